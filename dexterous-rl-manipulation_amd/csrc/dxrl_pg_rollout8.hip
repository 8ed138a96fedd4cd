// dxrl_pg_rollout8.hip -- the fused policy-gradient rollout for >= 32 envs per CU (config C4:
// 8192 envs on 256 CUs).  SURVEY.md §7 mapping (ii): an env on 8 lanes -- lane f < 5 owns finger f
// (its three joints, envs/manipulation_env.py:285-310 per-finger contact loop), lanes 5..7 the
// object axes -- so one 8-wave workgroup holds 32 envs and 8192 envs run in ONE round of 256
// workgroups (k_pg_rollout_ws holds 16 envs per workgroup: two rounds).
//
// Same step structure as k_pg_rollout_ws (dxrl_pg.hip): env waves 0..3 hold the envs, aux waves
// 4..7 are their lane-for-lane twins; all 8 waves split the actor MLP, now on two 16-row tiles.
// Every value is produced by the same instruction sequence on the same operands:
//   * the MLP: the same 16x16x32 MFMA chains in the same k order (a row's result does not depend
//     on the other rows of its tile) and the same tanh sequence;
//   * the Philox blocks: same keys, counters, streams and block ids;
//   * the env arithmetic op for op (ME:198-252), the reward (RS:50-187) in the reference's order.
// So the tapes, records and env state are bit-identical to k_pg_rollout_ws
// (tests/test_gpu_pg.py::test_lane_split_rollout_matches_64_env_kernel, diag 1024).
//
// What the 8-lane layout changes besides the envs per workgroup:
//   * a finger's three joints are lane-local: the finger sum, the closure term's negative-joint sum
//     and the contact test need no cross-lane shifts; the contact mask is the ballot itself;
//   * the drawing lanes finish the reset values (joint positions, sampler values) from the
//     uniforms, so the env lanes' reset path is LDS reads;
//   * the step's 480 Philox blocks (128 action-noise, 352 reset) are drawn by all 8 waves, one
//     per lane, in the head phase;
//   * the env lanes form dmin (the root of the least squared tip distance) for the aux twin's
//     reward settle, as k_pg_rollout_ws does, and the 15 log-density terms of the action and the
//     act tape; the aux twin sums the terms in action order one step later (beside the reward
//     settle), so log pi costs no cross-lane broadcast chain.
#include "dxrl_pg_rollout.h"

#include <stdio.h>

#include <vector>

using namespace dxrl;
using namespace dxrl::pg;

namespace dxrl {
namespace {

constexpr int kE8Waves = 8, kE8Threads = 64 * kE8Waves;

constexpr int kObsLd = 48;  // observation-noise row (floats): element k of env e at [e][k]

// lanes 0..7 of each 16-lane DPP row read lane K of the row, lanes 8..15 read lane 8 + K:
// row_newbcast restricted to the row's first / second pair of 4-lane banks (bank_mask 0x3 / 0xC)
template <int K>
__device__ __forceinline__ uint32_t bcast8_u32(uint32_t x) {
    const int lo = __builtin_amdgcn_update_dpp((int)x, (int)x, 0x150 + K, 0xF, 0x3, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(lo, (int)x, 0x150 + 8 + K, 0xF, 0xC, false);
}
template <int K>
__device__ __forceinline__ float bcast8(float x) {
    return __uint_as_float(bcast8_u32<K>(__float_as_uint(x)));
}
template <int K>
__device__ __forceinline__ double bcast8(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    const uint64_t lo = bcast8_u32<K>((uint32_t)u), hi = bcast8_u32<K>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)((hi << 32) | lo));
}

// The env's contact mask on its 8 lanes (ME:285-310): finger lane f sums its own three joint
// positions in order, forms the f64 tip and the squared distance to the object (axes on lanes
// 5..7) and tests it against the threshold without the root (sqrt_below, bit-exact); the ballot of
// the group's lanes 0..4 is the mask.  x: the finger's squared distance (finger lanes).
__device__ __forceinline__ uint32_t contacts8(const float (&jp)[kJ], double opd, double size, bool finger, int gbit,
                                              double& x) {
    const float sum = (jp[0] + jp[1]) + jp[2];  // np.sum of the finger's f32 joints, in order
    const double tip = (double)(sum * kC01);
    const double o0 = bcast8<5>(opd), o1 = bcast8<6>(opd), o2 = bcast8<7>(opd);
    const double dx = tip - o0, dy = tip - o1, dz = tip - o2;
    x = (dx * dx + dy * dy) + dz * dz;
    const bool hit = finger && sqrt_below(x, size * 1.5);
    return (uint32_t)(__ballot(hit) >> gbit) & 0x1Fu;
}

// 16x16x32 MFMA layer on TWO 16-row tiles (32 activation rows): per k-step each weight fragment
// feeds both row tiles.  Per row the chain is wave_layer16's (same fragments, same k order, same
// tanh), so the hidden units are bit-identical to k_pg_rollout_ws's.  Rows 16 + r are swizzled
// like row r (swz16).
template <int KS, int NT, bool kSwzA, bool kSwzOut, typename WF>
__device__ __forceinline__ void wave_layer16x2(const bf16* A, int lda, const WF& wfrag, int n0, bf16* out, int ldo,
                                               int lane, const float* bias_v = nullptr) {
    const int r = lane & 15, g = lane >> 4;
    f32x4 acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int kD = KS < 2 ? KS : 2;
    const auto afrag = [&](int i, int k) {
        const int col = 32 * k + 8 * g;
        return *reinterpret_cast<const bf16x8*>(A + (16 * i + r) * lda + (kSwzA ? swz16(r, col) : col));
    };
    bf16x8 a[kD][2];
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        a[k][0] = afrag(0, k);
        a[k][1] = afrag(1, k);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const bf16x8 w = wfrag(j, k);
            acc[0][j] = mfma16(w, a[k % kD][0], acc[0][j]);
            acc[1][j] = mfma16(w, a[k % kD][1], acc[1][j]);
        }
        if (k + kD < KS) {
            a[k % kD][0] = afrag(0, k + kD);
            a[k % kD][1] = afrag(1, k + kD);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            bf16x4 v;
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const f32x2 b = bias_v ? f32x2{tanh_bias(bias_v[4 * j + q]), tanh_bias(bias_v[4 * j + q + 1])}
                                       : f32x2{0.0f, 0.0f};
                const f32x2 t = tanh_pre2(f32x2{acc[i][j][q], acc[i][j][q + 1]}, b);
                v[q] = to_bf16(t.x);
                v[q + 1] = to_bf16(t.y);
            }
            const int col = n0 + 16 * j + 4 * g;
            *reinterpret_cast<bf16x4*>(out + (16 * i + r) * ldo + (kSwzOut ? swz16(r, col) : col)) = v;
        }
}

// Per-step draws of the 32 envs, written by the aux lanes in the head phase, read by the env
// lanes (and their aux twins) in P4.  jp0 / v2: the reset values themselves (the drawing lane
// applies the curriculum samplers, config.py:44-113), so the env lanes' reset is LDS reads.
struct __attribute__((aligned(16))) E8Draws {
    float eps[kE8Envs * 16];          // action noise, [env][dim]
    float dzn[kE8Envs * 16];          // dynamics noise (C5), [env][dim]
    float on[2][kE8Envs * kObsLd];    // observation noise, [row parity][env][element]
    float jp0[kE8Envs * 16];          // reset joint positions, [env][joint]
    double v2[kE8Envs * 8];           // reset sampler values: size, mass, friction, spawn x, y, z
};
struct E8Samplers {  // per env and extra slot: lo + span u with a range, the constant (span NaN) without
    double lo[kE8Envs * 8], span[kE8Envs * 8];
};
struct __attribute__((aligned(16))) E8Reward {  // an env's reward / log pi inputs and episode end of one step
    float term[16];      // log-density terms of the policy's action, action order (15 used)
    double dmin;         // np.min of the fingers' tip-object distances
    uint32_t c, prev;    // contacts, previous contacts (0x100: none)
    float nacc[kF];      // per finger: sum of its negative joint positions
    int32_t len, done, te;
    unsigned long long rctr;  // reset counter after the step (the next step's reset draws use it)
};

template <bool kNoise, bool kDiag>
__global__ __launch_bounds__(kE8Threads, 1) void k_pg_rollout_e8(PgRolloutArgs p) {
    constexpr int kHeadWave0 = 2;  // env waves 2, 3: the mu head of row tiles 0, 1
    constexpr int kW1sW = kIn + 16, kW3sW = kH + 16, kXsW = kIn + 16, kHsW = kH;
    constexpr int kHeadRows = 16;  // head rows 0..14 live (kAct), 15 padding
    __shared__ __attribute__((aligned(16))) bf16 W1s[kH * kW1sW];
    __shared__ __attribute__((aligned(16))) bf16 W3s[kHeadRows * kW3sW];
    __shared__ __attribute__((aligned(16))) bf16 X[kE8Envs * kXsW];
    __shared__ __attribute__((aligned(16))) bf16 H1[kE8Envs * kHsW];
    __shared__ __attribute__((aligned(16))) bf16 H2[kE8Envs * kHsW];
    __shared__ float MU[kE8Envs * (kOut + 1)];
    __shared__ float LS[kActPad], SIG[kActPad], ISIG[kActPad];
    __shared__ E8Draws DR;
    __shared__ E8Reward RW[2][kE8Envs];
    __shared__ E8Samplers RSMP;
    __shared__ uint32_t KEYS[kE8Envs][4];  // per env: reset key ek0, ek1, policy key pk0, pk1
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool aux = wave >= 4;
    const int et_tid = tid & 255;                 // the env lane this thread is (env wave) or twins (aux)
    const int eg = et_tid >> 3, s = et_tid & 7;   // env of the workgroup, lane of the env
    const int gbit = 8 * (lane >> 3);
    const bool finger = s < kF;
    const int ax = s - kF;  // object axis (lanes 5..7)
    const int64_t n = p.s.n;
    const int64_t i = (int64_t)blockIdx.x * kE8Envs + eg;
    const bool live = i < n;
    const int64_t T = p.horizon;
    if (tid < kAct) {
        const float ls = p.params[kOffLogStd + tid];
        LS[tid] = ls;
        SIG[tid] = __expf(ls);
        ISIG[tid] = __expf(-ls);
    }
    // this wave's L2 columns 32 wave .. + 31 as two 16-column tiles of 16x16x32 fragments
    bf16x8 w2[2][kH / 32];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < kH / 32; ++k)
            w2[j][k] = *reinterpret_cast<const bf16x8*>(p.wbf + kBfW2a + (int64_t)(32 * wave + 16 * j + (lane & 15)) * kHx +
                                                        32 * k + 8 * (lane >> 4));
    for (int c = tid; c < kH * (kIn / 8); c += kE8Threads) {
        const int row = c / (kIn / 8), col = 8 * (c % (kIn / 8));
        *reinterpret_cast<bf16x8*>(W1s + row * kW1sW + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW1a + (int64_t)row * kIn + col);
    }
    for (int c = tid; c < kHeadRows * (kH / 8); c += kE8Threads) {
        const int row = c / (kH / 8), col = 8 * (c % (kH / 8));
        *reinterpret_cast<bf16x8*>(W3s + row * kW3sW + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW3a + (int64_t)row * kHx + col);
    }
    for (int c = tid; c < kE8Envs * kXsW; c += kE8Threads) X[c] = (c % kXsW == kObsIn) ? (bf16)1.0f : (bf16)0.0f;
    const int r16 = lane & 15, g16 = lane >> 4;  // 16x16x32 fragment row / k group
    const auto w1frag = [&](int j, int k) {
        return *reinterpret_cast<const bf16x8*>(W1s + (32 * wave + 16 * j + r16) * kW1sW + 32 * k + 8 * g16);
    };
    const auto w2frag = [&](int j, int k) { return w2[j][k]; };
    float b2_reg[8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            b2_reg[4 * j + q] = p.params[kOffW2a + (int64_t)(32 * wave + 16 * j + 4 * g16 + q) * kHx + kH];
    const float b3_reg = p.params[kOffW3a + (int64_t)r16 * kHx + kH];

    // ---- env-lane state (env waves) / episode bookkeeping (aux waves)
    float jp[kJ] = {0.0f, 0.0f, 0.0f}, jv[kJ] = {0.0f, 0.0f, 0.0f};
    double opd = 0.0;
    float ovd = 0.0f;
    uint32_t flags = 0;
    int32_t et = 0;
    double size = 0.0, mass = 0.0, fric = 0.0, ep_ret = 0.0, sum_ret = 0.0;
    int32_t cnt = 0, sum_len = 0, succ = 0;
    uint64_t rctr = 0;
    bool fric64 = false;
    if (live) {
        if (!aux) {
            if (finger) {
#pragma unroll
                for (int j = 0; j < kJ; ++j) {
                    jp[j] = p.s.jp[(int64_t)(kJ * s + j) * n + i];
                    jv[j] = p.s.jv[(int64_t)(kJ * s + j) * n + i];
                }
            } else {
                opd = p.s.op[(int64_t)ax * n + i];
                ovd = p.s.ov[(int64_t)ax * n + i];
            }
            flags = p.s.flags[i];
            et = p.s.t[i];
            size = p.s.size[i];
            mass = p.s.mass[i];
            fric = p.s.fric[i];
            rctr = p.s.reset_ctr[i];
            const dxrl_curriculum& cu = p.s.curricula[p.s.cfg[i]];
            fric64 = cu.friction_is_f64_scalar != 0;
            if (s < DXRL_RESET_EXTRA) {  // this lane's extra reset sampler (config.py:44-113)
                const double* rg = s == 0 ? cu.size_range
                                          : s == 1 ? cu.mass_range
                                                   : s == 2 ? cu.friction_range
                                                            : s == 3 ? cu.spawn_x_range
                                                                     : s == 4 ? cu.spawn_y_range : cu.spawn_z_range;
                const double cst = s == 0 ? cu.object_size : s == 1 ? cu.object_mass : cu.friction_coefficient;
                const bool has = s == 0 ? cu.has_size_range != 0
                                        : s == 1 ? cu.has_mass_range != 0 : s == 2 ? cu.has_friction_range != 0 : true;
                RSMP.lo[eg * 8 + s] = has ? rg[0] : cst;
                RSMP.span[eg * 8 + s] = has ? rg[1] - rg[0] : __builtin_nan("");
            }
            if (s == 0) {
                uint32_t k0, k1;
                env_key(p.env_seed, p.gid0 + i, k0, k1);
                KEYS[eg][0] = k0;
                KEYS[eg][1] = k1;
                env_key(p.policy_seed, p.gid0 + i, k0, k1);
                KEYS[eg][2] = k0;
                KEYS[eg][3] = k1;
                RW[1][eg].rctr = rctr;  // "after step -1"
            }
        } else {
            ep_ret = p.ep_ret[i];
        }
    }
    const bool obs_noise = kNoise && p.obs_noise > 0.0f, dyn_noise = kNoise && p.dyn_noise > 0.0f;
    const auto env_live = [&](int e) { return (int64_t)blockIdx.x * kE8Envs + e < n; };

    // ---- head phase: this step's Philox blocks, one per lane of ALL 8 waves (480 tasks on 512
    // lanes): tasks 0..127 the action noise (env q / 4, block q % 4), 128..479 the reset uniforms at
    // each env's exact counter (env r / 11, block r % 11; slots 2 b, 2 b + 1: joint slots 0..14,
    // extra slots 15..20).  Same blocks and arithmetic as k_pg_rollout_ws's step_draws.  Waves
    // 0, 1 (SIMDs 0, 1) draw the action noise, waves 4..7 and 2 the reset blocks, and wave 3 --
    // which also runs the second row tile of the mu head -- the last 32.
    constexpr int kResetBlocks = (kReset + 1) / 2;
    constexpr int kActTasks = kE8Envs * 4, kTasks = kActTasks + kE8Envs * kResetBlocks;
    static_assert(kTasks <= kE8Threads && kActTasks == 128, "one draw task per lane");
    const auto step_draws = [&](uint64_t ctr, int64_t t_) {
        // the task index re-derived from a volatile lane id each step (not hoisted into a
        // long-lived register)
        int l;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        // wave -> first task: 0, 64 | 384, 448 | 128, 192, 256, 320
        const int base = wave < 2 ? 64 * wave : wave < 4 ? 384 + 64 * (wave - 2) : 128 + 64 * (wave - 4);
        const int q = base + l;
        if (q >= kTasks) return;
        if (wave < 2) {  // action noise (wave-uniform branch)
            const int e = q >> 2, b = q & 3;
            if (!env_live(e)) return;
            const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamPolicy, (uint32_t)b},
                                   KEYS[e][2], KEYS[e][3]);
            float4 nz;
            box_muller(r.x, r.y, nz.x, nz.y);
            box_muller(r.z, r.w, nz.z, nz.w);
            *reinterpret_cast<float4*>(&DR.eps[16 * e + 4 * b]) = nz;
            return;
        }
        const int rq = q - kActTasks, e = rq / kResetBlocks, b = rq % kResetBlocks;
        if (!env_live(e)) return;
        const uint64_t rc = RW[(t_ - 1) & 1][e].rctr;
        const u32x4 r = philox(u32x4{(uint32_t)rc, (uint32_t)(rc >> 32), kStreamReset, (uint32_t)b}, KEYS[e][0],
                               KEYS[e][1]);
        const double ua = u01_53(r.x, r.y), ub = u01_53(r.z, r.w);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = 2 * b + h;
            const double u = h ? ub : ua;
            if (k < kD) {
                DR.jp0[16 * e + k] = (float)(-0.1 + (0.1 - -0.1) * u);
            } else if (k < kReset) {
                const double lo = RSMP.lo[8 * e + k - kD], span = RSMP.span[8 * e + k - kD];
                DR.v2[8 * e + k - kD] = span == span ? lo + span * u : lo;
            }
        }
    };
    // ---- aux, P0: the next observation row's noise (12 blocks per env) and this step's dynamics
    // noise (4 blocks per env), two tasks per aux lane (512 per workgroup)
    constexpr int kOb = (kObs + 3) / 4, kObsTasks = kE8Envs * kOb, kNoiseTasks = kObsTasks + kE8Envs * 4;
    static_assert(kNoiseTasks <= 512, "two noise tasks per aux lane");
    const auto obs_draws = [&](uint64_t ctr, int buf, bool dyn, uint64_t dctr) {
        if (!(obs_noise || (dyn && dyn_noise))) return;
        const int L = 64 * (wave - 4) + lane;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = L + 256 * h;
            const bool is_obs = q < kObsTasks;
            const int e = is_obs ? q / kOb : (q - kObsTasks) >> 2, b = is_obs ? q % kOb : (q - kObsTasks) & 3;
            const bool want = is_obs ? obs_noise : (dyn && dyn_noise);
            if (!want || !env_live(e)) continue;
            const uint64_t c = is_obs ? ctr : dctr;
            float n4[4];
            noise_normals4(c, is_obs ? kStreamObs : kStreamDyn, (uint32_t)b, KEYS[e][2], KEYS[e][3], n4);
            const float4 nz = float4{n4[0], n4[1], n4[2], n4[3]};
            if (!is_obs) {
                *reinterpret_cast<float4*>(&DR.dzn[16 * e + 4 * b]) = nz;
                continue;
            }
            *reinterpret_cast<float4*>(&DR.on[buf][kObsLd * e + 4 * b]) = nz;
            if (kDiag && p.obs_noise_tape) {  // parity tape: the value write_obs_row adds
                const int64_t row = (int64_t)(c - p.iteration * (uint64_t)T);
                const int64_t ie = (int64_t)blockIdx.x * kE8Envs + e;
                float4 v;
                v.x = 4 * b + 0 < kObs ? p.obs_noise * nz.x : 0.0f;
                v.y = 4 * b + 1 < kObs ? p.obs_noise * nz.y : 0.0f;
                v.z = 4 * b + 2 < kObs ? p.obs_noise * nz.z : 0.0f;
                v.w = 4 * b + 3 < kObs ? p.obs_noise * nz.w : 0.0f;
                *reinterpret_cast<float4*>(p.obs_noise_tape + (row * n + ie) * kObsNoiseLd + 4 * b) = v;
            }
        }
    };
    // ---- aux: the dense reward (RS:50-187) and the episode bookkeeping of a finished step
    const auto settle = [&](int64_t t_) {
        const E8Reward& w = RW[t_ & 1][eg];
        const double dist = exp(-5.0 * w.dmin);
        const double con = count_over_f_f64(__popc(w.c));
        float sum = 0.0f;
#pragma unroll
        for (int f = 0; f < kF; ++f) sum = sum + (-w.nacc[f]);
        const float avg = div_f(sum);
        const float clo = clipf(div_f(avg), 0.0f, 1.0f);
        float st = 0.0f;
        if (w.prev != 0x100u) {
            float ch = 0.0f;
#pragma unroll
            for (int f = 0; f < kF; ++f) ch = ch + (float)(((w.c ^ w.prev) >> f) & 1u);
            st = clipf(1.0f - count_over_f_f32((uint32_t)ch), 0.0f, 1.0f);
        }
        const double r = ((p.w.w_dist * dist + p.w.w_con * con) + p.w.w_clo * (double)clo) + p.w.w_st * (double)st;
        ep_ret += r;
        if (s == 0) p.rew[t_ * n + i] = (float)r;
        if (w.done) {
            if (s == 0 && cnt < p.record_cap) {
                const int64_t o = i * p.record_cap + cnt;
                p.rec_return[o] = ep_ret;
                p.rec_length[o] = w.len;
                p.rec_success[o] = p.success_terminated ? (uint8_t)w.te : (uint8_t)0;
                p.rec_end_step[o] = (int32_t)t_;
            }
            ++cnt;
            sum_ret += ep_ret;
            sum_len += w.len;
            succ += w.te;
            ep_ret = 0.0;
        }
    };
    // ---- env lanes, P0: the observation row (ME:254-264): finger lane f its joint positions /
    // velocities 3 f .. 3 f + 2 and contact flag f, object lane 5 + a the object position /
    // velocity of axis a and quaternion element a (lane 5 also the last one)
    const auto write_obs_row = [&](int buf) {
        bf16* xr = X + eg * kXsW;
        const float* on = DR.on[buf] + kObsLd * eg;
        const auto put = [&](int k, float v) {
            if (obs_noise) v = v + p.obs_noise * on[k];
            xr[k] = to_bf16(v);
        };
        if (finger) {
#pragma unroll
            for (int j = 0; j < kJ; ++j) {
                put(kJ * s + j, jp[j]);
                put(kD + kJ * s + j, jv[j]);
            }
            put(2 * kD + 10 + s, (float)((flags >> s) & 1u));
        } else {
            put(2 * kD + ax, (float)opd);
            put(2 * kD + 7 + ax, ovd);
            put(2 * kD + 3 + ax, ax == 0 ? 1.0f : 0.0f);  // identity quaternion (ME:164)
            if (ax == 0) put(2 * kD + 6, 0.0f);
        }
    };
    const auto tape_obs_row = [&](int64_t m) {
        *reinterpret_cast<bf16x8*>(p.obs_rm + m * kIn + 8 * s) = *reinterpret_cast<const bf16x8*>(X + eg * kXsW + 8 * s);
    };
    const bool mlp = !kDiag || !(p.diag & 1), env_on = !kDiag || !(p.diag & 2);
    // ---- env lanes, head phase: the object's damping, gravity, position and wall stops
    // (ME:212-235; independent of the action)
    const auto env_object_step = [&]() {
        const double damp = 1.0 - (fric * 0.1 * 0.01);
        const float dampf = (float)damp;
        const bool op32 = (flags & kOpIsF32) != 0, fric_f64 = (flags & kFricF64) != 0;
        const int a3 = finger ? 0 : ax;
        const double gz = a3 == 2 ? kGz : 0.0, lo = a3 == 2 ? 0.0 : -0.2, hi = a3 == 2 ? 0.3 : 0.2;
        float v = fric_f64 ? (float)((double)ovd * damp) : ovd * dampf;
        v = (float)((double)v + gz);
        const float inc = v * kDt;
        double q = op32 ? (double)((float)opd + inc) : opd + (double)inc;
        q = clipd(q, lo, hi);
        if ((q <= lo && v < 0.0f) || (q >= hi && v > 0.0f)) v = 0.0f;
        if (!finger) {
            opd = q;
            ovd = v;
        }
        flags &= ~kOpIsF32;
    };
    // ---- env lanes, P4: action, dynamics, contacts (and dmin for the aux twin's reward),
    // termination, auto-reset
    const auto env_lane_step = [&](int64_t t, int64_t m) {
        bool te = false, tr = false;
        float a0[kJ], mu0[kJ];  // the policy's action and mean (log pi at the end of the step)
        if (finger) {
#pragma unroll
            for (int j = 0; j < kJ; ++j) {
                const int k = kJ * s + j;
                mu0[j] = mlp ? MU[eg * (kOut + 1) + k] : 0.0f;
                a0[j] = mu0[j] + SIG[k] * DR.eps[16 * eg + k];
                p.act[m * kActPad + k] = a0[j];
                float a = a0[j];
                if (dyn_noise)  // robustness_tests.py:180-187 (the tape keeps the policy's action)
                    a = clipf(a + p.dyn_noise * DR.dzn[16 * eg + k], -1.0f, 1.0f);
                if (kDiag && p.applied_act) p.applied_act[m * kActPad + k] = a;
                if (kDiag && p.dyn_noise_tape)
                    p.dyn_noise_tape[m * kActPad + k] = dyn_noise ? p.dyn_noise * DR.dzn[16 * eg + k] : 0.0f;
                if (env_on) {
                    const float ak = clipf(a, -1.0f, 1.0f);
                    jv[j] = kC09 * jv[j] + kC01 * ak;
                    jp[j] = clipf(jp[j] + jv[j] * kDt, -1.0f, 1.0f);
                }
            }
        } else if (s == kF) {  // the tapes' padding slot
            p.act[m * kActPad + kAct] = 0.0f;
            if (kDiag && p.applied_act) p.applied_act[m * kActPad + kAct] = 0.0f;
            if (kDiag && p.dyn_noise_tape) p.dyn_noise_tape[m * kActPad + kAct] = 0.0f;
        }
        if (env_on) {
            double x;
            const uint32_t c = contacts8(jp, opd, size, finger, gbit, x);
            E8Reward& rw = RW[t & 1][eg];
            if (finger) {  // the reward's inputs for the aux twin (RS:101-187)
                float nacc = 0.0f;
#pragma unroll
                for (int j = 0; j < kJ; ++j)
                    if (jp[j] < 0.0f) nacc = nacc + jp[j];
                rw.nacc[s] = nacc;
            }
            // dmin = min_f sqrt_rn(x_f) = sqrt_rn(min_f x_f) (the rounded root is monotone)
            double xm = bcast8<0>(x);
            const double x1 = bcast8<1>(x), x2 = bcast8<2>(x), x3 = bcast8<3>(x), x4 = bcast8<4>(x);
            xm = x1 < xm ? x1 : xm;
            xm = x2 < xm ? x2 : xm;
            xm = x3 < xm ? x3 : xm;
            xm = x4 < xm ? x4 : xm;
            if (s == 0) {
                rw.dmin = sqrt(xm);
                rw.c = c;
                rw.prev = (flags & kHasPrev) ? ((flags >> kPrevShift) & 0xFFu) : 0x100u;
            }
            flags = (flags & ~(0xFFu << kPrevShift)) | (c << kPrevShift) | kHasPrev;
            flags = (flags & ~0xFFu) | c;
            te = __popc(c) >= 3;
            tr = et >= p.max_episode_steps;
            et += 1;
        }
        const bool d = env_on && (te || tr || et >= p.max_steps);
        if (s == 0) {
            p.done[m] = d;
            if (p.ep_code)
                p.ep_code[m] = d ? (uint16_t)((et << 1) | (p.success_terminated && te ? 1 : 0)) : (uint16_t)0;
            E8Reward& rw = RW[t & 1][eg];
            rw.done = d;
            rw.te = te;
            rw.len = et;
        }
        if (d) {
            // ---- reset (ME:124-182) from the values the drawing lanes finished
            if (finger) {
#pragma unroll
                for (int j = 0; j < kJ; ++j) {
                    jp[j] = DR.jp0[16 * eg + kJ * s + j];
                    jv[j] = 0.0f;
                }
            }
            size = DR.v2[8 * eg + 0];
            mass = DR.v2[8 * eg + 1];
            fric = DR.v2[8 * eg + 2];
            const bool has = (flags & kHasObject) != 0;
            if (!finger) {
                const double spawn = DR.v2[8 * eg + 3 + ax];
                opd = (double)(float)(has ? opd : spawn);
                ovd = 0.0f;
            }
            et = 0;
            flags = kOpIsF32 | kHasObject | (fric64 ? kFricF64 : 0u);
            double x;
            flags |= contacts8(jp, opd, size, finger, gbit, x);  // ME:176
            ++rctr;
        }
        if (s == 0) RW[t & 1][eg].rctr = rctr;
        // log N(a | mu, sigma) terms of the finger's action dims (gauss_logp), off the step's
        // chain (its own basic block after the reset); the aux twin sums them next step.  Forming
        // only the first term here and the other two on the aux twin balances the two waves' P4
        // stamps but measured no faster (profiles/r05/ab_e8_logpi_terms.log)
        __builtin_amdgcn_sched_barrier(0);
        if (finger) {
#pragma unroll
            for (int j = 0; j < kJ; ++j) {
                const int k = kJ * s + j;
                const float z = (a0[j] - mu0[j]) * ISIG[k];
                RW[t & 1][eg].term[k] = -0.5f * z * z - LS[k] - 0.5f * kLog2Pi;
            }
        }
    };
    // ---- aux lanes: log pi(a|s) of step t_ -- the env lanes' 15 terms summed in action order
    // (gauss_logp / row_sum_in_order's order), one step after they were written
    const auto settle_logp = [&](int64_t t_) {
        const float4* tv = reinterpret_cast<const float4*>(RW[t_ & 1][eg].term);
        float lp = 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = tv[q];
            lp += v.x;
            lp += v.y;
            lp += v.z;
            if (4 * q + 3 < kAct) lp += v.w;
        }
        if (s == 0) p.logp[t_ * n + i] = lp;
    };

    // diag & 128: s_memtime segment stamps per step: env waves into stamps[16 i + k], aux waves
    // into stamps[16 i + 8 + k]
    unsigned long long st_acc[8], st_last = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) st_acc[q] = 0;
#define E8_STAMP(k)                                                                              \
    do {                                                                                         \
        if (kDiag && (p.diag & 128)) {                                                           \
            __builtin_amdgcn_sched_barrier(0);                                                   \
            unsigned long long t_;                                                               \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
            __builtin_amdgcn_sched_barrier(0);                                                   \
            st_acc[k] += t_ - st_last;                                                           \
            st_last = t_;                                                                        \
        }                                                                                        \
    } while (0)
    __syncthreads();  // KEYS, RSMP visible to the drawing lanes
    if (aux) obs_draws(p.iteration * (uint64_t)T, 0, false, 0);
    __syncthreads();
    E8_STAMP(7);
    for (int64_t t = 0; t < T; ++t) {
        const int64_t m = t * n + i;
        const uint64_t ctr = p.iteration * (uint64_t)T + (uint64_t)t;
        if (!aux && live) write_obs_row((int)(t & 1));
        if (aux) obs_draws(ctr + 1, (int)((t + 1) & 1), true, ctr);
        E8_STAMP(0);
        lds_barrier();
        if (!aux && live) tape_obs_row(m);
        if (mlp) wave_layer16x2<kIn / 32, 2, false, true>(X, kXsW, w1frag, 32 * wave, H1, kHsW, lane);  // b: col 45
        E8_STAMP(1);
        lds_barrier();
        if (mlp) wave_layer16x2<kH / 32, 2, true, true>(H1, kHsW, w2frag, 32 * wave, H2, kHsW, lane, b2_reg);
        E8_STAMP(2);
        lds_barrier();
        if (!aux && live && env_on) env_object_step();
        if (mlp && (wave == kHeadWave0 || wave == kHeadWave0 + 1)) {
            // mu head of row tile rt: 16 env rows x head rows 0..15 (15 live), k ring of 4
            const int rt = wave - kHeadWave0;
            const bf16* h2 = H2 + (16 * rt + r16) * kHsW;
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            constexpr int kDh = 4;
            bf16x8 ah[kDh], bw[kDh];
#pragma unroll
            for (int k = 0; k < kDh; ++k) {
                ah[k] = *reinterpret_cast<const bf16x8*>(h2 + swz16(r16, 32 * k + 8 * g16));
                bw[k] = *reinterpret_cast<const bf16x8*>(W3s + r16 * kW3sW + 32 * k + 8 * g16);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < kH / 32; ++k) {
                acc = mfma16(ah[k % kDh], bw[k % kDh], acc);
                if (k + kDh < kH / 32) {
                    ah[k % kDh] = *reinterpret_cast<const bf16x8*>(h2 + swz16(r16, 32 * (k + kDh) + 8 * g16));
                    bw[k % kDh] = *reinterpret_cast<const bf16x8*>(W3s + r16 * kW3sW + 32 * (k + kDh) + 8 * g16);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) MU[(16 * rt + 4 * g16 + q) * (kOut + 1) + r16] = acc[q] + b3_reg;
        }
        if (mlp && p.h2_tape) {
            // the step's H2 rows (32 envs x 32 chunks of 16 bytes; chunk c of row r at c ^ (r & 15))
            // to the actor's layer-2 tape, two chunks per thread
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = tid + 512 * u, row = q >> 5, c = q & 31;
                const int64_t ie = (int64_t)blockIdx.x * kE8Envs + row;
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(H2 + row * kHsW + ((c ^ (row & 15)) << 3));
                if (ie < n) __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p.h2_tape + (t * n + ie) * kH2Ld + 8 * c));
            }
        }
        step_draws(ctr, t);
        E8_STAMP(3);
        lds_barrier();
        E8_STAMP(4);
        if (live) {
            if (aux) {
                if (t > 0) {  // step t-1's log pi, reward and bookkeeping
                    settle_logp(t - 1);
                    if (env_on) settle(t - 1);
                }
            } else {
                env_lane_step(t, m);
            }
        }
        E8_STAMP(5);
        lds_barrier();  // this step's reward inputs / the next row's noise visible
        E8_STAMP(6);
    }
#undef E8_STAMP
    if (kDiag && (p.diag & 128) && s == 0 && live) {
#pragma unroll
        for (int q = 0; q < 8; ++q) p.stamps[16 * i + (aux ? 8 : 0) + q] = st_acc[q];
    }
    if (live && aux) {
        if (T > 0) settle_logp(T - 1);
        if (T > 0 && env_on) settle(T - 1);
        if (kDiag && (p.diag & 2))
            for (int64_t t = 0; t < T && s == 0; ++t) p.rew[t * n + i] = 0.0f;
        if (s == 0) {
            p.ep_ret[i] = ep_ret;
            p.ep_count[i] = cnt;
            p.ep_sum_ret[i] = sum_ret;
            p.ep_sum_len[i] = sum_len;
            p.ep_succ[i] = succ;
        }
    }
    if (live && !aux) {
        // bootstrap observation (slot T), then the state back to the slab
        write_obs_row((int)(T & 1));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        tape_obs_row(T * n + i);
        if (finger) {
#pragma unroll
            for (int j = 0; j < kJ; ++j) {
                p.s.jp[(int64_t)(kJ * s + j) * n + i] = jp[j];
                p.s.jv[(int64_t)(kJ * s + j) * n + i] = jv[j];
            }
        } else {
            p.s.op[(int64_t)ax * n + i] = opd;
            p.s.ov[(int64_t)ax * n + i] = ovd;
        }
        if (s == 0) {
            p.s.flags[i] = flags;
            p.s.t[i] = et;
            p.s.size[i] = size;
            p.s.mass[i] = mass;
            p.s.fric[i] = fric;
            p.s.reset_ctr[i] = rctr;
        }
    }
}

}  // namespace

int launch_pg_rollout_e8(const PgRolloutArgs& p, int64_t n, bool noise, bool diag, hipStream_t st) {
    const dim3 grid((unsigned)((n + kE8Envs - 1) / kE8Envs)), block(kE8Threads);
    if (noise && diag) hipLaunchKernelGGL((k_pg_rollout_e8<true, true>), grid, block, 0, st, p);
    else if (noise) hipLaunchKernelGGL((k_pg_rollout_e8<true, false>), grid, block, 0, st, p);
    else if (diag) hipLaunchKernelGGL((k_pg_rollout_e8<false, true>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((k_pg_rollout_e8<false, false>), grid, block, 0, st, p);
    if (int rc = launch_check("k_pg_rollout_e8")) return rc;
    if (p.diag & 128) {  // diagnostics: mean cycles per env per step segment, env / aux waves
        std::vector<unsigned long long> h((size_t)n * 16);
        (void)hipStreamSynchronize(st);
        (void)hipMemcpy(h.data(), p.stamps, h.size() * 8, hipMemcpyDeviceToHost);
        for (int w = 0; w < 2; ++w) {
            fprintf(stderr, "rollout_e8 %s cycles/step:", w ? "aux" : "env");
            for (int k = 0; k < 7; ++k) {
                double sum = 0;
                for (int64_t e = 0; e < n; ++e) sum += (double)h[e * 16 + 8 * w + k];
                fprintf(stderr, " s%d=%.0f", k, sum / n / p.horizon);
            }
            fprintf(stderr, "\n");
            for (int wv = 0; wv < 4; ++wv) {  // per wave of the workgroup (envs 8 wv .. 8 wv + 7)
                fprintf(stderr, "  wave %d:", 4 * w + wv);
                for (int k = 0; k < 7; ++k) {
                    double sum = 0;
                    int64_t cnt = 0;
                    for (int64_t e = 0; e < n; ++e)
                        if ((e % kE8Envs) / 8 == wv) {
                            sum += (double)h[e * 16 + 8 * w + k];
                            ++cnt;
                        }
                    fprintf(stderr, " s%d=%.0f", k, cnt ? sum / cnt / p.horizon : 0.0);
                }
                fprintf(stderr, "\n");
            }
        }
    }
    return DXRL_OK;
}

}  // namespace dxrl
