// dxrl_pg.hip -- policy-gradient learner on MI355X (no reference counterpart:
// the reference's only learner is the SimpleLearner hill-climber; SURVEY.md
// §8(a) A11-A13).  Actor-critic MLP, GAE(gamma, lambda) reverse scan,
// two-pass advantage normalisation, PPO-clip heads, Adam.
//
// k_pg_rollout is the hot loop: one workgroup owns 64 envs for the whole
// horizon.  Per env step it runs the actor MLP on its 64-row tile with bf16
// MFMA (weights streamed from L2, activations in LDS), samples
// a = mu + sigma * eps (Philox), optionally injects dynamics / observation
// noise (robustness_tests.py:140-211, config C5), steps the 64 envs (the
// same env_step as dxrl_env_step), writes the training tape and auto-resets.
// No inter-workgroup communication: envs and weights are independent/read-only.
#include "dxrl_gemm.h"
#include "dxrl_pg.h"
#include "dxrl_pg_rollout.h"

#include <stdio.h>

#include <vector>

using namespace dxrl;
using namespace dxrl::pg;

namespace dxrl {

// log N(a | mu, sigma) summed over the action dims
__device__ __forceinline__ float gauss_logp(const float* a, const float* mu, const float* logstd) {
    float lp = 0.0f;
#pragma unroll
    for (int k = 0; k < kAct; ++k) {
        const float z = (a[k] - mu[k]) * __expf(-logstd[k]);
        lp += -0.5f * z * z - logstd[k] - 0.5f * kLog2Pi;
    }
    return lp;
}

// 15 (or more) standard normals from one Philox stream position
template <int N>
__device__ __forceinline__ void philox_normals(float* out, uint32_t k0, uint32_t k1, uint64_t ctr, uint32_t stream) {
#pragma unroll
    for (int b = 0; b < (N + 3) / 4; ++b) {
        float n0, n1, n2, n3;
        if (stream == kStreamPolicy) {
            const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), stream, (uint32_t)b}, k0, k1);
            box_muller(r.x, r.y, n0, n1);
            box_muller(r.z, r.w, n2, n3);
        } else {  // a noise stream
            float nz[4];
            noise_normals4(ctr, stream, (uint32_t)b, k0, k1, nz);
            n0 = nz[0];
            n1 = nz[1];
            n2 = nz[2];
            n3 = nz[3];
        }
        if (4 * b + 0 < N) out[4 * b + 0] = n0;
        if (4 * b + 1 < N) out[4 * b + 1] = n1;
        if (4 * b + 2 < N) out[4 * b + 2] = n2;
        if (4 * b + 3 < N) out[4 * b + 3] = n3;
    }
}


constexpr int kTile = 64;           // envs per workgroup
constexpr int kXs = kIn + 8;        // LDS row strides (bf16) -- conflict-free b128 fragment reads
constexpr int kHs = kH + 8;

// observation element k of ME:254-264 (k is a compile-time constant after unrolling)
__device__ __forceinline__ float obs_elem(const Env& e, int k) {
    if (k < kD) return e.jp[k];
    if (k < 2 * kD) return e.jv[k - kD];
    if (k < 2 * kD + 3) return (float)e.op[k - 2 * kD];
    if (k < 2 * kD + 7) return k == 2 * kD + 3 ? 1.0f : 0.0f;  // identity quaternion
    if (k < 2 * kD + 10) return e.ov[k - 2 * kD - 7];
    return (float)((e.flags >> (k - 2 * kD - 10)) & 1u);
}

// Policy input row: obs (+ observation noise, robustness_tests.py:199-207: obs + f32(N(0, s))),
// streamed 4 elements per Philox block into the bf16 LDS row and the tape.
__device__ __forceinline__ void write_policy_obs(const Env& e, bf16* xrow, float obs_noise, uint32_t k0, uint32_t k1,
                                                 uint64_t ctr, bf16* tape_rm, bf16* tape_fm, int64_t m,
                                                 int64_t ld_fm) {
#pragma unroll
    for (int b = 0; b < (kObs + 3) / 4; ++b) {
        float nz[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (obs_noise > 0.0f) noise_normals4(ctr, kStreamObs, (uint32_t)b, k0, k1, nz);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = 4 * b + q;
            if (k >= kObs) break;
            float v = obs_elem(e, k);
            if (obs_noise > 0.0f) v = v + obs_noise * nz[q];
            xrow[k] = to_bf16(v);
        }
    }
    if (tape_rm) {
#pragma unroll
        for (int q = 0; q < kIn / 8; ++q) {
            bf16x8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 8 * q + j;
                v[j] = k < kObs ? xrow[k] : (k == kObsIn ? (bf16)1.0f : (bf16)0.0f);
            }
            reinterpret_cast<bf16x8*>(tape_rm + m * kIn)[q] = v;
        }
    }
    if (tape_fm) {
#pragma unroll
        for (int k = 0; k < kObs; ++k) tape_fm[(int64_t)k * ld_fm + m] = xrow[k];
    }
}

// Register-resident weight fragments: one 32-column N tile of a layer, all of
// K (K/16 MFMA k-steps): b[k] = W[n0 + r][16k + 8h .. 16k + 8h + 7].  Loaded
// once per rollout launch, so the per-step MLP reads no weights from memory.
template <int KS>
struct WTile {
    bf16x8 b[KS];
};

template <int KS>
__device__ __forceinline__ void load_wtile(WTile<KS>& w, const bf16* W, int ldw, int n0, int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int k = 0; k < KS; ++k) w.b[k] = *reinterpret_cast<const bf16x8*>(W + (int64_t)(n0 + r) * ldw + 16 * k + 8 * h);
}

// One wave: 64 rows x 32*NT columns of act(A . W^T + b) into LDS.  A: LDS [64][lda]
// bf16; the weight fragment of N-tile j, k-step k comes from wfrag(j, k) (registers
// or LDS); bias: f32 master column (bias[n * ldb]), the values the training GEMMs use, or
// bias_v[j] = that value already in a register (a persistent kernel hoists the load: a global
// load inside the step loop puts a vmcnt(0) -- which also drains every outstanding tape store --
// on the step's critical path).
template <int KS, int NT, bool kTanh, int RT = 2, typename WF, bool kRing = false>
__device__ __forceinline__ void wave_layer(const bf16* A, int lda, const WF& wfrag, int n0, const float* bias_p,
                                           int ldb, bf16* out, int ldo, int lane, const float* bias_v = nullptr) {
    // RT row tiles of 32 (RT == 1: 16 live rows -- accumulator registers q < 8)
    constexpr int kQ = RT == 1 ? 8 : 16;
    const int r = lane & 31, h = lane >> 5;
    f32x16 acc[RT][NT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;
    if constexpr (RT == 1 && !kRing) {
        // one row tile: issue every activation fragment up front (KS LDS reads in flight),
        // then the MFMA chain consumes them with counted waits
        bf16x8 a[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) a[k] = *reinterpret_cast<const bf16x8*>(A + r * lda + 16 * k + 8 * h);
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[0][j] = mfma32(a[k], wfrag(j, k), acc[0][j]);
    } else if constexpr (RT == 1) {
        // one row tile: a ring of kD activation fragments, refilled kD k-steps ahead; the
        // scheduling barriers keep the refills where they are (under register pressure the
        // scheduler otherwise sinks every read next to its MFMA, exposing one LDS latency per
        // k-step instead of one per chain)
        constexpr int kD = KS < 4 ? KS : 4;
        bf16x8 a[kD];
#pragma unroll
        for (int k = 0; k < kD; ++k) a[k] = *reinterpret_cast<const bf16x8*>(A + r * lda + 16 * k + 8 * h);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[0][j] = mfma32(a[k % kD], wfrag(j, k), acc[0][j]);
            if (k + kD < KS) a[k % kD] = *reinterpret_cast<const bf16x8*>(A + r * lda + 16 * (k + kD) + 8 * h);
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            bf16x8 a[RT];
#pragma unroll
            for (int i = 0; i < RT; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + (32 * i + r) * lda + 16 * k + 8 * h);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const bf16x8 b = wfrag(j, k);
#pragma unroll
                for (int i = 0; i < RT; ++i) acc[i][j] = mfma32(a[i], b, acc[i][j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = n0 + 32 * j + r;
        const float bias = bias_v ? bias_v[j] : bias_p ? bias_p[(int64_t)n * ldb] : 0.0f;
        const float bk = tanh_bias(bias);
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const float v = kTanh ? tanh_pre(acc[i][j][q], bk) : acc[i][j][q] + bias;
                out[(32 * i + acc_row(q, lane)) * ldo + n] = to_bf16(v);
            }
    }
}

// 16-row tiles on v_mfma_f32_16x16x32_bf16 for a 16-env workgroup: one wave computes the 16
// activation rows x 16*NT columns with no dead MFMA rows (wave_layer's RT == 1 tile carries 16
// live rows in a 32-row MFMA: twice the matrix-core cycles per output).  A chain of 16x16x32
// MFMAs over k-steps of 32 rounds exactly like the 32x32x16 chain over the same k order
// (tools/mfma_order.hip: 0 of 131,072 outputs differ), so the hidden units stay bit-identical to
// the learner's forward and to the one-lane k_pg_rollout.  Transposed formulation (weights as the A
// operand, as in the learner): lane l's accumulator holds columns n0 + 16 j + 4 (l >> 4) .. +3 of
// activation row l & 15, so the tanh epilogue runs on packed pairs and leaves as one 8-byte LDS
// store per tile.  Fragments: A row l & 15, k 32 k + 8 (l >> 4) ..+7; wfrag(j, k) =
// W[n0 + 16 j + (l & 15)][32 k + 8 (l >> 4) ..+7].  Activation fragments stream through a ring
// kD k-steps ahead (pinned by scheduling barriers).  bias_v[4 j + q]: the bias of column
// n0 + 16 j + 4 (l >> 4) + q (or null: none).
// kSwzA / kSwzOut: the activation rows A / out are 256-element rows stored with their 16-byte
// chunks XOR-swizzled by the row (chunk c of row r at chunk c ^ r, r < 16; swz16): the fragment
// reads (ds_read_b128, lane groups of 16) are then conflict-free and the 8-byte epilogue stores
// stay 2-way, where the padded 264-element pitch made every fragment read 2-way.
template <int KS, int NT, bool kSwzA = false, bool kSwzOut = false, typename WF>
__device__ __forceinline__ void wave_layer16(const bf16* A, int lda, const WF& wfrag, int n0, bf16* out, int ldo,
                                             int lane, const float* bias_v = nullptr) {
    const int r = lane & 15, g = lane >> 4;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int kD = KS < 4 ? KS : 4;
    const auto afrag = [&](int k) {
        const int col = 32 * k + 8 * g;
        return *reinterpret_cast<const bf16x8*>(A + r * lda + (kSwzA ? swz16(r, col) : col));
    };
    bf16x8 a[kD];
#pragma unroll
    for (int k = 0; k < kD; ++k) a[k] = afrag(k);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = mfma16(wfrag(j, k), a[k % kD], acc[j]);
        if (k + kD < KS) a[k % kD] = afrag(k + kD);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        bf16x4 v;
#pragma unroll
        for (int q = 0; q < 4; q += 2) {
            const f32x2 b = bias_v ? f32x2{tanh_bias(bias_v[4 * j + q]), tanh_bias(bias_v[4 * j + q + 1])}
                                   : f32x2{0.0f, 0.0f};
            const f32x2 t = tanh_pre2(f32x2{acc[j][q], acc[j][q + 1]}, b);
            v[q] = to_bf16(t.x);
            v[q + 1] = to_bf16(t.y);
        }
        const int col = n0 + 16 * j + 4 * g;
        *reinterpret_cast<bf16x4*>(out + r * ldo + (kSwzOut ? swz16(r, col) : col)) = v;
    }
}

// 4 waves (one per SIMD, so a wave may use 256 VGPRs + 256 AGPRs): wave w owns hidden
// columns kCpw*w .. kCpw*w + kCpw - 1 of both hidden layers; waves 2, 3 compute the mu head.
constexpr int kRolloutWaves = 4, kCpw = kH / kRolloutWaves, kNT = kCpw / 32;

constexpr int kW1s = kIn + 8, kW3s = kH + 8;  // LDS-resident W1 [256][72], W3 [32][264]

__global__ __launch_bounds__(64 * kRolloutWaves, 1) void k_pg_rollout(PgRolloutArgs p) {
    __shared__ __attribute__((aligned(16))) bf16 W1s[kH * kW1s];
    __shared__ __attribute__((aligned(16))) bf16 W3s[kOut * kW3s];
    __shared__ __attribute__((aligned(16))) bf16 X[kTile * kXs];
    __shared__ __attribute__((aligned(16))) bf16 H1[kTile * kHs];
    __shared__ __attribute__((aligned(16))) bf16 H2[kTile * kHs];
    __shared__ __attribute__((aligned(16))) float MU[kTile * (kOut + 1)];
    __shared__ float LS[kActPad], SIG[kActPad], ISIG[kActPad];  // log_std, exp(log_std), exp(-log_std)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t n = p.s.n;
    const int64_t i = (int64_t)blockIdx.x * kTile + lane;  // env of this lane (wave 0)
    const bool live = i < n;
    const int64_t T = p.horizon;
    if (threadIdx.x < kAct) {
        const float ls = p.params[kOffLogStd + threadIdx.x];
        LS[threadIdx.x] = ls;
        SIG[threadIdx.x] = __expf(ls);
        ISIG[threadIdx.x] = __expf(-ls);
    }
    // ---- weights, loaded once per launch: W2 slab in registers (wave w: columns 32w..),
    //      W1 and the mu head W3 in LDS
    WTile<kH / 16> w2[kNT];
#pragma unroll
    for (int j = 0; j < kNT; ++j) load_wtile(w2[j], p.wbf + kBfW2a, kHx, kCpw * wave + 32 * j, lane);
    for (int c = threadIdx.x; c < kH * (kIn / 8); c += 64 * kRolloutWaves) {
        const int row = c / (kIn / 8), col = 8 * (c % (kIn / 8));
        *reinterpret_cast<bf16x8*>(W1s + row * kW1s + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW1a + (int64_t)row * kIn + col);
    }
    for (int c = threadIdx.x; c < kOut * (kH / 8); c += 64 * kRolloutWaves) {
        const int row = c / (kH / 8), col = 8 * (c % (kH / 8));
        *reinterpret_cast<bf16x8*>(W3s + row * kW3s + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW3a + (int64_t)row * kHx + col);
    }
    const int r32 = lane & 31, h2 = lane >> 5;
    const auto w1frag = [&](int j, int k) {
        return *reinterpret_cast<const bf16x8*>(W1s + (kCpw * wave + 32 * j + r32) * kW1s + 16 * k + 8 * h2);
    };
    const auto w2frag = [&](int j, int k) { return w2[j].b[k]; };
    Env e;
    double ep_ret = 0.0;
    int32_t cnt = 0, sum_len = 0, succ = 0;
    double sum_ret = 0.0;
    uint32_t ek0 = 0, ek1 = 0, pk0 = 0, pk1 = 0;
    uint64_t rctr = 0;
    if (wave == 0) {
        // constant padding of the X tile: bias column, zeros
        for (int k = kObs; k < kIn; ++k) X[lane * kXs + k] = k == kObsIn ? (bf16)1.0f : (bf16)0.0f;
        if (live) {
            load_env(p.s, i, e);
            ep_ret = p.ep_ret[i];
            rctr = p.s.reset_ctr[i];
            env_key(p.env_seed, p.gid0 + i, ek0, ek1);
            env_key(p.policy_seed, p.gid0 + i, pk0, pk1);
        } else {
            for (int k = 0; k < kObs; ++k) X[lane * kXs + k] = (bf16)0.0f;
        }
    }
    const bool mlp = !(p.diag & 1);
    for (int64_t t = 0; t < T; ++t) {
        const int64_t m = t * n + i;
        const uint64_t ctr = p.iteration * (uint64_t)T + (uint64_t)t;
        if (wave == 0 && live)
            write_policy_obs(e, X + lane * kXs, p.obs_noise, pk0, pk1, ctr, p.obs_rm, p.obs_fm, m, T * n);
        __syncthreads();
        if (mlp) wave_layer<kIn / 16, kNT, true>(X, kXs, w1frag, kCpw * wave, nullptr, 0, H1, kHs, lane);  // b: col 45
        __syncthreads();
        if (mlp)
            wave_layer<kH / 16, kNT, true>(H1, kHs, w2frag, kCpw * wave, p.params + kOffW2a + kH, kHx, H2, kHs, lane);
        __syncthreads();
        if (mlp && wave >= kRolloutWaves - 2) {  // mu head: 32 rows per wave, 32 output columns
            const int r = lane & 31, h = lane >> 5, row0 = 32 * (wave - (kRolloutWaves - 2));
            f32x16 acc;
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
            for (int k = 0; k < kH / 16; ++k) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(H2 + (row0 + r) * kHs + 16 * k + 8 * h);
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(W3s + r * kW3s + 16 * k + 8 * h);
                acc = mfma32(a, b, acc);
            }
            const float bias = p.params[kOffW3a + (int64_t)r * kHx + kH];
#pragma unroll
            for (int q = 0; q < 16; ++q) MU[(row0 + acc_row(q, lane)) * (kOut + 1) + r] = acc[q] + bias;
        }
        __syncthreads();
        if (wave == 0 && live) {
            // a = mu + sigma * eps and log pi(a|s) accumulated in gauss_logp's exact order
            float a[kAct];
            float lp = 0.0f;
#pragma unroll
            for (int b = 0; b < (kAct + 3) / 4; ++b) {
                const u32x4 rr = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamPolicy, (uint32_t)b},
                                        pk0, pk1);
                float nz[4];
                box_muller(rr.x, rr.y, nz[0], nz[1]);
                box_muller(rr.z, rr.w, nz[2], nz[3]);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = 4 * b + q;
                    if (k >= kAct) break;
                    const float mu = mlp ? MU[lane * (kOut + 1) + k] : 0.0f;
                    a[k] = mu + SIG[k] * nz[q];
                    const float z = (a[k] - mu) * ISIG[k];
                    lp += -0.5f * z * z - LS[k] - 0.5f * kLog2Pi;
                }
            }
            p.logp[m] = lp;
            float4* arow = reinterpret_cast<float4*>(p.act + m * kActPad);
            arow[0] = float4{a[0], a[1], a[2], a[3]};
            arow[1] = float4{a[4], a[5], a[6], a[7]};
            arow[2] = float4{a[8], a[9], a[10], a[11]};
            arow[3] = float4{a[12], a[13], a[14], 0.0f};
            if (p.dyn_noise > 0.0f) {  // robustness_tests.py:180-187 (the tape keeps the policy's action)
                float dn[kAct];
                philox_normals<kAct>(dn, pk0, pk1, ctr, kStreamDyn);
#pragma unroll
                for (int k = 0; k < kAct; ++k) a[k] = clipf(a[k] + p.dyn_noise * dn[k], -1.0f, 1.0f);
            }
            if (p.applied_act) {
#pragma unroll
                for (int k = 0; k < kActPad; ++k) p.applied_act[m * kActPad + k] = k < kAct ? a[k] : 0.0f;
            }
            bool te = false, tr = false;
            double cp[4], r = 0.0;
            if (!(p.diag & 2)) r = env_step(e, a, true, p.w, p.max_episode_steps, te, tr, cp);
            ep_ret += r;
            const bool d = !(p.diag & 2) && (te || tr || e.t >= p.max_steps);
            p.rew[m] = (float)r;
            p.done[m] = d;
            if (p.ep_code)
                p.ep_code[m] = d ? (uint16_t)((e.t << 1) | (p.success_terminated && te ? 1 : 0)) : (uint16_t)0;
            if (d) {
                if (cnt < p.record_cap) {
                    const int64_t o = i * p.record_cap + cnt;
                    p.rec_return[o] = ep_ret;
                    p.rec_length[o] = e.t;
                    p.rec_success[o] = p.success_terminated ? (uint8_t)te : (uint8_t)0;
                    p.rec_end_step[o] = (int32_t)t;
                }
                ++cnt;
                sum_ret += ep_ret;
                sum_len += e.t;
                succ += te;
                env_reset_philox(e, p.s.curricula[e.cfg], ek0, ek1, rctr);
                ++rctr;
                ep_ret = 0.0;
            }
        }
    }
    if (wave == 0 && live) {
        // bootstrap observation (slot T) -- with observation noise as the policy would see it
        bf16 tmp[kObs];
        const uint64_t ctr = p.iteration * (uint64_t)T + (uint64_t)T;
        write_policy_obs(e, tmp, p.obs_noise, pk0, pk1, ctr, p.obs_rm, nullptr, T * n + i, 0);
        store_env(p.s, i, e);
        p.s.reset_ctr[i] = rctr;
        p.ep_ret[i] = ep_ret;
        p.ep_count[i] = cnt;
        p.ep_sum_ret[i] = sum_ret;
        p.ep_sum_len[i] = sum_len;
        p.ep_succ[i] = succ;
    }
}

// 16 lanes per env (k_pg_rollout_ws): envs per 256 env lanes.  (Round 5 retired the 4-wave
// lane-split kernel k_pg_rollout_ls, diag 64: k_pg_rollout_ws is its 8-wave successor and the
// one-lane k_pg_rollout and 32-env k_pg_rollout_e8 remain its bit-identity twins.)
constexpr int kLsEnvs = 16;

// ------------------------------------------------------------------ warp-specialised rollout
// k_pg_rollout_ws: the lane-split rollout -- each env spread over the 16 lanes of one DPP row
// (lane s owns joint s, lanes 0..2 the object's axis s, every lane a copy of the env's scalars)
// -- with the work that does not depend on this step's env state taken off the env lanes'
// serial chain.  A workgroup owns 16 envs with 8 waves (two per SIMD):
//   * env waves 0..3: lane (env 4w + row, s) -- observation row, sampling, dynamics, contacts,
//     termination, auto-reset;
//   * aux waves 4..7: wave 4 + w is the lane-for-lane twin of env wave w.  While the env lanes
//     step, the twin computes log pi and the act / log pi tape and settles the PREVIOUS step's
//     dense reward and episode bookkeeping (return, records, sums) from the inputs the env lanes
//     left in LDS;
//   * in the head phase, one drawing aux wave per SIMD computes the step's Philox draws for all
//     16 envs (step_draws) while the env waves run the action-independent object update;
//   * all 8 waves split the actor MLP: one 32-column tile of L1 and of L2 each (two waves per
//     SIMD, so one wave's tanh epilogue overlaps the other's MFMAs); aux wave 7 runs the mu head.
// Every value is computed by the same instruction sequence as in k_pg_rollout (same MFMA
// tiles and K order, same Philox calls, same reward ops), so the tapes are bit-identical.
// Exchanges inside an env's 16 lanes are DPP row broadcasts (an env is one DPP row).
constexpr int kWsWaves = 8, kWsThreads = 64 * kWsWaves;


// One env lane's draws, computed by its aux twin (structure of arrays over the 256 env lanes):
// the action / dynamics noise normals and the reset uniforms (at the env's exact reset counter)
// of the current step, and the observation-noise normals of the lane's obs elements
// (row_obs_elem) for the next observation row.  The step's draws are single-buffered (written in
// the head phase, read before the next head phase); the observation noise is double-buffered by
// row parity (row t + 1's is written in step t's P0 while the env lanes read row t's).  The reward inputs (WsReward) are double-buffered
// by step parity: the env lanes write step t's while the aux lanes settle step t-1's.
struct __attribute__((aligned(16))) WsDraws {
    // on: the observation noise, double-buffered by row parity, element k of env e at [e][k]
    float eps[256], dzn[256], on[2][kLsEnvs * 48];
    double u1[256], u2[256];
};
// one env lane's extra reset draw (config.py:44-113 samplers): lo + span u with a range, the
// constant (lo = cst, span = NaN: u is never NaN) without one -- structure of arrays, so the reset
// path's two reads are conflict-free 8-byte loads
struct WsSamplers {
    double lo[256], span[256];
};
struct WsReward {      // an env's dense-reward inputs and episode end of one step
    double dmin;
    uint32_t c, prev;  // contacts, previous contacts (0x100: none)
    float nacc[kF];    // per finger: sum of its negative joint positions
    int32_t len;       // episode length after the step
    int32_t done, te;
    unsigned long long rctr;  // reset counter after the step (the next step's reset draws use it)
};

// Step t of a workgroup (16 envs, 8 waves):
//   P0  env lanes write the observation row (+ its observation noise, drawn in step t-1's P0);
//       aux lanes meanwhile draw the next row's observation noise (other parity buffer) and this
//       step's dynamics noise
//   P1  all waves: L1, one 32-column tile each            (the env lanes also store the obs row)
//   P2  all waves: L2, one 32-column tile each
//   P3  env wave 3: the mu head; all env waves: the object update (env_object_step).  In their
//       shadow, one drawing aux wave per SIMD (step_draws): wave 4 step t's action noise, waves
//       5, 6, 7 the reset uniforms at each env's exact counter (step t-1's episode end is known)
//   P4  env lanes: a = mu + sigma eps, dynamics, contacts, termination, auto-reset.
//       Aux lanes: the same a, log pi (DPP row sum in action order), the act / log pi tape, then
//       settle step t-1's reward and episode bookkeeping
// kNoise: configs with fused noise (or the noise parity tapes); kDiag: diag_flags / parity tapes
// set.  The production instantiations compile out every runtime check of the other's features
// (branches and SGPRs inside the step loop: -8 % rollout time for <false, false>).
#ifndef DXRL_WS_PRIO
#define DXRL_WS_PRIO -1  // -1: by instantiation (env waves first with fused noise)
#endif
// Observation row t + 1 written at the end of step t's P4 instead of in step t + 1's P0 (no P0
// phase, no barrier for it) -- in the instantiations without fused noise only: there the rollout
// runs 1 % faster; with fused noise the aux waves' P0 draw stays and the env lanes' longer P4
// (the row's noise add) made it 7 % slower (profiles/r05/ab_ws_obs_in_p4.log)
#ifndef DXRL_WS_OBS_IN_P4
#define DXRL_WS_OBS_IN_P4 1
#endif
template <bool kNoise, bool kDiag>
__global__ __launch_bounds__(kWsThreads, 1) void k_pg_rollout_ws(PgRolloutArgs p) {
    constexpr int kRows = 32;
    // the env wave running the mu head: the env lanes idle while it runs (wave 0 instead, beside
    // the action-noise wave rather than a reset-draw wave: +-0.5 %, profiles/r05/ab_ws_head_wave_rejected.log)
    constexpr int kHeadWave = 3;
    // LDS images laid out for conflict-free 16-byte fragment reads (16-lane groups, 64 banks):
    // the read-only W1 / W3 and the observation rows padded to a 40 / 136-dword pitch, the hidden
    // rows unpadded with XOR-swizzled chunks (swz16; the padded 36 / 132-dword pitches of the
    // other rollout kernels make every fragment read 2-way)
    constexpr int kW1sW = kIn + 16, kW3sW = kH + 16, kXsW = kIn + 16, kHsW = kH;
    __shared__ __attribute__((aligned(16))) bf16 W1s[kH * kW1sW];
    __shared__ __attribute__((aligned(16))) bf16 W3s[kOut * kW3sW];
    __shared__ __attribute__((aligned(16))) bf16 X[kRows * kXsW];
    __shared__ __attribute__((aligned(16))) bf16 H1[kLsEnvs * kHsW];
    __shared__ __attribute__((aligned(16))) bf16 H2[kLsEnvs * kHsW];
    __shared__ float MU[kLsEnvs * (kOut + 1)];
    __shared__ float LS[kActPad], SIG[kActPad], ISIG[kActPad];
    __shared__ WsDraws DR;
    __shared__ WsReward RW[2][kLsEnvs];
    __shared__ WsSamplers RSMP;
    __shared__ uint32_t KEYS[kLsEnvs][4];           // per env: reset key ek0, ek1, policy key pk0, pk1
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool aux = wave >= 4;
    // waves w and w + 4 share SIMD w; with fused noise the env waves issue first (P0's aux lanes
    // run a Philox round beside the observation row): noise configs -2.2 % rollout, the others
    // +1 % (so they keep equal priorities); aux first or per-phase priorities lose 5-10 %
    // (rollout_time A/B, profiles/r04/ab_rollout_wave_priority.log)
    constexpr int kPrio = DXRL_WS_PRIO >= 0 ? DXRL_WS_PRIO : (kNoise ? 1 : 0);
    constexpr bool kObsInP4 = DXRL_WS_OBS_IN_P4 != 0 && !kNoise;
    if (kPrio != 0 && (__builtin_amdgcn_readfirstlane(wave) >= 4) == (kPrio == 2))
        __builtin_amdgcn_s_setprio(1);
    const int et_tid = tid & 255;  // the env lane this thread is (env wave) or twins (aux wave)
    const int eg = et_tid >> 4, s = et_tid & 15, gbit = 16 * (eg & 3);
    const int rbase = et_tid & ~15;
    const int64_t n = p.s.n;
    const int64_t i = (int64_t)blockIdx.x * kLsEnvs + eg;
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
    for (int c = tid; c < kH * (kIn / 8); c += kWsThreads) {
        const int row = c / (kIn / 8), col = 8 * (c % (kIn / 8));
        *reinterpret_cast<bf16x8*>(W1s + row * kW1sW + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW1a + (int64_t)row * kIn + col);
    }
    for (int c = tid; c < kOut * (kH / 8); c += kWsThreads) {
        const int row = c / (kH / 8), col = 8 * (c % (kH / 8));
        *reinterpret_cast<bf16x8*>(W3s + row * kW3sW + col) =
            *reinterpret_cast<const bf16x8*>(p.wbf + kBfW3a + (int64_t)row * kHx + col);
    }
    for (int c = tid; c < kRows * kXsW; c += kWsThreads) {
        const int row = c / kXsW, col = c % kXsW;
        X[c] = (row < kLsEnvs && col == kObsIn) ? (bf16)1.0f : (bf16)0.0f;
    }
    const int r16 = lane & 15, g16 = lane >> 4;  // 16x16x32 fragment row / k group
    const auto w1frag = [&](int j, int k) {
        return *reinterpret_cast<const bf16x8*>(W1s + (32 * wave + 16 * j + r16) * kW1sW + 32 * k + 8 * g16);
    };
    const auto w2frag = [&](int j, int k) { return w2[j][k]; };
    // step-invariant biases in registers: L2 columns 32 wave + 16 j + 4 g16 + q, head row r16
    float b2_reg[8];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            b2_reg[4 * j + q] = p.params[kOffW2a + (int64_t)(32 * wave + 16 * j + 4 * g16 + q) * kHx + kH];
    const float b3_reg = p.params[kOffW3a + (int64_t)r16 * kHx + kH];

    // ---- env-lane state (env waves) / episode bookkeeping (aux waves)
    float jp = 0.0f, jv = 0.0f;
    double opd = 0.0;
    float ovd = 0.0f;
    uint32_t flags = 0;
    int32_t et = 0, cfg = 0;
    double size = 0.0, mass = 0.0, fric = 0.0, ep_ret = 0.0, sum_ret = 0.0;
    int32_t cnt = 0, sum_len = 0, succ = 0;
    uint64_t rctr = 0;
    uint32_t ek0 = 0, ek1 = 0, pk0 = 0, pk1 = 0;
    if (live) {
        if (!aux) {
            if (s < kD) {
                jp = p.s.jp[(int64_t)s * n + i];
                jv = p.s.jv[(int64_t)s * n + i];
            }
            if (s < 3) {
                opd = p.s.op[(int64_t)s * n + i];
                ovd = p.s.ov[(int64_t)s * n + i];
            }
            flags = p.s.flags[i];
            et = p.s.t[i];
            size = p.s.size[i];
            mass = p.s.mass[i];
            fric = p.s.fric[i];
        } else {
            ep_ret = p.ep_ret[i];
        }
        cfg = p.s.cfg[i];
        rctr = p.s.reset_ctr[i];
        env_key(p.env_seed, p.gid0 + i, ek0, ek1);
        env_key(p.policy_seed, p.gid0 + i, pk0, pk1);
    }
    const int s2 = s < DXRL_RESET_EXTRA ? s : 0;
    // this lane's extra reset sampler (config.py:44-113) -- read only when an episode ends, so
    // kept in LDS rather than in registers: RSMP.lo / span[et_tid] = {lo, hi - lo} or {constant, NaN}
    double lo2 = 0.0, hi2 = 0.0, cst2 = 0.0;
    bool has2 = true, fric64 = false;
    if (live && !aux) {
        const dxrl_curriculum& cu = p.s.curricula[cfg];
        const double* rg = s2 == 0 ? cu.size_range
                                   : s2 == 1 ? cu.mass_range
                                             : s2 == 2 ? cu.friction_range
                                                       : s2 == 3 ? cu.spawn_x_range : s2 == 4 ? cu.spawn_y_range : cu.spawn_z_range;
        lo2 = rg[0];
        hi2 = rg[1];
        cst2 = s2 == 0 ? cu.object_size : s2 == 1 ? cu.object_mass : cu.friction_coefficient;
        has2 = s2 == 0 ? cu.has_size_range != 0 : s2 == 1 ? cu.has_mass_range != 0 : s2 == 2 ? cu.has_friction_range != 0 : true;
        RSMP.lo[et_tid] = has2 ? lo2 : cst2;
        RSMP.span[et_tid] = has2 ? hi2 - lo2 : __builtin_nan("");
        fric64 = cu.friction_is_f64_scalar != 0;
    }
    const int sa = s < kAct ? s : 0;
    const bool obs_noise = kNoise && p.obs_noise > 0.0f, dyn_noise = kNoise && p.dyn_noise > 0.0f;
    if (live && !aux && s == 0) {
        KEYS[eg][0] = ek0;
        KEYS[eg][1] = ek1;
        KEYS[eg][2] = pk0;
        KEYS[eg][3] = pk1;
        RW[1][eg].rctr = rctr;  // "after step -1"
    }

    // ---- aux: Philox draws.  Each block is computed once per env row and its values written
    // straight into the LDS slots of the env lanes that use them (a lane-split kernel that draws on
    // shared blocks on every lane): lanes 0..10 reset block s (slots 2s, 2s + 1: joint slots 0..14
    // -> u1 of lane k, extra slots 15..20 -> u2 of lane k - 15); lanes 11..14 action- and
    // dynamics-noise block s - 11 (normals 4(s-11) .. +3); lanes 0..11 observation-noise block s
    // (obs elements 4s .. 4s + 3).  Same blocks and arithmetic as philox_normal_at /
    // reset_uniform_at, so the values are identical.
    const auto normals4 = [&](uint64_t ctr, uint32_t stream, int blk, float nz[4]) {  // noise streams only
        noise_normals4(ctr, stream, (uint32_t)blk, pk0, pk1, nz);
    };
    // Step t's action / dynamics noise and reset uniforms, computed in the head phase by the aux
    // waves, one per SIMD (waves w and w + 4 share SIMD w; Philox's 64-bit products are
    // quarter-rate, so two drawing waves on one SIMD serialise), while the env waves run the
    // action-independent object update (env_object_step) and wave 3 the mu head: one Philox block
    // per lane, keys (KEYS) and reset counters (RW[.].rctr) of all 16 envs from LDS, values
    // written straight into the consumers' slots.
    //   wave 4 (SIMD 0)        action noise: lane -> (env lane >> 2, block lane & 3) (the
    //                          dynamics noise is drawn in P0: obs_draws)
    //   waves 5, 6, 7 (SIMD 1, 2, 3 -- 3 also runs the head on the matrix core): group lane
    //                          g < 176 reset block g % 11 of env g / 11 (u01_53 of both halves:
    //                          joint slots 0..14 -> u1, extra slots 15..20 -> u2)
    constexpr int kResetBlocks = (kReset + 1) / 2;
    const auto step_draws = [&](uint64_t ctr, int64_t t_) {
        // the lane id re-read each step (volatile): the task indices and LDS addresses derived
        // from it are then not hoisted out of the step loop, where they only raise register
        // pressure into spills (each reload a vmcnt(0))
        int lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        if (wave == 4) {
            const int e = lane >> 2, blk = lane & 3;
            if ((int64_t)blockIdx.x * kLsEnvs + e >= n) return;
            const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamPolicy, (uint32_t)blk},
                                   KEYS[e][2], KEYS[e][3]);
            float4 nz;
            box_muller(r.x, r.y, nz.x, nz.y);
            box_muller(r.z, r.w, nz.z, nz.w);
            // one 16-byte store per lane (slot 15 of the row is never read: kAct = 15); four
            // 4-byte stores at a 16-byte lane stride were 4-way bank conflicts
            *reinterpret_cast<float4*>(&DR.eps[16 * e + 4 * blk]) = nz;
            return;
        }
        if (wave < 5) return;
        const int g = 64 * (wave - 5) + lane;
        if (g >= kLsEnvs * kResetBlocks) return;
        const int e = g / kResetBlocks, blk = g % kResetBlocks;
        if ((int64_t)blockIdx.x * kLsEnvs + e >= n) return;
        const uint64_t rc = RW[(t_ - 1) & 1][e].rctr;
        const u32x4 r = philox(u32x4{(uint32_t)rc, (uint32_t)(rc >> 32), kStreamReset, (uint32_t)blk},
                               KEYS[e][0], KEYS[e][1]);
        const double ua = u01_53(r.x, r.y), ub = u01_53(r.z, r.w);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = 2 * blk + h;
            const double u = h ? ub : ua;
            if (k < kD) DR.u1[16 * e + k] = u;
            else if (k < kReset) DR.u2[16 * e + k - kD] = u;
        }
    };
    // P0 draws of the aux lanes (counter-only, so drawn where the aux waves would wait for the env
    // lanes' observation row): lanes s < 12 of env row eg the observation noise of row ctr (block
    // s) into DR.on[buf]; lanes 12..15 (dyn = true) the dynamics noise of step dctr (block s - 12,
    // normals 4 (s - 12) .. + 3) -- 64 busy lanes per aux wave, one Philox block each.
    const auto obs_draws = [&](uint64_t ctr, int buf, bool dyn = false, uint64_t dctr = 0) {
        constexpr int kOb = (kObs + 3) / 4;  // 12 observation blocks per row
        const bool is_obs = s < kOb, want = is_obs ? obs_noise : (dyn && dyn_noise);
        if (!(obs_noise || (dyn && dyn_noise))) return;
        // one Philox block per lane, the stream / counter / block selected per lane, so the wave
        // runs ONE Philox + Box-Muller sequence (lanes 12..15 branching into a second stream
        // would serialise the two)
        float nz[4];
        normals4(is_obs ? ctr : dctr, is_obs ? kStreamObs : kStreamDyn, is_obs ? s : s - kOb, nz);
        if (!want) return;
        if (!is_obs) {  // one 16-byte store (slot 15 never read), as the action noise
            *reinterpret_cast<float4*>(&DR.dzn[rbase + 4 * (s - kOb)]) = float4{nz[0], nz[1], nz[2], nz[3]};
            return;
        }
        // elements 4 s .. 4 s + 3 of the env's row (45..47 never read): one 16-byte store
        *reinterpret_cast<float4*>(&DR.on[buf][48 * eg + 4 * s]) = float4{nz[0], nz[1], nz[2], nz[3]};
        if (kDiag && p.obs_noise_tape) {  // parity tape: the value write_obs_row adds (row ctr - iteration T)
            const int64_t row = (int64_t)(ctr - p.iteration * (uint64_t)T);
            float4 v;
            v.x = 4 * s + 0 < kObs ? p.obs_noise * nz[0] : 0.0f;
            v.y = 4 * s + 1 < kObs ? p.obs_noise * nz[1] : 0.0f;
            v.z = 4 * s + 2 < kObs ? p.obs_noise * nz[2] : 0.0f;
            v.w = 4 * s + 3 < kObs ? p.obs_noise * nz[3] : 0.0f;
            *reinterpret_cast<float4*>(p.obs_noise_tape + (row * n + i) * kObsNoiseLd + 4 * s) = v;
        }
    };
    // ---- aux: the dense reward (RS:50-187) and the episode bookkeeping of a finished step
    const auto settle = [&](int64_t t_) {
        const WsReward& w = RW[t_ & 1][eg];
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
    // lane s's elements row_obs_elem(s, 0..3): joint position, joint velocity, object position /
    // identity quaternion (ME:164) / finger contact, object velocity -- the values selected
    // without divergent branches, then at most four predicated 2-byte stores (the if / else-if
    // chain compiled to a serial walk of exec-masked regions on the env waves' critical path)
    const auto write_obs_row = [&](int buf) {  // buf: the row's noise buffer (row parity)
        bf16* xr = X + eg * kXsW;
        const auto put = [&](int j, float v, int k) {
            (void)j;
            if (obs_noise) v = v + p.obs_noise * DR.on[buf][48 * eg + k];
            xr[k] = to_bf16(v);
        };
        const float v2 = s < 3 ? (float)opd : (s < 7 ? (s == 3 ? 1.0f : 0.0f) : (float)((flags >> ((s - 7) & 31)) & 1u));
        if (s < kD) {
            put(0, jp, s);
            put(1, jv, kD + s);
        }
        if (s < 7 + kF) put(2, v2, s < 7 ? 2 * kD + s : 2 * kD + 3 + s);
        if (s < 3) put(3, ovd, 2 * kD + 7 + s);
    };
    const auto tape_obs_row = [&](int64_t m) {
        *reinterpret_cast<bf16x4*>(p.obs_rm + m * kIn + 4 * s) = *reinterpret_cast<const bf16x4*>(X + eg * kXsW + 4 * s);
    };
    const bool mlp = !kDiag || !(p.diag & 1), env_on = !kDiag || !(p.diag & 2);
    // ---- env lanes, P4 of step t: action, dynamics, contacts, termination, auto-reset
    // ---- env lanes, head phase of step t: the object's velocity damping, gravity, position and
    // wall stops (ME:212-235) -- independent of the action, so off the P4 chain (the env waves
    // wait for the head and the draws here anyway)
    const auto env_object_step = [&]() {
        const double damp = 1.0 - (fric * 0.1 * 0.01);
        const float dampf = (float)damp;
        const bool op32 = (flags & kOpIsF32) != 0, fric_f64 = (flags & kFricF64) != 0;
        const int ax = s < 3 ? s : 0;
        const double gz = ax == 2 ? kGz : 0.0, lo = ax == 2 ? 0.0 : -0.2, hi = ax == 2 ? 0.3 : 0.2;
        float v = fric_f64 ? (float)((double)ovd * damp) : ovd * dampf;
        v = (float)((double)v + gz);
        const float inc = v * kDt;
        double q = op32 ? (double)((float)opd + inc) : opd + (double)inc;
        q = clipd(q, lo, hi);
        if ((q <= lo && v < 0.0f) || (q >= hi && v > 0.0f)) v = 0.0f;
        if (s < 3) {
            opd = q;
            ovd = v;
        }
        flags &= ~kOpIsF32;
    };
    const auto env_lane_step = [&](int64_t t, int64_t m) {
        const float mu = mlp ? MU[eg * (kOut + 1) + sa] : 0.0f;
        float a = mu + SIG[sa] * DR.eps[et_tid];
        if (dyn_noise)  // robustness_tests.py:180-187 (the tape keeps the policy's action)
            a = clipf(a + p.dyn_noise * DR.dzn[et_tid], -1.0f, 1.0f);
        bool te = false, tr = false;
        if (env_on) {
            // ---- env_step, lane-split (ME:198-252)
            if (s < kD) {
                const float ak = clipf(a, -1.0f, 1.0f);
                jv = kC09 * jv + kC01 * ak;
                jp = clipf(jp + jv * kDt, -1.0f, 1.0f);
            }
            // (the object's update, which does not depend on the action, ran in the head phase:
            // env_object_step)
            double op3[3];
            row_object(opd, op3);
            double dmin;
            float g3[3];
            const uint32_t c = row_contacts(jp, op3, size, s, gbit, dmin, g3);
            // the reward's inputs for the aux twin (RS:101-187)
            WsReward& rw = RW[t & 1][eg];
            float nacc = 0.0f;
#pragma unroll
            for (int j = 0; j < kJ; ++j)
                if (g3[j] < 0.0f) nacc = nacc + g3[j];
            if (finger_lane(s)) rw.nacc[s / kJ] = nacc;  // finger f on lane 3 f
            if (s == 0) {
                rw.dmin = dmin;
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
            WsReward& rw = RW[t & 1][eg];
            rw.done = d;
            rw.te = te;
            rw.len = et;
        }
        if (d) {
            // ---- env_reset_philox, lane-split: lane s holds slot s (joint) and slot 15 + s
            const double u1 = DR.u1[et_tid], u2 = DR.u2[et_tid];
            const double slo = RSMP.lo[et_tid], span = RSMP.span[et_tid];
            const double v2 = span == span ? slo + span * u2 : slo;  // config.py:44-113 samplers
            if (s < kD) {
                jp = (float)(-0.1 + (0.1 - -0.1) * u1);
                jv = 0.0f;
            }
            size = row_bcast<0>(v2);
            mass = row_bcast<1>(v2);
            fric = row_bcast<2>(v2);
            const double sx = row_bcast<3>(v2), sy = row_bcast<4>(v2), sz = row_bcast<5>(v2);
            const double spawn = s == 1 ? sy : (s == 2 ? sz : sx);
            const bool has = (flags & kHasObject) != 0;
            if (s < 3) {
                opd = (double)(float)(has ? opd : spawn);
                ovd = 0.0f;
            }
            et = 0;
            flags = kOpIsF32 | kHasObject | (fric64 ? kFricF64 : 0u);
            double op3[3];
            row_object(opd, op3);
            double dmin;
            float g3[3];
            flags |= row_contacts<false>(jp, op3, size, s, gbit, dmin, g3);  // ME:176 (no dmin)
            ++rctr;
        }
        if (s == 0) RW[t & 1][eg].rctr = rctr;
    };
    // ---- aux lanes, P4 of step t: the policy sample, log pi(a|s) (gauss_logp's order), tapes
    const auto aux_lane_step = [&](int64_t m) {
        const float mu = mlp ? MU[eg * (kOut + 1) + sa] : 0.0f;
        float a = mu + SIG[sa] * DR.eps[et_tid];
        const float z = (a - mu) * ISIG[sa];
        const float term = -0.5f * z * z - LS[sa] - 0.5f * kLog2Pi;
        float lp = 0.0f;
        row_sum_in_order<kAct>(term, lp);
        p.act[m * kActPad + s] = s < kAct ? a : 0.0f;
        if (s == 0) p.logp[m] = lp;
        if (kDiag && p.applied_act) {
            if (dyn_noise) a = clipf(a + p.dyn_noise * DR.dzn[et_tid], -1.0f, 1.0f);
            p.applied_act[m * kActPad + s] = s < kAct ? a : 0.0f;
        }
        if (kDiag && p.dyn_noise_tape)  // parity tape: the value env_lane_step adds to the action
            p.dyn_noise_tape[m * kActPad + s] = (dyn_noise && s < kAct) ? p.dyn_noise * DR.dzn[et_tid] : 0.0f;
    };

    // diag & 128: s_memtime segment stamps per step (diagnostics only): env waves into
    // stamps[16 i + k], aux waves into stamps[16 i + 8 + k]
    unsigned long long st_acc[8], st_last = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) st_acc[q] = 0;
#define WS_STAMP(k)                                                                              \
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
    if (aux && live) obs_draws(p.iteration * (uint64_t)T, 0);
    // kObsInP4: observation row t + 1 is written by the env lanes at the end of step t's P4
    // (right after the state it shows), so step t + 1 opens with layer 1 -- no P0 phase and no
    // barrier for it (row 0 here, before the first one)
    if (kObsInP4) {
        __syncthreads();  // row 0's noise (drawn just above) visible
        if (!aux && live) write_obs_row(0);
    }
    __syncthreads();
    WS_STAMP(7);
    for (int64_t t = 0; t < T; ++t) {
        const int64_t m = t * n + i;
        const uint64_t ctr = p.iteration * (uint64_t)T + (uint64_t)t;
        if (!kObsInP4 && !aux && live) write_obs_row((int)(t & 1));
        // the next observation row's noise (aux lanes, own rows; counter-only, so drawn here where
        // the aux waves wait for the env lanes' row, not in the head phase beside the draws)
        if (aux && live && (!kDiag || !(p.diag & 256))) obs_draws(ctr + 1, (int)((t + 1) & 1), true, ctr);
        WS_STAMP(0);
        if (!kObsInP4) lds_barrier();
        if (!aux && live) tape_obs_row(m);
        if (mlp) wave_layer16<kIn / 32, 2, false, true>(X, kXsW, w1frag, 32 * wave, H1, kHsW, lane);  // b: col 45
        WS_STAMP(1);
        lds_barrier();
        if (mlp) wave_layer16<kH / 32, 2, true, true>(H1, kHsW, w2frag, 32 * wave, H2, kHsW, lane, b2_reg);
        WS_STAMP(2);
        lds_barrier();
        if (!aux && live && env_on) env_object_step();
        if (mlp && wave == kHeadWave) {  // mu head: 16 env rows x head rows 0..15 (15 live)
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            // H2 rows and W3 rows (head outputs) from LDS as 16x16x32 fragments: a ring of 4
            // k-steps, refilled 4 ahead (pinned by scheduling barriers, as in wave_layer16)
            constexpr int kD = 4;
            bf16x8 ah[kD], bw[kD];
#pragma unroll
            for (int k = 0; k < kD; ++k) {
                ah[k] = *reinterpret_cast<const bf16x8*>(H2 + r16 * kHsW + swz16(r16, 32 * k + 8 * g16));
                bw[k] = *reinterpret_cast<const bf16x8*>(W3s + r16 * kW3sW + 32 * k + 8 * g16);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < kH / 32; ++k) {
                acc = mfma16(ah[k % kD], bw[k % kD], acc);
                if (k + kD < kH / 32) {
                    ah[k % kD] = *reinterpret_cast<const bf16x8*>(H2 + r16 * kHsW + swz16(r16, 32 * (k + kD) + 8 * g16));
                    bw[k % kD] = *reinterpret_cast<const bf16x8*>(W3s + r16 * kW3sW + 32 * (k + kD) + 8 * g16);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) MU[(4 * g16 + q) * (kOut + 1) + r16] = acc[q] + b3_reg;
        }
        if (!aux && mlp && p.h2_tape) {
            // the step's H2 rows (16 envs x 32 chunks of 16 bytes, chunk c of row r at c ^ r) to
            // the tape that the actor's train pass reads instead of recomputing layer 2; env lane
            // et_tid copies chunks et_tid and et_tid + 256 (wave 3 after its head)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = et_tid + 256 * u, row = q >> 5, c = q & 31;
                const int64_t ie = (int64_t)blockIdx.x * kLsEnvs + row;
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(H2 + row * kHsW + ((c ^ row) << 3));
                if (ie < n)  // non-temporal: read back once, by the actor's train pass (ab_h2_tape_nt.log)
                    __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p.h2_tape + (t * n + ie) * kH2Ld + 8 * c));
            }
        }
        if (!kDiag || !(p.diag & 256)) {
            // this step's draws (RW[(t - 1) & 1].rctr: the counters after step t-1's resets)
            if (aux) step_draws(ctr, t);
        }
        WS_STAMP(3);
        lds_barrier();
        WS_STAMP(4);
        if (live) {
            if (aux) {
                aux_lane_step(m);
                if (t > 0 && env_on && !(kDiag && (p.diag & 512))) settle(t - 1);  // step t-1's reward and bookkeeping
            } else {
                env_lane_step(t, m);
                if (kObsInP4) write_obs_row((int)((t + 1) & 1));  // row t + 1 (row T: the bootstrap)
            }
        }
        WS_STAMP(5);
        lds_barrier();  // this step's reward inputs / the next row's noise visible
        WS_STAMP(6);
    }
#undef WS_STAMP
    if (kDiag && (p.diag & 128) && s == 0 && live) {
#pragma unroll
        for (int q = 0; q < 8; ++q) p.stamps[16 * i + (aux ? 8 : 0) + q] = st_acc[q];
    }
    if (live && aux) {
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
        // bootstrap observation (slot T; with kObsInP4 already written by the last step's P4),
        // then the state back to the slab
        if (!kObsInP4 || T == 0) write_obs_row((int)(T & 1));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        tape_obs_row(T * n + i);
        if (s < kD) {
            p.s.jp[(int64_t)s * n + i] = jp;
            p.s.jv[(int64_t)s * n + i] = jv;
        }
        if (s < 3) {
            p.s.op[(int64_t)s * n + i] = opd;
            p.s.ov[(int64_t)s * n + i] = ovd;
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

// ------------------------------------------------------------------ GAE
// delta_t = r_t + gamma V_{t+1} (1 - d_t) - V_t ; A_t = delta_t + gamma lambda (1 - d_t) A_{t+1}
// One thread per env scans t = T-1 .. 0 (coalesced across envs), 64-env workgroups so the scan
// spreads over 64 CUs.  The loads of kGaeChunk steps go out together before that chunk's
// recurrence runs (one HBM latency per chunk, not per step).
//
// Normalisation moments without cancellation: each env accumulates f64 sums of (A - K) and
// (A - K)^2 about its own first value K = A_{T-1}, giving (count, mean, M2) with M2 the sum of
// squared deviations; workgroups, the block partials and the ranks then merge these triples
// with Chan et al.'s pairwise update in a fixed order (deterministic).  A plain
// sum(A^2) - mean sum(A) loses ~(mean/std)^2 ulps (2.8e-6 relative at mean/std = 4.6e4).
struct Moments {
    double n, mean, m2;
};
__device__ __forceinline__ Moments merge(Moments a, Moments b) {
    const double n = a.n + b.n;
    if (b.n == 0.0) return a;
    if (a.n == 0.0) return b;
    const double d = b.mean - a.mean;
    return Moments{n, a.mean + d * (b.n / n), a.m2 + b.m2 + d * d * (a.n * b.n / n)};
}
// workgroup tree merge in LDS (fixed pairing), result in red[0]
template <int NT>
__device__ void block_merge(Moments v, Moments* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] = merge(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
}

constexpr int kGaeChunk = 32, kGaeThreads = 64;
__global__ __launch_bounds__(kGaeThreads) void k_gae(const float* __restrict__ rew, const uint8_t* __restrict__ done,
                                                     const float* __restrict__ V, int64_t n, int64_t T, float gamma,
                                                     float lam, float* __restrict__ adv, float* __restrict__ ret,
                                                     Moments* __restrict__ partial) {
    __shared__ Moments red[kGaeThreads];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ic = i < n ? i : n - 1;  // clamped: every lane loads, only real envs store
    double s = 0.0, s2 = 0.0, K = 0.0;
    float next_adv = 0.0f;
    float next_v = V[T * n + ic];
    for (int64_t hi = T; hi > 0; hi -= kGaeChunk) {
        const int64_t lo = hi - kGaeChunk > 0 ? hi - kGaeChunk : 0;
        float rv[kGaeChunk], vv[kGaeChunk];
        uint8_t dv[kGaeChunk];
#pragma unroll
        for (int k = 0; k < kGaeChunk; ++k) {
            const int64_t t = lo + k < hi ? lo + k : hi - 1;
            const int64_t m = t * n + ic;
            rv[k] = rew[m];
            vv[k] = V[m];
            dv[k] = done[m];
        }
#pragma unroll
        for (int k = kGaeChunk - 1; k >= 0; --k) {
            if (lo + k >= hi) continue;
            const float nd = dv[k] ? 0.0f : 1.0f;
            const float delta = rv[k] + gamma * next_v * nd - vv[k];
            const float a = delta + gamma * lam * nd * next_adv;
            const int64_t m = (lo + k) * n + ic;
            if (lo + k == T - 1) K = (double)a;
            if (i < n) {
                adv[m] = a;
                ret[m] = a + vv[k];
                const double d = (double)a - K;
                s += d;
                s2 += d * d;
            }
            next_adv = a;
            next_v = vv[k];
        }
    }
    Moments mo{0.0, 0.0, 0.0};
    if (i < n) {
        const double c = (double)T;
        mo = Moments{c, K + s / c, fmax(s2 - s * (s / c), 0.0)};
    }
    block_merge<kGaeThreads>(mo, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// k_gae_lds: the same per-env recurrence (k_gae's expressions), with everything but the
// recurrence itself taken off the serial chain and the recurrence itself a 16-lane wavefront
// prefix per env (round 6, step 2 below).  A 256-thread workgroup owns 16 envs:
//   1. all 256 threads load the envs' whole horizon (rew, V_t, V_{t+1}, done; batches of
//      independent loads) and write delta_t = r_t + gamma V_{t+1} (1 - d_t) - V_t and the chain
//      coefficient c_t = (gamma lambda)(1 - d_t) (selected from the done byte) into env-major LDS
//      rows, zero-padded to a multiple of 8 steps;
//   2. A_t = delta_t + c_t A_{t+1} down the rows as a segmented scan (16 lanes per env, below);
//   3. all 256 threads write adv / ret back coalesced and accumulate the moments.
// The padded steps run first, on zeros: A stays +0, which the chain starts from anyway.
// Round 5: the chain read its operands as 16 scalar loads (delta, done byte) per 8 steps from
// time-major rows and selected c_t on it: 11.7 of the phase's 23.7 us (DXRL_GAE_DIAG ablation,
// profiles/r05/ab_gae_phases.log).
// k_gae (64 single-wave workgroups, the whole step on the chain, a memory latency per 32-step
// chunk) remains for horizons whose staging exceeds the LDS.
#ifndef DXRL_GAE_XCD
#define DXRL_GAE_XCD 1
#endif
// ablation bits for phase timing (A/B builds only; results are wrong when set): 1 no recurrence,
// 2 no moments / merge, 4 no stores of adv / ret
#ifndef DXRL_GAE_DIAG
#define DXRL_GAE_DIAG 0
#endif
constexpr int kGlEnvs = 16, kGlThreads = 256;
// Workgroups are dispatched to the 8 XCDs round robin (block b on XCD b % 8): env group g of
// block b chosen so each XCD owns one contiguous run of groups, and the 64-byte row pieces of
// neighbouring groups (one 128-byte line) are fetched into one L2, not two.  A permutation of
// the groups for any dispatch order; partial[] stays indexed by group, so every sum is unchanged.
__device__ __forceinline__ int64_t xcd_contiguous(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, j = b / 8;
    return x * q + (x < rem ? x : rem) + j;
}
// env-major row pitch (floats) of the delta / coefficient rows: the horizon padded to 8 steps,
// + 4 so the 16 lanes' 16-byte reads start on distinct bank quads (T = 200: pitch 204)
__host__ __device__ constexpr int64_t gae_pitch(int64_t T) { return (T + 7) / 8 * 8 + 4; }
// delta, coefficient and advantage rows [16][pitch] (env-major), V_t [T][16]
__host__ __device__ constexpr int64_t gae_lds_bytes(int64_t T) { return kGlEnvs * (12 * gae_pitch(T) + 4 * T); }
__global__ __launch_bounds__(kGlThreads) void k_gae_lds(const float* __restrict__ rew,
                                                        const uint8_t* __restrict__ done, const float* __restrict__ V,
                                                        int64_t n, int T, float gamma, float lam,
                                                        float* __restrict__ adv, float* __restrict__ ret,
                                                        Moments* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) float gl_lds[];
    const int P = (int)gae_pitch(T), T8 = (T + 7) / 8 * 8;
    float* Le = gl_lds;                            // [16][P] delta_t (env-major, zero past T)
    float* Ce = Le + kGlEnvs * P;                  // [16][P] c_t
    float* Vs = Ce + kGlEnvs * P;                  // [T][16] V_t (for ret)
    float* Ae = Vs + (int64_t)T * kGlEnvs;         // [16][P] A_t (env-major; the padded steps' A past T)
    __shared__ Moments red[kGlThreads];
    const int tid = threadIdx.x;
    const int64_t grp = DXRL_GAE_XCD ? xcd_contiguous(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t e0 = grp * kGlEnvs;
    const int64_t cnt = (int64_t)T * kGlEnvs;
    const float gl = gamma * lam;
    // 1. batches of kGlBatch elements per thread, every load issued before any lands
    constexpr int kGlBatch = 16;
    for (int64_t q0 = 0; q0 < cnt; q0 += (int64_t)kGlBatch * kGlThreads) {
        float rv[kGlBatch], v0[kGlBatch], v1[kGlBatch];
        uint8_t dv[kGlBatch];
#pragma unroll
        for (int u = 0; u < kGlBatch; ++u) {
            const int64_t q = q0 + (int64_t)u * kGlThreads + tid;
            const int64_t qc = q < cnt ? q : cnt - 1;
            const int64_t t = qc / kGlEnvs, e = qc % kGlEnvs;
            const int64_t ic = e0 + e < n ? e0 + e : n - 1;
            rv[u] = rew[t * n + ic];
            v0[u] = V[t * n + ic];
            v1[u] = V[(t + 1) * n + ic];
            dv[u] = done[t * n + ic];
        }
#pragma unroll
        for (int u = 0; u < kGlBatch; ++u) {
            const int64_t q = q0 + (int64_t)u * kGlThreads + tid;
            if (q < cnt) {
                const int t = (int)(q / kGlEnvs), e = (int)(q % kGlEnvs);
                const float nd = dv[u] ? 0.0f : 1.0f;
                Le[e * P + t] = rv[u] + gamma * v1[u] * nd - v0[u];
                Ce[e * P + t] = dv[u] ? 0.0f : gl;  // (gamma lambda) (1 - d_t), exactly
                Vs[q] = v0[u];
            }
        }
    }
    for (int k = tid; k < kGlEnvs * (T8 - T); k += kGlThreads) {  // padded steps: zeros
        const int e = k / (T8 - T), t = T + k % (T8 - T);
        Le[e * P + t] = 0.0f;
        Ce[e * P + t] = 0.0f;
    }
    __syncthreads();
    // 2. the recurrence A_t = delta_t + c_t A_{t+1} as a wavefront prefix: 16 lanes per env (one
    //    wave holds 4 envs), lane s owns the 8-step chunks [s nc / 16, (s + 1) nc / 16) of its env's
    //    nc = T8 / 8 chunks.  (a) each lane composes its segment into the affine map A_start =
    //    D + C A_in (D = the segment's recurrence from A_in = 0, C = the product of its c_t); (b) a
    //    Hillis-Steele suffix scan over the 16 lanes (offsets 1, 2, 4, 8: map_s <- map_s o map_{s+off})
    //    gives each lane A at the start of its segment, and lane s + 1's value is lane s's A_in;
    //    (c) each lane reruns its segment's recurrence from A_in, storing A_t.  The chain is
    //    2 (nc / 16) chunks + 4 scan steps long instead of nc chunks; inside a segment every A_t is
    //    the sequential expression, the segment boundaries' A_in carry the composition's rounding
    //    (pg_reference.gae restates this exact order).  Against one lane per env running the
    //    whole chain (round 5): advantages phase 16.0-16.7 -> 13.1-14.0 us
    //    (profiles/r06/ab_gae_scan.log).
    if (!(DXRL_GAE_DIAG & 1)) {
        const int e = tid >> 4, sg = tid & 15;
        const int nc = T8 / 8, c_lo = sg * nc / 16, c_hi = (sg + 1) * nc / 16;
        const float4* L4 = reinterpret_cast<const float4*>(Le + e * P);
        const float4* C4 = reinterpret_cast<const float4*>(Ce + e * P);
        float D = 0.0f, C = 1.0f;
        for (int k = c_hi - 1; k >= c_lo; --k) {
            const float4 l0 = L4[2 * k], l1 = L4[2 * k + 1], q0 = C4[2 * k], q1 = C4[2 * k + 1];
            const float lq[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
            const float cq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
            for (int j = 7; j >= 0; --j) {
                D = lq[j] + cq[j] * D;
                C = cq[j] * C;
            }
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const float Dn = __shfl_down(D, off, 16), Cn = __shfl_down(C, off, 16);
            if (sg + off < 16) {
                D = D + C * Dn;
                C = C * Cn;
            }
        }
        const float Dnext = __shfl_down(D, 1, 16);
        float next_adv = sg == 15 ? 0.0f : Dnext;
        for (int k = c_hi - 1; k >= c_lo; --k) {
            const float4 l0 = L4[2 * k], l1 = L4[2 * k + 1], q0 = C4[2 * k], q1 = C4[2 * k + 1];
            const float lq[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
            const float cq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
            float aq[8];
#pragma unroll
            for (int j = 7; j >= 0; --j) {
                aq[j] = lq[j] + cq[j] * next_adv;
                next_adv = aq[j];
            }
            float4* A4 = reinterpret_cast<float4*>(Ae + e * P + 8 * k);
            A4[0] = make_float4(aq[0], aq[1], aq[2], aq[3]);
            A4[1] = make_float4(aq[4], aq[5], aq[6], aq[7]);
        }
    }
    __syncthreads();
    // 3. store, and the moments of this thread's elements about its first one (merged with Chan's
    // update below and across workgroups: any shift point gives the same moments up to rounding)
    double s = 0.0, s2 = 0.0, K = 0.0, c = 0.0;
    for (int64_t q = tid; q < cnt; q += kGlThreads) {
        const int64_t t = q / kGlEnvs, e = q % kGlEnvs;
        if (e0 + e < n) {
            const float a = Ae[e * P + t];
            if (!(DXRL_GAE_DIAG & 4)) {
                adv[t * n + e0 + e] = a;
                ret[t * n + e0 + e] = a + Vs[q];
            }
            if (DXRL_GAE_DIAG & 2) continue;
            if (c == 0.0) K = (double)a;
            const double d = (double)a - K;
            s += d;
            s2 += d * d;
            c += 1.0;
        }
    }
    const Moments mo = c > 0.0 ? Moments{c, K + s / c, fmax(s2 - s * (s / c), 0.0)} : Moments{0.0, 0.0, 0.0};
    if (DXRL_GAE_DIAG & 2) {
        if (tid == 0) partial[grp] = mo;
        return;
    }
    block_merge<kGlThreads>(mo, red);
    if (tid == 0) partial[grp] = red[0];
}

// Local moments of the rank, contiguous so ranks exchange them as one 3-element block:
// stats[5] = count, stats[6] = mean, stats[7] = M2 (sum of squared deviations).
__global__ void k_gae_sums(const Moments* __restrict__ partial, int nb, double* __restrict__ stats) {
    __shared__ Moments red[256];
    Moments a{0.0, 0.0, 0.0};
    for (int k = threadIdx.x; k < nb; k += blockDim.x) a = merge(a, partial[k]);
    block_merge<256>(a, red);
    if (threadIdx.x == 0) {
        const Moments m = red[0];
        stats[5] = m.n;
        stats[6] = m.mean;
        stats[7] = m.m2;
        // the single-rank statistics as well (== dxrl_pg_adv_combine(stats + 5, world = 1), which
        // a multi-rank caller runs afterwards over the all-gathered triples, overwriting these)
        const Moments a1 = merge(Moments{0.0, 0.0, 0.0}, m);
        stats[0] = a1.n;
        stats[1] = a1.n * a1.mean;
        stats[2] = a1.mean;
        stats[3] = a1.m2;
        stats[4] = sqrt(a1.m2 / (a1.n > 1.0 ? a1.n - 1.0 : 1.0));
    }
}

// Global statistics from the ranks' (count, mean, M2) triples, merged in rank order:
// stats[0] count, [1] sum, [2] mean, [3] sum of squared deviations, [4] unbiased std
__global__ void k_stats_combine(const double* __restrict__ moments, int world, double* stats) {
    Moments a{0.0, 0.0, 0.0};
    for (int r = 0; r < world; ++r) a = merge(a, Moments{moments[3 * r], moments[3 * r + 1], moments[3 * r + 2]});
    stats[0] = a.n;
    stats[1] = a.n * a.mean;
    stats[2] = a.mean;
    stats[3] = a.m2;
    stats[4] = sqrt(a.m2 / (a.n > 1.0 ? a.n - 1.0 : 1.0));
}

// out[slot] = sum(partials) (fixed order)
// Sum of nb partials by a 256-thread block in one fixed order: thread-strided sums, a butterfly
// inside each wave (lane pairs add the same two values, so every lane holds the same bits), then
// the four wave sums in wave order.  k_sum_partials and every k_adam_pack workgroup use it, so the
// two optimiser paths clip with bit-identical norms.
__device__ __forceinline__ double block_sum256(double s, double* red4) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = s;
    __syncthreads();
    return ((red4[0] + red4[1]) + red4[2]) + red4[3];
}
// (thread t adds partial[t], partial[t + 256], ... in that order; the loads go out in batches of 8
// ahead of their adds -- one L2 latency per batch, not per partial, for the ~2.6 k partials of
// dxrl_pg_fused_pair_gnorm -- and the + 0.0 of a batch's tail leaves the sum's bits unchanged)
__device__ __forceinline__ double block_sum_partials(const double* __restrict__ partial, int nb, double* red4) {
    constexpr int kB = 8;
    double s = 0.0;
    for (int k0 = threadIdx.x; k0 < nb; k0 += 256 * kB) {
        double v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) v[u] = k0 + 256 * u < nb ? partial[k0 + 256 * u] : 0.0;
#pragma unroll
        for (int u = 0; u < kB; ++u) s += v[u];
    }
    return block_sum256(s, red4);
}

__global__ __launch_bounds__(256) void k_sum_partials(const double* __restrict__ partial, int nb,
                                                      double* __restrict__ out, int slot) {
    __shared__ double red4[4];
    const double s = block_sum_partials(partial, nb, red4);
    if (threadIdx.x == 0) out[slot] = s;
}


// ------------------------------------------------------------------ PPO heads
struct HeadArgs {
    const float* mu;       // [M][kOut] f32 (actor head)
    const float* V;        // [M] f32 (critic head row 0, feature-major)
    const float* act;      // [M][kActPad]
    const float* logp_old; // [M]
    const float* adv;      // [M]
    const float* ret;      // [M]
    const double* stats;   // normalisation stats
    const float* params;   // log_std
    int64_t M;
    double inv_total;      // 1 / global sample count (mean over all ranks)
    float clip_eps, vf_coef;
    bf16* dmu_rm;          // [M][kOut]
    bf16* dmu_fm;          // [kOut][M]
    bf16* dv_rm;           // [M][kOut] (col 0)
    bf16* dv_fm;           // [kOut][M] (row 0)
    float* dlogstd_partial;// [blocks][kActPad]
    double* loss_partial;  // [blocks][4]: policy loss, value loss, clip fraction, approx kl
};

__global__ __launch_bounds__(256) void k_ppo_heads(HeadArgs h) {
    __shared__ float red[256][kActPad];
    __shared__ double lred[256][4];
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float dls[kAct];
#pragma unroll
    for (int k = 0; k < kAct; ++k) dls[k] = 0.0f;
    double lp_loss = 0.0, lv = 0.0, clipped = 0.0, kl = 0.0;
    if (m < h.M) {
        float ls[kAct], mu[kAct], a[kAct];
#pragma unroll
        for (int k = 0; k < kAct; ++k) {
            ls[k] = h.params[kOffLogStd + k];
            mu[k] = h.mu[m * kOut + k];
            a[k] = h.act[m * kActPad + k];
        }
        const float lp = gauss_logp(a, mu, ls);
        const float ratio = __expf(lp - h.logp_old[m]);
        const float A = (float)(((double)h.adv[m] - h.stats[2]) / (h.stats[4] + 1e-8));
        const float s1 = ratio * A;
        const float rc = fminf(fmaxf(ratio, 1.0f - h.clip_eps), 1.0f + h.clip_eps);
        const float s2 = rc * A;
        // d(-min(s1, s2))/d logp
        float g = 0.0f;
        if (s1 <= s2) g = -A * ratio;
        else if (ratio == rc) g = -A * ratio;
        const float sc = (float)h.inv_total;
        g *= sc;
#pragma unroll
        for (int k = 0; k < kAct; ++k) {
            const float iv = __expf(-2.0f * ls[k]);
            const float d = a[k] - mu[k];
            const float dmu = g * d * iv;              // dlogp/dmu = (a - mu) / sigma^2
            dls[k] = g * (d * d * iv - 1.0f);          // dlogp/dlogstd = (a-mu)^2/sigma^2 - 1
            h.dmu_rm[m * kOut + k] = to_bf16(dmu);
            if (h.dmu_fm) h.dmu_fm[(int64_t)k * h.M + m] = to_bf16(dmu);
        }
        const float v = h.V[m];
        const float dv = 2.0f * h.vf_coef * (v - h.ret[m]) * sc;
        h.dv_rm[m * kOut] = to_bf16(dv);
        if (h.dv_fm) h.dv_fm[m] = to_bf16(dv);
        lp_loss = -(double)fminf(s1, s2);
        lv = (double)(v - h.ret[m]) * (double)(v - h.ret[m]);
        clipped = fabsf(ratio - 1.0f) > h.clip_eps ? 1.0 : 0.0;
        kl = (double)(h.logp_old[m] - lp);
    }
#pragma unroll
    for (int k = 0; k < kAct; ++k) red[threadIdx.x][k] = dls[k];
    lred[threadIdx.x][0] = lp_loss;
    lred[threadIdx.x][1] = lv;
    lred[threadIdx.x][2] = clipped;
    lred[threadIdx.x][3] = kl;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
#pragma unroll
            for (int k = 0; k < kAct; ++k) red[threadIdx.x][k] += red[threadIdx.x + w][k];
#pragma unroll
            for (int k = 0; k < 4; ++k) lred[threadIdx.x][k] += lred[threadIdx.x + w][k];
        }
        __syncthreads();
    }
    if (threadIdx.x < kActPad)
        h.dlogstd_partial[(int64_t)blockIdx.x * kActPad + threadIdx.x] = threadIdx.x < kAct ? red[0][threadIdx.x] : 0.0f;
    if (threadIdx.x < 4) h.loss_partial[(int64_t)blockIdx.x * 4 + threadIdx.x] = lred[0][threadIdx.x];
}

// grads[kOffLogStd + k] = sum_b partial[b][k] - ent_coef  (entropy bonus: d(-c H)/d logstd = -c)
__global__ __launch_bounds__(256) void k_logstd_grad(const float* __restrict__ partial, int nb, float ent_coef,
                                                     float* __restrict__ grads) {
    __shared__ float red[256][kActPad + 1];
    float s[kActPad];
#pragma unroll
    for (int k = 0; k < kActPad; ++k) s[k] = 0.0f;
    for (int b = threadIdx.x; b < nb; b += 256) {  // fixed partition + fixed tree: deterministic
#pragma unroll
        for (int k = 0; k < kActPad; ++k) s[k] += partial[(int64_t)b * kActPad + k];
    }
#pragma unroll
    for (int k = 0; k < kActPad; ++k) red[threadIdx.x][k] = s[k];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
#pragma unroll
            for (int k = 0; k < kActPad; ++k) red[threadIdx.x][k] += red[threadIdx.x + w][k];
        __syncthreads();
    }
    const int k = threadIdx.x;
    if (k < kActPad) grads[kOffLogStd + k] = k < kAct ? red[0][k] - ent_coef : 0.0f;
}

// ------------------------------------------------------------------ optimiser
// grad-norm^2 partials, then Adam with global-norm clipping (scale on device)
__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ x, int64_t n, double* __restrict__ partial) {
    __shared__ double red4[4];
    double s = 0.0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        s += (double)x[k] * (double)x[k];
    s = block_sum256(s, red4);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m1,
                       float* __restrict__ m2, int64_t n, float lr, float b1, float b2, float eps, float bc1,
                       float bc2, const double* __restrict__ gnorm2, float max_norm) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    float scale = 1.0f;
    if (max_norm > 0.0f) {
        const float nrm = (float)sqrt(gnorm2[0]);
        scale = nrm > max_norm ? max_norm / (nrm + 1e-6f) : 1.0f;
    }
    const float gk = g[k] * scale;
    const float a = b1 * m1[k] + (1.0f - b1) * gk;
    const float b = b2 * m2[k] + (1.0f - b2) * gk * gk;
    m1[k] = a;
    m2[k] = b;
    p[k] -= lr * (a / bc1) / (sqrtf(b / bc2) + eps);
}

// f32 master -> bf16 forward weights + transposed copies for input gradients: work item k of the
// pack, reading master element j as p(j)
template <typename Src>
__device__ __forceinline__ void pack_item(int64_t k, const Src& p, bf16* __restrict__ w) {
    // forward copies (same layout as the master blocks)
    if (k < kW1) {
        w[kBfW1a + k] = to_bf16(p(kOffW1a + k));
        w[kBfW1c + k] = to_bf16(p(kOffW1c + k));
    }
    if (k < kW2) {
        w[kBfW2a + k] = to_bf16(p(kOffW2a + k));
        w[kBfW2c + k] = to_bf16(p(kOffW2c + k));
    }
    if (k < kW3) {
        w[kBfW3a + k] = to_bf16(p(kOffW3a + k));
        w[kBfW3c + k] = to_bf16(p(kOffW3c + k));
    }
    if (k < kW2T) {  // W2T[i][o] = W2[o][i]
        const int64_t i = k / kH, o = k % kH;
        w[kBfW2aT + k] = to_bf16(p(kOffW2a + o * kHx + i));
        w[kBfW2cT + k] = to_bf16(p(kOffW2c + o * kHx + i));
    }
    if (k < kW3T) {  // W3T[i][o] = W3[o][i]
        const int64_t i = k / kOut, o = k % kOut;
        w[kBfW3aT + k] = to_bf16(p(kOffW3a + o * kHx + i));
        w[kBfW3cT + k] = to_bf16(p(kOffW3c + o * kHx + i));
    }
    // fragment-ordered copies (dxrl_pg.h): element k of a [N][K] matrix's fragment stream
    const auto frag_rc = [](int64_t k, int K, int64_t& row, int64_t& col) {
        const int e = (int)(k & 7), lane = (int)((k >> 3) & 63);
        const int64_t fk = k >> 9, ks = K / 16, ft = fk / ks, kk = fk % ks;
        row = 32 * ft + (lane & 31);
        col = 16 * kk + 8 * (lane >> 5) + e;
    };
#pragma unroll
    for (int net = 0; net < 2; ++net) {
        const int64_t o1 = net ? kOffW1c : kOffW1a, o2 = net ? kOffW2c : kOffW2a, o3 = net ? kOffW3c : kOffW3a;
        bf16* f = w + kFr + net * kFrNet;
        int64_t row, col;
        if (k < kFrW1) {
            frag_rc(k, kIn, row, col);
            f[kFrOffW1 + k] = to_bf16(p(o1 + row * kIn + col));
        }
        if (k < kFrW2) {
            frag_rc(k, kH, row, col);
            f[kFrOffW2 + k] = to_bf16(p(o2 + row * kHx + col));
            f[kFrOffW2T + k] = to_bf16(p(o2 + col * kHx + row));  // W2T[row][col] = W2[col][row]
        }
        if (k < kFrW3) {
            frag_rc(k, kH, row, col);
            f[kFrOffW3 + k] = to_bf16(p(o3 + row * kHx + col));
        }
        if (k < kFrW3T) {
            frag_rc(k, kOut, row, col);
            f[kFrOffW3T + k] = to_bf16(p(o3 + col * kHx + row));  // W3T[row][col] = W3[col][row]
        }
    }
}

__global__ void k_pack_weights(const float* __restrict__ p, bf16* __restrict__ w) {
    pack_item((int64_t)blockIdx.x * blockDim.x + threadIdx.x, [p](int64_t j) { return p[j]; }, w);
}

// Position of element (row, col) of a [N][K] matrix in its fragment stream (the inverse of
// pack_item's frag_rc: 64-lane x 8-element fragments, 32 rows x 16 columns each, k-steps inner)
__device__ __forceinline__ int64_t frag_index(int row, int col, int K) {
    const int lane = (row & 31) + 32 * ((col >> 3) & 1);
    return ((int64_t)((row >> 5) * (K / 16) + (col >> 4)) << 9) + lane * 8 + (col & 7);
}

// Every packed bf16 copy of master element j (value v): the scatter form of pack_item's gathers --
// the forward copy, the transposed copy and the fragment streams of W1 / W2 / W3 (log σ and the
// pad slots between the nets are master-only)
__device__ __forceinline__ void pack_scatter(int64_t j, float v, bf16* __restrict__ w) {
    const bf16 b = to_bf16(v);
    const bool c = j >= kOffW1c;
    const int64_t r = j - (c ? kOffW1c : kOffW1a);
    bf16* f = w + kFr + (c ? kFrNet : 0);
    if (r < 0) return;
    if (r < kW1) {  // W1 [kH][kIn]
        const int row = (int)(r / kIn), col = (int)(r % kIn);
        w[(c ? kBfW1c : kBfW1a) + r] = b;
        f[kFrOffW1 + frag_index(row, col, kIn)] = b;
    } else if (r < kW1 + kW2) {  // W2 [kH][kHx], column kH = bias
        const int64_t q = r - kW1;
        const int row = (int)(q / kHx), col = (int)(q % kHx);
        w[(c ? kBfW2c : kBfW2a) + q] = b;
        if (col < kH) {
            w[(c ? kBfW2cT : kBfW2aT) + (int64_t)col * kH + row] = b;
            f[kFrOffW2 + frag_index(row, col, kH)] = b;
            f[kFrOffW2T + frag_index(col, row, kH)] = b;
        }
    } else if (r < kW1 + kW2 + kW3) {  // W3 [kOut][kHx]
        const int64_t q = r - kW1 - kW2;
        const int row = (int)(q / kHx), col = (int)(q % kHx);
        w[(c ? kBfW3c : kBfW3a) + q] = b;
        if (col < kH) {
            w[(c ? kBfW3cT : kBfW3aT) + (int64_t)col * kOut + row] = b;
            f[kFrOffW3 + frag_index(row, col, kH)] = b;
            f[kFrOffW3T + frag_index(col, row, kOut)] = b;
        }
    }
}

// One optimiser launch after k_sumsq: every workgroup sums the grad-norm partials in
// k_sum_partials' order (so the clip scale is bit for bit k_adam's); thread j applies Adam to
// master element j (k_adam's expression, once) and scatters the updated value into every packed
// bf16 copy (pack_scatter).  The updated master goes to a second buffer (the trainer swaps the
// pair).  The gather form (k_pack_weights / pack_item, which recomputed the update of every
// element it packed: up to 20 updates per thread) took 13.3 us per step.
struct AdamPackArgs {
    const float *p, *g, *m1, *m2;
    float *po, *m1o, *m2o;
    int64_t n;
    float lr, b1, b2, eps, bc1, bc2, max_norm;
    const double* partial;
    int nb;
    double* gnorm2;
    bf16* w;
};

__global__ __launch_bounds__(256) void k_adam_pack(AdamPackArgs a) {
    __shared__ double red4[4];
    const double g2 = block_sum_partials(a.partial, a.nb, red4);
    if (blockIdx.x == 0 && threadIdx.x == 0) a.gnorm2[0] = g2;
    float scale = 1.0f;
    if (a.max_norm > 0.0f) {
        const float nrm = (float)sqrt(g2);
        scale = nrm > a.max_norm ? a.max_norm / (nrm + 1e-6f) : 1.0f;
    }
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const float gk = a.g[j] * scale;
    const float m = a.b1 * a.m1[j] + (1.0f - a.b1) * gk;
    const float v = a.b2 * a.m2[j] + (1.0f - a.b2) * gk * gk;
    const float pn = a.p[j] - a.lr * (m / a.bc1) / (sqrtf(v / a.bc2) + a.eps);
    a.po[j] = pn;
    a.m1o[j] = m;
    a.m2o[j] = v;
    pack_scatter(j, pn, a.w);
}

static int reduce_to(const double* partial, int nb, double* out, int slot, hipStream_t st) {
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(256), 0, st, partial, nb, out, slot);
    return launch_check("k_sum_partials");
}

}  // namespace dxrl

// =========================================================================== C ABI
extern "C" {

int dxrl_pg_sizes(int64_t* params, int64_t* packed_bf16) {
    DXRL_REQUIRE(params && packed_bf16, "null outputs");
    *params = kParams;
    *packed_bf16 = kBf;
    return DXRL_OK;
}

int dxrl_pg_pack_weights(int32_t device, const float* params, void* packed, void* stream) {
    DXRL_REQUIRE(params && packed, "null params/packed");
    DeviceGuard g(device);
    const int64_t n = kW2 > kW2T ? kW2 : kW2T;  // largest block
    hipLaunchKernelGGL(k_pack_weights, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), params,
                       static_cast<bf16*>(packed));
    return launch_check("k_pack_weights");
}

}  // extern "C"
namespace dxrl {
namespace {
// The rollout kernel dxrl_pg_rollout launches for n envs: 0 the 64-env reference kernel (feature-
// major tape / diag 16), 1 the 16-env kernel, 2 the 32-env kernel (>= 32 envs per CU: one round
// where the 16-env kernel would need two; diag 1024 / 2048 force it / the 16-env kernel).
int rollout_kernel(int64_t n, int32_t diag_flags, bool obs_fm) {
    if (obs_fm || (diag_flags & 16)) return 0;
    static const int cus = [] {
        int dev = 0, c = 0;
        (void)hipGetDevice(&dev);
        return hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0 ? c : 256;
    }();
    const bool e8 = !(diag_flags & 2048) && ((diag_flags & 1024) || n >= (int64_t)kE8Envs * cus);
    return e8 ? 2 : 1;
}
}  // namespace
}  // namespace dxrl
extern "C" {

int dxrl_pg_rollout_kernel(const dxrl_env* env, int32_t diag_flags, int32_t* kernel) {
    DXRL_REQUIRE(env && kernel, "null argument");
    DeviceGuard g(env->device);
    *kernel = rollout_kernel(env->cfg.num_envs, diag_flags, false);
    return DXRL_OK;
}

int dxrl_pg_rollout(dxrl_env* env, const void* packed, const float* params, const dxrl_pg_rollout_args* a,
                    void* stream) {
    DXRL_REQUIRE(env && packed && params && a, "null argument");
    DXRL_REQUIRE(a->horizon > 0 && a->max_steps > 0, "horizon and max_steps must be > 0");
    DXRL_REQUIRE(a->obs_rm && a->act && a->logp && a->rew && a->done && a->ep_return && a->ep_count &&
                     a->ep_sum_return && a->ep_sum_length && a->ep_successes,
                 "null tape / episode buffer");
    DXRL_REQUIRE(env->cfg.reward_type == DXRL_REWARD_DENSE, "the policy-gradient rollout uses the dense reward");
    DXRL_REQUIRE(a->record_cap == 0 || (a->rec_return && a->rec_length && a->rec_success && a->rec_end_step),
                 "record_cap > 0 needs all four record buffers");
    DXRL_REQUIRE(!a->ep_code || (a->max_steps < 16384 && env->cfg.max_episode_steps < 16383),
                 "ep_code holds episode lengths below 2^14: max_steps / max_episode_steps too large");
    PgRolloutArgs p{env->soa,
                    weights_of(env->cfg),
                    env->cfg.max_episode_steps,
                    a->max_steps,
                    a->horizon,
                    static_cast<const bf16*>(packed),
                    params,
                    env->cfg.seed,
                    a->policy_seed,
                    env->cfg.global_env_offset,
                    a->iteration,
                    (float)a->obs_noise_std,
                    (float)a->dyn_noise_std,
                    static_cast<bf16*>(a->obs_rm),
                    static_cast<bf16*>(a->obs_fm),
                    a->act,
                    a->logp,
                    a->rew,
                    a->done,
                    a->ep_return,
                    a->ep_count,
                    a->ep_sum_return,
                    a->ep_sum_length,
                    a->ep_successes,
                    a->diag_flags,
                    a->success_rule == DXRL_SUCCESS_TERMINATED,
                    a->record_cap,
                    a->rec_return,
                    a->rec_length,
                    a->rec_success,
                    a->rec_end_step,
                    a->ep_code,
                    a->applied_act,
                    a->dyn_noise_tape,
                    a->obs_noise_tape,
                    static_cast<bf16*>(a->h2_tape)};

    DXRL_REQUIRE(!(a->dyn_noise_tape || a->obs_noise_tape) || !(a->obs_fm || (a->diag_flags & 16)),
                 "the noise tapes are written by the 16- and 32-env rollout kernels only");
    DeviceGuard g(env->device);
    const int64_t n = env->cfg.num_envs;
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(a->h2_tape) & 15) == 0, "pg_rollout: h2_tape must be 16-byte aligned");
    DXRL_REQUIRE(!a->h2_tape || rollout_kernel(n, a->diag_flags, a->obs_fm != nullptr) != 0,
                 "h2_tape is written by the 16- and 32-env rollout kernels only (dxrl_pg_rollout_kernel)");
    if (a->obs_fm || (a->diag_flags & 16)) {  // feature-major tape / A-B reference: the 64-env kernel
        hipLaunchKernelGGL(k_pg_rollout, dim3((unsigned)((n + kTile - 1) / kTile)), dim3(64 * kRolloutWaves), 0,
                           as_stream(stream), p);
        return launch_check("k_pg_rollout");
    }
    DXRL_REQUIRE(!(a->diag_flags & (32 | 64)), "diag_flags 32 / 64 named the retired k_pg_rollout_ls");
    static unsigned long long* stamps = nullptr;
    static int64_t stamps_n = 0;
    if ((a->diag_flags & 128) && stamps_n < n) {
        if (stamps) (void)hipFree(stamps);
        (void)hipMalloc(&stamps, (size_t)n * 16 * sizeof(unsigned long long));
        stamps_n = n;
    }
    p.stamps = stamps;
    const bool e8 = rollout_kernel(n, a->diag_flags, false) == 2;
    if (e8) {
        const bool noise = a->obs_noise_std > 0.0 || a->dyn_noise_std > 0.0 || a->dyn_noise_tape || a->obs_noise_tape;
        const bool diag = (a->diag_flags & ~(1024 | 2048)) != 0 || a->applied_act || a->dyn_noise_tape ||
                          a->obs_noise_tape;
        return launch_pg_rollout_e8(p, n, noise, diag, as_stream(stream));
    }
    {  // the 16-env warp-specialised kernel
        const bool noise = a->obs_noise_std > 0.0 || a->dyn_noise_std > 0.0 || a->dyn_noise_tape || a->obs_noise_tape;
        const bool diag = (a->diag_flags & ~(1024 | 2048)) != 0 || a->applied_act || a->dyn_noise_tape ||
                          a->obs_noise_tape;
        const dim3 grid((unsigned)((n + kLsEnvs - 1) / kLsEnvs)), block(kWsThreads);
        if (noise && diag) hipLaunchKernelGGL((k_pg_rollout_ws<true, true>), grid, block, 0, as_stream(stream), p);
        else if (noise) hipLaunchKernelGGL((k_pg_rollout_ws<true, false>), grid, block, 0, as_stream(stream), p);
        else if (diag) hipLaunchKernelGGL((k_pg_rollout_ws<false, true>), grid, block, 0, as_stream(stream), p);
        else hipLaunchKernelGGL((k_pg_rollout_ws<false, false>), grid, block, 0, as_stream(stream), p);
        if (int rc = launch_check("k_pg_rollout_ws")) return rc;
        if (a->diag_flags & 128) {  // diagnostics: mean cycles per env per step segment, env / aux waves
            std::vector<unsigned long long> h((size_t)n * 16);
            (void)hipStreamSynchronize(as_stream(stream));
            (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
            for (int w = 0; w < 2; ++w) {
                fprintf(stderr, "rollout_ws %s cycles/step:", w ? "aux" : "env");
                for (int k = 0; k < 7; ++k) {
                    double sum = 0;
                    for (int64_t e = 0; e < n; ++e) sum += (double)h[e * 16 + 8 * w + k];
                    fprintf(stderr, " s%d=%.0f", k, sum / n / a->horizon);
                }
                fprintf(stderr, "\n");
                for (int wv = 0; wv < 4; ++wv) {  // per wave of the workgroup (envs 4 wv .. 4 wv + 3)
                    fprintf(stderr, "  wave %d:", 4 * w + wv);
                    for (int k = 0; k < 7; ++k) {
                        double sum = 0;
                        int64_t cnt = 0;
                        for (int64_t e = 0; e < n; ++e)
                            if ((e % kLsEnvs) / 4 == wv) {
                                sum += (double)h[e * 16 + 8 * w + k];
                                ++cnt;
                            }
                        fprintf(stderr, " s%d=%.0f", k, cnt ? sum / cnt / a->horizon : 0.0);
                    }
                    fprintf(stderr, "\n");
                }
            }
        }
        return DXRL_OK;
    }
}

int dxrl_pg_gae_partial_doubles(int64_t num_envs, int64_t horizon, int64_t* doubles) {
    DXRL_REQUIRE(doubles && num_envs >= 1 && horizon >= 1, "bad argument");
    // one Moments triple per workgroup; k_gae_lds (16 envs per workgroup) launches the most
    static_assert(kGlEnvs <= kGaeThreads, "k_gae_lds must be the kernel with the most workgroups");
    *doubles = 3 * ((num_envs + kGlEnvs - 1) / kGlEnvs);
    return DXRL_OK;
}

int dxrl_pg_gae(int32_t device, const float* rew, const uint8_t* done, const float* values, int64_t num_envs,
                int64_t horizon, double gamma, double lam, float* adv, float* ret, double* partial, double* stats,
                void* stream) {
    DXRL_REQUIRE(rew && done && values && adv && ret && partial && stats, "null argument");
    DXRL_REQUIRE(num_envs >= 1 && horizon >= 1, "num_envs and horizon must be >= 1");
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    static const bool seq = [] {  // A/B: k_gae, the chunked-load scan (DXRL_GAE_SEQ=1)
        const char* v = getenv("DXRL_GAE_SEQ");
        return v && atoi(v) != 0;
    }();
    int nb;
    const int64_t lds = gae_lds_bytes(horizon);
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(k_gae_lds),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 8 * 1024) == hipSuccess;
    if (!seq && attr && lds <= 152 * 1024) {
        nb = (int)((num_envs + kGlEnvs - 1) / kGlEnvs);
        hipLaunchKernelGGL(k_gae_lds, dim3(nb), dim3(kGlThreads), (size_t)lds, st, rew, done, values, num_envs,
                           (int)horizon, (float)gamma, (float)lam, adv, ret, reinterpret_cast<Moments*>(partial));
        if (int rc = launch_check("k_gae_lds")) return rc;
    } else {
        nb = (int)((num_envs + kGaeThreads - 1) / kGaeThreads);
        hipLaunchKernelGGL(k_gae, dim3(nb), dim3(kGaeThreads), 0, st, rew, done, values, num_envs, horizon,
                           (float)gamma, (float)lam, adv, ret, reinterpret_cast<Moments*>(partial));
        if (int rc = launch_check("k_gae")) return rc;
    }
    hipLaunchKernelGGL(k_gae_sums, dim3(1), dim3(256), 0, st, reinterpret_cast<const Moments*>(partial), nb, stats);
    return launch_check("k_gae_sums");
}

int dxrl_pg_adv_combine(int32_t device, const double* moments, int32_t world, double* stats, void* stream) {
    DXRL_REQUIRE(moments && stats && world >= 1, "bad argument");
    DeviceGuard g(device);
    hipLaunchKernelGGL(k_stats_combine, dim3(1), dim3(1), 0, as_stream(stream), moments, world, stats);
    return launch_check("k_stats_combine");
}

int dxrl_pg_adv_finalize(int32_t device, int32_t phase, const float* adv, int64_t count, double* partial,
                         double* stats, void* stream) {
    DXRL_REQUIRE(stats, "null argument");
    DXRL_REQUIRE(phase == 2, "phase must be 2 (the two-pass phases 0 / 1 were retired for the merged moments)");
    (void)adv, (void)count, (void)partial;
    return dxrl_pg_adv_combine(device, stats + 5, 1, stats, stream);
}

int dxrl_pg_heads(int32_t device, const dxrl_pg_heads_args* a, void* stream) {
    DXRL_REQUIRE(a, "null args");
    DeviceGuard g(device);
    HeadArgs h{a->mu, a->values, a->act, a->logp_old, a->adv, a->ret, a->stats, a->params, a->num_samples,
               a->inv_total_samples, (float)a->clip_eps, (float)a->vf_coef,
               static_cast<bf16*>(a->dmu_rm), static_cast<bf16*>(a->dmu_fm), static_cast<bf16*>(a->dv_rm),
               static_cast<bf16*>(a->dv_fm), a->dlogstd_partial, a->loss_partial};
    const int nb = (int)((a->num_samples + 255) / 256);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_ppo_heads, dim3(nb), dim3(256), 0, st, h);
    if (int rc = launch_check("k_ppo_heads")) return rc;
    hipLaunchKernelGGL(k_logstd_grad, dim3(1), dim3(256), 0, st, a->dlogstd_partial, nb, (float)a->ent_coef,
                       a->grads);
    return launch_check("k_logstd_grad");
}

int dxrl_pg_grad_sumsq(int32_t device, const float* grads, int64_t n, double* partial, double* out, void* stream) {
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_sumsq, dim3(512), dim3(256), 0, st, grads, n, partial);
    if (int rc = launch_check("k_sumsq")) return rc;
    return reduce_to(partial, 512, out, 0, st);
}

int dxrl_pg_optimizer_step(int32_t device, const float* params, const float* grads, const float* m1, const float* m2,
                           float* params_out, float* m1_out, float* m2_out, int64_t n, double lr, double beta1,
                           double beta2, double eps, int64_t step, double max_norm, double* partial, double* gnorm2,
                           void* packed, void* stream) {
    DXRL_REQUIRE(params && grads && m1 && m2 && params_out && m1_out && m2_out && partial && gnorm2 && packed &&
                     step >= 1,
                 "bad optimizer arguments");
    DXRL_REQUIRE(n == kParams, "optimizer: n must be the padded parameter count %lld", (long long)kParams);
    DXRL_REQUIRE(params != params_out && m1 != m1_out && m2 != m2_out, "optimizer: outputs must not alias inputs");
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    constexpr int kNb = 512;
    hipLaunchKernelGGL(k_sumsq, dim3(kNb), dim3(256), 0, st, grads, n, partial);
    if (int rc = launch_check("k_sumsq")) return rc;
    AdamPackArgs a{params, grads, m1, m2, params_out, m1_out, m2_out, n, (float)lr, (float)beta1, (float)beta2,
                   (float)eps, (float)(1.0 - pow(beta1, (double)step)), (float)(1.0 - pow(beta2, (double)step)),
                   (float)max_norm, partial, kNb, gnorm2, static_cast<bf16*>(packed)};
    hipLaunchKernelGGL(k_adam_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
    return launch_check("k_adam_pack");
}

int dxrl_pg_adam_step(int32_t device, const float* params, const float* grads, const float* m1, const float* m2,
                      float* params_out, float* m1_out, float* m2_out, int64_t n, double lr, double beta1, double beta2,
                      double eps, int64_t step, double max_norm, const double* gnorm_partial, int32_t gnorm_blocks,
                      double* gnorm2, void* packed, void* stream) {
    DXRL_REQUIRE(params && grads && m1 && m2 && params_out && m1_out && m2_out && gnorm_partial && gnorm2 && packed &&
                     step >= 1 && gnorm_blocks >= 1,
                 "bad adam_step arguments");
    DXRL_REQUIRE(n == kParams, "adam_step: n must be the padded parameter count %lld", (long long)kParams);
    DXRL_REQUIRE(params != params_out && m1 != m1_out && m2 != m2_out, "adam_step: outputs must not alias inputs");
    DeviceGuard g(device);
    AdamPackArgs a{params, grads, m1, m2, params_out, m1_out, m2_out, n, (float)lr, (float)beta1, (float)beta2,
                   (float)eps, (float)(1.0 - pow(beta1, (double)step)), (float)(1.0 - pow(beta2, (double)step)),
                   (float)max_norm, gnorm_partial, gnorm_blocks, gnorm2, static_cast<bf16*>(packed)};
    hipLaunchKernelGGL(k_adam_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), a);
    return launch_check("k_adam_pack");
}

int dxrl_pg_adam(int32_t device, float* params, const float* grads, float* m1, float* m2, int64_t n, double lr,
                 double beta1, double beta2, double eps, int64_t step, const double* gnorm2, double max_norm,
                 void* stream) {
    DXRL_REQUIRE(params && grads && m1 && m2 && step >= 1, "bad adam arguments");
    DeviceGuard g(device);
    const float bc1 = (float)(1.0 - pow(beta1, (double)step)), bc2 = (float)(1.0 - pow(beta2, (double)step));
    hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), params, grads, m1,
                       m2, n, (float)lr, (float)beta1, (float)beta2, (float)eps, bc1, bc2, gnorm2,
                       (float)max_norm);
    return launch_check("k_adam");
}

}  // extern "C"
