// dxrl_eval.hip -- evaluation episode programs.
//
// Replaces the per-episode Python loops of
//   evaluation/evaluator.py:71-181        Evaluator.evaluate_episode (EV)
//   evaluation/evaluator.py:183-262       Evaluator.evaluate_heldout_set
//   evaluation/robustness_tests.py:240-310 RobustnessTester.evaluate_with_noise (RT)
//   evaluation/robustness_tests.py:312-407 RobustnessTester.run_robustness_sweep
// One lane = one chain of segments (fresh env instances, see include/dxrl.h);
// the env state, the frozen policy and both random streams live in registers
// for the whole chain.  Records go out once per episode; the optional
// per-step contact history is one byte per step.
#include "dxrl_internal.h"

#include <stdio.h>
#include <stdlib.h>

using namespace dxrl;

namespace dxrl {

constexpr uint32_t kStreamEvalNoise = 0x45564e00u;

struct EvalParams {
    Weights w;
    int max_episode_steps;  // env truncation (ME:245)
    int dense;
    int has_object;         // env constructed with object_position (ME:28, :156-161)
    int n_curricula;
    double obj[3];
    dxrl_eval_args a;
    unsigned long long* diag_iters;  // DXRL_EVAL_DIAG: step iterations executed per wave, summed
};

// Draw-by-draw reader over a tape row or a Philox stream.  Philox blocks are
// consumed four u32 at a time: two 53-bit uniforms, or four f32 normals.
struct Stream {
    const double* tape;
    int64_t avail;
    int64_t cur;
    uint32_t k0, k1, tag;
    uint64_t ctr;
    bool ok;

    __device__ __forceinline__ u32x4 block() {
        const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), tag, 0u}, k0, k1);
        ++ctr;
        return r;
    }
    // n raw draws from the tape (cursor advances; false once the tape is exhausted)
    __device__ __forceinline__ bool take(double* out, int n) {
        if (cur + n > avail) {
            ok = false;
            return false;
        }
        for (int k = 0; k < n; ++k) out[k] = tape[cur + k];
        cur += n;
        return true;
    }
    __device__ __forceinline__ void skip(int n) {
        if (cur + n > avail) ok = false;
        cur += n;
    }
};

// f32 noise terms of one policy step (kD values) in the policy's own arithmetic.
template <bool kTape>
__device__ __forceinline__ bool policy_terms(int policy, double sigma, Stream& s, float* nz) {
    if (kTape) {
        double g[kD];
        if (!s.take(g, kD)) return false;
#pragma unroll
        for (int k = 0; k < kD; ++k) {
            if (policy == DXRL_EVAL_POLICY_SIMPLE)
                nz[k] = (float)(0.0 + sigma * g[k]);          // np.random.normal(0, s) (SL:60)
            else if (policy == DXRL_EVAL_POLICY_HEURISTIC)
                nz[k] = (float)(-0.1 + (0.1 - -0.1) * g[k]);  // np.random.uniform(-0.1, 0.1)
            else
                nz[k] = (float)(-1.0 + (1.0 - -1.0) * g[k]);  // Box.sample: uniform(low, high)
        }
        return true;
    }
    if (policy == DXRL_EVAL_POLICY_SIMPLE) {
        const float fs = (float)sigma;
#pragma unroll
        for (int b = 0; b < (kD + 3) / 4; ++b) {
            const u32x4 r = s.block();
            float n[4];
            box_muller(r.x, r.y, n[0], n[1]);
            box_muller(r.z, r.w, n[2], n[3]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * b + q < kD) nz[4 * b + q] = fs * n[q];
        }
    } else {
        const double lo = policy == DXRL_EVAL_POLICY_HEURISTIC ? -0.1 : -1.0;
#pragma unroll
        for (int b = 0; b < (kD + 1) / 2; ++b) {
            const u32x4 r = s.block();
            nz[2 * b] = (float)(lo + (-lo - lo) * u01_53(r.x, r.y));
            if (2 * b + 1 < kD) nz[2 * b + 1] = (float)(lo + (-lo - lo) * u01_53(r.z, r.w));
        }
    }
    return true;
}

// Dynamics noise of one wrapper step: f32(0 + s g) per joint (RT:180-187).
__device__ __forceinline__ void dyn_terms(bool tape, double sigma, Stream& s, float* nz) {
    if (tape) {
        double g[kD];
        if (!s.take(g, kD)) {
#pragma unroll
            for (int k = 0; k < kD; ++k) nz[k] = 0.0f;
            return;
        }
#pragma unroll
        for (int k = 0; k < kD; ++k) nz[k] = (float)(0.0 + sigma * g[k]);
        return;
    }
    const float fs = (float)sigma;
#pragma unroll
    for (int b = 0; b < (kD + 3) / 4; ++b) {
        const u32x4 r = s.block();
        float n[4];
        box_muller(r.x, r.y, n[0], n[1]);
        box_muller(r.z, r.w, n[2], n[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * b + q < kD) nz[4 * b + q] = fs * n[q];
    }
}

template <bool kTape>
__global__ __launch_bounds__(64) void k_eval(const dxrl_curriculum* __restrict__ curricula, EvalParams p) {
    const dxrl_eval_args& a = p.a;
    const int lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= a.num_lanes) return;
    Stream ps{};
    ps.ok = true;
    if (kTape) {
        ps.tape = a.policy_tape + (int64_t)lane * a.policy_stride;
        ps.avail = a.policy_stride;
    } else {
        env_key(a.policy_seed, lane, ps.k0, ps.k1);
        ps.tag = kStreamPolicy;
    }
    float mean[kD];
#pragma unroll
    for (int k = 0; k < kD; ++k) mean[k] = a.mean_action ? a.mean_action[(int64_t)lane * kD + k] : 0.0f;
    const int s0 = a.lane_segments[lane], s1 = a.lane_segments[lane + 1];
    const bool ntape = a.noise_tape != nullptr;
    bool ok = true;
    for (int si = s0; si < s1 && ok; ++si) {
        const dxrl_eval_segment sg = a.segments[si];
        const bool noisy = sg.obs_noise_std > 0.0 || sg.dyn_noise_std > 0.0;
        if (sg.curriculum_row < 0 || sg.curriculum_row >= p.n_curricula || sg.first_episode < 0 ||
            (ntape && noisy && sg.noise_offset < 0)) {
            ok = false;
            break;
        }
        const dxrl_curriculum cu = curricula[sg.curriculum_row];
        Stream ns{};
        ns.ok = true;
        if (ntape) {
            ns.tape = a.noise_tape + sg.noise_offset;
            ns.avail = sg.noise_count;
        } else {
            env_key(a.noise_seed, si, ns.k0, ns.k1);
            ns.tag = kStreamEvalNoise;
        }
        const bool obs_noise = sg.obs_noise_std > 0.0, dyn_noise = sg.dyn_noise_std > 0.0;
        // DexterousManipulationEnv(curriculum_config=row) (EV:94-98, RT:266-270)
        Env e;
#pragma unroll
        for (int k = 0; k < kD; ++k) e.jp[k] = e.jv[k] = 0.0f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            e.op[i] = p.obj[i];
            e.ov[i] = 0.0f;
        }
        e.flags = p.has_object ? kHasObject : 0u;
        e.t = 0;
        e.cfg = sg.curriculum_row;
        for (int ep = 0; ep < sg.num_episodes && ok; ++ep) {
            const int64_t rec = (int64_t)sg.first_episode + ep;
            if (rec >= a.total_episodes) {
                ok = false;
                break;
            }
            // env.reset(seed=episode_seed) (EV:127, RT:281) [+ wrapper obs noise, RT:193-197]
            if (ntape && obs_noise) ns.skip(kObs);
            if (a.reset_tape) {
                double d[kReset];
#pragma unroll
                for (int k = 0; k < kReset; ++k) d[k] = a.reset_tape[rec * kReset + k];
                env_reset(e, d, cu);
            } else {
                uint32_t rk0, rk1;
                env_key(a.reset_seed, rec, rk0, rk1);
                env_reset_philox(e, cu, rk0, rk1, 0);
            }
            float* otraj = a.obs_traj ? a.obs_traj + rec * (int64_t)(a.max_steps + 1) * kObs : nullptr;
            float* atraj = a.act_traj ? a.act_traj + rec * (int64_t)a.max_steps * kD : nullptr;
            if (otraj) write_obs(e, otraj);
            double ret = 0.0;
            bool te = false, tr = false;
            uint32_t nc = 0;
            int steps = 0;
            uint8_t* hist = a.contact_hist ? a.contact_hist + rec * a.max_steps : nullptr;
            for (int step = 0; step < a.max_steps; ++step) {
                float nz[kD], act[kD];
                if (!policy_terms<kTape>(a.policy, a.exploration_noise, ps, nz)) {
                    ok = false;
                    break;
                }
#pragma unroll
                for (int k = 0; k < kD; ++k)
                    act[k] = a.policy == DXRL_EVAL_POLICY_SIMPLE      ? clipf(mean[k] + nz[k], -1.0f, 1.0f)
                             : a.policy == DXRL_EVAL_POLICY_HEURISTIC ? clipf(-0.5f + nz[k], -1.0f, 1.0f)
                                                                      : nz[k];
                if (atraj) {
#pragma unroll
                    for (int k = 0; k < kD; ++k) atraj[step * kD + k] = act[k];
                }
                if (dyn_noise) {  // RT:180-187: clip(a + f32(N(0, s)), low, high)
                    float dz[kD];
                    dyn_terms(ntape, sg.dyn_noise_std, ns, dz);
#pragma unroll
                    for (int k = 0; k < kD; ++k) act[k] = clipf(act[k] + dz[k], -1.0f, 1.0f);
                }
                double cp[4];
                const double r = env_step(e, act, p.dense != 0, p.w, p.max_episode_steps, te, tr, cp);
                if (ntape && obs_noise) ns.skip(kObs);
                ret += r;  // EV:143 / RT:291 episode_reward += reward
                steps = step + 1;
                nc = (uint32_t)__popc(e.flags & 0x1Fu);
                if (hist) hist[step] = (uint8_t)nc;
                if (otraj) write_obs(e, otraj + (int64_t)(step + 1) * kObs);
                if (te || tr) break;
            }
            if (!ok) break;
            a.ep_return[rec] = ret;
            a.ep_length[rec] = steps;
            a.ep_success[rec] = (uint8_t)te;  // success = terminated (EV:157, RT:303)
            if (a.ep_contacts) a.ep_contacts[rec] = (uint8_t)nc;
        }
        if (!ns.ok) ok = false;
    }
    if (!ps.ok) ok = false;
    if (a.policy_used) a.policy_used[lane] = (int32_t)ps.cur;
    if (!ok && a.status) atomicOr(a.status, 1);
}

// ------------------------------------------------------------------ lane-split programs
// k_eval_ls: the same episode programs with each env spread over the 16 lanes of a DPP row (the
// rollout's layout: lane s owns joint s / action s, lanes 0..2 the object axes, the per-row
// sums and minima exchanged by row broadcasts) and the rows fed from a work queue: a row takes
// the next program lane whenever its current one ends, so no row idles behind a long episode.
// Every draw is the one k_eval takes (tape cursors advance by the step's draw count; Philox
// blocks are addressed by their position in the lane's stream), so records, histories,
// trajectories and tape consumption are identical (test_lane_split_eval_matches_one_lane_kernel).
constexpr int kEvalRows = 16, kEvalThreads = 16 * kEvalRows;

template <bool kTape>
__global__ __launch_bounds__(kEvalThreads) void k_eval_ls(const dxrl_curriculum* __restrict__ curricula,
                                                         EvalParams p, int32_t* __restrict__ queue) {
    const dxrl_eval_args& a = p.a;
    const int s = threadIdx.x & 15, gbit = 16 * ((threadIdx.x & 63) >> 4);
    const int sa = s < kD ? s : 0;
    const int s2 = s < DXRL_RESET_EXTRA ? s : 0;
    const bool ntape = a.noise_tape != nullptr;
    const bool simple = a.policy == DXRL_EVAL_POLICY_SIMPLE, heur = a.policy == DXRL_EVAL_POLICY_HEURISTIC;
    enum { kNeedLane, kNeedEp, kStep, kDone };
    int phase = kNeedLane;
    int lane = 0, si = 0, s1 = 0, ep = 0, step = 0;
    bool ok = true;
    // policy stream (tape cursor or Philox counter) and noise stream of the current segment
    int64_t pcur = 0, ncur = 0, navail = 0;
    uint64_t pctr = 0, nctr = 0;
    bool pok = true, nok = true;
    uint32_t pk0 = 0, pk1 = 0, nk0 = 0, nk1 = 0;
    const double* ptape = nullptr;
    const double* ntp = nullptr;
    float mean = 0.0f;
    double dyn_sigma = 0.0;
    bool obs_noise = false, dyn_noise = false;
    int first_ep = 0, n_eps = 0, cfg = 0;
    double lo2 = 0.0, hi2 = 0.0, cst2 = 0.0;
    bool has2 = true, fric64 = false;
    // env (lane-split)
    float jp = 0.0f, jv = 0.0f, ovd = 0.0f;
    double opd = 0.0, size = 0.0;
    double fric = 0.0;
    uint32_t flags = 0;
    int32_t et = 0;
    int64_t rec = 0;
    float *otraj = nullptr, *atraj = nullptr;
    uint8_t* hist = nullptr;
    double ret = 0.0;
    bool te = false;
    uint32_t nc = 0;
    int steps = 0;
    uint32_t iters = 0;  // step iterations this lane executed (diagnostics)

    const auto write_obs_row = [&](float* o) {  // ME:254-264, lane s's elements (row_obs_elem)
        if (s < kD) {
            o[s] = jp;
            o[kD + s] = jv;
        }
        if (s < 3) {
            o[2 * kD + s] = (float)opd;
            o[2 * kD + 7 + s] = ovd;
        } else if (s < 7) {
            o[2 * kD + s] = s == 3 ? 1.0f : 0.0f;
        } else if (s < 7 + kF) {
            o[2 * kD + 10 + (s - 7)] = (float)((flags >> (s - 7)) & 1u);
        }
    };
    const auto finish_lane = [&]() {
        if (!pok) ok = false;
        if (s == 0) {
            if (a.policy_used) a.policy_used[lane] = (int32_t)pcur;
            if (!ok && a.status) atomicOr(a.status, 1);
        }
        phase = kNeedLane;
    };
    // the next segment of the lane (si), or the lane's end
    const auto next_segment = [&]() {
        if (!ok || si >= s1) {
            finish_lane();
            return;
        }
        const dxrl_eval_segment sg = a.segments[si];
        const bool noisy = sg.obs_noise_std > 0.0 || sg.dyn_noise_std > 0.0;
        if (sg.curriculum_row < 0 || sg.curriculum_row >= p.n_curricula || sg.first_episode < 0 ||
            (ntape && noisy && sg.noise_offset < 0)) {
            ok = false;
            finish_lane();
            return;
        }
        cfg = sg.curriculum_row;
        const dxrl_curriculum& cu = curricula[cfg];
        const double* rg = s2 == 0 ? cu.size_range
                                   : s2 == 1 ? cu.mass_range
                                             : s2 == 2 ? cu.friction_range
                                                       : s2 == 3 ? cu.spawn_x_range : s2 == 4 ? cu.spawn_y_range : cu.spawn_z_range;
        lo2 = rg[0];
        hi2 = rg[1];
        cst2 = s2 == 0 ? cu.object_size : s2 == 1 ? cu.object_mass : cu.friction_coefficient;
        has2 = s2 == 0 ? cu.has_size_range != 0 : s2 == 1 ? cu.has_mass_range != 0 : s2 == 2 ? cu.has_friction_range != 0 : true;
        fric64 = cu.friction_is_f64_scalar != 0;
        nok = true;
        if (ntape) {
            ntp = a.noise_tape + sg.noise_offset;
            navail = sg.noise_count;
            ncur = 0;
        } else {
            env_key(a.noise_seed, si, nk0, nk1);
            nctr = 0;
        }
        obs_noise = sg.obs_noise_std > 0.0;
        dyn_noise = sg.dyn_noise_std > 0.0;
        dyn_sigma = sg.dyn_noise_std;
        first_ep = sg.first_episode;
        n_eps = sg.num_episodes;
        // DexterousManipulationEnv(curriculum_config=row) (EV:94-98, RT:266-270)
        jp = jv = 0.0f;
        opd = s < 3 ? p.obj[s] : 0.0;
        ovd = 0.0f;
        flags = p.has_object ? kHasObject : 0u;
        et = 0;
        ep = 0;
        phase = kNeedEp;
    };
    const auto next_episode = [&]() {
        if (ep >= n_eps) {  // end of the segment
            if (!nok) ok = false;
            ++si;
            next_segment();
            return;
        }
        rec = (int64_t)first_ep + ep;
        if (rec >= a.total_episodes) {
            ok = false;
            finish_lane();
            return;
        }
        // env.reset(seed=episode_seed) (EV:127, RT:281) [+ wrapper obs noise, RT:193-197]
        if (ntape && obs_noise) {
            if (ncur + kObs > navail) nok = false;
            ncur += kObs;
        }
        double u1, v2;
        if (a.reset_tape) {
            u1 = a.reset_tape[rec * kReset + sa];
            v2 = has2 ? a.reset_tape[rec * kReset + kD + s2] : cst2;
        } else {
            uint32_t rk0, rk1;
            env_key(a.reset_seed, rec, rk0, rk1);
            u1 = -0.1 + (0.1 - -0.1) * reset_uniform_at(sa, rk0, rk1, 0);
            v2 = has2 ? lo2 + (hi2 - lo2) * reset_uniform_at(kD + s2, rk0, rk1, 0) : cst2;
        }
        jp = s < kD ? (float)u1 : 0.0f;  // ME:143-145 .astype(float32)
        jv = 0.0f;
        size = row_bcast<0>(v2);
        fric = row_bcast<2>(v2);
        const double sx = row_bcast<3>(v2), sy = row_bcast<4>(v2), sz = row_bcast<5>(v2);
        const double spawn = s == 1 ? sy : (s == 2 ? sz : sx);
        const bool has = (flags & kHasObject) != 0;  // ME:156-161 sticky position
        if (s < 3) {
            opd = (double)(float)(has ? opd : spawn);
            ovd = 0.0f;
        }
        et = 0;
        flags = kOpIsF32 | kHasObject | (fric64 ? kFricF64 : 0u);
        double op3[3], dmin;
        float g3[3];
        row_object(opd, op3);
        flags |= row_contacts<false>(jp, op3, size, s, gbit, dmin, g3);  // ME:176 (no dmin)
        otraj = a.obs_traj ? a.obs_traj + rec * (int64_t)(a.max_steps + 1) * kObs : nullptr;
        atraj = a.act_traj ? a.act_traj + rec * (int64_t)a.max_steps * kD : nullptr;
        if (otraj) write_obs_row(otraj);
        ret = 0.0;
        te = false;
        nc = 0;
        steps = 0;
        step = 0;
        hist = a.contact_hist ? a.contact_hist + rec * a.max_steps : nullptr;
        phase = kStep;
    };
    const auto end_episode = [&]() {
        if (s == 0) {
            a.ep_return[rec] = ret;
            a.ep_length[rec] = steps;
            a.ep_success[rec] = (uint8_t)te;  // success = terminated (EV:157, RT:303)
            if (a.ep_contacts) a.ep_contacts[rec] = (uint8_t)nc;
        }
        ++ep;
        next_episode();
    };
    while (true) {
        while (phase != kStep && phase != kDone) {
            if (phase == kNeedLane) {
                int L = 0;
                if (s == 0) L = atomicAdd(queue, 1);
                lane = (int)row_bcast_u32<0>((uint32_t)L);
                if (lane >= a.num_lanes) {
                    phase = kDone;
                    break;
                }
                ok = pok = true;
                pcur = 0;
                pctr = 0;
                if (kTape) {
                    ptape = a.policy_tape + (int64_t)lane * a.policy_stride;
                } else {
                    env_key(a.policy_seed, lane, pk0, pk1);
                }
                mean = a.mean_action ? a.mean_action[(int64_t)lane * kD + sa] : 0.0f;
                si = a.lane_segments[lane];
                s1 = a.lane_segments[lane + 1];
                next_segment();
            } else {
                next_episode();
            }
        }
        if (phase == kDone) break;
        ++iters;
        // ---- the policy's action (one frozen-policy step; policy_terms' draws, lane s: dim s)
        float nz;
        if (kTape) {
            if (pcur + kD > a.policy_stride) {
                pok = false;
                ok = false;
                finish_lane();
                continue;
            }
            const double g = ptape[pcur + sa];
            pcur += kD;
            nz = simple ? (float)(0.0 + a.exploration_noise * g)       // np.random.normal(0, s) (SL:60)
                 : heur ? (float)(-0.1 + (0.1 - -0.1) * g)            // np.random.uniform(-0.1, 0.1)
                        : (float)(-1.0 + (1.0 - -1.0) * g);           // Box.sample: uniform(low, high)
        } else if (simple) {
            const uint64_t c = pctr + (uint64_t)(sa >> 2);
            const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), kStreamPolicy, 0u}, pk0, pk1);
            float n0, n1;
            const bool hi = (sa & 2) != 0;
            box_muller(hi ? r.z : r.x, hi ? r.w : r.y, n0, n1);
            nz = (float)a.exploration_noise * ((sa & 1) ? n1 : n0);
            pctr += (kD + 3) / 4;
        } else {
            const double lo = heur ? -0.1 : -1.0;
            const uint64_t c = pctr + (uint64_t)(sa >> 1);
            const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), kStreamPolicy, 0u}, pk0, pk1);
            nz = (float)(lo + (-lo - lo) * ((sa & 1) ? u01_53(r.z, r.w) : u01_53(r.x, r.y)));
            pctr += (kD + 1) / 2;
        }
        float act = simple ? clipf(mean + nz, -1.0f, 1.0f) : heur ? clipf(-0.5f + nz, -1.0f, 1.0f) : nz;
        if (atraj && s < kD) atraj[step * kD + s] = act;
        if (dyn_noise) {  // RT:180-187: clip(a + f32(N(0, s)), low, high)
            float dz = 0.0f;
            if (ntape) {
                if (ncur + kD > navail) {
                    nok = false;
                } else {
                    dz = (float)(0.0 + dyn_sigma * ntp[ncur + sa]);
                    ncur += kD;
                }
            } else {
                const uint64_t c = nctr + (uint64_t)(sa >> 2);
                const u32x4 r = philox(u32x4{(uint32_t)c, (uint32_t)(c >> 32), kStreamEvalNoise, 0u}, nk0, nk1);
                float n0, n1;
                const bool hi = (sa & 2) != 0;
                box_muller(hi ? r.z : r.x, hi ? r.w : r.y, n0, n1);
                dz = (float)dyn_sigma * ((sa & 1) ? n1 : n0);
                nctr += (kD + 3) / 4;
            }
            act = clipf(act + dz, -1.0f, 1.0f);
        }
        // ---- env_step, lane-split (ME:198-252)
        if (s < kD) {
            const float ak = clipf(act, -1.0f, 1.0f);
            jv = kC09 * jv + kC01 * ak;
            jp = clipf(jp + jv * kDt, -1.0f, 1.0f);
        }
        {
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
        }
        flags &= ~kOpIsF32;
        double op3[3], dmin;
        float g3[3];
        row_object(opd, op3);
        const uint32_t c = row_contacts(jp, op3, size, s, gbit, dmin, g3);
        double r;
        if (p.dense) {  // RS:50-187
            const double dist = exp(-5.0 * dmin);
            const double con = count_over_f_f64(__popc(c));
            float nacc = 0.0f;
#pragma unroll
            for (int j = 0; j < kJ; ++j)
                if (g3[j] < 0.0f) nacc = nacc + g3[j];
            float sum = 0.0f;
            row_neg_sum_fingers(nacc, sum);  // nacc of finger f on lane 3 f
            const float avg = div_f(sum);
            const float clo = clipf(div_f(avg), 0.0f, 1.0f);
            float st = 0.0f;
            if (flags & kHasPrev) {
                const uint32_t prev = (flags >> kPrevShift) & 0xFFu;
                float ch = 0.0f;
#pragma unroll
                for (int f = 0; f < kF; ++f) ch = ch + (float)(((c ^ prev) >> f) & 1u);
                st = clipf(1.0f - count_over_f_f32((uint32_t)ch), 0.0f, 1.0f);
            }
            flags = (flags & ~(0xFFu << kPrevShift)) | (c << kPrevShift) | kHasPrev;
            r = ((p.w.w_dist * dist + p.w.w_con * con) + p.w.w_clo * (double)clo) + p.w.w_st * (double)st;
        } else {
            r = (__popc(c) >= 3) ? 1.0 : -0.01;  // RS:226-231
        }
        flags = (flags & ~0xFFu) | c;
        te = __popc(c) >= 3;                   // ME:332-336
        const bool tr = et >= p.max_episode_steps;  // ME:245 (before the increment)
        et += 1;
        if (ntape && obs_noise) {
            if (ncur + kObs > navail) nok = false;
            ncur += kObs;
        }
        ret += r;  // EV:143 / RT:291 episode_reward += reward
        steps = step + 1;
        nc = (uint32_t)__popc(c);
        if (hist && s == 0) hist[step] = (uint8_t)nc;
        if (otraj) write_obs_row(otraj + (int64_t)(step + 1) * kObs);
        ++step;
        if (te || tr || step >= a.max_steps) end_episode();
    }
    if (p.diag_iters) {  // the wave ran as many iterations as its busiest lane: 4 env-step slots each
        uint32_t m = iters;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
        if ((threadIdx.x & 63) == 0) atomicAdd(p.diag_iters, (unsigned long long)m);
    }
}

}  // namespace dxrl

extern "C" int dxrl_evaluate(dxrl_env* env, const dxrl_eval_args* args, void* stream) {
    DXRL_REQUIRE(env && args, "null env / args");
    const dxrl_eval_args& a = *args;
    DXRL_REQUIRE(a.num_lanes > 0 && a.num_lanes <= env->cfg.num_envs, "num_lanes must be in [1, num_envs]");
    DXRL_REQUIRE(a.policy >= DXRL_EVAL_POLICY_SIMPLE && a.policy <= DXRL_EVAL_POLICY_RANDOM, "unknown policy %d",
                 a.policy);
    DXRL_REQUIRE(a.max_steps > 0 && a.total_episodes >= 0, "max_steps must be > 0, total_episodes >= 0");
    DXRL_REQUIRE(a.lane_segments && a.segments, "null segment table");
    DXRL_REQUIRE(a.ep_return && a.ep_length && a.ep_success, "null episode record buffers");
    const bool tape = a.policy_tape != nullptr;
    DXRL_REQUIRE(!tape || a.policy_stride >= 0, "bad policy tape stride");
    EvalParams p{weights_of(env->cfg),
                 env->cfg.max_episode_steps,
                 env->cfg.reward_type == DXRL_REWARD_DENSE,
                 env->cfg.has_object_position,
                 env->n_curricula,
                 {env->cfg.object_position[0], env->cfg.object_position[1], env->cfg.object_position[2]},
                 a,
                 nullptr};
    DeviceGuard g(env->device);
    hipStream_t st = as_stream(stream);
    const char* one_env = getenv("DXRL_EVAL_ONE_LANE");  // A/B: the one-lane-per-chain kernel
    const bool one_lane = one_env && atoi(one_env) != 0;
    if (one_lane) {
        const dim3 grid((unsigned)((a.num_lanes + 63) / 64)), block(64);
        if (tape)
            hipLaunchKernelGGL(k_eval<true>, grid, block, 0, st, env->curricula, p);
        else
            hipLaunchKernelGGL(k_eval<false>, grid, block, 0, st, env->curricula, p);
        return launch_check("k_eval");
    }
    // k_eval_ls: rows of 16 lanes over a work queue.  The counter is the caller's scratch
    // (a.work_queue), zeroed on the launch stream: no state shared between launches, so
    // evaluations on different streams / handles / threads cannot reset each other's queue.
    DXRL_REQUIRE(a.work_queue, "null work_queue (device i32[1] scratch of this launch)");
    const int dev = env->device;
    DXRL_REQUIRE(dev >= 0 && dev < 64, "device index out of range");
    if (int rc = hip_check(hipMemsetAsync(a.work_queue, 0, sizeof(int32_t), st), "eval queue reset")) return rc;
    const void* fn = tape ? reinterpret_cast<const void*>(k_eval_ls<true>) : reinterpret_cast<const void*>(k_eval_ls<false>);
    int per_cu = 0, cus = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kEvalThreads, 0);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int64_t blocks = (a.num_lanes + kEvalRows - 1) / kEvalRows;
    // One workgroup (16 rows) per CU by default: with more rows than that the queue runs dry
    // while the first long episodes are still running and most rows then idle in lockstep with
    // them (measured on 40,960 held-out episodes: wave efficiency 46 % -> 72 % on hard objects,
    // kernel time -26 %; 59 % -> 68 %, -5 % on the variable curriculum).  DXRL_EVAL_BPC: A/B.
    static const int bpc_env = [] {
        const char* v = getenv("DXRL_EVAL_BPC");
        return v ? atoi(v) : 1;
    }();
    if (bpc_env > 0 && (per_cu <= 0 || bpc_env < per_cu)) per_cu = bpc_env;
    const int64_t resident = (int64_t)(per_cu > 0 ? per_cu : 2) * (cus > 0 ? cus : 256);
    if (blocks > resident) blocks = resident;
    static unsigned long long* diag[64] = {nullptr};
    const char* dg = getenv("DXRL_EVAL_DIAG");
    if (dg && atoi(dg) != 0) {  // diagnostics: wave step iterations -> stderr after the launch
        if (!diag[dev]) (void)hipMalloc(&diag[dev], sizeof(unsigned long long));
        (void)hipMemsetAsync(diag[dev], 0, sizeof(unsigned long long), st);
        p.diag_iters = diag[dev];
    }
    if (tape)
        hipLaunchKernelGGL(k_eval_ls<true>, dim3((unsigned)blocks), dim3(kEvalThreads), 0, st, env->curricula, p,
                           a.work_queue);
    else
        hipLaunchKernelGGL(k_eval_ls<false>, dim3((unsigned)blocks), dim3(kEvalThreads), 0, st, env->curricula, p,
                           a.work_queue);
    if (int rc = launch_check("k_eval_ls")) return rc;
    if (p.diag_iters) {
        unsigned long long it = 0;
        (void)hipStreamSynchronize(st);
        (void)hipMemcpy(&it, p.diag_iters, sizeof(it), hipMemcpyDeviceToHost);
        fprintf(stderr, "k_eval_ls wave_iterations=%llu rows_per_wave=4 blocks=%lld per_cu=%d\n", it, (long long)blocks,
                per_cu);
    }
    return DXRL_OK;
}
