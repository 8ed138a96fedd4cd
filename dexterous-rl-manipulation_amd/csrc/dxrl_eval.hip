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
                 a};
    DeviceGuard g(env->device);
    const dim3 grid((unsigned)((a.num_lanes + 63) / 64)), block(64);
    if (tape)
        hipLaunchKernelGGL(k_eval<true>, grid, block, 0, as_stream(stream), env->curricula, p);
    else
        hipLaunchKernelGGL(k_eval<false>, grid, block, 0, as_stream(stream), env->curricula, p);
    return launch_check("k_eval");
}
