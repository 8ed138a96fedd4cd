// dxrl_rollout.hip -- fused multi-step rollout with per-env SimpleLearner.
//
// Replaces the run_episode loop (training/episode_utils.py:13-55) driving a
// SimpleLearner (policies/simple_learner.py:49-99) over consecutive episodes.
// One lane = one env + its learner; T steps run inside one launch with all
// state in registers (loaded once, stored once), so a 200-step rollout costs
// one launch instead of 200 x (select, step, update) round trips.
//
// RNG: parity mode consumes host tapes (legacy MT19937 gauss values for the
// learner, resolved PCG64 reset draws for the env) with the reference's
// data-dependent consumption order; throughput mode draws from per-env
// Philox4x32-10 streams on device.
#include "dxrl_internal.h"

using namespace dxrl;

namespace dxrl {

struct LearnerSoA {
    float* mean;
    double* best;
    double* ep_return;
    uint64_t* noise_ctr;
    int64_t n;
};

static int learner_layout(int64_t n, dxrl_learner_layout* L) {
    auto a256 = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    int64_t off = 0;
    L->mean = off;
    off = a256(off + 4 * kD * n);
    L->best = off;
    off = a256(off + 8 * n);
    L->ep_return = off;
    off = a256(off + 8 * n);
    L->noise_ctr = off;
    off = a256(off + 8 * n);
    L->total_bytes = off;
    return DXRL_OK;
}

static LearnerSoA learner_soa(void* base, int64_t n) {
    dxrl_learner_layout L;
    learner_layout(n, &L);
    char* b = static_cast<char*>(base);
    return LearnerSoA{reinterpret_cast<float*>(b + L.mean), reinterpret_cast<double*>(b + L.best),
                      reinterpret_cast<double*>(b + L.ep_return), reinterpret_cast<uint64_t*>(b + L.noise_ctr), n};
}

__global__ void k_learner_init(LearnerSoA L) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
#pragma unroll
    for (int k = 0; k < kD; ++k) L.mean[k * L.n + i] = 0.0f;  // SL:46
    L.best[i] = -__builtin_inf();                             // SL:47
    L.ep_return[i] = 0.0;
    L.noise_ctr[i] = 0;
}

__global__ void k_learner_reset(LearnerSoA L, const uint8_t* __restrict__ mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n || (mask && !mask[i])) return;
    L.best[i] = -__builtin_inf();  // SL:97-99
    L.ep_return[i] = 0.0;
}

// SL:59-71 for N learners: a = clip(mean + f32(0 + s*g), -1, 1)
__global__ void k_learner_select(LearnerSoA L, double noise, const double* __restrict__ gauss,
                                 float* __restrict__ act) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n) return;
#pragma unroll
    for (int k = 0; k < kD; ++k)
        act[i * kD + k] = clipf(L.mean[k * L.n + i] + (float)(0.0 + noise * gauss[i * kD + k]), -1.0f, 1.0f);
}

// SL:82-95 for the masked learners: mean = clip(f32(f64(mean) + (0 + lr*g)), +-clip); best = r
__global__ void k_learner_update(LearnerSoA L, double lr, float clip, const double* __restrict__ gauss,
                                 const double* __restrict__ reward, const uint8_t* __restrict__ mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L.n || !mask[i]) return;
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        const float m = (float)((double)L.mean[k * L.n + i] + (0.0 + lr * gauss[i * kD + k]));
        L.mean[k * L.n + i] = clipf(m, -clip, clip);
    }
    L.best[i] = reward[i];
}

struct RolloutParams {
    Weights w;
    int max_episode_steps;
    int max_steps;  // run_episode loop bound (episode_utils.py:38-42)
    int num_steps;
    int success_terminated;
    double lr, noise, clip;
    uint64_t env_seed, learner_seed;
    int64_t gid0;
};

// Fill g[0..kD) with the next kD normals of this env's learner stream.
template <bool kTape>
__device__ __forceinline__ bool draw_normals(double* g, const double* tape_row, int64_t stride, int& cur,
                                             uint32_t k0, uint32_t k1, uint64_t& ctr) {
    if (kTape) {
        if (cur + kD > stride) return false;
#pragma unroll
        for (int k = 0; k < kD; ++k) g[k] = tape_row[cur + k];
        cur += kD;
    } else {
#pragma unroll
        for (int b = 0; b < (kD + 3) / 4; ++b) {
            const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamPolicy, 0u}, k0, k1);
            ++ctr;
            float n0, n1, n2, n3;
            box_muller(r.x, r.y, n0, n1);
            box_muller(r.z, r.w, n2, n3);
            if (4 * b + 0 < kD) g[4 * b + 0] = n0;
            if (4 * b + 1 < kD) g[4 * b + 1] = n1;
            if (4 * b + 2 < kD) g[4 * b + 2] = n2;
            if (4 * b + 3 < kD) g[4 * b + 3] = n3;
        }
    }
    return true;
}

template <bool kDense, bool kTape>
__global__ __launch_bounds__(64) void k_rollout_simple(EnvSoA s, LearnerSoA L, RolloutParams p, dxrl_rollout_io io) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n) return;
    Env e;
    load_env(s, i, e);
    float mean[kD];
#pragma unroll
    for (int k = 0; k < kD; ++k) mean[k] = L.mean[k * L.n + i];
    double best = L.best[i];
    double ep_ret = L.ep_return[i];
    uint64_t nctr = L.noise_ctr[i];
    uint64_t rctr = s.reset_ctr[i];
    uint32_t ek0, ek1, lk0, lk1;
    env_key(p.env_seed, p.gid0 + i, ek0, ek1);
    env_key(p.learner_seed, p.gid0 + i, lk0, lk1);
    const double* grow = kTape ? io.gauss + i * io.gauss_stride : nullptr;
    const double* rrow = kTape ? io.reset_draws + i * io.reset_stride : nullptr;
    int gcur = 0, done_eps = 0;
    const int budget = io.episode_budget ? io.episode_budget[i] : 0x7fffffff;
    bool ok = true;
    const float fnoise = (float)p.noise, fclip = (float)p.clip;

    for (int step = 0; step < p.num_steps && done_eps < budget; ++step) {
        // select_action (SL:59-71)
        double g[kD];
        if (!draw_normals<kTape>(g, grow, io.gauss_stride, gcur, lk0, lk1, nctr)) {
            ok = false;
            break;
        }
        float a[kD];
#pragma unroll
        for (int k = 0; k < kD; ++k) {
            const float nz = kTape ? (float)(0.0 + p.noise * g[k]) : fnoise * (float)g[k];
            a[k] = clipf(mean[k] + nz, -1.0f, 1.0f);
        }
        bool te, tr;
        double cp[4];
        const double r = env_step(e, a, kDense, p.w, p.max_episode_steps, te, tr, cp);
        ep_ret += r;  // episode_utils.py:45 (f64, sequential)
        // update (SL:82-95)
        if (r > best) {
            if (!draw_normals<kTape>(g, grow, io.gauss_stride, gcur, lk0, lk1, nctr)) {
                ok = false;
                break;
            }
#pragma unroll
            for (int k = 0; k < kD; ++k) {
                const float m = kTape ? (float)((double)mean[k] + (0.0 + p.lr * g[k]))
                                      : mean[k] + (float)p.lr * (float)g[k];
                mean[k] = clipf(m, -fclip, fclip);
            }
            best = r;
        }
        if (te || tr || e.t >= p.max_steps) {  // episode_utils.py:42,51-53
            if (done_eps < io.record_cap) {
                const int64_t o = i * io.record_cap + done_eps;
                if (io.ep_return) io.ep_return[o] = ep_ret;
                if (io.ep_length) io.ep_length[o] = e.t;  // step + 1
                if (io.ep_success) io.ep_success[o] = p.success_terminated ? (uint8_t)te : (uint8_t)0;
                if (io.ep_end_step) io.ep_end_step[o] = step;
            }
            if (done_eps + 1 >= budget) {  // the driver's loop ends here: no further env.reset()
                ++done_eps;
                best = -__builtin_inf();
                ep_ret = 0.0;
                break;
            }
            // next run_episode: env.reset() (no seed) + policy.reset()
            const dxrl_curriculum cu = s.curricula[e.cfg];
            if (kTape) {
                if ((int64_t)(done_eps + 1) * kReset > io.reset_stride) {
                    ok = false;
                    break;
                }
                double d[kReset];
#pragma unroll
                for (int k = 0; k < kReset; ++k) d[k] = rrow[done_eps * kReset + k];
                env_reset(e, d, cu);
            } else {
                env_reset_philox(e, cu, ek0, ek1, rctr);
            }
            ++rctr;
            ++done_eps;
            best = -__builtin_inf();
            ep_ret = 0.0;
        }
    }
    store_env(s, i, e);
    s.reset_ctr[i] = rctr;
#pragma unroll
    for (int k = 0; k < kD; ++k) L.mean[k * L.n + i] = mean[k];
    L.best[i] = best;
    L.ep_return[i] = ep_ret;
    L.noise_ctr[i] = nctr;
    if (io.ep_count) io.ep_count[i] = done_eps;
    if (io.gauss_used) io.gauss_used[i] = gcur;
    if (!ok && io.status) atomicOr(io.status, 1);
}

}  // namespace dxrl

extern "C" {

int dxrl_learner_layout_for(int32_t num_envs, int32_t action_dim, dxrl_learner_layout* out) {
    DXRL_REQUIRE(out && num_envs > 0, "null layout / num_envs <= 0");
    if (action_dim != kD) {
        set_error("this build compiles action_dim=%d (got %d)", kD, action_dim);
        return DXRL_E_UNSUPPORTED;
    }
    return learner_layout(num_envs, out);
}

int dxrl_learner_init(int32_t device, int32_t num_envs, void* learner_state, void* stream) {
    DXRL_REQUIRE(learner_state && num_envs > 0, "null learner state / num_envs <= 0");
    DeviceGuard g(device);
    const int64_t n = num_envs;
    hipLaunchKernelGGL(k_learner_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       learner_soa(learner_state, n));
    return launch_check("k_learner_init");
}

int dxrl_learner_reset(int32_t device, int32_t num_envs, void* learner_state, const uint8_t* mask, void* stream) {
    DXRL_REQUIRE(learner_state && num_envs > 0, "null learner state / num_envs <= 0");
    DeviceGuard g(device);
    const int64_t n = num_envs;
    hipLaunchKernelGGL(k_learner_reset, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       learner_soa(learner_state, n), mask);
    return launch_check("k_learner_reset");
}

int dxrl_learner_select(int32_t device, int32_t num_envs, const void* learner_state, double exploration_noise,
                        const double* gauss, float* actions, void* stream) {
    DXRL_REQUIRE(learner_state && gauss && actions && num_envs > 0, "null argument / num_envs <= 0");
    DeviceGuard g(device);
    const int64_t n = num_envs;
    hipLaunchKernelGGL(k_learner_select, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       learner_soa(const_cast<void*>(learner_state), n), exploration_noise, gauss, actions);
    return launch_check("k_learner_select");
}

int dxrl_learner_update(int32_t device, int32_t num_envs, void* learner_state, double learning_rate,
                        double action_clip_range, const double* gauss, const double* reward, const uint8_t* mask,
                        void* stream) {
    DXRL_REQUIRE(learner_state && gauss && reward && mask && num_envs > 0, "null argument / num_envs <= 0");
    DeviceGuard g(device);
    const int64_t n = num_envs;
    hipLaunchKernelGGL(k_learner_update, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       learner_soa(learner_state, n), learning_rate, (float)action_clip_range, gauss, reward, mask);
    return launch_check("k_learner_update");
}

int dxrl_rollout_simple(dxrl_env* env, void* learner_state, const dxrl_learner_config* lc, int32_t num_steps,
                        int32_t max_steps, int32_t success_rule, const dxrl_rollout_io* io_in, void* stream) {
    DXRL_REQUIRE(env && learner_state && lc, "null env/learner/config");
    DXRL_REQUIRE(num_steps >= 0, "num_steps must be >= 0");
    DXRL_REQUIRE(max_steps > 0, "max_steps must be > 0");
    dxrl_rollout_io io{};
    if (io_in) io = *io_in;
    const bool tape = io.gauss != nullptr;
    DXRL_REQUIRE(tape == (io.reset_draws != nullptr), "parity mode needs both the gauss and the reset-draw tapes");
    DXRL_REQUIRE(!tape || (io.gauss_stride > 0 && io.reset_stride >= kReset), "bad tape strides");
    DXRL_REQUIRE(io.record_cap >= 0, "record_cap must be >= 0");
    const int64_t n = env->cfg.num_envs;
    RolloutParams p{weights_of(env->cfg),
                    env->cfg.max_episode_steps,
                    max_steps,
                    num_steps,
                    success_rule == DXRL_SUCCESS_TERMINATED,
                    lc->learning_rate,
                    lc->exploration_noise,
                    lc->action_clip_range,
                    env->cfg.seed,
                    lc->seed,
                    env->cfg.global_env_offset};
    DeviceGuard g(env->device);
    const LearnerSoA L = learner_soa(learner_state, n);
    const dim3 grid((unsigned)((n + 63) / 64)), block(64);
    hipStream_t st = as_stream(stream);
    const bool dense = env->cfg.reward_type == DXRL_REWARD_DENSE;
    if (dense && tape)
        hipLaunchKernelGGL((k_rollout_simple<true, true>), grid, block, 0, st, env->soa, L, p, io);
    else if (dense)
        hipLaunchKernelGGL((k_rollout_simple<true, false>), grid, block, 0, st, env->soa, L, p, io);
    else if (tape)
        hipLaunchKernelGGL((k_rollout_simple<false, true>), grid, block, 0, st, env->soa, L, p, io);
    else
        hipLaunchKernelGGL((k_rollout_simple<false, false>), grid, block, 0, st, env->soa, L, p, io);
    return launch_check("k_rollout_simple");
}

}  // extern "C"
