// dxrl_env.hip -- batched env reset/step kernels and the env half of the C ABI.
//
// Replaces envs/manipulation_env.py (DexterousManipulationEnv) + the reward
// plugins of rewards/reward_shaping.py.  State is a struct-of-arrays slab in
// HBM (layout in include/dxrl.h): component-major, env-contiguous, so every
// per-component access of a wave is one coalesced 256-B (f32) / 512-B (f64)
// transaction.  Row-major I/O tensors (actions [N][15], obs [N][45]) are
// staged through LDS so their HBM traffic is coalesced too.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

#include "dxrl_internal.h"

using namespace dxrl;

namespace dxrl {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

// ----------------------------------------------------------------------- init
__global__ void k_init(EnvSoA s, int has_obj, double ox, double oy, double oz) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n) return;
    Env e;
#pragma unroll
    for (int k = 0; k < kD; ++k) e.jp[k] = e.jv[k] = 0.0f;
    e.op[0] = ox;
    e.op[1] = oy;
    e.op[2] = oz;
    e.ov[0] = e.ov[1] = e.ov[2] = 0.0f;
    e.flags = has_obj ? kHasObject : 0u;
    e.t = 0;
    e.size = e.mass = e.fric = 0.0;
    store_env(s, i, e);
    s.cfg[i] = 0;
    s.reset_ctr[i] = 0;
}

// ----------------------------------------------------------------------- reset
// ME:124-182.  One lane per env; reset is per-episode, not per-step, so the
// obs row is written directly.
__global__ __launch_bounds__(kBlock) void k_reset(EnvSoA s, const uint8_t* __restrict__ mask,
                                                  const double* __restrict__ draws, float* __restrict__ obs,
                                                  uint64_t seed, int64_t gid0) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n) return;
    if (mask && !mask[i]) return;
    Env e;
    load_env(s, i, e);
    const dxrl_curriculum cu = s.curricula[e.cfg];
    if (draws) {
        double d[kReset];
#pragma unroll
        for (int k = 0; k < kReset; ++k) d[k] = draws[i * kReset + k];
        env_reset(e, d, cu);
    } else {
        uint32_t k0, k1;
        env_key(seed, gid0 + i, k0, k1);
        env_reset_philox(e, cu, k0, k1, s.reset_ctr[i]);
    }
    s.reset_ctr[i] += 1;
    store_env(s, i, e);
    if (obs) write_obs(e, obs + i * kObs);
}

// ----------------------------------------------------------------------- step
// ME:184-252 fused with the reward plugin.  Block = 256 envs; actions and
// observations move HBM<->LDS as contiguous float4 streams.
// Cache policy of the streamed accesses: bit0 = non-temporal stores, bit1 = non-temporal loads.
// By batch size (interleaved medians of 7 per N on one box, tools/step_policy_ab.sh,
// profiles/r06/step_policy_ab*.log): up to 2^19 envs (311 MB of traffic) the default policy
// (2^19: 0.0525 ms plain vs 0.0615 ms with both non-temporal -- round 5's threshold sat here);
// from 2^20 non-temporal stores only (0.114 vs 0.119 plain, 0.122 both); from 2^21 both
// (0.223 vs 0.231 stores only, 0.242 plain; 2^22: 0.444 vs 0.461 / 0.478).
// DXRL_STEP_VARIANT=0..3 overrides the choice (measurement).
constexpr int64_t kNtStoreMinEnvs = 1 << 20, kNtLoadMinEnvs = 1 << 21;
template <int kNt, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr ((kNt & 2) != 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int kNt, typename T>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr ((kNt & 1) != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool kDense, int kNt>
__global__ __launch_bounds__(kBlock) void k_step(EnvSoA s, const float* __restrict__ act, float* __restrict__ obs,
                                                 double* __restrict__ rew, uint8_t* __restrict__ term,
                                                 uint8_t* __restrict__ trunc, double* __restrict__ comps, Weights w,
                                                 int max_episode_steps) {
    __shared__ __attribute__((aligned(16))) float lds[kBlock * kObs];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kBlock;
    const int nb = (int)min((int64_t)kBlock, s.n - base);

    // actions [nb][15] -> LDS (coalesced float4; tail scalar)
    {
        const float* src = act + base * kD;
        const int nf = nb * kD;
        const int n4 = nf >> 2;
        using v4 = float __attribute__((ext_vector_type(4)));
        const v4* s4 = reinterpret_cast<const v4*>(src);
        v4* l4 = reinterpret_cast<v4*>(lds);
        for (int k = tid; k < n4; k += kBlock) l4[k] = ld<kNt>(s4 + k);
        for (int k = (n4 << 2) + tid; k < nf; k += kBlock) lds[k] = ld<kNt>(src + k);
    }
    __syncthreads();
    Env e;
    bool te = false, tr = false;
    double r = 0.0, cp[4];
    const int64_t i = base + tid;
    const int64_t n = s.n;
    if (tid < nb) {
        // load_env_dyn: the step reads size and friction, never mass or the curriculum row
#pragma unroll
        for (int k = 0; k < kD; ++k) {
            e.jp[k] = ld<kNt>(s.jp + k * n + i);
            e.jv[k] = ld<kNt>(s.jv + k * n + i);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            e.op[k] = ld<kNt>(s.op + k * n + i);
            e.ov[k] = ld<kNt>(s.ov + k * n + i);
        }
        e.flags = ld<kNt>(s.flags + i);
        e.t = ld<kNt>(s.t + i);
        e.size = ld<kNt>(s.size + i);
        e.fric = ld<kNt>(s.fric + i);
        float a[kD];
#pragma unroll
        for (int k = 0; k < kD; ++k) a[k] = lds[tid * kD + k];
        r = env_step(e, a, kDense, w, max_episode_steps, te, tr, cp);
#pragma unroll
        for (int k = 0; k < kD; ++k) {
            st<kNt>(s.jp + k * n + i, e.jp[k]);
            st<kNt>(s.jv + k * n + i, e.jv[k]);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            st<kNt>(s.op + k * n + i, e.op[k]);
            st<kNt>(s.ov + k * n + i, e.ov[k]);
        }
        st<kNt>(s.flags + i, e.flags);
        st<kNt>(s.t + i, e.t);
        st<kNt>(rew + i, r);
        st<kNt>(term + i, (uint8_t)te);
        st<kNt>(trunc + i, (uint8_t)tr);
        if (comps) {
            double2* c2 = reinterpret_cast<double2*>(comps + i * 4);
            c2[0] = double2{cp[0], cp[1]};
            c2[1] = double2{cp[2], cp[3]};
        }
    }
    if (!obs) return;
    __syncthreads();
    if (tid < nb) write_obs(e, lds + tid * kObs);
    __syncthreads();
    {
        float* dst = obs + base * kObs;
        const int nf = nb * kObs;
        const int n4 = nf >> 2;
        using v4 = float __attribute__((ext_vector_type(4)));
        v4* d4 = reinterpret_cast<v4*>(dst);
        const v4* l4 = reinterpret_cast<const v4*>(lds);
        for (int k = tid; k < n4; k += kBlock) st<kNt>(d4 + k, l4[k]);
        for (int k = (n4 << 2) + tid; k < nf; k += kBlock) st<kNt>(dst + k, lds[k]);
    }
}

__global__ void k_observe(EnvSoA s, float* __restrict__ obs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s.n) return;
    Env e;
    load_env(s, i, e);
    write_obs(e, obs + i * kObs);
}

// RewardShaping.compute / SparseReward.compute on caller-given inputs (RS:50-99, RS:205-242), one
// thread per item.  The dense terms come from dense_reward() -- the function every step kernel
// fuses -- fed with the min fingertip distance of the GIVEN finger_tips (RS:111-113,
// np.linalg.norm axis=1 = sqrt((dx^2 + dy^2) + dz^2) in f64) and the contact mask contacts > 0.5
// (RS:130).  Stability (RS:166-187) is restated on the f32 contact values themselves
// (np.abs(c - prev) summed in order, / len, 1 - x, clip), which for the env's 0 / 1 contacts is
// dense_reward's bitmask form bit for bit and also covers fractional contacts; prev / has_prev
// are the plugin's prev_contacts state, updated in place.
__global__ void k_reward_compute(int64_t count, bool dense, Weights w, const float* __restrict__ jp,
                                 const double* __restrict__ tips, const double* __restrict__ op,
                                 const float* __restrict__ contacts, float* __restrict__ prev,
                                 uint8_t* __restrict__ has_prev, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    float c[kF];
    uint32_t mask = 0;
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        c[f] = contacts[i * kF + f];
        mask |= (c[f] > 0.5f ? 1u : 0u) << f;
    }
    double* o = out + i * 5;
    if (!dense) {  // RS:228-242
        o[0] = __popc(mask) >= 3 ? 1.0 : -0.01;
        o[1] = o[2] = o[3] = o[4] = 0.0;
        return;
    }
    double dmin = 0.0;
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        const double* t = tips + (i * kF + f) * 3;
        const double dx = t[0] - op[i * 3 + 0], dy = t[1] - op[i * 3 + 1], dz = t[2] - op[i * 3 + 2];
        const double d = sqrt((dx * dx + dy * dy) + dz * dz);
        dmin = (f == 0 || d < dmin) ? d : dmin;  // np.min
    }
    Env e{};
#pragma unroll
    for (int k = 0; k < kD; ++k) e.jp[k] = jp[i * kD + k];
    e.flags = 0;  // stability is taken from the float restatement below
    double comp[4];
    (void)dense_reward(e, mask, dmin, w, comp);
    float st = 0.0f;
    if (has_prev[i]) {
        float ch = 0.0f;
#pragma unroll
        for (int f = 0; f < kF; ++f) ch = ch + fabsf(c[f] - prev[i * kF + f]);
        st = clipf(1.0f - div_f(ch), 0.0f, 1.0f);
    }
#pragma unroll
    for (int f = 0; f < kF; ++f) prev[i * kF + f] = c[f];
    has_prev[i] = 1;
    comp[3] = (double)st;
    o[0] = ((w.w_dist * comp[0] + w.w_con * comp[1]) + w.w_clo * comp[2]) + w.w_st * comp[3];  // RS:86-91
    o[1] = comp[0];
    o[2] = comp[1];
    o[3] = comp[2];
    o[4] = comp[3];
}

static int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

int layout_for(const dxrl_env_config* cfg, dxrl_env_layout* L) {
    const int64_t n = cfg->num_envs;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
        const int64_t o = off;
        off = align256(off + bytes);
        return o;
    };
    L->jp = take(4 * kD * n);
    L->jv = take(4 * kD * n);
    L->op = take(8 * 3 * n);
    L->ov = take(4 * 3 * n);
    L->flags = take(4 * n);
    L->step_count = take(4 * n);
    L->size = take(8 * n);
    L->mass = take(8 * n);
    L->friction = take(8 * n);
    L->cfg_index = take(4 * n);
    L->reset_ctr = take(8 * n);
    L->curricula = take((int64_t)sizeof(dxrl_curriculum) * DXRL_MAX_CURRICULA);
    L->total_bytes = off;
    return DXRL_OK;
}

static int validate_cfg(const dxrl_env_config* c) {
    DXRL_REQUIRE(c != nullptr, "null config");
    DXRL_REQUIRE(c->num_envs > 0, "num_envs must be > 0 (got %d)", c->num_envs);
    if (c->num_fingers != kF || c->joints_per_finger != kJ) {
        set_error("this build compiles num_fingers=%d, joints_per_finger=%d (got %d, %d)", kF, kJ, c->num_fingers,
                  c->joints_per_finger);
        return DXRL_E_UNSUPPORTED;
    }
    DXRL_REQUIRE(c->reward_type == DXRL_REWARD_DENSE || c->reward_type == DXRL_REWARD_SPARSE,
                 "reward_type must be DXRL_REWARD_DENSE or DXRL_REWARD_SPARSE");
    return DXRL_OK;
}

}  // namespace dxrl

// =========================================================================== C ABI
extern "C" {

int dxrl_abi_version(void) { return DXRL_ABI_VERSION; }
const char* dxrl_last_error(void) { return dxrl::g_err.c_str(); }

int dxrl_env_layout_for(const dxrl_env_config* cfg, dxrl_env_layout* out) {
    if (int rc = validate_cfg(cfg)) return rc;
    DXRL_REQUIRE(out != nullptr, "null layout");
    return layout_for(cfg, out);
}

int dxrl_env_create(const dxrl_env_config* cfg, int32_t device, void* state, void* stream, dxrl_env** out) {
    if (int rc = validate_cfg(cfg)) return rc;
    DXRL_REQUIRE(state != nullptr && out != nullptr, "null state/out");
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(state) & 255) == 0, "state slab must be 256-byte aligned");
    dxrl_env* e = new (std::nothrow) dxrl_env();
    if (!e) {
        set_error("host allocation failed");
        return DXRL_E_INVALID;
    }
    e->cfg = *cfg;
    e->device = device;
    layout_for(cfg, &e->layout);
    e->base = static_cast<char*>(state);
    const dxrl_env_layout& L = e->layout;
    char* b = e->base;
    e->curricula = reinterpret_cast<dxrl_curriculum*>(b + L.curricula);
    e->soa = EnvSoA{reinterpret_cast<float*>(b + L.jp),       reinterpret_cast<float*>(b + L.jv),
                    reinterpret_cast<double*>(b + L.op),      reinterpret_cast<float*>(b + L.ov),
                    reinterpret_cast<uint32_t*>(b + L.flags), reinterpret_cast<int32_t*>(b + L.step_count),
                    reinterpret_cast<double*>(b + L.size),    reinterpret_cast<double*>(b + L.mass),
                    reinterpret_cast<double*>(b + L.friction), reinterpret_cast<int32_t*>(b + L.cfg_index),
                    reinterpret_cast<uint64_t*>(b + L.reset_ctr), nullptr, e->curricula, cfg->num_envs};
    e->n_curricula = 1;
    DeviceGuard g(device);
    const int64_t n = cfg->num_envs;
    hipLaunchKernelGGL(k_init, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream), e->soa,
                       cfg->has_object_position, cfg->object_position[0], cfg->object_position[1],
                       cfg->object_position[2]);
    if (int rc = launch_check("k_init")) {
        delete e;
        return rc;
    }
    // default curriculum row 0 = CurriculumConfig() (experiments/config.py:24-42)
    dxrl_curriculum def{};
    def.object_size = 0.05;
    def.object_mass = 0.1;
    def.friction_coefficient = 0.5;
    def.spawn_x_range[0] = -0.1, def.spawn_x_range[1] = 0.1;
    def.spawn_y_range[0] = -0.1, def.spawn_y_range[1] = 0.1;
    def.spawn_z_range[0] = 0.05, def.spawn_z_range[1] = 0.2;
    if (int rc = hip_check(hipMemcpyAsync(e->curricula, &def, sizeof def, hipMemcpyHostToDevice, as_stream(stream)),
                           "curriculum upload") | hip_check(hipStreamSynchronize(as_stream(stream)), "create sync")) {
        delete e;
        return rc;
    }
    *out = e;
    return DXRL_OK;
}

int dxrl_env_destroy(dxrl_env* env) {
    delete env;
    return DXRL_OK;
}

static int set_curricula(dxrl_env* env, const dxrl_curriculum* table, int32_t n, const int32_t* env_index,
                         void* stream, bool sync) {
    DXRL_REQUIRE(env && table, "null env/table");
    DXRL_REQUIRE(n >= 1 && n <= DXRL_MAX_CURRICULA, "curriculum table size %d outside [1, %d]", n,
                 DXRL_MAX_CURRICULA);
    for (int k = 0; k < n; ++k) {
        const dxrl_curriculum& c = table[k];
        DXRL_REQUIRE(c.object_size > 0.0 || c.has_size_range, "curriculum row %d: object_size must be > 0", k);
    }
    if (env_index)
        for (int64_t i = 0; i < env->cfg.num_envs; ++i)
            DXRL_REQUIRE(env_index[i] >= 0 && env_index[i] < n, "env %lld: curriculum row %d out of range",
                         (long long)i, env_index[i]);
    DeviceGuard g(env->device);
    hipStream_t st = as_stream(stream);
    if (int rc = hip_check(hipMemcpyAsync(env->curricula, table, sizeof(dxrl_curriculum) * n, hipMemcpyHostToDevice, st),
                           "curricula upload"))
        return rc;
    if (env_index) {
        if (int rc = hip_check(hipMemcpyAsync(env->soa.cfg, env_index, sizeof(int32_t) * env->cfg.num_envs,
                                              hipMemcpyHostToDevice, st),
                               "env index upload"))
            return rc;
    } else {
        if (int rc = hip_check(hipMemsetAsync(env->soa.cfg, 0, sizeof(int32_t) * env->cfg.num_envs, st), "index zero"))
            return rc;
    }
    // synchronous form: the host arrays may be temporaries of the caller
    if (sync)
        if (int rc = hip_check(hipStreamSynchronize(st), "curricula sync")) return rc;
    env->n_curricula = n;
    return DXRL_OK;
}

int dxrl_env_set_curricula(dxrl_env* env, const dxrl_curriculum* table, int32_t n, const int32_t* env_index,
                           void* stream) {
    return set_curricula(env, table, n, env_index, stream, true);
}

int dxrl_env_set_curricula_async(dxrl_env* env, const dxrl_curriculum* table, int32_t n, const int32_t* env_index,
                                 void* stream) {
    return set_curricula(env, table, n, env_index, stream, false);
}


int dxrl_env_reset(dxrl_env* env, const uint8_t* mask, const double* draws, float* obs, void* stream) {
    DXRL_REQUIRE(env, "null env");
    DeviceGuard g(env->device);
    const int64_t n = env->cfg.num_envs;
    hipLaunchKernelGGL(k_reset, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream),
                       env->soa, mask, draws, obs, env->cfg.seed, (int64_t)env->cfg.global_env_offset);
    return launch_check("k_reset");
}

int dxrl_env_step(dxrl_env* env, const float* actions, float* obs, double* reward, uint8_t* terminated,
                  uint8_t* truncated, double* components, void* stream) {
    DXRL_REQUIRE(env && actions && reward && terminated && truncated, "null env/actions/reward/flags");
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(actions) & 15) == 0 && (reinterpret_cast<uintptr_t>(obs) & 15) == 0,
                 "actions/obs must be 16-byte aligned");
    DeviceGuard g(env->device);
    const int64_t n = env->cfg.num_envs;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    const Weights w = weights_of(env->cfg);
    const bool dense = env->cfg.reward_type == DXRL_REWARD_DENSE;
    hipStream_t st = as_stream(stream);
    const int mes = env->cfg.max_episode_steps;
    const char* vs = getenv("DXRL_STEP_VARIANT");
    const int variant = vs ? atoi(vs) & 3 : (n >= kNtLoadMinEnvs ? 3 : (n >= kNtStoreMinEnvs ? 1 : 0));
#define DXRL_STEP_LAUNCH(D, V)                                                                                  \
    hipLaunchKernelGGL((k_step<D, V>), grid, dim3(kBlock), 0, st, env->soa, actions, obs, reward, terminated, \
                       truncated, components, w, mes)
    switch ((dense ? 4 : 0) | variant) {
        case 0: DXRL_STEP_LAUNCH(false, 0); break;
        case 1: DXRL_STEP_LAUNCH(false, 1); break;
        case 2: DXRL_STEP_LAUNCH(false, 2); break;
        case 3: DXRL_STEP_LAUNCH(false, 3); break;
        case 4: DXRL_STEP_LAUNCH(true, 0); break;
        case 5: DXRL_STEP_LAUNCH(true, 1); break;
        case 6: DXRL_STEP_LAUNCH(true, 2); break;
        default: DXRL_STEP_LAUNCH(true, 3); break;
    }
#undef DXRL_STEP_LAUNCH
    return launch_check("k_step");
}

int dxrl_env_set_max_episode_steps(dxrl_env* env, int32_t max_episode_steps) {
    DXRL_REQUIRE(env, "null env");
    env->cfg.max_episode_steps = max_episode_steps;
    return DXRL_OK;
}

int dxrl_reward_compute(int32_t device, int32_t reward_type, const double* weights, int64_t count,
                        int32_t num_fingers, int32_t joints_per_finger, const float* joint_positions,
                        const double* finger_tips, const double* object_position, const float* contacts,
                        float* prev_contacts, uint8_t* has_prev, double* out, void* stream) {
    DXRL_REQUIRE(reward_type == DXRL_REWARD_DENSE || reward_type == DXRL_REWARD_SPARSE,
                 "reward_type must be DXRL_REWARD_DENSE or DXRL_REWARD_SPARSE");
    if (num_fingers != kF || joints_per_finger != kJ) {
        set_error("this build compiles num_fingers=%d, joints_per_finger=%d (got %d, %d)", kF, kJ, num_fingers,
                  joints_per_finger);
        return DXRL_E_UNSUPPORTED;
    }
    DXRL_REQUIRE(count >= 0, "count must be >= 0");
    DXRL_REQUIRE(contacts && out, "null contacts/out");
    const bool dense = reward_type == DXRL_REWARD_DENSE;
    DXRL_REQUIRE(!dense || (weights && joint_positions && finger_tips && object_position && prev_contacts && has_prev),
                 "the dense reward needs weights, joint_positions, finger_tips, object_position and the prev state");
    if (count == 0) return DXRL_OK;
    const Weights w = dense ? Weights{weights[0], weights[1], weights[2], weights[3]} : Weights{0.0, 0.0, 0.0, 0.0};
    DeviceGuard g(device);
    hipLaunchKernelGGL(k_reward_compute, dim3((unsigned)((count + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       as_stream(stream), count, dense, w, joint_positions, finger_tips, object_position, contacts,
                       prev_contacts, has_prev, out);
    return launch_check("k_reward_compute");
}

int dxrl_env_observe(dxrl_env* env, float* obs, void* stream) {
    DXRL_REQUIRE(env && obs, "null env/obs");
    DeviceGuard g(env->device);
    const int64_t n = env->cfg.num_envs;
    hipLaunchKernelGGL(k_observe, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream),
                       env->soa, obs);
    return launch_check("k_observe");
}

}  // extern "C"
