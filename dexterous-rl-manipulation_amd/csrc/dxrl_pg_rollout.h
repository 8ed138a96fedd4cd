// dxrl_pg_rollout.h -- what the fused policy-gradient rollout kernels share (dxrl_pg.hip: the
// 16-env kernels k_pg_rollout_ws / _ls / k_pg_rollout; dxrl_pg_rollout8.hip: the 32-env kernel
// k_pg_rollout_e8 for >= 32 envs per CU): the launch arguments, the LDS-only barrier and the
// hidden-row swizzle.  No reference counterpart beyond the env step itself.
#pragma once
#include "dxrl_gemm.h"
#include "dxrl_pg.h"

namespace dxrl {

constexpr float kLog2Pi = 1.8378770664093453f;

struct PgRolloutArgs {
    EnvSoA s;
    Weights w;
    int max_episode_steps, max_steps, horizon;
    const bf16* wbf;
    const float* params;
    uint64_t env_seed, policy_seed;
    int64_t gid0;
    uint64_t iteration;
    float obs_noise, dyn_noise;
    bf16* obs_rm;   // [(T+1) N][kIn]
    bf16* obs_fm;   // [kIn][T N]
    float* act;     // [T N][kActPad]
    float* logp;    // [T N]
    float* rew;     // [T N]
    uint8_t* done;  // [T N]
    double* ep_ret; // [N] open-episode return (persists across calls)
    int32_t* ep_count;
    double* ep_sum_ret;
    int32_t* ep_sum_len;
    int32_t* ep_succ;
    int diag;       // timing ablations: bit0 skip actor MLP, bit1 skip env step
    int success_terminated;
    int record_cap;
    double* rec_return;
    int32_t* rec_length;
    uint8_t* rec_success;
    int32_t* rec_end_step;
    uint16_t* ep_code;   // [T N] scheduler feed: 0, or (episode length << 1) | success (nullable)
    float* applied_act;  // [T N][kActPad] the action the env integrated (nullable; parity checks)
    float* dyn_noise_tape;  // [T N][kActPad] f32(sigma) * z as added to the action (nullable; ws kernel)
    float* obs_noise_tape;  // [(T+1) N][kObsNoiseLd] f32(sigma) * z per observation element (nullable)
    bf16* h2_tape;          // [T N][kH2Ld] the actor's layer-2 activations of every step (nullable)
    unsigned long long* stamps;  // diag & 128: cycles per step segment (16- / 32-env kernels)
};
constexpr int kObsNoiseLd = 48;
constexpr int kH2Ld = 264;  // h2_tape row pitch (bf16): the fused learner's H2 tile rows (kHp)

// Workgroup barrier for LDS hand-offs only: __syncthreads() also drains every outstanding
// global store (s_waitcnt vmcnt(0)) before s_barrier, which puts the tape stores' write
// latency on each step's critical path.  Nothing here is handed between waves through global
// memory, so only LDS is fenced.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// hidden rows of 256 bf16 with their 16-byte chunks XOR-swizzled by the row (chunk c of row r < 16
// at chunk c ^ r; the 32-row kernel swizzles row 16 + r like row r): 16-lane fragment reads
// conflict-free, 8-byte epilogue stores 2-way
__device__ __forceinline__ int swz16(int r, int col) { return ((((col >> 3) ^ r) << 3) | (col & 7)); }

// The 32-env rollout (dxrl_pg_rollout8.hip): one workgroup of 8 waves per 32 envs, each env on 8
// lanes.  Same tapes, records and env state as k_pg_rollout_ws bit for bit.
constexpr int kE8Envs = 32;
int launch_pg_rollout_e8(const PgRolloutArgs& p, int64_t n, bool noise, bool diag, hipStream_t st);

}  // namespace dxrl
