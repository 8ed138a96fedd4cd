// dxrl_gemm.h -- bf16 MFMA GEMM launcher shared by the learner kernels.
#pragma once
#include "dxrl_internal.h"
#include "dxrl_mfma.h"

namespace dxrl {

struct GemmArgs {
    const bf16* A;
    int64_t lda;
    const bf16* Bt;
    int64_t ldb;
    int64_t M;
    int N, K;
    int64_t k_chunk;        // split-K: K range per blockIdx.z (multiple of 32)
    const float* bias;      // bias[n * bias_stride] (nullable)
    int64_t bias_stride;
    int act;                // 0 identity, 1 tanh
    const bf16* gate;       // (1 - gate[m][n]^2) multiplier (tanh'), nullable
    int64_t ldg;
    float* Cf;              // f32 row-major out (nullable)
    int64_t ldcf;
    bf16* Crm;              // bf16 row-major out (nullable)
    int64_t ldc;
    bf16* Cfm;              // bf16 feature-major out Cfm[n][m] (nullable)
    int64_t ldfm;
    float* partial;         // split-K partial slab [z][M][N] f32 (nullable -> epilogue)
    float* Cffm;            // f32 feature-major out Cffm[n][m] (nullable)
    int64_t ldffm;
};

// Launch C = epi(A . Bt^T); splits > 1 -> split-K partial slabs reduced into
// reduce_out (f32 [M][N], += when accumulate).
int launch_gemm(const GemmArgs& g, int splits, float* reduce_out, int accumulate, hipStream_t st);
// out (+)= sum of z slabs of `slab` floats, deterministic; z > kReduceGroups runs two levels through
// tmp [kReduceGroups][slab] (callers reserve it right after their z partial slabs).
constexpr int kReduceGroups = 16;
// cols > 0: the slab is [rows][cols] and lands in out with row stride ldo.
int launch_slab_reduce(const float* partial, int64_t slab, int z, float* tmp, float* out, int accumulate,
                       hipStream_t st, int cols = 0, int64_t ldo = 0);
// out[O][I] = sum_m Y[m][o] X[m][i] (row-major operands, split-K over m; partial holds
// [splits + kReduceGroups][O][I]).
int launch_wgrad(const bf16* Y, int64_t ldy, int O, const bf16* X, int64_t ldx, int I, int64_t M, int splits,
                 float* partial, float* out, hipStream_t st, int64_t ldo = 0);
// out[256][ldo] = sum_m Y[m][o] tanh(obs[m] . W1^T)[i] for the 256-wide first hidden layer of the
// actor-critic MLP (obs [M][ldobs] bf16, 64 used columns; W1 [256][64]); H1 is recomputed on chip
// exactly as the fused learner's forward computes it.  M % 32 == 0; partial as launch_wgrad.
// reduce = 0: the split-K partials are left for the caller to sum (slab_reduce_block, e.g. in one
// launch with other reductions); returns the number of partial slabs written in *nslabs.
int launch_wgrad_l1(const bf16* Y, int64_t ldy, const bf16* obs, int64_t ldobs, const bf16* W1, int64_t M,
                    int splits, float* partial, float* out, hipStream_t st, int64_t ldo, int reduce = 1,
                    int* nslabs = nullptr);
// Both networks' dW2 in one launch (same observation rows, same M): splits0 workgroups run the
// first contraction, splits1 the second, each split exactly as a single launch_wgrad_l1 with that
// split count would run it (so each net's partial slabs are that launch's); the partials are left
// for the caller to sum (*nslabs0 / *nslabs1 slabs).
int launch_wgrad_l1_pair(const bf16* Y0, const bf16* W10, int splits0, float* partial0, float* out0, const bf16* Y1,
                         const bf16* W11, int splits1, float* partial1, float* out1, int64_t ldy, const bf16* obs,
                         int64_t ldobs, int64_t M, int64_t ldo, hipStream_t st, int* nslabs0, int* nslabs1);

// s += partial[k * stride4 + i] for k = k0 .. k1 - 1, in that order, with the loads issued in
// batches of 8 ahead of their adds (the plain loop waits out one load latency per slab: the
// reductions read their slabs from the Infinity Cache at a fraction of its bandwidth).  Same adds
// in the same order, so bit for bit the plain loop's sum.
__device__ __forceinline__ float4 ordered_slab_sum(const float4* __restrict__ partial, int64_t stride4, int64_t i,
                                                   int k0, int k1, float4 s) {
    constexpr int kB = 8;
    int k = k0;
    for (; k + kB <= k1; k += kB) {
        float4 v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) v[u] = partial[(int64_t)(k + u) * stride4 + i];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            s.x += v[u].x;
            s.y += v[u].y;
            s.z += v[u].z;
            s.w += v[u].w;
        }
    }
    for (; k < k1; ++k) {
        const float4 v = partial[(int64_t)k * stride4 + i];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
    }
    return s;
}

// One 256-thread block of the two-level fixed-order slab sum (k_slab_reduce2_4): float4 columns
// 16 blk .. 16 blk + 15 of z slabs; 16 groups of threads sum contiguous slab ranges, then group 0
// adds the 16 group sums in group order.  grp: the block's [16][16] float4 scratch in LDS.
// Returns the thread's f64 sum of squares of the four values it stored (0 on the other threads;
// unused by callers that do not need a norm, so the compiler drops it there).
__device__ __forceinline__ double slab_reduce_block(const float4* __restrict__ partial, int64_t slab4, int z,
                                                    float* __restrict__ out, int accumulate, int cols, int64_t ldo,
                                                    int64_t blk, float4 (*grp)[16]) {
    constexpr int kRX = 16;
    const int x = threadIdx.x % kRX, g = threadIdx.x / kRX;
    const int64_t i = blk * kRX + x;
    const int k0 = (int)((int64_t)g * z / kReduceGroups), k1 = (int)((int64_t)(g + 1) * z / kReduceGroups);
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (i < slab4) s = ordered_slab_sum(partial, slab4, i, k0, k1, s);
    grp[g][x] = s;
    __syncthreads();
    if (g != 0 || i >= slab4) return 0.0;
    float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int q = 0; q < kReduceGroups; ++q) {
        const float4 v = grp[q][x];
        r.x += v.x;
        r.y += v.y;
        r.z += v.z;
        r.w += v.w;
    }
    const int64_t e = 4 * i;
    const int64_t o = cols ? (e / cols) * ldo + e % cols : e;
    float4* dst = reinterpret_cast<float4*>(out + o);
    if (accumulate) {
        const float4 a = *dst;
        r = make_float4(a.x + r.x, a.y + r.y, a.z + r.z, a.w + r.w);
    }
    *dst = r;
    return (((double)r.x * r.x + (double)r.y * r.y) + (double)r.z * r.z) + (double)r.w * r.w;
}

}  // namespace dxrl
