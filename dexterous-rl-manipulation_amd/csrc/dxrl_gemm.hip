// dxrl_gemm.hip -- bf16 MFMA GEMM with fused epilogues for the actor-critic.
//
// C[M][N] = epi( A[M][K] . Bt[N][K]^T ), f32 accumulate.  Used for every
// dense obs x W contraction of the policy-gradient learner (forward, input
// gradients, weight gradients with split-K over samples).  Workgroup = 4
// waves (2x2), wave tile 64x64 = 2x2 MFMA 32x32x16 tiles, K step 32.
// Operand fragments are loaded straight from global memory (16 B / lane);
// the weight operand is L2-resident (<= 150 KB per matrix), activations
// stream once per column block.
#include "dxrl_internal.h"
#include "dxrl_gemm.h"

using namespace dxrl;

namespace dxrl {

constexpr int kWaveTile = 64, kBlockM = 128, kBlockN = 128;

__global__ __launch_bounds__(256) void k_gemm_bf16(GemmArgs g) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t m0 = (int64_t)blockIdx.x * kBlockM + (wave & 1) * kWaveTile;
    const int n0 = blockIdx.y * kBlockN + (wave >> 1) * kWaveTile;
    const int64_t kb = (int64_t)blockIdx.z * g.k_chunk;
    const int64_t ke = min((int64_t)g.K, kb + g.k_chunk);
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;

    if (n0 < g.N && m0 < g.M) {
        for (int64_t k = kb; k < ke; k += 32) {
            bf16x8 a[2][2], b[2][2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kk = (int)(k + 16 * s + 8 * h);
#pragma unroll
                for (int i = 0; i < 2; ++i) a[s][i] = load_frag(g.A, g.lda, m0 + 32 * i + r, g.M, kk);
#pragma unroll
                for (int j = 0; j < 2; ++j) b[s][j] = load_frag(g.Bt, g.ldb, n0 + 32 * j + r, g.N, kk);
            }
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[s][i], b[s][j], acc[i][j]);
        }
    }
    // ---- epilogue
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + 32 * j + r;
        if (n >= g.N) continue;
        const float bias = g.bias ? g.bias[(int64_t)n * g.bias_stride] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t m = m0 + 32 * i + acc_row(q, lane);
                if (m >= g.M) continue;
                float v = acc[i][j][q];
                if (g.partial) {
                    g.partial[((int64_t)blockIdx.z * g.M + m) * g.N + n] = v;
                    continue;
                }
                v += bias;
                if (g.act == 1) v = tanh_f(v);
                if (g.gate) {
                    const float y = from_bf16(g.gate[m * g.ldg + n]);
                    v = v * (1.0f - y * y);
                }
                if (g.Cf) g.Cf[m * g.ldcf + n] = v;
                if (g.Cffm) g.Cffm[(int64_t)n * g.ldffm + m] = v;
                const bf16 vb = to_bf16(v);
                if (g.Crm) g.Crm[m * g.ldc + n] = vb;
                if (g.Cfm) g.Cfm[(int64_t)n * g.ldfm + m] = vb;
            }
        }
    }
}

// out[i] (+)= sum_z partial[z][i], fixed order (deterministic)
__global__ void k_splitk_reduce(const float* __restrict__ partial, int64_t slab, int z, float* __restrict__ out,
                                int accumulate) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= slab) return;
    float s = 0.0f;
    for (int k = 0; k < z; ++k) s += partial[(int64_t)k * slab + i];
    out[i] = accumulate ? out[i] + s : s;
}

int launch_gemm(const GemmArgs& g0, int splits, float* reduce_out, int accumulate, hipStream_t st) {
    GemmArgs g = g0;
    DXRL_REQUIRE(g.K % 32 == 0 && g.N > 0 && g.M > 0, "gemm: K must be a multiple of 32 (got %d)", g.K);
    DXRL_REQUIRE((g.lda % 8) == 0 && (g.ldb % 8) == 0, "gemm: lda/ldb must be multiples of 8 elements");
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.Bt) & 15) == 0,
                 "gemm: operands must be 16-byte aligned");
    if (splits < 1) splits = 1;
    int64_t chunk = (g.K + splits - 1) / splits;
    chunk = (chunk + 31) / 32 * 32;
    splits = (int)((g.K + chunk - 1) / chunk);
    g.k_chunk = chunk;
    if (splits > 1) DXRL_REQUIRE(g.partial && reduce_out, "gemm: split-K needs a partial slab and an output");
    const dim3 grid((unsigned)((g.M + kBlockM - 1) / kBlockM), (unsigned)((g.N + kBlockN - 1) / kBlockN),
                    (unsigned)splits);
    hipLaunchKernelGGL(k_gemm_bf16, grid, dim3(256), 0, st, g);
    if (int rc = launch_check("k_gemm_bf16")) return rc;
    if (g.partial) {
        const int64_t slab = g.M * (int64_t)g.N;
        hipLaunchKernelGGL(k_splitk_reduce, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, g.partial, slab,
                           splits, reduce_out, accumulate);
        if (int rc = launch_check("k_splitk_reduce")) return rc;
    }
    return DXRL_OK;
}

}  // namespace dxrl

extern "C" {

// Test/diagnostic entry: C = epi(A . Bt^T) (see dxrl.h).
int dxrl_gemm_bf16(int32_t device, const void* A, int64_t lda, const void* Bt, int64_t ldb, int64_t M, int32_t N,
                   int32_t K, const float* bias, int64_t bias_stride, int32_t act, const void* gate, int64_t ldg,
                   float* Cf, int64_t ldcf, void* Crm, int64_t ldc, void* Cfm, int64_t ldfm, float* Cffm,
                   int64_t ldffm, int32_t splits, float* partial, void* stream) {
    DeviceGuard dg(device);
    GemmArgs g{static_cast<const bf16*>(A), lda, static_cast<const bf16*>(Bt), ldb, M, N, K, 0, bias, bias_stride,
               act, static_cast<const bf16*>(gate), ldg, Cf, ldcf, static_cast<bf16*>(Crm), ldc,
               static_cast<bf16*>(Cfm), ldfm, splits > 1 ? partial : nullptr, Cffm, ldffm};
    return launch_gemm(g, splits, splits > 1 ? Cf : nullptr, 0, as_stream(stream));
}

}  // extern "C"
