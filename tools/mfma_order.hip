// tools/mfma_order.hip -- do v_mfma_f32_16x16x32_bf16 chains round like v_mfma_f32_32x32x16_bf16
// chains over the same k order?  (If yes, 16-row rollout tiles keep the rollout's hidden units
// bit-identical to the learner's 32x32x16 forward.)
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_order tools/mfma_order.hip && tools/mfma_order
//
// One wave: C1 = A Bt^T by 16 chained 32x32x16 MFMAs (K = 256; rows 16..31 of A zero),
// C2 = the same 16 x 32 block by 2 tiles x 8 chained 16x16x32 MFMAs.  Prints the count of
// bitwise-different outputs over many random trials (magnitudes spread over 2^-8 .. 2^8).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>
#include <string.h>
#include <random>
#include <vector>

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int K = 256;

__global__ void k_cmp(const bf16* A, const bf16* Bt, float* C1, float* C2, int trials) {
    const int l = threadIdx.x;
    for (int t = 0; t < trials; ++t) {
        const bf16* a = A + (size_t)t * 32 * K;
        const bf16* b = Bt + (size_t)t * 32 * K;
        // 32x32x16: lane l holds A[l & 31][16k + 8 (l >> 5) ..], Bt[l & 31][...]
        f32x16 acc;
        for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
        const int r = l & 31, h = l >> 5;
        for (int k = 0; k < K / 16; ++k) {
            const bf16x8 fa = *reinterpret_cast<const bf16x8*>(a + r * K + 16 * k + 8 * h);
            const bf16x8 fb = *reinterpret_cast<const bf16x8*>(b + r * K + 16 * k + 8 * h);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
        }
        for (int q = 0; q < 16; ++q) {
            const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
            C1[(size_t)t * 1024 + row * 32 + r] = acc[q];
        }
        // 16x16x32: lane l holds A[l & 15][32k + 8 (l >> 4) ..], Bt[16 j + (l & 15)][...]
        const int r16 = l & 15, g = l >> 4;
        for (int j = 0; j < 2; ++j) {
            f32x4 c = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int k = 0; k < K / 32; ++k) {
                const bf16x8 fa = *reinterpret_cast<const bf16x8*>(a + r16 * K + 32 * k + 8 * g);
                const bf16x8 fb = *reinterpret_cast<const bf16x8*>(b + (16 * j + r16) * K + 32 * k + 8 * g);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, c, 0, 0, 0);
            }
            for (int q = 0; q < 4; ++q) C2[(size_t)t * 512 + (4 * g + q) * 32 + 16 * j + r16] = c[q];
        }
    }
}

int main() {
    const int T = 256;
    std::mt19937 rng(12345);
    std::normal_distribution<float> nd(0.0f, 1.0f);
    std::uniform_real_distribution<float> ud(-8.0f, 8.0f);
    std::vector<bf16> A((size_t)T * 32 * K), B((size_t)T * 32 * K);
    for (int t = 0; t < T; ++t)
        for (int i = 0; i < 32; ++i)
            for (int k = 0; k < K; ++k) {
                const float sa = t % 2 ? 1.0f : exp2f(ud(rng)), sb = t % 2 ? 1.0f : exp2f(ud(rng));
                A[((size_t)t * 32 + i) * K + k] = (bf16)(i < 16 ? nd(rng) * sa : 0.0f);
                B[((size_t)t * 32 + i) * K + k] = (bf16)(nd(rng) * sb);
            }
    bf16 *dA, *dB;
    float *dC1, *dC2;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC1, (size_t)T * 1024 * 4);
    hipMalloc(&dC2, (size_t)T * 512 * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_cmp, dim3(1), dim3(64), 0, 0, dA, dB, dC1, dC2, T);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    std::vector<float> C1((size_t)T * 1024), C2((size_t)T * 512);
    hipMemcpy(C1.data(), dC1, C1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(C2.data(), dC2, C2.size() * 4, hipMemcpyDeviceToHost);
    long diff = 0, total = 0;
    double maxrel = 0.0;
    for (int t = 0; t < T; ++t)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 32; ++j) {
                const float x = C1[(size_t)t * 1024 + i * 32 + j], y = C2[(size_t)t * 512 + i * 32 + j];
                ++total;
                if (memcmp(&x, &y, 4) != 0) {
                    ++diff;
                    const double rel = fabs((double)x - y) / fmax(1e-30, fabs((double)x));
                    if (rel > maxrel) maxrel = rel;
                }
            }
    printf("{\"outputs\": %ld, \"bit_different\": %ld, \"max_rel_diff\": %.3e}\n", total, diff, maxrel);
    return 0;
}
