// Philox4x32-10 latency micro-benchmark: one wave per workgroup, dependent chains
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
struct u4 { uint32_t x, y, z, w; };
__device__ __forceinline__ void mul_a(uint32_t m, uint32_t x, uint32_t& lo, uint32_t& hi) {
    const uint64_t p = (uint64_t)m * x; lo = (uint32_t)p; hi = (uint32_t)(p >> 32);
}
__device__ __forceinline__ void mul_b(uint32_t m, uint32_t x, uint32_t& lo, uint32_t& hi) {
    lo = m * x; hi = __umulhi(m, x);
}
// 16-bit halves through the full-rate 24-bit multiplier
template <uint32_t M>
__device__ __forceinline__ void mul_c(uint32_t x, uint32_t& lo, uint32_t& hi) {
    constexpr uint32_t ml = M & 0xFFFFu, mh = M >> 16;
    const uint32_t xl = x & 0xFFFFu, xh = x >> 16;
    const uint32_t p0 = xl * ml;             // < 2^32
    const uint32_t p1 = xl * mh;
    const uint32_t p2 = xh * ml;
    const uint32_t p3 = xh * mh;
    const uint64_t mid = (uint64_t)p1 + p2;  // < 2^33
    const uint64_t lo64 = (uint64_t)p0 + ((mid & 0xFFFFu) << 16);
    lo = (uint32_t)lo64;
    hi = p3 + (uint32_t)(mid >> 16) + (uint32_t)(lo64 >> 32);
}
template <int V>
__global__ void k(uint32_t* out, int iters, uint32_t seed) {
    u4 c{threadIdx.x ^ seed, seed, 7u, threadIdx.x};
    uint32_t k0 = seed * 3u, k1 = seed * 5u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            uint32_t lo0, hi0, lo1, hi1;
            if (V == 0) { mul_a(0xD2511F53u, c.x, lo0, hi0); mul_a(0xCD9E8D57u, c.z, lo1, hi1); }
            else if (V == 1) { mul_b(0xD2511F53u, c.x, lo0, hi0); mul_b(0xCD9E8D57u, c.z, lo1, hi1); }
            else { mul_c<0xD2511F53u>(c.x, lo0, hi0); mul_c<0xCD9E8D57u>(c.z, lo1, hi1); }
            c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
            k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = c.x ^ c.y ^ c.z ^ c.w;
}
int main() {
    uint32_t* d; hipMalloc(&d, 256 * 64 * 4 * 4);
    uint32_t h[3][64];
    for (int v = 0; v < 3; ++v) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (v == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(64), 0, 0, d, 1000, 12345u);
            if (v == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(64), 0, 0, d, 1000, 12345u);
            if (v == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(64), 0, 0, d, 1000, 12345u);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("variant %d: %.3f ms for 1000 Philox calls per lane (one wave per CU) = %.1f ns per call\n", v, ms, ms * 1e6 / 1000);
        }
        hipMemcpy(h[v], d, 64 * 4, hipMemcpyDeviceToHost);
    }
    int same = 1;
    for (int i = 0; i < 64; ++i) same &= h[0][i] == h[1][i] && h[0][i] == h[2][i];
    printf("results identical: %d\n", same);
    return 0;
}
