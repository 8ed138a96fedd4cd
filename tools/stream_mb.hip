// Streaming micro-benchmark for k_wgrad_l1's access pattern: 256 workgroups x 512 threads walk
// 20 KB chunks (chunk c of workgroup b at (b + c * grid) * 20 KB, 524 MB in all) three ways:
//   dma   the kernel's LDS-DMA (global_load_lds_dwordx4, waves 0..3 issue five 1 KiB pieces per
//         chunk, a 4-slot LDS ring, one barrier per chunk)
//   reg   every wave loads its 2.5 KiB of the chunk into registers (global_load_dwordx4), the same
//         barrier per chunk, values folded into one XOR so nothing is dead
//   regnb the same without barriers
//   dma2  as dma, but from two buffers like k_wgrad_l1's sources: 16 KB of dH2 rows and 4 KB of
//         observation rows per chunk (four pieces from the first, one from the second per wave)
//   dma2w dma2 right after the whole buffer was rewritten (as dH2 is by the pass before
//         k_wgrad_l1: dirty lines in the caches when the stream starts)
// hipcc --offload-arch=gfx950 -O3 tools/stream_mb.hip -o tools/stream_mb && ./tools/stream_mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kChunk = 20 * 1024, kRing = 4, kGrid = 256, kThreads = 512;

__device__ __forceinline__ void glds_x4(const void* src, const void* lds_dst) {
    const uint32_t lds_addr =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_dst);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_addr)
                 : "memory");
}

template <bool kTwo>
__global__ __launch_bounds__(kThreads, 1) void k_dma(const char* src, int64_t nchunks, uint32_t* out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nch = (int)((nchunks - blockIdx.x + gridDim.x - 1) / gridDim.x);
    const auto issue = [&](int c) {
        if (wave >= 4) return;
        const int64_t g = (int64_t)blockIdx.x + (int64_t)c * gridDim.x;
        char* slot = lds + (c % kRing) * kChunk;
        if (kTwo) {
            const char* y = src + g * 16384;
            const char* x = src + nchunks * 16384 + g * 4096;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int piece = 4 * wave + i;
                glds_x4(y + piece * 1024 + 16 * lane, slot + piece * 1024);
            }
            glds_x4(x + wave * 1024 + 16 * lane, slot + 16384 + wave * 1024);
            return;
        }
        const char* base = src + g * kChunk;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int piece = 5 * wave + i;  // 20 pieces of 1 KiB
            glds_x4(base + piece * 1024 + 16 * lane, slot + piece * 1024);
        }
    };
    for (int c = 0; c < kRing - 1 && c < nch; ++c) issue(c);
    uint32_t acc = 0;
    for (int c = 0; c < nch; ++c) {
        // chunk c landed (at most kRing - 2 younger chunks of 5 pieces in flight)
        if (c + kRing - 2 < nch) __builtin_amdgcn_s_waitcnt(0xF70 | 10);  // vmcnt(10)
        else __builtin_amdgcn_s_waitcnt(0xF70);
        __syncthreads();
        if (c + kRing - 1 < nch) issue(c + kRing - 1);
        acc ^= *reinterpret_cast<const uint32_t*>(lds + (c % kRing) * kChunk + 4 * threadIdx.x);
    }
    out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

template <bool kBarrier>
__global__ __launch_bounds__(kThreads, 1) void k_reg(const char* src, int64_t nchunks, uint32_t* out) {
    const int nch = (int)((nchunks - blockIdx.x + gridDim.x - 1) / gridDim.x);
    uint4 acc = make_uint4(0, 0, 0, 0);
    constexpr int kPer = kChunk / 16 / kThreads;  // 2.5 -> 2 full + a half wave
    for (int c = 0; c < nch; ++c) {
        const char* base = src + ((int64_t)blockIdx.x + (int64_t)c * gridDim.x) * kChunk;
        uint4 v[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int off = 16 * (threadIdx.x + kThreads * u);
            v[u] = off < kChunk ? *reinterpret_cast<const uint4*>(base + off) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            acc.x ^= v[u].x;
            acc.y ^= v[u].y;
            acc.z ^= v[u].z;
            acc.w ^= v[u].w;
        }
        if (kBarrier) __syncthreads();
    }
    (void)kPer;
    out[blockIdx.x * kThreads + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main() {
    const int64_t bytes = 524LL * 1024 * 1024, nchunks = bytes / kChunk;
    char* src;
    uint32_t* out;
    if (hipMalloc(&src, nchunks * kChunk) != hipSuccess || hipMalloc(&out, kGrid * kThreads * 4) != hipSuccess) return 1;
    hipMemset(src, 1, nchunks * kChunk);
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_dma<false>), hipFuncAttributeMaxDynamicSharedMemorySize, kRing * kChunk);
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_dma<true>), hipFuncAttributeMaxDynamicSharedMemorySize, kRing * kChunk);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int v = 0; v < 5; ++v) {
        float best = 1e9f;
        for (int rep = 0; rep < 6; ++rep) {
            if (v == 4) {
                hipMemsetAsync(src, rep, nchunks * kChunk);
                hipDeviceSynchronize();
            }
            hipEventRecord(a);
            if (v == 0) hipLaunchKernelGGL(k_dma<false>, dim3(kGrid), dim3(kThreads), kRing * kChunk, 0, src, nchunks, out);
            if (v == 1) hipLaunchKernelGGL(k_reg<true>, dim3(kGrid), dim3(kThreads), 0, 0, src, nchunks, out);
            if (v == 2) hipLaunchKernelGGL(k_reg<false>, dim3(kGrid), dim3(kThreads), 0, 0, src, nchunks, out);
            if (v >= 3) hipLaunchKernelGGL(k_dma<true>, dim3(kGrid), dim3(kThreads), kRing * kChunk, 0, src, nchunks, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep && ms < best) best = ms;
        }
        printf("%-6s %8.1f us  %.2f TB/s\n", v == 0 ? "dma" : v == 1 ? "reg" : v == 2 ? "regnb" : v == 3 ? "dma2" : "dma2w", best * 1e3,
               (double)nchunks * kChunk / (best * 1e-3) / 1e12);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
