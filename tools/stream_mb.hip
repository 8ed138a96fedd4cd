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
//   w-*   dma2 right after a kernel rewrote the buffer with plain / nt / sc1 / sc0 sc1 stores
// hipcc --offload-arch=gfx950 -O3 tools/stream_mb.hip -o tools/stream_mb && ./tools/stream_mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

// rewrite the buffer with 16-byte vector stores of one cache policy: 0 plain, 1 nt, 2 sc1,
// 3 sc0 sc1 (what the producer of a streamed buffer can choose)
template <int kPol>
__global__ __launch_bounds__(256) void k_fill(uint4* dst, int64_t n16, uint32_t v) {
    const uint4 x = make_uint4(v, v ^ 1u, v ^ 2u, v ^ 3u);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        if (kPol == 0) dst[i] = x;
        if (kPol == 1) {
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(v4u{x.x, x.y, x.z, x.w}, reinterpret_cast<v4u*>(dst + i));
        }
        typedef unsigned int v4r __attribute__((ext_vector_type(4)));
        const v4r xr = {x.x, x.y, x.z, x.w};
        if (kPol == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst + i), "v"(xr) : "memory");
        if (kPol == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dst + i), "v"(xr) : "memory");
    }
}

int main(int argc, char** argv) {
    // argv[1]: MiB streamed (default 524: k_wgrad_l1's bytes per network at C2); smaller sizes
    // show what the memory-side cache (256 MiB) does for a buffer written just before
    const int64_t bytes = (argc > 1 ? atoll(argv[1]) : 524LL) * 1024 * 1024, nchunks = bytes / kChunk;
    char* src;
    uint32_t* out;
    if (hipMalloc(&src, nchunks * kChunk) != hipSuccess || hipMalloc(&out, kGrid * kThreads * 4) != hipSuccess) return 1;
    hipMemset(src, 1, nchunks * kChunk);
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_dma<false>), hipFuncAttributeMaxDynamicSharedMemorySize, kRing * kChunk);
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_dma<true>), hipFuncAttributeMaxDynamicSharedMemorySize, kRing * kChunk);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int v = 0; v < 9; ++v) {
        float best = 1e9f;
        for (int rep = 0; rep < 6; ++rep) {
            if (v == 4) {
                hipMemsetAsync(src, rep, nchunks * kChunk);
                hipDeviceSynchronize();
            }
            if (v >= 5) {  // rewritten by a kernel with store policy v - 5
                const int64_t n16 = nchunks * kChunk / 16;
                uint4* d = reinterpret_cast<uint4*>(src);
                if (v == 5) hipLaunchKernelGGL(k_fill<0>, dim3(2048), dim3(256), 0, 0, d, n16, (uint32_t)rep);
                if (v == 6) hipLaunchKernelGGL(k_fill<1>, dim3(2048), dim3(256), 0, 0, d, n16, (uint32_t)rep);
                if (v == 7) hipLaunchKernelGGL(k_fill<2>, dim3(2048), dim3(256), 0, 0, d, n16, (uint32_t)rep);
                if (v == 8) hipLaunchKernelGGL(k_fill<3>, dim3(2048), dim3(256), 0, 0, d, n16, (uint32_t)rep);
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
        printf("%5lld MiB %-6s %8.1f us  %.2f TB/s\n", (long long)(bytes >> 20), v == 0 ? "dma" : v == 1 ? "reg" : v == 2 ? "regnb" : v == 3 ? "dma2" : v == 4 ? "dma2w" : v == 5 ? "w-plain" : v == 6 ? "w-nt" : v == 7 ? "w-sc1" : "w-sc01", best * 1e3,
               (double)nchunks * kChunk / (best * 1e-3) / 1e12);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
