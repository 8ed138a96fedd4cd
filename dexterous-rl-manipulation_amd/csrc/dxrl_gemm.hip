// dxrl_gemm.hip -- bf16 MFMA GEMMs with fused epilogues for the actor-critic.
//
// k_gemm_bf16 : C[M][N] = epi(A[M][K] . Bt[N][K]^T)  (forward layers, input grads)
// k_wgrad_bf16: C[O][I] = sum_m Y[m][O] X[m][I]       (weight grads, split-K over samples)
//
// Both stage 128x64 / 64x128 bf16 tiles through LDS with coalesced 16-byte
// global loads (8 or 16 lanes per contiguous row segment), double-buffered
// through registers: the next tile's global loads are issued before the
// current tile's MFMAs.  Workgroup = 4 waves (2x2), wave tile 64x64 =
// 2x2 v_mfma_f32_32x32x16_bf16.  The weight-gradient kernel reads both
// row-major operands k-major straight out of LDS with ds_read_b64_tr_b16
// (gfx950 transpose read, cdna_hip_programming.md T10), so no feature-major
// copy of any activation is ever written.
#include <stdlib.h>

#include "dxrl_internal.h"
#include "dxrl_gemm.h"

using namespace dxrl;

namespace dxrl {

constexpr int kBM = 128, kBN = 128, kBK = 64;
constexpr int kAPitch = kBK + 8;  // 144-B rows: conflict-free ds_read_b128 fragment reads

// ------------------------------------------------------------------ C = A . Bt^T
__global__ __launch_bounds__(256) void k_gemm_bf16(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) bf16 As[kBM * kAPitch];
    __shared__ __attribute__((aligned(16))) bf16 Bs[kBN * kAPitch];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
    const int64_t m0 = (int64_t)blockIdx.x * kBM;
    const int n0 = blockIdx.y * kBN;
    const int64_t kb = (int64_t)blockIdx.z * g.k_chunk;
    const int64_t ke = min((int64_t)g.K, kb + g.k_chunk);
    const bool wave_live = (n0 + wn) < g.N;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;

    // each thread moves 4 A chunks and 4 B chunks of 16 B per tile: chunk c -> row c>>3, col 8*(c&7)
    bf16x8 ra[4], rb[4];
    auto fetch = [&](int64_t k0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = tid + 256 * q, row = c >> 3, col = 8 * (c & 7);
            const int64_t k = k0 + col;
            const int64_t m = m0 + row;
            ra[q] = (m < g.M && k < ke) ? *reinterpret_cast<const bf16x8*>(g.A + m * g.lda + k) : zero8();
            const int n = n0 + row;
            rb[q] = (n < g.N && k < ke) ? *reinterpret_cast<const bf16x8*>(g.Bt + (int64_t)n * g.ldb + k) : zero8();
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = tid + 256 * q, row = c >> 3, col = 8 * (c & 7);
            *reinterpret_cast<bf16x8*>(As + row * kAPitch + col) = ra[q];
            *reinterpret_cast<bf16x8*>(Bs + row * kAPitch + col) = rb[q];
        }
    };
    if (kb < ke) fetch(kb);
    for (int64_t k0 = kb; k0 < ke; k0 += kBK) {
        __syncthreads();  // previous tile's fragment reads are done
        stash();
        __syncthreads();
        if (k0 + kBK < ke) fetch(k0 + kBK);  // overlaps with the MFMAs below
        if (wave_live) {
#pragma unroll
            for (int kk = 0; kk < kBK; kk += 16) {
                bf16x8 a[2], b[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    a[i] = *reinterpret_cast<const bf16x8*>(As + (wm + 32 * i + r) * kAPitch + kk + 8 * h);
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    b[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn + 32 * j + r) * kAPitch + kk + 8 * h);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
            }
        }
    }
    if (!wave_live) return;
    // ---- epilogue
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + 32 * j + r;
        if (n >= g.N) continue;
        const float bias = g.bias ? g.bias[(int64_t)n * g.bias_stride] : 0.0f;
        const float bk = tanh_bias(bias);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t m = m0 + wm + 32 * i + acc_row(q, lane);
                if (m >= g.M) continue;
                float v = acc[i][j][q];
                if (g.partial) {
                    g.partial[((int64_t)blockIdx.z * g.M + m) * g.N + n] = v;
                    continue;
                }
                v = g.act == 1 ? tanh_pre(v, bk) : v + bias;
                if (g.gate) v = tanh_gate(v, from_bf16(g.gate[m * g.ldg + n]));
                if (g.Cf) g.Cf[m * g.ldcf + n] = v;
                if (g.Cffm) g.Cffm[(int64_t)n * g.ldffm + m] = v;
                const bf16 vb = to_bf16(v);
                if (g.Crm) g.Crm[m * g.ldc + n] = vb;
                if (g.Cfm) g.Cfm[(int64_t)n * g.ldfm + m] = vb;
            }
        }
    }
}

// ------------------------------------------------------------------ panel GEMM
// Tall-skinny layers of the learner (M ~ 1e6 samples, N <= 256, K <= 256):
// a workgroup owns a 64-row panel and ALL output columns, so each activation
// row is read from HBM exactly once.  The whole A panel (and the tanh' gate
// panel) is fetched with every 16-byte load in flight at once, then each wave
// computes 64 rows x 64 columns with B fragments from L2; the bf16 result is
// staged in LDS and leaves as full 16-byte-per-lane row segments.
constexpr int kPM = 64, kPK = 256, kPPitch = kPK + 8;  // 528-B LDS rows

__global__ __launch_bounds__(256) void k_gemm_panel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) bf16 Ap[kPM * kPPitch];  // A panel, then the bf16 output stage
    __shared__ __attribute__((aligned(16))) bf16 Gp[kPM * kPPitch];  // gate panel (tanh')
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t m0 = (int64_t)blockIdx.x * kPM;
    const int K = g.K, Nn = g.N;
    const int kc = K >> 3;  // 16-byte chunks per row
    // ---- panel loads: every chunk of the A (and gate) panel in flight together
    {
        bf16x8 ta[8], tg[8];
        const int na = kPM * kc, ng = g.gate ? kPM * (Nn >> 3) : 0, gc = Nn >> 3;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = tid + 256 * q;
            if (c < na) {
                const int64_t m = m0 + c / kc;
                ta[q] = m < g.M ? *reinterpret_cast<const bf16x8*>(g.A + m * g.lda + 8 * (c % kc)) : zero8();
            }
            if (c < ng) {
                const int64_t m = m0 + c / gc;
                tg[q] = m < g.M ? *reinterpret_cast<const bf16x8*>(g.gate + m * g.ldg + 8 * (c % gc)) : zero8();
            }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = tid + 256 * q;
            if (c < na) *reinterpret_cast<bf16x8*>(Ap + (c / kc) * kPPitch + 8 * (c % kc)) = ta[q];
            if (c < ng) *reinterpret_cast<bf16x8*>(Gp + (c / gc) * kPPitch + 8 * (c % gc)) = tg[q];
        }
    }
    __syncthreads();
    const int wn = 64 * wave;
    const bool live = wn < Nn;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;
    if (live) {
        const bf16* B0 = g.Bt + (int64_t)(wn + r) * g.ldb + 8 * h;
        const bf16* B1 = g.Bt + (int64_t)(wn + 32 + r) * g.ldb + 8 * h;
        const bool b1ok = wn + 32 + r < Nn, b0ok = wn + r < Nn;
        // B fragments (weights, L2-resident): issue four k-steps of loads ahead of their MFMAs
        for (int k0 = 0; k0 < K; k0 += 64) {
            bf16x8 b0[4], b1[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = k0 + 16 * s;
                b0[s] = (b0ok && k < K) ? *reinterpret_cast<const bf16x8*>(B0 + k) : zero8();
                b1[s] = (b1ok && k < K) ? *reinterpret_cast<const bf16x8*>(B1 + k) : zero8();
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = k0 + 16 * s;
                if (k >= K) break;
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Ap + r * kPPitch + k + 8 * h);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Ap + (32 + r) * kPPitch + k + 8 * h);
                acc[0][0] = mfma32(a0, b0[s], acc[0][0]);
                acc[0][1] = mfma32(a0, b1[s], acc[0][1]);
                acc[1][0] = mfma32(a1, b0[s], acc[1][0]);
                acc[1][1] = mfma32(a1, b1[s], acc[1][1]);
            }
        }
    }
    __syncthreads();  // A panel reads done: Ap becomes the output stage
    if (live) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = wn + 32 * j + r;
            const bool nv = n < Nn;
            const float bias = (g.bias && nv) ? g.bias[(int64_t)n * g.bias_stride] : 0.0f;
            const float bk = tanh_bias(bias);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int row = 32 * i + acc_row(q, lane);
                    const int64_t m = m0 + row;
                    float v = g.act == 1 ? tanh_pre(acc[i][j][q], bk) : acc[i][j][q] + bias;
                    if (g.gate) v = tanh_gate(v, from_bf16(Gp[row * kPPitch + n]));
                    if (nv && m < g.M) {
                        if (g.Cf) g.Cf[m * g.ldcf + n] = v;
                        if (g.Cffm) g.Cffm[(int64_t)n * g.ldffm + m] = v;
                    }
                    Ap[row * kPPitch + n] = to_bf16(v);
                }
        }
    }
    if (!g.Crm) return;
    __syncthreads();
    const int nc = Nn >> 3;
    for (int c = tid; c < kPM * nc; c += 256) {
        const int row = c / nc, col = 8 * (c % nc);
        const int64_t m = m0 + row;
        if (m < g.M) *reinterpret_cast<bf16x8*>(g.Crm + m * g.ldc + col) =
            *reinterpret_cast<const bf16x8*>(Ap + row * kPPitch + col);
    }
}

static bool panel_ok(const GemmArgs& g, int splits) {
    return splits == 1 && !g.partial && !g.Cfm && g.K <= kPK && g.N <= 256 && (g.N % 8) == 0 && (g.ldc % 8) == 0 &&
           (!g.gate || (g.ldg % 8) == 0) && (reinterpret_cast<uintptr_t>(g.Crm) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(g.gate) & 15) == 0;
}

// ------------------------------------------------------------------ C[O][I] = Y^T X
// LDS images are [64 samples][128 features] bf16 with 320-B rows: the
// transposed reads (rows 16kk + 8(g>>1) + q, columns 16(g&1) + 4p of a
// 16-lane group g) then touch all 64 banks once per 32-lane half.
constexpr int kWO = 128, kWI = 128, kWK = 64, kWPitch = 128 + 32;

struct WgradArgs {
    const bf16* Y;  // [M][ldy], O used columns
    int64_t ldy;
    const bf16* X;  // [M][ldx], I used columns
    int64_t ldx;
    int O, I;
    int64_t M, m_chunk;
    float* out;      // [O][ldo] f32 (splits == 1)
    float* partial;  // [splits][O][I] (splits > 1)
    int64_t ldo;     // output row stride (>= I)
    int diag;        // timing ablation (DXRL_WGRAD_DIAG): 1 = stream only, no fragment reads / MFMAs
    const bf16* W1;  // k_wgrad_l1: [256][64] first-layer weights (X is then the observation matrix)
};

__global__ __launch_bounds__(256) void k_wgrad_bf16(WgradArgs w) {
    __shared__ __attribute__((aligned(16))) bf16 Ys[kWK * kWPitch];
    __shared__ __attribute__((aligned(16))) bf16 Xs[kWK * kWPitch];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wo = (wave & 1) * 64, wi = (wave >> 1) * 64;
    const int o0 = blockIdx.x * kWO, i0 = blockIdx.y * kWI;
    const int64_t mb = (int64_t)blockIdx.z * w.m_chunk;
    const int64_t me = min(w.M, mb + w.m_chunk);
    const bool wave_live = (o0 + wo) < w.O && (i0 + wi) < w.I;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.0f;
    // tile = 64 rows x 16 chunks of 16 B: chunk c -> row c >> 4, col 8 (c & 15)
    bf16x8 ry[4], rx[4];
    auto fetch = [&](int64_t m0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = tid + 256 * q, row = c >> 4, col = 8 * (c & 15);
            const int64_t m = m0 + row;
            const bool mv = m < me;
            ry[q] = (mv && o0 + col < w.O) ? *reinterpret_cast<const bf16x8*>(w.Y + m * w.ldy + o0 + col) : zero8();
            rx[q] = (mv && i0 + col < w.I) ? *reinterpret_cast<const bf16x8*>(w.X + m * w.ldx + i0 + col) : zero8();
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = tid + 256 * q, row = c >> 4, col = 8 * (c & 15);
            *reinterpret_cast<bf16x8*>(Ys + row * kWPitch + col) = ry[q];
            *reinterpret_cast<bf16x8*>(Xs + row * kWPitch + col) = rx[q];
        }
    };
    if (mb < me) fetch(mb);
    for (int64_t m0 = mb; m0 < me; m0 += kWK) {
        __syncthreads();
        stash();
        __syncthreads();
        if (m0 + kWK < me) fetch(m0 + kWK);
        // every lane of the wave issues the transposed reads (EXEC must be all ones)
#pragma unroll
        for (int kk = 0; kk < kWK; kk += 16) {
            bf16x8 a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = tr_frag<kWPitch>(Ys, wo + 32 * i, kk, lane);
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = tr_frag<kWPitch>(Xs, wi + 32 * j, kk, lane);
            if (wave_live) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
            }
        }
    }
    if (!wave_live) return;
    float* dst = w.partial ? w.partial + (int64_t)blockIdx.z * w.O * w.I : w.out;
    const int64_t ld = w.partial ? w.I : w.ldo;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = i0 + wi + 32 * j + (lane & 31);
        if (i >= w.I) continue;
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int o = o0 + wo + 32 * ii + acc_row(q, lane);
                if (o < w.O) dst[(int64_t)o * ld + i] = acc[ii][j][q];
            }
    }
}

// ------------------------------------------------------------------ whole-output weight gradient
// k_wgrad_full: C[O][I] = sum_m Y[m][o] X[m][i] for O, I <= 256 (the learner's dW2 = dH2^T H1;
// the bias column is summed by the fused kernel).  Every workgroup owns a contiguous range of
// samples and the WHOLE output (8 waves x 32 output rows x 8 column tiles = 128 accumulator
// registers per lane), so each activation row is read from HBM exactly once -- the tiled
// k_wgrad_bf16 re-reads Y once per column tile and X once per row tile.  64-sample chunks are
// staged through two LDS buffers (576-B rows: conflict-free transposed reads); two chunks'
// global loads are in flight in registers while the current chunk's MFMAs run (one chunk per
// CU in flight left HBM at 3.6 TB/s).  Partials [grid][O][I] are summed in a fixed order.
constexpr int kFO = 256, kFI = 256, kFK = 64, kFPitch = 288;
constexpr int kFPieces = kFK * (kFO / 8 + kFI / 8), kFPer = (kFPieces + 511) / 512;

// Chunk loads through buffer descriptors based at the workgroup's first row: rows past the end
// of the array come back as zeros from the hardware range check, so every load is issued
// unconditionally (no per-piece branch) and the wait for a chunk is a counted vmcnt that leaves
// the next chunk in flight.  Columns past O / I only feed accumulator rows / columns that are
// never stored.
template <int kU>
__device__ __forceinline__ void wfull_fetch(__amdgpu_buffer_rsrc_t ry, __amdgpu_buffer_rsrc_t rx, int64_t ldy,
                                            int64_t ldx, int64_t r0, int tid, bf16x8 (&v)[kU]) {
    asm volatile("" : "+v"(tid));  // recompute the piece offsets per chunk (not hoisted into registers)
    static_assert(kFK * (kFO / 8) == 4 * 512, "pieces 0..3 of a thread are Y, 4..7 are X");
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const bool isy = u < 4;  // compile-time per piece: one uniform descriptor per load
        const int cc = tid + 512 * (isy ? u : u - 4);
        const int row = cc >> 5, col = 8 * (cc & 31);
        const int64_t m = r0 + row;  // row relative to the workgroup's first row
        const auto t = isy ? __builtin_amdgcn_raw_buffer_load_b128(ry, (int)((m * ldy + col) * 2), 0, 0)
                           : __builtin_amdgcn_raw_buffer_load_b128(rx, (int)((m * ldx + col) * 2), 0, 0);
        v[u] = __builtin_bit_cast(bf16x8, t);
    }
}

template <int kU>
__device__ __forceinline__ void wfull_stash(bf16* Ysb, bf16* Xsb, int tid, const bf16x8 (&v)[kU]) {
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int c = tid + 512 * u;
        const bool isy = c < kFK * (kFO / 8);
        const int cc = isy ? c : c - kFK * (kFO / 8);
        const int row = cc >> 5, col = 8 * (cc & 31);
        *reinterpret_cast<bf16x8*>((isy ? Ysb : Xsb) + row * kFPitch + col) = v[u];
    }
}

__global__ __launch_bounds__(512, 1) void k_wgrad_full(WgradArgs w) {
    extern __shared__ __attribute__((aligned(16))) bf16 fsm[];
    bf16* const Y0 = fsm;
    bf16* const Y1 = fsm + kFK * kFPitch;
    bf16* const X0 = fsm + 2 * kFK * kFPitch;
    bf16* const X1 = fsm + 3 * kFK * kFPitch;
    const bf16* const Y = w.Y;
    const bf16* const X = w.X;
    const int64_t ldy = w.ldy, ldx = w.ldx;
    const int O = w.O, I = w.I;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t mb = (int64_t)blockIdx.x * w.m_chunk;
    const int64_t me = min(w.M, mb + w.m_chunk);
    const bool wave_live = 32 * wave < O;
    f32x16 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[j][q] = 0.0f;
    const auto compute = [&](const bf16* Ysb, const bf16* Xsb) {
#pragma unroll
        for (int kk = 0; kk < kFK; kk += 16) {
            // issue every fragment of this k-step before its MFMAs (one LDS latency per k-step,
            // not one per MFMA)
            const bf16x8 a = tr_frag<kFPitch>(Ysb, 32 * wave, kk, lane);
            bf16x8 bb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) bb[j] = tr_frag<kFPitch>(Xsb, 32 * j, kk, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (wave_live) acc[j] = mfma32(a, bb[j], acc[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // LDS-only barrier: the register-staged loads of the chunks in flight must survive it
    // (__syncthreads' fence would drain them with vmcnt(0))
    const auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // descriptors from wave-uniform values: based at row mb, bounded by the array end (M rows)
    const int64_t yb = min((int64_t)0x7fffffff, (w.M - mb) * ldy * 2), xb = min((int64_t)0x7fffffff, (w.M - mb) * ldx * 2);
    const auto uniform_ptr = [](const void* q) {
        const uint64_t a = reinterpret_cast<uint64_t>(q);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
        return reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    };
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(Y + mb * ldy), 0,
                                                                        __builtin_amdgcn_readfirstlane((int)yb), 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(X + mb * ldx), 0,
                                                                        __builtin_amdgcn_readfirstlane((int)xb), 0x00020000);
    bf16x8 f0[kFPer], f1[kFPer];
    wfull_fetch(ry, rx, ldy, ldx, 0, tid, f0);
    wfull_stash(Y0, X0, tid, f0);
    wfull_fetch(ry, rx, ldy, ldx, kFK, tid, f0);  // chunk 1 in flight
    __syncthreads();
    // chunk c sits in LDS buffer c & 1, chunk c + 1 in registers; chunk c + 2 is issued first.
    // Chunks past the workgroup's range are fetched but never computed; rows past M read as 0.
    for (int64_t m0 = mb; m0 < me; m0 += 2 * kFK) {
        wfull_fetch(ry, rx, ldy, ldx, m0 - mb + 2 * kFK, tid, f1);
        compute(Y0, X0);
        lds_barrier();  // every wave is done reading buffer 1 (chunk c - 1)
        wfull_stash(Y1, X1, tid, f0);
        lds_barrier();
        if (m0 + kFK >= me) break;
        wfull_fetch(ry, rx, ldy, ldx, m0 - mb + 3 * kFK, tid, f0);
        compute(Y1, X1);
        lds_barrier();
        wfull_stash(Y0, X0, tid, f1);
        lds_barrier();
    }
    if (!wave_live) return;
    float* dst = w.partial ? w.partial + (int64_t)blockIdx.x * O * I : w.out;
    const int64_t ld = w.partial ? I : w.ldo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = 32 * j + (lane & 31);
        if (i >= I) continue;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int o = 32 * wave + acc_row(q, lane);
            if (o < O) dst[(int64_t)o * ld + i] = acc[j][q];
        }
    }
}

// ------------------------------------------------------------------ dW2 via LDS-DMA
// k_wgrad_glds: the same whole-output contraction for O = I = 256 with the sample chunks
// streamed HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging): a 4-buffer ring of
// 32-sample chunks keeps three chunks (96 KB per CU) in flight across raw s_barriers with
// counted vmcnt waits.  LDS rows are 512 B unpadded; the 16-byte chunks of row r are XOR-
// swizzled by 4 (r & 3) on the SOURCE address (the LDS-DMA destination is lane-linear), which
// keeps the transposed fragment reads conflict-free.
constexpr int kGK = 32, kGNB = 4, kGRowB = 512;
constexpr int kGChunkB = 2 * kGK * kGRowB;  // Y + X bytes of one chunk

__device__ __forceinline__ bf16x8 tr_frag_swz(const bf16* tile, int col0, int kk, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p;
    lds_bf16* base = (lds_bf16*)(tile);
    const auto at = [&](int row) {
        return (lds_bf16x4*)(base + row * (kGRowB / 2) + (((col >> 3) ^ (4 * (row & 3))) << 3) + (col & 7));
    };
    const int row = kk + 8 * (g >> 1) + q;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(at(row));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(at(row + 4));
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = lo[j];
        v[4 + j] = hi[j];
    }
    return v;
}

__global__ __launch_bounds__(512, 1) void k_wgrad_glds(WgradArgs w) {
    extern __shared__ __attribute__((aligned(16))) char gsm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // chunks blockIdx.x, blockIdx.x + grid, ...: at any moment the workgroups stream neighbouring
    // 32-row chunks, spread over all HBM channels (contiguous per-workgroup ranges 1.6 MB apart
    // made every CU hit the same channels in lockstep)
    const int64_t total = w.M / kGK;
    const int nch = (int)((total - blockIdx.x + gridDim.x - 1) / gridDim.x);
    const bf16* const Y = w.Y;
    const bf16* const X = w.X;
    const int64_t ldy = w.ldy, ldx = w.ldx;
    f32x16 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[j][q] = 0.0f;
    // chunk c -> ring slot c % 4; wave w issues pieces 4w .. 4w + 3 (2 rows of Y or X each)
    const auto issue = [&](int c) {
        char* buf = gsm + (c % kGNB) * kGChunkB;
        const int64_t m0 = ((int64_t)blockIdx.x + (int64_t)c * gridDim.x) * kGK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = 4 * wave + i;
            const bool isy = pc < 16;
            const int prow = 2 * (pc & 15);
            const int r = prow + (lane >> 5), slot = lane & 31;
            const int gchunk = slot ^ (4 * (r & 3));
            const bf16* src = isy ? Y + (m0 + r) * ldy + 8 * gchunk : X + (m0 + r) * ldx + 8 * gchunk;
            char* dst = buf + (isy ? 0 : kGK * kGRowB) + prow * kGRowB;
            // issued from inline asm so the compiler's waitcnt pass does not see an LDS write in
            // flight (it would put vmcnt(0) before every LDS read); the counted waits below own it
            const uint32_t lds_addr = __builtin_amdgcn_readfirstlane(
                (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)dst);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(src), "s"(lds_addr)
                : "memory");
        }
    };
#pragma unroll
    for (int c = 0; c < 3; ++c)
        if (c < nch) issue(c);
    for (int c = 0; c < nch; ++c) {
        // chunk c has landed once at most the chunks issued after it are outstanding
        const int after = min(2, nch - 1 - c);
        if (after == 2) __builtin_amdgcn_s_waitcnt(0xF78);       // vmcnt(8)
        else if (after == 1) __builtin_amdgcn_s_waitcnt(0xF74);  // vmcnt(4)
        else __builtin_amdgcn_s_waitcnt(0xF70);                  // vmcnt(0)
        __builtin_amdgcn_s_barrier();  // every wave's DMA for chunk c is in; compute(c - 1) is done
        if (c + 3 < nch) issue(c + 3);  // into the slot compute(c - 1) just released
        const bf16* Ys = (const bf16*)(gsm + (c % kGNB) * kGChunkB);
        const bf16* Xs = (const bf16*)(gsm + (c % kGNB) * kGChunkB + kGK * kGRowB);
        if (w.diag & 1) continue;
        // both k-steps' fragments are issued before the first MFMA (one LDS latency per chunk)
        bf16x8 a[2], bb[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            a[h] = tr_frag_swz(Ys, 32 * wave, 16 * h, lane);
#pragma unroll
            for (int j = 0; j < 8; ++j) bb[h][j] = tr_frag_swz(Xs, 32 * j, 16 * h, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = mfma32(a[h], bb[h][j], acc[j]);
        __builtin_amdgcn_sched_barrier(0);
    }
    float* dst = w.partial ? w.partial + (int64_t)blockIdx.x * w.O * w.I : w.out;
    const int64_t ld = w.partial ? w.I : w.ldo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = 32 * j + (lane & 31);
#pragma unroll
        for (int q = 0; q < 16; ++q) dst[(int64_t)(32 * wave + acc_row(q, lane)) * ld + i] = acc[j][q];
    }
}

// k_wgrad_l1: dW2 = dH2^T H1 without H1 in HBM.  H1 = tanh(obs W1^T) is recomputed per 32-sample
// chunk from the 128-byte observation rows (a quarter of H1's bytes) with exactly the fused
// learner's L1 sequence -- same MFMA, operand roles, k order and tanh -- so the bf16 H1 is bit for
// bit the one the learner's forward used (test_h1_recompute_is_bit_exact).  The chunk ring is
// k_wgrad_glds's (dH2 rows 512 B, source-swizzled by 4 (r & 3)); observation rows land 128 B
// unpadded with their 16-byte chunks swizzled by (r >> 1) & 7, which keeps the row-fragment reads
// conflict-free.  Waves 0..3 issue every LDS-DMA op of a chunk (each: four dH2 pieces of 2 rows,
// one piece of 8 observation rows); waves 4..7 issue none (below).  Software-pipelined by one chunk: iteration c recomputes
// H1(c + 1) into one of two H1 buffers while contracting chunk c against the other, one barrier per
// chunk; the H1(c + 1) products sit between the two k-steps of chunk c in the MFMA pipe, so their
// tanh issues on the VALU while the second k-step runs on the matrix cores.
#ifndef DXRL_WL1_RING
#define DXRL_WL1_RING 4  // chunk slots (4: 166 us, 5: 174 us per 819 k rows, kernel-level A/B)
#endif
constexpr int kLK = 32, kLNB = DXRL_WL1_RING;
constexpr int kLYB = kLK * 512, kLXB = kLK * 128, kLSlot = kLYB + kLXB;
constexpr int kLH1 = kLNB * kLSlot;          // two recomputed H1 chunks [32][256] (h1_swz rows)
constexpr int kLLds = kLH1 + 2 * kLK * 512;  // 112 KiB at 4 slots

// one 16-byte-per-lane LDS-DMA piece (non-temporal loads of the read-once dH2 stream measured
// within noise, profiles/r05/ab_dh2_nt.log: removed in round 6)
__device__ __forceinline__ void glds_x4(const void* src, const void* lds_dst) {
    const uint32_t lds_addr =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_dst);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_addr)
                 : "memory");
}

// H1 chunk layout: 512-B rows, 16-byte chunk c of row r at c ^ (4 (r & 3) ^ ((r >> 2) & 3)).  The
// 4 (r & 3) term keeps the transposed reads conflict-free (as tr_frag_swz); the (r >> 2) & 3 term
// spreads the 16 rows of one ds_write_b64 lane group over 8 chunk slots (2-way, not 8-way).
__device__ __forceinline__ int h1_swz(int row) { return (4 * (row & 3)) ^ ((row >> 2) & 3); }
__device__ __forceinline__ bf16x8 tr_frag_h1(const bf16* tile, int col0, int kk, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 16 * (g & 1) + 4 * p;
    lds_bf16* base = (lds_bf16*)(tile);
    const auto at = [&](int row) {
        return (lds_bf16x4*)(base + row * 256 + (((col >> 3) ^ h1_swz(row)) << 3) + (col & 7));
    };
    const int row = kk + 8 * (g >> 1) + q;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(at(row));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(at(row + 4));
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = lo[j];
        v[4 + j] = hi[j];
    }
    return v;
}

// Which waves issue a chunk's LDS-DMA pieces.  1 (default): waves 0..3 five each (four dH2, one
// observation piece), waves 4..7 none; 0: every wave three (two dH2 pieces, one half-wave
// observation piece).  The first-dispatched half waits at the chunk barrier for its SIMD partners,
// so the pieces' issue cost (~0.4 k cycles per wave and chunk) moves into that slack: 182 -> 171
// us per 819 k rows (kernel-level A/B; the second half issuing them: 180 us)
#ifndef DXRL_WL1_DMA_HALF
#define DXRL_WL1_DMA_HALF 1
#endif
// s_waitcnt vmcnt(k n) (n = 0..4 chunks of k LDS-DMA ops each still in flight)
// (gfx9 vmcnt: 6 bits, the low four at [3:0] and the high two at [15:14])
constexpr int vmcnt_imm(int v) { return 0xF70 | (v & 15) | ((v >> 4) << 14); }
template <int k>
__device__ __forceinline__ void wait_chunks_k(int n) {
    static_assert(4 * k <= 63, "vmcnt field");
    if (n >= 4) __builtin_amdgcn_s_waitcnt(vmcnt_imm(4 * k));
    else if (n == 3) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * k));
    else if (n == 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * k));
    else if (n == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(k));
    else __builtin_amdgcn_s_waitcnt(0xF70);
}
__device__ __forceinline__ void wait_chunks(int n) { wait_chunks_k<3>(n); }

// kDiag: the DXRL_WGRAD_DIAG ablations compiled in (a run-time branch in the chunk loop costs the
// production kernel measurable time)
// Two contractions in one launch (both networks' dW2 of a PPO step): workgroups [0, nb0) run n[0]
// over nb0 splits, the rest n[1] over gridDim.x - nb0; a single contraction sets nb0 = gridDim.x.
struct WgradPair {
    WgradArgs n[2];
    int nb0;
};
template <bool kDiag>
__global__ __launch_bounds__(512, 1) void k_wgrad_l1(WgradPair pr) {
    extern __shared__ __attribute__((aligned(16))) char gsm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const bool second = (int)blockIdx.x >= pr.nb0;
    const WgradArgs& w = second ? pr.n[1] : pr.n[0];
    // this workgroup's split of its contraction and the contraction's split count
    const int bx = second ? (int)blockIdx.x - pr.nb0 : (int)blockIdx.x;
    const int gx = second ? (int)gridDim.x - pr.nb0 : pr.nb0;
    const int64_t total = w.M / kLK;
    const int nch = (int)((total - bx + gx - 1) / gx);
    const bf16* const Y = w.Y;
    const bf16* const X = w.X;
    const int64_t ldy = w.ldy, ldx = w.ldx;
    f32x16 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[j][q] = 0.0f;
    // this wave's 32 hidden units of W1 (A operand of the recompute), register-resident
    bf16x8 w1f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w1f[k] = *(const __attribute__((address_space(1))) bf16x8*)(w.W1 + (32 * wave + r) * 64 + 16 * k + 8 * h);
#if DXRL_WL1_DMA_HALF
    // the issuing half: wave q = wave mod 4 loads dH2 rows 8 q .. 8 q + 7 and observation rows 8 q ..
    const bool dma_wave = __builtin_amdgcn_readfirstlane(wave) < 4;
    const auto wait_in = [&](int n) {
        if (dma_wave) wait_chunks_k<5>(n);
        else __builtin_amdgcn_s_waitcnt(0xF70);
    };
    const auto issue = [&](int c) {
        if (!dma_wave) return;
        const int q = wave & 3;
        char* slot = gsm + (c % kLNB) * kLSlot;
        const int64_t m0 = ((int64_t)bx + (int64_t)c * gx) * kLK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // dH2 rows 8 q + 2 i, + 1
            const int prow = 8 * q + 2 * i;
            const int rr = prow + (lane >> 5), gchunk = (lane & 31) ^ (4 * (rr & 3));
            glds_x4(Y + (m0 + rr) * ldy + 8 * gchunk, slot + prow * 512);
        }
        {  // observation rows 8 q .. + 7
            const int row = 8 * q + (lane >> 3), pc = (lane & 7) ^ ((row >> 1) & 7);
            glds_x4(X + (m0 + row) * ldx + 8 * pc, slot + kLYB + 1024 * q);
        }
    };
#else
    const auto wait_in = [](int n) { wait_chunks(n); };
    const auto issue = [&](int c) {
        char* slot = gsm + (c % kLNB) * kLSlot;
        const int64_t m0 = ((int64_t)bx + (int64_t)c * gx) * kLK;
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // dH2 rows 4 wave + 2 i, + 1
            const int prow = 4 * wave + 2 * i;
            const int rr = prow + (lane >> 5), gchunk = (lane & 31) ^ (4 * (rr & 3));
            glds_x4(Y + (m0 + rr) * ldy + 8 * gchunk, slot + prow * 512);
        }
        if (lane < 32) {  // observation rows 4 wave .. + 3
            const int row = 4 * wave + (lane >> 3), pc = (lane & 7) ^ ((row >> 1) & 7);
            glds_x4(X + (m0 + row) * ldx + 8 * pc, slot + kLYB + 512 * wave);
        }
    };
#endif
    // H1[32 samples][hidden 32 wave ..] of chunk c = tanh(obs W1^T): the fused learner's L1, one tile
    // (products and tanh split so the caller can put MFMA work between them)
    const auto recompute_mfma = [&](int c, f32x16& ha) {
        const bf16* Os = (const bf16*)(gsm + (c % kLNB) * kLSlot + kLYB);
        bf16x8 b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = *reinterpret_cast<const bf16x8*>(Os + r * 64 + 8 * ((2 * k + h) ^ ((r >> 1) & 7)));
#pragma unroll
        for (int q = 0; q < 16; ++q) ha[q] = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) ha = mfma32(w1f[k], b[k], ha);
    };
    const auto recompute_store = [&](int c, const f32x16& ha) {
        bf16* H1 = (bf16*)(gsm + kLH1 + (c & 1) * kLK * 512);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f0 = 32 * wave + 8 * g + 4 * h;
            bf16x4 v;
#pragma unroll
            for (int u = 0; u < 4; u += 2) {
                const f32x2 t = tanh_pre2(f32x2{ha[4 * g + u], ha[4 * g + u + 1]}, f32x2{0.0f, 0.0f});
                v[u] = to_bf16(t.x);
                v[u + 1] = to_bf16(t.y);
            }
            *reinterpret_cast<bf16x4*>(H1 + r * 256 + (((f0 >> 3) ^ h1_swz(r)) << 3) + (f0 & 7)) = v;
        }
    };
    // dW2 += dH2(c)^T H1(c), k-step hh (16 samples)
    const auto contract = [&](int c, int hh) {
        const bf16* Ys = (const bf16*)(gsm + (c % kLNB) * kLSlot);
        const bf16* H1 = (const bf16*)(gsm + kLH1 + (c & 1) * kLK * 512);
        bf16x8 bb[8];
        const bf16x8 a = tr_frag_swz(Ys, 32 * wave, 16 * hh, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = tr_frag_h1(H1, 32 * j, 16 * hh, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = mfma32(a, bb[j], acc[j]);
    };
    constexpr int kLead = kLNB - 1;  // chunks in flight ahead of the one being contracted
#pragma unroll
    for (int c = 0; c < kLead; ++c)
        if (c < nch) issue(c);
    if (nch > 0) {
        wait_in(min(kLead - 1, nch - 1));  // chunk 0 in
        __builtin_amdgcn_s_barrier();
        f32x16 ha;
        recompute_mfma(0, ha);
        recompute_store(0, ha);
    }
    for (int c = 0; c < nch; ++c) {
        // chunk c + 1 in (chunks c + 2 .. c + kLead - 1 may still fly); H1(c) complete; chunk c - 1 done
        wait_in(max(0, min(kLead - 2, nch - 2 - c)));
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (c + kLead < nch) issue(c + kLead);  // into the slot chunk c - 1 released
        const bool next = c + 1 < nch && !(kDiag && (w.diag & 2)), mm = !(kDiag && (w.diag & 1));
        if (mm) contract(c, 0);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 ha;
        if (next) recompute_mfma(c + 1, ha);
        __builtin_amdgcn_sched_barrier(0);
        if (mm) contract(c, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (next) recompute_store(c + 1, ha);
    }
    float* dst = w.partial ? w.partial + (int64_t)bx * 256 * 256 : w.out;
    const int64_t ld = w.partial ? 256 : w.ldo;
    if (kDiag && (w.diag & 4)) return;  // ablation: no partial-slab stores
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = 32 * j + (lane & 31);
#pragma unroll
        for (int q = 0; q < 16; ++q) dst[(int64_t)(32 * wave + acc_row(q, lane)) * ld + i] = acc[j][q];
    }
}

namespace {
int wgrad_l1_args(const bf16* Y, int64_t ldy, const bf16* obs, int64_t ldobs, const bf16* W1, int64_t M, int& splits,
                  float* partial, float* out, int64_t ldo, WgradArgs& w) {
    DXRL_REQUIRE(Y && obs && W1 && out && M > 0 && M % kLK == 0, "wgrad_l1: M must be a positive multiple of %d", kLK);
    DXRL_REQUIRE(ldy >= 256 && ldy % 8 == 0 && ldobs >= 64 && ldobs % 8 == 0 && ldo >= 256, "wgrad_l1: bad strides");
    if (splits < 1) splits = 1;
    if (splits > M / kLK) splits = (int)(M / kLK);
    if (splits > 1) DXRL_REQUIRE(partial, "wgrad_l1: split-K needs a partial slab");
    w = WgradArgs{};
    w.Y = Y;
    w.ldy = ldy;
    w.X = obs;
    w.ldx = ldobs;
    w.W1 = W1;
    w.O = 256;
    w.I = 256;
    w.M = M;
    w.out = out;
    w.partial = splits > 1 ? partial : nullptr;
    w.ldo = ldo;
    return DXRL_OK;
}
int wgrad_l1_launch(const WgradPair& pr, int grid, hipStream_t st) {
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(k_wgrad_l1<false>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLLds) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(k_wgrad_l1<true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLLds) == hipSuccess;
    }();
    DXRL_REQUIRE(attr, "wgrad_l1: could not raise the dynamic LDS limit");
    static const int diag = [] {
        const char* v = getenv("DXRL_WGRAD_DIAG");
        return v ? atoi(v) : 0;
    }();
    WgradPair p = pr;
    p.n[0].diag = p.n[1].diag = diag;
    if (diag) hipLaunchKernelGGL(k_wgrad_l1<true>, dim3((unsigned)grid), dim3(512), kLLds, st, p);
    else hipLaunchKernelGGL(k_wgrad_l1<false>, dim3((unsigned)grid), dim3(512), kLLds, st, p);
    return launch_check("k_wgrad_l1");
}
}  // namespace

int launch_wgrad_l1_pair(const bf16* Y0, const bf16* W10, int splits0, float* partial0, float* out0, const bf16* Y1,
                         const bf16* W11, int splits1, float* partial1, float* out1, int64_t ldy, const bf16* obs,
                         int64_t ldobs, int64_t M, int64_t ldo, hipStream_t st, int* nslabs0, int* nslabs1) {
    WgradPair pr{};
    if (int rc = wgrad_l1_args(Y0, ldy, obs, ldobs, W10, M, splits0, partial0, out0, ldo, pr.n[0])) return rc;
    if (int rc = wgrad_l1_args(Y1, ldy, obs, ldobs, W11, M, splits1, partial1, out1, ldo, pr.n[1])) return rc;
    pr.nb0 = splits0;
    if (int rc = wgrad_l1_launch(pr, splits0 + splits1, st)) return rc;
    *nslabs0 = splits0 > 1 ? splits0 : 0;
    *nslabs1 = splits1 > 1 ? splits1 : 0;
    return DXRL_OK;
}

int launch_wgrad_l1(const bf16* Y, int64_t ldy, const bf16* obs, int64_t ldobs, const bf16* W1, int64_t M,
                    int splits, float* partial, float* out, hipStream_t st, int64_t ldo, int reduce, int* nslabs) {
    WgradPair pr{};
    if (int rc = wgrad_l1_args(Y, ldy, obs, ldobs, W1, M, splits, partial, out, ldo, pr.n[0])) return rc;
    pr.n[1] = pr.n[0];
    pr.nb0 = splits;
    if (int rc = wgrad_l1_launch(pr, splits, st)) return rc;
    if (nslabs) *nslabs = splits > 1 ? splits : 0;
    if (splits > 1 && reduce) {
        const int64_t slab = 256 * 256;
        return launch_slab_reduce(partial, slab, splits, partial + (int64_t)splits * slab, out, 0, st, 256, ldo);
    }
    return DXRL_OK;
}

// out[i] (+)= sum_z partial[z][i], fixed order (deterministic)
__global__ void k_splitk_reduce(const float* __restrict__ partial, int64_t slab, int z, float* __restrict__ out,
                                int accumulate, int cols, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= slab) return;
    float s = 0.0f;
    for (int k = 0; k < z; ++k) s += partial[(int64_t)k * slab + i];
    const int64_t o = cols ? (i / cols) * ldo + i % cols : i;  // [rows][cols] slab -> [rows][ldo] output
    out[o] = accumulate ? out[o] + s : s;
}

// First level of a two-level slab sum: tmp[g][i] = sum of slabs g*z/G .. (g+1)*z/G - 1 (in order),
// grid.y = G groups, so G x more loads are in flight than in a one-level sum over z slabs.
__global__ void k_slab_group_sum(const float* __restrict__ partial, int64_t slab, int z, float* __restrict__ tmp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= slab) return;
    const int G = gridDim.y, g = blockIdx.y;
    const int k0 = (int)((int64_t)g * z / G), k1 = (int)((int64_t)(g + 1) * z / G);
    float s = 0.0f;
    for (int k = k0; k < k1; ++k) s += partial[(int64_t)k * slab + i];
    tmp[(int64_t)g * slab + i] = s;
}

// float4 forms (slab, cols and ldo multiples of 4, 16-byte aligned bases): the same per-element
// k order, four elements per thread (a quarter of the load instructions)
__global__ void k_splitk_reduce4(const float4* __restrict__ partial, int64_t slab4, int z, float* __restrict__ out,
                                 int accumulate, int cols, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= slab4) return;
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int k = 0; k < z; ++k) {
        const float4 v = partial[(int64_t)k * slab4 + i];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
    }
    const int64_t e = 4 * i;
    const int64_t o = cols ? (e / cols) * ldo + e % cols : e;  // 4 | cols: the four stay in one row
    float4* dst = reinterpret_cast<float4*>(out + o);
    if (accumulate) {
        const float4 a = *dst;
        s = make_float4(a.x + s.x, a.y + s.y, a.z + s.z, a.w + s.w);
    }
    *dst = s;
}

// Both levels in one launch: a 256-thread block owns 16 float4 columns; thread (g, x) sums group g's
// slabs of column x (in order), then the x column's 16 group sums are added in group order from
// LDS -- exactly the two-launch sequence's per-element order, one launch and no tmp round trip.
constexpr int kRX = 16;  // float4 columns per block (x 16 groups = 256 threads)
__global__ __launch_bounds__(256) void k_slab_reduce2_4(const float4* __restrict__ partial, int64_t slab4, int z,
                                                        float* __restrict__ out, int accumulate, int cols, int64_t ldo) {
    __shared__ float4 grp[kReduceGroups][kRX];
    slab_reduce_block(partial, slab4, z, out, accumulate, cols, ldo, blockIdx.x, grp);
}

int launch_slab_reduce(const float* partial, int64_t slab, int z, float* tmp, float* out, int accumulate,
                       hipStream_t st, int cols, int64_t ldo) {
    const bool v4 = slab % 4 == 0 && cols % 4 == 0 && (cols == 0 || ldo % 4 == 0) &&
                    (reinterpret_cast<uintptr_t>(partial) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    (!tmp || (reinterpret_cast<uintptr_t>(tmp) & 15) == 0);
    if (v4) {
        const int64_t slab4 = slab / 4;
        const unsigned nb4 = (unsigned)((slab4 + 255) / 256);
        if (z > kReduceGroups && tmp) {
            hipLaunchKernelGGL(k_slab_reduce2_4, dim3((unsigned)((slab4 + kRX - 1) / kRX)), dim3(256), 0, st,
                               reinterpret_cast<const float4*>(partial), slab4, z, out, accumulate, cols, ldo);
            return launch_check("k_slab_reduce2_4");
        }
        hipLaunchKernelGGL(k_splitk_reduce4, dim3(nb4), dim3(256), 0, st, reinterpret_cast<const float4*>(partial), slab4,
                           z, out, accumulate, cols, ldo);
        return launch_check("k_splitk_reduce4");
    }
    const unsigned nb = (unsigned)((slab + 255) / 256);
    if (z > kReduceGroups && tmp) {
        hipLaunchKernelGGL(k_slab_group_sum, dim3(nb, kReduceGroups), dim3(256), 0, st, partial, slab, z, tmp);
        if (int rc = launch_check("k_slab_group_sum")) return rc;
        partial = tmp;
        z = kReduceGroups;
    }
    hipLaunchKernelGGL(k_splitk_reduce, dim3(nb), dim3(256), 0, st, partial, slab, z, out, accumulate, cols, ldo);
    return launch_check("k_splitk_reduce");
}

int launch_gemm(const GemmArgs& g0, int splits, float* reduce_out, int accumulate, hipStream_t st) {
    GemmArgs g = g0;
    DXRL_REQUIRE(g.K % 32 == 0 && g.N > 0 && g.M > 0, "gemm: K must be a multiple of 32 (got %d)", g.K);
    DXRL_REQUIRE((g.lda % 8) == 0 && (g.ldb % 8) == 0, "gemm: lda/ldb must be multiples of 8 elements");
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.Bt) & 15) == 0,
                 "gemm: operands must be 16-byte aligned");
    if (splits < 1) splits = 1;
    if (panel_ok(g, splits)) {
        g.k_chunk = g.K;
        hipLaunchKernelGGL(k_gemm_panel, dim3((unsigned)((g.M + kPM - 1) / kPM)), dim3(256), 0, st, g);
        return launch_check("k_gemm_panel");
    }
    int64_t chunk = (g.K + splits - 1) / splits;
    chunk = (chunk + kBK - 1) / kBK * kBK;
    splits = (int)((g.K + chunk - 1) / chunk);
    g.k_chunk = chunk;
    if (splits > 1) DXRL_REQUIRE(g.partial && reduce_out, "gemm: split-K needs a partial slab and an output");
    if (splits == 1) g.partial = nullptr;
    const dim3 grid((unsigned)((g.M + kBM - 1) / kBM), (unsigned)((g.N + kBN - 1) / kBN), (unsigned)splits);
    hipLaunchKernelGGL(k_gemm_bf16, grid, dim3(256), 0, st, g);
    if (int rc = launch_check("k_gemm_bf16")) return rc;
    if (g.partial) {
        const int64_t slab = g.M * (int64_t)g.N;
        if (int rc = launch_slab_reduce(g.partial, slab, splits, g.partial + (int64_t)splits * slab, reduce_out,
                                        accumulate, st))
            return rc;
    }
    return DXRL_OK;
}

int launch_wgrad(const bf16* Y, int64_t ldy, int O, const bf16* X, int64_t ldx, int I, int64_t M, int splits,
                 float* partial, float* out, hipStream_t st, int64_t ldo) {
    if (ldo <= 0) ldo = I;
    DXRL_REQUIRE(Y && X && out && O > 0 && I > 0 && M > 0, "wgrad: bad arguments");
    DXRL_REQUIRE(ldy % 8 == 0 && ldx % 8 == 0 && O % 8 == 0 && I % 8 == 0,
                 "wgrad: leading dims and feature counts must be multiples of 8");
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(Y) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0,
                 "wgrad: operands must be 16-byte aligned");
    if (splits < 1) splits = 1;
    const int requested = splits;
    int64_t chunk = (M + splits - 1) / splits;
    chunk = (chunk + kWK - 1) / kWK * kWK;
    splits = (int)((M + chunk - 1) / chunk);
    DXRL_REQUIRE(splits == 1 || partial, "wgrad: split-K needs a partial slab");
    WgradArgs w{Y, ldy, X, ldx, O, I, M, chunk, out, splits > 1 ? partial : nullptr, ldo, 0};
    if (O == kFO && I == kFI && M % kGK == 0 && ldy >= kFO && ldx >= kFI &&
        getenv("DXRL_WGRAD_REGSTAGE") == nullptr) {  // LDS-DMA stream (A/B: DXRL_WGRAD_REGSTAGE=1)
        static bool attr = [] {
            return hipFuncSetAttribute(reinterpret_cast<const void*>(k_wgrad_glds),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kGNB * kGChunkB) == hipSuccess;
        }();
        DXRL_REQUIRE(attr, "wgrad: could not raise the dynamic LDS limit");
        static const int diag = [] {
            const char* v = getenv("DXRL_WGRAD_DIAG");
            return v ? atoi(v) : 0;
        }();
        w.diag = diag;
        // 32-row chunks dealt round robin over the workgroups: the caller's split count (at most
        // one chunk each), not the range-normalised one above -- the same rule as launch_wgrad_l1,
        // so the H1-copy and recompute paths give each slab the same rows (bit-identical dW2)
        const int gs = (int)(requested < M / kGK ? requested : M / kGK);
        DXRL_REQUIRE(gs == 1 || partial, "wgrad: split-K needs a partial slab");
        w.partial = gs > 1 ? partial : nullptr;
        hipLaunchKernelGGL(k_wgrad_glds, dim3((unsigned)gs), dim3(512), kGNB * kGChunkB, st, w);
        if (int rc = launch_check("k_wgrad_glds")) return rc;
        if (gs > 1) {
            const int64_t slab = (int64_t)O * I;
            return launch_slab_reduce(partial, slab, gs, partial + (int64_t)gs * slab, out, 0, st, I, ldo);
        }
        return DXRL_OK;
    }
    if (O <= kFO && I <= kFI && O > 128 && M >= (int64_t)splits * kFK && chunk % kFK == 0 &&
        (M + 3 * kFK) * (ldy > ldx ? ldy : ldx) * 2 < 0x7fffffff) {  // whole output per workgroup
        static bool attr = [] {
            return hipFuncSetAttribute(reinterpret_cast<const void*>(k_wgrad_full),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 4 * kFK * kFPitch * 2) == hipSuccess;
        }();
        DXRL_REQUIRE(attr, "wgrad: could not raise the dynamic LDS limit");
        hipLaunchKernelGGL(k_wgrad_full, dim3((unsigned)splits), dim3(512), 4 * kFK * kFPitch * 2, st, w);
        if (int rc = launch_check("k_wgrad_full")) return rc;
        if (splits > 1) {
            const int64_t slab = (int64_t)O * I;
            return launch_slab_reduce(partial, slab, splits, partial + (int64_t)splits * slab, out, 0, st, I, ldo);
        }
        return DXRL_OK;
    }
    const dim3 grid((unsigned)((O + kWO - 1) / kWO), (unsigned)((I + kWI - 1) / kWI), (unsigned)splits);
    hipLaunchKernelGGL(k_wgrad_bf16, grid, dim3(256), 0, st, w);
    if (int rc = launch_check("k_wgrad_bf16")) return rc;
    if (splits > 1) {
        const int64_t slab = (int64_t)O * I;
        if (int rc = launch_slab_reduce(partial, slab, splits, partial + (int64_t)splits * slab, out, 0, st, I, ldo))
            return rc;
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

int dxrl_wgrad_bf16(int32_t device, const void* Y, int64_t ldy, int32_t O, const void* X, int64_t ldx, int32_t I,
                    int64_t M, int32_t splits, float* partial, float* out, void* stream) {
    DeviceGuard dg(device);
    return launch_wgrad(static_cast<const bf16*>(Y), ldy, O, static_cast<const bf16*>(X), ldx, I, M, splits, partial,
                        out, as_stream(stream));
}

}  // extern "C"
