// dxrl_pg_fused.hip -- one-pass training step of one MLP(256,256) head network.
//
// k_pg_fused runs, per 128-sample tile and entirely out of LDS (160 KiB, one
// workgroup of 8 waves per CU, persistent over tiles):
//
//   forward   H1 = tanh(X W1^T)  H2 = tanh(H1 W2^T + b2)  out = H2 W3^T + b3
//   heads     actor: PPO-clip surrogate -> dL/dmu, dL/dlog_std, losses
//             critic: value loss -> dL/dV            (forward mode: write V)
//   backward  dW3 += dout^T H2            (registers, whole launch)
//             dH2 = (dout W3) * (1 - H2^2)            -> HBM (for dW2)
//             dH1 = (dH2 W2) * (1 - H1^2)
//             dW1 += dH1^T X              (registers, whole launch)
//
// H1 and dH2 go to HBM once so the one contraction too large to keep in
// registers, dW2 = dH2^T H1, runs as the whole-output weight-gradient GEMM
// (launch_wgrad) right after.  Nothing else of the activations ever leaves
// the CU: compared with the layer-by-layer GEMM chain this removes the H2,
// dH1, mu / dout round trips and five of the eight launches.
//
// MFMA formulation: hidden layers are computed transposed (weights as the A
// operand from L2, activations as the B operand from LDS), so each lane's
// accumulator holds 4 consecutive features of one sample -> 8-byte LDS stores
// of the row-major activation tile.  Transposed operands of the weight
// gradients come straight from the row-major tiles through ds_read_b64_tr_b16.
//
// Gradients are deterministic: each workgroup owns a fixed tile set and writes
// its dW1 / dW3 / dlog_std partials once; launch_slab_reduce sums them in a fixed order.
#include "dxrl_gemm.h"
#include "dxrl_pg.h"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

using namespace dxrl;
using namespace dxrl::pg;

namespace dxrl {
namespace {

constexpr float kLog2PiF = 1.8378770664093453f;
constexpr int kXp = kIn + 8;             // 72:  X rows (conflict-free b128 row reads)
constexpr int kHp = kH + 8;              // 264: H1 / H2 rows
constexpr int kDp = kOut + 8;            // 40:  dout rows

// LDS image of one kTR-sample tile: X [kTR][kXp], H1 / H2 [kTR][kHp], dout [kTR][kDp] (bf16).
// kTR = 128: 160 KiB, one workgroup per CU; kTR = 64: 80 KiB, two workgroups per CU.
template <int kTR>
struct TileLds {
    static constexpr int kOffX = 0;
    static constexpr int kOffH1 = kOffX + kTR * kXp;
    static constexpr int kOffH2 = kOffH1 + kTR * kHp;
    static constexpr int kOffD = kOffH2 + kTR * kHp;
    static constexpr int kElems = kOffD + kTR * kDp;
    static_assert(kElems * 2 * (128 / kTR) == 163840, "one CU's 160 KiB of LDS per 128 samples");
};

// per-workgroup gradient partial slab (f32)
// Workgroup partial slab: only what a pass can make nonzero -- dW1 input columns 0..47 (45
// observation features + the bias column; X is zero beyond), dW3 head rows 0..15 (15 mu rows /
// the value row) with their bias column, padded to a float4 multiple; the scatter writes the
// zeros of the rest of the grads blocks
constexpr int kPW1C = 48;                        // dW1 columns kept
constexpr int kPW3C = kH + 4;                    // dW3 columns kept: 0..255, bias 256, pad 257..259
constexpr int kPartW1 = 0;                       // [256][48]
constexpr int kPartW3 = kPartW1 + kH * kPW1C;    // [16][260]
constexpr int kPartLs = kPartW3 + 16 * kPW3C;
constexpr int kPartB2 = kPartLs + 16;            // [256]: dL/db2 column sums
constexpr int kPartSize = kPartB2 + kH;

// global-address-space views: loads through them compile to global_load (vmcnt only); a
// generic pointer the compiler cannot place compiles to flat_load, which also counts in
// lgkmcnt and so holds every LDS wait until the global data is back
typedef __attribute__((address_space(1))) const bf16x8 gbf16x8;
typedef __attribute__((address_space(1))) const float gf32;

struct FusedArgs {
    int net;    // 0 actor, 1 critic
    int train;  // 0: forward only (critic values), 1: forward + heads + backward
    int diag;   // timing ablations (DXRL_FUSED_DIAG): 1 no HBM copies, 4 no dW MFMAs, 8 stamps,
                // 16 no L2 epilogue, 32 no L2 MFMAs
    int64_t rows;
    const bf16* X;  // [rows][64], column 45 = 1
    const bf16 *W1, *W2, *W3, *W2T, *W3T;  // fragment-ordered streams (dxrl_pg.h kFr*)
    const bf16* W3rm;  // the head's row-major bf16 copy [kOut][kHx] (16-row critic head)
    const float* b2;  // bias of hidden unit n: b2[n * kHx]
    const float* b3;  // bias of head row o:   b3[o * kHx]
    const float* logstd;
    const float* act;
    const float* logp_old;
    const float* adv;
    const float* ret;
    const double* stats;
    float sc, clip_eps, vf2;
    float* v_out;   // forward mode: [rows]
    bf16* h1_out;   // [rows][kHx] (columns 0..255 written)
    bf16* dh2_out;  // [rows][kH]
    const bf16* h2_in;  // train, kH2: layer-2 activations [rows][kHp] from the rollout / values pass
    bf16* h2_out;       // forward (k_pg_values): write H2 [rows][kHp] for the critic's train pass
    float* part;    // [grid][kPartSize]
    double* loss;   // [loss_rows][4]: row b = workgroup b's loss sums, rows >= gridDim.x zeroed
    int loss_rows;  // the caller's row count (dxrl_pg_fused_args.grid)
    unsigned long long* stamps;  // diag & 8: [grid][waves][16] cycles per segment
};

// one 16-byte-per-lane LDS-DMA piece: lane l's 16 bytes at src land at lds_dst + 16 l (M0 = the
// wave's LDS destination; global_load_lds_dwordx4, no VGPR staging)
__device__ __forceinline__ void glds_x4(const void* src, const void* lds_dst) {
    const uint32_t lds_addr =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds_dst);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_addr)
                 : "memory");
}

__device__ __forceinline__ void zero_acc(f32x16& a) {
#pragma unroll
    for (int q = 0; q < 16; ++q) a[q] = 0.0f;
}

struct NoHook {
    __device__ void operator()() const {}
};
struct NoKHook {
    __device__ void operator()(int) const {}
};
// The first kD weight fragments of a fwd_tiles call, issuable ahead of the call (before the
// barrier in front of its phase, so their L2 latency overlaps the barrier wait).
template <int KS>
struct WPre {
    // weight prefetch distance (k-steps; 12 or 16, all of W2 issued ahead of the barrier in front
    // of its layer, measured within 0.7 %: profiles/r06/ab_wpf_gatepk_rejected.log)
    static constexpr int kD = KS < 8 ? KS : 8;
    bf16x8 wf[kD];
    const gbf16x8* wp;
};
// (W: fragment-ordered stream of a matrix with kst k-steps per feature tile, dxrl_pg.h; loads
// through the global address space -- global_load: vmcnt only, a flat load would also hold every
// LDS wait)
template <int KS>
__device__ __forceinline__ void w_prefetch(WPre<KS>& w, const bf16* W, int kst, int ft0, int lane) {
    w.wp = (const gbf16x8*)W + (int64_t)ft0 * kst * 64 + lane;
#pragma unroll
    for (int k = 0; k < WPre<KS>::kD; ++k) w.wf[k] = w.wp[64 * k];
}
template <int KS, int kLda, int MT, typename Hook = NoHook>
__device__ __forceinline__ void fwd_run(WPre<KS>& w, const bf16* A, f32x16 (&acc)[MT], int lane, Hook hook = Hook{},
                                        bool no_mfma = false) {
    const int r = lane & 31, h = lane >> 5;
    constexpr int kD = WPre<KS>::kD;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) zero_acc(acc[mt]);
    // activation fragments double-buffered one k-step ahead
    const bf16* ap = A + r * kLda + 8 * h;
    bf16x8 bq[2][MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) bq[0][mt] = *reinterpret_cast<const bf16x8*>(ap + 32 * mt * kLda);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        if (k + 1 < KS) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                bq[(k + 1) & 1][mt] = *reinterpret_cast<const bf16x8*>(ap + 32 * mt * kLda + 16 * (k + 1));
        }
        const bf16x8 a = w.wf[k % kD];
        if (k + kD < KS) w.wf[k % kD] = w.wp[64 * (k + kD)];
        // loads the caller wants behind the last weight fragment (vmcnt retires in issue order:
        // issued earlier they would hold every weight wait of this call)
        if (k + kD == KS) hook();
        // keep the prefetches above issued ahead of this k-step's MFMAs (the scheduler would
        // otherwise sink every load next to its use and expose its full latency)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            if (!no_mfma) acc[mt] = mfma32(a, bq[k & 1][mt], acc[mt]);
        __builtin_amdgcn_sched_barrier(0);
    }
}
// acc[mt] (features 32 ft0.. x samples 32 mt..) = W[32 ft0 + r][:] . A[32 mt + r][:] over KS
// k-steps; weight fragments stream from L2 kD k-steps ahead, each feeds MT MFMAs.
template <int KS, int kLda, int MT, typename Hook = NoHook>
__device__ __forceinline__ void fwd_tiles(const bf16* __restrict__ W, int kst, int ft0, const bf16* A,
                                          f32x16 (&acc)[MT], int lane, Hook hook = Hook{}, bool no_mfma = false) {
    WPre<KS> w;
    w_prefetch(w, W, kst, ft0, lane);
    fwd_run<KS, kLda, MT>(w, A, acc, lane, hook, no_mfma);
}

// Sample-tile-major variant with the epilogue software-pipelined under the MFMAs: all KS weight
// fragments stay in registers, the MT 32-sample tiles run one after another, and while tile mt's
// MFMA chain runs the epilogue of tile mt - 1 issues into its gaps one value pair at a time
// (epi(acc, mt, p): pair p = 0..7 of the lane's 16 values, group p >> 1).  Two accumulators live
// instead of MT.  Per output the k order -- and so every bit -- is the same as fwd_run's.
// (fwd_pipe_w: the same with all KS weight fragments already in registers -- the forward-only
// pass keeps them resident for the launch)
template <int KS, int kLda, int MT, typename Epi, typename KHook = NoKHook, typename THook = NoKHook>
__device__ __forceinline__ void fwd_pipe_w(const bf16x8 (&wf)[KS], const bf16* A, int lane, Epi& epi,
                                           bool no_mfma = false, KHook khook = KHook{}, THook thook = THook{}) {
    static_assert(KS >= 4 && KS % 4 == 0, "pair schedule assumes KS in {4, 8, 16, ...}");
    const int r = lane & 31, h = lane >> 5;
    constexpr int kPairsPerK = KS >= 8 ? 1 : 8 / KS;  // epilogue pairs issued per k-step
    constexpr int kKPerPair = KS >= 8 ? KS / 8 : 1;   // k-steps per epilogue pair
    const bf16* ap = A + r * kLda + 8 * h;
    f32x16 acc, prev;
    // activation fragments kBD k-steps ahead (one MFMA per k-step now covers a read, not four)
    constexpr int kBD = 3;
    bf16x8 bq[kBD + 1];
#pragma unroll
    for (int i = 0; i < kBD; ++i)
        bq[i] = *reinterpret_cast<const bf16x8*>(ap + 32 * (i / KS) * kLda + 16 * (i % KS));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        zero_acc(acc);
        if (mt > 0) epi.prime(mt - 1);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const int sidx = mt * KS + k;
            if (sidx + kBD < MT * KS) {
                const int nmt = (sidx + kBD) / KS, nk = (sidx + kBD) % KS;
                bq[(sidx + kBD) % (kBD + 1)] = *reinterpret_cast<const bf16x8*>(ap + 32 * nmt * kLda + 16 * nk);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (!no_mfma) acc = mfma32(wf[k], bq[sidx % (kBD + 1)], acc);
            if (mt > 0 && (k % kKPerPair) == kKPerPair - 1) {
#pragma unroll
                for (int q = 0; q < kPairsPerK; ++q) epi(prev, mt - 1, (k / kKPerPair) * kPairsPerK + q);
            }
            khook(sidx);  // caller work spread over the MT * KS steps
            __builtin_amdgcn_sched_barrier(0);
        }
        prev = acc;
    }
    epi.prime(MT - 1);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        epi(prev, MT - 1, q);
        thook(q);  // caller work beside the last tile's epilogue (which has no MFMAs of its own)
    }
}
template <int KS, int kLda, int MT, typename Epi, typename Hook = NoHook, typename KHook = NoKHook,
          typename THook = NoKHook>
__device__ __forceinline__ void fwd_pipe(WPre<KS>& w, const bf16* A, int lane, Epi& epi, Hook hook = Hook{},
                                         bool no_mfma = false, KHook khook = KHook{}, THook thook = THook{}) {
    constexpr int kD = WPre<KS>::kD;
    bf16x8 wf[KS];
#pragma unroll
    for (int k = 0; k < kD; ++k) wf[k] = w.wf[k];
#pragma unroll
    for (int k = kD; k < KS; ++k) wf[k] = w.wp[64 * k];
    hook();  // loads the caller wants behind the last weight fragment (vmcnt retires in order)
    fwd_pipe_w<KS, kLda, MT>(wf, A, lane, epi, no_mfma, khook, thook);
}

// fwd_pipe epilogues.  EpiTanh: tanh(acc + bias) -> bf16 H rows (store_hidden, pair by pair);
// EpiGate: acc * (1 - Y^2) -> bf16 in place of Y (gate_in_place), Y read one pair group ahead.
struct EpiTanh {
    bf16* H;
    int f0;        // 32 ft + 4 h
    int r;
    const float* bk;  // 16 pre-scaled biases (registers) or null
    bf16x4 v;
    __device__ void prime(int) {}
    __device__ __forceinline__ void operator()(const f32x16& acc, int mt, int p) {
        const int g = p >> 1, u = 2 * (p & 1);
        const f32x2 b = bk ? f32x2{bk[4 * g + u], bk[4 * g + u + 1]} : f32x2{0.0f, 0.0f};
        const f32x2 t = tanh_pre2(f32x2{acc[4 * g + u], acc[4 * g + u + 1]}, b);
        v[u] = to_bf16(t.x);
        v[u + 1] = to_bf16(t.y);
        if (u == 2) *reinterpret_cast<bf16x4*>(H + (32 * mt + r) * kHp + f0 + 8 * g) = v;
    }
};
// EpiTanh with the 16 pre-scaled biases held by value (k_pg_values: through a pointer the
// run-time tile-count dispatch kept them in scratch memory)
struct EpiTanhB {
    bf16* H;
    int f0;
    int r;
    float bk[16];
    bf16x4 v;
    __device__ void prime(int) {}
    __device__ __forceinline__ void operator()(const f32x16& acc, int mt, int p) {
        const int g = p >> 1, u = 2 * (p & 1);
        const f32x2 t = tanh_pre2(f32x2{acc[4 * g + u], acc[4 * g + u + 1]}, f32x2{bk[4 * g + u], bk[4 * g + u + 1]});
        v[u] = to_bf16(t.x);
        v[u + 1] = to_bf16(t.y);
        if (u == 2) *reinterpret_cast<bf16x4*>(H + (32 * mt + r) * kHp + f0 + 8 * g) = v;
    }
};
struct EpiGate {
    bf16* Y;
    int f0;
    int r;
    bf16x4 y, v;
    __device__ __forceinline__ void prime(int mt) { y = *reinterpret_cast<const bf16x4*>(Y + (32 * mt + r) * kHp + f0); }
    __device__ __forceinline__ void operator()(const f32x16& acc, int mt, int p) {
        const int g = p >> 1, u = 2 * (p & 1);
        const f32x2 t = tanh_gate2(f32x2{acc[4 * g + u], acc[4 * g + u + 1]},
                                   f32x2{from_bf16(y[u]), from_bf16(y[u + 1])});
        v[u] = to_bf16(t.x);
        v[u + 1] = to_bf16(t.y);
        if (u == 2) {
            *reinterpret_cast<bf16x4*>(Y + (32 * mt + r) * kHp + f0 + 8 * g) = v;
            if (g < 3) y = *reinterpret_cast<const bf16x4*>(Y + (32 * mt + r) * kHp + f0 + 8 * (g + 1));
        }
    }
};

// tanh(acc + bias) -> bf16 row-major activation tile (4 consecutive features per 8-byte store)
// (bk: the lane's 16 pre-scaled biases tanh_bias(b[32 ft + 8 g + 4 h + u]) at [4 g + u], or null)
template <int MT>
__device__ __forceinline__ void store_hidden(const f32x16 (&acc)[MT], int ft, const float* bk, bf16* H, int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f0 = 32 * ft + 8 * g + 4 * h;
            float b[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            if (bk) {
#pragma unroll
                for (int u = 0; u < 4; ++u) b[u] = bk[4 * g + u];
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                bf16x4 v;
#pragma unroll
                for (int u = 0; u < 4; u += 2) {
                    const f32x2 t = tanh_pre2(f32x2{acc[mt][4 * g + u], acc[mt][4 * g + u + 1]},
                                              f32x2{b[u], b[u + 1]});
                    v[u] = to_bf16(t.x);
                    v[u + 1] = to_bf16(t.y);
                }
                *reinterpret_cast<bf16x4*>(H + (32 * mt + r) * kHp + f0) = v;
            }
        }
}

// Y[m][f] <- bf16(acc[f][m] * (1 - Y[m][f]^2)) for this wave's features (tanh' gate, in place)
// Y[m][f] <- bf16(acc[f][m] * (1 - Y[m][f]^2)) for this wave's features (tanh' gate, in place).
// gate_load reads all 4 x MT Y pieces first (the caller issues it ahead of the MFMAs that make acc,
// so one LDS latency hides under them; read one by one right before use, the compiler's schedule
// waited out each read in turn: lgkmcnt(0) eight times per tile)
template <int MT>
__device__ __forceinline__ void gate_load(bf16x4 (&ys)[4][MT], int ft, const bf16* Y, int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            ys[g][mt] = *reinterpret_cast<const bf16x4*>(Y + (32 * mt + r) * kHp + 32 * ft + 8 * g + 4 * h);
}
template <int MT>
__device__ __forceinline__ void gate_store(const f32x16 (&acc)[MT], const bf16x4 (&ys)[4][MT], int ft, bf16* Y,
                                           int lane) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int f0 = 32 * ft + 8 * g + 4 * h;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const bf16x4 y = ys[g][mt];
            bf16x4 v;
#pragma unroll
            for (int u = 0; u < 4; u += 2) {
                const f32x2 t = tanh_gate2(f32x2{acc[mt][4 * g + u], acc[mt][4 * g + u + 1]},
                                           f32x2{from_bf16(y[u]), from_bf16(y[u + 1])});
                v[u] = to_bf16(t.x);
                v[u + 1] = to_bf16(t.y);
            }
            *reinterpret_cast<bf16x4*>(Y + (32 * mt + r) * kHp + f0) = v;
        }
    }
}

// A [kTR][kH] bf16 tile of LDS (pitch kHp) -> rows m0.. of an HBM matrix (leading dimension ld),
// nthr threads from thread index t0 (16-byte chunks, rows past `rows` skipped)
template <int kThreads, int kTR>
__device__ __forceinline__ void copy_tile_out_n(const bf16* T, bf16* out, int64_t ld, int64_t m0, int64_t rows,
                                                int t, int diag) {
    constexpr int kChunks = kTR * (kH / 8);
    static_assert(kChunks % kThreads == 0, "whole chunks per thread");
    if (diag & 1) return;
    asm volatile("" : "+v"(t));  // per-call addresses (hoisted out of the tile loop they would spill)
#pragma unroll
    for (int u = 0; u < kChunks / kThreads; ++u) {
        const int c = t + kThreads * u, row = c >> 5, col = 8 * (c & 31);
        const int64_t m = m0 + row;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(T + row * kHp + col);
        if (m < rows) *(__attribute__((address_space(1))) bf16x8*)(out + m * ld + col) = v;
    }
}

// One 16-byte chunk of the dH2 tile to HBM, a plain store (non-temporal stores were measured +1-1.7 %
// on most boxes and -10 % on others, profiles/r05/ab_dh2_nt.log: removed in round 6)
__device__ __forceinline__ void store_dh2(bf16* dst, const bf16x8& v) { *(__attribute__((address_space(1))) bf16x8*)dst = v; }

// Hide a pointer's provenance from the optimiser so loads through it are not hoisted
// out of the tile loop (loop-invariant weight / bias loads would otherwise pin registers
// for the whole launch).
template <typename T>
__device__ __forceinline__ T* opaque(T* ptr) {
    asm volatile("" : "+s"(ptr));
    return ptr;
}

// A/B switches: DXRL_L2_PIPE layer 2 as fwd_pipe (tanh epilogue under the next sample tile's
// MFMAs) instead of the k-major chain + store_hidden; DXRL_FUSED_PRIO s_setprio 1 for waves 4..7
#ifndef DXRL_L2_PIPE
#define DXRL_L2_PIPE 1
#endif
#ifndef DXRL_DH2_IN_DH1
#define DXRL_DH2_IN_DH1 1
#endif
// The critic's value head on 16x16x32 tiles run by all eight waves (16 samples each, only head row
// 0 nonzero) instead of 32x32x16 tiles on four waves (32 samples each, 31 dead head rows, four
// waves idle): critic train 384 -> 375 us, critic values 215 -> 209 us (kernel-level A/B)
#ifndef DXRL_CRITIC_HEAD16
#define DXRL_CRITIC_HEAD16 1
#endif
// The actor's head on 16x16x32 tiles run by all eight waves (16 samples each, head rows 0..15; a
// sample's 16 log-density terms gathered by shuffles and summed in action order as before):
// actor train 427.6 -> 423.3 us (kernel-level A/B), 249 -> 231 VGPRs
#ifndef DXRL_ACTOR_HEAD16
#define DXRL_ACTOR_HEAD16 1
#endif
#ifndef DXRL_HEAD_PF
#define DXRL_HEAD_PF 1
#endif
#ifndef DXRL_FWD_RESIDENT_W
#define DXRL_FWD_RESIDENT_W 1
#endif
#ifndef DXRL_TRAIN_RESIDENT_HEAD
#define DXRL_TRAIN_RESIDENT_HEAD 1
#endif
// the train passes' layer-2 biases and (DXRL_TRAIN_RESIDENT_HEAD) the heads' constants in
// registers for the launch: actor 400 -> 384 us, critic 377 -> 363 us (kernel-level A/B,
// profiles/r04/ab_kernels_train_resident_consts.log); W1's 16 registers as well: no change
#ifndef DXRL_TRAIN_RESIDENT_B2
#define DXRL_TRAIN_RESIDENT_B2 1
#endif
#ifndef DXRL_FUSED_PRIO
#define DXRL_FUSED_PRIO 1
#endif

// forward-only pass with resident weights: the next tile's X fetched at the start of the tile
#ifndef DXRL_FWD_EARLY_X
#define DXRL_FWD_EARLY_X 1
#endif
// dW1 without the barrier after dH1: a wave's dW1 reads only its own dH1 columns (and X), so the
// MFMAs of the first three 32-sample blocks issue beside dH1's last epilogue (VALU only) and the
// db2 column sums' second stage moves behind the end-of-tile barrier
#ifndef DXRL_DW1_TAIL
#define DXRL_DW1_TAIL 1
#endif

// stamps (DXRL_FUSED_DIAG=8) of the kH2 passes: a diagnostic build only
#ifndef DXRL_H2_STAMPS
#define DXRL_H2_STAMPS 0
#endif

// dW3 / dW1 operands through tr_frag16_eo (even / odd sample order inside each 8-sample group:
// the transposed reads conflict-free) instead of tr_frag16 (2-way)
#ifndef DXRL_TR_EO
#define DXRL_TR_EO 1
#endif
template <int kPitch>
__device__ __forceinline__ bf16x8 wg_frag(const bf16* tile, int col0, int kk, int lane) {
    if constexpr (DXRL_TR_EO) return tr_frag16_eo<kPitch>(tile, col0, kk, lane);
    else return tr_frag16<kPitch>(tile, col0, kk, lane);
}

// kFW waves per workgroup: 4 (one per SIMD, 512 registers each) or 8 (two per SIMD)
// kTrain: forward + heads + backward; otherwise the forward-only critic-value pass, which keeps
// no launch-long accumulators and so fits two waves per SIMD.
// kNet: 0 actor, 1 critic, -1 read from the arguments; kDiag: the DXRL_FUSED_DIAG ablations /
// stamps compiled in (production instantiations do not test them at run time: fewer branches and
// SGPRs in the tile loop)
// kH2 (train, production geometry): the tile's layer-2 activations come from HBM (p.h2_in,
// written by the rollout for the actor / by k_pg_values for the critic with the same weights,
// bit for bit this pass's own L2) by LDS-DMA into the H2 slot while layer 1 runs, instead of
// being recomputed: no L2 phase (round 6).
template <int kFW, int kTR, bool kTrain, int kNet, bool kDiag, bool kH2 = false>
__global__ __launch_bounds__(64 * kFW, kTR == 64 ? 2 : 1) void k_pg_fused(FusedArgs p) {
    static_assert(!kH2 || (kTrain && kFW == 8 && kTR == 128 && (!kDiag || DXRL_H2_STAMPS)), "kH2: production train instantiations");
    const int diag = kDiag ? p.diag : 0;
    const bool actor = kNet < 0 ? p.net == 0 : kNet == 0;  // kNet -1: the net read at run time
    using L = TileLds<kTR>;
    constexpr int kOffX = L::kOffX, kOffH1 = L::kOffH1, kOffH2 = L::kOffH2, kOffD = L::kOffD;
    constexpr int kHW = kTR / 32;  // waves running the heads (one 32-sample tile each)
    // critic, 8 waves x 128 samples: every wave runs a 16-sample value head (DXRL_CRITIC_HEAD16)
    constexpr bool kCH16 = DXRL_CRITIC_HEAD16 && kNet == 1 && kFW == 8 && kTR == 128;
    constexpr bool kAH16 = DXRL_ACTOR_HEAD16 && kNet == 0 && kTrain && kFW == 8 && kTR == 128;
    constexpr bool kH16 = kCH16 || kAH16;
    constexpr int kMT = kTR / 32;  // 32-sample MFMA tiles of a tile
    constexpr int kFThreads = 64 * kFW;
    constexpr int kNT = kH / 32 / kFW;  // 32-wide feature tiles per wave
    [[maybe_unused]] constexpr int kCopyU = kTR * (kH / 8) / kFThreads;  // 16-byte chunks per thread, [kTR][kH] tile
    static_assert(kHW <= kFW, "one 32-sample head tile per wave");
    __shared__ __attribute__((aligned(16))) bf16 lds[L::kElems];
    bf16* X = lds + kOffX;
    bf16* H1 = lds + kOffH1;
    bf16* H2 = lds + kOffH2;
    bf16* D = lds + kOffD;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if DXRL_FUSED_PRIO
    // the second-dispatched half of the waves loses VALU arbitration to its SIMD partner
    if (__builtin_amdgcn_readfirstlane(wave) >= kFW / 2) __builtin_amdgcn_s_setprio(1);
#endif
    const int ft0 = kNT * wave;  // this wave's first 32-wide feature tile
    const int64_t ntiles = (p.rows + kTR - 1) / kTR;

    // launch-long accumulators: dW3 columns of this wave's tiles, dW1 rows of this wave's tiles
    // (16x16x32 tiles: only head rows 0..15 and input columns 0..47 can be nonzero -- 15 mu rows /
    // one value row, 45 observation features + the bias column -- so 8 + 24 registers, not 16 + 32)
    f32x4 acc3[kNT][2], acc1[kNT][2][3];
#pragma unroll
    for (int j = 0; j < kNT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc3[j][0][q] = acc3[j][1][q] = 0.0f;
#pragma unroll
            for (int ri = 0; ri < 2; ++ri)
#pragma unroll
                for (int ci = 0; ci < 3; ++ci) acc1[j][ri][ci][q] = 0.0f;
        }
    float dls[8], db3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dls[j] = db3[j] = 0.0f;
    float db2 = 0.0f;  // threads < 256: dL/db2 of column tid
    float lsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // per-thread sums over <= ~25 tiles (f64 across threads)

    // workgroup-uniform: pinned to scalar registers (as VGPR pairs they were spilled across the tile loop)
    const auto uniform_f64 = [](double v) {
        const uint64_t u = __double_as_longlong(v);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
        return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    };
    const double adv_mean = uniform_f64(kTrain && actor ? p.stats[2] : 0.0);
    // 1 / (std + 1e-8) once per launch: one f64 multiply per sample instead of an f64 division
    // sequence (~12 f64 instructions and their registers in the head)
    const double adv_inv = uniform_f64(kTrain && actor ? 1.0 / (p.stats[4] + 1e-8) : 1.0);

    // X tile prefetch: 128 rows x 8 chunks of 16 B = 1024 chunks, 4 per thread
    constexpr int kXU = kTR * (kIn / 8) / kFThreads;
    bf16x8 xr[kXU];
    auto fetch_x = [&](int64_t tile) {
        int t = tid;
        asm volatile("" : "+v"(t));
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int c = t + kFThreads * u, row = c >> 3, col = 8 * (c & 7);
            const int64_t m = tile * kTR + row;
            xr[u] = m < p.rows ? *reinterpret_cast<const bf16x8*>(p.X + m * kIn + col) : zero8();
        }
    };
    unsigned long long st_acc[16], st_last = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) st_acc[k] = 0;
#define STAMP(k)                                                                                 \
    do {                                                                                         \
        if (diag & 8) {                                                                        \
            __builtin_amdgcn_sched_barrier(0);                                                   \
            unsigned long long t_;                                                               \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
            __builtin_amdgcn_sched_barrier(0);                                                   \
            st_acc[k] += t_ - st_last;                                                           \
            st_last = t_;                                                                        \
        }                                                                                        \
    } while (0)
    // forward-only pass (critic values): this wave's W1 / W2 fragments stay in registers for the
    // whole launch (80 VGPRs; the train instantiations have no room for them) instead of streaming
    // 160 KB of weight fragments from L2 per tile and workgroup
    constexpr bool kResW = !kTrain && kNT == 1 && DXRL_FWD_RESIDENT_W && DXRL_L2_PIPE;
    constexpr bool kEarlyX = kResW && DXRL_FWD_EARLY_X;
    // kH2: W1 resident too, so layer 1 issues no global loads -- the LDS-DMA pieces in flight
    // beside it are invisible to the compiler, and a vmcnt wait for a weight fragment issued
    // before them would wait for them as well
    constexpr bool kResW1 = kResW || kH2;
    constexpr bool kDw1Tail = kTrain && kNT == 1 && kMT == 4 && DXRL_DW1_TAIL && DXRL_DH2_IN_DH1;
    bf16x8 w1res[kResW1 ? kIn / 16 : 1], w2res[kResW ? kH / 16 : 1];
    if constexpr (kResW1) {
        const gbf16x8* p1 = (const gbf16x8*)p.W1 + (int64_t)ft0 * (kIn / 16) * 64 + lane;
#pragma unroll
        for (int k = 0; k < kIn / 16; ++k) w1res[k] = p1[64 * k];
    }
    if constexpr (kH2) __builtin_amdgcn_s_waitcnt(0xF70);  // (vmcnt(0): retired before any LDS-DMA piece)
    if constexpr (kResW) {
        const gbf16x8* p2 = (const gbf16x8*)p.W2 + (int64_t)ft0 * (kH / 16) * 64 + lane;
#pragma unroll
        for (int k = 0; k < kH / 16; ++k) w2res[k] = p2[64 * k];
    }
    // ... and so do the layer-2 biases of its feature tile and (16-row critic head) the value row
    // (the train passes too: the biases fit beside their accumulators, W2 / W2T do not)
    constexpr bool kResB = kNT == 1 && (kResW || (kTrain && DXRL_TRAIN_RESIDENT_B2));
    float bkres[kResB ? 16 : 1];
    constexpr bool kResH = kCH16 && (kResW || (kTrain && DXRL_TRAIN_RESIDENT_HEAD));
    bf16x8 w3res[kResH ? 8 : 1];
    float b3res = 0.0f;
    // the actor head's per-lane constants (head rows 4 (lane >> 4) .. + 3): log sigma and mu bias
    constexpr bool kResA = kAH16 && DXRL_TRAIN_RESIDENT_HEAD;
    float ahls[kResA ? 4 : 1], ahb3[kResA ? 4 : 1];
    if constexpr (kResA) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = 4 * (lane >> 4) + i;
            ahls[i] = o < kAct ? ((gf32*)p.logstd)[o] : 0.0f;
            ahb3[i] = ((gf32*)p.b3)[(int64_t)o * kHx];
        }
    }
    if constexpr (kResB) {
        const int h0 = (threadIdx.x & 63) >> 5;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            bkres[q] = tanh_bias(((gf32*)p.b2)[(int64_t)(32 * ft0 + 8 * (q >> 2) + 4 * h0 + (q & 3)) * kHx]);
    }
    if constexpr (kResH) {
        {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                w3res[k] = (lane & 15) == 0 ? *(const gbf16x8*)(p.W3rm + 32 * k + 8 * (lane >> 4)) : zero8();
            b3res = ((gf32*)p.b3)[0];
        }
    }
    int64_t tile = blockIdx.x;
    if (tile < ntiles) fetch_x(tile);
    STAMP(15);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t m0 = tile * kTR;
        // lane-derived addresses are recomputed per tile instead of being hoisted out of the
        // loop by the compiler (dozens of loop-invariant address registers otherwise)
        int tid_l = (int)threadIdx.x;
        asm volatile("" : "+v"(tid_l));
        const int lane = tid_l & 63, r = lane & 31, h = lane >> 5;
        (void)r;
        (void)h;
        const bf16 *W1 = opaque(p.W1), *W2 = opaque(p.W2), *W3 = opaque(p.W3), *W2T = opaque(p.W2T),
                   *W3T = opaque(p.W3T);
        const float *b2 = opaque(p.b2), *b3 = opaque(p.b3), *logstd = opaque(p.logstd);
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int c = tid + kFThreads * u, row = c >> 3, col = 8 * (c & 7);
            *reinterpret_cast<bf16x8*>(X + row * kXp + col) = xr[u];
        }
        // resident-weight forward pass: no weight fragment loads in the tile loop, so nothing
        // waits behind the next tile's X -- it goes out now and lands under this tile's layers
        // (fetched after the head it was a full HBM latency at the next tile's start)
        if constexpr (kEarlyX) {
            if (tile + gridDim.x < ntiles) fetch_x(tile + gridDim.x);
        }
        // the first W1 fragments go out before the barrier (their L2 latency overlaps its wait;
        // issued after the X stores, so they do not queue behind the X tile's HBM loads)
        WPre<kIn / 16> pw1;
        if constexpr (kResW1) {
#pragma unroll
            for (int k = 0; k < kIn / 16; ++k) pw1.wf[k] = w1res[k];
        } else {
            w_prefetch(pw1, W1, kIn / 16, ft0, lane);
        }
        // kH2: the head's HBM inputs here; the tile's H2 rows (rows m0 .. m0 + 127 of p.h2_in, [kTR][kHp]
        // bf16 = 66 contiguous 1 KiB pieces) go straight into the H2 slot -- free since the last tile's
        // end barrier -- at layer 1's first k-step, issued by waves 4..7 only (16-17 pieces each).
        // Issuing stalls a wave for ~2.4 k cycles per tile (the CU's memory path); waves 4..7 are the
        // s_setprio 1 half, so while one stalls its SIMD runs the partner's layer 1 (issued by every
        // wave before the barrier instead, the stall sat on every wave's path: profiles/r06/
        // ab_h2_dma_waves47_sched.log, fused_stamps_h2_dma_place.log)
        float hv2 = 0.0f, adv2 = 0.0f;
        float4 a02 = make_float4(0.f, 0.f, 0.f, 0.f);
        constexpr int kPieces = kTR * kHp * 2 / 1024;  // 66
        static_assert(kTR * kHp * 2 % 1024 == 0, "whole 1 KiB pieces");
        if constexpr (kH2) {
            const int64_t m16 = m0 + 16 * wave + (lane & 15), mc = m16 < p.rows ? m16 : p.rows - 1;
            if constexpr (kNet == 1) {
                hv2 = p.ret[mc];
            } else {
                hv2 = p.logp_old[mc];
                a02 = *reinterpret_cast<const float4*>(p.act + mc * kActPad + 4 * (lane >> 4));
                adv2 = p.adv[mc];
            }
        }
        const bool h2_issuer = kH2 && __builtin_amdgcn_readfirstlane(wave) >= kFW / 2;
        const auto h2_dma_k = [&](int sidx) {
            if constexpr (kH2) {
                if (sidx != 0 || !h2_issuer) return;
                const int64_t valid = (p.rows - m0 < kTR ? p.rows - m0 : kTR) * (int64_t)kHp * 2;  // bytes of real rows
                const char* src = reinterpret_cast<const char*>(p.h2_in + m0 * kHp);
                char* dst = reinterpret_cast<char*>(H2);
                for (int q = __builtin_amdgcn_readfirstlane(wave) - kFW / 2; q < kPieces; q += kFW / 2) {
                    int64_t off = (int64_t)q * 1024 + 16 * lane;
                    off = off < valid ? off : valid - 16;  // past the last row: a finite copy of real data
                    glds_x4(src + off, dst + q * 1024);
                }
            }
        };
        STAMP(0);
        __syncthreads();
        STAMP(1);
        // (the next tile's X is fetched late in this one: vmcnt retires in issue order, so an
        // HBM load issued here would make every weight-fragment wait below wait for it too)

        // ---- L1, L2 (wave w: hidden features 64w .. 64w + 63, all 128 samples)
#pragma unroll 1
        for (int j = 0; j < kNT; ++j) {
            // bias = W1 column 45 (X column 45 = 1)
            if (j > 0) w_prefetch(pw1, W1, kIn / 16, ft0 + j, lane);
            EpiTanh e1{H1, 32 * (ft0 + j) + 4 * h, r, nullptr};
            if constexpr (kH2) fwd_pipe<kIn / 16, kXp, kMT>(pw1, X, lane, e1, NoHook{}, false, h2_dma_k);
            else fwd_pipe<kIn / 16, kXp, kMT>(pw1, X, lane, e1);
        }
        // the first W2 fragments go out before the barrier (their L2 latency overlaps its wait)
        WPre<kH / 16> pw2;
        if constexpr (!kResW && !kH2) w_prefetch(pw2, W2, kH / 16, ft0, lane);
        STAMP(2);
        if constexpr (!kH2) __syncthreads();  // (kH2: no L2, so H1 is next read after the head barrier)
        STAMP(3);
        // head inputs (HBM), issued halfway through L2 so their latency hides behind its second half
        const int ml = 32 * wave + r;
        const int64_t m = m0 + ml;
        const bool valid = m < p.rows;
        float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
        // hv: the head's per-sample target -- old log pi (actor) or return (critic); one variable,
        // not two assigned on the two net branches (the compiler merged those stores into one
        // through a selected pointer and kept both in scratch memory)
        float hv = 0.0f, adv = 0.0f;
        float bk[16];
        int bft = ft0;  // feature tile whose biases bk holds
        auto head_inputs = [&]() {
            // the bias loads first: store_hidden waits for them, and must not wait for the HBM loads
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                if constexpr (kResB) bk[q] = bkres[q];
                else bk[q] = tanh_bias(((gf32*)b2)[(int64_t)(32 * bft + 8 * (q >> 2) + 4 * h + (q & 3)) * kHx]);
            }
            if constexpr (kCH16) {
                if (kTrain) {
                    const int64_t m16 = m0 + 16 * wave + (lane & 15);
                    hv = p.ret[m16 < p.rows ? m16 : p.rows - 1];
                }
                return;
            }
            if constexpr (kAH16) {  // sample 16 w + (lane & 15), actions 4 (lane >> 4) .. + 3
                const int64_t m16 = m0 + 16 * wave + (lane & 15), mc = m16 < p.rows ? m16 : p.rows - 1;
                hv = p.logp_old[mc];
                a0 = *reinterpret_cast<const float4*>(p.act + mc * kActPad + 4 * (lane >> 4));
                adv = p.adv[mc];
                return;
            }
            if (!kTrain || __builtin_amdgcn_readfirstlane(wave) >= kHW) return;
            const int64_t mc = valid ? m : p.rows - 1;  // clamped: unconditional loads, no branch
            hv = (actor ? p.logp_old : p.ret)[mc];
            if (actor) {
                a0 = *reinterpret_cast<const float4*>(p.act + mc * kActPad + 4 * h);
                a1 = *reinterpret_cast<const float4*>(p.act + mc * kActPad + 8 + 4 * h);
                adv = p.adv[mc];
            }
        };
#pragma unroll 1
        for (int j = 0; j < (kH2 ? 0 : kNT); ++j) {
            bft = ft0 + j;
            const auto l2_hook = [&]() {
                if (j == kNT - 1) head_inputs();
                else {
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        bk[q] = tanh_bias(((gf32*)b2)[(int64_t)(32 * bft + 8 * (q >> 2) + 4 * h + (q & 3)) * kHx]);
                }
            };
            if (j > 0) w_prefetch(pw2, W2, kH / 16, ft0 + j, lane);
            // (fwd_pipe measured 1 % slower here than the k-major chain + store_hidden)
#if DXRL_L2_PIPE
            EpiTanh e2{H2, 32 * (ft0 + j) + 4 * h, r, bk};
            if constexpr (kResW) {  // biases and head inputs resident: nothing to load
                EpiTanh e2r{H2, 32 * (ft0 + j) + 4 * h, r, bkres};
                fwd_pipe_w<kH / 16, kHp, kMT>(w2res, H1, lane, e2r, (diag & 32) != 0);
            } else {
                fwd_pipe<kH / 16, kHp, kMT>(pw2, H1, lane, e2, l2_hook, (diag & 32) != 0);
            }
#else
            f32x16 acc[kMT];
            fwd_run<kH / 16, kHp, kMT>(pw2, H1, acc, lane, l2_hook, (diag & 32) != 0);
            if (!(diag & 16)) store_hidden(acc, ft0 + j, bk, H2, lane);
#endif
        }
        // forward mode: the head waves' W3 fragments, all 16 k-steps, go out before the barrier
        // (their L2 latency overlaps its wait instead of opening the head phase twice).  Train
        // mode keeps two batches of 8 issued in the head: 16 in flight there spill (the
        // launch-long gradient accumulators are live)
        constexpr int kW3K = kH / 16;
        // (critic train mode, DXRL_HEAD_PF: the first half of the fragments and the head's biases go
        // out here too, so the head opens without an L2 round trip; across the barrier the actor's
        // extra registers spill, so its head keeps its loads)
        constexpr bool kHeadPf = kTrain && DXRL_HEAD_PF && kNet == 1;
        constexpr int kW3P = kTrain ? (kHeadPf ? kW3K / 2 : 1) : kW3K;
        bf16x8 w3p[kW3P];
        float b3p[8];
        const gbf16x8* w3row = (const gbf16x8*)W3 + lane;  // fragment stream, feature tile 0
        // 16-row critic head: the 8 A fragments (head row lane & 15 -- only row 0, the value row,
        // is loaded -- over k 32 ks + 8 (lane >> 4) ..) and the value bias, on every wave
        bf16x8 w3h[kH16 ? 8 : 1];
        float b3h = 0.0f;
        if constexpr (kAH16) {  // head rows lane & 15 (0..14 the means, 15 zero)
            const bf16* W3rm = opaque(p.W3rm) + (lane & 15) * kHx + 8 * (lane >> 4);
#pragma unroll
            for (int k = 0; k < 8; ++k) w3h[k] = *(const gbf16x8*)(W3rm + 32 * k);
        }
        if constexpr (kResH) {
#pragma unroll
            for (int k = 0; k < 8; ++k) w3h[k] = w3res[k];
            b3h = b3res;
        } else if constexpr (kCH16) {
            const bf16* W3rm = opaque(p.W3rm);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                w3h[k] = (lane & 15) == 0 ? *(const gbf16x8*)(W3rm + 32 * k + 8 * (lane >> 4)) : zero8();
            b3h = ((gf32*)b3)[0];
        }
        if (!kH16 && (!kTrain || kHeadPf)) {
            if (wave < kHW) {
#pragma unroll
                for (int k = 0; k < kW3P; ++k) w3p[k] = w3row[64 * k];
                if (kTrain) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) b3p[q] = ((gf32*)b3)[(int64_t)((q & 3) + 8 * (q >> 2) + 4 * h) * kHx];
                }
            }
        }
        if constexpr (kH2) {
            hv = hv2;
            a0 = a02;
            adv = adv2;
            // vmcnt(0) on the issuing waves: their H2 pieces landed before the head barrier (the other
            // waves' own loads are waited for by the compiler where they are used; a vmcnt(0) there
            // too only waited out the head's weight loads: profiles/r06/ab_h2_dma_wait_issuers.log)
            if (h2_issuer) __builtin_amdgcn_s_waitcnt(0xF70);
        }
        STAMP(4);
        __syncthreads();
        STAMP(5);

        // ---- head: wave w < kHW owns samples 32w .. 32w + 31 (lane: sample r, head rows of half h)
        // H1 tile -> HBM (B operand of the dW2 GEMM) by the waves that have no head tile; their
        // stores then retire while the head runs instead of holding the head's load waits
        if constexpr (kTrain && kFW > kHW && !kH16) {
            if (wave >= kHW && p.h1_out)
                copy_tile_out_n<64 * (kFW - kHW), kTR>(H1, p.h1_out, kHx, m0, p.rows, tid - 64 * kHW, diag);
        }
        if constexpr (kCH16) {
            // wave w: samples 16 w .. 16 w + 15; V of sample 16 w + l in lane l < 16 (row 0, reg 0)
            const int s16 = 16 * wave + (lane & 15);
            const bf16* hb = H2 + s16 * kHp + 8 * (lane >> 4);
            f32x4 a16 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 8; ++k) a16 = mfma16(w3h[k], *reinterpret_cast<const bf16x8*>(hb + 32 * k), a16);
            const int64_t m16 = m0 + s16;
            const bool v16 = m16 < p.rows && lane < 16;
            const float v = a16[0] + b3h;
            float d0 = 0.0f;
            if (!kTrain) {
                if (v16) p.v_out[m16] = v;
            } else if (v16) {
                const float e = v - hv;  // hv: the return
                d0 = from_bf16(to_bf16(p.vf2 * e * p.sc));
                db3[0] += d0;
                lsum[1] += e * e;
            }
            if (kTrain) {  // dout row of sample s16: d0 in column 0, zeros in 1..31 (lane >> 4: 8 columns)
                bf16x8 dv = zero8();
                if (lane < 16) dv[0] = to_bf16(d0);
                *reinterpret_cast<bf16x8*>(D + s16 * kDp + 8 * (lane >> 4)) = dv;
            }
        } else if constexpr (kAH16) {
            // wave w: samples 16 w .. + 15; lane l holds head rows o = 4 (l >> 4) + i of sample l & 15
            const int s16 = 16 * wave + (lane & 15), g4 = lane >> 4;
            const bf16* hb = H2 + s16 * kHp + 8 * g4;
            f32x4 a16 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 8; ++k) a16 = mfma16(w3h[k], *reinterpret_cast<const bf16x8*>(hb + 32 * k), a16);
            const int64_t m16 = m0 + s16;
            const bool v16 = m16 < p.rows;
            float mu[4], a[4], lsv[4], iv2[4], t[4], d[4];
            a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = 4 * g4 + i;
                if constexpr (kResA) lsv[i] = ahls[i];
                else lsv[i] = o < kAct ? ((gf32*)logstd)[o] : 0.0f;
                iv2[i] = __expf(-2.0f * lsv[i]);
                if constexpr (kResA) mu[i] = a16[i] + ahb3[i];
                else mu[i] = a16[i] + ((gf32*)b3)[(int64_t)o * kHx];
                const float z = (a[i] - mu[i]) * __expf(-lsv[i]);
                t[i] = o < kAct ? -0.5f * z * z - lsv[i] - 0.5f * kLog2PiF : 0.0f;
                d[i] = 0.0f;
            }
            // log pi(a|s): the sample's 15 terms gathered from its four lanes, summed in action order
            float tt[16];
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) tt[4 * g + i] = __shfl(t[i], (lane & 15) + 16 * g);
            float lp = 0.0f;
#pragma unroll
            for (int o = 0; o < kAct; ++o) lp += tt[o];
            const float lo = hv;
            const float ratio = __expf(lp - lo);
            const float A = (float)(((double)adv - adv_mean) * adv_inv);
            const float s1 = ratio * A;
            const float rc = fminf(fmaxf(ratio, 1.0f - p.clip_eps), 1.0f + p.clip_eps);
            const float s2 = rc * A;
            float g = 0.0f;
            if (s1 <= s2 || ratio == rc) g = -A * ratio;  // d(-min(s1, s2)) / d logp
            g *= p.sc;
            if (v16) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int o = 4 * g4 + i;
                    if (o < kAct) {
                        const float dd = a[i] - mu[i];
                        d[i] = from_bf16(to_bf16(g * dd * iv2[i]));  // dlogp/dmu = (a - mu) / sigma^2
                        dls[i] += g * (dd * dd * iv2[i] - 1.0f);       // dlogp/dlogstd
                        db3[i] += d[i];
                    }
                }
                if (g4 == 0) {
                    lsum[0] += -fminf(s1, s2);
                    lsum[2] += fabsf(ratio - 1.0f) > p.clip_eps ? 1.0f : 0.0f;
                    lsum[3] += lo - lp;
                }
            }
            bf16x4 dv, zv;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dv[i] = to_bf16(d[i]);
                zv[i] = (bf16)0.0f;
            }
            *reinterpret_cast<bf16x4*>(D + s16 * kDp + 4 * g4) = dv;        // head rows 4 g4 .. + 3
            *reinterpret_cast<bf16x4*>(D + s16 * kDp + 16 + 4 * g4) = zv;   // rows 16 .. 31: zero
        } else if (wave < kHW) {
            f32x16 acc;
            zero_acc(acc);
            if constexpr (!kTrain) {
#pragma unroll
                for (int k = 0; k < kW3K; ++k) {
                    const bf16x8 b = *reinterpret_cast<const bf16x8*>(H2 + (32 * wave + r) * kHp + 16 * k + 8 * h);
                    acc = mfma32(w3p[k], b, acc);
                }
            } else {
                constexpr int kB = kW3K / 2;  // fragments per batch (32 registers in flight)
                bf16x8 w3f[kB];
                if constexpr (kHeadPf) {
                    // second batch in flight under the first (prefetched) batch's MFMAs
#pragma unroll
                    for (int k = 0; k < kB; ++k) w3f[k] = w3row[64 * (k + kB)];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = 0; k < kB; ++k) {
                        const bf16x8 b = *reinterpret_cast<const bf16x8*>(H2 + (32 * wave + r) * kHp + 16 * k + 8 * h);
                        acc = mfma32(w3p[k], b, acc);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                } else {
#pragma unroll
                    for (int k = 0; k < kB; ++k) w3f[k] = w3row[64 * k];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = 0; k < kB; ++k) {
                        const bf16x8 b = *reinterpret_cast<const bf16x8*>(H2 + (32 * wave + r) * kHp + 16 * k + 8 * h);
                        acc = mfma32(w3f[k], b, acc);
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = 0; k < kB; ++k) w3f[k] = w3row[64 * (k + kB)];
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const bf16x8 b = *reinterpret_cast<const bf16x8*>(H2 + (32 * wave + r) * kHp + 16 * (k + kB) + 8 * h);
                    acc = mfma32(w3f[k], b, acc);
                }
            }
            float d[8], b3v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                d[q] = 0.0f;
                // head row o of register q
                b3v[q] = kHeadPf ? b3p[q] : ((gf32*)b3)[(int64_t)((q & 3) + 8 * (q >> 2) + 4 * h) * kHx];
            }
            if (actor) {
                if (kTrain) {
                    float mu[8], a[8], lsv[8], iv2[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int o = (q & 3) + 8 * (q >> 2) + 4 * h;
                        lsv[q] = o < kAct ? ((gf32*)logstd)[o] : 0.0f;
                        iv2[q] = __expf(-2.0f * lsv[q]);
                    }
                    a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w;
                    a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
                    // log pi(a|s): the 15 terms summed in action order (as the rollout sampled
                    // them), so the first update's ratios are exactly 1
                    float t[8], u[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int o = (q & 3) + 8 * (q >> 2) + 4 * h;
                        mu[q] = acc[q] + b3v[q];
                        const float z = (a[q] - mu[q]) * __expf(-lsv[q]);
                        t[q] = o < kAct ? -0.5f * z * z - lsv[q] - 0.5f * kLog2PiF : 0.0f;
                    }
#pragma unroll
                    for (int q = 0; q < 8; ++q) u[q] = __shfl_xor(t[q], 32);
                    float lp = 0.0f;
#pragma unroll
                    for (int q = 0; q < 4; ++q) lp += h ? u[q] : t[q];      // o = 0..3
#pragma unroll
                    for (int q = 0; q < 4; ++q) lp += h ? t[q] : u[q];      // o = 4..7
#pragma unroll
                    for (int q = 4; q < 8; ++q) lp += h ? u[q] : t[q];      // o = 8..11
#pragma unroll
                    for (int q = 4; q < 7; ++q) lp += h ? t[q] : u[q];      // o = 12..14
                    const float lo = hv;
                    const float ratio = __expf(lp - lo);
                    const float A = (float)(((double)adv - adv_mean) * adv_inv);
                    const float s1 = ratio * A;
                    const float rc = fminf(fmaxf(ratio, 1.0f - p.clip_eps), 1.0f + p.clip_eps);
                    const float s2 = rc * A;
                    float g = 0.0f;
                    if (s1 <= s2 || ratio == rc) g = -A * ratio;  // d(-min(s1, s2)) / d logp
                    g *= p.sc;
                    if (valid) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const int o = (q & 3) + 8 * (q >> 2) + 4 * h;
                            if (o < kAct) {
                                const float dd = a[q] - mu[q];
                                d[q] = from_bf16(to_bf16(g * dd * iv2[q]));  // dlogp/dmu = (a - mu) / sigma^2
                                dls[q] += g * (dd * dd * iv2[q] - 1.0f);       // dlogp/dlogstd
                                db3[q] += d[q];
                            }
                        }
                        if (h == 0) {
                            lsum[0] += -fminf(s1, s2);
                            lsum[2] += fabsf(ratio - 1.0f) > p.clip_eps ? 1.0f : 0.0f;
                            lsum[3] += lo - lp;
                        }
                    }
                }
            } else {
                const float v = acc[0] + b3v[0];  // lanes h == 0 hold head row 0
                if (!kTrain) {
                    if (valid && h == 0) p.v_out[m] = v;
                } else if (valid && h == 0) {
                    const float e = v - hv;  // hv: the return
                    d[0] = from_bf16(to_bf16(p.vf2 * e * p.sc));
                    db3[0] += d[0];
                    lsum[1] += e * e;
                }
            }
            if (kTrain) {
#pragma unroll
                for (int g2 = 0; g2 < 4; ++g2) {  // head rows 8 g2 + 4 h .. + 3
                    bf16x4 v;
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = g2 < 2 ? to_bf16(d[4 * g2 + u]) : (bf16)0.0f;
                    *reinterpret_cast<bf16x4*>(D + ml * kDp + 8 * g2 + 4 * h) = v;
                }
            }
        }
        STAMP(6);
        if (!kTrain) {
            // (h2_out: H2 for the critic's train pass, as k_pg_values writes it)
            if (p.h2_out) copy_tile_out_n<kFThreads, kTR>(H2, p.h2_out, kHp, m0, p.rows, tid, diag);
            if (!kEarlyX && tile + gridDim.x < ntiles) fetch_x(tile + gridDim.x);
            __syncthreads();  // X / H1 / H2 are rewritten by the next tile
            STAMP(7);
            continue;
        }
        if constexpr (kFW == kHW || kH16) {
            if (p.h1_out) copy_tile_out_n<kFThreads, kTR>(H1, p.h1_out, kHx, m0, p.rows, tid, diag);
        }
        WPre<1> pw3t;  // dH2's one W3T fragment, ahead of the barrier
        w_prefetch(pw3t, W3T, kOut / 16, ft0, lane);
        STAMP(7);
        __syncthreads();
        STAMP(8);

        // ---- dW3 += dout^T H2 (wave w: H2 columns of its tiles), then dH2 in place of H2
#pragma unroll
        for (int kk = 0; kk < kTR; kk += 32) {
            const bf16x8 a = wg_frag<kDp>(D, 0, kk, lane);
#pragma unroll
            for (int j = 0; j < kNT; ++j)
#pragma unroll
                for (int ci = 0; ci < 2; ++ci)
                    if (!(diag & 4))
                        acc3[j][ci] = mfma16(a, wg_frag<kHp>(H2, 32 * (ft0 + j) + 16 * ci, kk, lane), acc3[j][ci]);
        }
#pragma unroll 1
        for (int j = 0; j < kNT; ++j) {
            f32x16 acc[kMT];
            bf16x4 ys[4][kMT];
            gate_load(ys, ft0 + j, H2, lane);
            // dH2^T = W3^T dout^T over head rows 0..15 (dout rows 16..31 are zero)
            if (j == 0) fwd_run<1, kDp, kMT>(pw3t, D, acc, lane);
            else fwd_tiles<1, kDp, kMT>(W3T, kOut / 16, ft0 + j, D, acc, lane);
            gate_store(acc, ys, ft0 + j, H2, lane);
        }
        WPre<kH / 16> pw2t;  // dH1's first W2T fragments, ahead of the barrier
        w_prefetch(pw2t, W2T, kH / 16, ft0, lane);
        STAMP(9);
        __syncthreads();
        STAMP(10);

        // ---- db2 column sums of dH2, stage 1: wave w sums rows w * kTR / kFW.. for the 4 columns
        //      4 lane..; the per-wave sums go to the (dead) dout region, stage 2 follows in dW1.
        //      dH1 = (dH2 W2) * (1 - H1^2)  (wave w: L2 inputs of its tiles, rows = samples)
        {
            constexpr int kRows = kTR / kFW;
            float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);  // padding rows carry dH2 = 0 (their dout is 0)
            const bf16* hp = H2 + (kRows * wave) * kHp + 4 * lane;
            // every row read before the first add (read and summed row by row, the compiler waited
            // out each pair of reads in turn: eight LDS round trips per tile); same adds, same order
            bf16x4 rv[kRows];
#pragma unroll
            for (int rr = 0; rr < kRows; ++rr) rv[rr] = *reinterpret_cast<const bf16x4*>(hp + rr * kHp);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int rr = 0; rr < kRows; ++rr) {
                const bf16x4 v = rv[rr];
                cs.x += from_bf16(v[0]);
                cs.y += from_bf16(v[1]);
                cs.z += from_bf16(v[2]);
                cs.w += from_bf16(v[3]);
            }
            reinterpret_cast<float4*>(lds + kOffD)[wave * 64 + lane] = cs;
        }
#pragma unroll 1
        for (int j = 0; j < kNT; ++j) {
            // dH1^T = W2^T dH2^T, gated in place of H1
            if (j > 0) w_prefetch(pw2t, W2T, kH / 16, ft0 + j, lane);
            EpiGate eg{H1, 32 * (ft0 + j) + 4 * h, r};
#if DXRL_DH2_IN_DH1
            // dH2 tile -> HBM (Y of the dW2 GEMM) in this phase's shadow: one 16-byte chunk per
            // thread every 8th step (the stores go out after every weight fragment, so no
            // fragment wait queues behind them; H2 holds dH2 read-only here)
            // The chunks go out from the second sample tile on (k-step 16 + kEvery i): a store
            // issued among the first tile's k-steps, while W2T fragments still stream in, made
            // the compiler's vmcnt waits for them one fragment deeper (and the last one a full
            // drain, the store's row guard being a branch).  Each chunk is read from LDS three
            // steps ahead of its store (read right before it, its wait drained every LDS read in
            // flight, the B-operand prefetch included).
            bf16x8 cv;
            const auto copy_k = [&](int sidx) {
                // (64-sample tiles: too few steps after the first tile; they start at step 3)
                constexpr int kSteps = kMT * (kH / 16);
                constexpr int kFirst = (kSteps - kH / 16) / kCopyU >= 4 ? kH / 16 : 2;
                constexpr int kEvery = (kSteps - kFirst) / kCopyU, kAhead = kEvery >= 4 ? 3 : kEvery - 1;
                static_assert(kAhead >= 1 && kFirst >= kAhead && kFirst + kEvery * kCopyU <= kSteps, "copy schedule");
                if (diag & 1 || sidx < kFirst - kAhead) return;
                const int i = (sidx - (kFirst - kAhead)) / kEvery, ph = (sidx - (kFirst - kAhead)) % kEvery;
                const int c = tid_l + kFThreads * i, row = c >> 5, col = 8 * (c & 31);
                if (ph == 0 && i < kCopyU) cv = *reinterpret_cast<const bf16x8*>(H2 + row * kHp + col);
                if (ph == kAhead && i < kCopyU && m0 + row < p.rows) store_dh2(p.dh2_out + (m0 + row) * kH + col, cv);
            };
            if constexpr (kDw1Tail) {
                // dW1 of sample blocks 0..2 (gated during the tile loop) beside the tail epilogue
                // of block 3; block 3's dW1 follows it (same MFMAs, same kk order as below)
                const auto dw1_tail = [&](int q) {
                    if (q != 1 && q != 3 && q != 5) return;
                    const int kk = 32 * (q >> 1);
                    if (kk == 0 && tile + gridDim.x < ntiles) fetch_x(tile + gridDim.x);
                    bf16x8 b[3];
#pragma unroll
                    for (int ci = 0; ci < 3; ++ci) b[ci] = wg_frag<kXp>(X, 16 * ci, kk, lane);
#pragma unroll
                    for (int ri = 0; ri < 2; ++ri) {
                        const bf16x8 a = wg_frag<kHp>(H1, 32 * ft0 + 16 * ri, kk, lane);
#pragma unroll
                        for (int ci = 0; ci < 3; ++ci)
                            if (!(diag & 4)) acc1[0][ri][ci] = mfma16(a, b[ci], acc1[0][ri][ci]);
                    }
                };
                fwd_pipe<kH / 16, kHp, kMT>(pw2t, H2, lane, eg, NoHook{}, false, copy_k, dw1_tail);
            } else {
                fwd_pipe<kH / 16, kHp, kMT>(pw2t, H2, lane, eg, NoHook{}, false, copy_k);
            }
#else
            fwd_pipe<kH / 16, kHp, kMT>(pw2t, H2, lane, eg);
#endif
        }
        STAMP(11);
        const auto db2_stage2 = [&]() {
            if (tid < kH) {  // db2 stage 2: the kFW row-group sums of column tid, in row order
                const float* cs = reinterpret_cast<const float*>(lds + kOffD);
#pragma unroll
                for (int w = 0; w < kFW; ++w) db2 += cs[w * kH + tid_l];
            }
        };
        if constexpr (!kDw1Tail) {
            __syncthreads();
            STAMP(12);
            // ---- dW1 += dH1^T X (wave w: hidden rows of its tiles, input columns 0..63); LDS only,
            //      so the next tile's X loads go out now
            if (tile + gridDim.x < ntiles) fetch_x(tile + gridDim.x);
#if !DXRL_DH2_IN_DH1
            // dH2 tile -> HBM (Y of the dW2 GEMM; H2 holds dH2 until the next tile's L2)
            copy_tile_out_n<kFThreads, kTR>(H2, p.dh2_out, kH, m0, p.rows, tid, diag);
#endif
            db2_stage2();
        }
#pragma unroll
        for (int kk = kDw1Tail ? 96 : 0; kk < kTR; kk += 32) {
            bf16x8 b[3];
#pragma unroll
            for (int ci = 0; ci < 3; ++ci) b[ci] = wg_frag<kXp>(X, 16 * ci, kk, lane);
#pragma unroll
            for (int j = 0; j < kNT; ++j)
#pragma unroll
                for (int ri = 0; ri < 2; ++ri) {
                    const bf16x8 a = wg_frag<kHp>(H1, 32 * (ft0 + j) + 16 * ri, kk, lane);
#pragma unroll
                    for (int ci = 0; ci < 3; ++ci)
                        if (!(diag & 4)) acc1[j][ri][ci] = mfma16(a, b[ci], acc1[j][ri][ci]);
                }
        }
        STAMP(13);
        __syncthreads();
        STAMP(14);
        // (kDw1Tail: the dout region holding the row-group sums is not written again before the
        // next tile's head, two barriers on)
        if constexpr (kDw1Tail) db2_stage2();
    }
    if ((diag & 8) && lane == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) p.stamps[((int64_t)blockIdx.x * kFW + wave) * 16 + k] = st_acc[k];
    }
#undef STAMP
    if (!kTrain) return;

    // ---- workgroup partials (fixed layout; summed in a fixed order by launch_slab_reduce)
    float* part = p.part + (int64_t)blockIdx.x * kPartSize;
    {
        const int c16 = lane & 15, g16 = lane >> 4;
#pragma unroll
        for (int j = 0; j < kNT; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = 4 * g16 + i;  // head row (rows 16..31 stay zero: k_fused_scatter)
#pragma unroll
                for (int ci = 0; ci < 2; ++ci) part[kPartW3 + o * kPW3C + 32 * (ft0 + j) + 16 * ci + c16] = acc3[j][ci][i];
#pragma unroll
                for (int ri = 0; ri < 2; ++ri) {
                    float* row = part + kPartW1 + (32 * (ft0 + j) + 16 * ri + o) * kPW1C;
#pragma unroll
                    for (int ci = 0; ci < 3; ++ci) row[16 * ci + c16] = acc1[j][ri][ci][i];
                }
            }
    }
    if (tid < kH) part[kPartB2 + tid] = db2;
    if constexpr (kCH16) {
        // value-head bias gradient and value loss: lanes 0..15 of every wave, summed in
        // (wave, lane) order
        float* red = reinterpret_cast<float*>(lds);
        double* lred = reinterpret_cast<double*>(lds + kOffH1);
        red[tid] = db3[0];
        lred[tid] = (double)lsum[1];
        __syncthreads();
        if (tid < 32) {
            float sb = 0.0f;
            if (tid == 0)
                for (int w = 0; w < kFW; ++w)
                    for (int rr = 0; rr < 16; ++rr) sb += red[64 * w + rr];
            if (tid < 16) {
                part[kPartW3 + tid * kPW3C + kH] = sb;  // bias column of head row tid (rows > 0: zero)
                part[kPartLs + tid] = 0.0f;
            }
        } else if (tid == 33) {
            double s = 0.0;
            for (int w = 0; w < kFW; ++w)
                for (int rr = 0; rr < 16; ++rr) s += lred[64 * w + rr];
            p.loss[(int64_t)blockIdx.x * 4 + 1] = s;
            for (int r = blockIdx.x + gridDim.x; r < p.loss_rows; r += gridDim.x) p.loss[(int64_t)r * 4 + 1] = 0.0;
        }
        return;
    }
    if constexpr (kAH16) {
        // head rows o = 4 g + i of lanes 16 g .. 16 g + 15 of every wave, summed in (wave, lane)
        // order; the loss terms over every lane in thread order
        float* red = reinterpret_cast<float*>(lds);              // [512][8]: dls[0..3], db3[0..3]
        double* lred = reinterpret_cast<double*>(lds + kOffH1);  // [512][4]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            red[tid * 8 + i] = dls[i];
            red[tid * 8 + 4 + i] = db3[i];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) lred[tid * 4 + k] = (double)lsum[k];
        __syncthreads();
        if (tid < 32) {
            const int o = tid, g = (o >> 2) & 3, i = o & 3;
            float sl = 0.0f, sb = 0.0f;
            if (o < 16) {
                for (int w = 0; w < kFW; ++w)
                    for (int rr = 0; rr < 16; ++rr) {
                        const int t = 64 * w + 16 * g + rr;
                        sl += red[t * 8 + i];
                        sb += red[t * 8 + 4 + i];
                    }
            }
            if (o < 16) {
                part[kPartW3 + o * kPW3C + kH] = sb;  // bias column of the head
                part[kPartLs + o] = sl;
            }
        } else if (tid < 36) {
            const int k = tid - 32;
            if (k != 1) {
                double s = 0.0;
                for (int t = 0; t < kFThreads; ++t) s += lred[t * 4 + k];
                p.loss[(int64_t)blockIdx.x * 4 + k] = s;
                for (int r = blockIdx.x + gridDim.x; r < p.loss_rows; r += gridDim.x) p.loss[(int64_t)r * 4 + k] = 0.0;
            }
        }
        return;
    }
    float* red = reinterpret_cast<float*>(lds);              // [head lanes][16]
    double* lred = reinterpret_cast<double*>(lds + kOffH1);  // [head lanes][4]
    if (wave < kHW) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            red[tid * 16 + q] = dls[q];
            red[tid * 16 + 8 + q] = db3[q];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) lred[tid * 4 + k] = (double)lsum[k];
    }
    __syncthreads();
    if (tid < 32) {  // head row o: lanes with h = (o >> 2) & 1, register q = (o & 3) + 4 (o >> 3)
        const int o = tid, hh = (o >> 2) & 1, q = (o & 3) + 4 * (o >> 3);
        float sl = 0.0f, sb = 0.0f;
        if (o < 16) {
            for (int w = 0; w < kHW; ++w)
                for (int rr = 0; rr < 32; ++rr) {
                    const int t = 64 * w + 32 * hh + rr;
                    sl += red[t * 16 + q];
                    sb += red[t * 16 + 8 + q];
                }
        }
        if (o < 16) {
            part[kPartW3 + o * kPW3C + kH] = sb;  // bias column of the head
            part[kPartLs + o] = sl;
        }
    } else if (tid < 36) {
        const int k = tid - 32;
        double s = 0.0;
        for (int t = 0; t < 64 * kHW; ++t) s += lred[t * 4 + k];
        if (actor == (k != 1)) {
            p.loss[(int64_t)blockIdx.x * 4 + k] = s;
            // rows of workgroups this launch does not have (fewer tiles than the caller's grid):
            // zeroed, so a sum over all rows never picks up an earlier, larger pass
            for (int r = blockIdx.x + gridDim.x; r < p.loss_rows; r += gridDim.x) p.loss[(int64_t)r * 4 + k] = 0.0;
        }
    }
}

// One element of the grads blocks W1 / W3 / log_std (actor) / W2's column 256 + pads from the
// workgroup sum s = sum[j] (k_fused_scatter's mapping; `j` indexes the partial-slab layout).
// Returns the value stored into the gradient element slab entry j maps to (0 when it maps to
// none; the pads it zeroes contribute nothing to a norm).
__device__ __forceinline__ float fused_scatter_one(int j, float s, float* __restrict__ gW1, float* __restrict__ gW3,
                                                   float* __restrict__ gLs, float* __restrict__ gW2, float ent_coef) {
    if (j >= kPartB2) {  // W2 block column 256 (bias) and the zero pad columns 257..287 of row n
        const int n = j - kPartB2;
        if (n < kH) {
            gW2[(int64_t)n * kHx + kH] = s;
            for (int c = kH + 1; c < kHx; ++c) gW2[(int64_t)n * kHx + c] = 0.0f;
            return s;
        }
        return 0.0f;
    }
    if (j < kPartW3) {  // dW1 [256][64]: columns 0..47 from the slab, 48..63 zero
        const int row = j / kPW1C, col = j % kPW1C;
        gW1[row * kIn + col] = s;
        if (col < kIn - kPW1C) gW1[row * kIn + kPW1C + col] = 0.0f;
        return s;
    }
    if (j < kPartLs) {  // dW3 [32][288]: rows 0..15 columns 0..256 from the slab, the rest zero
        const int o = (j - kPartW3) / kPW3C, col = (j - kPartW3) % kPW3C;
        if (col <= kH) gW3[o * kHx + col] = s;
        if (col < kH) {
            gW3[(16 + o) * kHx + col] = 0.0f;  // rows 16..31
        } else if (col == kH) {  // row o's pad columns 257..287, row 16 + o's columns 256..287
            for (int c = kH + 1; c < kHx; ++c) gW3[o * kHx + c] = 0.0f;
            for (int c = kH; c < kHx; ++c) gW3[(16 + o) * kHx + c] = 0.0f;
        }
        return col <= kH ? s : 0.0f;
    }
    if (gLs) {
        const int k = j - kPartLs;
        const float v = k < kAct ? s - ent_coef : 0.0f;
        gLs[k] = v;
        return v;
    }
    return 0.0f;
}

// f64 squares of four stored gradient values, summed in one fixed order
__device__ __forceinline__ double sumsq4(float a, float b, float c, float d) {
    return (((double)a * a + (double)b * b) + (double)c * c) + (double)d * d;
}

// Critic values (the forward-only pass) as its own kernel, pipelined across tiles: the layer-by-layer
// instantiation k_pg_fused<8, 128, false, 1> closes four barriers per tile (X stored, L1 -> L2,
// L2 -> head, end of tile).  Here the next tile's X is stored while L2 runs (X is free once L1 is
// done) and the next tile's L1 runs beside this tile's value head (H1 is free once L2 is done, H2
// is not written again until the next L2): two barriers per tile.  Rows: every workgroup runs the
// same number of whole 128-row tiles, then one share of the remaining rows (< 128 per workgroup,
// ceil(remainder / grid) each) as a short tile of 1-4 32-row MFMA tiles -- at the bench shape the
// T + 1 observation blocks are 25 tiles and 16 rows per workgroup, where the layer-by-layer grid
// ran a 26th round of whole tiles on 32 workgroups.  Same resident W1 / W2 / biases / value row,
// same fwd_pipe_w chains, epilogues and 16x16x32 head as the layer-by-layer pass, and a row's V
// depends only on its own observation row, so V is bit for bit that pass's V
// (test_values_kernel_equals_layer_by_layer_pass).
#ifndef DXRL_FWD_VALUES
#define DXRL_FWD_VALUES 1
#endif
#ifndef DXRL_VALUES_HEAD_SPLIT
#define DXRL_VALUES_HEAD_SPLIT 1
#endif
template <int KS, int kLda, typename Epi>
__device__ __forceinline__ void fwd_pipe_w_mt(int mt, const bf16x8 (&wf)[KS], const bf16* A, int lane, Epi& epi) {
    switch (mt) {  // workgroup-uniform
        case 1: fwd_pipe_w<KS, kLda, 1>(wf, A, lane, epi); break;
        case 2: fwd_pipe_w<KS, kLda, 2>(wf, A, lane, epi); break;
        case 3: fwd_pipe_w<KS, kLda, 3>(wf, A, lane, epi); break;
        default: fwd_pipe_w<KS, kLda, 4>(wf, A, lane, epi); break;
    }
}
__global__ __launch_bounds__(512, 1) void k_pg_values(FusedArgs p) {
    using L = TileLds<128>;
    constexpr int kXU = 128 * (kIn / 8) / 512;
    __shared__ __attribute__((aligned(16))) bf16 lds[L::kElems];
    bf16* X = lds + L::kOffX;
    bf16* H1 = lds + L::kOffH1;
    bf16* H2 = lds + L::kOffH2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
#if DXRL_FUSED_PRIO
    if (__builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);
#endif
    // this workgroup's tiles: k < full -> rows (b + k G) 128 .. + 127; k == full -> its share of the rest
    const int64_t G = gridDim.x, b = blockIdx.x;
    const int64_t full = p.rows / 128 / G, main_rows = full * G * 128, rem = p.rows - main_rows;
    const int64_t rper = (rem + G - 1) / G;  // <= 128 (rem < 128 G)
    const int64_t r_lo = main_rows + b * rper, r_hi = min(p.rows, r_lo + rper);
    const int64_t ntile = full + (r_hi > r_lo ? 1 : 0);
    if (ntile == 0) return;  // workgroup-uniform
    const auto row0 = [&](int64_t k) { return k < full ? (b + k * G) * 128 : r_lo; };
    const auto count = [&](int64_t k) { return k < full ? (int64_t)128 : r_hi - r_lo; };
    bf16x8 xr[kXU];
    const auto fetch_x = [&](int64_t k) {
        const int64_t base = row0(k), cnt = count(k);
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int c = tid + 512 * u, row = c >> 3, col = 8 * (c & 7);
            xr[u] = row < cnt ? *reinterpret_cast<const bf16x8*>(p.X + (base + row) * kIn + col) : zero8();
        }
    };
    const auto store_x = [&]() {
#pragma unroll
        for (int u = 0; u < kXU; ++u) {
            const int c = tid + 512 * u, row = c >> 3, col = 8 * (c & 7);
            *reinterpret_cast<bf16x8*>(X + row * kXp + col) = xr[u];
        }
    };
    int64_t k = 0;
    fetch_x(k);
    // this wave's 32 hidden units: W1 / W2 fragments, layer-2 biases, the value row (resident)
    bf16x8 w1[kIn / 16], w2[kH / 16], w3h[8];
    {
        const gbf16x8* p1 = (const gbf16x8*)p.W1 + (int64_t)wave * (kIn / 16) * 64 + lane;
#pragma unroll
        for (int q = 0; q < kIn / 16; ++q) w1[q] = p1[64 * q];
        const gbf16x8* p2 = (const gbf16x8*)p.W2 + (int64_t)wave * (kH / 16) * 64 + lane;
#pragma unroll
        for (int q = 0; q < kH / 16; ++q) w2[q] = p2[64 * q];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            w3h[q] = (lane & 15) == 0 ? *(const gbf16x8*)(p.W3rm + 32 * q + 8 * (lane >> 4)) : zero8();
    }
    float bk[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) bk[q] = tanh_bias(((gf32*)p.b2)[(int64_t)(32 * wave + 8 * (q >> 2) + 4 * h + (q & 3)) * kHx]);
    const float b3h = ((gf32*)p.b3)[0];
    EpiTanh e1{H1, 32 * wave + 4 * h, r, nullptr};
    EpiTanhB e2{H2, 32 * wave + 4 * h, r, {}, {}};
#pragma unroll
    for (int q = 0; q < 16; ++q) e2.bk[q] = bk[q];
    const auto mts = [&](int64_t kk) { return (int)((count(kk) + 31) / 32); };  // 32-row MFMA tiles
    store_x();
    if (k + 1 < ntile) fetch_x(k + 1);
    __syncthreads();
    fwd_pipe_w_mt<kIn / 16, kXp>(mts(k), w1, X, lane, e1);
    __syncthreads();  // H1 of the first tile complete, X free
    for (;;) {
        fwd_pipe_w_mt<kH / 16, kHp>(mts(k), w2, H1, lane, e2);
        if (k + 1 < ntile) {
            store_x();  // X(k + 1): every wave finished L1(k) before the last barrier
            if (k + 2 < ntile) fetch_x(k + 2);
        }
        __syncthreads();  // H2(k) and X(k + 1) complete; H1 free
        // h2_out: this tile's H2 rows for the critic's train pass (the slot is rewritten only by
        // the next tile's L2, after the next barrier)
        if (p.h2_out) {
            // non-temporal stores: the stream is read back once, by the critic's train pass (plain
            // stores: iteration 1.66-1.67 vs 1.62-1.63 ms, profiles/r06/ab_h2_variants.log; the
            // copy spread over the next layer 1's steps was slower still, ab_h2_spread_rejected.log;
            // issued by waves 4..7 only: no change, ab_values_h2_half_rejected.log)
            const int64_t h2_m0 = row0(k), h2_end = row0(k) + count(k);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int c = tid + 512 * u, row = c >> 5, col = 8 * (c & 31);
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(H2 + row * kHp + col);
                if (h2_m0 + row < h2_end)
                    __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p.h2_out + (h2_m0 + row) * kHp + col));
            }
        }
        const auto head = [&]() {  // value head: wave w, samples 16 w .. + 15; V of sample 16 w + l in lane l < 16
            const int s16 = 16 * wave + (lane & 15);
            if (s16 < 32 * mts(k)) {  // (rows past the tile's MFMA tiles were never computed)
                const bf16* hb = H2 + s16 * kHp + 8 * (lane >> 4);
                f32x4 a16 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int q = 0; q < 8; ++q) a16 = mfma16(w3h[q], *reinterpret_cast<const bf16x8*>(hb + 32 * q), a16);
                if (s16 < count(k) && lane < 16) p.v_out[row0(k) + s16] = a16[0] + b3h;
            }
        };
        if (k + 1 >= ntile) {
            head();
            break;
        }
        // L1(k + 1) beside the heads: the two waves of a SIMD in opposite orders, so one's head MFMAs
        // run beside the other's L1 epilogue (DXRL_VALUES_HEAD_SPLIT; 0: head first on every wave)
        if (DXRL_VALUES_HEAD_SPLIT && __builtin_amdgcn_readfirstlane(wave) >= 4) {
            fwd_pipe_w_mt<kIn / 16, kXp>(mts(k + 1), w1, X, lane, e1);
            head();
        } else {
            head();
            fwd_pipe_w_mt<kIn / 16, kXp>(mts(k + 1), w1, X, lane, e1);
        }
        __syncthreads();  // H1(k + 1) complete; H2 and X free
        ++k;
    }
}

// The workgroup partials summed and scattered in one launch: a 256-thread block owns 16 float4
// columns of the [z][kPartSize] slabs; with z > kReduceGroups thread (g, x) sums group g's slabs
// of column x in order and the 16 group sums are added in group order (launch_slab_reduce's two
// levels), else one thread sums the z slabs in order (its one level) -- the same per-element order
// either way -- and the column goes straight into the grads blocks.  Returns the thread's f64 sum
// of squares of the gradient values it stored (0 on threads that store none).
__device__ __forceinline__ double fused_reduce_block(const float4* __restrict__ partial, int z, float* __restrict__ gW1,
                                                     float* __restrict__ gW3, float* __restrict__ gLs,
                                                     float* __restrict__ gW2, float ent_coef, int64_t blk,
                                                     float4 (*grp)[16]) {
    constexpr int kRX = 16;
    constexpr int64_t kSlab4 = kPartSize / 4;
    static_assert(kPartSize % 4 == 0 && 256 == kRX * kReduceGroups, "layout");
    const int x = threadIdx.x % kRX, g = threadIdx.x / kRX;
    const int64_t i = blk * kRX + x;
    const auto add = [](float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); };
    float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (z > kReduceGroups) {
        const int k0 = (int)((int64_t)g * z / kReduceGroups), k1 = (int)((int64_t)(g + 1) * z / kReduceGroups);
        float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (i < kSlab4) s = ordered_slab_sum(partial, kSlab4, i, k0, k1, s);  // == the in-order loop
        grp[g][x] = s;
        __syncthreads();
        if (g != 0 || i >= kSlab4) return 0.0;
#pragma unroll
        for (int q = 0; q < kReduceGroups; ++q) r = add(r, grp[q][x]);
    } else {
        if (g != 0 || i >= kSlab4) return 0.0;
        r = ordered_slab_sum(partial, kSlab4, i, 0, z, r);
    }
    const int j = (int)(4 * i);
    const float v0 = fused_scatter_one(j, r.x, gW1, gW3, gLs, gW2, ent_coef);
    const float v1 = fused_scatter_one(j + 1, r.y, gW1, gW3, gLs, gW2, ent_coef);
    const float v2 = fused_scatter_one(j + 2, r.z, gW1, gW3, gLs, gW2, ent_coef);
    const float v3 = fused_scatter_one(j + 3, r.w, gW1, gW3, gLs, gW2, ent_coef);
    return sumsq4(v0, v1, v2, v3);
}

__global__ __launch_bounds__(256) void k_fused_reduce_scatter(const float4* __restrict__ partial, int z,
                                                              float* __restrict__ gW1, float* __restrict__ gW3,
                                                              float* __restrict__ gLs, float* __restrict__ gW2,
                                                              float ent_coef) {
    __shared__ float4 grp[kReduceGroups][16];
    fused_reduce_block(partial, z, gW1, gW3, gLs, gW2, ent_coef, blockIdx.x, grp);
}

// The pass's two gradient reductions in one launch: blocks [0, nb1) sum the fused kernel's
// workgroup partials and scatter them (W1 / W3 / log σ / the W2 bias column), the rest sum the
// dW2 split-K slabs into W2's columns 0..255 -- disjoint outputs, each in its usual fixed order.
__global__ __launch_bounds__(256) void k_grad_reduce_pair(const float4* __restrict__ fpart, int fz,
                                                          float* __restrict__ gW1, float* __restrict__ gW3,
                                                          float* __restrict__ gLs, float* __restrict__ gW2,
                                                          float ent_coef, const float4* __restrict__ wpart, int wz,
                                                          int64_t ldo, int nb1) {
    __shared__ float4 grp[kReduceGroups][16];
    if ((int)blockIdx.x < nb1) fused_reduce_block(fpart, fz, gW1, gW3, gLs, gW2, ent_coef, blockIdx.x, grp);
    else slab_reduce_block(wpart, (int64_t)kH * kH / 4, wz, gW2, 0, kH, ldo, (int64_t)blockIdx.x - nb1, grp);
}

// Both networks' reductions of a paired learner step in one launch: blocks [0, nbA) are net A's
// k_grad_reduce_pair blocks, the rest net B's -- each element summed in the order its own pass's
// reduction would use.
struct GradReduceNet {
    const float4* fpart;
    int fz;
    float *gW1, *gW3, *gLs, *gW2;
    float ent_coef;
    const float4* wpart;
    int wz;
    int64_t ldo;
    int nb1, nb2;
};
// gn (optional): gn[block] = the f64 sum of squares of every gradient value the block stored, in
// one fixed order (a butterfly inside each wave, then the four wave sums in wave order).  The
// blocks together store every element of the master-layout gradient (pads as zeros), so at one
// rank these partials are the global norm's: the optimiser step reads them instead of running
// k_sumsq over the finished gradient (dxrl_pg_fused_pair_gnorm + dxrl_pg_adam_step).
__global__ __launch_bounds__(256) void k_grad_reduce_nets(GradReduceNet a, GradReduceNet b, double* __restrict__ gn) {
    __shared__ float4 grp[kReduceGroups][16];
    __shared__ double red4[4];
    const bool second = (int)blockIdx.x >= a.nb1 + a.nb2;
    const GradReduceNet& r = second ? b : a;
    const int64_t blk = second ? (int64_t)blockIdx.x - (a.nb1 + a.nb2) : (int64_t)blockIdx.x;
    double q;
    if (blk < r.nb1) q = fused_reduce_block(r.fpart, r.fz, r.gW1, r.gW3, r.gLs, r.gW2, r.ent_coef, blk, grp);
    else q = slab_reduce_block(r.wpart, (int64_t)kH * kH / 4, r.wz, r.gW2, 0, kH, r.ldo, blk - r.nb1, grp);
    if (gn) {  // launch-uniform; every thread of the block is still here
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
        if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = q;
        __syncthreads();
        if (threadIdx.x == 0) gn[blockIdx.x] = ((red4[0] + red4[1]) + red4[2]) + red4[3];
    }
}

// grads blocks W1 / W3 (and log_std for the actor) from the workgroup sum (launch_slab_reduce)
__global__ void k_fused_scatter(const float* __restrict__ sum, float* __restrict__ gW1, float* __restrict__ gW3,
                                float* __restrict__ gLs, float* __restrict__ gW2, float ent_coef) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= kPartSize) return;
    fused_scatter_one(j, sum[j], gW1, gW3, gLs, gW2, ent_coef);
}

}  // namespace
}  // namespace dxrl

// =========================================================================== C ABI
extern "C" {

int dxrl_pg_fused_sizes(int32_t* tile_rows, int64_t* partial_floats_per_block) {
    DXRL_REQUIRE(tile_rows && partial_floats_per_block, "null outputs");
    *tile_rows = 128;  // the largest tile; launches use up to two workgroups per CU (grid <= 2 CUs)
    *partial_floats_per_block = kPartSize;
    return DXRL_OK;
}

}  // extern "C"

namespace dxrl {
namespace {
// k_pg_fused itself (no dW2 contraction, no reductions); the grid it ran in *grid_out
int fused_kernel(const dxrl_pg_fused_args* a, hipStream_t st, int* grid_out);
}  // namespace
}  // namespace dxrl

extern "C" {

int dxrl_pg_fused(int32_t device, const dxrl_pg_fused_args* a, void* stream) {
    DXRL_REQUIRE(a && a->packed && a->params && a->obs && a->rows > 0, "fused: null arguments");
    DXRL_REQUIRE(a->net == 0 || a->net == 1, "fused: net must be 0 (actor) or 1 (critic)");
    DXRL_REQUIRE(a->grid >= 1 && a->grid <= 65535, "fused: grid out of range");
    const bool train = a->train != 0;
    if (!train) DXRL_REQUIRE(a->net == 1 && a->values, "fused: forward mode computes critic values only");
    if (train) {
        DXRL_REQUIRE(a->h1_mode == 0 || a->h1_mode == 1, "fused: h1_mode must be 0 or 1");
        DXRL_REQUIRE((a->h1 || (a->h1_mode == 0 && a->rows % 32 == 0)) && a->dh2 && a->partial && a->loss_partial && a->grads && a->wgrad_partial &&
                         a->wgrad_splits >= 1,
                     "fused: training needs h1/dh2 scratch, partial slabs and grads");
        DXRL_REQUIRE(a->net == 1 ? (a->ret != nullptr) : (a->act && a->logp_old && a->adv && a->stats),
                     "fused: missing head inputs");
        DXRL_REQUIRE((reinterpret_cast<uintptr_t>(a->act) & 15) == 0, "fused: act must be 16-byte aligned");
    }
    DXRL_REQUIRE((reinterpret_cast<uintptr_t>(a->obs) & 15) == 0, "fused: obs must be 16-byte aligned");
    // (read by 16-byte LDS-DMA pieces / written by 16-byte stores)
    DXRL_REQUIRE(((reinterpret_cast<uintptr_t>(a->h2_in) | reinterpret_cast<uintptr_t>(a->h2_out)) & 15) == 0,
                 "fused: h2_in / h2_out must be 16-byte aligned");
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    int grid = 0;
    if (int rc = fused_kernel(a, st, &grid)) return rc;
    if (!train) return DXRL_OK;
    const bf16* w = static_cast<const bf16*>(a->packed);
    const bool c = a->net == 1;
    const int64_t o2 = c ? kOffW2c : kOffW2a, o3 = c ? kOffW3c : kOffW3a;
    const bool recompute = a->rows % 32 == 0 && a->h1_mode == 0;
    float* G = a->grads;
    // the pad columns 257..287 of the W3 slab are never written: the scatter zeroes them
    float* tmp = a->partial + (int64_t)grid * kPartSize;
    float* sum = tmp + (int64_t)kReduceGroups * kPartSize;
    const bool aligned = (reinterpret_cast<uintptr_t>(a->partial) & 15) == 0;
    if (aligned && recompute && (reinterpret_cast<uintptr_t>(a->wgrad_partial) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(G + o2) & 15) == 0) {
        // dW2 first (its partials only), then both reductions in one launch
        int ns = 0;
        if (int rc = launch_wgrad_l1(static_cast<const bf16*>(a->dh2), kH, static_cast<const bf16*>(a->obs), kIn,
                                     w + (c ? kBfW1c : kBfW1a), a->rows, a->wgrad_splits, a->wgrad_partial, G + o2, st,
                                     kHx, 0, &ns))
            return rc;
        const int nb1 = (int)((kPartSize / 4 + 15) / 16);
        int nb2 = 0;
        if (ns > kReduceGroups) {
            nb2 = kH * kH / 4 / 16;
        } else if (ns > 0) {  // few slabs: the one-level sum (k_slab_reduce2_4 is the two-level form)
            if (int rc = launch_slab_reduce(a->wgrad_partial, (int64_t)kH * kH, ns, nullptr, G + o2, 0, st, kH, kHx))
                return rc;
        }
        hipLaunchKernelGGL(k_grad_reduce_pair, dim3((unsigned)(nb1 + nb2)), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(a->partial), grid, G + (c ? kOffW1c : kOffW1a), G + o3,
                           c ? nullptr : G + kOffLogStd, G + o2, (float)a->ent_coef,
                           reinterpret_cast<const float4*>(a->wgrad_partial), ns, (int64_t)kHx, nb1);
        return launch_check("k_grad_reduce_pair");
    }
    if (aligned) {
        (void)tmp;
        (void)sum;
        hipLaunchKernelGGL(k_fused_reduce_scatter, dim3((unsigned)((kPartSize / 4 + 15) / 16)), dim3(256), 0, st,
                           reinterpret_cast<const float4*>(a->partial), grid, G + (c ? kOffW1c : kOffW1a), G + o3,
                           c ? nullptr : G + kOffLogStd, G + o2, (float)a->ent_coef);
        if (int rc = launch_check("k_fused_reduce_scatter")) return rc;
    } else {
        if (int rc = launch_slab_reduce(a->partial, kPartSize, grid, tmp, sum, 0, st)) return rc;
        hipLaunchKernelGGL(k_fused_scatter, dim3((kPartSize + 255) / 256), dim3(256), 0, st, sum,
                           G + (c ? kOffW1c : kOffW1a), G + o3, c ? nullptr : G + kOffLogStd, G + o2,
                           (float)a->ent_coef);
        if (int rc = launch_check("k_fused_scatter")) return rc;
    }
    // dW2[:, 0..255] = dH2^T H1 (the bias column 256 came from the column sums above)
    if (recompute)
        return launch_wgrad_l1(static_cast<const bf16*>(a->dh2), kH, static_cast<const bf16*>(a->obs), kIn,
                               w + (c ? kBfW1c : kBfW1a), a->rows, a->wgrad_splits, a->wgrad_partial, G + o2, st, kHx);
    return launch_wgrad(static_cast<const bf16*>(a->dh2), kH, kH, static_cast<const bf16*>(a->h1), kHx, kH, a->rows,
                        a->wgrad_splits, a->wgrad_partial, G + o2, st, kHx);
}

int dxrl_pg_fused_pair(int32_t device, const dxrl_pg_fused_args* c, const dxrl_pg_fused_args* a, void* stream) {
    return dxrl_pg_fused_pair_gnorm(device, c, a, nullptr, 0, nullptr, stream);
}

int dxrl_pg_fused_pair_gnorm(int32_t device, const dxrl_pg_fused_args* c, const dxrl_pg_fused_args* a,
                             double* gnorm_partial, int32_t gnorm_capacity, int32_t* gnorm_blocks, void* stream) {
    DXRL_REQUIRE(c && a, "fused_pair: null arguments");
    DXRL_REQUIRE(!gnorm_partial || gnorm_blocks, "fused_pair: gnorm_partial needs gnorm_blocks");
    const int nb1 = (int)((kPartSize / 4 + 15) / 16), nb2 = kH * kH / 4 / 16;  // reduction blocks per network
    // (checked before anything is launched: a failed call leaves the gradient untouched)
    DXRL_REQUIRE(!gnorm_partial || gnorm_capacity >= 2 * (nb1 + nb2), "fused_pair: gnorm_partial needs %d doubles",
                 2 * (nb1 + nb2));
    DXRL_REQUIRE(c->net == 1 && a->net == 0 && c->train && a->train, "fused_pair: a critic and an actor train pass");
    DXRL_REQUIRE(c->rows == a->rows && c->rows > 0 && c->rows % 32 == 0 && c->obs == a->obs && c->packed == a->packed &&
                     c->grads == a->grads && c->params == a->params,
                 "fused_pair: both passes over the same samples, weights and gradient buffer (rows % 32 == 0)");
    DXRL_REQUIRE(c->h1_mode == 0 && a->h1_mode == 0, "fused_pair: H1 recomputed on chip (h1_mode 0)");
    DXRL_REQUIRE(c->dh2 && a->dh2 && c->dh2 != a->dh2 && c->partial && a->partial && c->partial != a->partial &&
                     c->wgrad_partial && a->wgrad_partial && c->wgrad_partial != a->wgrad_partial,
                 "fused_pair: each pass needs its own dh2, partial and wgrad_partial buffers");
    // the dW2 launch caps each split count at the 32-row chunk count (launch_wgrad_l1_pair): the
    // capped counts must still exceed kReduceGroups (checked after the launches, a
    // small batch overwrote dH2's partial slabs -- or dW2 itself at one split -- before failing)
    DXRL_REQUIRE(c->wgrad_splits > kReduceGroups && a->wgrad_splits > kReduceGroups &&
                     c->rows / 32 > kReduceGroups,
                 "fused_pair: wgrad_splits > %d per network and rows / 32 > %d", kReduceGroups, kReduceGroups);
    DXRL_REQUIRE(c->act == nullptr || (reinterpret_cast<uintptr_t>(c->act) & 15) == 0, "fused_pair: alignment");
    for (const dxrl_pg_fused_args* x : {c, a}) {
        DXRL_REQUIRE(x->packed && x->params && x->obs && x->loss_partial && x->grid >= 1 && x->grid <= 65535,
                     "fused_pair: null arguments");
        DXRL_REQUIRE(x->net == 1 ? (x->ret != nullptr) : (x->act && x->logp_old && x->adv && x->stats),
                     "fused_pair: missing head inputs");
        DXRL_REQUIRE(((reinterpret_cast<uintptr_t>(x->partial) | reinterpret_cast<uintptr_t>(x->wgrad_partial) |
                       reinterpret_cast<uintptr_t>(x->obs) | reinterpret_cast<uintptr_t>(x->act)) & 15) == 0,
                     "fused_pair: partial / wgrad_partial / obs / act must be 16-byte aligned");
        DXRL_REQUIRE((reinterpret_cast<uintptr_t>(x->h2_in) & 15) == 0, "fused_pair: h2_in must be 16-byte aligned");
    }
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    int grid_c = 0, grid_a = 0;
    if (int rc = fused_kernel(c, st, &grid_c)) return rc;
    if (int rc = fused_kernel(a, st, &grid_a)) return rc;
    const bf16* w = static_cast<const bf16*>(a->packed);
    float* G = a->grads;
    int ns_c = 0, ns_a = 0;
    // both dW2 contractions in one launch (their split counts side by side on the CUs), then both
    // networks' reductions in one launch
    if (int rc = launch_wgrad_l1_pair(static_cast<const bf16*>(c->dh2), w + kBfW1c, c->wgrad_splits, c->wgrad_partial,
                                      G + kOffW2c, static_cast<const bf16*>(a->dh2), w + kBfW1a, a->wgrad_splits,
                                      a->wgrad_partial, G + kOffW2a, kH, static_cast<const bf16*>(a->obs), kIn, a->rows,
                                      kHx, st, &ns_c, &ns_a))
        return rc;
    // (ns_c, ns_a = min(splits, rows / 32) > kReduceGroups by the checks above)
    if (gnorm_partial) *gnorm_blocks = 2 * (nb1 + nb2);
    GradReduceNet rc_{reinterpret_cast<const float4*>(c->partial), grid_c, G + kOffW1c, G + kOffW3c, nullptr,
                      G + kOffW2c, (float)c->ent_coef, reinterpret_cast<const float4*>(c->wgrad_partial), ns_c,
                      (int64_t)kHx, nb1, nb2};
    GradReduceNet ra_{reinterpret_cast<const float4*>(a->partial), grid_a, G + kOffW1a, G + kOffW3a, G + kOffLogStd,
                      G + kOffW2a, (float)a->ent_coef, reinterpret_cast<const float4*>(a->wgrad_partial), ns_a,
                      (int64_t)kHx, nb1, nb2};
    hipLaunchKernelGGL(k_grad_reduce_nets, dim3((unsigned)(2 * (nb1 + nb2))), dim3(256), 0, st, rc_, ra_,
                       gnorm_partial);
    return launch_check("k_grad_reduce_nets");
}

int dxrl_pg_gnorm_blocks(int32_t* blocks) {
    DXRL_REQUIRE(blocks, "null output");
    *blocks = (int32_t)(2 * ((kPartSize / 4 + 15) / 16 + kH * kH / 4 / 16));
    return DXRL_OK;
}

}  // extern "C"

namespace dxrl {
namespace {
int fused_kernel(const dxrl_pg_fused_args* a, hipStream_t st, int* grid_out) {
    const bool train = a->train != 0;
    const bf16* w = static_cast<const bf16*>(a->packed);
    const bool c = a->net == 1;
    const int64_t o2 = c ? kOffW2c : kOffW2a, o3 = c ? kOffW3c : kOffW3a;
    FusedArgs f{};
    f.net = a->net;
    f.train = train;
    f.rows = a->rows;
    f.X = static_cast<const bf16*>(a->obs);
    const bf16* fr = w + kFr + (c ? kFrNet : 0);
    f.W1 = fr + kFrOffW1;
    f.W2 = fr + kFrOffW2;
    f.W3 = fr + kFrOffW3;
    f.W2T = fr + kFrOffW2T;
    f.W3T = fr + kFrOffW3T;
    f.W3rm = w + (c ? kBfW3c : kBfW3a);
    f.b2 = a->params + o2 + kH;
    f.b3 = a->params + o3 + kH;
    f.logstd = a->params + kOffLogStd;
    f.act = a->act;
    f.logp_old = a->logp_old;
    f.adv = a->adv;
    f.ret = a->ret;
    f.stats = a->stats;
    f.sc = (float)a->inv_total_samples;
    f.clip_eps = (float)a->clip_eps;
    f.vf2 = (float)(2.0 * a->vf_coef);
    f.v_out = a->values;
    // H1 reaches the dW2 contraction either recomputed on chip from the observations
    // (launch_wgrad_l1: rows % 32 == 0) or as an HBM copy written by this kernel
    const bool recompute = train && a->rows % 32 == 0 && a->h1_mode == 0;
    f.h1_out = recompute ? nullptr : static_cast<bf16*>(a->h1);
    f.dh2_out = static_cast<bf16*>(a->dh2);
    f.h2_in = train ? static_cast<const bf16*>(a->h2_in) : nullptr;
    f.h2_out = train ? nullptr : static_cast<bf16*>(a->h2_out);
    f.part = a->partial;
    f.loss = a->loss_partial;
    f.loss_rows = a->grid;
    // tile geometry: 128-sample tiles, one 8-wave workgroup per CU (160 KiB LDS), or 64-sample
    // tiles, two 4-wave workgroups per CU (80 KiB each) -- DXRL_FUSED_TILE=64|128 (A/B)
    static const int tile = [] {
        const char* v = getenv("DXRL_FUSED_TILE");
        return v && atoi(v) == 64 ? 64 : 128;
    }();
    static const int cus = [] {
        int n = 0, device = 0;
        (void)hipGetDevice(&device);  // the caller's DeviceGuard made it current
        return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n > 0 ? n
                                                                                                            : 256;
    }();
    const int waves = tile == 64 ? 4 : 8;  // the instantiations launched below (128-sample tiles: 8 waves)
    const int64_t ntiles = (a->rows + tile - 1) / tile;
    const int64_t cap = (int64_t)cus * (tile == 64 ? 2 : 1);
    int64_t g64 = a->grid < cap ? a->grid : cap;
    if (ntiles < g64) g64 = ntiles;
    const int grid = (int)g64;
    static const int diag = [] {
        const char* v = getenv("DXRL_FUSED_DIAG");
        return v ? atoi(v) : 0;
    }();
    f.diag = diag;
    static unsigned long long* stamps = nullptr;
    if ((diag & 8) && !stamps) (void)hipMalloc(&stamps, (size_t)65536 * 8 * 16 * 8);
    f.stamps = stamps;
    const bool dg = diag != 0;
    if (tile == 64) {  // A/B geometry: the diagnostic instantiations only
        if (!train) hipLaunchKernelGGL((k_pg_fused<4, 64, false, 1, true>), dim3(grid), dim3(256), 0, st, f);
        else if (!c) hipLaunchKernelGGL((k_pg_fused<4, 64, true, 0, true>), dim3(grid), dim3(256), 0, st, f);
        else hipLaunchKernelGGL((k_pg_fused<4, 64, true, 1, true>), dim3(grid), dim3(256), 0, st, f);
    } else if (!train) {
        // A/B and the bit-identity test: the layer-by-layer instantiation (DXRL_FWD_LAYERED=1, read per call)
        const char* lv = getenv("DXRL_FWD_LAYERED");
        const bool layered = lv && atoi(lv) != 0;
        if (dg) hipLaunchKernelGGL((k_pg_fused<8, 128, false, 1, true>), dim3(grid), dim3(512), 0, st, f);
        else if (DXRL_FWD_VALUES && !layered) hipLaunchKernelGGL(k_pg_values, dim3(grid), dim3(512), 0, st, f);
        else hipLaunchKernelGGL((k_pg_fused<8, 128, false, 1, false>), dim3(grid), dim3(512), 0, st, f);
    } else if (!c) {
        // (h2_in: the layer-2 activations from the rollout; the diagnostic instantiations recompute
        // them -- the same bits either way)
        if (dg && DXRL_H2_STAMPS && f.h2_in) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 0, true, DXRL_H2_STAMPS != 0>), dim3(grid), dim3(512), 0, st, f);
        else if (dg) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 0, true>), dim3(grid), dim3(512), 0, st, f);
        else if (f.h2_in) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 0, false, true>), dim3(grid), dim3(512), 0, st, f);
        else hipLaunchKernelGGL((k_pg_fused<8, 128, true, 0, false>), dim3(grid), dim3(512), 0, st, f);
    } else {
        if (dg && DXRL_H2_STAMPS && f.h2_in) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 1, true, DXRL_H2_STAMPS != 0>), dim3(grid), dim3(512), 0, st, f);
        else if (dg) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 1, true>), dim3(grid), dim3(512), 0, st, f);
        else if (f.h2_in) hipLaunchKernelGGL((k_pg_fused<8, 128, true, 1, false, true>), dim3(grid), dim3(512), 0, st, f);
        else hipLaunchKernelGGL((k_pg_fused<8, 128, true, 1, false>), dim3(grid), dim3(512), 0, st, f);
    }
    if (int rc = launch_check("k_pg_fused")) return rc;
    if (diag & 8) {  // print the mean cycles per segment per wave (diagnostic builds only)
        std::vector<unsigned long long> h((size_t)grid * waves * 16);
        (void)hipStreamSynchronize(st);
        (void)hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost);
        fprintf(stderr, "fused net=%d train=%d tile=%d waves=%d cycles/wave:", a->net, (int)train, tile, waves);
        // (first half of the waves / second half: the two waves sharing a SIMD are w and w + waves / 2)
        for (int k = 0; k < 16; ++k) {
            double sum[2] = {0, 0};
            for (size_t w = 0; w < (size_t)grid * waves; ++w) sum[(w % waves) >= (size_t)waves / 2] += (double)h[w * 16 + k];
            fprintf(stderr, " s%d=%.0f/%.0f", k, 2 * sum[0] / (grid * waves), 2 * sum[1] / (grid * waves));
        }
        fprintf(stderr, "\n");
    }
    *grid_out = grid;
    return DXRL_OK;
}
}  // namespace
}  // namespace dxrl
