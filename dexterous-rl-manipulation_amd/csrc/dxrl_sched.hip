// dxrl_sched.hip -- the CurriculumScheduler feed on the device (config C3).
//
// The reference feeds its scheduler one finished episode at a time
// (evaluation/component_ablation.py:160-170 -> experiments/curriculum_scheduler.py:116-140):
// append (success, steps), then progress when
//   total_episodes >= min_episodes  and  len(successes) >= window  and
//   mean(successes[-window:]) >= threshold          (curriculum_scheduler.py:142-170)
// and interpolate the config one 1/progression_steps notch further (:172-222).  A
// vectorised iteration finishes up to T*N episodes per rank (700 k at 4096 envs on the
// easy curriculum), so the feed runs here: the rollout writes one u16 code per (step,
// env) -- 0, or (episode length << 1) | success -- and these kernels walk the codes in
// the order the host would have fed them, (end step, global env id), across all ranks'
// (all-gathered) tapes.  They return what the host scheduler needs to replay the batch
// exactly: the episode / step / success totals, the first P episodes at which the
// progression test holds (with the cumulative steps and window successes there), and the
// new tail of the last `window` episodes.  Only those few numbers cross PCIe.
//
// Global order index g = t * (world N) + r N + i  ->  codes[(r T + t) N + i].
//   k_sched_count    per 2048-code chunk: episodes, steps, successes
//   k_sched_offsets  one workgroup: exclusive chunk offsets, totals, the tail's prefix
//   k_sched_scatter  per chunk: episode index k of every end -> cumulative steps[k] and the
//                    success prefix cs[tail + k + 1]
//   k_sched_ok       per 256 episodes: the progression test, the block's first candidates
//   k_sched_collect  one workgroup: the first P candidates overall, the new tail
#include "dxrl_internal.h"

using namespace dxrl;

namespace {

constexpr int kThreads = 256, kPer = 8, kChunk = kThreads * kPer;
constexpr int kCollectThreads = 1024;

struct CodeView {
    const uint16_t* codes;
    int64_t n, T, world, L;
    __device__ __forceinline__ uint16_t at(int64_t g) const {
        const int64_t wn = world * n;
        const int64_t t = g / wn, rem = g - t * wn;
        const int64_t r = rem / n, i = rem - r * n;
        return codes[(r * T + t) * n + i];
    }
};

struct Tri {
    int64_t c, s, u;  // episodes, steps, successes
};
__device__ __forceinline__ Tri add(Tri a, Tri b) { return Tri{a.c + b.c, a.s + b.s, a.u + b.u}; }

// exclusive scan of one Tri per thread over a workgroup: inclusive scans of the 64-lane waves by
// shuffles, then the wave totals through LDS (lds: >= NT / 64 entries; integer sums, so any
// association gives the same result).  Ends with a barrier: lds is free again on return.
template <int NT>
__device__ Tri block_exclusive_scan(Tri v, Tri* lds, Tri& total) {
    static_assert(NT % 64 == 0 && NT <= 4096, "whole waves");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    Tri inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Tri o{__shfl_up(inc.c, d), __shfl_up(inc.s, d), __shfl_up(inc.u, d)};
        if (lane >= d) inc = add(inc, o);
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    Tri pre{0, 0, 0}, tot{0, 0, 0};
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
        const Tri s = lds[k];
        if (k < w) pre = add(pre, s);
        tot = add(tot, s);
    }
    total = tot;
    __syncthreads();
    return Tri{pre.c + inc.c - v.c, pre.s + inc.s - v.s, pre.u + inc.u - v.u};
}

// the kPer codes g0 .. g0 + kPer - 1 (0 past the end): one 16-byte load when the view is one
// contiguous rank (the order (t, r, i) is then the buffer's own) and the run is aligned
__device__ __forceinline__ void load_codes(const CodeView& v, int64_t g0, uint16_t (&x)[kPer]) {
    static_assert(kPer == 8, "one 16-byte load");
    if (v.world == 1 && g0 + kPer <= v.L && ((reinterpret_cast<uintptr_t>(v.codes) & 15) == 0)) {
        const uint4 q = *reinterpret_cast<const uint4*>(v.codes + g0);  // g0 % 8 == 0
        const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[2 * k] = (uint16_t)(w4[k] & 0xFFFFu);
            x[2 * k + 1] = (uint16_t)(w4[k] >> 16);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) x[k] = g0 + k < v.L ? v.at(g0 + k) : (uint16_t)0;
}

__global__ __launch_bounds__(kThreads) void k_sched_count(CodeView v, Tri* blk) {
    __shared__ Tri lds[kThreads];
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kPer;
    uint16_t x[kPer];
    load_codes(v, g0, x);
    Tri a{0, 0, 0};
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (x[k]) {
            a.c += 1;
            a.s += x[k] >> 1;
            a.u += x[k] & 1;
        }
    }
    Tri tot;
    (void)block_exclusive_scan<kThreads>(a, lds, tot);
    if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// off[b] = exclusive prefix of blk; summary[0..2] = totals; cs[0..tail_len] = tail success prefix
__global__ __launch_bounds__(kCollectThreads) void k_sched_offsets(const Tri* blk, int nb, Tri* off,
                                                                   const uint16_t* tail, const int32_t* tail_len,
                                                                   int32_t* cs, int64_t* summary) {
    __shared__ Tri lds[kCollectThreads];
    const int per = (nb + kCollectThreads - 1) / kCollectThreads;
    const int lo = threadIdx.x * per, hi = min(nb, lo + per);
    Tri a{0, 0, 0};
    for (int b = lo; b < hi; ++b) a = add(a, blk[b]);
    Tri tot;
    Tri run = block_exclusive_scan<kCollectThreads>(a, lds, tot);
    for (int b = lo; b < hi; ++b) {
        off[b] = run;
        run = add(run, blk[b]);
    }
    if (threadIdx.x == 0) {
        summary[0] = tot.c;
        summary[1] = tot.s;
        summary[2] = tot.u;
        const int tl = *tail_len;
        int32_t c = 0;
        cs[0] = 0;
        for (int j = 0; j < tl; ++j) {
            c += tail[j] & 1;
            cs[j + 1] = c;
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_sched_scatter(CodeView v, const Tri* off, const int32_t* tail_len,
                                                            int32_t* cs, int64_t* csteps) {
    __shared__ Tri lds[kThreads];
    const int64_t g0 = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kPer;
    uint16_t x[kPer];
    load_codes(v, g0, x);
    Tri a{0, 0, 0};
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (x[k]) {
            a.c += 1;
            a.s += x[k] >> 1;
            a.u += x[k] & 1;
        }
    }
    Tri tot;
    Tri run = add(off[blockIdx.x], block_exclusive_scan<kThreads>(a, lds, tot));
    const int tl = *tail_len;
    const int32_t tail_succ = cs[tl];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (x[k]) {
            run.s += x[k] >> 1;
            run.u += x[k] & 1;
            csteps[run.c] = run.s;                            // steps through episode k = run.c
            cs[tl + run.c + 1] = tail_succ + (int32_t)run.u;  // successes through history index tl + k
            run.c += 1;
        }
    }
}

struct OkParams {
    int32_t window;
    double threshold;
    int64_t min_episodes, episodes_before;
};

__device__ __forceinline__ int32_t window_successes(const int32_t* cs, int tl, int64_t k, int32_t w) {
    const int64_t e = tl + k + 1;  // history prefix length through episode k
    const int64_t b = e - w > 0 ? e - w : 0;
    return cs[e] - cs[b];
}

__device__ __forceinline__ bool progression_test(const OkParams& q, int64_t k, int32_t win) {
    const int64_t total = q.episodes_before + k + 1;  // total_episodes == len(episode_successes)
    return total >= q.min_episodes && total >= q.window && (double)win / (double)q.window >= q.threshold;
}

// one thread per episode; per 256-episode block: number of candidates and the first kCap of them
template <int kCap>
__global__ __launch_bounds__(kThreads) void k_sched_ok(const int64_t* summary, const int32_t* tail_len,
                                                       const int32_t* cs, OkParams q, int32_t* okcnt,
                                                       int64_t* okfirst) {
    __shared__ int wave_cnt[kThreads / 64];
    const int64_t E = summary[0];
    const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int tl = *tail_len;
    bool ok = false;
    if (k < E) ok = progression_test(q, k, window_successes(cs, tl, k, q.window));
    const unsigned long long m = __ballot(ok);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) wave_cnt[wave] = __popcll(m);
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        before += w < wave ? wave_cnt[w] : 0;
        total += wave_cnt[w];
    }
    if (ok) {
        const int rank = before + __popcll(m & ((1ull << lane) - 1ull));
        if (rank < kCap) okfirst[(int64_t)blockIdx.x * kCap + rank] = k;
    }
    if (threadIdx.x == 0) okcnt[blockIdx.x] = total;
}

// the first P candidates in episode order (P <= kCap), their cumulative steps and window
// successes; the new tail = the last min(window, tail_len + E) history codes
template <int kCap>
__global__ __launch_bounds__(kCollectThreads) void k_sched_collect(
    int nb, int32_t P, const int32_t* okcnt, const int64_t* okfirst, const int32_t* cs, const int64_t* csteps,
    int32_t window, const uint16_t* tail_in, const int32_t* tail_len_in, uint16_t* tail_out, int32_t* tail_len_out,
    int64_t* summary) {
    __shared__ int64_t lds[kCollectThreads];
    __shared__ int64_t found_total;
    const int per = (nb + kCollectThreads - 1) / kCollectThreads;
    const int lo = threadIdx.x * per, hi = min(nb, lo + per);
    int64_t a = 0;
    for (int b = lo; b < hi; ++b) a += okcnt[b];
    lds[threadIdx.x] = a;
    __syncthreads();
    for (int d = 1; d < kCollectThreads; d <<= 1) {
        const int64_t o = threadIdx.x >= d ? lds[threadIdx.x - d] : 0;
        __syncthreads();
        lds[threadIdx.x] += o;
        __syncthreads();
    }
    int64_t run = threadIdx.x ? lds[threadIdx.x - 1] : 0;
    if (threadIdx.x == kCollectThreads - 1) found_total = lds[kCollectThreads - 1];
    const int tl = *tail_len_in;
    for (int b = lo; b < hi && run < P; ++b) {
        const int c = okcnt[b];
        for (int j = 0; j < c && j < kCap && run + j < P; ++j) {
            const int64_t k = okfirst[(int64_t)b * kCap + j];
            int64_t* o = summary + 4 + 3 * (run + j);
            o[0] = k;
            o[1] = csteps[k];
            o[2] = window_successes(cs, tl, k, window);
        }
        run += c;
    }
    __syncthreads();
    const int64_t E = summary[0];
    if (threadIdx.x == 0) summary[3] = found_total < P ? found_total : P;
    const int64_t hist = tl + E;
    const int32_t nl = (int32_t)(hist < window ? hist : window);
    for (int j = threadIdx.x; j < nl; j += kCollectThreads) {
        const int64_t x = hist - nl + j;  // history index
        uint16_t code;
        if (x < tl) {
            code = tail_in[x];
        } else {
            const int64_t k = x - tl;
            const int64_t len = csteps[k] - (k ? csteps[k - 1] : 0);
            code = (uint16_t)((len << 1) | (int64_t)(cs[x + 1] - cs[x]));
        }
        tail_out[j] = code;
    }
    if (threadIdx.x == 0) *tail_len_out = nl;
}

constexpr int kCap = DXRL_SCHED_MAX_CANDIDATES;

// ------------------------------------------------------------------ the compacted exchange
// A rank's pack (u32 words, fixed size for an all-gather):
//   [0] E_r episodes of this rank   [1] tailn_r = min(window, E_r)
//   [2 + 3 t ..] per step t: episodes, steps, successes ending at t (this rank's envs)
//   tail: the rank's last tailn_r codes (u16, episode order)
//   bits (only when progressions are still possible): the success bit of every episode of the
//        rank, in (end step, env) order
// Global episode order (end step t, global env id) = blocks (t, r) in order t-major, rank-minor;
// block (t, r) holds rank r's episodes local [loff(t), loff(t) + count) -- so the last `window`
// episodes of the whole batch are all inside the ranks' own tails, and the success prefix at any
// episode needs the bits only.
struct PackLayout {
    int64_t steps_at, tail_at, bits_at, words;  // word offsets
};
__host__ __device__ inline PackLayout pack_layout(int64_t T, int64_t N, int32_t window, int32_t bits) {
    PackLayout p;
    p.steps_at = 2;
    p.tail_at = p.steps_at + 3 * T;
    p.bits_at = p.tail_at + (window + 1) / 2;
    p.words = p.bits_at + (bits ? (T * N + 31) / 32 : 0);
    return p;
}

template <typename V>
__device__ V block_exclusive_scan_v(V v, V* lds, V& total) {  // as block_exclusive_scan, one value
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    V inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const V o = __shfl_up(inc, d);
        if (lane >= d) inc = inc + o;
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    V pre{}, tot{};
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) {
        const V s = lds[k];
        if (k < w) pre = pre + s;
        tot = tot + s;
    }
    total = tot;
    __syncthreads();
    return pre + inc - v;
}

// one workgroup per step: this rank's (episodes, steps, successes) ending at t
__global__ __launch_bounds__(kThreads) void k_pack_count(const uint16_t* __restrict__ codes, int64_t N,
                                                         uint32_t* __restrict__ pack, PackLayout L) {
    __shared__ Tri lds[kThreads];
    const int64_t t = blockIdx.x;
    Tri a{0, 0, 0};
    for (int64_t i = threadIdx.x; i < N; i += kThreads) {
        const uint16_t x = codes[t * N + i];
        if (x) {
            a.c += 1;
            a.s += x >> 1;
            a.u += x & 1;
        }
    }
    Tri tot;
    (void)block_exclusive_scan<kThreads>(a, lds, tot);
    if (threadIdx.x == 0) {
        uint32_t* o = pack + L.steps_at + 3 * t;
        o[0] = (uint32_t)tot.c;
        o[1] = (uint32_t)tot.s;
        o[2] = (uint32_t)tot.u;
    }
}

// one workgroup per step: episode indices of the step's ends -> success bits, the rank's tail
__global__ __launch_bounds__(kThreads) void k_pack_bits(const uint16_t* __restrict__ codes, int64_t T, int64_t N,
                                                        int32_t window, int32_t bits, uint32_t* __restrict__ pack,
                                                        PackLayout L) {
    __shared__ int64_t red[kThreads];
    __shared__ int64_t off_s, e_s;
    const int64_t t = blockIdx.x;
    int64_t before = 0, all = 0;
    for (int64_t q = threadIdx.x; q < T; q += kThreads) {
        const int64_t c = pack[L.steps_at + 3 * q];
        all += c;
        before += q < t ? c : 0;
    }
    {
        int64_t tb;
        const int64_t eb = block_exclusive_scan_v<int64_t>(before, red, tb);
        (void)eb;
        int64_t ta;
        (void)block_exclusive_scan_v<int64_t>(all, red, ta);
        if (threadIdx.x == 0) {
            off_s = tb;
            e_s = ta;
        }
        __syncthreads();
    }
    const int64_t off = off_s, E = e_s;
    const int64_t tailn = E < window ? E : window, tail0 = E - tailn;
    if (t == 0 && threadIdx.x == 0) {
        pack[0] = (uint32_t)E;
        pack[1] = (uint32_t)tailn;
    }
    uint16_t* tail = reinterpret_cast<uint16_t*>(pack + L.tail_at);
    uint32_t* bw = pack + L.bits_at;
    int64_t run = 0;  // episodes of this step before the current chunk
    for (int64_t c0 = 0; c0 < N; c0 += (int64_t)kThreads * kPer) {
        const int64_t i0 = c0 + (int64_t)threadIdx.x * kPer;
        uint16_t x[kPer];
        int64_t cnt = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            x[k] = i0 + k < N ? codes[t * N + i0 + k] : (uint16_t)0;
            cnt += x[k] != 0;
        }
        int64_t ctot;
        int64_t idx = off + run + block_exclusive_scan_v<int64_t>(cnt, red, ctot);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (!x[k]) continue;
            if (bits && (x[k] & 1)) atomicOr(bw + (idx >> 5), 1u << (idx & 31));
            if (idx >= tail0) tail[idx - tail0] = x[k];
            ++idx;
        }
        run += ctot;
    }
}

// block (t, r) -> exclusive prefix (episodes, steps, successes) in global order, the rank-local
// offset of the block, the totals; the tail's success prefix cs[0..tl]
__global__ __launch_bounds__(kCollectThreads) void k_sp_blocks(const uint32_t* __restrict__ packs, PackLayout L,
                                                               int32_t world, int64_t T, Tri* __restrict__ boff,
                                                               int64_t* __restrict__ loff, const uint16_t* tail,
                                                               const int32_t* tail_len, int32_t* cs,
                                                               int64_t* summary) {
    __shared__ Tri lds[kCollectThreads];
    const int64_t nb = (int64_t)world * T;
    const int64_t per = (nb + kCollectThreads - 1) / kCollectThreads;
    const int64_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    const auto blk = [&](int64_t b) {
        const int64_t t = b / world, r = b % world;
        const uint32_t* o = packs + r * L.words + L.steps_at + 3 * t;
        return Tri{(int64_t)o[0], (int64_t)o[1], (int64_t)o[2]};
    };
    Tri a{0, 0, 0};
    for (int64_t b = lo; b < hi; ++b) a = add(a, blk(b));
    Tri tot;
    Tri run = block_exclusive_scan<kCollectThreads>(a, lds, tot);
    for (int64_t b = lo; b < hi; ++b) {
        boff[b] = run;
        run = add(run, blk(b));
    }
    // rank-local offsets: loff[t * world + r] = sum_{t' < t} count(t', r)
    for (int64_t r = threadIdx.x; r < world; r += kCollectThreads) {
        int64_t c = 0;
        for (int64_t t = 0; t < T; ++t) {
            loff[t * world + r] = c;
            c += packs[r * L.words + L.steps_at + 3 * t];
        }
    }
    if (threadIdx.x == 0) {
        summary[0] = tot.c;
        summary[1] = tot.s;
        summary[2] = tot.u;
        summary[3] = 0;
        const int tl = *tail_len;
        int32_t c = 0;
        cs[0] = 0;
        for (int j = 0; j < tl; ++j) {
            c += tail[j] & 1;
            cs[j + 1] = c;
        }
    }
}

// bits mode: cs[tl + k + 1] = successes through history index tl + k, one workgroup per block
__global__ __launch_bounds__(kThreads) void k_sp_cs(const uint32_t* __restrict__ packs, PackLayout L, int32_t world,
                                                    const Tri* __restrict__ boff, const int64_t* __restrict__ loff,
                                                    const int32_t* tail_len, int32_t* cs) {
    __shared__ int64_t red[kThreads];
    const int64_t b = blockIdx.x;
    const int64_t r = b % world;
    const Tri o = boff[b];
    const int64_t c = (int64_t)packs[r * L.words + L.steps_at + 3 * (b / world)];
    const uint32_t* bw = packs + r * L.words + L.bits_at;
    const int tl = *tail_len;
    const int32_t base = cs[tl] + (int32_t)o.u;
    const int64_t l0 = loff[b];
    int64_t run = 0;
    for (int64_t j0 = 0; j0 < c; j0 += (int64_t)kThreads * kPer) {
        const int64_t j1 = j0 + (int64_t)threadIdx.x * kPer;
        uint32_t s[kPer];
        int64_t n = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int64_t idx = l0 + j1 + k;
            s[k] = j1 + k < c ? (bw[idx >> 5] >> (idx & 31)) & 1u : 0u;
            n += s[k];
        }
        int64_t ntot;
        int64_t acc = run + block_exclusive_scan_v<int64_t>(n, red, ntot);
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (j1 + k < c) {
                acc += s[k];
                cs[tl + o.c + j1 + k + 1] = base + (int32_t)acc;
            }
        }
        run += ntot;
    }
}

// the block holding global episode k (the last block whose first episode is <= k and that is
// non-empty): binary search over the exclusive prefix
__device__ __forceinline__ int64_t block_of(const Tri* boff, int64_t nb, int64_t k) {
    int64_t lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (boff[mid].c <= k) lo = mid;
        else hi = mid - 1;
    }
    return lo;  // boff[lo].c <= k < boff[lo + 1].c, so block lo is non-empty
}

// the first P candidates (block-prefix steps; the owner completes them) and the new tail from
// the ranks' own tails
template <int kCapT>
__global__ __launch_bounds__(kCollectThreads) void k_sp_collect(
    int nbk, int32_t P, const int32_t* okcnt, const int64_t* okfirst, const int32_t* cs, const uint32_t* packs,
    PackLayout L, int32_t world, int64_t T, const Tri* boff, const int64_t* loff, int32_t window,
    const uint16_t* tail_in, const int32_t* tail_len_in, uint16_t* tail_out, int32_t* tail_len_out,
    int32_t* where, int64_t* summary) {
    __shared__ int64_t lds[kCollectThreads];
    __shared__ int64_t found_total;
    const int64_t nb = (int64_t)world * T;
    const int tl = *tail_len_in;
    if (P > 0) {
        const int per = (nbk + kCollectThreads - 1) / kCollectThreads;
        const int lo = threadIdx.x * per, hi = min(nbk, lo + per);
        int64_t a = 0;
        for (int b = lo; b < hi; ++b) a += okcnt[b];
        lds[threadIdx.x] = a;
        __syncthreads();
        for (int d = 1; d < kCollectThreads; d <<= 1) {
            const int64_t o = threadIdx.x >= d ? lds[threadIdx.x - d] : 0;
            __syncthreads();
            lds[threadIdx.x] += o;
            __syncthreads();
        }
        int64_t run = threadIdx.x ? lds[threadIdx.x - 1] : 0;
        if (threadIdx.x == kCollectThreads - 1) found_total = lds[kCollectThreads - 1];
        for (int b = lo; b < hi && run < P; ++b) {
            const int c = okcnt[b];
            for (int j = 0; j < c && j < kCapT && run + j < P; ++j) {
                const int64_t k = okfirst[(int64_t)b * kCapT + j];
                const int64_t bk = block_of(boff, nb, k);
                int64_t* o = summary + 4 + 3 * (run + j);
                o[0] = k;
                o[1] = boff[bk].s;  // + the owner's steps through k within the block (dxrl_sched_candidate_steps)
                o[2] = window_successes(cs, tl, k, window);
                int32_t* w = where + 3 * (run + j);
                w[0] = (int32_t)(bk % world);
                w[1] = (int32_t)(bk / world);
                w[2] = (int32_t)(k - boff[bk].c);
            }
            run += c;
        }
        __syncthreads();
        if (threadIdx.x == 0) summary[3] = found_total < P ? found_total : P;
    }
    const int64_t E = summary[0];
    const int64_t hist = tl + E;
    const int32_t nl = (int32_t)(hist < window ? hist : window);
    for (int j = threadIdx.x; j < nl; j += kCollectThreads) {
        const int64_t x = hist - nl + j;  // history index
        uint16_t code;
        if (x < tl) {
            code = tail_in[x];
        } else {
            const int64_t k = x - tl;
            const int64_t bk = block_of(boff, nb, k);
            const int64_t r = bk % world;
            const uint32_t* pr = packs + r * L.words;
            const int64_t local = loff[bk] + (k - boff[bk].c);
            const int64_t t0 = (int64_t)pr[0] - (int64_t)pr[1];  // the rank's tail starts at local t0
            code = reinterpret_cast<const uint16_t*>(pr + L.tail_at)[local - t0];
        }
        tail_out[j] = code;
    }
    if (threadIdx.x == 0) *tail_len_out = nl;
}

// one workgroup per candidate this rank owns: steps of the block's first j + 1 episodes
__global__ __launch_bounds__(kThreads) void k_sp_cand_steps(const uint16_t* __restrict__ codes, int64_t N, int32_t rank,
                                                            const int32_t* __restrict__ where,
                                                            const int64_t* __restrict__ summary,
                                                            int64_t* __restrict__ partial) {
    __shared__ Tri lds[kThreads];
    __shared__ int64_t result;
    const int c = blockIdx.x;
    const bool mine = c < summary[3] && where[3 * c] == rank;
    if (threadIdx.x == 0) result = 0;
    __syncthreads();
    if (mine) {
        const int64_t t = where[3 * c + 1], j = where[3 * c + 2];
        Tri run{0, 0, 0};
        for (int64_t c0 = 0; c0 < N && run.c <= j; c0 += (int64_t)kThreads * kPer) {
            const int64_t i0 = c0 + (int64_t)threadIdx.x * kPer;
            uint16_t x[kPer];
            Tri a{0, 0, 0};
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                x[k] = i0 + k < N ? codes[t * N + i0 + k] : (uint16_t)0;
                if (x[k]) {
                    a.c += 1;
                    a.s += x[k] >> 1;
                }
            }
            Tri tot;
            Tri ex = add(run, block_exclusive_scan<kThreads>(a, lds, tot));
            if (ex.c <= j && j < ex.c + a.c) {  // episode j of the block is in this thread's codes
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    if (x[k] && ex.c <= j) {
                        ex.s += x[k] >> 1;
                        ex.c += 1;
                    }
                }
                result = ex.s;
            }
            run = add(run, tot);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) partial[c] = result;
}

__global__ void k_sp_finish(const int64_t* __restrict__ partial, int64_t* __restrict__ summary) {
    const int c = threadIdx.x;
    if (c < summary[3]) summary[4 + 3 * c + 1] += partial[c];
}

struct PackedScratch {
    Tri* boff;
    int64_t* loff;
    int32_t* cs;
    int32_t* okcnt;
    int64_t* okfirst;
    size_t bytes;
};

PackedScratch carve_packed(char* base, int32_t world, int64_t T, int64_t N, int32_t window) {
    const int64_t nb = (int64_t)world * T, L = nb * N, nb4 = (L + kThreads - 1) / kThreads;
    PackedScratch s{};
    size_t o = 0;
    const auto take = [&](size_t bytes) {
        char* p = base ? base + o : nullptr;
        o += (bytes + 255) & ~(size_t)255;
        return p;
    };
    s.boff = reinterpret_cast<Tri*>(take(sizeof(Tri) * (size_t)nb));
    s.loff = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (size_t)nb));
    s.cs = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)(window + L + 1)));
    s.okcnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)nb4));
    s.okfirst = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (size_t)kCap * (size_t)nb4));
    s.bytes = o;
    return s;
}

struct Scratch {
    Tri* blk;
    Tri* off;
    int32_t* cs;
    int64_t* csteps;
    int32_t* okcnt;
    int64_t* okfirst;
    size_t bytes;
};

Scratch carve(char* base, int64_t L, int32_t window) {
    const int64_t nb = (L + kChunk - 1) / kChunk, nb4 = (L + kThreads - 1) / kThreads;
    Scratch s{};
    size_t o = 0;
    const auto take = [&](size_t bytes) {
        char* p = base ? base + o : nullptr;
        o += (bytes + 255) & ~(size_t)255;
        return p;
    };
    s.blk = reinterpret_cast<Tri*>(take(sizeof(Tri) * (size_t)nb));
    s.off = reinterpret_cast<Tri*>(take(sizeof(Tri) * (size_t)nb));
    s.cs = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)(window + L + 1)));
    s.csteps = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (size_t)(L > 0 ? L : 1)));
    s.okcnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (size_t)(nb4 > 0 ? nb4 : 1)));
    s.okfirst = reinterpret_cast<int64_t*>(take(sizeof(int64_t) * (size_t)kCap * (size_t)(nb4 > 0 ? nb4 : 1)));
    s.bytes = o;
    return s;
}

}  // namespace

extern "C" {

int dxrl_sched_scratch_bytes(int32_t world, int32_t horizon, int64_t num_envs, int32_t window, int64_t* bytes) {
    DXRL_REQUIRE(bytes && world >= 1 && horizon >= 1 && num_envs >= 1 && window >= 1, "bad scheduler-scan shape");
    *bytes = (int64_t)carve(nullptr, (int64_t)world * horizon * num_envs, window).bytes;
    return DXRL_OK;
}

int dxrl_sched_scan(int32_t device, const dxrl_sched_args* a, void* stream) {
    DXRL_REQUIRE(a && a->codes && a->tail_in && a->tail_out && a->tail_len_in && a->tail_len_out && a->scratch &&
                     a->summary,
                 "null argument");
    DXRL_REQUIRE(a->world >= 1 && a->horizon >= 1 && a->num_envs >= 1, "bad codes shape");
    DXRL_REQUIRE(a->window >= 1, "window must be >= 1");
    DXRL_REQUIRE(a->max_candidates >= 0 && a->max_candidates <= kCap, "max_candidates outside [0, %d]", kCap);
    DXRL_REQUIRE(a->tail_in != a->tail_out, "tail_in and tail_out must differ");
    const int64_t L = (int64_t)a->world * a->horizon * a->num_envs;
    Scratch s = carve(static_cast<char*>(a->scratch), L, a->window);
    DXRL_REQUIRE(a->scratch_bytes >= (int64_t)s.bytes, "scratch too small: %lld < %lld bytes",
                 (long long)a->scratch_bytes, (long long)s.bytes);
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    const CodeView v{a->codes, a->num_envs, a->horizon, a->world, L};
    const int nb = (int)((L + kChunk - 1) / kChunk), nb4 = (int)((L + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(k_sched_count, dim3(nb), dim3(kThreads), 0, st, v, s.blk);
    if (int rc = launch_check("k_sched_count")) return rc;
    hipLaunchKernelGGL(k_sched_offsets, dim3(1), dim3(kCollectThreads), 0, st, s.blk, nb, s.off, a->tail_in,
                       a->tail_len_in, s.cs, a->summary);
    if (int rc = launch_check("k_sched_offsets")) return rc;
    hipLaunchKernelGGL(k_sched_scatter, dim3(nb), dim3(kThreads), 0, st, v, s.off, a->tail_len_in, s.cs, s.csteps);
    if (int rc = launch_check("k_sched_scatter")) return rc;
    const OkParams q{a->window, a->threshold, a->min_episodes, a->episodes_before};
    hipLaunchKernelGGL(k_sched_ok<kCap>, dim3(nb4), dim3(kThreads), 0, st, a->summary, a->tail_len_in, s.cs, q,
                       s.okcnt, s.okfirst);
    if (int rc = launch_check("k_sched_ok")) return rc;
    hipLaunchKernelGGL(k_sched_collect<kCap>, dim3(1), dim3(kCollectThreads), 0, st, nb4, a->max_candidates,
                       s.okcnt, s.okfirst, s.cs, s.csteps, a->window, a->tail_in, a->tail_len_in, a->tail_out,
                       a->tail_len_out, a->summary);
    return launch_check("k_sched_collect");
}

int dxrl_sched_pack_words(int32_t horizon, int64_t num_envs, int32_t window, int32_t bits, int64_t* words) {
    DXRL_REQUIRE(words && horizon >= 1 && num_envs >= 1 && window >= 1, "bad scheduler-pack shape");
    *words = pack_layout(horizon, num_envs, window, bits).words;
    return DXRL_OK;
}

int dxrl_sched_pack(int32_t device, const uint16_t* codes, int32_t horizon, int64_t num_envs, int32_t window,
                    int32_t bits, uint32_t* pack, void* stream) {
    DXRL_REQUIRE(codes && pack && horizon >= 1 && num_envs >= 1 && window >= 1, "bad scheduler-pack arguments");
    DXRL_REQUIRE(num_envs < (1ll << 18), "num_envs >= 2^18: a step's episode steps may overflow the u32 pack field");
    DXRL_REQUIRE((int64_t)horizon * num_envs < (1ll << 32), "horizon * num_envs >= 2^32");
    const PackLayout L = pack_layout(horizon, num_envs, window, bits);
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    if (int rc = hip_check(hipMemsetAsync(pack, 0, (size_t)L.words * 4, st), "pack zero")) return rc;
    hipLaunchKernelGGL(k_pack_count, dim3((unsigned)horizon), dim3(kThreads), 0, st, codes, num_envs, pack, L);
    if (int rc = launch_check("k_pack_count")) return rc;
    hipLaunchKernelGGL(k_pack_bits, dim3((unsigned)horizon), dim3(kThreads), 0, st, codes, (int64_t)horizon, num_envs,
                       window, bits, pack, L);
    return launch_check("k_pack_bits");
}

int dxrl_sched_packed_scratch_bytes(int32_t world, int32_t horizon, int64_t num_envs, int32_t window,
                                    int64_t* bytes) {
    DXRL_REQUIRE(bytes && world >= 1 && horizon >= 1 && num_envs >= 1 && window >= 1, "bad scheduler-scan shape");
    *bytes = (int64_t)carve_packed(nullptr, world, horizon, num_envs, window).bytes;
    return DXRL_OK;
}

int dxrl_sched_scan_packed(int32_t device, const dxrl_sched_packed_args* a, void* stream) {
    DXRL_REQUIRE(a && a->packs && a->tail_in && a->tail_out && a->tail_len_in && a->tail_len_out && a->scratch &&
                     a->summary && a->where,
                 "null argument");
    DXRL_REQUIRE(a->world >= 1 && a->horizon >= 1 && a->num_envs >= 1 && a->window >= 1, "bad packs shape");
    DXRL_REQUIRE(a->max_candidates >= 0 && a->max_candidates <= kCap, "max_candidates outside [0, %d]", kCap);
    DXRL_REQUIRE(a->max_candidates == 0 || a->bits, "candidates need the packs' success bits (bits = 1)");
    DXRL_REQUIRE(a->tail_in != a->tail_out, "tail_in and tail_out must differ");
    const PackLayout L = pack_layout(a->horizon, a->num_envs, a->window, a->bits);
    DXRL_REQUIRE(a->pack_words == L.words, "pack_words %lld != dxrl_sched_pack_words %lld", (long long)a->pack_words,
                 (long long)L.words);
    PackedScratch s = carve_packed(static_cast<char*>(a->scratch), a->world, a->horizon, a->num_envs, a->window);
    DXRL_REQUIRE(a->scratch_bytes >= (int64_t)s.bytes, "scratch too small: %lld < %lld bytes",
                 (long long)a->scratch_bytes, (long long)s.bytes);
    DeviceGuard g(device);
    hipStream_t st = as_stream(stream);
    const int64_t nb = (int64_t)a->world * a->horizon;
    const uint32_t* packs = static_cast<const uint32_t*>(a->packs);
    hipLaunchKernelGGL(k_sp_blocks, dim3(1), dim3(kCollectThreads), 0, st, packs, L, a->world, (int64_t)a->horizon,
                       s.boff, s.loff, a->tail_in, a->tail_len_in, s.cs, a->summary);
    if (int rc = launch_check("k_sp_blocks")) return rc;
    const int64_t Lmax = nb * a->num_envs;
    const int nb4 = (int)((Lmax + kThreads - 1) / kThreads);
    if (a->max_candidates > 0) {
        hipLaunchKernelGGL(k_sp_cs, dim3((unsigned)nb), dim3(kThreads), 0, st, packs, L, a->world, s.boff, s.loff,
                           a->tail_len_in, s.cs);
        if (int rc = launch_check("k_sp_cs")) return rc;
        const OkParams q{a->window, a->threshold, a->min_episodes, a->episodes_before};
        hipLaunchKernelGGL(k_sched_ok<kCap>, dim3(nb4), dim3(kThreads), 0, st, a->summary, a->tail_len_in, s.cs, q,
                           s.okcnt, s.okfirst);
        if (int rc = launch_check("k_sched_ok")) return rc;
    }
    hipLaunchKernelGGL(k_sp_collect<kCap>, dim3(1), dim3(kCollectThreads), 0, st, nb4, a->max_candidates, s.okcnt,
                       s.okfirst, s.cs, packs, L, a->world, (int64_t)a->horizon, s.boff, s.loff, a->window,
                       a->tail_in, a->tail_len_in, a->tail_out, a->tail_len_out, a->where, a->summary);
    return launch_check("k_sp_collect");
}

int dxrl_sched_candidate_steps(int32_t device, const uint16_t* codes, int32_t horizon, int64_t num_envs,
                               int32_t rank, int32_t max_candidates, const int32_t* where, const int64_t* summary,
                               int64_t* partial, void* stream) {
    DXRL_REQUIRE(codes && where && summary && partial && horizon >= 1 && num_envs >= 1 && rank >= 0,
                 "bad candidate-steps arguments");
    DXRL_REQUIRE(max_candidates >= 1 && max_candidates <= kCap, "max_candidates outside [1, %d]", kCap);
    DeviceGuard g(device);
    hipLaunchKernelGGL(k_sp_cand_steps, dim3((unsigned)max_candidates), dim3(kThreads), 0, as_stream(stream), codes,
                       num_envs, rank, where, summary, partial);
    return launch_check("k_sp_cand_steps");
}

int dxrl_sched_finish(int32_t device, const int64_t* partial, int64_t* summary, void* stream) {
    DXRL_REQUIRE(partial && summary, "null argument");
    DeviceGuard g(device);
    hipLaunchKernelGGL(k_sp_finish, dim3(1), dim3(kCap), 0, as_stream(stream), partial, summary);
    return launch_check("k_sp_finish");
}

}  // extern "C"
