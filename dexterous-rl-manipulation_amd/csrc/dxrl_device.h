// dxrl_device.h -- per-env physics, contacts and reward terms for gfx950.
//
// One lane owns one env; every per-env quantity lives in registers.  The
// arithmetic restates the reference op by op under NumPy-2 (NEP 50) scalar
// promotion -- f32 where the reference's arrays are f32, f64 where NumPy
// promotes -- and the library is compiled with -ffp-contract=off so no
// multiply-add is fused (the reference never fuses).  Citations are into the
// reference checkout (envs/manipulation_env.py = ME, rewards/reward_shaping.py = RS,
// policies/simple_learner.py = SL).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dxrl.h"

namespace dxrl {

constexpr int kF = 5, kJ = 3, kD = kF * kJ;  // ME:26-27 defaults (compiled shape)
constexpr int kObs = 2 * kD + 10 + kF;       // ME:96-100 -> 45
constexpr int kReset = kD + DXRL_RESET_EXTRA;

// Python-float literals as NumPy sees them next to an f32 array: the double
// rounded to f32 (NEP 50 weak scalar), not the decimal rounded to f32.
constexpr float kC09 = (float)0.9, kC01 = (float)0.1, kDt = (float)0.01;
constexpr double kGz = -9.81 * 0.01;  // ME:211-212 gravity (f64)
constexpr double kLo[3] = {-0.2, -0.2, 0.0}, kHi[3] = {0.2, 0.2, 0.3};  // ME:119

// flag word bits
constexpr uint32_t kPrevShift = 8, kHasPrev = 1u << 16, kOpIsF32 = 1u << 17, kHasObject = 1u << 18,
                   kFricF64 = 1u << 19;  // episode friction is a numpy.float64 (NEP 50 f64 damping)

struct Weights {
    double w_dist, w_con, w_clo, w_st;
};

// np.clip / np.minimum(np.maximum(x, lo), hi) without NaN canonicalisation.
__device__ __forceinline__ float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ double clipd(double x, double lo, double hi) {
    double y = x < lo ? lo : x;  // np.maximum(x, lo)
    return y > hi ? hi : y;      // np.minimum(., hi)
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // each 32x32 -> 64-bit product as one v_mad_u64_u32 (both halves), not mul_lo + mul_hi
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
// 53-bit uniform in [0,1), as numpy's next_double((u64 >> 11) * 2^-53)
__device__ __forceinline__ double u01_53(uint32_t hi, uint32_t lo) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    return (double)(v >> 11) * (1.0 / 9007199254740992.0);
}
// 24-bit uniform in (0,1]
__device__ __forceinline__ float u01_24(uint32_t v) { return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f); }
// Box-Muller on the hardware transcendentals, for uniforms u1 = (v + 1) 2^-kBits (v = the
// kBits-bit integer of the first source, u1 formed exactly) and u2 (the angle in revolutions,
// which v_sin_f32 / v_cos_f32 take directly): r = sqrt(-2 ln 2 log2 u1) with v_log_f32 (log2) of
// u1 itself (log2 of v + 1 minus kBits would cancel near u1 = 1).  The same values as
// sqrt(-2 __logf(u1)) and __sincosf(2 pi u2) up to the hardware approximations, in 12 vector
// instructions + 4 transcendentals per pair instead of 23 + 4 (__logf is libm-accurate: a
// denormal rescale and a two-term ln 2 product around its v_log_f32; __sincosf scales by 2 pi
// and back).  The clamp keeps r real should log2 of u1 <= 1 round above zero.
template <int kBits>
__device__ __forceinline__ void box_muller_hw(uint32_t v, float u2_rev, float& n0, float& n1) {
    constexpr float kM2Ln2 = -1.38629436111989061883f, kUlp = 1.0f / (float)(1u << kBits);
    const float l = __builtin_amdgcn_logf((float)(v + 1u) * kUlp);
    const float r = __builtin_amdgcn_sqrtf(fmaxf(l * kM2Ln2, 0.0f));
    n0 = r * __builtin_amdgcn_cosf(u2_rev);
    n1 = r * __builtin_amdgcn_sinf(u2_rev);
}
// two standard normals (Box-Muller, f32) from two u32 (24-bit uniforms in (0, 1]): the policy
// noise.  Network-noise math, not parity math (no CPU restatement replays these values: parity
// runs replay the device's action tape).  Kept on __logf / __sincosf: box_muller_hw<24> here
// made the C2 rollout 1.2-1.8 % slower (its draws run in the head phase beside the mu head) while
// the fused noise gained from it (profiles/r05/ab_box_muller.log)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
    const float r = __builtin_amdgcn_sqrtf(-2.0f * __logf(u01_24(a)));
    float s, c;
    __sincosf(6.28318530717958647692f * u01_24(b), &s, &c);
    n0 = r * c;
    n1 = r * s;
}

// Stream ids for the Philox counter's third word.
constexpr uint32_t kStreamReset = 0x52535400u, kStreamPolicy = 0x504f4c00u, kStreamDyn = 0x44594e00u,
                   kStreamObs = 0x4f425300u;

// ---------------------------------------------------------------- fused noise (config C5)
// Block `blk` of a noise stream (kStreamDyn / kStreamObs) at counter ctr: four standard normals,
// normal 4 blk + j in nz[j].  Throughput-mode robustness noise has distributional parity with the
// reference's default_rng normals only (robustness_tests.py:177-207; the host-tape path replays
// those exactly), so its generator is the build's own (round 6):
//   Philox2x32-10 (Random123: M = 0xD256D193, Weyl 0x9E3779B9) of the counter
//   (lo ctr, hi ctr << 8 ^ stream ^ blk) under the key k0 ^ k1 * 0x9E3779B9 -> words (w0, w1), and
//   s = the generator's first word after round 5 of the 10; pair 0 = Box-Muller of w0, pair 1 of
//   w1: the angle is the word's high 16 bits, the radius uniform the 24-bit integer
//   (word & 0xFFFF) << 8 | byte of s (byte 0 for w0, byte 1 for w1).
// The 24-bit radius uniform keeps the normal tail to |z| <= sqrt(-2 ln 2^-24) = 5.77 (round 5 drew
// it from 16 bits: |z| <= 4.71, a tail quantised to a few radius values above 3.5 sigma).  s costs
// no product: it is a state the ten rounds pass through anyway, five rounds of mixing from the
// counter and five from the output words.  oracle/dx_oracle.py device_normals_f64 restates it.
__device__ __forceinline__ void philox2x32_10(uint32_t& c0, uint32_t& c1, uint32_t k, uint32_t& mid) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p = (uint64_t)0xD256D193u * c0;  // one v_mad_u64_u32
        const uint32_t hi = (uint32_t)(p >> 32), lo = (uint32_t)p;
        c0 = hi ^ k ^ c1;
        c1 = lo;
        k += 0x9E3779B9u;
        if (r == 4) mid = c0;
    }
}
// One Box-Muller pair: angle = the high 16 bits of w, u2 = (hi + 1) 2^-16 as 1 + (hi + 1) 2^-16
// revolutions (one period on: the bits of hi placed in the mantissa of 1.0 and 2^-16 added, both
// exact); radius uniform (v24 + 1) 2^-24, v24 = (w & 0xFFFF) << 8 | e (e: one byte of s)
__device__ __forceinline__ void box_muller24(uint32_t w, uint32_t e, float& n0, float& n1) {
    const float rev = __uint_as_float(0x3F800000u | ((w >> 16) << 7)) + (1.0f / 65536.0f);
    box_muller_hw<24>(((w & 0xFFFFu) << 8) | (e & 0xFFu), rev, n0, n1);
}
__device__ __forceinline__ void noise_normals4(uint64_t ctr, uint32_t stream, uint32_t blk, uint32_t k0, uint32_t k1,
                                               float nz[4]) {
    uint32_t c0 = (uint32_t)ctr, c1 = ((uint32_t)(ctr >> 32) << 8) ^ stream ^ blk, s = 0;
    philox2x32_10(c0, c1, k0 ^ (k1 * 0x9E3779B9u), s);
    box_muller24(c0, s, nz[0], nz[1]);
    box_muller24(c1, s >> 8, nz[2], nz[3]);
}

__device__ __forceinline__ void env_key(uint64_t seed, int64_t gid, uint32_t& k0, uint32_t& k1) {
    k0 = (uint32_t)gid ^ (uint32_t)(seed >> 32) * 0x85EBCA6Bu;
    k1 = (uint32_t)seed ^ (uint32_t)((uint64_t)gid >> 32) * 0xC2B2AE35u;
}

// ---------------------------------------------------------------- env registers
struct Env {
    float jp[kD], jv[kD];
    double op[3];
    float ov[3];
    uint32_t flags;
    int32_t t;
    double size, mass, fric;
    int32_t cfg;
};

// ME:285-310 _update_contacts.  tip_f = f64(f32(f32(sum_seq joints) * 0.1f)),
// d_f = sqrt(((tx-ox)^2 + (ty-oy)^2) + (tz-oz)^2) in f64 (np.linalg.norm axis=1),
// contact_f = d_f < size * 1.5.  Returns the contact bitmask; min distance out.
__device__ __forceinline__ uint32_t contacts_of(const Env& e, double& dmin) {
    const double thr = e.size * 1.5;
    uint32_t mask = 0;
    dmin = 0.0;
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        float s = e.jp[kJ * f];
#pragma unroll
        for (int j = 1; j < kJ; ++j) s = s + e.jp[kJ * f + j];
        const double tip = (double)(s * kC01);
        const double dx = tip - e.op[0], dy = tip - e.op[1], dz = tip - e.op[2];
        const double d = sqrt((dx * dx + dy * dy) + dz * dz);
        mask |= (d < thr ? 1u : 0u) << f;
        dmin = (f == 0 || d < dmin) ? d : dmin;  // np.min
    }
    return mask;
}

// k / kF for a contact count k = 0..kF, bit for bit the correctly rounded quotient (the quotients
// are compile-time constants, selected: no division instruction sequence on the step's path)
__device__ __forceinline__ double count_over_f_f64(uint32_t k) {
    double r = 0.0;
#pragma unroll
    for (int q = 1; q <= kF; ++q) r = k == (uint32_t)q ? (double)q / (double)kF : r;
    return r;
}
__device__ __forceinline__ float count_over_f_f32(uint32_t k) {
    float r = 0.0f;
#pragma unroll
    for (int q = 1; q <= kF; ++q) r = k == (uint32_t)q ? (float)q / (float)kF : r;
    return r;
}

// x / 5 in f32, correctly rounded, without the division sequence (-fhip-fp32-correctly-rounded-
// divide-sqrt compiles x / 5.0f to ~10 dependent instructions): RN32(RN64(x * RN64(0.2))).  For a
// normal f32 x = M 2^k the exact quotient is at least ulp(q) / 10 from every f32 midpoint (the
// numerator of q - mid is a nonzero multiple of 2^(j - 1) over 5), while the f64 product is within
// ~2^-52 q of x / 5, so both roundings land on the same f32 (tests/test_host_logic.py checks it
// against IEEE f32 division over whole binades).
static_assert(kF == 5, "div_f: the finger count's reciprocal constant");
__device__ __forceinline__ float div_f(float x) { return (float)((double)x * 0.2); }

// RS:101-187 dense terms + weighted total (RS:84-89); updates prev contacts.
__device__ __forceinline__ double dense_reward(Env& e, uint32_t c, double dmin, const Weights& w, double comp[4]) {
    const double dist = exp(-5.0 * dmin);                 // RS:111-116
    const int n = __popc(c);
    const double con = count_over_f_f64((uint32_t)n);     // RS:128-134 (n / 5)
    float sum = 0.0f;                                     // RS:147-162
#pragma unroll
    for (int f = 0; f < kF; ++f) {
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
            const float v = e.jp[kJ * f + j];
            if (v < 0.0f) acc = acc + v;
        }
        sum = sum + (-acc);
    }
    const float avg = div_f(sum);                         // np.mean(...)  (f32 / 5)
    const float clo = clipf(div_f(avg), 0.0f, 1.0f);      // avg / num_fingers
    float st = 0.0f;                                      // RS:166-187
    if (e.flags & kHasPrev) {
        const uint32_t prev = (e.flags >> kPrevShift) & 0xFFu;
        float ch = 0.0f;
#pragma unroll
        for (int f = 0; f < kF; ++f) ch = ch + (float)(((c ^ prev) >> f) & 1u);
        st = clipf(1.0f - count_over_f_f32((uint32_t)ch), 0.0f, 1.0f);
    }
    e.flags = (e.flags & ~(0xFFu << kPrevShift)) | (c << kPrevShift) | kHasPrev;
    comp[0] = dist;
    comp[1] = con;
    comp[2] = (double)clo;
    comp[3] = (double)st;
    return ((w.w_dist * dist + w.w_con * con) + w.w_clo * (double)clo) + w.w_st * (double)st;
}

// ME:198-252 one step.  a[] = raw action (clipped here, ME:199).
// Returns reward; term/trunc flags; comp[] the reward components.
__device__ __forceinline__ double env_step(Env& e, const float* a, bool dense, const Weights& w,
                                           int max_episode_steps, bool& term, bool& trunc, double comp[4]) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        const float ak = clipf(a[k], -1.0f, 1.0f);
        e.jv[k] = kC09 * e.jv[k] + kC01 * ak;                  // ME:203 (f32, no FMA)
        e.jp[k] = clipf(e.jp[k] + e.jv[k] * kDt, -1.0f, 1.0f);  // ME:204-207
    }
    const double damp = 1.0 - (e.fric * 0.1 * 0.01);  // ME:215
    const float dampf = (float)damp;
    const double g[3] = {0.0, 0.0, kGz};
    const bool op32 = (e.flags & kOpIsF32) != 0;
    const bool fric_f64 = (e.flags & kFricF64) != 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float v = fric_f64 ? (float)((double)e.ov[i] * damp) : e.ov[i] * dampf;  // ME:216 (NEP 50)
        v = (float)((double)v + g[i]);                                          // ME:219 f32 += f64
        const float inc = v * kDt;                                              // ME:222
        double p = op32 ? (double)((float)e.op[i] + inc) : e.op[i] + (double)inc;
        p = clipd(p, kLo[i], kHi[i]);                                           // ME:225-229 -> f64
        if ((p <= kLo[i] && v < 0.0f) || (p >= kHi[i] && v > 0.0f)) v = 0.0f;   // ME:232-235
        e.op[i] = p;
        e.ov[i] = v;
    }
    e.flags &= ~kOpIsF32;
    double dmin;
    const uint32_t c = contacts_of(e, dmin);                                    // ME:238
    double r;
    if (dense) {
        r = dense_reward(e, c, dmin, w, comp);
    } else {
        r = (__popc(c) >= 3) ? 1.0 : -0.01;  // RS:226-231
        comp[0] = comp[1] = comp[2] = comp[3] = 0.0;
    }
    e.flags = (e.flags & ~0xFFu) | c;
    term = __popc(c) >= 3;                   // ME:332-336
    trunc = e.t >= max_episode_steps;        // ME:245 (before the increment)
    e.t += 1;                                // ME:247
    return r;
}

// ME:124-182 reset from resolved draws (see DXRL_RESET_EXTRA slot order).
__device__ __forceinline__ void env_reset(Env& e, const double* draw, const dxrl_curriculum& cu) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        e.jp[k] = (float)draw[k];  // ME:143-145 .astype(float32)
        e.jv[k] = 0.0f;
    }
    e.size = cu.has_size_range ? draw[kD + 0] : cu.object_size;  // config.py:44-84
    e.mass = cu.has_mass_range ? draw[kD + 1] : cu.object_mass;
    e.fric = cu.has_friction_range ? draw[kD + 2] : cu.friction_coefficient;
    const bool has = (e.flags & kHasObject) != 0;  // ME:156-161 sticky position
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        e.op[i] = (double)(float)(has ? e.op[i] : draw[kD + 3 + i]);
        e.ov[i] = 0.0f;
    }
    e.t = 0;
    // prev_contacts = None (RS:45-48); the host marks rows whose episode friction is a numpy.float64
    e.flags = kOpIsF32 | kHasObject | (cu.friction_is_f64_scalar ? kFricF64 : 0u);
    double dmin;
    e.flags |= contacts_of(e, dmin);  // ME:176
}

// Device-RNG reset draws: the same slots, uniform(lo, hi) = lo + (hi-lo)*u.
__device__ __forceinline__ void philox_reset_draws(double* d, const dxrl_curriculum& cu, uint32_t k0, uint32_t k1,
                                                   uint64_t ctr) {
    uint32_t u[2 * kReset + 2];
#pragma unroll
    for (int b = 0; b < (2 * kReset + 3) / 4; ++b) {
        const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamReset, (uint32_t)b}, k0, k1);
        if (4 * b + 0 < 2 * kReset + 2) u[4 * b + 0] = r.x;
        if (4 * b + 1 < 2 * kReset + 2) u[4 * b + 1] = r.y;
        if (4 * b + 2 < 2 * kReset + 2) u[4 * b + 2] = r.z;
        if (4 * b + 3 < 2 * kReset + 2) u[4 * b + 3] = r.w;
    }
#pragma unroll
    for (int k = 0; k < kD; ++k) d[k] = -0.1 + (0.1 - -0.1) * u01_53(u[2 * k], u[2 * k + 1]);
    const double* rng[6] = {cu.size_range, cu.mass_range, cu.friction_range,
                            cu.spawn_x_range, cu.spawn_y_range, cu.spawn_z_range};
#pragma unroll
    for (int k = 0; k < 6; ++k)
        d[kD + k] = rng[k][0] + (rng[k][1] - rng[k][0]) * u01_53(u[2 * (kD + k)], u[2 * (kD + k) + 1]);
}

// env_reset(philox_reset_draws(...)) without materialising the 21 draws: each
// Philox block yields two 53-bit uniforms (slots 2b, 2b+1) that are consumed
// on the spot.  Bit-identical to the two-step form (same slots, same arithmetic).
__device__ __forceinline__ void env_reset_philox(Env& e, const dxrl_curriculum& cu, uint32_t k0, uint32_t k1,
                                                 uint64_t ctr) {
    const bool has = (e.flags & kHasObject) != 0;
    double spawn[3];
#pragma unroll
    for (int b = 0; b < (kReset + 1) / 2; ++b) {
        const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamReset, (uint32_t)b}, k0, k1);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int k = 2 * b + half;
            if (k >= kReset) break;
            const double u = half ? u01_53(r.z, r.w) : u01_53(r.x, r.y);
            if (k < kD) {
                e.jp[k] = (float)(-0.1 + (0.1 - -0.1) * u);
                e.jv[k] = 0.0f;
            } else if (k == kD + 0) {
                e.size = cu.has_size_range ? cu.size_range[0] + (cu.size_range[1] - cu.size_range[0]) * u : cu.object_size;
            } else if (k == kD + 1) {
                e.mass = cu.has_mass_range ? cu.mass_range[0] + (cu.mass_range[1] - cu.mass_range[0]) * u : cu.object_mass;
            } else if (k == kD + 2) {
                e.fric = cu.has_friction_range ? cu.friction_range[0] + (cu.friction_range[1] - cu.friction_range[0]) * u
                                               : cu.friction_coefficient;
            } else {
                const double* rg = k == kD + 3 ? cu.spawn_x_range : (k == kD + 4 ? cu.spawn_y_range : cu.spawn_z_range);
                spawn[k - kD - 3] = rg[0] + (rg[1] - rg[0]) * u;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        e.op[i] = (double)(float)(has ? e.op[i] : spawn[i]);
        e.ov[i] = 0.0f;
    }
    e.t = 0;
    e.flags = kOpIsF32 | kHasObject | (cu.friction_is_f64_scalar ? kFricF64 : 0u);
    double dmin;
    e.flags |= contacts_of(e, dmin);
}

__device__ __forceinline__ void write_obs(const Env& e, float* o) {  // ME:254-264
#pragma unroll
    for (int k = 0; k < kD; ++k) o[k] = e.jp[k];
#pragma unroll
    for (int k = 0; k < kD; ++k) o[kD + k] = e.jv[k];
#pragma unroll
    for (int i = 0; i < 3; ++i) o[2 * kD + i] = (float)e.op[i];
    o[2 * kD + 3] = 1.0f;  // identity quaternion (ME:164)
    o[2 * kD + 4] = 0.0f;
    o[2 * kD + 5] = 0.0f;
    o[2 * kD + 6] = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) o[2 * kD + 7 + i] = e.ov[i];
#pragma unroll
    for (int f = 0; f < kF; ++f) o[2 * kD + 10 + f] = (float)((e.flags >> f) & 1u);
}

// ---------------------------------------------------------------- SoA access
struct EnvSoA {
    float* jp;
    float* jv;
    double* op;
    float* ov;
    uint32_t* flags;
    int32_t* t;
    double *size, *mass, *fric;
    int32_t* cfg;
    uint64_t* reset_ctr;
    double* comps;
    const dxrl_curriculum* curricula;
    int64_t n;
};

__device__ __forceinline__ void load_env(const EnvSoA& s, int64_t i, Env& e) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        e.jp[k] = s.jp[k * s.n + i];
        e.jv[k] = s.jv[k * s.n + i];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        e.op[k] = s.op[k * s.n + i];
        e.ov[k] = s.ov[k * s.n + i];
    }
    e.flags = s.flags[i];
    e.t = s.t[i];
    e.size = s.size[i];
    e.mass = s.mass[i];
    e.fric = s.fric[i];
    e.cfg = s.cfg[i];
}

// Step-only traffic: the episode constants (size, friction) are read, never
// written; mass and the curriculum row are not touched by a step.
__device__ __forceinline__ void load_env_dyn(const EnvSoA& s, int64_t i, Env& e) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        e.jp[k] = s.jp[k * s.n + i];
        e.jv[k] = s.jv[k * s.n + i];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        e.op[k] = s.op[k * s.n + i];
        e.ov[k] = s.ov[k * s.n + i];
    }
    e.flags = s.flags[i];
    e.t = s.t[i];
    e.size = s.size[i];
    e.fric = s.fric[i];
}

__device__ __forceinline__ void store_env_dyn(const EnvSoA& s, int64_t i, const Env& e) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        s.jp[k * s.n + i] = e.jp[k];
        s.jv[k * s.n + i] = e.jv[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s.op[k * s.n + i] = e.op[k];
        s.ov[k * s.n + i] = e.ov[k];
    }
    s.flags[i] = e.flags;
    s.t[i] = e.t;
}

__device__ __forceinline__ void store_env(const EnvSoA& s, int64_t i, const Env& e) {
#pragma unroll
    for (int k = 0; k < kD; ++k) {
        s.jp[k * s.n + i] = e.jp[k];
        s.jv[k * s.n + i] = e.jv[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s.op[k * s.n + i] = e.op[k];
        s.ov[k * s.n + i] = e.ov[k];
    }
    s.flags[i] = e.flags;
    s.t[i] = e.t;
    s.size[i] = e.size;
    s.mass[i] = e.mass;
    s.fric[i] = e.fric;
}

// standard normal k of Philox block k / 4 (Box-Muller pairs (x, y), (z, w)), as philox_normals
__device__ __forceinline__ float philox_normal_at(int k, uint32_t k0, uint32_t k1, uint64_t ctr, uint32_t stream) {
    if (stream != kStreamPolicy) {  // a noise stream: its own generator (noise_normals4)
        float nz[4];
        noise_normals4(ctr, stream, (uint32_t)(k >> 2), k0, k1, nz);
        return nz[k & 3];
    }
    const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), stream, (uint32_t)(k >> 2)}, k0, k1);
    float n0, n1;  // operands selected first: one branch-free Box-Muller (schedulable into MFMA gaps)
    const bool hi = (k & 2) != 0;
    box_muller(hi ? r.z : r.x, hi ? r.w : r.y, n0, n1);
    return (k & 1) ? n1 : n0;
}

// 53-bit uniform of reset slot k (Philox block k / 2, half k % 2), as env_reset_philox
__device__ __forceinline__ double reset_uniform_at(int k, uint32_t k0, uint32_t k1, uint64_t ctr) {
    const u32x4 r = philox(u32x4{(uint32_t)ctr, (uint32_t)(ctr >> 32), kStreamReset, (uint32_t)(k >> 1)}, k0, k1);
    return (k & 1) ? u01_53(r.z, r.w) : u01_53(r.x, r.y);
}

// ---------------------------------------------------------------- lane-split envs
// An env spread over the 16 lanes of one DPP row (lane s: joint s, lanes 0..2 the object axes);
// row_newbcast:K (DPP control 0x150 + K) hands lane K's value to every lane of its row in one
// VALU op.  Used by the rollout (k_pg_rollout_ws) and the evaluation programs (k_eval_ls);
// call only where the whole row is active.
template <int K>
__device__ __forceinline__ uint32_t row_bcast_u32(uint32_t x) {
    // every lane of the row reads a valid source lane, so the "old" operand is never used: the
    // undefined-old form (mov_dpp) spares the v_mov_b32 0 the update_dpp(0, ...) form put in front
    // of each broadcast
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + K, 0xF, 0xF, true);  // row_newbcast:K
}
template <int K>
__device__ __forceinline__ float row_bcast(float x) {
    return __uint_as_float(row_bcast_u32<K>(__float_as_uint(x)));
}
template <int K>
__device__ __forceinline__ double row_bcast(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    const uint64_t lo = row_bcast_u32<K>((uint32_t)u), hi = row_bcast_u32<K>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)((hi << 32) | lo));
}
// acc = ((acc + x_0) + x_1) + ... + x_{N-1} with x_k = lane k's x (the reference's sequential order)
template <int N, int K = 0>
__device__ __forceinline__ void row_sum_in_order(float x, float& acc) {
    if constexpr (K < N) {
        acc += row_bcast<K>(x);
        row_sum_in_order<N, K + 1>(x, acc);
    }
}
template <int K = 0>
__device__ __forceinline__ void row_joints(float jp, float (&J)[kD]) {
    if constexpr (K < kD) {
        J[K] = row_bcast<K>(jp);
        row_joints<K + 1>(jp, J);
    }
}
// sqrt_rn(x) < t for doubles x >= 0, t > 0, without the square root on the common path:
// q = fl(t t); x < q (1 - 2^-40) implies sqrt(x) < t (1 - 2^-42), so the correctly rounded root
// is < t; x > q (1 + 2^-40) implies sqrt(x) > t (1 + 2^-43), so it is >= t.  Only an x within
// ~2^-40 relative of t^2 (a lane essentially on the contact threshold) takes the exact root.
__device__ __forceinline__ bool sqrt_below(double x, double t) {
    const double q = t * t;
    if (x < q * (1.0 - 0x1p-40)) return true;
    if (x > q * (1.0 + 0x1p-40)) return false;
    return sqrt(x) < t;
}
// lane s receives lane s + N's value within its 16-lane row (row_shl:N; lanes past the row end
// read 0 -- they are never finger lanes)
template <int N>
__device__ __forceinline__ float row_shl(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x100 + N, 0xF, 0xF, true));
}
// finger lanes of a row: lane 3 f holds finger f's joints 3 f .. 3 f + 2 after two row shifts
__device__ __forceinline__ bool finger_lane(int s) { return s < kD && s % kJ == 0; }
// Lane-split contacts_of (ME:285-310) over a DPP row: finger lane 3f gathers its finger's three
// joint positions with two row shifts (no LDS round trip: the ds_bpermute gather sat on the step's
// dependent chain twice per reset step) and sums them in the reference's order; every lane gets
// the mask (ballot, the finger lanes' bits compressed to bit f) and the minimum distance.
// g3: the finger's joints (finger lanes).
// The contact test d_f < size * 1.5 runs on the squared distance (sqrt_below: bit-exact), and
// dmin = min_f sqrt_rn(x_f) = sqrt_rn(min_f x_f) (the correctly rounded root is monotone), so one
// root per row, off the mask's dependency chain; kDmin = false (the contacts of a reset state,
// ME:176) skips it.
template <bool kDmin = true>
__device__ __forceinline__ uint32_t row_contacts(float jp, const double op[3], double size, int s, int gbit,
                                                 double& dmin, float g3[3]) {
    static_assert(kJ == 3 && kF * kJ <= 16, "finger lanes 3 f of a 16-lane row");
    g3[0] = jp;
    g3[1] = row_shl<1>(jp);
    g3[2] = row_shl<2>(jp);
    const float sum = (g3[0] + g3[1]) + g3[2];  // np.sum of the finger's f32 joints, in order
    const double tip = (double)(sum * kC01);
    const double dx = tip - op[0], dy = tip - op[1], dz = tip - op[2];
    const double x = (dx * dx + dy * dy) + dz * dz;
    const bool hit = finger_lane(s) && sqrt_below(x, size * 1.5);
    const uint32_t r16 = (uint32_t)(__ballot(hit) >> gbit);  // bit 3 f: finger f
    const uint32_t mask = (r16 & 1u) | ((r16 >> 2) & 2u) | ((r16 >> 4) & 4u) | ((r16 >> 6) & 8u) | ((r16 >> 8) & 16u);
    if constexpr (kDmin) {
        double xm = row_bcast<0>(x);
        const double x1 = row_bcast<3>(x), x2 = row_bcast<6>(x), x3 = row_bcast<9>(x), x4 = row_bcast<12>(x);
        xm = x1 < xm ? x1 : xm;
        xm = x2 < xm ? x2 : xm;
        xm = x3 < xm ? x3 : xm;
        xm = x4 < xm ? x4 : xm;
        dmin = sqrt(xm);
    } else {
        dmin = 0.0;
    }
    return mask;
}
__device__ __forceinline__ void row_object(double opd, double op[3]) {
    op[0] = row_bcast<0>(opd);
    op[1] = row_bcast<1>(opd);
    op[2] = row_bcast<2>(opd);
}

// acc = ((acc + (-x_0)) + (-x_1)) + ...  over the finger lanes 0, 3, .., 12 (x_f on lane 3 f: the
// closure term's sum of finger sums, RS:147-162)
template <int K = 0>
__device__ __forceinline__ void row_neg_sum_fingers(float x, float& acc) {
    if constexpr (K < kF) {
        acc = acc + (-row_bcast<kJ * K>(x));
        row_neg_sum_fingers<K + 1>(x, acc);
    }
}

// observation element k written by lane s (ME:254-264), slot j of at most 4; -1 = none
__device__ __forceinline__ int row_obs_elem(int s, int j) {
    if (j == 0) return s < kD ? s : -1;
    if (j == 1) return s < kD ? kD + s : -1;
    if (j == 2) return s < 7 ? 2 * kD + s : (s < 7 + kF ? 2 * kD + 10 + (s - 7) : -1);
    return s < 3 ? 2 * kD + 7 + s : -1;
}

}  // namespace dxrl
