// dxrl_pg.h -- shapes and parameter layout of the actor-critic learner.
//
// Actor  : obs(45) -> 256 -> 256 -> mu(15), tanh hidden units, state-independent log_std(15)
// Critic : obs(45) -> 256 -> 256 -> V(1)
// 159,263 logical parameters.  Padded storage:
//   L1 [256][64]  : inputs = 45 obs features, column 45 = constant 1 (the bias), 46..63 zero
//   L2 [256][288] : columns 0..255 weights, column 256 = bias, 257..287 zero
//   L3 [32][288]  : rows 0..14 (actor) / row 0 (critic) used; column 256 = bias
// Feature-major activation buffers carry a constant-1 row 256 so the split-K
// weight-gradient GEMM yields the bias gradient as column 256 for free.
#pragma once
#include <stdint.h>

namespace dxrl {
namespace pg {

constexpr int kObsIn = 45;   // observation features
constexpr int kIn = 64;      // padded L1 input (bias column at kObsIn)
constexpr int kH = 256;      // hidden width
constexpr int kHx = 288;     // hidden + bias column + pad (multiple of 32)
constexpr int kOut = 32;     // padded head rows
constexpr int kAct = 15;     // action dim
constexpr int kActPad = 16;  // action tape row

// f32 master parameter block offsets (elements)
constexpr int64_t kW1 = (int64_t)kH * kIn;    // 16384
constexpr int64_t kW2 = (int64_t)kH * kHx;    // 73728
constexpr int64_t kW3 = (int64_t)kOut * kHx;  // 9216
constexpr int64_t kOffW1a = 0;
constexpr int64_t kOffW2a = kOffW1a + kW1;
constexpr int64_t kOffW3a = kOffW2a + kW2;
constexpr int64_t kOffLogStd = kOffW3a + kW3;  // 32 slots, 15 used
constexpr int64_t kOffW1c = kOffLogStd + 32;
constexpr int64_t kOffW2c = kOffW1c + kW1;
constexpr int64_t kOffW3c = kOffW2c + kW2;
constexpr int64_t kParams = kOffW3c + kW3;     // padded f32 master size

// bf16 pack (forward weights + transposed copies for input gradients)
constexpr int64_t kW2T = (int64_t)kH * kH;     // Bt[i][o] = W2[o][i]
constexpr int64_t kW3T = (int64_t)kH * kOut;   // Bt[i][o] = W3[o][i]
constexpr int64_t kBfW1a = 0;
constexpr int64_t kBfW2a = kBfW1a + kW1;
constexpr int64_t kBfW3a = kBfW2a + kW2;
constexpr int64_t kBfW2aT = kBfW3a + kW3;
constexpr int64_t kBfW3aT = kBfW2aT + kW2T;
constexpr int64_t kBfW1c = kBfW3aT + kW3T;
constexpr int64_t kBfW2c = kBfW1c + kW1;
constexpr int64_t kBfW3c = kBfW2c + kW2;
constexpr int64_t kBfW2cT = kBfW3c + kW3;
constexpr int64_t kBfW3cT = kBfW2cT + kW2T;
// MFMA-fragment-ordered copies for the fused learner's weight streams: a [N][K] matrix as
// [N / 32][K / 16][64 lanes][8], lane l of (feature tile ft, k-step k) holding W[32 ft + (l & 31)]
// [16 k + 8 (l >> 5) .. + 7] -- every fragment load is one contiguous 1 KiB wave read.
constexpr int64_t kFrW1 = (int64_t)kH * kIn, kFrW2 = (int64_t)kH * kH, kFrW3 = (int64_t)kOut * kH;
constexpr int64_t kFrW2T = (int64_t)kH * kH, kFrW3T = (int64_t)kH * kOut;
constexpr int64_t kFrNet = kFrW1 + kFrW2 + kFrW3 + kFrW2T + kFrW3T;
constexpr int64_t kFr = kBfW3cT + kW3T;  // actor block, then critic block
constexpr int64_t kFrOffW1 = 0, kFrOffW2 = kFrW1, kFrOffW3 = kFrOffW2 + kFrW2, kFrOffW2T = kFrOffW3 + kFrW3,
                  kFrOffW3T = kFrOffW2T + kFrW2T;
constexpr int64_t kBf = kFr + 2 * kFrNet;

}  // namespace pg
}  // namespace dxrl
