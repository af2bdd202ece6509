// sk_partial.hpp — layout of the per-workgroup gradient partials that the
// gradient kernels (sk_update.hip, sk_learn32.hip) write and k_adam_flat sums.
//
// torch parameters() order (update_kernel.flatten_module), except the
// critic's W2 [128][258]: its 256 main columns are stored as 256-float rows
// (so the 32 lanes of a store write one aligned 128-byte line instead of
// straddling two), followed by the two action columns as [128][2].  Every
// other offset equals the flat parameter offset, and the actor's W2 is
// already [128][256].
#pragma once

namespace skpart {

constexpr int kIn = 12, kH1 = 256, kH2 = 128;
constexpr int kPW2 = kH1 * kIn + kH1;  // W1, b1 first
constexpr int kCriticParams = 36609;

__host__ __device__ constexpr int critic_w2_main(int o, int i) { return kPW2 + o * kH1 + i; }
__host__ __device__ constexpr int critic_w2_action(int o, int j) { return kPW2 + kH2 * kH1 + 2 * o + j; }

// partial offset of flat parameter p of a net with n_params parameters
__host__ __device__ inline int index(int p, int n_params) {
  if (n_params != kCriticParams || p < kPW2 || p >= kPW2 + kH2 * (kH1 + 2)) return p;
  const int q = p - kPW2, o = q / (kH1 + 2), i = q - o * (kH1 + 2);
  return i < kH1 ? critic_w2_main(o, i) : critic_w2_action(o, i - kH1);
}

}  // namespace skpart
