// sk_mlp.hpp — shared pieces of the fused MLP kernels (actor, critic) on
// gfx950 MFMA: bf16 fragment types, the packed-dword square, Philox4x32-10
// normals, and the fragment layouts of the 12 -> 256 and 256 -> 128 layers.
//
// Fragment layouts (v_mfma_f32_32x32x16_bf16; activations kept transposed,
// H^T = W X^T, batch row on the lane):
//   W1 [256][12]: A fragment of hidden chunk c (32 units), lane (r, h),
//       element j = W1[32c + r][8h + j] (k >= 12 -> 0)
//   W2 [128][>=256]: out chunk t, k-step kk, lane (r, h), element j =
//       W2[32t + r][32(kk>>1) + 16(kk&1) + 8(j>>2) + 4h + (j&3)]  (the row
//       order of the previous accumulator's registers 8s..8s+7, s = kk&1)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace skmlp {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kIn = 12, kH1 = 256, kH2 = 128, kOut = 2;
constexpr int kW1Frag = 8 * 64 * 16;        // 8 hidden chunks x 64 lanes x 8 bf16
constexpr int kW2Frag = 4 * 16 * 64 * 16;   // 4 out chunks x 16 k-steps x 64 lanes x 8 bf16

__device__ __forceinline__ short f2bf(float f) {  // round-to-nearest-even (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(short, (__bf16)f);
}

// elementwise square of a bf16 fragment (the variance chain's operand x^2 is
// derived at use instead of stored: keeps the noise kernel inside 256 VGPRs).
// Written on the packed dwords: the per-element __bf16 form of this loop was
// compiled (ROCm 7.2 clang, gfx950) into element 0's square broadcast to all
// eight elements.
__device__ __forceinline__ uint32_t sq_bf16x2(uint32_t w) {
  const float lo = __uint_as_float(w << 16), hi = __uint_as_float(w & 0xFFFF0000u);
  const uint32_t a = (uint32_t)(uint16_t)f2bf(lo * lo), b = (uint32_t)(uint16_t)f2bf(hi * hi);
  return a | (b << 16);
}
__device__ __forceinline__ bf16x8 sq_bf16(bf16x8 a) {
  uint4 u = __builtin_bit_cast(uint4, a);
  u.x = sq_bf16x2(u.x);
  u.y = sq_bf16x2(u.y);
  u.z = sq_bf16x2(u.z);
  u.w = sq_bf16x2(u.w);
  return __builtin_bit_cast(bf16x8, u);
}

// actor packed buffer layout (bytes), written by k_actor_pack
constexpr size_t kOffW1 = 0, kOffW1s = kOffW1 + kW1Frag;
constexpr size_t kOffW2 = kOffW1s + kW1Frag, kOffW2s = kOffW2 + kW2Frag;
constexpr size_t kOffB = kOffW2s + kW2Frag;  // fp32: b1[256] b2[128] b3[2] (pad 512)
constexpr size_t kOffW3f = kOffB + 512 * 4;  // fp32 W3[2][128] then W3^2[2][128] (layer 3 on the VALU)
constexpr size_t kPackedBytes = kOffW3f + 512 * 4;

// k index (input unit) of element j of lane half h in layer-2 k-step kk
__host__ __device__ __forceinline__ int w2_k(int kk, int h, int j) {
  return 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}

// ---------------------------------------------------------------- noise
template <int ROUNDS = 10>
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < ROUNDS; ++i) {
    uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 16 standard normals for (row, stream, lane half h): Box-Muller on 2 Philox
// draws, each 32-bit word split into a 16-bit radius uniform and a 16-bit
// angle uniform (one word per normal pair; radius truncated at 4.86 sigma,
// P = 1.2e-6).  The two lane halves hold different hidden units of the same
// row, so h is part of the counter (independent noise per unit).  The RNG
// was half of the noisy actor's VALU instructions (PMC, profiles/r01t_*).
__device__ __forceinline__ void normals16(uint64_t seed, uint64_t call, uint32_t row, uint32_t stream, int h,
                                          float z[16]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    uint4 u = philox(make_uint4(row, (stream * 2 + (uint32_t)h) * 2 + q, (uint32_t)call, (uint32_t)(call >> 32)),
                     (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float u1 = ((float)(w[p] & 0xFFFFu) + 0.5f) * 0x1p-16f;  // (0, 1)
      float u2 = (float)(w[p] >> 16) * 0x1p-16f;               // [0, 1)
      float rad = __builtin_amdgcn_sqrtf(-2.0f * __logf(u1));  // v_sqrt_f32 (1 ulp): noise scale
      float sn, cs;
      __sincosf(6.283185307179586f * u2, &sn, &cs);
      z[8 * q + 2 * p] = rad * cs;
      z[8 * q + 2 * p + 1] = rad * sn;
    }
  }
}

}  // namespace skmlp
