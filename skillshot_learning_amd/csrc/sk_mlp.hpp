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
// Philox rounds of the bf16 actor's parameter-noise draws (normals16 /
// pairs8; A/B builds override).  Philox4x32-7 is the fewest rounds of the
// family that pass TestU01 BigCrush (Salmon et al., SC'11; 10 is the library
// default, kept as a safety margin everywhere else: the fp32 path's noise,
// the Dropout masks, the replay sampling, action noise).  The noisy bf16
// forward is VALU-issue-bound (~29 % of its cycles were Philox's 64-bit
// multiplies): 7 rounds take the 131,072-row launch 60.4 -> 55.8 us
// (profiles/r03y3_bf16_noise_pair_philox_ab.jsonl); the noise is pinned
// statistically (the two-sample KS test against explicit weight noise).
#ifndef SK_NOISE_ROUNDS
#define SK_NOISE_ROUNDS 7
#endif
template <int ROUNDS = 10>
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < ROUNDS; ++i) {
    // one v_mad_u64_u32 gives both halves of each product (instead of a
    // v_mul_lo_u32 + v_mul_hi_u32 pair), one v_bitop3_b32 (0x96: a^b^c) each xor
    const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u, p1 = (uint64_t)c.z * 0xCD9E8D57u;
    c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                   __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 16 normals of standard deviation sd for (row, stream, lane half h):
// Box-Muller on 2 Philox draws, each 32-bit word split into a 16-bit radius
// uniform and a 16-bit angle uniform (one word per normal pair; radius
// truncated at 4.86 sigma, P = 1.2e-6).  The two lane halves hold different
// hidden units of the same row, so h is part of the counter (independent noise
// per unit).  k2 = noise_k2(sd) = -2 ln2 sd^2 folds sd and ln -> log2 into the
// radius: rad = sqrt(k2 log2 u1) on v_log_f32 (u1 >= 2^-17: no denormal
// scaling), and the angle goes to v_sin_f32 / v_cos_f32 in revolutions, so a
// pair costs ~10 VALU instructions.  The RNG was half of the noisy actor's
// VALU instructions (PMC, profiles/r01t_*, r02_pmc_mfma_learner.json).
__host__ __device__ __forceinline__ float noise_k2(float sd) { return -1.3862943611198906f * sd * sd; }

__device__ __forceinline__ void normals16(uint64_t seed, uint64_t call, uint32_t row, uint32_t stream, int h,
                                          float k2, float z[16]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    uint4 u = philox<SK_NOISE_ROUNDS>(make_uint4(row, (stream * 2 + (uint32_t)h) * 2 + q, (uint32_t)call,
                                                 (uint32_t)(call >> 32)),
                     (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float u1 = ((float)(w[p] & 0xFFFFu) + 0.5f) * 0x1p-16f;  // (0, 1)
      const float rev = (float)(w[p] >> 16) * 0x1p-16f;               // [0, 1) revolutions
      const float rad = __builtin_amdgcn_sqrtf(k2 * __builtin_amdgcn_logf(u1));
      z[8 * q + 2 * p] = rad * __builtin_amdgcn_cosf(rev);
      z[8 * q + 2 * p + 1] = rad * __builtin_amdgcn_sinf(rev);
    }
  }
}

// The same 16 draws as normals16 in Box-Muller pair form, for the noisy
// pre-activations: pair p holds L = k2 log2 u1 (the squared radius) and the
// angle's cos / sin, so y_i = m + b + sqrt((b^2 + v) L) * {cos, sin} takes one
// square root per element (noisy_pre_pair) instead of the radius's plus the
// element's: 5 transcendentals per pair instead of 6 (the noisy bf16 forward is
// VALU-issue-bound; profiles/r03y3_bf16_noise_pair_philox_ab.jsonl)
struct Pairs8 {
  float L[8], c[8], s[8];
};
__device__ __forceinline__ void pairs8(uint64_t seed, uint64_t call, uint32_t row, uint32_t stream, int h, float k2,
                                       Pairs8& n) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    uint4 u = philox<SK_NOISE_ROUNDS>(make_uint4(row, (stream * 2 + (uint32_t)h) * 2 + q, (uint32_t)call,
                                                 (uint32_t)(call >> 32)),
                     (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float u1 = ((float)(w[p] & 0xFFFFu) + 0.5f) * 0x1p-16f;  // (0, 1)
      const float rev = (float)(w[p] >> 16) * 0x1p-16f;               // [0, 1) revolutions
      n.L[4 * q + p] = k2 * __builtin_amdgcn_logf(u1);
      n.c[4 * q + p] = __builtin_amdgcn_cosf(rev);
      n.s[4 * q + p] = __builtin_amdgcn_sinf(rev);
    }
  }
}
// element i of the pair form (normal i of normals16, for diagnostics)
__device__ __forceinline__ float pair_normal(const Pairs8& n, int i) {
  return __builtin_amdgcn_sqrtf(n.L[i >> 1]) * ((i & 1) ? n.s[i >> 1] : n.c[i >> 1]);
}
__device__ __forceinline__ float noisy_pre_pair(float m, float b, float v, const Pairs8& n, int i) {
  return __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v) * n.L[i >> 1]),
                        (i & 1) ? n.s[i >> 1] : n.c[i >> 1], m + b);
}

// 2 normals of standard deviation sd (model_act_action_noise's N(0, sd) on
// the two tanh outputs): one Philox draw, the first word as in normals16
__device__ __forceinline__ void normals2(uint64_t seed, uint64_t call, uint32_t row, uint32_t stream, float k2,
                                         float z[2]) {
  const uint4 u = philox(make_uint4(row, stream * 4u, (uint32_t)call, (uint32_t)(call >> 32)), (uint32_t)seed,
                         (uint32_t)(seed >> 32));
  const float u1 = ((float)(u.x & 0xFFFFu) + 0.5f) * 0x1p-16f;
  const float rev = (float)(u.x >> 16) * 0x1p-16f;
  const float rad = __builtin_amdgcn_sqrtf(k2 * __builtin_amdgcn_logf(u1));
  z[0] = rad * __builtin_amdgcn_cosf(rev);
  z[1] = rad * __builtin_amdgcn_sinf(rev);
}

// noisy pre-activation y = m + b + sqrt(v + b^2) * zs (zs already scaled by
// sd).  v is a sum of products of squares (>= 0), so v + b^2 needs no clamp.
__device__ __forceinline__ float noisy_pre(float m, float b, float v, float zs) {
  return __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v)), zs, m + b);
}

// ---------------------------------------------------------------- replay minibatch
// A minibatch drawn from the HBM replay ring inside a gradient launch
// (sk_critic_grad_f32_sampled, sk_critic_grad_bootstrap_sampled): batch row b
// is ring row floor(u_b size), u_b from Philox4x32-10 keyed (seed; b, draw,
// total), exactly k_replay_sample's row (csrc/sk_replay.hip), so the step
// equals sk_replay_sample + the step on the sampled rows, bit for bit.
struct RingSample {
  const float* ring;  // [cap][28]; NULL: no gather
  int64_t cap;
  const int64_t* total;
  uint64_t seed;
  int draw;
  float *s, *a, *r, *s2, *d;  // the sample buffers
  int64_t excl;  // rows a concurrent insert writes (0: every min(total, cap) row)
};
// excl == 0: floor(u min(t, cap)), k_replay_sample's row.  excl = E > 0 (the
// learner tick with the update beside the insert): the min(t, cap - E) most
// recent rows as of count t, i.e. none of the E rows the insert running
// beside it overwrites or adds, drawn with the same key.
__device__ __forceinline__ int64_t ring_row(const RingSample& q, int64_t b, int64_t t) {
  const uint4 u = philox<10>(make_uint4((uint32_t)b, (uint32_t)q.draw, (uint32_t)t, (uint32_t)(t >> 32)),
                             (uint32_t)q.seed, (uint32_t)(q.seed >> 32));
  const uint64_t u53 = (((uint64_t)u.x << 32) | u.y) >> 11;
  if (q.excl <= 0) {
    const uint64_t size = (uint64_t)(t < q.cap ? t : q.cap);
    return (int64_t)(((unsigned __int128)u53 * size) >> 53);
  }
  // the entry points reject excl outside [0, cap); the clamp keeps a bad
  // value from indexing outside the ring regardless
  const int64_t lim = q.cap - q.excl, el0 = t < lim ? t : lim, el = el0 > 0 ? el0 : 0;
  const int64_t k = (int64_t)(((unsigned __int128)u53 * (uint64_t)el) >> 53);
  return (t - el + k) % q.cap;
}
// float f (0..27) of a gathered ring row into the sample buffers: one store
// to an address chosen by selects (a store per branch let the waitcnt pass,
// its tracking lost across the branches, put a vmcnt(0) before each store, i.e.
// wait for the previous store's acknowledgement)
__device__ __forceinline__ void ring_scatter(const RingSample& q, int64_t b, int f, float v) {
  float* dst = f < 12 ? q.s + b * 12 + f
               : f < 14 ? q.a + b * 2 + (f - 12)
               : f == 14 ? q.r + b
               : f < 27 ? q.s2 + b * 12 + (f - 15)
               : q.d + b;
  *dst = v;
}

}  // namespace skmlp
