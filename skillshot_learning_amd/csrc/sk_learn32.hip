// sk_learn32.hip — the learner at the reference's precision: fp32 operands
// and fp32 accumulation on v_mfma_f32_32x32x2_f32 (exact f32 products, the
// f32 VECTOR rate of MI355X: 157 TF), for the Keras fp32 nets of
// SkillshotLearner.py:70-121 and their update (:386-443).
//
//   k_actor_fwd32   actor forward 12 -> 256 relu -> 128 relu -> 2 tanh for a
//                   [rows, 12] batch, optionally with the reference's parameter
//                   noise w <- w (1 + sd N(0,1)) (:245-281) sampled exactly in
//                   distribution per row by local reparameterisation
//   k_critic_grad32 critic train step: (bootstrap target from the target nets,)
//                   Dropout(0.2) forward, MSE, backward -> per-workgroup
//                   gradient partials
//   k_actor_grad32  actor step: actor forward, critic forward at inference,
//                   dQ/da, backward of -sum Q -> per-workgroup partials
// The partials are summed (and Adam applied) by k_adam_flat (sk_update.hip).
//
// No packing: the kernels read the weights straight from the nets' flat fp32
// parameter vectors in torch parameters() order (update_kernel.flatten_module)
// W1 [256][12], b1, W2 [128][ld2], b2, W3 [n_out][128], b3 (ld2 = 258 for the
// critic: the last two columns multiply the action).
//
// MFMA operand trick.  v_mfma_f32_32x32x2_f32 contracts K = 2: lane l holds
// A[l%32][k0 + l/32] and B[k0 + l/32][l%32]; D register v of lane l is
// D[8(v/4) + 4(l/32) + v%4][l%32].  A GEMM whose operands are both
// k-contiguous loads a float4 per lane (lane half h = l/32 takes k0 + 4h ..
// k0 + 4h + 3) and issues 4 MFMAs, MFMA t contracting the pair {k0 + t,
// k0 + 4 + t}: every k appears exactly once, so the sum is the GEMM's (in a
// different order, which fp32 tolerates: tests hold it to 1e-5 of fp64).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <cstring>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"
#include "sk_partial.hpp"
#include "sk_split.hpp"
#include "sk_step.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // W2 rows of the critic are 8-B aligned

constexpr int kIn = 12, kH1 = 256, kH2 = 128;
constexpr int kLdH1 = 260, kLdH2 = 132;  // LDS row strides (floats): 16-B aligned, banks rotated
constexpr int kThreads = 512;                        // grad kernels: 8 waves per 32-row sub-tile
constexpr int kFwdThreads = 256;                     // forward: 4 waves per 32-row tile

// flat parameter offsets (torch parameters() order)
constexpr int kPW1 = 0, kPB1 = kH1 * kIn, kPW2 = kPB1 + kH1;
__host__ __device__ constexpr int pB2(int ld2) { return kPW2 + kH2 * ld2; }
__host__ __device__ constexpr int pW3(int ld2) { return pB2(ld2) + kH2; }
__host__ __device__ constexpr int pB3(int ld2, int n_out) { return pW3(ld2) + n_out * kH2; }
constexpr int kCLd = kH1 + 2, kALd = kH1;
constexpr int kCP = pB3(kCLd, 1) + 1, kAP = pB3(kALd, 2) + 2;
static_assert(kCP == 36609 && kAP == 36482 && kCP == skpart::kCriticParams && kPW2 == skpart::kPW2, "parameter counts");

// Weights are read through GLOBAL-address-space pointers: laundered (below)
// generic pointers would become FLAT loads, which count on lgkmcnt too, so
// every LDS wait would also wait for the in-flight weight loads
typedef const __attribute__((address_space(1))) float* gfp;
typedef const __attribute__((address_space(1))) f4u* gf4u;
struct Net {  // views into one flat parameter vector
  gfp W1, b1, W2, b2, W3, b3;
  int ld2;
};
__device__ __forceinline__ Net net_of(const float* f, int ld2, int n_out) {
  const gfp g = (gfp)f;
  return Net{g + kPW1, g + kPB1, g + kPW2, g + pB2(ld2), g + pW3(ld2), g + pB3(ld2, n_out), ld2};
}

// Re-derive a net's bases (and the lane id) inside a sub-tile loop: without
// this LICM hoists every per-lane load address out of the loop and spills
// them (the same trap as sk_update.hip's fragment loads)
__device__ __forceinline__ const float* launder(const float* base) {
  asm volatile("" : "+s"(base));  // one SGPR pair per net; the parameter offsets are immediates
  return base;
}
__device__ __forceinline__ int launder_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

__device__ __forceinline__ int drow(int v, int lane) { return 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3); }

__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u, p1 = (uint64_t)c.z * 0xCD9E8D57u;  // v_mad_u64_u32
    c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                   __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Phase timestamps of the first and last workgroup (diagnostic builds only:
// -DSK_TRACE32, read back with sk_debug_trace32; tools/trace_learn32.py)
#ifdef SK_TRACE32
__device__ unsigned long long g_sk_trace32[2][32][2];
#define TP32(k)                                                                              \
  do {                                                                                       \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1)) {              \
      const int wg_ = blockIdx.x == 0 ? 0 : 1;                                               \
      g_sk_trace32[wg_][k][0] = __builtin_amdgcn_s_memtime();                                \
      g_sk_trace32[wg_][k][1] = wall_clock64();                                              \
    }                                                                                        \
  } while (0)
#else
#define TP32(k) \
  do {          \
  } while (0)
#endif

// ------------------------------------------------------------------ the acting tile's GEMMs
// fp32 products from bf16 pieces (sk_split.hpp): D[i][n] += sum_k X[i][k]
// W[n][k] as six v_mfma_f32_32x32x16_bf16 per 16 k — the small piece
// products first, the hi x hi last — into one fp32 accumulator; the
// variance GEMM of parameter noise (x^2 W^2, which only scales the noise) is
// one more on bf16 squares.  A = the activations, row-major bf16 planes in
// LDS (hi, mid, lo, square: `xp` elements apart), lane (r, h) reading row r,
// k = 16 kk + 8 h + 0..7 (16 bytes); B = the weights' split pack in global
// memory (fragment order, planes `wp` elements apart), one 16-byte load per
// lane and k-step.  D register v of lane l is D[8(v/4) + 4(l/32) + v%4][l%32],
// the layout of the f32 MFMA these replace: every epilogue is unchanged.
typedef const __attribute__((address_space(1))) skmlp::bf16x8* gbf8;
using skmlp::bf16x8;
__device__ __forceinline__ f32x16 mfb(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mf6(const bf16x8 x[3], const bf16x8 w[3], f32x16 m) {
  m = mfb(x[2], w[0], m);
  m = mfb(x[0], w[2], m);
  m = mfb(x[1], w[1], m);
  m = mfb(x[1], w[0], m);
  m = mfb(x[0], w[1], m);
  return mfb(x[0], w[0], m);
}
// kk k-steps of the tile: X rows at X (row stride ldx elements), W fragments
// of n-tile `frag0` (kk-th at frag0 + 64 kk lanes); VAR adds the variance GEMM
template <int KK, bool VAR>
__device__ __forceinline__ void gemm6(f32x16& m, f32x16& v, const short* X, int ldx, int xp, gbf8 W, int wp,
                                      int lane) {
  const int i = lane & 31, h = lane >> 5;
  const short* xr = X + i * ldx + 8 * h;
  gbf8 wr = W + lane;
  constexpr int NP = VAR ? 4 : 3;
  bf16x8 wn[2][NP];  // two k-steps of weight fragments in flight
#pragma unroll
  for (int d = 0; d < 2 && d < KK; ++d)
#pragma unroll
    for (int q = 0; q < NP; ++q) wn[d][q] = wr[(size_t)q * (wp / 8) + 64 * d];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    bf16x8 wc[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) wc[q] = wn[kk & 1][q];
    if (kk + 2 < KK) {
#pragma unroll
      for (int q = 0; q < NP; ++q) wn[kk & 1][q] = wr[(size_t)q * (wp / 8) + 64 * (kk + 2)];
    }
    bf16x8 x[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) x[q] = *(const bf16x8*)(xr + q * xp + 16 * kk);
    m = mf6(x, wc, m);
    if (VAR) v = mfb(x[3], wc[3], v);
  }
}

// ================================================================ gradient kernels
// 16-row sub-tiles on v_mfma_f32_16x16x4_f32 (the fp32 MFMA rate is the
// bound: a 16-row sub-tile per workgroup spreads a minibatch over twice the
// CUs of 32-row tiles).  Lane l = (i = l % 16, g = l / 16): A[i][k = g],
// B[k = g][i], D register r = D[4g + r][i] (4 consecutive rows of column i).
// The float4 trick of the 32x32 GEMMs: lane (i, g) loads k0 + 4g .. + 3 and
// MFMA t contracts {k0 + t, k0 + 4 + t, k0 + 8 + t, k0 + 12 + t}.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kR = 16;                         // rows per sub-tile
constexpr int kLdS16 = 20, kLdT16 = 20;        // [16][20] states; transposed [unit][16 rows (+4)]

__device__ __forceinline__ f32x4 m16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 m16x4(f4 a, f4 b, f32x4 c) {
  c = m16(a.x, b.x, c);
  c = m16(a.y, b.y, c);
  c = m16(a.z, b.z, c);
  return m16(a.w, b.w, c);
}

// layer 1 (K = 12): k 0..11 by lane groups 0-2 (group 3's 12..15 are zero
// operands: S is zero-padded, W1 is not read)
__device__ __forceinline__ f32x4 g16_l1(const float* S, gfp W1, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const f4 x = *(const f4*)(S + i * kLdS16 + 4 * g);
  f4 w = {0.f, 0.f, 0.f, 0.f};
  if (g < 3) w = *(gf4u)(W1 + (n0 + i) * kIn + 4 * g);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  return m16x4(x, w, acc);
}
// D[row][n0 + j] = sum_k X[row][k] W[n0 + j][k] over the 256 inputs (X in
// LDS [16][ldx], W global row-major), for one net (a) or two nets' chains
// interleaved (b); the weight loads of the next 4 steps are in flight
__device__ __forceinline__ f32x4 g16_xwT256(const float* X, int ldx, gfp W, int ldw, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const float* xr = X + i * ldx + 4 * g;
  const gfp wr = W + (size_t)(n0 + i) * ldw + 4 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f4 wn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + 16 * t);
#pragma unroll
  for (int k = 0; k < 256; k += 64) {
    f4 wc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wc[t] = wn[t];
    if (k + 64 < 256) {
#pragma unroll
      for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + k + 64 + 16 * t);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = m16x4(*(const f4*)(xr + k + 16 * t), wc[t], acc);
  }
  return acc;
}
__device__ __forceinline__ void g16_xwT256x2(f32x4& a0, f32x4& a1, const float* X0, gfp W0, int ldw0, const float* X1,
                                             gfp W1, int ldw1, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const float* x0 = X0 + i * kLdH1 + 4 * g;
  const float* x1 = X1 + i * kLdH1 + 4 * g;
  const gfp w0 = W0 + (size_t)(n0 + i) * ldw0 + 4 * g;
  const gfp w1 = W1 + (size_t)(n0 + i) * ldw1 + 4 * g;
  a0 = f32x4{0.f, 0.f, 0.f, 0.f};
  a1 = f32x4{0.f, 0.f, 0.f, 0.f};
  f4 n0w[2], n1w[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    n0w[t] = *(gf4u)(w0 + 16 * t);
    n1w[t] = *(gf4u)(w1 + 16 * t);
  }
#pragma unroll
  for (int k = 0; k < 256; k += 32) {
    f4 c0[2], c1[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      c0[t] = n0w[t];
      c1[t] = n1w[t];
    }
    if (k + 32 < 256) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        n0w[t] = *(gf4u)(w0 + k + 32 + 16 * t);
        n1w[t] = *(gf4u)(w1 + k + 32 + 16 * t);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a0 = m16x4(*(const f4*)(x0 + k + 16 * t), c0[t], a0);
      a1 = m16x4(*(const f4*)(x1 + k + 16 * t), c1[t], a1);
    }
  }
}
// D[row][n0 + j] = sum_{u < 128} DZ[row][u] W[u][n0 + j]: DZ in LDS [16][ldz],
// W global row-major read down its columns (16 lanes: 64 contiguous bytes)
__device__ __forceinline__ f32x4 g16_xw128(const float* DZ, int ldz, gfp W, int ldw, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const float* zr = DZ + i * ldz + 4 * g;
  const gfp wc = W + (size_t)(4 * g) * ldw + n0 + i;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f4 bn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    bn[t] = f4{wc[(16 * t + 0) * ldw], wc[(16 * t + 1) * ldw], wc[(16 * t + 2) * ldw], wc[(16 * t + 3) * ldw]};
#pragma unroll
  for (int k = 0; k < 128; k += 64) {
    f4 bc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) bc[t] = bn[t];
    if (k + 64 < 128) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = k + 64 + 16 * t;
        bn[t] = f4{wc[(r + 0) * ldw], wc[(r + 1) * ldw], wc[(r + 2) * ldw], wc[(r + 3) * ldw]};
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = m16x4(*(const f4*)(zr + k + 16 * t), bc[t], acc);
  }
  return acc;
}
// weight gradient of one 16 x 16 tile over the sub-tile's 16 rows: acc[m][n]
// += sum_row AT[m0 + m][row] BT[n0 + n][row] (both transposed in LDS)
__device__ __forceinline__ f32x4 g16_wgrad(f32x4 acc, const float* AT, int m0, const float* BT, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  return m16x4(*(const f4*)(AT + (m0 + i) * kLdT16 + 4 * g), *(const f4*)(BT + (n0 + i) * kLdT16 + 4 * g), acc);
}

// inclusive prefix sum over the 16 lanes of a DPP row (row_shr 1, 2, 4, 8,
// zero fill): lane 15 of each row holds the row's total
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float rowsum16(float v) {
  v += dpp_f<0x111>(v);
  v += dpp_f<0x112>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  return v;
}

// LDS-only workgroup barrier (outstanding global loads stay in flight)
__device__ __forceinline__ void lds_sync32() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// fp32 tails of a net staged in LDS (1024 floats, the bf16 grad-pack tail
// layout): b1 [256], b2 [128], critic action columns W2[u][256 + j] as [128][2],
// W3 [n_out][128], b3
constexpr int kT1 = 0, kT2 = 256, kTA = 384, kT3 = 640, kTB = 896;
// One load per element from an index chosen by selects: a load per branch
// put each element's candidate loads in one VGPR, and the write-after-write
// between them cost an s_waitcnt vmcnt(0) -- a full round trip of every load
// in flight -- per branch a wave took (profiles/r04ao_trace_slice_bwd.jsonl).
__device__ __forceinline__ float tail_src(gfp f, int ld2, int n_out, int e) {
  const int ea = e - kTA, e3 = e - kT3, eb = e - kTB;
  int idx = e < kT2 ? kPB1 + e : pB2(ld2) + e - kT2;
  // (a 24-bit product: the 32-bit one became a v_mad_u64_u32 whose unused
  // high addend half was a register with a load in flight)
  idx = e < kTA ? idx : kPW2 + (int)__umul24((unsigned)ea >> 1, (unsigned)ld2) + kH1 + (ea & 1);
  idx = e < kT3 ? idx : pW3(ld2) + e3;
  idx = e < kTB ? idx : pB3(ld2, n_out) + eb;
  const bool ok = e < kTA || (e < kT3 ? ld2 != kH1 : e < kTB ? e3 < n_out * kH2 : eb < n_out);
  const float v = f[ok ? idx : 0];
  return ok ? v : 0.f;
}

struct G32 {
  float *S, *S2, *ST, *H1, *H1a, *H1c, *H1T, *DZ2, *DZ2T, *DZ1T, *TL, *A, *R, *D, *Y, *QP, *MP, *YP, *DP, *RED;
};
constexpr int kG32Floats = 3 * kR * kLdS16 + 3 * kR * kLdH1 + kH1 * kLdT16 + kR * kLdH2 + kH2 * kLdT16 +
                           kH1 * kLdT16 + 3 * 1024 + 32 + 16 + 16 + 16 + 8 * 16 + 8 * 32 + 8 * 16 + 8 * 32 + 4;
constexpr size_t kLdsGrad32 = (size_t)kG32Floats * 4;
static_assert(kLdsGrad32 <= 160 * 1024, "LDS budget of one CU");
__device__ __forceinline__ G32 carve32(float* p) {
  G32 L;
  L.S = p;    p += kR * kLdS16;
  L.S2 = p;   p += kR * kLdS16;
  L.ST = p;   p += kR * kLdS16;
  L.H1 = p;   p += kR * kLdH1;
  L.H1a = p;  p += kR * kLdH1;
  L.H1c = p;  p += kR * kLdH1;
  L.H1T = p;  p += kH1 * kLdT16;
  L.DZ2 = p;  p += kR * kLdH2;
  L.DZ2T = p; p += kH2 * kLdT16;
  L.DZ1T = p; p += kH1 * kLdT16;
  L.TL = p;   p += 3 * 1024;
  L.A = p;    p += 32;
  L.R = p;    p += 16;
  L.D = p;    p += 16;
  L.Y = p;    p += 16;
  L.QP = p;   p += 8 * 16;  // per-wave partial row sums: [wave][row]
  L.MP = p;   p += 8 * 32;  //                             [wave][row][2]
  L.YP = p;   p += 8 * 16;
  L.DP = p;   p += 8 * 32;
  L.RED = p;
  return L;
}
// Dropout keep bits of n-tiles w and w + 8 (16 units each): bit 4j + r is
// row 4g + r of the sub-tile, unit 16 (w + 8j) + i (rng.dropout_keep: the mask
// of global row key + row, Philox word row % 4 of counter (row / 4, unit))
__device__ __forceinline__ uint32_t dropout_bits16(uint64_t seed, uint64_t call, int64_t key, int w, int lane) {
  const int i = lane & 15, g = lane >> 4;
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint4 u = philox(make_uint4((uint32_t)((key + 4 * g) >> 2), (uint32_t)(16 * (w + 8 * j) + i), (uint32_t)call,
                                      (uint32_t)(call >> 32)),
                           (uint32_t)seed, (uint32_t)(seed >> 32));
    bits |= ((uint32_t)(u.x >= 858993460u) | ((uint32_t)(u.y >= 858993460u) << 1) |
             ((uint32_t)(u.z >= 858993460u) << 2) | ((uint32_t)(u.w >= 858993460u) << 3)) << (4 * j);
  }
  return bits;
}
// layer-1 epilogue of n-tile nt: relu(acc + b1) (x Dropout keep bits) ->
// H [row][unit] and, if HT, HT [unit][rows] (one 16-byte write)
__device__ __forceinline__ void l1_out(f32x4 acc, const float* tl, int nt, int lane, float* H, float* HT, bool drop,
                                       uint32_t bits4) {
  const int i = lane & 15, g = lane >> 4, n = 16 * nt + i;
  const float b = tl[kT1 + n];
  f4 z;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = fmaxf(acc[r] + b, 0.f);
    if (drop) v = (bits4 >> r) & 1u ? v * 1.25f : 0.f;
    z[r] = v;
    H[(4 * g + r) * kLdH1 + n] = v;
  }
  if (HT) *(f4*)(HT + n * kLdT16 + 4 * g) = z;
}

// ---------------------------------------------------------------- critic step
// Critic.forward in training mode + MSE backward (critic.fit,
// SkillshotLearner.py:434; DDPG.critic_step): dL/dq = grad_scale (q - y),
// grad_scale = 2 / global batch; Dropout keep-mask of global row key_row0 +
// row (rng.dropout_keep), keep -> x 1.25.  BOOT: y = r + gamma (1 - done)
// Q'(s', mu'(s')) from the target nets, in the same phases (wave w: layer-2
// unit tile w, layer-1 / dz1 tiles w and w + 8):
//   0  stage s, a (s', r, done), the nets' tails; Dropout bits meanwhile
//   1  layer 1 of the critic (Dropout), the target actor, the target critic
//   2  layer 2 of the critic and of the target actor (chains interleaved);
//      per-wave partial row sums of q and mu'
//   3  mu'(s') from the partials; the target critic's layer 2 -> Q' partials
//   4  y, dL/dq per row; dz2 of the wave's units
//   5  dW2 (16 tiles per wave), dz1;  6  dW1
template <bool BOOT>
__global__ void __launch_bounds__(kThreads) k_critic_grad32(
    const float* __restrict__ cflat, const float* __restrict__ Sg, const float* __restrict__ Ag,
    const float* __restrict__ Yg, int64_t B, int64_t key_row0, int sub_per_wg, float grad_scale, uint64_t seed,
    const int64_t* __restrict__ call_ctr, float* __restrict__ partial, float* step_ctr, int n_steps,
    float* __restrict__ loss_out, uint8_t* __restrict__ mask_out, const float* __restrict__ S2g,
    const float* __restrict__ Rg, const float* __restrict__ Dg, float gamma, const float* __restrict__ taflat,
    const float* __restrict__ tcflat) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  const G32 L = carve32(smem32);
  TP32(0);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t call = (uint64_t)*call_ctr;
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  const float* TLc = L.TL;
  const float* TLa = L.TL + 1024;
  const float* TLt = L.TL + 2048;
  f32x4 gW2[16], gW1[2];
#pragma unroll
  for (int t = 0; t < 16; ++t) gW2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  gW1[0] = gW1[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per-lane partial sums: b1 of units 16(w + 8j) + i, b2 / W2 action
  // columns / W3 of unit 16w + i (over the lane's rows), db3 and the loss
  float gb1[2] = {0.f, 0.f}, gb2 = 0.f, gwa0 = 0.f, gwa1 = 0.f, gw3 = 0.f, gb3 = 0.f, lsum = 0.f;
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * kR;
    if (row0 >= B) break;  // uniform across the workgroup
    const int tid = launder_lane(threadIdx.x), lane = tid & 63, i = lane & 15, g = lane >> 4;
    const int u = 16 * w + i;  // the lane's layer-2 unit
    const Net C = net_of(launder(cflat), kCLd, 1);
    // ---- phase 0: every global load, the Dropout bits while they fly, then LDS
    const int si = (tid & 255) >> 4, sk = tid & 15;
    const float* src = tid < 256 ? Sg : S2g;
    const bool want_s = tid < 256 || BOOT;
    const float sv = want_s && sk < kIn && row0 + si < B ? src[(row0 + si) * kIn + sk] : 0.f;
    const float av = tid < 32 && row0 + (tid >> 1) < B ? Ag[row0 * 2 + tid] : 0.f;
    const bool rok = tid < kR && row0 + tid < B;
    const float rv = rok ? (BOOT ? Rg[row0 + tid] : Yg[row0 + tid]) : 0.f;
    const float dv = BOOT && rok ? Dg[row0 + tid] : 0.f;
    float tv[6];
    if (sub == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const int net = k >> 1, e = tid + kThreads * (k & 1);
        tv[k] = net == 0 ? tail_src(C.W1, kCLd, 1, e)
                         : (BOOT ? (net == 1 ? tail_src((gfp)launder(taflat), kALd, 2, e)
                                             : tail_src((gfp)launder(tcflat), kCLd, 1, e))
                                 : 0.f);
      }
    }
    uint32_t keep = dropout_bits16(seed, call, key_row0 + row0, w, lane);
    asm volatile("" : "+v"(keep));  // computed here, under the loads' latency
    if (mask_out) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row0 + 4 * g + r < B) mask_out[(row0 + 4 * g + r) * kH1 + 16 * (w + 8 * j) + i] = (keep >> (4 * j + r)) & 1u;
    }
    if (tid < 256) {
      L.S[si * kLdS16 + sk] = sv;
      L.ST[sk * kLdT16 + si] = sv;  // feature rows 12..15 get zeros
    } else if (BOOT) {
      L.S2[si * kLdS16 + sk] = sv;
    }
    if (tid < 32) L.A[tid] = av;
    if (tid < kR) {
      if (BOOT) {
        L.R[tid] = rv;
        L.D[tid] = dv;
      } else {
        L.Y[tid] = rv;
      }
    }
    if (sub == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (k < 2 || BOOT) L.TL[(k >> 1) * 1024 + tid + kThreads * (k & 1)] = tv[k];
    }
    lds_sync32();
    TP32(1);
    // ---- phase 1: layer 1, n-tiles w and w + 8, of the critic (Dropout), target actor, target critic
    const Net TA = net_of(launder(BOOT ? taflat : cflat), kALd, 2), TC = net_of(launder(BOOT ? tcflat : cflat), kCLd, 1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 8 * j;
      l1_out(g16_l1(L.S, C.W1, 16 * nt, lane), TLc, nt, lane, L.H1, L.H1T, true, keep >> (4 * j));
      if (BOOT) {
        l1_out(g16_l1(L.S2, TA.W1, 16 * nt, lane), TLa, nt, lane, L.H1a, nullptr, false, 0);
        l1_out(g16_l1(L.S2, TC.W1, 16 * nt, lane), TLt, nt, lane, L.H1c, nullptr, false, 0);
      }
    }
    lds_sync32();
    TP32(2);
    // ---- phase 2: critic h2 (registers) and per-wave q partials; target actor mu' partials
    float h2[4];
    {
      f32x4 acc, acca;
      if (BOOT) g16_xwT256x2(acc, acca, L.H1, C.W2, kCLd, L.H1a, TA.W2, kALd, 16 * w, lane);
      else acc = g16_xwT256(L.H1, kLdH1, C.W2, kCLd, 16 * w, lane);
      const float b2 = TLc[kT2 + u], wa0 = TLc[kTA + 2 * u], wa1 = TLc[kTA + 2 * u + 1], w3 = TLc[kT3 + u];
      const f4 a01 = *(const f4*)(L.A + 8 * g), a23 = *(const f4*)(L.A + 8 * g + 4);  // a[4g + r][0..1]
      const float a0[4] = {a01.x, a01.z, a23.x, a23.z}, a1[4] = {a01.y, a01.w, a23.y, a23.w};
      f4 qp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h2[r] = fmaxf(acc[r] + b2 + a0[r] * wa0 + a1[r] * wa1, 0.f);
        qp[r] = rowsum16(h2[r] * w3);
      }
      if (i == 15) *(f4*)(L.QP + 16 * w + 4 * g) = qp;
      if (BOOT) {
        const float b2a = TLa[kT2 + u], w30 = TLa[kT3 + u], w31 = TLa[kT3 + kH2 + u];
        f4 m0, m1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float h = fmaxf(acca[r] + b2a, 0.f);
          m0[r] = rowsum16(h * w30);
          m1[r] = rowsum16(h * w31);
        }
        if (i == 15) {
          *(f4*)(L.MP + 32 * w + 8 * g) = f4{m0.x, m1.x, m0.y, m1.y};
          *(f4*)(L.MP + 32 * w + 8 * g + 4) = f4{m0.z, m1.z, m0.w, m1.w};
        }
      }
    }
    lds_sync32();
    TP32(3);
    // ---- phase 3 (BOOT): mu'(s') of the lane's rows, the target critic's layer 2 -> Q' partials
    if (BOOT) {
      f4 s01 = {0.f, 0.f, 0.f, 0.f}, s23 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        s01 += *(const f4*)(L.MP + 32 * v + 8 * g);
        s23 += *(const f4*)(L.MP + 32 * v + 8 * g + 4);
      }
      const float ap0[4] = {tanhf(s01.x + TLa[kTB]), tanhf(s01.z + TLa[kTB]), tanhf(s23.x + TLa[kTB]),
                            tanhf(s23.z + TLa[kTB])};
      const float ap1[4] = {tanhf(s01.y + TLa[kTB + 1]), tanhf(s01.w + TLa[kTB + 1]), tanhf(s23.y + TLa[kTB + 1]),
                            tanhf(s23.w + TLa[kTB + 1])};
      const f32x4 acc = g16_xwT256(L.H1c, kLdH1, TC.W2, kCLd, 16 * w, lane);
      const float b2 = TLt[kT2 + u], wa0 = TLt[kTA + 2 * u], wa1 = TLt[kTA + 2 * u + 1], w3 = TLt[kT3 + u];
      f4 yp;
#pragma unroll
      for (int r = 0; r < 4; ++r) yp[r] = rowsum16(fmaxf(acc[r] + b2 + ap0[r] * wa0 + ap1[r] * wa1, 0.f) * w3);
      if (i == 15) *(f4*)(L.YP + 16 * w + 4 * g) = yp;
      lds_sync32();
    }
    TP32(4);
    // ---- phase 4: y and dL/dq of the lane's rows; dz2 = dL/dq W3 relu'(h2) of unit u
    {
      f4 q = {TLc[kTB], TLc[kTB], TLc[kTB], TLc[kTB]}, yq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        q += *(const f4*)(L.QP + 16 * v + 4 * g);
        if (BOOT) yq += *(const f4*)(L.YP + 16 * v + 4 * g);
      }
      const f4 rr = *(const f4*)((BOOT ? L.R : L.Y) + 4 * g);
      const f4 dd = BOOT ? *(const f4*)(L.D + 4 * g) : f4{0.f, 0.f, 0.f, 0.f};
      const float w3 = TLc[kT3 + u];
      const f4 a01 = *(const f4*)(L.A + 8 * g), a23 = *(const f4*)(L.A + 8 * g + 4);
      const float a0[4] = {a01.x, a01.z, a23.x, a23.z}, a1[4] = {a01.y, a01.w, a23.y, a23.w};
      f4 dz;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float y = BOOT ? rr[r] + gamma * (1.f - dd[r]) * (TLt[kTB] + yq[r]) : rr[r];
        const float e = row0 + 4 * g + r < B ? q[r] - y : 0.f;
        const float dq = grad_scale * e;
        if (w == 0 && i == 0) {
          gb3 += dq;
          lsum += e * e;
        }
        const float d = h2[r] > 0.f ? dq * w3 : 0.f;
        dz[r] = d;
        L.DZ2[(4 * g + r) * kLdH2 + u] = d;
        gb2 += d;
        gwa0 += d * a0[r];
        gwa1 += d * a1[r];
        gw3 += dq * h2[r];
      }
      *(f4*)(L.DZ2T + u * kLdT16 + 4 * g) = dz;
    }
    lds_sync32();
    TP32(5);
    // ---- phase 5: dW2 (unit tile w x 16 input tiles), dz1 of n-tiles w, w + 8
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) gW2[kt] = g16_wgrad(gW2[kt], L.DZ2T, 16 * w, L.H1T, 16 * kt, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 16 * (w + 8 * j) + i;
      const f32x4 acc = g16_xw128(L.DZ2, kLdH2, C.W2, kCLd, 16 * (w + 8 * j), lane);
      f4 d;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        d[r] = L.H1[(4 * g + r) * kLdH1 + n] > 0.f ? acc[r] * 1.25f : 0.f;
        gb1[j] += d[r];
      }
      *(f4*)(L.DZ1T + n * kLdT16 + 4 * g) = d;
    }
    lds_sync32();
    TP32(6);
    // ---- phase 6: dW1 of unit tiles w, w + 8 (input columns 12..15 discarded)
#pragma unroll
    for (int j = 0; j < 2; ++j) gW1[j] = g16_wgrad(gW1[j], L.DZ1T, 16 * (w + 8 * j), L.ST, 0, lane);
    lds_sync32();  // the next sub-tile restages
    TP32(7);
  }
  // ---- this workgroup's partial gradient (sk_partial.hpp layout)
  float* P = partial + (int64_t)blockIdx.x * kCP;
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4, u = 16 * w + i;
#pragma unroll
  for (int kt = 0; kt < 16; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) P[skpart::critic_w2_main(16 * w + 4 * g + r, 16 * kt + i)] = gW2[kt][r];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (i < kIn) {
#pragma unroll
      for (int r = 0; r < 4; ++r) P[kPW1 + (16 * (w + 8 * j) + 4 * g + r) * kIn + i] = gW1[j][r];
    }
    float b = gb1[j] + __shfl_xor(gb1[j], 16, 64);
    b += __shfl_xor(b, 32, 64);
    if (g == 0) P[kPB1 + 16 * (w + 8 * j) + i] = b;
  }
  TP32(8);
  gb2 += __shfl_xor(gb2, 16, 64);
  gb2 += __shfl_xor(gb2, 32, 64);
  gwa0 += __shfl_xor(gwa0, 16, 64);
  gwa0 += __shfl_xor(gwa0, 32, 64);
  gwa1 += __shfl_xor(gwa1, 16, 64);
  gwa1 += __shfl_xor(gwa1, 32, 64);
  gw3 += __shfl_xor(gw3, 16, 64);
  gw3 += __shfl_xor(gw3, 32, 64);
  if (g == 0) {
    P[pB2(kCLd) + u] = gb2;
    P[skpart::critic_w2_action(u, 0)] = gwa0;
    P[skpart::critic_w2_action(u, 1)] = gwa1;
    P[pW3(kCLd) + u] = gw3;
  }
  if (w == 0 && i == 0) {  // wave 0, one lane per row group: db3 and loss partials
    atomicAdd(&L.RED[0], gb3);
    atomicAdd(&L.RED[1], lsum);
  }
  lds_sync32();
  if (threadIdx.x == 0) {
    P[pB3(kCLd, 1)] = L.RED[0];
    if (loss_out) atomicAdd(loss_out, L.RED[1]);
  }
  TP32(9);
}

// ---------------------------------------------------------------- actor step
// model_actor_fit_step (SkillshotLearner.py:386-417): gradient of
// -loss_scale * sum_b Q(s_b, mu(s_b)) w.r.t. the actor, critic at inference.
//   0  stage s, the nets' tails
//   1  layer 1 of the actor (-> H1, H1T) and of the critic (-> H1c)
//   2  the actor's layer 2 (-> h2 registers, mu partials) and the critic's
//      layer-2 MFMA (held; its action columns join in phase 3), interleaved
//   3  mu per row; critic z2 at (s, mu): dQ/da and Q partials
//   4  dL/dz3 = -loss_scale dQ/da (1 - a^2) per row; dz2 of unit 16w + i
//   5  dW2, dz1;  6  dW1
__global__ void __launch_bounds__(kThreads) k_actor_grad32(const float* __restrict__ aflat,
                                                           const float* __restrict__ cflat,
                                                           const float* __restrict__ Sg, int64_t B, int sub_per_wg,
                                                           float loss_scale, float* __restrict__ partial,
                                                           float* step_ctr, int n_steps, float* __restrict__ q_out) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  const G32 L = carve32(smem32);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;
  const float* TLa = L.TL;
  const float* TLc = L.TL + 1024;
  f32x4 gW2[16], gW1[2];
#pragma unroll
  for (int t = 0; t < 16; ++t) gW2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  gW1[0] = gW1[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gb1[2] = {0.f, 0.f}, gb2 = 0.f, gw30 = 0.f, gw31 = 0.f, gb30 = 0.f, gb31 = 0.f, qsum = 0.f;
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * kR;
    if (row0 >= B) break;
    const int tid = launder_lane(threadIdx.x), lane = tid & 63, i = lane & 15, g = lane >> 4;
    const int u = 16 * w + i;
    const Net A = net_of(launder(aflat), kALd, 2), C = net_of(launder(cflat), kCLd, 1);
    // ---- phase 0
    const int si = tid >> 4, sk = tid & 15;
    const float sv = tid < 256 && sk < kIn && row0 + si < B ? Sg[(row0 + si) * kIn + sk] : 0.f;
    float tv[4];
    if (sub == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid + kThreads * (k & 1);
        tv[k] = k < 2 ? tail_src(A.W1, kALd, 2, e) : tail_src(C.W1, kCLd, 1, e);
      }
    }
    if (tid < 256) {
      L.S[si * kLdS16 + sk] = sv;
      L.ST[sk * kLdT16 + si] = sv;
    }
    if (sub == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) L.TL[(k >> 1) * 1024 + tid + kThreads * (k & 1)] = tv[k];
    }
    lds_sync32();
    // ---- phase 1
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 8 * j;
      l1_out(g16_l1(L.S, A.W1, 16 * nt, lane), TLa, nt, lane, L.H1, L.H1T, false, 0);
      l1_out(g16_l1(L.S, C.W1, 16 * nt, lane), TLc, nt, lane, L.H1c, nullptr, false, 0);
    }
    lds_sync32();
    // ---- phase 2
    float h2[4];
    f32x4 zc;
    {
      f32x4 acc;
      g16_xwT256x2(acc, zc, L.H1, A.W2, kALd, L.H1c, C.W2, kCLd, 16 * w, lane);
      const float b2 = TLa[kT2 + u], w30 = TLa[kT3 + u], w31 = TLa[kT3 + kH2 + u];
      f4 m0, m1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h2[r] = fmaxf(acc[r] + b2, 0.f);
        m0[r] = rowsum16(h2[r] * w30);
        m1[r] = rowsum16(h2[r] * w31);
      }
      if (i == 15) {
        *(f4*)(L.MP + 32 * w + 8 * g) = f4{m0.x, m1.x, m0.y, m1.y};
        *(f4*)(L.MP + 32 * w + 8 * g + 4) = f4{m0.z, m1.z, m0.w, m1.w};
      }
    }
    lds_sync32();
    // ---- phase 3: mu of the lane's rows; the critic at (s, mu)
    float a0[4], a1[4];
    {
      f4 s01 = {0.f, 0.f, 0.f, 0.f}, s23 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        s01 += *(const f4*)(L.MP + 32 * v + 8 * g);
        s23 += *(const f4*)(L.MP + 32 * v + 8 * g + 4);
      }
      a0[0] = tanhf(s01.x + TLa[kTB]);
      a1[0] = tanhf(s01.y + TLa[kTB + 1]);
      a0[1] = tanhf(s01.z + TLa[kTB]);
      a1[1] = tanhf(s01.w + TLa[kTB + 1]);
      a0[2] = tanhf(s23.x + TLa[kTB]);
      a1[2] = tanhf(s23.y + TLa[kTB + 1]);
      a0[3] = tanhf(s23.z + TLa[kTB]);
      a1[3] = tanhf(s23.w + TLa[kTB + 1]);
      const float b2 = TLc[kT2 + u], wa0 = TLc[kTA + 2 * u], wa1 = TLc[kTA + 2 * u + 1], w3 = TLc[kT3 + u];
      f4 d0, d1, qp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = zc[r] + b2 + a0[r] * wa0 + a1[r] * wa1;
        const float dqdz = (z > 0.f && row0 + 4 * g + r < B) ? w3 : 0.f;  // dQ/dz2 (rows beyond B: 0)
        d0[r] = rowsum16(dqdz * wa0);
        d1[r] = rowsum16(dqdz * wa1);
        qp[r] = rowsum16(fmaxf(z, 0.f) * w3);
      }
      if (i == 15) {
        *(f4*)(L.DP + 32 * w + 8 * g) = f4{d0.x, d1.x, d0.y, d1.y};
        *(f4*)(L.DP + 32 * w + 8 * g + 4) = f4{d0.z, d1.z, d0.w, d1.w};
        *(f4*)(L.QP + 16 * w + 4 * g) = qp;
      }
    }
    lds_sync32();
    // ---- phase 4: dL/dz3 of the lane's rows, dz2 = (dz3 W3) relu'(h2) of unit u
    {
      f4 s01 = {0.f, 0.f, 0.f, 0.f}, s23 = {0.f, 0.f, 0.f, 0.f}, qs = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        s01 += *(const f4*)(L.DP + 32 * v + 8 * g);
        s23 += *(const f4*)(L.DP + 32 * v + 8 * g + 4);
        qs += *(const f4*)(L.QP + 16 * v + 4 * g);
      }
      const float da0[4] = {s01.x, s01.z, s23.x, s23.z}, da1[4] = {s01.y, s01.w, s23.y, s23.w};
      const float w30 = TLa[kT3 + u], w31 = TLa[kT3 + kH2 + u];
      f4 dz;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z0 = -loss_scale * da0[r] * (1.f - a0[r] * a0[r]);
        const float z1 = -loss_scale * da1[r] * (1.f - a1[r] * a1[r]);
        if (w == 0 && i == 0) {
          gb30 += z0;
          gb31 += z1;
          if (row0 + 4 * g + r < B) qsum += TLc[kTB] + qs[r];
        }
        const float d = h2[r] > 0.f ? z0 * w30 + z1 * w31 : 0.f;
        dz[r] = d;
        L.DZ2[(4 * g + r) * kLdH2 + u] = d;
        gb2 += d;
        gw30 += z0 * h2[r];
        gw31 += z1 * h2[r];
      }
      *(f4*)(L.DZ2T + u * kLdT16 + 4 * g) = dz;
    }
    lds_sync32();
    // ---- phase 5
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) gW2[kt] = g16_wgrad(gW2[kt], L.DZ2T, 16 * w, L.H1T, 16 * kt, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 16 * (w + 8 * j) + i;
      const f32x4 acc = g16_xw128(L.DZ2, kLdH2, A.W2, kALd, 16 * (w + 8 * j), lane);
      f4 d;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        d[r] = L.H1[(4 * g + r) * kLdH1 + n] > 0.f ? acc[r] : 0.f;
        gb1[j] += d[r];
      }
      *(f4*)(L.DZ1T + n * kLdT16 + 4 * g) = d;
    }
    lds_sync32();
    // ---- phase 6
#pragma unroll
    for (int j = 0; j < 2; ++j) gW1[j] = g16_wgrad(gW1[j], L.DZ1T, 16 * (w + 8 * j), L.ST, 0, lane);
    lds_sync32();
  }
  float* P = partial + (int64_t)blockIdx.x * kAP;
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4, u = 16 * w + i;
#pragma unroll
  for (int kt = 0; kt < 16; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) P[kPW2 + (16 * w + 4 * g + r) * kALd + 16 * kt + i] = gW2[kt][r];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (i < kIn) {
#pragma unroll
      for (int r = 0; r < 4; ++r) P[kPW1 + (16 * (w + 8 * j) + 4 * g + r) * kIn + i] = gW1[j][r];
    }
    float b = gb1[j] + __shfl_xor(gb1[j], 16, 64);
    b += __shfl_xor(b, 32, 64);
    if (g == 0) P[kPB1 + 16 * (w + 8 * j) + i] = b;
  }
  gb2 += __shfl_xor(gb2, 16, 64);
  gb2 += __shfl_xor(gb2, 32, 64);
  gw30 += __shfl_xor(gw30, 16, 64);
  gw30 += __shfl_xor(gw30, 32, 64);
  gw31 += __shfl_xor(gw31, 16, 64);
  gw31 += __shfl_xor(gw31, 32, 64);
  if (g == 0) {
    P[pB2(kALd) + u] = gb2;
    P[pW3(kALd) + u] = gw30;
    P[pW3(kALd) + kH2 + u] = gw31;
  }
  if (w == 0 && i == 0) {
    atomicAdd(&L.RED[0], gb30);
    atomicAdd(&L.RED[1], gb31);
    atomicAdd(&L.RED[2], qsum);
  }
  lds_sync32();
  if (threadIdx.x < 2) P[pB3(kALd, 2) + threadIdx.x] = L.RED[threadIdx.x];
  if (threadIdx.x == 0 && q_out) atomicAdd(q_out, L.RED[2]);
}

// ================================================================ sliced gradient kernels
// Small minibatches.  The kernels above give a 256-row
// minibatch 16 workgroups (one per 16-row tile), each running the whole
// phase chain on one CU at two waves per SIMD: MFMA-rate bound on 16 of 256
// CUs.  The sliced schedule splits layer 2 over kSlices workgroups per row
// tile (16 units each: RT x 8 workgroups, 128 at batch 256), two launches per
// step:
//   fwd (rt, s)  layer 1 of every net the step reads (all 256 units; the
//                critic's Dropout), then the slice's 16 layer-2 units with K
//                split over the 4 waves -> pre-activations z2 (no b2, no
//                action columns) [rt][net][row][unit] in the scratch buffer
//   bwd (rt, s)  per row, from all 128 units of z2 (read back: 8 KB per net
//                and row tile): q, mu', Q', y, dL/dq (critic) or mu, dQ/da,
//                dL/dz3 (actor); then the slice's dz2, its dW2 rows and its
//                b2 / action-column / W3 gradients; and the slice's share of
//                dz1 = dz2_s W2_s (dz1 is linear in dz2, the relu' and
//                Dropout masks are elementwise) -> dW1 / db1 contributions
//                written to a second partial buffer [RT * kSlices][3328]
//                that k_adam_flat sums for W1 and b1.
// Every partial entry is written by exactly one workgroup.  Block b is row
// tile b / 8, slice b % 8: slice s always lands on XCD s, whose L2 then holds
// that slice's W2 rows for every row tile.
constexpr int kSlices = 8, kSliceU = kH2 / kSlices;  // 16 units per slice
constexpr int kSlThreads = 256;                       // 4 waves: one per SIMD
constexpr int kZPlane = kR * kH2;                     // one net's z2 of a row tile
// LDS layouts of the sliced kernels, laid out against the gfx950 bank rules
// (MI355X_MICROARCH.md §LDS; VERDICT r05: conflict cycles were 100 / 61 / 91 %
// of the LDS instructions of fwd<1> / bwd<1> / fwd<2>).  SK_SL_SWZ=0 restores
// the padded row-major layouts (A/B only); the arithmetic is the same either way.
// Every XOR below touches only bits 2-3 of the column (which 16-B slot of a
// fragment) and depends only on a lane's own row, so each lane computes its
// addresses once and the unrolled accesses differ by immediate offsets (a
// swizzle that mixed the unrolled indices in cost ~80 VALU per wave).
//   [16][16] tiles read as 16-B MFMA fragments (lane (i, g): row i, floats
//     4g..4g+3; ds_read_b128 serves 16 lanes per cycle over 64 banks): rows of
//     16 floats, the slot XORed with (row >> 1) & 3 -- every lane group of the
//     fragment read and of the 8-lane ds_write_b128 of a transposed row covers
//     16 (8) distinct slots.  Also the [256][16] transposed layer 1.
//   [16][260] layer-1 outputs (written one float per lane, rows 4g + r, the
//     two 16-lane rows of a half 1,040 floats = 16 banks apart; read as
//     fragments, row i): the slot XORed with f(row >> 2), f = 0, 1, 1, 0, which
//     puts the four 4-row blocks of a ds_read_b128 lane group on disjoint slots.
//   [16][128 + 16] z2 planes: the row reductions read rows r and r + 1 in one
//     32-lane half, 16 banks apart.
//   the forward's K-split partials [wave][row][unit]: row r at 16 (r + r / 4),
//     so rows 4 apart (lanes g and g + 1 of one store) sit 16 banks apart.
#ifndef SK_SL_SWZ
#define SK_SL_SWZ 1
#endif
constexpr int kSlLdT = SK_SL_SWZ ? 16 : kLdT16;
constexpr int kSlLdH = kLdH1;
constexpr int kLdZ = SK_SL_SWZ ? kH2 + 16 : kH2 + 4;
constexpr int kSlRed = SK_SL_SWZ ? 20 * kSliceU : kR * kSliceU;  // floats per wave
__device__ __forceinline__ int sl_tmask(int row) { return SK_SL_SWZ ? ((row >> 1) & 3) << 2 : 0; }
__device__ __forceinline__ int sl_t16(int row, int col) { return row * kSlLdT + (col ^ sl_tmask(row)); }
__device__ __forceinline__ int sl_hmask(int row) { return SK_SL_SWZ ? (((row >> 2) ^ (row >> 3)) & 1) << 2 : 0; }
__device__ __forceinline__ int sl_red(int row, int j) { return (SK_SL_SWZ ? row + (row >> 2) : row) * kSliceU + j; }
constexpr int kW1Part = kPW2;                         // W1 + b1: floats per contribution row
enum { kSlCriticY = 0, kSlCriticBoot = 1, kSlActor = 2 };
__host__ __device__ constexpr int sl_planes(int mode) { return mode == kSlCriticBoot ? 3 : (mode == kSlActor ? 2 : 1); }
// net p of a step: critic modes 0 critic, 1 target actor, 2 target critic;
// actor mode 0 actor, 1 critic
__host__ __device__ constexpr int sl_ld(int mode, int p) {
  return (mode == kSlActor && p == 0) || (mode == kSlCriticBoot && p == 1) ? kALd : kCLd;
}
__host__ __device__ constexpr int sl_nout(int mode, int p) { return sl_ld(mode, p) == kALd ? 2 : 1; }
constexpr size_t sl_fwd_lds(int) { return (size_t)(kR * kSlLdT + kR * kSlLdH + kH1 + 4 * kSlRed) * 4; }
constexpr size_t sl_bwd_lds(int mode) {
  return (size_t)(2 * kR * kSlLdT + sl_planes(mode) * (kR * kLdZ + 1024) + kR * kSlLdH + kH1 * kSlLdT +
                  3 * kSliceU * kSlLdT + 32 + 2 * kR + 2 * kR + kR + 4) *
         4;
}
static_assert(sl_fwd_lds(kSlCriticBoot) <= 160 * 1024 && sl_bwd_lds(kSlCriticBoot) <= 160 * 1024, "LDS budget");

// layer-1 fragment of unit n0 + i (g16_l1 with the weights already loaded:
// the fragments are issued ahead of the staging barrier)
// p[i] where ok, else 0, as one unconditional load (of p[0] where !ok) and a
// select: a load under a branch put its value through a phi copy that the
// waitcnt pass guarded with a vmcnt(0), a round trip of every load in flight
__device__ __forceinline__ float ld_or0(const float* __restrict__ p, int64_t i, bool ok) {
  const float v = p[ok ? i : 0];
  return ok ? v : 0.f;
}

// (an unconditional load, zeroed by select where g = 3: the conditional load's
// phi cost the actor's backward a vmcnt(0) right after it)
__device__ __forceinline__ f4 w1_frag(gfp W1, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const f4 v = *(gf4u)(W1 + (n0 + i) * kIn + 4 * (g < 3 ? g : 0));
  const bool ok = g < 3;
  return f4{ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f};
}
__device__ __forceinline__ f32x4 g16_l1w(const float* S, f4 w, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  return m16x4(*(const f4*)(S + sl_t16(i, 4 * g)), w, z);
}
// (n = 16 nt + i: n's masks are i's)
// l1_out on the sliced layouts
__device__ __forceinline__ void l1_out_sl(f32x4 acc, const float* tl, int nt, int lane, float* H, float* HT, bool drop,
                                          uint32_t bits4) {
  const int i = lane & 15, g = lane >> 4, n = 16 * nt + i;
  const float b = tl[kT1 + n];
  f4 z;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float v = fmaxf(acc[r] + b, 0.f);
    if (drop) v = (bits4 >> r) & 1u ? v * 1.25f : 0.f;
    z[r] = v;
    H[(4 * g + r) * kSlLdH + 16 * nt + (i ^ sl_hmask(4 * g))] = v;
  }
  if (HT) *(f4*)(HT + n * kSlLdT + (4 * g ^ sl_tmask(i))) = z;
}
// g16_wgrad on the sliced layouts
__device__ __forceinline__ f32x4 g16_wgrad_sl(f32x4 acc, const float* AT, int m0, const float* BT, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int c = 4 * g ^ sl_tmask(i);  // m0, n0: multiples of 16
  return m16x4(*(const f4*)(AT + (m0 + i) * kSlLdT + c), *(const f4*)(BT + (n0 + i) * kSlLdT + c), acc);
}

// The replay minibatch gathered inside the critic's first launch
// (sk_critic_grad_f32_sampled): skmlp::RingSample / ring_row (sk_mlp.hpp).
// Each workgroup reads its own rows' states from the ring; the (slice 0, net
// 0) workgroup of every row tile also writes its 16 rows into the sample
// buffers, which the second launch and the actor step read.
using skmlp::RingSample;
using skmlp::ring_row;

template <int MODE>
__global__ void __launch_bounds__(kSlThreads) k_grad_slice_fwd(const float* __restrict__ f0, const float* __restrict__ f1,
                                                              const float* __restrict__ f2, const float* __restrict__ Sg,
                                                              const float* __restrict__ S2g, int64_t B,
                                                              int64_t key_row0, uint64_t seed,
                                                              const int64_t* __restrict__ call_ctr,
                                                              float* __restrict__ Z, float* step_ctr, int n_steps,
                                                              RingSample rs) {
  constexpr int NP = sl_planes(MODE);
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  float* sS = smem_sl;              // [16][16] (sl_t16)
  float* sH = sS + kR * kSlLdT;     // [16][260] layer-1 outputs (sl_hmask)
  float* sB1 = sH + kR * kSlLdH;    // [256]
  float* sRed = sB1 + kH1;          // [4 waves][16 rows][16 units] K-split partials (sl_red)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  // block = (row tile, net, slice), slice fastest
  const int b = blockIdx.x, s = b % kSlices, p = (b / kSlices) % NP, rt = b / (kSlices * NP);
  const int64_t row0 = (int64_t)rt * kR;
  if (b == 0 && tid < n_steps) step_ctr[tid] += 1.0f;  // Adam's step (read by k_adam_flat)
  const float* F = p == 0 ? f0 : (p == 1 ? f1 : f2);
  const int ld = (MODE == kSlActor && p == 0) || (MODE == kSlCriticBoot && p == 1) ? kALd : kCLd;
  const float* Ssrc = MODE == kSlCriticBoot && p > 0 ? S2g : Sg;
  const bool drop = MODE != kSlActor && p == 0;
  // the ring's insert count first: the row draw (Philox) needs it, and issued
  // after the weight fragments it made the draw wait for all of them
  const int64_t t_total = rs.ring ? *rs.total : 0;
  const float bv = F[kPB1 + tid];  // b1, with the weight fragments
  // the slice's W2 fragments, rows 16 s + i, k = 64 w + 16 t + 4 g, and the
  // layer-1 fragments of n-tiles w + 4q: in flight under the staging
  f4 wv[4], w1v[4];
  {
    const gfp wr = (gfp)F + kPW2 + (size_t)(kSliceU * s + i) * ld + 64 * w + 4 * g;
#pragma unroll
    for (int t = 0; t < 4; ++t) wv[t] = *(gf4u)(wr + 16 * t);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) w1v[q] = w1_frag((gfp)F + kPW1, 16 * (w + 4 * q), lane);
  const int si = tid >> 4, sk = tid & 15;
  float sv;
  f4 rowv = {0.f, 0.f, 0.f, 0.f};
  bool scat = false;
  if (rs.ring) {
    const int64_t b = row0 + si, t = t_total;
    const bool ok = b < B && t > 0;
    const int64_t idx = ok ? ring_row(rs, b, t) : 0;
    const float* src = rs.ring + idx * 28;
    sv = ld_or0(src, (MODE == kSlCriticBoot && p > 0 ? 15 : 0) + sk, ok && sk < kIn);
    // the row into the sample buffers (stored after the barrier below, so no
    // wait for the sample's operands also waits for these stores)
    scat = ok && s == 0 && p == 0 && sk < 7;
    rowv = *(const f4*)(src + 4 * (sk < 7 ? sk : 0));
  } else {
    sv = ld_or0(Ssrc, (row0 + si) * kIn + sk, sk < kIn && row0 + si < B);
  }
  uint32_t keep0 = 0, keep1 = 0;
  if (drop) {
    const uint64_t call = (uint64_t)*call_ctr;
    keep0 = dropout_bits16(seed, call, key_row0 + row0, w, lane);      // n-tiles w, w + 8
    keep1 = dropout_bits16(seed, call, key_row0 + row0, w + 4, lane);  // n-tiles w + 4, w + 12
  }
  sS[sl_t16(si, sk)] = sv;
  sB1[tid] = bv;
  lds_sync32();
  if (scat) {
#pragma unroll
    for (int c = 0; c < 4; ++c) skmlp::ring_scatter(rs, row0 + si, 4 * sk + c, rowv[c]);
  }
  // ---- layer 1, n-tiles w, w + 4, w + 8, w + 12
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t bits = ((q & 1) ? keep1 : keep0) >> (4 * (q >> 1));
    l1_out_sl(g16_l1w(sS, w1v[q], lane), sB1, w + 4 * q, lane, sH, nullptr, drop, bits);
  }
  lds_sync32();
  // ---- layer 2 of the slice: wave w contracts inputs 64 w .. 64 w + 63
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* xr = sH + i * kSlLdH + 64 * w + (4 * g ^ sl_hmask(i));
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = m16x4(*(const f4*)(xr + 16 * t), wv[t], acc);
    float* red = sRed + w * kSlRed + sl_red(4 * g, i);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[r * kSliceU] = acc[r];
  }
  lds_sync32();
  // ---- z2[row][16 s + j] = the 4 waves' partials (thread = (row, j))
  {
    const int row = tid >> 4, j = tid & 15;
    const float* red = sRed + sl_red(row, j);
    const float z = (red[0] + red[kSlRed]) + (red[2 * kSlRed] + red[3 * kSlRed]);
    Z[((int64_t)rt * NP + p) * kZPlane + row * kH2 + kSliceU * s + j] = z;
  }
}

// sum over the 16 lanes of a DPP row, in every lane of the row (xor 1, xor 2,
// half-row mirror, row mirror: each step adds a lane-symmetric pair, so every
// lane ends with the same bits)
template <int CTRL>
__device__ __forceinline__ float dpp_all(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float rowall16(float v) {
  v += dpp_all<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_all<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_all<0x141>(v);  // row_half_mirror
  v += dpp_all<0x140>(v);  // row_mirror
  return v;
}


// The backward launch's workgroup `bid` (row tile bid / kSlices, slice
// bid % kSlices) on the LDS at smem_sl (sl_bwd_lds(MODE) bytes): the body of
// k_grad_slice_bwd, and of k_bwd_act_step32's backward workgroups.
#define SK_SLICE_BWD_PARAMS                                                                                      \
  const float *__restrict__ f0, const float *__restrict__ f1, const float *__restrict__ f2,                       \
      const float *__restrict__ Sg, const float *__restrict__ Ag, const float *__restrict__ Yg,                  \
      const float *__restrict__ Rg, const float *__restrict__ Dg, float gamma, int64_t B, int64_t key_row0,      \
      float scale, uint64_t seed, const int64_t *__restrict__ call_ctr, const float *__restrict__ Z,             \
      float *__restrict__ partial, float *__restrict__ partial_w1, float *__restrict__ stat_out,                 \
      uint8_t *__restrict__ mask_out
#define SK_SLICE_BWD_ARGS \
  f0, f1, f2, Sg, Ag, Yg, Rg, Dg, gamma, B, key_row0, scale, seed, call_ctr, Z, partial, partial_w1, stat_out, mask_out

// The backward of a (row tile, slice) in SK_BWD_HALVES workgroups: half hq
// owns n-tiles w + 4q for q = hq, hq + 2 (layer 1 of the trained net, the
// dW2 columns, the dz1 share and its dW1 / db1 contributions), each half
// redoing the loads, the per-row reductions and dz2 that both need.  Every
// output entry is computed by exactly one workgroup with the same operations
// in the same order as by the one-workgroup form (SK_BWD_HALVES=1), so the
// results are the same bits; the launch has twice the workgroups on the 256
// CUs its 128 left half idle.
#ifndef SK_BWD_HALVES
#define SK_BWD_HALVES 2
#endif
constexpr int kBwdH = SK_BWD_HALVES, kBwdQ = 4 / kBwdH;
static_assert(kBwdH == 1 || kBwdH == 2 || kBwdH == 4, "1, 2 or 4 workgroups per (row tile, slice)");

template <int MODE>
__device__ __forceinline__ void grad_slice_bwd(int bid, float* smem_sl, SK_SLICE_BWD_PARAMS) {
  constexpr int NP = sl_planes(MODE);
  constexpr bool CRIT = MODE != kSlActor;
  constexpr int LD0 = sl_ld(MODE, 0), NPAR = CRIT ? kCP : kAP;
  float* sS = smem_sl;                  // [16][16] (sl_t16)
  float* sST = sS + kR * kSlLdT;        // [16 features][16 rows] (sl_t16)
  float* sZ = sST + kR * kSlLdT;        // [NP][16][kLdZ]
  float* sTL = sZ + NP * kR * kLdZ;     // [NP][1024] the nets' fp32 tails
  float* sH1 = sTL + NP * 1024;         // [16][260] layer 1 of the trained net, after Dropout (sl_hmask)
  float* sH1T = sH1 + kR * kSlLdH;      // [256][16] (sl_t16)
  float* sDZ2 = sH1T + kH1 * kSlLdT;    // [16 rows][16 slice units] (sl_t16)
  float* sDZ2T = sDZ2 + kSliceU * kSlLdT;  // [16 units][16 rows] (sl_t16)
  float* sH2T = sDZ2T + kSliceU * kSlLdT;  // [4 waves][16 units][4] per-unit gradient sums
  float* sA = sH2T + kSliceU * kSlLdT;  // [16][2] actions (critic)
  float* sRD = sA + 32;                 // [16] r or y, [16] done
  float* sDQ = sRD + 2 * kR;            // [16][2] dL/dq (critic) or dL/dz3 (actor)
  float* sST8 = sDQ + 2 * kR;           // [16] per-row e^2 (critic) or Q (actor)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  // block = (row tile, half, slice), slice fastest (slice s on XCD s)
  const int s = bid % kSlices, hq = (bid / kSlices) % kBwdH, rt = bid / (kSlices * kBwdH);
  const int64_t row0 = (int64_t)rt * kR;
  const float* fl[3] = {f0, f1, f2};
  const gfp W2 = (gfp)f0 + kPW2;
  TP32(20);
  // ---- phase 0: every global load; the tails first, their index arithmetic
  // ahead of every load (after the others it shared registers with loads in
  // flight and cost a full vmcnt(0) round trip)
  float tv[NP][4];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int k = 0; k < 4; ++k) tv[p][k] = tail_src((gfp)fl[p], sl_ld(MODE, p), sl_nout(MODE, p), tid + kSlThreads * k);
  // the slice's W2 rows down the columns of n-tiles w + 4q (the dz1 GEMM of
  // phase 3), q = hq + kBwdH k: this workgroup's n-tiles
  float wd[kBwdQ][4];
#pragma unroll
  for (int k = 0; k < kBwdQ; ++k)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      wd[k][c] = W2[(size_t)(kSliceU * s + 4 * g + c) * LD0 + 16 * (w + 4 * (hq + kBwdH * k)) + i];
  f4 w1v[kBwdQ];
#pragma unroll
  for (int k = 0; k < kBwdQ; ++k) w1v[k] = w1_frag((gfp)f0 + kPW1, 16 * (w + 4 * (hq + kBwdH * k)), lane);
  f4 zv[NP][2];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int m = 0; m < 2; ++m)
      zv[p][m] = *(const f4*)(Z + ((int64_t)rt * NP + p) * kZPlane + 4 * (tid + kSlThreads * m));
  const int si = tid >> 4, sk = tid & 15;
  const float sv = ld_or0(Sg, (row0 + si) * kIn + sk, sk < kIn && row0 + si < B);
  const bool rok = tid < kR && row0 + tid < B;
  const float av = CRIT && tid < 32 && row0 + (tid >> 1) < B ? Ag[row0 * 2 + tid] : 0.f;
  const float rv = CRIT && rok ? (MODE == kSlCriticBoot ? Rg[row0 + tid] : Yg[row0 + tid]) : 0.f;
  const float dv = MODE == kSlCriticBoot && rok ? Dg[row0 + tid] : 0.f;
  // keep0: n-tiles w, w + 8 (q = 0, 2); keep1: w + 4, w + 12 (q = 1, 3)
  uint32_t keep0 = 0, keep1 = 0;
  if (CRIT) {
    const uint64_t call = (uint64_t)*call_ctr;
    // (this workgroup's q = hq + kBwdH k all share hq's parity)
    if (kBwdH == 1 || (hq & 1) == 0) keep0 = dropout_bits16(seed, call, key_row0 + row0, w, lane);
    if (kBwdH == 1 || (hq & 1) == 1) keep1 = dropout_bits16(seed, call, key_row0 + row0, w + 4, lane);
  }
  sS[sl_t16(si, sk)] = sv;
  sST[sl_t16(sk, si)] = sv;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int q = tid + kSlThreads * m;
      *(f4*)(sZ + p * kR * kLdZ + (q >> 5) * kLdZ + 4 * (q & 31)) = zv[p][m];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) sTL[p * 1024 + tid + kSlThreads * k] = tv[p][k];
  }
  if (CRIT && tid < 32) sA[tid] = av;
  if (CRIT && tid < kR) {
    sRD[tid] = rv;
    sRD[kR + tid] = dv;
  }
  if (CRIT && mask_out && s == 0) {
#pragma unroll
    for (int k = 0; k < kBwdQ; ++k) {
      const int q = hq + kBwdH * k;
      const uint32_t bits = ((q & 1) ? keep1 : keep0) >> (4 * (q >> 1));
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (row0 + 4 * g + r < B) mask_out[(row0 + 4 * g + r) * kH1 + 16 * (w + 4 * q) + i] = (bits >> r) & 1u;
    }
  }
  lds_sync32();
  TP32(21);
  // ---- phase 1: layer 1 of the trained net (MFMA) and the per-row reductions (VALU)
#pragma unroll
  for (int k = 0; k < kBwdQ; ++k) {
    const int q = hq + kBwdH * k, nt = w + 4 * q;
    const uint32_t bits = ((q & 1) ? keep1 : keep0) >> (4 * (q >> 1));
    l1_out_sl(g16_l1w(sS, w1v[k], lane), sTL, nt, lane, sH1, sH1T, CRIT, bits);
  }
  {
    const int row = tid >> 4, c = tid & 15;
    const bool valid = row0 + row < B;
    const float* T0 = sTL;
    const float* T1 = sTL + 1024;
    const float* z0 = sZ + row * kLdZ;
    if (CRIT) {
      const float a0 = sA[2 * row], a1 = sA[2 * row + 1];
      float y;
      if (MODE == kSlCriticBoot) {
        const float* za = sZ + kR * kLdZ + row * kLdZ;
        const float* zt = sZ + 2 * kR * kLdZ + row * kLdZ;
        const float* T2 = sTL + 2048;
        float m0 = 0.f, m1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int u = c + 16 * k;
          const float h = fmaxf(za[u] + T1[kT2 + u], 0.f);
          m0 += h * T1[kT3 + u];
          m1 += h * T1[kT3 + kH2 + u];
        }
        const float mu0 = tanhf(rowall16((m0)) + T1[kTB]);
        const float mu1 = tanhf(rowall16((m1)) + T1[kTB + 1]);
        float qt = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int u = c + 16 * k;
          qt += fmaxf(zt[u] + T2[kT2 + u] + T2[kTA + 2 * u] * mu0 + T2[kTA + 2 * u + 1] * mu1, 0.f) * T2[kT3 + u];
        }
        y = sRD[row] + gamma * (1.f - sRD[kR + row]) * (T2[kTB] + rowall16((qt)));
      } else {
        y = sRD[row];
      }
      float qc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int u = c + 16 * k;
        qc += fmaxf(z0[u] + T0[kT2 + u] + T0[kTA + 2 * u] * a0 + T0[kTA + 2 * u + 1] * a1, 0.f) * T0[kT3 + u];
      }
      qc = rowsum16(qc);
      if (c == 15) {
        const float e = valid ? qc + T0[kTB] - y : 0.f;
        sDQ[2 * row] = scale * e;
        sST8[row] = e * e;
      }
    } else {
      const float* zc = sZ + kR * kLdZ + row * kLdZ;
      float m0 = 0.f, m1 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int u = c + 16 * k;
        const float h = fmaxf(z0[u] + T0[kT2 + u], 0.f);
        m0 += h * T0[kT3 + u];
        m1 += h * T0[kT3 + kH2 + u];
      }
      const float mu0 = tanhf(rowall16((m0)) + T0[kTB]);
      const float mu1 = tanhf(rowall16((m1)) + T0[kTB + 1]);
      float d0 = 0.f, d1 = 0.f, qs = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int u = c + 16 * k;
        const float wa0 = T1[kTA + 2 * u], wa1 = T1[kTA + 2 * u + 1], w3 = T1[kT3 + u];
        const float z = zc[u] + T1[kT2 + u] + wa0 * mu0 + wa1 * mu1;
        const float dq = z > 0.f ? w3 : 0.f;
        d0 += dq * wa0;
        d1 += dq * wa1;
        qs += fmaxf(z, 0.f) * w3;
      }
      d0 = rowsum16(d0);
      d1 = rowsum16(d1);
      qs = rowsum16(qs);
      if (c == 15) {
        sDQ[2 * row] = valid ? -scale * d0 * (1.f - mu0 * mu0) : 0.f;
        sDQ[2 * row + 1] = valid ? -scale * d1 * (1.f - mu1 * mu1) : 0.f;
        sST8[row] = valid ? qs + T1[kTB] : 0.f;
      }
    }
  }
  lds_sync32();
  TP32(22);
  // ---- phase 2: dz2 of the slice's units (thread = (row, j))
  {
    const int row = tid >> 4, j = tid & 15, u = kSliceU * s + j;
    const float* T0 = sTL;
    float dz, h2x;
    if (CRIT) {
      const float z = sZ[row * kLdZ + u] + T0[kT2 + u] + T0[kTA + 2 * u] * sA[2 * row] + T0[kTA + 2 * u + 1] * sA[2 * row + 1];
      const float h2 = fmaxf(z, 0.f), dq = sDQ[2 * row];
      dz = h2 > 0.f ? dq * T0[kT3 + u] : 0.f;
      h2x = dq * h2;
    } else {
      const float h2 = fmaxf(sZ[row * kLdZ + u] + T0[kT2 + u], 0.f);
      dz = h2 > 0.f ? sDQ[2 * row] * T0[kT3 + u] + sDQ[2 * row + 1] * T0[kT3 + kH2 + u] : 0.f;
      h2x = h2;
    }
    sDZ2[sl_t16(row, j)] = dz;
    sDZ2T[sl_t16(j, row)] = dz;
    // the unit's b2 and W3 (and, critic, action-column) gradients over the
    // wave's 4 rows (lanes j, j + 16, j + 32, j + 48), then across waves in phase 3
    float v[4];
    if (CRIT) {
      v[0] = dz;
      v[1] = dz * sA[2 * row];
      v[2] = dz * sA[2 * row + 1];
      v[3] = h2x;
    } else {
      v[0] = dz;
      v[1] = sDQ[2 * row] * h2x;
      v[2] = sDQ[2 * row + 1] * h2x;
      v[3] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] += __shfl_xor(v[k], 16, 64);
      v[k] += __shfl_xor(v[k], 32, 64);
    }
    if (lane < kSliceU) *(f4*)(sH2T + (w * kSliceU + j) * 4) = f4{v[0], v[1], v[2], v[3]};
  }
  lds_sync32();
  TP32(23);
  // ---- phase 3: the slice's per-unit gradients; dW2 rows; dz1 share -> dW1, db1
  float* P = partial + (int64_t)rt * NPAR;
  float* PW = partial_w1 + (int64_t)(rt * kSlices + s) * kW1Part;  // one contribution row per (row tile, slice)
  if (hq != 0) {
    // the slice's per-unit gradients and b3 / the stat: half 0's
  } else if (tid < kSliceU) {
    const int j = tid, u = kSliceU * s + j;
    const f4 v = (*(const f4*)(sH2T + j * 4) + *(const f4*)(sH2T + (kSliceU + j) * 4)) +
                 (*(const f4*)(sH2T + (2 * kSliceU + j) * 4) + *(const f4*)(sH2T + (3 * kSliceU + j) * 4));
    const float b2 = v.x, x0 = v.y, x1 = v.z, x3 = v.w;
    if (CRIT) {
      P[pB2(kCLd) + u] = b2;
      P[skpart::critic_w2_action(u, 0)] = x0;
      P[skpart::critic_w2_action(u, 1)] = x1;
      P[pW3(kCLd) + u] = x3;
    } else {
      P[pB2(kALd) + u] = b2;
      P[pW3(kALd) + u] = x0;
      P[pW3(kALd) + kH2 + u] = x1;
    }
  } else if (s == 0 && tid == 64) {  // a lane of wave 1: b3 and the step's loss / Q sum
    float b30 = 0.f, b31 = 0.f, st = 0.f;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      b30 += sDQ[2 * r];
      b31 += sDQ[2 * r + 1];
      st += sST8[r];
    }
    if (CRIT) {
      P[pB3(kCLd, 1)] = b30;
    } else {
      P[pB3(kALd, 2)] = b30;
      P[pB3(kALd, 2) + 1] = b31;
    }
    if (stat_out) atomicAdd(stat_out, st);
  }
  const float dscale = CRIT ? 1.25f : 1.f;  // Dropout(0.2): kept activations x 1.25
  const f4 dzr = *(const f4*)(sDZ2 + sl_t16(i, 4 * g));
  const f4 sT = *(const f4*)(sST + sl_t16(i, 4 * g));
#pragma unroll
  for (int k = 0; k < kBwdQ; ++k) {
    const int q = hq + kBwdH * k, nt = w + 4 * q, n = 16 * nt + i;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 gw2 = g16_wgrad_sl(z4, sDZ2T, 0, sH1T, 16 * nt, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = kSliceU * s + 4 * g + r;
      P[CRIT ? skpart::critic_w2_main(o, n) : kPW2 + o * kALd + n] = gw2[r];
    }
    const f32x4 acc = m16x4(dzr, f4{wd[k][0], wd[k][1], wd[k][2], wd[k][3]}, z4);
    f4 d;
    float b = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      d[r] = sH1[(4 * g + r) * kSlLdH + 16 * nt + (i ^ sl_hmask(4 * g))] > 0.f ? acc[r] * dscale : 0.f;
      b += d[r];
    }
    b += __shfl_xor(b, 16, 64);
    b += __shfl_xor(b, 32, 64);
    if (g == 0) PW[kPB1 + n] = b;
    const f32x4 gw1 = m16x4(d, sT, z4);
    if (i < kIn) {
#pragma unroll
      for (int r = 0; r < 4; ++r) PW[kPW1 + (16 * nt + 4 * g + r) * kIn + i] = gw1[r];
    }
  }
  TP32(24);
}

template <int MODE>
__global__ void __launch_bounds__(kSlThreads) k_grad_slice_bwd(SK_SLICE_BWD_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  grad_slice_bwd<MODE>(blockIdx.x, smem_sl, SK_SLICE_BWD_ARGS);
}

// ---------------------------------------------------------------- actor forward
// the last workgroup to arrive stores the call number the launch drew with.
// Grouped arrival (as the bf16 actor's advance_call, csrc/sk_actor.hip):
// workgroup b on group line call_ctr[2 + 16 (b % 8)], the last of each group
// on call_ctr[1] (SK_ACTOR_COUNTER_WORDS); nb = the launch's workgroups that
// arrive (the first nb of the grid)
__device__ __forceinline__ void advance_call32(uint64_t* call_ctr, uint64_t call, unsigned nb) {
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned long long members = (nb - g + 7u) / 8u;
    unsigned long long* gc = (unsigned long long*)&call_ctr[2 + 16 * g];
    if (atomicAdd(gc, 1ull) == members - 1) {
      *gc = 0;
      const unsigned long long groups = nb < 8u ? nb : 8u;
      if (atomicAdd((unsigned long long*)&call_ctr[1], 1ull) == groups - 1) {
        call_ctr[0] = call;
        call_ctr[1] = 0;
      }
    }
  }
}
// mean and variance GEMMs of parameter noise on 16-row tiles (g16_xwT256 with
// x^2 w^2 beside: every operand load feeds both chains)
__device__ __forceinline__ void g16_xwT256_mv(f32x4& m, f32x4& v, const float* X, gfp W, int n0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const float* xr = X + i * kLdH1 + 4 * g;
  const gfp wr = W + (size_t)(n0 + i) * kALd + 4 * g;
  m = f32x4{0.f, 0.f, 0.f, 0.f};
  v = f32x4{0.f, 0.f, 0.f, 0.f};
  f4 wn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + 16 * t);
#pragma unroll
  for (int k = 0; k < 256; k += 64) {
    f4 wc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wc[t] = wn[t];
    if (k + 64 < 256) {
#pragma unroll
      for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + k + 64 + 16 * t);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f4 x = *(const f4*)(xr + k + 16 * t);
      m = m16x4(x, wc[t], m);
      v = m16x4(x * x, wc[t] * wc[t], v);
    }
  }
}

// 4 normals for the rows r .. r+3 of unit `unit` of `layer` (Box-Muller on
// the 4 Philox words: two pairs)
__device__ __forceinline__ void normals4(uint64_t seed, uint64_t call, uint32_t r, uint32_t layer_unit, float z[4]) {
  const uint4 u = philox(make_uint4(r, layer_unit, (uint32_t)call, (uint32_t)(call >> 32)), (uint32_t)seed,
                         (uint32_t)(seed >> 32));
  const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float u1 = ((float)(wd[2 * q] >> 8) + 0.5f) * 0x1p-24f;  // (0, 1)
    const float u2 = (float)(wd[2 * q + 1] >> 8) * 0x1p-24f;       // [0, 1)
    const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln u1
    z[2 * q] = rad * __builtin_amdgcn_cosf(u2);  // v_cos_f32 / v_sin_f32 take revolutions
    z[2 * q + 1] = rad * __builtin_amdgcn_sinf(u2);
  }
}

// 4 noisy pre-activations of rows r .. r+3 of unit `layer_unit`:
// y = m + b + sd sqrt(b^2 + v) xi, the xi keyed as normals4's (the same
// Philox counter, 24-bit uniforms, Box-Muller in revolutions) but in pair
// form: sqrt((b^2 + v) L) with L = -2 ln(u1) sd^2 carries the radius, one
// square root per element instead of the radius's plus the element's, and
// Philox4x32 with SK_F32_NOISE_ROUNDS rounds (7: the fewest BigCrush-passing
// rounds, as the bf16 path's noise; sk_mlp.hpp).  k2 = noise_k2(sd).
#ifndef SK_F32_NOISE_ROUNDS
#define SK_F32_NOISE_ROUNDS 7
#endif
// noisy4 in two parts, bit for bit the same: the draws (Philox words ->
// the pairs' L and cos / sin; independent of the GEMM, so they can be issued
// ahead of it and run under its MFMAs) and the combination with m and v
// SK_NOISE_HOIST = 1 (A/B builds) draws layer 2's noise before its second
// half's GEMM instead of after it: neutral at two workgroups per CU
// (profiles/r04g_noise_hoist_ab.jsonl); at three its 24 live registers
// spilled (config 5 acting 119 vs 112 us, profiles/r04p_hoist_ab.jsonl)
#ifndef SK_NOISE_HOIST
#define SK_NOISE_HOIST 0
#endif
struct Draw4 {
  float L[2], c[2], s[2];
};
__device__ __forceinline__ Draw4 draw4n(uint64_t seed, uint64_t call, uint32_t r, uint32_t layer_unit, float k2) {
  const uint4 u = skmlp::philox<SK_F32_NOISE_ROUNDS>(
      make_uint4(r, layer_unit, (uint32_t)call, (uint32_t)(call >> 32)), (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
  Draw4 d;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float u1 = ((float)(wd[2 * q] >> 8) + 0.5f) * 0x1p-24f;  // (0, 1)
    const float u2 = (float)(wd[2 * q + 1] >> 8) * 0x1p-24f;       // [0, 1) revolutions
    d.L[q] = k2 * __builtin_amdgcn_logf(u1);                        // -2 ln(u1) sd^2
    d.c[q] = __builtin_amdgcn_cosf(u2);
    d.s[q] = __builtin_amdgcn_sinf(u2);
  }
  return d;
}
template <typename V>
__device__ __forceinline__ void noisy4_apply(const Draw4& d, float b, const V& m, const V& v, int o, float y[4]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    y[2 * q] = __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v[o + 2 * q]) * d.L[q]), d.c[q],
                              m[o + 2 * q] + b);
    y[2 * q + 1] = __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v[o + 2 * q + 1]) * d.L[q]), d.s[q],
                                  m[o + 2 * q + 1] + b);
  }
}
template <typename V>
__device__ __forceinline__ void noisy4(uint64_t seed, uint64_t call, uint32_t r, uint32_t layer_unit, float k2,
                                       float b, const V& m, const V& v, int o, float y[4]) {
  const uint4 u = skmlp::philox<SK_F32_NOISE_ROUNDS>(
      make_uint4(r, layer_unit, (uint32_t)call, (uint32_t)(call >> 32)), (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float u1 = ((float)(wd[2 * q] >> 8) + 0.5f) * 0x1p-24f;  // (0, 1)
    const float u2 = (float)(wd[2 * q + 1] >> 8) * 0x1p-24f;       // [0, 1) revolutions
    const float L = k2 * __builtin_amdgcn_logf(u1);                 // -2 ln(u1) sd^2
    const float c = __builtin_amdgcn_cosf(u2), s = __builtin_amdgcn_sinf(u2);
    y[2 * q] = __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v[o + 2 * q]) * L), c, m[o + 2 * q] + b);
    y[2 * q + 1] =
        __builtin_fmaf(__builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, v[o + 2 * q + 1]) * L), s, m[o + 2 * q + 1] + b);
  }
}

// Row maps of a 32-row actor tile: local row i -> global row of the [rows]
// batch, and whether it exists.  Contiguous: rows row0 .. row0 + 31.
// Players (the self-play tick, k_act_step32): games g0 .. g0 + 15, rows
// g0 + i (player 1) and N + g0 + i - 16 (player 2) of the actor's
// player-major [2N] order.  Parameter / action noise is keyed by the global
// row (the first row of an aligned 4-row group), so with N % 4 == 0 both maps
// draw the same noise for the same row.
struct RowsContig {
  int64_t row0, rows;
  __device__ int64_t operator()(int i) const { return row0 + i; }
  __device__ bool valid(int i) const { return row0 + i < rows; }
};
struct RowsPlayers {
  int64_t g0, n;
  __device__ int64_t operator()(int i) const { return i < 16 ? g0 + i : n + g0 + (i - 16); }
  __device__ bool valid(int i) const { return g0 + (i & 15) < n; }
};

// one 32-row tile per workgroup of 4 waves: layer 1 n-tiles w, 4 + w,
// layer 2 n-tile w, layer 3 by all threads.  NOISE: per layer y = xW + b +
// sd sqrt(x^2 W^2 + b^2) xi, xi ~ N(0,1) per (row, unit) (exact in
// distribution for w' = w (1 + sd N(0,1)) drawn per row, each noisy weight
// being used once per row).  The actions go to out[R(i)] and, if act_lds,
// to act_lds[i].  GEMMs on split bf16 pieces (gemm6, sk_split.hpp): fp32
// products at the bf16 MFMA rate, W1 / W2 read from the actor's split pack
// `pk`, biases and W3 from the flat vector.  LDS (ActorLds, kActorTileLds
// bytes): the observations and the layer-1 outputs as four bf16 planes each
// (hi, mid, lo, square; written once by the producing lane, read by every
// wave's A fragments), layer 2's fp32 outputs over the layer-1 planes once
// every wave has read them.  Round 3's f32-MFMA tile (128 dependent 32x32x2
// f32 MFMAs per wave in layer 2: 5.2 us of the 4,096-game acting launch,
// profiles/r03t_*) and its variance GEMM's bf16 operands are replaced.
// Layer 1 runs in two halves of 128 units (n-tile 4h + w per wave), each
// followed by its 8 k-steps of layer 2 into the same accumulators (the k
// order, hence every sum, of one 16-step chain): the planes hold one half,
// 41 KB of LDS per tile instead of 74 KB, so three workgroups share a CU
// instead of two.
// waves per SIMD the acting kernels are compiled for (their VGPR budget:
// 512 / waves): with the half-size planes three workgroups share a CU
// (config 5 acting 127 -> 112 us with SK_NOISE_HOIST 0; at two waves, 185
// VGPRs, no gain: profiles/r04o_act_waves_ab.jsonl).  The episode kernel at
// two: it held every loop-invariant weight fragment of the tile across the
// episode (512 VGPRs, one workgroup per CU, spills) until its weight
// addresses were made opaque per tick (180 -> 110 us per tick,
// profiles/r04o_episode_ab.jsonl)
#ifndef SK_ACT_WAVES
#define SK_ACT_WAVES 3
#endif
#ifndef SK_EPISODE_WAVES
#define SK_EPISODE_WAVES 2
#endif
constexpr int kLdX1 = 24, kLdX2 = 136;              // bf16 row strides (48 / 272 B: conflict-free 16-B reads)
constexpr int kX1Plane = 32 * kLdX1, kX2Plane = 32 * kLdX2;  // kX2Plane: one half of layer 1's units
constexpr size_t kActorTileLds = (size_t)(4 * kX1Plane + 4 * kX2Plane) * 2;
static_assert((size_t)32 * kLdH2 * 4 <= (size_t)4 * kX2Plane * 2, "layer 2's outputs fit over the layer-1 planes");
struct ActorLds {
  short* S;   // [4 planes][32][kLdX1]
  short* H1;  // [4 planes][32][kLdX2]
  float* H2;  // [32][kLdH2], aliasing H1
};
__device__ __forceinline__ ActorLds actor_lds(char* base) {
  ActorLds L;
  L.S = (short*)base;
  L.H1 = L.S + 4 * kX1Plane;
  L.H2 = (float*)L.H1;
  return L;
}
// the four planes of element (row, col) of a bf16-plane block
__device__ __forceinline__ void put4(short* P, int plane, int at, float v) {
  short hi, mid, lo, sq;
  sksplit::split4(v, hi, mid, lo, sq);
  P[at] = hi;
  P[plane + at] = mid;
  P[2 * plane + at] = lo;
  P[3 * plane + at] = sq;
}

template <bool NOISE, typename MAP>
__device__ __forceinline__ void actor_tile32(const Net& A, const char* __restrict__ pk,
                                             const float* __restrict__ X, float* __restrict__ out, const MAP& R,
                                             float sd, float action_sd, uint64_t seed, uint64_t call, ActorLds T,
                                             float2* act_lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int t = threadIdx.x; t < 32 * 16; t += kFwdThreads) {  // S[i][k] = obs (k < 12, valid rows), else 0
    const int i = t >> 4, k = t & 15;
    put4(T.S, kX1Plane, i * kLdX1 + k, (k < kIn && R.valid(i)) ? X[R(i) * kIn + k] : 0.f);
  }
  __syncthreads();
  TP32(2);
  const gbf8 W1 = (gbf8)(pk + sksplit::kOffW1), W2 = (gbf8)(pk + sksplit::kOffW2);
  const int u2 = 32 * w + (lane & 31);  // this wave's layer-2 unit
  const float k2 = skmlp::noise_k2(sd);
  Draw4 dr[4];
  f32x16 m2 = {0}, var2 = {0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    {  // layer 1, units 128 h .. 128 h + 127: n-tile 4 h + w, into the planes' column u - 128 h
      const int nt = 4 * h + w, u = 32 * nt + (lane & 31), col = u - 128 * h;
      f32x16 m = {0}, var = {0};
      gemm6<1, NOISE>(m, var, T.S, kLdX1, kX1Plane, W1 + 64 * nt, sksplit::kW1Plane, lane);
      const float b = A.b1[u];
      if (NOISE) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float y[4];
          noisy4(seed, call, (uint32_t)R(drow(4 * g, lane)), (uint32_t)u, k2, b, m, var, 4 * g, y);
#pragma unroll
          for (int q = 0; q < 4; ++q) put4(T.H1, kX2Plane, drow(4 * g + q, lane) * kLdX2 + col, fmaxf(y[q], 0.f));
        }
      } else {
#pragma unroll
        for (int v = 0; v < 16; ++v) put4(T.H1, kX2Plane, drow(v, lane) * kLdX2 + col, fmaxf(m[v] + b, 0.f));
      }
    }
    __syncthreads();
    if (h == 0) TP32(3);
    if (NOISE && SK_NOISE_HOIST && h == 1) {  // layer 2's draws among the MFMAs (A/B only)
#pragma unroll
      for (int g = 0; g < 4; ++g) dr[g] = draw4n(seed, call, (uint32_t)R(drow(4 * g, lane)), (uint32_t)(kH1 + u2), k2);
    }
    // layer 2, k = 128 h .. 128 h + 127 (k-steps 8 h .. 8 h + 7 of n-tile w)
    gemm6<8, NOISE>(m2, var2, T.H1, kLdX2, kX2Plane, W2 + 16 * 64 * w + 8 * 64 * h, sksplit::kW2Plane, lane);
    __syncthreads();  // every wave has read this half: the next half / layer 2's outputs go over it
  }
  {
    const float b = A.b2[u2];
    if (NOISE) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float y[4];
        if (!SK_NOISE_HOIST) dr[g] = draw4n(seed, call, (uint32_t)R(drow(4 * g, lane)), (uint32_t)(kH1 + u2), k2);
        noisy4_apply(dr[g], b, m2, var2, 4 * g, y);
#pragma unroll
        for (int q = 0; q < 4; ++q) T.H2[drow(4 * g + q, lane) * kLdH2 + u2] = fmaxf(y[q], 0.f);
      }
    } else {
#pragma unroll
      for (int v = 0; v < 16; ++v) T.H2[drow(v, lane) * kLdH2 + u2] = fmaxf(m2[v] + b, 0.f);
    }
  }
  __syncthreads();
  TP32(4);
  {  // layer 3: thread t -> row t / 8, units 16 (t % 8) .. (both outputs)
    const float* H2 = T.H2;
    const int i = threadIdx.x >> 3, c = threadIdx.x & 7;
    float m0 = 0.f, m1 = 0.f, v0 = 0.f, v1 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int u = 16 * c + k;
      const float h = H2[i * kLdH2 + u], w0 = A.W3[u], w1 = A.W3[kH2 + u];
      m0 += h * w0;
      m1 += h * w1;
      if (NOISE) {
        v0 += h * h * w0 * w0;
        v1 += h * h * w1 * w1;
      }
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {
      m0 += __shfl_xor(m0, off, 64);
      m1 += __shfl_xor(m1, off, 64);
      if (NOISE) {
        v0 += __shfl_xor(v0, off, 64);
        v1 += __shfl_xor(v1, off, 64);
      }
    }
    if (c == 0 && R.valid(i)) {
      const int64_t row = R(i);
      float y0 = m0 + A.b3[0], y1 = m1 + A.b3[1];
      if (NOISE) {
        float z[4];
        normals4(seed, call, (uint32_t)row, (uint32_t)(kH1 + kH2), z);
        y0 += sd * __builtin_amdgcn_sqrtf(v0 + A.b3[0] * A.b3[0]) * z[0];
        y1 += sd * __builtin_amdgcn_sqrtf(v1 + A.b3[1] * A.b3[1]) * z[1];
      }
      float o0 = tanhf(y0), o1 = tanhf(y1);
      if (action_sd != 0.f) {  // model_act_action_noise (:229-243): tanh output + N(0, sd), unclipped
        float z[4];
        normals4(seed, call, (uint32_t)row, (uint32_t)(kH1 + kH2 + 1), z);
        o0 += action_sd * z[0];
        o1 += action_sd * z[1];
      }
      *(float2*)(out + row * 2) = make_float2(o0, o1);
      if (act_lds) act_lds[i] = make_float2(o0, o1);
    }
  }
}

template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads, SK_ACT_WAVES) k_actor_fwd32(const float* __restrict__ aflat,
                                                             const char* __restrict__ apack,
                                                             const float* __restrict__ X, float* __restrict__ out,
                                                             int64_t rows, float sd, float action_sd, uint64_t seed,
                                                             uint64_t* __restrict__ call_ctr) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  const Net A = net_of(aflat, kALd, 2);
  // a launch that draws noise (parameter or action) uses call number
  // counter + 1 and its last workgroup stores that number back
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call = draws ? call_ctr[0] + 1 : 0;
  actor_tile32<NOISE>(A, apack, X, out, RowsContig{(int64_t)blockIdx.x * 32, rows}, sd, action_sd, seed, call,
                      actor_lds((char*)smem_sl), nullptr);
  if (draws) {  // the last workgroup to finish stores the call number it drew with
    __syncthreads();
    advance_call32(call_ctr, call, gridDim.x);
  }
}

// The self-play tick's act + step in ONE launch (VERDICT r02 item 3;
// SkillshotLearner.py:304-314 act -> do_actions -> game_tick -> get_state,
// with the replay ring insert of sk_env_step_insert): workgroup b owns games
// 16b .. 16b + 15.  Wave 0's lanes 0-31 issue k_step_split's state loads
// (both players of the 16 games) first, so they land under the actor's
// MFMA chain; the 4 waves run the fp32 actor tile on the games' 32
// observation rows (RowsPlayers); the actions meet in LDS; wave 0 then
// finishes k_step_split's tick for its lanes.  Equal, bit for bit, to
// sk_actor_forward_f32 (32-row tiles) followed by sk_env_step(_insert).
// Wave 0 counts its games into counter slot line b.
// act_step32: the body on the LDS at `smem` (the actor tile's, then sAct)
// for the first nb workgroups of the grid (k_act_step32: all of them;
// k_bwd_act_step32: the workgroups before the backward's)
constexpr size_t kActStepLds = kActorTileLds + 32 * sizeof(float2);
template <bool NOISE>
__device__ __forceinline__ void act_step32(const float* __restrict__ aflat, const char* __restrict__ apack,
                                           float* __restrict__ act_out, float sd, float action_sd, uint64_t seed,
                                           uint64_t* __restrict__ call_ctr, sk::StepArgs a, sk::Cfg c, char* smem,
                                           unsigned nb) {
  float2* sAct = (float2*)(smem + kActorTileLds);
  const int lane = threadIdx.x & 63;
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const int64_t g0 = (int64_t)blockIdx.x * 16;
  sk_counters* slot = a.ctr ? a.ctr + (size_t)blockIdx.x * SK_CTR_STRIDE : nullptr;
  TP32(0);
  sk::StepLane L;
  if (w0) L = sk::split_load(a, lane < 32 ? 2 * g0 + lane : 2 * a.n, slot);
  TP32(1);
  const Net A = net_of(aflat, kALd, 2);
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call = draws ? call_ctr[0] + 1 : 0;
  actor_tile32<NOISE>(A, apack, a.acting_obs, act_out, RowsPlayers{g0, a.n}, sd, action_sd, seed, call,
                      actor_lds(smem), sAct);
  TP32(5);
  __syncthreads();
  TP32(6);
  if (w0) {
    const float2 act = lane < 32 ? sAct[(lane & 1) * 16 + (lane >> 1)] : make_float2(0.f, 0.f);
    sk::split_finish(a, c, L, act, slot);
  }
  TP32(7);
  if (draws) {
    __syncthreads();
    advance_call32(call_ctr, call, nb);
  }
}

template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads, SK_ACT_WAVES) k_act_step32(const float* __restrict__ aflat,
                                                            const char* __restrict__ apack,
                                                            float* __restrict__ act_out, float sd, float action_sd,
                                                            uint64_t seed, uint64_t* __restrict__ call_ctr,
                                                            sk::StepArgs a, sk::Cfg c) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  act_step32<NOISE>(aflat, apack, act_out, sd, action_sd, seed, call_ctr, a, c, (char*)smem_sl, gridDim.x);
}


// The reference rule's episode collection (model_train, SkillshotLearner.py
// :289-318) in ONE launch: every game plays its episode
// from the current state, act (the actor held fixed for the epoch, fresh
// exploration noise per tick: tick t draws with call number call0 + 1 + t,
// as t sk_env_act_step calls would) -> do_actions -> game_tick -> get_state
// while game_live and ticks < tick_limit (:304); a game that has ended is
// stepped no further, as the reference's loop stops.  Workgroup b owns
// games 16b .. 16b + 15 for the whole episode (act_step32's geometry: no
// workgroup waits for another) and leaves once all of them have ended.
// Tick t reads the acting states at states[t] ([2][N][12], player-major;
// states[0] is the caller's observation of the start) and writes the
// actions to actions[t] ([2][N][2]), the post-tick observation to
// states[t + 1] and the reward to rewards[t] ([2][N]); lengths[i] = the
// ticks game i played.  The rows t < lengths[i] of both players are the
// episode's (s, a, r) for models_fit (:320-357); later rows are undefined.  The step counter and the
// noise call number advance by the ticks the per-tick loop would have run,
// max_i lengths[i] (it had been n_ticks, so the next epoch's
// restarts and noise diverged from the loop's whenever every game ended
// before the limit): k_episode_finish, one workgroup launched after this
// kernel on the same stream, reduces the lengths and stores both.
struct EpisodeArgs {
  float* states;
  float* actions;
  float* rewards;
  int32_t* lengths;
  int n_ticks;
};
template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads, SK_EPISODE_WAVES) k_act_episode32(const float* __restrict__ aflat,
                                                               const char* __restrict__ apack, float sd,
                                                               float action_sd, uint64_t seed,
                                                               uint64_t* __restrict__ call_ctr, sk::StepArgs a,
                                                               sk::Cfg c, EpisodeArgs ep) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  char* smem = (char*)smem_sl;
  float2* sAct = (float2*)(smem + kActorTileLds);
  int* sAlive = (int*)(sAct + 32);
  const int lane = threadIdx.x & 63;
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const int64_t g0 = (int64_t)blockIdx.x * 16;
  // no episode counters: a lane whose game has ended skips split_finish's
  // count, and the slot line is stored by lane 0 (the episode's outcome is
  // the final state and `lengths`)
  sk_counters* const slot = nullptr;
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call0 = draws ? call_ctr[0] : 0;
  const int64_t n = a.n, gt = 2 * g0 + lane, gi = gt >> 1;  // wave 0: lane -> (game, player)
  if (w0 && lane < 32 && (lane & 1) == 0 && gi < n) ep.lengths[gi] = 0;
  for (int t = 0; t < ep.n_ticks; ++t) {
    // the weights' addresses opaque per tick: otherwise every weight fragment
    // and bias the tile loads is loop-invariant, hoisted out of the loop and
    // held (or spilled) across the whole episode
    const float* af = aflat;
    const char* pk = apack;
    asm volatile("" : "+s"(af), "+s"(pk));
    const Net A = net_of(af, kALd, 2);
    sk::StepArgs at = a;
    at.acting_obs = ep.states + (int64_t)t * 24 * n;
    at.obs = ep.states + (int64_t)(t + 1) * 24 * n;
    at.reward = ep.rewards + (int64_t)t * 2 * n;
    sk::StepLane L;
    // the state loads fly under the actor tile (act_step32's order); the
    // loop test waits for them only after it
    if (w0) L = sk::split_load(at, lane < 32 ? gt : 2 * n, slot);
    actor_tile32<NOISE>(A, pk, at.acting_obs, ep.actions + (int64_t)t * 4 * n, RowsPlayers{g0, n}, sd,
                        action_sd, seed, call0 + 1 + (uint64_t)t, actor_lds(smem), sAct);
    if (w0) {
      // the reference's loop test (:304) on the pre-tick state; both lanes of a game agree
      const bool alive = L.in && ((L.mi.y >> 16) & 0xff) && L.mi.x < a.tick_limit;
      L.in = alive;  // an ended game is neither stepped nor written
      if (alive && L.p == 0) ep.lengths[L.i] = t + 1;
      const uint64_t any = __ballot(alive);
      if (lane == 0) *sAlive = any != 0;
    }
    __syncthreads();
    if (!*sAlive) break;  // workgroup-uniform: every game of the workgroup has ended
    if (w0) {
      const float2 act = lane < 32 ? sAct[(lane & 1) * 16 + (lane >> 1)] : make_float2(0.f, 0.f);
      sk::split_finish(at, c, L, act, slot);
    }
    __syncthreads();  // this tick's observations are the next tick's acting rows (this workgroup's own stores)
  }
}

// The episode's counter advance (see k_act_episode32): T = max lengths[i]
// (the per-tick loop's iterations: it runs while any game lives), then the
// step slot step0 + T and, when the episode drew, the call number call0 + T.
// Both start values are read here: the episode kernel leaves the counters
// alone, and this launch follows it on the stream.
__global__ void __launch_bounds__(256) k_episode_finish(const int32_t* __restrict__ lengths, int64_t n,
                                                        sk::StepRef step, uint64_t* __restrict__ call_ctr) {
  __shared__ int red[4];
  int m = 0;
  for (int64_t i = threadIdx.x; i < n; i += 256) m = max(m, lengths[i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t T = (uint64_t)max(max(red[0], red[1]), max(red[2], red[3]));
    step.slots[1 - step.parity] = step.slots[step.parity] + T;
    if (call_ctr) call_ctr[0] = call_ctr[0] + T;
  }
}

// ---------------------------------------------------------------- actor forward, 16-row tiles
// The same forward for small row counts: a 32-row tile is a serial chain of
// load latencies around 3.4 us of MFMA per workgroup (9.4 us at 256 rows);
// 16-row tiles on v_mfma_f32_16x16x4_f32 halve the per-workgroup MFMA chain
// (6.5 us at 256 rows).  Above ~4,096 rows the 32-row tiles win: the chip's
// fp32 MFMA time dominates and two 16-row workgroups per CU contend.  Every weight
// fragment a wave needs before layer 2 is issued ahead of the staging
// barrier.  Wave w: layer-1 n-tiles w + 4q (16 units each), layer-2 n-tiles w
// and w + 4; layer 3 from DPP row sums of the layer-2 tiles.  The noise draws
// are keyed exactly as k_actor_fwd32's: normals4 per (first row of a 4-row
// group, unit), z[r] for row + r.
// The 16-row tile on the LDS at S / H1 / MP (kActorTile16Lds bytes) for the
// row map R (local row i -> global row; noise keyed by the global first row of
// each aligned 4-row group, so with N % 4 == 0 the players' map draws what
// the contiguous map draws).  k_actor_fwd16 (contiguous rows) and
// k_act_step16 (8 games: rows g0 .. g0 + 7 and N + g0 .. N + g0 + 7, the
// actions also into act_lds) run it.
constexpr size_t kActorTile16Lds = (size_t)(kR * kLdS16 + kR * kLdH1) * 4 + 4 * kR * sizeof(f4);
template <bool NOISE, typename MAP>
__device__ __forceinline__ void actor_tile16(const Net& A, const float* __restrict__ X, float* __restrict__ out,
                                             const MAP& R, float sd, float action_sd, uint64_t seed, uint64_t call,
                                             float* S, float* H1, f4 (*MP)[kR], float2* act_lds) {
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // ---- every load ahead of the barrier: states, layer-1 fragments and biases, the
  // first layer-2 fragments (g16_xwT256's prefetch), W3 / b2 of the wave's units
  const int si = tid >> 4, sk = tid & 15;
  const float sv = sk < kIn && R.valid(si) ? X[R(si) * kIn + sk] : 0.f;
  f4 w1v[4];
  float b1v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w1v[q] = w1_frag(A.W1, 16 * (w + 4 * q), lane);
    b1v[q] = A.b1[16 * (w + 4 * q) + i];
  }
  float b2v[2], w30[2], w31[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int u = 16 * (w + 4 * t) + i;
    b2v[t] = A.b2[u];
    w30[t] = A.W3[u];
    w31[t] = A.W3[kH2 + u];
  }
  S[si * kLdS16 + sk] = sv;
  lds_sync32();
  // ---- layer 1
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = 16 * (w + 4 * q) + i;
    const f4 x = *(const f4*)(S + i * kLdS16 + 4 * g);
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 m = m16x4(x, w1v[q], z4);
    const float b = b1v[q];
    if (NOISE) {
      const f32x4 var = m16x4(x * x, w1v[q] * w1v[q], z4);
      float y[4];
      noisy4(seed, call, (uint32_t)R(4 * g), (uint32_t)u, skmlp::noise_k2(sd), b, m, var, 0, y);
#pragma unroll
      for (int r = 0; r < 4; ++r) H1[(4 * g + r) * kLdH1 + u] = fmaxf(y[r], 0.f);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) H1[(4 * g + r) * kLdH1 + u] = fmaxf(m[r] + b, 0.f);
    }
  }
  lds_sync32();
  // ---- layer 2 (n-tiles w, w + 4) and the layer-3 partials of the wave's units
  // per row 4g + r: the layer-3 dot products (and their variances) over this lane's two units
  float pm0[4] = {0.f, 0.f, 0.f, 0.f}, pm1[4] = {0.f, 0.f, 0.f, 0.f}, pv0[4] = {0.f, 0.f, 0.f, 0.f},
        pv1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int nt = w + 4 * t, u = 16 * nt + i;
    f32x4 m, var;
    if (NOISE) {
      g16_xwT256_mv(m, var, H1, A.W2, 16 * nt, lane);
    } else {
      m = g16_xwT256(H1, kLdH1, A.W2, kALd, 16 * nt, lane);
    }
    float yn[4];
    if (NOISE) noisy4(seed, call, (uint32_t)R(4 * g), (uint32_t)(kH1 + u), skmlp::noise_k2(sd), b2v[t], m, var, 0, yn);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float y = NOISE ? yn[r] : m[r] + b2v[t];
      const float h = fmaxf(y, 0.f);
      pm0[r] += h * w30[t];
      pm1[r] += h * w31[t];
      if (NOISE) {
        pv0[r] += h * h * w30[t] * w30[t];
        pv1[r] += h * h * w31[t] * w31[t];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const f4 v = {rowsum16(pm0[r]), rowsum16(pm1[r]), NOISE ? rowsum16(pv0[r]) : 0.f, NOISE ? rowsum16(pv1[r]) : 0.f};
    if (i == 15) MP[w][4 * g + r] = v;
  }
  lds_sync32();
  // ---- layer 3, tanh, action noise: one thread per row
  if (tid < kR && R.valid(tid)) {
    const int64_t row = R(tid);
    const f4 v = (MP[0][tid] + MP[1][tid]) + (MP[2][tid] + MP[3][tid]);
    const float b30 = A.b3[0], b31 = A.b3[1];
    float y0 = v.x + b30, y1 = v.y + b31;
    if (NOISE) {
      float z[4];
      normals4(seed, call, (uint32_t)row, (uint32_t)(kH1 + kH2), z);
      y0 += sd * __builtin_amdgcn_sqrtf(v.z + b30 * b30) * z[0];
      y1 += sd * __builtin_amdgcn_sqrtf(v.w + b31 * b31) * z[1];
    }
    float o0 = tanhf(y0), o1 = tanhf(y1);
    if (action_sd != 0.f) {
      float z[4];
      normals4(seed, call, (uint32_t)row, (uint32_t)(kH1 + kH2 + 1), z);
      o0 += action_sd * z[0];
      o1 += action_sd * z[1];
    }
    *(float2*)(out + row * 2) = make_float2(o0, o1);
    if (act_lds) act_lds[tid] = make_float2(o0, o1);
  }
}

template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads) k_actor_fwd16(const float* __restrict__ aflat,
                                                             const float* __restrict__ X, float* __restrict__ out,
                                                             int64_t rows, float sd, float action_sd, uint64_t seed,
                                                             uint64_t* __restrict__ call_ctr) {
  __shared__ __attribute__((aligned(16))) float S[kR * kLdS16];
  __shared__ __attribute__((aligned(16))) float H1[kR * kLdH1];
  __shared__ __attribute__((aligned(16))) f4 MP[4][kR];  // per wave and row: {m0, m1, v0, v1} of layer 3
  const Net A = net_of(aflat, kALd, 2);
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call = draws ? call_ctr[0] + 1 : 0;
  actor_tile16<NOISE>(A, X, out, RowsContig{(int64_t)blockIdx.x * kR, rows}, sd, action_sd, seed, call, S, H1, MP,
                      nullptr);
  if (draws) {
    __syncthreads();
    advance_call32(call_ctr, call, gridDim.x);
  }
}

// The self-play tick's act + step on 16-row tiles (SK_ACT16, the acting
// launch below kAct16MaxEnvs games): a workgroup owns 8 games, their 16
// player rows (RowsPlayers8) through actor_tile16, then wave 0's first 16
// lanes finish k_step_split's tick (split_load / split_finish) as
// act_step32's wave 0 does for 16 games.  Equal, bit for bit, to
// sk_actor_forward_f32 with 16-row tiles (SK_FWD16=1) + sk_env_step_insert.
struct RowsPlayers8 {
  int64_t g0, n;
  __device__ int64_t operator()(int i) const { return i < 8 ? g0 + i : n + g0 + (i - 8); }
  __device__ bool valid(int i) const { return g0 + (i & 7) < n; }
};
template <bool NOISE>
__device__ __forceinline__ void act_step16(const float* __restrict__ aflat, float* __restrict__ act_out, float sd,
                                           float action_sd, uint64_t seed, uint64_t* __restrict__ call_ctr,
                                           sk::StepArgs a, sk::Cfg c, float* lds, unsigned nb) {
  float* S = lds;
  float* H1 = S + kR * kLdS16;
  f4(*MP)[kR] = (f4(*)[kR])(H1 + kR * kLdH1);
  float2* sAct = (float2*)(MP[4]);
  const int lane = threadIdx.x & 63;
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const int64_t g0 = (int64_t)blockIdx.x * 8;
  sk_counters* slot = a.ctr ? a.ctr + (size_t)blockIdx.x * SK_CTR_STRIDE : nullptr;
  sk::StepLane L;
  if (w0) L = sk::split_load(a, lane < 16 ? 2 * g0 + lane : 2 * a.n, slot);
  const Net A = net_of(aflat, kALd, 2);
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call = draws ? call_ctr[0] + 1 : 0;
  actor_tile16<NOISE>(A, a.acting_obs, act_out, RowsPlayers8{g0, a.n}, sd, action_sd, seed, call, S, H1, MP, sAct);
  __syncthreads();
  if (w0) {
    const float2 act = lane < 16 ? sAct[(lane & 1) * 8 + (lane >> 1)] : make_float2(0.f, 0.f);
    sk::split_finish(a, c, L, act, slot);
  }
  if (draws) {
    __syncthreads();
    advance_call32(call_ctr, call, nb);
  }
}
constexpr size_t kActStep16Lds = kActorTile16Lds + 16 * sizeof(float2);
template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads) k_act_step16(const float* __restrict__ aflat, float* __restrict__ act_out,
                                                            float sd, float action_sd, uint64_t seed,
                                                            uint64_t* __restrict__ call_ctr, sk::StepArgs a,
                                                            sk::Cfg c) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  act_step16<NOISE>(aflat, act_out, sd, action_sd, seed, call_ctr, a, c, smem_sl, gridDim.x);
}

// A gradient step's backward launch with the next acting tick beside it
// (the fused overlapped learner tick: sk_critic_grad_f32_sampled_step carries
// it in the critic's backward, sk_actor_grad_f32_step in the actor's):
// workgroups [0, GA) run act_step32 (k_act_step32's 16 games each), the rest
// grad_slice_bwd<MODE> (k_grad_slice_bwd's workgroup blockIdx - GA).  The
// two share no data: the backward reads the minibatch, the nets and the
// forward's z2; the acting half reads the actor and the observations and
// writes the env, the actions and the ring (the minibatch was gathered
// before, excluding the rows this insert writes).  LDS is the larger of the
// two layouts: two workgroups per CU (the critic's 78,544 B twice fill the
// CU's 160 KiB).
constexpr size_t bwd_act_lds(int mode, bool a16 = false) {
  return (a16 ? kActStep16Lds : kActStepLds) > sl_bwd_lds(mode) ? (a16 ? kActStep16Lds : kActStepLds)
                                                                  : sl_bwd_lds(mode);
}
static_assert(2 * bwd_act_lds(kSlCriticBoot) <= 160 * 1024 && 2 * bwd_act_lds(kSlActor) <= 160 * 1024,
              "two fused workgroups per CU");
static_assert(kSlThreads == kFwdThreads, "one workgroup size for both halves");
template <int MODE, bool NOISE, bool A16>
__global__ void __launch_bounds__(kFwdThreads) k_bwd_act_step32(SK_SLICE_BWD_PARAMS, unsigned GA,
                                                                const float* __restrict__ aflat,
                                                                const char* __restrict__ apack,
                                                                float* __restrict__ act_out, float sd, float action_sd,
                                                                uint64_t aseed, uint64_t* __restrict__ acall_ctr,
                                                                sk::StepArgs a, sk::Cfg c) {
  extern __shared__ __attribute__((aligned(16))) float smem_sl[];
  if (A16 && blockIdx.x < GA) {
    act_step16<NOISE>(aflat, act_out, sd, action_sd, aseed, acall_ctr, a, c, smem_sl, GA);
  } else if (blockIdx.x < GA) {
    act_step32<NOISE>(aflat, apack, act_out, sd, action_sd, aseed, acall_ctr, a, c, (char*)smem_sl, GA);
  } else {
    grad_slice_bwd<MODE>((int)(blockIdx.x - GA), smem_sl, SK_SLICE_BWD_ARGS);
  }
}

int64_t subtiles_per_wg32(int64_t B) {  // 16-row sub-tiles; <= 256 workgroups, >= 1 sub-tile each
  const int64_t tiles = (B + kR - 1) / kR;
  return (tiles + 255) / 256;
}

template <typename K>
void set_lds32(K kernel, size_t bytes) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// 16-row actor forward up to 4,096 rows (at most half the CUs busy with 32-row
// tiles; profiles/r03u_actor_fwd.jsonl: 2,048 rows 9.6 -> 6.6 us, but 8,192
// rows 10.4 -> 10.9 us); SK_FWD16=0 / 1 forces the 32- / 16-row kernel
// the acting launch on 16-row tiles (8 games per workgroup): SK_ACT16=1 / 0
// forces, else up to kAct16MaxEnvs games
constexpr int64_t kAct16MaxEnvs = 0;
bool act16_games(int64_t n) {
  const char* e = getenv("SK_ACT16");
  const int v = e && *e ? atoi(e) : -1;
  return v == 1 || (v != 0 && n <= kAct16MaxEnvs);
}

bool fwd16_rows(int64_t rows) {
  const char* e = getenv("SK_FWD16");
  const int v = e && *e ? atoi(e) : -1;
  return v == 1 || (v != 0 && rows <= 4096);
}

// the sliced schedule: automatic up to kSliceMaxTiles row tiles (batch 512);
// SK_SLICE32=0 never, =1 at every batch (A/B and tests)
constexpr int64_t kSliceMaxTiles = 32;
int slice_env() {  // read at every call: tests switch it per case
  const char* e = getenv("SK_SLICE32");
  return e && *e ? atoi(e) : -1;
}

template <int MODE>
int launch_sliced(const float* f0, const float* f1, const float* f2, const float* S, const float* S2,
                  const float* A, const float* Y, const float* R, const float* D, float gamma, int64_t B,
                  int64_t key_row0, float scale, uint64_t seed, const int64_t* call_ctr, float* partials,
                  float* scratch, int64_t w1_rows, float* step_ctr, int n_steps, float* stat_out, uint8_t* mask_out,
                  hipStream_t st, RingSample rs = RingSample{}, const sk::ActStepJob* job = nullptr) {
  static bool attr = false;
  if (!attr) {
    set_lds32(k_grad_slice_fwd<MODE>, sl_fwd_lds(MODE));
    set_lds32(k_grad_slice_bwd<MODE>, sl_bwd_lds(MODE));
    set_lds32(k_bwd_act_step32<MODE, true, false>, bwd_act_lds(MODE));
    set_lds32(k_bwd_act_step32<MODE, false, false>, bwd_act_lds(MODE));
    set_lds32(k_bwd_act_step32<MODE, true, true>, bwd_act_lds(MODE, true));
    set_lds32(k_bwd_act_step32<MODE, false, true>, bwd_act_lds(MODE, true));
    attr = true;
  }
  float* Z = scratch + w1_rows * kW1Part;
  const unsigned G = (unsigned)w1_rows;  // row tiles x slices
  k_grad_slice_fwd<MODE><<<G * sl_planes(MODE), kSlThreads, sl_fwd_lds(MODE), st>>>(f0, f1, f2, S, S2, B, key_row0, seed, call_ctr, Z,
                                                                  step_ctr, n_steps, rs);
  if (job) {  // the acting tick's workgroups first, then the backward's
    sk::StepArgs a = job->a;
    const bool a16 = act16_games(a.n);
    const unsigned GA = (unsigned)(a16 ? (a.n + 7) / 8 : (a.n + 15) / 16);
    a.grid_blocks = GA;
    const size_t lds = bwd_act_lds(MODE, a16);
#define SK_BWD_ACT(NZ, A6)                                                                                          \
  k_bwd_act_step32<MODE, NZ, A6><<<GA + G * kBwdH, kFwdThreads, lds, st>>>(                                         \
      f0, f1, f2, S, A, Y, R, D, gamma, B, key_row0, scale, seed, call_ctr, Z, partials, scratch, stat_out, mask_out, \
      GA, job->aflat, job->apack, job->act_out, NZ ? job->sd : 0.f, job->action_sd, job->seed, job->call_ctr, a, \
      job->c)
    if (job->sd != 0.f) {
      if (a16) SK_BWD_ACT(true, true);
      else SK_BWD_ACT(true, false);
    } else {
      if (a16) SK_BWD_ACT(false, true);
      else SK_BWD_ACT(false, false);
    }
#undef SK_BWD_ACT
    return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
  }
  k_grad_slice_bwd<MODE><<<G * kBwdH, kSlThreads, sl_bwd_lds(MODE), st>>>(f0, f1, f2, S, A, Y, R, D, gamma, B, key_row0,
                                                                  scale, seed, call_ctr, Z, partials, scratch,
                                                                  stat_out, mask_out);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

// the split pack (sk_split.hpp) from the actor's flat fp32 parameters: one
// thread per plane element (the W1 padding k = 12..15 written as zero)
__global__ void k_split_pack32(const float* __restrict__ aflat, char* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  short* b;
  int idx, plane;
  float v;
  if (t < sksplit::kW1Plane) {
    idx = t;
    const int j = t & 7, lane = (t >> 3) & 63, nt = t >> 9;
    const int n = 32 * nt + (lane & 31), k = 8 * (lane >> 5) + j;
    v = k < kIn ? aflat[kPW1 + n * kIn + k] : 0.f;
    b = (short*)(out + sksplit::kOffW1);
    plane = sksplit::kW1Plane;
  } else if (t < sksplit::kW1Plane + sksplit::kW2Plane) {
    idx = t - sksplit::kW1Plane;
    const int j = idx & 7, lane = (idx >> 3) & 63, kk = (idx >> 9) & 15, nt = idx >> 13;
    const int o = 32 * nt + (lane & 31), i = 16 * kk + 8 * (lane >> 5) + j;
    v = aflat[kPW2 + o * kALd + i];
    b = (short*)(out + sksplit::kOffW2);
    plane = sksplit::kW2Plane;
  } else {
    return;
  }
  short hi, mid, lo, sq;
  sksplit::split4(v, hi, mid, lo, sq);
  b[idx] = hi;
  b[plane + idx] = mid;
  b[2 * plane + idx] = lo;
  b[3 * plane + idx] = sq;
}

}  // namespace

// csrc/sk_replay.hip
int replay_sample_excl(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                       int64_t batch, float* s, float* a, float* r, float* s2, float* d, int64_t excl,
                       hipStream_t stream);

// the self-play tick launch (sk_env_act_step, csrc/sk_engine.hip): a.n % 4 == 0
int sk_launch_act_step32(const float* aflat, const void* apack, float* act_out, float sd, float action_sd,
                         uint64_t seed, uint64_t* call_ctr, const sk::StepArgs& a, const sk::Cfg& c, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    set_lds32(k_act_step32<true>, kActStepLds);
    set_lds32(k_act_step32<false>, kActStepLds);
    attr = true;
  }
  if (act16_games(a.n)) {
    const unsigned G8 = (unsigned)((a.n + 7) / 8);
    if (sd != 0.f)
      k_act_step16<true><<<G8, kFwdThreads, kActStep16Lds, st>>>(aflat, act_out, sd, action_sd, seed, call_ctr, a, c);
    else
      k_act_step16<false><<<G8, kFwdThreads, kActStep16Lds, st>>>(aflat, act_out, 0.f, action_sd, seed, call_ctr, a,
                                                                  c);
    return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
  }
  if (!apack || (((uintptr_t)apack) & 15)) return SK_EINVAL;  // the 32-row tile reads the split pack
  const unsigned G = (unsigned)((a.n + 15) / 16);
  const char* pk = (const char*)apack;
  if (sd != 0.f)
    k_act_step32<true><<<G, kFwdThreads, kActStepLds, st>>>(aflat, pk, act_out, sd, action_sd, seed, call_ctr, a, c);
  else
    k_act_step32<false><<<G, kFwdThreads, kActStepLds, st>>>(aflat, pk, act_out, 0.f, action_sd, seed, call_ctr, a,
                                                             c);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

// the reference rule's episode collection (sk_env_act_episode, csrc/sk_engine.hip): a.n % 4 == 0
int sk_launch_act_episode32(const float* aflat, const void* apack, float sd, float action_sd, uint64_t seed,
                            uint64_t* call_ctr, const sk::StepArgs& a, const sk::Cfg& c, float* states,
                            float* actions, float* rewards, int32_t* lengths, int n_ticks, hipStream_t st) {
  constexpr size_t lds = kActStepLds + 16;
  static bool attr = false;
  if (!attr) {
    set_lds32(k_act_episode32<true>, lds);
    set_lds32(k_act_episode32<false>, lds);
    attr = true;
  }
  if (!apack || (((uintptr_t)apack) & 15)) return SK_EINVAL;
  const unsigned G = (unsigned)((a.n + 15) / 16);
  const EpisodeArgs ep{states, actions, rewards, lengths, n_ticks};
  const char* pk = (const char*)apack;
  if (sd != 0.f)
    k_act_episode32<true><<<G, kFwdThreads, lds, st>>>(aflat, pk, sd, action_sd, seed, call_ctr, a, c, ep);
  else
    k_act_episode32<false><<<G, kFwdThreads, lds, st>>>(aflat, pk, 0.f, action_sd, seed, call_ctr, a, c, ep);
  if (hipGetLastError() != hipSuccess) return SK_EHIP;
  const bool draws = (sd != 0.f || action_sd != 0.f) && call_ctr;
  k_episode_finish<<<1, 256, 0, st>>>(lengths, a.n, a.step, draws ? call_ctr : nullptr);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

extern "C" {

int64_t sk_update_scratch_f32(int64_t batch, int64_t* w1_rows) {
  int64_t rows = 0, floats = 0;
  if (batch > 0 && batch <= ((int64_t)1 << 30)) {
    const int64_t RT = (batch + kR - 1) / kR;
    const int m = slice_env();
    if (m == 1 || (m != 0 && RT <= kSliceMaxTiles)) {
      rows = RT * kSlices;
      floats = rows * kW1Part + RT * 3 * kZPlane;
    }
  }
  if (w1_rows) *w1_rows = rows;
  return floats;
}

int64_t sk_update_partials_f32(int64_t batch) {
  if (batch <= 0) return 0;
  if (sk_update_scratch_f32(batch, nullptr) > 0) return (batch + kR - 1) / kR;  // sliced: one row per row tile
  const int64_t spw = subtiles_per_wg32(batch);
  return ((batch + kR - 1) / kR + spw - 1) / spw;
}

static int critic_f32(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                      const float* next_obs, const float* rewards, const float* done, float gamma,
                      const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                      int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                      float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                      uint8_t* dropout_mask, float* scratch, const sk::ActStepJob* job, void* stream) {
  const bool boot = target_actor_flat != nullptr;
  if (boot && (!target_critic_flat || !next_obs || !rewards || !done)) return SK_EINVAL;
  if (!boot && !targets) return SK_EINVAL;
  if (!critic_flat || !obs || !actions || !call_counter || !partials || batch <= 0) return SK_EINVAL;
  if (row_offset < 0 || (row_offset & 3)) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  int64_t w1_rows = 0;
  if (sk_update_scratch_f32(batch, &w1_rows) > 0) {
    if (!scratch) return SK_EINVAL;
    if (boot)
      return launch_sliced<kSlCriticBoot>(critic_flat, target_actor_flat, target_critic_flat, obs, next_obs, actions,
                                          nullptr, rewards, done, gamma, batch, row_offset, grad_scale, seed,
                                          call_counter, partials, scratch, w1_rows, step_counters, n_steps, loss_sum,
                                          dropout_mask, (hipStream_t)stream, RingSample{}, job);
    return launch_sliced<kSlCriticY>(critic_flat, nullptr, nullptr, obs, nullptr, actions, targets, nullptr, nullptr,
                                     0.f, batch, row_offset, grad_scale, seed, call_counter, partials, scratch,
                                     w1_rows, step_counters, n_steps, loss_sum, dropout_mask, (hipStream_t)stream,
                                     RingSample{}, job);
  }
  static bool attr = false;
  if (!attr) {
    set_lds32(k_critic_grad32<true>, kLdsGrad32);
    set_lds32(k_critic_grad32<false>, kLdsGrad32);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg32(batch);
  const unsigned G = (unsigned)sk_update_partials_f32(batch);
  auto kern = boot ? k_critic_grad32<true> : k_critic_grad32<false>;
  kern<<<G, kThreads, kLdsGrad32, (hipStream_t)stream>>>(
      critic_flat, obs, actions, targets, batch, row_offset, (int)spw, grad_scale, seed, call_counter, partials,
      step_counters, n_steps, loss_sum, dropout_mask, next_obs, rewards, done, gamma, target_actor_flat,
      target_critic_flat);
  if (hipGetLastError() != hipSuccess) return SK_EHIP;
  if (!job) return SK_OK;
  return sk_launch_act_step32(job->aflat, job->apack, job->act_out, job->sd, job->action_sd, job->seed, job->call_ctr, job->a,
                              job->c, (hipStream_t)stream);
}

int sk_critic_grad_f32(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                       const float* next_obs, const float* rewards, const float* done, float gamma,
                       const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                       int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                       float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                       uint8_t* dropout_mask, float* scratch, void* stream) {
  return critic_f32(critic_flat, obs, actions, targets, next_obs, rewards, done, gamma, target_actor_flat,
                    target_critic_flat, batch, row_offset, grad_scale, seed, call_counter, partials, step_counters,
                    n_steps, loss_sum, dropout_mask, scratch, nullptr, stream);
}

int sk_critic_grad_f32_step(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                            const float* next_obs, const float* rewards, const float* done, float gamma,
                            const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                            int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                            float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                            uint8_t* dropout_mask, float* scratch, const sk_step_job* job, void* stream) {
  if (!job) return SK_EINVAL;
  sk::ActStepJob j;
  std::memcpy(&j, job, sizeof(j));
  if (j.magic != sk::kActStepJobMagic) return SK_EINVAL;
  return critic_f32(critic_flat, obs, actions, targets, next_obs, rewards, done, gamma, target_actor_flat,
                    target_critic_flat, batch, row_offset, grad_scale, seed, call_counter, partials, step_counters,
                    n_steps, loss_sum, dropout_mask, scratch, &j, stream);
}

static int critic_sampled(const float* critic_flat, const sk_ring_sample* q, float gamma,
                          const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                          int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                          float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                          uint8_t* dropout_mask, float* scratch, const sk::ActStepJob* job, void* stream) {
  if (!q || !q->ring || !q->total || !q->s || !q->a || !q->r || !q->s2 || !q->d || q->capacity <= 0) return SK_EINVAL;
  if (q->exclude < 0 || q->exclude >= q->capacity) return SK_EINVAL;  // as sk_replay_sample_excl
  if ((((uintptr_t)q->ring) & 15) || (((uintptr_t)q->s) & 15) || (((uintptr_t)q->s2) & 15) || (((uintptr_t)q->a) & 7))
    return SK_EINVAL;
  const bool boot = target_actor_flat != nullptr;
  if (boot && !target_critic_flat) return SK_EINVAL;
  if (!critic_flat || !call_counter || !partials || batch <= 0) return SK_EINVAL;
  if (row_offset < 0 || (row_offset & 3)) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  int64_t w1_rows = 0;
  if (sk_update_scratch_f32(batch, &w1_rows) > 0) {
    if (!scratch) return SK_EINVAL;
    const RingSample rs{q->ring, q->capacity, q->total, q->seed, q->draw, q->s, q->a, q->r, q->s2, q->d, q->exclude};
    if (boot)
      return launch_sliced<kSlCriticBoot>(critic_flat, target_actor_flat, target_critic_flat, q->s, q->s2, q->a,
                                          nullptr, q->r, q->d, gamma, batch, row_offset, grad_scale, seed,
                                          call_counter, partials, scratch, w1_rows, step_counters, n_steps, loss_sum,
                                          dropout_mask, (hipStream_t)stream, rs, job);
    return launch_sliced<kSlCriticY>(critic_flat, nullptr, nullptr, q->s, nullptr, q->a, q->r, nullptr, nullptr, 0.f,
                                     batch, row_offset, grad_scale, seed, call_counter, partials, scratch, w1_rows,
                                     step_counters, n_steps, loss_sum, dropout_mask, (hipStream_t)stream, rs, job);
  }
  // unsliced batches: the gather as its own launch
  const int rc = replay_sample_excl(q->ring, q->capacity, q->total, q->seed, q->draw, batch, q->s, q->a, q->r, q->s2,
                                    q->d, q->exclude, (hipStream_t)stream);
  if (rc != SK_OK) return rc;
  const int rc2 = sk_critic_grad_f32(critic_flat, q->s, q->a, boot ? nullptr : q->r, boot ? q->s2 : nullptr,
                                     boot ? q->r : nullptr, boot ? q->d : nullptr, gamma, target_actor_flat,
                                     target_critic_flat, batch, row_offset, grad_scale, seed, call_counter, partials,
                                     step_counters, n_steps, loss_sum, dropout_mask, scratch, stream);
  if (rc2 != SK_OK || !job) return rc2;
  return sk_launch_act_step32(job->aflat, job->apack, job->act_out, job->sd, job->action_sd, job->seed, job->call_ctr, job->a,
                              job->c, (hipStream_t)stream);
}

int sk_critic_grad_f32_sampled(const float* critic_flat, const sk_ring_sample* q, float gamma,
                               const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                               int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                               float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                               uint8_t* dropout_mask, float* scratch, void* stream) {
  return critic_sampled(critic_flat, q, gamma, target_actor_flat, target_critic_flat, batch, row_offset, grad_scale,
                        seed, call_counter, partials, step_counters, n_steps, loss_sum, dropout_mask, scratch, nullptr,
                        stream);
}

int sk_critic_grad_f32_sampled_step(const float* critic_flat, const sk_ring_sample* q, float gamma,
                                    const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                                    int64_t row_offset, float grad_scale, uint64_t seed,
                                    const int64_t* call_counter, float* partials, float* step_counters,
                                    int32_t n_steps, float* loss_sum, uint8_t* dropout_mask, float* scratch,
                                    const sk_step_job* job, void* stream) {
  if (!job) return SK_EINVAL;
  sk::ActStepJob j;
  std::memcpy(&j, job, sizeof(j));
  if (j.magic != sk::kActStepJobMagic) return SK_EINVAL;
  return critic_sampled(critic_flat, q, gamma, target_actor_flat, target_critic_flat, batch, row_offset, grad_scale,
                        seed, call_counter, partials, step_counters, n_steps, loss_sum, dropout_mask, scratch, &j,
                        stream);
}

int sk_actor_grad_f32(const float* actor_flat, const float* critic_flat, const float* obs, int64_t batch,
                      float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                      float* scratch, void* stream) {
  if (!actor_flat || !critic_flat || !obs || !partials || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  int64_t w1_rows = 0;
  if (sk_update_scratch_f32(batch, &w1_rows) > 0) {
    if (!scratch) return SK_EINVAL;
    return launch_sliced<kSlActor>(actor_flat, critic_flat, nullptr, obs, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   0.f, batch, 0, loss_scale, 0, nullptr, partials, scratch, w1_rows, step_counters,
                                   n_steps, q_sum, nullptr, (hipStream_t)stream);
  }
  static bool attr = false;
  if (!attr) {
    set_lds32(k_actor_grad32, kLdsGrad32);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg32(batch);
  const unsigned G = (unsigned)sk_update_partials_f32(batch);
  k_actor_grad32<<<G, kThreads, kLdsGrad32, (hipStream_t)stream>>>(actor_flat, critic_flat, obs, batch, (int)spw,
                                                                  loss_scale, partials, step_counters, n_steps,
                                                                  q_sum);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_grad_f32_step(const float* actor_flat, const float* critic_flat, const float* obs, int64_t batch,
                           float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                           float* scratch, const sk_step_job* job, void* stream) {
  if (!job) return SK_EINVAL;
  sk::ActStepJob j;
  std::memcpy(&j, job, sizeof(j));
  if (j.magic != sk::kActStepJobMagic) return SK_EINVAL;
  if (!actor_flat || !critic_flat || !obs || !partials || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  int64_t w1_rows = 0;
  if (sk_update_scratch_f32(batch, &w1_rows) > 0) {
    if (!scratch) return SK_EINVAL;
    return launch_sliced<kSlActor>(actor_flat, critic_flat, nullptr, obs, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   0.f, batch, 0, loss_scale, 0, nullptr, partials, scratch, w1_rows, step_counters,
                                   n_steps, q_sum, nullptr, (hipStream_t)stream, RingSample{}, &j);
  }
  const int rc = sk_actor_grad_f32(actor_flat, critic_flat, obs, batch, loss_scale, partials, step_counters, n_steps,
                                   q_sum, scratch, stream);
  if (rc != SK_OK) return rc;
  return sk_launch_act_step32(j.aflat, j.apack, j.act_out, j.sd, j.action_sd, j.seed, j.call_ctr, j.a, j.c,
                              (hipStream_t)stream);
}

int sk_actor_forward_f32(const float* actor_flat, const void* actor_pack, const float* obs, float* actions,
                         int64_t rows, float noise_sd, float action_sd, uint64_t seed, uint64_t* call_counter,
                         void* stream) {
  if (!actor_flat || !obs || !actions || rows <= 0) return SK_EINVAL;
  if ((((uintptr_t)actions) & 7)) return SK_EINVAL;
  if (fwd16_rows(rows)) {
    const unsigned G16 = (unsigned)((rows + kR - 1) / kR);
    if (noise_sd != 0.f)
      k_actor_fwd16<true><<<G16, kFwdThreads, 0, (hipStream_t)stream>>>(actor_flat, obs, actions, rows, noise_sd,
                                                                          action_sd, seed, call_counter);
    else
      k_actor_fwd16<false><<<G16, kFwdThreads, 0, (hipStream_t)stream>>>(actor_flat, obs, actions, rows, 0.f,
                                                                           action_sd, seed, call_counter);
    return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
  }
  if (!actor_pack || (((uintptr_t)actor_pack) & 15)) return SK_EINVAL;  // the 32-row tile reads the split pack
  static bool attr = false;
  if (!attr) {
    set_lds32(k_actor_fwd32<true>, kActorTileLds);
    set_lds32(k_actor_fwd32<false>, kActorTileLds);
    attr = true;
  }
  const unsigned G = (unsigned)((rows + 31) / 32);
  const char* pk = (const char*)actor_pack;
  if (noise_sd != 0.f)
    k_actor_fwd32<true><<<G, kFwdThreads, kActorTileLds, (hipStream_t)stream>>>(actor_flat, pk, obs, actions, rows,
                                                                                 noise_sd, action_sd, seed,
                                                                                 call_counter);
  else
    k_actor_fwd32<false><<<G, kFwdThreads, kActorTileLds, (hipStream_t)stream>>>(actor_flat, pk, obs, actions, rows,
                                                                                  0.f, action_sd, seed, call_counter);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

size_t sk_actor_split_pack_bytes(void) { return sksplit::kBytes; }

int sk_actor_split_pack_f32(const float* actor_flat, void* actor_pack, void* stream) {
  if (!actor_flat || !actor_pack || (((uintptr_t)actor_pack) & 15)) return SK_EINVAL;
  const int n = sksplit::kW1Plane + sksplit::kW2Plane;  // one thread per plane-0 element
  k_split_pack32<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(actor_flat, (char*)actor_pack);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

}  // extern "C"

#ifdef SK_TRACE32
// diagnostic builds only (not in include/skillshot.h): [2 wg][32 points][memtime, realtime]
extern "C" int sk_debug_trace32(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk_trace32), sizeof(g_sk_trace32)) == hipSuccess ? SK_OK : SK_EHIP;
}
#endif
