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

#include "../../include/skillshot.h"
#include "sk_partial.hpp"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));  // W2 rows of the critic are 8-B aligned

#ifndef UNROLL_XW
#define UNROLL_XW 4
#endif
constexpr int kIn = 12, kH1 = 256, kH2 = 128;
constexpr int kLdS = 36, kLdH1 = 260, kLdH2 = 132;  // LDS row strides (floats): 16-B aligned, banks rotated
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

__device__ __forceinline__ f32x16 mf(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mf4(f4 a, f4 b, f32x16 c) {
  c = mf(a.x, b.x, c);
  c = mf(a.y, b.y, c);
  c = mf(a.z, b.z, c);
  return mf(a.w, b.w, c);
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

// ------------------------------------------------------------------ GEMM tiles
// acc[i][j] += sum_{k0 <= k < k0+kc} X[i][k] W[n0 + j][k]: X in LDS row-major,
// W global row-major (ldw); kc a multiple of 8
// Software-pipelined: the weight loads of the next 4 steps (32 k) are in
// flight while the MFMAs of the current 4 run (the weights come from L2 and
// would otherwise stall both waves of a SIMD at every batch).
template <int KC>
__device__ __forceinline__ f32x16 gemm_xwT_p(f32x16 acc, const float* X, int ldx, gfp W, int ldw, int n0,
                                             int k0, int lane) {
  static_assert(KC % 32 == 0, "KC: multiple of 32");
  const int i = lane & 31, h = lane >> 5;
  const float* xr = X + i * ldx + k0 + 4 * h;
  const gfp wr = W + (size_t)(n0 + i) * ldw + k0 + 4 * h;
  f4 wn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + 8 * t);
#pragma unroll
  for (int k = 0; k < KC; k += 32) {
    f4 wc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wc[t] = wn[t];
    if (k + 32 < KC) {
#pragma unroll
      for (int t = 0; t < 4; ++t) wn[t] = *(gf4u)(wr + k + 32 + 8 * t);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = mf4(*(const f4*)(xr + k + 8 * t), wc[t], acc);
  }
  return acc;
}
__device__ __forceinline__ f32x16 gemm_xwT(f32x16 acc, const float* X, int ldx, gfp W, int ldw, int n0,
                                           int k0, int kc, int lane) {
  if (kc == 128) return gemm_xwT_p<128>(acc, X, ldx, W, ldw, n0, k0, lane);
  if (kc == 256) return gemm_xwT_p<256>(acc, X, ldx, W, ldw, n0, k0, lane);
  const int i = lane & 31, h = lane >> 5;
  const float* xr = X + i * ldx + k0 + 4 * h;
  const gfp wr = W + (size_t)(n0 + i) * ldw + k0 + 4 * h;
#pragma unroll UNROLL_XW
  for (int k = 0; k < kc; k += 8) acc = mf4(*(const f4*)(xr + k), *(gf4u)(wr + k), acc);
  return acc;
}
// mean and variance GEMMs of parameter noise in one pass: every operand load
// feeds both (x w and x^2 w^2: two independent accumulator chains per wave)
__device__ __forceinline__ void gemm_xwT_mv(f32x16& m, f32x16& v, const float* X, int ldx, gfp W, int ldw,
                                            int n0, int k0, int kc, int lane) {
  const int i = lane & 31, h = lane >> 5;
  const float* xr = X + i * ldx + k0 + 4 * h;
  const gfp wr = W + (size_t)(n0 + i) * ldw + k0 + 4 * h;
#pragma unroll 4
  for (int k = 0; k < kc; k += 8) {
    const f4 x = *(const f4*)(xr + k);
    const f4 w = *(gf4u)(wr + k);
    m = mf4(x, w, m);
    v = mf4(x * x, w * w, v);
  }
}
// layer 1 (K = 12): k 0..7 by both halves, k 8..11 by half 0 (half 1's
// 12..15 are zero operands, never loaded)
template <bool SQ>
__device__ __forceinline__ f32x16 gemm_l1(const float* S, gfp W1, int n0, int lane) {
  const int i = lane & 31, h = lane >> 5;
  f4 x0 = *(const f4*)(S + i * kLdS + 4 * h);
  f4 w0 = *(gf4u)(W1 + (n0 + i) * kIn + 4 * h);
  f4 x1 = {0.f, 0.f, 0.f, 0.f}, w1 = {0.f, 0.f, 0.f, 0.f};
  if (h == 0) {
    x1 = *(const f4*)(S + i * kLdS + 8);
    w1 = *(gf4u)(W1 + (n0 + i) * kIn + 8);
  }
  if (SQ) {
    x0 *= x0;
    w0 *= w0;
    x1 *= x1;
    w1 *= w1;
  }
  f32x16 acc = {0};
  acc = mf4(x0, w0, acc);
  return mf4(x1, w1, acc);
}
// acc[i][j] += sum_{k0 <= u < k0+kc} DZ[i][u] W[u][n0 + j]: DZ in LDS
// row-major, W global row-major (ldw), read down its columns (coalesced)
__device__ __forceinline__ f32x16 gemm_xw(f32x16 acc, const float* DZ, int ldz, gfp W, int ldw, int n0,
                                          int k0, int kc, int lane) {
  const int i = lane & 31, h = lane >> 5;
  const float* zr = DZ + i * ldz + k0 + 4 * h;
  const gfp wc = W + (size_t)(k0 + 4 * h) * ldw + n0 + i;
  // pipelined as gemm_xwT_p: 4 steps (16 column loads) in flight ahead
  f4 bn[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    bn[t] = f4{wc[(8 * t + 0) * ldw], wc[(8 * t + 1) * ldw], wc[(8 * t + 2) * ldw], wc[(8 * t + 3) * ldw]};
  for (int k = 0; k < kc; k += 32) {
    f4 bc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) bc[t] = bn[t];
    if (k + 32 < kc) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = k + 32 + 8 * t;
        bn[t] = f4{wc[(r + 0) * ldw], wc[(r + 1) * ldw], wc[(r + 2) * ldw], wc[(r + 3) * ldw]};
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = mf4(*(const f4*)(zr + k + 8 * t), bc[t], acc);
  }
  return acc;
}
// weight gradient over the 32 rows of a sub-tile:
// acc[m][n] += sum_i DZ[i][m0 + m] X[i][n0 + n] (both in LDS)
__device__ __forceinline__ f32x16 gemm_wgrad(f32x16 acc, const float* DZ, int ldz, int m0, const float* X, int ldx,
                                             int n0, int lane) {
  const int j = lane & 31, h = lane >> 5;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = k + 4 * h;
    const f4 a = {DZ[(r + 0) * ldz + m0 + j], DZ[(r + 1) * ldz + m0 + j], DZ[(r + 2) * ldz + m0 + j],
                  DZ[(r + 3) * ldz + m0 + j]};
    const f4 b = {X[(r + 0) * ldx + n0 + j], X[(r + 1) * ldx + n0 + j], X[(r + 2) * ldx + n0 + j],
                  X[(r + 3) * ldx + n0 + j]};
    acc = mf4(a, b, acc);
  }
  return acc;
}

// row reductions: thread t owns row t/16 and 8 of its 128 units; every lane
// of the 16-lane group returns the row's sum
__device__ __forceinline__ float row_dot128(const float* X, int ldx, gfp w, int ws) {
  const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += X[i * ldx + 8 * c + k] * w[(8 * c + k) * ws];
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
  return s;
}
__device__ __forceinline__ float row_sum128(const float* X, int ldx) {
  const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += X[i * ldx + 8 * c + k];
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
  return s;
}

// ------------------------------------------------------------ shared layers
// relu(S W1^T + b1) of n-tile w into H (inference; no Dropout)
__device__ __forceinline__ void layer1_relu(const float* S, const Net& n, float* H, int w, int lane) {
  const f32x16 acc = gemm_l1<false>(S, n.W1, 32 * w, lane);
  const int u = 32 * w + (lane & 31);
  const float b = n.b1[u];
#pragma unroll
  for (int v = 0; v < 16; ++v) H[drow(v, lane) * kLdH1 + u] = fmaxf(acc[v] + b, 0.f);
}

// layer 2 pre-activation over the 256 hidden inputs, split over the 8 waves:
// wave w computes n-tile w & 3 over inputs 128 (w >> 2) ..; the upper half's
// partial goes through XCH.  Returns the full sum in waves 0..3.
__device__ __forceinline__ f32x16 layer2_split(const float* H, const Net& n, float* XCH, int w, int lane) {
  const int nt = w & 3, kh = w >> 2;
  f32x16 acc = {0};
  acc = gemm_xwT(acc, H, kLdH1, n.W2, n.ld2, 32 * nt, 128 * kh, 128, lane);
  if (kh) {
#pragma unroll
    for (int v = 0; v < 16; ++v) XCH[(nt * 16 + v) * 64 + lane] = acc[v];
  }
  __syncthreads();
  if (!kh) {
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] += XCH[(nt * 16 + v) * 64 + lane];
  }
  return acc;
}

// actor layer 3: a = tanh(W3 h2 + b3) per row into ACT[32][2] (all threads)
__device__ __forceinline__ void actor_out(const float* H2, const Net& n, float* ACT) {
  const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
  const float z0 = row_dot128(H2, kLdH2, n.W3, 1);
  const float z1 = row_dot128(H2, kLdH2, n.W3 + kH2, 1);
  if (c < 2) ACT[2 * i + c] = tanhf((c ? z1 : z0) + n.b3[c]);
}

// ---------------------------------------------------------------- LDS layout
struct L32 {
  float *S, *H1, *H2, *DZ2, *DZ1, *XCH, *H1C, *QZ, *S2, *A, *Y, *DQ, *A2, *R, *D, *DZ3, *RED;
};
constexpr int kFS = 32 * kLdS, kFH1 = 32 * kLdH1, kFH2 = 32 * kLdH2, kFX = 4 * 16 * 64;
constexpr int kSmall = 64 + 32 + 32 + 64 + 32 + 32 + 64 + 8;
// critic: S, H1 (the dropped-out h1), H2, DZ2, DZ1 (aliases XCH), S2, small
constexpr size_t kLdsCritic = (size_t)(kFS + kFH1 + kFH2 + kFH2 + kFH1 + kFS + kSmall) * 4;
// actor: S, H1 (actor), H1C (critic h1; DZ1 aliases it), H2 (actor h2),
// DZ2 (also the critic's dQ/dz2), QZ, XCH, small
constexpr size_t kLdsActor = (size_t)(kFS + kFH1 + kFH1 + kFH2 + kFH2 + kFH2 + kFX + kSmall) * 4;
static_assert(kFX <= kFH1, "XCH aliases DZ1 in the critic kernel");

__device__ __forceinline__ void carve_small(L32& L, float* p) {
  L.A = p;   p += 64;
  L.Y = p;   p += 32;
  L.DQ = p;  p += 32;
  L.A2 = p;  p += 64;
  L.R = p;   p += 32;
  L.D = p;   p += 32;
  L.DZ3 = p; p += 64;
  L.RED = p;
}

// stage a sub-tile's states: S[i][k] = obs (k < 12, row < B), else 0
__device__ __forceinline__ void stage_states(float* S, const float* X, int64_t row0, int64_t B) {
  for (int t = threadIdx.x; t < 32 * kLdS; t += blockDim.x) {
    const int i = t / kLdS, k = t - i * kLdS;
    S[t] = (k < kIn && row0 + i < B) ? X[(row0 + i) * kIn + k] : 0.f;
  }
}

// ---------------------------------------------------------------- critic step
// Critic.forward in training mode + MSE backward (critic.fit,
// SkillshotLearner.py:434; DDPG.critic_step): dL/dq = grad_scale (q - y),
// grad_scale = 2 / global batch; Dropout keep-mask of global row key_row0 +
// row (rng.dropout_keep), keep -> x 1.25.  With tap (target actor): y = r +
// gamma (1 - done) Q'(s', mu'(s')) from the target nets first.
__global__ void __launch_bounds__(kThreads) k_critic_grad32(
    const float* __restrict__ cflat, const float* __restrict__ Sg, const float* __restrict__ Ag,
    const float* __restrict__ Yg, int64_t B, int64_t key_row0, int sub_per_wg, float grad_scale, uint64_t seed,
    const int64_t* __restrict__ call_ctr, float* __restrict__ partial, float* step_ctr, int n_steps,
    float* __restrict__ loss_out, uint8_t* __restrict__ mask_out, const float* __restrict__ S2g,
    const float* __restrict__ Rg, const float* __restrict__ Dg, float gamma, const float* __restrict__ taflat,
    const float* __restrict__ tcflat) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  L32 L;
  float* p = smem32;
  L.S = p;   p += kFS;
  L.H1 = p;  p += kFH1;
  L.H2 = p;  p += kFH2;
  L.DZ2 = p; p += kFH2;
  L.DZ1 = p; p += kFH1;
  L.XCH = L.DZ1;
  L.S2 = p;  p += kFS;
  carve_small(L, p);
  const int lane0 = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t call = (uint64_t)*call_ctr;
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  f32x16 gW2[4], gW1 = {0};
#pragma unroll
  for (int t = 0; t < 4; ++t) gW2[t] = f32x16{0};
  // per-unit sums over rows: thread t < 256 owns b1[t]; t < 128 b2, W2 action columns, W3
  float gb1 = 0.f, gb2 = 0.f, gwa0 = 0.f, gwa1 = 0.f, gw3 = 0.f, gb3 = 0.f, lsum = 0.f;
  const int u2 = w & 3;  // layer-2 n-tile of this wave (waves 0..3 hold the sums)
  TP32(0);
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;  // uniform across the workgroup
    const int lane = launder_lane(lane0);
    const Net C = net_of(launder(cflat), kCLd, 1);
    stage_states(L.S, Sg, row0, B);
    if (threadIdx.x < 64) L.A[threadIdx.x] = row0 + (threadIdx.x >> 1) < B ? Ag[row0 * 2 + threadIdx.x] : 0.f;
    if (taflat) {
      stage_states(L.S2, S2g, row0, B);
      if (threadIdx.x < 32) {
        const bool ok = row0 + threadIdx.x < B;
        L.R[threadIdx.x] = ok ? Rg[row0 + threadIdx.x] : 0.f;
        L.D[threadIdx.x] = ok ? Dg[row0 + threadIdx.x] : 0.f;
      }
      __syncthreads();
      TP32(1);
      // ---- bootstrap target: mu'(s') then Q'(s', mu'(s')), inference
      const Net TA = net_of(launder(taflat), kALd, 2), TC = net_of(launder(tcflat), kCLd, 1);
      layer1_relu(L.S2, TA, L.H1, w, lane);
      __syncthreads();
      {
        const f32x16 acc = layer2_split(L.H1, TA, L.XCH, w, lane);
        if (w < 4) {
          const int u = 32 * u2 + (lane & 31);
          const float b = TA.b2[u];
#pragma unroll
          for (int v = 0; v < 16; ++v) L.H2[drow(v, lane) * kLdH2 + u] = fmaxf(acc[v] + b, 0.f);
        }
      }
      __syncthreads();
      TP32(2);
      actor_out(L.H2, TA, L.A2);
      layer1_relu(L.S2, TC, L.H1, w, lane);  // H1 was last read before the previous barrier
      __syncthreads();
      {
        const f32x16 acc = layer2_split(L.H1, TC, L.XCH, w, lane);
        if (w < 4) {
          const int u = 32 * u2 + (lane & 31);
          const float b = TC.b2[u], wa0 = TC.W2[u * kCLd + kH1], wa1 = TC.W2[u * kCLd + kH1 + 1];
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            const int i = drow(v, lane);
            L.H2[i * kLdH2 + u] = fmaxf(acc[v] + b + L.A2[2 * i] * wa0 + L.A2[2 * i + 1] * wa1, 0.f);
          }
        }
      }
      __syncthreads();
      {
        const float q2 = TC.b3[0] + row_dot128(L.H2, kLdH2, TC.W3, 1);
        const int i = threadIdx.x >> 4;
        if ((threadIdx.x & 15) == 0) L.Y[i] = L.R[i] + gamma * (1.f - L.D[i]) * q2;
      }
      TP32(3);
    } else if (threadIdx.x < 32) {
      L.Y[threadIdx.x] = row0 + threadIdx.x < B ? Yg[row0 + threadIdx.x] : 0.f;
    }
    __syncthreads();
    // ---- layer 1 with Dropout: wave w -> units 32w ..
    {
      const f32x16 acc = gemm_l1<false>(L.S, C.W1, 32 * w, lane);
      const int u = 32 * w + (lane & 31);
      const float b = C.b1[u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        const uint4 r = philox(make_uint4((uint32_t)((key_row0 + row0 + i0) >> 2), (uint32_t)u, (uint32_t)call,
                                          (uint32_t)(call >> 32)),
                               (uint32_t)seed, (uint32_t)(seed >> 32));
        const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool keep = wd[q] >= 858993460u;  // P(drop) = 0.2 (Dropout(0.2), SkillshotLearner.py:105)
          const float z = fmaxf(acc[4 * g + q] + b, 0.f);
          L.H1[(i0 + q) * kLdH1 + u] = keep ? z * 1.25f : 0.f;
          if (mask_out && row0 + i0 + q < B) mask_out[(row0 + i0 + q) * kH1 + u] = keep;
        }
      }
    }
    __syncthreads();
    TP32(4);
    // ---- layer 2 (+ the two action columns) -> h2
    {
      const f32x16 acc = layer2_split(L.H1, C, L.XCH, w, lane);
      if (w < 4) {
        const int u = 32 * u2 + (lane & 31);
        const float b = C.b2[u], wa0 = C.W2[u * kCLd + kH1], wa1 = C.W2[u * kCLd + kH1 + 1];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int i = drow(v, lane);
          L.H2[i * kLdH2 + u] = fmaxf(acc[v] + b + L.A[2 * i] * wa0 + L.A[2 * i + 1] * wa1, 0.f);
        }
      }
    }
    __syncthreads();
    TP32(5);
    // ---- q, dL/dq (rows beyond B: 0)
    {
      const float q = C.b3[0] + row_dot128(L.H2, kLdH2, C.W3, 1);
      const int i = threadIdx.x >> 4;
      if ((threadIdx.x & 15) == 0) {
        const float e = row0 + i < B ? q - L.Y[i] : 0.f;
        L.DQ[i] = grad_scale * e;
        gb3 += grad_scale * e;
        lsum += e * e;
      }
    }
    __syncthreads();
    // ---- dz2 = dq W3 relu'(h2)
    for (int t = threadIdx.x; t < 32 * kH2; t += kThreads) {
      const int i = t >> 7, u = t & 127;
      const float h = L.H2[i * kLdH2 + u];
      L.DZ2[i * kLdH2 + u] = h > 0.f ? L.DQ[i] * C.W3[u] : 0.f;
    }
    __syncthreads();
    TP32(6);
    if (threadIdx.x < kH2) {  // per-unit sums: b2, the action columns of W2, W3
      const int u = threadIdx.x;
      for (int i = 0; i < 32; ++i) {
        const float d = L.DZ2[i * kLdH2 + u];
        gb2 += d;
        gwa0 += d * L.A[2 * i];
        gwa1 += d * L.A[2 * i + 1];
        gw3 += L.DQ[i] * L.H2[i * kLdH2 + u];
      }
    }
    // ---- dW2[u][k] += sum_i dz2[i][u] h1d[i][k]: wave w, u-tile w & 3, k-tiles 4 (w >> 2) ..
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      __builtin_amdgcn_sched_barrier(0); gW2[t] = gemm_wgrad(gW2[t], L.DZ2, kLdH2, 32 * u2, L.H1, kLdH1, 32 * (4 * (w >> 2) + t), lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- dz1 = (dz2 W2) x 1.25 relu'(kept h1): wave w -> units 32w ..
    {
      f32x16 acc = {0};
      acc = gemm_xw(acc, L.DZ2, kLdH2, C.W2, kCLd, 32 * w, 0, kH2, lane);
      const int u = 32 * w + (lane & 31);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = drow(v, lane);
        L.DZ1[i * kLdH1 + u] = L.H1[i * kLdH1 + u] > 0.f ? acc[v] * 1.25f : 0.f;
      }
    }
    __syncthreads();
    TP32(7);
    if (threadIdx.x < kH1) {
      for (int i = 0; i < 32; ++i) gb1 += L.DZ1[i * kLdH1 + threadIdx.x];
    }
    // ---- dW1[u][c] += sum_i dz1[i][u] s[i][c]: wave w, u-tile w (columns c >= 12 discarded)
    gW1 = gemm_wgrad(gW1, L.DZ1, kLdH1, 32 * w, L.S, kLdS, 0, lane);
    __syncthreads();  // the next sub-tile restages S / H1
    TP32(8);
  }
  // ---- this workgroup's partial gradient (torch parameters() order)
  float* P = partial + (int64_t)blockIdx.x * kCP;
  const int lane = lane0;
  {
    const int j = lane & 31;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 32 * (4 * (w >> 2) + t) + j;
#pragma unroll
      for (int v = 0; v < 16; ++v) P[skpart::critic_w2_main(32 * u2 + drow(v, lane), k)] = gW2[t][v];
    }
    if (j < kIn) {
#pragma unroll
      for (int v = 0; v < 16; ++v) P[kPW1 + (32 * w + drow(v, lane)) * kIn + j] = gW1[v];
    }
  }
  if (threadIdx.x < kH1) P[kPB1 + threadIdx.x] = gb1;
  if (threadIdx.x < kH2) {
    const int u = threadIdx.x;
    P[pB2(kCLd) + u] = gb2;
    P[skpart::critic_w2_action(u, 0)] = gwa0;
    P[skpart::critic_w2_action(u, 1)] = gwa1;
    P[pW3(kCLd) + u] = gw3;
  }
  if (threadIdx.x < 2) L.RED[threadIdx.x] = 0.f;
  __syncthreads();
  if ((threadIdx.x & 15) == 0) {
    atomicAdd(&L.RED[0], gb3);
    atomicAdd(&L.RED[1], lsum);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    P[pB3(kCLd, 1)] = L.RED[0];
    if (loss_out) atomicAdd(loss_out, L.RED[1]);
  }
  TP32(9);
}

// ---------------------------------------------------------------- actor step
// model_actor_fit_step (SkillshotLearner.py:386-417): gradient of
// -loss_scale * sum_b Q(s_b, mu(s_b)) w.r.t. the actor, critic at inference.
__global__ void __launch_bounds__(kThreads) k_actor_grad32(const float* __restrict__ aflat,
                                                           const float* __restrict__ cflat,
                                                           const float* __restrict__ Sg, int64_t B, int sub_per_wg,
                                                           float loss_scale, float* __restrict__ partial,
                                                           float* step_ctr, int n_steps, float* __restrict__ q_out) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  L32 L;
  float* p = smem32;
  L.S = p;   p += kFS;
  L.H1 = p;  p += kFH1;
  L.H1C = p; p += kFH1;
  L.DZ1 = L.H1C;
  L.H2 = p;  p += kFH2;
  L.DZ2 = p; p += kFH2;
  L.QZ = p;  p += kFH2;
  L.XCH = p; p += kFX;
  carve_small(L, p);
  const int lane0 = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;
  f32x16 gW2[4], gW1 = {0};
#pragma unroll
  for (int t = 0; t < 4; ++t) gW2[t] = f32x16{0};
  float gb1 = 0.f, gb2 = 0.f, gw30 = 0.f, gw31 = 0.f, gb3 = 0.f, qsum = 0.f;
  const int u2 = w & 3;
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;
    const int lane = launder_lane(lane0);
    const Net A = net_of(launder(aflat), kALd, 2), C = net_of(launder(cflat), kCLd, 1);
    stage_states(L.S, Sg, row0, B);
    __syncthreads();
    layer1_relu(L.S, A, L.H1, w, lane);
    layer1_relu(L.S, C, L.H1C, w, lane);
    __syncthreads();
    {  // actor h2
      const f32x16 acc = layer2_split(L.H1, A, L.XCH, w, lane);
      if (w < 4) {
        const int u = 32 * u2 + (lane & 31);
        const float b = A.b2[u];
#pragma unroll
        for (int v = 0; v < 16; ++v) L.H2[drow(v, lane) * kLdH2 + u] = fmaxf(acc[v] + b, 0.f);
      }
    }
    __syncthreads();
    actor_out(L.H2, A, L.A);  // mu(s)
    __syncthreads();
    {  // critic layer 2 at (s, mu(s)): dQ/dz2 = W3 relu'(z2) into DZ2 (rows beyond B: 0), Q terms into QZ
      const f32x16 acc = layer2_split(L.H1C, C, L.XCH, w, lane);
      if (w < 4) {
        const int u = 32 * u2 + (lane & 31);
        const float b = C.b2[u], wa0 = C.W2[u * kCLd + kH1], wa1 = C.W2[u * kCLd + kH1 + 1], w3 = C.W3[u];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int i = drow(v, lane);
          const float z = acc[v] + b + L.A[2 * i] * wa0 + L.A[2 * i + 1] * wa1;
          L.DZ2[i * kLdH2 + u] = (z > 0.f && row0 + i < B) ? w3 : 0.f;
          L.QZ[i * kLdH2 + u] = fmaxf(z, 0.f) * w3;
        }
      }
    }
    __syncthreads();
    {  // dL/dz3 = -loss_scale dQ/da (1 - a^2), dQ/da = sum_u dQ/dz2 W2[u][256 + c]
      const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
      const float da0 = row_dot128(L.DZ2, kLdH2, C.W2 + kH1, kCLd);
      const float da1 = row_dot128(L.DZ2, kLdH2, C.W2 + kH1 + 1, kCLd);
      const float qrow = row_sum128(L.QZ, kLdH2);
      if (c < 2) {
        const float a = L.A[2 * i + c];
        const float d = -loss_scale * (c ? da1 : da0) * (1.f - a * a);
        L.DZ3[2 * i + c] = d;
        gb3 += d;
      }
      if (c == 0 && row0 + i < B) qsum += C.b3[0] + qrow;
    }
    __syncthreads();
    // dz2 = (dz3 W3) relu'(h2) (DZ2 is free again)
    for (int t = threadIdx.x; t < 32 * kH2; t += kThreads) {
      const int i = t >> 7, u = t & 127;
      const float h = L.H2[i * kLdH2 + u];
      L.DZ2[i * kLdH2 + u] = h > 0.f ? L.DZ3[2 * i] * A.W3[u] + L.DZ3[2 * i + 1] * A.W3[kH2 + u] : 0.f;
    }
    __syncthreads();
    if (threadIdx.x < kH2) {
      const int u = threadIdx.x;
      for (int i = 0; i < 32; ++i) {
        const float h = L.H2[i * kLdH2 + u];
        gb2 += L.DZ2[i * kLdH2 + u];
        gw30 += L.DZ3[2 * i] * h;
        gw31 += L.DZ3[2 * i + 1] * h;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      __builtin_amdgcn_sched_barrier(0);
      gW2[t] = gemm_wgrad(gW2[t], L.DZ2, kLdH2, 32 * u2, L.H1, kLdH1, 32 * (4 * (w >> 2) + t), lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    {  // dz1 = (dz2 W2) relu'(h1) into DZ1 (aliases H1C: last read before the barrier above)
      f32x16 acc = {0};
      acc = gemm_xw(acc, L.DZ2, kLdH2, A.W2, kALd, 32 * w, 0, kH2, lane);
      const int u = 32 * w + (lane & 31);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = drow(v, lane);
        L.DZ1[i * kLdH1 + u] = L.H1[i * kLdH1 + u] > 0.f ? acc[v] : 0.f;
      }
    }
    __syncthreads();
    if (threadIdx.x < kH1) {
      for (int i = 0; i < 32; ++i) gb1 += L.DZ1[i * kLdH1 + threadIdx.x];
    }
    gW1 = gemm_wgrad(gW1, L.DZ1, kLdH1, 32 * w, L.S, kLdS, 0, lane);
    __syncthreads();
  }
  float* P = partial + (int64_t)blockIdx.x * kAP;
  const int lane = lane0;
  {
    const int j = lane & 31;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = 32 * (4 * (w >> 2) + t) + j;
#pragma unroll
      for (int v = 0; v < 16; ++v) P[kPW2 + (32 * u2 + drow(v, lane)) * kALd + k] = gW2[t][v];
    }
    if (j < kIn) {
#pragma unroll
      for (int v = 0; v < 16; ++v) P[kPW1 + (32 * w + drow(v, lane)) * kIn + j] = gW1[v];
    }
  }
  if (threadIdx.x < kH1) P[kPB1 + threadIdx.x] = gb1;
  if (threadIdx.x < kH2) {
    const int u = threadIdx.x;
    P[pB2(kALd) + u] = gb2;
    P[pW3(kALd) + u] = gw30;
    P[pW3(kALd) + kH2 + u] = gw31;
  }
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  __syncthreads();
  {
    const int c = threadIdx.x & 15;
    if (c < 2) atomicAdd(&L.RED[c], gb3);
    if (c == 0) atomicAdd(&L.RED[2], qsum);
  }
  __syncthreads();
  if (threadIdx.x < 2) P[pB3(kALd, 2) + threadIdx.x] = L.RED[threadIdx.x];
  if (threadIdx.x == 0 && q_out) atomicAdd(q_out, L.RED[2]);
}

// ---------------------------------------------------------------- actor forward
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

// one 32-row tile per workgroup of 4 waves: layer 1 n-tiles 2w, 2w+1,
// layer 2 n-tile w, layer 3 by all threads.  NOISE: per layer y = xW + b +
// sd sqrt(x^2 W^2 + b^2) xi, xi ~ N(0,1) per (row, unit) (exact in
// distribution for w' = w (1 + sd N(0,1)) drawn per row, each noisy weight
// being used once per row).
template <bool NOISE>
__global__ void __launch_bounds__(kFwdThreads) k_actor_fwd32(const float* __restrict__ aflat,
                                                             const float* __restrict__ X, float* __restrict__ out,
                                                             int64_t rows, float sd, float action_sd, uint64_t seed,
                                                             uint64_t* __restrict__ call_ctr) {
  __shared__ __attribute__((aligned(16))) float S[32 * kLdS];
  __shared__ __attribute__((aligned(16))) float H1[32 * kLdH1];
  __shared__ __attribute__((aligned(16))) float H2[32 * kLdH2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const Net A = net_of(aflat, kALd, 2);
  const int64_t row0 = (int64_t)blockIdx.x * 32;
  // a launch that draws noise (parameter or action) uses call number
  // counter + 1 and its last workgroup stores that number back
  const bool draws = (NOISE || action_sd != 0.f) && call_ctr;
  const uint64_t call = draws ? call_ctr[0] + 1 : 0;
  stage_states(S, X, row0, rows);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int nt = 2 * w + t, u = 32 * nt + (lane & 31);
    const f32x16 m = gemm_l1<false>(S, A.W1, 32 * nt, lane);
    const float b = A.b1[u];
    if (NOISE) {
      const f32x16 var = gemm_l1<true>(S, A.W1, 32 * nt, lane);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float z[4];
        normals4(seed, call, (uint32_t)(row0 + drow(4 * g, lane)), (uint32_t)u, z);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = 4 * g + q;
          const float y = __builtin_fmaf(sd * __builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, var[v])), z[q], m[v] + b);
          H1[drow(v, lane) * kLdH1 + u] = fmaxf(y, 0.f);
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < 16; ++v) H1[drow(v, lane) * kLdH1 + u] = fmaxf(m[v] + b, 0.f);
    }
  }
  __syncthreads();
  {
    const int u = 32 * w + (lane & 31);
    f32x16 m = {0}, var = {0};
    if (NOISE) gemm_xwT_mv(m, var, H1, kLdH1, A.W2, kALd, 32 * w, 0, kH1, lane);
    else m = gemm_xwT(m, H1, kLdH1, A.W2, kALd, 32 * w, 0, kH1, lane);
    const float b = A.b2[u];
    if (NOISE) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float z[4];
        normals4(seed, call, (uint32_t)(row0 + drow(4 * g, lane)), (uint32_t)(kH1 + u), z);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = 4 * g + q;
          const float y = __builtin_fmaf(sd * __builtin_amdgcn_sqrtf(__builtin_fmaf(b, b, var[v])), z[q], m[v] + b);
          H2[drow(v, lane) * kLdH2 + u] = fmaxf(y, 0.f);
        }
      }
    } else {
#pragma unroll
      for (int v = 0; v < 16; ++v) H2[drow(v, lane) * kLdH2 + u] = fmaxf(m[v] + b, 0.f);
    }
  }
  __syncthreads();
  {  // layer 3: thread t -> row t / 8, units 16 (t % 8) .. (both outputs)
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
    if (c == 0 && row0 + i < rows) {
      float y0 = m0 + A.b3[0], y1 = m1 + A.b3[1];
      if (NOISE) {
        float z[4];
        normals4(seed, call, (uint32_t)(row0 + i), (uint32_t)(kH1 + kH2), z);
        y0 += sd * __builtin_amdgcn_sqrtf(v0 + A.b3[0] * A.b3[0]) * z[0];
        y1 += sd * __builtin_amdgcn_sqrtf(v1 + A.b3[1] * A.b3[1]) * z[1];
      }
      float o0 = tanhf(y0), o1 = tanhf(y1);
      if (action_sd != 0.f) {  // model_act_action_noise (:229-243): tanh output + N(0, sd), unclipped
        float z[4];
        normals4(seed, call, (uint32_t)(row0 + i), (uint32_t)(kH1 + kH2 + 1), z);
        o0 += action_sd * z[0];
        o1 += action_sd * z[1];
      }
      *(float2*)(out + (row0 + i) * 2) = make_float2(o0, o1);
    }
  }
  if (draws) {  // the last workgroup to finish stores the call number it drew with
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long prev =
          atomicAdd((unsigned long long*)&call_ctr[1], 1ull);
      if (prev == gridDim.x - 1) {
        call_ctr[0] = call;
        call_ctr[1] = 0;
      }
    }
  }
}

int64_t subtiles_per_wg32(int64_t B) {  // <= 256 workgroups, >= 1 sub-tile each
  const int64_t tiles = (B + 31) / 32;
  return (tiles + 255) / 256;
}

template <typename K>
void set_lds32(K kernel, size_t bytes) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" {

int64_t sk_update_partials_f32(int64_t batch) {
  if (batch <= 0) return 0;
  const int64_t spw = subtiles_per_wg32(batch);
  return ((batch + 31) / 32 + spw - 1) / spw;
}

int sk_critic_grad_f32(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                       const float* next_obs, const float* rewards, const float* done, float gamma,
                       const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                       int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                       float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                       uint8_t* dropout_mask, void* stream) {
  const bool boot = target_actor_flat != nullptr;
  if (boot && (!target_critic_flat || !next_obs || !rewards || !done)) return SK_EINVAL;
  if (!boot && !targets) return SK_EINVAL;
  if (!critic_flat || !obs || !actions || !call_counter || !partials || batch <= 0) return SK_EINVAL;
  if (row_offset < 0 || (row_offset & 3)) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds32(k_critic_grad32, kLdsCritic);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg32(batch);
  const unsigned G = (unsigned)sk_update_partials_f32(batch);
  k_critic_grad32<<<G, kThreads, kLdsCritic, (hipStream_t)stream>>>(
      critic_flat, obs, actions, targets, batch, row_offset, (int)spw, grad_scale, seed, call_counter, partials,
      step_counters, n_steps, loss_sum, dropout_mask, next_obs, rewards, done, gamma, target_actor_flat,
      target_critic_flat);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_grad_f32(const float* actor_flat, const float* critic_flat, const float* obs, int64_t batch,
                      float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                      void* stream) {
  if (!actor_flat || !critic_flat || !obs || !partials || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds32(k_actor_grad32, kLdsActor);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg32(batch);
  const unsigned G = (unsigned)sk_update_partials_f32(batch);
  k_actor_grad32<<<G, kThreads, kLdsActor, (hipStream_t)stream>>>(actor_flat, critic_flat, obs, batch, (int)spw,
                                                                  loss_scale, partials, step_counters, n_steps,
                                                                  q_sum);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_forward_f32(const float* actor_flat, const float* obs, float* actions, int64_t rows, float noise_sd,
                         float action_sd, uint64_t seed, uint64_t* call_counter, void* stream) {
  if (!actor_flat || !obs || !actions || rows <= 0) return SK_EINVAL;
  if ((((uintptr_t)actions) & 7)) return SK_EINVAL;
  const unsigned G = (unsigned)((rows + 31) / 32);
  if (noise_sd != 0.f)
    k_actor_fwd32<true><<<G, kFwdThreads, 0, (hipStream_t)stream>>>(actor_flat, obs, actions, rows, noise_sd,
                                                                      action_sd, seed, call_counter);
  else
    k_actor_fwd32<false><<<G, kFwdThreads, 0, (hipStream_t)stream>>>(actor_flat, obs, actions, rows, 0.f, action_sd,
                                                                       seed, call_counter);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

}  // extern "C"

#ifdef SK_TRACE32
// diagnostic builds only (not in include/skillshot.h): [2 wg][32 points][memtime, realtime]
extern "C" int sk_debug_trace32(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk_trace32), sizeof(g_sk_trace32)) == hipSuccess ? SK_OK : SK_EHIP;
}
#endif
