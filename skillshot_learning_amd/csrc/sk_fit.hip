// sk_fit.hip — the reference rule's models_fit (SkillshotLearner.py:419-443)
// as resident launches.
//
// models_fit is sequential SGD at batch 16: a critic pass (critic.fit, one
// epoch: MSE to the immediate reward, Dropout 0.2 active, :434) over every
// shuffled minibatch, then an actor pass (model_actor_fit_step per
// minibatch, :386-417, the final critic at inference).  Each step depends on
// the last, so the pass is a chain of ~10^7 tiny steps (16 rows x 36.6 k
// parameters); as three launches per step (gradient forward, backward, Adam)
// a step costs 13-14 us of launch boundaries and dependent phase chains.
//
// Here ONE launch runs M consecutive steps of a pass on P workgroups (P = 16
// by default, 8 with SK_FIT_P=8; one CU each, on one XCD by default, spread
// over the XCDs with SK_FIT_XCD=0) that keep the net, its Adam moments and the
// step's activations on chip for the whole launch.  The 36 k weights of layers 1
// and 2 are split by LAYER-2 INPUT COLUMNS (the layer-1 units): workgroup d
// owns
//   layer-1 units C_d = [C d, C d + C), C = 256 / P: W1 rows and b1, and the
//     Dropout mask of those units (keyed by the global unit, as
//     rng.dropout_keep);
//   W2[:, C_d], the layer-2 weights of those inputs for all 128 units;
// with their Adam moments.  The few hundred "unit" parameters after layer 2
// (b2, W3, b3 and the critic's action columns W2[:, 256:258]) are held and
// stepped by EVERY workgroup, redundantly and bit-identically.  A step then
// needs two in-launch exchanges (data-tagged 8-byte granules in pairs, 16-byte
// stores, every load of a sweep in flight, as csrc/sk_xchg.hpp describes; the
// stores plain when the launch finds all its workgroups on one XCD, whose L2
// then carries the exchange, write-through otherwise: fit_placement):
//   R  reduce-scatter of the layer-2 partial products (each workgroup's
//      16 x 128 over its own input columns; workgroup e sums the P slices of
//      units U_e = [U e, U e + U), U = 128 / P, in source order and adds b2
//      and the action columns),
//   H  all-gather of those 16 x U sums (the critic's h2 = relu(z2); the
//      actor's h2), each wave gathering its own four rows: every workgroup
//      then forms q (critic) or a = tanh(z3) and dQ/da (actor), dL/dz2 of all
//      128 units and the unit parameters' gradients and Adam steps itself,
//      and dW2[:, C_d], dL/dh1[:, C_d] with its own columns.
// Two round trips per step instead of the four (critic) or six (actor) of a
// per-quantity exchange (all-reduce q, all-gather dz2, ...); the bytes are
// half the row split's (tools/seam_bench.py, profiles/r05f_seam_bench.jsonl).
// The actor pass reads the frozen critic's action-free layer-2
// pre-activations from a parallel launch ahead of it (k_fit_critic_z2).
//
// The rest of a step is a phase chain (tools/trace_fit.py, -DSK_TRACE_FIT):
// a first version holding everything in LDS spent 9 of its 12.8 us per
// critic step in serial LDS-latency chains.  So the weights live in
// REGISTERS in the layout of the MFMA operand that reads them, and every
// gradient GEMM is oriented to produce its output in that same layout, so
// Adam runs in the GEMM's epilogue on registers:
//   W2[:, C_d]  lane (i, g) of wave w holds W2[16 nt + i][16 mk + 4 g .. + 3]
//               for n-tiles nt = w, w + 4 and column tiles mk < C / 16: the B
//               operand of the forward partials (h1 W2^T) and the output of
//               dW2^T = h1^T dz2 (v_mfma_f32_16x16x4_f32: lane (i, g) holds
//               A[i][k = g], B[k = g][i], D[4 g + r][i]); an LDS mirror feeds
//               the backward dz2 W2;
//   W1 | b1     lane (i, g) of wave w < C / 16 holds W1[C d + 16 w + i][4 g ..
//               + 3] (g = 3: b1 and zeros): the B operand of layer 1 as a
//               K = 16 GEMM on s with a column of ones (the bias folded in),
//               and the output of dW1^T = s^T dz1; layer 1's output rows
//               4 g .. 4 g + 3 of one unit per lane also make ONE Philox call
//               per lane give the four rows' Dropout bits;
// 16-lane sums are DPP row operations.  GEMMs are exact fp32 products with
// fp32 sums in another order than the three-launch chain: the tests hold both
// to 1e-5 of each other and of the fp64 Keras restatement.  Adam is Keras'
// formula with k_adam_flat's step-count arithmetic.
//
// Device counters advance as M three-launch steps would: the Dropout call
// number (calls += M), the Adam step counts (steps[i] += 1 per step, fp32)
// and the exchange epoch (epoch += 2 M; tags are epochs, so a slot's previous
// contents never match and no memset is needed between launches).  A wait
// that runs out of spins (a lost workgroup) sets *timeout and ends the launch
// uniformly; the host checks it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"
#include "sk_xchg.hpp"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

constexpr int kB = 16, kS = 12, kH1 = 256, kH2 = 128, kT = 256;  // rows, inputs, units, threads
constexpr int kCLd = kH1 + 2;                                     // critic W2 row: 256 h1 + 2 action
// flat offsets (torch parameters() order; update_kernel.flatten_module)
constexpr int kW1 = 0, kB1 = kH1 * kS, kW2 = kB1 + kH1;
constexpr int kCB2 = kW2 + kH2 * kCLd, kCW3 = kCB2 + kH2, kCB3 = kCW3 + kH2, kCP = kCB3 + 1;
constexpr int kAB2 = kW2 + kH2 * kH1, kAW3 = kAB2 + kH2, kAB3 = kAW3 + 2 * kH2, kAP = kAB3 + 2;
static_assert(kCP == 36609 && kAP == 36482, "parameter counts");
constexpr unsigned kDropThreshold = 858993460u;  // rng.DROP_THRESHOLD: keep with p = 0.8

// LDS strides (floats)
constexpr int LS = 16;       // s_ext rows: 12 inputs, 1 (the bias column), 3 zeros
constexpr int LHT = kB + 4;  // [C][16 rows]
constexpr int LZ = kH2 + 4;  // [16 rows][128]
constexpr int LZT = kB + 4;  // [128][16 rows]

// The split over PW workgroups (8 or 16, SK_FIT_P): C own layer-1 units (=
// W2 input columns) per workgroup in NT1 16-unit tiles, U layer-2 units summed
// per workgroup in the R exchange; the dL/dh1 GEMM splits its K = 128 over KS
// waves per n-tile
template <int PW>
struct Geo {
  static constexpr int P = PW, C = kH1 / P, U = kH2 / P, NT1 = C / 16, KS = 4 / NT1;
  static constexpr int LH = C + 4;  // [16 rows][C] activations
  static constexpr int LW = C + 4;  // the W2 mirror [128][C]
  static_assert(C % 16 == 0 && NT1 <= 2 && U % 8 == 0, "geometry");
};

__device__ __forceinline__ f32x4 m16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 m16x4(f4 a, f4 b, f32x4 c) {
  c = m16(a.x, b.x, c);
  c = m16(a.y, b.y, c);
  c = m16(a.z, b.z, c);
  return m16(a.w, b.w, c);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, -1, 0x00020000);
}
// one granule pair {a, tag, b, tag}: ONE 16-byte store.  local (every
// workgroup of the launch on one XCD, fit_placement): a plain store, which
// keeps the line in that XCD's L2, where the readers' sc1 loads find it;
// otherwise write-through (aux 16 = sc1), which drops the line from the
// writer's L2 so the other XCDs' readers see it (a same-XCD reader then pays
// the cross-XCD rate: critic 5.1 vs 4.4 us per step)
__device__ __forceinline__ void put2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, unsigned tag, float a, float b,
                                     bool local) {
  const u4v v = {__float_as_uint(a), tag, __float_as_uint(b), tag};
  if (local)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 16);
}
// N granule pairs per lane at byte offsets off[k], every load issued before
// the checks, re-read until the wave's tags all equal `tag` (bounded spin)
template <int N>
__device__ __forceinline__ bool get2(__amdgpu_buffer_rsrc_t r, const uint32_t (&off)[N], unsigned tag,
                                     float (&v)[2 * N], unsigned* timeout) {
  for (unsigned spins = 0;; ++spins) {
    u4v x[N];
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = __builtin_amdgcn_raw_buffer_load_b128(r, off[k], 0, 16);
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      v[2 * k] = __uint_as_float(x[k].x);
      v[2 * k + 1] = __uint_as_float(x[k].z);
      ok &= (x[k].y == tag) & (x[k].w == tag);
    }
    if (__all(ok)) return true;
    if (spins >= skx::kSpinLimit) {
      if ((threadIdx.x & 63) == 0) atomicMax(timeout, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The launch's placement, decided once before the first step: every
// workgroup publishes its XCD (HW_REG_XCC_ID) in granule pair kXPlace + 2 d
// (write-through; tag ~epoch, which no earlier launch's slot and no zeroed
// slot holds) and wave 0 reads all P of them.  Every workgroup sees the same P
// values, so all pick the same store flavour (put2): correct under any
// block -> XCD map, fast when the stride-8 grid lands on one XCD.  Returns
// 2 (one XCD), 1 (spread) or 0 (a workgroup never arrived: *timeout is set).
constexpr int kXPlace = 65536 - 64;  // granules: the placement slots, past every step exchange
template <int P>
__device__ __forceinline__ int fit_placement(__amdgpu_buffer_rsrc_t xr, int d, unsigned ep0, unsigned* timeout) {
  __shared__ int s_place;
  const unsigned tag = ~ep0;
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID [3:0]
  if (threadIdx.x == 0) put2(xr, (uint32_t)(kXPlace + 2 * d) * 8u, tag, __uint_as_float(xcc), 0.f, false);
  if (threadIdx.x < 64) {
    const uint32_t off[1] = {(uint32_t)(kXPlace + 2 * (int)(threadIdx.x % P)) * 8u};
    float v[2];
    const bool ok = get2<1>(xr, off, tag, v, timeout);
    const bool same = __all(__float_as_uint(v[0]) == xcc);
    if (threadIdx.x == 0) s_place = ok ? (same ? 2 : 1) : 0;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(s_place);
}

// whether any thread of the workgroup has f set, at a workgroup barrier: one
// barrier (__syncthreads_or is two and an LDS atomic).  slot: 4 ints of LDS
// per call site, alternated by the caller so the next write to a slot is
// behind barriers after this call's reads
__device__ __forceinline__ bool wg_any(bool f, int* slot) {
  const bool w = __any(f);
  if ((threadIdx.x & 63) == 0) slot[threadIdx.x >> 6] = w;
  __syncthreads();
  const int4 v = *(const int4*)slot;
  return (v.x | v.y | v.z | v.w) != 0;
}

// DPP row (16-lane) moves: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// the sum of v over this lane's 16-lane row; every lane of the row gets the
// same bits (each stage adds two equal partial sums in either order)
__device__ __forceinline__ float sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  return v + dpp<0x140>(v);
}

// Keras Adam (learner.KerasAdam, k_adam_flat) on registers; returns the new
// parameter.  The square root and the quotient by the hardware's v_sqrt_f32
// and v_rcp_f32 (1 ulp each, against a 14-instruction correctly rounded
// sqrtf; the tests bound the parameters at 1e-5)
__device__ __forceinline__ float adam(float w, float& m, float& v, float g, float alpha, float b1c, float b2c,
                                      float eps) {
  m = m + (g - m) * b1c;
  v = v + (g * g - v) * b2c;
  return w - (m * alpha) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) + eps);
}
// the same on four parameters (the element-wise arithmetic as packed fp32 pairs)
__device__ __forceinline__ void adam4(f4& w, f4& m, f4& v, f4 g, float alpha, float b1c, float b2c, float eps) {
  m = m + (g - m) * b1c;
  v = v + (g * g - v) * b2c;
  f4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v[t]) + eps);
  w = w - (m * alpha) * r;
}
// tanh without branches: sign(x) (1 - 2 / (e^{2|x|} + 1)) on v_exp_f32 and
// v_rcp_f32, absolutely within ~1e-7 of tanhf (whose range split made both
// outputs' chains run both paths under exec masks, one after the other)
__device__ __forceinline__ float tanh_nb(float x) {
  const float e = __builtin_amdgcn_exp2f(fabsf(x) * 2.8853900817779268f);  // 2 log2(e) |x|
  return copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f), x);
}
__device__ __forceinline__ void adam_lds(float* w, float* m, float* v, int i, float g, float alpha, float b1c,
                                         float b2c, float eps) {
  float mm = m[i], vv = v[i];
  w[i] = adam(w[i], mm, vv, g, alpha, b1c, b2c, eps);
  m[i] = mm;
  v[i] = vv;
}
// N parameters at once: every read issued before the first write (one LDS
// round trip; one adam_lds after another waited for each in turn)
template <int N>
__device__ __forceinline__ void adam_lds_n(float* w, float* m, float* v, const int (&i)[N], const float (&g)[N],
                                           float alpha, float b1c, float b2c, float eps) {
  float ww[N], mm[N], vv[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    ww[n] = w[i[n]];
    mm[n] = m[i[n]];
    vv[n] = v[i[n]];
  }
#pragma unroll
  for (int n = 0; n < N; ++n) ww[n] = adam(ww[n], mm[n], vv[n], g[n], alpha, b1c, b2c, eps);
#pragma unroll
  for (int n = 0; n < N; ++n) {
    w[i[n]] = ww[n];
    m[i[n]] = mm[n];
    v[i[n]] = vv[n];
  }
}

struct FitArgs {
  float* flat;           // the net's flat parameters (in / out)
  float* m;              // its Adam moments (flat, in / out)
  float* v;
  float* steps;          // Adam step counters (fp32, n_steps of them; all advance by 1 per step)
  int n_steps;
  const float* states;   // [M * 16][12] the pass's minibatches, consecutive
  const float* actions;  // [M * 16][2] (critic)
  const float* targets;  // [M * 16] (critic)
  int M;                 // minibatch steps in this launch
  uint64_t drop_seed;
  int64_t* drop_calls;   // Dropout call number (in / out; critic)
  float lr, beta1, beta2, eps;
  unsigned long long* xbuf;
  unsigned long long* epoch;
  unsigned* timeout;      // [0] a lost exchange (atomicMax 1); [1] the placement (fit_placement's value)
  float* losses;         // [M] per-step MSE (nullable; critic)
  int stride;            // grid = P x stride; blocks b % stride == 0 work (stride 8: one XCD under
                         // round-robin placement, a speed choice only, never correctness)
  const float* critic;   // the actor pass: the (frozen) critic's flat parameters
};

// Measurement build only (-DSK_TRACE_FIT; tools/trace_fit.py): thread 0 of
// every workgroup records s_memrealtime (100 MHz) at 11 points of steps
// 64 .. 95 of a launch into LDS (no memory write inside the steps to wait
// for), copied to sk_fit_trace[workgroup][step - 64][12] at the end.
#ifdef SK_TRACE_FIT
__device__ unsigned long long* sk_fit_trace;
#define SK_FT_DECL __shared__ unsigned long long ft_lds[32 * 12];
#define SK_FT(k, i)                                                                    \
  do {                                                                                 \
    if (threadIdx.x == 0 && (k) >= 64 && (k) < 96)                                     \
      ft_lds[((k) - 64) * 12 + (i)] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
#define SK_FT_FLUSH()                                                                    \
  do {                                                                                   \
    __syncthreads();                                                                     \
    for (int j = threadIdx.x; j < 32 * 12; j += kT) sk_fit_trace[(size_t)d * 384 + j] = ft_lds[j]; \
  } while (0)
#else
#define SK_FT_DECL
#define SK_FT(k, i) \
  do {              \
  } while (0)
#define SK_FT_FLUSH() \
  do {                \
  } while (0)
#endif
// -DSK_TRACE_FIT_P5 moves stamps 7 .. 9 into phase 5 (tools/trace_fit.py --p5)
#ifdef SK_TRACE_FIT_P5
#define SK_FT5(k, i) SK_FT(k, i)
#define SK_FT7(k, i) \
  do {               \
  } while (0)
#else
#define SK_FT5(k, i) \
  do {               \
  } while (0)
#define SK_FT7(k, i) SK_FT(k, i)
#endif

// ---------------------------------------------------------------- shared pieces
// The W2[:, C_d] slice in registers: r[q][mk][t] = W[u = 16 (w + 4 q) + i][c = 16 mk + 4 g + t]
template <class G>
struct W2Reg {
  f4 w[2][G::NT1];
};
// flat index of W2 entry (u, own column c) for row length ld
template <class G>
__device__ __forceinline__ int w2_index(int u, int c, int d, int ld) { return kW2 + u * ld + G::C * d + c; }

template <class G, int LD>
__device__ __forceinline__ void w2_load(W2Reg<G>& r, const float* src, int d, int wv, int li, int lg) {
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int mk = 0; mk < G::NT1; ++mk) {
      const int u = 16 * (wv + 4 * q) + li;
#pragma unroll
      for (int t = 0; t < 4; ++t) r.w[q][mk][t] = src[w2_index<G>(u, 16 * mk + 4 * lg + t, d, LD)];
    }
}
template <class G, int LD>
__device__ __forceinline__ void w2_store(const W2Reg<G>& r, float* dst, int d, int wv, int li, int lg) {
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int mk = 0; mk < G::NT1; ++mk) {
      const int u = 16 * (wv + 4 * q) + li;
#pragma unroll
      for (int t = 0; t < 4; ++t) dst[w2_index<G>(u, 16 * mk + 4 * lg + t, d, LD)] = r.w[q][mk][t];
    }
}
template <class G>
__device__ __forceinline__ void w2_mirror(const W2Reg<G>& r, float* sW2, int wv, int li, int lg) {
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int mk = 0; mk < G::NT1; ++mk) {
      const int u = 16 * (wv + 4 * q) + li;
      *(f4*)(sW2 + u * G::LW + 16 * mk + 4 * lg) = r.w[q][mk];
    }
}

// W1 | b1 of n-tile wt in registers: lane (i, g): W1[C d + 16 wt + i][4 g + t], g = 3: {b1, 0, 0, 0}
template <class G>
__device__ __forceinline__ f4 w1_load(const float* src, int d, int wt, int li, int lg) {
  const int cg = G::C * d + 16 * wt + li;
  f4 r = {0.f, 0.f, 0.f, 0.f};
  if (lg < 3) {
#pragma unroll
    for (int t = 0; t < 4; ++t) r[t] = src[kW1 + cg * kS + 4 * lg + t];
  } else {
    r[0] = src[kB1 + cg];
  }
  return r;
}
template <class G>
__device__ __forceinline__ void w1_store(f4 r, float* dst, int d, int wt, int li, int lg) {
  const int cg = G::C * d + 16 * wt + li;
  if (lg < 3) {
#pragma unroll
    for (int t = 0; t < 4; ++t) dst[kW1 + cg * kS + 4 * lg + t] = r[t];
  } else {
    dst[kB1 + cg] = r[0];
  }
}

// layer 1 of n-tile wt as a K = 16 GEMM on s_ext (the bias column folded
// in): lane (i, g) gets z[r] of rows 4 g + r, unit 16 wt + i
__device__ __forceinline__ f32x4 layer1(const float* sS, f4 w1, int li, int lg) {
  const f4 x = *(const f4*)(sS + li * LS + 4 * lg);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  return m16x4(x, w1, acc);
}

// the layer-2 partial products of X [16][LH] (own columns) with the
// register slice W for n-tiles wv and wv + 4, each unit's row published to
// its summer e at slot(e) (granule index of a [U units][16 rows] slice)
template <class G, typename Slot>
__device__ __forceinline__ void partials_publish(const float* X, const W2Reg<G>& W, __amdgpu_buffer_rsrc_t xr,
                                                 unsigned tag, bool local, int wv, int li, int lg, Slot slot) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int nt = wv + 4 * q;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mk = 0; mk < G::NT1; ++mk)
      acc = m16x4(*(const f4*)(X + li * G::LH + 16 * mk + 4 * lg), W.w[q][mk], acc);
    // unit 16 nt + li is summed by workgroup (16 nt + li) / U: its slice row
    const int u = 16 * nt + li;
    const uint32_t base = (uint32_t)(slot(u / G::U) + (u % G::U) * 16 + 4 * lg) * 8u;
    put2(xr, base, tag, acc[0], acc[1], local);
    put2(xr, base + 16u, tag, acc[2], acc[3], local);
  }
}

// the R sums of this workgroup's U units: lane pr < 8 U sums granule pair
// pr ([U][16]) of the P source slices in source order; {rows r0, r0 + 1} of
// unit 2 pr / 16 (local)
template <class G, typename Slot>
__device__ __forceinline__ bool r_sum(__amdgpu_buffer_rsrc_t xr, unsigned tag, int pr, Slot slot, float& z0,
                                      float& z1, unsigned* timeout) {
  constexpr int P = G::P;
  uint32_t off[P];
#pragma unroll
  for (int s = 0; s < P; ++s) off[s] = (uint32_t)(slot(s) + 2 * pr) * 8u;
  float v[2 * P];
  const bool ok = get2<P>(xr, off, tag, v, timeout);
  z0 = 0.f;
  z1 = 0.f;
#pragma unroll
  for (int s = 0; s < P; ++s) {
    z0 += v[2 * s];
    z1 += v[2 * s + 1];
  }
  return ok;
}

// The H exchange: each source's [8 row pairs][U units] granule pairs (row
// pair major), so the rows 4 w .. 4 w + 3 a wave works on are 2 U contiguous
// pairs per source.  h_pair: the pair index of (source s, row pair rp, unit ul)
template <class G>
__device__ __forceinline__ int h_pair(int s, int rp, int ul) {
  return s * G::U * 8 + rp * G::U + ul;
}
// wave w gathers its own rows' h2 (row pairs 2 w, 2 w + 1 of all 128 units)
// into dst [16][LZ]: its phase-5 reads need no workgroup barrier
template <class G>
__device__ __forceinline__ bool gather_h_rows(__amdgpu_buffer_rsrc_t xr, int base, unsigned tag, float* dst, int wv,
                                              int lane, unsigned* timeout) {
  constexpr int U = G::U, PER = (G::P * 2 * U) / 64;  // granule pairs per lane
  static_assert(PER == 4, "256 pairs per wave");
  uint32_t off[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int q = lane + 64 * j, s = q / (2 * U), w = q % (2 * U);
    off[j] = (uint32_t)(base + 2 * h_pair<G>(s, 2 * wv + w / U, w % U)) * 8u;
  }
  float v[2 * PER];
  const bool ok = get2<PER>(xr, off, tag, v, timeout);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int q = lane + 64 * j, s = q / (2 * U), w = q % (2 * U);
    const int r0 = 2 * (2 * wv + w / U), u = U * s + w % U;
    dst[r0 * LZ + u] = v[2 * j];
    dst[(r0 + 1) * LZ + u] = v[2 * j + 1];
  }
  // the wave's own LDS writes, in order before its reads (no other wave reads these rows this phase)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok;
}

// dL/dh1 of the own columns = dz2 W2[:, C_d] from the LDS mirror (the
// weights before this step's update): waves (n-tile w % NT1, k part w / NT1);
// waves w < NT1 return their n-tile's result (lane (i, g): rows 4 g + r,
// column 16 w + i — layer 1's output layout)
template <class G>
__device__ __forceinline__ f32x4 backward_dh1(const float* sDZ, const float* sW2, float* sPart, int wv, int lane,
                                              int li, int lg) {
  constexpr int NT1 = G::NT1, KW = kH2 / G::KS, LW = G::LW;
  const int nt = wv % NT1, ks = wv / NT1;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < KW; kk += 16) {
    const int k0 = KW * ks + kk;
    const f4 x = *(const f4*)(sDZ + li * LZ + k0 + 4 * lg);
    const float* wc = sW2 + (k0 + 4 * lg) * LW + 16 * nt + li;
    const f4 w = {wc[0], wc[LW], wc[2 * LW], wc[3 * LW]};
    acc = m16x4(x, w, acc);
  }
  if (ks) *(f32x4*)(sPart + ((wv - NT1) * 64 + lane) * 4) = acc;
  __syncthreads();
  if (!ks) {
#pragma unroll
    for (int j = 1; j < G::KS; ++j) acc += *(const f32x4*)(sPart + ((j * NT1 + wv - NT1) * 64 + lane) * 4);
  }
  return acc;
}

// dW2^T tiles (column tile mk, unit tile nt = wv + 4 q) = h1^T dz2 and their
// Adam steps on the register slice; the mirror rewritten
template <class G>
__device__ __forceinline__ void dw2_adam(W2Reg<G>& W, W2Reg<G>& Mo, W2Reg<G>& Vo, const float* sHT,
                                         const float* sDZT, float* sW2, float alpha, float b1c, float b2c, float eps,
                                         int wv, int li, int lg) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int nt = wv + 4 * q;
    const f4 dz = *(const f4*)(sDZT + (16 * nt + li) * LZT + 4 * lg);
#pragma unroll
    for (int mk = 0; mk < G::NT1; ++mk) {
      const f4 h = *(const f4*)(sHT + (16 * mk + li) * LHT + 4 * lg);
      f32x4 g = {0.f, 0.f, 0.f, 0.f};
      g = m16x4(h, dz, g);
      adam4(W.w[q][mk], Mo.w[q][mk], Vo.w[q][mk], g, alpha, b1c, b2c, eps);
    }
  }
  w2_mirror<G>(W, sW2, wv, li, lg);
}

// dW1^T of n-tile wv (waves 0 / 1) = s_ext^T dz1 and its Adam step: lane (i,
// g) holds dz1 of rows 4 g .. 4 g + 3, unit 16 wv + i (layer 1's layout) and
// W1 | b1 in w1_load's layout
__device__ __forceinline__ void dw1_adam(f4& w1, f4& m1, f4& v1, f4 dz1, const float* sS, float alpha, float b1c,
                                         float b2c, float eps, int li, int lg) {
  const f4 x = {sS[(4 * lg) * LS + li], sS[(4 * lg + 1) * LS + li], sS[(4 * lg + 2) * LS + li],
                sS[(4 * lg + 3) * LS + li]};
  f32x4 g = {0.f, 0.f, 0.f, 0.f};
  g = m16x4(x, dz1, g);  // D[4 g + t][i] = dW1ext^T[j = 4 g + t][unit i]
  const int n = lg < 3 ? 4 : 1;  // j = 12 is b1; 13 .. 15 are the zero pad
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < n) {
      float mm = m1[t], vv = v1[t];
      w1[t] = adam(w1[t], mm, vv, g[t], alpha, b1c, b2c, eps);
      m1[t] = mm;
      v1[t] = vv;
    }
  }
}

// the Dropout bits of layer-1 unit C d + c, rows 4 g .. 4 g + 3, for call
// number `call` (rng.dropout_keep's keys: (row >> 2, unit, call); word row & 3)
template <class G>
__device__ __forceinline__ uint4 drop_bits(const FitArgs& a, uint64_t call, int d, int c, int lg) {
  return skmlp::philox<10>(make_uint4((uint32_t)lg, (uint32_t)(G::C * d + c), (uint32_t)call, (uint32_t)(call >> 32)),
                           (uint32_t)a.drop_seed, (uint32_t)(a.drop_seed >> 32));
}

__device__ __forceinline__ float keras_alpha(const FitArgs& a, float tk) {
  return a.lr * sqrtf(1.f - powf(a.beta2, tk)) / (1.f - powf(a.beta1, tk));
}
// The Adam step count after j steps from tk0, as the three-launch chain
// produces it: j fp32 additions of 1 (k_grad_slice_fwd / k_critic_grad32),
// which stop changing the count at 2^24 (2^24 + 1 rounds to even, 2^24).
// Above 2^24 (a loaded count) only the first addition can change it (an odd
// mantissa rounds up to even), so one addition stands for all
__host__ __device__ __forceinline__ float adam_count(float tk0, int j) {
  if (j <= 0) return tk0;
  return tk0 < 16777216.f ? fminf(tk0 + (float)j, 16777216.f) : tk0 + 1.0f;
}
// Adam's step sizes of steps k0 .. k0 + kAlphaN - 1 into LDS, computed in
// parallel once per kAlphaN steps (two powf per step off the step chain);
// step k applies the count adam_count(tk0, k + 1) (k_adam_flat reads it incremented)
constexpr int kAlphaN = 2048;
__device__ __forceinline__ void alpha_fill(const FitArgs& a, float* sAlpha, float tk0, int k0) {
  for (int j = threadIdx.x; j < kAlphaN && k0 + j < a.M; j += kT)
    sAlpha[j] = keras_alpha(a, adam_count(tk0, k0 + j + 1));
  __syncthreads();
}

// ------------------------------------------------------------------ critic
// unit parameters in LDS (w, m, v planes of kUN), all 128 units in every workgroup
constexpr int uW3 = 0, uB2 = kH2, uWA = 2 * kH2, uB3 = 4 * kH2, kUN = 4 * kH2 + 4;
// per-step buffers, two of each (step k uses k & 1, so the next step's rows
// and layer-1 activations never wait for this step's last readers):
// rows [s_ext 16 x 16 | a 16 x 2 | y 16], activations [hd 16 x LH | hd^T C x LHT]
template <class G>
struct CriticLayout {
  static constexpr int kRowsN = kB * LS + 2 * kB + kB, kActN = kB * G::LH + G::C * LHT;
  static constexpr int cRows = 3 * kUN, cAct = cRows + 2 * kRowsN, cDQ = cAct + 2 * kActN, cL = cDQ + kB,
                       cH2 = cL + kB, cDZ = cH2 + kB * LZ, cDZT = cDZ + kB * LZ, cW2 = cDZT + kH2 * LZT,
                       cPart = cW2 + kH2 * G::LW, cAlpha = cPart + 3 * 64 * 4, cEnd = cAlpha + kAlphaN;
  static constexpr size_t kLds = (size_t)cEnd * 4;
  // exchanges (granules): R [P src][P dst][U][16], H [P][U][16]
  static constexpr int cxR = 0, cxH = cxR + G::P * G::P * G::U * 16, cxN = cxH + G::P * G::U * 16;
  static_assert(kLds <= 150 * 1024 && cxN <= kXPlace, "LDS / xbuf");
};

template <int PW>
__global__ void __launch_bounds__(kT) k_fit_critic(FitArgs a) {
  using G = Geo<PW>;
  using Y = CriticLayout<G>;
  constexpr int P = G::P, U = G::U, LH = G::LH, NT1 = G::NT1;
  constexpr int kRowsN = Y::kRowsN, kActN = Y::kActN, cRows = Y::cRows, cAct = Y::cAct, cxR = Y::cxR,
                cxH = Y::cxH;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ __attribute__((aligned(16))) int sFail[8];
  SK_FT_DECL
  if (blockIdx.x % a.stride) return;
  float* uW = sm;
  float* uM = sm + kUN;
  float* uV = sm + 2 * kUN;
  float* sDQ = sm + Y::cDQ;
  float* sL = sm + Y::cL;
  float* sH2 = sm + Y::cH2;
  float* sAlpha = sm + Y::cAlpha;
  float* sDZ = sm + Y::cDZ;
  float* sDZT = sm + Y::cDZT;
  float* sW2 = sm + Y::cW2;
  float* sPart = sm + Y::cPart;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, li = lane & 15, lg = lane >> 4;
  const int d = blockIdx.x / a.stride;
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(a.xbuf);

  // the owned slice: W2 (+ moments) and W1 | b1 in registers; every unit parameter in LDS
  W2Reg<G> W2, M2, V2;
  w2_load<G, kCLd>(W2, a.flat, d, wv, li, lg);
  w2_load<G, kCLd>(M2, a.m, d, wv, li, lg);
  w2_load<G, kCLd>(V2, a.v, d, wv, li, lg);
  w2_mirror<G>(W2, sW2, wv, li, lg);
  f4 W1 = {0.f, 0.f, 0.f, 0.f}, M1 = W1, V1 = W1;
  if (wv < NT1) {
    W1 = w1_load<G>(a.flat, d, wv, li, lg);
    M1 = w1_load<G>(a.m, d, wv, li, lg);
    V1 = w1_load<G>(a.v, d, wv, li, lg);
  }
  // a use of the loaded slice here, so their vmcnt wait is placed before the
  // step loop (first used inside it, the wait went inside it: a vmcnt(0) at
  // every step's layer-1 MFMAs, behind whatever memory traffic was in flight)
  asm volatile("" ::"v"(W1), "v"(M1), "v"(V1));
  if (t < kH2) {
    const int gi[4] = {kCW3 + t, kCB2 + t, kW2 + t * kCLd + kH1, kW2 + t * kCLd + kH1 + 1};
    const int l4[4] = {uW3 + t, uB2 + t, uWA + 2 * t, uWA + 2 * t + 1};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uW[l4[j]] = a.flat[gi[j]];
      uM[l4[j]] = a.m[gi[j]];
      uV[l4[j]] = a.v[gi[j]];
    }
  } else if (t == kH2) {
    uW[uB3] = a.flat[kCB3];
    uM[uB3] = a.m[kCB3];
    uV[uB3] = a.v[kCB3];
  }
  const int64_t call0 = a.drop_calls[0];
  const unsigned ep0 = (unsigned)a.epoch[0];
  const float tk0 = a.steps[0];
  const int place = fit_placement<P>(xr, d, ep0, a.timeout);
  const bool local = place == 2;
  const int M = place ? a.M : 0;  // a lost workgroup: no step runs (*timeout is set)
  // s_ext: 12 inputs, the bias column (1), zeros (both buffers); step 0's rows
  if (t < kB * LS) {
    const int r = t / LS, j = t % LS;
    sm[cRows + t] = j < kS ? a.states[r * kS + j] : (j == kS ? 1.f : 0.f);
    sm[cRows + kRowsN + t] = j == kS ? 1.f : 0.f;
  }
  if (t < 2 * kB) sm[cRows + kB * LS + t] = a.actions[t];
  if (t < kB) sm[cRows + kB * LS + 2 * kB + t] = a.targets[t];
  const float b1c = 1.f - a.beta1, b2c = 1.f - a.beta2;
  bool fail = false;  // this thread's exchange ran out of spins (decided uniformly at the barriers)
  // waves w < NT1: this step's Dropout bits (the next step's are drawn in the R wait)
  uint4 bits = {0u, 0u, 0u, 0u};
  if (wv < NT1) bits = drop_bits<G>(a, (uint64_t)call0, d, 16 * wv + li, lg);

  for (int k = 0; k < M; ++k) {
    const unsigned E = ep0 + 2u * (unsigned)k;
    if (k % kAlphaN == 0) alpha_fill(a, sAlpha, tk0, k);  // (its barrier also publishes step 0's rows)
    const float alpha = sAlpha[k % kAlphaN];
    float* sS = sm + cRows + (k & 1) * kRowsN;
    float* sA = sS + kB * LS;
    float* sY = sA + 2 * kB;
    float* sHD = sm + cAct + (k & 1) * kActN;
    float* sHDT = sHD + kB * LH;
    SK_FT(k, 0);
    const bool more = k + 1 < a.M;

    // (1) layer 1 of the own units with Dropout (SkillshotLearner.py:106-108):
    //     waves w < NT1, one n-tile each; one Philox call gives the 4 rows' bits
    f4 mask = {0.f, 0.f, 0.f, 0.f};
    if (wv < NT1) {
      const f32x4 z = layer1(sS, W1, li, lg);
      const int c = 16 * wv + li;
      const uint32_t bw[4] = {bits.x, bits.y, bits.z, bits.w};
      f4 hd;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool keep = bw[r] >= kDropThreshold;
        hd[r] = keep ? fmaxf(z[r], 0.f) * 1.25f : 0.f;
        mask[r] = (keep && z[r] > 0.f) ? 1.25f : 0.f;
        sHD[(4 * lg + r) * LH + c] = hd[r];
      }
      *(f4*)(sHDT + c * LHT + 4 * lg) = hd;
    }
    __syncthreads();
    SK_FT(k, 1);

    // (2) the layer-2 partial products of the own columns for all 128 units,
    //     each 16-unit tile to its summer: slice (d -> e) = [U units][16 rows]
    partials_publish<G>(sHD, W2, xr, E + 1, local, wv, li, lg, [&](int e) { return cxR + (d * P + e) * U * 16; });
    SK_FT(k, 2);
    // the next step's rows into registers, stored into the other buffer after
    // phase 5: issued here they land under the exchange waits (at the top of
    // the step the layer-1 MFMAs' vmcnt(0) waited for them)
    float nx = 0.f;
    if (more) {
      const int64_t r0 = (int64_t)(k + 1) * kB;
      if (t < kB * kS) nx = a.states[r0 * kS + t];
      else if (t < kB * kS + 2 * kB) nx = a.actions[r0 * 2 + (t - kB * kS)];
      else if (t < kB * kS + 3 * kB) nx = a.targets[r0 + (t - kB * kS - 2 * kB)];
    }

    // (3) workgroup d sums the P slices of units U_d (source order), adds b2
    //     and the action columns: h2 = relu(z2), published to all (H); the
    //     next step's Dropout bits first (VALU work hidden by the wait; the
    //     summing lanes t < 8 U are the layer-1 waves w < NT1)
    static_assert(U * 8 == NT1 * 64, "the summing waves are the layer-1 waves");
    if (t < U * 8) {
      if (more) bits = drop_bits<G>(a, (uint64_t)(call0 + k + 1), d, 16 * wv + li, lg);
      float z0, z1;
      fail |= !r_sum<G>(xr, E + 1, t, [&](int s) { return cxR + (s * P + d) * U * 16; }, z0, z1, a.timeout);
      const int ug = U * d + (2 * t) / 16, r0 = (2 * t) % 16;
      const float b2 = uW[uB2 + ug], wa0 = uW[uWA + 2 * ug], wa1 = uW[uWA + 2 * ug + 1];
      z0 = z0 + sA[2 * r0] * wa0 + sA[2 * r0 + 1] * wa1 + b2;
      z1 = z1 + sA[2 * r0 + 2] * wa0 + sA[2 * r0 + 3] * wa1 + b2;
      put2(xr, (uint32_t)(cxH + 2 * h_pair<G>(d, r0 / 2, ug - U * d)) * 8u, E + 2, fmaxf(z0, 0.f), fmaxf(z1, 0.f),
           local);
    }
    SK_FT(k, 3);

    // (4) h2 of all 128 units for this wave's rows
    fail |= !gather_h_rows<G>(xr, cxH, E + 2, sH2, wv, lane, a.timeout);
    SK_FT(k, 4);

    // (5) q of the 16 rows, every workgroup: lane (row t / 16, units t % 16 +
    //     16 i; each wave its own gathered rows), a DPP row sum; dL/dq =
    //     2 (q - y) / 16; dL/dz2 of all units
    //     (every operand read into registers first: read again after the
    //     first stores, each re-read waited for its own round trip)
    {
      const int r = t >> 4, j = t & 15;
      float h[8], w3[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        h[i] = sH2[r * LZ + j + 16 * i];
        w3[i] = uW[uW3 + j + 16 * i];
      }
      const float b3 = uW[uB3], yr = sY[r];
      float qp = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) qp += w3[i] * h[i];
      SK_FT5(k, 7);
      const float q = sum16(qp) + b3;
      const float e = q - yr, dq = e * (2.f / kB);
      SK_FT5(k, 8);
      float g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = h[i] > 0.f ? dq * w3[i] : 0.f;
      if (j == 0) {
        sDQ[r] = dq;
        sL[r] = e * e;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int u = j + 16 * i;
        sDZ[r * LZ + u] = g[i];
        sDZT[u * LZT + r] = g[i];
      }
    }
    SK_FT5(k, 9);
    if (wg_any(fail, sFail + 4 * (k & 1))) break;  // a lost exchange ends the launch (uniformly)
    SK_FT(k, 5);
    if (more) {  // the next step's rows (that buffer's last readers were in step k - 1)
      float* nS = sm + cRows + ((k + 1) & 1) * kRowsN;
      if (t < kB * kS) nS[(t / kS) * LS + t % kS] = nx;
      else if (t < kB * kS + 3 * kB) nS[kB * LS + (t - kB * kS)] = nx;
    }
    if (a.losses && d == 0 && t == 0) {
      float l = 0.f;
#pragma unroll
      for (int r = 0; r < kB; ++r) l += sL[r];
      a.losses[k] = l / kB;
    }

    // (7) dL/dh1d of the own columns (waves 0 / 1 end with layer 1's layout),
    //     dz1 = dh1d x the Dropout / relu mask, (8) dW1 | db1 and their Adam
    //     steps on registers; (9) dW2[:, C_d] and its Adam steps in the
    //     epilogue (the W2 mirror's reads by (7) are behind its barrier)
    const f32x4 dh = backward_dh1<G>(sDZ, sW2, sPart, wv, lane, li, lg);
    SK_FT(k, 6);
    if (wv < NT1) {
      const f4 dz1 = {dh[0] * mask[0], dh[1] * mask[1], dh[2] * mask[2], dh[3] * mask[3]};
      dw1_adam(W1, M1, V1, dz1, sS, alpha, b1c, b2c, a.eps, li, lg);
    }
    if (wv >= 2) {
      // (6) meanwhile waves 2 / 3: the unit parameters' 16-row gradient sums
      //     (one unit per lane) and Adam steps (every W3 / b2 / W2A read of
      //     this step is behind the barriers above; the next are behind the
      //     next step's first)
      const int u = t - 2 * 64;
      float gw3 = 0.f, gb2 = 0.f, ga0 = 0.f, ga1 = 0.f;
#pragma unroll
      for (int r = 0; r < kB; ++r) {
        const float dz = sDZ[r * LZ + u];
        gw3 += sDQ[r] * sH2[r * LZ + u];
        gb2 += dz;
        ga0 += dz * sA[2 * r];
        ga1 += dz * sA[2 * r + 1];
      }
      adam_lds_n<4>(uW, uM, uV, {uW3 + u, uB2 + u, uWA + 2 * u, uWA + 2 * u + 1}, {gw3, gb2, ga0, ga1}, alpha, b1c,
                    b2c, a.eps);
      if (wv == 2) {  // b3: the 16 rows' dL/dq in row 0 of wave 2
        const float gb3 = sum16(lane < kB ? sDQ[lane] : 0.f);
        if (lane == 0) adam_lds(uW, uM, uV, uB3, gb3, alpha, b1c, b2c, a.eps);
      }
    }
    SK_FT7(k, 7);
    SK_FT7(k, 8);
    dw2_adam<G>(W2, M2, V2, sHDT, sDZT, sW2, alpha, b1c, b2c, a.eps, wv, li, lg);
    SK_FT7(k, 9);
    SK_FT(k, 10);
    // no barrier: the next step writes only the other buffers before its first
    // one; the W2 mirror's next reader (dh1) is behind three more
  }
  const float tk = adam_count(tk0, a.M);
  SK_FT_FLUSH();

  // the owned slice back; workgroup 0 the unit parameters and the counters
  w2_store<G, kCLd>(W2, a.flat, d, wv, li, lg);
  w2_store<G, kCLd>(M2, a.m, d, wv, li, lg);
  w2_store<G, kCLd>(V2, a.v, d, wv, li, lg);
  if (wv < NT1) {
    w1_store<G>(W1, a.flat, d, wv, li, lg);
    w1_store<G>(M1, a.m, d, wv, li, lg);
    w1_store<G>(V1, a.v, d, wv, li, lg);
  }
  __syncthreads();
  if (d == 0) {
    if (t < kH2) {
      const int gi[4] = {kCW3 + t, kCB2 + t, kW2 + t * kCLd + kH1, kW2 + t * kCLd + kH1 + 1};
      const int l4[4] = {uW3 + t, uB2 + t, uWA + 2 * t, uWA + 2 * t + 1};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.flat[gi[j]] = uW[l4[j]];
        a.m[gi[j]] = uM[l4[j]];
        a.v[gi[j]] = uV[l4[j]];
      }
    } else if (t == kH2) {
      a.flat[kCB3] = uW[uB3];
      a.m[kCB3] = uM[uB3];
      a.v[kCB3] = uV[uB3];
    }
    if (t == 0) {
      a.drop_calls[0] = call0 + a.M;
      a.epoch[0] = (unsigned long long)(ep0 + 2u * (unsigned)a.M);
      a.timeout[1] = (unsigned)place;  // the placement report
    }
    if (t < a.n_steps) a.steps[t] = tk;
  }
}

// ------------------------------------------------------------------ actor
// model_actor_fit_step (SkillshotLearner.py:386-417): the gradient of
// -sum_b Q(s_b, mu(s_b)) with the critic fixed (inference: no Dropout), one
// Adam step of the actor per minibatch.  The critic is frozen for the whole
// pass, so its part of Q that depends on s alone — the layer-2
// pre-activations without the action columns, zc = b2 + W2[:, :256]
// relu(W1 s + b1) — is computed for every row of the launch up front by one
// parallel kernel (k_fit_critic_z2, one workgroup per minibatch), and each
// step streams its 16 rows of zc in (prefetched a step ahead) instead of
// running the critic's layers 1 and 2 in the chain.  The actor itself takes
// the critic kernel's column split: workgroup d owns the actor's W1 | b1 of
// C_d and W2[:, C_d] in registers; its unit parameters (b2, W3, b3 with their
// moments) are in every workgroup's LDS, and each lane holds the critic's
// (W3, action columns) of the 8 units it reduces over in registers for the
// launch.  R reduce-scatters the actor's layer-2 partials, H all-gathers its
// h2; then every workgroup forms a = tanh(z3), the critic's dQ/da at (s, a),
// the actor's dL/dz2 and its unit parameters' Adam steps itself.

// zc[row][u] of the critic, for `M` minibatches of states (float [16 M][128])
constexpr int LH1 = kH1 + 4;
__global__ void __launch_bounds__(kT) k_fit_critic_z2(const float* __restrict__ critic,
                                                      const float* __restrict__ states, float* __restrict__ zc) {
  __shared__ __attribute__((aligned(16))) float sS[kB * LS];
  __shared__ __attribute__((aligned(16))) float sH[kB * LH1];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, li = lane & 15, lg = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * kB;
  if (t < kB * LS) {
    const int r = t / LS, j = t % LS;
    sS[t] = j < kS ? states[(row0 + r) * kS + j] : (j == kS ? 1.f : 0.f);
  }
  __syncthreads();
  // layer 1 (s with a column of ones against W1 | b1): wave w, unit tiles w + 4 q
  const f4 x = *(const f4*)(sS + li * LS + 4 * lg);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = 16 * (wv + 4 * q) + li;
    f4 w = {0.f, 0.f, 0.f, 0.f};
    if (lg < 3) {
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = critic[kW1 + u * kS + 4 * lg + j];
    } else {
      w[0] = critic[kB1 + u];
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = m16x4(x, w, acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) sH[(4 * lg + r) * LH1 + u] = fmaxf(acc[r], 0.f);
  }
  __syncthreads();
  // layer 2 over the 256 h1 columns: wave w, unit tiles w, w + 4
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int u = 16 * (wv + 4 * q) + li;
    const float* wr = critic + kW2 + u * kCLd;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int kk = 0; kk < kH1; kk += 16) {
      const f4 h = *(const f4*)(sH + li * LH1 + kk + 4 * lg);
      const f4 w = {wr[kk + 4 * lg], wr[kk + 4 * lg + 1], wr[kk + 4 * lg + 2], wr[kk + 4 * lg + 3]};
      acc = m16x4(h, w, acc);
    }
    const float b2 = critic[kCB2 + u];
#pragma unroll
    for (int r = 0; r < 4; ++r) zc[(row0 + 4 * lg + r) * kH2 + u] = acc[r] + b2;
  }
}

constexpr int aW3 = 0, aB2 = 2 * kH2, aB3 = 3 * kH2, kAUN = 3 * kH2 + 4;  // actor units: W3 [128][2], b2, b3[2]
// two of each per-step buffer (as the critic's): rows [s_ext 16 x 16],
// activations [h1 16 x LH | its transpose C x LHT], the critic's zc [16 x LZ]
template <class G>
struct ActorLayout {
  static constexpr int kARowsN = kB * LS, kAActN = kB * G::LH + G::C * LHT;
  static constexpr int xS = 3 * kAUN, xAct = xS + 2 * kARowsN, xZC = xAct + 2 * kAActN,
                       xDZ3 = xZC + 2 * kB * LZ, xH2 = xDZ3 + 2 * kB, xDZ = xH2 + kB * LZ, xDZT = xDZ + kB * LZ,
                       xW2 = xDZT + kH2 * LZT, xPart = xW2 + kH2 * G::LW, xAlpha = xPart + 3 * 64 * 4,
                       xEnd = xAlpha + kAlphaN;
  static constexpr size_t kLds = (size_t)xEnd * 4;
  // exchanges: R [P src][P dst][U][16], H [P][U][16]
  static constexpr int axR = 0, axH = axR + G::P * G::P * G::U * 16, axN = axH + G::P * G::U * 16;
  static_assert(kLds <= 150 * 1024 && axN <= kXPlace, "LDS / xbuf");
};
constexpr int kZPer = kB * kH2 / kT;  // zc floats per thread and step

template <int PW>
__global__ void __launch_bounds__(kT) k_fit_actor(FitArgs a, const float* __restrict__ zc) {
  using G = Geo<PW>;
  using Y = ActorLayout<G>;
  constexpr int P = G::P, U = G::U, LH = G::LH, NT1 = G::NT1;
  constexpr int kARowsN = Y::kARowsN, kAActN = Y::kAActN, xS = Y::xS, xAct = Y::xAct, xZC = Y::xZC,
                axR = Y::axR, axH = Y::axH;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ __attribute__((aligned(16))) int sFail[8];
  SK_FT_DECL
  if (blockIdx.x % a.stride) return;
  float* uW = sm;
  float* uM = sm + kAUN;
  float* uV = sm + 2 * kAUN;
  float* sDZ3 = sm + Y::xDZ3;
  float* sH2 = sm + Y::xH2;
  float* sDZ = sm + Y::xDZ;
  float* sDZT = sm + Y::xDZT;
  float* sW2 = sm + Y::xW2;
  float* sPart = sm + Y::xPart;
  float* sAlpha = sm + Y::xAlpha;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, li = lane & 15, lg = lane >> 4;
  const int d = blockIdx.x / a.stride;
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(a.xbuf);

  W2Reg<G> W2, M2, V2;
  w2_load<G, kH1>(W2, a.flat, d, wv, li, lg);
  w2_load<G, kH1>(M2, a.m, d, wv, li, lg);
  w2_load<G, kH1>(V2, a.v, d, wv, li, lg);
  w2_mirror<G>(W2, sW2, wv, li, lg);
  // waves w < NT1: the actor's W1 | b1 (n-tile wv)
  f4 W1 = {0.f, 0.f, 0.f, 0.f}, M1 = W1, V1 = W1;
  if (wv < NT1) {
    W1 = w1_load<G>(a.flat, d, wv, li, lg);
    M1 = w1_load<G>(a.m, d, wv, li, lg);
    V1 = w1_load<G>(a.v, d, wv, li, lg);
  }
  // a use of the loaded slice here, so their vmcnt wait is placed before the
  // step loop (first used inside it, the wait went inside it: a vmcnt(0) at
  // every step's layer-1 MFMAs, behind whatever memory traffic was in flight)
  asm volatile("" ::"v"(W1), "v"(M1), "v"(V1));
  if (t < kH2) {
    const int gi[3] = {kAW3 + t, kAW3 + kH2 + t, kAB2 + t};
    const int l3[3] = {aW3 + 2 * t, aW3 + 2 * t + 1, aB2 + t};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      uW[l3[j]] = a.flat[gi[j]];
      uM[l3[j]] = a.m[gi[j]];
      uV[l3[j]] = a.v[gi[j]];
    }
  } else if (t < kH2 + 2) {
    const int j = t - kH2;
    uW[aB3 + j] = a.flat[kAB3 + j];
    uM[aB3 + j] = a.m[kAB3 + j];
    uV[aB3 + j] = a.v[kAB3 + j];
  }
  const unsigned ep0 = (unsigned)a.epoch[0];
  const float tk0 = a.steps[0];
  const int place = fit_placement<P>(xr, d, ep0, a.timeout);
  const bool local = place == 2;
  const int M = place ? a.M : 0;  // a lost workgroup: no step runs (*timeout is set)
  if (t < kB * LS) {
    const int r = t / LS, j = t % LS;
    sm[xS + t] = j < kS ? a.states[r * kS + j] : (j == kS ? 1.f : 0.f);
    sm[xS + kARowsN + t] = j == kS ? 1.f : 0.f;
  }
#pragma unroll
  for (int i = 0; i < kZPer; ++i) {
    const int idx = t + kT * i;
    sm[xZC + (idx / kH2) * LZ + idx % kH2] = zc[idx];
  }
  const float b1c = 1.f - a.beta1, b2c = 1.f - a.beta2;
  bool fail = false;
  // the frozen critic's unit parameters of this lane's 8 units (t % 16 + 16 i), held for the launch
  float cwa0[8], cwa1[8], cw3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int u = (t & 15) + 16 * i;
    cw3[i] = a.critic[kCW3 + u];
    cwa0[i] = a.critic[kW2 + u * kCLd + kH1];
    cwa1[i] = a.critic[kW2 + u * kCLd + kH1 + 1];
  }

  for (int k = 0; k < M; ++k) {
    const unsigned E = ep0 + 2u * (unsigned)k;
    if (k % kAlphaN == 0) alpha_fill(a, sAlpha, tk0, k);
    const float alpha = sAlpha[k % kAlphaN];
    float* sS = sm + xS + (k & 1) * kARowsN;
    float* sH1 = sm + xAct + (k & 1) * kAActN;
    float* sH1T = sH1 + kB * LH;
    const float* sZC = sm + xZC + (k & 1) * kB * LZ;
    SK_FT(k, 0);
    const bool more = k + 1 < a.M;

    // (1) layer 1 of the own units on waves w < NT1 (the relu mask kept in registers)
    f4 hmask = {0.f, 0.f, 0.f, 0.f};
    if (wv < NT1) {
      const f32x4 z = layer1(sS, W1, li, lg);
      const int c = 16 * wv + li;
      f4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = fmaxf(z[r], 0.f);
        hmask[r] = z[r] > 0.f ? 1.f : 0.f;
        sH1[(4 * lg + r) * LH + c] = h[r];
      }
      *(f4*)(sH1T + c * LHT + 4 * lg) = h;
    }
    __syncthreads();
    SK_FT(k, 1);

    // (2) the layer-2 partials over the own columns, to the unit summers
    partials_publish<G>(sH1, W2, xr, E + 1, local, wv, li, lg, [&](int e) { return axR + (d * P + e) * U * 16; });
    // the next step's rows and zc into registers (stored after phase 5;
    // issued here they land under the exchange waits)
    float nx = 0.f;
    float nz[kZPer];
    if (more) {
      if (t < kB * kS) nx = a.states[(int64_t)(k + 1) * kB * kS + t];
#pragma unroll
      for (int i = 0; i < kZPer; ++i) nz[i] = zc[(int64_t)(k + 1) * kB * kH2 + t + kT * i];
    }
    SK_FT(k, 2);

    // (3) the sums of U_d: h2 = relu(z2 + b2), published to all (H)
    if (t < U * 8) {
      float z0, z1;
      fail |= !r_sum<G>(xr, E + 1, t, [&](int s) { return axR + (s * P + d) * U * 16; }, z0, z1, a.timeout);
      const float b2 = uW[aB2 + U * d + (2 * t) / 16];
      put2(xr, (uint32_t)(axH + 2 * h_pair<G>(d, (t % 8), t / 8)) * 8u, E + 2, fmaxf(z0 + b2, 0.f),
           fmaxf(z1 + b2, 0.f), local);
    }
    SK_FT(k, 3);

    // (4) h2 of all 128 units for this wave's rows
    fail |= !gather_h_rows<G>(xr, axH, E + 2, sH2, wv, lane, a.timeout);
    SK_FT(k, 4);

    // (5) every workgroup, lane (row t / 16, units t % 16 + 16 i), DPP row
    //     sums: z3 -> a = tanh(z3); the critic at (s, a): dQ/dz2 = W3 [z2 > 0],
    //     dQ/da; dL/dz3 = -dQ/da (1 - a^2) (L = -sum Q); the actor's dL/dz2
    //     (every operand read into registers first: read again after the
    //     first stores, each re-read waited for its own round trip)
    {
      const int r = t >> 4, j = t & 15;
      float h[8], zr[8];
      float2 w3[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int u = j + 16 * i;
        h[i] = sH2[r * LZ + u];
        w3[i] = *(const float2*)(uW + aW3 + 2 * u);
        zr[i] = sZC[r * LZ + u];
      }
      const float2 b3 = *(const float2*)(uW + aB3);
      float p0 = 0.f, p1 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        p0 += w3[i].x * h[i];
        p1 += w3[i].y * h[i];
      }
      SK_FT5(k, 7);
      const float a0 = tanh_nb(sum16(p0) + b3.x), a1 = tanh_nb(sum16(p1) + b3.y);
      float g0 = 0.f, g1 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float wa0 = cwa0[i], wa1 = cwa1[i];
        const float z = zr[i] + a0 * wa0 + a1 * wa1;
        const float dz = z > 0.f ? cw3[i] : 0.f;
        g0 += dz * wa0;
        g1 += dz * wa1;
      }
      SK_FT5(k, 8);
      const float e0 = -sum16(g0) * (1.f - a0 * a0), e1 = -sum16(g1) * (1.f - a1 * a1);
      float g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = h[i] > 0.f ? e0 * w3[i].x + e1 * w3[i].y : 0.f;
      if (j == 0) {
        sDZ3[2 * r] = e0;
        sDZ3[2 * r + 1] = e1;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int u = j + 16 * i;
        sDZ[r * LZ + u] = g[i];
        sDZT[u * LZT + r] = g[i];
      }
    }
    SK_FT5(k, 9);
    if (wg_any(fail, sFail + 4 * (k & 1))) break;  // a lost exchange ends the launch (uniformly)
    SK_FT(k, 5);
    if (more) {  // the next step's rows and zc (those buffers' last readers were in step k - 1)
      if (t < kB * kS) sm[xS + ((k + 1) & 1) * kARowsN + (t / kS) * LS + t % kS] = nx;
      float* nZ = sm + xZC + ((k + 1) & 1) * kB * LZ;
#pragma unroll
      for (int i = 0; i < kZPer; ++i) {
        const int idx = t + kT * i;
        nZ[(idx / kH2) * LZ + idx % kH2] = nz[i];
      }
    }

    // (7) dL/dh1[:, C_d], dz1 = dh1 [h1 > 0], dW1 | db1 (waves 0 / 1) and
    //     dW2[:, C_d] with their Adam steps
    const f32x4 dh = backward_dh1<G>(sDZ, sW2, sPart, wv, lane, li, lg);
    SK_FT(k, 6);
    if (wv < NT1) {
      const f4 dz1 = {dh[0] * hmask[0], dh[1] * hmask[1], dh[2] * hmask[2], dh[3] * hmask[3]};
      dw1_adam(W1, M1, V1, dz1, sS, alpha, b1c, b2c, a.eps, li, lg);
    }
    if (wv >= 2) {
      // (6) meanwhile waves 2 / 3: the actor's unit parameters' 16-row
      //     gradient sums (one unit per lane) and Adam steps
      const int u = t - 2 * 64;
      float gw0 = 0.f, gw1 = 0.f, gb2 = 0.f;
#pragma unroll
      for (int r = 0; r < kB; ++r) {
        const float hv = sH2[r * LZ + u];
        gw0 += sDZ3[2 * r] * hv;
        gw1 += sDZ3[2 * r + 1] * hv;
        gb2 += sDZ[r * LZ + u];
      }
      adam_lds_n<3>(uW, uM, uV, {aW3 + 2 * u, aW3 + 2 * u + 1, aB2 + u}, {gw0, gw1, gb2}, alpha, b1c, b2c, a.eps);
      if (wv == 2) {  // b3: dL/dz3 of the 16 rows, output j in row j of wave 2
        const float gb3 = sum16(lane < 2 * kB ? sDZ3[2 * (lane & 15) + (lane >> 4)] : 0.f);
        if (lane == 0 || lane == 16) adam_lds(uW, uM, uV, aB3 + (lane >> 4), gb3, alpha, b1c, b2c, a.eps);
      }
    }
    SK_FT7(k, 7);
    SK_FT7(k, 8);
    dw2_adam<G>(W2, M2, V2, sH1T, sDZT, sW2, alpha, b1c, b2c, a.eps, wv, li, lg);
    SK_FT7(k, 9);
    SK_FT(k, 10);
  }
  const float tk = adam_count(tk0, a.M);
  SK_FT_FLUSH();

  w2_store<G, kH1>(W2, a.flat, d, wv, li, lg);
  w2_store<G, kH1>(M2, a.m, d, wv, li, lg);
  w2_store<G, kH1>(V2, a.v, d, wv, li, lg);
  if (wv < NT1) {
    w1_store<G>(W1, a.flat, d, wv, li, lg);
    w1_store<G>(M1, a.m, d, wv, li, lg);
    w1_store<G>(V1, a.v, d, wv, li, lg);
  }
  __syncthreads();
  if (d == 0) {
    if (t < kH2) {
      const int gi[3] = {kAW3 + t, kAW3 + kH2 + t, kAB2 + t};
      const int l3[3] = {aW3 + 2 * t, aW3 + 2 * t + 1, aB2 + t};
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        a.flat[gi[j]] = uW[l3[j]];
        a.m[gi[j]] = uM[l3[j]];
        a.v[gi[j]] = uV[l3[j]];
      }
    } else if (t < kH2 + 2) {
      const int j = t - kH2;
      a.flat[kAB3 + j] = uW[aB3 + j];
      a.m[kAB3 + j] = uM[aB3 + j];
      a.v[kAB3 + j] = uV[aB3 + j];
    }
    if (t == 0) {
      a.epoch[0] = (unsigned long long)(ep0 + 2u * (unsigned)a.M);
      a.timeout[1] = (unsigned)place;  // the placement report
    }
    if (t < a.n_steps) a.steps[t] = tk;
  }
}

// The resident kernels need up to ~150 KB of dynamic LDS per workgroup and
// their P workgroups resident together (include/skillshot.h,
// INTEGRATION.md): a device whose opt-in LDS limit is smaller, or a failed
// attribute call, is reported as SK_EHIP before anything is launched, and
// the Python layer takes the three-launch steps instead
template <typename K, typename... X>
int launch_fit(K kernel, int P, size_t lds, bool& attr, const FitArgs& a, hipStream_t st, X... extra) {
  if (!attr) {
    int dev = 0, optin = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess ||
        (size_t)optin < lds)
      return SK_EHIP;
    if (hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return SK_EHIP;
    attr = true;
  }
  kernel<<<P * a.stride, kT, lds, st>>>(a, extra...);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

// SK_FIT_P: the workgroups per pass (8 or 16; default 16)
int fit_p() {
  const char* e = getenv("SK_FIT_P");
  return (e && atoi(e) == 8) ? 8 : 16;
}

// The workgroups' placement: by default a grid of 8 P blocks, every 8th
// working, which the round-robin dispatch puts on ONE XCD, so the exchanges
// run through that XCD's L2 (fit_placement checks it in every launch; with
// write-through stores one XCD had been no faster than spread: critic
// 5.25-5.30 vs 5.32-5.36 us, profiles/r05u_bench_fit.jsonl; with plain stores
// 4.4 / 4.6 us, profiles/r05zi_bench_fit_local.jsonl).  SK_FIT_XCD=0: P blocks,
// spread over the XCDs (write-through stores).
int fit_stride() {
  const char* e = getenv("SK_FIT_XCD");
  return (e && atoi(e) == 0) ? 1 : 8;
}

}  // namespace

extern "C" {

#ifdef SK_TRACE_FIT
int skdiag_set_fit_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(sk_fit_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

size_t sk_fit_xbuf_bytes(void) { return (size_t)65536 * 8; }

int sk_fit_critic_f32(float* critic_flat, float* m, float* v, float* steps, int32_t n_steps, const float* states,
                      const float* actions, const float* targets, int32_t n_minibatches, uint64_t drop_seed,
                      int64_t* drop_calls, float lr, float beta1, float beta2, float eps, void* xbuf,
                      uint64_t* epoch, uint32_t* timeout, float* losses, void* stream) {
  if (!critic_flat || !m || !v || !steps || n_steps < 1 || n_steps > 64 || !states || !actions || !targets ||
      n_minibatches < 1 || !drop_calls || !xbuf || !epoch || !timeout)
    return SK_EINVAL;
  if (((uintptr_t)xbuf) & 15) return SK_EINVAL;
  FitArgs a{critic_flat, m, v, steps, n_steps, states, actions, targets, n_minibatches, drop_seed, drop_calls,
            lr, beta1, beta2, eps, (unsigned long long*)xbuf, (unsigned long long*)epoch, timeout, losses,
            fit_stride(), nullptr};
  static bool attr8 = false, attr16 = false;
  if (fit_p() == 8)
    return launch_fit(k_fit_critic<8>, 8, CriticLayout<Geo<8>>::kLds, attr8, a, (hipStream_t)stream);
  return launch_fit(k_fit_critic<16>, 16, CriticLayout<Geo<16>>::kLds, attr16, a, (hipStream_t)stream);
}

int sk_fit_actor_f32(float* actor_flat, float* adam_m, float* adam_v, float* step_counters, int32_t n_steps,
                     const float* critic_flat, const float* states, int32_t n_minibatches, float lr, float beta1,
                     float beta2, float eps, void* xbuf, uint64_t* epoch, uint32_t* timeout, float* zbuf,
                     void* stream) {
  if (!actor_flat || !adam_m || !adam_v || !step_counters || n_steps < 1 || n_steps > 64 || !critic_flat ||
      !states || n_minibatches < 1 || !xbuf || !epoch || !timeout || !zbuf)
    return SK_EINVAL;
  if (((uintptr_t)xbuf) & 15) return SK_EINVAL;
  const hipStream_t st = (hipStream_t)stream;
  k_fit_critic_z2<<<n_minibatches, kT, 0, st>>>(critic_flat, states, zbuf);
  if (hipGetLastError() != hipSuccess) return SK_EHIP;
  FitArgs a{actor_flat, adam_m, adam_v, step_counters, n_steps, states, nullptr, nullptr, n_minibatches, 0, nullptr,
            lr, beta1, beta2, eps, (unsigned long long*)xbuf, (unsigned long long*)epoch, timeout, nullptr,
            fit_stride(), critic_flat};
  static bool attr8 = false, attr16 = false;
  if (fit_p() == 8)
    return launch_fit(k_fit_actor<8>, 8, ActorLayout<Geo<8>>::kLds, attr8, a, st, (const float*)zbuf);
  return launch_fit(k_fit_actor<16>, 16, ActorLayout<Geo<16>>::kLds, attr16, a, st, (const float*)zbuf);
}

}  // extern "C"
