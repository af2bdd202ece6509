// sk_update.hip — the DDPG update on MFMA (gfx950): critic and actor
// forward + backward over a minibatch in one launch each, then one launch
// that reduces the per-workgroup weight gradients and applies Adam (and the
// soft target update).  Replaces, per update, the ~100 small torch kernels
// of DDPG.critic_step / model_actor_fit_step / soft_update
// (skillshot_learning_amd/learner.py; reference rule SkillshotLearner.py
// :386-443, nets :70-121).
//
//   k_grad_pack    a net's weights -> bf16 MFMA fragments (W1, W2, W2^T) +
//                  fp32 tail (biases, critic action columns, W3)
//   k_critic_grad  critic train step: Dropout(0.2) forward, MSE to the
//                  targets, backward; per-workgroup gradient partials
//   k_actor_grad   actor step: actor forward, critic forward (inference),
//                  dQ/da, actor backward of -sum Q; gradient partials
//   k_adam_flat    sum of the partials (+ optional flat-gradient output for an
//                  RCCL all-reduce), Adam (torch formulation, Keras eps),
//                  optional soft update of a target net
//
// Layout.  Activations are batch-major in LDS (row = batch row, k
// contiguous) so that every MFMA operand is a 16-byte LDS read or a 1 KiB
// coalesced fragment load: v_mfma_f32_32x32x16_bf16 computes D[32x32] +=
// A[32x16] B[16x32]; lane l holds A[l%32][8(l/32)+j] and B[8(l/32)+j][l%32]
// (j = 0..7), and D register v of lane l is D[8(v/4) + 4(l/32) + v%4][l%32].
// An operand is "k-contiguous" when stored as [M][K] (A) or [N][K] (B); the
// weight-gradient GEMMs contract over the batch, so the activations they
// need are written to LDS twice, batch-major and transposed.
//
// A workgroup of 8 waves (two per SIMD: one wave's VALU epilogue overlaps the
// other's MFMA chain) owns a contiguous range of 32-row sub-tiles and keeps
// its weight-gradient accumulators (AGPRs) across them: wave w holds dW2 rows
// 32(w%4).. x columns 128(w/4).. (4 MFMA tiles) and dW1 rows 32w.. (1 tile);
// layer 1 / dH1 use the 32-unit tile w.  Layer 2 (128 units) takes four
// waves per net, so waves 0-3 and 4-7 run two nets' layer 2 side by side.
// Operands are bf16, accumulation fp32; biases, the critic's action columns,
// layer 3 and the losses are fp32 VALU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"
#include "sk_partial.hpp"
#include "sk_split.hpp"

namespace {

using namespace skmlp;

constexpr int kThreads = 512;  // 8 waves, two per SIMD

// Phase timestamps of the first and last workgroup (diagnostic builds only:
// -DSK_TRACE, read back with sk_debug_update_trace; tools/trace_update.py)
#ifdef SK_TRACE
__device__ unsigned long long g_sk_trace[2][32][2];
#define SK_TP(k)                                                                             \
  do {                                                                                       \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1)) {              \
      const int wg_ = blockIdx.x == 0 ? 0 : 1;                                               \
      g_sk_trace[wg_][k][0] = __builtin_amdgcn_s_memtime();                                  \
      g_sk_trace[wg_][k][1] = wall_clock64();                                                \
    }                                                                                        \
  } while (0)
#else
#define SK_TP(k) \
  do {           \
  } while (0)
#endif

// grad pack layout (bytes)
constexpr size_t kGW1 = 0;                        // 8 frags   (n-tile of 256 hidden)
constexpr size_t kGW2 = kGW1 + 8 * 1024;          // 64 frags  (nt 0..3 of 128 out) x (kk 0..15 of 256 in)
constexpr size_t kGW2T = kGW2 + 64 * 1024;        // 64 frags  (nt 0..7 of 256 in)  x (kk 0..7 of 128 out)
constexpr size_t kGTail = kGW2T + 64 * 1024;      // fp32 [1024]
constexpr size_t kGPackBytes = kGTail + 1024 * 4;
// tail (fp32 offsets)
constexpr int kTB1 = 0, kTB2 = 256, kTW2a = 384, kTW3 = 640, kTB3 = 896;

// flat parameter offsets (torch parameters() order)
constexpr int kPW1 = 0, kPB1 = kPW1 + kH1 * kIn, kPW2 = kPB1 + kH1;
constexpr int kCPW2ld = kH1 + 2;  // critic W2 row length (h1 then the action)
constexpr int kCPB2 = kPW2 + kH2 * kCPW2ld, kCPW3 = kCPB2 + kH2, kCPB3 = kCPW3 + kH2, kCP = kCPB3 + 1;
constexpr int kAPB2 = kPW2 + kH2 * kH1, kAPW3 = kAPB2 + kH2, kAPB3 = kAPW3 + kOut * kH2, kAP = kAPB3 + kOut;
static_assert(kCP == 36609 && kAP == 36482 && kCP == skpart::kCriticParams && kPW2 == skpart::kPW2, "parameter counts");

// LDS leading dimensions (bf16 elements unless noted): +8 (16 B) per row
// rotates the banks of successive rows for the 16-byte fragment reads
constexpr int kLdS = 24, kLdT = 40, kLdH1 = 264, kLdH2f = 132, kLdZ2 = 136;

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// k-contiguous fragment from LDS: lane l gets X[row0 + l%32][k0 + 8(l/32) .. +7]
__device__ __forceinline__ bf16x8 lfrag(const short* X, int ld, int row0, int k0, int lane) {
  return *(const bf16x8*)(X + (row0 + (lane & 31)) * ld + k0 + 8 * (lane >> 5));
}
__device__ __forceinline__ int drow(int v, int lane) { return 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3); }
__device__ __forceinline__ float bf2f(short s) { return __uint_as_float(((uint32_t)(uint16_t)s) << 16); }

// D registers 4g..4g+3 of a lane are 4 consecutive rows: store them to a
// transposed [col][row] bf16 array with one 8-byte write
__device__ __forceinline__ void store_t4(short* XT, int ld, int col, int row, float a, float b, float c, float d) {
  const uint32_t lo = (uint32_t)(uint16_t)f2bf(a) | ((uint32_t)(uint16_t)f2bf(b) << 16);
  const uint32_t hi = (uint32_t)(uint16_t)f2bf(c) | ((uint32_t)(uint16_t)f2bf(d) << 16);
  *(uint2*)(XT + col * ld + row) = make_uint2(lo, hi);
}

// ---------------------------------------------------------------- pack
// W1 [256][12], W2 [128][ld2] (first 256 columns on MFMA; critic: columns
// 256, 257 are the action), W3 [n_out][128]
__device__ __forceinline__ void grad_pack_body(int t, const float* W1, const float* b1, const float* W2, int ld2,
                                               const float* b2, const float* W3, const float* b3, int n_out,
                                               char* out) {
  if (t < 8 * 64) {  // W1: B operand of layer 1 (n = hidden unit, k = input)
    short* o = (short*)(out + kGW1) + t * 8;
    const int nt = t >> 6, lane = t & 63;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * (lane >> 5) + j;
      o[j] = f2bf(k < kIn ? W1[(32 * nt + (lane & 31)) * kIn + k] : 0.f);
    }
  } else if (t < 8 * 64 + 64 * 64) {  // W2: B operand of layer 2 (n = out unit, k = in unit)
    const int u = t - 8 * 64, f = u >> 6, lane = u & 63, nt = f >> 4, kk = f & 15;
    short* o = (short*)(out + kGW2) + u * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(W2[(32 * nt + (lane & 31)) * ld2 + 16 * kk + 8 * (lane >> 5) + j]);
  } else if (t < 8 * 64 + 2 * 64 * 64) {  // W2^T: B operand of dH1 = dZ2 W2 (n = in unit, k = out unit)
    const int u = t - 8 * 64 - 64 * 64, f = u >> 6, lane = u & 63, nt = f >> 3, kk = f & 7;
    short* o = (short*)(out + kGW2T) + u * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(W2[(16 * kk + 8 * (lane >> 5) + j) * ld2 + 32 * nt + (lane & 31)]);
  } else if (t < 8 * 64 + 2 * 64 * 64 + 1024) {
    const int u = t - 8 * 64 - 2 * 64 * 64;
    float v = 0.f;
    if (u < kTB2) v = b1[u];
    else if (u < kTW2a) v = b2[u - kTB2];
    else if (u < kTW3) v = ld2 > kH1 ? W2[((u - kTW2a) >> 1) * ld2 + kH1 + ((u - kTW2a) & 1)] : 0.f;
    else if (u < kTB3) v = (u - kTW3) < n_out * kH2 ? W3[u - kTW3] : 0.f;
    else if (u < kTB3 + n_out) v = b3[u - kTB3];
    ((float*)(out + kGTail))[u] = v;
  }
}
constexpr int kPackThreads = 8 * 64 + 2 * 64 * 64 + 1024;

__global__ void k_grad_pack(const float* W1, const float* b1, const float* W2, int ld2, const float* b2,
                            const float* W3, const float* b3, int n_out, char* out) {
  grad_pack_body(blockIdx.x * blockDim.x + threadIdx.x, W1, b1, W2, ld2, b2, W3, b3, n_out, out);
}

// up to 4 nets stored flat in torch parameters() order (W1 [256][12], b1,
// W2 [128][ld2], b2, W3 [n_out][128], b3), one per blockIdx.y
struct PackJobs {
  const float* flat[4];
  char* out[4];
  int ld2[4];
  int n_out[4];
};

__global__ void k_grad_pack_flat(PackJobs j) {
  const int y = blockIdx.y;
  const float* f = j.flat[y];
  const int ld2 = j.ld2[y];
  const float* W2 = f + kPW2;
  const float* b2 = W2 + kH2 * ld2;
  const float* W3 = b2 + kH2;
  grad_pack_body(blockIdx.x * blockDim.x + threadIdx.x, f + kPW1, f + kPB1, W2, ld2, b2, W3, W3 + j.n_out[y] * kH2,
                 j.n_out[y], j.out[y]);
}

// ---------------------------------------------------------------- shared pieces
// LDS-only workgroup barrier: waits for this wave's LDS traffic but not its
// global loads, so the weight fragments prefetched for the next phase stay
// in flight across it (the waves of these kernels exchange data through LDS
// only; global results are written after the last barrier)
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// Pointers laundered through inline asm (against LICM, below) lose their
// address space, and a FLAT load counts on lgkmcnt too, so every LDS wait
// (lds_sync) would also wait for the weight prefetches: loads through these
// casts stay GLOBAL loads
typedef const __attribute__((address_space(1))) bf16x8* gfrag_t;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f4v* gf4_t;

// Re-derive the lane id inside a sub-tile loop: without this LICM hoists every
// lane-dependent LDS / tail address of the loop body out of it and spills them
__device__ __forceinline__ int launder_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}
// a wave's LDS write, then its read of another lane's value: LDS operations of
// one wave complete in order, this only keeps the compiler from reordering
__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local"); }

// LDS of both gradient kernels.  H1a (the critic kernel's target-actor h1,
// phases 1-2) aliases DZ1T (dz1, phase 5); H1B holds the second net's h1
// (critic: target critic, actor: critic).  QP / MP / YP / DP are per-wave
// partial row sums (halfsum32) of the layer-2 epilogues.
struct Lds {
  short *Sr, *S2r, *ST, *H1, *H1B, *H1T, *DZ2, *DZ2T, *DZ1T, *H1a;
  float *H2f, *TL, *A, *Y, *RB, *DB, *RED, *AW, *DW, *QP, *MP, *YP, *DP;
};
constexpr size_t kSzS = 32 * kLdS * 2, kSzT = 32 * kLdT * 2, kSzH1 = 32 * kLdH1 * 2, kSzH1T = kH1 * kLdT * 2;
constexpr size_t kSzZ2 = 32 * kLdZ2 * 2, kSzZ2T = kH2 * kLdT * 2, kSzH2f = 32 * kLdH2f * 4;
constexpr int kSmallF = 64 + 32 + 32 + 32 + 4 + 8 * 64 + 8 * 64 + 4 * 32 + 4 * 64 + 4 * 32 + 4 * 64;
constexpr size_t kLdsGrad = 2 * kSzS + kSzT + 2 * kSzH1 + kSzH1T + kSzZ2 + kSzZ2T + kSzH1T + kSzH2f +
                            3 * 1024 * 4 + kSmallF * 4;
static_assert(kSzH1 <= kSzH1T, "LDS alias");
static_assert(kLdsGrad <= 160 * 1024, "LDS budget of one CU");

__device__ __forceinline__ Lds carve(char* smem) {
  Lds L;
  char* p = smem;
  L.Sr = (short*)p;   p += kSzS;
  L.S2r = (short*)p;  p += kSzS;
  L.ST = (short*)p;   p += kSzT;
  L.H1 = (short*)p;   p += kSzH1;
  L.H1B = (short*)p;  p += kSzH1;
  L.H1T = (short*)p;  p += kSzH1T;
  L.DZ2 = (short*)p;  p += kSzZ2;
  L.DZ2T = (short*)p; p += kSzZ2T;
  L.DZ1T = (short*)p; p += kSzH1T;
  L.H2f = (float*)p;  p += kSzH2f;
  L.TL = (float*)p;   p += 3 * 1024 * 4;
  float* f = (float*)p;
  L.A = f;   f += 64;
  L.Y = f;   f += 32;
  L.RB = f;  f += 32;
  L.DB = f;  f += 32;
  L.RED = f; f += 4;
  L.AW = f;  f += 8 * 64;
  L.DW = f;  f += 8 * 64;
  L.QP = f;  f += 4 * 32;  // per-wave partial row sums over a wave's 32 units: [wave][row]
  L.MP = f;  f += 4 * 64;  //                                                  [wave][row][2]
  L.YP = f;  f += 4 * 32;
  L.DP = f;
  L.H1a = L.DZ1T;
  return L;
}

// Phase 0 of a sub-tile issues every global load first (states, actions or
// targets, s', r, done; on the first sub-tile also the nets' fp32 tails) so
// that their latencies overlap, then writes LDS.  Thread t < 512 owns state
// element (row t / 16, input t % 16) and tail float4s t and t + 512.
__device__ __forceinline__ float load_state(const float* S, int64_t row0, int64_t B, int tid) {
  const int i = tid >> 4, k = tid & 15;
  return (k < kIn && row0 + i < B) ? S[(row0 + i) * kIn + k] : 0.f;
}
__device__ __forceinline__ void put_state(short* Xr, short* XT, float v, int tid) {
  const int i = tid >> 4, k = tid & 15;
  const short b = f2bf(v);
  Xr[i * kLdS + k] = b;
  if (XT && k < kIn) XT[k * kLdT + i] = b;  // rows 12..31 of XT stay zero from the kernel start
}
// tails of n <= 3 nets: waves 0-3 load net 0's 256 float4s, waves 4-7 net 1's,
// and waves 0-3 also net 2's (wave-uniform pointer choice: global loads)
__device__ __forceinline__ void load_tails(f4v& a, f4v& b, const char* p0, const char* p1, const char* p2, int n,
                                           int w, int tid) {
  if (w < 4 || n > 1) a = ((gf4_t)((w < 4 ? p0 : p1) + kGTail))[tid & 255];
  if (n > 2 && w < 4) b = ((gf4_t)(p2 + kGTail))[tid];
}
__device__ __forceinline__ void put_tails(float* TL, f4v a, f4v b, int n, int w, int tid) {
  if (w < 4 || n > 1) ((f4v*)TL)[tid] = a;
  if (n > 2 && w < 4) ((f4v*)TL)[512 + tid] = b;
}

// keep bits of the critic's training Dropout for n-tile nt: bit 4g + q is row
// drow(4g, lane) + q of the sub-tile, unit 32 nt + lane % 32.  The mask of
// GLOBAL batch row key + i (the 1-rank batch's row numbering; key is a
// multiple of 4: learner.DDPG, rng.dropout_keep), P(drop) = 0.2 (Dropout(0.2),
// SkillshotLearner.py:110).  Data-independent: computed while phase 0's loads fly.
__device__ __forceinline__ uint32_t dropout_bits(uint64_t seed, uint64_t call, int64_t key, int nt, int lane) {
  const uint32_t n = 32 * nt + (lane & 31);
  uint32_t bits = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint4 u = philox(make_uint4((uint32_t)((key + drow(4 * g, lane)) >> 2), n, (uint32_t)call,
                                      (uint32_t)(call >> 32)),
                           (uint32_t)seed, (uint32_t)(seed >> 32));
    bits |= ((uint32_t)(u.x >= 858993460u) | ((uint32_t)(u.y >= 858993460u) << 1) |
             ((uint32_t)(u.z >= 858993460u) << 2) | ((uint32_t)(u.w >= 858993460u) << 3)) << (4 * g);
  }
  return bits;
}

// per-row LDS values for the 4 consecutive rows i0 .. i0 + 3 of an
// accumulator register group (i0 a multiple of 4): X[i], and X[2i], X[2i+1]
__device__ __forceinline__ float4 rows4(const float* X, int i0) { return *(const float4*)(X + i0); }
__device__ __forceinline__ void pairs4(const float* X, int i0, float x0[4], float x1[4]) {
  const float4 p = *(const float4*)(X + 2 * i0), q = *(const float4*)(X + 2 * i0 + 4);
  x0[0] = p.x; x1[0] = p.y; x0[1] = p.z; x1[1] = p.w;
  x0[2] = q.x; x1[2] = q.y; x0[3] = q.z; x1[3] = q.w;
}

// layer-1 fragment of n-tile w
__device__ __forceinline__ bf16x8 load_l1(const char* pack, int w, int lane) {
  return ((gfrag_t)(pack + kGW1))[w * 64 + lane];
}

// layer 1 of one net for n-tile nt (its fragment prefetched): relu(S W1^T +
// b1) -> batch-major (and, if HT, transposed) bf16; DROP applies the
// critic's training Dropout with the precomputed keep bits
template <bool DROP>
__device__ __forceinline__ void layer1(const short* Sx, bf16x8 wfrag, const float* tail, int nt, int lane, short* H,
                                       short* HT, uint32_t keep_bits) {
  f32x16 acc = {0};
  acc = mfma(lfrag(Sx, kLdS, 0, 0, lane), wfrag, acc);
  const int n = 32 * nt + (lane & 31);
  const float b = tail[kTB1 + n];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float hv[4];
    const int i0 = drow(4 * g, lane);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float z = fmaxf(acc[4 * g + q] + b, 0.f);
      if (DROP) {
        z = (keep_bits >> (4 * g + q)) & 1u ? z * 1.25f : 0.f;
      }
      hv[q] = z;
      H[(i0 + q) * kLdH1 + n] = f2bf(z);
    }
    if (HT) store_t4(HT, kLdT, n, i0, hv[0], hv[1], hv[2], hv[3]);
  }
}

// layer 2: the 16 weight fragments of out n-tile nt (issued a phase ahead),
// then the MFMA chain over the 256 hidden inputs
__device__ __forceinline__ void load_l2(bf16x8 wf[16], const char* pack, int nt, int lane) {
  const gfrag_t g = (gfrag_t)(pack + kGW2);
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) wf[kk] = g[(nt * 16 + kk) * 64 + lane];
}
__device__ __forceinline__ f32x16 l2_mfma(const short* H, const bf16x8 wf[16], int lane) {
  f32x16 acc = {0};
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    acc = mfma(lfrag(H, kLdH1, 0, 16 * kk, lane), wf[kk], acc);
    if ((kk & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // cap the hoisted LDS fragments (VGPRs)
  }
  return acc;
}
// W2^T fragments of the dH1 n-tile w (phase 5)
__device__ __forceinline__ void load_w2t(bf16x8 wt[8], const char* pack, int w, int lane) {
  const gfrag_t g = (gfrag_t)(pack + kGW2T);
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) wt[kk] = g[(w * 8 + kk) * 64 + lane];
}

// sum over the 32 lanes of each wave half (the 32 units of a layer-2 tile,
// per register = per row): DPP row_shr 1, 2, 4, 8 (16-lane inclusive scan,
// zero fill), then row_bcast:15 into rows 1 and 3; lanes 31 and 63 return
// their half's total
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, true));
}
__device__ __forceinline__ float halfsum32(float v) {
  v += dpp_f<0x111, 0xf>(v);
  v += dpp_f<0x112, 0xf>(v);
  v += dpp_f<0x114, 0xf>(v);
  v += dpp_f<0x118, 0xf>(v);
  v += dpp_f<0x142, 0xa>(v);
  return v;
}
// a lane-31 / lane-63 register group's row totals (4 consecutive rows from
// i0) into X[row], or interleaved as X[2 row + j]
__device__ __forceinline__ void put_rows4(float* X, const float v[4], int i0) {
  *(float4*)(X + i0) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void put_rows4x2(float* X, const float v0[4], const float v1[4], int i0) {
  *(float4*)(X + 2 * i0) = make_float4(v0[0], v1[0], v0[1], v1[1]);
  *(float4*)(X + 2 * i0 + 4) = make_float4(v0[2], v1[2], v0[3], v1[3]);
}

// the backward GEMMs shared by both kernels, given dZ2 (batch-major and
// transposed) in LDS and the W2^T fragments wt (prefetched):
//   dW2 tiles (w%4, 4(w/4)..+3) += dZ2^T H1     (accumulators gW2[4])
//   dZ1 = (dZ2 W2) * d relu1 (* 1.25 under Dropout) -> DZ1T; db1 partial
//   dW1 tile w += dZ1^T S                       (accumulator gW1)
template <bool DROP>
__device__ __forceinline__ void backward_12(const Lds& L, const bf16x8 wt[8], int w, int lane, f32x16 gW2[4],
                                            f32x16& gW1, float& gb1) {
  const int mt = w & 3, nt0 = 4 * (w >> 2);
  const bf16x8 a0 = lfrag(L.DZ2T, kLdT, 32 * mt, 0, lane), a1 = lfrag(L.DZ2T, kLdT, 32 * mt, 16, lane);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    gW2[t] = mfma(a0, lfrag(L.H1T, kLdT, 32 * (nt0 + t), 0, lane), gW2[t]);
    gW2[t] = mfma(a1, lfrag(L.H1T, kLdT, 32 * (nt0 + t), 16, lane), gW2[t]);
    __builtin_amdgcn_sched_barrier(0);
  }
  {
    f32x16 acc = {0};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) acc = mfma(lfrag(L.DZ2, kLdZ2, 0, 16 * kk, lane), wt[kk], acc);
    const int n = 32 * w + (lane & 31);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int i0 = drow(4 * g, lane);
      float d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float h = bf2f(L.H1[(i0 + q) * kLdH1 + n]);
        d[q] = h > 0.f ? acc[4 * g + q] * (DROP ? 1.25f : 1.0f) : 0.f;
        gb1 += d[q];
      }
      store_t4(L.DZ1T, kLdT, n, i0, d[0], d[1], d[2], d[3]);
    }
  }
  lds_sync();
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) gW1 = mfma(lfrag(L.DZ1T, kLdT, 32 * w, 16 * kk, lane), lfrag(L.ST, kLdT, 0, 16 * kk, lane), gW1);
}

// write a sub-tile's W1 / W2 gradients (W2: main 256 columns, the partial
// layout's 256-float rows) into the workgroup's partial row, or add them to it
// (later sub-tiles: each lane re-reads only what it wrote).  Storing per
// sub-tile keeps the 80 accumulator registers out of phases 0-4.  32 lanes of
// a register write 128 contiguous bytes.
__device__ __forceinline__ void store_w12(float* P, int w, int lane, const f32x16 gW2[4], const f32x16& gW1,
                                          bool add) {
  const int mt = w & 3, nt0 = 4 * (w >> 2);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      float* d = P + kPW2 + (32 * mt + drow(v, lane)) * kH1 + 32 * (nt0 + t) + (lane & 31);
      *d = add ? *d + gW2[t][v] : gW2[t][v];
    }
  const int k = lane & 31;
  if (k < kIn) {
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      float* d = P + kPW1 + (32 * w + drow(v, lane)) * kIn + k;
      *d = add ? *d + gW1[v] : gW1[v];
    }
  }
}
__device__ __forceinline__ void store_b1(float* P, int w, int lane, float gb1) {
  const float b = gb1 + __shfl_xor(gb1, 32, 64);
  if (lane < 32) P[kPB1 + 32 * w + lane] = b;
}

__device__ __forceinline__ int64_t ring_row_of(const skmlp::RingSample& q, int64_t b, int64_t t) {
  return skmlp::ring_row(q, b, t);
}

// ---------------------------------------------------------------- critic step
// Critic.forward in train mode + F.mse_loss(q, y) backward
// (DDPG.critic_step; critic.fit, SkillshotLearner.py:434): dL/dq =
// grad_scale * (q - y) with grad_scale = 2 / (global batch).  BOOT: y = r +
// gamma (1 - done) Q'(s', mu'(s')) from the target nets' packs, computed in
// the same phases as the training forward:
//   0  stage s, a (s', r, done); layer-1 fragments in flight
//   1  layer 1 (n-tile w) of the critic (Dropout), target actor, target critic
//   2  waves 0-3: critic layer 2 -> h2;  waves 4-7: target actor layer 2
//   3  waves 0-3: q = W3 h2 + b3;  waves 4-7: mu'(s') (each wave, all rows)
//      and the target critic's layer 2 at (s', mu'(s')) -> Q' terms
//   4  waves 0-3: y and dL/dq (each wave, all rows), dz2 of its units
//   5  dW2, dz1;  6  dW1
// Weight fragments are loaded one phase ahead of their MFMAs and the
// barriers are LDS-only (lds_sync), so no phase waits on a global load.
template <bool BOOT>
__global__ void __launch_bounds__(kThreads) k_critic_grad(const float* __restrict__ S, const float* __restrict__ A,
                                                          const float* __restrict__ Y, int64_t B, int64_t key_row0,
                                                          int sub_per_wg, float grad_scale, uint64_t seed,
                                                          const int64_t* __restrict__ call_ctr,
                                                          const char* __restrict__ gpack, float* __restrict__ partial,
                                                          float* step_ctr, int n_steps, float* __restrict__ loss_out,
                                                          uint8_t* __restrict__ mask_out, const float* __restrict__ S2,
                                                          const float* __restrict__ R, const float* __restrict__ D,
                                                          float gamma, const char* __restrict__ tapack,
                                                          const char* __restrict__ tcpack,
                                                          skmlp::RingSample rs = skmlp::RingSample{}) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve(smem);
  SK_TP(0);
  const int lane0 = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool l2 = w < 4;  // waves of the critic's own layer 2 (4-7: the target nets')
  const uint64_t call = (uint64_t)*call_ctr;
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  for (int t = threadIdx.x; t < 32 * kLdT; t += kThreads) L.ST[t] = 0;
  const float* TLc = L.TL;
  const float* TLa = L.TL + 1024;
  const float* TLt = L.TL + 2048;
  float* P = partial + (int64_t)blockIdx.x * kCP;
  float gb1 = 0.f, gb2 = 0.f, gw2a0 = 0.f, gw2a1 = 0.f, gw3 = 0.f, gb3 = 0.f, lsum = 0.f;
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  SK_TP(1);
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;  // uniform across the workgroup
    const int tid = launder_lane(threadIdx.x), lane = tid & 63, hh = lane >> 5, col = lane & 31;
    const int u = 32 * (w & 3) + col;  // the lane's layer-2 unit (of the critic or a target net)
    // launder the pack bases every sub-tile: otherwise LICM hoists every
    // (loop-invariant) fragment load out of the loop and spills
    const char* cp = gpack;
    const char* ap = tapack;
    const char* tp = tcpack;
    asm volatile("" : "+s"(cp), "+s"(ap), "+s"(tp));
    const bf16x8 f1c = load_l1(cp, w, lane);
    bf16x8 f1a = {}, f1t = {};
    if (BOOT) {
      f1a = load_l1(ap, w, lane);
      f1t = load_l1(tp, w, lane);
    }
    // ---- phase 0: every global load of the sub-tile, the Dropout bits while they fly, then LDS
    float sv, s2v, av, rv, dv;
    const bool rok = tid < 32 && row0 + tid < B;
    if (rs.ring) {  // the minibatch drawn from the replay ring here (sk_critic_grad_bootstrap_sampled)
      const int64_t t = *rs.total;
      const int64_t bs = row0 + (tid >> 4), ba = row0 + (tid >> 1), br = row0 + tid;
      const int ks = tid & 15;
      const bool oks = bs < B && t > 0 && ks < kIn, oka = tid < 64 && ba < B && t > 0, okr = rok && t > 0;
      const float* rows = rs.ring;
      const float* srow = rows + (oks ? ring_row_of(rs, bs, t) : 0) * 28;
      sv = oks ? srow[ks] : 0.f;
      s2v = BOOT && oks ? srow[15 + ks] : 0.f;
      av = oka ? rows[ring_row_of(rs, ba, t) * 28 + 12 + (tid & 1)] : 0.f;
      const float* rrow = rows + (okr ? ring_row_of(rs, br, t) : 0) * 28;
      rv = okr ? rrow[14] : 0.f;
      dv = BOOT && okr ? rrow[27] : 0.f;
      if (tid < 32 * 7 && row0 + tid / 7 < B && t > 0) {  // the sub-tile's rows into the sample buffers
        const int64_t b = row0 + tid / 7;
        const int k = tid - (tid / 7) * 7;
        const float4 v = *(const float4*)(rows + ring_row_of(rs, b, t) * 28 + 4 * k);
        skmlp::ring_scatter(rs, b, 4 * k, v.x);
        skmlp::ring_scatter(rs, b, 4 * k + 1, v.y);
        skmlp::ring_scatter(rs, b, 4 * k + 2, v.z);
        skmlp::ring_scatter(rs, b, 4 * k + 3, v.w);
      }
    } else {
      sv = load_state(S, row0, B, tid);
      s2v = BOOT ? load_state(S2, row0, B, tid) : 0.f;
      av = tid < 64 && row0 + (tid >> 1) < B ? A[row0 * 2 + tid] : 0.f;
      rv = rok ? (BOOT ? R[row0 + tid] : Y[row0 + tid]) : 0.f;
      dv = BOOT && rok ? D[row0 + tid] : 0.f;
    }
    f4v tla = {}, tlb = {};
    if (sub == 0) load_tails(tla, tlb, cp, ap, tp, BOOT ? 3 : 1, w, tid);
    uint32_t keep = dropout_bits(seed, call, key_row0 + row0, w, lane);
    asm volatile("" : "+v"(keep));  // computed here, under the loads' latency (not sunk into phase 1)
    if (mask_out) {  // the Dropout mask (tests): byte per (row, unit)
      const int n = 32 * w + col;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = drow(v, lane);
        if (row0 + i < B) mask_out[(row0 + i) * kH1 + n] = (keep >> v) & 1u;
      }
    }
    put_state(L.Sr, L.ST, sv, tid);
    if (BOOT) put_state(L.S2r, nullptr, s2v, tid);
    if (tid < 64) L.A[tid] = av;
    if (tid < 32) {
      if (BOOT) {
        L.RB[tid] = rv;
        L.DB[tid] = dv;
      } else {
        L.Y[tid] = rv;
      }
    }
    if (sub == 0) put_tails(L.TL, tla, tlb, BOOT ? 3 : 1, w, tid);
    lds_sync();
    SK_TP(2);
    // ---- phase 1: layer 1 (n-tile w) of the critic with Dropout, the target actor, the target critic
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch in phase 1 (hoisted into phase 0 it spills)
    bf16x8 wf[16];
    if (l2) load_l2(wf, cp, w, lane);
    else if (BOOT) load_l2(wf, ap, w - 4, lane);
    SK_TP(12);
    layer1<true>(L.Sr, f1c, TLc, w, lane, L.H1, L.H1T, keep);
    SK_TP(13);
    if (BOOT) {
      layer1<false>(L.S2r, f1a, TLa, w, lane, L.H1a, nullptr, 0);
      SK_TP(14);
      layer1<false>(L.S2r, f1t, TLt, w, lane, L.H1B, nullptr, 0);
    }
    SK_TP(15);
    lds_sync();
    SK_TP(3);
    // ---- phase 2
    if (l2) {  // critic h2 = relu(W2 [h1; a] + b2) -> fp32 LDS (dz2); q partial row sums
      const f32x16 acc = l2_mfma(L.H1, wf, lane);
      const float b2 = TLc[kTB2 + u], wa0 = TLc[kTW2a + 2 * u], wa1 = TLc[kTW2a + 2 * u + 1], w3 = TLc[kTW3 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        float a0[4], a1[4], qv[4];
        pairs4(L.A, i0, a0, a1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = fmaxf(acc[4 * g + q] + b2 + a0[q] * wa0 + a1[q] * wa1, 0.f);
          L.H2f[(i0 + q) * kLdH2f + u] = h;
          qv[q] = halfsum32(h * w3);
        }
        if (col == 31) put_rows4(L.QP + 32 * w, qv, i0);
      }
    } else if (BOOT) {  // target actor h2 -> mu' partial row sums; then the target critic's layer-2 fragments
      const f32x16 acc = l2_mfma(L.H1a, wf, lane);
      __builtin_amdgcn_sched_barrier(0);
      load_l2(wf, tp, w - 4, lane);
      const float b2 = TLa[kTB2 + u], w30 = TLa[kTW3 + u], w31 = TLa[kTW3 + kH2 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float m0[4], m1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = fmaxf(acc[4 * g + q] + b2, 0.f);
          m0[q] = halfsum32(h * w30);
          m1[q] = halfsum32(h * w31);
        }
        if (col == 31) put_rows4x2(L.MP + 64 * (w - 4), m0, m1, drow(4 * g, lane));
      }
    }
    lds_sync();
    SK_TP(4);
    // ---- phase 3
    bf16x8 wt[8];  // W2^T fragments of phase 5 (waves 4-7: after the target critic's fragments are consumed)
    if (l2 || !BOOT) load_w2t(wt, cp, w, lane);
    if (!l2 && BOOT) {  // mu'(s') per row from the partials, then Q' partial row sums of the wave's units
      const f32x16 acc = l2_mfma(L.H1B, wf, lane);
      __builtin_amdgcn_sched_barrier(0);
      load_w2t(wt, cp, w, lane);
      float* aw = L.AW + 64 * w;
      {  // lane (row col, output hh)
        float sm = TLa[kTB3 + hh];
#pragma unroll
        for (int v = 0; v < 4; ++v) sm += L.MP[64 * v + 2 * col + hh];
        aw[2 * col + hh] = tanhf(sm);
      }
      wave_lds_order();
      const float b2 = TLt[kTB2 + u], wa0 = TLt[kTW2a + 2 * u], wa1 = TLt[kTW2a + 2 * u + 1], w3 = TLt[kTW3 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        float a0[4], a1[4], yq[4];
        pairs4(aw, i0, a0, a1);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          yq[q] = halfsum32(fmaxf(acc[4 * g + q] + b2 + a0[q] * wa0 + a1[q] * wa1, 0.f) * w3);
        if (col == 31) put_rows4(L.YP + 32 * (w - 4), yq, i0);
      }
    }
    if (BOOT) lds_sync();
    SK_TP(5);
    // ---- phase 4 (waves 0-3): y and dL/dq for all rows (each wave), then dz2 = dL/dq W3 relu'(h2) of its units
    if (l2) {
      float q = TLc[kTB3], yq = TLt[kTB3];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        q += L.QP[32 * v + col];
        if (BOOT) yq += L.YP[32 * v + col];
      }
      const float yv = BOOT ? L.RB[col] + gamma * (1.f - L.DB[col]) * yq : L.Y[col];
      const float e = row0 + col < B ? q - yv : 0.f;
      float* dw = L.DW + 64 * w;
      if (hh == 0) dw[col] = grad_scale * e;
      if (w == 0 && hh == 0) {
        gb3 += grad_scale * e;
        lsum += e * e;
      }
      wave_lds_order();
      const float w3 = TLc[kTW3 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        const float4 dq4 = rows4(dw, i0);
        const float dqs[4] = {dq4.x, dq4.y, dq4.z, dq4.w};
        float a0[4], a1[4], d[4];
        pairs4(L.A, i0, a0, a1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = L.H2f[(i0 + q) * kLdH2f + u];
          d[q] = h > 0.f ? dqs[q] * w3 : 0.f;
          L.DZ2[(i0 + q) * kLdZ2 + u] = f2bf(d[q]);
          gb2 += d[q];
          gw2a0 += d[q] * a0[q];
          gw2a1 += d[q] * a1[q];
          gw3 += dqs[q] * h;
        }
        store_t4(L.DZ2T, kLdT, u, i0, d[0], d[1], d[2], d[3]);
      }
    }
    lds_sync();
    SK_TP(6);
    // ---- phases 5, 6
    {
      f32x16 gW2[4], gW1 = {0};
#pragma unroll
      for (int k = 0; k < 4; ++k) gW2[k] = f32x16{0};
      backward_12<true>(L, wt, w, lane, gW2, gW1, gb1);
      store_w12(P, w, lane, gW2, gW1, sub > 0);
    }
    lds_sync();  // the next sub-tile restages
    SK_TP(7);
  }
  const int lane = lane0, hh = lane >> 5;
  const int u = 32 * (w & 3) + (lane & 31);
  store_b1(P, w, lane, gb1);
  SK_TP(8);
  gb2 += __shfl_xor(gb2, 32, 64);
  gw2a0 += __shfl_xor(gw2a0, 32, 64);
  gw2a1 += __shfl_xor(gw2a1, 32, 64);
  gw3 += __shfl_xor(gw3, 32, 64);
  if (l2 && hh == 0) {
    P[kCPB2 + u] = gb2;
    P[skpart::critic_w2_action(u, 0)] = gw2a0;
    P[skpart::critic_w2_action(u, 1)] = gw2a1;
    P[kCPW3 + u] = gw3;
  }
  if (w == 0 && hh == 0) {  // wave 0's row lanes hold the db3 / loss partials
    atomicAdd(&L.RED[0], gb3);
    atomicAdd(&L.RED[1], lsum);
  }
  lds_sync();
  if (threadIdx.x == 0) {
    P[kCPB3] = L.RED[0];
    if (loss_out) atomicAdd(loss_out, L.RED[1]);
  }
  SK_TP(9);
}

// ---------------------------------------------------------------- actor step
// model_actor_fit_step (SkillshotLearner.py:386-417; DDPG.model_actor_fit_step):
// gradient of -loss_scale * sum_b Q(s_b, mu(s_b)) w.r.t. the actor, critic in
// inference mode (no Dropout).  q_out (optional) receives sum_b Q.  Phases:
//   0  stage s; layer-1 fragments in flight
//   1  layer 1 (n-tile w) of the actor and of the critic (both read s)
//   2  waves 0-3: actor layer 2 -> h2;  waves 4-7: the critic's layer-2 MFMA
//      (its action columns join in phase 3)
//   3  mu(s) (each wave, all rows); waves 4-7: critic z2 at (s, mu(s)),
//      dQ/dz2 = W3 relu'(z2), Q terms
//   4  waves 0-3: dL/dz3 = -loss_scale dQ/da (1 - a^2) (each wave, all rows),
//      dz2 of its units; wave 4: sum Q
//   5  dW2, dz1;  6  dW1
__global__ void __launch_bounds__(kThreads) k_actor_grad(const float* __restrict__ S, int64_t B, int sub_per_wg,
                                                         float loss_scale, const char* __restrict__ apack,
                                                         const char* __restrict__ cpack, float* __restrict__ partial,
                                                         float* step_ctr, int n_steps, float* __restrict__ q_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve(smem);
  SK_TP(0);
  const int lane0 = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool l2 = w < 4;  // waves of the actor's layer 2 (4-7: the critic's)
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  for (int t = threadIdx.x; t < 32 * kLdT; t += kThreads) L.ST[t] = 0;
  const float* TLa = L.TL;
  const float* TLc = L.TL + 1024;
  float* P = partial + (int64_t)blockIdx.x * kAP;
  // the actor kernel has the registers to keep its weight-gradient
  // accumulators across sub-tiles (the critic stores per sub-tile)
  f32x16 gW2[4], gW1 = {0};
#pragma unroll
  for (int k = 0; k < 4; ++k) gW2[k] = f32x16{0};
  float gb1 = 0.f, gb2 = 0.f, gw30 = 0.f, gw31 = 0.f, gb3 = 0.f, qsum = 0.f;
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  SK_TP(1);
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;  // uniform across the workgroup
    const int tid = launder_lane(threadIdx.x), lane = tid & 63, hh = lane >> 5, col = lane & 31;
    const int u = 32 * (w & 3) + col;  // the lane's layer-2 unit (actor: waves 0-3, critic: 4-7)
    const char* ap = apack;
    const char* cp = cpack;
    asm volatile("" : "+s"(ap), "+s"(cp));  // no LICM of the fragment loads (see k_critic_grad)
    const bf16x8 f1a = load_l1(ap, w, lane), f1c = load_l1(cp, w, lane);
    // ---- phase 0: states (and, first sub-tile, the tails) loaded together, then LDS
    const float sv = load_state(S, row0, B, tid);
    f4v tla = {}, tlb = {};
    if (sub == 0) load_tails(tla, tlb, ap, cp, nullptr, 2, w, tid);
    put_state(L.Sr, L.ST, sv, tid);
    if (sub == 0) put_tails(L.TL, tla, tlb, 2, w, tid);
    lds_sync();
    SK_TP(2);
    // ---- phase 1: layer 1 (n-tile w) of the actor and of the critic
    bf16x8 wf[16];
    if (l2) load_l2(wf, ap, w, lane);
    else load_l2(wf, cp, w - 4, lane);
    layer1<false>(L.Sr, f1a, TLa, w, lane, L.H1, L.H1T, 0);
    layer1<false>(L.Sr, f1c, TLc, w, lane, L.H1B, nullptr, 0);
    lds_sync();
    SK_TP(3);
    // ---- phase 2
    f32x16 zc = {0};
    if (l2) {  // actor h2 -> fp32 LDS (dz2); mu partial row sums
      const f32x16 acc = l2_mfma(L.H1, wf, lane);
      const float b2 = TLa[kTB2 + u], w30 = TLa[kTW3 + u], w31 = TLa[kTW3 + kH2 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        float m0[4], m1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = fmaxf(acc[4 * g + q] + b2, 0.f);
          L.H2f[(i0 + q) * kLdH2f + u] = h;
          m0[q] = halfsum32(h * w30);
          m1[q] = halfsum32(h * w31);
        }
        if (col == 31) put_rows4x2(L.MP + 64 * w, m0, m1, i0);
      }
    } else {
      zc = l2_mfma(L.H1B, wf, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 wt[8];  // W2^T fragments of phase 5
    load_w2t(wt, ap, w, lane);
    lds_sync();
    SK_TP(4);
    // ---- phase 3: mu(s) = tanh(W3 h2 + b3) from the partials, lane (row col, output hh), every wave
    float a;
    {
      float sm = TLa[kTB3 + hh];
#pragma unroll
      for (int v = 0; v < 4; ++v) sm += L.MP[64 * v + 2 * col + hh];
      a = tanhf(sm);
    }
    if (!l2) {  // the critic at (s, mu(s)): partial row sums of dQ/da = W3 relu'(z2) W2a (rows beyond B: 0) and Q
      float* aw = L.AW + 64 * w;
      aw[2 * col + hh] = a;
      wave_lds_order();
      const float b2 = TLc[kTB2 + u], wa0 = TLc[kTW2a + 2 * u], wa1 = TLc[kTW2a + 2 * u + 1], w3 = TLc[kTW3 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        float a0[4], a1[4], d0[4], d1[4], qz[4];
        pairs4(aw, i0, a0, a1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float z = zc[4 * g + q] + b2 + a0[q] * wa0 + a1[q] * wa1;
          const float dqdz = (z > 0.f && row0 + i0 + q < B) ? w3 : 0.f;
          d0[q] = halfsum32(dqdz * wa0);
          d1[q] = halfsum32(dqdz * wa1);
          qz[q] = q_out ? halfsum32(fmaxf(z, 0.f) * w3) : 0.f;
        }
        if (col == 31) {
          put_rows4x2(L.DP + 64 * (w - 4), d0, d1, i0);
          if (q_out) put_rows4(L.QP + 32 * (w - 4), qz, i0);
        }
      }
    }
    lds_sync();
    SK_TP(5);
    // ---- phase 4
    if (l2) {  // dL/dz3[row col][hh], then dz2 = (dz3 W3) relu'(h2) of its units
      float da = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) da += L.DP[64 * v + 2 * col + hh];
      const float dz3 = -loss_scale * da * (1.f - a * a);
      float* dw = L.DW + 64 * w;
      dw[2 * col + hh] = dz3;
      if (w == 0) {
        gb3 += dz3;  // db3[hh] partial of row col
        if (q_out && hh == 0 && row0 + col < B) {
          float sq = TLc[kTB3];
#pragma unroll
          for (int v = 0; v < 4; ++v) sq += L.QP[32 * v + col];
          qsum += sq;
        }
      }
      wave_lds_order();
      const float w30 = TLa[kTW3 + u], w31 = TLa[kTW3 + kH2 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i0 = drow(4 * g, lane);
        float z0[4], z1[4], d[4];
        pairs4(dw, i0, z0, z1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float h = L.H2f[(i0 + q) * kLdH2f + u];
          d[q] = h > 0.f ? z0[q] * w30 + z1[q] * w31 : 0.f;
          L.DZ2[(i0 + q) * kLdZ2 + u] = f2bf(d[q]);
          gb2 += d[q];
          gw30 += z0[q] * h;
          gw31 += z1[q] * h;
        }
        store_t4(L.DZ2T, kLdT, u, i0, d[0], d[1], d[2], d[3]);
      }
    }
    lds_sync();
    SK_TP(6);
    // ---- phases 5, 6
    backward_12<false>(L, wt, w, lane, gW2, gW1, gb1);
    lds_sync();
    SK_TP(7);
  }
  const int lane = lane0, hh = lane >> 5;
  const int u = 32 * (w & 3) + (lane & 31);
  store_w12(P, w, lane, gW2, gW1, false);
  store_b1(P, w, lane, gb1);
  SK_TP(8);
  gb2 += __shfl_xor(gb2, 32, 64);
  gw30 += __shfl_xor(gw30, 32, 64);
  gw31 += __shfl_xor(gw31, 32, 64);
  if (l2 && hh == 0) {
    P[kAPB2 + u] = gb2;
    P[kAPW3 + u] = gw30;
    P[kAPW3 + kH2 + u] = gw31;
  }
  if (w == 0) atomicAdd(&L.RED[hh], gb3);  // db3[hh]: wave 0, lane (row, hh)
  if (w == 0 && hh == 0 && q_out) atomicAdd(&L.RED[2], qsum);
  lds_sync();
  if (threadIdx.x < 2) P[kAPB3 + threadIdx.x] = L.RED[threadIdx.x];
  if (threadIdx.x == 0 && q_out) atomicAdd(q_out, L.RED[2]);
  SK_TP(9);
}

// ---------------------------------------------------------------- Adam
// g = sum of the G partials (+ written to grad_out, if given, e.g. for an
// RCCL all-reduce between this kernel with apply=0 and a second with G=0).
// Keras Adam (tf.keras.optimizers.Adam of SkillshotLearner.py:68, :118;
// learner.KerasAdam): m += (g - m)(1-b1), v += (g^2 - v)(1-b2),
// p -= m alpha / (sqrt(v) + eps) with alpha = lr sqrt(1-b2^t) / (1-b1^t),
// t = the step counter (advanced by the grad kernel).  Then target += tau
// (p - target) (torch._foreach_lerp_, DDPG.soft_update) when a target is
// given.
// Housekeeping of the step, by thread 0 when applying (after the gradient
// kernel consumed them, before the next one): stat_out = stat_acc * scale and
// stat_acc = 0 (the loss accumulator of the gradient kernel), ++*counter (its
// dropout call number) — one launch fewer each than torch ops would cost.
// ---------------------------------------------------------------- packs from Adam
// Every packed entry is a function of one parameter, so the Adam launch that
// produces a parameter also writes its packed copies (replacing the separate
// k_grad_pack / k_grad_pack_flat / k_actor_pack launches of a step):
// scatter_grad_pack is the inverse of grad_pack_body's index map, and
// scatter_fwd_pack of k_actor_pack's (sk_actor.hip).  Padding entries (W1 k
// >= 12, unused tail slots) are never written: they keep the zeros of the
// initial full pack.
struct PackOut {
  char* gp;   // grad pack of the stepped net (nullable)
  char* tp;   // grad pack of its soft-updated target (nullable)
  char* fp;   // actor forward pack (sk_actor_pack layout; nullable, actor only)
  int ld2, n_out;
  char* sp;   // the fp32 actor's split pack (sk_split.hpp; nullable, actor only)
};

__device__ __forceinline__ void scatter_grad_pack(char* out, int p, float v, int ld2, int n_out) {
  float* tail = (float*)(out + kGTail);
  if (p < kPB1) {  // W1[n][k]
    const int n = p / kIn, k = p - n * kIn;
    const int lane = (n & 31) + 32 * (k >> 3);
    ((short*)(out + kGW1))[((n >> 5) * 64 + lane) * 8 + (k & 7)] = f2bf(v);
    return;
  }
  if (p < kPW2) {
    tail[kTB1 + p - kPB1] = v;
    return;
  }
  const int q = p - kPW2;
  if (q < kH2 * ld2) {  // W2[o][i]
    const int o = q / ld2, i = q - o * ld2;
    if (i < kH1) {
      const short b = f2bf(v);
      const int l2 = (o & 31) + 32 * ((i >> 3) & 1);
      ((short*)(out + kGW2))[(((o >> 5) * 16 + (i >> 4)) * 64 + l2) * 8 + (i & 7)] = b;
      const int lt = (i & 31) + 32 * ((o >> 3) & 1);
      ((short*)(out + kGW2T))[(((i >> 5) * 8 + (o >> 4)) * 64 + lt) * 8 + (o & 7)] = b;
    } else {
      tail[kTW2a + 2 * o + (i - kH1)] = v;
    }
    return;
  }
  const int r = q - kH2 * ld2;
  if (r < kH2) tail[kTB2 + r] = v;
  else if (r < kH2 + n_out * kH2) tail[kTW3 + r - kH2] = v;
  else tail[kTB3 + r - kH2 - n_out * kH2] = v;
}

__device__ __forceinline__ void scatter_fwd_pack(char* out, int p, float v) {  // actor: ld2 = 256, n_out = 2
  float* bias = (float*)(out + kOffB);
  if (p < kPB1) {
    const int n = p / kIn, k = p - n * kIn;
    const int idx = ((n >> 5) * 64 + (n & 31) + 32 * (k >> 3)) * 8 + (k & 7);
    ((short*)(out + kOffW1))[idx] = f2bf(v);
    ((short*)(out + kOffW1s))[idx] = f2bf(v * v);
    return;
  }
  if (p < kPW2) {
    bias[p - kPB1] = v;
    return;
  }
  const int q = p - kPW2;
  if (q < kH2 * kH1) {
    const int o = q / kH1, i = q - o * kH1;
    const int kk = 2 * (i >> 5) + ((i >> 4) & 1), j = 4 * ((i >> 3) & 1) + (i & 3);
    const int lane = (o & 31) + 32 * ((i >> 2) & 1);
    const int idx = (((o >> 5) * 16 + kk) * 64 + lane) * 8 + j;
    ((short*)(out + kOffW2))[idx] = f2bf(v);
    ((short*)(out + kOffW2s))[idx] = f2bf(v * v);
    return;
  }
  const int r = q - kH2 * kH1;
  if (r < kH2) {
    bias[kH1 + r] = v;
  } else if (r < kH2 + kOut * kH2) {
    float* w3f = (float*)(out + kOffW3f);
    w3f[r - kH2] = v;
    w3f[256 + r - kH2] = v * v;
  } else {
    bias[kH1 + kH2 + r - kH2 - kOut * kH2] = v;
  }
}

#ifndef SK_ADAM_SLICES
#define SK_ADAM_SLICES 4
#endif
#ifndef SK_ADAM_PARAMS
#define SK_ADAM_PARAMS 64
#endif
#ifndef SK_ADAM_INFLIGHT
#define SK_ADAM_INFLIGHT 8
#endif
constexpr int kAdamParams = SK_ADAM_PARAMS, kAdamSlices = SK_ADAM_SLICES, kAdamInflight = SK_ADAM_INFLIGHT;
// partials per lane loaded in one round (k_adam_flat): 32 = the sliced fp32
// kernels' W1 / b1 contributions at batch 256 (128 rows over 4 slices)
constexpr int kAdamOnce = 32 + kAdamInflight;
static_assert(kAdamParams == 64, "one wave per slice: the partial count is wave-uniform");
static_assert(kAdamInflight >= 2 && (kAdamInflight & (kAdamInflight - 1)) == 0, "a power of two");
static_assert(skpart::kPW2 % kAdamParams == 0, "the W1 rows stay workgroup-uniform");

__global__ void __launch_bounds__(kAdamParams * kAdamSlices) k_adam_flat(const float* __restrict__ partial, int G, int P, const float* __restrict__ grad_in,
                            float* __restrict__ grad_out, int apply, float* __restrict__ param, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ step_ctr, float lr, float beta1,
                            float beta2, float eps, float* __restrict__ target, float tau, float* stat_acc,
                            float stat_scale, float* stat_out, int64_t* counter, PackOut po,
                            const float* __restrict__ partial_w1, int G1) {
  // a workgroup owns kAdamParams consecutive parameters; its kAdamSlices
  // waves each sum every kAdamSlices-th partial of them (64-lane coalesced
  // rows, 8 loads in flight per lane), then fold through LDS: 4x the waves
  // of one-thread-per-parameter, for the latency of the partial reads
  __shared__ float red[kAdamSlices - 1][kAdamParams];
  const int lane = threadIdx.x % kAdamParams, slice = threadIdx.x / kAdamParams;
  const int p = blockIdx.x * kAdamParams + lane;
  if (apply && p == 0 && slice == 0) {
    if (stat_acc) {
      if (stat_out) *stat_out = *stat_acc * stat_scale;
      *stat_acc = 0.f;
    }
    if (counter) *counter += 1;
  }
  const bool in = p < P;
  int pp = skpart::index(p, P);  // the partial layout (sk_partial.hpp)
  // W1 / b1 of the sliced fp32 kernels (sk_learn32.hip): G1 contribution
  // rows of kPW2 floats (workgroup-uniform: kPW2 is a multiple of kAdamParams)
  const bool w1 = partial_w1 && p < skpart::kPW2;
  const float* src = w1 ? partial_w1 : partial;
  const int64_t ld = w1 ? skpart::kPW2 : P;
  const int GG = w1 ? G1 : G;
  // the step's own operands are loaded up front, under the partial reads
  float g0 = 0.f, mm = 0.f, vv = 0.f, w0 = 0.f, tw0 = 0.f, t = 0.f;
  if (in && slice == 0) {
    if (grad_in) g0 = grad_in[p];
    if (apply) {
      t = step_ctr[0];
      mm = m[p];
      vv = v[p];
      w0 = param[p];
      if (target) tw0 = target[p];
    }
  }
  // kAdamInflight independent loads in flight per lane: the sliced fp32
  // kernels' W1 / b1 gradient is 128 contribution rows at batch 256 (32 per
  // slice), so 8 in flight made those workgroups wait four load latencies
  float acc[kAdamInflight];
#pragma unroll
  for (int j = 0; j < kAdamInflight; ++j) acc[j] = 0.f;
  // this lane's partials are k = slice + i * kAdamSlices, i < cnt (wave-uniform)
  const int cnt = in && GG > slice ? (GG - slice + kAdamSlices - 1) / kAdamSlices : 0;
  float alpha = 0.f;
  if (cnt <= kAdamOnce) {
    // every partial in flight at once (one load latency; the loop below
    // waited for each group of kAdamInflight and the tail one load at a
    // time: at batch 256 every W2 lane's 4 partials were 4 dependent round
    // trips, every W1 lane's 32 were 4), summed in the loop's order:
    // group g (i = 8g .. 8g + 7, while 8g + 7 < cnt) into acc[i % 8], the
    // tail (i >= 8 * groups) into acc[0], each in increasing i.  Same sums.
    float x[kAdamOnce];
#pragma unroll
    for (int g = 0; g < kAdamOnce / kAdamInflight; ++g) {
      if (kAdamInflight * g < cnt) {  // wave-uniform (one wave per slice): only the groups in use
#pragma unroll
        for (int j = 0; j < kAdamInflight; ++j) {
          const int i = kAdamInflight * g + j;
          x[i] = src[(int64_t)(i < cnt ? slice + i * kAdamSlices : slice) * ld + pp];  // unconditional within the group
        }
      } else {
#pragma unroll
        for (int j = 0; j < kAdamInflight; ++j) x[kAdamInflight * g + j] = 0.f;
      }
    }
    // Adam's step size under the loads (it needs only the step count)
    if (apply && in && slice == 0) {
      alpha = lr * sqrtf(1.f - powf(beta2, t)) / (1.f - powf(beta1, t));
      asm volatile("" : "+v"(alpha));
    }
    __builtin_amdgcn_sched_barrier(0);
    const int full = (cnt / kAdamInflight) * kAdamInflight;
#pragma unroll
    for (int i = 0; i < kAdamOnce; ++i) {
      const int j = i % kAdamInflight;
      acc[j] = i < full ? acc[j] + x[i] : acc[j];
    }
#pragma unroll
    for (int i = 0; i < kAdamOnce; ++i) acc[0] = (i >= full && i < cnt) ? acc[0] + x[i] : acc[0];
  } else if (in) {
    int k = slice;
    for (; k + (kAdamInflight - 1) * kAdamSlices < GG; k += kAdamInflight * kAdamSlices) {
#pragma unroll
      for (int j = 0; j < kAdamInflight; ++j) acc[j] += src[(int64_t)(k + j * kAdamSlices) * ld + pp];
    }
    for (; k < GG; k += kAdamSlices) acc[0] += src[(int64_t)k * ld + pp];
  }
  // adjacent pairs first, ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7)):
  // the round-3 summation order, so Adam results stay bit-identical to it
  // (round 4's halving tree summed (a0 + a4) + ... first)
#pragma unroll
  for (int s = 1; s < kAdamInflight; s *= 2)
#pragma unroll
    for (int j = 0; j + s < kAdamInflight; j += 2 * s) acc[j] += acc[j + s];
  const float part = acc[0];
  if (slice > 0) red[slice - 1][lane] = part;
  __syncthreads();
  if (slice > 0 || !in) return;
  float g = g0;
  g += part;
#pragma unroll
  for (int j = 0; j < kAdamSlices - 1; ++j) g += red[j][lane];
  if (grad_out) grad_out[p] = g;
  if (!apply) return;
  if (cnt > kAdamOnce) alpha = lr * sqrtf(1.f - powf(beta2, t)) / (1.f - powf(beta1, t));
  mm = mm + (g - mm) * (1.f - beta1);
  vv = vv + (g * g - vv) * (1.f - beta2);
  m[p] = mm;
  v[p] = vv;
  const float w = w0 - (mm * alpha) / (sqrtf(vv) + eps);
  param[p] = w;
  if (po.gp) scatter_grad_pack(po.gp, p, w, po.ld2, po.n_out);
  if (po.fp) scatter_fwd_pack(po.fp, p, w);
  if (po.sp) sksplit::scatter_split_pack(po.sp, p, w);
  if (target) {
    const float tw = tw0 + tau * (w - tw0);
    target[p] = tw;
    if (po.tp) scatter_grad_pack(po.tp, p, tw, po.ld2, po.n_out);
  }
}

int64_t subtiles_per_wg(int64_t B) {  // <= 128 workgroups, >= 1 sub-tile each
  const int64_t tiles = (B + 31) / 32;
  return (tiles + 127) / 128;
}

template <typename K>
void set_lds(K kernel, size_t bytes) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" {

size_t sk_grad_packed_bytes(void) { return kGPackBytes; }

int sk_grad_pack_flat(const float* const* flats, const int32_t* ld2s, const int32_t* n_outs, void* const* outs,
                      int32_t n_nets, void* stream) {
  if (!flats || !ld2s || !n_outs || !outs || n_nets < 1 || n_nets > 4) return SK_EINVAL;
  PackJobs j = {};
  for (int k = 0; k < n_nets; ++k) {
    if (!flats[k] || !outs[k] || (((uintptr_t)outs[k]) & 15)) return SK_EINVAL;
    if ((ld2s[k] != kH1 && ld2s[k] != kH1 + 2) || (n_outs[k] != 1 && n_outs[k] != 2)) return SK_EINVAL;
    j.flat[k] = flats[k];
    j.out[k] = (char*)outs[k];
    j.ld2[k] = ld2s[k];
    j.n_out[k] = n_outs[k];
  }
  k_grad_pack_flat<<<dim3((kPackThreads + 255) / 256, n_nets), 256, 0, (hipStream_t)stream>>>(j);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int64_t sk_update_partials(int64_t batch) {
  if (batch <= 0) return 0;
  const int64_t spw = subtiles_per_wg(batch);
  return ((batch + 31) / 32 + spw - 1) / spw;
}

int sk_grad_pack(const float* W1, const float* b1, const float* W2, int32_t ld2, const float* b2, const float* W3,
                 const float* b3, int32_t n_out, void* packed, void* stream) {
  if (!W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !packed) return SK_EINVAL;
  if ((ld2 != kH1 && ld2 != kH1 + 2) || (n_out != 1 && n_out != 2) || (((uintptr_t)packed) & 15)) return SK_EINVAL;
  k_grad_pack<<<(kPackThreads + 255) / 256, 256, 0, (hipStream_t)stream>>>(W1, b1, W2, ld2, b2, W3, b3, n_out,
                                                                          (char*)packed);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_critic_grad(const void* cpack, const float* obs, const float* actions, const float* targets, int64_t batch,
                   int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter, float* partial,
                   float* step_counters, int32_t n_steps, float* loss_sum, uint8_t* dropout_mask, void* stream) {
  return sk_critic_grad_bootstrap(cpack, obs, actions, targets, nullptr, nullptr, nullptr, 0.f, nullptr, nullptr,
                                  batch, row_offset, grad_scale, seed, call_counter, partial, step_counters, n_steps,
                                  loss_sum, dropout_mask, stream);
}

int sk_critic_grad_bootstrap(const void* cpack, const float* obs, const float* actions, const float* targets,
                             const float* next_obs, const float* rewards, const float* done, float gamma,
                             const void* target_actor_gpack, const void* target_critic_gpack, int64_t batch,
                             int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                             float* partial, float* step_counters, int32_t n_steps, float* loss_sum,
                             uint8_t* dropout_mask, void* stream) {
  const bool boot = target_actor_gpack != nullptr;
  if (row_offset < 0 || (row_offset & 3)) return SK_EINVAL;
  if (boot && (!target_critic_gpack || !next_obs || !rewards || !done)) return SK_EINVAL;
  if (!boot && !targets) return SK_EINVAL;
  if (boot && ((((uintptr_t)target_actor_gpack) & 15) || (((uintptr_t)target_critic_gpack) & 15))) return SK_EINVAL;
  if (!cpack || !obs || !actions || !call_counter || !partial || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  if ((((uintptr_t)cpack) & 15) || (((uintptr_t)obs) & 3) || (((uintptr_t)actions) & 3)) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds(k_critic_grad<true>, kLdsGrad);
    set_lds(k_critic_grad<false>, kLdsGrad);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg(batch);
  const unsigned G = (unsigned)sk_update_partials(batch);
  auto kern = boot ? k_critic_grad<true> : k_critic_grad<false>;
  kern<<<G, kThreads, kLdsGrad, (hipStream_t)stream>>>(
      obs, actions, targets, batch, row_offset, (int)spw, grad_scale, seed, call_counter, (const char*)cpack, partial,
      step_counters, n_steps, loss_sum, dropout_mask, next_obs, rewards, done, gamma,
      (const char*)target_actor_gpack, (const char*)target_critic_gpack, skmlp::RingSample{});
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_critic_grad_bootstrap_sampled(const void* cpack, const sk_ring_sample* q, float gamma,
                                     const void* target_actor_gpack, const void* target_critic_gpack, int64_t batch,
                                     int64_t row_offset, float grad_scale, uint64_t seed,
                                     const int64_t* call_counter, float* partial, float* step_counters,
                                     int32_t n_steps, float* loss_sum, uint8_t* dropout_mask, void* stream) {
  if (!q || !q->ring || !q->total || !q->s || !q->a || !q->r || !q->s2 || !q->d || q->capacity <= 0) return SK_EINVAL;
  if (q->exclude < 0 || q->exclude >= q->capacity) return SK_EINVAL;  // as sk_replay_sample_excl
  if ((((uintptr_t)q->ring) & 15) || (((uintptr_t)q->s) & 15) || (((uintptr_t)q->s2) & 15) || (((uintptr_t)q->a) & 7))
    return SK_EINVAL;
  const bool boot = target_actor_gpack != nullptr;
  if (row_offset < 0 || (row_offset & 3)) return SK_EINVAL;
  if (boot && !target_critic_gpack) return SK_EINVAL;
  if (boot && ((((uintptr_t)target_actor_gpack) & 15) || (((uintptr_t)target_critic_gpack) & 15))) return SK_EINVAL;
  if (!cpack || !call_counter || !partial || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  if (((uintptr_t)cpack) & 15) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds(k_critic_grad<true>, kLdsGrad);
    set_lds(k_critic_grad<false>, kLdsGrad);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg(batch);
  const unsigned G = (unsigned)sk_update_partials(batch);
  const skmlp::RingSample rs{q->ring, q->capacity, q->total, q->seed, q->draw, q->s, q->a, q->r, q->s2, q->d, q->exclude};
  auto kern = boot ? k_critic_grad<true> : k_critic_grad<false>;
  kern<<<G, kThreads, kLdsGrad, (hipStream_t)stream>>>(
      q->s, q->a, q->r, batch, row_offset, (int)spw, grad_scale, seed, call_counter, (const char*)cpack, partial,
      step_counters, n_steps, loss_sum, dropout_mask, q->s2, q->r, q->d, gamma, (const char*)target_actor_gpack,
      (const char*)target_critic_gpack, rs);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_grad(const void* apack, const void* cpack, const float* obs, int64_t batch, float loss_scale,
                  float* partial, float* step_counters, int32_t n_steps, float* q_sum, void* stream) {
  if (!apack || !cpack || !obs || !partial || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  if ((((uintptr_t)apack) & 15) || (((uintptr_t)cpack) & 15) || (((uintptr_t)obs) & 3)) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds(k_actor_grad, kLdsGrad);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg(batch);
  const unsigned G = (unsigned)sk_update_partials(batch);
  k_actor_grad<<<G, kThreads, kLdsGrad, (hipStream_t)stream>>>(obs, batch, (int)spw, loss_scale, (const char*)apack,
                                                                (const char*)cpack, partial, step_counters, n_steps,
                                                                q_sum);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_adam_flat_sliced(const float* partial, int32_t n_partials, const float* partials_w1, int32_t n_w1,
                        int32_t n_params, const float* grad_in, float* grad_out, int32_t apply, float* param,
                        float* exp_avg, float* exp_avg_sq, const float* step_counter, float lr, float beta1,
                        float beta2, float eps, float* target, float tau, float* stat_acc, float stat_scale,
                        float* stat_out, int64_t* counter, const sk_pack_targets* packs, void* stream) {
  if (n_params <= 0 || n_partials < 0 || (n_partials > 0 && !partial)) return SK_EINVAL;
  if (n_w1 < 0 || (n_w1 > 0 && !partials_w1) || (partials_w1 && n_params < skpart::kPW2)) return SK_EINVAL;
  if (apply && (!param || !exp_avg || !exp_avg_sq || !step_counter)) return SK_EINVAL;
  PackOut po = {nullptr, nullptr, nullptr, kH1, 1, nullptr};
  if (packs && apply) {
    const int ld2 = packs->ld2, n_out = packs->n_out;
    if ((ld2 != kH1 && ld2 != kH1 + 2) || (n_out != 1 && n_out != 2)) return SK_EINVAL;
    if (n_params != kPW2 + kH2 * ld2 + kH2 + n_out * kH2 + n_out) return SK_EINVAL;
    if ((packs->actor_fwd_pack || packs->actor_split_pack) && (ld2 != kH1 || n_out != kOut)) return SK_EINVAL;
    if (packs->target_gpack && !target) return SK_EINVAL;
    for (const void* b : {packs->param_gpack, packs->target_gpack, packs->actor_fwd_pack, packs->actor_split_pack})
      if (((uintptr_t)b) & 15) return SK_EINVAL;
    po = {(char*)packs->param_gpack, (char*)packs->target_gpack, (char*)packs->actor_fwd_pack, ld2, n_out,
          (char*)packs->actor_split_pack};
  }
  k_adam_flat<<<(n_params + kAdamParams - 1) / kAdamParams, kAdamParams * kAdamSlices, 0, (hipStream_t)stream>>>(
      partial, n_partials, n_params, grad_in, grad_out, apply, param, exp_avg, exp_avg_sq, step_counter, lr, beta1,
      beta2, eps, target, tau, stat_acc, stat_scale, stat_out, counter, po, partials_w1, n_w1);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_adam_flat_packed(const float* partial, int32_t n_partials, int32_t n_params, const float* grad_in,
                        float* grad_out, int32_t apply, float* param, float* exp_avg, float* exp_avg_sq,
                        const float* step_counter, float lr, float beta1, float beta2, float eps, float* target,
                        float tau, float* stat_acc, float stat_scale, float* stat_out, int64_t* counter,
                        const sk_pack_targets* packs, void* stream) {
  return sk_adam_flat_sliced(partial, n_partials, nullptr, 0, n_params, grad_in, grad_out, apply, param, exp_avg,
                             exp_avg_sq, step_counter, lr, beta1, beta2, eps, target, tau, stat_acc, stat_scale,
                             stat_out, counter, packs, stream);
}

int sk_adam_flat(const float* partial, int32_t n_partials, int32_t n_params, const float* grad_in, float* grad_out,
                 int32_t apply, float* param, float* exp_avg, float* exp_avg_sq, const float* step_counter, float lr,
                 float beta1, float beta2, float eps, float* target, float tau, float* stat_acc, float stat_scale,
                 float* stat_out, int64_t* counter, void* stream) {
  return sk_adam_flat_packed(partial, n_partials, n_params, grad_in, grad_out, apply, param, exp_avg, exp_avg_sq,
                             step_counter, lr, beta1, beta2, eps, target, tau, stat_acc, stat_scale, stat_out, counter,
                             nullptr, stream);
}

}  // extern "C"

#ifdef SK_TRACE
// diagnostic builds only (not in include/skillshot.h): [2 wg][32 points][memtime, realtime]
extern "C" int sk_debug_update_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk_trace), sizeof(g_sk_trace)) == hipSuccess ? SK_OK : SK_EHIP;
}
#endif
