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
// A workgroup (8 waves) owns a contiguous range of 32-row sub-tiles and
// keeps its weight-gradient accumulators in registers across them: wave w
// holds dW2 rows 32(w%4).. x columns 128(w/4).. (4 MFMA tiles) and dW1 rows
// 32w..32w+31 (1 tile); layer 1 / dH1 use one 32-unit tile per wave, layer
// 2 (128 units) waves 0-3.  Operands are bf16, accumulation fp32; biases, the critic's action
// columns, layer 3 and the losses are fp32 VALU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"

namespace {

using namespace skmlp;

constexpr int kThreads = 512;  // 8 waves

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
static_assert(kCP == 36609 && kAP == 36482, "parameter counts");

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

// sum over the 128 layer-2 units of X[i][k] * w[k * ws] for the row
// i = threadIdx.x / 16 of this thread (all 512 threads: 32 rows x 16
// 8-unit chunks, then a 4-step butterfly inside each 16-lane group; every
// lane of the group returns the row sum)
__device__ __forceinline__ float row_dot128(const float* X, int ld, const float* w, int ws) {
  const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += X[i * ld + 8 * c + k] * w[(8 * c + k) * ws];
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
  return s;
}
__device__ __forceinline__ float row_sum128(const float* X, int ld) {
  const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += X[i * ld + 8 * c + k];
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, 64);
  return s;
}

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
struct Lds {
  short *Sr, *ST, *H1, *H1T, *DZ2, *DZ2T, *DZ1T, *H1C, *S2r;
  float *H2f, *DZC, *A, *Y, *DQ, *DZ3, *RED, *A2, *RB, *DB;
};

__device__ __forceinline__ Lds carve(char* smem, bool actor) {
  Lds L;
  char* p = smem;
  L.Sr = (short*)p;   p += 32 * kLdS * 2;
  L.ST = (short*)p;   p += 32 * kLdT * 2;
  L.H1 = (short*)p;   p += 32 * kLdH1 * 2;
  L.H1T = (short*)p;  p += kH1 * kLdT * 2;
  L.DZ2 = (short*)p;  p += 32 * kLdZ2 * 2;
  L.DZ2T = (short*)p; p += kH2 * kLdT * 2;
  L.DZ1T = (short*)p; p += kH1 * kLdT * 2;
  L.H2f = (float*)p;  p += 32 * kLdH2f * 4;
  L.A = (float*)p;    p += 64 * 4;
  L.Y = (float*)p;    p += 32 * 4;
  L.DQ = (float*)p;   p += 32 * 4;
  L.DZ3 = (float*)p;  p += 64 * 4;
  L.RED = (float*)p;  p += 4 * 4;
  L.S2r = (short*)p;  p += 32 * kLdS * 2;  // bootstrap target: s', mu'(s'), r, done
  L.A2 = (float*)p;   p += 64 * 4;
  L.RB = (float*)p;   p += 32 * 4;
  L.DB = (float*)p;   p += 32 * 4;
  L.H1C = nullptr;
  L.DZC = nullptr;
  if (actor) {
    L.H1C = (short*)p; p += 32 * kLdH1 * 2;
    L.DZC = (float*)p; p += 32 * kLdH2f * 4;
  }
  return L;
}
constexpr size_t kLdsBase = 32 * kLdS * 2 + 32 * kLdT * 2 + 32 * kLdH1 * 2 + kH1 * kLdT * 2 + 32 * kLdZ2 * 2 +
                            kH2 * kLdT * 2 + kH1 * kLdT * 2 + 32 * kLdH2f * 4 + (64 + 32 + 32 + 64 + 4) * 4 +
                            32 * kLdS * 2 + (64 + 32 + 32) * 4;
constexpr size_t kLdsCritic = kLdsBase;
constexpr size_t kLdsActor = kLdsBase + 32 * kLdH1 * 2 + 32 * kLdH2f * 4;

// this sub-tile's states into Sr (batch-major) and ST (transposed, inputs
// padded to 32 rows; rows 12..31 stay zero from the kernel start)
__device__ __forceinline__ void load_states(const Lds& L, const float* S, int64_t row0, int64_t B) {
  for (int t = threadIdx.x; t < 32 * 16; t += kThreads) {
    const int i = t >> 4, k = t & 15;
    const float v = (k < kIn && row0 + i < B) ? S[(row0 + i) * kIn + k] : 0.f;
    const short b = f2bf(v);
    L.Sr[i * kLdS + k] = b;
    if (k < kIn) L.ST[k * kLdT + i] = b;
  }
}

// layer 1 of one net for n-tile nt: relu(S W1^T + b1) -> batch-major (and,
// if HT, transposed) bf16; `drop` applies the critic's training Dropout
template <bool DROP>
__device__ __forceinline__ void layer1(const short* Sx, const bf16x8* gW1, const float* tail, int nt, int lane,
                                       short* H, short* HT, uint64_t seed, uint64_t call, int64_t row0,
                                       uint8_t* mask_out, int64_t B, int64_t key_row0 = 0) {
  f32x16 acc = {0};
  acc = mfma(lfrag(Sx, kLdS, 0, 0, lane), gW1[nt * 64 + lane], acc);
  const int n = 32 * nt + (lane & 31);
  const float b = tail[kTB1 + n];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float hv[4];
    uint4 u = make_uint4(0, 0, 0, 0);
    const int i0 = drow(4 * g, lane);
    // the mask of GLOBAL batch row key_row0 + row0 + i (the 1-rank batch's
    // row numbering; key_row0 is a multiple of 4): learner.DDPG, rng.dropout_keep
    if (DROP) u = philox(make_uint4((uint32_t)((key_row0 + row0 + i0) >> 2), (uint32_t)n, (uint32_t)call,
                                    (uint32_t)(call >> 32)),
                         (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float z = fmaxf(acc[4 * g + q] + b, 0.f);
      if (DROP) {
        const bool keep = uw[q] >= 858993460u;  // P(drop) = 0.2 (Dropout(0.2), SkillshotLearner.py:110)
        z = keep ? z * 1.25f : 0.f;
        if (mask_out && row0 + i0 + q < B) mask_out[(row0 + i0 + q) * kH1 + n] = keep;
      }
      hv[q] = z;
      H[(i0 + q) * kLdH1 + n] = f2bf(z);
    }
    if (HT) store_t4(HT, kLdT, n, i0, hv[0], hv[1], hv[2], hv[3]);
  }
}

// layer 2 MFMA of one net for out n-tile nt over the 256 hidden inputs
// (all 16 weight fragments issued up front: one memory round trip)
__device__ __forceinline__ f32x16 layer2(const short* H, const bf16x8* gW2, int nt, int lane) {
  bf16x8 wf[16];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) wf[kk] = gW2[(nt * 16 + kk) * 64 + lane];
  f32x16 acc = {0};
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) acc = mfma(lfrag(H, kLdH1, 0, 16 * kk, lane), wf[kk], acc);
  return acc;
}

// the backward GEMMs shared by both kernels, given dZ2 (batch-major and
// transposed) in LDS:
//   dW2 tiles (w%4, 4(w/4)..+3) += dZ2^T H1     (accumulators gW2[4])
//   dZ1 = (dZ2 W2) * d relu1 (* 1.25 under Dropout) -> DZ1T; db1 partial
//   dW1 tile w += dZ1^T S                       (accumulator gW1)
template <bool DROP>
__device__ __forceinline__ void backward_12(const Lds& L, const bf16x8* gW2T, int w, int lane, f32x16 gW2[4],
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
    bf16x8 wf[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wf[kk] = gW2T[(w * 8 + kk) * 64 + lane];
    f32x16 acc = {0};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) acc = mfma(lfrag(L.DZ2, kLdZ2, 0, 16 * kk, lane), wf[kk], acc);
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
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) gW1 = mfma(lfrag(L.DZ1T, kLdT, 32 * w, 16 * kk, lane), lfrag(L.ST, kLdT, 0, 16 * kk, lane), gW1);
}

// write the register-held gradients of W1 / W2 (main 256 columns) / b1
__device__ __forceinline__ void store_w12(float* P, int ld2, int w, int lane, const f32x16 gW2[4], const f32x16& gW1,
                                          float gb1) {
  const int mt = w & 3, nt0 = 4 * (w >> 2);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int v = 0; v < 16; ++v)
      P[kPW2 + (32 * mt + drow(v, lane)) * ld2 + 32 * (nt0 + t) + (lane & 31)] = gW2[t][v];
  const int k = lane & 31;
  if (k < kIn) {
#pragma unroll
    for (int v = 0; v < 16; ++v) P[kPW1 + (32 * w + drow(v, lane)) * kIn + k] = gW1[v];
  }
  const float b = gb1 + __shfl_xor(gb1, 32, 64);
  if (lane < 32) P[kPB1 + 32 * w + lane] = b;
}

// ---------------------------------------------------------------- bootstrap target
// y = r + gamma (1 - done) Q'(s', mu'(s')) for the sub-tile's rows with the
// target nets' grad packs (the same batch-major layers as the steps), into
// L.Y; uses H1 / H2f as scratch (they are rewritten by the step after it).
// Inputs in L.S2r, L.RB, L.DB; all threads of the workgroup call it.
__device__ __forceinline__ void bootstrap_target(const Lds& L, const char* tap, const char* tcp, float gamma, int w,
                                                 int lane) {
  asm volatile("" : "+s"(tap), "+s"(tcp));  // no LICM of the fragment loads out of the sub-tile loop
  const bf16x8* aW1 = (const bf16x8*)(tap + kGW1);
  const bf16x8* aW2 = (const bf16x8*)(tap + kGW2);
  const float* at = (const float*)(tap + kGTail);
  const bf16x8* cW1 = (const bf16x8*)(tcp + kGW1);
  const bf16x8* cW2 = (const bf16x8*)(tcp + kGW2);
  const float* ct = (const float*)(tcp + kGTail);
  const bool l2 = w < 4;
  const int u = 32 * (w & 3) + (lane & 31);
  __syncthreads();  // S2r in
  layer1<false>(L.S2r, aW1, at, w, lane, L.H1, nullptr, 0, 0, 0, nullptr, 0);
  __syncthreads();
  if (l2) {
    const f32x16 acc = layer2(L.H1, aW2, w, lane);
    const float b2 = at[kTB2 + u];
#pragma unroll
    for (int v = 0; v < 16; ++v) L.H2f[drow(v, lane) * kLdH2f + u] = fmaxf(acc[v] + b2, 0.f);
  }
  __syncthreads();
  {  // mu'(s')
    const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
    const float z0 = row_dot128(L.H2f, kLdH2f, at + kTW3, 1);
    const float z1 = row_dot128(L.H2f, kLdH2f, at + kTW3 + kH2, 1);
    if (c < 2) L.A2[2 * i + c] = tanhf((c ? z1 : z0) + at[kTB3 + c]);
  }
  __syncthreads();
  layer1<false>(L.S2r, cW1, ct, w, lane, L.H1, nullptr, 0, 0, 0, nullptr, 0);
  __syncthreads();
  if (l2) {  // Q' terms relu(z2) W3 per (row, unit)
    const f32x16 acc = layer2(L.H1, cW2, w, lane);
    const float b2 = ct[kTB2 + u], wa0 = ct[kTW2a + 2 * u], wa1 = ct[kTW2a + 2 * u + 1], w3 = ct[kTW3 + u];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int i = drow(v, lane);
      const float z = acc[v] + b2 + L.A2[2 * i] * wa0 + L.A2[2 * i + 1] * wa1;
      L.H2f[i * kLdH2f + u] = fmaxf(z, 0.f) * w3;
    }
  }
  __syncthreads();
  {
    const int i = threadIdx.x >> 4;
    const float q = ct[kTB3] + row_sum128(L.H2f, kLdH2f);
    if ((threadIdx.x & 15) == 0) L.Y[i] = L.RB[i] + gamma * (1.f - L.DB[i]) * q;
  }
  __syncthreads();
}

// ---------------------------------------------------------------- critic step
// Critic.forward in train mode + F.mse_loss(q, y) backward
// (DDPG.critic_step; critic.fit, SkillshotLearner.py:434): dL/dq =
// grad_scale * (q - y) with grad_scale = 2 / (global batch).
__global__ void __launch_bounds__(kThreads) k_critic_grad(const float* __restrict__ S, const float* __restrict__ A,
                                                          const float* __restrict__ Y, int64_t B, int64_t key_row0,
                                                          int sub_per_wg,
                                                          float grad_scale, uint64_t seed,
                                                          const int64_t* __restrict__ call_ctr,
                                                          const char* __restrict__ gpack, float* __restrict__ partial,
                                                          float* step_ctr, int n_steps, float* __restrict__ loss_out,
                                                          uint8_t* __restrict__ mask_out, const float* __restrict__ S2,
                                                          const float* __restrict__ R, const float* __restrict__ D,
                                                          float gamma, const char* __restrict__ tapack,
                                                          const char* __restrict__ tcpack) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve(smem, false);
  SK_TP(0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5;
  const uint64_t call = (uint64_t)*call_ctr;
  const bf16x8* fW1_ = (const bf16x8*)(gpack + kGW1);
  const bf16x8* fW2_ = (const bf16x8*)(gpack + kGW2);
  const bf16x8* fW2T_ = (const bf16x8*)(gpack + kGW2T);
  const float* tail_ = (const float*)(gpack + kGTail);
  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  for (int t = threadIdx.x; t < 32 * kLdT; t += kThreads) L.ST[t] = 0;
  f32x16 gW2[4], gW1 = {0};
#pragma unroll
  for (int k = 0; k < 4; ++k) gW2[k] = f32x16{0};
  float gb1 = 0.f, gb2 = 0.f, gw2a0 = 0.f, gw2a1 = 0.f, gw3 = 0.f, gb3 = 0.f, lsum = 0.f;
  const bool l2 = w < 4;               // layer-2 waves
  const int u = 32 * (w & 3) + (lane & 31);  // their layer-2 unit
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  __syncthreads();
  SK_TP(1);
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;  // uniform across the workgroup
    // launder the weight bases every sub-tile: otherwise LICM hoists every
    // (loop-invariant) fragment load out of the loop and spills
    const bf16x8* fW1 = fW1_;
    const bf16x8* fW2 = fW2_;
    const bf16x8* fW2T = fW2T_;
    const float* tail = tail_;
    asm volatile("" : "+s"(fW1), "+s"(fW2), "+s"(fW2T), "+s"(tail));
    load_states(L, S, row0, B);
    if (threadIdx.x < 64) L.A[threadIdx.x] = row0 + (threadIdx.x >> 1) < B ? A[row0 * 2 + threadIdx.x] : 0.f;
    if (tapack) {  // the DDPG target y = r + gamma (1 - done) Q'(s', mu'(s')) of this sub-tile, in LDS
      for (int t = threadIdx.x; t < 32 * 16; t += kThreads) {
        const int i = t >> 4, k = t & 15;
        L.S2r[i * kLdS + k] = f2bf((k < kIn && row0 + i < B) ? S2[(row0 + i) * kIn + k] : 0.f);
      }
      if (threadIdx.x < 32) {
        const bool ok = row0 + threadIdx.x < B;
        L.RB[threadIdx.x] = ok ? R[row0 + threadIdx.x] : 0.f;
        L.DB[threadIdx.x] = ok ? D[row0 + threadIdx.x] : 0.f;
      }
      SK_TP(2);
      bootstrap_target(L, tapack, tcpack, gamma, w, lane);
      SK_TP(3);
    } else if (threadIdx.x < 32) {
      L.Y[threadIdx.x] = row0 + threadIdx.x < B ? Y[row0 + threadIdx.x] : 0.f;
    }
    __syncthreads();
    SK_TP(4);
    layer1<true>(L.Sr, fW1, tail, w, lane, L.H1, L.H1T, seed, call, row0, mask_out, B, key_row0);
    __syncthreads();
    SK_TP(5);
    float h2v[16];
    if (l2) {
      const f32x16 acc = layer2(L.H1, fW2, w, lane);
      const float b2 = tail[kTB2 + u], wa0 = tail[kTW2a + 2 * u], wa1 = tail[kTW2a + 2 * u + 1];
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = drow(v, lane);
        h2v[v] = fmaxf(acc[v] + b2 + L.A[2 * i] * wa0 + L.A[2 * i + 1] * wa1, 0.f);
        L.H2f[i * kLdH2f + u] = h2v[v];
      }
    }
    __syncthreads();
    SK_TP(6);
    {  // q and dL/dq per row (all threads: row_dot128)
      const int i = threadIdx.x >> 4;
      const float q = tail[kTB3] + row_dot128(L.H2f, kLdH2f, tail + kTW3, 1);
      if ((threadIdx.x & 15) == 0) {
        const float e = row0 + i < B ? q - L.Y[i] : 0.f;
        L.DQ[i] = grad_scale * e;
        gb3 += grad_scale * e;
        lsum += e * e;
      }
    }
    __syncthreads();
    SK_TP(7);
    if (l2) {
      const float w3 = tail[kTW3 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = drow(4 * g + q, lane);
          const float dq = L.DQ[i];
          d[q] = h2v[4 * g + q] > 0.f ? dq * w3 : 0.f;
          L.DZ2[i * kLdZ2 + u] = f2bf(d[q]);
          gb2 += d[q];
          gw2a0 += d[q] * L.A[2 * i];
          gw2a1 += d[q] * L.A[2 * i + 1];
          gw3 += dq * h2v[4 * g + q];
        }
        store_t4(L.DZ2T, kLdT, u, drow(4 * g, lane), d[0], d[1], d[2], d[3]);
      }
    }
    __syncthreads();
    SK_TP(8);
    backward_12<true>(L, fW2T, w, lane, gW2, gW1, gb1);
    __syncthreads();
    SK_TP(9);
  }
  float* P = partial + (int64_t)blockIdx.x * kCP;
  store_w12(P, kCPW2ld, w, lane, gW2, gW1, gb1);
  SK_TP(10);
  gb2 += __shfl_xor(gb2, 32, 64);
  gw2a0 += __shfl_xor(gw2a0, 32, 64);
  gw2a1 += __shfl_xor(gw2a1, 32, 64);
  gw3 += __shfl_xor(gw3, 32, 64);
  if (l2 && hh == 0) {
    P[kCPB2 + u] = gb2;
    P[kPW2 + u * kCPW2ld + kH1] = gw2a0;
    P[kPW2 + u * kCPW2ld + kH1 + 1] = gw2a1;
    P[kCPW3 + u] = gw3;
  }
  if ((threadIdx.x & 15) == 0) {  // the row-owner threads hold db3 / loss partials
    atomicAdd(&L.RED[0], gb3);
    atomicAdd(&L.RED[1], lsum);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    P[kCPB3] = L.RED[0];
    if (loss_out) atomicAdd(loss_out, L.RED[1]);
  }
  SK_TP(11);
}

// ---------------------------------------------------------------- actor step
// model_actor_fit_step (SkillshotLearner.py:386-417; DDPG.model_actor_fit_step):
// gradient of -loss_scale * sum_b Q(s_b, mu(s_b)) w.r.t. the actor, critic in
// inference mode (no Dropout).  q_out (optional) receives sum_b Q.
__global__ void __launch_bounds__(kThreads) k_actor_grad(const float* __restrict__ S, int64_t B, int sub_per_wg,
                                                         float loss_scale, const char* __restrict__ apack,
                                                         const char* __restrict__ cpack, float* __restrict__ partial,
                                                         float* step_ctr, int n_steps, float* __restrict__ q_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const Lds L = carve(smem, true);
  SK_TP(0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5;

  if (blockIdx.x == 0 && threadIdx.x < n_steps) step_ctr[threadIdx.x] += 1.0f;  // Adam's step (read by k_adam_flat)
  for (int t = threadIdx.x; t < 32 * kLdT; t += kThreads) L.ST[t] = 0;
  f32x16 gW2[4], gW1 = {0};
#pragma unroll
  for (int k = 0; k < 4; ++k) gW2[k] = f32x16{0};
  float gb1 = 0.f, gb2 = 0.f, gw30 = 0.f, gw31 = 0.f, gb3 = 0.f, qsum = 0.f;
  const bool l2 = w < 4;                     // layer-2 waves
  const int u = 32 * (w & 3) + (lane & 31);  // their layer-2 unit
  if (threadIdx.x < 4) L.RED[threadIdx.x] = 0.f;
  __syncthreads();
  SK_TP(1);
  for (int sub = 0; sub < sub_per_wg; ++sub) {
    const int64_t row0 = ((int64_t)blockIdx.x * sub_per_wg + sub) * 32;
    if (row0 >= B) break;  // uniform across the workgroup
    const char* ap = apack;
    const char* cp = cpack;
    asm volatile("" : "+s"(ap), "+s"(cp));  // no LICM of the fragment loads (see k_critic_grad)
    const bf16x8* aW1 = (const bf16x8*)(ap + kGW1);
    const bf16x8* aW2 = (const bf16x8*)(ap + kGW2);
    const bf16x8* aW2T = (const bf16x8*)(ap + kGW2T);
    const float* at = (const float*)(ap + kGTail);
    const bf16x8* cW1 = (const bf16x8*)(cp + kGW1);
    const bf16x8* cW2 = (const bf16x8*)(cp + kGW2);
    const float* ct = (const float*)(cp + kGTail);
    load_states(L, S, row0, B);
    __syncthreads();
    SK_TP(2);
    layer1<false>(L.Sr, aW1, at, w, lane, L.H1, L.H1T, 0, 0, 0, nullptr, B);
    layer1<false>(L.Sr, cW1, ct, w, lane, L.H1C, nullptr, 0, 0, 0, nullptr, B);
    __syncthreads();
    SK_TP(3);
    if (l2) {  // actor h2 -> H2f (fp32, kept for the backward)
      const f32x16 acc = layer2(L.H1, aW2, w, lane);
      const float b2 = at[kTB2 + u];
#pragma unroll
      for (int v = 0; v < 16; ++v) L.H2f[drow(v, lane) * kLdH2f + u] = fmaxf(acc[v] + b2, 0.f);
    }
    __syncthreads();
    SK_TP(4);
    {  // mu(s) = tanh(W3 h2 + b3) (all threads: row_dot128)
      const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
      const float z0 = row_dot128(L.H2f, kLdH2f, at + kTW3, 1);
      const float z1 = row_dot128(L.H2f, kLdH2f, at + kTW3 + kH2, 1);
      if (c < 2) L.A[2 * i + c] = tanhf((c ? z1 : z0) + at[kTB3 + c]);
    }
    __syncthreads();
    SK_TP(5);
    {  // critic layer 2 at (s, mu(s)): dQ/dz2 = W3 relu'(z2) (rows beyond B: 0)
      f32x16 acc = {0};
      if (l2) acc = layer2(L.H1C, cW2, w, lane);
      __syncthreads();  // every wave is done reading H1C: its space takes the Q terms
      float* QZ = (float*)L.H1C;  // [32][kLdH2f] fp32 relu(z2) W3 (q_out)
      if (l2) {
        const float b2 = ct[kTB2 + u], wa0 = ct[kTW2a + 2 * u], wa1 = ct[kTW2a + 2 * u + 1], w3 = ct[kTW3 + u];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int i = drow(v, lane);
          const float z = acc[v] + b2 + L.A[2 * i] * wa0 + L.A[2 * i + 1] * wa1;
          L.DZC[i * kLdH2f + u] = (z > 0.f && row0 + i < B) ? w3 : 0.f;
          if (q_out) QZ[i * kLdH2f + u] = fmaxf(z, 0.f) * w3;
        }
      }
      __syncthreads();
      // dL/dz3 = -loss_scale * dQ/da * (1 - a^2), dQ/da = sum_u dQ/dz2 W2[u][256 + j]
      const int i = threadIdx.x >> 4, c = threadIdx.x & 15;
      const float da0 = row_dot128(L.DZC, kLdH2f, ct + kTW2a, 2);
      const float da1 = row_dot128(L.DZC, kLdH2f, ct + kTW2a + 1, 2);
      const float qrow = q_out ? row_sum128(QZ, kLdH2f) : 0.f;
      if (c < 2) {
        const float a = L.A[2 * i + c];
        const float d = -loss_scale * (c ? da1 : da0) * (1.f - a * a);
        L.DZ3[2 * i + c] = d;
        gb3 += d;  // db3[c] partial (threads with c < 2)
      }
      if (c == 0 && q_out && row0 + i < B) qsum += ct[kTB3] + qrow;
    }
    __syncthreads();
    SK_TP(6);
    if (l2) {  // dZ2 = (dz3 W3) relu'(h2);  dW3[j][u] += sum_i dz3[i][j] h2[i][u]
      const float w30 = at[kTW3 + u], w31 = at[kTW3 + kH2 + u];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = drow(4 * g + q, lane);
          const float z0 = L.DZ3[2 * i], z1 = L.DZ3[2 * i + 1];
          const float h = L.H2f[i * kLdH2f + u];
          d[q] = h > 0.f ? z0 * w30 + z1 * w31 : 0.f;
          L.DZ2[i * kLdZ2 + u] = f2bf(d[q]);
          gb2 += d[q];
          gw30 += z0 * h;
          gw31 += z1 * h;
        }
        store_t4(L.DZ2T, kLdT, u, drow(4 * g, lane), d[0], d[1], d[2], d[3]);
      }
    }
    __syncthreads();
    SK_TP(7);
    backward_12<false>(L, aW2T, w, lane, gW2, gW1, gb1);
    __syncthreads();
    SK_TP(8);
  }
  float* P = partial + (int64_t)blockIdx.x * kAP;
  store_w12(P, kH1, w, lane, gW2, gW1, gb1);
  SK_TP(9);
  gb2 += __shfl_xor(gb2, 32, 64);
  gw30 += __shfl_xor(gw30, 32, 64);
  gw31 += __shfl_xor(gw31, 32, 64);
  if (l2 && hh == 0) {
    P[kAPB2 + u] = gb2;
    P[kAPW3 + u] = gw30;
    P[kAPW3 + kH2 + u] = gw31;
  }
  {  // db3[j]: threads with c == j; sum Q: threads with c == 0
    const int c = threadIdx.x & 15;
    if (c < 2) atomicAdd(&L.RED[c], gb3);
    if (c == 0) atomicAdd(&L.RED[2], qsum);
  }
  __syncthreads();
  if (threadIdx.x < 2) P[kAPB3 + threadIdx.x] = L.RED[threadIdx.x];
  if (threadIdx.x == 0 && q_out) atomicAdd(q_out, L.RED[2]);
  SK_TP(10);
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

constexpr int kAdamParams = 64, kAdamSlices = 4;

__global__ void __launch_bounds__(kAdamParams * kAdamSlices) k_adam_flat(const float* __restrict__ partial, int G, int P, const float* __restrict__ grad_in,
                            float* __restrict__ grad_out, int apply, float* __restrict__ param, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ step_ctr, float lr, float beta1,
                            float beta2, float eps, float* __restrict__ target, float tau, float* stat_acc,
                            float stat_scale, float* stat_out, int64_t* counter, PackOut po) {
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
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 independent loads in flight
  if (in) {
    int k = slice;
    for (; k + 7 * kAdamSlices < G; k += 8 * kAdamSlices) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += partial[(int64_t)(k + j * kAdamSlices) * P + p];
    }
    for (; k < G; k += kAdamSlices) acc[0] += partial[(int64_t)k * P + p];
  }
  const float part = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (slice > 0) red[slice - 1][lane] = part;
  __syncthreads();
  if (slice > 0 || !in) return;
  float g = grad_in ? grad_in[p] : 0.f;
  g += part;
#pragma unroll
  for (int j = 0; j < kAdamSlices - 1; ++j) g += red[j][lane];
  if (grad_out) grad_out[p] = g;
  if (!apply) return;
  const float t = step_ctr[0];
  const float alpha = lr * sqrtf(1.f - powf(beta2, t)) / (1.f - powf(beta1, t));
  float mm = m[p], vv = v[p];
  mm = mm + (g - mm) * (1.f - beta1);
  vv = vv + (g * g - vv) * (1.f - beta2);
  m[p] = mm;
  v[p] = vv;
  const float w = param[p] - (mm * alpha) / (sqrtf(vv) + eps);
  param[p] = w;
  if (po.gp) scatter_grad_pack(po.gp, p, w, po.ld2, po.n_out);
  if (po.fp) scatter_fwd_pack(po.fp, p, w);
  if (target) {
    const float tw = target[p] + tau * (w - target[p]);
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
    set_lds(k_critic_grad, kLdsCritic);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg(batch);
  const unsigned G = (unsigned)sk_update_partials(batch);
  k_critic_grad<<<G, kThreads, kLdsCritic, (hipStream_t)stream>>>(
      obs, actions, targets, batch, row_offset, (int)spw, grad_scale, seed, call_counter, (const char*)cpack, partial,
      step_counters, n_steps, loss_sum, dropout_mask, next_obs, rewards, done, gamma,
      (const char*)target_actor_gpack, (const char*)target_critic_gpack);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_grad(const void* apack, const void* cpack, const float* obs, int64_t batch, float loss_scale,
                  float* partial, float* step_counters, int32_t n_steps, float* q_sum, void* stream) {
  if (!apack || !cpack || !obs || !partial || batch <= 0) return SK_EINVAL;
  if ((n_steps > 0 && !step_counters) || n_steps < 0 || n_steps > 64) return SK_EINVAL;
  if ((((uintptr_t)apack) & 15) || (((uintptr_t)cpack) & 15) || (((uintptr_t)obs) & 3)) return SK_EINVAL;
  static bool attr = false;
  if (!attr) {
    set_lds(k_actor_grad, kLdsActor);
    attr = true;
  }
  const int64_t spw = subtiles_per_wg(batch);
  const unsigned G = (unsigned)sk_update_partials(batch);
  k_actor_grad<<<G, kThreads, kLdsActor, (hipStream_t)stream>>>(obs, batch, (int)spw, loss_scale, (const char*)apack,
                                                                (const char*)cpack, partial, step_counters, n_steps,
                                                                q_sum);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_adam_flat_packed(const float* partial, int32_t n_partials, int32_t n_params, const float* grad_in,
                        float* grad_out, int32_t apply, float* param, float* exp_avg, float* exp_avg_sq,
                        const float* step_counter, float lr, float beta1, float beta2, float eps, float* target,
                        float tau, float* stat_acc, float stat_scale, float* stat_out, int64_t* counter,
                        const sk_pack_targets* packs, void* stream) {
  if (n_params <= 0 || n_partials < 0 || (n_partials > 0 && !partial)) return SK_EINVAL;
  if (apply && (!param || !exp_avg || !exp_avg_sq || !step_counter)) return SK_EINVAL;
  PackOut po = {nullptr, nullptr, nullptr, kH1, 1};
  if (packs && apply) {
    const int ld2 = packs->ld2, n_out = packs->n_out;
    if ((ld2 != kH1 && ld2 != kH1 + 2) || (n_out != 1 && n_out != 2)) return SK_EINVAL;
    if (n_params != kPW2 + kH2 * ld2 + kH2 + n_out * kH2 + n_out) return SK_EINVAL;
    if (packs->actor_fwd_pack && (ld2 != kH1 || n_out != kOut)) return SK_EINVAL;
    if (packs->target_gpack && !target) return SK_EINVAL;
    for (const void* b : {packs->param_gpack, packs->target_gpack, packs->actor_fwd_pack})
      if (((uintptr_t)b) & 15) return SK_EINVAL;
    po = {(char*)packs->param_gpack, (char*)packs->target_gpack, (char*)packs->actor_fwd_pack, ld2, n_out};
  }
  k_adam_flat<<<(n_params + kAdamParams - 1) / kAdamParams, kAdamParams * kAdamSlices, 0, (hipStream_t)stream>>>(
      partial, n_partials, n_params, grad_in, grad_out, apply, param, exp_avg, exp_avg_sq, step_counter, lr, beta1,
      beta2, eps, target, tau, stat_acc, stat_scale, stat_out, counter, po);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
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
