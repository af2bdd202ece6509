// sk_actor.hip — fused actor MLP forward on MFMA (gfx950), with per-row
// parameter noise by local reparameterisation.
//
// Replaces the batched form of model_actor.predict (SkillshotLearner.py:222,
// 235, 271) on the actor of model_define_actor (:70-96):
//     a = tanh(W3 relu(W2 relu(W1 s + b1) + b2) + b3),  s: 12 -> 256 -> 128 -> 2
// and model_act_param_noise (:245-281), where every weight and bias becomes
// w(1 + sd*eps) afresh per call: with one independent noisy actor per row,
// each noisy weight is used once per row, so every pre-activation is exactly
//     y = W x + b + sd * sqrt(W^2 x^2 + b^2) * xi,  xi ~ N(0,1) per unit and row.
//
// Layout (cdna_hip_programming.md §3 "accumulator tile as the next MFMA's
// operand"): activations are kept TRANSPOSED, H^T = W X^T, with the batch row
// on the lane and hidden units in the 16 accumulator registers of a
// v_mfma_f32_32x32x16_bf16 tile, so each layer's accumulator converts in
// registers to the next layer's B operand; the weights are pre-packed
// (k_actor_pack) into A fragments in the matching permuted k order.
// Per 32-row tile: layer 1 8 MFMAs, layer 2 64 (x2 with noise); layer 3 (2 x 128) in
// fp32 on the VALU from layer 2's accumulators.
// W2 (and W2^2) fragments are staged once per workgroup in LDS (64/128 KiB);
// W1 fragments (8 KiB, + squares) are read through L1.  bf16 operands, fp32
// accumulate, fp32 bias/noise/activation epilogues.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"

namespace {

using namespace skmlp;

// deterministic: 8 waves (two per SIMD, 141 VGPRs); noise: 4 waves (one per
// SIMD) so the mean and variance chains' operands (h1, h1^2: 128 VGPRs) plus
// both accumulators fit the 512-register budget without spilling (332 VGPRs;
// 8 waves force 256 and 77 spilled: 61 -> 72 us at 131,072 rows,
// profiles/r02_actor_threads_ab.jsonl)
#ifndef SK_NOISE_THREADS  // A/B builds only
#define SK_NOISE_THREADS 256
#endif
template <bool NOISE>
constexpr int threads_for() { return NOISE ? SK_NOISE_THREADS : 512; }


// ---------------------------------------------------------------- packing
// W1: [256][12] row-major (torch Linear weight [out][in]); A fragment of
// hidden chunk c, lane (r, h), element j = W1[32c + r][8h + j] (k >= 12 -> 0).
// W2: [128][256]; chunk t, k-step kk, lane (r, h), element j =
//     W2[32t + r][32(kk>>1) + 16(kk&1) + 8(j>>2) + 4h + (j&3)]  (the row order
//     of the previous accumulator's registers 8s..8s+7, s = kk&1).
// W3: [2][128] copied as fp32 (with its squares) for the VALU layer 3.
__global__ void k_actor_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                             const float* b3, char* out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  short* w1 = (short*)(out + kOffW1);
  short* w1s = (short*)(out + kOffW1s);
  short* w2 = (short*)(out + kOffW2);
  short* w2s = (short*)(out + kOffW2s);
  float* bias = (float*)(out + kOffB);
  // one thread per (fragment, lane): layer 1 (8*64), layer 2 (64*64); then biases, W3
  if (t < 8 * 64) {
    int c = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    for (int j = 0; j < 8; ++j) {
      int k = 8 * h + j;
      float v = k < kIn ? W1[(32 * c + r) * kIn + k] : 0.f;
      w1[t * 8 + j] = f2bf(v);
      w1s[t * 8 + j] = f2bf(v * v);
    }
  } else if (t < 8 * 64 + 64 * 64) {
    int u = t - 8 * 64;
    int frag = u >> 6, lane = u & 63, r = lane & 31, h = lane >> 5;
    int tt = frag >> 4, kk = frag & 15;
    for (int j = 0; j < 8; ++j) {
      int k = 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
      float v = W2[(32 * tt + r) * kH1 + k];
      w2[u * 8 + j] = f2bf(v);
      w2s[u * 8 + j] = f2bf(v * v);
    }
  } else if (t < 8 * 64 + 64 * 64 + 512) {
    int u = t - 8 * 64 - 64 * 64;
    float v = 0.f;
    if (u < kH1) v = b1[u];
    else if (u < kH1 + kH2) v = b2[u - kH1];
    else if (u < kH1 + kH2 + kOut) v = b3[u - kH1 - kH2];
    bias[u] = v;
  } else if (t < 8 * 64 + 64 * 64 + 512 + 256) {
    int u = t - 8 * 64 - 64 * 64 - 512;  // o * 128 + k
    float v = W3[u];
    float* w3f = (float*)(out + kOffW3f);
    w3f[u] = v;
    w3f[256 + u] = v * v;
  }
}

// ---------------------------------------------------------------- forward
// DBG (diagnostics build only): dbg[row][kDbgCols] receives every unit's
// post-activation value (256 layer-1, 128 layer-2, 2 layer-3 pre-tanh), then
// layer 2's pre-bias mean accumulator, variance accumulator and normal draw
// (3 x 128).
constexpr int kDbgCols = 386 + 3 * 128;
// With a device call counter adv = {call number, arrivals}: every workgroup has
// read adv[0] before its first barrier; the last to finish stores the number
// it used, so the next launch draws fresh noise without a separate add.
// grouped (sk_actor_forward_noise, adv = uint64[SK_ACTOR_COUNTER_WORDS]):
// workgroup b arrives first on group counter b % 8 (its own 128-byte line,
// adv[2 + 16 (b % 8)]), the last of each group on adv[1]; device-scope
// atomics on one address serialise, and 256 arrivals on adv[1] cost up to
// 3 us of a bf16 launch (store-only ablation, profiles/r02_actor_arrival_ab.jsonl)
__device__ __forceinline__ void advance_call(uint64_t* adv, uint64_t call, int grouped = 0) {
  if (threadIdx.x != 0) return;
  unsigned long long last = (unsigned long long)gridDim.x - 1;
  if (grouped) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned long long members = (gridDim.x - g + 7u) / 8u;  // workgroups b with b % 8 == g
    unsigned long long* gc = (unsigned long long*)&adv[2 + 16 * g];
    if (atomicAdd(gc, 1ull) != members - 1) return;
    *gc = 0;  // every member of the group has arrived
    last = (gridDim.x < 8u ? gridDim.x : 8u) - 1;
  }
  const unsigned long long prev = atomicAdd((unsigned long long*)&adv[1], 1ull);
  if (prev == last) {
    adv[1] = 0;
    adv[0] = call;
  }
}

template <bool NOISE, bool DBG = false>
__global__ void __launch_bounds__(threads_for<NOISE>()) k_actor_fwd(const float* __restrict__ X, float* __restrict__ out,
                                                        int64_t M, const char* __restrict__ packed, float sd,
                                                        uint64_t seed, uint64_t call,
                                                        const uint64_t* __restrict__ call_dev = nullptr,
                                                        float* dbg = nullptr, uint64_t* adv = nullptr,
                                                        float action_sd = 0.f, int grouped = 0) {
  // the noise call number comes from device memory when given (graph replays
  // then draw fresh noise per replay): *call_dev, advanced by the caller, or,
  // with adv, adv[0] + 1, stored back by the last workgroup (advance_call)
  const bool draws = NOISE || action_sd != 0.f;  // parameter and/or action noise
  if (draws && call_dev) call = *call_dev;  // wave-uniform scalar load
  if (draws && adv) call = adv[0] + 1;
  asm volatile("" : "+s"(call));  // read before the staging barrier (advance_call relies on it)
  const float k2 = noise_k2(sd);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* sW2 = (bf16x8*)smem;                               // [4][16][64]
  bf16x8* sW2s = (bf16x8*)(smem + kW2Frag);                  // NOISE only
  float* sB = (float*)(smem + (NOISE ? 2 : 1) * kW2Frag);    // b1 b2 b3 (512), W3 (256), W3^2 (256)
  float* sW3 = sB + 512;

  constexpr int kThreads = threads_for<NOISE>();
  {  // stage W2 fragments (+ squares) and biases once per workgroup
    const uint4* g = (const uint4*)(packed + kOffW2);
    uint4* s = (uint4*)smem;
    const int n16 = (NOISE ? 2 : 1) * kW2Frag / 16;
    for (int k = threadIdx.x; k < n16; k += kThreads) s[k] = g[k];  // W2s follows W2 in the buffer
    const float* gb = (const float*)(packed + kOffB);
    for (int k = threadIdx.x; k < 1024; k += kThreads) sB[k] = gb[k];  // biases then W3, W3^2 (contiguous)
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (M + 31) / 32;
  const int64_t wave = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kThreads / 64);

  for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
    // launder the weight base each tile: otherwise LICM hoists all 32 W1/W3
    // fragment loads out of the tile loop and spills them
    const char* pk = packed;
    asm volatile("" : "+s"(pk));
    const bf16x8* gW1 = (const bf16x8*)(pk + kOffW1);
    const bf16x8* gW1s = (const bf16x8*)(pk + kOffW1s);
    const int64_t row = tile * 32 + r;
    const bool valid = row < M;
    // ---- X^T fragment: B[k = 8h + j][col r] = X[row][8h + j]
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = 0.f;
    if (valid) {
      const float* xr = X + row * kIn + 8 * h;
      if (h == 0) {
        float4 a = *(const float4*)xr, b = *(const float4*)(xr + 4);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      } else {
        float4 a = *(const float4*)xr;
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      }
    }
    bf16x8 xb, xs;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xb[j] = f2bf(x[j]);
      xs[j] = f2bf(x[j] * x[j]);
    }

    // ---- layer 1: H1^T = relu(W1 X^T + b1 [+ noise]) -> 16 B fragments (k-steps of layer 2)
    bf16x8 h1[16];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      f32x16 acc = {0}, var = {0};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gW1[c * 64 + lane], xb, acc, 0, 0, 0);
      if (NOISE) var = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gW1s[c * 64 + lane], xs, var, 0, 0, 0);
      Pairs8 z;
      if (NOISE) pairs8(seed, call, (uint32_t)row, (uint32_t)c, h, k2, z);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int hid = 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
        const float b = sB[hid];
        float y = NOISE ? noisy_pre_pair(acc[i], b, var[i], z, i) : acc[i] + b;
        y = fmaxf(y, 0.f);
        acc[i] = y;
        if (DBG && valid) dbg[row * kDbgCols + hid] = y;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = f2bf(acc[8 * s + j]);
        h1[2 * c + s] = f;
      }
      __builtin_amdgcn_sched_barrier(0);  // one chunk's accumulators live at a time
    }

    // ---- layer 2: H2^T = relu(W2 H1^T + b2 [+ noise]), and layer 3 on the VALU:
    // each lane accumulates fp32 partial dot products of W3 (and W3^2 for the
    // noise variance) over the 64 layer-2 units it holds; the two lane halves
    // are combined with one cross-half shuffle.
    // k-step outer, output chunk inner: the 4 chunks' accumulator chains (8
    // with the variance GEMM) are independent, so no MFMA waits on its
    // predecessor's result, and each k-step's h1^2 fragment is squared once
    // (not once per chunk).  Every accumulator sums its k-steps in the same
    // order as a chunk-outer loop: the results are bit-identical.
    f32x16 accs[4], vars[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      accs[t] = f32x16{0};
      vars[t] = f32x16{0};
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const bf16x8 hs = NOISE ? sq_bf16(h1[kk]) : h1[kk];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        accs[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sW2[(t * 16 + kk) * 64 + lane], h1[kk], accs[t], 0, 0, 0);
        if (NOISE)
          vars[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sW2s[(t * 16 + kk) * 64 + lane], hs, vars[t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // cap hoisted LDS fragments
    }
    float m0 = 0.f, m1 = 0.f, q0 = 0.f, q1 = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x16 acc = accs[t], var = vars[t];
      Pairs8 z;
      if (NOISE) pairs8(seed, call, (uint32_t)row, (uint32_t)(8 + t), h, k2, z);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int hid = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
        const float b = sB[kH1 + hid];
        float y = NOISE ? noisy_pre_pair(acc[i], b, var[i], z, i) : acc[i] + b;
        y = fmaxf(y, 0.f);
        if (DBG && valid) {
          dbg[row * kDbgCols + kH1 + hid] = y;
          dbg[row * kDbgCols + 386 + hid] = acc[i];
          dbg[row * kDbgCols + 386 + kH2 + hid] = NOISE ? var[i] : 0.f;
          dbg[row * kDbgCols + 386 + 2 * kH2 + hid] = NOISE ? pair_normal(z, i) / sd : 0.f;
        }
        m0 = __builtin_fmaf(sW3[hid], y, m0);
        m1 = __builtin_fmaf(sW3[kH2 + hid], y, m1);
        if (NOISE) {
          const float yy = y * y;
          q0 = __builtin_fmaf(sW3[2 * kH2 + hid], yy, q0);
          q1 = __builtin_fmaf(sW3[3 * kH2 + hid], yy, q1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    m0 += __shfl_xor(m0, 32, 64);
    m1 += __shfl_xor(m1, 32, 64);
    if (NOISE) {
      q0 += __shfl_xor(q0, 32, 64);
      q1 += __shfl_xor(q1, 32, 64);
    }

    // ---- layer 3 epilogue: a = tanh(W3 h2 + b3 [+ noise]) for this lane's row
    if (h == 0 && valid) {
      float z[16];
      if (NOISE) normals16(seed, call, (uint32_t)row, 12u, h, k2, z);
      const float mm[2] = {m0, m1}, qq[2] = {q0, q1};
      float o[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float b = sB[kH1 + kH2 + i];
        const float y = NOISE ? noisy_pre(mm[i], b, qq[i], z[i]) : mm[i] + b;
        if (DBG) dbg[row * kDbgCols + kH1 + kH2 + i] = y;
        o[i] = tanhf(y);
      }
      if (action_sd != 0.f) {  // model_act_action_noise (:229-243): tanh output + N(0, sd), unclipped
        float za[2];
        normals2(seed, call, (uint32_t)row, 13u, noise_k2(action_sd), za);
        o[0] += za[0];
        o[1] += za[1];
      }
      *(float2*)(out + row * kOut) = make_float2(o[0], o[1]);
    }
  }
  if (draws && adv) advance_call(adv, call, grouped);
}

// One 32-row tile per WORKGROUP: for batches too small to give every SIMD its
// own tile (the 4,096-game learner has 8,192 rows = 256 tiles for 1,024
// SIMDs).  Wave w computes layer-1 chunks 2w, 2w+1 and layer-2 chunk w.  The
// layer-1 output fragments meet in LDS in the B-operand lane layout, so every
// wave reads fragment kk at [kk][lane]; layer 3's per-wave partial dot
// products are summed across the four waves in LDS.  Same noise counters as
// k_actor_fwd (row, unit chunk, lane half): the two modes draw identical
// noise and differ only in layer 3's fp32 summation order.
constexpr int kWgThreads = 256;
constexpr size_t kWgExtra = 16 * 64 * 16 + 4 * 32 * 16;  // h1 fragments + layer-3 partials

template <bool NOISE>
__global__ void __launch_bounds__(kWgThreads) k_actor_fwd_wg(const float* __restrict__ X, float* __restrict__ out,
                                                            int64_t M, const char* __restrict__ packed, float sd,
                                                            uint64_t seed, uint64_t call,
                                                            const uint64_t* __restrict__ call_dev,
                                                            uint64_t* adv = nullptr, float action_sd = 0.f,
                                                            int grouped = 0) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* sW2 = (bf16x8*)smem;
  bf16x8* sW2s = (bf16x8*)(smem + kW2Frag);
  float* sB = (float*)(smem + (NOISE ? 2 : 1) * kW2Frag);
  float* sW3 = sB + 512;
  bf16x8* sH1 = (bf16x8*)(sB + 1024);            // [16 k-steps][64 lanes]
  float4* sPart = (float4*)(sH1 + 16 * 64);      // [4 waves][32 rows]: m0 m1 q0 q1
  const bool draws = NOISE || action_sd != 0.f;  // parameter and/or action noise
  if (draws && call_dev) call = *call_dev;
  if (draws && adv) call = adv[0] + 1;
  asm volatile("" : "+s"(call));  // read before the staging barrier (advance_call)
  const float k2 = noise_k2(sd);
  {
    const uint4* g = (const uint4*)(packed + kOffW2);
    uint4* sm = (uint4*)smem;
    const int n16 = (NOISE ? 2 : 1) * kW2Frag / 16;
    for (int k = threadIdx.x; k < n16; k += kWgThreads) sm[k] = g[k];
    const float* gb = (const float*)(packed + kOffB);
    for (int k = threadIdx.x; k < 1024; k += kWgThreads) sB[k] = gb[k];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5, w = threadIdx.x >> 6;
  const int64_t ntiles = (M + 31) / 32;
  const bf16x8* gW1 = (const bf16x8*)(packed + kOffW1);
  const bf16x8* gW1s = (const bf16x8*)(packed + kOffW1s);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row = tile * 32 + r;
    const bool valid = row < M;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = 0.f;
    if (valid) {
      const float* xr = X + row * kIn + 8 * h;
      float4 a = *(const float4*)xr;
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      if (h == 0) {
        float4 b = *(const float4*)(xr + 4);
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      }
    }
    bf16x8 xb, xs;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xb[j] = f2bf(x[j]);
      xs[j] = f2bf(x[j] * x[j]);
    }
    // ---- layer 1, chunks 2w and 2w+1 -> LDS
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int c = 2 * w + cc;
      f32x16 acc = {0}, var = {0};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gW1[c * 64 + lane], xb, acc, 0, 0, 0);
      if (NOISE) var = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gW1s[c * 64 + lane], xs, var, 0, 0, 0);
      Pairs8 z;
      if (NOISE) pairs8(seed, call, (uint32_t)row, (uint32_t)c, h, k2, z);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int hid = 32 * c + (i & 3) + 8 * (i >> 2) + 4 * h;
        const float b = sB[hid];
        float y = NOISE ? noisy_pre_pair(acc[i], b, var[i], z, i) : acc[i] + b;
        acc[i] = fmaxf(y, 0.f);
      }
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) {
        bf16x8 f;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = f2bf(acc[8 * sidx + j]);
        sH1[(2 * c + sidx) * 64 + lane] = f;
      }
    }
    __syncthreads();
    // ---- layer 2, chunk t = w, and this wave's share of layer 3
    float m0 = 0.f, m1 = 0.f, q0 = 0.f, q1 = 0.f;
    {
      const int t = w;
      f32x16 acc = {0}, var = {0};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const bf16x8 hb = sH1[kk * 64 + lane];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sW2[(t * 16 + kk) * 64 + lane], hb, acc, 0, 0, 0);
        if (NOISE)
          var = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sW2s[(t * 16 + kk) * 64 + lane], sq_bf16(hb), var, 0, 0, 0);
      }
      Pairs8 z;
      if (NOISE) pairs8(seed, call, (uint32_t)row, (uint32_t)(8 + t), h, k2, z);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int hid = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * h;
        const float b = sB[kH1 + hid];
        float y = NOISE ? noisy_pre_pair(acc[i], b, var[i], z, i) : acc[i] + b;
        y = fmaxf(y, 0.f);
        m0 = __builtin_fmaf(sW3[hid], y, m0);
        m1 = __builtin_fmaf(sW3[kH2 + hid], y, m1);
        if (NOISE) {
          const float yy = y * y;
          q0 = __builtin_fmaf(sW3[2 * kH2 + hid], yy, q0);
          q1 = __builtin_fmaf(sW3[3 * kH2 + hid], yy, q1);
        }
      }
    }
    m0 += __shfl_xor(m0, 32, 64);
    m1 += __shfl_xor(m1, 32, 64);
    if (NOISE) {
      q0 += __shfl_xor(q0, 32, 64);
      q1 += __shfl_xor(q1, 32, 64);
    }
    if (h == 0) sPart[w * 32 + r] = make_float4(m0, m1, q0, q1);
    __syncthreads();
    // ---- layer 3 epilogue on wave 0
    if (w == 0 && h == 0 && valid) {
      float4 p = sPart[r];
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float4 o = sPart[k * 32 + r];
        p.x += o.x; p.y += o.y; p.z += o.z; p.w += o.w;
      }
      float z[16];
      if (NOISE) normals16(seed, call, (uint32_t)row, 12u, 0, k2, z);
      const float mm[2] = {p.x, p.y}, qq[2] = {p.z, p.w};
      float o2[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float b = sB[kH1 + kH2 + i];
        const float y = NOISE ? noisy_pre(mm[i], b, qq[i], z[i]) : mm[i] + b;
        o2[i] = tanhf(y);
      }
      if (action_sd != 0.f) {  // model_act_action_noise (:229-243), as k_actor_fwd
        float za[2];
        normals2(seed, call, (uint32_t)row, 13u, noise_k2(action_sd), za);
        o2[0] += za[0];
        o2[1] += za[1];
      }
      *(float2*)(out + row * kOut) = make_float2(o2[0], o2[1]);
    }
  }
  if (draws && adv) advance_call(adv, call, grouped);
}

// launch-mode override for tests and sweeps: 0 auto, 1 tile per wave, 2 tile per workgroup
int g_actor_mode = 0;

}  // namespace

extern "C" {

size_t sk_actor_packed_bytes(void) { return kPackedBytes; }

int sk_actor_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                  const float* b3, void* packed, void* stream) {
  if (!W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !packed) return SK_EINVAL;
  if (((uintptr_t)packed) & 15) return SK_EINVAL;
  const int total = 8 * 64 + 64 * 64 + 512 + 256;
  k_actor_pack<<<(total + 255) / 256, 256, 0, (hipStream_t)stream>>>(W1, b1, W2, b2, W3, b3, (char*)packed);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

static int actor_forward(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                         uint64_t seed, uint64_t call, const uint64_t* call_dev, void* stream,
                         uint64_t* adv = nullptr, float action_sd = 0.f, int grouped = 0) {
  if (!packed || !obs || !actions || rows < 0) return SK_EINVAL;
  if ((((uintptr_t)obs) & 15) || (((uintptr_t)actions) & 7) || (((uintptr_t)packed) & 15)) return SK_EINVAL;
  if (call_dev && (((uintptr_t)call_dev) & 7)) return SK_EINVAL;
  if (adv && (((uintptr_t)adv) & 7)) return SK_EINVAL;
  if (rows == 0) return SK_OK;
  int dev = 0;
  (void)hipGetDevice(&dev);
  static int cus_of[64] = {0};  // CU count per device, queried once
  if (dev < 0 || dev >= 64) return SK_EINVAL;
  if (!cus_of[dev]) {
    int c = 256;
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    cus_of[dev] = c;
  }
  const int cus = cus_of[dev];
  const bool noise = noise_sd != 0.f;
  const int threads = noise ? threads_for<true>() : threads_for<false>();
  const int64_t tiles = (rows + 31) / 32;
  int64_t grid = (tiles + threads / 64 - 1) / (threads / 64);
  if (grid > cus) grid = cus;  // one workgroup per CU (LDS-limited), 32-row tiles grid-strided
  const size_t lds = (noise ? 2 : 1) * kW2Frag + 1024 * 4;
  static bool attr_set = false;  // dynamic LDS above 64 KiB must be opted into once
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)k_actor_fwd<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * kW2Frag + 1024 * 4);
    (void)hipFuncSetAttribute((const void*)k_actor_fwd<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kW2Frag + 1024 * 4);
    attr_set = true;
  }
  // tile per workgroup when tile-per-wave would leave SIMDs idle
  const bool wg_mode = g_actor_mode == 2 || (g_actor_mode == 0 && tiles < (int64_t)cus * (threads / 64));
  if (wg_mode) {
    static bool wg_attr_set = false;
    if (!wg_attr_set) {
      (void)hipFuncSetAttribute((const void*)k_actor_fwd_wg<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * kW2Frag + 1024 * 4 + kWgExtra);
      (void)hipFuncSetAttribute((const void*)k_actor_fwd_wg<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kW2Frag + 1024 * 4 + kWgExtra);
      wg_attr_set = true;
    }
    const int64_t wgrid = tiles < cus ? tiles : cus;
    if (noise)
      k_actor_fwd_wg<true><<<(unsigned)wgrid, kWgThreads, lds + kWgExtra, (hipStream_t)stream>>>(
          obs, actions, rows, (const char*)packed, noise_sd, seed, call, call_dev, adv, action_sd, grouped);
    else
      k_actor_fwd_wg<false><<<(unsigned)wgrid, kWgThreads, lds + kWgExtra, (hipStream_t)stream>>>(
          obs, actions, rows, (const char*)packed, 0.f, seed, call, call_dev, adv, action_sd, grouped);
    return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
  }
  if (noise) {
    k_actor_fwd<true><<<(unsigned)grid, threads, lds, (hipStream_t)stream>>>(obs, actions, rows, (const char*)packed,
                                                                            noise_sd, seed, call, call_dev, nullptr,
                                                                            adv, action_sd, grouped);
  } else {
    k_actor_fwd<false><<<(unsigned)grid, threads, lds, (hipStream_t)stream>>>(
        obs, actions, rows, (const char*)packed, 0.f, seed, call, call_dev, nullptr, adv, action_sd, grouped);
  }
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_actor_forward(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                     uint64_t seed, uint64_t call, void* stream) {
  return actor_forward(packed, obs, actions, rows, noise_sd, seed, call, nullptr, stream);
}

int sk_actor_forward_dev(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                         uint64_t seed, const uint64_t* call_counter, void* stream) {
  if (!call_counter) return SK_EINVAL;
  return actor_forward(packed, obs, actions, rows, noise_sd, seed, 0, call_counter, stream);
}

int sk_actor_forward_advance(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                             uint64_t seed, uint64_t* call_counter, void* stream) {
  if (!call_counter) return SK_EINVAL;
  if (noise_sd == 0.f) return actor_forward(packed, obs, actions, rows, 0.f, seed, 0, nullptr, stream);
  return actor_forward(packed, obs, actions, rows, noise_sd, seed, 0, nullptr, stream, call_counter);
}

int sk_actor_forward_noise(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                           float action_sd, uint64_t seed, uint64_t* call_counter, void* stream) {
  if (!call_counter || !(action_sd >= 0.f) || !(noise_sd >= 0.f)) return SK_EINVAL;
  if (noise_sd == 0.f && action_sd == 0.f) return actor_forward(packed, obs, actions, rows, 0.f, seed, 0, nullptr, stream);
  return actor_forward(packed, obs, actions, rows, noise_sd, seed, 0, nullptr, stream, call_counter, action_sd, 1);
}

// diagnostics only (not in include/skillshot.h): force the launch mode
// (0 auto, 1 one tile per wave, 2 one tile per workgroup)
int skdiag_actor_set_mode(int mode) {
  if (mode < 0 || mode > 2) return SK_EINVAL;
  g_actor_mode = mode;
  return SK_OK;
}

// diagnostics only (not in include/skillshot.h): the noisy forward with every
// unit's activation dumped to dbg[rows][kDbgCols]
int skdiag_actor_forward_dbg(const void* packed, const float* obs, float* actions, float* dbg, int64_t rows,
                             float noise_sd, uint64_t seed, uint64_t call, void* stream) {
  const int threads = threads_for<true>();
  const int64_t tiles = (rows + 31) / 32;
  int64_t grid = (tiles + threads / 64 - 1) / (threads / 64);
  if (grid > 256) grid = 256;
  const size_t lds = 2 * kW2Frag + 1024 * 4;
  (void)hipFuncSetAttribute((const void*)k_actor_fwd<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  k_actor_fwd<true, true><<<(unsigned)grid, threads, lds, (hipStream_t)stream>>>(
      obs, actions, rows, (const char*)packed, noise_sd, seed, call, nullptr, dbg);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

}  // extern "C"
