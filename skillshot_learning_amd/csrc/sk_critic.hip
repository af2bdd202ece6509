// sk_critic.hip — fused critic-Q forward on MFMA (gfx950), alone and fused
// behind the actor as the DDPG bootstrap target Q'(s, mu'(s)).
//
// The critic of model_define_critic (SkillshotLearner.py:98-121):
//     h1 = Dropout(relu(W1 s + b1))            12 -> 256   (Dropout is the
//                                                identity at inference)
//     h2 = relu(W2 [h1; a] + b2)              258 -> 128
//     q  = W3 h2 + b3                          128 -> 1
// Same transposed layout as the actor (sk_actor.hip, sk_mlp.hpp): the batch
// row on the lane, hidden units in the 16 accumulator registers of a
// v_mfma_f32_32x32x16_bf16 tile, each layer's accumulator converted in
// registers to the next layer's B operand.  W2's first 256 input columns run
// on MFMA (bf16 operands, fp32 accumulate); its two action columns are a
// rank-2 fp32 update in the layer-2 epilogue (each lane holds its row's
// action), and layer 3 is an fp32 VALU dot product combined across the two
// lane halves with one __shfl_xor.
//
// k_target_q runs the (target) actor and then the (target) critic on the same
// 32-row tile in one launch: the DDPG bootstrap term Q'(s', mu'(s')) with no
// intermediate in memory.  Its actor half is the same instruction sequence as
// k_actor_fwd<false>, so its actions equal the actor kernel's bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"

namespace {

using namespace skmlp;

constexpr int kCIn2 = kH1 + 2;  // critic layer-2 inputs: h1 then the action

// critic packed buffer layout (bytes)
constexpr size_t kCOffW1 = 0;
constexpr size_t kCOffW2 = kCOffW1 + kW1Frag;
constexpr size_t kCOffB = kCOffW2 + kW2Frag;    // fp32: b1[256] b2[128] b3[1] (pad 512)
constexpr size_t kCOffW2a = kCOffB + 512 * 4;   // fp32: W2[u][256 + j] as [128][2]
constexpr size_t kCOffW3 = kCOffW2a + 256 * 4;  // fp32: W3[128] (pad 256)
constexpr size_t kCPackedBytes = kCOffW3 + 256 * 4;
constexpr int kCThreads = 512;  // 8 waves, one 32-row tile each

__global__ void k_critic_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                              const float* b3, char* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 8 * 64) {
    short* w1 = (short*)(out + kCOffW1);
    const int c = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * h + j;
      w1[t * 8 + j] = f2bf(k < kIn ? W1[(32 * c + r) * kIn + k] : 0.f);
    }
  } else if (t < 8 * 64 + 64 * 64) {
    short* w2 = (short*)(out + kCOffW2);
    const int u = t - 8 * 64;
    const int frag = u >> 6, lane = u & 63, r = lane & 31, h = lane >> 5;
    const int tt = frag >> 4, kk = frag & 15;
    for (int j = 0; j < 8; ++j) w2[u * 8 + j] = f2bf(W2[(32 * tt + r) * kCIn2 + w2_k(kk, h, j)]);
  } else if (t < 8 * 64 + 64 * 64 + 512) {
    const int u = t - 8 * 64 - 64 * 64;
    float v = 0.f;
    if (u < kH1) v = b1[u];
    else if (u < kH1 + kH2) v = b2[u - kH1];
    else if (u == kH1 + kH2) v = b3[0];
    ((float*)(out + kCOffB))[u] = v;
  } else if (t < 8 * 64 + 64 * 64 + 512 + 256) {
    const int u = t - 8 * 64 - 64 * 64 - 512;  // unit * 2 + j
    ((float*)(out + kCOffW2a))[u] = W2[(u >> 1) * kCIn2 + kH1 + (u & 1)];
  } else if (t < 8 * 64 + 64 * 64 + 512 + 256 + 256) {
    const int u = t - 8 * 64 - 64 * 64 - 512 - 256;
    ((float*)(out + kCOffW3))[u] = u < kH2 ? W3[u] : 0.f;
  }
}
constexpr int kCPackThreads = 8 * 64 + 64 * 64 + 512 + 256 + 256;

// stage 64 KiB of layer-2 fragments + 1024 fp32 (biases and the fp32 tail)
// from a packed buffer into LDS
__device__ __forceinline__ void stage(const char* packed, size_t off_w2, size_t off_tail, char* s_w2, float* s_tail) {
  const uint4* g = (const uint4*)(packed + off_w2);
  uint4* s = (uint4*)s_w2;
  for (int k = threadIdx.x; k < kW2Frag / 16; k += blockDim.x) s[k] = g[k];
  const float* gb = (const float*)(packed + off_tail);
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) s_tail[k] = gb[k];
}

// X^T fragment of a 32-row tile: lane (r, h) holds X[row][8h .. 8h+7] (k >= 12 -> 0)
__device__ __forceinline__ bf16x8 x_fragment(const float* X, int64_t row, bool valid, int h) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = 0.f;
  if (valid) {
    const float* xr = X + row * kIn + 8 * h;
    const float4 a = *(const float4*)xr;
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    if (h == 0) {
      const float4 b = *(const float4*)(xr + 4);
      x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    }
  }
  bf16x8 xb;
#pragma unroll
  for (int j = 0; j < 8; ++j) xb[j] = f2bf(x[j]);
  return xb;
}

// layer 1 (12 -> 256, relu) into 16 bf16 B fragments of layer 2.  Epilogue
// operands are read from per-lane-half bases (+4h folded in once) so every
// LDS read is base + immediate.
__device__ __forceinline__ void layer1(const bf16x8* gW1, const float* sb1, bf16x8 xb, int lane, int h,
                                       bf16x8 h1[16]) {
  const float* b1h = sb1 + 4 * h;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    f32x16 acc = {0};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gW1[c * 64 + lane], xb, acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * s + j;
        f[j] = f2bf(fmaxf(acc[i] + b1h[32 * c + (i & 3) + 8 * (i >> 2)], 0.f));
      }
      h1[2 * c + s] = f;
    }
    __builtin_amdgcn_sched_barrier(0);  // one chunk's accumulators live at a time
  }
}

// the critic's q for this lane's row, given the layer-1 fragments and the action
__device__ __forceinline__ float critic_q(const bf16x8* sW2, const float* sb, const float* sW2a, const float* sW3,
                                          const bf16x8 h1[16], float a0, float a1, int lane, int h) {
  const float* b2h = sb + kH1 + 4 * h;
  const float* w2ah = sW2a + 8 * h;
  const float* w3h = sW3 + 4 * h;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 acc = {0};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sW2[(t * 16 + kk) * 64 + lane], h1[kk], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int u = 32 * t + (i & 3) + 8 * (i >> 2);  // hidden unit - 4h
      float y = acc[i] + b2h[u];
      y += w2ah[2 * u] * a0 + w2ah[2 * u + 1] * a1;
      q += w3h[u] * fmaxf(y, 0.f);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return q + __shfl_xor(q, 32, 64) + sb[kH1 + kH2];
}

// Q(s, a) for given actions
__global__ void __launch_bounds__(kCThreads) k_critic_fwd(const float* __restrict__ S, const float* __restrict__ A,
                                                          float* __restrict__ Q, int64_t M,
                                                          const char* __restrict__ packed) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sTail = (float*)(smem + kW2Frag);
  stage(packed, kCOffW2, kCOffB, smem, sTail);
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (M + 31) / 32;
  const int64_t wave = (int64_t)blockIdx.x * (kCThreads / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kCThreads / 64);
  for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
    // launder the weight bases each tile: otherwise LICM hoists the W1
    // fragment loads and the ~256 fp32 LDS operands of the epilogues out of
    // the tile loop and spills them
    const char* pk = packed;
    int toff = 0;
    asm volatile("" : "+s"(pk), "+v"(toff));
    const bf16x8* sW2 = (const bf16x8*)smem + toff;
    const float* sb = sTail + toff;
    const float* sW2a = sTail + 512 + toff;
    const float* sW3 = sTail + 768 + toff;
    const int64_t row = tile * 32 + r;
    const bool valid = row < M;
    float a0 = 0.f, a1 = 0.f;
    if (valid) {
      const float2 a = *(const float2*)(A + row * 2);
      a0 = a.x;
      a1 = a.y;
    }
    bf16x8 h1[16];
    layer1((const bf16x8*)(pk + kCOffW1), sb, x_fragment(S, row, valid, h), lane, h, h1);
    const float q = critic_q(sW2, sb, sW2a, sW3, h1, a0, a1, lane, h);
    if (h == 0 && valid) Q[row] = q;
  }
}

// Q'(s, mu'(s)): the actor then the critic on the same tile
// With R given, Q receives the bootstrapped target R + gamma (1 - D) Q'
// (DDPG.replay_update) instead of Q'.
__global__ void __launch_bounds__(kCThreads) k_target_q(const float* __restrict__ S, float* __restrict__ Q,
                                                        float* __restrict__ A_out, int64_t M,
                                                        const char* __restrict__ apacked,
                                                        const char* __restrict__ cpacked, const float* __restrict__ R,
                                                        const float* __restrict__ D, float gamma) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sAW2 = smem;
  float* sATail = (float*)(smem + kW2Frag);            // actor b1 b2 b3 (512), W3 (256), W3^2 (256)
  char* sCW2 = smem + kW2Frag + 1024 * 4;
  float* sCTail = (float*)(sCW2 + kW2Frag);            // critic b (512), W2a (256), W3 (256)
  stage(apacked, kOffW2, kOffB, sAW2, sATail);
  stage(cpacked, kCOffW2, kCOffB, sCW2, sCTail);
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (M + 31) / 32;
  const int64_t wave = (int64_t)blockIdx.x * (kCThreads / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kCThreads / 64);
  for (int64_t tile = wave; tile < ntiles; tile += nwaves) {
    const char* ap = apacked;
    const char* cp = cpacked;
    int toff = 0;
    asm volatile("" : "+s"(ap), "+s"(cp), "+v"(toff));
    const int64_t row = tile * 32 + r;
    const bool valid = row < M;
    const bf16x8 xb = x_fragment(S, row, valid, h);
    bf16x8 h1[16];
    // ---- actor mu'(s): as k_actor_fwd<false>
    layer1((const bf16x8*)(ap + kOffW1), sATail + toff, xb, lane, h, h1);
    const bf16x8* aW2 = (const bf16x8*)sAW2;
    const float* ab2h = sATail + toff + kH1 + 4 * h;
    const float* aw3h = sATail + toff + 512 + 4 * h;
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 acc = {0};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aW2[(t * 16 + kk) * 64 + lane], h1[kk], acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int u = 32 * t + (i & 3) + 8 * (i >> 2);  // hidden unit - 4h
        const float y = fmaxf(acc[i] + ab2h[u], 0.f);
        m0 = __builtin_fmaf(aw3h[u], y, m0);  // the actor kernel's layer-3 order (sk_actor.hip): same bits
        m1 = __builtin_fmaf(aw3h[kH2 + u], y, m1);
      }
    }
    m0 += __shfl_xor(m0, 32, 64);
    m1 += __shfl_xor(m1, 32, 64);
    const float a0 = tanhf(m0 + sATail[toff + kH1 + kH2]);
    const float a1 = tanhf(m1 + sATail[toff + kH1 + kH2 + 1]);
    if (A_out && h == 0 && valid) *(float2*)(A_out + row * 2) = make_float2(a0, a1);
    // ---- critic Q'(s, a)
    layer1((const bf16x8*)(cp + kCOffW1), sCTail + toff, xb, lane, h, h1);
    const float q = critic_q((const bf16x8*)sCW2, sCTail + toff, sCTail + toff + 512, sCTail + toff + 768, h1, a0,
                             a1, lane, h);
    if (h == 0 && valid) Q[row] = R ? R[row] + gamma * (1.f - D[row]) * q : q;
  }
}

int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int c = 256;
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    cus[dev] = c;
  }
  return cus[dev];
}

int64_t grid_for(int64_t rows) {
  const int64_t tiles = (rows + 31) / 32;
  int64_t g = (tiles + kCThreads / 64 - 1) / (kCThreads / 64);
  const int64_t cus = cu_count();
  return g > cus ? cus : g;  // one workgroup per CU (LDS-limited), tiles grid-strided
}

}  // namespace

extern "C" {

size_t sk_critic_packed_bytes(void) { return kCPackedBytes; }

int sk_critic_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                   const float* b3, void* packed, void* stream) {
  if (!W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !packed) return SK_EINVAL;
  if (((uintptr_t)packed) & 15) return SK_EINVAL;
  k_critic_pack<<<(kCPackThreads + 255) / 256, 256, 0, (hipStream_t)stream>>>(W1, b1, W2, b2, W3, b3,
                                                                                (char*)packed);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_critic_forward(const void* packed, const float* obs, const float* actions, float* q, int64_t rows,
                      void* stream) {
  if (!packed || !obs || !actions || !q || rows < 0) return SK_EINVAL;
  if ((((uintptr_t)obs) & 15) || (((uintptr_t)actions) & 7) || (((uintptr_t)packed) & 15)) return SK_EINVAL;
  if (rows == 0) return SK_OK;
  const size_t lds = kW2Frag + 1024 * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_critic_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  k_critic_fwd<<<(unsigned)grid_for(rows), kCThreads, lds, (hipStream_t)stream>>>(obs, actions, q, rows,
                                                                                  (const char*)packed);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_target_q(const void* actor_packed, const void* critic_packed, const float* obs, float* q, float* actions,
                int64_t rows, void* stream) {
  if (!actor_packed || !critic_packed || !obs || !q || rows < 0) return SK_EINVAL;
  if ((((uintptr_t)obs) & 15) || (((uintptr_t)actor_packed) & 15) || (((uintptr_t)critic_packed) & 15) ||
      (actions && (((uintptr_t)actions) & 7)))
    return SK_EINVAL;
  if (rows == 0) return SK_OK;
  const size_t lds = 2 * (kW2Frag + 1024 * 4);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_target_q, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  k_target_q<<<(unsigned)grid_for(rows), kCThreads, lds, (hipStream_t)stream>>>(
      obs, q, actions, rows, (const char*)actor_packed, (const char*)critic_packed, nullptr, nullptr, 0.f);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_target_y(const void* actor_packed, const void* critic_packed, const float* next_obs, const float* rewards,
                const float* done, float gamma, float* y, int64_t rows, void* stream) {
  if (!actor_packed || !critic_packed || !next_obs || !rewards || !done || !y || rows < 0) return SK_EINVAL;
  if ((((uintptr_t)next_obs) & 15) || (((uintptr_t)actor_packed) & 15) || (((uintptr_t)critic_packed) & 15))
    return SK_EINVAL;
  if (rows == 0) return SK_OK;
  const size_t lds = 2 * (kW2Frag + 1024 * 4);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_target_q, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  k_target_q<<<(unsigned)grid_for(rows), kCThreads, lds, (hipStream_t)stream>>>(
      next_obs, y, nullptr, rows, (const char*)actor_packed, (const char*)critic_packed, rewards, done, gamma);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

}  // extern "C"
