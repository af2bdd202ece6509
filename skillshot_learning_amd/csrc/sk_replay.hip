// sk_replay.hip — the learner's HBM replay ring on device (F1; SURVEY §8(d)
// config 3: "replay buffer in HBM, capacity 1M transitions, 112 B each"):
// the insert of a tick's 2N transitions and the minibatch gather, one launch
// each, with the ring position on device so a captured hipGraph replays them
// (replaces ~16 small torch kernels per tick: cat, remainder, index_copy_,
// head/size arithmetic, rand/mul/long/minimum/index, contiguous copies).
//
// Ring: float[cap][28] rows (s 12, a 2, r 1, s' 12, done 1 = 112 B,
// learner.ReplayRing.WIDTH); total (int64, device) counts the rows ever
// inserted: head = total % cap, size = min(total, cap).
//   k_replay_insert  tick row r (player r / N of game r % N: the actor's
//                    [2N] order) -> ring row (total + r) % cap; the last
//                    workgroup to finish advances total (every workgroup
//                    read total before it signalled, so none reads the new
//                    value)
//   k_replay_sample  batch row b -> ring row floor(u_b * size), u_b from
//                    Philox4x32-10 keyed (seed; b, draw, total), gathered
//                    into contiguous s / a / r / s' / d
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_mlp.hpp"

namespace {

constexpr int kW = 28;  // floats per ring row
constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) k_replay_insert(float* __restrict__ ring, int64_t cap,
                                                            int64_t* __restrict__ total, unsigned* __restrict__ arrivals,
                                                            const float* __restrict__ obs, const float* __restrict__ act,
                                                            const float* __restrict__ rew,
                                                            const float* __restrict__ obs2,
                                                            const uint8_t* __restrict__ done, int64_t n_games,
                                                            int64_t rows) {
  __shared__ int64_t s_base;
  if (threadIdx.x == 0) s_base = *total;
  __syncthreads();
  const int64_t base = s_base;
  const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r < rows) {
    const float4* o = (const float4*)(obs + r * 12);
    const float4* o2 = (const float4*)(obs2 + r * 12);
    const float4 s0 = o[0], s1 = o[1], s2 = o[2];
    const float4 t0 = o2[0], t1 = o2[1], t2 = o2[2];
    const float2 a = *(const float2*)(act + r * 2);
    const float rr = rew[r];
    const float d = (float)done[r % n_games];
    float4* dst = (float4*)(ring + ((base + r) % cap) * kW);
    dst[0] = s0;
    dst[1] = s1;
    dst[2] = s2;
    dst[3] = make_float4(a.x, a.y, rr, t0.x);
    dst[4] = make_float4(t0.y, t0.z, t0.w, t1.x);
    dst[5] = make_float4(t1.y, t1.z, t1.w, t2.x);
    dst[6] = make_float4(t2.y, t2.z, t2.w, d);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(arrivals, 1u);
    if (prev == gridDim.x - 1) {  // the last workgroup: every other one has read total
      *total = base + rows;
      *arrivals = 0u;
    }
  }
}

__global__ void __launch_bounds__(kThreads) k_replay_sample(const float* __restrict__ ring, int64_t cap,
                                                            const int64_t* __restrict__ total, uint64_t seed,
                                                            int draw, int64_t batch, float* __restrict__ s,
                                                            float* __restrict__ a, float* __restrict__ r,
                                                            float* __restrict__ s2, float* __restrict__ d,
                                                            int64_t excl) {
  const int64_t t = *total;
  const uint64_t size = (uint64_t)(t < cap ? t : cap);
  const int64_t b = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (b >= batch || size == 0) return;
  // floor(u * size), or with excl the rows skmlp::ring_row draws (sk_mlp.hpp)
  const skmlp::RingSample q{ring, cap, total, seed, draw, s, a, r, s2, d, excl};
  const int64_t idx = skmlp::ring_row(q, b, t);
  const float4* src = (const float4*)(ring + idx * kW);
  float4 v[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) v[k] = src[k];
  float4* so = (float4*)(s + b * 12);
  so[0] = v[0];
  so[1] = v[1];
  so[2] = v[2];
  *(float2*)(a + b * 2) = make_float2(v[3].x, v[3].y);
  r[b] = v[3].z;
  float4* s2o = (float4*)(s2 + b * 12);
  s2o[0] = make_float4(v[3].w, v[4].x, v[4].y, v[4].z);
  s2o[1] = make_float4(v[4].w, v[5].x, v[5].y, v[5].z);
  s2o[2] = make_float4(v[5].w, v[6].x, v[6].y, v[6].z);
  d[b] = v[6].w;
}

// Insert and sample in ONE launch (the learner tick's two consecutive ring
// launches): workgroups [0, gi) insert as k_replay_insert, [gi, gi + gs)
// sample as k_replay_sample would AFTER the insert, with the same Philox key
// (total after the insert) and range.  A sampled ring row that this launch is
// writing is read from the insert's sources instead (the same floats the
// insert stores), every other row from the ring, which this launch does not
// touch there; so no workgroup waits for another.  Every workgroup reads
// total first and signals its arrival last; the last to arrive advances it.
__global__ void __launch_bounds__(kThreads) k_replay_insert_sample(
    float* __restrict__ ring, int64_t cap, int64_t* __restrict__ total, unsigned* __restrict__ arrivals,
    const float* __restrict__ obs, const float* __restrict__ act, const float* __restrict__ rew,
    const float* __restrict__ obs2, const uint8_t* __restrict__ done, int64_t n_games, int64_t rows, unsigned gi,
    uint64_t seed, int draw, int64_t batch, float* __restrict__ s, float* __restrict__ a, float* __restrict__ r,
    float* __restrict__ s2, float* __restrict__ d) {
  __shared__ int64_t s_base;
  if (threadIdx.x == 0) s_base = *total;
  __syncthreads();
  const int64_t base = s_base;
  if (blockIdx.x < gi) {
    const int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (q < rows) {
      const float4* o = (const float4*)(obs + q * 12);
      const float4* o2 = (const float4*)(obs2 + q * 12);
      const float4 s0 = o[0], s1 = o[1], s2v = o[2];
      const float4 t0 = o2[0], t1 = o2[1], t2 = o2[2];
      const float2 av = *(const float2*)(act + q * 2);
      const float rr = rew[q];
      const float dv = (float)done[q % n_games];
      float4* dst = (float4*)(ring + ((base + q) % cap) * kW);
      dst[0] = s0;
      dst[1] = s1;
      dst[2] = s2v;
      dst[3] = make_float4(av.x, av.y, rr, t0.x);
      dst[4] = make_float4(t0.y, t0.z, t0.w, t1.x);
      dst[5] = make_float4(t1.y, t1.z, t1.w, t2.x);
      dst[6] = make_float4(t2.y, t2.z, t2.w, dv);
    }
  } else {
    const int64_t t = base + rows;  // total after the insert: k_replay_sample's key and range
    const uint64_t size = (uint64_t)(t < cap ? t : cap);
    const int64_t b = (int64_t)(blockIdx.x - gi) * kThreads + threadIdx.x;
    if (b < batch) {
      const uint4 u = skmlp::philox(make_uint4((uint32_t)b, (uint32_t)draw, (uint32_t)t, (uint32_t)(t >> 32)),
                                    (uint32_t)seed, (uint32_t)(seed >> 32));
      const uint64_t u53 = (((uint64_t)u.x << 32) | u.y) >> 11;
      const int64_t idx = (int64_t)(((unsigned __int128)u53 * size) >> 53);
      const int64_t off = ((idx - base % cap) % cap + cap) % cap;  // its tick row if written now
      float4 v[7];
      if (off < rows) {
        const float4* o = (const float4*)(obs + off * 12);
        const float4* o2 = (const float4*)(obs2 + off * 12);
        const float4 t0 = o2[0], t1 = o2[1], t2 = o2[2];
        const float2 av = *(const float2*)(act + off * 2);
        v[0] = o[0];
        v[1] = o[1];
        v[2] = o[2];
        v[3] = make_float4(av.x, av.y, rew[off], t0.x);
        v[4] = make_float4(t0.y, t0.z, t0.w, t1.x);
        v[5] = make_float4(t1.y, t1.z, t1.w, t2.x);
        v[6] = make_float4(t2.y, t2.z, t2.w, (float)done[off % n_games]);
      } else {
        const float4* src = (const float4*)(ring + idx * kW);
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = src[k];
      }
      float4* so = (float4*)(s + b * 12);
      so[0] = v[0];
      so[1] = v[1];
      so[2] = v[2];
      *(float2*)(a + b * 2) = make_float2(v[3].x, v[3].y);
      r[b] = v[3].z;
      float4* s2o = (float4*)(s2 + b * 12);
      s2o[0] = make_float4(v[3].w, v[4].x, v[4].y, v[4].z);
      s2o[1] = make_float4(v[4].w, v[5].x, v[5].y, v[5].z);
      s2o[2] = make_float4(v[5].w, v[6].x, v[6].y, v[6].z);
      d[b] = v[6].w;
    }
  }
  __syncthreads();
  // grouped arrival (arrivals = uint32[SK_REPLAY_ARRIVAL_WORDS]): workgroup b
  // on group line arrivals[32 (1 + b % 8)], the last of each group on
  // arrivals[0]; 500+ workgroups on one address serialise for microseconds
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned members = (gridDim.x - g + 7u) / 8u;
    unsigned* gc = arrivals + 32u * (1u + g);
    if (atomicAdd(gc, 1u) == members - 1u) {
      *gc = 0u;
      const unsigned groups = gridDim.x < 8u ? gridDim.x : 8u;
      if (atomicAdd(arrivals, 1u) == groups - 1u) {  // the last workgroup: every other one has read total
        *total = base + rows;
        *arrivals = 0u;
      }
    }
  }
}

}  // namespace

extern "C" {

int sk_replay_insert(float* ring, int64_t capacity, int64_t* total, uint32_t* arrivals, const float* obs,
                     const float* actions, const float* rewards, const float* next_obs, const uint8_t* done,
                     int64_t n_games, int64_t rows, void* stream) {
  if (!ring || !total || !arrivals || !obs || !actions || !rewards || !next_obs || !done) return SK_EINVAL;
  if (capacity <= 0 || rows <= 0 || n_games <= 0 || rows > capacity) return SK_EINVAL;
  if ((((uintptr_t)ring) & 15) || (((uintptr_t)obs) & 15) || (((uintptr_t)next_obs) & 15) ||
      (((uintptr_t)actions) & 7) || (((uintptr_t)total) & 7))
    return SK_EINVAL;
  const unsigned grid = (unsigned)((rows + kThreads - 1) / kThreads);
  k_replay_insert<<<grid, kThreads, 0, (hipStream_t)stream>>>(ring, capacity, total, arrivals, obs, actions, rewards,
                                                              next_obs, done, n_games, rows);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_replay_sample(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                     int64_t batch, float* s, float* a, float* r, float* s2, float* d, void* stream) {
  return sk_replay_sample_excl(ring, capacity, total, seed, draw, batch, s, a, r, s2, d, 0, stream);
}

int sk_replay_sample_excl(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                          int64_t batch, float* s, float* a, float* r, float* s2, float* d, int64_t exclude,
                          void* stream) {
  if (!ring || !total || !s || !a || !r || !s2 || !d || capacity <= 0 || batch <= 0) return SK_EINVAL;
  if (exclude < 0 || exclude >= capacity) return SK_EINVAL;
  if ((((uintptr_t)ring) & 15) || (((uintptr_t)s) & 15) || (((uintptr_t)s2) & 15) || (((uintptr_t)a) & 7))
    return SK_EINVAL;
  const unsigned grid = (unsigned)((batch + kThreads - 1) / kThreads);
  k_replay_sample<<<grid, kThreads, 0, (hipStream_t)stream>>>(ring, capacity, total, seed, draw, batch, s, a, r, s2,
                                                              d, exclude);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

int sk_replay_insert_sample(float* ring, int64_t capacity, int64_t* total, uint32_t* arrivals, const float* obs,
                            const float* actions, const float* rewards, const float* next_obs, const uint8_t* done,
                            int64_t n_games, int64_t rows, uint64_t seed, int32_t draw, int64_t batch, float* s,
                            float* a, float* r, float* s2, float* d, void* stream) {
  if (!ring || !total || !arrivals || !obs || !actions || !rewards || !next_obs || !done) return SK_EINVAL;
  if (!s || !a || !r || !s2 || !d || batch <= 0) return SK_EINVAL;
  if (capacity <= 0 || rows <= 0 || n_games <= 0 || rows > capacity) return SK_EINVAL;
  if ((((uintptr_t)ring) & 15) || (((uintptr_t)obs) & 15) || (((uintptr_t)next_obs) & 15) ||
      (((uintptr_t)actions) & 7) || (((uintptr_t)total) & 7) || (((uintptr_t)s) & 15) || (((uintptr_t)s2) & 15) ||
      (((uintptr_t)a) & 7))
    return SK_EINVAL;
  const unsigned gi = (unsigned)((rows + kThreads - 1) / kThreads);
  const unsigned gs = (unsigned)((batch + kThreads - 1) / kThreads);
  k_replay_insert_sample<<<gi + gs, kThreads, 0, (hipStream_t)stream>>>(ring, capacity, total, arrivals, obs, actions,
                                                                       rewards, next_obs, done, n_games, rows, gi,
                                                                       seed, draw, batch, s, a, r, s2, d);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}

}  // extern "C"

// sk_replay_sample with the ring_row exclusion (sk_critic_grad_f32_sampled's
// unsliced batches)
int replay_sample_excl(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                       int64_t batch, float* s, float* a, float* r, float* s2, float* d, int64_t excl,
                       hipStream_t stream) {
  if (!ring || !total || !s || !a || !r || !s2 || !d || capacity <= 0 || batch <= 0 || excl < 0 || excl >= capacity)
    return SK_EINVAL;
  const unsigned grid = (unsigned)((batch + kThreads - 1) / kThreads);
  k_replay_sample<<<grid, kThreads, 0, stream>>>(ring, capacity, total, seed, draw, batch, s, a, r, s2, d, excl);
  return hipGetLastError() == hipSuccess ? SK_OK : SK_EHIP;
}
