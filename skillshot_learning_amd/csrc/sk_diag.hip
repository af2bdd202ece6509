// sk_diag.hip — measurement-only kernels (not part of the drop-in ABI in
// include/skillshot.h): they bound the fused step's per-launch cost from
// below at the same grid and byte traffic.
//   kind 0  empty : same grid as k_step, each lane writes its done byte
//   kind 1  copy  : k_step's exact loads and stores (state planes, actions,
//                   done) with no game logic — the memory + launch floor
#include <hip/hip_runtime.h>
#include <stdint.h>

static constexpr int kDiagBlock = 256;

__global__ void __launch_bounds__(kDiagBlock) kd_empty(uint8_t* done, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * kDiagBlock + threadIdx.x;
  if (i < n) done[i] = 0;
}

__global__ void __launch_bounds__(kDiagBlock) kd_copy(int4* pos, double2* rot, int4* qpos, double2* qrot,
                                                      int4* qcdage, int2* misc, const float2* act, uint8_t* done,
                                                      int64_t n) {
  int64_t i = (int64_t)blockIdx.x * kDiagBlock + threadIdx.x;
  if (i >= n) return;
  int4 p = pos[i];
  double2 r = rot[i];
  int4 q = qpos[i];
  double2 qr = qrot[i];
  int4 ca = qcdage[i];
  int2 m = misc[i];
  float2 a0 = act[i], a1 = act[n + i];
  // data-dependent so nothing is elided; values written back unchanged
  int t = (a0.x > 2.f) + (a1.y > 2.f);
  pos[i] = make_int4(p.x + t, p.y, p.z, p.w);
  rot[i] = r;
  qpos[i] = q;
  qrot[i] = qr;
  qcdage[i] = ca;
  misc[i] = m;
  done[i] = (uint8_t)t;
}

// kind 2 copy_xcc : the same copy, env chunk chosen from the block's physical
//                  XCD (HW_REG_XCC_ID) and its ordinal among blocks b%8 — if
//                  the dispatcher keeps b, b+8, ... on one XCD, every chunk is
//                  touched by the same XCD each launch (speed probe only: the
//                  mapping is placement-dependent, never used in the product)
// kind 3 copy_b8   : chunk from b%8 grouping only (control for kind 2)
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

template <int MODE>
__global__ void __launch_bounds__(kDiagBlock) kd_copy_map(int4* pos, double2* rot, int4* qpos, double2* qrot,
                                                          int4* qcdage, int2* misc, const float2* act,
                                                          uint8_t* done, int64_t n) {
  unsigned G = gridDim.x, b = blockIdx.x;
  unsigned group = MODE == 2 ? xcc_id() : (b & 7);
  unsigned chunk = group * (G / 8) + (b >> 3);
  int64_t i = (int64_t)chunk * kDiagBlock + threadIdx.x;
  if (i >= n) return;
  int4 p = pos[i];
  double2 r = rot[i];
  int4 q = qpos[i];
  double2 qr = qrot[i];
  int4 ca = qcdage[i];
  int2 m = misc[i];
  float2 a0 = act[i], a1 = act[n + i];
  int t = (a0.x > 2.f) + (a1.y > 2.f);
  pos[i] = make_int4(p.x + t, p.y, p.z, p.w);
  rot[i] = r;
  qpos[i] = q;
  qrot[i] = qr;
  qcdage[i] = ca;
  misc[i] = m;
  done[i] = (uint8_t)t;
}

// kind 4 copy_full : the full-contract tick's traffic (k_step_split layout:
//                    lanes 2i, 2i+1 own players 1, 2 of game i, 8-byte plane
//                    halves) — state in/out, action in, obs row 48 B and
//                    reward 4 B out per player, done per game; no game logic.
//                    obs/reward go to `obs` = [2][n][12] f32 followed by
//                    [2][n] f32 (one buffer the caller sizes 104 n bytes)
__global__ void __launch_bounds__(kDiagBlock) kd_copy_full(int2* pos, double* rot, int2* qpos, double* qrot,
                                                           int2* qcdage, int2* misc, const float2* act,
                                                           uint8_t* done, float* obs, int64_t n) {
  const int64_t gt = (int64_t)blockIdx.x * kDiagBlock + threadIdx.x;
  const int64_t i = gt >> 1;
  const int p = (int)(gt & 1);
  if (i >= n) return;
  const int64_t h = 2 * i + p;
  int2 pp = pos[h], qq = qpos[h], ca = qcdage[h];
  double r = rot[h], qr = qrot[h];
  int2 m = misc[i];
  float2 a = act[(int64_t)p * n + i];
  int t = (a.x > 2.f) + (a.y > 2.f);
  pos[h] = make_int2(pp.x + t, pp.y);
  rot[h] = r;
  qpos[h] = qq;
  qrot[h] = qr;
  qcdage[h] = ca;
  if (p == 0) {
    misc[i] = m;
    done[i] = (uint8_t)t;
  }
  float4* o = reinterpret_cast<float4*>(obs + ((int64_t)p * n + i) * 12);
  const float f = (float)pp.x;
  o[0] = make_float4(f, f, f, f);
  o[1] = make_float4(f, f, (float)r, f);
  o[2] = make_float4(f, (float)qr, f, f);
  obs[24 * n + (int64_t)p * n + i] = f;
}

extern "C" int skdiag_launch_full(void* const* planes, const float* actions, uint8_t* done, float* obs, int64_t n,
                                  void* stream) {
  unsigned grid = (unsigned)((2 * n + kDiagBlock - 1) / kDiagBlock);
  kd_copy_full<<<grid, kDiagBlock, 0, (hipStream_t)stream>>>(
      (int2*)planes[0], (double*)planes[1], (int2*)planes[2], (double*)planes[3], (int2*)planes[4],
      (int2*)planes[5], (const float2*)actions, done, obs, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int skdiag_launch(int kind, void* const* planes, const float* actions, uint8_t* done, int64_t n,
                             void* stream) {
  unsigned grid = (unsigned)((n + kDiagBlock - 1) / kDiagBlock);
  if (kind == 0) {
    kd_empty<<<grid, kDiagBlock, 0, (hipStream_t)stream>>>(done, n);
  } else if (kind == 1) {
    kd_copy<<<grid, kDiagBlock, 0, (hipStream_t)stream>>>(
        (int4*)planes[0], (double2*)planes[1], (int4*)planes[2], (double2*)planes[3], (int4*)planes[4],
        (int2*)planes[5], (const float2*)actions, done, n);
  } else if (kind == 2 || kind == 3) {
    if (grid % 8) return -1;
    auto k = kind == 2 ? kd_copy_map<2> : kd_copy_map<3>;
    k<<<grid, kDiagBlock, 0, (hipStream_t)stream>>>(
        (int4*)planes[0], (double2*)planes[1], (int4*)planes[2], (double2*)planes[3], (int4*)planes[4],
        (int2*)planes[5], (const float2*)actions, done, n);
  } else {
    return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
