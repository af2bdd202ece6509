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
