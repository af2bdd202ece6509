// sk_xchg.hpp — in-launch exchanges among the workgroups of one persistent
// launch (the resident models_fit kernels, csrc/sk_fit.hip; the seam
// microbenchmark, tools/seam_bench.hip).
//
// Data-tagged granules (MI355X_MICROARCH.md "handoff-1to1", cdna_hip_
// programming.md Guideline 16, R2): every value travels as one naturally
// aligned 8-byte {value, tag} word written by ONE agent-scope relaxed store
// (global_store_dwordx2 sc1: write-through, so no release fence), and the
// consumer re-reads its granules with agent-scope relaxed loads (sc1: past
// the CU's L1) until every tag equals the phase's epoch.  The data IS the
// flag: no separate flag store, no acquire fence, no ordering between the
// granules.  Tags are epochs counted on device across launches (never a
// launch argument, which a replayed graph would freeze), so a slot still
// holding an earlier phase's granule never matches.
//
// Every wait is bounded: a spin that runs out sets *timeout (the host reads
// it after the launch and fails loudly) and the caller leaves the phase with
// whatever it holds, so a lost producer cannot hang the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace skx {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ gu64* g64(void* p) { return (gu64*)p; }

__device__ __forceinline__ void put(gu64* slot, unsigned epoch, float v) {
  __hip_atomic_store(slot, ((unsigned long long)epoch << 32) | (unsigned long long)__float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long peek(gu64* slot) {
  return __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned kSpinLimit = 1u << 22;  // ~4 s of polling: a lost producer, not a slow one

// N granules per lane at slots[k * stride] (k < N), re-read until every tag
// of the WAVE's granules is `epoch`; values into v.  Returns false (and sets
// *timeout) when the spin limit runs out.
template <int N>
__device__ __forceinline__ bool gather(gu64* slots, int stride, unsigned epoch, float (&v)[N], unsigned* timeout) {
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const unsigned long long x = peek(slots + (size_t)k * stride);
      v[k] = __uint_as_float((unsigned)x);
      ok &= (unsigned)(x >> 32) == epoch;
    }
    if (__all(ok)) return true;
    if (spins >= kSpinLimit) {
      if ((threadIdx.x & 63) == 0) atomicMax(timeout, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace skx
