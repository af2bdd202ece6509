// sk_split.hpp — the fp32 actor's split pack: its weights as three bf16
// pieces (and the bf16 square for the parameter noise's variance GEMM), in
// the fragment order of v_mfma_f32_32x32x16_bf16, so the acting tile's
// GEMMs run at the bf16 MFMA rate while computing fp32 products.
//
// Split products.  Any fp32 value v is hi + mid + lo with hi = bf16(v),
// mid = bf16(v - hi), lo = bf16(v - hi - mid), each subtraction exact in fp32;
// v - (hi + mid + lo) is below 2^-26 |v| (three round-to-nearest 8-bit pieces
// of a 24-bit significand).  A product x w is then the sum of the nine piece
// products, each exact in the MFMA's fp32 accumulation (8 x 8 significant
// bits); the three whose pieces' orders add to 3 or more (mid lo, lo mid,
// lo lo) are below 2^-26 |x w| and are dropped.  So six bf16 MFMAs give
// every product within ~2^-25 of x w — the accuracy of the fp32 product
// itself (one rounding, 2^-24) — at 6 x 32 = 192 cycles per 16 k against
// the f32 MFMA's 8 x 64 = 512 (MI355X: f32 MFMA 157 TF, bf16 2.5 PF).  The
// sum order differs from an f32 MFMA's, as any GEMM's may; the acting tile
// is held to 1e-5 of the fp64 Keras restatement (tests/test_learn32_gpu.py).
//
// Layout (bytes; written by k_split_pack32 from the flat fp32 parameters and
// by the actor's Adam launch, scatter_split_pack):
//   W1 planes p = 0..3 (hi, mid, lo, bf16(w^2)): [8 n-tiles][64 lanes][8]
//       lane (r, h), element j = W1[32 nt + r][8 h + j] (k >= 12 -> 0)
//   W2 planes p = 0..3: [4 n-tiles][16 k-steps][64 lanes][8]
//       lane (r, h), element j = W2[32 nt + r][16 kk + 8 h + j]
// A lane's 8 elements of a k-step are one 16-byte load; the activations'
// A fragment is the same k order read from row-major LDS rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sksplit {

constexpr int kW1Plane = 8 * 64 * 8;         // bf16 elements per W1 plane
constexpr int kW2Plane = 4 * 16 * 64 * 8;    // per W2 plane
constexpr size_t kOffW1 = 0;
constexpr size_t kOffW2 = kOffW1 + 4 * (size_t)kW1Plane * 2;
constexpr size_t kBytes = kOffW2 + 4 * (size_t)kW2Plane * 2;

__device__ __forceinline__ short bf(float f) { return __builtin_bit_cast(short, (__bf16)f); }
__device__ __forceinline__ float unbf(short s) { return __uint_as_float((uint32_t)(uint16_t)s << 16); }

// v -> (hi, mid, lo) bf16 pieces and bf16(v * v)
__device__ __forceinline__ void split4(float v, short& hi, short& mid, short& lo, short& sq) {
  hi = bf(v);
  const float r1 = v - unbf(hi);
  mid = bf(r1);
  lo = bf(r1 - unbf(mid));
  sq = bf(v * v);
}

// element index (within a plane) of W1[n][k] (k < 12) and W2[o][i]
__device__ __forceinline__ int w1_index(int n, int k) {
  return ((n >> 5) * 64 + (n & 31) + 32 * (k >> 3)) * 8 + (k & 7);
}
__device__ __forceinline__ int w2_index(int o, int i) {
  return (((o >> 5) * 16 + (i >> 4)) * 64 + (o & 31) + 32 * ((i >> 3) & 1)) * 8 + (i & 7);
}

// the pack entries of flat actor parameter p (torch parameters() order:
// W1 [256][12], b1, W2 [128][256], ...) holding value w; other parameters
// (biases, W3) are read from the flat vector by the kernels
__device__ __forceinline__ void scatter_split_pack(char* out, int p, float w) {
  constexpr int kPB1 = 256 * 12, kPW2 = kPB1 + 256, kPB2 = kPW2 + 128 * 256;
  int idx, plane;
  short* base;
  if (p < kPB1) {
    idx = w1_index(p / 12, p % 12);
    plane = kW1Plane;
    base = (short*)(out + kOffW1);
  } else if (p >= kPW2 && p < kPB2) {
    const int q = p - kPW2;
    idx = w2_index(q >> 8, q & 255);
    plane = kW2Plane;
    base = (short*)(out + kOffW2);
  } else {
    return;
  }
  short hi, mid, lo, sq;
  split4(w, hi, mid, lo, sq);
  base[idx] = hi;
  base[plane + idx] = mid;
  base[2 * plane + idx] = lo;
  base[3 * plane + idx] = sq;
}

}  // namespace sksplit
