// Device helpers shared by the MFMA conv translation units (conv_igemm.hip, halo_conv.hip).
#pragma once
#include "tde_common.h"

// Division by a runtime constant d >= 1 for 0 <= n < 2^31: q = (umulhi(n, m) + n) >> s with
// s = ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1.  Replaces the ~30-instruction integer division
// in the im2col decode of every k-tile by three instructions.
struct FDiv {
  unsigned m; int s;
};

__host__ __device__ inline FDiv make_fdiv(int d) {
  FDiv f;
  f.s = 0;
  while ((1 << f.s) < d) ++f.s;
  f.m = (unsigned)((((unsigned long long)1 << 32) * (((unsigned long long)1 << f.s) - (unsigned)d)) / (unsigned)d + 1);
  return f;
}

__device__ __forceinline__ int fdiv(int n, FDiv f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s);
}

// Exact three-way bf16 split of an fp32 value (bf16x6 conv math; see conv_igemm.hip for the error
// analysis): x = hi + mid + lo, each part's top 16 bits are a bf16 and its low 16 bits are zero.
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
  const unsigned u = __float_as_uint(x);
  h = u & 0xFFFF0000u;
  const float r = x - __uint_as_float(h);
  m = __float_as_uint(r) & 0xFFFF0000u;
  l = __float_as_uint(r - __uint_as_float(m));
}
__device__ __forceinline__ unsigned pack_hi16(unsigned a, unsigned b) { return (a >> 16) | (b & 0xFFFF0000u); }

__device__ __forceinline__ void split4x3(f4 v, uint2& hi, uint2& mi, uint2& lo) {
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split3(v[j], h[j], m[j], l[j]);
  hi = make_uint2(pack_hi16(h[0], h[1]), pack_hi16(h[2], h[3]));
  mi = make_uint2(pack_hi16(m[0], m[1]), pack_hi16(m[2], m[3]));
  lo = make_uint2(pack_hi16(l[0], l[1]), pack_hi16(l[2], l[3]));
}

