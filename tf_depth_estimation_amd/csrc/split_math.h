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


// ---------------------------------------------------------------- fp16x3 (conv math 4)
// Two-way fp16 split of a SCALED fp32 value x*s: hi = fp16_rne(x*s), lo = fp16_rne(x*s - hi).  hi carries
// 11 significant bits, the exact remainder is rounded to another 11, so |x*s - hi - lo| <= 2^-22 |x*s| while
// lo is a normal fp16 (|x*s| >= 2^-3), and <= 2^-25 absolute below that (fp16 subnormal half-quantum).  The
// product keeps hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_f16 (fp32 accumulation): the dropped lo*lo
// and the two split residuals are <= ~3 * 2^-22 of |x*y| (bf16x6: < 2^-21) at HALF the MFMAs of bf16x6.
// fp16's range (max 65504) is what the power-of-two operand scale s handles: s = 2^(14 - e) puts an
// operand with |x| <= bound (frexp exponent e) below 2^14, so nothing overflows and everything down to
// 2^-16 of the bound keeps the full 22 bits; the accumulator is multiplied by 1/(s_a s_b) (exact).
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

// fixed scale of an operand with no bound: weights (|w| < 256 with full precision down to |w| ~ 5e-4)
constexpr float F16X3_WSCALE = 256.f;

__device__ __forceinline__ float f16x3_scale(const float* bound, float dflt) {
  if (bound == nullptr) return dflt;
  float m = bound[0];   // TDE_BOUND_SLOTS slots (one scalar load), the bound is their max
#pragma unroll
  for (int i = 1; i < TDE_BOUND_SLOTS; ++i) m = fmaxf(m, bound[i]);
  int e;
  (void)frexpf(m, &e);
  e = e < -100 ? -100 : (e > 100 ? 100 : e);   // 2^(14 - e) stays a finite normal float
  return ldexpf(1.f, 14 - e);
}

typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

// hi = fp16_rne(x*s) by pairs (v_pk_mul_f32 + v_cvt_pk_f16_f32), lo = fp16_rne(fma(x, s, -hi)) read from the
// packed hi register by v_fma_mix (op_sel picks the f16 half): 2 VALU instructions per element.  hipcc's own
// lowering of the same arithmetic unpacked hi back to fp32 first (3.25 per element).  Bit-identical: x*s is
// exact (power-of-two s), x*s - hi is exact in fp32, and both forms round that value once to fp16.
__device__ __forceinline__ unsigned f16_lo_pair(float x0, float x1, float s, unsigned hi_pair) {
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %4, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo) : "v"(x0), "v"(s), "v"(hi_pair), "v"(x1));
  return lo;
}

// hi = fp16_rne(x*s) by pairs with v_fma_mix too (fma(x, s, 0): x*s is exact, one rounding to fp16, as
// v_pk_mul_f32 + v_cvt_pk_f16_f32): its fp32 sources are single VGPRs, where v_pk_mul_f32 needs each pair in
// an aligned register pair -- for the transposed staging (a row of 4 k gathered from 4 loaded vectors) hipcc
// spent 2 v_mov per pair building them (32 per 128x128 WGRAD k-tile).  Only the sign of an exact zero can
// differ (-0 * s + 0 = +0), which no fp32 sum of the products can observe.
__device__ __forceinline__ unsigned f16_hi_pair(float x0, float x1, float s) {
  unsigned hi;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %2, 0"
      : "=&v"(hi) : "v"(x0), "v"(s), "v"(x1));
  return hi;
}

#ifndef TDE_F16_MIX_HI
#define TDE_F16_MIX_HI 1
#endif

__device__ __forceinline__ void split4x2h(f4 v, float s, h4& hi, h4& lo) {
#if TDE_F16_MIX_HI
  const h2v a = __builtin_bit_cast(h2v, f16_hi_pair(v[0], v[1], s));
  const h2v b = __builtin_bit_cast(h2v, f16_hi_pair(v[2], v[3], s));
#else
  const h2v a = __builtin_convertvector(f2v{v[0], v[1]} * s, h2v);
  const h2v b = __builtin_convertvector(f2v{v[2], v[3]} * s, h2v);
#endif
  const h2v c = __builtin_bit_cast(h2v, f16_lo_pair(v[0], v[1], s, __builtin_bit_cast(unsigned, a)));
  const h2v d = __builtin_bit_cast(h2v, f16_lo_pair(v[2], v[3], s, __builtin_bit_cast(unsigned, b)));
  hi = h4{a[0], a[1], b[0], b[1]};
  lo = h4{c[0], c[1], d[0], d[1]};
}

// 8 consecutive-k fp32 values (two f4) -> hi / lo fp16x8 fragments
__device__ __forceinline__ void split8x2h(f4 a, f4 b, float s, h8& hi, h8& lo) {
  h4 h0, l0, h1, l1;
  split4x2h(a, s, h0, l0);
  split4x2h(b, s, h1, l1);
  hi = h8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
  lo = h8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
}
