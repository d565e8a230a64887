// MFMA implicit-GEMM convolution for gfx950 (fp32 in, fp32 accumulate, exact fp32 MFMA).
//
// Replaces TF's Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter as emitted by slim.conv2d and
// slim.conv2d_transpose in nets_optflow_depth.py:88-144, nets_depth.py:88-191 (SURVEY.md §8a rows a1,a2).
// One kernel template, three operand-gather modes over the *virtual forward conv*
//   y[n,oh,ow,k] = sum_{kh,kw,c} x[n, oh*S-PT+kh, ow*S-PL+kw, c] * w[kh,kw,c,k]:
//   FWD  : C[m=(n,oh,ow)][k]      = sum_{(kh,kw,c)}  x(...) w            (conv fwd, deconv bwd-data)
//   DGRAD: C[m=(n,ih,iw)][c]      = sum_{(th,tw,k)}  dy(...) w           (conv bwd-data, deconv fwd)
//          stride-S problems split into S*S output-parity classes, each a dense stride-1 GEMM
//          over only the taps that hit it (sub-pixel decomposition, no zero-insertion).
//   WGRAD: C[m=(kh,kw,c)][k]      = sum_{pixels}     x(...) dy           (conv/deconv bwd-filter)
// Tiles: BM x BN x 32 per 256-thread block (4 waves), each wave TM x TN 16x16 accumulators.  Both
// operands live m-major in a double-buffered LDS image ([row][k], padded rows); an operand whose
// 16-byte global vectors run along rows (not k) is transposed in registers (4 rows x 4 k per thread),
// so every global load is a coalesced dwordx4, every LDS store a ds_write_b128 (fp32) and every
// fragment read a ds_read_b128 issued up front for the whole k-tile.  Five math modes (MATH template
// argument, TDE_CONV_MATH / tde_set_conv_math):
//   0 fp32    : 8 v_mfma_f32_16x16x4_f32 per tile pair (exact f32 products, fp32 accumulate);
//   1 bf16x3  : 3 v_mfma_f32_16x16x32_bf16 per tile pair on a hi/lo split of each operand;
//   2 bf16x6  : 6 bf16 MFMAs on an exact hi/mid/lo split, split once at LDS staging;
//   3 bf16x6r : the same products, split per fragment in registers after the LDS read;
//   4 fp16x3  : 3 v_mfma_f32_16x16x32_f16 on a power-of-two-scaled hi/lo fp16 split (the default).
// Split-K partials go to a caller workspace and are reduced by a second kernel (deterministic; no
// float atomics).
#include "tde_common.h"

#include <vector>
#include "bn_internal.h"
#include "split_math.h"
#include "conv_common.h"
using namespace tdeconv;

#include <utility>
#include "halo_conv.h"

#include <cstdlib>

namespace {

// TDE_DBG_PHASE (timing-diagnostic BUILDS only, -DTDE_DBG_PHASE=..., wrong results; never a runtime switch), a
// bit mask: 1 no k-loop global loads, 2 no MFMAs, 4 no staging (split + LDS stores), 8 no B-operand loads or
// staging (its fragments read whatever LDS holds), 16 the same for the A operand.  (Round 3's row-of-4 WGRAD
// decode, XCD-grouped WGRAD order, write-through epilogue stores and software-pipelined two-tile k-loop were
// measured neutral and removed in round 4: DESIGN.md section 6.)
#ifndef TDE_DBG_PHASE
#define TDE_DBG_PHASE 0
#endif
constexpr int NT = 256;


// ------------------------------------------------------------------ bf16x3 split-precision variant
// Same three gather modes, but each fp32 operand element x is split at staging time into
// hi = bf16_rne(x), lo = bf16_rne(x - hi) and the product is formed by three
// v_mfma_f32_16x16x32_bf16 (lo*hi + hi*lo + hi*hi, fp32 accumulate).  The dropped lo*lo term and the
// two roundings leave ~2^-16 relative error per product (vs 2^-24 for fp32) at 16/3 = 5.3x the
// fp32-MFMA rate.  LDS holds hi/lo planes as [row][BK=32 (+8 pad)] bf16; an operand whose 16-byte
// global vectors run along rows is transposed in registers (4 rows x 4 k per thread).
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;
constexpr int BK3 = 32;
// LDS row strides: the 16 lanes of a ds_read_b128 lane group read rows r16 at 16-byte column q; that is
// conflict-free when the row stride in 16-byte units is 2 mod 4 (an odd stride, e.g. 80 or 144 bytes,
// costs 2 LDS cycles per group; halo_conv.hip measured 50% conflict cycles with one)
constexpr int LDR = BK3 + 16;   // 96-byte bf16 plane rows

__device__ __forceinline__ unsigned bf16_rne_bits(float x) {
  const unsigned u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void split4(f4 v, uint2& hi, uint2& lo) {
  unsigned h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = bf16_rne_bits(v[j]);
    l[j] = bf16_rne_bits(v[j] - __uint_as_float(h[j] << 16));
  }
  hi = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  lo = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
}

template <int ROWS>
struct Img3 {
  static constexpr int PLANE = ROWS * LDR;     // u16 elements per plane
  static constexpr int SIZE = 2 * PLANE;       // hi + lo
  __device__ static __forceinline__ void put(u16* s, int row, int k, f4 v) {
    uint2 hi, lo;
    split4(v, hi, lo);
    *reinterpret_cast<uint2*>(s + row * LDR + k) = hi;
    *reinterpret_cast<uint2*>(s + PLANE + row * LDR + k) = lo;
  }
  __device__ static __forceinline__ bf8 hi(const u16* s, int row, int q) {
    return *reinterpret_cast<const bf8*>(s + row * LDR + 8 * q);
  }
  __device__ static __forceinline__ bf8 lo(const u16* s, int row, int q) {
    return *reinterpret_cast<const bf8*>(s + PLANE + row * LDR + 8 * q);
  }
};

// fp32 image: [row][BK3 + 4] floats (144-byte rows), read as f4 = the 4 k of one v_mfma_f32_16x16x4_f32
// lane (MATH 0) or two f4 at k = 4q and 16 + 4q (MATH 3, see compute()).  144 B is an odd 16-byte count
// (2-way conflicts per lane group); the conflict-free 160 B was measured 2% slower per step: it pushes
// the 128x128 double-buffered image to 80 KiB, one workgroup per CU.
constexpr int LDF = BK3 + 4;

template <int ROWS>
struct Img1 {
  using T = float;
  static constexpr int SIZE = ROWS * LDF;
  __device__ static __forceinline__ void put(float* s, int row, int k, f4 v) {
    *reinterpret_cast<f4*>(s + row * LDF + k) = v;
  }
  __device__ static __forceinline__ f4 frag(const float* s, int row, int k) {
    return *reinterpret_cast<const f4*>(s + row * LDF + k);
  }
};

// ------------------------------------------------------------------ bf16x6: fp32-accurate split MFMA
// x = hi + mid + lo EXACTLY for normal fp32 x: hi = x with the low 16 mantissa bits cleared (8
// significant bits), r = x - hi (exact, <= 16 significant bits), mid = r truncated the same way,
// lo = r - mid (exact, <= 8 significant bits, so representable in bf16).  The product keeps the six
// terms of order <= 2^-14 (hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid) on v_mfma_f32_16x16x32_bf16
// with fp32 accumulation; the dropped mid*lo + lo*mid + lo*lo are < 2^-21 of |x*y| (worst case; fp32
// rounding itself is 2^-24 per operation), at 16/6 = 2.7x the fp32-MFMA rate.
// Measured per conv against float64 (tests/diag_conv_err.py): rms error 2.9e-7 of rms(ref) (fp32 MFMA:
// 3.5e-7) with a small negative bias (-4e-8 of rms; fp32 MFMA: ~1e-10).  The bias is the bf16 MFMA's
// accumulation, not the split: a round-to-nearest split (+1 VALU op per level) left it unchanged and cost
// 2% of the step, so the split truncates.
//   MATH 2: split once per element at LDS staging, three bf16 planes in LDS;
//   MATH 3: fp32 LDS image (as MATH 0), split per fragment in registers after the LDS read.
typedef unsigned u4v __attribute__((ext_vector_type(4)));
// 8 consecutive-k fp32 values (two f4) -> hi / mid / lo bf16x8 fragments
__device__ __forceinline__ void split8x3(f4 a, f4 b, bf8& hi, bf8& mi, bf8& lo) {
  uint2 h0, m0, l0, h1, m1, l1;
  split4x3(a, h0, m0, l0);
  split4x3(b, h1, m1, l1);
  hi = __builtin_bit_cast(bf8, u4v{h0.x, h0.y, h1.x, h1.y});
  mi = __builtin_bit_cast(bf8, u4v{m0.x, m0.y, m1.x, m1.y});
  lo = __builtin_bit_cast(bf8, u4v{l0.x, l0.y, l1.x, l1.y});
}

template <int ROWS>
struct Img6 {
  static constexpr int PLANE = ROWS * LDR;
  static constexpr int SIZE = 3 * PLANE;       // hi + mid + lo
  __device__ static __forceinline__ void put(u16* s, int row, int k, f4 v) {
    uint2 hi, mi, lo;
    split4x3(v, hi, mi, lo);
    *reinterpret_cast<uint2*>(s + row * LDR + k) = hi;
    *reinterpret_cast<uint2*>(s + PLANE + row * LDR + k) = mi;
    *reinterpret_cast<uint2*>(s + 2 * PLANE + row * LDR + k) = lo;
  }
  __device__ static __forceinline__ bf8 plane(const u16* s, int pl, int row, int q) {
    return *reinterpret_cast<const bf8*>(s + pl * PLANE + row * LDR + 8 * q);
  }
};

// fp16x3 staged image (MATH 4): each scaled fp32 operand element is split ONCE, at LDS staging, into fp16
// hi / lo planes [row][32 k] (64-byte rows) -- not once per reading wave per k-tile, which made the split's
// VALU work (~3 instructions per element, 2 waves reading every element) the limiter of the whole k-loop
// (313 VALU vs 48 MFMAs per wave per 128x128 k-tile).  Bank mapping for gfx950's lane groups (MI355X_MICROARCH
// LDS table; checked exhaustively for every tile shape, scripts/lds_swizzle_check.py): the four 16-byte
// k-chunks of row r sit at chunk ^ g[(r >> 2) & 3], g = {0, 2, 3, 1}, so each ds_read_b128 group ({0-3,
// 12-15, 20-27}, ... : two k-chunks over 16 rows) hits 16 distinct 4-bank units; and rows r, r ^ 1 trade
// places in odd 16-row blocks, which halves the conflicts of the transposed staging stores (4 rows x 4 k
// per lane: 4-way -> 2-way; plain stores stay conflict-free).  The first layout (chunk ^ (r >> 2) & 3)
// spent 60-67 % of the LDS cycles of the deep-layer GEMMs in conflicts (SQ_LDS_BANK_CONFLICT).
// TDE_F16_STAGE=0 builds the previous register-split variant (fp32 image) for A/B runs.
#ifndef TDE_F16_STAGE
#define TDE_F16_STAGE 1
#endif
template <int ROWS>
struct Img2h {
  static constexpr int PLANE = ROWS * 32;   // u16 elements per plane
  static constexpr int SIZE = 2 * PLANE;    // hi + lo
  __device__ static __forceinline__ int off(int row, int chunk) {
    const int g = (0x1320 >> (4 * ((row >> 2) & 3))) & 3;
    return (row ^ ((row >> 4) & 1)) * 32 + ((chunk ^ g) << 3);
  }
  __device__ static __forceinline__ void put(u16* s, int row, int k, f4 v, float sc) {
    h4 hi, lo;
    split4x2h(v, sc, hi, lo);
    const int o = off(row, k >> 3) + (k & 7);
    *reinterpret_cast<h4*>(s + o) = hi;
    *reinterpret_cast<h4*>(s + PLANE + o) = lo;
  }
  __device__ static __forceinline__ h8 hi(const u16* s, int row, int q) {
    return *reinterpret_cast<const h8*>(s + off(row, q));
  }
  __device__ static __forceinline__ h8 lo(const u16* s, int row, int q) {
    return *reinterpret_cast<const h8*>(s + PLANE + off(row, q));
  }
};

template <int MATH, int ROWS>
struct ImgSel;
template <int ROWS>
struct ImgSel<0, ROWS> { using type = Img1<ROWS>; using T = float; };
template <int ROWS>
struct ImgSel<1, ROWS> { using type = Img3<ROWS>; using T = u16; };
template <int ROWS>
struct ImgSel<2, ROWS> { using type = Img6<ROWS>; using T = u16; };
template <int ROWS>
struct ImgSel<3, ROWS> { using type = Img1<ROWS>; using T = float; };
#if TDE_F16_STAGE
template <int ROWS>
struct ImgSel<4, ROWS> { using type = Img2h<ROWS>; using T = u16; };
#else
template <int ROWS>
struct ImgSel<4, ROWS> { using type = Img1<ROWS>; using T = float; };
#endif

// MATH 0: exact fp32 (2 x 4 v_mfma_f32_16x16x4_f32 per 32-deep k-tile); MATH 1: bf16x3.
template <int MATH, int BM, int BN>
struct SmemSize {
  using IA = typename ImgSel<MATH, BM>::type;
  using IB = typename ImgSel<MATH, BN>::type;
  using ET = typename ImgSel<MATH, BM>::T;
  static constexpr int N = 2 * (IA::SIZE + IB::SIZE);
};

// One output tile (bx, by) of split / class bz.  The kernels below map blocks onto tiles.
template <int MATH, int MODE, int BM, int BN, int WM, int WN, int PF>
__device__ __forceinline__ void conv_tile(const ConvArgs& p, const int bx, const int by, const int bz,
                                          typename ImgSel<MATH, BM>::T* smem) {
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(WM * WN == 4 && TM >= 1 && TN >= 1, "tile");
  constexpr bool A_T = (MODE == MODE_WGRAD || MODE == MODE_PSW);   // A global vectors along rows -> register transpose
  constexpr bool B_T = (MODE != MODE_DGRAD && MODE != MODE_PS);   // B global vectors along rows (n) -> transpose
  constexpr bool FWDLIKE = (MODE == MODE_FWD || MODE == MODE_PS);  // A = the forward im2col gather of x
  using IA = typename ImgSel<MATH, BM>::type;
  using IB = typename ImgSel<MATH, BN>::type;
  using ET = typename ImgSel<MATH, BM>::T;
  ET* const As0 = smem;
  ET* const Bs0 = smem + 2 * IA::SIZE;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;

  // fp16x3 operand scales (powers of two): A = x (FWD, WGRAD) or dy (DGRAD), B = w (FWD, DGRAD) or dy (WGRAD)
  float sA = 1.f, sB = 1.f;
  if constexpr (MATH == 4) {
    sA = f16x3_scale(MODE == MODE_DGRAD ? p.ymax : p.xmax, 1.f);
    sB = (MODE == MODE_WGRAD || MODE == MODE_PSW) ? f16x3_scale(p.ymax, 1.f) : f16x3_scale(p.wmax, F16X3_WSCALE);
  }

  int M, Nn, Kd;
  DgClass g{};
  int zsplit;
  if constexpr (MODE == MODE_DGRAD) {
    const int ncls = p.S * p.S;
    const int cls = bz % ncls;
    zsplit = bz / ncls;
    g = dg_class(p, cls);
    M = g.M; Nn = p.C; Kd = g.Kd;
  } else if constexpr (FWDLIKE) {
    zsplit = bz;
    M = p.N * p.OH * p.OW; Nn = p.K; Kd = p.KH * p.KW * p.C;
  } else {
    zsplit = bz;
    M = p.KH * p.KW * p.C; Nn = MODE == MODE_PSW ? p.ps_T * p.ps_T * p.K : p.K; Kd = p.N * p.OH * p.OW;
  }
  FDiv fntw{};
  if constexpr (MODE == MODE_DGRAD) fntw = make_fdiv(g.ntw);
  const int m0 = bx * BM, n0 = by * BN;
  if (m0 >= M || n0 >= Nn) return;
  const int nkt = (Kd + BK3 - 1) / BK3;
  const int kt0 = zsplit * p.kt_per;
  const int kt1 = min(nkt, kt0 + p.kt_per);

  // A slots: plain -> (row = s >> 3, kq = s & 7); transposed -> (rq = s % (BM/4), kq = s / (BM/4))
  constexpr int A_SLOTS = A_T ? (BM / 4) * (BK3 / 4) : BM * (BK3 / 4);
  constexpr int B_SLOTS = B_T ? (BN / 4) * (BK3 / 4) : BN * (BK3 / 4);
  constexpr int A_PER = (A_SLOTS + NT - 1) / NT, B_PER = (B_SLOTS + NT - 1) / NT;
  constexpr int A_V = A_T ? 4 : 1, B_V = B_T ? 4 : 1;   // f4 loads per slot

  // Operands are read through raw buffer resources: an invalid element (padding tap, tile edge, k
  // tail) gets offset OOB >= num_records and loads as zero -- no branches, no zero-fill moves.
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, (long)p.N * p.OH * p.OW * p.ycs);
  const __amdgpu_buffer_rsrc_t rw =
      make_rsrc(p.w, MODE == MODE_PS ? (long)p.ps_KS * p.ps_KS * p.ps_C * p.ps_K : (long)p.KH * p.KW * p.wcin * p.K);

  // per-slot row geometry (float offsets; `pb` = element offset of the row at tap/k origin)
  int a_pb[A_PER], a_i1[A_PER], a_i2[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int s = tid + i * NT;
    a_pb[i] = 0; a_i1[i] = -(1 << 28); a_i2[i] = -(1 << 28);   // invalid row -> every tap out of range
    if constexpr (FWDLIKE) {
      const int m = m0 + (s >> 3);
      if (s < A_SLOTS && m < M) {
        const int ohw = p.OH * p.OW;
        const int n = m / ohw, r = m - n * ohw, oh = r / p.OW, ow = r - oh * p.OW;
        a_i1[i] = oh * p.S - p.PT; a_i2[i] = ow * p.S - p.PL;
        a_pb[i] = ((n * p.H + a_i1[i]) * p.W + a_i2[i]) * p.xcs + p.xco;
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      const int m = m0 + (s >> 3);
      if (s < A_SLOTS && m < M) {
        const int hw = g.HH * g.WW;
        const int n = m / hw, r = m - n * hw, ihh = r / g.WW, iww = r - ihh * g.WW;
        a_i1[i] = ihh + g.dh; a_i2[i] = iww + g.dw;
        a_pb[i] = ((n * p.OH + a_i1[i]) * p.OW + a_i2[i]) * p.ycs + p.yco;
      }
    } else {
      const int m = m0 + 4 * (s % (BM / 4));
      if (s < A_SLOTS && m < M) {
        const int tap = m / p.C, c = m - tap * p.C, kh = tap / p.KW, kw = tap - kh * p.KW;
        a_i1[i] = kh - p.PT; a_i2[i] = kw - p.PL;
        a_pb[i] = (a_i1[i] * p.W + a_i2[i]) * p.xcs + p.xco + c;
      }
    }
  }

  // register staging sets: set 0, and set 1 for the second tile in flight when PF == 2
  f4 ra0[A_PER][A_V], rb0[B_PER][B_V];
  f4 ra1[PF == 2 ? A_PER : 1][A_V], rb1[PF == 2 ? B_PER : 1][B_V];

  auto load_tiles = [&](int kt, auto& ra, auto& rb) {
#if TDE_DBG_PHASE & 1
    // timing diagnostic (not a result): no global loads in the k-loop
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
#pragma unroll
      for (int j = 0; j < A_V; ++j) ra[i][j] = f4{1.f, 1.f, 1.f, (float)kt};
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
#pragma unroll
      for (int j = 0; j < B_V; ++j) rb[i][j] = f4{1.f, 1.f, 1.f, (float)kt};
    return;
#endif
    const int kbase = kt * BK3;
    // k decode shared by every A slot (and the DGRAD B slots): s & 7 == tid & 7 for all slots
    const int kq = kbase + 4 * (tid & 7);
    int t_h = 0, t_w = 0, koff = 0, kx = 0, dg_wtap = 0;
    if constexpr (FWDLIKE) {
      const int tap = fdiv(kq, p.fC), c = kq - tap * p.C;
      t_h = fdiv(tap, p.fKW); t_w = tap - t_h * p.KW;
      koff = (t_h * p.W + t_w) * p.xcs + c;
    } else if constexpr (MODE == MODE_DGRAD) {
      const int tap = fdiv(kq, p.fK);
      kx = kq - tap * p.K;                       // output channel co
      t_h = fdiv(tap, fntw); t_w = tap - t_h * g.ntw;
      koff = -(t_h * p.OW + t_w) * p.ycs + kx;
      // weight offset of this thread's (tap, co) shared by all its B slots (which differ in ci only)
      dg_wtap = ((g.khs + p.S * t_h) * p.KW + g.kws + p.S * t_w) * p.wcin * p.K + kx;
    }
#if !(TDE_DBG_PHASE & 16)
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      if constexpr (FWDLIKE) {
        const bool ok = kq < Kd && (unsigned)(a_i1[i] + t_h) < (unsigned)p.H &&
                        (unsigned)(a_i2[i] + t_w) < (unsigned)p.W;
        ra[i][0] = bload(rx, ok ? 4 * (a_pb[i] + koff) : OOB);
      } else if constexpr (MODE == MODE_DGRAD) {
        const bool ok = kq < Kd && (unsigned)(a_i1[i] - t_h) < (unsigned)p.OH &&
                        (unsigned)(a_i2[i] - t_w) < (unsigned)p.OW;
        ra[i][0] = bload(rdy, ok ? 4 * (a_pb[i] + koff) : OOB);
      } else {
        const int s = tid + i * NT;
        const int pix0 = kbase + 4 * (s / (BM / 4));
        int n = fdiv(pix0, p.fOHW);
        const int r = pix0 - n * p.OH * p.OW;
        int oh = fdiv(r, p.fOW), ow = r - oh * p.OW;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ih = oh * p.S, iw = ow * p.S;
          const bool ok = pix0 + j < Kd && (unsigned)(ih + a_i1[i]) < (unsigned)p.H &&
                          (unsigned)(iw + a_i2[i]) < (unsigned)p.W;
          ra[i][j] = bload(rx, ok ? 4 * (a_pb[i] + ((n * p.H + ih) * p.W + iw) * p.xcs) : OOB);
          if (++ow == p.OW) { ow = 0; if (++oh == p.OH) { oh = 0; ++n; } }
        }
      }
    }
#endif
#if TDE_DBG_PHASE & 8
    if (true) return;
#endif
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int s = tid + i * NT;
      const bool slot = s < B_SLOTS;
      if constexpr (MODE == MODE_FWD) {
        const int n = n0 + 4 * (s % (BN / 4)), k0 = kbase + 4 * (s / (BN / 4));
        const int tap = fdiv(k0, p.fC), c0 = k0 - tap * p.C;   // k0..k0+3 share the tap (C % 4 == 0)
        const bool ok = slot && n < Nn && k0 < Kd;
        const int wo = (tap * p.wcin + c0) * p.K + n;            // weight row k0, column n (one multiply)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rb[i][j] = bload(rw, ok && c0 + j < p.wcin ? 4 * (wo + j * p.K) : OOB);
      } else if constexpr (MODE == MODE_DGRAD) {
        const int ci = n0 + (s >> 3);
        const bool ok = slot && kq < Kd && ci < p.wcin;
        rb[i][0] = bload(rw, ok ? 4 * (dg_wtap + ci * p.K) : OOB);
      } else if constexpr (MODE == MODE_PS) {
        // column n = (py, px, c), k quad kq = (th, tw, kin..kin+3): w[kh0 + py - 2 th][kh0 + px - 2 tw][c][kin..]
        const int n = n0 + (s >> 3);
        const int gq = fdiv(n, p.fpsC), c = n - gq * p.ps_C;
        const int tap = fdiv(kq, p.fC), kin = kq - tap * p.C;
        const int th = fdiv(tap, p.fKW), tw = tap - th * p.KW;
        const int kh = p.ps_kh0 + (gq >> 1) - 2 * th, kw = p.ps_kh0 + (gq & 1) - 2 * tw;
        const bool ok = slot && n < Nn && kq < Kd && (unsigned)kh < (unsigned)p.ps_KS && (unsigned)kw < (unsigned)p.ps_KS;
        rb[i][0] = bload(rw, ok ? 4 * (((kh * p.ps_KS + kw) * p.ps_C + c) * p.ps_K + kin) : OOB);
      } else if constexpr (MODE == MODE_PSW) {
        // columns n..n+3 = (th, tw, k..k+3): dy at (a - PW + th, b - PW + tw) of pixels pix0..pix0+3 = (img, a, b)
        const int n = n0 + 4 * (s % (BN / 4)), pix0 = kbase + 4 * (s / (BN / 4));
        const bool ok = slot && n < Nn;
        const int tap = fdiv(n, p.fK), k = n - tap * p.K;
        const int th = fdiv(tap, p.fpsT), tw = tap - th * p.ps_T;
        int img = fdiv(pix0, p.fOHW);
        const int r = pix0 - img * p.OH * p.OW;
        int aa = fdiv(r, p.fOW), bb = r - aa * p.OW;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ia = aa + th - p.ps_PW, ib = bb + tw - p.ps_PW;
          const bool okj = ok && pix0 + j < Kd && (unsigned)ia < (unsigned)p.OH && (unsigned)ib < (unsigned)p.OW;
          rb[i][j] = bload(rdy, okj ? 4 * (((img * p.OH + ia) * p.OW + ib) * p.ycs + p.yco + k) : OOB);
          if (++bb == p.OW) { bb = 0; if (++aa == p.OH) { aa = 0; ++img; } }
        }
      } else {
        const int n = n0 + 4 * (s % (BN / 4)), pix0 = kbase + 4 * (s / (BN / 4));
        const bool ok = slot && n < Nn;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rb[i][j] = bload(rdy, ok && pix0 + j < Kd ? 4 * ((pix0 + j) * p.ycs + p.yco + n) : OOB);
      }
    }
  };

  // staging store of one 4-k row segment (the staged fp16x3 image splits here, with the operand's scale)
  auto putA = [&](ET* A, int row, int k, f4 v) {
    if constexpr (MATH == 4 && TDE_F16_STAGE) IA::put(A, row, k, v, sA);
    else IA::put(A, row, k, v);
  };
  auto putB = [&](ET* Bm, int row, int k, f4 v) {
    if constexpr (MATH == 4 && TDE_F16_STAGE) IB::put(Bm, row, k, v, sB);
    else IB::put(Bm, row, k, v);
  };
  auto store_tiles = [&](int buf, auto& ra, auto& rb) {
#if TDE_DBG_PHASE & 4
    // timing diagnostic (not a result): no split / LDS staging stores (loads kept alive by one cheap use)
    if (ra[0][0][0] == 12345.f && rb[0][0][0] == 54321.f) As0[tid] = 0;
    return;
#endif
    ET* A = As0 + buf * IA::SIZE;
    ET* Bm = Bs0 + buf * IB::SIZE;
#if !(TDE_DBG_PHASE & 16)
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int s = tid + i * NT;
      if (s >= A_SLOTS) continue;
      if constexpr (A_T) {
        const int r0 = 4 * (s % (BM / 4)), k0 = 4 * (s / (BM / 4));
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          putA(A, r0 + rr, k0, f4{ra[i][0][rr], ra[i][1][rr], ra[i][2][rr], ra[i][3][rr]});
      } else {
        putA(A, s >> 3, 4 * (s & 7), ra[i][0]);
      }
    }
#endif
#if !(TDE_DBG_PHASE & 8)
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int s = tid + i * NT;
      if (s >= B_SLOTS) continue;
      if constexpr (B_T) {
        const int r0 = 4 * (s % (BN / 4)), k0 = 4 * (s / (BN / 4));
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          putB(Bm, r0 + rr, k0, f4{rb[i][0][rr], rb[i][1][rr], rb[i][2][rr], rb[i][3][rr]});
      } else {
        putB(Bm, s >> 3, 4 * (s & 7), rb[i][0]);
      }
    }
#endif
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};

  const int r16 = lane & 15, q = lane >> 4;
  const int wrow0 = wm * TM * 16, wcol0 = wn * TN * 16;

  // one k-tile from LDS buffer `cur`: fragment reads first, then `issue` (the global loads of a later
  // tile: their address arithmetic overlaps the LDS latency), then the MFMAs
  auto compute = [&](int cur, auto&& issue) {
    const ET* A = As0 + cur * IA::SIZE;
    const ET* Bm = Bs0 + cur * IB::SIZE;
    if constexpr (MATH == 1) {
      bf8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        ah[a] = IA::hi(A, wrow0 + a * 16 + r16, q);
        al[a] = IA::lo(A, wrow0 + a * 16 + r16, q);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        bh[b] = IB::hi(Bm, wcol0 + b * 16 + r16, q);
        bl[b] = IB::lo(Bm, wcol0 + b * 16 + r16, q);
      }
      issue();
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    } else if constexpr (MATH == 4 && TDE_F16_STAGE && (TDE_DBG_PHASE & 2)) {
      // timing diagnostic (not a result): fragment reads, no MFMAs
      h8 ah[TM], bh[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) ah[a] = IA::hi(A, wrow0 + a * 16 + r16, q);
#pragma unroll
      for (int b = 0; b < TN; ++b) bh[b] = IB::hi(Bm, wcol0 + b * 16 + r16, q);
      issue();
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b][0] += (float)ah[a][0] * (float)bh[b][0];
    } else if constexpr (MATH == 4 && TDE_F16_STAGE) {
      // fp16x3, staged image: hi / lo fragments straight from the planes (k-chunk q = k 8q..8q+7 for A and B)
      h8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        ah[a] = IA::hi(A, wrow0 + a * 16 + r16, q);
        al[a] = IA::lo(A, wrow0 + a * 16 + r16, q);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        bh[b] = IB::hi(Bm, wcol0 + b * 16 + r16, q);
        bl[b] = IB::lo(Bm, wcol0 + b * 16 + r16, q);
      }
      issue();
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    } else if constexpr (MATH == 4) {
      // fp16x3 (TDE_F16_STAGE=0): fp32 LDS image as MATH 3, each fragment scaled and split in registers
      f4 fa[TM][2], fb[TN][2];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        fa[a][0] = IA::frag(A, wrow0 + a * 16 + r16, 4 * q);
        fa[a][1] = IA::frag(A, wrow0 + a * 16 + r16, 16 + 4 * q);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        fb[b][0] = IB::frag(Bm, wcol0 + b * 16 + r16, 4 * q);
        fb[b][1] = IB::frag(Bm, wcol0 + b * 16 + r16, 16 + 4 * q);
      }
      issue();
      h8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) split8x2h(fa[a][0], fa[a][1], sA, ah[a], al[a]);
#pragma unroll
      for (int b = 0; b < TN; ++b) split8x2h(fb[b][0], fb[b][1], sB, bh[b], bl[b]);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    } else if constexpr (MATH == 2 || MATH == 3) {
      bf8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
      if constexpr (MATH == 2) {
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          ah[a] = IA::plane(A, 0, wrow0 + a * 16 + r16, q);
          am[a] = IA::plane(A, 1, wrow0 + a * 16 + r16, q);
          al[a] = IA::plane(A, 2, wrow0 + a * 16 + r16, q);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          bh[b] = IB::plane(Bm, 0, wcol0 + b * 16 + r16, q);
          bm[b] = IB::plane(Bm, 1, wcol0 + b * 16 + r16, q);
          bl[b] = IB::plane(Bm, 2, wcol0 + b * 16 + r16, q);
        }
        issue();
      } else {
        f4 fa[TM][2], fb[TN][2];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          // lane q feeds MFMA k-slots 8q..8q+7 with image k = 4q..4q+3, 16+4q..16+4q+3 (the same permutation
          // for A and B, so the contraction is unchanged): 16-byte column q, conflict-free reads
          fa[a][0] = IA::frag(A, wrow0 + a * 16 + r16, 4 * q);
          fa[a][1] = IA::frag(A, wrow0 + a * 16 + r16, 16 + 4 * q);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          fb[b][0] = IB::frag(Bm, wcol0 + b * 16 + r16, 4 * q);
          fb[b][1] = IB::frag(Bm, wcol0 + b * 16 + r16, 16 + 4 * q);
        }
        issue();
#pragma unroll
        for (int a = 0; a < TM; ++a) split8x3(fa[a][0], fa[a][1], ah[a], am[a], al[a]);
#pragma unroll
        for (int b = 0; b < TN; ++b) split8x3(fb[b][0], fb[b][1], bh[b], bm[b], bl[b]);
      }
      // smallest terms first
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[a], bm[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bm[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    } else {
      // lane (r16, q) holds k = 16*kc + 4*q + j of MFMA (kc, j): same permutation for A and B
      f4 fa[2][TM], fb[2][TN];
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
#pragma unroll
        for (int a = 0; a < TM; ++a) fa[kc][a] = IA::frag(A, wrow0 + a * 16 + r16, 16 * kc + 4 * q);
#pragma unroll
        for (int b = 0; b < TN; ++b) fb[kc][b] = IB::frag(Bm, wcol0 + b * 16 + r16, 16 * kc + 4 * q);
      }
      issue();
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[kc][a][j], fb[kc][b][j], acc[a][b], 0, 0, 0);
    }
  };

  if (kt0 < kt1) {
    load_tiles(kt0, ra0, rb0);
    store_tiles(0, ra0, rb0);
    __syncthreads();
    int cur = 0;
    if constexpr (PF == 1) {
      // one tile in flight: the load of tile kt+1 overlaps the MFMAs of tile kt
      for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = (kt + 1 < kt1);
        compute(cur, [&] { if (more) load_tiles(kt + 1, ra0, rb0); });
        if (more) store_tiles(cur ^ 1, ra0, rb0);
        __syncthreads();
        cur ^= 1;
      }
    } else {
      // two tiles in flight (register sets 0/1 alternate; the loop is unrolled by two so every register
      // index is static): tile kt is consumed from LDS while kt+1 and kt+2 are loading.  For the small
      // tiles of the deep, weight-streaming layers one tile's MFMAs are shorter than a memory latency.
      // Loads and stores are issued unconditionally (past the last tile they re-load tile kt1-1 into
      // the idle buffer): a conditional issue makes hipcc wait vmcnt(0) at the merge point, which
      // would drain the second tile in flight.
      const int klast = kt1 - 1;
      load_tiles(min(kt0 + 1, klast), ra1, rb1);
      int kt = kt0;
      while (true) {
        compute(cur, [&] { load_tiles(min(kt + 2, klast), ra0, rb0); });
        store_tiles(cur ^ 1, ra1, rb1);
        __syncthreads();
        cur ^= 1;
        if (++kt >= kt1) break;
        compute(cur, [&] { load_tiles(min(kt + 2, klast), ra1, rb1); });
        store_tiles(cur ^ 1, ra0, rb0);
        __syncthreads();
        cur ^= 1;
        if (++kt >= kt1) break;
      }
    }
  }

  if constexpr (MATH == 4) {
    // undo the operand scales (a power of two: exact) before any statistics, partial or store
    const float inv = 1.f / (sA * sB);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] *= inv;
  }

  tile_epilogue<MODE, BM, BN, WM, WN>(p, acc, bx, by, bz, M, Nn, zsplit, g, reinterpret_cast<float*>(smem));
}

// Tile order = hardware order.  (An XCD-contiguous remap -- each XCD walking a run of tiles that
// share a pixel slab -- was measured 5-20% SLOWER on config 2's layers, and an XCD-grouped WGRAD order neutral:
// the round-robin order already lets neighbouring tiles, dispatched together, share the slab through the
// Infinity Cache.)
// TDE_PF2_WAVES: waves per SIMD the two-tiles-in-flight (PF 2) variants must fit (register cap 512 / W)
#ifndef TDE_PF2_WAVES
#define TDE_PF2_WAVES 2
#endif
// TDE_GEMM_WAVES: waves per SIMD the fp16x3 one-tile-in-flight tiles are allocated for (round 6: 3 -- the 128 x 64 tiles
// and the fused backward's 64 x 128 tiles drop from 172-184 to 143-151 registers, no spills, 2 -> 3 waves per SIMD,
// which their 48 KB of LDS already allowed; tiles over 128 x 64 cannot fit 3 and keep the default allocation)
#ifndef TDE_GEMM_WAVES
#define TDE_GEMM_WAVES 3
#endif
template <int MATH, int MODE, int BM, int BN, int WM, int WN, int PF>
__global__ void __launch_bounds__(NT)
__attribute__((amdgpu_waves_per_eu(MATH == 4 ? (BM * BN <= 8192 ? TDE_GEMM_WAVES : 1) : (PF == 2 ? TDE_PF2_WAVES : 1))))
igemmx_kernel(const ConvArgs p) {
  __shared__ __attribute__((aligned(16))) typename ImgSel<MATH, BM>::T smem[SmemSize<MATH, BM, BN>::N];
  conv_tile<MATH, MODE, BM, BN, WM, WN, PF>(p, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// The two backward GEMMs of one layer in ONE launch (horizontal fusion): blocks [0, nd) compute the
// data gradient (MODE1: DGRAD of a conv, FWD of a deconv's virtual conv), blocks [nd, nd + nw) the
// filter gradient (WGRAD).  Both
// only read dz, so they are independent; at the deep levels neither fills the chip alone.
template <int MATH, int MODE1, int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MATH == 4 && BM * BN <= 8192 ? TDE_GEMM_WAVES : 1)))
igemm_bwd2_kernel(const ConvArgs pd, const ConvArgs pw, int gxd, int gyd,
                                                        int gxw, int gyw, int nd) {
  __shared__ __attribute__((aligned(16))) typename ImgSel<MATH, BM>::T smem[SmemSize<MATH, BM, BN>::N];
  int id = blockIdx.x;
  if (id < nd) {
    const int bx = id % gxd;
    id /= gxd;
    conv_tile<MATH, MODE1, BM, BN, WM, WN, 1>(pd, bx, id % gyd, id / gyd, smem);
  } else {
    id -= nd;
    const int bx = id % gxw;
    id /= gxw;
    conv_tile<MATH, MODE_WGRAD, BM, BN, WM, WN, 1>(pw, bx, id % gyw, id / gyw, smem);
  }
}

// ------------------------------------------------------------------ skinny-M path (deep levels)
// At the 3x4 / 2x2 levels (M = N*OH*OW <= 96 output rows) FWD and stride-1 DGRAD are weight streams:
// the operand W is read exactly once and the activations are a few hundred KB.  A tiled GEMM stages W
// through LDS one 32-deep k-tile per barrier and cannot keep enough bytes in flight.  Here each wave
// owns a k-slice of KG x 16 and issues ALL its loads (activations and weights, straight to registers)
// before the first MFMA; the block's 4 waves are 4 consecutive k-slices of the same 64 output
// columns, combined through LDS in wave order.  Grid = (64-column tiles, k splits); the per-split
// partials go to the usual slab and splitk_reduce_kernel (fixed order: deterministic).
//   MFMA operand mapping (v_mfma_f32_16x16x4_f32, MFMA m of a 16-deep group uses k = k0 + 4q + m):
//     A  lane (i, q) = X[row 16a + i][k0 + 4q + m]      (one f4 per row fragment and group)
//     B  FWD  : lane (i, q) f4 = W[k0 + 4q + m][n0 + 4i .. 4i+3]  -> column fragment j = output
//               columns n0 + 4i + j (weights are [k][n], n contiguous)
//        DGRAD: lane (i, q) f4 = W[tap][c = n0 + 16f + i][kx .. kx+3] -> column fragment f
//               (the [k][c] operand is contiguous along k)
template <int MODE, int TM, int KG>
__global__ void __launch_bounds__(NT) skinny_kernel(const ConvArgs p) {
  constexpr int KW = 16 * KG, KB = 4 * KW;   // k per wave, k per block (one split)
  __shared__ float red[4 * TM * 16 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 64, zsplit = blockIdx.y;
  int M, Nn, Kd;
  if constexpr (MODE == MODE_FWD) {
    M = p.N * p.OH * p.OW; Nn = p.K; Kd = p.KH * p.KW * p.C;
  } else {
    M = p.N * p.H * p.W; Nn = p.C; Kd = p.KH * p.KW * p.K;
  }
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, (long)p.N * p.OH * p.OW * p.ycs);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w, (long)p.KH * p.KW * p.wcin * p.K);
  // row geometry of this lane's TM rows
  int rb[TM], r1[TM], r2[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int m = 16 * a + i;
    rb[a] = 0; r1[a] = -(1 << 28); r2[a] = -(1 << 28);
    if (m < M) {
      if constexpr (MODE == MODE_FWD) {
        const int ohw = p.OH * p.OW;
        const int n = m / ohw, r = m - n * ohw, oh = r / p.OW, ow = r - oh * p.OW;
        r1[a] = oh * p.S - p.PT; r2[a] = ow * p.S - p.PL;
        rb[a] = ((n * p.H + r1[a]) * p.W + r2[a]) * p.xcs + p.xco;
      } else {
        const int hw = p.H * p.W;
        const int n = m / hw, r = m - n * hw, ih = r / p.W, iw = r - ih * p.W;
        r1[a] = ih + p.PT; r2[a] = iw + p.PL;
        rb[a] = ((n * p.OH + r1[a]) * p.OW + r2[a]) * p.ycs + p.yco;
      }
    }
  }
  // issue every load of this wave's k-slice
  f4 xa[KG][TM], wb[KG][4];
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    const int kq = zsplit * KB + wv * KW + 16 * g + 4 * q;
    const bool kok = kq < Kd;
    if constexpr (MODE == MODE_FWD) {
      const int tap = fdiv(kq, p.fC), c = kq - tap * p.C;
      const int th = fdiv(tap, p.fKW), tw = tap - th * p.KW;
      const int koff = (th * p.W + tw) * p.xcs + c;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const bool ok = kok && (unsigned)(r1[a] + th) < (unsigned)p.H && (unsigned)(r2[a] + tw) < (unsigned)p.W;
        xa[g][a] = bload(rx, ok ? 4 * (rb[a] + koff) : OOB);
      }
      const int n = n0 + 4 * i;
#pragma unroll
      for (int mm = 0; mm < 4; ++mm)
        wb[g][mm] = bload(rw, kok && c + mm < p.wcin && n < Nn ? 4 * ((tap * p.wcin + c + mm) * p.K + n) : OOB);
    } else {
      const int tap = fdiv(kq, p.fK), kx = kq - tap * p.K;
      const int th = fdiv(tap, p.fKW), tw = tap - th * p.KW;
      const int koff = -(th * p.OW + tw) * p.ycs + kx;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const bool ok = kok && (unsigned)(r1[a] - th) < (unsigned)p.OH && (unsigned)(r2[a] - tw) < (unsigned)p.OW;
        xa[g][a] = bload(rdy, ok ? 4 * (rb[a] + koff) : OOB);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int c = n0 + 16 * f + i;
        wb[g][f] = bload(rw, kok && c < p.wcin ? 4 * ((tap * p.wcin + c) * p.K + kx) : OOB);
      }
    }
  }
  f4 acc[TM][4];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[a][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const float bv = MODE == MODE_FWD ? wb[g][mm][j] : wb[g][j][mm];
          acc[a][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[g][a][mm], bv, acc[a][j], 0, 0, 0);
        }
  // combine the 4 waves (k-slices) in wave order; thread t then owns output columns n0 + (t & 63)
  float* mine = red + wv * (TM * 16 * 64);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) mine[((a * 4 + j) * 4 + r) * 64 + lane] = acc[a][j][r];
  __syncthreads();
  const int cc = tid & 63;                     // column within the tile
  const int col = n0 + cc;
  // this column's (fragment, lane i) in the accumulator layout
  const int jf = MODE == MODE_FWD ? (cc & 3) : (cc >> 4);
  const int il = MODE == MODE_FWD ? (cc >> 2) : (cc & 15);
  const bool direct = p.splits == 1;
  float* base;
  if constexpr (MODE == MODE_FWD) base = direct ? p.y : p.ws;
  else base = direct ? p.dx : p.ws;
  for (int rr = tid >> 6; rr < 16 * TM; rr += 4) {   // rows of the tile
    const int a = rr >> 4, qq = (rr & 15) >> 2, r = rr & 3;
    const int e = ((a * 4 + jf) * 4 + r) * 64 + qq * 16 + il;
    const float v = ((red[e] + red[TM * 1024 + e]) + red[2 * TM * 1024 + e]) + red[3 * TM * 1024 + e];
    if (rr >= M || col >= Nn) continue;
    long off;
    if (direct) off = (long)rr * (MODE == MODE_FWD ? p.ycs : p.xcs) + (MODE == MODE_FWD ? p.yco : p.xco) + col;
    else off = ((long)zsplit * M + rr) * Nn + col;
    base[off] = direct ? (p.accumulate ? base[off] + v : bias_act(v, p.bias, col, p.relu)) : v;
  }
}

// Split-K reduction: dst(row, col) (+)= sum_z ws[z][row][col].  A block is ZL z-lanes x (256/ZL)
// output quads: lane l sums splits l, l+ZL, ... with 4 loads in flight, then the ZL lanes of a quad are
// combined through LDS in lane order (fixed order: deterministic).  ZL > 1 only when the output is too
// small to fill the chip otherwise (few outputs, hundreds of splits: the WGRAD of 192x256 layers).
// (The body takes the block's index among the nblk blocks of its reduction: splitk_reduce2_kernel runs a layer's data-
// and filter-gradient reductions as one launch.)
template <int MODE>
__device__ __forceinline__ void splitk_reduce_body(const ConvArgs& p, int rows, int cols, int zl, int blk, int nblk,
                                                   f4* tmp) {
  const long total4 = (long)rows * (cols / 4);
  const long stride = (long)rows * cols;
  const int zlane = threadIdx.x % zl, ql = threadIdx.x / zl, qpb = 256 / zl;
  for (long i0 = (long)blk * qpb; i0 < total4; i0 += (long)nblk * qpb) {
    const long i = i0 + ql;
    f4 s = {0.f, 0.f, 0.f, 0.f}, prev = {0.f, 0.f, 0.f, 0.f};
    int row = 0, col = 0;
    float* dst = nullptr;
    if (i < total4) {
      row = (int)(i / (cols / 4));
      col = 4 * (int)(i - (long)row * (cols / 4));
      if constexpr (MODE == MODE_FWD) {
        dst = p.y + (long)row * p.ycs + p.yco + col;
      } else if constexpr (MODE == MODE_DGRAD) {
        dst = p.dx + (long)row * p.xcs + p.xco + col;
      } else if constexpr (MODE == MODE_PSW) {
        // row (py, px, c), columns col..col+3 = (th, tw, k..k+3) -> dw[kh0 + py - 2 th][kh0 + px - 2 tw][c][k..k+3]
        const int gq = row / p.C, c = row - gq * p.C;
        const int tap = col / p.K, k = col - tap * p.K;
        const int th = tap / p.ps_T, tw = tap - th * p.ps_T;
        const int kh = p.ps_kh0 + (gq >> 1) - 2 * th, kw = p.ps_kh0 + (gq & 1) - 2 * tw;
        dst = ((unsigned)kh < (unsigned)p.ps_KS && (unsigned)kw < (unsigned)p.ps_KS)
                  ? p.dw + ((long)(kh * p.ps_KS + kw) * p.wcin + c) * p.K + k
                  : nullptr;
      } else {
        const int tap = row / p.C, c = row - tap * p.C;
        dst = c < p.wcin ? p.dw + (long)(tap * p.wcin + c) * p.K + col : nullptr;
      }
      // the accumulated-into value is loaded with the slabs (not after the sum: one round trip less)
      if (p.accumulate && zlane == 0 && dst) prev = ld4(dst);
      const float* src = p.ws + (long)row * cols + col;
      f4 s4[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      int z = zlane;
      for (; z + 3 * zl < p.splits; z += 4 * zl) {
#pragma unroll
        for (int u = 0; u < 4; ++u) s4[u] += ld4(src + (z + u * zl) * stride);
      }
      for (int u = 0; z < p.splits; z += zl, ++u) s4[u] += ld4(src + z * stride);
      s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
    if (zl > 1) {
      tmp[threadIdx.x] = s;
      __syncthreads();
      if (zlane == 0) {
        for (int k = 1; k < zl; ++k) s += tmp[threadIdx.x + k];
      }
      __syncthreads();
    }
    if (zlane != 0 || i >= total4 || !dst) continue;
    if (p.accumulate) s += prev;
    if constexpr (MODE != MODE_WGRAD && MODE != MODE_PSW) {
      if (p.bias || p.relu) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] = bias_act(s[j], p.bias, col + j, p.relu);
      }
    }
    tde_st(reinterpret_cast<f4*>(dst), s);
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const ConvArgs p, int rows, int cols, int zl) {
  __shared__ f4 tmp[256];
  splitk_reduce_body<MODE>(p, rows, cols, zl, blockIdx.x, gridDim.x, tmp);
}

// Both split-K reductions of one layer's backward (data gradient in MODE1, filter gradient) in one launch: blocks
// [0, nb1) reduce the first, the rest the second (per element the same sums as two launches).
template <int MODE1, int MODE2 = MODE_WGRAD>
__global__ void __launch_bounds__(256) splitk_reduce2_kernel(const ConvArgs p1, int rows1, int cols1, int zl1, int nb1,
                                                             const ConvArgs p2, int rows2, int cols2, int zl2) {
  __shared__ f4 tmp[256];
  if ((int)blockIdx.x < nb1) splitk_reduce_body<MODE1>(p1, rows1, cols1, zl1, blockIdx.x, nb1, tmp);
  else splitk_reduce_body<MODE2>(p2, rows2, cols2, zl2, blockIdx.x - nb1, gridDim.x - nb1, tmp);
}

// Split-K reduction for a conv followed by batch norm: z = sum_z ws[z] (same fixed order as
// splitk_reduce_kernel) written densely, plus per-row-chunk fp64 statistics partials [chunk][2][cols].
// Grid (row chunk, 64-channel group): a thread owns one channel quad of a row lane.
__global__ void __launch_bounds__(256) splitk_reduce_bn_kernel(const float* ws, int splits, int rows, int cols,
                                                               float* z, const BnChunks cp, double* part) {
  __shared__ double sh[2][256 * 4];
  const int q0 = blockIdx.y * 16;
  const int nq = min(16, cols / 4 - q0);
  const int ty_n = 256 / nq;
  const int tx = threadIdx.x % nq, ty = threadIdx.x / nq;
  const int c = 4 * (q0 + tx);
  const long stride = (long)rows * cols;
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  int r0, r1;
  bn_chunk_rows(cp, blockIdx.x, r0, r1);   // row groups: every chunk inside one group (group-major partials)
  if (ty < ty_n) {
    float f0[4] = {0, 0, 0, 0}, f1[4] = {0, 0, 0, 0};
    for (int r = r0 + ty; r < r1; r += ty_n) {
      const float* src = ws + (long)r * cols + c;
      f4 a[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      int zi = 0;
      for (; zi + 3 < splits; zi += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] += ld4(src + (zi + u) * stride);
      }
      for (int u = 0; zi < splits; ++zi, ++u) a[u] += ld4(src + zi * stride);
      const f4 v = (a[0] + a[1]) + (a[2] + a[3]);
      tde_st(reinterpret_cast<f4*>(z + (long)r * cols + c), v);
#pragma unroll
      for (int j = 0; j < 4; ++j) { f0[j] += v[j]; f1[j] += v[j] * v[j]; }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { s0[j] = f0[j]; s1[j] = f1[j]; }
  }
  rowlane_combine(s0, s1, nq, ty_n, &sh[0][0]);
  if (ty == 0) {
    double* o = part + (long)blockIdx.x * 2 * cols;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[c + j] = s0[j]; o[cols + c + j] = s1[j]; }
  }
}

// ------------------------------------------------------------------ host dispatch
struct Plan {
  int bm, bn, splits, kt_per, gx, gy, gz;
  int skinny_tm, skinny_kg;   // > 0: skinny_kernel<MODE, TM, KG> (weight-streaming deep layers)
  int rows, cols;  // reduce extent
  size_t slab_bytes, ws_bytes;
};

static void gemm_dims(const tde_conv_desc_t& d, int mode, long& M, long& Nn, long& Kd, int& ncls) {
  ncls = 1;
  if (mode == MODE_FWD) {
    M = (long)d.N * d.OH * d.OW; Nn = d.K; Kd = (long)d.KH * d.KW * d.C;
  } else if (mode == MODE_DGRAD) {
    ncls = d.stride * d.stride;
    const long hh = (d.H + d.stride - 1) / d.stride, ww = (d.W + d.stride - 1) / d.stride;
    M = (long)d.N * hh * ww;  // largest class
    Nn = d.C;
    const long th = (d.KH + d.stride - 1) / d.stride, tw = (d.KW + d.stride - 1) / d.stride;
    Kd = th * tw * d.K;
  } else {
    M = (long)d.KH * d.KW * d.C; Nn = d.K; Kd = (long)d.N * d.OH * d.OW;
  }
}

// Split-K policy (environment overrides are for tuning experiments; read once at load time).
static long env_long(const char* name, long dflt) {
  const char* v = getenv(name);
  return v ? atol(v) : dflt;
}
// 0 fp32 MFMA, 1 bf16x3, 2/3 bf16x6, 4 fp16x3 (process-wide, see tde_set_conv_math; TDE_CONV_MATH sets the
// initial mode for A/B runs).  Default 4: the scaled two-way fp16 split, the fastest mode within the parity
// bars (half the MFMAs of bf16x6 at the same accuracy class).
static int g_conv_math = []() {
  const long m = env_long("TDE_CONV_MATH", 4);
  return (int)(m >= 0 && m <= 4 ? m : 4);
}();
static const long g_split_target = tde_env_pos("TDE_SPLIT_TARGET", 384);   // blocks to aim for (round 4: 384, see make_plan)
static const long g_split_minkt = tde_env_pos("TDE_SPLIT_MINKT", 4);       // >= k-tiles per split
static const long g_split_slab = tde_env_pos("TDE_SPLIT_SLAB_MB", 128) << 20;
// tile / split overrides for kernel exploration (scripts/conv_micro.py); 0 = planner's choice
static const long g_force_bn = env_long("TDE_FORCE_BN", 0);
static const long g_force_bm = env_long("TDE_FORCE_BM", 0);
static const long g_force_splits = env_long("TDE_FORCE_SPLITS", 0);

static const long g_skinny_m = env_long("TDE_SKINNY_M", 32);   // rows up to which FWD / DGRAD go skinny
// FWD / DGRAD GEMMs with at most this many rows (and < 256 tiles) take 64-row tiles (more blocks); above it, and
// for every WGRAD, 128 (half the weight re-reads of a weight-streaming deep layer per row tile)
static const long g_bm64_maxm = env_long("TDE_BM64_MAXM", 4096);
static const long g_tile_ovh = env_long("TDE_TILE_OVH", 24);   // per-tile overhead of the N-tile rule, in columns
static const long g_maxbn = env_long("TDE_MAXBN", 0);           // cap on the N tile (0: none; A/B of the 3-wave tiles)
static const long g_maxbn_modes = env_long("TDE_MAXBN_MODES", 7);   // bit m: the cap applies to mode m

// fix_bm / fix_bn > 0: plan with that tile (the fused backward launch needs one tile for both GEMMs)
static Plan make_plan(const tde_conv_desc_t& d, int mode, int fix_bm = 0, int fix_bn = 0) {
  const int BK = BK3;
  long M, Nn, Kd; int ncls;
  gemm_dims(d, mode, M, Nn, Kd, ncls);
  Plan pl{};
  if ((mode == MODE_FWD || (mode == MODE_DGRAD && d.stride == 1)) && M <= g_skinny_m && M <= 96 && !fix_bm &&
      g_conv_math != 1) {
    // skinny path (fp32 MFMA in every exact math mode: a weight stream, not MFMA-bound): 64-column
    // tiles, 4 waves x KG x 16 of k per block; the largest KG (fewest splits) that still gives >= 256
    // blocks, TM x KG <= 8 register fragments
    pl.skinny_tm = (int)((M + 15) / 16);
    pl.gx = tde_cdiv(Nn, 64);
    pl.skinny_kg = 1;
    for (int kg = 4; kg >= 1; kg /= 2) {
      if (pl.skinny_tm * kg > 8) continue;
      if ((long)pl.gx * tde_cdiv(Kd, 64 * kg) >= 256 || kg == 1) { pl.skinny_kg = kg; break; }
    }
    pl.splits = tde_cdiv(Kd, 64 * pl.skinny_kg);
    pl.kt_per = 0;
    pl.gy = pl.splits;
    pl.gz = 1;
    pl.bm = 0; pl.bn = 64;
    pl.rows = (int)M; pl.cols = (int)Nn;
    pl.slab_bytes = pl.splits > 1 ? (size_t)pl.splits * pl.rows * pl.cols * sizeof(float) : 0;
    pl.ws_bytes = pl.slab_bytes;
    return pl;
  }
  // N tile: minimise computed columns + a per-tile overhead (~24 columns' worth), so odd widths such
  // as the decoder concats in DGRAD (68, 132, 260 channels) do not run half-empty 128-wide tiles
  {
    static const int cands[] = {16, 32, 48, 64, 96, 128};
    long best = -1;
    for (int bn : cands) {
      if (g_maxbn && ((g_maxbn_modes >> mode) & 1) && bn > g_maxbn) continue;
      const long t = tde_cdiv(Nn, bn);
      const long cost = t * bn + g_tile_ovh * t;
      if (best < 0 || cost < best || (cost == best && bn > pl.bn)) { best = cost; pl.bn = bn; }
    }
  }
  if (g_force_bn) pl.bn = (int)g_force_bn;
  if (fix_bn) pl.bn = fix_bn;
  pl.bm = 128;
  long tiles = tde_cdiv(M, pl.bm) * (long)tde_cdiv(Nn, pl.bn) * ncls;
  // WGRAD reduces over every pixel (Kd ~ 1e5): parallelism comes from split-K, so keep the
  // MFMA-dense 128-row tile; FWD/DGRAD with few tiles trade tile size for more blocks.  (64-row filter-gradient
  // tiles for the low-resolution layers and a column cap on the 64-row tiles were measured no better and removed in
  // round 5.)
  if ((mode != MODE_WGRAD && tiles < 256 && M <= g_bm64_maxm) || g_force_bm == 64 || fix_bm == 64) {
    pl.bm = 64;
    tiles = tde_cdiv(M, pl.bm) * (long)tde_cdiv(Nn, pl.bn) * ncls;
  }
  if (fix_bm == 128 && pl.bm != 128) {
    pl.bm = 128;
    tiles = tde_cdiv(M, pl.bm) * (long)tde_cdiv(Nn, pl.bn) * ncls;
  }
  const int nkt = tde_cdiv(Kd, BK);
  // split K until ~1.5 blocks per CU (g_split_target 384), keeping >= 4 k-tiles (128 reduction elements) per split.
  // Round 4: 384 instead of 512 -- with config 4's two networks on two streams each GEMM no longer has to fill the
  // chip alone, and fewer splits mean fewer slab bytes and shorter reduces (same box, alternating x2: config 4
  // 1043-1047 -> 1066-1067 pairs/s, config 2 2917-2918 -> 2924-2927; 256: config 4 1065, config 2 -1.3 %;
  // profiles/r04/ab_r04e_split.txt)
  int splits = 1;
  const long target = g_split_target;
  if (tiles < target) {
    splits = (int)((target + tiles - 1) / tiles);
    splits = splits > nkt / g_split_minkt ? (int)(nkt / g_split_minkt) : splits;
    if (splits < 1) splits = 1;
    if (splits > 512) splits = 512;
    // keep the fp32 partial slabs under 128 MB
    long rows = mode == MODE_DGRAD ? (long)d.N * d.H * d.W : M;
    long cols = mode == MODE_DGRAD ? d.C : Nn;
    while (splits > 1 && (long)splits * rows * cols * 4 > g_split_slab) splits /= 2;
  }
  if (g_force_splits) splits = (int)(g_force_splits < nkt ? g_force_splits : nkt);
  pl.kt_per = tde_cdiv(nkt, splits);
  pl.splits = tde_cdiv(nkt, pl.kt_per);
  pl.gx = tde_cdiv(M, pl.bm);
  pl.gy = tde_cdiv(Nn, pl.bn);
  pl.gz = pl.splits * ncls;
  if (mode == MODE_FWD) { pl.rows = (int)M; pl.cols = (int)Nn; }
  else if (mode == MODE_DGRAD) { pl.rows = d.N * d.H * d.W; pl.cols = d.C; }
  else { pl.rows = (int)M; pl.cols = (int)Nn; }
  pl.slab_bytes = pl.splits > 1 ? (size_t)pl.splits * pl.rows * pl.cols * sizeof(float) : 0;
  pl.ws_bytes = pl.slab_bytes;
  return pl;
}

// Fused conv + BN + ReLU (tde_conv2d_fwd_bn / tde_deconv2d_fwd_bn, workspace op 3).  Where the BN
// statistics come from:
//   BN_SMALL : <= 2048 output rows -- [split-K reduce], then one BN kernel (bn.hip) does it all;
//   BN_EPI   : no split -- the conv epilogue writes one fp64 partial per row tile;
//   BN_REDUCE: split-K -- the reduce kernel writes z and one partial per row chunk;
//   BN_STANDALONE: row groups (tde_bn_train_t.groups > 1) the tiles above would straddle -- [split-K reduce], then
//              bn.hip's grouped partial pass over z;
// then bn.hip finalizes and applies (two launches).
enum { BN_SMALL = 0, BN_EPI = 1, BN_REDUCE = 2, BN_STANDALONE = 3 };
struct BnPlan {
  int path, nparts;
  BnChunks ch;
  size_t part_bytes;
};

static BnPlan bn_plan(const tde_conv_desc_t& d, int mode, const Plan& pl, int G = 1) {
  BnPlan b{};
  if (G < 1) G = 1;
  const int Mg = pl.rows / G;
  // a deconv's parity classes: every class's rows per group whole row tiles (group-major epilogue partials)
  bool cls_aligned = true;
  if (mode == MODE_DGRAD)
    for (int c = 0; c < d.stride * d.stride; ++c) {
      const int py = c / d.stride, px = c - py * d.stride;
      const long mc = (long)d.N * ((d.H - py + d.stride - 1) / d.stride) * ((d.W - px + d.stride - 1) / d.stride);
      if (mc % G != 0 || (mc / G) % pl.bm != 0) cls_aligned = false;
    }
  if (Mg <= BN_SMALL_M) {
    b.path = BN_SMALL;
  } else if (G > 1 && pl.splits == 1 && (mode == MODE_DGRAD ? !cls_aligned : Mg % pl.bm != 0)) {
    // row groups whose boundaries the epilogue's row tiles (or a deconv's parity-class tiles) do not respect:
    // the statistics come from a separate grouped partial pass over z
    b.path = BN_STANDALONE;
    b.nparts = 0;
  } else if (pl.splits == 1) {
    b.path = BN_EPI;
    if (mode == MODE_DGRAD)
      for (int c = 0; c < d.stride * d.stride; ++c) {
        const int py = c / d.stride, px = c - py * d.stride;
        const long mc = (long)d.N * ((d.H - py + d.stride - 1) / d.stride) * ((d.W - px + d.stride - 1) / d.stride);
        b.nparts += tde_cdiv(mc, pl.bm);
      }
    else
      b.nparts = pl.gx;
  } else {
    // split-K: the reduce kernel writes z and the partials, one per row chunk, every chunk inside one row group
    b.path = BN_REDUCE;
    b.ch = bn_chunk_plan(pl.rows, pl.cols, pl.splits, G);
    b.nparts = b.ch.chunks;
  }
  b.part_bytes = (size_t)b.nparts * 2 * pl.cols * sizeof(double);
  if (pl.splits > 1) {
    // the workspace query does not know G: a grouped split-K reduce may cut up to G - 1 more row chunks than the
    // G = 1 plan (per_g is a ceiling per group), so size for the worst G
    for (int g = 1; g <= BN_MAX_GROUPS; ++g) {
      if (pl.rows % g != 0) continue;
      const size_t pb = (size_t)bn_chunk_plan(pl.rows, pl.cols, pl.splits, g).chunks * 2 * pl.cols * sizeof(double);
      if (pb > b.part_bytes) b.part_bytes = pb;
    }
  }
  // room for the grouped standalone statistics pass (any G: the workspace query does not know it)
  const size_t sa = bn_part_bytes(pl.rows, pl.cols);
  if (sa > b.part_bytes) b.part_bytes = sa;
  return b;
}

// Halo path workspace: split weights + BN partials.  Sized for both split maths whatever the current mode
// (a caller may size once and switch tde_set_conv_math later).
static size_t halo_ws_bytes(const tde_conv_desc_t& d, int mode, bool bn) {
  // the larger of the bf16x6 and fp16x3 plans (planes and LDS budget differ, so may the tile shape)
  size_t b = 0;
  for (int math = 3; math <= 4; ++math) {
    HaloPlan hp;
    if (mode == MODE_WGRAD || !halo_plan(d, mode == MODE_FWD ? 0 : 1, math, hp)) continue;
    size_t pb = bn ? (size_t)hp.nparts * 2 * hp.Ncols * sizeof(double) : 0;
    if (bn) {
      const long Mz = (long)d.N * (mode == MODE_FWD ? (long)d.OH * d.OW : (long)d.H * d.W);
      if (bn_part_bytes(Mz, hp.Ncols) > pb) pb = bn_part_bytes(Mz, hp.Ncols);
    }
    const size_t m = hp.wbytes + pb;
    b = m > b ? m : b;
  }
  return b;
}

// halo-WGRAD partials: the larger of the fp32 and fp16x3 plans (0: neither applies)
static size_t hwg_ws_bytes(const tde_conv_desc_t& d) {
  size_t b = 0;
  for (int math = 3; math <= 4; ++math) {
    HwgPlan wp;
    if (hwg_plan(d, wp, math) && wp.part_bytes > b) b = wp.part_bytes;
  }
  return b;
}

static bool ps_ok(const tde_conv_desc_t& d, int* bm = nullptr, int* bn = nullptr);
static bool psw_ok(const tde_conv_desc_t& d);
static Plan psw_plan(const tde_conv_desc_t& d);

static size_t plan_ws_bytes(const tde_conv_desc_t& d, int mode, bool bn) {
  const Plan pl = make_plan(d, mode);
  const size_t igemm = pl.ws_bytes + (bn ? bn_plan(d, mode, pl).part_bytes : 0);
  const size_t halo = halo_ws_bytes(d, mode, bn);
  size_t b = igemm > halo ? igemm : halo;
  int pbm = 0, pbn = 0;
  if (mode == MODE_DGRAD && ps_ok(d, &pbm, &pbn)) {
    // pixel-shuffle path: one partial record [2][C] per (row tile, column tile)
    const size_t pb = bn ? std::max((size_t)tde_cdiv((long)d.N * d.OH * d.OW, pbm) * (4 * d.C / pbn) * 2 * d.C *
                                        sizeof(double),
                                    bn_part_bytes((long)d.N * d.H * d.W, d.C))
                         : 0;
    if (pb > b) b = pb;
  }
  if (mode == MODE_WGRAD && hwg_ws_bytes(d) > b) b = hwg_ws_bytes(d);
  if (mode == MODE_WGRAD && psw_ok(d) && psw_plan(d).ws_bytes > b) b = psw_plan(d).ws_bytes;
  return b;
}

// fp16x3 64-row FWD / DGRAD tiles with two tiles in flight (round 6): at the 3-wave register cap (TDE_GEMM_WAVES) they
// fit in 138-152 registers without spills, so the second tile no longer costs a wave per SIMD (round 3's attempt
// ran them at 2 waves: neutral, see below).  0: one tile in flight (A/B).
static const long g_f16_pf2 = env_long("TDE_F16_PF2", 1);
// prefetch depth (tiles in flight): 1 for 128-row tiles; for the 64-row tiles of the deep layers 2 in the
// register-split maths, 1 in fp16x3 (depth 2 costs 187 VGPR+AGPR = 2 waves/SIMD, depth 1 136 = 3; measured
// (scripts/r02zm.sh) icnv5 DGRAD 43.6 -> 36.6 us, config 2 2.82 -> 2.80 ms, config 4 13.30 -> 13.18 ms).
// (Two tiles in flight for the fp16x3 tiles, with or without the staging interleaved with the MFMAs, measured
// neutral in round 3 -- 604 vs 602 us on big3x3 WGRAD, config 4 within 0.5 % -- and removed.)
// wave layout of a tile: 2 x 2 waves when BN is a multiple of TDE_WN_DIV, else 4 x 1 (all rows split)
#ifndef TDE_WN_DIV
#define TDE_WN_DIV 32
#endif

// bf16x6 register split (math 3) costs ~44 VALU instructions per 8-element fragment per wave: it pays
// only where a wave's fragments feed enough MFMAs (measured: 128x128 1.45x faster than fp32, 128x32
// 10% slower), so narrower tiles run exact fp32 MFMA in that mode.
static const long g_math3_min_bn = env_long("TDE_MATH3_MIN_BN", 64);
static const long g_narrow_math = env_long("TDE_NARROW_MATH", 0);   // math of those narrow tiles (0 or 2)
static const long g_math3_wgrad_min_bn = env_long("TDE_MATH3_WGRAD_MIN_BN", 64);   // the same for WGRAD alone
// fp16x3 (math 4): split cost per fragment ~half of bf16x6's; narrow-tile threshold measured separately
static const long g_math4_min_bn = env_long("TDE_MATH4_MIN_BN", 16);
static int tile_math(int bn, int mode = -1) {
  if (g_conv_math == 4) return bn < g_math4_min_bn ? 0 : 4;
  const long lim = mode == MODE_WGRAD ? g_math3_wgrad_min_bn : g_math3_min_bn;
  return (g_conv_math == 3 && bn < lim) ? (int)g_narrow_math : g_conv_math;
}

template <int MODE, int BM, int BN>
static void launch_cfg(const ConvArgs& a0, dim3 grid, hipStream_t st) {
  ConvArgs a = a0;
  constexpr int WN = BN % TDE_WN_DIV == 0 ? 2 : 1;
  constexpr int WM = 4 / WN;
  const int math = tile_math(BN, MODE);
  const int pf = (BM == 64 && (math != 4 || g_f16_pf2)) ? 2 : 1;
  constexpr bool F16_PF2 = BM == 64 && MODE != MODE_WGRAD && MODE != MODE_PSW;
  if (math == 1) hipLaunchKernelGGL((igemmx_kernel<1, MODE, BM, BN, WM, WN, 1>), grid, dim3(NT), 0, st, a);
  else if (math == 2) hipLaunchKernelGGL((igemmx_kernel<2, MODE, BM, BN, WM, WN, 1>), grid, dim3(NT), 0, st, a);
  else if (math == 4 && F16_PF2 && pf == 2)
    hipLaunchKernelGGL((igemmx_kernel<4, MODE, BM, BN, WM, WN, F16_PF2 ? 2 : 1>), grid, dim3(NT), 0, st, a);
  else if (math == 4) hipLaunchKernelGGL((igemmx_kernel<4, MODE, BM, BN, WM, WN, 1>), grid, dim3(NT), 0, st, a);
  else if (math == 3 && pf == 2) hipLaunchKernelGGL((igemmx_kernel<3, MODE, BM, BN, WM, WN, 2>), grid, dim3(NT), 0, st, a);
  else if (math == 3) hipLaunchKernelGGL((igemmx_kernel<3, MODE, BM, BN, WM, WN, 1>), grid, dim3(NT), 0, st, a);
  else if (pf == 2) hipLaunchKernelGGL((igemmx_kernel<0, MODE, BM, BN, WM, WN, 2>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((igemmx_kernel<0, MODE, BM, BN, WM, WN, 1>), grid, dim3(NT), 0, st, a);
}

template <int MODE, int TM>
static void launch_skinny_tm(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  const dim3 grid(pl.gx, pl.gy);
  switch (pl.skinny_kg) {
    case 4: if constexpr (TM <= 2) hipLaunchKernelGGL((skinny_kernel<MODE, TM, 4>), grid, dim3(NT), 0, st, a); break;
    case 2: if constexpr (TM <= 4) hipLaunchKernelGGL((skinny_kernel<MODE, TM, 2>), grid, dim3(NT), 0, st, a); break;
    default: hipLaunchKernelGGL((skinny_kernel<MODE, TM, 1>), grid, dim3(NT), 0, st, a); break;
  }
}

template <int MODE>
static void launch_skinny(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  if constexpr (MODE == MODE_WGRAD) return;
  else {
    switch (pl.skinny_tm) {
      case 1: launch_skinny_tm<MODE, 1>(pl, a, st); break;
      case 2: launch_skinny_tm<MODE, 2>(pl, a, st); break;
      case 3: launch_skinny_tm<MODE, 3>(pl, a, st); break;
      case 4: launch_skinny_tm<MODE, 4>(pl, a, st); break;
      case 5: launch_skinny_tm<MODE, 5>(pl, a, st); break;
      default: launch_skinny_tm<MODE, 6>(pl, a, st); break;
    }
  }
}

template <int MODE>
static void launch_mode(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  if (pl.skinny_tm > 0) {
    launch_skinny<MODE>(pl, a, st);
    return;
  }
  dim3 grid(pl.gx, pl.gy, pl.gz);
  if (pl.bm == 128) {
    switch (pl.bn) {
      case 16: launch_cfg<MODE, 128, 16>(a, grid, st); break;
      case 32: launch_cfg<MODE, 128, 32>(a, grid, st); break;
      case 48: launch_cfg<MODE, 128, 48>(a, grid, st); break;
      case 64: launch_cfg<MODE, 128, 64>(a, grid, st); break;
      case 96: launch_cfg<MODE, 128, 96>(a, grid, st); break;
      default: launch_cfg<MODE, 128, 128>(a, grid, st); break;
    }
  } else {
    switch (pl.bn) {
      case 16: launch_cfg<MODE, 64, 16>(a, grid, st); break;
      case 32: launch_cfg<MODE, 64, 32>(a, grid, st); break;
      case 48: launch_cfg<MODE, 64, 48>(a, grid, st); break;
      case 64: launch_cfg<MODE, 64, 64>(a, grid, st); break;
      case 96: launch_cfg<MODE, 64, 96>(a, grid, st); break;
      default: launch_cfg<MODE, 64, 128>(a, grid, st); break;
    }
  }
}

static bool desc_ok(const tde_conv_desc_t* d) {
  if (!d) return false;
  if (d->N <= 0 || d->H <= 0 || d->W <= 0 || d->C <= 0 || d->OH <= 0 || d->OW <= 0 || d->K <= 0) return false;
  if (d->KH <= 0 || d->KW <= 0 || d->stride <= 0 || d->pad_top < 0 || d->pad_left < 0) return false;
  if (d->C % 4 || d->K % 4 || d->x_cstride % 4 || d->x_coff % 4 || d->y_cstride % 4 || d->y_coff % 4) return false;
  if (d->w_cin <= 0 || d->w_cin > d->C) return false;
  if (d->x_coff + d->C > d->x_cstride || d->y_coff + d->K > d->y_cstride) return false;
  return true;
}

static ConvArgs make_args(const tde_conv_desc_t& d) {
  ConvArgs a{};
  a.N = d.N; a.H = d.H; a.W = d.W; a.C = d.C; a.OH = d.OH; a.OW = d.OW; a.K = d.K;
  a.KH = d.KH; a.KW = d.KW; a.S = d.stride; a.PT = d.pad_top; a.PL = d.pad_left; a.wcin = d.w_cin;
  a.xcs = d.x_cstride; a.xco = d.x_coff; a.ycs = d.y_cstride; a.yco = d.y_coff;
  a.fC = make_fdiv(d.C); a.fK = make_fdiv(d.K); a.fKW = make_fdiv(d.KW); a.fOW = make_fdiv(d.OW);
  a.fOHW = make_fdiv(d.OH * d.OW);
  a.xmax = d.x_absmax; a.ymax = d.y_absmax; a.wmax = d.w_absmax;
  return a;
}

// Conv-kernel spans for bench.py's graph-timed roofline (tde_conv_span_arm): when the calling thread has armed a
// pair of device timestamp slots, the next conv entry call launches a one-wave stamp kernel right before its first
// conv-family kernel (GEMM, halo, halo-WGRAD or pixel-shuffle kernel) and one right after its last (split-K reduce
// included; the BatchNorm launches of a fused conv + BN call come after it).  Kernels of one stream (and dependent
// graph nodes) run one after another, so the two stamps bracket the call's kernels where a captured graph replays
// them.  (Timing events cannot serve: recording one inside the trainer's thread-local capture is refused,
// hipErrorStreamCaptureUnsupported.)  The stamp is the 100 MHz constant real-time counter.  Unarmed (always,
// outside bench's timing capture): no launch, no cost.
__global__ void __launch_bounds__(64) span_stamp_kernel(unsigned long long* slot) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) slot[threadIdx.x] = t;      // a per-lane (vector) address
}
static thread_local unsigned long long* g_span_slot[2] = {nullptr, nullptr};
static thread_local int g_span_marks = 0;
static void span_mark(int which, hipStream_t st) {
  if (g_span_slot[which] == nullptr) return;
  hipLaunchKernelGGL(span_stamp_kernel, dim3(1), dim3(64), 0, st, g_span_slot[which]);
  ++g_span_marks;
}

// Timing experiments only (results are garbage), compiled in ONLY by a diagnostic build (-DTDE_TIMING_DIAG; never
// in the shipped libtde.so, so no environment variable can make the product skip work -- VERDICT r03): skip every
// conv launch of layers whose forward output has <= / > this many pixels (TDE_SKIP_CONV_LE / _GT; TDE_SKIP_WHAT
// bit 0: GEMM kernels, bit 1: reduces), or every filter gradient (TDE_SKIP_WGRAD), to measure what they cost.
#ifdef TDE_TIMING_DIAG
static const long g_skip_le = env_long("TDE_SKIP_CONV_LE", -1);
static const long g_skip_gt = env_long("TDE_SKIP_CONV_GT", -1);
static const long g_skip_what = env_long("TDE_SKIP_WHAT", 3);
static const long g_skip_wgrad = env_long("TDE_SKIP_WGRAD", 0);
#else
static constexpr long g_skip_le = -1, g_skip_gt = -1, g_skip_what = 3, g_skip_wgrad = 0;
#endif
static bool skip_conv(const tde_conv_desc_t* d) {
  const long m = (long)d->N * d->OH * d->OW;
  return (g_skip_le >= 0 && m <= g_skip_le) || (g_skip_gt >= 0 && m > g_skip_gt);
}

// z-lanes per output quad (fill >= ~256 blocks, keep >= 4 splits per lane) and blocks of a split-K reduction
static void reduce_shape(const Plan& pl, int& zl, int& blocks) {
  const long n4 = (long)pl.rows * (pl.cols / 4);
  zl = 1;
  while (zl < 64 && (n4 * zl * 2 + 255) / 256 <= 256 && pl.splits / (zl * 2) >= 4) zl *= 2;
  long b = (n4 * zl + 255) / 256;
  blocks = (int)(b > 4096 ? 4096 : b);
}

template <int MODE>
static void launch_reduce(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  if (pl.splits <= 1) return;
  int zl, blocks;
  reduce_shape(pl, zl, blocks);
  hipLaunchKernelGGL(splitk_reduce_kernel<MODE>, dim3(blocks), dim3(256), 0, st, a, pl.rows, pl.cols, zl);
}

// The data- and filter-gradient reductions of a layer's backward: one launch when both GEMMs split K.
// (MODE2 = MODE_PSW: the pixel-shuffle filter gradient, whose slab is reduced -- and scattered -- even at one split)
template <int MODE1, int MODE2 = MODE_WGRAD>
static void launch_reduce2(const Plan& p1, const ConvArgs& a1, const Plan& p2, const ConvArgs& a2, hipStream_t st) {
  if (p1.splits <= 1 || (p2.splits <= 1 && MODE2 != MODE_PSW)) {
    launch_reduce<MODE1>(p1, a1, st);
    if constexpr (MODE2 == MODE_PSW) {
      int zl, blocks;
      reduce_shape(p2, zl, blocks);
      hipLaunchKernelGGL(splitk_reduce_kernel<MODE_PSW>, dim3(blocks), dim3(256), 0, st, a2, p2.rows, p2.cols, zl);
    } else {
      launch_reduce<MODE2>(p2, a2, st);
    }
    return;
  }
  int zl1, b1, zl2, b2;
  reduce_shape(p1, zl1, b1);
  reduce_shape(p2, zl2, b2);
  hipLaunchKernelGGL((splitk_reduce2_kernel<MODE1, MODE2>), dim3(b1 + b2), dim3(256), 0, st, a1, p1.rows, p1.cols, zl1, b1, a2,
                     p2.rows, p2.cols, zl2);
}

// Pixel-shuffle path of the stride-2 k x k virtual DGRAD (deconv forward, conv data gradient; MODE_PS above; k = 3,
// 5, 7).  TDE_DECONV_PS_MINM: input pixels (N x OH x OW) from which it replaces the four parity-class GEMMs (0:
// never).  Split-K never runs here (below that size the class GEMMs and their split-K remain).  The 5x5 / 7x7 forms
// (round 5: exp_upcnv1 / exp_upcnv2 forwards, cnv2's data gradient; before, 16 / 32-column class GEMMs) moved config
// 4 from 1077-1079 to 1092-1095 pairs/s (profiles/r05/ps_ab.md).
static const long g_ps_minm = env_long("TDE_DECONV_PS_MINM", 8192);
// ... and only with enough tiles to fill the chip (the class GEMMs have 4x the tiles and split K): >= 512 blocks of
// 128 rows, else >= 512 of 64 rows (measured, batch 8, us: upcnv1 48.2 -> 35.5 with 768 blocks of 128 rows;
// upcnv2 28.7 -> 29.7 with 192, upcnv3 32.8 -> 37.7 with 96, upcnv4 29.5 -> 57.3 with 24: r03x)
static const long g_ps_minblocks = env_long("TDE_DECONV_PS_MINBLOCKS", 512);

// The pixel-shuffle GEMM's tap window over the deconv input for a k x k kernel at pad pt: input row a - PW + th
// (th < T) feeds output row 2a + py through kernel row kh = kh0 + py - 2 th, kh0 = pt + 2 PW -- the union over
// py = 0, 1 of the rows a + (py + pt - kh) / 2 with kh = py + pt (mod 2), 0 <= kh < k.
struct PsWindow { int T, PW, kh0; };
static PsWindow ps_window(int k, int pt) {
  int lo = 1 << 20, hi = -(1 << 20);
  for (int py = 0; py < 2; ++py)
    for (int kh = 0; kh < k; ++kh)
      if (((py + pt - kh) & 1) == 0) {
        const int di = (py + pt - kh) / 2;
        lo = di < lo ? di : lo;
        hi = di > hi ? di : hi;
      }
  return PsWindow{hi - lo + 1, -lo, pt - 2 * lo};
}
static bool ps_ok(const tde_conv_desc_t& d, int* bm, int* bn) {
  if (!(g_ps_minm > 0 && g_conv_math == 4 && d.stride == 2 && d.KH == d.KW && (d.KH & 1) && d.KH <= 7 &&
        d.pad_top == d.pad_left && d.pad_top >= 0 && d.pad_top < d.KH && d.H == 2 * d.OH && d.W == 2 * d.OW &&
        d.w_cin == d.C && d.C % 16 == 0 && d.K % 4 == 0 && (long)d.N * d.OH * d.OW >= g_ps_minm))
    return false;
  const long M = (long)d.N * d.OH * d.OW;
  const int Nn = 4 * d.C, BN = Nn % 128 == 0 ? 128 : 64;
  int BM = 0;
  if ((long)tde_cdiv(M, 128) * (Nn / BN) >= g_ps_minblocks) BM = 128;
  else if ((long)tde_cdiv(M, 64) * (Nn / BN) >= g_ps_minblocks) BM = 64;
  if (!BM) return false;
  if (bm) *bm = BM;
  if (bn) *bn = BN;
  return true;
}

// The pixel-shuffle GEMM's arguments: the virtual DGRAD's input = a0.dy (view y of d, K channels), its output =
// a0.dx (view x of d, C channels).
static ConvArgs ps_args(const tde_conv_desc_t* d, const ConvArgs& a0, int accumulate) {
  ConvArgs a{};
  const PsWindow pw = ps_window(d->KH, d->pad_top);
  a.N = d->N; a.H = d->OH; a.W = d->OW; a.C = d->K; a.OH = d->OH; a.OW = d->OW; a.K = 4 * d->C;
  a.KH = pw.T; a.KW = pw.T; a.S = 1; a.PT = pw.PW; a.PL = pw.PW; a.wcin = d->K;
  a.xcs = d->y_cstride; a.xco = d->y_coff; a.ycs = d->x_cstride; a.yco = d->x_coff;
  a.fC = make_fdiv(d->K); a.fK = make_fdiv(4 * d->C); a.fKW = make_fdiv(pw.T); a.fOW = make_fdiv(d->OW);
  a.fOHW = make_fdiv(d->OH * d->OW);
  a.xmax = a0.ymax; a.wmax = a0.wmax;
  a.x = a0.dy; a.w = a0.w; a.y = a0.dx; a.bias = a0.bias; a.relu = a0.relu;
  a.ps_C = d->C; a.ps_H = d->H; a.ps_W = d->W; a.ps_K = d->K; a.ps_KS = d->KH; a.ps_kh0 = pw.kh0;
  a.fpsC = make_fdiv(d->C);
  a.splits = 1; a.kt_per = tde_cdiv((long)pw.T * pw.T * d->K, BK3); a.accumulate = accumulate;
  return a;
}

// One pixel-shuffle GEMM launch (register-staged tile).
static void launch_ps(ConvArgs& a, int BM, int BN, dim3 grid, hipStream_t st) {
  if (BM == 128 && BN == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PS, 128, 128, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else if (BM == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PS, 128, 64, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else if (BN == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PS, 64, 128, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((igemmx_kernel<4, MODE_PS, 64, 64, 2, 2, 1>), grid, dim3(NT), 0, st, a);
}

static int run_ps(const tde_conv_desc_t* d, const ConvArgs& a0, int accumulate, const tde_bn_train_t* bn, void* ws,
                  size_t ws_bytes, void* stream) {
  ConvArgs a = ps_args(d, a0, accumulate);
  const long M = (long)d->N * d->OH * d->OW, rows = (long)d->N * d->H * d->W;
  const int Nn = 4 * d->C;
  const int G = bn && bn->groups > 1 ? bn->groups : 1;
  if (rows % G != 0) return TDE_ERR_ARG;
  int BM = 0, BN = 0;
  ps_ok(*d, &BM, &BN);
  const dim3 grid(tde_cdiv(M, BM), Nn / BN, 1);
  // BN statistics from the epilogue (one record per (row tile, column tile)) when every row group is whole row tiles
  // and a tile covers whole classes; else a grouped partial pass over z
  const bool epi = bn && rows / G > BN_SMALL_M && (M % G == 0) && ((M / G) % BM == 0) && BN % d->C == 0;
  const size_t epi_bytes = (size_t)grid.x * grid.y * 2 * d->C * sizeof(double);
  const size_t part_bytes = bn ? std::max(bn_part_bytes(rows, d->C), epi ? epi_bytes : (size_t)0) : 0;
  if (bn && (!ws || !tde_aligned16(ws) || part_bytes > ws_bytes)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  double* part = bn ? reinterpret_cast<double*>(tde_ws_body(ws)) : nullptr;
  if (epi) {
    a.bnp = part;
    a.bn_gy = (int)grid.y;
  }
  span_mark(0, st);
  launch_ps(a, BM, BN, grid, st);
  span_mark(1, st);
  if (bn) {
    BnOut o{bn->beta, bn->eps, bn->decay, bn->bessel, bn->moving_mean, bn->moving_var, bn->save_mean,
                  bn->save_invstd, bn->y, bn->y_cstride, bn->y_coff, bn->relu, G, bn->sums};
    if (rows / G <= BN_SMALL_M) bn_fwd_small_launch((int)rows, d->C, a.y, o, part, st);
    else if (epi) bn_fwd_from_partials_launch((int)rows, d->C, a.y, (int)(grid.x * grid.y), part, o, st);
    else bn_fwd_standalone_launch((int)rows, d->C, a.y, o, part, st);
  }
  return tde_launch_status();
}

// Pixel-shuffle filter gradient (MODE_PSW) of a stride-2 k x k layer with the MODE_PS geometry (k = 3, 5, 7; no
// ps_ok tile-count rule: the reduction over every dy pixel splits K) from TDE_PSW_MINM dy pixels (0: never), for
// 16 input channels only: measured per layer at config 4's twin batch (scripts/conv_micro.py, profiles/r05/psw_micro.txt)
// it wins for the 16-channel deconvs -- upcnv1 71.5 -> 58.6 us, exp_upcnv1 173 -> 137 us, whose direct GEMM is
// k^2 x 16 rows by 32 columns -- and loses for 8 / 32 / 64 channels (cnv1 110 -> 138, upcnv3 35 -> 40 us).
static const long g_psw_minm = env_long("TDE_PSW_MINM", 8192);
static bool psw_ok(const tde_conv_desc_t& d) {
  return g_psw_minm > 0 && g_conv_math == 4 && d.C == 16 && d.stride == 2 && d.KH == d.KW && (d.KH & 1) && d.KH <= 7 &&
         d.pad_top == d.pad_left && d.pad_top >= 0 && d.pad_top < d.KH && d.H == 2 * d.OH && d.W == 2 * d.OW &&
         d.w_cin == d.C && (long)d.N * d.OH * d.OW >= g_psw_minm;
}
// rows 4 C, columns T^2 K, K = dy pixels; 64-row tiles for 4 C <= 64, 64 / 128 columns by make_plan's cost rule,
// split-K to make_plan's block target.  Every tile writes the slab (splits >= 1), the reduce scatters.
static Plan psw_plan(const tde_conv_desc_t& d) {
  const PsWindow pw = ps_window(d.KH, d.pad_top);
  const long M = 4L * d.C, Nn = (long)pw.T * pw.T * d.K, Kd = (long)d.N * d.OH * d.OW;
  Plan pl{};
  pl.bm = M <= 64 ? 64 : 128;
  pl.bn = (tde_cdiv(Nn, 64) * 88 < tde_cdiv(Nn, 128) * 152) ? 64 : 128;
  const long tiles = tde_cdiv(M, pl.bm) * tde_cdiv(Nn, pl.bn);
  const int nkt = tde_cdiv(Kd, BK3);
  long splits = tiles < g_split_target ? (g_split_target + tiles - 1) / tiles : 1;
  if (splits > nkt / g_split_minkt) splits = nkt / g_split_minkt;
  if (splits < 1) splits = 1;
  if (splits > 512) splits = 512;
  while (splits > 1 && splits * M * Nn * 4 > g_split_slab) splits /= 2;
  pl.kt_per = tde_cdiv(nkt, (int)splits);
  pl.splits = tde_cdiv(nkt, pl.kt_per);
  pl.gx = (int)tde_cdiv(M, pl.bm); pl.gy = (int)tde_cdiv(Nn, pl.bn); pl.gz = pl.splits;
  pl.rows = (int)M; pl.cols = (int)Nn;
  pl.slab_bytes = (size_t)pl.splits * M * Nn * sizeof(float);
  pl.ws_bytes = pl.slab_bytes;
  return pl;
}
// The PSW GEMM's arguments from the layer's filter-gradient arguments (x, dy, dw, accumulate of the virtual conv).
static ConvArgs psw_args(const tde_conv_desc_t* d, const ConvArgs& a0, const Plan& pl) {
  const PsWindow pw = ps_window(d->KH, d->pad_top);
  ConvArgs a = a0;
  a.KH = 2; a.KW = 2; a.S = 2; a.PT = 0; a.PL = 0; a.fKW = make_fdiv(2);
  a.ps_T = pw.T; a.ps_PW = pw.PW; a.ps_KS = d->KH; a.ps_kh0 = pw.kh0; a.fpsT = make_fdiv(pw.T);
  a.splits = pl.splits; a.kt_per = pl.kt_per; a.bnp = nullptr;
  return a;
}
static void launch_psw(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  const dim3 grid(pl.gx, pl.gy, pl.gz);
  if (pl.bm == 128 && pl.bn == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PSW, 128, 128, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else if (pl.bm == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PSW, 128, 64, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else if (pl.bn == 128) hipLaunchKernelGGL((igemmx_kernel<4, MODE_PSW, 64, 128, 2, 2, 1>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((igemmx_kernel<4, MODE_PSW, 64, 64, 2, 2, 1>), grid, dim3(NT), 0, st, a);
}
static void launch_psw_reduce(const Plan& pl, const ConvArgs& a, hipStream_t st) {
  int zl, blocks;
  reduce_shape(pl, zl, blocks);
  hipLaunchKernelGGL(splitk_reduce_kernel<MODE_PSW>, dim3(blocks), dim3(256), 0, st, a, pl.rows, pl.cols, zl);
}

template <int MODE>
static int run(const tde_conv_desc_t* d, ConvArgs a, int accumulate, const tde_bn_train_t* bn, void* ws,
               size_t ws_bytes, void* stream) {
  if constexpr (MODE == MODE_DGRAD) {
    if (ps_ok(*d) && !skip_conv(d)) return run_ps(d, a, accumulate, bn, ws, ws_bytes, stream);
  }
  const bool skipm = skip_conv(d);
  const bool skip = skipm && (g_skip_what & 1), skipr = skipm && (g_skip_what & 2);
  HwgPlan wp;
  if (MODE == MODE_WGRAD && hwg_plan(*d, wp, g_conv_math)) {
    // narrow, high-resolution layer (stride 1, or stride 2 over few input channels): halo-tiled filter gradient (halo_wgrad.hip)
    if (wp.part_bytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
    span_mark(0, static_cast<hipStream_t>(stream));
    if (!skip) hwg_launch(wp, *d, a.x, a.dy, a.dw, accumulate, tde_ws_body(ws), static_cast<hipStream_t>(stream));
    span_mark(1, static_cast<hipStream_t>(stream));
    return tde_launch_status();
  }
  if (MODE == MODE_WGRAD && psw_ok(*d)) {
    const Plan pl = psw_plan(*d);
    if (pl.ws_bytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
    a.ws = reinterpret_cast<float*>(tde_ws_body(ws));
    a.accumulate = accumulate;
    const ConvArgs ap = psw_args(d, a, pl);
    hipStream_t st = static_cast<hipStream_t>(stream);
    span_mark(0, st);
    if (!skip) launch_psw(pl, ap, st);
    if (!skipr) launch_psw_reduce(pl, ap, st);
    span_mark(1, st);
    return tde_launch_status();
  }
  HaloPlan hp;
  if (MODE != MODE_WGRAD && halo_plan(*d, MODE == MODE_FWD ? 0 : 1, g_conv_math, hp)) {
    // stride-1, few-channel, high-resolution layer: halo-tiled kernel (halo_conv.hip)
    const int G = bn && bn->groups > 1 ? bn->groups : 1;
    const long Mz = (long)d->N * (MODE == MODE_FWD ? (long)d->OH * d->OW : (long)d->H * d->W);
    // halo partials are image-major (one per pixel tile of one image): group-aligned when G divides N
    if (Mz % G != 0) return TDE_ERR_ARG;
    const bool grouped_sa = G > 1 && (d->N % G != 0 || Mz / G <= BN_SMALL_M);
    size_t pbytes = bn ? (size_t)hp.nparts * 2 * hp.Ncols * sizeof(double) : 0;
    if (bn && bn_part_bytes(Mz, hp.Ncols) > pbytes) pbytes = bn_part_bytes(Mz, hp.Ncols);
    if (hp.wbytes + pbytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
    char* body = tde_ws_body(ws);
    double* part = bn ? reinterpret_cast<double*>(body + hp.wbytes) : nullptr;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const float* in = MODE == MODE_FWD ? a.x : a.dy;
    float* z = MODE == MODE_FWD ? a.y : a.dx;
    span_mark(0, st);
    if (!skip) halo_launch(hp, *d, in, a.w, z, accumulate, body, grouped_sa ? nullptr : part, st, a.bias, a.relu);
    span_mark(1, st);
    if (bn) {
      BnOut o{bn->beta, bn->eps, bn->decay, bn->bessel, bn->moving_mean, bn->moving_var, bn->save_mean,
                    bn->save_invstd, bn->y, bn->y_cstride, bn->y_coff, bn->relu, G, bn->sums};
      if (grouped_sa) bn_fwd_standalone_launch((int)Mz, hp.Ncols, z, o, part, st);
      else bn_fwd_from_partials_launch((int)Mz, hp.Ncols, z, hp.nparts, part, o, st);
    }
    return tde_launch_status();
  }
  const Plan pl = make_plan(*d, MODE);
  BnPlan bp{};
  const int G = bn && bn->groups > 1 ? bn->groups : 1;
  if (pl.rows % G != 0) return TDE_ERR_ARG;
  if (bn) bp = bn_plan(*d, MODE, pl, G);
  if (pl.ws_bytes + bp.part_bytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  char* body = tde_ws_body(ws);
  double* part = reinterpret_cast<double*>(body + pl.slab_bytes);
  a.ws = reinterpret_cast<float*>(body);
  a.splits = pl.splits;
  a.kt_per = pl.kt_per;
  a.accumulate = accumulate;
  a.bnp = (bn && bp.path == BN_EPI) ? part : nullptr;
  a.bn_gx = pl.gx;
  a.bn_G = G;
  hipStream_t st = static_cast<hipStream_t>(stream);
  span_mark(0, st);
  if (!skip) launch_mode<MODE>(pl, a, st);
  float* z = MODE == MODE_FWD ? a.y : (MODE == MODE_DGRAD ? a.dx : a.dw);
  if (!skipr && !(bn && bp.path == BN_REDUCE)) launch_reduce<MODE>(pl, a, st);
  if (bn && bp.path == BN_REDUCE && !skipr)
    hipLaunchKernelGGL(splitk_reduce_bn_kernel, dim3(bp.ch.chunks, bp.ch.groups), dim3(256), 0, st, a.ws, pl.splits,
                       pl.rows, pl.cols, z, bp.ch, part);
  span_mark(1, st);
  if (bn) {
    // slim.batch_norm + ReLU of z (nets_optflow_depth.py:82-87)
    BnOut o{bn->beta, bn->eps, bn->decay, bn->bessel, bn->moving_mean, bn->moving_var, bn->save_mean,
                  bn->save_invstd, bn->y, bn->y_cstride, bn->y_coff, bn->relu, G, bn->sums};
    if (bp.path == BN_SMALL) {
      bn_fwd_small_launch(pl.rows, pl.cols, z, o, part, st);
    } else if (bp.path == BN_STANDALONE) {
      bn_fwd_standalone_launch(pl.rows, pl.cols, z, o, part, st);
    } else {
      bn_fwd_from_partials_launch(pl.rows, pl.cols, z, bp.nparts, part, o, st);
    }
  }
  return tde_launch_status();
}

template <int MODE1, int BM, int BN>
static void launch_bwd2_cfg(const Plan& p1, const ConvArgs& a1, const Plan& p2, const ConvArgs& a2, hipStream_t st) {
  constexpr int WN = BN % TDE_WN_DIV == 0 ? 2 : 1;
  constexpr int WM = 4 / WN;
  const int nd = p1.gx * p1.gy * p1.gz, nw = p2.gx * p2.gy * p2.gz;
  const int math = tile_math(BN);
  if (math == 2)
    hipLaunchKernelGGL((igemm_bwd2_kernel<2, MODE1, BM, BN, WM, WN>), dim3(nd + nw), dim3(NT), 0, st, a1, a2, p1.gx,
                       p1.gy, p2.gx, p2.gy, nd);
  else if (math == 3)
    hipLaunchKernelGGL((igemm_bwd2_kernel<3, MODE1, BM, BN, WM, WN>), dim3(nd + nw), dim3(NT), 0, st, a1, a2, p1.gx,
                       p1.gy, p2.gx, p2.gy, nd);
  else if (math == 4)
    hipLaunchKernelGGL((igemm_bwd2_kernel<4, MODE1, BM, BN, WM, WN>), dim3(nd + nw), dim3(NT), 0, st, a1, a2, p1.gx,
                       p1.gy, p2.gx, p2.gy, nd);
  else
    hipLaunchKernelGGL((igemm_bwd2_kernel<0, MODE1, BM, BN, WM, WN>), dim3(nd + nw), dim3(NT), 0, st, a1, a2, p1.gx,
                       p1.gy, p2.gx, p2.gy, nd);
}

template <int MODE1>
static void launch_bwd2(const Plan& p1, const ConvArgs& a1, const Plan& p2, const ConvArgs& a2, hipStream_t st) {
  switch (p1.bm * 1000 + p1.bn) {
#define BWD2_CASE(BM_, BN_) case BM_ * 1000 + BN_: launch_bwd2_cfg<MODE1, BM_, BN_>(p1, a1, p2, a2, st); break;
    BWD2_CASE(128, 16) BWD2_CASE(128, 32) BWD2_CASE(128, 48) BWD2_CASE(128, 64) BWD2_CASE(128, 96)
    BWD2_CASE(128, 128) BWD2_CASE(64, 16) BWD2_CASE(64, 32) BWD2_CASE(64, 48) BWD2_CASE(64, 64)
    BWD2_CASE(64, 96) BWD2_CASE(64, 128)
#undef BWD2_CASE
    default: break;
  }
}

static const long g_bwd_fuse = env_long("TDE_BWD_FUSE", 1);   // 0: two launches (A/B experiments)



// Data + filter gradient of one layer.  MODE1 = the data-gradient GEMM of the virtual conv (DGRAD for a
// conv, FWD for a deconv); the filter gradient is always its WGRAD.  One fused launch when the data
// gradient's tile fits the filter gradient (re-planned on that tile), then the split-K reduces.
template <int MODE1>
static int run_bwd(const tde_conv_desc_t* d, ConvArgs a1, int acc1, ConvArgs a2, int acc2, void* ws, size_t ws_bytes,
                   void* stream) {
  const bool skipm = skip_conv(d);
  const bool skip = skipm && (g_skip_what & 1), skipr = skipm && (g_skip_what & 2);
  HaloPlan hp;
  HwgPlan wp;
  if (MODE1 == MODE_DGRAD && d->stride == 1 && hwg_plan(*d, wp, g_conv_math)) {
    // filter gradient on the halo-tiled WGRAD kernel; data gradient on the halo path or the implicit GEMM
    hipStream_t st = static_cast<hipStream_t>(stream);
    const bool hd = halo_plan(*d, 1, g_conv_math, hp);
    const Plan p1 = hd ? Plan{} : make_plan(*d, MODE1);
    const size_t b1 = hd ? hp.wbytes : p1.slab_bytes;
    if (b1 + wp.part_bytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
    char* body = tde_ws_body(ws);
    if (hd) {
      if (!skip) halo_launch(hp, *d, a1.dy, a1.w, a1.dx, acc1, body, nullptr, st);
    } else {
      a1.ws = reinterpret_cast<float*>(body);
      a1.splits = p1.splits; a1.kt_per = p1.kt_per; a1.accumulate = acc1; a1.bnp = nullptr;
      if (!skip) launch_mode<MODE1>(p1, a1, st);
      if (!skipr) launch_reduce<MODE1>(p1, a1, st);
    }
    if (!skip && !g_skip_wgrad) hwg_launch(wp, *d, a2.x, a2.dy, a2.dw, acc2, body + b1, st);
    return tde_launch_status();
  }
  if (MODE1 == MODE_DGRAD && halo_plan(*d, 1, g_conv_math, hp)) {
    // data gradient on the halo path, filter gradient on the implicit GEMM (two launches + its reduce)
    const Plan p2 = make_plan(*d, MODE_WGRAD);
    if (hp.wbytes + p2.slab_bytes > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
    char* body = tde_ws_body(ws);
    a2.ws = reinterpret_cast<float*>(body + hp.wbytes);
    a2.splits = p2.splits; a2.kt_per = p2.kt_per; a2.accumulate = acc2; a2.bnp = nullptr;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (!skip) {
      halo_launch(hp, *d, a1.dy, a1.w, a1.dx, acc1, body, nullptr, st);
      if (!g_skip_wgrad) launch_mode<MODE_WGRAD>(p2, a2, st);
    }
    if (!skipr && !g_skip_wgrad) launch_reduce<MODE_WGRAD>(p2, a2, st);
    return tde_launch_status();
  }
  // a stride-2 conv whose data gradient fits the pixel-shuffle GEMM (ps_ok: the high-resolution 3x3 / 5x5 / 7x7 layers)
  // runs it as one 4 x C-wide launch without split-K, then the filter gradient as its own launch (config 4, cnv2's
  // 5x5: 1090 -> 1092-1095 pairs/s against the fused class-GEMM launch, profiles/r05/ps_ab.md); else the fused data +
  // filter gradient launch
  Plan p1;
  int pbm = 0, pbn = 0;
  const bool ps1 = MODE1 == MODE_DGRAD && ps_ok(*d, &pbm, &pbn);
  if (ps1) {
    p1 = Plan{};
    p1.bm = pbm; p1.bn = pbn; p1.splits = 1; p1.gz = 1;
    p1.gx = (int)tde_cdiv((long)d->N * d->OH * d->OW, pbm); p1.gy = 4 * d->C / pbn;
  } else {
    p1 = make_plan(*d, MODE1);
  }
  // the filter gradient of a stride-2 layer on the halo-tiled kernel (few input channels: hwg_plan) or in the
  // pixel-shuffle form (MODE_PSW) where they apply
  const bool hw2 = !g_skip_wgrad && d->stride == 2 && hwg_plan(*d, wp, g_conv_math);
  const bool psw2 = !g_skip_wgrad && !hw2 && psw_ok(*d);
  // fused data + filter gradient launch only when the filter gradient is an implicit GEMM and the data gradient is
  // not a pixel-shuffle GEMM
  const bool fuse = !ps1 && !psw2 && !hw2 && g_bwd_fuse != 0 && g_conv_math != 1 && p1.skinny_tm == 0 &&
                    !g_skip_wgrad;
  const Plan p2 = hw2 ? Plan{} : psw2 ? psw_plan(*d) : make_plan(*d, MODE_WGRAD, fuse ? p1.bm : 0, fuse ? p1.bn : 0);
  const size_t b2 = hw2 ? wp.part_bytes : p2.slab_bytes;
  if (p1.slab_bytes + b2 > ws_bytes || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  char* body = tde_ws_body(ws);
  a1.ws = reinterpret_cast<float*>(body);
  a1.splits = p1.splits; a1.kt_per = p1.kt_per; a1.accumulate = acc1; a1.bnp = nullptr;
  a2.ws = reinterpret_cast<float*>(body + p1.slab_bytes);
  a2.splits = p2.splits; a2.kt_per = p2.kt_per; a2.accumulate = acc2; a2.bnp = nullptr;
  const ConvArgs a2p = psw2 ? psw_args(d, a2, p2) : a2;
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto wgrad = [&] {
    if (g_skip_wgrad) return;
    if (hw2) hwg_launch(wp, *d, a2.x, a2.dy, a2.dw, acc2, body + p1.slab_bytes, st);   // + its chunk reduce
    else if (psw2) launch_psw(p2, a2p, st);
    else launch_mode<MODE_WGRAD>(p2, a2, st);
  };
  if (skip) {
  } else if (ps1) {
    ConvArgs ap = ps_args(d, a1, acc1);
    launch_ps(ap, p1.bm, p1.bn, dim3(p1.gx, p1.gy, 1), st);
    wgrad();
  } else if (fuse) {
    launch_bwd2<MODE1>(p1, a1, p2, a2, st);
  } else {
    launch_mode<MODE1>(p1, a1, st);
    wgrad();
  }
  if (!skipr) {
    if (g_skip_wgrad || hw2) launch_reduce<MODE1>(p1, a1, st);
    else if (psw2) launch_reduce2<MODE1, MODE_PSW>(p1, a1, p2, a2p, st);
    else launch_reduce2<MODE1>(p1, a1, p2, a2, st);
  }
  return tde_launch_status();
}

static size_t bwd_ws_bytes(const tde_conv_desc_t& d, int mode1) {
  const Plan p1 = make_plan(d, mode1);
  const size_t fused = p1.skinny_tm ? 0 : p1.slab_bytes + make_plan(d, MODE_WGRAD, p1.bm, p1.bn).slab_bytes;
  const size_t split = p1.slab_bytes + make_plan(d, MODE_WGRAD).slab_bytes;
  size_t b = fused > split ? fused : split;
  {
    const size_t w2 = make_plan(d, MODE_WGRAD).slab_bytes;
    if (p1.slab_bytes + w2 > b) b = p1.slab_bytes + w2;
    if (psw_ok(d)) {
      // the pixel-shuffle filter gradient beside any data gradient above
      const size_t r = p1.slab_bytes + psw_plan(d).slab_bytes;
      if (r > b) b = r;
    }
  }
  const size_t h = mode1 == MODE_DGRAD ? halo_ws_bytes(d, MODE_DGRAD, false) : 0;
  if (h) {
    const size_t w2 = make_plan(d, MODE_WGRAD).slab_bytes;
    if (h + w2 > b) b = h + w2;
  }
  const size_t hw = hwg_ws_bytes(d);
  if (hw) {
    const size_t b1 = h > p1.slab_bytes ? h : p1.slab_bytes;   // halo or igemm data gradient (math-dependent)
    if (b1 + hw > b) b = b1 + hw;
  }
  return b + 64;
}

static bool bn_ok(const tde_bn_train_t* bn, int C) {
  return bn && bn->beta && bn->save_mean && bn->save_invstd && bn->y && C <= 1024 && bn->groups >= 0 &&
         bn->groups <= BN_MAX_GROUPS &&
         ((bn->moving_mean == nullptr) == (bn->moving_var == nullptr)) && bn->y_cstride % 4 == 0 &&
         bn->y_coff % 4 == 0 && bn->y_coff + C <= bn->y_cstride && tde_aligned16(bn->y) && tde_aligned16(bn->beta);
}

}  // namespace

// Gradient-operand bound for fp16x3 (conv math 4) when the caller passes none: the split scales each operand by
// a power of two from its bound, and an unscaled gradient (|dy| ~ 1e-6) would keep only ~2^-25 absolute precision.
// One pre-pass (16 blocks, each the max|.| of a strided share of the view into its own slot: no atomics) writes
// the bound into the last 256 bytes of the caller's workspace, past everything the conv plans use (every
// workspace query includes them: with_bound_scratch).
static size_t with_bound_scratch(size_t n) { return (n + 255) / 256 * 256 + 256; }

__global__ void __launch_bounds__(256) operand_absmax_kernel(long quads, int cq, const float* p, int cs, int co,
                                                             float* out) {
  __shared__ float sm[4];
  float m = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < quads; i += 256L * gridDim.x) {
    const long r = i / cq;
    const int q = (int)(i - r * cq);
    const f4 v = *reinterpret_cast<const f4*>(p + r * cs + co + 4 * q);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
  __syncthreads();
  // |values| >= 0 order as their bit patterns: an unsigned max into one of the TDE_BOUND_SLOTS slots (zeroed
  // before the launch), spread over the slots so few blocks meet on one address
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned*>(out) + (blockIdx.x & (TDE_BOUND_SLOTS - 1)),
              __float_as_uint(fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]))));
}

// db = *d, with the gradient operand's bound (view 1: y of d; view 0: x of d) computed when math 4 needs one
// and the caller gave none.
static int bound_grad_operand(const tde_conv_desc_t* d, tde_conv_desc_t& db, int yview, const float* g, void* ws,
                              size_t ws_bytes, void* stream) {
  db = *d;
  const float* have = yview ? d->y_absmax : d->x_absmax;
  if (g_conv_math != 4 || have != nullptr) return TDE_OK;
  if (!ws || ws_bytes < 256 + 64 || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  float* slot = reinterpret_cast<float*>(static_cast<char*>(ws) + ((ws_bytes - 256) & ~(size_t)15));
  const long rows = yview ? (long)d->N * d->OH * d->OW : (long)d->N * d->H * d->W;
  const int C = yview ? d->K : d->C;
  const int cs = yview ? d->y_cstride : d->x_cstride, co = yview ? d->y_coff : d->x_coff;
  static_assert((TDE_BOUND_SLOTS & (TDE_BOUND_SLOTS - 1)) == 0, "slot spread mask");
  // ~4 quads per lane, at least one block per slot, at most 1024 blocks (the first version used one block per
  // slot: 350 us for a 67 MB dy)
  const long quads = rows * (C / 4);
  const int blocks = (int)std::min(1024L, std::max((long)TDE_BOUND_SLOTS, (long)tde_cdiv(quads, 1024L)));
  const hipError_t me = hipMemsetAsync(slot, 0, TDE_BOUND_SLOTS * sizeof(float), static_cast<hipStream_t>(stream));
  if (me != hipSuccess) return TDE_ERR_HIP;
  hipLaunchKernelGGL(operand_absmax_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     quads, C / 4, g, cs, co, slot);
  if (yview) db.y_absmax = slot; else db.x_absmax = slot;
  return tde_launch_status();
}

extern "C" {

int tde_set_conv_math(int mode) {
  tde_clear_error();
  if (mode < 0 || mode > 4) return TDE_ERR_ARG;
  g_conv_math = mode;
  return TDE_OK;
}

int tde_get_conv_math(void) { return g_conv_math; }

size_t tde_conv2d_split_weights_size(const tde_conv_desc_t* d, int op) {
  if (!desc_ok(d) || op < 0 || op > 3) return 0;
  HaloPlan hp;
  if (halo_plan(*d, op & 1, g_conv_math, hp)) return hp.wbytes;
  return 0;
}

int tde_conv2d_split_weights(int n, const tde_conv_desc_t* const* descs, const int* ops, const float* const* weights,
                             void* const* outs, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(n >= 0 && (n == 0 || (descs && ops && weights && outs)));
  // halo-path images (halo_wprep_batch), one batched launch
  std::vector<HaloPlan> hps;
  std::vector<const tde_conv_desc_t*> hd;
  std::vector<const float*> hw;
  std::vector<void*> ho;
  for (int i = 0; i < n; ++i) {
    TDE_CHECK_ARG(desc_ok(descs[i]) && ops[i] >= 0 && ops[i] <= 3 && weights[i] && outs[i] && tde_aligned16(outs[i]));
    HaloPlan hp;
    if (halo_plan(*descs[i], ops[i] & 1, g_conv_math, hp)) {
      hps.push_back(hp); hd.push_back(descs[i]); hw.push_back(weights[i]); ho.push_back(outs[i]);
    } else {
      return TDE_ERR_ARG;   // a layer / op that takes no split (tde_conv2d_split_weights_size == 0): the caller's error
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!hps.empty()) halo_wprep_batch((int)hps.size(), hps.data(), hd.data(), hw.data(), ho.data(), st);
  return tde_launch_status();
}

size_t tde_conv2d_workspace_size(const tde_conv_desc_t* d, int op) {
  // op 3 = forward + batch norm + ReLU (tde_conv2d_fwd_bn)
  if (!desc_ok(d) || op < 0 || op > 3) return 0;
  return with_bound_scratch(
      plan_ws_bytes(*d, op == 0 || op == 3 ? MODE_FWD : (op == 1 ? MODE_DGRAD : MODE_WGRAD), op == 3));
}

size_t tde_deconv2d_workspace_size(const tde_conv_desc_t* d, int op) {
  // deconv fwd = DGRAD, bwd_data = FWD, bwd_filter = WGRAD of the virtual conv; op 3 = fwd + BN + ReLU
  if (!desc_ok(d) || op < 0 || op > 3) return 0;
  return with_bound_scratch(
      plan_ws_bytes(*d, op == 0 || op == 3 ? MODE_DGRAD : (op == 1 ? MODE_FWD : MODE_WGRAD), op == 3));
}

int tde_conv2d_fwd(const tde_conv_desc_t* d, const float* x, const float* w, float* y, int accumulate,
                   void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x) && tde_aligned16(w) && tde_aligned16(y));
  ConvArgs a = make_args(*d);
  a.x = x; a.w = w; a.y = y;
  return run<MODE_FWD>(d, a, accumulate, nullptr, ws, ws_bytes, stream);
}

int tde_conv2d_fwd_bn(const tde_conv_desc_t* d, const float* x, const float* w, float* z, const tde_bn_train_t* bn,
                      void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x) && tde_aligned16(w) && tde_aligned16(z) && bn_ok(bn, d->K));
  TDE_CHECK_ARG(d->y_cstride == d->K && d->y_coff == 0);   // z is the dense pre-BN output
  ConvArgs a = make_args(*d);
  a.x = x; a.w = w; a.y = z;
  return run<MODE_FWD>(d, a, 0, bn, ws, ws_bytes, stream);
}

int tde_conv2d_bwd_data(const tde_conv_desc_t* d, const float* dy, const float* w, float* dx, int accumulate,
                        void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(dy) && tde_aligned16(w) && tde_aligned16(dx));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 1, dy, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a = make_args(db);
  a.dy = dy; a.w = w; a.dx = dx;
  return run<MODE_DGRAD>(&db, a, accumulate, nullptr, ws, ws_bytes, stream);
}

int tde_conv2d_bwd_filter(const tde_conv_desc_t* d, const float* x, const float* dy, float* dw, int accumulate,
                          void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x) && tde_aligned16(dy) && tde_aligned16(dw));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 1, dy, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a = make_args(db);
  a.x = x; a.dy = dy; a.dw = dw;
  return run<MODE_WGRAD>(&db, a, accumulate, nullptr, ws, ws_bytes, stream);
}

int tde_deconv2d_fwd(const tde_conv_desc_t* d, const float* x_small, const float* w, float* y_big,
                     int accumulate, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  // the deconv input is an activation (no gradient-operand bound needed): the virtual DGRAD directly
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x_small) && tde_aligned16(w) && tde_aligned16(y_big));
  ConvArgs a = make_args(*d);
  a.dy = x_small; a.w = w; a.dx = y_big;
  return run<MODE_DGRAD>(d, a, accumulate, nullptr, ws, ws_bytes, stream);
}

// Folded-BN inference conv: y = relu?(conv(x, w_folded) + bias) into the y view of d.
int tde_conv2d_fwd_bias_act(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias, int relu,
                            float* y, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x) && tde_aligned16(w) && tde_aligned16(y) && (relu == 0 || relu == 1));
  ConvArgs a = make_args(*d);
  a.x = x; a.w = w; a.y = y; a.bias = bias; a.relu = relu;
  return run<MODE_FWD>(d, a, 0, nullptr, ws, ws_bytes, stream);
}

int tde_deconv2d_fwd_bias_act(const tde_conv_desc_t* d, const float* x_small, const float* w, const float* bias,
                              int relu, float* y_big, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x_small) && tde_aligned16(w) && tde_aligned16(y_big) &&
                (relu == 0 || relu == 1) && d->w_cin == d->C);
  ConvArgs a = make_args(*d);
  a.dy = x_small; a.w = w; a.dx = y_big; a.bias = bias; a.relu = relu;
  return run<MODE_DGRAD>(d, a, 0, nullptr, ws, ws_bytes, stream);
}

int tde_deconv2d_fwd_bn(const tde_conv_desc_t* d, const float* x_small, const float* w, float* z_big,
                        const tde_bn_train_t* bn, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x_small) && tde_aligned16(w) && tde_aligned16(z_big) && bn_ok(bn, d->C));
  TDE_CHECK_ARG(d->x_cstride == d->C && d->x_coff == 0);   // z is the dense pre-BN output
  ConvArgs a = make_args(*d);
  a.dy = x_small; a.w = w; a.dx = z_big;
  return run<MODE_DGRAD>(d, a, 0, bn, ws, ws_bytes, stream);
}

size_t tde_conv2d_bwd_workspace_size(const tde_conv_desc_t* d) {
  return desc_ok(d) ? with_bound_scratch(bwd_ws_bytes(*d, MODE_DGRAD)) : 0;
}

size_t tde_deconv2d_bwd_workspace_size(const tde_conv_desc_t* d) {
  return desc_ok(d) ? with_bound_scratch(bwd_ws_bytes(*d, MODE_FWD)) : 0;
}

int tde_conv2d_bwd(const tde_conv_desc_t* d, const float* x, const float* dy, const float* w, float* dx,
                   int accumulate_dx, float* dw, int accumulate_dw, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(x) && tde_aligned16(dy) && tde_aligned16(w) && tde_aligned16(dx) &&
                tde_aligned16(dw));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 1, dy, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a1 = make_args(db), a2 = make_args(db);
  a1.dy = dy; a1.w = w; a1.dx = dx;
  a2.x = x; a2.dy = dy; a2.dw = dw;
  span_mark(0, static_cast<hipStream_t>(stream));
  const int r = run_bwd<MODE_DGRAD>(&db, a1, accumulate_dx, a2, accumulate_dw, ws, ws_bytes, stream);
  span_mark(1, static_cast<hipStream_t>(stream));
  return r;
}

int tde_deconv2d_bwd(const tde_conv_desc_t* d, const float* dy_big, const float* x_small, const float* w,
                     float* dx_small, int accumulate_dx, float* dw, int accumulate_dw, void* ws, size_t ws_bytes,
                     void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(dy_big) && tde_aligned16(x_small) && tde_aligned16(w) &&
                tde_aligned16(dx_small) && tde_aligned16(dw));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 0, dy_big, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a1 = make_args(db), a2 = make_args(db);
  a1.x = dy_big; a1.w = w; a1.y = dx_small;          // data gradient = Conv2D(dy_big) (virtual FWD)
  a2.x = dy_big; a2.dy = x_small; a2.dw = dw;        // filter gradient (virtual WGRAD)
  span_mark(0, static_cast<hipStream_t>(stream));
  const int r = run_bwd<MODE_FWD>(&db, a1, accumulate_dx, a2, accumulate_dw, ws, ws_bytes, stream);
  span_mark(1, static_cast<hipStream_t>(stream));
  return r;
}

int tde_deconv2d_bwd_data(const tde_conv_desc_t* d, const float* dy_big, const float* w, float* dx_small,
                          int accumulate, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(dy_big) && tde_aligned16(w) && tde_aligned16(dx_small));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 0, dy_big, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a = make_args(db);   // the virtual conv's forward, in a data-gradient role
  a.x = dy_big; a.w = w; a.y = dx_small;
  return run<MODE_FWD>(&db, a, accumulate, nullptr, ws, ws_bytes, stream);
}

int tde_deconv2d_bwd_filter(const tde_conv_desc_t* d, const float* dy_big, const float* x_small, float* dw,
                            int accumulate, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(desc_ok(d) && tde_aligned16(dy_big) && tde_aligned16(x_small) && tde_aligned16(dw));
  tde_conv_desc_t db;
  const int rc = bound_grad_operand(d, db, 0, dy_big, ws, ws_bytes, stream);
  if (rc != TDE_OK) return rc;
  ConvArgs a = make_args(db);
  a.x = dy_big; a.dy = x_small; a.dw = dw;
  return run<MODE_WGRAD>(&db, a, accumulate, nullptr, ws, ws_bytes, stream);
}

int tde_stamp(unsigned long long* slot, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(slot != nullptr);
  hipLaunchKernelGGL(span_stamp_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), slot);
  return tde_launch_status();
}

// bench.py's graph-timed roofline: arm the calling thread's conv-kernel span stamp slots (device uint64, 8-byte
// aligned; null, null disarms).  Returns how many stamps the previous arming launched (2 after one conv entry call).
int tde_conv_span_arm(unsigned long long* stamp_begin, unsigned long long* stamp_end) {
  tde_clear_error();
  const int n = g_span_marks;
  g_span_slot[0] = stamp_begin;
  g_span_slot[1] = stamp_end;
  g_span_marks = 0;
  return n;
}

}  // extern "C"
