// Halo-tiled filter gradient (TF Conv2DBackpropFilter) of the stride-1, narrow (K <= 32 output channels),
// high-resolution layers: cnv1b 7x7 32->32 @96x128, icnv1 3x3 17->16 @192x256, icnv2 3x3 65->32 @96x128
// (nets_optflow_depth.py:89,141,134).
//
// dW[kh][kw][c][n] = sum_pixels x[p + (kh - PT, kw - PL)][c] * dy[p][n].  The implicit GEMM runs this as
// a (taps*C) x K GEMM over ~1e5 pixels with a 128 x 32 tile: its im2col operand re-reads every input pixel
// from L2 once per tap (49x for cnv1b), and with K = 16/32 the tile is too narrow for the bf16x6 path,
// so those layers ran at 30-50 TF/s.  Here:
//   * block = (kernel row kh, pixel chunk); it walks 128-pixel output row segments of its chunk;
//   * per segment the ONE input row the kernel row reads (128 + KW - 1 pixels x C channels) and the dy
//     segment (128 x K) are staged in LDS (register prefetch of the next segment overlaps the MFMAs);
//   * wave w owns (kw, channel fragment, column fragment) items w, w+4, ...: per 4-pixel k-step one
//     v_mfma_f32_16x16x4_f32 per item -- A = x[pixel + kw][c] straight out of the halo row at the tap
//     offset (any offset: 4-byte LDS reads), B = dy[pixel][n] shared by all items of a column fragment;
//   * exact fp32 products, fp32 accumulation in registers across the whole chunk; one fp32 partial
//     dW per (chunk, kh) and a fixed-order reduce over chunks (deterministic).
// LDS rows hold an odd multiple of 16 floats, so the four 4-lane-group pixel rows of one A / B fragment
// read land in four distinct 16-bank quarters (conflict-free ds_read_b32).
#include "halo_conv.h"

#include <cstdlib>

#include "split_math.h"

namespace {

constexpr int TP = 128;       // output pixels per row segment
constexpr int MAXI = 8;       // (kw, cf, nf) items per wave
constexpr int XQ = 8;         // f4 prefetch registers per thread: input row
constexpr int DQ = 4;         // f4 prefetch registers per thread: dy segment

struct HwgArgs {
  int N, H, W, C, K, KH, KW, PT, PL, wcin;
  int OH, OW, S;      // output rows / columns (the segments tile them) and stride (1; 2 in the fp16x3 kernel)
  int CF, NF, CPS, KPS, nitems, ntw, chunks;
  int ntiles;
  const float* x; int xcs, xco;
  const float* dy; int ycs, yco;
  float* part;
  int diag;   // timing experiments only (results garbage): bit 0 skip the MFMA loop, bit 1 skip the loads
};

__device__ __forceinline__ void tile_coords(const HwgArgs& a, int t, int& n, int& oh, int& ow0) {
  const int r = t / a.ntw;
  ow0 = (t - r * a.ntw) * TP;
  n = r / a.OH;
  oh = r - n * a.OH;
}

// per-thread (pixel, channel) coordinates of its prefetch quads: constant over the tiles
template <int XQN, int DQN>
struct QuadsT {
  int xhp[XQN], xc[XQN], dp[DQN], dc[DQN];
};
using Quads = QuadsT<XQ, DQ>;

// global -> registers: this thread's quads of the input row (kernel row kh) and the dy segment of tile t.
// Branch-free raw buffer loads (out of the image / past the row -> offset OOB -> 0), all in flight at once;
// the w_cin channel mask is applied when the registers are stored to LDS.
template <int XQN, int DQN>
__device__ __forceinline__ void prefetch(const HwgArgs& a, const QuadsT<XQN, DQN>& q, __amdgpu_buffer_rsrc_t rx,
                                         __amdgpu_buffer_rsrc_t rd, int kh, int t, f4 (&xr)[XQN], f4 (&dr)[DQN]) {
  const bool tv = t < a.ntiles && !(a.diag & 2);
  int n = 0, oh = 0, ow0 = 0;
  if (tv) tile_coords(a, t, n, oh, ow0);
  const int ih = oh * a.S + kh - a.PT;
  const bool rowok = tv && (unsigned)ih < (unsigned)a.H;
  const int xrow = ((n * a.H + ih) * a.W) * a.xcs + a.xco;
#pragma unroll
  for (int i = 0; i < XQN; ++i) {
    const int iw = ow0 * a.S - a.PL + q.xhp[i];
    const bool ok = rowok && (unsigned)iw < (unsigned)a.W;      // xhp < 0: past this thread's quads
    xr[i] = bload(rx, ok ? 4 * (xrow + iw * a.xcs + q.xc[i]) : OOB);
  }
  const int drow = ((n * a.OH + oh) * a.OW) * a.ycs + a.yco;
#pragma unroll
  for (int i = 0; i < DQN; ++i) {
    const bool ok = tv && q.dp[i] >= 0 && ow0 + q.dp[i] < a.OW;
    dr[i] = bload(rd, ok ? 4 * (drow + (ow0 + q.dp[i]) * a.ycs + q.dc[i]) : OOB);
  }
}

// NI = items per wave (compile time: the per-item A reads and MFMAs of a k-step are straight-line code,
// all LDS reads issued before the MFMAs); items past nitems are dummies whose results are dropped.
template <int NI>
__global__ void __launch_bounds__(256) hwg_kernel(const HwgArgs a) {
  extern __shared__ float lds[];
  float* xs = lds;                                   // [TP + KW - 1][CPS]
  float* ds = lds + (TP + a.KW - 1) * a.CPS;         // [TP][KPS]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int kh = blockIdx.y;
  const int cq = a.CF * 4, nq = a.NF * 4;
  // this wave's items: it = wv + 4m -> (kw, cf, nf), LDS offsets of its A / B fragment reads
  int aoff[NI], bsel[NI];
#pragma unroll
  for (int m = 0; m < NI; ++m) {
    const int it = wv + 4 * m;
    const int itc = it < a.nitems ? it : 0;
    const int nf = itc % a.NF, r = itc / a.NF, cf = r % a.CF, kw = r / a.CF;
    aoff[m] = (lq + kw) * a.CPS + cf * 16 + li;
    bsel[m] = nf;
  }
  f4 acc[NI];
#pragma unroll
  for (int m = 0; m < NI; ++m) acc[m] = f4{0.f, 0.f, 0.f, 0.f};
  f4 xr[XQ], dr[DQ];
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (long)a.N * a.H * a.W * a.xcs);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (long)a.N * a.OH * a.OW * a.ycs);
  Quads q;
  {
    const int nx = (TP + a.KW - 1) * cq;
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int hp = e / cq, c = 4 * (e - hp * cq);
      const bool ok = e < nx && c < a.C;
      q.xhp[i] = ok ? hp : -(1 << 20);
      q.xc[i] = c;
    }
#pragma unroll
    for (int i = 0; i < DQ; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int p = e / nq, c = 4 * (e - p * nq);
      const bool ok = e < TP * nq && c < a.K;
      q.dp[i] = ok ? p : -1;
      q.dc[i] = c;
    }
  }
  int t = blockIdx.x;
  prefetch(a, q, rx, rd, kh, t, xr, dr);
  for (; t < a.ntiles; t += a.chunks) {
    int n, oh, ow0;
    tile_coords(a, t, n, oh, ow0);
    const bool live = (unsigned)(oh + kh - a.PT) < (unsigned)a.H;   // uniform over the block
    __syncthreads();                                   // the previous segment's reads are done
#pragma unroll
    for (int i = 0; i < XQ; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < (TP + a.KW - 1) * cq) {
        const int hp = e / cq, c = 4 * (e - hp * cq);
        f4 v = xr[i];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j >= a.wcin) v[j] = 0.f;
        *reinterpret_cast<f4*>(xs + hp * a.CPS + c) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < DQ; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < TP * nq) {
        const int p = e / nq, c = 4 * (e - p * nq);
        *reinterpret_cast<f4*>(ds + p * a.KPS + c) = dr[i];
      }
    }
    __syncthreads();
    prefetch(a, q, rx, rd, kh, t + a.chunks, xr, dr);             // next segment's loads in flight under the MFMAs
    if (!live || (a.diag & 1)) continue;
#pragma unroll 2
    for (int s = 0; s < TP / 4; ++s) {
      const float b0 = ds[(4 * s + lq) * a.KPS + li];
      const float b1 = ds[(4 * s + lq) * a.KPS + 16 + li];   // NF == 1: the pad row, never selected
      float av[NI];
#pragma unroll
      for (int m = 0; m < NI; ++m) av[m] = xs[aoff[m] + 4 * s * a.CPS];
#pragma unroll
      for (int m = 0; m < NI; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bsel[m] ? b1 : b0, acc[m], 0, 0, 0);
    }
  }
  // lane (li, lq) holds dW[c = cf*16 + 4 lq + r][n = nf*16 + li]; partial [chunk][kh][kw][wcin][K]
  float* out = a.part + ((long)blockIdx.x * a.KH + kh) * a.KW * a.wcin * a.K;
#pragma unroll
  for (int m = 0; m < NI; ++m) {
    const int it = wv + 4 * m;
    if (it >= a.nitems) continue;
    const int nf = it % a.NF, r = it / a.NF, cf = r % a.CF, kw = r / a.CF;
    const int nn = nf * 16 + li;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = cf * 16 + 4 * lq + j;
      if (c < a.wcin && nn < a.K) out[((long)kw * a.wcin + c) * a.K + nn] = acc[m][j];
    }
  }
}

// ------------------------------------------------------------------ fp16x3 variant (conv math 4)
// Same blocking (block = (kernel row, pixel chunk), 128-pixel output row segments, input row + dy segment
// staged once per segment), but the operands are split into power-of-two-scaled fp16 hi / lo planes at
// staging (split_math.h) and each 32-pixel k-step of an item is 3 v_mfma_f32_16x16x32_f16 instead of 8
// v_mfma_f32_16x16x4_f32 (5.3x the product rate).  The contraction runs over pixels, but the LDS images
// stay pixel-major ([pixel][channel], as loaded): fragments are read with ds_read_b64_tr_b16, which hands
// lane i of a 16-lane group column i (= channel / output column i) of a 4-pixel x 16-column block, so the
// tap shift kw is just a row offset.  k order inside a 32-pixel step (identical for A and B): element j of
// lane group g is pixel 4g + j (j < 4) or 16 + 4g + j - 4; a 32-lane half then reads 8 consecutive rows,
// conflict-free with a row stride of an odd multiple of 32 bytes (odd16 fp16 elements).
// A wave owns NA (kw, channel fragment) items and computes each against all NF column fragments.
struct HwhArgs {
  int N, H, W, C, K, KH, KW, PT, PL, wcin;
  int OH, OW;
  int CF, NF, XS, DS, nA, ntw, chunks;
  int ntiles;
  const float* x; int xcs, xco;
  const float* dy; int ycs, yco;
  float* part;
  const float* xmax; const float* dmax;   // operand bounds (tde_conv_desc_t x_absmax / y_absmax) or null
};

typedef unsigned short u16;
typedef __fp16 hp4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
typedef __attribute__((address_space(3))) hp4* lds_hp4_t;

// one 8-element fp16 fragment (k = 32-pixel step starting at pixel row `row0` of the plane, columns col0..+15)
__device__ __forceinline__ h8 tr_frag(const u16* plane, int S, int row0, int col0, int g, int li) {
  const int qq = li >> 2, p = li & 3;
  const u16* a0 = plane + (row0 + 4 * g + qq) * S + col0 + 4 * p;
  const hp4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hp4_t)(a0));
  const hp4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hp4_t)(a0 + 16 * S));
  const h4 l4 = __builtin_bit_cast(h4, lo), h4v = __builtin_bit_cast(h4, hi);
  return h8{l4[0], l4[1], l4[2], l4[3], h4v[0], h4v[1], h4v[2], h4v[3]};
}

// the same fragment from a per-lane pointer p = plane + (row0 + 4g + qq) S + col0 + 4p; `up` = 16 rows
__device__ __forceinline__ h8 tr_frag2(const u16* p, int up) {
  const hp4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hp4_t)(p));
  const hp4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hp4_t)(p + up));
  const h4 l4 = __builtin_bit_cast(h4, lo), h4v = __builtin_bit_cast(h4, hi);
  return h8{l4[0], l4[1], l4[2], l4[3], h4v[0], h4v[1], h4v[2], h4v[3]};
}

constexpr int XQ16 = 12, DQ16 = 4;   // most prefetch quads per thread (input row, dy segment)

// XQN input-row quads per thread (4, 8 or 12: as few registers as the row needs), DQN = 2 NF dy quads.
// S = stride (1 or 2).  At stride 2 a segment's input row (2 TP + KW - 1 pixels from 2 ow0 - PL) is staged as two
// parity planes of R = TP + (KW - 1) / 2 rows -- plane q row r = pixel 2 r + q -- so tap kw of output pixel p reads
// plane kw & 1 at row p + kw / 2: still a plain row offset for the transposing reads, and each input pixel is
// staged once (round 6: cnv1, whose 3 / 6 input channels left the implicit GEMM's filter gradient at ~23 TF/s).
template <int NA, int NF, int XQN, int S>
__global__ void __launch_bounds__(256) hwh_kernel(const HwhArgs a) {
  constexpr int DQN = 2 * NF;
  extern __shared__ __attribute__((aligned(16))) u16 lds16[];
  const int R = TP + (a.KW - 1) / S;              // rows per parity plane
  const int XP = S * R * a.XS, DP = TP * a.DS;
  u16* const xh = lds16;
  u16* const xl = xh + XP;
  u16* const dh = xl + XP;
  u16* const dl = dh + DP;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  // (chunk, kernel row) of this block.  (An XCD-grouped order -- the KH blocks of one chunk, which read the same dy
  // segments, on one XCD -- measured neutral on every layer: profiles/r06/hwh_s2_micro.txt.)
  const int chunk = blockIdx.x, kh = blockIdx.y;
  // only the real channel quads are staged: the pad channels / columns of the last fragment hold whatever the
  // LDS holds, which reaches only dW rows c >= C and columns n >= K (dropped)
  const int cq = a.C / 4, nq = a.K / 4;
  const float sx = f16x3_scale(a.xmax, 1.f), sd = f16x3_scale(a.dmax, 1.f);
  int akw[NA], acol[NA], aoff[NA];
#pragma unroll
  for (int m = 0; m < NA; ++m) {
    const int ia = wv + 4 * m;
    const int ic = ia < a.nA ? ia : 0;   // dummy items read item 0 (every lane takes part: EXEC all ones)
    akw[m] = ic / a.CF;
    acol[m] = (ic - akw[m] * a.CF) * 16;
    aoff[m] = ((akw[m] % S) * R + akw[m] / S) * a.XS;   // parity plane + row offset of tap kw
  }
  f4 acc[NA][NF];
#pragma unroll
  for (int m = 0; m < NA; ++m)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[m][f] = f4{0.f, 0.f, 0.f, 0.f};
  f4 xr[XQN], dr[DQN];
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x, (long)a.N * a.H * a.W * a.xcs);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (long)a.N * a.OH * a.OW * a.ycs);
  // the fp32 kernel's prefetch (same quads; HwgArgs view of the geometry)
  HwgArgs ga{};
  ga.N = a.N; ga.H = a.H; ga.W = a.W; ga.C = a.C; ga.K = a.K; ga.KW = a.KW; ga.PT = a.PT; ga.PL = a.PL;
  ga.OH = a.OH; ga.OW = a.OW; ga.S = S;
  ga.ntw = a.ntw; ga.ntiles = a.ntiles; ga.xcs = a.xcs; ga.xco = a.xco; ga.ycs = a.ycs; ga.yco = a.yco;
  const int nx = S * R * cq;                      // input-row quads of a segment
  QuadsT<XQN, DQN> q;
  {
#pragma unroll
    for (int i = 0; i < XQN; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int hp = e / cq, c = 4 * (e - hp * cq);
      const bool ok = e < nx;
      q.xhp[i] = ok ? hp : -(1 << 20);
      q.xc[i] = c;
    }
#pragma unroll
    for (int i = 0; i < DQN; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int p = e / nq, c = 4 * (e - p * nq);
      const bool ok = e < TP * nq;
      q.dp[i] = ok ? p : -1;
      q.dc[i] = c;
    }
  }
  int t = chunk;
  prefetch(ga, q, rx, rd, kh, t, xr, dr);
  for (; t < a.ntiles; t += a.chunks) {
    int n, oh, ow0;
    tile_coords(ga, t, n, oh, ow0);
    const bool live = (unsigned)(oh * S + kh - a.PT) < (unsigned)a.H;   // uniform over the block
    __syncthreads();                                   // the previous segment's reads are done
    // the quads' (pixel, channel) coordinates come from the prefetch table (no per-segment divisions: round 6,
    // the integer divisions by C / 4 and K / 4 were ~40 % of the kernel's VALU instructions)
#pragma unroll
    for (int i = 0; i < XQN; ++i) {
      if (q.xhp[i] >= 0) {
        const int hp = q.xhp[i], c = q.xc[i];
        const int row = (hp % S) * R + hp / S;         // parity plane hp % S, row hp / S
        // no pad-channel mask: channel c of the view only ever meets MFMA A row c, i.e. dW row c, and rows
        // c >= w_cin are dropped at the store (round 6: the per-quad masks cost ~60 VALU per segment)
        h4 hi, lo;
        split4x2h(xr[i], sx, hi, lo);
        *reinterpret_cast<h4*>(xh + row * a.XS + c) = hi;
        *reinterpret_cast<h4*>(xl + row * a.XS + c) = lo;
      }
    }
#pragma unroll
    for (int i = 0; i < DQN; ++i) {
      if (q.dp[i] >= 0) {
        const int p = q.dp[i], c = q.dc[i];
        h4 hi, lo;
        split4x2h(dr[i], sd, hi, lo);
        *reinterpret_cast<h4*>(dh + p * a.DS + c) = hi;
        *reinterpret_cast<h4*>(dl + p * a.DS + c) = lo;
      }
    }
    __syncthreads();
    prefetch(ga, q, rx, rd, kh, t + a.chunks, xr, dr);   // next segment's loads in flight under the MFMAs
    if (!live) continue;
    // per-lane read pointers advanced by one 32-pixel step per iteration; the lo planes and the upper 16 pixels are
    // immediate offsets (round 6: recomputing each fragment's address cost 60 VALU per 24 MFMAs)
    const u16* pb = dh + (4 * g + (li >> 2)) * a.DS + 4 * (li & 3);
    const u16* pa = xh + (4 * g + (li >> 2)) * a.XS + 4 * (li & 3);
#pragma unroll 1
    for (int s0 = 0; s0 < TP; s0 += 32, pb += 32 * a.DS, pa += 32 * a.XS) {
      h8 bh[NF], bl[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        bh[f] = tr_frag2(pb + 16 * f, 16 * a.DS);
        bl[f] = tr_frag2(pb + DP + 16 * f, 16 * a.DS);
      }
#pragma unroll
      for (int m = 0; m < NA; ++m) {
        const h8 ah = tr_frag2(pa + aoff[m] + acol[m], 16 * a.XS);
        const h8 al = tr_frag2(pa + XP + aoff[m] + acol[m], 16 * a.XS);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          acc[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[f], acc[m][f], 0, 0, 0);
          acc[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[f], acc[m][f], 0, 0, 0);
          acc[m][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[f], acc[m][f], 0, 0, 0);
        }
      }
    }
  }
  // lane (li, g) holds dW[kw][c = cf*16 + 4g + r][n = nf*16 + li] (scaled); partial [chunk][kh][kw][wcin][K]
  const float inv = 1.f / (sx * sd);   // power of two: exact
  float* out = a.part + ((long)chunk * a.KH + kh) * a.KW * a.wcin * a.K;
#pragma unroll
  for (int m = 0; m < NA; ++m) {
    const int ia = wv + 4 * m;
    if (ia >= a.nA) continue;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int nn = f * 16 + li;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = acol[m] + 4 * g + j;
        if (c < a.wcin && nn < a.K) out[((long)akw[m] * a.wcin + c) * a.K + nn] = acc[m][f][j] * inv;
      }
    }
  }
}

// dw[e] (+)= sum over chunks of part[chunk][e] (e = ((kh*KW + kw)*wcin + c)*K + n): a block is 16 output
// quads x 16 z-lanes; lane z sums chunks z, z+16, ... and the 16 lanes of a quad are combined through LDS
// in lane order (fixed order: deterministic).
__global__ void __launch_bounds__(256) hwg_reduce_kernel(const float* part, int chunks, long E4, float* dw,
                                                         int accumulate) {
  __shared__ f4 tmp[256];
  const int zl = threadIdx.x & 15;
  const long i = blockIdx.x * 16L + (threadIdx.x >> 4);
  f4 s = {0.f, 0.f, 0.f, 0.f};
  if (i < E4) {
    const f4* p = reinterpret_cast<const f4*>(part) + i;
    f4 s2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    int u = 0;
    for (int z = zl; z < chunks; z += 16, u ^= 1) s2[u] += p[(long)z * E4];
    s = s2[0] + s2[1];
  }
  tmp[threadIdx.x] = s;
  __syncthreads();
  if (zl == 0 && i < E4) {
#pragma unroll
    for (int k = 1; k < 16; ++k) s += tmp[threadIdx.x + k];
    f4* d = reinterpret_cast<f4*>(dw) + i;
    if (accumulate) s += *d;
    *d = s;
  }
}

long env_hwg(const char* name, long dflt) {
  const char* v = std::getenv(name);
  return v ? std::atol(v) : dflt;
}
const long g_hwg = env_hwg("TDE_HWG", 1);                 // 0: never (A/B)
const long g_hwg_blocks = tde_env_pos("TDE_HWG_BLOCKS", 768);  // grid size to aim for
const long g_hwg_min_m = tde_env_pos("TDE_HWG_MIN_M", 16384);
// TDE_HWG_DIAG (timing experiments, results garbage): read only by a diagnostic build (-DTDE_TIMING_DIAG)
#ifdef TDE_TIMING_DIAG
const long g_hwg_diag = env_hwg("TDE_HWG_DIAG", 0);
#else
constexpr long g_hwg_diag = 0;
#endif
const long g_hwg_min_items = env_hwg("TDE_HWG_MIN_ITEMS", 25);
const long g_hwh = env_hwg("TDE_HWH", 1);                 // 0: fp32 halo WGRAD also in math 4 (A/B)
const long g_hwh_min_items = env_hwg("TDE_HWH_MIN_ITEMS", 1);
// stride-2 layers on the fp16x3 kernel for input views of TDE_HWH_S2_MINC..TDE_HWH_S2_MAXC channels (MAXC 0: none).
// Measured per layer at config 4's twin batch (scripts/conv_micro.py, profiles/r06/hwh_s2_micro.txt), against the
// implicit GEMM / pixel-shuffle filter gradient: cnv1 over 8 channels 114.7 -> 93-95 us, exp_upcnv1 (16) 139-143 ->
// 111 us, upcnv1 (16) 57-59 -> 54 us; cnv1 over 4 channels 70 -> 89-94 us (loses: a 16-row fragment holds 4).
const long g_hwh_s2_minc = env_hwg("TDE_HWH_S2_MINC", 8);
const long g_hwh_s2_maxc = env_hwg("TDE_HWH_S2_MAXC", 16);

int odd16(int c) {   // smallest odd multiple of 16 >= c
  int f = (c + 15) / 16;
  if (!(f & 1)) ++f;
  return 16 * f;
}

}  // namespace

bool hwg_plan(const tde_conv_desc_t& d, HwgPlan& hp, int math) {
  hp = HwgPlan{};
  if (!g_hwg) return false;
  const bool s1 = d.stride == 1 && d.OH == d.H && d.OW == d.W;
  if (math == 4 && g_hwh) {
    // fp16x3 kernel: (kw, channel fragment) items per wave x all column fragments; stride 1, or stride 2 (parity
    // planes) for input views of TDE_HWH_S2_MINC..MAXC channels
    const bool s2 = d.stride == 2 && d.C >= g_hwh_s2_minc && d.C <= g_hwh_s2_maxc;
    if (!s1 && !s2) return false;
    const int S = d.stride;
    if ((long)d.N * d.OH * d.OW < g_hwg_min_m) return false;
    if (d.K > 32 || d.K % 4 || d.C % 4 || d.C > 128 || d.KW > 7 || d.KH > 7) return false;
    if (d.x_cstride % 4 || d.x_coff % 4 || d.y_cstride % 4 || d.y_coff % 4) return false;
    const int CF = (d.C + 15) / 16, NF = (d.K + 15) / 16;
    const int nA = d.KW * CF;
    if (nA > 4 * 8 || nA * NF < g_hwh_min_items) return false;
    const int R = TP + (d.KW - 1) / S;   // rows per parity plane
    if (S * R * (d.C / 4) > 256 * XQ16 || TP * (d.K / 4) > 256 * 2 * NF) return false;
    hp.ok = 1; hp.f16 = 1; hp.S = S;
    hp.CF = CF; hp.NF = NF; hp.nitems = nA;
    hp.CPS = odd16(CF * 16);   // fp16 elements per LDS row
    hp.KPS = odd16(NF * 16);
    hp.ntw = (d.OW + TP - 1) / TP;
    hp.ntiles = (long)d.N * d.OH * hp.ntw;
    long chunks = (g_hwg_blocks + d.KH - 1) / d.KH;
    const long maxc = (hp.ntiles + 3) / 4;
    if (chunks > maxc) chunks = maxc;
    if (chunks < 1) chunks = 1;
    hp.chunks = (int)chunks;
    // two fp16 planes each of the input row (S parity planes of R rows) and the dy segment
    hp.lds_bytes = (size_t)(2 * S * R * hp.CPS + 2 * TP * hp.KPS) * sizeof(u16);
    hp.part_bytes = ((size_t)chunks * d.KH * d.KW * d.w_cin * d.K * sizeof(float) + 255) / 256 * 256;
    return true;
  }
  if (!s1) return false;
  if ((long)d.N * d.H * d.W < g_hwg_min_m) return false;
  if (d.K > 32 || d.K % 4 || d.C % 4 || d.C > 128 || d.KW > 7 || d.KH > 7) return false;
  if (d.x_cstride % 4 || d.x_coff % 4 || d.y_cstride % 4 || d.y_coff % 4) return false;
  const int CF = (d.C + 15) / 16, NF = (d.K + 15) / 16;
  const int nitems = d.KW * CF * NF;
  // measured (scripts/conv_micro.py, TDE_HWG_DIAG): the fp32-MFMA loop runs at ~56% of its peak and the
  // per-segment staging + partial reduce cost ~45 us on cnv1b, so the kernel only beats the implicit GEMM
  // where the MFMA work per segment is large (cnv1b: 180 vs 201 us; icnv1 with 6 items of 3x3 taps: 93 vs
  // 79 us) -- >= 25 items (7 per wave) unless TDE_HWG_MIN_ITEMS says otherwise
  if (nitems > 4 * MAXI || nitems < g_hwg_min_items) return false;
  if ((TP + d.KW - 1) * CF * 4 > 256 * XQ || TP * NF * 4 > 256 * DQ) return false;
  hp.ok = 1; hp.S = 1;
  hp.CF = CF; hp.NF = NF; hp.nitems = nitems;
  hp.CPS = odd16(CF * 16);
  hp.KPS = odd16(NF * 16);
  hp.ntw = (d.W + TP - 1) / TP;
  hp.ntiles = (long)d.N * d.H * hp.ntw;
  long chunks = (g_hwg_blocks + d.KH - 1) / d.KH;
  const long maxc = (hp.ntiles + 3) / 4;   // >= 4 segments per block
  if (chunks > maxc) chunks = maxc;
  if (chunks < 1) chunks = 1;
  hp.chunks = (int)chunks;
  hp.lds_bytes = (size_t)((TP + d.KW - 1) * hp.CPS + TP * hp.KPS + 16) * sizeof(float);   // + pad row
  hp.part_bytes = ((size_t)chunks * d.KH * d.KW * d.w_cin * d.K * sizeof(float) + 255) / 256 * 256;
  return true;
}

template <int NA, int XQN, int S>
void launch_hwh_x(const HwgPlan& hp, const HwhArgs& a, dim3 grid, hipStream_t st) {
  if (hp.NF == 1) hipLaunchKernelGGL((hwh_kernel<NA, 1, XQN, S>), grid, dim3(256), hp.lds_bytes, st, a);
  else hipLaunchKernelGGL((hwh_kernel<NA, 2, XQN, S>), grid, dim3(256), hp.lds_bytes, st, a);
}
template <int NA, int S>
void launch_hwh_s(const HwgPlan& hp, const HwhArgs& a, dim3 grid, hipStream_t st) {
  const int need = (S * (TP + (a.KW - 1) / S) * (a.C / 4) + 255) / 256;
  if (need <= 4) launch_hwh_x<NA, 4, S>(hp, a, grid, st);
  else if (need <= 8) launch_hwh_x<NA, 8, S>(hp, a, grid, st);
  else launch_hwh_x<NA, 12, S>(hp, a, grid, st);
}
template <int NA>
void launch_hwh(const HwgPlan& hp, const HwhArgs& a, dim3 grid, hipStream_t st) {
  if (hp.S == 2) launch_hwh_s<NA, 2>(hp, a, grid, st);
  else launch_hwh_s<NA, 1>(hp, a, grid, st);
}

void hwg_launch(const HwgPlan& hp, const tde_conv_desc_t& d, const float* x, const float* dy, float* dw,
                int accumulate, void* ws, hipStream_t st) {
  if (hp.f16) {
    HwhArgs a{};
    a.N = d.N; a.H = d.H; a.W = d.W; a.C = d.C; a.K = d.K; a.KH = d.KH; a.KW = d.KW;
    a.PT = d.pad_top; a.PL = d.pad_left; a.wcin = d.w_cin;
    a.OH = d.OH; a.OW = d.OW;
    a.CF = hp.CF; a.NF = hp.NF; a.XS = hp.CPS; a.DS = hp.KPS; a.nA = hp.nitems; a.ntw = hp.ntw;
    a.chunks = hp.chunks; a.ntiles = (int)hp.ntiles;
    a.x = x; a.xcs = d.x_cstride; a.xco = d.x_coff;
    a.dy = dy; a.ycs = d.y_cstride; a.yco = d.y_coff;
    a.part = static_cast<float*>(ws);
    a.xmax = d.x_absmax; a.dmax = d.y_absmax;
    const dim3 grid(hp.chunks, d.KH);
    switch ((hp.nitems + 3) / 4) {
      case 1: launch_hwh<1>(hp, a, grid, st); break;
      case 2: launch_hwh<2>(hp, a, grid, st); break;
      case 3: launch_hwh<3>(hp, a, grid, st); break;
      case 4: launch_hwh<4>(hp, a, grid, st); break;
      case 5: launch_hwh<5>(hp, a, grid, st); break;
      case 6: launch_hwh<6>(hp, a, grid, st); break;
      case 7: launch_hwh<7>(hp, a, grid, st); break;
      default: launch_hwh<8>(hp, a, grid, st); break;
    }
    const long E4 = (long)d.KH * d.KW * d.w_cin * d.K / 4;
    hipLaunchKernelGGL(hwg_reduce_kernel, dim3((int)((E4 + 15) / 16)), dim3(256), 0, st, a.part, hp.chunks, E4, dw,
                       accumulate);
    return;
  }
  HwgArgs a{};
  a.N = d.N; a.H = d.H; a.W = d.W; a.C = d.C; a.K = d.K; a.KH = d.KH; a.KW = d.KW;
  a.PT = d.pad_top; a.PL = d.pad_left; a.wcin = d.w_cin;
  a.OH = d.H; a.OW = d.W; a.S = 1;
  a.CF = hp.CF; a.NF = hp.NF; a.CPS = hp.CPS; a.KPS = hp.KPS; a.nitems = hp.nitems; a.ntw = hp.ntw;
  a.chunks = hp.chunks; a.ntiles = (int)hp.ntiles;
  a.x = x; a.xcs = d.x_cstride; a.xco = d.x_coff;
  a.dy = dy; a.ycs = d.y_cstride; a.yco = d.y_coff;
  a.part = static_cast<float*>(ws);
  a.diag = (int)g_hwg_diag;
  const dim3 grid(hp.chunks, d.KH);
  switch ((hp.nitems + 3) / 4) {
    case 1: hipLaunchKernelGGL(hwg_kernel<1>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 2: hipLaunchKernelGGL(hwg_kernel<2>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 3: hipLaunchKernelGGL(hwg_kernel<3>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 4: hipLaunchKernelGGL(hwg_kernel<4>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 5: hipLaunchKernelGGL(hwg_kernel<5>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 6: hipLaunchKernelGGL(hwg_kernel<6>, grid, dim3(256), hp.lds_bytes, st, a); break;
    case 7: hipLaunchKernelGGL(hwg_kernel<7>, grid, dim3(256), hp.lds_bytes, st, a); break;
    default: hipLaunchKernelGGL(hwg_kernel<8>, grid, dim3(256), hp.lds_bytes, st, a); break;
  }
  const long E4 = (long)d.KH * d.KW * d.w_cin * d.K / 4;
  hipLaunchKernelGGL(hwg_reduce_kernel, dim3((int)((E4 + 15) / 16)), dim3(256), 0, st, a.part, hp.chunks, E4, dw,
                     accumulate);
}
