// Shared by the implicit-GEMM conv translation units (conv_igemm.hip: the register-staged tiles, skinny and
// split-K kernels, host planning; conv_ring.hip: the LDS-DMA ring tiles): GEMM argument block, DGRAD class
// geometry and the tile epilogue (BN statistics partials, stores), in namespace tdeconv (inline device code: each
// translation unit keeps its own copy; the argument block is one type across them).
#pragma once
#include "tde_common.h"
#include "split_math.h"

namespace tdeconv {

constexpr int MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2;
// MODE_PS: the forward of a k x k stride-2 deconv (slim.conv2d_transpose, nets_optflow_depth.py:103-140; k = 3, 5, 7)
// -- equally the data gradient of a k x k stride-2 conv -- as ONE pixel-shuffle GEMM instead of 4 parity-class DGRAD
// GEMMs: rows = input pixels (n, a, b), columns = the 2x2 output block (py, px) x Cout, K = the T x T input
// neighbourhood (a - PW + th, b - PW + tw) x Cin -- a stride-1 T x T forward conv (KH = KW = T, PT = PL = PW: the
// union of the four classes' tap windows, T = 2 / 3 / 4 for k = 3 / 5 / 7) whose B operand is the deconv weight
// w[kh][kw][c][k] gathered at kh = ps_kh0 + py - 2 th, kw = ps_kh0 + px - 2 tw (zero outside the k x k kernel: 9 of
// 16, 25 of 36, 49 of 64 tap x class pairs), and whose epilogue scatters column (py, px, c) to output pixel
// (2a + py, 2b + px).  Each input pixel is staged once per tile for all four classes, and the GEMM is 4 x Cout wide
// where the class GEMMs are Cout wide (16 / 32 columns for the high-resolution layers).
constexpr int MODE_PS = 3;
// MODE_PSW: the filter gradient of the same stride-2 layers in the pixel-shuffle form.  dw[kh][kw][c][k] =
// sum_(n,a,b) x[n, 2a + py, 2b + px, c] dy[n, a - PW + th, b - PW + tw, k] with kh = kh0 + py - 2 th (the MODE_PS
// relation read the other way): rows = (py, px, c) -- the WGRAD im2col gather of x with a 2x2 "kernel" at stride 2 --
// columns = (th, tw, k) -- the T x T stride-1 window of dy over its own grid -- reduction over dy's pixels.  4 x C
// rows and T^2 x K columns where the direct filter-gradient GEMM has k^2 x C rows and K columns (16 / 32 for the
// high-resolution layers); every output goes through the split-K slab, whose reduce scatters (row, column) to
// dw[kh][kw][c][k] and drops the (py, th) pairs outside the kernel.
constexpr int MODE_PSW = 4;

struct ConvArgs {
  int N, H, W, C, OH, OW, K, KH, KW, S, PT, PL, wcin;
  const float* x; float* dx; int xcs, xco;
  const float* dy; float* y; int ycs, yco;
  const float* w; float* dw;
  float* ws; int splits; int accumulate;
  int kt_per;  // k-tiles per split
  FDiv fC, fK, fKW, fOW, fOHW;
  double* bnp;  // BN statistics partials [row tile][2][Nn] from the epilogue (FWD/DGRAD/PS, splits == 1)
  int bn_gx;    // row tiles per DGRAD class (grid x)
  int bn_G;     // BN row groups (DGRAD: partials ordered group-major over the parity classes; the host checks that
                // every class's rows per group are whole row tiles)
  int bn_gy;    // MODE_PS: column tiles (one partial record [2][ps_C] per (row tile, column tile))
  // inference epilogue (FWD / DGRAD outputs only; accumulate == 0): v = conv + bias[col], then ReLU
  // (BN folded into the weights, tde_conv2d_fwd_bias_act); bias null and relu 0 = plain conv
  const float* bias; int relu;
  // fp16x3 (math 4) operand bounds |x| <= *bound of the x view, the y view and the weights (null: unscaled
  // x / y, fixed weight scale; split_math.h)
  const float* xmax; const float* ymax; const float* wmax;
  // MODE_PS: deconv output channels / height / width, weight input channels (w[ps_KS][ps_KS][ps_C][ps_K]), kernel size
  // and the kernel-row origin of the B gather (kh = ps_kh0 + py - 2 th)
  int ps_C, ps_H, ps_W, ps_K, ps_KS, ps_kh0;
  FDiv fpsC;
  // MODE_PSW: the dy window (T x T from -PW) and its division
  int ps_T, ps_PW;
  FDiv fpsT;
};

// The folded-BN epilogue: TF's Relu keeps NaN (same test as bn_apply_kernel).
__device__ __forceinline__ float bias_act(float v, const float* bias, int col, int relu) {
  if (bias) v += bias[col];
  return (relu && v < 0.f) ? 0.f : v;
}

// Per-class geometry of the DGRAD sub-pixel decomposition.
struct DgClass {
  int py, px, khs, kws, dh, dw, nth, ntw, HH, WW, M, Kd;
};

__device__ __forceinline__ DgClass dg_class(const ConvArgs& p, int cls) {
  DgClass g;
  g.py = cls / p.S;
  g.px = cls - g.py * p.S;
  g.khs = (g.py + p.PT) % p.S;
  g.kws = (g.px + p.PL) % p.S;
  g.dh = (g.py + p.PT - g.khs) / p.S;
  g.dw = (g.px + p.PL - g.kws) / p.S;
  g.nth = (p.KH - g.khs + p.S - 1) / p.S;
  g.ntw = (p.KW - g.kws + p.S - 1) / p.S;
  g.HH = (p.H - g.py + p.S - 1) / p.S;
  g.WW = (p.W - g.px + p.S - 1) / p.S;
  g.M = p.N * g.HH * g.WW;
  g.Kd = g.nth * g.ntw * p.K;
  return g;
}

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// Epilogue shared by the implicit-GEMM tiles (conv_tile, ring_tile): BN statistics partials of the output tile,
// then the stores (direct or split-K slab), accumulate / bias / ReLU as the ConvArgs say.  acc is the wave's TM x TN
// 16x16 accumulators (scales already undone); red: >= 2 * WM * BN floats of LDS, free (the k-loop ended with a
// barrier).  Works for any block size >= BN threads (waves laid out WM x WN).
template <int MODE, int BM, int BN, int WM, int WN>
__device__ __forceinline__ void tile_epilogue(const ConvArgs& p, f4 (&acc)[BM / (16 * WM)][BN / (16 * WN)], const int bx,
                                              const int by, const int bz, const int M, const int Nn, const int zsplit,
                                              const DgClass& g, float* red) {
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr bool FWDLIKE = (MODE == MODE_FWD || MODE == MODE_PS);
  constexpr bool WGLIKE = (MODE == MODE_WGRAD || MODE == MODE_PSW);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int r16 = lane & 15, q = lane >> 4;
  const int wrow0 = wm * TM * 16, wcol0 = wn * TN * 16;
  const int m0 = bx * BM, n0 = by * BN;
  // ---- batch-norm statistics of the output tile (slim.batch_norm after this conv, bn.hip): per-channel
  // sum and sum of squares over the tile's rows (rows past M hold exact zeros: their operand rows loaded
  // as zero), lanes -> waves in a fixed order, one fp64 partial per row tile.  Workgroup-local: the
  // cross-tile reduction is the next kernel's (a launch costs what an in-kernel hand-off costs).
  if constexpr (!WGLIKE) {
    if (p.bnp != nullptr) {
      float cs[TN], cq[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        cs[b] = 0.f; cq[b] = 0.f;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r) { const float v = acc[a][b][r]; cs[b] += v; cq[b] += v * v; }
        cs[b] += __shfl_xor(cs[b], 16, 64); cq[b] += __shfl_xor(cq[b], 16, 64);
        cs[b] += __shfl_xor(cs[b], 32, 64); cq[b] += __shfl_xor(cq[b], 32, 64);
      }
      // red: [2][WM][BN]; the main loop ended with a barrier
      if (lane < 16) {
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          red[wm * BN + wcol0 + b * 16 + lane] = cs[b];
          red[(WM + wm) * BN + wcol0 + b * 16 + lane] = cq[b];
        }
      }
      __syncthreads();
      if constexpr (MODE == MODE_PS) {
        // column (py, px, c) is channel c of output-pixel class (py, px): a tile of BN columns covers whole classes
        // (the host checks BN % ps_C == 0), so channel c's record sums its classes' columns in class order
        const int Cc = p.ps_C;
        if (tid < Cc) {
          double sv = 0.0, sq = 0.0;
          for (int k = 0; k * Cc < BN; ++k) {
            const int col = k * Cc + tid;
            if (n0 + col >= Nn) break;
#pragma unroll
            for (int w = 0; w < WM; ++w) { sv += red[w * BN + col]; sq += red[(WM + w) * BN + col]; }
          }
          const size_t j = (size_t)bx * p.bn_gy + by;
          p.bnp[j * 2 * Cc + tid] = sv;
          p.bnp[j * 2 * Cc + Cc + tid] = sq;
        }
      } else if (tid < BN && n0 + tid < Nn) {
        // dense row-tile index (class-major for DGRAD: classes own disjoint pixel sets; with row groups group-major,
        // each group's tiles of every class before the next group's)
        int j = bx;
        if constexpr (MODE == MODE_DGRAD) {
          const int ncls = p.S * p.S, cls = bz % ncls;
          if (p.bn_G > 1) {
            int off = 0, tot = 0, tg = 1;
            for (int c = 0; c < ncls; ++c) {
              const int t = dg_class(p, c).M / p.bn_G / BM;
              if (c < cls) off += t;
              if (c == cls) tg = t;
              tot += t;
            }
            const int gi = bx / tg;
            j = gi * tot + off + (bx - gi * tg);
          } else {
            for (int c = 0; c < cls; ++c) j += (dg_class(p, c).M + BM - 1) / BM;
          }
        }
        double sv = 0.0, sq = 0.0;
#pragma unroll
        for (int w = 0; w < WM; ++w) { sv += red[w * BN + tid]; sq += red[(WM + w) * BN + tid]; }
        p.bnp[(size_t)j * 2 * Nn + n0 + tid] = sv;
        p.bnp[(size_t)j * 2 * Nn + Nn + n0 + tid] = sq;
      }
    }
  }

  // ---- epilogue (16x16 C/D map is dtype-independent on gfx950).  Row addresses first; when
  // accumulating into the destination, ALL old values are loaded before any store (a store may alias a
  // later load, so an interleaved read-modify-write would serialise one memory latency per element).
  const bool direct = (p.splits == 1) && MODE != MODE_PSW;    // MODE_PSW: always the slab (its reduce scatters)
  float* base;
  if constexpr (FWDLIKE) base = direct ? p.y : p.ws;
  else if constexpr (MODE == MODE_DGRAD) base = direct ? p.dx : p.ws;
  else base = direct ? p.dw : p.ws;
  long rowaddr[TM][4];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wrow0 + a * 16 + 4 * q + r;
      long ra_ = -1;
      if (m < M) {
        if constexpr (MODE == MODE_FWD) {
          ra_ = direct ? (long)m * p.ycs + p.yco : ((long)zsplit * M + m) * Nn;
        } else if constexpr (MODE == MODE_PS) {
          // output pixel (2a, 2b) of row (n, a, b); split-K never runs in this mode (the host keeps splits 1)
          const int ohw = p.OH * p.OW;
          const int ni = m / ohw, rr = m - ni * ohw, aa = rr / p.OW, bb = rr - aa * p.OW;
          ra_ = ((long)(ni * p.ps_H + 2 * aa) * p.ps_W + 2 * bb) * p.ycs + p.yco;
        } else if constexpr (MODE == MODE_DGRAD) {
          const int hw = g.HH * g.WW;
          const int n = m / hw, rr = m - n * hw, ihh = rr / g.WW, iww = rr - ihh * g.WW;
          const long P = ((long)n * p.H + (ihh * p.S + g.py)) * p.W + (iww * p.S + g.px);
          ra_ = direct ? P * p.xcs + p.xco : ((long)zsplit * p.N * p.H * p.W + P) * Nn;
        } else {
          if (direct) {
            const int tap = m / p.C, c = m - tap * p.C;
            if (c < p.wcin) ra_ = (long)(tap * p.wcin + c) * p.K;
          } else {
            ra_ = ((long)zsplit * M + m) * Nn;
          }
        }
      }
      rowaddr[a][r] = ra_;
    }
  }
  // element offset of column n from its row address, and the channel of n (bias index): n itself, except MODE_PS
  // (column (py, px, c) -> pixel (2a + py, 2b + px), channel c)
  long coff[TN];
  int ccol[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int n = n0 + wcol0 + b * 16 + r16;
    coff[b] = n; ccol[b] = n;
    if constexpr (MODE == MODE_PS) {
      const int gq = fdiv(n, p.fpsC);
      ccol[b] = n - gq * p.ps_C;
      coff[b] = (long)((gq >> 1) * p.ps_W + (gq & 1)) * p.ycs + ccol[b];
    }
  }
  if (direct && p.accumulate) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int n = n0 + wcol0 + b * 16 + r16;
          if (rowaddr[a][r] >= 0 && n < Nn) acc[a][b][r] += base[rowaddr[a][r] + coff[b]];
        }
  }
  if constexpr (!WGLIKE) {
    if (direct && (p.bias || p.relu)) {
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wcol0 + b * 16 + r16;
        const int nb = n < Nn ? ccol[b] : 0;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][r] = bias_act(acc[a][b][r], p.bias, nb, p.relu);
      }
    }
  }
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int n = n0 + wcol0 + b * 16 + r16;
        if (rowaddr[a][r] >= 0 && n < Nn) tde_st(base + rowaddr[a][r] + coff[b], acc[a][b][r]);
      }
}

}  // namespace tdeconv
