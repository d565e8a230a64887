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

namespace {

constexpr int TP = 128;       // output pixels per row segment
constexpr int MAXI = 8;       // (kw, cf, nf) items per wave
constexpr int XQ = 8;         // f4 prefetch registers per thread: input row
constexpr int DQ = 4;         // f4 prefetch registers per thread: dy segment

struct HwgArgs {
  int N, H, W, C, K, KH, KW, PT, PL, wcin;
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
  n = r / a.H;
  oh = r - n * a.H;
}

// per-thread (pixel, channel) coordinates of its prefetch quads: constant over the tiles
struct Quads {
  int xhp[XQ], xc[XQ], dp[DQ], dc[DQ];
};

// global -> registers: this thread's quads of the input row (kernel row kh) and the dy segment of tile t.
// Branch-free raw buffer loads (out of the image / past the row -> offset OOB -> 0), all in flight at once;
// the w_cin channel mask is applied when the registers are stored to LDS.
__device__ __forceinline__ void prefetch(const HwgArgs& a, const Quads& q, __amdgpu_buffer_rsrc_t rx,
                                         __amdgpu_buffer_rsrc_t rd, int kh, int t, f4 (&xr)[XQ], f4 (&dr)[DQ]) {
  const bool tv = t < a.ntiles && !(a.diag & 2);
  int n = 0, oh = 0, ow0 = 0;
  if (tv) tile_coords(a, t, n, oh, ow0);
  const int ih = oh + kh - a.PT;
  const bool rowok = tv && (unsigned)ih < (unsigned)a.H;
  const int xrow = ((n * a.H + ih) * a.W) * a.xcs + a.xco;
#pragma unroll
  for (int i = 0; i < XQ; ++i) {
    const int iw = ow0 - a.PL + q.xhp[i];
    const bool ok = rowok && (unsigned)iw < (unsigned)a.W;      // xhp < 0: past this thread's quads
    xr[i] = bload(rx, ok ? 4 * (xrow + iw * a.xcs + q.xc[i]) : OOB);
  }
  const int drow = ((n * a.H + oh) * a.W) * a.ycs + a.yco;
#pragma unroll
  for (int i = 0; i < DQ; ++i) {
    const bool ok = tv && q.dp[i] >= 0 && ow0 + q.dp[i] < a.W;
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
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dy, (long)a.N * a.H * a.W * a.ycs);
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
const long g_hwg_diag = env_hwg("TDE_HWG_DIAG", 0);
const long g_hwg_min_items = env_hwg("TDE_HWG_MIN_ITEMS", 25);

int odd16(int c) {   // smallest odd multiple of 16 >= c
  int f = (c + 15) / 16;
  if (!(f & 1)) ++f;
  return 16 * f;
}

}  // namespace

bool hwg_plan(const tde_conv_desc_t& d, HwgPlan& hp) {
  hp = HwgPlan{};
  if (!g_hwg || d.stride != 1 || d.OH != d.H || d.OW != d.W) return false;
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
  hp.ok = 1;
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

void hwg_launch(const HwgPlan& hp, const tde_conv_desc_t& d, const float* x, const float* dy, float* dw,
                int accumulate, void* ws, hipStream_t st) {
  HwgArgs a{};
  a.N = d.N; a.H = d.H; a.W = d.W; a.C = d.C; a.K = d.K; a.KH = d.KH; a.KW = d.KW;
  a.PT = d.pad_top; a.PL = d.pad_left; a.wcin = d.w_cin;
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
