// Few-output-channel conv heads (K in {1,2,3,6}): disparity heads (nets_optflow_depth.py:122-144,
// DISP_SCALING*sigmoid(conv+b) [+MIN_DISP]; nets.py:122-144, 3-ch linear), flow heads (nets_depth.py:169-191,
// 2-ch linear), exp-mask
// logits (nets_optflow_depth.py:193-198, k 3/5/7) and pose/pred 1x1 (:181).  These GEMMs have N = 1..6
// and are HBM/L2-bound (arithmetic intensity ~K flop/B), so they are direct convolutions on the vector
// ALU with the activation and its derivative fused, not MFMA tiles padded to 16 columns.
//
//   fwd   : L lanes per output pixel split the (tap, channel-quad) reduction, xor-shuffle combine.
//   dz    : dz = dL/d(pre-activation) once per output element (workspace), reused by dgrad and wgrad.
//   dgrad : one thread per (input pixel, channel quad) gathers dz over the taps (stride 1).
//   wgrad : block = (pixel chunk, tap group); thread = (channel quad, pixel lane) keeps a
//           TT-tap x 4-channel x K register tile over its pixels, LDS combine over pixel lanes, then a
//           deterministic fixed-order reduction over chunks.
#include "tde_common.h"

typedef float f2 __attribute__((ext_vector_type(2)));

#include <cstdlib>

namespace {

struct HeadArgs {
  int N, H, W, C, OH, OW, K, KH, KW, S, PT, PL, wcin;
  const float* x; int xcs, xco;
  const float* w; const float* b;
  float* y; const float* yin; const float* dy; int ycs, yco;
  float* dx; int acc_dx;
  const float* dz;   // [M][K] dense (backward)
  float* dzw;        // same buffer, written by the wgrad pass
  int act; float scale, offset;
};

__device__ __forceinline__ float head_act(float z, int act, float scale, float offset) {
  return act ? scale / (1.f + __expf(-z)) + offset : z;
}

// dL/dz from y and dL/dy
__device__ __forceinline__ float head_dz(float y, float dy, int act, float scale, float offset) {
  if (!act) return dy;
  const float s = (y - offset) / scale;
  return dy * scale * s * (1.f - s);
}

template <int KC, int L>
__global__ void __launch_bounds__(256) head_fwd_kernel(const HeadArgs p) {
  constexpr int PPB = 256 / L;
  const int lane = threadIdx.x & (L - 1);
  const long M = (long)p.N * p.OH * p.OW;
  const int ohw = p.OH * p.OW;
  for (long m0 = (long)blockIdx.x * PPB; m0 < M; m0 += (long)gridDim.x * PPB) {
    const long m = m0 + threadIdx.x / L;
    float acc[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[k] = 0.f;
    if (m < M) {
      const int n = (int)(m / ohw), r = (int)(m - (long)n * ohw), oh = r / p.OW, ow = r - oh * p.OW;
      for (int kh = 0; kh < p.KH; ++kh) {
        const int ih = oh * p.S - p.PT + kh;
        if ((unsigned)ih >= (unsigned)p.H) continue;
        for (int kw = 0; kw < p.KW; ++kw) {
          const int iw = ow * p.S - p.PL + kw;
          if ((unsigned)iw >= (unsigned)p.W) continue;
          const float* xp = p.x + ((long)(n * p.H + ih) * p.W + iw) * p.xcs + p.xco;
          const float* wp = p.w + (long)(kh * p.KW + kw) * p.wcin * KC;
          for (int c = 4 * lane; c < p.wcin; c += 4 * L) {
            const f4 xv = *reinterpret_cast<const f4*>(xp + c);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c + j < p.wcin) {
#pragma unroll
                for (int k = 0; k < KC; ++k) acc[k] = fmaf(xv[j], wp[(c + j) * KC + k], acc[k]);
              }
          }
        }
      }
    }
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1)
#pragma unroll
      for (int k = 0; k < KC; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
    if (m < M && lane == 0) {
      float* yp = p.y + m * p.ycs + p.yco;
#pragma unroll
      for (int k = 0; k < KC; ++k) yp[k] = head_act(acc[k] + p.b[k], p.act, p.scale, p.offset);
    }
  }
}

// Weights of a head staged in LDS once per block: [tap][wcin][KC] (<= HEAD_WMAX floats; every head of
// the reference nets fits: 3x3x128x2, 7x7x16x2, 1x1x256x6).
constexpr int HEAD_WMAX = 4608;

__device__ __forceinline__ void stage_weights(const float* w, int n, float* sw) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
}

// Forward, taps unrolled (KS x KS, stride 1): L lanes per output pixel, each lane QPL channel quads;
// all of a lane's activation loads (KS*KS*QPL branch-free buffer loads) are issued before the FMAs,
// weights from LDS, xor-shuffle combine, bias + activation fused.
template <int KC, int KS, int L, int QPL>
__global__ void __launch_bounds__(256) head_fwd2_kernel(const HeadArgs p) {
  __shared__ __attribute__((aligned(16))) float sw[HEAD_WMAX];
  stage_weights(p.w, KS * KS * p.wcin * KC, sw);
  constexpr int PPB = 256 / L;
  const int lane = threadIdx.x & (L - 1);
  const long M = (long)p.N * p.OH * p.OW;
  const long m = (long)blockIdx.x * PPB + threadIdx.x / L;
  const int CQ = (p.wcin + 3) / 4;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  float acc[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) acc[k] = 0.f;
  const long mm = m < M ? m : 0;
  const int ohw = p.OH * p.OW;
  const int n = (int)(mm / ohw), r = (int)(mm - (long)n * ohw), oh = r / p.OW, ow = r - oh * p.OW;
  const int base = ((n * p.H + oh - p.PT) * p.W + ow - p.PL) * p.xcs + p.xco;
  f4 xv[KS * KS][QPL];
#pragma unroll
  for (int kh = 0; kh < KS; ++kh)
#pragma unroll
    for (int kw = 0; kw < KS; ++kw) {
      const bool ok = m < M && (unsigned)(oh - p.PT + kh) < (unsigned)p.H && (unsigned)(ow - p.PL + kw) < (unsigned)p.W;
#pragma unroll
      for (int u = 0; u < QPL; ++u) {
        const int cq = lane + u * L;
        xv[kh * KS + kw][u] = bload(rx, ok && cq < CQ ? 4 * (base + (kh * p.W + kw) * p.xcs + 4 * cq) : OOB);
      }
    }
#pragma unroll
  for (int t = 0; t < KS * KS; ++t) {
    const float* wp = sw + t * p.wcin * KC;
#pragma unroll
    for (int u = 0; u < QPL; ++u) {
      const int c0 = 4 * (lane + u * L);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c < p.wcin) {
#pragma unroll
          for (int k = 0; k < KC; ++k) acc[k] = fmaf(xv[t][u][j], wp[c * KC + k], acc[k]);
        }
      }
    }
  }
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
  if (m < M && lane == 0) {
    float* yp = p.y + m * p.ycs + p.yco;
#pragma unroll
    for (int k = 0; k < KC; ++k) yp[k] = head_act(acc[k] + p.b[k], p.act, p.scale, p.offset);
  }
}

// Data gradient, taps unrolled, weights from LDS: thread = (input pixel, channel quad), stride 1.
template <int KC, int KS>
__global__ void __launch_bounds__(256) head_dgrad2_kernel(const HeadArgs p) {
  __shared__ __attribute__((aligned(16))) float sw[HEAD_WMAX];
  stage_weights(p.w, KS * KS * p.wcin * KC, sw);
  const int CQ = p.C / 4;
  const long total = (long)p.N * p.H * p.W * CQ;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / CQ;
    const int c = 4 * (int)(i - pix * CQ);
    const int hw = p.H * p.W;
    const int n = (int)(pix / hw), r = (int)(pix - (long)n * hw), ih = r / p.W, iw = r - ih * p.W;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c < p.wcin) {
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        const int oh = ih + p.PT - kh;
        if ((unsigned)oh >= (unsigned)p.OH) continue;
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const int ow = iw + p.PL - kw;
          if ((unsigned)ow >= (unsigned)p.OW) continue;
          const float* dzp = p.dz + ((long)(n * p.OH + oh) * p.OW + ow) * KC;
          const float* wp = sw + ((kh * KS + kw) * p.wcin + c) * KC;
#pragma unroll
          for (int k = 0; k < KC; ++k) {
            const float dz = dzp[k];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c + j < p.wcin) acc[j] = fmaf(dz, wp[j * KC + k], acc[j]);
          }
        }
      }
    }
    float* dst = p.dx + pix * p.xcs + p.xco + c;
    f4 out = acc;
    if (p.acc_dx) out += *reinterpret_cast<const f4*>(dst);
    *reinterpret_cast<f4*>(dst) = out;
  }
}

__global__ void __launch_bounds__(256) head_dz_kernel(long M, int K, const float* y, const float* dy, int ycs,
                                                      int yco, int act, float scale, float offset, float* dz) {
  const long total = M * K;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long m = i / K;
    const int k = (int)(i - m * K);
    const long o = m * ycs + yco + k;
    dz[i] = head_dz(y[o], dy[o], act, scale, offset);
  }
}

// dx[n,ih,iw,c..c+3] = sum_{kh,kw,k} dz[n,oh,ow,k] w[kh,kw,c,k], stride-1 heads only.
template <int KC>
__global__ void __launch_bounds__(256) head_dgrad_kernel(const HeadArgs p) {
  const int CQ = p.C / 4;
  const long total = (long)p.N * p.H * p.W * CQ;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / CQ;
    const int c = 4 * (int)(i - pix * CQ);
    const int hw = p.H * p.W;
    const int n = (int)(pix / hw), r = (int)(pix - (long)n * hw), ih = r / p.W, iw = r - ih * p.W;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c < p.wcin) {
      for (int kh = 0; kh < p.KH; ++kh) {
        const int oh = ih + p.PT - kh;
        if ((unsigned)oh >= (unsigned)p.OH) continue;
        for (int kw = 0; kw < p.KW; ++kw) {
          const int ow = iw + p.PL - kw;
          if ((unsigned)ow >= (unsigned)p.OW) continue;
          const float* dzp = p.dz + ((long)(n * p.OH + oh) * p.OW + ow) * KC;
          const float* wp = p.w + (long)(kh * p.KW + kw) * p.wcin * KC;
#pragma unroll
          for (int k = 0; k < KC; ++k) {
            const float dz = dzp[k];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c + j < p.wcin) acc[j] = fmaf(dz, wp[(c + j) * KC + k], acc[j]);
          }
        }
      }
    }
    float* dst = p.dx + pix * p.xcs + p.xco + c;
    f4 out = acc;
    if (p.acc_dx) out += *reinterpret_cast<const f4*>(dst);
    *reinterpret_cast<f4*>(dst) = out;
  }
}

// ------------------------------------------------------------------ tiled heads (high resolution, C <= 64)
// The direct kernels above re-read every activation once per tap from L1/L2 (49x for the 7x7 mask1 head of
// depth_net: 1.2 GB of cache traffic per config-4 call).  These stage an output tile's input halo in LDS once
// per 4-channel chunk and slide a register window along each thread's row segment, so each staged value
// feeds KS x PX x KC FMAs.  Weights are wave-uniform (scalar loads).  Stride 1, KS x KS, K <= 2.
//   tfwd  : thread = 4 consecutive output pixels of one row, all K outputs; halo chunks double-buffered.
//   tdgrad: thread = 4 consecutive input pixels x 16 channels; the dz halo (computed from y, dy at staging).
//   twgrad: thread = (kernel row, row lane); a KS x 4 x K register tile per chunk, lane sums by xor shuffles,
//           one partial row per tile (head_wgrad_reduce_kernel sums the tiles in a fixed order).
constexpr int HT_TW = 64, HT_TH = 16, HT_PX = 4, HT_SEG = HT_TW / HT_PX;

template <int KS, int TH = HT_TH>
struct HaloGeom {
  static constexpr int HW = HT_TW + KS - 1;        // halo width (pixels)
  static constexpr int PITCH = HW | 1;             // odd f4 row pitch: rows of a lane group hit distinct banks
  static constexpr int HH = TH + KS - 1;
  static constexpr int NSLOT = HH * PITCH;
  static constexpr int LPT = (HH * HW + 255) / 256;   // staging loads per thread
};

struct TileIdx {
  int n, oh0, ow0;
};
__device__ __forceinline__ TileIdx tile_of(int b, int tiles_w, int tiles_h, int th) {
  TileIdx t;
  const int tw = b % tiles_w;
  const int r = b / tiles_w;
  t.oh0 = (r % tiles_h) * th;
  t.n = r / tiles_h;
  t.ow0 = tw * HT_TW;
  return t;
}

// halo element i of channel chunk cq: byte offset into x (or OOB)
template <int KS, int TH = HT_TH>
__device__ __forceinline__ int halo_off(const HeadArgs& p, const TileIdx& t, int i, int cq) {
  using G = HaloGeom<KS, TH>;
  const int hr = i / G::HW, hc = i - hr * G::HW;
  const int ih = t.oh0 - p.PT + hr, iw = t.ow0 - p.PL + hc;
  const bool ok = i < G::HH * G::HW && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W && 4 * cq < p.wcin;
  return ok ? 4 * (((t.n * p.H + ih) * p.W + iw) * p.xcs + p.xco + 4 * cq) : OOB;
}

template <int KS, int TH = HT_TH>
__device__ __forceinline__ void halo_fetch(const HeadArgs& p, __amdgpu_buffer_rsrc_t rx, const TileIdx& t, int cq,
                                           f4 (&r)[HaloGeom<KS, TH>::LPT]) {
#pragma unroll
  for (int u = 0; u < HaloGeom<KS, TH>::LPT; ++u) r[u] = bload(rx, halo_off<KS, TH>(p, t, threadIdx.x + 256 * u, cq));
}

template <int KS, int TH = HT_TH>
__device__ __forceinline__ void halo_store(f4* sx, const f4 (&r)[HaloGeom<KS, TH>::LPT]) {
  using G = HaloGeom<KS, TH>;
#pragma unroll
  for (int u = 0; u < G::LPT; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < G::HH * G::HW) {
      const int hr = i / G::HW, hc = i - hr * G::HW;
      sx[hr * G::PITCH + hc] = r[u];
    }
  }
}

// Weights staged in LDS as [tap][k][c] over the channel count padded to 4 (zeros past w_cin), so the quad
// of 4 channels a thread multiplies is one wave-uniform (broadcast) ds_read_b128.  Capacity: KS^2 * C * K
// <= 3200 floats (head_tiled: C <= 32 at KS 7, C <= 64 at KS <= 5).
constexpr int HT_WMAX = 3200;

template <int KC, int KS>
__device__ __forceinline__ void stage_wt(const HeadArgs& p, float* sw) {
  const int cp = (p.wcin + 3) & ~3;
  const int n = KS * KS * KC * cp;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = i % cp, r = i / cp, k = r % KC, tap = r / KC;
    sw[i] = c < p.wcin ? p.w[((long)tap * p.wcin + c) * KC + k] : 0.f;
  }
}

__device__ __forceinline__ f4 wquad(const float* sw, int tap, int c, int cp, int KC, int k) {
  return *reinterpret_cast<const f4*>(sw + (tap * KC + k) * cp + c);
}

template <int KC, int KS>
__global__ void __launch_bounds__(256) head_tfwd_kernel(const HeadArgs p, int tiles_w, int tiles_h) {
  using G = HaloGeom<KS>;
  __shared__ f4 sx[2][G::NSLOT];
  __shared__ __attribute__((aligned(16))) float sw[HT_WMAX];
  const TileIdx t = tile_of(blockIdx.x, tiles_w, tiles_h, HT_TH);
  const int row = threadIdx.x % HT_TH, x0 = (threadIdx.x / HT_TH) * HT_PX;
  const int cp = (p.wcin + 3) & ~3;
  stage_wt<KC, KS>(p, sw);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const int CQ = (p.wcin + 3) / 4;
  float acc[HT_PX][KC];
#pragma unroll
  for (int i = 0; i < HT_PX; ++i)
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[i][k] = 0.f;
  f4 r[G::LPT];
  halo_fetch<KS>(p, rx, t, 0, r);
  halo_store<KS>(sx[0], r);
  __syncthreads();
  for (int cq = 0; cq < CQ; ++cq) {
    if (cq + 1 < CQ) halo_fetch<KS>(p, rx, t, cq + 1, r);
    const f4* s = sx[cq & 1];
#pragma unroll 1
    for (int kh = 0; kh < KS; ++kh) {
      f4 win[HT_PX + KS - 1];
#pragma unroll
      for (int j = 0; j < HT_PX + KS - 1; ++j) win[j] = s[(row + kh) * G::PITCH + x0 + j];
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const f4 wv = wquad(sw, kh * KS + kw, 4 * cq, cp, KC, k);
#pragma unroll
          for (int i = 0; i < HT_PX; ++i) {
            const f4 xv = win[i + kw];
            acc[i][k] = fmaf(xv[0], wv[0], fmaf(xv[1], wv[1], fmaf(xv[2], wv[2], fmaf(xv[3], wv[3], acc[i][k]))));
          }
        }
        // keep each tap's weight reads next to their FMAs (hoisting all taps' reads costs occupancy)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (cq + 1 < CQ) halo_store<KS>(sx[(cq + 1) & 1], r);
    __syncthreads();
  }
  const int oh = t.oh0 + row;
  if (oh >= p.OH) return;
#pragma unroll
  for (int i = 0; i < HT_PX; ++i) {
    const int ow = t.ow0 + x0 + i;
    if (ow < p.OW) {
      float* yp = p.y + ((long)(t.n * p.OH + oh) * p.OW + ow) * p.ycs + p.yco;
#pragma unroll
      for (int k = 0; k < KC; ++k) yp[k] = head_act(acc[i][k] + p.b[k], p.act, p.scale, p.offset);
    }
  }
}

// dz = dL/d(pre-activation) of output pixel (oh, ow), zero outside the image
template <int KC>
__device__ __forceinline__ void dz_at(const HeadArgs& p, int n, int oh, int ow, float (&d)[KC]) {
  const bool ok = (unsigned)oh < (unsigned)p.OH && (unsigned)ow < (unsigned)p.OW;
  const long o = ((long)(n * p.OH + (ok ? oh : 0)) * p.OW + (ok ? ow : 0)) * p.ycs + p.yco;
#pragma unroll
  for (int k = 0; k < KC; ++k) d[k] = ok ? head_dz(p.yin[o + k], p.dy[o + k], p.act, p.scale, p.offset) : 0.f;
}

// NG channel groups of 16 (C = 16 * NG); rows per tile 16 / NG
template <int KC, int KS, int NG>
__global__ void __launch_bounds__(256) head_tdgrad_kernel(const HeadArgs p, int tiles_w, int tiles_h) {
  constexpr int TH = HT_TH / NG, HW = HT_TW + KS - 1, PITCH = HW | 1, HH = TH + KS - 1;
  constexpr int CG = 16;
  __shared__ float sdz[HH * PITCH * KC];
  __shared__ __attribute__((aligned(16))) float sw[HT_WMAX];
  const TileIdx t = tile_of(blockIdx.x, tiles_w, tiles_h, TH);
  const int cp = (p.wcin + 3) & ~3;
  stage_wt<KC, KS>(p, sw);
  // dz halo: output pixels (ih0 + PT - (KS-1) + hr, iw0 + PL - (KS-1) + hc)
  for (int i = threadIdx.x; i < HH * HW; i += 256) {
    const int hr = i / HW, hc = i - hr * HW;
    float d[KC];
    dz_at<KC>(p, t.n, t.oh0 + p.PT - (KS - 1) + hr, t.ow0 + p.PL - (KS - 1) + hc, d);
#pragma unroll
    for (int k = 0; k < KC; ++k) sdz[(hr * PITCH + hc) * KC + k] = d[k];
  }
  __syncthreads();
  const int row = threadIdx.x % TH, seg = (threadIdx.x / TH) % HT_SEG, g = threadIdx.x / (TH * HT_SEG);
  const int x0 = seg * HT_PX, c0 = g * CG;
  f4 acc[HT_PX][CG / 4];
#pragma unroll
  for (int i = 0; i < HT_PX; ++i)
#pragma unroll
    for (int q = 0; q < CG / 4; ++q) acc[i][q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kh = 0; kh < KS; ++kh) {
#pragma unroll 1
    for (int kw = 0; kw < KS; ++kw) {
      // dz of the 4 output pixels this tap maps the thread's input pixels to, and the tap's weight quads
      const float* dzp = sdz + ((row + KS - 1 - kh) * PITCH + x0 + KS - 1 - kw) * KC;
      float dv[HT_PX][KC];
#pragma unroll
      for (int i = 0; i < HT_PX; ++i)
#pragma unroll
        for (int k = 0; k < KC; ++k) dv[i][k] = dzp[i * KC + k];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
#pragma unroll
        for (int q = 0; q < CG / 4; ++q) {
          const f4 wv = c0 + 4 * q < cp ? wquad(sw, kh * KS + kw, c0 + 4 * q, cp, KC, k) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < HT_PX; ++i) acc[i][q] += dv[i][k] * wv;
        }
      }
    }
  }
  const int ih = t.oh0 + row;
  if (ih >= p.H) return;
#pragma unroll
  for (int i = 0; i < HT_PX; ++i) {
    const int iw = t.ow0 + x0 + i;
    if (iw < p.W) {
      float* dst = p.dx + ((long)(t.n * p.H + ih) * p.W + iw) * p.xcs + p.xco + c0;
#pragma unroll
      for (int q = 0; q < CG / 4; ++q) {
        f4 o = acc[i][q];
        if (p.acc_dx) o += *reinterpret_cast<const f4*>(dst + 4 * q);
        *reinterpret_cast<f4*>(dst + 4 * q) = o;
      }
    }
  }
}

// lanes per tap: L consecutive lanes share one tap's outputs and split the tile's pixels (xor-shuffle sum
// within L <= 16 lanes); KS 3 / 5 / 7 -> 144 / 200 / 196 active threads
template <int KS>
struct TwLanes { static constexpr int L = KS == 3 ? 16 : (KS == 5 ? 8 : 4); };
constexpr int HT_TWG_TH = 8;   // filter-gradient tile rows (more tiles than the forward's 16: fills the chip)

template <int KC, int KS>
__global__ void __launch_bounds__(256) head_twgrad_kernel(const HeadArgs p, int tiles_w, int tiles_h, float* part) {
  constexpr int TH = HT_TWG_TH;
  using G = HaloGeom<KS, TH>;
  constexpr int L = TwLanes<KS>::L, NPX = TH * HT_TW;
  __shared__ f4 sx[2][G::NSLOT];
  __shared__ float sdz[NPX * KC];
  __shared__ float sb[4][KC];
  const TileIdx t = tile_of(blockIdx.x, tiles_w, tiles_h, TH);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const int E = KS * KS * p.wcin;
  // partials transposed, part[output][tile]: head_wgrad_reduce_t_kernel reads each output's row contiguously
  const long R = gridDim.x;
  float* out = part + blockIdx.x;
  f4 r[G::LPT];
  halo_fetch<KS, TH>(p, rx, t, 0, r);
  // dz of the tile's own output pixels, and their sums (the bias gradient)
  float bs[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) bs[k] = 0.f;
  for (int i = threadIdx.x; i < NPX; i += 256) {
    float d[KC];
    dz_at<KC>(p, t.n, t.oh0 + i / HT_TW, t.ow0 + i % HT_TW, d);
#pragma unroll
    for (int k = 0; k < KC; ++k) { sdz[i * KC + k] = d[k]; bs[k] += d[k]; }
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bs[k] += __shfl_xor(bs[k], o, 64);
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6][k] = bs[k];
  }
  halo_store<KS, TH>(sx[0], r);
  __syncthreads();
  if (threadIdx.x < KC)
    out[(E * KC + threadIdx.x) * R] = ((sb[0][threadIdx.x] + sb[1][threadIdx.x]) + sb[2][threadIdx.x]) + sb[3][threadIdx.x];
  const int tap = threadIdx.x / L, l = threadIdx.x % L;
  const int kh = tap / KS, kw = tap - kh * KS;
  const bool active = tap < KS * KS;
  const int CQ = (p.wcin + 3) / 4;
  for (int cq = 0; cq < CQ; ++cq) {
    if (cq + 1 < CQ) halo_fetch<KS, TH>(p, rx, t, cq + 1, r);
    float acc[4][KC];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) acc[j][k] = 0.f;
    if (active) {
      const f4* s = sx[cq & 1] + kh * G::PITCH + kw;
#pragma unroll 8
      for (int px = l; px < NPX; px += L) {
        const int row = px / HT_TW, col = px - row * HT_TW;
        const f4 xv = s[row * G::PITCH + col];
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const float d = sdz[px * KC + k];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j][k] = fmaf(xv[j], d, acc[j][k]);
        }
      }
    }
    // sum over the L lanes of this tap (fixed xor order), lane 0 writes the tile's partial
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        float v = acc[j][k];
#pragma unroll
        for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[j][k] = v;
      }
    if (active && l == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 4 * cq + j;
        if (c < p.wcin)
#pragma unroll
          for (int k = 0; k < KC; ++k) out[((tap * p.wcin + c) * KC + k) * R] = acc[j][k];
      }
    }
    if (cq + 1 < CQ) halo_store<KS, TH>(sx[(cq + 1) & 1], r);
    __syncthreads();
  }
}

// taps per wgrad block: TT * 4 * KC accumulators per thread
template <int KC>
struct WgTaps { static constexpr int TT = KC == 1 ? 9 : (KC == 2 ? 5 : (KC == 3 ? 3 : 2)); };

constexpr int WG_MAX_CHUNKS = 1024;

// part[chunk][e * KC + k] for e = tap * wcin + c (only this block's taps), plus part[chunk][E*KC + k]
// = bias sums (tap group 0).
template <int KC>
__global__ void __launch_bounds__(256) head_wgrad_partial_kernel(const HeadArgs p, float* part, int pix_per_chunk) {
  constexpr int TT = WgTaps<KC>::TT;
  constexpr int NV = TT * 4 * KC;
  __shared__ float sred[256 * NV];
  const long M = (long)p.N * p.OH * p.OW;
  const int CQ = p.C / 4;
  const int P = 256 / CQ;                     // pixel lanes (CQ <= 64)
  const int q = (int)threadIdx.x % CQ, pl = (int)threadIdx.x / CQ;
  const int ntaps = p.KH * p.KW;
  const int t0 = blockIdx.y * TT;
  const int nt = min(TT, ntaps - t0);
  const long cbeg = (long)blockIdx.x * pix_per_chunk;
  const long cend = min(M, cbeg + pix_per_chunk);
  const int ohw = p.OH * p.OW;
  int tkh[TT], tkw[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int tap = min(t0 + t, ntaps - 1);
    tkh[t] = tap / p.KW - p.PT;
    tkw[t] = tap - (tap / p.KW) * p.KW - p.PL;
  }
  float acc[TT][4][KC];
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) acc[t][j][k] = 0.f;
  float bacc[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) bacc[k] = 0.f;
  if (pl < P) {
    for (long pix = cbeg + pl; pix < cend; pix += P) {
      // dL/dz from y and dL/dy (sigmoid head) computed here; tap group 0's first channel-quad lane
      // stores it for the data-gradient pass
      float dz[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const long o = pix * p.ycs + p.yco + k;
        dz[k] = head_dz(p.yin[o], p.dy[o], p.act, p.scale, p.offset);
      }
      if (blockIdx.y == 0 && q == 0) {
#pragma unroll
        for (int k = 0; k < KC; ++k) p.dzw[pix * KC + k] = dz[k];
      }
#pragma unroll
      for (int k = 0; k < KC; ++k) bacc[k] += dz[k];
      const int n = (int)(pix / ohw), r = (int)(pix - (long)n * ohw), oh = r / p.OW, ow = r - oh * p.OW;
      const float* xb = p.x + (long)n * p.H * p.W * p.xcs + p.xco + 4 * q;
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const int ih = oh * p.S + tkh[t], iw = ow * p.S + tkw[t];
        if (t < nt && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) {
          const f4 xv = *reinterpret_cast<const f4*>(xb + ((long)ih * p.W + iw) * p.xcs);
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < KC; ++k) acc[t][j][k] = fmaf(xv[j], dz[k], acc[t][j][k]);
        }
      }
    }
  }
  // combine the P pixel lanes: sred[thread][t][j][k]
  float* mine = sred + threadIdx.x * NV;
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) mine[(t * 4 + j) * KC + k] = acc[t][j][k];
  __syncthreads();
  const int E = ntaps * p.wcin;
  float* out = part + (long)blockIdx.x * (E * KC + KC);
  const int nout = nt * CQ * 4 * KC;
  for (int o = threadIdx.x; o < nout; o += 256) {
    const int k = o % KC, cj = (o / KC) % (CQ * 4), t = o / (KC * CQ * 4);
    const int qq = cj >> 2, j = cj & 3;
    const int c = 4 * qq + j;
    if (c >= p.wcin) continue;
    float s = 0.f;
    for (int l = 0; l < P; ++l) s += sred[(l * CQ + qq) * NV + (t * 4 + j) * KC + k];
    out[((t0 + t) * p.wcin + c) * KC + k] = s;
  }
  if (blockIdx.y == 0) {
    __syncthreads();
    if (q == 0 && pl < P)
#pragma unroll
      for (int k = 0; k < KC; ++k) sred[pl * KC + k] = bacc[k];
    __syncthreads();
    if (threadIdx.x < KC) {
      float s = 0.f;
      for (int l = 0; l < P; ++l) s += sred[l * KC + threadIdx.x];
      out[E * KC + threadIdx.x] = s;
    }
  }
}

// 64 outputs per block, 16 waves split the chunk range with 4 loads in flight each, fp64 fixed-order
// combine through LDS.
__global__ void __launch_bounds__(1024) head_wgrad_reduce_kernel(const float* part, int chunks, int total,
                                                                  int nw, float* dw, float* db, int accumulate) {
  __shared__ double sh[1024];
  const int il = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + il;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (i < total) {
    int ch = w;
    for (; ch + 48 < chunks; ch += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(long)(ch + 16 * u) * total + i];
    }
    for (int u = 0; ch < chunks; ch += 16, ++u) a[u & 3] += part[(long)ch * total + i];
  }
  sh[threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w != 0 || i >= total) return;
  double s = 0.0;
#pragma unroll
  for (int v = 0; v < 16; ++v) s += sh[il + 64 * v];
  float* dst = (i < nw) ? dw + i : db + (i - nw);
  *dst = accumulate ? *dst + (float)s : (float)s;
}

// Sum of the transposed tiled partials part[output][rows]: one wave per output, lanes over rows in a fixed
// order (fp64), xor-tree combine.
__global__ void __launch_bounds__(64) head_wgrad_reduce_t_kernel(const float* part, int rows, int nw, float* dw,
                                                                  float* db, int accumulate) {
  const float* src = part + (long)blockIdx.x * rows;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  int r = threadIdx.x;
  for (; r + 192 < rows; r += 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += src[r + 64 * u];
  }
  for (int u = 0; r < rows; r += 64, ++u) a[u & 3] += src[r];
  double s = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (threadIdx.x == 0) {
    const int i = blockIdx.x;
    float* dst = (i < nw) ? dw + i : db + (i - nw);
    *dst = accumulate ? *dst + (float)s : (float)s;
  }
}

// ------------------------------------------------------------------ row-walk 3x3 heads (round 4)
// The disparity heads (nets_optflow_depth.py:122-144: 3x3, stride 1, one output; the masks' 3x3 level too) at the
// high resolutions are pure streams -- ~9 FMAs per input byte -- and the halo-tiled kernels above ran them at a
// quarter to a sixth of the HBM rate (rocprofv3, config 4: disp fwd 23 us, wgrad 31 us per call against ~8 us of
// reads for disp1).  Here no LDS staging and no barrier in the loop: thread = (channel quad q, 16-pixel segment of
// one row); it walks its segment with a 3 x 3 window of f4 in registers, loading one new input column (3 f4) per
// pixel (unrolled by 4: 12 loads in flight), weights in registers.  The CQ = C/4 lanes of a pixel are adjacent, so a
// pixel's channels are one contiguous read and its quads combine by xor shuffles.  Rows r-1..r+1 of one image are
// walked by neighbouring threads of the same block (their reads meet in L1/L2): x leaves HBM about once.
constexpr int RW_SEG = 16;    // output pixels per thread

struct RwGeom {
  int CQ, segs, rows;   // lanes per pixel, segments per row, N * OH rows
};
__device__ __forceinline__ void rw_decode(const HeadArgs& p, int CQ, int segs, long t, int& q, int& x0, int& n,
                                          int& r) {
  q = (int)(t % CQ);
  const long u = t / CQ;
  x0 = (int)(u % segs) * RW_SEG;
  const long rr = u / segs;
  n = (int)(rr / p.OH);
  r = (int)(rr - (long)n * p.OH);
}

// x quad at (n, ih, iw) or 0 outside the image (buffer load: branch-free)
__device__ __forceinline__ f4 rw_x(const HeadArgs& p, __amdgpu_buffer_rsrc_t rx, int n, int ih, int iw, int q) {
  const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
  return bload(rx, ok ? 4 * (((n * p.H + ih) * p.W + iw) * p.xcs + p.xco + 4 * q) : OOB);
}

template <int KC>
__global__ void __launch_bounds__(256) head_rw_fwd_kernel(const HeadArgs p, int CQ, int segs, long threads) {
  const long t = blockIdx.x * 256L + threadIdx.x;
  int q, x0, n, r;
  rw_decode(p, CQ, segs, t < threads ? t : 0, q, x0, n, r);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  float w[9][4][KC];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) w[tap][j][k] = p.w[(tap * p.wcin + 4 * q + j) * KC + k];
  // window columns x0-1, x0 (rows r-1 .. r+1); column x0+1+i is loaded at step i
  f4 win[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    win[kh][0] = rw_x(p, rx, n, r + kh - 1, x0 - 1, q);
    win[kh][1] = rw_x(p, rx, n, r + kh - 1, x0, q);
  }
  const int lanebase = (int)(threadIdx.x & 63) & ~(CQ - 1);
  for (int i0 = 0; i0 < RW_SEG; i0 += 4) {
    f4 col[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) col[u][kh] = rw_x(p, rx, n, r + kh - 1, x0 + i0 + u + 1, q);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) win[kh][2] = col[u][kh];
      float acc[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) acc[k] = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < KC; ++k) acc[k] = fmaf(win[kh][kw][j], w[kh * 3 + kw][j][k], acc[k]);
      // the CQ quads of this pixel: xor tree over the adjacent lanes (fixed order)
      for (int o = 1; o < CQ; o <<= 1)
#pragma unroll
        for (int k = 0; k < KC; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
      const int ow = x0 + i0 + u;
      if (q == 0 && t < threads && ow < p.OW) {
        float* yp = p.y + ((long)(n * p.OH + r) * p.OW + ow) * p.ycs + p.yco;
#pragma unroll
        for (int k = 0; k < KC; ++k) yp[k] = head_act(acc[k] + p.b[k], p.act, p.scale, p.offset);
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) { win[kh][0] = win[kh][1]; win[kh][1] = win[kh][2]; }
    }
  }
  (void)lanebase;
}

// dz (dL / d pre-activation) at output pixel (n, oh, ow), zero outside the image
template <int KC>
__device__ __forceinline__ void rw_dz(const HeadArgs& p, int n, int oh, int ow, float (&d)[KC]) {
  dz_at<KC>(p, n, oh, ow, d);
}

// Filter gradient partials: per block, dW[tap][c][k] (+ the bias sums) over its threads' pixels, written
// transposed part[output][block] for head_wgrad_reduce_t_kernel (fixed-order fp64 sums over blocks).
template <int KC>
__global__ void __launch_bounds__(256) head_rw_wgrad_kernel(const HeadArgs p, int CQ, int segs, long threads,
                                                            float* part) {
  constexpr int NA = 9 * 4 * KC;
  __shared__ float red[4 * 16 * (NA + KC)];
  const long t = blockIdx.x * 256L + threadIdx.x;
  int q, x0, n, r;
  rw_decode(p, CQ, segs, t < threads ? t : 0, q, x0, n, r);
  const bool live = t < threads;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  float acc[9][4][KC], bacc[KC];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) acc[tap][j][k] = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) bacc[k] = 0.f;
  f4 win[3][3];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    win[kh][0] = rw_x(p, rx, n, r + kh - 1, x0 - 1, q);
    win[kh][1] = rw_x(p, rx, n, r + kh - 1, x0, q);
  }
  for (int i0 = 0; i0 < RW_SEG; i0 += 4) {
    f4 col[4][3];
    float d[4][KC];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) col[u][kh] = rw_x(p, rx, n, r + kh - 1, x0 + i0 + u + 1, q);
      const int ow = x0 + i0 + u;
      rw_dz<KC>(p, n, live ? r : p.OH, ow, d[u]);          // outside the image (or a dead thread): 0
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) win[kh][2] = col[u][kh];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < KC; ++k) acc[kh * 3 + kw][j][k] = fmaf(win[kh][kw][j], d[u][k], acc[kh * 3 + kw][j][k]);
#pragma unroll
      for (int k = 0; k < KC; ++k) bacc[k] += d[u][k];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) { win[kh][0] = win[kh][1]; win[kh][1] = win[kh][2]; }
    }
  }
  // block combine (fixed order): xor tree over the lanes of a wave that hold the same quad (lane bits >= log2 CQ),
  // then the 4 waves' sums through LDS in wave order
  for (int o = CQ; o < 64; o <<= 1) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < KC; ++k) acc[tap][j][k] += __shfl_xor(acc[tap][j][k], o, 64);
#pragma unroll
    for (int k = 0; k < KC; ++k) bacc[k] += __shfl_xor(bacc[k], o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < CQ) {
    float* mine = red + (wv * 16 + lane) * (NA + KC);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < KC; ++k) mine[(tap * 4 + j) * KC + k] = acc[tap][j][k];
#pragma unroll
    for (int k = 0; k < KC; ++k) mine[NA + k] = bacc[k];     // (every quad lane summed the same dz: quad 0's is used)
  }
  __syncthreads();
  const int E = 9 * p.wcin;
  const long R = gridDim.x;
  const int nout = E * KC + KC;
  for (int o = threadIdx.x; o < nout; o += 256) {
    int qq = 0, slot;
    if (o < E * KC) {
      const int k = o % KC, e = o / KC, tap = e / p.wcin, c = e - tap * p.wcin;
      qq = c >> 2;
      slot = (tap * 4 + (c & 3)) * KC + k;
    } else {
      slot = NA + (o - E * KC);
    }
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += red[(w * 16 + qq) * (NA + KC) + slot];
    part[(long)o * R + blockIdx.x] = s;
  }
}

// ------------------------------------------------------------------ row-walk 5x5 / 7x7 filter gradients (round 5)
// The explainability-mask heads' filter gradients (nets_optflow_depth_pairtest.py:198-206: mask2 5x5 over 32
// channels at 1/2 resolution, mask1 7x7 over 16 channels at full resolution, 2 outputs each) on the halo-tiled
// kernel read every staged value once per tap from LDS with ~3 LDS reads per 8 FMAs: 97 us for mask1 (config 4)
// against ~16 us of packed-FMA work.  Here block row y = kernel row kh; thread = (channel quad q, SEG-pixel segment of
// one output row r) walks its segment with a KS-wide window of x quads (input row r + kh - PT) in registers, one new
// quad and one dz pair per pixel, and accumulates dW[kh][kw][4q..4q+3][0..1] for all KS kw as float2 (k0, k1) pairs:
// KS x 4 packed FMAs per pixel, no LDS in the loop.  The CQ lanes of a pixel are adjacent (its channels one
// contiguous read); blocks combine their lanes in a fixed order and write one partial per output, summed over the
// blocks by head_wgrad_reduce_t_kernel.
// Segment = 4 groups of KS pixels: within a group the window is a ring of KS registers indexed by (pixel + kw) % KS
// at compile time (fully unrolled), so sliding it costs no moves; dz comes from the dense dz pass (one float2 per
// pixel).
template <int KS>
struct Rwk { static constexpr int SEG = 4 * KS; };

template <int KS>
__global__ void __launch_bounds__(256) head_rwk_wgrad_kernel(const HeadArgs p, int CQ, int segs, long threads,
                                                             float* part) {
  constexpr int NA = KS * 4;          // float2 accumulators per thread (kw, channel)
  constexpr int SEG = Rwk<KS>::SEG;
  __shared__ f2 red[4][16][NA + 1];
  const int kh = blockIdx.y;
  const long t = blockIdx.x * 256L + threadIdx.x;
  const bool live = t < threads;
  const long tt = live ? t : 0;
  const int q = (int)(tt % CQ);
  const long u_ = tt / CQ;
  const int x0 = (int)(u_ % segs) * SEG;
  const long rr = u_ / segs;
  const int n = (int)(rr / p.OH), r = (int)(rr - (long)n * p.OH);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const __amdgpu_buffer_rsrc_t rdz = make_rsrc(p.dz, (long)p.N * p.OH * p.OW * 2);
  const int ih = live ? r + kh - p.PT : -1;   // a dead thread reads zeros
  const long dzrow = ((long)n * p.OH + r) * p.OW;
  f2 acc[KS][4], bacc = {0.f, 0.f};
#pragma unroll
  for (int kw = 0; kw < KS; ++kw)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[kw][j] = f2{0.f, 0.f};
  // ring slot m % KS holds input column x0 - PL + m
  f4 win[KS];
#pragma unroll
  for (int m = 0; m < KS - 1; ++m) win[m] = rw_x(p, rx, n, ih, x0 - p.PL + m, q);
  // per group: its KS new input columns and dz pairs, all loads issued before the first FMA.  (Prefetching the next
  // group's beside this one's FMAs measured slower: 220 VGPRs, 2 waves per SIMD; mask1 at batch 16 96 vs 78 us.)
#pragma unroll 1
  for (int g0 = 0; g0 < SEG; g0 += KS) {
    f4 col[KS];
    f2 d[KS];
#pragma unroll
    for (int u = 0; u < KS; ++u) {
      const int ow = x0 + g0 + u;
      col[u] = rw_x(p, rx, n, ih, ow - p.PL + KS - 1, q);
      const bool ok = live && ow < p.OW;
      d[u] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rdz, ok ? 8 * (int)(dzrow + ow) : OOB, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < KS; ++u) {
      win[(u + KS - 1) % KS] = col[u];
#pragma unroll
      for (int kw = 0; kw < KS; ++kw)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[kw][j] = win[(u + kw) % KS][j] * d[u] + acc[kw][j];
      bacc += d[u];
    }
  }
  // block combine (fixed order): xor tree over the lanes of a wave holding the same quad, then the 4 waves via LDS
  for (int o = CQ; o < 64; o <<= 1) {
#pragma unroll
    for (int kw = 0; kw < KS; ++kw)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[kw][j].x += __shfl_xor(acc[kw][j].x, o, 64);
        acc[kw][j].y += __shfl_xor(acc[kw][j].y, o, 64);
      }
    bacc.x += __shfl_xor(bacc.x, o, 64);
    bacc.y += __shfl_xor(bacc.y, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < CQ) {
#pragma unroll
    for (int kw = 0; kw < KS; ++kw)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wv][lane][kw * 4 + j] = acc[kw][j];
    red[wv][lane][NA] = bacc;
  }
  __syncthreads();
  // outputs of this kernel row: e = ((kh KS + kw) wcin + c) K + k for c < wcin; kernel row 0 also the bias sums
  const long R = gridDim.x;
  const int nrow = KS * p.wcin * 2;
  const int nout = nrow + (kh == 0 ? 2 : 0);
  for (int o = threadIdx.x; o < nout; o += 256) {
    int qq = 0, slot = NA, k = o & 1;
    long dst;
    if (o < nrow) {
      const int e = o >> 1, kw = e / p.wcin, c = e - kw * p.wcin;
      qq = c >> 2;
      slot = kw * 4 + (c & 3);
      dst = (long)((kh * KS + kw) * p.wcin + c) * 2 + k;
    } else {
      k = o - nrow;
      dst = (long)KS * KS * p.wcin * 2 + k;   // (every quad lane summed the same dz: quad 0's is used)
    }
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += k ? red[w][qq][slot].y : red[w][qq][slot].x;
    part[dst * R + blockIdx.x] = v;
  }
}

// Data gradient: thread = (channel quad, 16-pixel segment of one input row); a 3 x 3 window of dz (KC floats each,
// recomputed from y, dy) slides along the row, weights in registers.
template <int KC>
__global__ void __launch_bounds__(256) head_rw_dgrad_kernel(const HeadArgs p, int CQ, int segs, long threads) {
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= threads) return;
  int q, x0, n, r;
  rw_decode(p, CQ, segs, t, q, x0, n, r);     // (input pixels: H = OH, W = OW for the stride-1 SAME heads)
  float w[9][4][KC];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < KC; ++k) w[tap][j][k] = p.w[(tap * p.wcin + 4 * q + j) * KC + k];
  // dz window: rows r+1, r, r-1 (tap kh = 0, 1, 2 reads output row r + 1 - kh), columns iw+1, iw, iw-1
  float dw_[3][3][KC];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    rw_dz<KC>(p, n, r + 1 - kh, x0 - 1, dw_[kh][0]);
    rw_dz<KC>(p, n, r + 1 - kh, x0, dw_[kh][1]);
  }
  for (int i0 = 0; i0 < RW_SEG; i0 += 4) {
    float nd[4][3][KC];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) rw_dz<KC>(p, n, r + 1 - kh, x0 + i0 + u + 1, nd[u][kh]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int k = 0; k < KC; ++k) dw_[kh][2][k] = nd[u][kh][k];
      // dx[iw] = sum_{kh,kw} dz[r + 1 - kh][iw + 1 - kw] w[kh][kw]: column iw + 1 - kw is window slot 2 - kw
      f4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int k = 0; k < KC; ++k) {
            const float dv = dw_[kh][2 - kw][k];
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = fmaf(dv, w[kh * 3 + kw][j][k], o[j]);
          }
      const int iw = x0 + i0 + u;
      if (iw < p.W) {
        float* dst = p.dx + ((long)(n * p.H + r) * p.W + iw) * p.xcs + p.xco + 4 * q;
        if (p.acc_dx) o += *reinterpret_cast<const f4*>(dst);
        *reinterpret_cast<f4*>(dst) = o;
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int k = 0; k < KC; ++k) { dw_[kh][0][k] = dw_[kh][1][k]; dw_[kh][1][k] = dw_[kh][2][k]; }
    }
  }
}

// Measured per call (scripts/head_micro.py, r04k, us): forward disp1 / disp2 / disp3 at twin batch 16 19.6 / 14.3 /
// 12.1 against 30.5 / 15.3 / 17.6 halo-tiled; filter gradient (with its reduce) 31 / 19 / 16 against 39 / 33 / 25;
// equal at batch 8.
// row-walk path: 3x3, stride 1, SAME, K <= 2, every channel a weight row (w_cin == C), C / 4 lanes per pixel a power
// of two <= 16 (C = 16 / 32 / 64), at least TDE_HEAD_TILE_MIN pixels; TDE_HEAD_RW=0 keeps the halo-tiled kernels
static const bool g_head_rw_on = !(std::getenv("TDE_HEAD_RW") && std::atol(std::getenv("TDE_HEAD_RW")) == 0);
bool head_rw(const tde_conv_desc_t* d) {
  const int cq = d->C / 4;
  return g_head_rw_on && d->stride == 1 && d->KH == 3 && d->KW == 3 && d->pad_top == 1 && d->pad_left == 1 &&
         (d->K == 1 || d->K == 2) && d->w_cin == d->C && (cq == 4 || cq == 8 || cq == 16) && d->OH == d->H &&
         d->OW == d->W && (long)d->N * d->H * d->W >= 32768;
}
long rw_threads(const tde_conv_desc_t* d) {
  return (long)d->N * d->OH * ((d->OW + RW_SEG - 1) / RW_SEG) * (d->C / 4);
}

bool head_tiled(const tde_conv_desc_t* d);

// row-walk 5x5 / 7x7 filter gradient (head_rwk_wgrad_kernel): the tiled heads' shapes with K = 2, SAME padding and
// every channel a weight row; TDE_HEAD_RWK=0 keeps head_twgrad_kernel (A/B)
static const bool g_head_rwk_on = !(std::getenv("TDE_HEAD_RWK") && std::atol(std::getenv("TDE_HEAD_RWK")) == 0);
bool head_rwk(const tde_conv_desc_t* d) {
  const int cq = d->C / 4;
  return g_head_rwk_on && head_tiled(d) && (d->KH == 5 || d->KH == 7) && d->K == 2 && d->w_cin == d->C &&
         (cq == 4 || cq == 8 || cq == 16) && d->pad_top == (d->KH - 1) / 2 && d->pad_left == (d->KW - 1) / 2;
}
int rwk_seg(const tde_conv_desc_t* d) { return 4 * d->KH; }   // Rwk<KS>::SEG
long rwk_threads(const tde_conv_desc_t* d) {
  return (long)d->N * d->OH * ((d->OW + rwk_seg(d) - 1) / rwk_seg(d)) * (d->C / 4);
}

struct WgPlan {
  int chunks, ppc, tgroups;
};

// pixels per thread lane at least: 2 (config-2 step, scripts/layer_profile.py: disp2/3/4 backward 50/42/40 ->
// 41/32/27 us against 8; disp1 unchanged) -- more blocks for the low-resolution heads
static const long g_head_ppl = tde_env_pos("TDE_HEAD_PPL", 2);
static const long g_head_blocks = tde_env_pos("TDE_HEAD_BLOCKS", 2048);

WgPlan wg_plan(const tde_conv_desc_t* d) {
  WgPlan w;
  const long M = (long)d->N * d->OH * d->OW;
  const int TT = d->K == 1 ? 9 : (d->K == 2 ? 5 : (d->K == 3 ? 3 : 2));
  w.tgroups = (d->KH * d->KW + TT - 1) / TT;
  const int P = 256 / (d->C / 4);
  // >= g_head_ppl pixels per thread lane, ~2048 blocks in total, <= WG_MAX_CHUNKS partial rows
  long chunks = (g_head_blocks + w.tgroups - 1) / w.tgroups;
  const long maxc = (M + g_head_ppl * P - 1) / (g_head_ppl * P);
  if (chunks > maxc) chunks = maxc;
  if (chunks > WG_MAX_CHUNKS) chunks = WG_MAX_CHUNKS;
  if (chunks < 1) chunks = 1;
  w.ppc = (int)((M + chunks - 1) / chunks);
  w.chunks = (int)((M + w.ppc - 1) / w.ppc);
  return w;
}

// tiled path (head_t*_kernel): stride-1 square KS in {3,5,7}, K <= 2, C = 16 * {1,2,4}, at least
// TDE_HEAD_TILE_MIN output pixels (default 32768; below it the direct kernels' parallelism wins); TDE_HEAD_TILE=0
// turns it off
static const long g_head_tile_min = tde_env_pos("TDE_HEAD_TILE_MIN", 32768);
static const bool g_head_tile_on = !(std::getenv("TDE_HEAD_TILE") && std::atol(std::getenv("TDE_HEAD_TILE")) == 0);

bool head_tiled(const tde_conv_desc_t* d) {
  return g_head_tile_on && d->stride == 1 && d->KH == d->KW && (d->KH == 3 || d->KH == 5 || d->KH == 7) &&
         (d->K == 1 || d->K == 2) && (d->C == 16 || d->C == 32 || d->C == 64) && d->OH == d->H && d->OW == d->W &&
         d->KH * d->KH * d->C * d->K <= HT_WMAX &&
         d->W >= 32 && (long)d->N * d->H * d->W >= g_head_tile_min;
}

int head_ng(const tde_conv_desc_t* d) { return d->C / 16; }

long head_tiles(const tde_conv_desc_t* d, int th) {
  return (long)d->N * ((d->OH + th - 1) / th) * ((d->OW + HT_TW - 1) / HT_TW);
}

bool head_desc_ok(const tde_conv_desc_t* d) {
  if (!d) return false;
  if (d->K < 1 || d->K > 8 || d->C % 4 || d->w_cin > d->C || d->w_cin <= 0) return false;
  if (d->C > 256) return false;   // wgrad: one channel quad per thread, >= 1 pixel lane per block
  if (d->x_coff + d->C > d->x_cstride || d->y_coff + d->K > d->y_cstride) return false;
  return d->N > 0 && d->H > 0 && d->W > 0 && d->OH > 0 && d->OW > 0;
}

HeadArgs make_head_args(const tde_conv_desc_t* d) {
  HeadArgs a{};
  a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C; a.OH = d->OH; a.OW = d->OW; a.K = d->K;
  a.KH = d->KH; a.KW = d->KW; a.S = d->stride; a.PT = d->pad_top; a.PL = d->pad_left; a.wcin = d->w_cin;
  a.xcs = d->x_cstride; a.xco = d->x_coff; a.ycs = d->y_cstride; a.yco = d->y_coff;
  return a;
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

size_t dz_bytes(const tde_conv_desc_t* d) {
  const size_t n = (size_t)d->N * d->OH * d->OW * d->K * sizeof(float);
  return (n + 255) / 256 * 256;
}

template <int KC, int KS, int QPL>
void launch_fwd_l(const HeadArgs& a, long M, int L, hipStream_t st) {
  const dim3 g((unsigned)((M * L + 255) / 256));
  switch (L) {
    case 1: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 1, QPL>), g, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 2, QPL>), g, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 4, QPL>), g, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 8, QPL>), g, dim3(256), 0, st, a); break;
    case 16: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 16, QPL>), g, dim3(256), 0, st, a); break;
    case 32: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 32, QPL>), g, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((head_fwd2_kernel<KC, KS, 64, QPL>), g, dim3(256), 0, st, a); break;
  }
}

template <int KC, int KS>
void launch_fwd_ks(const HeadArgs& a, long M, hipStream_t st) {
  // lanes per pixel: enough threads (~64K) in flight, then quads per lane (QPL) from the channel count;
  // at most 36 activation vectors in flight per lane
  const int cq = (a.wcin + 3) / 4;
  constexpr int QMAX = KS * KS >= 25 ? 1 : (KS == 3 ? 4 : 8);
  int L = 1;
  while (L < 64 && (M * L < 65536 || (cq + L - 1) / L > QMAX)) L *= 2;
  const int qpl = (cq + L - 1) / L;
  if (qpl <= 1) launch_fwd_l<KC, KS, 1>(a, M, L, st);
  else if (qpl <= 2) launch_fwd_l<KC, KS, (QMAX >= 2 ? 2 : 1)>(a, M, L, st);
  else if (qpl <= 4) launch_fwd_l<KC, KS, (QMAX >= 4 ? 4 : 1)>(a, M, L, st);
  else launch_fwd_l<KC, KS, (QMAX >= 8 ? 8 : 1)>(a, M, L, st);
}

template <int KC>
int launch_fwd(const HeadArgs& a, long M, hipStream_t st) {
  if (a.KH != a.KW || a.S != 1 || a.KH * a.KW * a.wcin * KC > HEAD_WMAX) {
    // generic fallback (unused by the reference nets): lanes split channels, weights from global
    const int cq = (a.wcin + 3) / 4;
    const int L = cq <= 4 ? 4 : (cq <= 8 ? 8 : 16);
    const long blocks = (M * L + 255) / 256;
    const dim3 g((unsigned)(blocks > 16384 ? 16384 : blocks));
    if (L == 4) hipLaunchKernelGGL((head_fwd_kernel<KC, 4>), g, dim3(256), 0, st, a);
    else if (L == 8) hipLaunchKernelGGL((head_fwd_kernel<KC, 8>), g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((head_fwd_kernel<KC, 16>), g, dim3(256), 0, st, a);
    return TDE_OK;
  }
  switch (a.KH) {
    case 1: launch_fwd_ks<KC, 1>(a, M, st); break;
    case 3: launch_fwd_ks<KC, 3>(a, M, st); break;
    case 5: launch_fwd_ks<KC, 5>(a, M, st); break;
    case 7: launch_fwd_ks<KC, 7>(a, M, st); break;
    default: return TDE_ERR_UNSUPPORTED;
  }
  return TDE_OK;
}

template <int KC, int KS>
void launch_tiled_ks(const tde_conv_desc_t* d, const HeadArgs& a, int which, float* part, hipStream_t st) {
  const int tw = (d->OW + HT_TW - 1) / HT_TW;
  if (which == 0) {
    hipLaunchKernelGGL((head_tfwd_kernel<KC, KS>), dim3(head_tiles(d, HT_TH)), dim3(256), 0, st, a, tw,
                       (d->OH + HT_TH - 1) / HT_TH);
  } else if (which == 1) {
    const int ng = head_ng(d), th = HT_TH / ng;
    const dim3 g(head_tiles(d, th));
    const int thn = (d->H + th - 1) / th;
    if (ng == 1) hipLaunchKernelGGL((head_tdgrad_kernel<KC, KS, 1>), g, dim3(256), 0, st, a, tw, thn);
    else if (ng == 2) hipLaunchKernelGGL((head_tdgrad_kernel<KC, KS, 2>), g, dim3(256), 0, st, a, tw, thn);
    else hipLaunchKernelGGL((head_tdgrad_kernel<KC, KS, 4>), g, dim3(256), 0, st, a, tw, thn);
  } else {
    hipLaunchKernelGGL((head_twgrad_kernel<KC, KS>), dim3(head_tiles(d, HT_TWG_TH)), dim3(256), 0, st, a, tw,
                       (d->OH + HT_TWG_TH - 1) / HT_TWG_TH, part);
  }
}

// which: 0 forward, 1 data gradient, 2 filter-gradient partials (one row per HT_TH x HT_TW tile)
void launch_tiled(const tde_conv_desc_t* d, const HeadArgs& a, int which, float* part, hipStream_t st) {
  const int key = d->K * 10 + d->KH;
  switch (key) {
    case 13: launch_tiled_ks<1, 3>(d, a, which, part, st); break;
    case 15: launch_tiled_ks<1, 5>(d, a, which, part, st); break;
    case 17: launch_tiled_ks<1, 7>(d, a, which, part, st); break;
    case 23: launch_tiled_ks<2, 3>(d, a, which, part, st); break;
    case 25: launch_tiled_ks<2, 5>(d, a, which, part, st); break;
    default: launch_tiled_ks<2, 7>(d, a, which, part, st); break;
  }
}

template <int KC>
int launch_dgrad(const HeadArgs& a, hipStream_t st) {
  const long n = (long)a.N * a.H * a.W * (a.C / 4);
  const dim3 g(grid_for(n));
  if (a.KH != a.KW || a.KH * a.KW * a.wcin * KC > HEAD_WMAX) {
    hipLaunchKernelGGL(head_dgrad_kernel<KC>, g, dim3(256), 0, st, a);
    return TDE_OK;
  }
  switch (a.KH) {
    case 1: hipLaunchKernelGGL((head_dgrad2_kernel<KC, 1>), g, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((head_dgrad2_kernel<KC, 3>), g, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((head_dgrad2_kernel<KC, 5>), g, dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL((head_dgrad2_kernel<KC, 7>), g, dim3(256), 0, st, a); break;
    default: return TDE_ERR_UNSUPPORTED;
  }
  return TDE_OK;
}

#define HEAD_DISPATCH(KVAL, KERNEL, GRID, ...)                                              \
  switch (KVAL) {                                                                            \
    case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(256), 0, st, __VA_ARGS__); break;       \
    case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(256), 0, st, __VA_ARGS__); break;       \
    case 3: hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(256), 0, st, __VA_ARGS__); break;       \
    case 6: hipLaunchKernelGGL(KERNEL<6>, GRID, dim3(256), 0, st, __VA_ARGS__); break;       \
    default: return TDE_ERR_UNSUPPORTED;                                                     \
  }

}  // namespace

extern "C" {

size_t tde_head_workspace_size(const tde_conv_desc_t* d) {
  if (!head_desc_ok(d)) return 0;
  const WgPlan w = wg_plan(d);
  long rows = head_tiled(d) ? head_tiles(d, HT_TWG_TH) : w.chunks;
  if (head_rw(d)) rows = (rw_threads(d) + 255) / 256;
  if (head_rwk(d)) rows = std::max(rows, (rwk_threads(d) + 255) / 256);
  const size_t part = (size_t)rows * (d->KH * d->KW * d->w_cin * d->K + d->K) * sizeof(float);
  return dz_bytes(d) + part;
}

int tde_head_fwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias, float* y,
                 int act, float scale, float offset, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(head_desc_ok(d) && x && w && bias && y && tde_aligned16(x) && d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  HeadArgs a = make_head_args(d);
  a.x = x; a.w = w; a.b = bias; a.y = y; a.act = act; a.scale = scale; a.offset = offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const long M = (long)d->N * d->OH * d->OW;
  if (head_rw(d)) {
    const long th = rw_threads(d);
    const int segs = (d->OW + RW_SEG - 1) / RW_SEG;
    if (d->K == 1)
      hipLaunchKernelGGL(head_rw_fwd_kernel<1>, dim3((th + 255) / 256), dim3(256), 0, st, a, d->C / 4, segs, th);
    else
      hipLaunchKernelGGL(head_rw_fwd_kernel<2>, dim3((th + 255) / 256), dim3(256), 0, st, a, d->C / 4, segs, th);
    return tde_launch_status();
  }
  if (head_tiled(d)) {
    launch_tiled(d, a, 0, nullptr, st);
    return tde_launch_status();
  }
  switch (d->K) {
    case 1: launch_fwd<1>(a, M, st); break;
    case 2: launch_fwd<2>(a, M, st); break;
    case 3: launch_fwd<3>(a, M, st); break;
    case 6: launch_fwd<6>(a, M, st); break;
    default: return TDE_ERR_UNSUPPORTED;
  }
  return tde_launch_status();
}

int tde_head_bwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* y, const float* dy,
                 float* dx, int accumulate_dx, float* dw, float* dbias, int accumulate_dw, int act, float scale,
                 float offset, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(head_desc_ok(d) && d->stride == 1 && x && w && y && dy && tde_aligned16(x));
  TDE_CHECK_ARG(d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  TDE_CHECK_ARG(d->K == 1 || d->K == 2 || d->K == 3 || d->K == 6);
  if (ws_bytes < tde_head_workspace_size(d) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  ws = tde_ws_body(ws);
  HeadArgs a = make_head_args(d);
  a.x = x; a.w = w; a.yin = y; a.dy = dy; a.dx = dx; a.acc_dx = accumulate_dx;
  a.act = act; a.scale = scale; a.offset = offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const long M = (long)d->N * d->OH * d->OW;
  float* dz = static_cast<float*>(ws);
  a.dz = dz;
  a.dzw = dz;
  TDE_CHECK_ARG(!dx || tde_aligned16(dx));
  TDE_CHECK_ARG(!dw || dbias != nullptr);
  if (head_rw(d)) {
    // dz recomputed from (y, dy) where each kernel needs it: no dz pass
    const long th = rw_threads(d);
    const int segs = (d->OW + RW_SEG - 1) / RW_SEG, CQ = d->C / 4;
    const int rows = (int)((th + 255) / 256);
    const int total = 9 * d->w_cin * d->K + d->K;
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + dz_bytes(d));
    if (dw) {
      if (d->K == 1) hipLaunchKernelGGL(head_rw_wgrad_kernel<1>, dim3(rows), dim3(256), 0, st, a, CQ, segs, th, part);
      else hipLaunchKernelGGL(head_rw_wgrad_kernel<2>, dim3(rows), dim3(256), 0, st, a, CQ, segs, th, part);
    }
    if (dx) {
      // the data gradient stays on the halo-tiled kernel where it applies: its dz halo is computed once per tile, while
      // every quad lane of the row walk recomputes its dz window (measured, scripts/head_micro.py r04k: disp2 / disp3
      // dgrad 15.2 / 9.8 us tiled vs 17.8 / 14.5 us row-walk at batch 16; flow1 47.8 vs 78.5 us)
      if (head_tiled(d)) launch_tiled(d, a, 1, nullptr, st);
      else if (d->K == 1) hipLaunchKernelGGL(head_rw_dgrad_kernel<1>, dim3(rows), dim3(256), 0, st, a, CQ, segs, th);
      else hipLaunchKernelGGL(head_rw_dgrad_kernel<2>, dim3(rows), dim3(256), 0, st, a, CQ, segs, th);
    }
    if (dw)
      hipLaunchKernelGGL(head_wgrad_reduce_t_kernel, dim3(total), dim3(64), 0, st, part, rows, 9 * d->w_cin * d->K, dw,
                         dbias, accumulate_dw);
    return tde_launch_status();
  }
  if (head_tiled(d)) {
    // dz recomputed from (y, dy) at each kernel's staging: no dz pass
    const int E = d->KH * d->KW * d->w_cin;
    const int total = E * d->K + d->K;
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + dz_bytes(d));
    long prow = head_tiles(d, HT_TWG_TH);
    if (dw && head_rwk(d)) {
      // the dense dz pass (K = 2 floats per pixel), then the row walk reads one float2 per pixel
      hipLaunchKernelGGL(head_dz_kernel, dim3(grid_for(M * d->K)), dim3(256), 0, st, M, d->K, y, dy, d->y_cstride,
                         d->y_coff, act, scale, offset, dz);
      const long th = rwk_threads(d);
      const int segs = (d->OW + rwk_seg(d) - 1) / rwk_seg(d);
      prow = (th + 255) / 256;
      const dim3 g((unsigned)prow, (unsigned)d->KH);
      if (d->KH == 5) hipLaunchKernelGGL(head_rwk_wgrad_kernel<5>, g, dim3(256), 0, st, a, d->C / 4, segs, th, part);
      else hipLaunchKernelGGL(head_rwk_wgrad_kernel<7>, g, dim3(256), 0, st, a, d->C / 4, segs, th, part);
    } else if (dw) {
      launch_tiled(d, a, 2, part, st);
    }
    if (dx) launch_tiled(d, a, 1, nullptr, st);
    if (dw)
      hipLaunchKernelGGL(head_wgrad_reduce_t_kernel, dim3(total), dim3(64), 0, st, part, (int)prow, E * d->K, dw,
                         dbias, accumulate_dw);
    return tde_launch_status();
  }
  // the wgrad pass computes dz on the fly and stores it; without a weight gradient a dz pass does that
  if (dw) {
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + dz_bytes(d));
    const WgPlan wp = wg_plan(d);
    HEAD_DISPATCH(d->K, head_wgrad_partial_kernel, dim3(wp.chunks, wp.tgroups), a, part, wp.ppc);
    if (dx) {
      int rc = TDE_OK;
      switch (d->K) {
        case 1: rc = launch_dgrad<1>(a, st); break;
        case 2: rc = launch_dgrad<2>(a, st); break;
        case 3: rc = launch_dgrad<3>(a, st); break;
        default: rc = launch_dgrad<6>(a, st); break;
      }
      if (rc != TDE_OK) return rc;
    }
    const int E = d->KH * d->KW * d->w_cin;
    const int total = E * d->K + d->K;
    hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(1024), 0, st, part, wp.chunks, total,
                       E * d->K, dw, dbias, accumulate_dw);
  } else if (dx) {
    hipLaunchKernelGGL(head_dz_kernel, dim3(grid_for(M * d->K)), dim3(256), 0, st, M, d->K, y, dy, d->y_cstride,
                       d->y_coff, act, scale, offset, dz);
    int rc = TDE_OK;
    switch (d->K) {
      case 1: rc = launch_dgrad<1>(a, st); break;
      case 2: rc = launch_dgrad<2>(a, st); break;
      case 3: rc = launch_dgrad<3>(a, st); break;
      default: rc = launch_dgrad<6>(a, st); break;
    }
    if (rc != TDE_OK) return rc;
  }
  return tde_launch_status();
}

}  // extern "C"
