// Few-output-channel conv heads (K <= 8): disparity heads (nets_optflow_depth.py:122-144,
// DISP_SCALING*sigmoid(conv+b) [+MIN_DISP]), flow heads (nets_depth.py:169-191, 2-ch linear), exp-mask
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

// taps per wgrad block: TT * 4 * KC accumulators per thread
template <int KC>
struct WgTaps { static constexpr int TT = KC == 1 ? 9 : (KC == 2 ? 5 : 2); };

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
  const int TT = d->K == 1 ? 9 : (d->K == 2 ? 5 : 2);
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
    case 6: hipLaunchKernelGGL(KERNEL<6>, GRID, dim3(256), 0, st, __VA_ARGS__); break;       \
    default: return TDE_ERR_UNSUPPORTED;                                                     \
  }

}  // namespace

extern "C" {

size_t tde_head_workspace_size(const tde_conv_desc_t* d) {
  if (!head_desc_ok(d)) return 0;
  const WgPlan w = wg_plan(d);
  const size_t part = (size_t)w.chunks * (d->KH * d->KW * d->w_cin * d->K + d->K) * sizeof(float);
  return dz_bytes(d) + part;
}

int tde_head_fwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias, float* y,
                 int act, float scale, float offset, void* stream) {
  TDE_CHECK_ARG(head_desc_ok(d) && x && w && bias && y && tde_aligned16(x) && d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  HeadArgs a = make_head_args(d);
  a.x = x; a.w = w; a.b = bias; a.y = y; a.act = act; a.scale = scale; a.offset = offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const long M = (long)d->N * d->OH * d->OW;
  switch (d->K) {
    case 1: launch_fwd<1>(a, M, st); break;
    case 2: launch_fwd<2>(a, M, st); break;
    case 6: launch_fwd<6>(a, M, st); break;
    default: return TDE_ERR_UNSUPPORTED;
  }
  return tde_launch_status();
}

int tde_head_bwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* y, const float* dy,
                 float* dx, int accumulate_dx, float* dw, float* dbias, int accumulate_dw, int act, float scale,
                 float offset, void* ws, size_t ws_bytes, void* stream) {
  TDE_CHECK_ARG(head_desc_ok(d) && d->stride == 1 && x && w && y && dy && tde_aligned16(x));
  TDE_CHECK_ARG(d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  TDE_CHECK_ARG(d->K == 1 || d->K == 2 || d->K == 6);
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
      default: rc = launch_dgrad<6>(a, st); break;
    }
    if (rc != TDE_OK) return rc;
  }
  return tde_launch_status();
}

}  // extern "C"
