// Few-output-channel conv heads (K <= 8): disparity heads (nets_optflow_depth.py:122-144,
// DISP_SCALING*sigmoid(conv+b) [+MIN_DISP]), flow heads (nets_depth.py:169-191, 2-ch linear), exp-mask
// logits (nets_optflow_depth.py:193-198) and pose/pred 1x1 (:181).  These GEMMs have N = 1..6 and are
// HBM/L2-bound (arithmetic intensity ~K flop/B), so they are direct convolutions on the vector ALU
// with the activation and its derivative fused, not MFMA tiles padded to 16 columns.
#include "tde_common.h"

namespace {

struct HeadArgs {
  int N, H, W, C, OH, OW, K, KH, KW, S, PT, PL, wcin;
  const float* x; int xcs, xco;
  const float* w; const float* b;
  float* y; const float* yin; const float* dy; int ycs, yco;
  float* dx; int acc_dx;
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

template <int KC>
__global__ void __launch_bounds__(256) head_fwd_kernel(const HeadArgs p) {
  const long M = (long)p.N * p.OH * p.OW;
  for (long m = blockIdx.x * (long)blockDim.x + threadIdx.x; m < M; m += (long)gridDim.x * blockDim.x) {
    const int ohw = p.OH * p.OW;
    const int n = (int)(m / ohw), r = (int)(m - (long)n * ohw), oh = r / p.OW, ow = r - oh * p.OW;
    float acc[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[k] = 0.f;
    for (int kh = 0; kh < p.KH; ++kh) {
      const int ih = oh * p.S - p.PT + kh;
      if ((unsigned)ih >= (unsigned)p.H) continue;
      for (int kw = 0; kw < p.KW; ++kw) {
        const int iw = ow * p.S - p.PL + kw;
        if ((unsigned)iw >= (unsigned)p.W) continue;
        const float* xp = p.x + ((long)(n * p.H + ih) * p.W + iw) * p.xcs + p.xco;
        const float* wp = p.w + (long)(kh * p.KW + kw) * p.wcin * KC;
        for (int c = 0; c < p.wcin; c += 4) {
          const f4 xv = *reinterpret_cast<const f4*>(xp + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (c + j < p.wcin) {
#pragma unroll
              for (int k = 0; k < KC; ++k) acc[k] = fmaf(xv[j], wp[(c + j) * KC + k], acc[k]);
            }
          }
        }
      }
    }
    float* yp = p.y + m * p.ycs + p.yco;
#pragma unroll
    for (int k = 0; k < KC; ++k) yp[k] = head_act(acc[k] + p.b[k], p.act, p.scale, p.offset);
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
    for (int kh = 0; kh < p.KH; ++kh) {
      const int oh = ih + p.PT - kh;
      if ((unsigned)oh >= (unsigned)p.OH) continue;
      for (int kw = 0; kw < p.KW; ++kw) {
        const int ow = iw + p.PL - kw;
        if ((unsigned)ow >= (unsigned)p.OW) continue;
        const long o = ((long)(n * p.OH + oh) * p.OW + ow) * p.ycs + p.yco;
        const float* wp = p.w + (long)(kh * p.KW + kw) * p.wcin * KC;
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const float dz = head_dz(p.yin[o + k], p.dy[o + k], p.act, p.scale, p.offset);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < p.wcin) acc[j] = fmaf(dz, wp[(c + j) * KC + k], acc[j]);
        }
      }
    }
    float* dst = p.dx + pix * p.xcs + p.xco + c;
    f4 out = acc;
    if (p.acc_dx) out += *reinterpret_cast<const f4*>(dst);
    *reinterpret_cast<f4*>(dst) = out;
  }
}

// Per-chunk partial dW / db: part[chunk][e*KC + k] for e = (tap, c) in [0, KH*KW*wcin), then KC bias sums.
constexpr int HW_PIX = 128;  // pixels per chunk (staged dz in LDS)

// One block per pixel chunk (<= HW_CHUNKS chunks).  Threads = (entry e, pixel lane g): when the weight
// has E < 256 entries, 256/E lanes split each staged sub-chunk's pixels and are combined through LDS.
constexpr int HW_CHUNKS = 1024;

template <int KC>
__global__ void __launch_bounds__(256) head_wgrad_partial_kernel(const HeadArgs p, float* part, int pix_per_chunk) {
  __shared__ float sdz[HW_PIX * KC];
  __shared__ float sred[256 * KC];
  __shared__ int3 spix[HW_PIX];
  const long M = (long)p.N * p.OH * p.OW;
  const long cbeg = (long)blockIdx.x * pix_per_chunk;
  const long cend = min(M, cbeg + pix_per_chunk);
  const int E = p.KH * p.KW * p.wcin;
  const int G = E >= 256 ? 1 : 256 / E;          // pixel lanes
  const int lane = (int)threadIdx.x / (E >= 256 ? 256 : E);
  const bool active = lane < G;
  const int ohw = p.OH * p.OW;
  // each thread owns entries e = e0, e0 + 256, ... (G == 1) or exactly one entry (G > 1)
  const int e0 = E >= 256 ? (int)threadIdx.x : (int)threadIdx.x % E;
  const int ne = E >= 256 ? (E - e0 + 255) / 256 : 1;
  constexpr int MAXE = 8;                        // E <= 2048 entries
  float acc[MAXE][KC];
#pragma unroll
  for (int j = 0; j < MAXE; ++j)
#pragma unroll
    for (int k = 0; k < KC; ++k) acc[j][k] = 0.f;
  float bacc[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) bacc[k] = 0.f;
  for (long p0 = cbeg; p0 < cend; p0 += HW_PIX) {
    const int np = (int)min((long)HW_PIX, cend - p0);
    __syncthreads();
    for (int t = threadIdx.x; t < HW_PIX * KC; t += blockDim.x) {
      const int pi = t / KC, k = t - pi * KC;
      float v = 0.f;
      if (pi < np) {
        const long o = (p0 + pi) * p.ycs + p.yco + k;
        v = head_dz(p.yin[o], p.dy[o], p.act, p.scale, p.offset);
      }
      sdz[t] = v;
    }
    for (int pi = threadIdx.x; pi < np; pi += blockDim.x) {   // pixel decode once per sub-chunk
      const long pix = p0 + pi;
      const int n = (int)(pix / ohw), r = (int)(pix - (long)n * ohw), oh = r / p.OW, ow = r - oh * p.OW;
      spix[pi] = make_int3(n * p.H, oh * p.S - p.PT, ow * p.S - p.PL);
    }
    __syncthreads();
    if (threadIdx.x < KC)
      for (int pi = 0; pi < np; ++pi) bacc[threadIdx.x] += sdz[pi * KC + threadIdx.x];
    if (!active) continue;
#pragma unroll
    for (int j = 0; j < MAXE; ++j) {
      if (j >= ne) break;
      const int e = e0 + j * 256;
      const int tap = e / p.wcin, c = e - tap * p.wcin, kh = tap / p.KW, kw = tap - kh * p.KW;
      for (int pi = lane; pi < np; pi += G) {
        const int3 q = spix[pi];
        const int ih = q.y + kh, iw = q.z + kw;
        if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) {
          const float xv = p.x[((long)(q.x + ih) * p.W + iw) * p.xcs + p.xco + c];
#pragma unroll
          for (int k = 0; k < KC; ++k) acc[j][k] = fmaf(xv, sdz[pi * KC + k], acc[j][k]);
        }
      }
    }
  }
  const int stride_out = E * KC + KC;
  float* out = part + (long)blockIdx.x * stride_out;
  if (G == 1) {
    if (active)
      for (int j = 0; j < ne; ++j)
#pragma unroll
        for (int k = 0; k < KC; ++k) out[(e0 + j * 256) * KC + k] = acc[j][k];
  } else {
    __syncthreads();
    if (active)
#pragma unroll
      for (int k = 0; k < KC; ++k) sred[threadIdx.x * KC + k] = acc[0][k];
    __syncthreads();
    if ((int)threadIdx.x < E) {
      for (int k = 0; k < KC; ++k) {
        float s = 0.f;
        for (int g = 0; g < G; ++g) s += sred[(g * E + threadIdx.x) * KC + k];
        out[threadIdx.x * KC + k] = s;
      }
    }
  }
  if (threadIdx.x < KC) out[E * KC + threadIdx.x] = bacc[threadIdx.x];
}

// 64 outputs per block, 4 waves split the chunk range, fp64 combine through LDS.
__global__ void __launch_bounds__(256) head_wgrad_reduce_kernel(const float* part, int chunks, int E, int KC,
                                                                 float* dw, float* db, int accumulate) {
  __shared__ double sh[256];
  const int total = E * KC + KC;
  const int il = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + il;
  double s = 0.0;
  if (i < total)
    for (int ch = w; ch < chunks; ch += 4) s += part[(long)ch * total + i];
  sh[threadIdx.x] = s;
  __syncthreads();
  if (w != 0 || i >= total) return;
  s = sh[il] + sh[il + 64] + sh[il + 128] + sh[il + 192];
  float* dst = (i < E * KC) ? dw + i : db + (i - E * KC);
  *dst = accumulate ? *dst + (float)s : (float)s;
}

int head_chunks(long M) {
  const long c = (M + HW_PIX - 1) / HW_PIX;
  return (int)(c < HW_CHUNKS ? c : HW_CHUNKS);
}

bool head_desc_ok(const tde_conv_desc_t* d) {
  if (!d) return false;
  if (d->K < 1 || d->K > 8 || d->C % 4 || d->w_cin > d->C || d->w_cin <= 0) return false;
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
  const long M = (long)d->N * d->OH * d->OW;
  const long chunks = head_chunks(M);
  return (size_t)chunks * (d->KH * d->KW * d->w_cin * d->K + d->K) * sizeof(float);
}

int tde_head_fwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias, float* y,
                 int act, float scale, float offset, void* stream) {
  TDE_CHECK_ARG(head_desc_ok(d) && x && w && bias && y && tde_aligned16(x) && d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  HeadArgs a = make_head_args(d);
  a.x = x; a.w = w; a.b = bias; a.y = y; a.act = act; a.scale = scale; a.offset = offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const long M = (long)d->N * d->OH * d->OW;
  HEAD_DISPATCH(d->K, head_fwd_kernel, dim3(grid_for(M)), a);
  return tde_launch_status();
}

int tde_head_bwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* y, const float* dy,
                 float* dx, int accumulate_dx, float* dw, float* dbias, int accumulate_dw, int act, float scale,
                 float offset, void* ws, size_t ws_bytes, void* stream) {
  TDE_CHECK_ARG(head_desc_ok(d) && d->stride == 1 && x && w && y && dy && tde_aligned16(x));
  TDE_CHECK_ARG(d->x_cstride % 4 == 0 && d->x_coff % 4 == 0);
  HeadArgs a = make_head_args(d);
  a.x = x; a.w = w; a.yin = y; a.dy = dy; a.dx = dx; a.acc_dx = accumulate_dx;
  a.act = act; a.scale = scale; a.offset = offset;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dx) {
    TDE_CHECK_ARG(tde_aligned16(dx));
    const long n = (long)d->N * d->H * d->W * (d->C / 4);
    HEAD_DISPATCH(d->K, head_dgrad_kernel, dim3(grid_for(n)), a);
  }
  if (dw) {
    TDE_CHECK_ARG(dbias != nullptr);
    if (ws_bytes < tde_head_workspace_size(d)) return TDE_ERR_WORKSPACE;
    float* part = static_cast<float*>(ws);
    const long M = (long)d->N * d->OH * d->OW;
    const int chunks = head_chunks(M);
    const int ppc = (int)((M + chunks - 1) / chunks);
    TDE_CHECK_ARG(d->KH * d->KW * d->w_cin <= 2048);
    HEAD_DISPATCH(d->K, head_wgrad_partial_kernel, dim3(chunks), a, part, ppc);
    const int E = d->KH * d->KW * d->w_cin;
    const int total = E * d->K + d->K;
    hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3((total + 63) / 64), dim3(256), 0, st, part, chunks, E,
                       d->K, dw, dbias, accumulate_dw);
  }
  return tde_launch_status();
}

}  // extern "C"
