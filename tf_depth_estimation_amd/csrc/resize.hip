// TF-1 legacy resize ops on channel views (align_corners=False, no half-pixel centres):
//   resize_nearest_neighbor  -> resize_like (nets_optflow_depth.py:11-16)
//   resize_bilinear          -> disp*_up (nets_optflow_depth.py:124,131,138)
//   resize_area (int factor) -> loss pyramids (train_depth_then_cam_lr.py:227-232)
// Scales are computed in fp32 exactly as TF does (scale = (float)in / out).  Backward passes are
// written as gathers over the (few) outputs that touch each input, so they need no atomics and
// are deterministic.
#include "tde_common.h"

namespace {

__device__ __forceinline__ int nn_src(int o, float s, int n_in) {
  const int i = (int)floorf((float)o * s);
  return i < n_in - 1 ? i : n_in - 1;
}

__global__ void __launch_bounds__(256) nearest_fwd_kernel(int N, int H, int W, int C, const float* x, int xcs, int xco,
                                                          int OH, int OW, float* y, int ycs, int yco) {
  const float sy = (float)H / (float)OH, sx = (float)W / (float)OW;
  const long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int ow = (int)(pix % OW);
    const long t = pix / OW;
    const int oh = (int)(t % OH), n = (int)(t / OH);
    const int ih = nn_src(oh, sy, H), iw = nn_src(ow, sx, W);
    y[pix * ycs + yco + c] = x[((long)(n * H + ih) * W + iw) * xcs + xco + c];
  }
}

__global__ void __launch_bounds__(256) nearest_bwd_kernel(int N, int H, int W, int C, float* dx, int dxcs, int dxco,
                                                          int acc, int OH, int OW, const float* dy, int dycs,
                                                          int dyco) {
  const float sy = (float)H / (float)OH, sx = (float)W / (float)OW;
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int iw = (int)(pix % W);
    const long t = pix / W;
    const int ih = (int)(t % H), n = (int)(t / H);
    // outputs o with nn_src(o) == i lie in [floor(i/s)-1, ceil((i+1)/s)+1]
    const int oh0 = max(0, (int)floorf(ih / sy) - 1), oh1 = min(OH - 1, (int)ceilf((ih + 1) / sy) + 1);
    const int ow0 = max(0, (int)floorf(iw / sx) - 1), ow1 = min(OW - 1, (int)ceilf((iw + 1) / sx) + 1);
    float s = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      if (nn_src(oh, sy, H) != ih) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        if (nn_src(ow, sx, W) != iw) continue;
        s += dy[((long)(n * OH + oh) * OW + ow) * dycs + dyco + c];
      }
    }
    float* d = dx + pix * dxcs + dxco + c;
    *d = acc ? *d + s : s;
  }
}

struct Lerp {
  int i0, i1;
  float l;
};

__device__ __forceinline__ Lerp lerp_src(int o, float s, int n_in) {
  Lerp r;
  const float in = (float)o * s;
  r.i0 = (int)floorf(in);
  r.i1 = r.i0 + 1 < n_in - 1 ? r.i0 + 1 : n_in - 1;
  r.l = in - (float)r.i0;
  return r;
}

__global__ void __launch_bounds__(256) bilinear_fwd_kernel(int N, int H, int W, int C, const float* x, int xcs,
                                                           int xco, int OH, int OW, float* y, int ycs, int yco) {
  const float sy = (float)H / (float)OH, sx = (float)W / (float)OW;
  const long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int ow = (int)(pix % OW);
    const long t = pix / OW;
    const int oh = (int)(t % OH), n = (int)(t / OH);
    const Lerp ly = lerp_src(oh, sy, H), lx = lerp_src(ow, sx, W);
    const float* b = x + (long)n * H * W * xcs + xco + c;
    const float tl = b[((long)ly.i0 * W + lx.i0) * xcs], tr = b[((long)ly.i0 * W + lx.i1) * xcs];
    const float bl = b[((long)ly.i1 * W + lx.i0) * xcs], br = b[((long)ly.i1 * W + lx.i1) * xcs];
    const float top = tl + (tr - tl) * lx.l;
    const float bot = bl + (br - bl) * lx.l;
    y[pix * ycs + yco + c] = top + (bot - top) * ly.l;
  }
}

// Exact x2 upsample (the disparity heads, nets_optflow_depth.py:124,131,138) with 32-bit indices: one thread
// per output pixel, the source offsets from shifts (in = o * 0.5: lower = o >> 1, lerp 0 or 0.5) -- the same
// float expressions as bilinear_fwd_kernel, so the same values.
__global__ void __launch_bounds__(256) bilinear_up2_fwd_kernel(int N, int H, int W, int C, const float* x, int xcs,
                                                               int xco, float* y, int ycs, int yco) {
  const int OH = 2 * H, OW = 2 * W;
  const int total = N * OH * OW;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < total; p += gridDim.x * 256) {
    const int ow = p % OW, t = p / OW;
    const int oh = t % OH, n = t / OH;
    const int y0 = oh >> 1, x0 = ow >> 1;
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = (oh & 1) ? 0.5f : 0.f, lx = (ow & 1) ? 0.5f : 0.f;
    const float* b = x + n * H * W * xcs + xco;
    for (int c = 0; c < C; ++c) {
      const float tl = b[(y0 * W + x0) * xcs + c], tr = b[(y0 * W + x1) * xcs + c];
      const float bl = b[(y1 * W + x0) * xcs + c], br = b[(y1 * W + x1) * xcs + c];
      const float top = tl + (tr - tl) * lx;
      const float bot = bl + (br - bl) * lx;
      y[p * ycs + yco + c] = top + (bot - top) * ly;
    }
  }
}

// Its gradient: an input row i receives from output rows 2i-1 (weight 0.5), 2i (1) and 2i+1 (0.5, plus the
// clamped upper tap 0.5 on the last row); columns alike.  Summed in the generic kernel's order (ascending
// output row, then column, zero weights skipped) with the same weight products: the same values.
__global__ void __launch_bounds__(256) bilinear_up2_bwd_kernel(int N, int H, int W, int C, float* dx, int dxcs,
                                                               int dxco, int acc, const float* dy, int dycs,
                                                               int dyco) {
  const int OH = 2 * H, OW = 2 * W;
  const int total = N * H * W;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < total; p += gridDim.x * 256) {
    const int iw = p % W, t = p / W;
    const int ih = t % H, n = t / H;
    float wys[3], wxs[3];
    wys[0] = ih > 0 ? 0.5f : 0.f;
    wys[1] = 1.f;
    wys[2] = ih == H - 1 ? 1.f : 0.5f;     // row 2i+1: lower tap 0.5, and on the last row its clamped upper too
    wxs[0] = iw > 0 ? 0.5f : 0.f;
    wxs[1] = 1.f;
    wxs[2] = iw == W - 1 ? 1.f : 0.5f;
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        if (wys[a] == 0.f) continue;
        const int oh = 2 * ih - 1 + a;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          if (wxs[b] == 0.f) continue;
          const int ow = 2 * iw - 1 + b;
          s += dy[((n * OH + oh) * OW + ow) * dycs + dyco + c] * (wys[a] * wxs[b]);
        }
      }
      float* d = dx + p * dxcs + dxco + c;
      *d = acc ? *d + s : s;
    }
  }
}

// ResizeBilinearGrad as a gather: dx[i] = sum over outputs o of dy[o] * weight(o -> i).
__global__ void __launch_bounds__(256) bilinear_bwd_kernel(int N, int H, int W, int C, float* dx, int dxcs,
                                                           int dxco, int acc, int OH, int OW, const float* dy,
                                                           int dycs, int dyco) {
  const float sy = (float)H / (float)OH, sx = (float)W / (float)OW;
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int iw = (int)(pix % W);
    const long t = pix / W;
    const int ih = (int)(t % H), n = (int)(t / H);
    // contributors have floor(o * s) in {i - 1, i} (or the clamped last row): o in [(i - 1) / s, (i + 1) / s];
    // the exact tap tests below decide, the window only has to contain them (25 candidates at x2, not 49)
    const int oh0 = max(0, (int)floorf((ih - 1) / sy)), oh1 = min(OH - 1, (int)ceilf((ih + 1) / sy));
    const int ow0 = max(0, (int)floorf((iw - 1) / sx)), ow1 = min(OW - 1, (int)ceilf((iw + 1) / sx));
    float s = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const Lerp ly = lerp_src(oh, sy, H);
      float wy = 0.f;
      if (ly.i0 == ih) wy += 1.f - ly.l;
      if (ly.i1 == ih) wy += ly.l;
      if (wy == 0.f) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const Lerp lx = lerp_src(ow, sx, W);
        float wx = 0.f;
        if (lx.i0 == iw) wx += 1.f - lx.l;
        if (lx.i1 == iw) wx += lx.l;
        if (wx == 0.f) continue;
        s += dy[((long)(n * OH + oh) * OW + ow) * dycs + dyco + c] * (wy * wx);
      }
    }
    float* d = dx + pix * dxcs + dxco + c;
    *d = acc ? *d + s : s;
  }
}

__global__ void __launch_bounds__(256) area_fwd_kernel(int N, int H, int W, int C, const float* x, int OH, int OW,
                                                       float* y) {
  const int fy = H / OH, fx = W / OW;
  const float inv = 1.f / (float)(fy * fx);
  const long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int ow = (int)(pix % OW);
    const long t = pix / OW;
    const int oh = (int)(t % OH), n = (int)(t / OH);
    float s = 0.f;
    for (int a = 0; a < fy; ++a)
      for (int b = 0; b < fx; ++b) s += x[((long)(n * H + oh * fy + a) * W + ow * fx + b) * C + c];
    y[i] = s * inv;
  }
}

int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

int tde_resize_nearest_fwd(int N, int H, int W, int C, const float* x, int x_cstride, int x_coff, int OH, int OW,
                           float* y, int y_cstride, int y_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && x && y);
  hipLaunchKernelGGL(nearest_fwd_kernel, dim3(ew_grid((long)N * OH * OW * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, H, W, C, x, x_cstride, x_coff, OH, OW, y, y_cstride, y_coff);
  return tde_launch_status();
}

int tde_resize_nearest_bwd(int N, int H, int W, int C, float* dx, int dx_cstride, int dx_coff, int accumulate, int OH,
                           int OW, const float* dy, int dy_cstride, int dy_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && dx && dy);
  hipLaunchKernelGGL(nearest_bwd_kernel, dim3(ew_grid((long)N * H * W * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, H, W, C, dx, dx_cstride, dx_coff, accumulate, OH, OW, dy,
                     dy_cstride, dy_coff);
  return tde_launch_status();
}

int tde_resize_bilinear_fwd(int N, int H, int W, int C, const float* x, int x_cstride, int x_coff, int OH, int OW,
                            float* y, int y_cstride, int y_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && x && y);
  if (OH == 2 * H && OW == 2 * W && (long)N * OH * OW * (y_cstride > x_cstride ? y_cstride : x_cstride) < (1L << 31)) {
    hipLaunchKernelGGL(bilinear_up2_fwd_kernel, dim3(ew_grid((long)N * OH * OW)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, H, W, C, x, x_cstride, x_coff, y, y_cstride, y_coff);
    return tde_launch_status();
  }
  hipLaunchKernelGGL(bilinear_fwd_kernel, dim3(ew_grid((long)N * OH * OW * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, H, W, C, x, x_cstride, x_coff, OH, OW, y, y_cstride, y_coff);
  return tde_launch_status();
}

int tde_resize_bilinear_bwd(int N, int H, int W, int C, float* dx, int dx_cstride, int dx_coff, int accumulate, int OH,
                            int OW, const float* dy, int dy_cstride, int dy_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && dx && dy);
  if (OH == 2 * H && OW == 2 * W && (long)N * OH * OW * (dy_cstride > dx_cstride ? dy_cstride : dx_cstride) < (1L << 31)) {
    hipLaunchKernelGGL(bilinear_up2_bwd_kernel, dim3(ew_grid((long)N * H * W)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, H, W, C, dx, dx_cstride, dx_coff, accumulate, dy,
                       dy_cstride, dy_coff);
    return tde_launch_status();
  }
  hipLaunchKernelGGL(bilinear_bwd_kernel, dim3(ew_grid((long)N * H * W * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, H, W, C, dx, dx_cstride, dx_coff, accumulate, OH, OW, dy,
                     dy_cstride, dy_coff);
  return tde_launch_status();
}

int tde_resize_area_fwd(int N, int H, int W, int C, const float* x, int OH, int OW, float* y, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0 && x && y);
  TDE_CHECK_ARG(H % OH == 0 && W % OW == 0);
  hipLaunchKernelGGL(area_fwd_kernel, dim3(ew_grid((long)N * OH * OW * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, H, W, C, x, OH, OW, y);
  return tde_launch_status();
}

}  // extern "C"
