// Inference pre/post-processing of the reference's prediction scripts, on the GPU:
//   batch_prediction.py:62  I = cv2.resize(I, (224, 224), interpolation=cv2.INTER_AREA)          uint8 RGB
//   batch_prediction.py:72  z = cv2.resize(pred[0][0,:,:,0], (image_width, image_height), INTER_CUBIC)  float
//   batch_prediction.py:73  z = cv2.bilateralFilter(z, 9, 75, 75)                                  float
// OpenCV is not vendored in the reference (a pip dependency, unpinned) and cv2 is not importable here, so each
// kernel restates the published algorithm of OpenCV 4.x's scalar reference code (imgproc resize.cpp
// resizeArea_ / resizeAreaFast_ / resizeGeneric_ + computeResizeAreaTab + interpolateCubic, bilateral_filter
// 32f) -- parity against cv2 itself is unpinned.  Where OpenCV's x86 SIMD paths round differently from its scalar
// code (the 8-bit 2x2 area average and the 8-bit linear vertical pass), the scalar code is what is restated.
// oracle/cv_ops.py is the NumPy restatement the tests compare with.
//
// All three are HBM/L2-bound stencils over small images (a 224x224 input, a 240x720 output map): one thread per
// output pixel, taps gathered through L1/L2, FMA contraction off so the float arithmetic is OpenCV's operation
// for operation (mult, then add).
#include <cfloat>
#include <cmath>

#include "tde_common.h"

namespace {

// ---------------------------------------------------------------- INTER_AREA (uint8)
// computeResizeAreaTab (resize.cpp): the source cells of destination index d along one axis, with their weights.
struct AreaSpan {
  int s0;         // first source index
  int n;          // number of taps (<= 2 + ceil(scale))
  float a_first;  // weight of s0 (partial cell, or the full weight)
  float a_mid;    // weight of the whole cells
  float a_last;   // weight of the last (partial) cell
  bool has_first_partial, has_last_partial;
  int mid0, mid1; // whole cells [mid0, mid1)
};

__device__ __forceinline__ AreaSpan area_span(int d, int ssize, double scale) {
  AreaSpan t;
  const double fs1 = d * scale;
  const double fs2 = fs1 + scale;
  const double cell = fmin(scale, (double)ssize - fs1);
  int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  t.has_first_partial = s1 - fs1 > 1e-3;
  t.a_first = (float)((s1 - fs1) / cell);
  t.mid0 = s1;
  t.mid1 = s2;
  t.a_mid = (float)(1.0 / cell);
  t.has_last_partial = fs2 - s2 > 1e-3;
  t.a_last = (float)(fmin(fmin(fs2 - s2, 1.0), cell) / cell);
  t.s0 = t.has_first_partial ? s1 - 1 : s1;
  t.n = (t.has_first_partial ? 1 : 0) + (s2 - s1) + (t.has_last_partial ? 1 : 0);
  return t;
}

// k-th tap of a span: source index and weight, in computeResizeAreaTab's order
__device__ __forceinline__ void area_tap(const AreaSpan& t, int k, int& s, float& a) {
  if (t.has_first_partial) {
    if (k == 0) { s = t.mid0 - 1; a = t.a_first; return; }
    --k;
  }
  if (k < t.mid1 - t.mid0) { s = t.mid0 + k; a = t.a_mid; return; }
  s = t.mid1;
  a = t.a_last;
}

__device__ __forceinline__ unsigned char sat_u8(float v) {   // saturate_cast<uchar>(float): cvRound = nearest even
  const int i = (int)rintf(v);
  return (unsigned char)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

struct AreaArgs {
  int B, H, W, C, OH, OW;
  const unsigned char* src;
  unsigned char* dst;
  float* dst_f;
  int f_cstride;
  double sx, sy, inv_sx, inv_sy;   // scale = src / dst (1 / inv_scale), inv_scale = dst / src
  int mode;                        // 0 copy, 1 fast integer area, 2 area tables, 3 area-emulating linear (upscale)
  int isx, isy;
};

__device__ __forceinline__ void area_store(const AreaArgs& a, long pix, int c, unsigned char v) {
  if (a.dst) a.dst[pix * a.C + c] = v;
  if (a.dst_f) a.dst_f[pix * a.f_cstride + c] = (float)v;
}

__global__ void __launch_bounds__(256) resize_area_kernel(const AreaArgs a) {
#pragma clang fp contract(off)
  const long total = (long)a.B * a.OH * a.OW;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int b = (int)(p / ((long)a.OH * a.OW));
    const int r = (int)(p - (long)b * a.OH * a.OW);
    const int dy = r / a.OW, dx = r - dy * a.OW;
    const unsigned char* S = a.src + (long)b * a.H * a.W * a.C;
    unsigned char area_out[4] = {0, 0, 0, 0};
    if (a.mode == 2) {
      // ResizeArea_Invoker: for each source row of the y-span (in table order) the row's x-span sum
      // buf = sum_k S*alpha_k (float, from 0), then sum = beta_0*buf_0, sum += beta_j*buf_j; round.  The spans are
      // computed once per output pixel, all channels accumulate together (same per-channel operation order).
      const AreaSpan ty = area_span(dy, a.H, a.sy), tx = area_span(dx, a.W, a.sx);
      float sum[4] = {0.f, 0.f, 0.f, 0.f};
      // up to kAreaTaps taps per axis (scales < kAreaTaps - 1) with every tap's load of a row issued before its
      // first use; wider cells take the plain loop
      constexpr int kAreaTaps = 6;
      int xs[kAreaTaps];
      float xa[kAreaTaps];
      const bool small = tx.n <= kAreaTaps;
#pragma unroll
      for (int k = 0; k < kAreaTaps; ++k) {
        xs[k] = 0;
        xa[k] = 0.f;
        if (k < tx.n) area_tap(tx, k, xs[k], xa[k]);
      }
      for (int j = 0; j < ty.n; ++j) {
        int sy;
        float beta;
        area_tap(ty, j, sy, beta);
        const unsigned char* row = S + (long)sy * a.W * a.C;
        float buf[4] = {0.f, 0.f, 0.f, 0.f};
        if (small) {
          unsigned char v[kAreaTaps][4];
#pragma unroll
          for (int k = 0; k < kAreaTaps; ++k)
#pragma unroll
            for (int c = 0; c < 4; ++c) v[k][c] = (k < tx.n && c < a.C) ? row[(long)xs[k] * a.C + c] : 0;
#pragma unroll
          for (int k = 0; k < kAreaTaps; ++k)
            if (k < tx.n) {
#pragma unroll
              for (int c = 0; c < 4; ++c) buf[c] = buf[c] + (float)v[k][c] * xa[k];
            }
        } else {
          for (int k = 0; k < tx.n; ++k) {
            int sx;
            float alpha;
            area_tap(tx, k, sx, alpha);
            const unsigned char* px = row + (long)sx * a.C;
#pragma unroll
            for (int c = 0; c < 4; ++c)
              if (c < a.C) buf[c] = buf[c] + (float)px[c] * alpha;
          }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) sum[c] = (j == 0) ? beta * buf[c] : sum[c] + beta * buf[c];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) area_out[c] = sat_u8(sum[c]);
    }
    for (int c = 0; c < a.C; ++c) {
      unsigned char out;
      if (a.mode == 0) {
        out = S[((long)dy * a.W + dx) * a.C + c];
      } else if (a.mode == 1) {
        // resizeAreaFast_ (scalar): int sum over the isx x isy cell, saturate_cast<uchar>(sum * (1.f / area)); a
        // cell cut by the image edge averages its in-range pixels (sum / count)
        const int sy0 = dy * a.isy, sx0 = dx * a.isx;
        const bool whole = sy0 + a.isy <= a.H && dx < a.W / a.isx;
        int sum = 0, count = 0;
        for (int yy = 0; yy < a.isy; ++yy) {
          if (sy0 + yy >= a.H) break;
          for (int xx = 0; xx < a.isx; ++xx) {
            if (sx0 + xx >= a.W) break;
            sum += S[((long)(sy0 + yy) * a.W + sx0 + xx) * a.C + c];
            ++count;
          }
        }
        if (whole) {
          out = sat_u8((float)sum * __fdiv_rn(1.f, (float)(a.isx * a.isy)));
        } else {
          out = count ? sat_u8(__fdiv_rn((float)sum, (float)count)) : (unsigned char)0;
        }
      } else if (a.mode == 2) {
        out = area_out[c];
      } else {
        // area-mode emulation by linear interpolation (resizeGeneric_ with area_mode, 8-bit fixed point):
        // sx = floor(dx*scale), fx = (dx+1) - (sx+1)*inv_scale, fx = fx <= 0 ? 0 : fx - floor(fx); coefficients
        // saturate_cast<short>(w * 2048); horizontal int sums, vertical (v0*b0 + v1*b1 + 2^21) >> 22
        // columns: xofs / alpha with the border rules of resizeGeneric_ (sx < 0 -> 0; sx >= W-1 -> W-1, fx = 0)
        int sx = (int)floor(dx * a.sx);
        float fx = (float)((dx + 1) - (sx + 1) * a.inv_sx);
        fx = fx <= 0.f ? 0.f : fx - floorf(fx);
        if (sx < 0) { fx = 0.f; sx = 0; }
        const bool xhi = sx + 1 >= a.W;            // dx >= xmax: HResizeLinear's tail (first tap at full weight)
        if (sx >= a.W - 1) { fx = 0.f; sx = a.W - 1; }
        // rows: yofs / beta as computed (no border rule), the two source rows clipped to [0, H-1]
        const int sy = (int)floor(dy * a.sy);
        float fy = (float)((dy + 1) - (sy + 1) * a.inv_sy);
        fy = fy <= 0.f ? 0.f : fy - floorf(fy);
        const int ax0 = (int)rintf((1.f - fx) * 2048.f), ax1 = (int)rintf(fx * 2048.f);
        const int by0 = (int)rintf((1.f - fy) * 2048.f), by1 = (int)rintf(fy * 2048.f);
        int v[2];
        for (int k = 0; k < 2; ++k) {
          const int yy = min(max(sy + k, 0), a.H - 1);
          const unsigned char* row = S + (long)yy * a.W * a.C;
          v[k] = xhi ? (int)row[(long)sx * a.C + c] * 2048
                     : (int)row[(long)sx * a.C + c] * ax0 + (int)row[(long)(sx + 1) * a.C + c] * ax1;
        }
        const int acc = (v[0] * by0 + v[1] * by1 + (1 << 21)) >> 22;
        out = (unsigned char)(acc < 0 ? 0 : (acc > 255 ? 255 : acc));
      }
      area_store(a, p, c, out);
    }
  }
}

// ---------------------------------------------------------------- INTER_CUBIC (float, one channel)
struct CubicArgs {
  int B, H, W, OH, OW;
  const float* src;
  int s_cstride, s_coff;
  float* dst;
  double sx, sy;
};

// interpolateCubic (resize.cpp), A = -0.75, float arithmetic
__device__ __forceinline__ void cubic_coeffs(float x, float* c) {
#pragma clang fp contract(off)
  const float A = -0.75f;
  c[0] = ((A * (x + 1.f) - 5.f * A) * (x + 1.f) + 8.f * A) * (x + 1.f) - 4.f * A;
  c[1] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  c[2] = ((A + 2.f) * (1.f - x) - (A + 3.f)) * (1.f - x) * (1.f - x) + 1.f;
  c[3] = 1.f - c[0] - c[1] - c[2];
}

__global__ void __launch_bounds__(256) resize_cubic_kernel(const CubicArgs a) {
#pragma clang fp contract(off)
  const long total = (long)a.B * a.OH * a.OW;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int b = (int)(p / ((long)a.OH * a.OW));
    const int r = (int)(p - (long)b * a.OH * a.OW);
    const int dy = r / a.OW, dx = r - dy * a.OW;
    const float* S = a.src + (long)b * a.H * a.W * a.s_cstride + a.s_coff;
    if (a.H == a.OH && a.W == a.OW) {      // cv::resize to the same size is a copy
      a.dst[p] = S[(long)r * a.s_cstride];
      continue;
    }
    float fx = (float)((dx + 0.5) * a.sx - 0.5);
    const int sx = (int)floorf(fx);
    fx -= (float)sx;
    float fy = (float)((dy + 0.5) * a.sy - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    float cx[4], cy[4];
    cubic_coeffs(fx, cx);
    cubic_coeffs(fy, cy);
    float rows[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // resizeGeneric_Invoker: source rows clipped to [0, H-1]; HResizeCubic: out-of-range taps replicate the edge
      const int yy = min(max(sy - 1 + k, 0), a.H - 1);
      const float* row = S + (long)yy * a.W * a.s_cstride;
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int xx = min(max(sx - 1 + j, 0), a.W - 1);
        v = v + row[(long)xx * a.s_cstride] * cx[j];
      }
      rows[k] = v;
    }
    // VResizeCubic: b0*S0 + b1*S1 + b2*S2 + b3*S3, left to right
    a.dst[p] = cy[0] * rows[0] + cy[1] * rows[1] + cy[2] * rows[2] + cy[3] * rows[3];
  }
}

// ---------------------------------------------------------------- bilateralFilter (float, one channel)
constexpr int kExpBins = 1 << 12;          // kExpNumBinsPerChannel (cn = 1)
constexpr int kMaxTaps = 31 * 31;          // d <= 31

struct BilateralArgs {
  int B, H, W, radius, maxk;
  const float* src;
  float* dst;
  float* ws;                 // per image: [min, max, scale_index, copy flag] then the exp LUT [kExpBins + 2]
  double color_coeff;        // -0.5 / sigma_color^2
};

struct SpaceTable {
  float w[kMaxTaps];
  short dy[kMaxTaps], dx[kMaxTaps];
};

constexpr int kBilWs = 4 + kExpBins + 2;   // floats per image (then the min / max partials, kMinMaxBlocks x 2 each)

constexpr int kMinMaxBlocks = 64;          // min / max partial blocks per image

struct BilPartials {
  float* p;                  // [B][kMinMaxBlocks][2] (min, max) partials
};

// per image min / max partials (minMaxLoc over the map, NaN skipped): block x of image y takes a strided share
__global__ void __launch_bounds__(256) bil_minmax_kernel(const BilateralArgs a, BilPartials bp) {
  const int b = blockIdx.y;
  const float* S = a.src + (long)b * a.H * a.W;
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < a.H * a.W; i += kMinMaxBlocks * 256) {
    const float v = S[i];
    if (v == v) {
      lo = fminf(lo, v);
      hi = fmaxf(hi, v);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_down(lo, o, 64));
    hi = fmaxf(hi, __shfl_down(hi, o, 64));
  }
  __shared__ float sl[4], sh[4];
  if ((threadIdx.x & 63) == 0) {
    sl[threadIdx.x >> 6] = lo;
    sh[threadIdx.x >> 6] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) {
      lo = fminf(lo, sl[w]);
      hi = fmaxf(hi, sh[w]);
    }
    bp.p[((long)b * kMinMaxBlocks + blockIdx.x) * 2] = lo;
    bp.p[((long)b * kMinMaxBlocks + blockIdx.x) * 2 + 1] = hi;
  }
}

// Each block first folds the image's min / max partials (min / max are order-free: every block gets the same
// values) -> scale_index and the copy flag (block 0 publishes them), then its share of the table:
// expLUT[i] = (float)exp(val*val*gauss_color_coeff), double val = i / scale_index (a float division: scale_index is
// a float)
__global__ void __launch_bounds__(256) bil_lut_kernel(const BilateralArgs a, BilPartials bp) {
  const int b = blockIdx.y;
  float* W = a.ws + (long)b * kBilWs;
  __shared__ float s_scale;
  if (threadIdx.x < 64) {
    float lo = bp.p[((long)b * kMinMaxBlocks + threadIdx.x) * 2], hi = bp.p[((long)b * kMinMaxBlocks + threadIdx.x) * 2 + 1];
    for (int o = 32; o > 0; o >>= 1) {
      lo = fminf(lo, __shfl_down(lo, o, 64));
      hi = fmaxf(hi, __shfl_down(hi, o, 64));
    }
    if (threadIdx.x == 0) {
      // len = (float)(maxVal - minVal) * cn (minMaxLoc returns doubles); scale_index = kExpNumBins / len (float)
      const float len = (float)((double)hi - (double)lo);
      s_scale = __fdiv_rn((float)kExpBins, len);
      if (blockIdx.x == 0) {
        W[0] = lo;
        W[1] = hi;
        W[2] = s_scale;
        W[3] = fabs((double)lo - (double)hi) < FLT_EPSILON ? 1.f : 0.f;
      }
    }
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kExpBins + 2) return;
  const double val = (double)__fdiv_rn((float)i, s_scale);
  W[4 + i] = (float)exp(val * val * a.color_coeff);
}

__global__ void __launch_bounds__(256) bil_filter_kernel(const BilateralArgs a, const SpaceTable sp) {
#pragma clang fp contract(off)
  const long total = (long)a.B * a.H * a.W;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int b = (int)(p / ((long)a.H * a.W));
    const int r = (int)(p - (long)b * a.H * a.W);
    const int y = r / a.W, x = r - y * a.W;
    const float* S = a.src + (long)b * a.H * a.W;
    const float* Wk = a.ws + (long)b * kBilWs;
    const float rval = S[r];
    if (Wk[3] != 0.f) {                      // a constant map: src.copyTo(dst)
      a.dst[p] = rval;
      continue;
    }
    const float scale_index = Wk[2];
    const float* lut = Wk + 4;
    float sum = 0.f, wsum = 0.f;
    for (int k = 0; k < a.maxk; ++k) {
      // copyMakeBorder(BORDER_REFLECT_101) of radius pixels, read at the tap offset
      int yy = y + sp.dy[k], xx = x + sp.dx[k];
      yy = yy < 0 ? -yy : (yy >= a.H ? 2 * a.H - 2 - yy : yy);
      xx = xx < 0 ? -xx : (xx >= a.W ? 2 * a.W - 2 - xx : xx);
      const float val = S[(long)yy * a.W + xx];
      float alpha = fabsf(val - rval) * scale_index;
      const int idx = (int)floorf(alpha);
      alpha -= (float)idx;
      if (val == val) {
        const float w = sp.w[k] * (rval != rval ? 1.f : (lut[idx] + alpha * (lut[idx + 1] - lut[idx])));
        wsum += w;
        sum += val * w;
      }
    }
    a.dst[p] = rval != rval ? __fdiv_rn(sum, wsum) : __fdiv_rn(sum + rval, wsum + 1.f);
  }
}

int blocks_for(long total) {
  long bl = (total + 255) / 256;
  return (int)(bl > 4096 ? 4096 : (bl < 1 ? 1 : bl));
}

}  // namespace

extern "C" {

int tde_resize_area_u8(int B, int H, int W, int C, const unsigned char* src, int OH, int OW, unsigned char* dst_u8,
                       float* dst_f32, int f32_cstride, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && C <= 4 && OH > 0 && OW > 0 && src && (dst_u8 || dst_f32));
  TDE_CHECK_ARG(!dst_f32 || f32_cstride >= C);
  AreaArgs a{};
  a.B = B; a.H = H; a.W = W; a.C = C; a.OH = OH; a.OW = OW;
  a.src = src; a.dst = dst_u8; a.dst_f = dst_f32; a.f_cstride = f32_cstride;
  // cv::resize: inv_scale = dsize / ssize (double), hal::resize: scale = 1 / inv_scale
  a.inv_sx = (double)OW / W;
  a.inv_sy = (double)OH / H;
  a.sx = 1. / a.inv_sx;
  a.sy = 1. / a.inv_sy;
  if (H == OH && W == OW) {
    a.mode = 0;
  } else {
    const int ix = (int)lrint(a.sx), iy = (int)lrint(a.sy);
    const bool fast = std::fabs(a.sx - ix) < DBL_EPSILON && std::fabs(a.sy - iy) < DBL_EPSILON;
    if (a.sx >= 1 && a.sy >= 1) {
      a.mode = fast ? 1 : 2;
      a.isx = ix;
      a.isy = iy;
    } else {
      a.mode = 3;
    }
  }
  hipLaunchKernelGGL(resize_area_kernel, dim3(blocks_for((long)B * OH * OW)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  return tde_launch_status();
}

int tde_resize_cubic_f32(int B, int H, int W, const float* src, int s_cstride, int s_coff, int OH, int OW, float* dst,
                         void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && src && dst && s_coff >= 0 && s_coff < s_cstride);
  CubicArgs a{};
  a.B = B; a.H = H; a.W = W; a.OH = OH; a.OW = OW;
  a.src = src; a.s_cstride = s_cstride; a.s_coff = s_coff; a.dst = dst;
  a.sx = 1. / ((double)OW / W);
  a.sy = 1. / ((double)OH / H);
  hipLaunchKernelGGL(resize_cubic_kernel, dim3(blocks_for((long)B * OH * OW)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  return tde_launch_status();
}

size_t tde_bilateral_workspace_size(int B) {
  return B > 0 ? (size_t)B * (kBilWs + 2 * kMinMaxBlocks) * sizeof(float) : 0;
}

int tde_bilateral_f32(int B, int H, int W, const float* src, float* dst, int d, double sigma_color,
                      double sigma_space, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 1 && W > 1 && src && dst && src != dst && d <= 31);
  if (ws_bytes < tde_bilateral_workspace_size(B) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  // bilateralFilter_32f: sigma <= 0 -> 1; radius = d > 0 ? d / 2 : cvRound(1.5 sigma_space), at least 1
  if (sigma_color <= 0) sigma_color = 1;
  if (sigma_space <= 0) sigma_space = 1;
  int radius = d <= 0 ? (int)lrint(sigma_space * 1.5) : d / 2;
  radius = radius < 1 ? 1 : radius;
  TDE_CHECK_ARG(radius <= 15 && radius < H && radius < W);
  const double space_coeff = -0.5 / (sigma_space * sigma_space);
  SpaceTable sp{};
  int maxk = 0;
  for (int i = -radius; i <= radius; ++i)
    for (int j = -radius; j <= radius; ++j) {
      const double r = std::sqrt((double)i * i + (double)j * j);
      if (r > radius || (i == 0 && j == 0)) continue;
      sp.w[maxk] = (float)std::exp(r * r * space_coeff);
      sp.dy[maxk] = (short)i;
      sp.dx[maxk] = (short)j;
      ++maxk;
    }
  BilateralArgs a{};
  a.B = B; a.H = H; a.W = W; a.radius = radius; a.maxk = maxk;
  a.src = src; a.dst = dst; a.ws = static_cast<float*>(ws);
  a.color_coeff = -0.5 / (sigma_color * sigma_color);
  hipStream_t st = static_cast<hipStream_t>(stream);
  BilPartials bp{static_cast<float*>(ws) + (size_t)B * kBilWs};
  hipLaunchKernelGGL(bil_minmax_kernel, dim3(kMinMaxBlocks, B), dim3(256), 0, st, a, bp);
  hipLaunchKernelGGL(bil_lut_kernel, dim3(tde_cdiv(kExpBins + 2, 256), B), dim3(256), 0, st, a, bp);
  hipLaunchKernelGGL(bil_filter_kernel, dim3(blocks_for((long)B * H * W)), dim3(256), 0, st, a, sp);
  return tde_launch_status();
}

}  // extern "C"
