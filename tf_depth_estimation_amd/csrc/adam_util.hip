// TF Adam over one flat parameter buffer (tf.train.AdamOptimizer, train_depth_then_cam_lr.py:413-417;
// TF ApplyAdam kernel: m += (g-m)(1-b1); v += (g*g-v)(1-b2); var -= lr_t*m/(sqrt(v)+eps)) plus small
// utilities.  Adam is HBM-bound: 4 reads + 3 writes of 4 B per parameter, 16-byte vectors.
#include <cstdio>

#include "tde_common.h"

namespace {

__global__ void step_begin_kernel(float* step) { step[0] += 1.f; }

// zero `bytes` bytes at p: n16 16-byte vectors (p 16-byte aligned; 0 otherwise), then the byte tail
__global__ void __launch_bounds__(256) zero_bytes_kernel(unsigned char* p, size_t bytes, size_t n16) {
  const size_t t = blockIdx.x * 256ull + threadIdx.x, nt = gridDim.x * 256ull;
  for (size_t i = t; i < n16; i += nt) reinterpret_cast<uint4*>(p)[i] = make_uint4(0, 0, 0, 0);
  for (size_t i = n16 * 16 + t; i < bytes; i += nt) p[i] = 0;
}

__global__ void __launch_bounds__(256) adam_kernel(long n4, f4* __restrict__ p, const f4* __restrict__ g,
                                                   f4* __restrict__ m, f4* __restrict__ v, const float* step,
                                                   float lr, float b1, float b2, float eps, float gs) {
  const double t = (double)step[0];
  const float lr_t = (float)((double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t)));
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f4 gi = g[i] * gs;   // gs == 1: exact, the gradient as stored
    f4 mi = m[i], vi = v[i], pi = p[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mi[j] += (gi[j] - mi[j]) * (1.f - b1);
      vi[j] += (gi[j] * gi[j] - vi[j]) * (1.f - b2);
      pi[j] -= lr_t * mi[j] / (sqrtf(vi[j]) + eps);
    }
    m[i] = mi; v[i] = vi; p[i] = pi;
  }
}

__global__ void __launch_bounds__(256) scale_kernel(long n, float* x, float a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= a;
}

__global__ void __launch_bounds__(256) fill_kernel(long n, float* x, float val) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] = val;
}

// I = unsigned when every element offset fits 32 bits (the row split is then a 32-bit division, not the
// long-division sequence of a 64-bit one)
template <typename I>
__global__ void __launch_bounds__(256) copy_view_kernel(int M, int C, const float* s, int scs, int sco, float* d,
                                                        int dcs, int dco, int acc) {
  const I total = (I)M * (I)C;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const I r = i / (I)C;
    const I c = i - r * (I)C;
    const float v = s[r * (I)scs + (I)sco + c];
    float* o = d + r * (I)dcs + (I)dco + c;
    *o = acc ? *o + v : v;
  }
}

// pose_avg = tf.reduce_mean(pose_pred, [1, 2]) (nets_optflow_depth.py:183): x [N,HW,C] -> y [N,C]
__global__ void spatial_mean_fwd_kernel(int N, int HW, int C, const float* x, int xcs, float* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += x[((long)n * HW + p) * xcs + c];
  y[i] = s / (float)HW;
}

__global__ void spatial_mean_bwd_kernel(int N, int HW, int C, float* dx, int dxcs, int acc, const float* dy) {
  const long total = (long)N * HW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = (int)(i - r * C);
    const int n = (int)(r / HW);
    const float g = dy[n * C + c] / (float)HW;
    float* o = dx + r * dxcs + c;
    *o = acc ? *o + g : g;
  }
}

int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

thread_local int tde_g_last_hip = 0;

extern "C" {

int tde_abi_version(void) { return TDE_ABI_VERSION; }

const char* tde_status_string(int s) {
  switch (s) {
    case TDE_OK: return "ok";
    case TDE_ERR_ARG: return "invalid argument (pointer, alignment or shape)";
    case TDE_ERR_WORKSPACE: return "workspace too small";
    case TDE_ERR_HIP: {
      static thread_local char buf[160];
      snprintf(buf, sizeof(buf), "HIP launch error: %s",
               hipGetErrorName(static_cast<hipError_t>(tde_g_last_hip)));
      return buf;
    }
    case TDE_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return "unknown status";
  }
}

int tde_adam_step_begin(float* step, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(step != nullptr);
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), step);
  return tde_launch_status();
}

int tde_adam_update(size_t n, float* param, const float* grad, float* m, float* v, const float* step, float lr,
                    float beta1, float beta2, float eps, float grad_scale, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(n % 4 == 0 && param && grad && m && v && step);
  TDE_CHECK_ARG(tde_aligned16(param) && tde_aligned16(grad) && tde_aligned16(m) && tde_aligned16(v));
  const long n4 = (long)(n / 4);
  hipLaunchKernelGGL(adam_kernel, dim3(ew_grid(n4)), dim3(256), 0, static_cast<hipStream_t>(stream), n4,
                     reinterpret_cast<f4*>(param), reinterpret_cast<const f4*>(grad), reinterpret_cast<f4*>(m),
                     reinterpret_cast<f4*>(v), step, lr, beta1, beta2, eps, grad_scale);
  return tde_launch_status();
}

int tde_zero_bytes(size_t bytes, void* p, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(p != nullptr);
  if (bytes == 0) return TDE_OK;
  // a kernel of our own, not hipMemsetAsync: a captured step then holds kernel nodes only (the runtime's
  // memset becomes a fill-kernel or memset node depending on size and alignment, 4.8 us per small launch)
  const size_t n16 = (reinterpret_cast<uintptr_t>(p) & 15) ? 0 : bytes / 16;
  long blocks = (long)((n16 + 255) / 256);
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  hipLaunchKernelGGL(zero_bytes_kernel, dim3((int)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<unsigned char*>(p), bytes, n16);
  return tde_launch_status();
}

int tde_spatial_mean_fwd(int N, int HW, int C, const float* x, int x_cstride, float* y, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && HW > 0 && C > 0 && x && y);
  hipLaunchKernelGGL(spatial_mean_fwd_kernel, dim3((N * C + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, HW, C, x, x_cstride, y);
  return tde_launch_status();
}

int tde_spatial_mean_bwd(int N, int HW, int C, float* dx, int dx_cstride, int accumulate, const float* dy,
                         void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && HW > 0 && C > 0 && dx && dy);
  hipLaunchKernelGGL(spatial_mean_bwd_kernel, dim3(ew_grid((long)N * HW * C)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), N, HW, C, dx, dx_cstride, accumulate, dy);
  return tde_launch_status();
}

int tde_scale(size_t n, float* x, float alpha, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(x != nullptr);
  hipLaunchKernelGGL(scale_kernel, dim3(ew_grid((long)n)), dim3(256), 0, static_cast<hipStream_t>(stream), (long)n, x,
                     alpha);
  return tde_launch_status();
}

int tde_fill(size_t n, float* x, float value, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(x != nullptr);
  hipLaunchKernelGGL(fill_kernel, dim3(ew_grid((long)n)), dim3(256), 0, static_cast<hipStream_t>(stream), (long)n, x,
                     value);
  return tde_launch_status();
}

int tde_copy_view(int M, int C, const float* src, int s_cstride, int s_coff, float* dst, int d_cstride, int d_coff,
                  int accumulate, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && src && dst);
  TDE_CHECK_ARG(s_cstride >= C && d_cstride >= C && s_coff >= 0 && d_coff >= 0);
  const long span = (long)M * (s_cstride > d_cstride ? s_cstride : d_cstride) + (s_coff > d_coff ? s_coff : d_coff);
  const dim3 grid(ew_grid((long)M * C));
  if (span < 0x7fffffffL)
    hipLaunchKernelGGL(copy_view_kernel<unsigned>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), M, C, src,
                       s_cstride, s_coff, dst, d_cstride, d_coff, accumulate);
  else
    hipLaunchKernelGGL(copy_view_kernel<long>, grid, dim3(256), 0, static_cast<hipStream_t>(stream), M, C, src,
                       s_cstride, s_coff, dst, d_cstride, d_coff, accumulate);
  return tde_launch_status();
}

}  // extern "C"
