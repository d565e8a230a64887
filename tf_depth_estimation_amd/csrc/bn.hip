// slim.batch_norm(center=True, scale=False, eps=1e-3) + ReLU, training and inference, forward and
// backward (TF FusedBatchNorm / FusedBatchNormGrad as used by the arg_scope of
// nets_optflow_depth.py:82-87).  HBM-bound: one read of z for the statistics,
// one read + one (strided) write for the apply; the backward reads z and dy twice and writes dz.
// Per-channel sums are accumulated in fp64 per block and reduced deterministically (no atomics).
#include "tde_common.h"

namespace {

// Grid: blockIdx.x = row chunk.  Threads: tx = channel quad (C/4 of them), ty = row lane.
struct RowSplit {
  int cq, ty_n, chunks, rows_per_chunk;
};

RowSplit row_split(int M, int C) {
  RowSplit r;
  r.cq = C / 4;
  r.ty_n = r.cq >= 256 ? 1 : 256 / r.cq;
  // <= 256 chunks (the finalize reads chunks x C partials), >= 4 rows per thread lane
  const int target = 256;
  r.rows_per_chunk = (M + target - 1) / target;
  if (r.rows_per_chunk < 4 * r.ty_n) r.rows_per_chunk = 4 * r.ty_n;
  r.rows_per_chunk = (r.rows_per_chunk + r.ty_n - 1) / r.ty_n * r.ty_n;
  r.chunks = (M + r.rows_per_chunk - 1) / r.rows_per_chunk;
  return r;
}

// Sum the per-chunk fp64 partials [chunks][2][C] for 64 channels per 1024-thread block: 16 waves
// split the chunk range, each keeping 4 chunks' loads in flight (the loop is L2-latency bound, not
// bandwidth bound), then one fixed-order LDS combine.  Returns (in wave 0) the totals for channel c.
constexpr int FIN_WAVES = 16;
__device__ __forceinline__ bool reduce_chunks(int C, int chunks, const double* part, double& s0, double& s1,
                                              int& c) {
  __shared__ double sh[2][FIN_WAVES * 64];
  const int cl = threadIdx.x & 63, w = threadIdx.x >> 6;
  c = blockIdx.x * 64 + cl;
  double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < C) {
    const long st = 2l * C;
    int k = w;
    for (; k + 3 * FIN_WAVES < chunks; k += 4 * FIN_WAVES) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] += part[(k + u * FIN_WAVES) * st + c];
        b[u] += part[(k + u * FIN_WAVES) * st + C + c];
      }
    }
    for (int u = 0; k < chunks; k += FIN_WAVES, ++u) {
      a[u & 3] += part[k * st + c];
      b[u & 3] += part[k * st + C + c];
    }
  }
  sh[0][threadIdx.x] = (a[0] + a[1]) + (a[2] + a[3]);
  sh[1][threadIdx.x] = (b[0] + b[1]) + (b[2] + b[3]);
  __syncthreads();
  if (w != 0 || c >= C) return false;
  s0 = 0.0; s1 = 0.0;
#pragma unroll
  for (int v = 0; v < FIN_WAVES; ++v) { s0 += sh[0][cl + 64 * v]; s1 += sh[1][cl + 64 * v]; }
  return true;
}

// MODE 0: sums of z and z^2.  MODE 1 (backward): sums of g and g*xhat where g = dy * relu'(y).
template <int MODE>
__global__ void __launch_bounds__(256) bn_partial_kernel(int M, int C, const float* z, const float* dy, int dycs,
                                                          int dyco, const float* mean, const float* invstd,
                                                          const float* beta, int relu, int rows_per_chunk,
                                                          double* part) {
  const int cq = C / 4;
  const int ty_n = cq >= 256 ? 1 : 256 / cq;
  const int tx = threadIdx.x % cq, ty = threadIdx.x / cq;
  __shared__ double sh[2][256 * 4];
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  for (int cbase = 0; cbase < cq; cbase += 256) {  // C > 1024 would loop; C <= 1024 in this net
    const int c4 = cbase + tx;
    if (ty < ty_n && c4 < cq) {
      f4 mu = {0, 0, 0, 0}, is = {0, 0, 0, 0}, bt = {0, 0, 0, 0};
      if (MODE == 1) {
        mu = *reinterpret_cast<const f4*>(mean + 4 * c4);
        is = *reinterpret_cast<const f4*>(invstd + 4 * c4);
        bt = *reinterpret_cast<const f4*>(beta + 4 * c4);
      }
      // fp32 partials over <= 64 rows per thread, flushed into fp64; unrolled so 8 rows' loads are
      // in flight at once (one load per iteration would expose the full memory latency each time)
      for (int rb = r0 + ty; rb < r1; rb += 64 * ty_n) {
        const int rend = min(r1, rb + 64 * ty_n);
        float f0[4] = {0, 0, 0, 0}, f1[4] = {0, 0, 0, 0};
#pragma unroll 8
        for (int r = rb; r < rend; r += ty_n) {
          const f4 zv = *reinterpret_cast<const f4*>(z + (long)r * C + 4 * c4);
          if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) { f0[j] += zv[j]; f1[j] += zv[j] * zv[j]; }
          } else {
            const f4 gv = *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + 4 * c4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float xh = (zv[j] - mu[j]) * is[j];
              const float g = (!relu || xh + bt[j] > 0.f) ? gv[j] : 0.f;
              f0[j] += g; f1[j] += g * xh;
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) { s0[j] += f0[j]; s1[j] += f1[j]; }
      }
    }
  }
  // reduce over ty within the block (cq <= 256 case; for cq > 256 each thread owns distinct channels)
#pragma unroll
  for (int j = 0; j < 4; ++j) { sh[0][threadIdx.x * 4 + j] = s0[j]; sh[1][threadIdx.x * 4 + j] = s1[j]; }
  __syncthreads();
  if (ty == 0 && tx < cq) {
    for (int t = 1; t < ty_n; ++t) {
      const int src = (t * cq + tx) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) { s0[j] += sh[0][src + j]; s1[j] += sh[1][src + j]; }
    }
    double* o = part + (long)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[4 * tx + j] = s0[j]; o[C + 4 * tx + j] = s1[j]; }
  }
}

__global__ void __launch_bounds__(1024) bn_stats_finalize_kernel(int M, int C, int chunks, const double* part, float eps, float decay,
                                         int bessel, float* mm, float* mv, float* save_mean, float* save_invstd) {
  double s, ss;
  int c;
  if (!reduce_chunks(C, chunks, part, s, ss, c)) return;
  const double mean = s / M;
  double var = ss / M - mean * mean;
  if (var < 0) var = 0;
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (mm) {
    const double vu = (bessel && M > 1) ? var * M / (M - 1) : var;
    mm[c] -= (mm[c] - (float)mean) * (1.f - decay);
    mv[c] -= (mv[c] - (float)vu) * (1.f - decay);
  }
}

__global__ void __launch_bounds__(256) bn_apply_kernel(int M, int C, const float* z, const float* mean,
                                                       const float* invstd, const float* beta, int relu, float* y,
                                                       int ycs, int yco) {
  const int cq = C / 4;
  const long total = (long)M * cq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cq;
    const int c = 4 * (int)(i - r * cq);
    const f4 zv = *reinterpret_cast<const f4*>(z + r * C + c);
    const f4 mu = *reinterpret_cast<const f4*>(mean + c);
    const f4 is = *reinterpret_cast<const f4*>(invstd + c);
    const f4 bt = *reinterpret_cast<const f4*>(beta + c);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = (zv[j] - mu[j]) * is[j] + bt[j];
      o[j] = (relu && v < 0.f) ? 0.f : v;
    }
    *reinterpret_cast<f4*>(y + r * ycs + yco + c) = o;
  }
}

__global__ void __launch_bounds__(256) bn_infer_kernel(int M, int C, const float* z, const float* mm,
                                                       const float* mv, float eps, const float* beta, int relu,
                                                       float* y, int ycs, int yco) {
  const int cq = C / 4;
  const long total = (long)M * cq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cq;
    const int c = 4 * (int)(i - r * cq);
    const f4 zv = *reinterpret_cast<const f4*>(z + r * C + c);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v = (zv[j] - mm[c + j]) / sqrtf(mv[c + j] + eps) + beta[c + j];
      o[j] = (relu && v < 0.f) ? 0.f : v;
    }
    *reinterpret_cast<f4*>(y + r * ycs + yco + c) = o;
  }
}

__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(int M, int C, int chunks, const double* part, float* dbeta, int acc,
                                       float* coef /*[2][C]: mean(g), mean(g*xhat)*/) {
  double s, sx;
  int c;
  if (!reduce_chunks(C, chunks, part, s, sx, c)) return;
  if (dbeta) dbeta[c] = acc ? dbeta[c] + (float)s : (float)s;
  coef[c] = (float)(s / M);
  coef[C + c] = (float)(sx / M);
}

__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(int M, int C, const float* z, const float* dy, int dycs,
                                                           int dyco, const float* mean, const float* invstd,
                                                           const float* beta, const float* coef, int relu,
                                                           float* dz) {
  const int cq = C / 4;
  const long total = (long)M * cq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cq;
    const int c = 4 * (int)(i - r * cq);
    const f4 zv = *reinterpret_cast<const f4*>(z + r * C + c);
    const f4 gv = *reinterpret_cast<const f4*>(dy + r * dycs + dyco + c);
    const f4 mu = *reinterpret_cast<const f4*>(mean + c);
    const f4 is = *reinterpret_cast<const f4*>(invstd + c);
    const f4 bt = *reinterpret_cast<const f4*>(beta + c);
    const f4 mg = *reinterpret_cast<const f4*>(coef + c);
    const f4 mgx = *reinterpret_cast<const f4*>(coef + C + c);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (zv[j] - mu[j]) * is[j];
      const float g = (!relu || xh + bt[j] > 0.f) ? gv[j] : 0.f;
      o[j] = is[j] * (g - mg[j] - xh * mgx[j]);
    }
    *reinterpret_cast<f4*>(dz + r * C + c) = o;
  }
}


// ------------------------------------------------------------------ small-M layers: one kernel each way
// The deep encoder/decoder levels (12x16 down to 1x1 at batch 8: M <= 2048 rows) are launch-latency
// bound as three kernels.  Here a block owns 16 channels over ALL rows (4 channel quads x 64 row lanes),
// so statistics (fp64), finalize and apply happen in one launch with one LDS combine.
constexpr int SMALL_M = 2048;

__global__ void __launch_bounds__(256) bn_small_fwd_kernel(int M, int C, const float* z, const float* beta,
                                                           float eps, float decay, int bessel, float* mm,
                                                           float* mv, float* save_mean, float* save_invstd,
                                                           float* y, int ycs, int yco, int relu) {
  __shared__ double sh[2][64][17];
  __shared__ float s_mu[16], s_is[16];
  const int qd = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int c = blockIdx.x * 16 + 4 * qd;
  const bool ok = c < C;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  if (ok)
    for (int r = rl; r < M; r += 64) {
      const f4 v = *reinterpret_cast<const f4*>(z + (long)r * C + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) { a[j] += v[j]; b[j] += (double)v[j] * v[j]; }
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) { sh[0][rl][4 * qd + j] = a[j]; sh[1][rl][4 * qd + j] = b[j]; }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int cl = threadIdx.x, cc = blockIdx.x * 16 + cl;
    double s = 0.0, ss = 0.0;
    for (int l = 0; l < 64; ++l) { s += sh[0][l][cl]; ss += sh[1][l][cl]; }
    const double mean = s / M;
    double var = ss / M - mean * mean;
    if (var < 0) var = 0;
    const float mu = (float)mean, is = (float)(1.0 / sqrt(var + (double)eps));
    s_mu[cl] = mu; s_is[cl] = is;
    if (cc < C) {
      save_mean[cc] = mu;
      save_invstd[cc] = is;
      if (mm) {
        const double vu = (bessel && M > 1) ? var * M / (M - 1) : var;
        mm[cc] -= (mm[cc] - mu) * (1.f - decay);
        mv[cc] -= (mv[cc] - (float)vu) * (1.f - decay);
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  const f4 bt = *reinterpret_cast<const f4*>(beta + c);
  for (int r = rl; r < M; r += 64) {
    const f4 v = *reinterpret_cast<const f4*>(z + (long)r * C + c);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = (v[j] - s_mu[4 * qd + j]) * s_is[4 * qd + j] + bt[j];
      o[j] = (relu && t < 0.f) ? 0.f : t;
    }
    *reinterpret_cast<f4*>(y + (long)r * ycs + yco + c) = o;
  }
}

__global__ void __launch_bounds__(256) bn_small_bwd_kernel(int M, int C, const float* z, const float* mean,
                                                           const float* invstd, const float* beta, const float* dy,
                                                           int dycs, int dyco, float* dz, float* dbeta, int acc,
                                                           int relu) {
  __shared__ double sh[2][64][17];
  __shared__ float s_mg[16], s_mgx[16];
  const int qd = threadIdx.x & 3, rl = threadIdx.x >> 2;
  const int c = blockIdx.x * 16 + 4 * qd;
  const bool ok = c < C;
  f4 mu = {0, 0, 0, 0}, is = {0, 0, 0, 0}, bt = {0, 0, 0, 0};
  if (ok) {
    mu = *reinterpret_cast<const f4*>(mean + c);
    is = *reinterpret_cast<const f4*>(invstd + c);
    bt = *reinterpret_cast<const f4*>(beta + c);
  }
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  if (ok)
    for (int r = rl; r < M; r += 64) {
      const f4 v = *reinterpret_cast<const f4*>(z + (long)r * C + c);
      const f4 gv = *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (v[j] - mu[j]) * is[j];
        const float g = (!relu || xh + bt[j] > 0.f) ? gv[j] : 0.f;
        a[j] += g; b[j] += (double)g * xh;
      }
    }
#pragma unroll
  for (int j = 0; j < 4; ++j) { sh[0][rl][4 * qd + j] = a[j]; sh[1][rl][4 * qd + j] = b[j]; }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int cl = threadIdx.x, cc = blockIdx.x * 16 + cl;
    double s = 0.0, sx = 0.0;
    for (int l = 0; l < 64; ++l) { s += sh[0][l][cl]; sx += sh[1][l][cl]; }
    s_mg[cl] = (float)(s / M);
    s_mgx[cl] = (float)(sx / M);
    if (cc < C && dbeta) dbeta[cc] = acc ? dbeta[cc] + (float)s : (float)s;
  }
  __syncthreads();
  if (!ok) return;
  for (int r = rl; r < M; r += 64) {
    const f4 v = *reinterpret_cast<const f4*>(z + (long)r * C + c);
    const f4 gv = *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + c);
    f4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (v[j] - mu[j]) * is[j];
      const float g = (!relu || xh + bt[j] > 0.f) ? gv[j] : 0.f;
      o[j] = is[j] * (g - s_mg[4 * qd + j] - xh * s_mgx[4 * qd + j]);
    }
    *reinterpret_cast<f4*>(dz + (long)r * C + c) = o;
  }
}

int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

size_t tde_bn_workspace_size(int M, int C) {
  if (M <= 0 || C <= 0 || C % 4) return 0;
  const RowSplit rs = row_split(M, C);
  return (size_t)rs.chunks * 2 * C * sizeof(double) + 2 * (size_t)C * sizeof(float) + 64;
}

int tde_bn_fwd_train(int M, int C, const float* z, const float* beta, float eps, float decay, int bessel,
                     float* moving_mean, float* moving_var, float* save_mean, float* save_invstd, float* y,
                     int y_cstride, int y_coff, int relu, void* ws, size_t ws_bytes, void* stream) {
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && beta && save_mean && save_invstd && y);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride && tde_aligned16(z) && tde_aligned16(y));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (M <= SMALL_M) {
    hipLaunchKernelGGL(bn_small_fwd_kernel, dim3((C + 15) / 16), dim3(256), 0, st, M, C, z, beta, eps, decay, bessel,
                       moving_mean, moving_var, save_mean, save_invstd, y, y_cstride, y_coff, relu);
    return tde_launch_status();
  }
  const RowSplit rs = row_split(M, C);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(bn_partial_kernel<0>, dim3(rs.chunks), dim3(256), 0, st, M, C, z, nullptr, 0, 0, nullptr,
                     nullptr, nullptr, 0, rs.rows_per_chunk, part);
  hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, st, M, C, rs.chunks, part, eps,
                     decay, bessel, moving_mean, moving_var, save_mean, save_invstd);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid((long)M * C / 4)), dim3(256), 0, st, M, C, z, save_mean,
                     save_invstd, beta, relu, y, y_cstride, y_coff);
  return tde_launch_status();
}

int tde_bn_fwd_infer(int M, int C, const float* z, const float* beta, float eps, const float* moving_mean,
                     const float* moving_var, float* y, int y_cstride, int y_coff, int relu, void* stream) {
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && z && beta && moving_mean && moving_var && y);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(bn_infer_kernel, dim3(ew_grid((long)M * C / 4)), dim3(256), 0, st, M, C, z, moving_mean,
                     moving_var, eps, beta, relu, y, y_cstride, y_coff);
  return tde_launch_status();
}

int tde_bn_bwd(int M, int C, const float* z, const float* save_mean, const float* save_invstd, const float* beta,
               const float* dy, int dy_cstride, int dy_coff, float* dz, float* dbeta, int accumulate_dbeta, int relu,
               void* ws, size_t ws_bytes, void* stream) {
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && save_mean && save_invstd && beta && dy && dz);
  TDE_CHECK_ARG(dy_cstride % 4 == 0 && dy_coff % 4 == 0 && tde_aligned16(dy) && tde_aligned16(dz));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (M <= SMALL_M) {
    hipLaunchKernelGGL(bn_small_bwd_kernel, dim3((C + 15) / 16), dim3(256), 0, st, M, C, z, save_mean, save_invstd,
                       beta, dy, dy_cstride, dy_coff, dz, dbeta, accumulate_dbeta, relu);
    return tde_launch_status();
  }
  const RowSplit rs = row_split(M, C);
  double* part = static_cast<double*>(ws);
  float* coef = reinterpret_cast<float*>(part + (size_t)rs.chunks * 2 * C);
  hipLaunchKernelGGL(bn_partial_kernel<1>, dim3(rs.chunks), dim3(256), 0, st, M, C, z, dy, dy_cstride, dy_coff,
                     save_mean, save_invstd, beta, relu, rs.rows_per_chunk, part);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * FIN_WAVES), 0, st, M, C, rs.chunks, part, dbeta,
                     accumulate_dbeta, coef);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_grid((long)M * C / 4)), dim3(256), 0, st, M, C, z, dy, dy_cstride,
                     dy_coff, save_mean, save_invstd, beta, coef, relu, dz);
  return tde_launch_status();
}

}  // extern "C"
