// Fused forward+backward loss-head kernels.  Each call adds
// weight*term into a device fp64 scalar and adds d(weight*term)/d(pred) into a gradient view, in one
// pass over the prediction: the loss is the top of the graph, so its backward needs no saved state.
#include "tde_common.h"

#include <cstdlib>

namespace {

// value of the smoothed map at (n,i,j): pred or 1/pred (train_depth_then_cam_lr.py:217 smooths 1/disp)
struct Map {
  const float* p; int H, W, cs, co, recip;
  __device__ __forceinline__ float operator()(int n, int i, int j) const {
    const float v = p[((long)(n * H + i) * W + j) * cs + co];
    return recip ? 1.f / v : v;
  }
};

// compute_smooth_loss (train_depth_then_cam_lr.py:59-68): with f the map, TF evaluates
//   dx = f[:, :, 1:] - f[:, :, :-1], dy = f[:, 1:] - f[:, :-1]
//   dx2 = dx[:, :, 1:] - dx[:, :, :-1]; dxdy = dx[:, 1:] - dx[:, :-1]
//   dydx = dy[:, :, 1:] - dy[:, :, :-1]; dy2 = dy[:, 1:] - dy[:, :-1]
// and sums mean|.| of each.  The four second differences are evaluated here in the same fp32 order.
__device__ __forceinline__ float t_dx2(const Map& f, int n, int i, int j) {
  return (f(n, i, j + 2) - f(n, i, j + 1)) - (f(n, i, j + 1) - f(n, i, j));
}
__device__ __forceinline__ float t_dxdy(const Map& f, int n, int i, int j) {
  return (f(n, i + 1, j + 1) - f(n, i + 1, j)) - (f(n, i, j + 1) - f(n, i, j));
}
__device__ __forceinline__ float t_dydx(const Map& f, int n, int i, int j) {
  return (f(n, i + 1, j + 1) - f(n, i, j + 1)) - (f(n, i + 1, j) - f(n, i, j));
}
__device__ __forceinline__ float t_dy2(const Map& f, int n, int i, int j) {
  return (f(n, i + 2, j) - f(n, i + 1, j)) - (f(n, i + 1, j) - f(n, i, j));
}

__global__ void __launch_bounds__(256) smooth2_kernel(int N, int H, int W, Map f, float weight, double* loss,
                                                      float* g, int gcs, int gco) {
  __shared__ double sh[4];
  const double n1 = (double)N * H * (W - 2), n23 = (double)N * (H - 1) * (W - 1), n4 = (double)N * (H - 2) * W;
  const float w1 = (float)(weight / n1), w23 = (float)(weight / n23), w4 = (float)(weight / n4);
  const long total = (long)N * H * W;
  double lsum = 0.0;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int j = (int)(idx % W);
    const long t = idx / W;
    const int i = (int)(t % H), n = (int)(t / H);
    // forward terms anchored at (i,j)
    float lv = 0.f;
    if (j < W - 2) lv += fabsf(t_dx2(f, n, i, j)) * w1;
    if (i < H - 1 && j < W - 1) lv += (fabsf(t_dxdy(f, n, i, j)) + fabsf(t_dydx(f, n, i, j))) * w23;
    if (i < H - 2) lv += fabsf(t_dy2(f, n, i, j)) * w4;
    lsum += lv;
    // gradient wrt f(n,i,j): every term that contains it, times d|t|/dt = sign(t)
    float gf = 0.f;
    if (j < W - 2) gf += tde_sign(t_dx2(f, n, i, j)) * w1;
    if (j >= 1 && j - 1 < W - 2) gf -= 2.f * tde_sign(t_dx2(f, n, i, j - 1)) * w1;
    if (j >= 2) gf += tde_sign(t_dx2(f, n, i, j - 2)) * w1;
    if (i < H - 2) gf += tde_sign(t_dy2(f, n, i, j)) * w4;
    if (i >= 1 && i - 1 < H - 2) gf -= 2.f * tde_sign(t_dy2(f, n, i - 1, j)) * w4;
    if (i >= 2) gf += tde_sign(t_dy2(f, n, i - 2, j)) * w4;
    // dxdy/dydx(a,b) = f(a+1,b+1) - f(a+1,b) - f(a,b+1) + f(a,b)
    if (i < H - 1 && j < W - 1) gf += (tde_sign(t_dxdy(f, n, i, j)) + tde_sign(t_dydx(f, n, i, j))) * w23;
    if (i < H - 1 && j >= 1) gf -= (tde_sign(t_dxdy(f, n, i, j - 1)) + tde_sign(t_dydx(f, n, i, j - 1))) * w23;
    if (i >= 1 && j < W - 1) gf -= (tde_sign(t_dxdy(f, n, i - 1, j)) + tde_sign(t_dydx(f, n, i - 1, j))) * w23;
    if (i >= 1 && j >= 1) gf += (tde_sign(t_dxdy(f, n, i - 1, j - 1)) + tde_sign(t_dydx(f, n, i - 1, j - 1))) * w23;
    if (f.recip) {
      const float p = f.p[((long)(n * H + i) * W + j) * f.cs + f.co];
      gf *= -1.f / (p * p);
    }
    g[((long)(n * H + i) * W + j) * gcs + gco] += gf;
  }
  const double bs = tde_block_sum_d(lsum, sh);
  if (threadIdx.x == 0) atomicAdd(loss, bs);
}

__global__ void __launch_bounds__(256) l1_kernel(long total, const float* pred, int cs, int co, const float* label,
                                                 int nonfinite, float weight, double* loss, float* g, int gcs,
                                                 int gco) {
  __shared__ double sh[4];
  const float wn = (float)(weight / (double)total);
  double lsum = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float d = label[i] - pred[i * cs + co];
    if (nonfinite && !isfinite(d)) d = 0.f;  // lmbspecialops.replace_nonfinite; gradient masked too
    lsum += fabsf(d);
    g[i * gcs + gco] += -tde_sign(d) * wn;
  }
  const double bs = tde_block_sum_d(lsum, sh);
  if (threadIdx.x == 0) atomicAdd(loss, bs * (double)weight / (double)total);
}

// ------------------------------------------------------------------ DeMoN scale-invariant-gradient loss
// my_losses.py:78-82 (compute_loss_single_depth; split_training.py:117):
//   sig(f)[2d](p)   = w_d (f(p + D_d x) - f(p)) / (|f(p + D_d x)| + |f(p)| + eps_s)     (0 off the image)
//   sig(f)[2d+1](p) = same along y
//   loss += weight * mean_p sqrt(sum_c nf(sig(pred)_c(p) - sig(label)_c(p))^2 + eps)
// (lmbspecialops.scale_invariant_gradient per delta, concatenated as depthmotionnet.v2.losses does, and
// its pointwise_l2_loss: replace_nonfinite of the difference, label under stop_gradient).  The gradient
// wrt pred at q gathers every sig term that reads f(q): its own (as the centre) and those anchored at
// q - D_d x / q - D_d y (as the neighbour); the per-pixel L2 factor of those anchors is recomputed.
constexpr int SIG_MAXD = 8;
struct SigArgs {
  int N, H, W, nd;
  int delta[SIG_MAXD];
  float wt[SIG_MAXD];
  float seps, l2eps, weight;
  const float* pred; int cs, co;
  const float* label;
  double* loss;
  float* g; int gcs, gco;
};

__device__ __forceinline__ float sig_term(float f0, float f1, float w, float eps) {
  return w * (f1 - f0) / (fabsf(f1) + fabsf(f0) + eps);
}

// dL/dsig_c at pixel (n,i,j) for all 2*nd components (0 where the difference is non-finite); returns
// the pixel's sqrt(.) value.
__device__ float sig_pixel(const SigArgs& a, int n, int i, int j, float* G) {
  const long base = (long)(n * a.H + i) * a.W + j;
  const float p0 = a.pred[base * a.cs + a.co], l0 = a.label[base];
  float d[2 * SIG_MAXD];
  float ss = 0.f;
  for (int k = 0; k < a.nd; ++k) {
    const int D = a.delta[k];
    float dx = 0.f, dy = 0.f;   // both sig values are 0 off the image
    if (j + D < a.W) {
      const long q = base + D;
      dx = sig_term(p0, a.pred[q * a.cs + a.co], a.wt[k], a.seps) - sig_term(l0, a.label[q], a.wt[k], a.seps);
    }
    if (i + D < a.H) {
      const long q = base + (long)D * a.W;
      dy = sig_term(p0, a.pred[q * a.cs + a.co], a.wt[k], a.seps) - sig_term(l0, a.label[q], a.wt[k], a.seps);
    }
    if (!isfinite(dx)) dx = 0.f;   // sops.replace_nonfinite (gradient masked too)
    if (!isfinite(dy)) dy = 0.f;
    d[2 * k] = dx; d[2 * k + 1] = dy;
    ss += dx * dx + dy * dy;
  }
  const float r = sqrtf(ss + a.l2eps);
  for (int c = 0; c < 2 * a.nd; ++c) G[c] = d[c] / r;
  return r;
}

__global__ void __launch_bounds__(256) sig_l2_kernel(const SigArgs a) {
  __shared__ double sh[4];
  const long total = (long)a.N * a.H * a.W;
  const float wn = (float)(a.weight / (double)total);
  double lsum = 0.0;
  float G[2 * SIG_MAXD];
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int j = (int)(idx % a.W);
    const long t = idx / a.W;
    const int i = (int)(t % a.H), n = (int)(t / a.H);
    const float fq = a.pred[idx * a.cs + a.co];
    const float sq = tde_sign(fq);
    lsum += sig_pixel(a, n, i, j, G);
    float gq = 0.f;
    // q as the centre (f0) of its own terms: dt/df0 = w (-1/D - u sign(f0) / D^2)
    for (int k = 0; k < a.nd; ++k) {
      const int D = a.delta[k];
      if (j + D < a.W) {
        const float f1 = a.pred[(idx + D) * a.cs + a.co];
        const float den = fabsf(f1) + fabsf(fq) + a.seps, u = f1 - fq;
        gq += G[2 * k] * a.wt[k] * (-1.f / den - u * sq / (den * den));
      }
      if (i + D < a.H) {
        const float f1 = a.pred[(idx + (long)D * a.W) * a.cs + a.co];
        const float den = fabsf(f1) + fabsf(fq) + a.seps, u = f1 - fq;
        gq += G[2 * k + 1] * a.wt[k] * (-1.f / den - u * sq / (den * den));
      }
    }
    // q as the neighbour (f1) of the terms anchored D to the left / above: dt/df1 = w (1/D - u sign(f1) / D^2)
    for (int k = 0; k < a.nd; ++k) {
      const int D = a.delta[k];
      if (j - D >= 0) {
        sig_pixel(a, n, i, j - D, G);
        const float f0 = a.pred[(idx - D) * a.cs + a.co];
        const float den = fabsf(fq) + fabsf(f0) + a.seps, u = fq - f0;
        gq += G[2 * k] * a.wt[k] * (1.f / den - u * sq / (den * den));
      }
      if (i - D >= 0) {
        sig_pixel(a, n, i - D, j, G);
        const float f0 = a.pred[(idx - (long)D * a.W) * a.cs + a.co];
        const float den = fabsf(fq) + fabsf(f0) + a.seps, u = fq - f0;
        gq += G[2 * k + 1] * a.wt[k] * (1.f / den - u * sq / (den * den));
      }
    }
    a.g[idx * a.gcs + a.gco] += gq * wn;
  }
  const double bs = tde_block_sum_d(lsum, sh);
  if (threadIdx.x == 0) atomicAdd(a.loss, bs * (double)a.weight / (double)total);
}

// grid-stride loss kernels end every block in fp64 atomics on one accumulator: a few hundred blocks, not
// thousands (the same contention measured on depth_pyramid_kernel)
int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 512 ? 512 : (b < 1 ? 1 : b));
}

// ------------------------------------------------------------------ fused multi-scale depth loss head
// One launch for every scale of train_depth_only.py:160-187 (and the per-scale smooth / depth-L1 terms
// of the other trainers): for scale s, compute_smooth_loss of pred_s (or 1/pred_s) and
// mean|nf(resize_area(label, s) - pred_s)|, values into two fp64 accumulators, gradients written (or
// added) into grad_s.  The area-downsampled label (train_depth_only.py:170) is formed on the fly from
// the full-resolution label (integer factor 2^s, same summation order as tde_resize_area_fwd).
struct PyrArgs {
  tde_depth_loss_t a;
  int bstart[TDE_MAX_SCALES + 1];   // first block of each scale (a block works on ONE scale, so the
                                    // per-scale parameters are indexed uniformly: scalar loads)
  float w1[TDE_MAX_SCALES], w23[TDE_MAX_SCALES], w4[TDE_MAX_SCALES];   // smooth weights / term counts
  double l1d[TDE_MAX_SCALES];       // depth-L1 weight / pixel count (value, fp64)
  float l1f[TDE_MAX_SCALES];        // the same rounded to float (gradient)
};

// Each pixel's smoothness value + gradient needs f on its 3x3 neighbourhood plus (i, j+-2) and (i+-2, j):
// those 13 values are loaded once into registers (clamped addresses; the edge tests below decide which
// terms exist) and every second difference is formed from them in the same fp32 order as t_dx2 / t_dxdy /
// t_dydx / t_dy2 (the same fp32 expressions as the per-term evaluation).  32-bit index math; the
// per-scale weights are precomputed on the host exactly as before (double, then rounded to float).
__device__ __forceinline__ void depth_pyramid_block(const PyrArgs& P, const int bid) {
  __shared__ double sh[4];
  const tde_depth_loss_t& a = P.a;
  double ls = 0.0, ll = 0.0;
  int s = 0;
  while (bid >= P.bstart[s + 1]) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  const int H = a.H >> s, W = a.W >> s;
  const int total = a.N * H * W;
  const int nb = P.bstart[s + 1] - P.bstart[s];
  const float* pr = a.pred[s];
  const int pcs = a.pred_cs[s], pco = a.pred_co[s];
  const bool smooth = a.smooth_w[s] != 0.f && H >= 3 && W >= 3;
  const float w1 = P.w1[s], w23 = P.w23[s], w4 = P.w4[s];
  for (int loc = (bid - P.bstart[s]) * 256 + threadIdx.x; loc < total; loc += nb * 256) {
    const int t = loc / W;
    const int j = loc - t * W;
    const int n = t / H, i = t - n * H;
    const int rowb = n * H;
    auto F = [&](int ii, int jj) __attribute__((always_inline)) {
      ii = min(max(ii, 0), H - 1);
      jj = min(max(jj, 0), W - 1);
      const float v = pr[((rowb + ii) * W + jj) * pcs + pco];
      return a.recip ? 1.f / v : v;
    };
    const float pv = pr[(loc)*pcs + pco];
    float gf = 0.f;
    if (smooth) {
      // f[r][c] = f(i + r - 1, j + c - 1) on the 3x3 block; fxm2/fxp2 = f(i, j-+2), fym2/fyp2 = f(i-+2, j)
      float f[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) f[r][c] = F(i + r - 1, j + c - 1);
      const float fxm2 = F(i, j - 2), fxp2 = F(i, j + 2), fym2 = F(i - 2, j), fyp2 = F(i + 2, j);
      // t_dx2(i, jj) = (f(i,jj+2) - f(i,jj+1)) - (f(i,jj+1) - f(i,jj))
      const float dx2_0 = (fxp2 - f[1][2]) - (f[1][2] - f[1][1]);         // jj = j
      const float dx2_m1 = (f[1][2] - f[1][1]) - (f[1][1] - f[1][0]);     // jj = j - 1
      const float dx2_m2 = (f[1][1] - f[1][0]) - (f[1][0] - fxm2);        // jj = j - 2
      const float dy2_0 = (fyp2 - f[2][1]) - (f[2][1] - f[1][1]);
      const float dy2_m1 = (f[2][1] - f[1][1]) - (f[1][1] - f[0][1]);
      const float dy2_m2 = (f[1][1] - f[0][1]) - (f[0][1] - fym2);
      // t_dxdy(a,b) = (f(a+1,b+1) - f(a+1,b)) - (f(a,b+1) - f(a,b)); t_dydx(a,b) = (f(a+1,b+1) - f(a,b+1)) - (f(a+1,b) - f(a,b))
#define DXDY(r, c) ((f[r + 1][c + 1] - f[r + 1][c]) - (f[r][c + 1] - f[r][c]))
#define DYDX(r, c) ((f[r + 1][c + 1] - f[r][c + 1]) - (f[r + 1][c] - f[r][c]))
      const float xy00 = DXDY(1, 1), yx00 = DYDX(1, 1);   // anchor (i, j)
      const float xy0m = DXDY(1, 0), yx0m = DYDX(1, 0);   // (i, j - 1)
      const float xym0 = DXDY(0, 1), yxm0 = DYDX(0, 1);   // (i - 1, j)
      const float xymm = DXDY(0, 0), yxmm = DYDX(0, 0);   // (i - 1, j - 1)
#undef DXDY
#undef DYDX
      float lv = 0.f;
      if (j < W - 2) lv += fabsf(dx2_0) * w1;
      if (i < H - 1 && j < W - 1) lv += (fabsf(xy00) + fabsf(yx00)) * w23;
      if (i < H - 2) lv += fabsf(dy2_0) * w4;
      ls += lv;
      if (j < W - 2) gf += tde_sign(dx2_0) * w1;
      if (j >= 1 && j - 1 < W - 2) gf -= 2.f * tde_sign(dx2_m1) * w1;
      if (j >= 2) gf += tde_sign(dx2_m2) * w1;
      if (i < H - 2) gf += tde_sign(dy2_0) * w4;
      if (i >= 1 && i - 1 < H - 2) gf -= 2.f * tde_sign(dy2_m1) * w4;
      if (i >= 2) gf += tde_sign(dy2_m2) * w4;
      if (i < H - 1 && j < W - 1) gf += (tde_sign(xy00) + tde_sign(yx00)) * w23;
      if (i < H - 1 && j >= 1) gf -= (tde_sign(xy0m) + tde_sign(yx0m)) * w23;
      if (i >= 1 && j < W - 1) gf -= (tde_sign(xym0) + tde_sign(yxm0)) * w23;
      if (i >= 1 && j >= 1) gf += (tde_sign(xymm) + tde_sign(yxmm)) * w23;
      if (a.recip) gf *= -1.f / (pv * pv);
    }
    if (a.l1_w[s] != 0.f) {
      const int fct = 1 << s;
      float lab;
      if (s == 0) {
        lab = a.label[(n * a.H + i) * a.W + j];
      } else {
        // the 2^s x 2^s box (<= 8 x 8): every load issued before the first add (a runtime-bounded loop
        // would serialise one L2 round trip per pixel), then summed in the u-major order of
        // tde_resize_area_fwd
        const float* lb = a.label + (n * a.H + i * fct) * a.W + j * fct;
        float box[8][8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int v = 0; v < 8; ++v) box[u][v] = (u < fct && v < fct) ? lb[u * a.W + v] : 0.f;
        float sum = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int v = 0; v < 8; ++v)
            if (u < fct && v < fct) sum += box[u][v];
        lab = sum * (1.f / (float)(fct * fct));
      }
      float d = lab - pv;
      if (a.nonfinite && !isfinite(d)) d = 0.f;   // replace_nonfinite: value and gradient masked
      ll += fabsf(d) * P.l1d[s];
      gf += -tde_sign(d) * P.l1f[s];
    }
    float* gp = a.grad[s] + loc * a.g_cs[s] + a.g_co[s];
    *gp = a.grad_accumulate ? *gp + gf : gf;
  }
  const double bs = tde_block_sum_d(ls, sh);
  __syncthreads();
  const double bl = tde_block_sum_d(ll, sh);
  if (threadIdx.x == 0) {
    if (a.loss_smooth) atomicAdd(a.loss_smooth, bs);
    if (a.loss_l1) atomicAdd(a.loss_l1, bl);
  }
}

__global__ void __launch_bounds__(256) depth_pyramid_kernel(const PyrArgs P) { depth_pyramid_block(P, blockIdx.x); }

// tde_loss_depth_pyramid_multi: map m owns blocks [mstart[m], mstart[m+1]) of the grid
struct PyrMulti {
  PyrArgs p[TDE_PYR_MULTI_MAX];
  int mstart[TDE_PYR_MULTI_MAX + 1];
  int n;
};

__global__ void __launch_bounds__(256) depth_pyramid_multi_kernel(const PyrMulti M) {
  int m = 0;
  while (m + 1 < M.n && (int)blockIdx.x >= M.mstart[m + 1]) ++m;
  depth_pyramid_block(M.p[m], (int)blockIdx.x - M.mstart[m]);
}

}  // namespace

extern "C" {

int tde_loss_smooth2(int N, int H, int W, const float* pred, int cstride, int coff, int recip, float weight,
                     double* loss, float* grad, int g_cstride, int g_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H >= 3 && W >= 3 && pred && loss && grad);
  Map f{pred, H, W, cstride, coff, recip};
  hipLaunchKernelGGL(smooth2_kernel, dim3(ew_grid((long)N * H * W)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     N, H, W, f, weight, loss, grad, g_cstride, g_coff);
  return tde_launch_status();
}

int tde_loss_l1(int N, int H, int W, const float* pred, int cstride, int coff, const float* label, int nonfinite,
                float weight, double* loss, float* grad, int g_cstride, int g_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && pred && label && loss && grad);
  const long total = (long)N * H * W;
  hipLaunchKernelGGL(l1_kernel, dim3(ew_grid(total)), dim3(256), 0, static_cast<hipStream_t>(stream), total, pred,
                     cstride, coff, label, nonfinite, weight, loss, grad, g_cstride, g_coff);
  return tde_launch_status();
}

int tde_loss_sig_l2(int N, int H, int W, const float* pred, int cstride, int coff, const float* label, int ndeltas,
                    const int* deltas, const float* weights, float sig_epsilon, float epsilon, float weight,
                    double* loss, float* grad, int g_cstride, int g_coff, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(N > 0 && H > 0 && W > 0 && pred && label && loss && grad && ndeltas >= 1 && ndeltas <= SIG_MAXD &&
                deltas && weights && cstride > coff && g_cstride > g_coff);
  SigArgs a{};
  a.N = N; a.H = H; a.W = W; a.nd = ndeltas;
  for (int k = 0; k < ndeltas; ++k) {
    TDE_CHECK_ARG(deltas[k] >= 1);
    a.delta[k] = deltas[k];
    a.wt[k] = weights[k];
  }
  a.seps = sig_epsilon; a.l2eps = epsilon; a.weight = weight;
  a.pred = pred; a.cs = cstride; a.co = coff; a.label = label; a.loss = loss;
  a.g = grad; a.gcs = g_cstride; a.gco = g_coff;
  hipLaunchKernelGGL(sig_l2_kernel, dim3(ew_grid((long)N * H * W)), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return tde_launch_status();
}

// blocks per scale at most: every block ends in two fp64 atomics on the same two accumulators, and the
// full-resolution scale's blocks each walk (scale pixels / cap) pixels (rocprofv3, config 2: 4096 -> 61 us,
// 512 -> 38 us, 128 -> 30 us per step; round 2 re-sweep, scripts/r02s7_pyrmaxb.sh: 128 / 160 / 192 / 224 ->
// 30.3 / 23.1 / 21.8 / 22.9 us (config 2), 28.4 / 23.5 / 20.9 / 19.9 us (config 4))
// (TDE_PYR_MAXB tuning knob; a missing, non-numeric or non-positive value means the default)
static const long g_pyr_maxb = tde_env_pos("TDE_PYR_MAXB", 192);

// host-side setup of one map's launch arguments (argument checks, per-scale block ranges and weights)
static int pyr_setup(const tde_depth_loss_t* a, PyrArgs& P) {
  TDE_CHECK_ARG(a && a->N > 0 && a->H > 0 && a->W > 0 && a->nscales >= 1 && a->nscales <= TDE_MAX_SCALES);
  P.a = *a;
  P.bstart[0] = 0;
  for (int s = 0; s < a->nscales; ++s) {
    TDE_CHECK_ARG(a->pred[s] && a->grad[s] && (a->H >> s) > 0 && (a->W >> s) > 0);
    TDE_CHECK_ARG(a->l1_w[s] == 0.f || (a->label && a->H % (1 << s) == 0 && a->W % (1 << s) == 0));
    // compute_smooth_loss takes reduce_mean over dx2 / dy2, which are empty below 3 rows / columns (the
    // reference's value is NaN there): same contract as tde_loss_smooth2
    TDE_CHECK_ARG(a->smooth_w[s] == 0.f || ((a->H >> s) >= 3 && (a->W >> s) >= 3));
    // the kernel's element offsets loc * cs + co assume 0 <= co < cs for every view
    TDE_CHECK_ARG(a->pred_co[s] >= 0 && a->pred_co[s] < a->pred_cs[s] && a->g_co[s] >= 0 && a->g_co[s] < a->g_cs[s]);
    long nbk = ew_grid((long)a->N * (a->H >> s) * (a->W >> s));
    nbk = nbk > g_pyr_maxb ? g_pyr_maxb : (nbk < 1 ? 1 : nbk);
    P.bstart[s + 1] = P.bstart[s] + (int)nbk;
  }
  for (int s = a->nscales; s < TDE_MAX_SCALES; ++s) P.bstart[s + 1] = P.bstart[s];
  long cs = 1;
  for (int s = 0; s < a->nscales; ++s) cs = a->pred_cs[s] > cs ? a->pred_cs[s] : cs;
  for (int s = 0; s < a->nscales; ++s) cs = a->g_cs[s] > cs ? a->g_cs[s] : cs;
  TDE_CHECK_ARG((long)a->N * a->H * a->W * cs < 0x7fffffffL);   // 32-bit pixel / element indices
  for (int s = 0; s < TDE_MAX_SCALES; ++s) {
    const int H = a->H >> s, W = a->W >> s;
    const double n1 = (double)a->N * H * (W - 2), n23 = (double)a->N * (H - 1) * (W - 1),
                 n4 = (double)a->N * (H - 2) * W, tot = (double)a->N * H * W;
    const bool on = s < a->nscales;
    P.w1[s] = on ? (float)(a->smooth_w[s] / n1) : 0.f;
    P.w23[s] = on ? (float)(a->smooth_w[s] / n23) : 0.f;
    P.w4[s] = on ? (float)(a->smooth_w[s] / n4) : 0.f;
    P.l1d[s] = on ? (double)a->l1_w[s] / tot : 0.0;
    P.l1f[s] = on ? (float)(a->l1_w[s] / tot) : 0.f;
  }
  return TDE_OK;
}

int tde_loss_depth_pyramid(const tde_depth_loss_t* a, void* stream) {
  tde_clear_error();
  PyrArgs P;
  const int rc = pyr_setup(a, P);
  if (rc != TDE_OK) return rc;
  hipLaunchKernelGGL(depth_pyramid_kernel, dim3(P.bstart[a->nscales]), dim3(256), 0,
                     static_cast<hipStream_t>(stream), P);
  return tde_launch_status();
}

int tde_loss_depth_pyramid_multi(const tde_depth_loss_t* args, int n, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(args && n > 0 && n <= TDE_PYR_MULTI_MAX);
  PyrMulti M;
  M.n = n;
  M.mstart[0] = 0;
  for (int m = 0; m < n; ++m) {
    const int rc = pyr_setup(args + m, M.p[m]);
    if (rc != TDE_OK) return rc;
    M.mstart[m + 1] = M.mstart[m] + M.p[m].bstart[args[m].nscales];
  }
  hipLaunchKernelGGL(depth_pyramid_multi_kernel, dim3(M.mstart[n]), dim3(256), 0, static_cast<hipStream_t>(stream),
                     M);
  return tde_launch_status();
}

}  // extern "C"
