// Fused self-supervised loss head: projective inverse warp + TF bilinear sampler + photometric /
// explainability / left-right consistency terms, forward value AND hand-derived backward in one pass
// (SURVEY.md §8a rows a10-a17, a21, a22).  Reference: utils_lr.py:106-366 (pose_vec2mat, pixel2cam,
// cam2pixel, projective_inverse_warp, bilinear_sampler), utils_lr.py:369-458 (consistent_depth_loss),
// utils_lr.py:258-274/472-489 (optflow_warp, depth_optflow), train_depth_then_cam_lr.py:253-340
// (per-scale loss assembly), train_optflow_combine.py:169-210, refine_depth.py:200-213.
//
// One thread per target pixel (grid.y = batch element); HBM-bound: it reads the target disparity
// (or flow), two RGB images and the 2 logits, gathers 4 taps of the source image (and of the other
// view's disparity), and writes the gradients of the disparity / flow / logits in place.  Only the
// consistency term scatters (into the other view's disparity gradient, 4 float atomics per pixel);
// d(loss)/d(projection matrix) is reduced per block in fp64 and added with 12 atomics per block.
#include "tde_common.h"

#include <algorithm>

namespace {

struct Tap4 {
  int x0, x1, y0, y1;        // clamped indices
  float wx0, wx1, wy0, wy1;  // masked weights (utils_lr.py:324-327)
  float mx0, mx1, my0, my1;  // in-range masks (= d wx1/du, -d wx0/du)
};

__device__ __forceinline__ Tap4 taps(float u, float v, int W, int H) {
  Tap4 t;
  const float fx0 = floorf(u), fy0 = floorf(v);
  const float fx1 = fx0 + 1.f, fy1 = fy0 + 1.f;
  const float xmax = (float)(W - 1), ymax = (float)(H - 1);
  const float cx0 = fminf(fmaxf(fx0, 0.f), xmax), cx1 = fminf(fmaxf(fx1, 0.f), xmax);
  const float cy0 = fminf(fmaxf(fy0, 0.f), ymax), cy1 = fminf(fmaxf(fy1, 0.f), ymax);
  t.mx0 = (fx0 == cx0) ? 1.f : 0.f;
  t.mx1 = (fx1 == cx1) ? 1.f : 0.f;
  t.my0 = (fy0 == cy0) ? 1.f : 0.f;
  t.my1 = (fy1 == cy1) ? 1.f : 0.f;
  t.wx0 = (fx1 - u) * t.mx0;
  t.wx1 = (u - fx0) * t.mx1;
  t.wy0 = (fy1 - v) * t.my0;
  t.wy1 = (v - fy0) * t.my1;
  t.x0 = (int)cx0; t.x1 = (int)cx1; t.y0 = (int)cy0; t.y1 = (int)cy1;
  return t;
}

// Deterministic mode (tde_warp_loss_t.det_ws != NULL): the consistency term's gather gradient is scattered as
// 64-bit fixed-point integers (integer addition is associative: the sum is the same in any order), scaled so
// that no destination can overflow: |sum| <= H*W * bound, bound = consist_w/(B*H*W) * max(1/disp_other)^2
// (warp_det_prep_kernel), scale = 2^(62 - ceil(log2(H*W*bound))); warp_det_finish_kernel adds the sums into
// g_other once.  The loss parts and dL/dP leave each block as partial rows reduced in block order (no fp64
// atomics).  Layout of det_ws: [B*H*W] int64 scatter sums | [blocks][15] fp64 partials | 4 B bound slot.
struct WarpDet {
  long long* acc;      // [B*H*W] fixed-point scatter sums (zeroed by the prep kernel)
  double* part;        // [gridDim.x * B][15]
  unsigned* bound;     // max over the other view of (1/disp)^2, float bits (atomicMax: order-independent)
};

__device__ __forceinline__ double det_scale(const tde_warp_loss_t& a, const WarpDet& d) {
  const double mo2 = (double)__uint_as_float(*d.bound);
  const double hw = (double)a.H * a.W;
  const double lim = hw * (double)a.consist_w / ((double)a.B * hw) * mo2;
  if (!(lim > 0.0) || !isfinite(lim)) return 1.0;
  int e;
  frexp(lim, &e);                         // lim < 2^e
  return ldexp(1.0, 62 - e);
}

// One block of one call: block bx of gdx along the pixels of batch element b.
template <bool NEED_G_P, bool DET>
__device__ __forceinline__ void warp_loss_block(const tde_warp_loss_t& a, const WarpDet& det, const int bx,
                                                const int b, const int gdx) {
  __shared__ double sh[16][4];
  const int HW = a.H * a.W;
  // per-thread fp64 accumulators over a grid-stride loop: a capped grid (tde_warp_loss) keeps the
  // block-end fp64 atomics on the shared loss / dL/dP words few
  double l_photo = 0, l_exp = 0, l_cons = 0;
  double gp[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) gp[i] = 0.0;
  const double inv_n3 = 1.0 / (3.0 * a.B * HW), inv_n = 1.0 / ((double)a.B * HW);
  const double dscale = DET ? det_scale(a, det) : 0.0;
  for (int idx = bx * blockDim.x + threadIdx.x; idx < HW; idx += gdx * blockDim.x) {
    const int y = idx / a.W, x = idx - y * a.W;
    const long pix = (long)b * HW + idx;
    // ---- coordinates (cam2pixel of pixel2cam) or grid + flow
    float u, v, z = 0.f, disp = 0.f, dep = 0.f, cam[3] = {0, 0, 0};
    const float* Pb = a.P + 12 * b;
    const float xf = (float)x, yf = (float)y;   // meshgrid gives integer pixel centres (utils_lr.py:212-213)
    if (a.disp) {
      disp = a.disp[pix * a.disp_cs + a.disp_co];
      dep = 1.f / disp;
      const float* Ki = a.Kinv + 9 * b;
#pragma unroll
      for (int i = 0; i < 3; ++i) cam[i] = (Ki[3 * i] * xf + Ki[3 * i + 1] * yf + Ki[3 * i + 2]) * dep;
      const float p0 = Pb[0] * cam[0] + Pb[1] * cam[1] + Pb[2] * cam[2] + Pb[3];
      const float p1 = Pb[4] * cam[0] + Pb[5] * cam[1] + Pb[6] * cam[2] + Pb[7];
      const float p2 = Pb[8] * cam[0] + Pb[9] * cam[1] + Pb[10] * cam[2] + Pb[11];
      z = p2;
      u = p0 / (p2 + 1e-10f);
      v = p1 / (p2 + 1e-10f);
    } else {
      const float* f = a.flow + pix * a.flow_cs + a.flow_co;
      u = xf + f[0];
      v = yf + f[1];
    }
    // ---- photometric: bilinear sample of the source image
    const Tap4 t = taps(u, v, a.W, a.H);
    const float* S = a.img_src + (long)b * HW * 3;
    const float* s00 = S + ((long)t.y0 * a.W + t.x0) * 3;
    const float* s01 = S + ((long)t.y1 * a.W + t.x0) * 3;
    const float* s10 = S + ((long)t.y0 * a.W + t.x1) * 3;
    const float* s11 = S + ((long)t.y1 * a.W + t.x1) * 3;
    const float w00 = t.wx0 * t.wy0, w01 = t.wx0 * t.wy1, w10 = t.wx1 * t.wy0, w11 = t.wx1 * t.wy1;
    const float* T = a.img_tgt + pix * 3;
    float err[3], sw[3];
    float esum = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      sw[c] = w00 * s00[c] + w01 * s01[c] + w10 * s10[c] + w11 * s11[c];
      err[c] = sw[c] - T[c];
      esum += fabsf(err[c]);
    }
    // ---- per-pixel photometric weight: softmax(logits)[1] (exp mask), wmask, or 1
    float wpix = 1.f, p1 = 1.f, l0 = 0.f, l1 = 0.f;
    if (a.logits) {
      const float* L = a.logits + pix * a.logit_cs + a.logit_co;
      l0 = L[0]; l1 = L[1];
      const float m = fmaxf(l0, l1);
      const float e0 = __expf(l0 - m), e1 = __expf(l1 - m);
      p1 = e1 / (e0 + e1);
      wpix = p1;
      // softmax_cross_entropy_with_logits, label [0,1] (get_reference_explain_mask, :76-85)
      l_exp += (double)(-(l1 - m) + logf(e0 + e1)) * a.exp_w * inv_n;
    } else if (a.wmask) {
      wpix = a.wmask[pix];
    }
    l_photo += (double)esum * wpix * a.photo_w * inv_n3;
    // ---- left-right consistency: |z - bilinear(1/disp_other)(u,v)| * p1 (utils_lr.py:369-458)
    float g_z = 0.f, g_o = 0.f, cons = 0.f, o = 0.f;
    const float* Do = a.disp_other ? a.disp_other + (long)b * HW * a.other_cs + a.other_co : nullptr;
    float o00 = 0, o01 = 0, o10 = 0, o11 = 0;
    if (Do) {
      o00 = 1.f / Do[((long)t.y0 * a.W + t.x0) * a.other_cs];
      o01 = 1.f / Do[((long)t.y1 * a.W + t.x0) * a.other_cs];
      o10 = 1.f / Do[((long)t.y0 * a.W + t.x1) * a.other_cs];
      o11 = 1.f / Do[((long)t.y1 * a.W + t.x1) * a.other_cs];
      o = w00 * o00 + w01 * o01 + w10 * o10 + w11 * o11;
      const float dzo = z - o;
      cons = fabsf(dzo);
      l_cons += (double)cons * p1 * a.consist_w * inv_n;
      const float gc = (float)(a.consist_w * inv_n) * p1 * tde_sign(dzo);
      g_z = gc;
      g_o = -gc;
    }
    // ---- backward: logits
    if (a.logits && a.g_logits) {
      const float Scoef = (float)(a.photo_w * inv_n3) * esum + (float)(a.consist_w * inv_n) * cons;
      const float q = p1 * (1.f - p1);
      const float gl1 = Scoef * q - (float)(a.exp_w * inv_n) * (1.f - p1);
      float* G = a.g_logits + pix * a.logit_cs + a.logit_co;
      G[0] += -gl1;
      G[1] += gl1;
    }
    // d/d sampled value (photometric), then d/d(u,v)
    const float gph = (float)(a.photo_w * inv_n3) * wpix;
    float gu = 0.f, gv = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float gs = gph * tde_sign(err[c]);
      // d sample / du = -mx0*(wy0*s00 + wy1*s01) + mx1*(wy0*s10 + wy1*s11)
      gu += gs * (-t.mx0 * (t.wy0 * s00[c] + t.wy1 * s01[c]) + t.mx1 * (t.wy0 * s10[c] + t.wy1 * s11[c]));
      gv += gs * (-t.my0 * (t.wx0 * s00[c] + t.wx1 * s10[c]) + t.my1 * (t.wx0 * s01[c] + t.wx1 * s11[c]));
    }
    if (Do) {
      gu += g_o * (-t.mx0 * (t.wy0 * o00 + t.wy1 * o01) + t.mx1 * (t.wy0 * o10 + t.wy1 * o11));
      gv += g_o * (-t.my0 * (t.wx0 * o00 + t.wx1 * o10) + t.my1 * (t.wx0 * o01 + t.wx1 * o11));
      if (a.g_other) {   // gather gradient -> scatter-add into the other view's disparity (d(1/d) = -1/d^2)
        float* Go = a.g_other + (long)b * HW * a.other_cs + a.other_co;
        const float* Dd = Do;
        const long i00 = ((long)t.y0 * a.W + t.x0) * a.other_cs, i01 = ((long)t.y1 * a.W + t.x0) * a.other_cs;
        const long i10 = ((long)t.y0 * a.W + t.x1) * a.other_cs, i11 = ((long)t.y1 * a.W + t.x1) * a.other_cs;
        if (DET) {
          // fixed-point integer scatter into det.acc (dense [B*H*W], one value per pixel of the other view)
          unsigned long long* A = reinterpret_cast<unsigned long long*>(det.acc) + (long)b * HW;
          const long j00 = (long)t.y0 * a.W + t.x0, j01 = (long)t.y1 * a.W + t.x0;
          const long j10 = (long)t.y0 * a.W + t.x1, j11 = (long)t.y1 * a.W + t.x1;
          if (w00 != 0.f) atomicAdd(A + j00, (unsigned long long)llrint((double)(-g_o * w00 * o00 * o00) * dscale));
          if (w01 != 0.f) atomicAdd(A + j01, (unsigned long long)llrint((double)(-g_o * w01 * o01 * o01) * dscale));
          if (w10 != 0.f) atomicAdd(A + j10, (unsigned long long)llrint((double)(-g_o * w10 * o10 * o10) * dscale));
          if (w11 != 0.f) atomicAdd(A + j11, (unsigned long long)llrint((double)(-g_o * w11 * o11 * o11) * dscale));
        } else {
          if (w00 != 0.f) atomicAdd(Go + i00, -g_o * w00 * o00 * o00);
          if (w01 != 0.f) atomicAdd(Go + i01, -g_o * w01 * o01 * o01);
          if (w10 != 0.f) atomicAdd(Go + i10, -g_o * w10 * o10 * o10);
          if (w11 != 0.f) atomicAdd(Go + i11, -g_o * w11 * o11 * o11);
        }
        (void)Dd;
      }
    }
    if (a.disp) {
      // (u, v, z) <- p = P[:, :3] cam + P[:, 3]
      const float den = Pb[8] * cam[0] + Pb[9] * cam[1] + Pb[10] * cam[2] + Pb[11] + 1e-10f;
      const float p0 = Pb[0] * cam[0] + Pb[1] * cam[1] + Pb[2] * cam[2] + Pb[3];
      const float p1v = Pb[4] * cam[0] + Pb[5] * cam[1] + Pb[6] * cam[2] + Pb[7];
      const float gp0 = gu / den, gp1 = gv / den;
      const float gp2 = -(gu * p0 + gv * p1v) / (den * den) + g_z;
      const float gcam0 = Pb[0] * gp0 + Pb[4] * gp1 + Pb[8] * gp2;
      const float gcam1 = Pb[1] * gp0 + Pb[5] * gp1 + Pb[9] * gp2;
      const float gcam2 = Pb[2] * gp0 + Pb[6] * gp1 + Pb[10] * gp2;
      if (NEED_G_P) {
        const float gps[3] = {gp0, gp1, gp2};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          gp[4 * i + 0] += gps[i] * cam[0];
          gp[4 * i + 1] += gps[i] * cam[1];
          gp[4 * i + 2] += gps[i] * cam[2];
          gp[4 * i + 3] += gps[i];
        }
      }
      // cam = dep * Kinv [x y 1]  ->  d dep = gcam . (cam / dep);  disp = 1/dep -> d disp = -d dep / disp^2
      const float gdep = (gcam0 * cam[0] + gcam1 * cam[1] + gcam2 * cam[2]) / dep;
      if (a.g_disp) a.g_disp[pix * a.disp_cs + a.disp_co] += -gdep / (disp * disp);
    } else if (a.g_flow) {
      float* G = a.g_flow + pix * a.flow_cs + a.flow_co;
      G[0] += gu;
      G[1] += gv;
    }
  }
  // ---- block reductions (loss parts; dL/dP)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double vals[15] = {l_photo, l_exp, l_cons};
#pragma unroll
  for (int i = 0; i < 12; ++i) vals[3 + i] = NEED_G_P ? gp[i] : 0.0;
  const int nv = NEED_G_P ? 15 : 3;
  for (int i = 0; i < nv; ++i) {
    double vv = vals[i];
    for (int off = 32; off > 0; off >>= 1) vv += __shfl_down(vv, off, 64);
    if (lane == 0) sh[i][wid] = vv;
  }
  __syncthreads();
  if (threadIdx.x < nv) {
    const int i = threadIdx.x;
    const double s = sh[i][0] + sh[i][1] + sh[i][2] + sh[i][3];
    if (DET) {
      det.part[((long)b * gdx + bx) * 15 + i] = s;
    } else if (i < 3) {
      if (s != 0.0) atomicAdd(a.loss + i, s);
    } else {
      atomicAdd(a.g_P + 12 * b + (i - 3), s);
    }
  }
}

template <bool NEED_G_P, bool DET>
__global__ void __launch_bounds__(256) warp_loss_kernel(const tde_warp_loss_t a, const WarpDet det) {
  warp_loss_block<NEED_G_P, DET>(a, det, blockIdx.x, blockIdx.y, gridDim.x);
}

// Several calls in ONE launch (tde_warp_loss_multi): call c owns blocks [start[c], start[c+1]) of a 1-D grid, gx[c]
// per batch element.  The calls' gradient outputs must be disjoint (float += without atomics on g_disp / g_logits).
struct WarpMulti {
  tde_warp_loss_t a[TDE_WARP_MULTI_MAX];
  int start[TDE_WARP_MULTI_MAX + 1];
  int gx[TDE_WARP_MULTI_MAX];
  int n;
};

template <bool NEED_G_P>
__global__ void __launch_bounds__(256) warp_loss_multi_kernel(const WarpMulti m) {
  const int id = blockIdx.x;
  int c = 0;
  while (c + 1 < m.n && id >= m.start[c + 1]) ++c;
  const int local = id - m.start[c], gx = m.gx[c];
  const WarpDet none{nullptr, nullptr, nullptr};
  warp_loss_block<NEED_G_P, false>(m.a[c], none, local % gx, local / gx, gx);
}

// Deterministic mode, before the loss kernel: zero the fixed-point sums and raise the bound slot to
// max (1/disp_other)^2 (atomicMax on the float bits of non-negative values: order-independent).
__global__ void __launch_bounds__(256) warp_det_prep_kernel(const tde_warp_loss_t a, const WarpDet det, long n) {
  float m = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += 256L * gridDim.x) {
    det.acc[i] = 0;
    if (a.disp_other) {
      const float o = 1.f / a.disp_other[i * a.other_cs + a.other_co];
      m = fmaxf(m, o * o);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(det.bound, __float_as_uint(m));
}

// Deterministic mode, after the loss kernel: g_other += fixed-point sums / scale (one add per pixel), and the
// last block sums the per-block partials of the loss parts and dL/dP in block order.
__global__ void __launch_bounds__(256) warp_det_finish_kernel(const tde_warp_loss_t a, const WarpDet det, long n,
                                                              int gx, int nv) {
  if (blockIdx.x == gridDim.x - 1) {
    // loss parts (3) and dL/dP (12 per batch element), fixed order over blocks
    for (int i = threadIdx.x; i < 3 + 12 * a.B; i += 256) {
      if (i < 3) {
        double s = 0.0;
        for (int bb = 0; bb < a.B; ++bb)
          for (int x = 0; x < gx; ++x) s += det.part[((long)bb * gx + x) * 15 + i];
        if (s != 0.0) a.loss[i] += s;
      } else if (nv == 15) {
        const int bb = (i - 3) / 12, k = (i - 3) % 12;
        double s = 0.0;
        for (int x = 0; x < gx; ++x) s += det.part[((long)bb * gx + x) * 15 + 3 + k];
        a.g_P[12 * bb + k] += s;
      }
    }
    return;
  }
  if (!a.g_other) return;
  const double inv = 1.0 / det_scale(a, det);
  const int HW = a.H * a.W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += 256L * (gridDim.x - 1)) {
    const long b = i / HW, idx = i - b * HW;
    float* g = a.g_other + (b * HW + idx) * a.other_cs + a.other_co;
    *g += (float)((double)det.acc[i] * inv);
  }
}

// ------------------------------------------------------------------ pose / intrinsics (per batch element)
__device__ void rodrigues(const float* r, float R[9]) {
  // utils_lr.py:106-134 + axis_angle_to_rotation_matrix :77-103; NaN at r = 0 like the reference
  const float th = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  const float a0 = r[0] / th, a1 = r[1] / th, a2 = r[2] / th;
  const float Kx[9] = {0.f, -a2, a1, a2, 0.f, -a0, -a1, a0, 0.f};
  const float s = sinf(th), c1 = 1.f - cosf(th);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float kk = 0.f;
      for (int m = 0; m < 3; ++m) kk += Kx[3 * i + m] * Kx[3 * m + j];
      R[3 * i + j] = (i == j ? 1.f : 0.f) + s * Kx[3 * i + j] + c1 * kk;
    }
}

__device__ void inv3(const float* K, float* Ki) {
  const float a = K[0], b = K[1], c = K[2], d = K[3], e = K[4], f = K[5], g = K[6], h = K[7], i = K[8];
  const float A = e * i - f * h, Bc = -(d * i - f * g), C = d * h - e * g;
  const float det = a * A + b * Bc + c * C;
  const float id = 1.f / det;
  Ki[0] = A * id; Ki[1] = -(b * i - c * h) * id; Ki[2] = (b * f - c * e) * id;
  Ki[3] = Bc * id; Ki[4] = (a * i - c * g) * id; Ki[5] = -(a * f - c * d) * id;
  Ki[6] = C * id; Ki[7] = -(a * h - b * g) * id; Ki[8] = (a * e - b * d) * id;
}

__device__ __forceinline__ void pose_prep_one(int b, const float* vec, const float* mat, const float* K, float* T,
                                              float* P, float* Kinv) {
  float Tm[16];
  if (vec) {
    float R[9];
    rodrigues(vec + 6 * b + 3, R);
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) Tm[4 * i + j] = R[3 * i + j];
      Tm[4 * i + 3] = vec[6 * b + i];
    }
    Tm[12] = 0.f; Tm[13] = 0.f; Tm[14] = 0.f; Tm[15] = 1.f;
  } else {
    for (int i = 0; i < 16; ++i) Tm[i] = mat[16 * b + i];
  }
  const float* Kb = K + 9 * b;
  if (T) for (int i = 0; i < 16; ++i) T[16 * b + i] = Tm[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j)
      P[12 * b + 4 * i + j] = Kb[3 * i] * Tm[j] + Kb[3 * i + 1] * Tm[4 + j] + Kb[3 * i + 2] * Tm[8 + j];
  inv3(Kb, Kinv + 9 * b);
}

__global__ void pose_prep_kernel(int B, const float* vec, const float* mat, const float* K, float* T, float* P,
                                 float* Kinv) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) pose_prep_one(b, vec, mat, K, T, P, Kinv);
}

// tde_pose_prep_multi: job blockIdx.y of up to TDE_WARP_MULTI_MAX independent tde_pose_prep calls
struct PoseMulti {
  tde_pose_prep_t j[TDE_WARP_MULTI_MAX];
};

__global__ void pose_prep_multi_kernel(const PoseMulti m) {
  const tde_pose_prep_t& j = m.j[blockIdx.y];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < j.B) pose_prep_one(b, j.pose_vec, j.pose_mat, j.K, j.T, j.P, j.Kinv);
}

// dL/dvec from dL/dP (all scales summed: gP[s][b][12], K_s at Ks + b*k_stride_b + 9*s) and an
// optional extra dL/dT [B][16] (cam loss).  Rodrigues backward (utils_lr.py:77-103,126-134).
__device__ void pose_grad_one(int b, int B, int nscales, const float* vec, const float* Ks, long k_stride_b,
                              const double* gP, const float* gT_extra, float* out);

__global__ void pose_grad_kernel(int B, int nscales, const float* vec, const float* Ks, long k_stride_b,
                                 const double* gP, const float* gT_extra, float* gvec, int accumulate) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float out[6];
  pose_grad_one(b, B, nscales, vec, Ks, k_stride_b, gP, gT_extra, out);
  for (int i = 0; i < 6; ++i) gvec[6 * b + i] = accumulate ? gvec[6 * b + i] + out[i] : out[i];
}

// tde_pose_grad_spread: job blockIdx.y; the pose gradient, then its spatial-mean backward into the pose map
struct PoseGradMulti {
  tde_pose_grad_t j[TDE_WARP_MULTI_MAX];
};

__global__ void pose_grad_spread_kernel(const PoseGradMulti m) {
  const tde_pose_grad_t& j = m.j[blockIdx.y];
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= j.B) return;
  float out[6];
  pose_grad_one(b, j.B, j.nscales, j.pose_vec, j.K, j.k_stride_b, j.gP, j.gT_extra, out);
  float g[6];
  for (int i = 0; i < 6; ++i) {
    g[i] = j.accumulate ? j.g_pose_vec[6 * b + i] + out[i] : out[i];
    j.g_pose_vec[6 * b + i] = g[i];
  }
  if (j.dpose) {   // pose_avg = reduce_mean(pose_pred, [1, 2]) backward (tde_spatial_mean_bwd's expression)
    for (int p = 0; p < j.hw; ++p) {
      float* o = j.dpose + ((long)b * j.hw + p) * j.dpose_cstride;
      for (int c = 0; c < 6; ++c) {
        const float v = g[c] / (float)j.hw;
        o[c] = j.dpose_accumulate ? o[c] + v : v;
      }
    }
  }
}

__device__ void pose_grad_one(int b, int B, int nscales, const float* vec, const float* Ks, long k_stride_b,
                              const double* gP, const float* gT_extra, float* out) {
  double G[12];  // dL/dT rows 0..2
  for (int i = 0; i < 12; ++i) G[i] = gT_extra ? gT_extra[16 * b + i] : 0.0;
  for (int s = 0; s < nscales; ++s) {
    const float* Kb = Ks + b * k_stride_b + 9 * s;
    const double* g = gP + ((long)s * B + b) * 12;   // layout [scale][B][12]
    // P = K @ T[0:3]  ->  dT[k][j] += sum_i K[i][k] dP[i][j]
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 4; ++j) G[4 * k + j] += Kb[k] * g[j] + Kb[3 + k] * g[4 + j] + Kb[6 + k] * g[8 + j];
  }
  const float* r = vec + 6 * b + 3;
  const double th = sqrt((double)r[0] * r[0] + (double)r[1] * r[1] + (double)r[2] * r[2]);
  const double a[3] = {r[0] / th, r[1] / th, r[2] / th};
  const double Kx[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
  const double s = sin(th), c = cos(th);
  double GR[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) GR[3 * i + j] = G[4 * i + j];
  // R = I + s K + (1-c) K^2
  double dS = 0, dC = 0, KK[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double kk = 0;
      for (int m = 0; m < 3; ++m) kk += Kx[3 * i + m] * Kx[3 * m + j];
      KK[3 * i + j] = kk;
    }
  for (int i = 0; i < 9; ++i) { dS += GR[i] * Kx[i]; dC -= GR[i] * KK[i]; }
  // dL/dK = s*GR + (1-c)*(GR K^T + K^T GR)
  double dK[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double t1 = 0, t2 = 0;
      for (int m = 0; m < 3; ++m) {
        t1 += GR[3 * i + m] * Kx[3 * j + m];   // GR K^T
        t2 += Kx[3 * m + i] * GR[3 * m + j];   // K^T GR
      }
      dK[3 * i + j] = s * GR[3 * i + j] + (1 - c) * (t1 + t2);
    }
  const double da[3] = {dK[7] - dK[5], dK[2] - dK[6], dK[3] - dK[1]};
  // dS = dL/ds, dC = dL/dc (c enters as 1-c); ds/dth = c, dc/dth = -s
  const double dth_total = dS * c - dC * s;
  const double ada = a[0] * da[0] + a[1] * da[1] + a[2] * da[2];
  for (int i = 0; i < 3; ++i) out[i] = (float)G[4 * i + 3];
  for (int i = 0; i < 3; ++i) out[3 + i] = (float)((da[i] - a[i] * ada) / th + dth_total * a[i]);
}

// Config 4 cam loss (train_depth_then_cam_lr.py:278-286):
//   w*mean((T_gt - T_lr)^2) + w*mean((inv(T_gt) - T_rl)^2), T_gt = pose_vec2mat(gt, angleaxis)
__global__ void cam_loss_kernel(int B, const float* gt_vec, const float* T_lr, const float* T_rl, float w,
                                double* loss, float* gT_lr, float* gT_rl) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float R[9];
  rodrigues(gt_vec + 6 * b + 3, R);
  float Tg[16], Ti[16];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Tg[4 * i + j] = R[3 * i + j];
    Tg[4 * i + 3] = gt_vec[6 * b + i];
  }
  Tg[12] = Tg[13] = Tg[14] = 0.f; Tg[15] = 1.f;
  // inverse of a rigid transform [R t; 0 1] = [R^T, -R^T t; 0 1] (tf.matrix_inverse of the same matrix)
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Ti[4 * i + j] = R[3 * j + i];
    Ti[4 * i + 3] = -(R[i] * Tg[3] + R[3 + i] * Tg[7] + R[6 + i] * Tg[11]);
  }
  Ti[12] = Ti[13] = Ti[14] = 0.f; Ti[15] = 1.f;
  const double inv = 1.0 / (16.0 * B);
  double l = 0;
  for (int i = 0; i < 16; ++i) {
    const float d1 = Tg[i] - T_lr[16 * b + i], d2 = Ti[i] - T_rl[16 * b + i];
    l += (double)d1 * d1 + (double)d2 * d2;
    gT_lr[16 * b + i] += (float)(-2.0 * w * inv * d1);
    gT_rl[16 * b + i] += (float)(-2.0 * w * inv * d2);
  }
  atomicAdd(loss, l * w * inv);
}

// Forward-only projective_inverse_warp (utils_lr.py:222-256) / bilinear_sampler (:276-366).
// coords from depth (or 1/disp) via P, Kinv; or, with depth == NULL, given coords [B,H,W,2].
__global__ void __launch_bounds__(256) warp_fwd_kernel(int B, int H, int W, int C, const float* depth, int is_disp,
                                                      const float* P, const float* Kinv, const float* coords_in,
                                                      const float* img, int Hs, int Ws, float* out, float* coords,
                                                      float* flow_x, float* flow_y, float* wmask, float* zout) {
  const int b = blockIdx.y;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (idx >= HW) return;
  const long pix = (long)b * HW + idx;
  const int y = idx / W, x = idx - y * W;
  float u, v, z = 0.f;
  if (depth) {
    const float dv = depth[pix];
    const float dep = is_disp ? 1.f / dv : dv;
    const float* Ki = Kinv + 9 * b;
    const float* Pb = P + 12 * b;
    float cam[3];
    for (int i = 0; i < 3; ++i) cam[i] = (Ki[3 * i] * x + Ki[3 * i + 1] * y + Ki[3 * i + 2]) * dep;
    const float p0 = Pb[0] * cam[0] + Pb[1] * cam[1] + Pb[2] * cam[2] + Pb[3];
    const float p1 = Pb[4] * cam[0] + Pb[5] * cam[1] + Pb[6] * cam[2] + Pb[7];
    const float p2 = Pb[8] * cam[0] + Pb[9] * cam[1] + Pb[10] * cam[2] + Pb[11];
    z = p2;
    u = p0 / (p2 + 1e-10f);
    v = p1 / (p2 + 1e-10f);
  } else {
    u = coords_in[2 * pix];
    v = coords_in[2 * pix + 1];
  }
  const Tap4 t = taps(u, v, Ws, Hs);
  const float w00 = t.wx0 * t.wy0, w01 = t.wx0 * t.wy1, w10 = t.wx1 * t.wy0, w11 = t.wx1 * t.wy1;
  if (out) {
    const float* S = img + (long)b * Hs * Ws * C;
    for (int c = 0; c < C; ++c)
      out[pix * C + c] = w00 * S[((long)t.y0 * Ws + t.x0) * C + c] + w01 * S[((long)t.y1 * Ws + t.x0) * C + c] +
                         w10 * S[((long)t.y0 * Ws + t.x1) * C + c] + w11 * S[((long)t.y1 * Ws + t.x1) * C + c];
  }
  if (coords) { coords[2 * pix] = u; coords[2 * pix + 1] = v; }
  if (flow_x) flow_x[pix] = u - (float)x;     // depth_optflow (utils_lr.py:472-489)
  if (flow_y) flow_y[pix] = v - (float)y;
  if (wmask) wmask[pix] = w00 + w01 + w10 + w11;
  if (zout) zout[pix] = z;
}

// ------------------------------------------------------------------ reference-named geometry ops
// (the un-fused utils_lr.py functions, for callers that build their own loss: pose_vec2mat,
// projective_inverse_warp, bilinear_sampler, optflow_warp, consistent_depth_loss) and their backward.

// euler2mat (utils_lr.py:26-75): R = Rx(x) @ Ry(y) @ Rz(z), angles clipped to [-pi, pi].
__device__ void euler_R(float z, float y, float x, float R[9]) {
  const float pi = 3.14159265358979f;
  z = fminf(fmaxf(z, -pi), pi); y = fminf(fmaxf(y, -pi), pi); x = fminf(fmaxf(x, -pi), pi);
  const float cz = cosf(z), sz = sinf(z), cy = cosf(y), sy = sinf(y), cx = cosf(x), sx = sinf(x);
  const float Rz[9] = {cz, -sz, 0.f, sz, cz, 0.f, 0.f, 0.f, 1.f};
  const float Ry[9] = {cy, 0.f, sy, 0.f, 1.f, 0.f, -sy, 0.f, cy};
  const float Rx[9] = {1.f, 0.f, 0.f, 0.f, cx, -sx, 0.f, sx, cx};
  float XY[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) XY[3 * i + j] = Rx[3 * i] * Ry[j] + Rx[3 * i + 1] * Ry[3 + j] + Rx[3 * i + 2] * Ry[6 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[3 * i + j] = XY[3 * i] * Rz[j] + XY[3 * i + 1] * Rz[3 + j] + XY[3 * i + 2] * Rz[6 + j];
}

// pose_vec2mat (utils_lr.py:106-149): format 0 'angleaxis', 1 'eular', 2 'test' (identity, no translation).
__global__ void pose_vec2mat_kernel(int B, const float* vec, int format, float* T) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* v = vec + 6 * b;
  float R[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f};
  if (format == 0) rodrigues(v + 3, R);
  else if (format == 1) euler_R(v[5], v[4], v[3], R);
  float* Tb = T + 16 * b;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) Tb[4 * i + j] = R[3 * i + j];
    Tb[4 * i + 3] = format == 2 ? 0.f : v[i];
  }
  Tb[12] = 0.f; Tb[13] = 0.f; Tb[14] = 0.f; Tb[15] = 1.f;
}

// Backward of the 'eular' branch: dL/d(rx,ry,rz) = <G, dR/dangle>, zero outside the clip range
// (tf.clip_by_value passes the gradient on [min, max]); translation gradient = G[:,3].
__global__ void pose_vec2mat_euler_bwd_kernel(int B, const float* vec, const float* dT, float* dvec, int accumulate) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float pi = 3.14159265358979f;
  const float* v = vec + 6 * b;
  const float* G = dT + 16 * b;
  const float ang[3] = {v[5], v[4], v[3]};   // z, y, x
  float out[6];
  for (int i = 0; i < 3; ++i) out[i] = G[4 * i + 3];
  float cl[3], c[3], s[3];
  for (int i = 0; i < 3; ++i) {
    cl[i] = fminf(fmaxf(ang[i], -pi), pi);
    c[i] = cosf(cl[i]); s[i] = sinf(cl[i]);
  }
  // matrices and their derivatives
  const float Rz[9] = {c[0], -s[0], 0.f, s[0], c[0], 0.f, 0.f, 0.f, 1.f};
  const float dRz[9] = {-s[0], -c[0], 0.f, c[0], -s[0], 0.f, 0.f, 0.f, 0.f};
  const float Ry[9] = {c[1], 0.f, s[1], 0.f, 1.f, 0.f, -s[1], 0.f, c[1]};
  const float dRy[9] = {-s[1], 0.f, c[1], 0.f, 0.f, 0.f, -c[1], 0.f, -s[1]};
  const float Rx[9] = {1.f, 0.f, 0.f, 0.f, c[2], -s[2], 0.f, s[2], c[2]};
  const float dRx[9] = {0.f, 0.f, 0.f, 0.f, -s[2], -c[2], 0.f, c[2], -s[2]};
  const float* A[3][3] = {{Rx, Ry, dRz}, {Rx, dRy, Rz}, {dRx, Ry, Rz}};
  float g[3];
  for (int k = 0; k < 3; ++k) {
    float M1[9], M[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        M1[3 * i + j] = A[k][0][3 * i] * A[k][1][j] + A[k][0][3 * i + 1] * A[k][1][3 + j] + A[k][0][3 * i + 2] * A[k][1][6 + j];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        M[3 * i + j] = M1[3 * i] * A[k][2][j] + M1[3 * i + 1] * A[k][2][3 + j] + M1[3 * i + 2] * A[k][2][6 + j];
    float acc = 0.f;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) acc += G[4 * i + j] * M[3 * i + j];
    g[k] = (ang[k] >= -pi && ang[k] <= pi) ? acc : 0.f;
  }
  out[3] = g[2]; out[4] = g[1]; out[5] = g[0];   // (rx, ry, rz)
  for (int i = 0; i < 6; ++i) dvec[6 * b + i] = accumulate ? dvec[6 * b + i] + out[i] : out[i];
}

// bilinear_sampler backward (utils_lr.py:276-366): out[c] = sum_taps w * img[tap][c], wmask = sum w.
// d_img[tap] += w * d_out (atomic scatter), d_coords = d_out . d out/d(u,v) + d_wmask * d wmask/d(u,v).
__global__ void __launch_bounds__(256) sampler_bwd_kernel(int B, int H, int W, int C, const float* coords,
                                                          const float* img, int Hs, int Ws, const float* d_out,
                                                          const float* d_wmask, float* d_img, float* d_coords) {
  const int b = blockIdx.y;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= H * W) return;
  const long pix = (long)b * H * W + idx;
  const float u = coords[2 * pix], v = coords[2 * pix + 1];
  const Tap4 t = taps(u, v, Ws, Hs);
  const float w00 = t.wx0 * t.wy0, w01 = t.wx0 * t.wy1, w10 = t.wx1 * t.wy0, w11 = t.wx1 * t.wy1;
  const long base = (long)b * Hs * Ws;
  const long i00 = (base + (long)t.y0 * Ws + t.x0) * C, i01 = (base + (long)t.y1 * Ws + t.x0) * C;
  const long i10 = (base + (long)t.y0 * Ws + t.x1) * C, i11 = (base + (long)t.y1 * Ws + t.x1) * C;
  float gu = 0.f, gv = 0.f;
  for (int c = 0; c < C; ++c) {
    const float g = d_out ? d_out[pix * C + c] : 0.f;
    if (g == 0.f) continue;
    if (d_coords) {
      const float s00 = img[i00 + c], s01 = img[i01 + c], s10 = img[i10 + c], s11 = img[i11 + c];
      gu += g * (-t.mx0 * (t.wy0 * s00 + t.wy1 * s01) + t.mx1 * (t.wy0 * s10 + t.wy1 * s11));
      gv += g * (-t.my0 * (t.wx0 * s00 + t.wx1 * s10) + t.my1 * (t.wx0 * s01 + t.wx1 * s11));
    }
    if (d_img) {
      if (w00 != 0.f) atomicAdd(d_img + i00 + c, w00 * g);
      if (w01 != 0.f) atomicAdd(d_img + i01 + c, w01 * g);
      if (w10 != 0.f) atomicAdd(d_img + i10 + c, w10 * g);
      if (w11 != 0.f) atomicAdd(d_img + i11 + c, w11 * g);
    }
  }
  if (d_coords) {
    if (d_wmask) {
      const float gw = d_wmask[pix];
      gu += gw * (t.mx1 - t.mx0) * (t.wy0 + t.wy1);
      gv += gw * (t.my1 - t.my0) * (t.wx0 + t.wx1);
    }
    d_coords[2 * pix] = gu;
    d_coords[2 * pix + 1] = gv;
  }
}

// Backward of (coords, z) = cam2pixel(P, pixel2cam(depth, meshgrid, Kinv)) (utils_lr.py:151-194):
// d_depth (+)= ..., gP[b][12] += dL/dP (fp64, block-reduced).  Intrinsics are data (no gradient).
__global__ void __launch_bounds__(256) cam_coords_bwd_kernel(int B, int H, int W, const float* depth, const float* P,
                                                             const float* Kinv, const float* d_coords,
                                                             const float* d_z, float* d_depth, int accumulate,
                                                             double* gP) {
  __shared__ double sh[12][4];
  const int b = blockIdx.y;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  double gp[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) gp[i] = 0.0;
  if (idx < H * W) {
    const long pix = (long)b * H * W + idx;
    const int y = idx / W, x = idx - y * W;
    const float dep = depth[pix];
    const float* Ki = Kinv + 9 * b;
    const float* Pb = P + 12 * b;
    float cam[3];
    for (int i = 0; i < 3; ++i) cam[i] = (Ki[3 * i] * x + Ki[3 * i + 1] * y + Ki[3 * i + 2]) * dep;
    const float p0 = Pb[0] * cam[0] + Pb[1] * cam[1] + Pb[2] * cam[2] + Pb[3];
    const float p1 = Pb[4] * cam[0] + Pb[5] * cam[1] + Pb[6] * cam[2] + Pb[7];
    const float den = Pb[8] * cam[0] + Pb[9] * cam[1] + Pb[10] * cam[2] + Pb[11] + 1e-10f;
    const float gu = d_coords ? d_coords[2 * pix] : 0.f, gv = d_coords ? d_coords[2 * pix + 1] : 0.f;
    const float gp0 = gu / den, gp1 = gv / den;
    const float gp2 = -(gu * p0 + gv * p1) / (den * den) + (d_z ? d_z[pix] : 0.f);
    const float gcam0 = Pb[0] * gp0 + Pb[4] * gp1 + Pb[8] * gp2;
    const float gcam1 = Pb[1] * gp0 + Pb[5] * gp1 + Pb[9] * gp2;
    const float gcam2 = Pb[2] * gp0 + Pb[6] * gp1 + Pb[10] * gp2;
    const float gps[3] = {gp0, gp1, gp2};
    for (int i = 0; i < 3; ++i) {
      gp[4 * i + 0] = gps[i] * cam[0];
      gp[4 * i + 1] = gps[i] * cam[1];
      gp[4 * i + 2] = gps[i] * cam[2];
      gp[4 * i + 3] = gps[i];
    }
    if (d_depth) {
      // cam = dep * (Kinv [x y 1]) -> d dep = gcam . (Kinv [x y 1])
      float gd = 0.f;
      const float gc[3] = {gcam0, gcam1, gcam2};
      for (int i = 0; i < 3; ++i) gd += gc[i] * (Ki[3 * i] * x + Ki[3 * i + 1] * y + Ki[3 * i + 2]);
      d_depth[pix] = accumulate ? d_depth[pix] + gd : gd;
    }
  }
  if (!gP) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = 0; i < 12; ++i) {
    double vv = gp[i];
    for (int off = 32; off > 0; off >>= 1) vv += __shfl_down(vv, off, 64);
    if (lane == 0) sh[i][wid] = vv;
  }
  __syncthreads();
  if (threadIdx.x < 12) {
    const int i = threadIdx.x;
    atomicAdd(gP + 12 * b + i, sh[i][0] + sh[i][1] + sh[i][2] + sh[i][3]);
  }
}

// dL/dT rows 0..2 from dL/dP with P = K @ T[0:3] (dT = K^T dP), row 3 zero; then to dvec via
// the pose backward of the chosen format (or left as dT for format 'matrix' == 3).
__global__ void dP_to_dT_kernel(int B, const float* K, const double* gP, float* dT) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* Kb = K + 9 * b;
  const double* g = gP + 12 * b;
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < 4; ++j)
      dT[16 * b + 4 * k + j] = (float)(Kb[k] * g[j] + Kb[3 + k] * g[4 + j] + Kb[6 + k] * g[8 + j]);
  for (int j = 0; j < 4; ++j) dT[16 * b + 12 + j] = 0.f;
}

}  // namespace

extern "C" {

int tde_pose_vec2mat(int B, const float* vec, int format, float* T, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && vec && T && format >= 0 && format <= 2);
  hipLaunchKernelGGL(pose_vec2mat_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B, vec,
                     format, T);
  return tde_launch_status();
}

int tde_pose_vec2mat_bwd(int B, const float* vec, int format, const float* dT, float* dvec, int accumulate,
                         void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && vec && dT && dvec && format >= 0 && format <= 2);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (format == 0)
    hipLaunchKernelGGL(pose_grad_kernel, dim3((B + 63) / 64), dim3(64), 0, st, B, 0, vec, (const float*)nullptr, 0L,
                       (const double*)nullptr, dT, dvec, accumulate);
  else if (format == 1)
    hipLaunchKernelGGL(pose_vec2mat_euler_bwd_kernel, dim3((B + 63) / 64), dim3(64), 0, st, B, vec, dT, dvec,
                       accumulate);
  else if (!accumulate)
    return tde_zero_bytes(sizeof(float) * 6 * (size_t)B, dvec, stream);   // 'test': constant
  return tde_launch_status();
}

int tde_sampler_bwd(int B, int H, int W, int C, const float* coords, const float* img, int Hs, int Ws,
                    const float* d_out, const float* d_wmask, float* d_img, float* d_coords, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && C > 0 && Hs > 0 && Ws > 0 && coords && img);
  TDE_CHECK_ARG(!d_img || d_out);
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(sampler_bwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), B, H, W, C, coords,
                     img, Hs, Ws, d_out, d_wmask, d_img, d_coords);
  return tde_launch_status();
}

int tde_cam_coords_bwd(int B, int H, int W, const float* depth, const float* P, const float* Kinv,
                       const float* d_coords, const float* d_z, float* d_depth, int accumulate, double* gP,
                       void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && depth && P && Kinv && (d_coords || d_z));
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(cam_coords_bwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), B, H, W, depth, P,
                     Kinv, d_coords, d_z, d_depth, accumulate, gP);
  return tde_launch_status();
}

int tde_pose_dp_to_dt(int B, const float* K, const double* gP, float* dT, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && K && gP && dT);
  hipLaunchKernelGGL(dP_to_dT_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B, K, gP,
                     dT);
  return tde_launch_status();
}

int tde_warp_fwd(int B, int H, int W, int C, const float* depth, int depth_is_disp, const float* P, const float* Kinv,
                 const float* coords_in, const float* img, int Hs, int Ws, float* out, float* coords, float* flow_x,
                 float* flow_y, float* wmask, float* z, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && (depth || coords_in) && (!depth || (P && Kinv)));
  TDE_CHECK_ARG(!out || (img && C > 0 && Hs > 0 && Ws > 0));
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(warp_fwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), B, H, W, C, depth,
                     depth_is_disp, P, Kinv, coords_in, img, Hs > 0 ? Hs : H, Ws > 0 ? Ws : W, out, coords, flow_x,
                     flow_y, wmask, z);
  return tde_launch_status();
}

int tde_warp_loss(const tde_warp_loss_t* a, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(a && a->B > 0 && a->H > 0 && a->W > 0 && a->img_src && a->img_tgt && a->loss);
  TDE_CHECK_ARG((a->disp != nullptr) != (a->flow != nullptr));
  TDE_CHECK_ARG(!a->disp || (a->P && a->Kinv));
  TDE_CHECK_ARG(!a->disp_other || a->disp);
  // <= ~512 blocks in all (each ends in up to 15 fp64 atomics on words shared by the whole grid / by its
  // batch element); threads loop over the rest
  static const long maxb = tde_env_pos("TDE_WARP_MAXB", 512);
  int gx = (a->H * a->W + 255) / 256;
  const int cap = (int)std::max(1L, maxb / a->B);
  if (gx > cap) gx = cap;
  dim3 grid(gx, a->B);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool gp = a->g_P && a->disp;
  if (a->det_ws == nullptr) {
    const WarpDet none{nullptr, nullptr, nullptr};
    if (gp) hipLaunchKernelGGL((warp_loss_kernel<true, false>), grid, dim3(256), 0, st, *a, none);
    else hipLaunchKernelGGL((warp_loss_kernel<false, false>), grid, dim3(256), 0, st, *a, none);
    return tde_launch_status();
  }
  const long n = (long)a->B * a->H * a->W;
  if (a->det_ws_bytes < tde_warp_loss_det_workspace_size(a->B, a->H, a->W) || !tde_aligned16(a->det_ws))
    return TDE_ERR_WORKSPACE;
  char* w = static_cast<char*>(a->det_ws);
  WarpDet det;
  det.acc = reinterpret_cast<long long*>(w);
  det.part = reinterpret_cast<double*>(w + 8 * n);
  det.bound = reinterpret_cast<unsigned*>(w + 8 * n + 8L * 15 * gx * a->B);
  const int pb = (int)std::min<long>(1024, (n + 255) / 256);
  if (hipMemsetAsync(det.bound, 0, 4, st) != hipSuccess) return TDE_ERR_HIP;
  hipLaunchKernelGGL(warp_det_prep_kernel, dim3(pb), dim3(256), 0, st, *a, det, n);
  if (gp) hipLaunchKernelGGL((warp_loss_kernel<true, true>), grid, dim3(256), 0, st, *a, det);
  else hipLaunchKernelGGL((warp_loss_kernel<false, true>), grid, dim3(256), 0, st, *a, det);
  hipLaunchKernelGGL(warp_det_finish_kernel, dim3(pb + 1), dim3(256), 0, st, *a, det, n, gx, gp ? 15 : 3);
  return tde_launch_status();
}

int tde_warp_loss_multi(const tde_warp_loss_t* args, int n, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(args && n > 0 && n <= TDE_WARP_MULTI_MAX);
  static const long maxb = tde_env_pos("TDE_WARP_MAXB", 512);
  WarpMulti m;
  m.n = n;
  m.start[0] = 0;
  const bool gp = args[0].g_P && args[0].disp;
  for (int c = 0; c < n; ++c) {
    const tde_warp_loss_t* a = args + c;
    TDE_CHECK_ARG(a->B > 0 && a->H > 0 && a->W > 0 && a->img_src && a->img_tgt && a->loss);
    TDE_CHECK_ARG((a->disp != nullptr) != (a->flow != nullptr));
    TDE_CHECK_ARG(!a->disp || (a->P && a->Kinv));
    TDE_CHECK_ARG(!a->disp_other || a->disp);
    TDE_CHECK_ARG(a->det_ws == nullptr);                   // the deterministic scatter runs per call (tde_warp_loss)
    TDE_CHECK_ARG((a->g_P && a->disp) == gp);               // one kernel variant for all calls
    int gx = (a->H * a->W + 255) / 256;
    const int cap = (int)std::max(1L, maxb / a->B);
    if (gx > cap) gx = cap;
    m.a[c] = *a;
    m.gx[c] = gx;
    m.start[c + 1] = m.start[c] + gx * a->B;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (gp) hipLaunchKernelGGL(warp_loss_multi_kernel<true>, dim3(m.start[n]), dim3(256), 0, st, m);
  else hipLaunchKernelGGL(warp_loss_multi_kernel<false>, dim3(m.start[n]), dim3(256), 0, st, m);
  return tde_launch_status();
}

size_t tde_warp_loss_det_workspace_size(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  static const long maxb = tde_env_pos("TDE_WARP_MAXB", 512);
  long gx = ((long)H * W + 255) / 256;
  const long cap = std::max(1L, maxb / B);
  if (gx > cap) gx = cap;
  return (size_t)(8L * B * H * W + 8L * 15 * gx * B + 16);
}

int tde_pose_prep(int B, const float* pose_vec, const float* pose_mat, const float* K, float* T, float* P,
                  float* Kinv, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && (pose_vec || pose_mat) && K && P && Kinv);
  hipLaunchKernelGGL(pose_prep_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B,
                     pose_vec, pose_mat, K, T, P, Kinv);
  return tde_launch_status();
}

int tde_pose_prep_multi(const tde_pose_prep_t* jobs, int n, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(jobs && n > 0 && n <= TDE_WARP_MULTI_MAX);
  PoseMulti m;
  int bmax = 0;
  for (int c = 0; c < n; ++c) {
    const tde_pose_prep_t& j = jobs[c];
    TDE_CHECK_ARG(j.B > 0 && (j.pose_vec || j.pose_mat) && j.K && j.P && j.Kinv);
    m.j[c] = j;
    bmax = std::max(bmax, j.B);
  }
  hipLaunchKernelGGL(pose_prep_multi_kernel, dim3((bmax + 63) / 64, n), dim3(64), 0, static_cast<hipStream_t>(stream),
                     m);
  return tde_launch_status();
}

int tde_pose_grad(int B, int nscales, const float* pose_vec, const float* K, long k_stride_b, const double* gP,
                  const float* gT_extra, float* g_pose_vec, int accumulate, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && nscales > 0 && pose_vec && K && gP && g_pose_vec);
  hipLaunchKernelGGL(pose_grad_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B,
                     nscales, pose_vec, K, k_stride_b, gP, gT_extra, g_pose_vec, accumulate);
  return tde_launch_status();
}

int tde_pose_grad_spread(const tde_pose_grad_t* jobs, int n, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(jobs && n > 0 && n <= TDE_WARP_MULTI_MAX);
  PoseGradMulti m;
  int bmax = 0;
  for (int c = 0; c < n; ++c) {
    const tde_pose_grad_t& j = jobs[c];
    TDE_CHECK_ARG(j.B > 0 && j.nscales > 0 && j.pose_vec && j.K && j.gP && j.g_pose_vec);
    TDE_CHECK_ARG(!j.dpose || (j.hw > 0 && j.dpose_cstride >= 6));
    m.j[c] = j;
    bmax = std::max(bmax, j.B);
  }
  hipLaunchKernelGGL(pose_grad_spread_kernel, dim3((bmax + 63) / 64, n), dim3(64), 0,
                     static_cast<hipStream_t>(stream), m);
  return tde_launch_status();
}

int tde_cam_loss(int B, const float* gt_vec, const float* T_lr, const float* T_rl, float weight, double* loss,
                 float* gT_lr, float* gT_rl, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(B > 0 && gt_vec && T_lr && T_rl && loss && gT_lr && gT_rl);
  hipLaunchKernelGGL(cam_loss_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B, gt_vec,
                     T_lr, T_rl, weight, loss, gT_lr, gT_rl);
  return tde_launch_status();
}

}  // extern "C"
