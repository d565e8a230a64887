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

template <bool NEED_G_P>
__global__ void __launch_bounds__(256) warp_loss_kernel(const tde_warp_loss_t a) {
  __shared__ double sh[16][4];
  const int b = blockIdx.y;
  const int HW = a.H * a.W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  double l_photo = 0, l_exp = 0, l_cons = 0;
  double gp[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) gp[i] = 0.0;
  const double inv_n3 = 1.0 / (3.0 * a.B * HW), inv_n = 1.0 / ((double)a.B * HW);
  if (idx < HW) {
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
      l_exp = (double)(-(l1 - m) + logf(e0 + e1)) * a.exp_w * inv_n;
    } else if (a.wmask) {
      wpix = a.wmask[pix];
    }
    l_photo = (double)esum * wpix * a.photo_w * inv_n3;
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
      l_cons = (double)cons * p1 * a.consist_w * inv_n;
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
        if (w00 != 0.f) atomicAdd(Go + i00, -g_o * w00 * o00 * o00);
        if (w01 != 0.f) atomicAdd(Go + i01, -g_o * w01 * o01 * o01);
        if (w10 != 0.f) atomicAdd(Go + i10, -g_o * w10 * o10 * o10);
        if (w11 != 0.f) atomicAdd(Go + i11, -g_o * w11 * o11 * o11);
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
          gp[4 * i + 0] = gps[i] * cam[0];
          gp[4 * i + 1] = gps[i] * cam[1];
          gp[4 * i + 2] = gps[i] * cam[2];
          gp[4 * i + 3] = gps[i];
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
    if (i < 3) {
      if (s != 0.0) atomicAdd(a.loss + i, s);
    } else {
      atomicAdd(a.g_P + 12 * b + (i - 3), s);
    }
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

__global__ void pose_prep_kernel(int B, const float* vec, const float* mat, const float* K, float* T, float* P,
                                 float* Kinv) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
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

// dL/dvec from dL/dP (all scales summed: gP[s][b][12], K_s at Ks + b*k_stride_b + 9*s) and an
// optional extra dL/dT [B][16] (cam loss).  Rodrigues backward (utils_lr.py:77-103,126-134).
__global__ void pose_grad_kernel(int B, int nscales, const float* vec, const float* Ks, long k_stride_b,
                                 const double* gP, const float* gT_extra, float* gvec, int accumulate) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
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
  float out[6];
  for (int i = 0; i < 3; ++i) out[i] = (float)G[4 * i + 3];
  for (int i = 0; i < 3; ++i) out[3 + i] = (float)((da[i] - a[i] * ada) / th + dth_total * a[i]);
  for (int i = 0; i < 6; ++i) gvec[6 * b + i] = accumulate ? gvec[6 * b + i] + out[i] : out[i];
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

}  // namespace

extern "C" {

int tde_warp_fwd(int B, int H, int W, int C, const float* depth, int depth_is_disp, const float* P, const float* Kinv,
                 const float* coords_in, const float* img, int Hs, int Ws, float* out, float* coords, float* flow_x,
                 float* flow_y, float* wmask, float* z, void* stream) {
  TDE_CHECK_ARG(B > 0 && H > 0 && W > 0 && (depth || coords_in) && (!depth || (P && Kinv)));
  TDE_CHECK_ARG(!out || (img && C > 0 && Hs > 0 && Ws > 0));
  dim3 grid((H * W + 255) / 256, B);
  hipLaunchKernelGGL(warp_fwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream), B, H, W, C, depth,
                     depth_is_disp, P, Kinv, coords_in, img, Hs > 0 ? Hs : H, Ws > 0 ? Ws : W, out, coords, flow_x,
                     flow_y, wmask, z);
  return tde_launch_status();
}

int tde_warp_loss(const tde_warp_loss_t* a, void* stream) {
  TDE_CHECK_ARG(a && a->B > 0 && a->H > 0 && a->W > 0 && a->img_src && a->img_tgt && a->loss);
  TDE_CHECK_ARG((a->disp != nullptr) != (a->flow != nullptr));
  TDE_CHECK_ARG(!a->disp || (a->P && a->Kinv));
  TDE_CHECK_ARG(!a->disp_other || a->disp);
  dim3 grid((a->H * a->W + 255) / 256, a->B);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a->g_P && a->disp) hipLaunchKernelGGL(warp_loss_kernel<true>, grid, dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(warp_loss_kernel<false>, grid, dim3(256), 0, st, *a);
  return tde_launch_status();
}

int tde_pose_prep(int B, const float* pose_vec, const float* pose_mat, const float* K, float* T, float* P,
                  float* Kinv, void* stream) {
  TDE_CHECK_ARG(B > 0 && (pose_vec || pose_mat) && K && P && Kinv);
  hipLaunchKernelGGL(pose_prep_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B,
                     pose_vec, pose_mat, K, T, P, Kinv);
  return tde_launch_status();
}

int tde_pose_grad(int B, int nscales, const float* pose_vec, const float* K, long k_stride_b, const double* gP,
                  const float* gT_extra, float* g_pose_vec, int accumulate, void* stream) {
  TDE_CHECK_ARG(B > 0 && nscales > 0 && pose_vec && K && gP && g_pose_vec);
  hipLaunchKernelGGL(pose_grad_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B,
                     nscales, pose_vec, K, k_stride_b, gP, gT_extra, g_pose_vec, accumulate);
  return tde_launch_status();
}

int tde_cam_loss(int B, const float* gt_vec, const float* T_lr, const float* T_rl, float weight, double* loss,
                 float* gT_lr, float* gT_rl, void* stream) {
  TDE_CHECK_ARG(B > 0 && gt_vec && T_lr && T_rl && loss && gT_lr && gT_rl);
  hipLaunchKernelGGL(cam_loss_kernel, dim3((B + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), B, gt_vec,
                     T_lr, T_rl, weight, loss, gT_lr, gT_rl);
  return tde_launch_status();
}

}  // extern "C"
