// slim.batch_norm(center=True, scale=False, eps=1e-3) + ReLU, training and inference, forward and
// backward (TF FusedBatchNorm / FusedBatchNormGrad as used by the arg_scope of
// nets_optflow_depth.py:82-87).
//
// At the shapes of the reference nets these passes are launch-latency bound (~5 us per kernel on
// MI355X) or per-CU-bandwidth bound, so:
//   M <= BN_SMALL_M = 512 rows per group (the deepest levels): ONE kernel per direction; a block owns one channel
//     quad over all rows (row values held in registers), statistics, finalize, moving averages and apply in place.
//     (512, not 2048: the partial-sum path's wider grids measured +0.5 % on the config-4 step, round 4.)
//   larger M, forward: the statistics partials come from the producing conv (its epilogue or its
//     split-K reduce, conv_igemm.hip) -- or from bn_part_kernel for the standalone entry point -- then a
//     finalize launch and an apply launch.
//   larger M, backward: partial sums (many-block grid), finalize, apply.
// Per-channel sums are fp64 and reduced in a fixed order: deterministic, no atomics.
#include "tde_common.h"

#include "bn_internal.h"

#include <cstdlib>

#ifndef TDE_BN_XCD
#define TDE_BN_XCD 1
#endif

namespace {

// channel-quad block of the M <= BN_SMALL_M forward / backward kernels: XCD-contiguous, so the 8 quads of one 128-byte
// row line share an L2 (rocprofv3, config 2: bn_fwd_small 6.41 -> 5.27 us, bn_bwd_small 8.90 -> 7.67 us; the
// finalize kernel, 32-byte fp64 pieces, was neutral-to-slower and keeps hardware order).  TDE_BN_XCD=0: hardware
// order everywhere, for A/B builds.
__device__ __forceinline__ int bn_quad_block() {
  return TDE_BN_XCD ? tde_xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// MODE 0 (forward): sums of z and z^2.  MODE 1 (backward): sums of g and g*xhat, g = dy * relu'(y).
// Grid (row chunk, group of 16 channel quads); part[chunk][2][C] (fp64).
template <int MODE>
__global__ void __launch_bounds__(256) bn_part_kernel(int M, int C, const float* z, const float* dy, int dycs, int dyco,
                                                      const float* mean, const float* invstd, const float* beta,
                                                      int relu, const BnChunks cp, double* part) {
  __shared__ double sh[2][256 * 4];
  const int q0 = blockIdx.y * 16;
  const int nq = min(16, C / 4 - q0);
  const int ty_n = 256 / nq;
  const int tx = threadIdx.x % nq, ty = threadIdx.x / nq;
  const int c = 4 * (q0 + tx);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  int r0, r1;
  bn_chunk_rows(cp, blockIdx.x, r0, r1);
  if (ty < ty_n) {
    f4 mu = {0, 0, 0, 0}, is = {0, 0, 0, 0}, bt = {0, 0, 0, 0};
    if (MODE == 1) {
      const int g = blockIdx.x / cp.per_g;      // the chunk's row group: its statistics
      mu = *reinterpret_cast<const f4*>(mean + (long)g * C + c);
      is = *reinterpret_cast<const f4*>(invstd + (long)g * C + c);
      bt = *reinterpret_cast<const f4*>(beta + c);
    }
    // fp32 partials over <= 64 rows per lane, flushed into fp64; unrolled so several rows' loads are
    // in flight at once
    for (int rb = r0 + ty; rb < r1; rb += 64 * ty_n) {
      const int rend = min(r1, rb + 64 * ty_n);
      float f0[4] = {0, 0, 0, 0}, f1[4] = {0, 0, 0, 0};
#pragma unroll 8
      for (int r = rb; r < rend; r += ty_n) {
        const f4 zv = *reinterpret_cast<const f4*>(z + (long)r * C + c);
        if (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) { f0[j] += zv[j]; f1[j] += zv[j] * zv[j]; }
        } else {
          const f4 gv = *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + c);
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
  rowlane_combine(s0, s1, nq, ty_n, &sh[0][0]);
  if (ty == 0) {
    double* o = part + (long)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[c + j] = s0[j]; o[C + c + j] = s1[j]; }
  }
}

// Reduce `nparts` partials per channel.  Block = one channel quad x 64 stripes (256 lanes; four
// neighbouring lanes read 32 contiguous bytes), so a C-channel layer runs C/4 blocks; 8 loads in flight
// per lane, then a fixed-order combine: an xor-shuffle tree over a wave's 16 stripes of a channel and the 4
// waves through LDS (one barrier; the round-1 version walked 1024 lanes down 9 LDS levels with a barrier
// each).  MODE 0 publishes mean / invstd and updates the moving averages; MODE 1 writes
// coef = (mean g, mean g*xhat) and dbeta; MODE 2 the raw sums.
// Row groups (G >= 1; M = rows per group): group g reduces partials [g * nparts/G, (g+1) * nparts/G) and writes
// its statistics at [g][C] (coef [g][2][C]); the moving averages take one update per group and dbeta the
// groups' sums in group order -- what G consecutive slim.batch_norm calls of a shared-variable network do.
// NT = 256 lanes for up to 512 partial rows, 1024 above (more loads in flight for the long reductions).
template <int MODE, int NT>
__global__ void __launch_bounds__(NT) bn_finalize_kernel(int M, int C, int nparts, const double* part, float eps,
                                                         float decay, int bessel, float* mm, float* mv,
                                                         float* save_mean, float* save_invstd, float* dbeta,
                                                         int acc, float* coef, double* sums = nullptr, int G = 1,
                                                         double* sums2 = nullptr) {
  constexpr int FIN_ST = NT / 4, NWV = NT / 64;
  __shared__ double sh[2][NWV][4];
  const int cl = threadIdx.x & 3, st = threadIdx.x >> 2;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 4 + cl;
  // the read-modify-write operands of the 4 publishing lanes, loaded before the reduction so their
  // latency overlaps the partial-sum loads (after the barrier they would add one dependent round trip)
  float mm0 = 0.f, mv0 = 0.f, db0 = 0.f;
  if (threadIdx.x < 4) {
    if (MODE == 0 && mm) { mm0 = mm[c]; mv0 = mv[c]; }
    if (MODE == 1 && dbeta && acc) db0 = dbeta[c];
  }
  const int pg = nparts / G;
  bool first = !acc;
  for (int g = 0; g < G; ++g) {
    const double* pp = part + (long)g * pg * 2 * C;
    double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    int k = st;
    for (; k + 3 * FIN_ST < pg; k += 4 * FIN_ST) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] += pp[(long)(k + u * FIN_ST) * 2 * C + c];
        b[u] += pp[(long)(k + u * FIN_ST) * 2 * C + C + c];
      }
    }
    for (int u = 0; k < pg; k += FIN_ST, ++u) {
      a[u] += pp[(long)k * 2 * C + c];
      b[u] += pp[(long)k * 2 * C + C + c];
    }
    double ra = (a[0] + a[1]) + (a[2] + a[3]), rb = (b[0] + b[1]) + (b[2] + b[3]);
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) {   // the 16 lanes of this wave with the same channel (lane bits 2..5)
      ra += __shfl_xor(ra, o, 64);
      rb += __shfl_xor(rb, o, 64);
    }
    if (g > 0) __syncthreads();          // the publishing lanes have read the previous group's sums
    if (lane < 4) { sh[0][wv][lane] = ra; sh[1][wv][lane] = rb; }
    __syncthreads();
    if (threadIdx.x < 4) {
      double s = 0, s2 = 0;
#pragma unroll
      for (int w = 0; w < NWV; ++w) { s += sh[0][w][cl]; s2 += sh[1][w][cl]; }
      if (MODE == 2) {   // raw per-channel sums (SyncBN: all-reduced by the caller, then *_from_sums)
        sums[(long)g * 2 * C + c] = s;
        sums[(long)g * 2 * C + C + c] = s2;
        if (sums2) { sums2[(long)g * 2 * C + c] = s; sums2[(long)g * 2 * C + C + c] = s2; }
      } else if (MODE == 0) {
        const double mean = s / M;
        double var = s2 / M - mean * mean;
        if (var < 0) var = 0;
        save_mean[(long)g * C + c] = (float)mean;
        save_invstd[(long)g * C + c] = (float)(1.0 / sqrt(var + (double)eps));
        if (mm) {
          const double vu = (bessel && M > 1) ? var * M / (M - 1) : var;
          mm0 = mm0 - (mm0 - (float)mean) * (1.f - decay);
          mv0 = mv0 - (mv0 - (float)vu) * (1.f - decay);
        }
      } else {
        db0 = first ? (float)s : db0 + (float)s;
        first = false;
        coef[(long)g * 2 * C + c] = (float)(s / M);
        coef[(long)g * 2 * C + C + c] = (float)(s2 / M);
      }
    }
  }
  if (threadIdx.x < 4) {
    if (MODE == 0 && mm) { mm[c] = mm0; mv[c] = mv0; }
    if (MODE == 1 && dbeta) dbeta[c] = db0;
  }
}

// SyncBN statistics of channels c..c+3 of row group g from the (all-reduced) sums [G][2][C] over Mt rows: fp64
// mean / variance, rounded to fp32 once (the expressions publish_fwd stores, so every block applies the statistics
// block 0 publishes).
__device__ __forceinline__ void stats_from_sums(const double* sums, int C, int g, int c, double Mt, float eps,
                                                f4& mu, f4& is) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double sv = sums[(long)g * 2 * C + c + j], s2 = sums[(long)g * 2 * C + C + c + j];
    const double mean = sv / Mt;
    double var = s2 / Mt - mean * mean;
    if (var < 0) var = 0;
    mu[j] = (float)mean;
    is[j] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// What the SyncBN one-launch apply passes publish from block 0 (per row group, in group order): forward the batch
// statistics and the moving averages, backward dbeta from this replica's own sums.
struct SumsPub {
  const double* sums;        // all-reduced [G][2][C]
  const double* lsums;       // backward: this replica's [G][2][C] (dbeta)
  double Mt;                 // rows per group over all replicas
  float eps, decay;
  int bessel, G, acc;
  float *mm, *mv, *save_mean, *save_invstd, *dbeta;
};

__device__ __forceinline__ void publish_fwd(const SumsPub& P, int C, int c) {
  float mm0[4] = {0, 0, 0, 0}, mv0[4] = {0, 0, 0, 0};
  if (P.mm) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { mm0[j] = P.mm[c + j]; mv0[j] = P.mv[c + j]; }
  }
  for (int g = 0; g < P.G; ++g) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double sv = P.sums[(long)g * 2 * C + c + j], s2 = P.sums[(long)g * 2 * C + C + c + j];
      const double mean = sv / P.Mt;
      double var = s2 / P.Mt - mean * mean;
      if (var < 0) var = 0;
      P.save_mean[(long)g * C + c + j] = (float)mean;
      P.save_invstd[(long)g * C + c + j] = (float)(1.0 / sqrt(var + (double)P.eps));
      if (P.mm) {
        const double vu = (P.bessel && P.Mt > 1) ? var * P.Mt / (P.Mt - 1) : var;
        mm0[j] -= (mm0[j] - (float)mean) * (1.f - P.decay);
        mv0[j] -= (mv0[j] - (float)vu) * (1.f - P.decay);
      }
    }
  }
  if (P.mm) {
#pragma unroll
    for (int j = 0; j < 4; ++j) { P.mm[c + j] = mm0[j]; P.mv[c + j] = mv0[j]; }
  }
}

__device__ __forceinline__ void publish_bwd(const SumsPub& P, int C, int c) {
  if (!P.dbeta) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float db = P.acc ? P.dbeta[c + j] : 0.f;
    for (int g = 0; g < P.G; ++g) {
      const float l = (float)P.lsums[(long)g * 2 * C + c + j];
      db = (g == 0 && !P.acc) ? l : db + l;
    }
    P.dbeta[c + j] = db;
  }
}

constexpr int APPLY_RB = 8;   // rows in flight per lane in the apply passes

// y = relu((z - mean) * invstd + beta): rows split over blocks, a thread owns one channel quad of a row
// lane (no 64-bit division in the index math).
// Row groups: rows [g*Mg, (g+1)*Mg) use the statistics at [g][C] (a thread moves to the next group's
// statistics when its row walk crosses a group boundary).
// SUMS (SyncBN, one launch instead of from-sums + apply): the statistics come from the all-reduced sums (P), and
// block 0 publishes them and the moving averages.
template <bool SUMS>
__global__ void __launch_bounds__(256) bn_apply_kernel(int M, int C, const float* z, const float* mean,
                                                       const float* invstd, const float* beta, int relu, float* y,
                                                       int ycs, int yco, int rows_per_block, int Mg, SumsPub P) {
  const int cq = C / 4;
  const int rstep = cq >= 256 ? 1 : 256 / cq;
  if (cq < 256 && threadIdx.x >= rstep * cq) return;
  const int rl = cq >= 256 ? 0 : threadIdx.x / cq;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int qq = (cq >= 256 ? threadIdx.x : threadIdx.x % cq); qq < cq; qq += (cq >= 256 ? 256 : cq)) {
    const int c = 4 * qq;
    if (SUMS && blockIdx.x == 0 && rl == 0) publish_fwd(P, C, c);
    int g = (r0 + rl) / Mg, gend = (g + 1) * Mg;
    f4 mu, is;
    if (SUMS) {
      stats_from_sums(P.sums, C, g, c, P.Mt, P.eps, mu, is);
    } else {
      mu = *reinterpret_cast<const f4*>(mean + (long)g * C + c);
      is = *reinterpret_cast<const f4*>(invstd + (long)g * C + c);
    }
    const f4 bt = *reinterpret_cast<const f4*>(beta + c);
    // APPLY_RB rows' loads issued before the first is used (a load -> store chain per row left these passes at
    // ~1/4 of HBM rate)
    for (int rb = r0 + rl; rb < r1; rb += APPLY_RB * rstep) {
      f4 zv[APPLY_RB];
#pragma unroll
      for (int i = 0; i < APPLY_RB; ++i) {
        const int r = rb + i * rstep;
        zv[i] = r < r1 ? *reinterpret_cast<const f4*>(z + (long)r * C + c) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < APPLY_RB; ++i) {
        const int r = rb + i * rstep;
        if (r >= r1) break;
        if (r >= gend) {
          g = r / Mg;
          gend = (g + 1) * Mg;
          if (SUMS) {
            stats_from_sums(P.sums, C, g, c, P.Mt, P.eps, mu, is);
          } else {
            mu = *reinterpret_cast<const f4*>(mean + (long)g * C + c);
            is = *reinterpret_cast<const f4*>(invstd + (long)g * C + c);
          }
        }
        f4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = (zv[i][j] - mu[j]) * is[j] + bt[j];
          o[j] = (relu && v < 0.f) ? 0.f : v;
        }
        tde_st(reinterpret_cast<f4*>(y + (long)r * ycs + yco + c), o);
      }
    }
  }
}

// max|dz| of a block's values into one of the TDE_BOUND_SLOTS slots of amax (slot = block % slots, so that
// at most blocks / 16 atomics contend for an address; a bound is the max of its slots): the fp16x3 conv
// math's operand bound of the gradient (tde_conv_desc_t.y_absmax).  uint order = float order for
// non-negative floats; fmaxf from 0 keeps NaN out of the bound.  Every thread of the block must call it.
__device__ __forceinline__ void block_absmax_to(float m, float* amax) {
  __shared__ float wmx[4];
  if (amax == nullptr) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmx[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wmx[0], wmx[1]), fmaxf(wmx[2], wmx[3]));
    if (m > 0.f) atomicMax(reinterpret_cast<unsigned*>(amax + (blockIdx.x & (TDE_BOUND_SLOTS - 1))), __float_as_uint(m));
  }
}

// coef = (mean g, mean g*xhat) of row group g: from the finalize's coef, or (SUMS) from the all-reduced sums over
// P.Mt rows (fp64 quotient, one fp32 rounding)
template <bool SUMS>
__device__ __forceinline__ void bwd_coef(const float* coef, const SumsPub& P, int C, int g, int c, f4& mg, f4& mgx) {
  if (SUMS) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mg[j] = (float)(P.sums[(long)g * 2 * C + c + j] / P.Mt);
      mgx[j] = (float)(P.sums[(long)g * 2 * C + C + c + j] / P.Mt);
    }
  } else {
    mg = *reinterpret_cast<const f4*>(coef + (long)g * 2 * C + c);
    mgx = *reinterpret_cast<const f4*>(coef + (long)g * 2 * C + C + c);
  }
}

template <bool SUMS>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(int M, int C, const float* z, const float* dy, int dycs,
                                                           int dyco, const float* mean, const float* invstd,
                                                           const float* beta, const float* coef, int relu,
                                                           float* dz, int rows_per_block, float* amax, int Mg,
                                                           SumsPub P) {
  const int cq = C / 4;
  const int rstep = cq >= 256 ? 1 : 256 / cq;
  const bool active = cq >= 256 || threadIdx.x < rstep * cq;
  const int rl = cq >= 256 ? 0 : threadIdx.x / cq;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float mx = 0.f;
  for (int qq = (cq >= 256 ? threadIdx.x : threadIdx.x % cq); active && qq < cq; qq += (cq >= 256 ? 256 : cq)) {
    const int c = 4 * qq;
    if (SUMS && blockIdx.x == 0 && rl == 0) publish_bwd(P, C, c);
    int g = (r0 + rl) / Mg, gend = (g + 1) * Mg;
    f4 mu = *reinterpret_cast<const f4*>(mean + (long)g * C + c);
    f4 is = *reinterpret_cast<const f4*>(invstd + (long)g * C + c);
    const f4 bt = *reinterpret_cast<const f4*>(beta + c);
    f4 mg, mgx;
    bwd_coef<SUMS>(coef, P, C, g, c, mg, mgx);
    for (int rb = r0 + rl; rb < r1; rb += APPLY_RB * rstep) {
      f4 zv[APPLY_RB], gv[APPLY_RB];
#pragma unroll
      for (int i = 0; i < APPLY_RB; ++i) {
        const int r = rb + i * rstep;
        zv[i] = r < r1 ? *reinterpret_cast<const f4*>(z + (long)r * C + c) : f4{0.f, 0.f, 0.f, 0.f};
        gv[i] = r < r1 ? *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + c) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < APPLY_RB; ++i) {
        const int r = rb + i * rstep;
        if (r >= r1) break;
        if (r >= gend) {
          g = r / Mg;
          gend = (g + 1) * Mg;
          mu = *reinterpret_cast<const f4*>(mean + (long)g * C + c);
          is = *reinterpret_cast<const f4*>(invstd + (long)g * C + c);
          bwd_coef<SUMS>(coef, P, C, g, c, mg, mgx);
        }
        f4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (zv[i][j] - mu[j]) * is[j];
          const float gg = (!relu || xh + bt[j] > 0.f) ? gv[i][j] : 0.f;
          o[j] = is[j] * (gg - mg[j] - xh * mgx[j]);
          mx = fmaxf(mx, fabsf(o[j]));
        }
        tde_st(reinterpret_cast<f4*>(dz + (long)r * C + c), o);
      }
    }
  }
  block_absmax_to(mx, amax);
}

// ------------------------------------------------------------------ M <= BN_SMALL_M (512): one kernel
// Block = one channel quad; each lane keeps its <= BN_SMALL_M / 256 rows per group in registers between the statistics and the
// apply (fp32 per lane, fp64 across lanes, fixed-order wave/LDS combine).  GT row groups are in flight at once (all
// their loads issued before the first reduction, one barrier round for all of them): a twin run's two groups cost
// one load -> reduce -> apply latency chain instead of two.  The moving averages and dbeta still take the groups'
// values in group order (one thread per channel walks them).
constexpr int SMALL_R = BN_SMALL_M / 256;
#ifndef TDE_SMALL_GT2   // diagnostic A/B build flag: 0 = one row group in flight (the round-3 kernels)
#define TDE_SMALL_GT2 1
#endif

template <int GT>
__global__ void __launch_bounds__(256) bn_fwd_small_kernel(int M, int C, const float* z, const float* beta, float eps,
                                                           float decay, int bessel, float* mm, float* mv,
                                                           float* save_mean, float* save_invstd, float* y, int ycs,
                                                           int yco, int relu, int G) {
  // M = rows per group (<= BN_SMALL_M); groups g0 .. g0+GT-1 together, G / GT rounds one after the other
  __shared__ double sh[GT][2][4][4];
  __shared__ float s_mu[GT][4], s_is[GT][4];
  const int c = bn_quad_block() * 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // beta and the moving averages loaded up front (off the reduce -> publish -> apply chain)
  const f4 bt = *reinterpret_cast<const f4*>(beta + c);
  float mm0 = 0.f, mv0 = 0.f;
  if (threadIdx.x < 4 && mm) { mm0 = mm[c + threadIdx.x]; mv0 = mv[c + threadIdx.x]; }
  for (int g0 = 0; g0 < G; g0 += GT) {
    f4 v[GT][SMALL_R];
    float fa[GT][4], fb[GT][4];
#pragma unroll
    for (int k = 0; k < GT; ++k) {
      const float* zg = z + (long)(g0 + k) * M * C;
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[k][j] = fb[k][j] = 0.f;
#pragma unroll
      for (int i = 0; i < SMALL_R; ++i) {
        const int r = threadIdx.x + 256 * i;
        v[k][i] = r < M ? *reinterpret_cast<const f4*>(zg + (long)r * C + c) : f4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) { fa[k][j] += v[k][i][j]; fb[k][j] += v[k][i][j] * v[k][i][j]; }
      }
    }
    if (g0 > 0) __syncthreads();          // the previous round's apply has read s_mu / s_is
#pragma unroll
    for (int k = 0; k < GT; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double a = wave_sum_d((double)fa[k][j]), b = wave_sum_d((double)fb[k][j]);
        if (lane == 0) { sh[k][0][wv][j] = a; sh[k][1][wv][j] = b; }
      }
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      const int j = threadIdx.x, cc = c + j;
#pragma unroll
      for (int k = 0; k < GT; ++k) {
        const double s = ((sh[k][0][0][j] + sh[k][0][1][j]) + sh[k][0][2][j]) + sh[k][0][3][j];
        const double s2 = ((sh[k][1][0][j] + sh[k][1][1][j]) + sh[k][1][2][j]) + sh[k][1][3][j];
        const double mean = s / M;
        double var = s2 / M - mean * mean;
        if (var < 0) var = 0;
        const float mu = (float)mean, is = (float)(1.0 / sqrt(var + (double)eps));
        s_mu[k][j] = mu; s_is[k][j] = is;
        save_mean[(long)(g0 + k) * C + cc] = mu;
        save_invstd[(long)(g0 + k) * C + cc] = is;
        if (mm) {
          const double vu = (bessel && M > 1) ? var * M / (M - 1) : var;
          mm0 = mm0 - (mm0 - mu) * (1.f - decay);
          mv0 = mv0 - (mv0 - (float)vu) * (1.f - decay);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GT; ++k) {
      float* yg = y + (long)(g0 + k) * M * ycs;
#pragma unroll
      for (int i = 0; i < SMALL_R; ++i) {
        const int r = threadIdx.x + 256 * i;
        if (r < M) {
          f4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = (v[k][i][j] - s_mu[k][j]) * s_is[k][j] + bt[j];
            o[j] = (relu && t < 0.f) ? 0.f : t;
          }
          tde_st(reinterpret_cast<f4*>(yg + (long)r * ycs + yco + c), o);
        }
      }
    }
  }
  if (threadIdx.x < 4 && mm) { mm[c + threadIdx.x] = mm0; mv[c + threadIdx.x] = mv0; }
}

template <int GT>
__global__ void __launch_bounds__(256) bn_bwd_small_kernel(int M, int C, const float* z, const float* mean,
                                                           const float* invstd, const float* beta, const float* dy,
                                                           int dycs, int dyco, float* dz, float* dbeta, int acc,
                                                           int relu, float* amax, int G) {
  // M = rows per group (<= BN_SMALL_M); groups g0 .. g0+GT-1 together; dbeta takes the groups' sums in group
  // order (the first overwrites unless accumulating)
  __shared__ double sh[GT][2][4][4];
  __shared__ float s_mg[GT][4], s_mgx[GT][4];
  const int c = bn_quad_block() * 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const f4 bt = *reinterpret_cast<const f4*>(beta + c);
  float db = (threadIdx.x < 4 && dbeta && acc) ? dbeta[c + threadIdx.x] : 0.f;
  bool first = !acc;
  float mx = 0.f;
  for (int g0 = 0; g0 < G; g0 += GT) {
    f4 mu[GT], is[GT];
    f4 xr[GT][SMALL_R], gr[GT][SMALL_R];
    float fa[GT][4], fb[GT][4];
#pragma unroll
    for (int k = 0; k < GT; ++k) {
      mu[k] = *reinterpret_cast<const f4*>(mean + (long)(g0 + k) * C + c);
      is[k] = *reinterpret_cast<const f4*>(invstd + (long)(g0 + k) * C + c);
    }
#pragma unroll
    for (int k = 0; k < GT; ++k) {
      const long row0 = (long)(g0 + k) * M;
#pragma unroll
      for (int j = 0; j < 4; ++j) fa[k][j] = fb[k][j] = 0.f;
#pragma unroll
      for (int i = 0; i < SMALL_R; ++i) {
        const int r = threadIdx.x + 256 * i;
        xr[k][i] = f4{0, 0, 0, 0}; gr[k][i] = f4{0, 0, 0, 0};
        if (r < M) {
          const f4 v = *reinterpret_cast<const f4*>(z + (row0 + r) * C + c);
          const f4 gv = *reinterpret_cast<const f4*>(dy + (row0 + r) * dycs + dyco + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xh = (v[j] - mu[k][j]) * is[k][j];
            const float gg = (!relu || xh + bt[j] > 0.f) ? gv[j] : 0.f;
            xr[k][i][j] = xh; gr[k][i][j] = gg;
            fa[k][j] += gg; fb[k][j] += gg * xh;
          }
        }
      }
    }
    if (g0 > 0) __syncthreads();          // the previous round's apply has read s_mg / s_mgx
#pragma unroll
    for (int k = 0; k < GT; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double a = wave_sum_d((double)fa[k][j]), b = wave_sum_d((double)fb[k][j]);
        if (lane == 0) { sh[k][0][wv][j] = a; sh[k][1][wv][j] = b; }
      }
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      const int j = threadIdx.x;
#pragma unroll
      for (int k = 0; k < GT; ++k) {
        const double s = ((sh[k][0][0][j] + sh[k][0][1][j]) + sh[k][0][2][j]) + sh[k][0][3][j];
        const double sx = ((sh[k][1][0][j] + sh[k][1][1][j]) + sh[k][1][2][j]) + sh[k][1][3][j];
        s_mg[k][j] = (float)(s / M);
        s_mgx[k][j] = (float)(sx / M);
        db = first ? (float)s : db + (float)s;
        first = false;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GT; ++k) {
      const long row0 = (long)(g0 + k) * M;
#pragma unroll
      for (int i = 0; i < SMALL_R; ++i) {
        const int r = threadIdx.x + 256 * i;
        if (r < M) {
          f4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] = is[k][j] * (gr[k][i][j] - s_mg[k][j] - xr[k][i][j] * s_mgx[k][j]);
            mx = fmaxf(mx, fabsf(o[j]));
          }
          tde_st(reinterpret_cast<f4*>(dz + (row0 + r) * C + c), o);
        }
      }
    }
  }
  if (threadIdx.x < 4 && dbeta) dbeta[c + threadIdx.x] = db;
  block_absmax_to(mx, amax);
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

// Inference-mode batch norm folded into the preceding conv (batch_prediction.py:41-44 runs disp_net with
// is_training=False): y = (conv(x, w) - mm) * rsqrt(mv + eps) + beta = conv(x, w * s) + (beta - mm * s),
// s = rsqrt(mv + eps) per output channel k.  layout 0: conv weights [taps][cin][K] (k = idx % K);
// layout 1: conv2d_transpose weights [taps][K][cin] (k = (idx / cin) % K).  fp64 scale and products.
__global__ void __launch_bounds__(256) bn_fold_kernel(long total, int cin, int K, int layout, const float* w,
                                                      const float* mm, const float* mv, const float* beta,
                                                      float eps, float* w_out, float* bias_out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int k = layout == 0 ? (int)(i % K) : (int)((i / cin) % K);
    const double s = 1.0 / sqrt((double)mv[k] + (double)eps);
    w_out[i] = (float)((double)w[i] * s);
    if (i < K) bias_out[i] = (float)((double)beta[i] - (double)mm[i] * (1.0 / sqrt((double)mv[i] + (double)eps)));
  }
}

// BN-free conv / deconv layers (nets_optflow_depth_pairtest.py:76-147: normalizer_fn commented out at :83-84,
// so slim adds biases and applies ReLU): dz = dy * relu'(y) written dense [M][C] (the conv backward's gradient
// operand), per-chunk fp64 bias sums part[chunk][C], max|dz| into the operand bound.  Grid (row chunk, group of
// 16 channel quads) as bn_part_kernel.
__global__ void __launch_bounds__(256) bias_relu_part_kernel(int M, int C, const float* y, int ycs, int yco,
                                                             const float* dy, int dycs, int dyco, int relu,
                                                             int rows_per_chunk, float* dz, double* part, float* amax) {
  __shared__ double sh[2][256 * 4];
  const int q0 = blockIdx.y * 16;
  const int nq = min(16, C / 4 - q0);
  const int ty_n = 256 / nq;
  const int tx = threadIdx.x % nq, ty = threadIdx.x / nq;
  const int c = 4 * (q0 + tx);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  float mx = 0.f;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(M, r0 + rows_per_chunk);
  if (ty < ty_n) {
    for (int rb = r0 + ty; rb < r1; rb += 64 * ty_n) {
      const int rend = min(r1, rb + 64 * ty_n);
      float f0[4] = {0, 0, 0, 0};
#pragma unroll 8
      for (int r = rb; r < rend; r += ty_n) {
        const f4 yv = *reinterpret_cast<const f4*>(y + (long)r * ycs + yco + c);
        const f4 gv = *reinterpret_cast<const f4*>(dy + (long)r * dycs + dyco + c);
        f4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = (!relu || yv[j] > 0.f) ? gv[j] : 0.f;
          f0[j] += o[j];
          mx = fmaxf(mx, fabsf(o[j]));
        }
        *reinterpret_cast<f4*>(dz + (long)r * C + c) = o;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) s0[j] += f0[j];
    }
  }
  rowlane_combine(s0, s1, nq, ty_n, &sh[0][0]);
  if (ty == 0) {
    double* o = part + (long)blockIdx.x * C;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[c + j] = s0[j];
  }
  block_absmax_to(mx, amax);
}

// dbias[c] (+)= sum over the chunk partials in chunk order (fixed order: deterministic).
__global__ void __launch_bounds__(256) bias_sum_kernel(int C, int nparts, const double* part, float* dbias, int acc) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double a[4] = {0, 0, 0, 0};
  int p = 0;
  for (; p + 3 < nparts; p += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += part[(long)(p + u) * C + c];
  }
  for (; p < nparts; ++p) a[0] += part[(long)p * C + c];
  const double s = (a[0] + a[1]) + (a[2] + a[3]);
  dbias[c] = acc ? dbias[c] + (float)s : (float)s;
}

int ew_grid(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

// apply grid: ~8 rows per row lane, <= 2048 blocks (diagnostic A/B build flags TDE_APPLY_RPL / TDE_APPLY_MAXB)
#ifndef TDE_APPLY_RPL
#define TDE_APPLY_RPL 8
#endif
#ifndef TDE_APPLY_MAXB
#define TDE_APPLY_MAXB 2048
#endif
int apply_rows_per_block(int M, int C) {
  const int cq = C / 4;
  const int rstep = cq >= 256 ? 1 : 256 / cq;
  long rpb = (long)rstep * TDE_APPLY_RPL;
  if ((M + rpb - 1) / rpb > TDE_APPLY_MAXB) rpb = (M + TDE_APPLY_MAXB - 1) / TDE_APPLY_MAXB;
  rpb = (rpb + rstep - 1) / rstep * rstep;
  return (int)rpb;
}

int finalize_blocks(int C) { return C / 4; }

// M = rows per group; nparts = all groups' partials (G | nparts, group-major)
template <int MODE>
void finalize_launch(int nparts, int C, hipStream_t st, int M, const double* part, float eps, float decay, int bessel,
                     float* mm, float* mv, float* save_mean, float* save_invstd, float* dbeta, int acc, float* coef,
                     double* sums, int G = 1, double* sums2 = nullptr) {
  if (nparts / G <= 512)
    hipLaunchKernelGGL((bn_finalize_kernel<MODE, 256>), dim3(finalize_blocks(C)), dim3(256), 0, st, M, C, nparts, part,
                       eps, decay, bessel, mm, mv, save_mean, save_invstd, dbeta, acc, coef, sums, G, sums2);
  else
    hipLaunchKernelGGL((bn_finalize_kernel<MODE, 1024>), dim3(finalize_blocks(C)), dim3(1024), 0, st, M, C, nparts,
                       part, eps, decay, bessel, mm, mv, save_mean, save_invstd, dbeta, acc, coef, sums, G, sums2);
}

}  // namespace

// ------------------------------------------------------------------ internal launchers (bn_internal.h)
// tuning knobs; a missing, non-numeric or non-positive value means the default (a 0 would divide by zero in
// bn_chunk_plan)
static long bn_env(const char* n, long d) { return tde_env_pos(n, d); }
// elements per partial-sum block and row chunks at most: 8K / 1024 (config-2 step: BN backward 473 -> 441 us
// against 16K / 256, which left the 192x256 and 96x128 layers at <= 256 blocks on 256 CUs)
static const long g_bn_elems = bn_env("TDE_BN_ELEMS", 8192);
static const long g_bn_maxch = bn_env("TDE_BN_MAXCH", 1024);

BnChunks bn_chunk_plan(long M, int C, int work_mult, int G) {
  // ~g_bn_elems elements (x work_mult, e.g. split-K slabs) per block, <= g_bn_maxch chunks; with G row groups the
  // same count split evenly over the groups (every chunk inside one group)
  BnChunks p;
  const int cq = C / 4;
  p.groups = (cq + 15) / 16;
  const int nq = cq < 16 ? cq : 16;
  const int ty_n = 256 / nq;
  if (G < 1) G = 1;
  const long Mg = M / G;
  long ch = M * (long)C * (work_mult > 1 ? work_mult : 1) / g_bn_elems / p.groups;
  if (ch > g_bn_maxch) ch = g_bn_maxch;
  ch = ch / G;
  if (ch < 1) ch = 1;
  long rpc = (Mg + ch - 1) / ch;
  rpc = (rpc + ty_n - 1) / ty_n * ty_n;
  p.rows_per_chunk = (int)rpc;
  p.per_g = (int)((Mg + rpc - 1) / rpc);
  p.Mg = (int)Mg;
  p.chunks = p.per_g * G;
  return p;
}

size_t bn_part_bytes(long M, int C) {
  // any plan of bn_chunk_plan(M, C, 1, G <= BN_MAX_GROUPS) has per_g <= max(1, ch / G) chunks per group, i.e. at
  // most max(ch, G) partials (ch = the chunk target before the per-group split)
  const long groups = (C / 4 + 15) / 16;
  long n = M * (long)C / g_bn_elems / groups;
  if (n > g_bn_maxch) n = g_bn_maxch;
  if (n < BN_MAX_GROUPS) n = BN_MAX_GROUPS;
  return (size_t)n * 2 * C * sizeof(double);
}

void bn_fwd_small_launch(int M, int C, const float* z, const BnOut& o, double* part, hipStream_t st) {
  const int G = o.groups > 1 ? o.groups : 1;
  if (o.sums) {   // SyncBN phase 1: the grouped sums only
    const BnChunks pp = bn_chunk_plan(M, C, 1, G);
    hipLaunchKernelGGL(bn_part_kernel<0>, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, z, nullptr, 0, 0,
                       nullptr, nullptr, nullptr, 0, pp, part);
    bn_fwd_from_partials_launch(M, C, z, pp.chunks, part, o, st);
    return;
  }
  if (G % 2 == 0 && TDE_SMALL_GT2)
    hipLaunchKernelGGL(bn_fwd_small_kernel<2>, dim3(C / 4), dim3(256), 0, st, M / G, C, z, o.beta, o.eps, o.decay,
                       o.bessel, o.mm, o.mv, o.save_mean, o.save_invstd, o.y, o.ycs, o.yco, o.relu, G);
  else
    hipLaunchKernelGGL(bn_fwd_small_kernel<1>, dim3(C / 4), dim3(256), 0, st, M / G, C, z, o.beta, o.eps, o.decay,
                       o.bessel, o.mm, o.mv, o.save_mean, o.save_invstd, o.y, o.ycs, o.yco, o.relu, G);
}

void bn_fwd_from_partials_launch(int M, int C, const float* z, int nparts, const double* part, const BnOut& o,
                                 hipStream_t st) {
  const int G = o.groups > 1 ? o.groups : 1;
  if (o.sums) {   // SyncBN phase 1: the per-group (sum z, sum z^2) for the caller's all-reduce; nothing applied
    finalize_launch<2>(nparts, C, st, M / G, part, 0.f, 0.f, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                       nullptr, o.sums, G);
    return;
  }
  finalize_launch<0>(nparts, C, st, M / G, part, o.eps, o.decay, o.bessel, o.mm, o.mv, o.save_mean, o.save_invstd,
                     nullptr, 0, nullptr, nullptr, G);
  const int rpb = apply_rows_per_block(M, C);
  hipLaunchKernelGGL(bn_apply_kernel<false>, dim3((M + rpb - 1) / rpb), dim3(256), 0, st, M, C, z, o.save_mean,
                     o.save_invstd, o.beta, o.relu, o.y, o.ycs, o.yco, rpb, M / G, SumsPub{});
}

void bn_fwd_standalone_launch(int M, int C, const float* z, const BnOut& o, double* part, hipStream_t st) {
  const int G = o.groups > 1 ? o.groups : 1;
  if (M / G <= BN_SMALL_M) {
    bn_fwd_small_launch(M, C, z, o, part, st);
    return;
  }
  const BnChunks pp = bn_chunk_plan(M, C, 1, G);
  hipLaunchKernelGGL(bn_part_kernel<0>, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, z, nullptr, 0, 0, nullptr,
                     nullptr, nullptr, 0, pp, part);
  bn_fwd_from_partials_launch(M, C, z, pp.chunks, part, o, st);
}

extern "C" {

size_t tde_bn_workspace_size(int M, int C) {
  if (M <= 0 || C <= 0 || C % 4) return 0;
  return bn_part_bytes(M, C) + (size_t)BN_MAX_GROUPS * 2 * C * sizeof(float) + 64;
}

int tde_bn_fwd_train(int M, int C, int groups, const float* z, const float* beta, float eps, float decay, int bessel,
                     float* moving_mean, float* moving_var, float* save_mean, float* save_invstd, float* y,
                     int y_cstride, int y_coff, int relu, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && beta && save_mean && save_invstd && y);
  TDE_CHECK_ARG(groups >= 1 && groups <= BN_MAX_GROUPS && M % groups == 0);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride && tde_aligned16(z) && tde_aligned16(y));
  TDE_CHECK_ARG((moving_mean == nullptr) == (moving_var == nullptr));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const BnOut o{beta, eps, decay, bessel, moving_mean, moving_var, save_mean, save_invstd, y, y_cstride, y_coff, relu,
                groups};
  bn_fwd_standalone_launch(M, C, z, o, reinterpret_cast<double*>(tde_ws_body(ws)), st);
  return tde_launch_status();
}

int tde_bn_fwd_infer(int M, int C, const float* z, const float* beta, float eps, const float* moving_mean,
                     const float* moving_var, float* y, int y_cstride, int y_coff, int relu, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && z && beta && moving_mean && moving_var && y);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(bn_infer_kernel, dim3(ew_grid((long)M * C / 4)), dim3(256), 0, st, M, C, z, moving_mean,
                     moving_var, eps, beta, relu, y, y_cstride, y_coff);
  return tde_launch_status();
}

int tde_bn_fold(int taps, int cin, int K, int layout, const float* w, const float* moving_mean,
                const float* moving_var, const float* beta, float eps, float* w_out, float* bias_out, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(taps > 0 && cin > 0 && K > 0 && (layout == 0 || layout == 1) && w && moving_mean && moving_var &&
                beta && w_out && bias_out && w != w_out);
  const long total = (long)taps * cin * K;
  hipLaunchKernelGGL(bn_fold_kernel, dim3(ew_grid(total)), dim3(256), 0, static_cast<hipStream_t>(stream), total, cin,
                     K, layout, w, moving_mean, moving_var, beta, eps, w_out, bias_out);
  return tde_launch_status();
}

int tde_bn_bwd(int M, int C, int groups, const float* z, const float* save_mean, const float* save_invstd,
               const float* beta, const float* dy, int dy_cstride, int dy_coff, float* dz, float* dbeta,
               int accumulate_dbeta, int relu, float* dz_absmax, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && save_mean && save_invstd && beta && dy && dz);
  TDE_CHECK_ARG(groups >= 1 && groups <= BN_MAX_GROUPS && M % groups == 0);
  TDE_CHECK_ARG(dy_cstride % 4 == 0 && dy_coff % 4 == 0 && tde_aligned16(dy) && tde_aligned16(dz));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int G = groups, Mg = M / groups;
  if (Mg <= BN_SMALL_M) {
    if (G % 2 == 0 && TDE_SMALL_GT2)
      hipLaunchKernelGGL(bn_bwd_small_kernel<2>, dim3(C / 4), dim3(256), 0, st, Mg, C, z, save_mean, save_invstd, beta,
                         dy, dy_cstride, dy_coff, dz, dbeta, accumulate_dbeta, relu, dz_absmax, G);
    else
      hipLaunchKernelGGL(bn_bwd_small_kernel<1>, dim3(C / 4), dim3(256), 0, st, Mg, C, z, save_mean, save_invstd, beta,
                         dy, dy_cstride, dy_coff, dz, dbeta, accumulate_dbeta, relu, dz_absmax, G);
    return tde_launch_status();
  }
  const BnChunks pp = bn_chunk_plan(M, C, 1, G);
  double* part = reinterpret_cast<double*>(tde_ws_body(ws));
  float* coef = reinterpret_cast<float*>(tde_ws_body(ws) + bn_part_bytes(M, C));
  hipLaunchKernelGGL(bn_part_kernel<1>, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, z, dy, dy_cstride, dy_coff,
                     save_mean, save_invstd, beta, relu, pp, part);
  finalize_launch<1>(pp.chunks, C, st, Mg, part, 0.f, 0.f, 0, nullptr, nullptr, nullptr, nullptr, dbeta, accumulate_dbeta,
                     coef, nullptr, G);
  const int rpb = apply_rows_per_block(M, C);
  hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3((M + rpb - 1) / rpb), dim3(256), 0, st, M, C, z, dy,
                     dy_cstride, dy_coff, save_mean, save_invstd, beta, coef, relu, dz, rpb, dz_absmax, Mg, SumsPub{});
  return tde_launch_status();
}


int tde_bn_sums(int M, int C, int groups, const float* z, const float* dy, int dy_cstride, int dy_coff,
                const float* save_mean, const float* save_invstd, const float* beta, int relu, int mode, double* sums,
                double* sums_copy, void* ws, size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && sums && (mode == 0 || mode == 1));
  TDE_CHECK_ARG(groups >= 1 && groups <= BN_MAX_GROUPS && M % groups == 0);
  TDE_CHECK_ARG(tde_aligned16(z) && (mode == 0 || (dy && save_mean && save_invstd && beta && tde_aligned16(dy) &&
                                                   dy_cstride % 4 == 0 && dy_coff % 4 == 0)));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const BnChunks pp = bn_chunk_plan(M, C, 1, groups);
  double* part = reinterpret_cast<double*>(tde_ws_body(ws));
  if (mode == 0)
    hipLaunchKernelGGL(bn_part_kernel<0>, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, z, nullptr, 0, 0,
                       nullptr, nullptr, nullptr, 0, pp, part);
  else
    hipLaunchKernelGGL(bn_part_kernel<1>, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, z, dy, dy_cstride,
                       dy_coff, save_mean, save_invstd, beta, relu, pp, part);
  finalize_launch<2>(pp.chunks, C, st, M / groups, part, 0.f, 0.f, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                     nullptr, sums, groups, sums_copy);
  return tde_launch_status();
}

int tde_bn_fwd_from_sums(int M, int C, int groups, long M_total, const float* z, const double* sums, const float* beta,
                         float eps, float decay, int bessel, float* moving_mean, float* moving_var, float* save_mean,
                         float* save_invstd, float* y, int y_cstride, int y_coff, int relu, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(groups >= 1 && groups <= BN_MAX_GROUPS && M % groups == 0 && M_total >= M / groups);
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && sums && beta && save_mean && save_invstd && y);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride && tde_aligned16(z) &&
                tde_aligned16(y) && (moving_mean == nullptr) == (moving_var == nullptr));
  hipStream_t st = static_cast<hipStream_t>(stream);
  SumsPub P{};
  P.sums = sums; P.Mt = (double)M_total; P.eps = eps; P.decay = decay; P.bessel = bessel; P.G = groups;
  P.mm = moving_mean; P.mv = moving_var; P.save_mean = save_mean; P.save_invstd = save_invstd;
  const int rpb = apply_rows_per_block(M, C);
  hipLaunchKernelGGL(bn_apply_kernel<true>, dim3((M + rpb - 1) / rpb), dim3(256), 0, st, M, C, z, nullptr, nullptr,
                     beta, relu, y, y_cstride, y_coff, rpb, M / groups, P);
  return tde_launch_status();
}

int tde_bn_bwd_from_sums(int M, int C, int groups, long M_total, const float* z, const float* save_mean,
                         const float* save_invstd, const float* beta, const float* dy, int dy_cstride, int dy_coff,
                         const double* global_sums, const double* local_sums, float* dz, float* dbeta,
                         int accumulate_dbeta, int relu, float* dz_absmax, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(groups >= 1 && groups <= BN_MAX_GROUPS && M % groups == 0 && M_total >= M / groups);
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && z && save_mean && save_invstd && beta && dy && dz &&
                global_sums && local_sums);
  TDE_CHECK_ARG(dy_cstride % 4 == 0 && dy_coff % 4 == 0 && tde_aligned16(dy) && tde_aligned16(dz));
  hipStream_t st = static_cast<hipStream_t>(stream);
  SumsPub P{};
  P.sums = global_sums; P.lsums = local_sums; P.Mt = (double)M_total; P.G = groups; P.acc = accumulate_dbeta;
  P.dbeta = dbeta;
  const int rpb = apply_rows_per_block(M, C);
  hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3((M + rpb - 1) / rpb), dim3(256), 0, st, M, C, z, dy, dy_cstride,
                     dy_coff, save_mean, save_invstd, beta, nullptr, relu, dz, rpb, dz_absmax, M / groups, P);
  return tde_launch_status();
}

int tde_bias_relu_bwd(int M, int C, const float* y, int y_cstride, int y_coff, const float* dy, int dy_cstride,
                      int dy_coff, int relu, float* dz, float* dbias, int accumulate_dbias, float* dz_absmax, void* ws,
                      size_t ws_bytes, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(M > 0 && C > 0 && C % 4 == 0 && C <= 1024 && y && dy && dz && dbias);
  TDE_CHECK_ARG(y_cstride % 4 == 0 && y_coff % 4 == 0 && y_coff + C <= y_cstride && dy_cstride % 4 == 0 &&
                dy_coff % 4 == 0 && dy_coff + C <= dy_cstride);
  TDE_CHECK_ARG(tde_aligned16(y) && tde_aligned16(dy) && tde_aligned16(dz));
  if (ws_bytes < tde_bn_workspace_size(M, C) || !ws || !tde_aligned16(ws)) return TDE_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const BnChunks pp = bn_chunk_plan(M, C, 1);
  double* part = reinterpret_cast<double*>(tde_ws_body(ws));
  hipLaunchKernelGGL(bias_relu_part_kernel, dim3(pp.chunks, pp.groups), dim3(256), 0, st, M, C, y, y_cstride, y_coff,
                     dy, dy_cstride, dy_coff, relu, pp.rows_per_chunk, dz, part, dz_absmax);
  hipLaunchKernelGGL(bias_sum_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, pp.chunks, part, dbias,
                     accumulate_dbias);
  return tde_launch_status();
}

}  // extern "C"
