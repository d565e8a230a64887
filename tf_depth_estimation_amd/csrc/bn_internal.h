// Batch-norm launchers shared between bn.hip and the conv translation unit (conv_igemm.hip), which
// produces the BN statistics partials itself (conv epilogue, or its split-K reduce) for a fused
// conv + BN + ReLU layer.
#pragma once
#include "tde_common.h"

#ifndef TDE_BN_SMALL_M   // diagnostic A/B build flag
#define TDE_BN_SMALL_M 512
#endif
constexpr int BN_SMALL_M = TDE_BN_SMALL_M;   // rows (per row group) of the single-kernel BN path
constexpr int BN_MAX_GROUPS = 8;   // row groups of a grouped BN (tde_bn_train_t.groups)

// What a training-mode BN forward writes: statistics, moving averages (mm/mv null: no update) and
// y = relu?((z - mean) * invstd + beta) into a channel view.  groups G >= 1: the M rows are G equal consecutive
// row groups, each normalised over its own rows (G slim.batch_norm calls of one shared-variable network batched
// into one launch); save_mean / save_invstd are [G][C] and the moving averages take G updates in group order.
struct BnOut {
  const float* beta;
  float eps, decay;
  int bessel;
  float *mm, *mv, *save_mean, *save_invstd;
  float* y;
  int ycs, yco, relu;
  int groups;
  double* sums = nullptr;   // SyncBN phase 1 (tde_bn_train_t.sums): the per-group sums only, nothing applied
};

// Row-chunk x 64-channel-group grid of the partial-statistics passes (bn.hip and the conv's split-K
// reduce): `chunks` fp64 partials [chunk][2][C]; with row groups, `per_g` chunks per group of Mg rows (chunk
// k covers rows (k / per_g) * Mg + (k % per_g) * rows_per_chunk .. of its group), so every partial belongs to
// exactly one group and group g owns partials [g * per_g, (g + 1) * per_g).
struct BnChunks {
  int chunks, rows_per_chunk, groups;
  int per_g, Mg;
};
BnChunks bn_chunk_plan(long M, int C, int work_mult, int G = 1);
__device__ __forceinline__ void bn_chunk_rows(const BnChunks& p, int k, int& r0, int& r1) {
  const int gi = k / p.per_g, kk = k - gi * p.per_g;
  r0 = gi * p.Mg + kk * p.rows_per_chunk;
  r1 = min(gi * p.Mg + p.Mg, r0 + p.rows_per_chunk);
}
// fp64 partial bytes a grouped standalone forward / backward BN of M rows x C channels may use
size_t bn_part_bytes(long M, int C);

// Mg <= BN_SMALL_M: statistics + finalize + apply in one launch.
void bn_fwd_small_launch(int M, int C, const float* z, const BnOut& o, double* part, hipStream_t st);
// From `nparts` fp64 partials [part][2][C] of z (G | nparts, group-aligned): finalize (one small launch) + apply
// (one launch).
void bn_fwd_from_partials_launch(int M, int C, const float* z, int nparts, const double* part, const BnOut& o,
                                 hipStream_t st);
// The whole training-mode forward BN of z (partials computed here): small path or partials + finalize + apply.
void bn_fwd_standalone_launch(int M, int C, const float* z, const BnOut& o, double* part, hipStream_t st);

// Row-lane combine of the partial-sum kernels (bn_part_kernel, splitk_reduce_bn_kernel): thread = ty * nq + tx
// (256 threads, nq channel quads), s0 / s1 its 4-channel sums.  Leaves the block's sums for quad tx in the
// threads with ty == 0 (tid < nq), combined in a fixed order: an xor-shuffle tree over a wave's row lanes and
// one LDS level over the 4 waves when nq is a power of two (64 % nq == 0), else the serial LDS loop.
__device__ __forceinline__ void rowlane_combine(double (&s0)[4], double (&s1)[4], int nq, int ty_n,
                                                double* sh /* [2][256*4] */) {
  const int tid = threadIdx.x;
  if ((nq & (nq - 1)) == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      for (int o = nq; o < 64; o <<= 1) {
        s0[j] += __shfl_xor(s0[j], o, 64);
        s1[j] += __shfl_xor(s1[j], o, 64);
      }
    const int lane = tid & 63, wv = tid >> 6;
    if (lane < nq) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { sh[(wv * 16 + lane) * 4 + j] = s0[j]; sh[1024 + (wv * 16 + lane) * 4 + j] = s1[j]; }
    }
    __syncthreads();
    if (tid < nq) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0[j] = sh[tid * 4 + j]; s1[j] = sh[1024 + tid * 4 + j];
        for (int w = 1; w < 4; ++w) { s0[j] += sh[(w * 16 + tid) * 4 + j]; s1[j] += sh[1024 + (w * 16 + tid) * 4 + j]; }
      }
    }
    return;
  }
  const int tx = tid % nq;
#pragma unroll
  for (int j = 0; j < 4; ++j) { sh[tid * 4 + j] = s0[j]; sh[1024 + tid * 4 + j] = s1[j]; }
  __syncthreads();
  if (tid < nq) {
    for (int t = 1; t < ty_n; ++t) {
      const int o = (t * nq + tx) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) { s0[j] += sh[o + j]; s1[j] += sh[1024 + o + j]; }
    }
  }
}
