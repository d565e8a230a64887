// Batch-norm launchers shared between bn.hip and the conv translation unit (conv_igemm.hip), which
// produces the BN statistics partials itself (conv epilogue, or its split-K reduce) for a fused
// conv + BN + ReLU layer.
#pragma once
#include "tde_common.h"

constexpr int BN_SMALL_M = 2048;   // rows of the single-kernel BN path

// What a training-mode BN forward writes: statistics, moving averages (mm/mv null: no update) and
// y = relu?((z - mean) * invstd + beta) into a channel view.
struct BnOut {
  const float* beta;
  float eps, decay;
  int bessel;
  float *mm, *mv, *save_mean, *save_invstd;
  float* y;
  int ycs, yco, relu;
};

// Row-chunk x 64-channel-group grid of the partial-statistics passes (bn.hip and the conv's split-K
// reduce): `chunks` fp64 partials [chunk][2][C].
struct BnChunks {
  int chunks, rows_per_chunk, groups;
};
BnChunks bn_chunk_plan(long M, int C, int work_mult);

// M <= BN_SMALL_M: statistics + finalize + apply in one launch.
void bn_fwd_small_launch(int M, int C, const float* z, const BnOut& o, hipStream_t st);
// From `nparts` fp64 partials [part][2][C] of z: finalize (one small launch) + apply (one launch).
void bn_fwd_from_partials_launch(int M, int C, const float* z, int nparts, const double* part, const BnOut& o,
                                 hipStream_t st);
