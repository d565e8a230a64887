// Internal helpers shared by the HIP translation units of libtde.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tde.h"

typedef float f4 __attribute__((ext_vector_type(4)));

#define TDE_CHECK_ARG(cond)            \
  do {                                 \
    if (!(cond)) return TDE_ERR_ARG;   \
  } while (0)

static inline int tde_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? TDE_OK : TDE_ERR_HIP;
}

static inline bool tde_aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static inline int tde_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Every workspace starts with TDE_WS_HEADER_BYTES of uint32 arrival counters (include/tde.h): the
// deterministic "last block reduces" steps of the conv and BN kernels count tile arrivals there and
// reset their counter to zero before exiting, so a workspace zeroed once stays valid for every call.
constexpr size_t TDE_WS_HDR = TDE_WS_HEADER_BYTES;
constexpr int TDE_CNT_SPLIT = 0;        // [0, 8192): split-K tiles of one conv launch
constexpr int TDE_CNT_SPLIT_MAX = 8192;
constexpr int TDE_CNT_BN = 8192;        // [8192, 16384): BN statistics groups and column tiles
constexpr int TDE_CNT_BN_MAX = 8192;
static inline unsigned* tde_ws_counters(void* ws) { return static_cast<unsigned*>(ws); }
static inline char* tde_ws_body(void* ws) { return static_cast<char*>(ws) + TDE_WS_HDR; }

__device__ __forceinline__ float tde_sign(float x) { return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f); }

// Block-wide sum of a double (blockDim.x == 256), result valid in thread 0.
__device__ __forceinline__ double tde_block_sum_d(double v, double* sh /*[4]*/) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) r += sh[i];
  }
  return r;
}
