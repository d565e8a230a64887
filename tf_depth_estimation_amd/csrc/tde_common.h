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

// the HIP error behind the calling thread's last TDE_ERR_HIP (named by tde_status_string)
extern thread_local int tde_g_last_hip;

// Launch status of an ABI entry: every entry point that launches starts with tde_clear_error(), which drops
// whatever another library left in the calling thread's last-error slot (an event query's hipErrorNotReady from
// the framework's allocator or the collective layer, any other stale code), so tde_launch_status() at its end
// reports exactly the launches of this call.  (Round 4 whitelisted hipErrorNotReady after the fact instead: any
// other stale code still failed a capture, and a real failure could be read as someone else's.)
static inline void tde_clear_error() { (void)hipGetLastError(); }
static inline int tde_launch_status() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return TDE_OK;
  tde_g_last_hip = (int)e;
  return TDE_ERR_HIP;
}

static inline bool tde_aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static inline int tde_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

static inline char* tde_ws_body(void* ws) { return static_cast<char*>(ws); }

// Tuning knob that must be positive (tile counts, chunk sizes, block caps): a missing, non-numeric, zero or
// negative value means the default, so a bad setting can neither divide by zero nor empty a grid.
#include <cstdlib>
static inline long tde_env_pos(const char* name, long dflt) {
  const char* v = std::getenv(name);
  const long x = v ? std::atol(v) : 0L;
  return x > 0 ? x : dflt;
}

// Raw buffer resource over n floats (byte range clamped below 2^31 so OOB is always out of range;
// 0x00020000 = DATA_FORMAT 32 for gfx9-family raw buffers).  An access at byte offset OOB reads zero:
// branch-free predicated loads.
constexpr int OOB = (int)0x80000000;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, long n) {
  const long bytes = 4 * n;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0,
                                           (int)(bytes < 0x7fffffffl ? bytes : 0x7fffffffl), 0x00020000);
}
__device__ __forceinline__ f4 bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// XCD-contiguous logical block index: the hardware deals blocks round-robin over the 8 XCDs (each with its
// own L2), so logical blocks [x*q + min(x, r), ...) of XCD x = physical b with b % 8 == x.  A bijection for any
// nb; used where neighbouring blocks read neighbouring 16-byte pieces of the same cache lines (per-channel-quad
// BatchNorm kernels), so a line is pulled into one L2 instead of eight.  Placement is a speed hint only.
__device__ __forceinline__ int tde_xcd_block(int b, int nb) {
  const int x = b & 7, q = nb >> 3, r = nb & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// Output stores of the big producer kernels (conv epilogues, split-K slabs and reduces, BatchNorm apply passes).
// (Round 4's TDE_NT_STORES build flag -- non-temporal stores -- measured slower and was removed in round 5.)
template <typename T>
__device__ __forceinline__ void tde_st(T* p, T v) {
  *p = v;
}

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
