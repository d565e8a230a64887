// Halo-tiled stride-1 convolution on bf16x6 MFMA (gfx950).
//
// Replaces TF's Conv2D / Conv2DBackpropInput for the stride-1, few-channel, high-resolution layers of
// the reference networks (cnv1b 7x7 32->32 @96x128, cnv2b 5x5 @48x64, icnv1/icnv2/icnv3 3x3 on the
// decoder concats; nets_optflow_depth.py:89-141).  There the
// implicit GEMM (conv_igemm.hip) re-gathers its im2col operand once per 32-deep k-tile: every input
// pixel crosses L2 -> LDS KH*KW times (49x for cnv1b), and that traffic, not the MFMAs, sets the time.
//
// Here a block owns a (2*NW) x 16 output-pixel tile of one image and 16*TN output columns:
//   1. its input halo ((2*NW + KH - 1) x (16 + KW - 1) pixels x one channel chunk) is loaded ONCE,
//      split into exact bf16 hi/mid/lo planes (split_math.h) and kept in LDS for all KH*KW taps;
//   2. the weights, pre-split by halo_wprep_kernel into [k-step][plane][column][32] bf16 tiles, stream
//      through a double-buffered LDS slot, one 32-deep k-step per barrier;
//   3. each wave owns two 16-pixel rows x all TN column fragments: per k-step it reads its A fragments
//      straight out of the halo (row = pixel + tap offset) and issues 6 v_mfma_f32_16x16x32_bf16 per
//      fragment pair (the bf16x6 product, fp32 accumulation).
// The reduction index is (chunk, tap, channel-in-chunk) with the chunk width a multiple of 8, so the 8
// consecutive k of one MFMA lane never straddle a tap.  DGRAD is the same kernel on dy with the taps
// flipped, the pads mirrored and the weights transposed (done by the prep kernel).  Optional fp64 BN
// statistics partials (one per pixel tile) feed bn_fwd_from_partials_launch exactly like the
// implicit GEMM's epilogue partials.
#include "halo_conv.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "split_math.h"

namespace {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;
// LDS row strides: a 16-lane group of ds_read_b128 fragment reads (rows r16, 16-byte column q) is
// conflict-free when the row stride in 16-byte units is 2 mod 4 (gfx950 lane groups {0-3,12-15,20-27},
// ...; an odd stride such as 80 B costs 2 cycles per group -- measured SQ_LDS_BANK_CONFLICT = 50% of the
// LDS cycles).  B rows: 32 k + 16 pad = 96 bytes.
constexpr int LDB = 48;

struct HaloArgs {
  int N, H, W;
  int HWd, HP, CC, nch, SA, steps, ntap, KW, PT, PL;
  int Cv, ics, ico, Ncols, ocs, oco, ncolt, NcolsP;
  int accumulate;
  int swz;             // halo row layout: 0 padded rows (SA from lds_stride); 4 / 8 = 16-byte chunks per row, XOR-swizzled
  FDiv fCC, fKW, fC4, fHWd;
  const float* in;
  float* out;
  const u16* wp;
  double* bnp;
  const float* bias;   // folded-BN inference epilogue (accumulate == 0); null / 0: plain conv
  int relu;
  const float* inmax;  // fp16x3 (math 4): bounds of the input view and of the weights (split_math.h)
  const float* wmax;
};

// Split weights, one contiguous B tile per (k-step g, column tile ct):
//   wp[(((g * ncolt + ct) * 3 + plane) * NCP + cl) * LDB + rl]   (rl < 32; rl 32..47 = 0, the LDS row pad)
// g = chunk * steps + step, r = step * 32 + rl = tap * CC + cc within the chunk, reduction channel
// c = chunk * CC + cc, column col = ct * NCP + cl:
//   FWD  : B[(tap, c)][col] = w[tap][c][col]                     (w [KH][KW][wcin][K], c < wcin)
//   DGRAD: B[(tap, k)][col] = w[ntap - 1 - tap][col][k]          (col = dx channel < wcin, k < K)
// The tile is copied byte-for-byte into its LDS ring slot by LDS-DMA, so this IS the LDS image.
//   planes 3: bf16x6 hi / mid / lo (split3); planes 2: fp16x3 hi / lo of w * f16x3_scale(wmax) (split4x2h)
struct WprepJob {
  const float* w;
  u16* wp;
  const float* wmax;
  long total;
  int block0, nblocks;    // the job's blocks in a batched launch
  int mode, steps, CC, ntap, Cred, Ncols, NCP, ncolt, wcin, K, planes;
};
constexpr int WPREP_MAXJ = 16;
struct WprepBatch {
  int njobs;
  WprepJob j[WPREP_MAXJ];
};

__device__ __forceinline__ void wprep_elem(const WprepJob& J, float ws, long idx) {
  const float* __restrict__ w = J.w;
  u16* __restrict__ wp = J.wp;
  const int mode = J.mode, steps = J.steps, CC = J.CC, ntap = J.ntap, Cred = J.Cred, Ncols = J.Ncols;
  const int NCP = J.NCP, ncolt = J.ncolt, wcin = J.wcin, K = J.K, planes = J.planes;
  {
    const int rl = (int)(idx % LDB);
    long t = idx / LDB;
    const int cl = (int)(t % NCP);
    t /= NCP;
    const int ct = (int)(t % ncolt);
    const int g = (int)(t / ncolt);
    const int col = ct * NCP + cl;
    const int ch = g / steps, s = g - ch * steps;
    const int r = s * 32 + rl, tap = r / CC, cc = r - tap * CC, c = ch * CC + cc;
    float v = 0.f;
    if (rl < 32 && tap < ntap && c < Cred && col < Ncols) {   // rl 32..47: LDS row pad
      if (mode == 0) v = w[((long)tap * wcin + c) * K + col];
      else if (col < wcin) v = w[((long)(ntap - 1 - tap) * wcin + col) * K + c];
    }
    const long base = ((((long)g * ncolt + ct) * planes) * NCP + cl) * LDB + rl;
    if (planes == 2) {
      const float x = v * ws;
      const _Float16 h = (_Float16)x, l = (_Float16)(x - (float)h);
      wp[base] = __builtin_bit_cast(u16, h);
      wp[base + (long)NCP * LDB] = __builtin_bit_cast(u16, l);
    } else {
      unsigned h, m, l;
      split3(v, h, m, l);
      wp[base] = (u16)(h >> 16);
      wp[base + (long)NCP * LDB] = (u16)(m >> 16);
      wp[base + 2l * NCP * LDB] = (u16)(l >> 16);
    }
  }
}

__global__ void __launch_bounds__(256) halo_wprep_kernel(const WprepJob J) {
  const float ws = J.planes == 2 ? f16x3_scale(J.wmax, F16X3_WSCALE) : 1.f;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < J.total; idx += (long)gridDim.x * 256)
    wprep_elem(J, ws, idx);
}

// Several layers' splits in one launch (tde_conv2d_split_weights): a block works on ONE job (block ranges).
__global__ void __launch_bounds__(256) halo_wprep_batch_kernel(const WprepBatch B) {
  int k = 0;
  while (k + 1 < B.njobs && (int)blockIdx.x >= B.j[k + 1].block0) ++k;
  const WprepJob& J = B.j[k];
  const float ws = J.planes == 2 ? f16x3_scale(J.wmax, F16X3_WSCALE) : 1.f;
  for (long idx = (long)(blockIdx.x - J.block0) * 256 + threadIdx.x; idx < J.total; idx += (long)J.nblocks * 256)
    wprep_elem(J, ws, idx);
}

// 16-byte chunk `chunk` of halo row `row` (u16 offset within the row).  Padded layout (swz 0): rows of SA u16 whose
// 16-byte count is 2 mod 4.  Swizzled layouts (round 6, fp16x3): rows of exactly 4 / 8 chunks (SA 32 / 64), chunk ^
// (row >> 1) & 3 or chunk ^ row & 7 -- conflict-free for the fragment reads of every tap shift (bank model over
// gfx950's ds_read_b128 lane groups), with 1/3 (32 channels) / 1/5 (64) less LDS per halo row than
// the padding, so e.g. cnv1b's 7x7 blocks fit two per CU.
__device__ __forceinline__ int halo_chunk_off(int swz, int row, int chunk) {
  const int x = swz == 8 ? (row & 7) : (swz == 4 ? ((row >> 1) & 3) : 0);
  return 8 * (chunk ^ x);
}

// Workgroup barrier that waits only for this wave's LDS operations.  __syncthreads() is a release/acquire
// fence + s_barrier, and the fence makes the compiler drain every outstanding global load (vmcnt(0))
// first, which would retire the weight-tile DMAs still in flight.  The "memory" clobber keeps the
// compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// MATH 3: bf16x6 (three bf16 planes, 6 MFMAs per fragment pair); MATH 4: fp16x3 (two fp16 planes, 3 MFMAs)
template <int NW, int TN, int MATH>
__global__ void __launch_bounds__(64 * NW) halo_conv_kernel(const HaloArgs p) {
  extern __shared__ __attribute__((aligned(16))) u16 lds[];
  constexpr int PL = MATH == 4 ? 2 : 3;                      // planes
  constexpr int NT = 64 * NW, NCP = 16 * TN;
  constexpr int BPL = NCP * LDB, BTILE = PL * BPL;          // u16 per B tile
  constexpr int NI = (BTILE * 2 + 1023) / 1024;             // 1-KiB DMA wave-instructions per tile
  constexpr int DI = (NI + NW - 1) / NW;                    // per wave (uniform: extra ones duplicate)
  constexpr int BSLOT = NI * 512;                           // u16 per ring slot (whole 1-KiB pieces)
  constexpr int NSLOT = 3;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r16 = lane & 15, q = lane >> 4;
  const int x0 = blockIdx.x * 16, y0 = blockIdx.y * (2 * NW);
  const int n = blockIdx.z / p.ncolt, ct = blockIdx.z - n * p.ncolt;
  const int col0 = ct * NCP;
  const int PLANE = p.HP * p.SA;
  u16* const As = lds;
  u16* const Bs = lds + PL * PLANE;
  const float sIn = MATH == 4 ? f16x3_scale(p.inmax, 1.f) : 1.f;
  const float sW = MATH == 4 ? f16x3_scale(p.wmax, F16X3_WSCALE) : 1.f;
  const __amdgpu_buffer_rsrc_t rin = make_rsrc(p.in, (long)p.N * p.H * p.W * p.ics);

  // B tiles reach their ring slot by LDS-DMA (global_load_lds_dwordx4: each wave-instruction copies 1 KiB,
  // lane i -> slot + 16 i); the tile of step s + 2 is issued while step s computes, and a counted
  // vmcnt wait + raw barrier retires one tile per step, so two tiles stay in flight across barriers.
  // Lanes past the tile re-read its last 16 bytes into the slot's tail padding.
  auto dma_b = [&](int g, int slot) __attribute__((always_inline)) {
    const u16* src = p.wp + ((long)g * p.ncolt + ct) * BTILE;
#pragma unroll
    for (int j = 0; j < DI; ++j) {
      const int piece = min(wv + j * NW, NI - 1);
      const int off = min((piece * 64 + lane) * 8, BTILE - 8);   // u16
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + off), (lds_ptr_t)(Bs + slot * BSLOT + piece * 512), 16, 0,
                                       0);
    }
  };

  // halo of channel chunk ch -> PL split planes [HP][SA]; 8 loads in flight per thread
  auto stage_a = [&](int ch) __attribute__((always_inline)) {
    const int nc4 = p.CC >> 2, total = p.HP * nc4;
    for (int base = 0; base < total; base += 8 * NT) {
      f4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * NT + tid;
        const int hp = fdiv(idx, p.fC4), c4 = idx - hp * nc4;
        const int hy = fdiv(hp, p.fHWd), hx = hp - hy * p.HWd;
        const int iy = y0 - p.PT + hy, ix = x0 - p.PL + hx, c = ch * p.CC + 4 * c4;
        const bool ok = idx < total && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && c < p.Cv;
        v[u] = bload(rin, ok ? 4 * (((n * p.H + iy) * p.W + ix) * p.ics + p.ico + c) : OOB);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int idx = base + u * NT + tid;
        if (idx < total) {
          const int hp = fdiv(idx, p.fC4), c4 = idx - hp * nc4;
          u16* d = As + hp * p.SA + halo_chunk_off(p.swz, hp, c4 >> 1) + 4 * (c4 & 1);
          if constexpr (MATH == 4) {
            h4 hi, lo;
            split4x2h(v[u], sIn, hi, lo);
            *reinterpret_cast<h4*>(d) = hi;
            *reinterpret_cast<h4*>(d + PLANE) = lo;
          } else {
            uint2 hi, mi, lo;
            split4x3(v[u], hi, mi, lo);
            *reinterpret_cast<uint2*>(d) = hi;
            *reinterpret_cast<uint2*>(d + PLANE) = mi;
            *reinterpret_cast<uint2*>(d + 2 * PLANE) = lo;
          }
        }
      }
    }
  };

  f4 acc[2][TN];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};

  // halo row of this lane's A fragment rows at tap (0, 0): pixel rows 2*wv + a, column r16
  const int hrow0 = (2 * wv) * p.HWd + r16, hrow1 = hrow0 + p.HWd;

  // one k-step s from ring slot `slot`
  auto compute = [&](int s, int slot) __attribute__((always_inline)) {
    // reduction index of this lane's 8 k: tap and channel in the chunk (k past the taps: weights are 0)
    const int r0 = s * 32 + 8 * q;
    int tap = fdiv(r0, p.fCC), cc = r0 - tap * p.CC;
    if (tap >= p.ntap) { tap = 0; cc = 0; }
    const int kh = fdiv(tap, p.fKW), kw = tap - kh * p.KW;
    const int trow = kh * p.HWd + kw;
    if constexpr (MATH == 4) {
      h8 ah[2], al[2], bh[TN], bl[TN];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int row = (a ? hrow1 : hrow0) + trow;
        const u16* src = As + row * p.SA + halo_chunk_off(p.swz, row, cc >> 3);
        ah[a] = *reinterpret_cast<const h8*>(src);
        al[a] = *reinterpret_cast<const h8*>(src + PLANE);
      }
      const u16* bsrc = Bs + slot * BSLOT + r16 * LDB + 8 * q;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        bh[b] = *reinterpret_cast<const h8*>(bsrc + b * 16 * LDB);
        bl[b] = *reinterpret_cast<const h8*>(bsrc + BPL + b * 16 * LDB);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
      return;
    }
    bf8 ah[2], am[2], al[2], bh[TN], bm[TN], bl[TN];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const u16* src = As + ((a ? hrow1 : hrow0) + trow) * p.SA + cc;   // (padded rows only: swz 0 in bf16x6)
      ah[a] = *reinterpret_cast<const bf8*>(src);
      am[a] = *reinterpret_cast<const bf8*>(src + PLANE);
      al[a] = *reinterpret_cast<const bf8*>(src + 2 * PLANE);
    }
    const u16* bsrc = Bs + slot * BSLOT + r16 * LDB + 8 * q;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      bh[b] = *reinterpret_cast<const bf8*>(bsrc + b * 16 * LDB);
      bm[b] = *reinterpret_cast<const bf8*>(bsrc + BPL + b * 16 * LDB);
      bl[b] = *reinterpret_cast<const bf8*>(bsrc + 2 * BPL + b * 16 * LDB);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[a], bm[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[a], bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bm[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
      }
  };

  for (int ch = 0; ch < p.nch; ++ch) {
    const int g0 = ch * p.steps, gl = g0 + p.steps - 1;
    if (ch > 0) {
      vm_wait<0>();     // the previous chunk's trailing DMAs have landed before their slots are reused
      lds_barrier();    // and nobody still reads its halo or slots
    }
    dma_b(g0, 0);
    dma_b(min(g0 + 1, gl), 1);
    stage_a(ch);        // its loads are younger than the two DMAs and waited for inside
    vm_wait<DI>();      // this wave's part of tile 0 has landed (tile 1 may still fly)
    lds_barrier();
    int slot = 0;
    for (int s = 0; s < p.steps; ++s) {
      // slot (slot + 2) % 3 was read by step s - 1, which every wave finished before the last barrier
      dma_b(min(g0 + s + 2, gl), slot == 0 ? 2 : slot - 1);
      compute(s, slot);
      vm_wait<DI>();    // tile s + 1 landed (tile s + 2 may still fly)
      lds_barrier();
      slot = slot == 2 ? 0 : slot + 1;
    }
  }
  vm_wait<0>();
  if constexpr (MATH == 4) {
    const float inv = 1.f / (sIn * sW);   // power of two: exact
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] *= inv;
  }

  // ---- epilogue: acc[a][b][r] = out(pixel (y0 + 2*wv + a, x0 + 4q + r), column col0 + 16b + r16)
  bool rowok[2][4];
  long rowaddr[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int y = y0 + 2 * wv + a, x = x0 + 4 * q + r;
      rowok[a][r] = y < p.H && x < p.W;
      rowaddr[a][r] = ((long)(n * p.H + y) * p.W + x) * p.ocs + p.oco;
    }
  if (p.bnp != nullptr) {
    // fp64 BN statistics partial of this pixel tile, per column (the main loop ended with a barrier)
    float* red = reinterpret_cast<float*>(lds);   // [2][NW][NCP]
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      float cs = 0.f, cq = 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = rowok[a][r] ? acc[a][b][r] : 0.f;
          cs += v; cq += v * v;
        }
      cs += __shfl_xor(cs, 16, 64); cq += __shfl_xor(cq, 16, 64);
      cs += __shfl_xor(cs, 32, 64); cq += __shfl_xor(cq, 32, 64);
      if (lane < 16) {
        red[wv * NCP + b * 16 + lane] = cs;
        red[(NW + wv) * NCP + b * 16 + lane] = cq;
      }
    }
    __syncthreads();
    if (tid < NCP && col0 + tid < p.Ncols) {
      double sv = 0.0, sq = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) { sv += red[w * NCP + tid]; sq += red[(NW + w) * NCP + tid]; }
      const long j = ((long)n * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
      p.bnp[j * 2 * p.Ncols + col0 + tid] = sv;
      p.bnp[j * 2 * p.Ncols + p.Ncols + col0 + tid] = sq;
    }
  }
  if (p.accumulate) {
    // every old value in flight before the first add (branch-free buffer loads; invalid -> 0, unused)
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(p.out, (long)p.N * p.H * p.W * p.ocs);
    float old[2][4][TN];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int col = col0 + b * 16 + r16;
          const bool ok = rowok[a][r] && col < p.Ncols;
          old[a][r][b] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rout, ok ? (int)(4 * (rowaddr[a][r] + col)) : OOB, 0, 0));
        }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b][r] += old[a][r][b];
  }
  if (p.bias || p.relu) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = col0 + b * 16 + r16;
      const float bv = (p.bias && col < p.Ncols) ? p.bias[col] : 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[a][b][r] + bv;
          acc[a][b][r] = (p.relu && v < 0.f) ? 0.f : v;
        }
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = col0 + b * 16 + r16;
        if (rowok[a][r] && col < p.Ncols) tde_st(p.out + rowaddr[a][r] + col, acc[a][b][r]);
      }
}

long env_l(const char* name, long dflt) {
  const char* v = getenv(name);
  return v ? atol(v) : dflt;
}
const long g_halo = env_l("TDE_HALO", 1);                 // 0: never take the halo path (A/B)
const long g_halo_min_m = tde_env_pos("TDE_HALO_MIN_M", 8192);  // output pixels (N*H*W) from which it pays (r04: 16384 -> 8192, +0.5 %)
const long g_halo_nw = env_l("TDE_HALO_NW", 0);           // force 4 or 8 waves per block
const long g_halo_tn = env_l("TDE_HALO_TN", 0);           // force 1-4 column fragments per wave (A/B)
const long g_halo_verbose = env_l("TDE_HALO_VERBOSE", 0); // print every plan to stderr (tuning runs)
const long g_halo_lds = tde_env_pos("TDE_HALO_LDS_KB", 150) << 10;
const long g_halo_minch = tde_env_pos("TDE_HALO_MINCH", 1);     // force at least this many channel chunks
const long g_halo_swz = env_l("TDE_HALO_SWZ", 1);         // 0: padded halo rows only (A/B)

int lds_stride(int cc) {   // smallest row stride (u16) >= cc whose 16-byte count is 2 mod 4
  int s = cc;
  while ((s / 8) % 4 != 2) s += 8;
  return s;
}

template <int NW, int TN, int MATH>
void launch_m(const HaloPlan& hp, const HaloArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&halo_conv_kernel<NW, TN, MATH>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((halo_conv_kernel<NW, TN, MATH>), dim3(hp.gx, hp.gy, hp.gz), dim3(64 * NW), hp.lds_bytes, st,
                     a);
}
template <int NW, int TN>
void launch_t(const HaloPlan& hp, const HaloArgs& a, hipStream_t st) {
  if (hp.planes == 2) launch_m<NW, TN, 4>(hp, a, st);
  else launch_m<NW, TN, 3>(hp, a, st);
}

}  // namespace

bool halo_plan(const tde_conv_desc_t& d, int mode, int math, HaloPlan& hp) {
  hp = HaloPlan{};
  if (!g_halo || (math != 2 && math != 3 && math != 4) || d.stride != 1 || (mode != 0 && mode != 1)) return false;
  if (d.OH != d.H || d.OW != d.W || (long)d.N * d.H * d.W < g_halo_min_m) return false;
  hp.mode = mode;
  hp.planes = math == 4 ? 2 : 3;
  hp.KH = d.KH; hp.KW = d.KW;
  if (mode == 0) {
    hp.PT = d.pad_top; hp.PL = d.pad_left;
    hp.Cv = d.C; hp.ics = d.x_cstride; hp.ico = d.x_coff; hp.Cred = d.w_cin;
    hp.Ncols = d.K; hp.ocs = d.y_cstride; hp.oco = d.y_coff;
  } else {
    hp.PT = d.KH - 1 - d.pad_top; hp.PL = d.KW - 1 - d.pad_left;
    hp.Cv = d.K; hp.ics = d.y_cstride; hp.ico = d.y_coff; hp.Cred = d.K;
    hp.Ncols = d.C; hp.ocs = d.x_cstride; hp.oco = d.x_coff;
  }
  if (hp.PT < 0 || hp.PL < 0 || hp.PT >= hp.KH || hp.PL >= hp.KW) return false;
  hp.ntap = d.KH * d.KW;
  hp.HWd = 16 + d.KW - 1;
  // columns: TN fragments per block, fewest padded columns (+ a per-tile overhead of 32 columns)
  long best = -1;
  for (int tn = 1; tn <= 4; ++tn) {
    const long nt = tde_cdiv(hp.Ncols, 16 * tn), cost = nt * (16 * tn + 32);
    if (g_halo_tn ? tn == g_halo_tn : (best < 0 || cost < best)) { best = cost; hp.TN = tn; }
  }
  hp.ncolt = tde_cdiv(hp.Ncols, 16 * hp.TN);
  hp.NcolsP = hp.ncolt * 16 * hp.TN;
  // Tile shape by a throughput model fitted to the measured layers (scripts/conv_micro.py sweep): per-SIMD
  // MFMA work = rounds of concurrently resident blocks x k-steps x TN, divided by an efficiency that is
  // low for one wave per SIMD (nothing hides its LDS / barrier latency) -- the grid must also cover the
  // chip (cnv2b at 16-row tiles is 96 blocks: 8-row tiles won by 1.4x).
  const int cp8 = (hp.Cv + 7) / 8 * 8;
  const int nws[2] = {8, 4};
  const size_t btile = (size_t)hp.planes * 16 * hp.TN * LDB * 2;                      // bytes
  const size_t ring = 3 * ((btile + 1023) / 1024 * 1024);
  double best_est = -1.0;
  for (int i = 0; i < 2; ++i) {
    const int nw = nws[i];
    if (g_halo_nw && nw != g_halo_nw) continue;
    const int hh = 2 * nw + d.KH - 1;
    int tried = 0;
    for (int nch = (int)g_halo_minch; nch <= cp8 / 8 && tried < 3; ++nch) {
      const int cc = ((cp8 + nch - 1) / nch + 7) / 8 * 8;
      if (nch > 1 && (cp8 + cc - 1) / cc < nch) continue;   // same chunking as a smaller nch
      int sa = lds_stride(cc), swz = 0;
      if (g_halo_swz && hp.planes == 2) {   // fp16x3: swizzled rows of 4 / 8 chunks where they beat the padding
        if (cc > 16 && cc <= 32 && sa > 32) { sa = 32; swz = 4; }
        else if (cc > 32 && cc <= 64 && sa > 64) { sa = 64; swz = 8; }
      }
      const size_t lds = (size_t)hp.planes * hh * hp.HWd * sa * 2 + ring;
      if (lds > (size_t)g_halo_lds) continue;
      ++tried;
      const int nchr = (cp8 + cc - 1) / cc;
      const long blocks = (long)tde_cdiv(d.W, 16) * tde_cdiv(d.H, 2 * nw) * d.N * hp.ncolt;
      int bpc = (int)((160 * 1024) / lds);
      if (bpc > 12 / nw) bpc = 12 / nw;            // ~130-170 VGPRs: <= 3 waves per SIMD
      if (bpc < 1) bpc = 1;
      const long rounds = (blocks + 256L * bpc - 1) / (256L * bpc);
      const long res = blocks < 256L * bpc ? (blocks + 255) / 256 : bpc;   // blocks per busy CU
      const double share = (double)(nw * res) / 4.0;                        // waves per SIMD
      const double eff = share >= 2.0 ? 1.0 : (share >= 1.0 ? 0.6 : 0.6 * share);
      const double est = (double)rounds * nchr * tde_cdiv((long)hp.ntap * cc, 32) * hp.TN * share / eff +
                         2.0 * nchr;   // + halo staging per chunk
      if (best_est < 0 || est < best_est - 1e-9) {
        best_est = est;
        hp.NW = nw; hp.CC = cc; hp.nch = nchr; hp.SA = sa; hp.swz = swz; hp.HP = hh * hp.HWd;
        hp.lds_bytes = lds; hp.ok = 1;
      }
    }
  }
  if (!hp.ok) return false;
  if (g_halo_verbose)
    fprintf(stderr, "[halo] mode %d N %d H %d W %d C %d K %d k %d: NW %d TN %d CC %d nch %d SA %d swz %d lds %zu\n",
            mode, d.N, d.H, d.W, hp.Cv, hp.Ncols, d.KH, hp.NW, hp.TN, hp.CC, hp.nch, hp.SA, hp.swz, hp.lds_bytes);
  hp.steps = tde_cdiv((long)hp.ntap * hp.CC, 32);
  hp.gx = tde_cdiv(d.W, 16);
  hp.gy = tde_cdiv(d.H, 2 * hp.NW);
  hp.gz = d.N * hp.ncolt;
  hp.nparts = hp.gx * hp.gy * d.N;
  hp.wbytes = ((size_t)hp.nch * hp.steps * hp.planes * hp.NcolsP * LDB * 2 + 255) / 256 * 256;
  return true;
}

static WprepJob wprep_job(const HaloPlan& hp, const tde_conv_desc_t& d, const float* w, void* out) {
  WprepJob J{};
  J.w = w; J.wp = static_cast<u16*>(out); J.wmax = d.w_absmax;
  J.total = (long)hp.nch * hp.steps * hp.NcolsP * LDB;
  long blocks = (J.total + 255) / 256;
  J.nblocks = (int)(blocks > 2048 ? 2048 : blocks);
  J.mode = hp.mode; J.steps = hp.steps; J.CC = hp.CC; J.ntap = hp.ntap; J.Cred = hp.Cred; J.Ncols = hp.Ncols;
  J.NCP = 16 * hp.TN; J.ncolt = hp.ncolt; J.wcin = d.w_cin; J.K = d.K; J.planes = hp.planes;
  return J;
}

void halo_wprep_batch(int n, const HaloPlan* hps, const tde_conv_desc_t* const* ds, const float* const* ws,
                      void* const* outs, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += WPREP_MAXJ) {
    WprepBatch B{};
    int blocks = 0;
    for (int i = i0; i < n && B.njobs < WPREP_MAXJ; ++i) {
      WprepJob J = wprep_job(hps[i], *ds[i], ws[i], outs[i]);
      J.block0 = blocks;
      blocks += J.nblocks;
      B.j[B.njobs++] = J;
    }
    hipLaunchKernelGGL(halo_wprep_batch_kernel, dim3(blocks), dim3(256), 0, st, B);
  }
}

void halo_launch(const HaloPlan& hp, const tde_conv_desc_t& d, const float* in, const float* w, float* out,
                 int accumulate, void* ws, double* bnp, hipStream_t st, const float* bias, int relu) {
  // weights split beforehand (tde_conv2d_split_weights, d.w_split[mode]) or here, into the workspace
  const u16* wp = static_cast<const u16*>(d.w_split[hp.mode]);
  if (wp == nullptr) {
    const WprepJob J = wprep_job(hp, d, w, ws);
    hipLaunchKernelGGL(halo_wprep_kernel, dim3(J.nblocks), dim3(256), 0, st, J);
    wp = static_cast<const u16*>(ws);
  }
  HaloArgs a{};
  a.N = d.N; a.H = d.H; a.W = d.W;
  a.HWd = hp.HWd; a.HP = hp.HP; a.CC = hp.CC; a.nch = hp.nch; a.SA = hp.SA; a.steps = hp.steps; a.ntap = hp.ntap;
  a.KW = hp.KW; a.PT = hp.PT; a.PL = hp.PL;
  a.Cv = hp.Cv; a.ics = hp.ics; a.ico = hp.ico; a.Ncols = hp.Ncols; a.ocs = hp.ocs; a.oco = hp.oco;
  a.ncolt = hp.ncolt; a.NcolsP = hp.NcolsP; a.accumulate = accumulate; a.swz = hp.swz;
  a.fCC = make_fdiv(hp.CC); a.fKW = make_fdiv(hp.KW); a.fC4 = make_fdiv(hp.CC / 4); a.fHWd = make_fdiv(hp.HWd);
  a.in = in; a.out = out; a.wp = wp; a.bnp = bnp; a.bias = bias; a.relu = relu;
  a.inmax = hp.mode == 0 ? d.x_absmax : d.y_absmax;
  a.wmax = d.w_absmax;
  const int key = hp.NW * 10 + hp.TN;
  switch (key) {
    case 81: launch_t<8, 1>(hp, a, st); break;
    case 82: launch_t<8, 2>(hp, a, st); break;
    case 83: launch_t<8, 3>(hp, a, st); break;
    case 84: launch_t<8, 4>(hp, a, st); break;
    case 41: launch_t<4, 1>(hp, a, st); break;
    case 42: launch_t<4, 2>(hp, a, st); break;
    case 43: launch_t<4, 3>(hp, a, st); break;
    default: launch_t<4, 4>(hp, a, st); break;
  }
}
