// LDS-DMA ring implicit-GEMM tiles for gfx950, fp16x3 conv math (round 5).
//
// Opt-in (tde_set_conv_ring / TDE_RING; measured slower overall, conv_igemm.hip) replacement of the register-staged
// k-loop of conv_igemm.hip (conv_tile) for the FWD / DGRAD / pixel-shuffle GEMMs of
// slim.conv2d / slim.conv2d_transpose (nets_optflow_depth.py:88-144) that do not take the
// halo or skinny paths -- the encoder's strided convs, the deep levels, the decoder's icnv* and the deconvs.  The
// register-staged tile keeps ONE k-tile in flight: each 32-deep step waits for its global loads (~1-2 us under
// load) and then for its split + LDS stores behind a barrier, so at 1-2 waves per SIMD the MFMAs idle most of the
// step (round 3's phase-removal builds: loads + staging cost 2.4x the MFMA phase).  Here both operands stream into an
// NS-slot LDS ring by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction), NS - 1 k-tiles in flight across
// the barriers (counted vmcnt, raw s_barrier -- __syncthreads() would drain the DMAs):
//   A (the im2col gather of x, or of dy for DGRAD) lands as fp32 [BM][32]; each lane's 16-byte source is one
//     4-channel piece of one pixel (C % 4 == 0), padding taps / tails get an out-of-range offset and land as 0;
//     the 16-byte slots of a row are XOR-swizzled (ring_fa) on the SOURCE side, so the lane-linear DMA image
//     reads conflict-free; each wave splits its A fragments in registers (2 v_fma_mix per element);
//   B (the weights) is pre-split in HBM by ring_wprep_kernel into exactly its LDS image: fp16 hi / lo planes
//     [BN][32] per (class, k-tile, column tile), slots swizzled by ring_fb -- once per step for every layer
//     (tde_conv2d_split_weights), so B costs the k-loop no VALU at all.
// The k order inside a fragment is permuted (lane group q holds k 4q..4q+3 and 16+4q..16+4q+3) identically for A
// (which fp32 slots it reads) and B (which k the prep kernel puts in chunk q), so the contraction is unchanged.
// Products: hi*lo + lo*hi + hi*hi on v_mfma_f32_16x16x32_f16 with fp32 accumulation, the split of split_math.h
// (same operand scales as conv_tile), then conv_tile's epilogue (tile_epilogue: BN partials, stores, split-K slab).
#include "conv_common.h"

namespace tdeconv {

typedef unsigned short u16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

namespace {   // kernels: internal linkage (their host stubs live in this translation unit)

// Workgroup barrier waiting only for this wave's LDS operations (see halo_conv.hip: __syncthreads()' fence would
// make the compiler drain the DMAs in flight).
__device__ __forceinline__ void ring_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void ring_vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// 16 bytes per lane from buffer r at byte offset voff (out of range: zeros) to LDS base + 16 * lane.  (A helper, not
// the builtin inside the kernel's lambda: hipcc's host pass then dropped the kernels' launch stubs.)
__device__ __forceinline__ void ring_dma16(__amdgpu_buffer_rsrc_t r, void* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, 0, 0, 0);
}

// Float offset into w of the GEMM's B value at reduction index kk, column n; OOB (a zero read) past the tensor.
// `g` = the class geometry (DGRAD: khs, kws, ntw, nth * ntw * K) computed once per tile.
__device__ __forceinline__ int ring_bsrc(const RingJob& J, const int4 g, int kk, int n) {
  if (n >= J.Nn) return OOB;
  if (J.mode == MODE_FWD) {
    // B[(tap, c)][k] = w[tap][c][k]   (w [KH][KW][wcin][K]; channels c >= wcin of a padded view: 0)
    if (kk >= J.Kd) return OOB;
    const int tap = fdiv(kk, J.fC), c = kk - tap * J.C;
    return c < J.wcin ? 4 * ((tap * J.wcin + c) * J.K + n) : OOB;
  }
  if (J.mode == MODE_DGRAD) {
    // class (py, px) of the sub-pixel decomposition: B[(th, tw, kx)][ci] = w[khs + S th][kws + S tw][ci][kx]
    if (kk >= g.w || n >= J.wcin) return OOB;
    const int tap = fdiv(kk, J.fK), kx = kk - tap * J.K;
    const int th = tap / g.z, tw = tap - th * g.z;   // ntw <= 7: a short division
    return 4 * ((((g.x + J.S * th) * J.KW + g.y + J.S * tw) * J.wcin + n) * J.K + kx);
  }
  // MODE_PS: column n = (py, px, c), reduction kk = (th, tw, kin): w[2 (1 - th) + py][2 (1 - tw) + px][c][kin]
  if (kk >= J.Kd) return OOB;
  const int gq = fdiv(n, J.fpsC), c = n - gq * J.ps_C;
  const int tap = fdiv(kk, J.fC), kin = kk - tap * J.C;
  const int kh = 2 - 2 * (tap >> 1) + (gq >> 1), kw = 2 - 2 * (tap & 1) + (gq & 1);
  if (kh >= 3 || kw >= 3) return OOB;
  return 4 * (((kh * 3 + kw) * J.ps_C + c) * J.ps_K + kin);
}

// One B tile per block iteration: [2 planes][BN][32 u16] of (class, k-tile, column tile) t of job J.  The 32 x BN
// fp32 values pass through LDS so both sides stay coalesced: read along n where the weights are n-contiguous (FWD:
// w[tap][c][k]), along k where they are k-contiguous (DGRAD w[tap][ci][kx], PS w[kh][kw][c][kin]); written as whole
// 16-byte chunks.  A lane's BN / 8 reads are all issued before the first is used (the first version read one value
// per loop trip with the index decode's divisions between: latency-bound, ~100 us per network launch).
// Row cl's 16-byte slot s holds logical chunk j = s ^ ring_fb(cl), element el of chunk j is k-in-tile 4j + el (el < 4)
// or 16 + 4j + el - 4; plane 0 = fp16(x s), plane 1 = fp16(x s - hi), s the weights' fp16x3 scale (split_math.h: the
// same two roundings as split4x2h).
constexpr int RING_PREP_MAXBN = 128;
constexpr int RING_PREP_PER = RING_BK * RING_PREP_MAXBN / 256;
__global__ void __launch_bounds__(256) ring_wprep_kernel(const RingJobs B) {
  __shared__ float T[RING_BK][RING_PREP_MAXBN + 1];
  int k = 0;
  while (k + 1 < B.njobs && (int)blockIdx.x >= B.j[k + 1].block0) ++k;
  const RingJob& J = B.j[k];
  const float ws = f16x3_scale(J.wmax, F16X3_WSCALE);
  const int BNc = J.bn, nel = RING_BK * BNc;
  const FDiv fbn = make_fdiv(BNc);
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(J.w, J.wn);
  for (int t = blockIdx.x - J.block0; t < J.ncls * J.nkt * J.ncolt; t += J.nblocks) {
    const int ct = t % J.ncolt, kt = (t / J.ncolt) % J.nkt, cls = t / (J.ncolt * J.nkt);
    int4 g = make_int4(0, 0, 1, 0);
    if (J.mode == MODE_DGRAD) {
      const int S = J.S, py = cls / S, px = cls - py * S;
      const int khs = (py + J.PT) % S, kws = (px + J.PL) % S;
      const int nth = (J.KH - khs + S - 1) / S, ntw = (J.KW - kws + S - 1) / S;
      g = make_int4(khs, kws, ntw, nth * ntw * J.K);
    }
    float v[RING_PREP_PER];
#pragma unroll
    for (int i = 0; i < RING_PREP_PER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      int kl, n;
      if (J.mode == MODE_FWD) { kl = fdiv(idx, fbn); n = idx - kl * BNc; }
      else { n = idx >> 5; kl = idx & 31; }
      const int off = idx < nel ? ring_bsrc(J, g, kt * RING_BK + kl, ct * BNc + n) : OOB;
      v[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < RING_PREP_PER; ++i) {
      const int idx = threadIdx.x + 256 * i;
      if (idx < nel) {
        int kl, n;
        if (J.mode == MODE_FWD) { kl = fdiv(idx, fbn); n = idx - kl * BNc; }
        else { n = idx >> 5; kl = idx & 31; }
        T[kl][n] = v[i] * ws;
      }
    }
    __syncthreads();
    u16* out = J.out + (long)t * (2 * BNc * RING_BK);
    for (int c = threadIdx.x; c < 8 * BNc; c += 256) {   // 16-byte chunks: (plane, row cl, slot s)
      const int s = c & 3, cl = (c >> 2) % BNc, plane = c / (4 * BNc);
      const int j = s ^ ring_fb(cl & 15);
      u16 v[8];
#pragma unroll
      for (int el = 0; el < 8; ++el) {
        const float x = T[el < 4 ? 4 * j + el : 16 + 4 * j + (el - 4)][cl];
        const _Float16 h = (_Float16)x;
        v[el] = __builtin_bit_cast(u16, plane == 0 ? h : (_Float16)(x - (float)h));
      }
      *reinterpret_cast<uint4*>(out + (long)(plane * BNc + cl) * RING_BK + 8 * s) =
          make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
    }
    __syncthreads();
  }
}

}  // namespace

void ring_wprep_launch(const RingJobs& jobs, int blocks, hipStream_t st) {
  if (jobs.njobs > 0 && blocks > 0) hipLaunchKernelGGL(ring_wprep_kernel, dim3(blocks), dim3(256), 0, st, jobs);
}

namespace {

// One (row tile, column tile, split * class) block.  NW = WM x WN waves, each TM x TN 16x16 fragments.
template <int MODE, int BM, int BN, int WM, int WN, int NS>
__global__ void __launch_bounds__(64 * WM * WN) ring_kernel(const ConvArgs p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int A_BYTES = BM * RING_BK * 4, B_BYTES = BN * RING_BK * 4;   // B: 2 planes x BN x 32 fp16
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024, B_INS = B_BYTES / 1024;           // 1-KiB DMA wave-instructions
  static_assert(A_INS % NW == 0 && B_BYTES % 1024 == 0 && TM >= 1 && TN >= 1, "ring tile");
  constexpr int DA = A_INS / NW, DB = (B_INS + NW - 1) / NW, DI = DA + DB;
  constexpr bool FWDLIKE = (MODE == MODE_FWD || MODE == MODE_PS);
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int r16 = lane & 15, q = lane >> 4;
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  const float sA = f16x3_scale(MODE == MODE_DGRAD ? p.ymax : p.xmax, 1.f);
  const float sB = f16x3_scale(p.wmax, F16X3_WSCALE);

  int M, Nn, Kd, zsplit, cls = 0;
  DgClass g{};
  if constexpr (MODE == MODE_DGRAD) {
    const int ncls = p.S * p.S;
    cls = bz % ncls;
    zsplit = bz / ncls;
    g = dg_class(p, cls);
    M = g.M; Nn = p.C; Kd = g.Kd;
  } else {
    zsplit = bz;
    M = p.N * p.OH * p.OW; Nn = p.K; Kd = p.KH * p.KW * p.C;
  }
  FDiv fntw{};
  if constexpr (MODE == MODE_DGRAD) fntw = make_fdiv(g.ntw);
  const int m0 = bx * BM, n0 = by * BN;
  if (m0 >= M || n0 >= Nn) return;
  const int nkt = (Kd + RING_BK - 1) / RING_BK;
  const int kt0 = zsplit * p.kt_per;
  const int kt1 = min(nkt, kt0 + p.kt_per);

  const __amdgpu_buffer_rsrc_t ra = FWDLIKE ? make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs)
                                            : make_rsrc(p.dy, (long)p.N * p.OH * p.OW * p.ycs);
  const long img_floats = (long)(MODE == MODE_DGRAD ? p.S * p.S : 1) * p.img_nkt * p.img_ncolt * (B_BYTES / 4);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(reinterpret_cast<const float*>(p.wimg), img_floats);

  // A DMA pieces of this lane: instruction i of this wave covers tile rows (wid + i * NW) * 8 .. + 7, lane ->
  // row + (lane >> 3), slot lane & 7 = logical chunk jA (ring_fa depends on row bits 1-2 = bits of lane >> 3 only)
  const int jA = (lane & 7) ^ ring_fa(lane >> 3);
  int a_pb[DA], a_i1[DA], a_i2[DA];
#pragma unroll
  for (int i = 0; i < DA; ++i) {
    const int m = m0 + (wid + i * NW) * 8 + (lane >> 3);
    a_pb[i] = 0; a_i1[i] = -(1 << 28); a_i2[i] = -(1 << 28);   // rows past M: every tap out of range -> 0
    if (m < M) {
      if constexpr (FWDLIKE) {
        const int ohw = p.OH * p.OW;
        const int n = m / ohw, r = m - n * ohw, oh = r / p.OW, ow = r - oh * p.OW;
        a_i1[i] = oh * p.S - p.PT; a_i2[i] = ow * p.S - p.PL;
        a_pb[i] = ((n * p.H + a_i1[i]) * p.W + a_i2[i]) * p.xcs + p.xco;
      } else {
        const int hw = g.HH * g.WW;
        const int n = m / hw, r = m - n * hw, ihh = r / g.WW, iww = r - ihh * g.WW;
        a_i1[i] = ihh + g.dh; a_i2[i] = iww + g.dw;
        a_pb[i] = ((n * p.OH + a_i1[i]) * p.OW + a_i2[i]) * p.ycs + p.yco;
      }
    }
  }
  const int bimg0 = ((cls * p.img_nkt) * p.img_ncolt + by) * B_BYTES;   // + kt * ncolt * B_BYTES

  auto issue = [&](int kt, int slot) __attribute__((always_inline)) {
    char* const sb = smem + slot * STAGE;
    const int kq = kt * RING_BK + 4 * jA;
    int t_h, t_w, koff;
    if constexpr (FWDLIKE) {
      const int tap = fdiv(kq, p.fC), c = kq - tap * p.C;
      t_h = fdiv(tap, p.fKW); t_w = tap - t_h * p.KW;
      koff = (t_h * p.W + t_w) * p.xcs + c;
    } else {
      const int tap = fdiv(kq, p.fK), kx = kq - tap * p.K;
      t_h = fdiv(tap, fntw); t_w = tap - t_h * g.ntw;
      koff = -(t_h * p.OW + t_w) * p.ycs + kx;
    }
#pragma unroll
    for (int i = 0; i < DA; ++i) {
      bool ok;
      if constexpr (FWDLIKE)
        ok = kq < Kd && (unsigned)(a_i1[i] + t_h) < (unsigned)p.H && (unsigned)(a_i2[i] + t_w) < (unsigned)p.W;
      else
        ok = kq < Kd && (unsigned)(a_i1[i] - t_h) < (unsigned)p.OH && (unsigned)(a_i2[i] - t_w) < (unsigned)p.OW;
      ring_dma16(ra, sb + (wid + i * NW) * 1024, ok ? 4 * (a_pb[i] + koff) : OOB);
    }
    const int tb = bimg0 + kt * p.img_ncolt * B_BYTES;
#pragma unroll
    for (int i = 0; i < DB; ++i) {
      const int piece = min(wid + i * NW, B_INS - 1);   // (waves past the last piece copy it again: same bytes)
      ring_dma16(rb, sb + A_BYTES + piece * 1024, tb + piece * 1024 + lane * 16);
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * TM * 16, wcol0 = wn * TN * 16;
  const int fa = ring_fa(r16), fb = ring_fb(r16);

  auto compute = [&](int slot) __attribute__((always_inline)) {
    const float* A = reinterpret_cast<const float*>(smem + slot * STAGE);
    const u16* Bp = reinterpret_cast<const u16*>(smem + slot * STAGE + A_BYTES);
    h8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const u16* br = Bp + (wcol0 + b * 16 + r16) * RING_BK + 8 * (q ^ fb);
      bh[b] = *reinterpret_cast<const h8*>(br);
      bl[b] = *reinterpret_cast<const h8*>(br + BN * RING_BK);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const float* ar = A + (wrow0 + a * 16 + r16) * RING_BK;
      const f4 x0 = *reinterpret_cast<const f4*>(ar + 4 * (q ^ fa));
      const f4 x1 = *reinterpret_cast<const f4*>(ar + 4 * ((q + 4) ^ fa));
      split8x2h(x0, x1, sA, ah[a], al[a]);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
      }
  };

  if (kt0 < kt1) {
    const int klast = kt1 - 1;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(min(kt0 + s, klast), s);
    int rs = 0, wsl = NS - 1;
    for (int kt = kt0; kt < kt1; ++kt) {
      ring_vm_wait<(NS - 2) * DI>();   // this wave's pieces of tile kt have landed (NS - 2 tiles still in flight)
      ring_barrier();                  // every wave's pieces landed; slot wsl (tile kt - 1) read by every wave
      issue(min(kt + NS - 1, klast), wsl);
      compute(rs);
      rs = rs + 1 == NS ? 0 : rs + 1;
      wsl = wsl + 1 == NS ? 0 : wsl + 1;
    }
    ring_vm_wait<0>();
  }
  ring_barrier();   // the ring is free before the epilogue reuses LDS

  const float inv = 1.f / (sA * sB);   // powers of two: exact
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] *= inv;
  tile_epilogue<MODE, BM, BN, WM, WN>(p, acc, bx, by, bz, M, Nn, zsplit, g, reinterpret_cast<float*>(smem));
}

// WGRAD (Conv2DBackpropFilter): C[(tap, c)][k] = sum_p x[p + tap][c] dy[p][k], the reduction over the output pixels p
// in 32-pixel k-tiles.  Both operands are pixel-major in HBM (channels contiguous), so each stage DMA's them as they
// lie: [32 pixels][BM] of the x gather (out-of-image taps land as 0) and [32 pixels][BN] of dy, fp32.  A fragment
// (8 pixels of one channel) is 8 ds_read_b32 -- rows 8 pixels apart are kept 16 floats apart by XOR-ing bit 2 of
// the 16-byte chunk index with row bit 3 (source-side swizzle), so both halves of a ds_read_b32 lane group hit
// distinct banks -- then split in registers like the A operand of ring_kernel.  No register transposes, no staging
// stores (the register-staged WGRAD transposes 4x4 blocks in registers and stores them with 2-way LDS conflicts).
template <int BM, int BN, int WM, int WN, int NS>
__global__ void __launch_bounds__(64 * WM * WN) ring_wgrad_kernel(const ConvArgs p) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int A_BYTES = RING_BK * BM * 4, B_BYTES = RING_BK * BN * 4;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024, B_INS = B_BYTES / 1024;
  static_assert(A_INS % NW == 0 && B_BYTES % 1024 == 0 && TM >= 1 && TN >= 1 && BM % 32 == 0 && BN % 32 == 0, "tile");
  constexpr int DA = A_INS / NW, DB = (B_INS + NW - 1) / NW, DI = DA + DB;
  constexpr int ACH = BM / 4, BCH = BN / 4;   // 16-byte chunks per pixel row
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int r16 = lane & 15, q = lane >> 4;
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  const float sA = f16x3_scale(p.xmax, 1.f);
  const float sB = f16x3_scale(p.ymax, 1.f);
  const int M = p.KH * p.KW * p.C, Nn = p.K, npix = p.N * p.OH * p.OW;
  const int zsplit = bz;
  const int m0 = bx * BM, n0 = by * BN;
  if (m0 >= M || n0 >= Nn) return;
  const int nkt = (npix + RING_BK - 1) / RING_BK;
  const int kt0 = zsplit * p.kt_per;
  const int kt1 = min(nkt, kt0 + p.kt_per);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x, (long)p.N * p.H * p.W * p.xcs);
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, (long)npix * p.ycs);

  // per A piece of this lane: its pixel row, the (tap, channel) of its 4-column chunk (fixed over the k-loop)
  int a_pr[DA], a_dh[DA], a_dw[DA], a_c[DA];
#pragma unroll
  for (int i = 0; i < DA; ++i) {
    const int e = (wid + i * NW) * 64 + lane;
    const int pr = e / ACH, sl = e - pr * ACH;
    const int m = m0 + 4 * (sl ^ (((pr >> 3) & 1) << 2));
    a_pr[i] = pr;
    a_dh[i] = -(1 << 28); a_dw[i] = 0; a_c[i] = 0;   // rows past M: always out of range
    if (m < M) {
      const int tap = m / p.C, c = m - tap * p.C, kh = tap / p.KW, kw = tap - kh * p.KW;
      a_dh[i] = kh - p.PT; a_dw[i] = kw - p.PL; a_c[i] = c;
    }
  }
  int b_pr[DB], b_n[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) {
    const int piece = min(wid + i * NW, B_INS - 1);
    const int e = piece * 64 + lane;
    const int pr = e / BCH, sl = e - pr * BCH;
    b_pr[i] = pr;
    b_n[i] = n0 + 4 * (sl ^ (((pr >> 3) & 1) << 2));
  }

  auto issue = [&](int kt, int slot) __attribute__((always_inline)) {
    char* const sb = smem + slot * STAGE;
#pragma unroll
    for (int i = 0; i < DA; ++i) {
      const int pix = kt * RING_BK + a_pr[i];
      const int n = fdiv(pix, p.fOHW), r = pix - n * p.OH * p.OW;
      const int oh = fdiv(r, p.fOW), ow = r - oh * p.OW;
      const int ih = oh * p.S + a_dh[i], iw = ow * p.S + a_dw[i];
      const bool ok = pix < npix && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      ring_dma16(rx, sb + (wid + i * NW) * 1024, ok ? 4 * (((n * p.H + ih) * p.W + iw) * p.xcs + p.xco + a_c[i]) : OOB);
    }
#pragma unroll
    for (int i = 0; i < DB; ++i) {
      const int piece = min(wid + i * NW, B_INS - 1);
      const int pix = kt * RING_BK + b_pr[i];
      const bool ok = pix < npix && b_n[i] < Nn;
      ring_dma16(rdy, sb + A_BYTES + piece * 1024, ok ? 4 * (pix * p.ycs + p.yco + b_n[i]) : OOB);
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * TM * 16, wcol0 = wn * TN * 16;
  const int flip = (q & 1) << 4;   // rows 8q .. 8q+7: physical column = column ^ 16 for odd q

  auto compute = [&](int slot) __attribute__((always_inline)) {
    const float* A = reinterpret_cast<const float*>(smem + slot * STAGE);
    const float* Bm = reinterpret_cast<const float*>(smem + slot * STAGE + A_BYTES);
    h8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const float* bc = Bm + 8 * q * BN + ((wcol0 + b * 16 + r16) ^ flip);
      const f4 x0 = f4{bc[0], bc[BN], bc[2 * BN], bc[3 * BN]};
      const f4 x1 = f4{bc[4 * BN], bc[5 * BN], bc[6 * BN], bc[7 * BN]};
      split8x2h(x0, x1, sB, bh[b], bl[b]);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const float* ac = A + 8 * q * BM + ((wrow0 + a * 16 + r16) ^ flip);
      const f4 x0 = f4{ac[0], ac[BM], ac[2 * BM], ac[3 * BM]};
      const f4 x1 = f4{ac[4 * BM], ac[5 * BM], ac[6 * BM], ac[7 * BM]};
      split8x2h(x0, x1, sA, ah[a], al[a]);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[a], bh[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bl[b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[a], bh[b], acc[a][b], 0, 0, 0);
      }
  };

  if (kt0 < kt1) {
    const int klast = kt1 - 1;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(min(kt0 + s, klast), s);
    int rs = 0, wsl = NS - 1;
    for (int kt = kt0; kt < kt1; ++kt) {
      ring_vm_wait<(NS - 2) * DI>();
      ring_barrier();
      issue(min(kt + NS - 1, klast), wsl);
      compute(rs);
      rs = rs + 1 == NS ? 0 : rs + 1;
      wsl = wsl + 1 == NS ? 0 : wsl + 1;
    }
    ring_vm_wait<0>();
  }
  ring_barrier();
  const float inv = 1.f / (sA * sB);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] *= inv;
  const DgClass g{};
  tile_epilogue<MODE_WGRAD, BM, BN, WM, WN>(p, acc, bx, by, bz, M, Nn, zsplit, g, reinterpret_cast<float*>(smem));
}

}  // namespace

// Tiles: 64 rows on 4 waves (2 x 2, each 32 rows x BN/2), 128 rows on 8 waves (4 x 2); BN in {32, 64, 96, 128};
// 3 ring slots (2 k-tiles in flight): 64 x 128 = 72 KiB (two workgroups per CU), 128 x 128 = 96 KiB.
#ifndef TDE_RING_NS
#define TDE_RING_NS 3
#endif
template <int MODE, int BM>
static void ring_launch_bm(int bn, dim3 grid, const ConvArgs& a, hipStream_t st) {
  constexpr int WM = BM == 128 ? 4 : 2, NTH = 64 * WM * 2, NS = TDE_RING_NS;
  switch (bn) {
    case 32: hipLaunchKernelGGL((ring_kernel<MODE, BM, 32, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    case 64: hipLaunchKernelGGL((ring_kernel<MODE, BM, 64, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    case 96: hipLaunchKernelGGL((ring_kernel<MODE, BM, 96, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    default: hipLaunchKernelGGL((ring_kernel<MODE, BM, 128, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
  }
}

template <int MODE>
static void ring_launch_mode(int bm, int bn, dim3 grid, const ConvArgs& a, hipStream_t st) {
  if (bm == 128) ring_launch_bm<MODE, 128>(bn, grid, a, st);
  else ring_launch_bm<MODE, 64>(bn, grid, a, st);
}

template <int BM>
static void ring_wgrad_bm(int bn, dim3 grid, const ConvArgs& a, hipStream_t st) {
  constexpr int WM = BM == 128 ? 4 : 2, NTH = 64 * WM * 2, NS = TDE_RING_NS;
  switch (bn) {
    case 32: hipLaunchKernelGGL((ring_wgrad_kernel<BM, 32, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    case 64: hipLaunchKernelGGL((ring_wgrad_kernel<BM, 64, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    case 96: hipLaunchKernelGGL((ring_wgrad_kernel<BM, 96, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
    default: hipLaunchKernelGGL((ring_wgrad_kernel<BM, 128, WM, 2, NS>), grid, dim3(NTH), 0, st, a); break;
  }
}

void ring_launch(int mode, int bm, int bn, dim3 grid, const ConvArgs& a, hipStream_t st) {
  if (mode == MODE_WGRAD) {
    if (bm == 128) ring_wgrad_bm<128>(bn, grid, a, st);
    else ring_wgrad_bm<64>(bn, grid, a, st);
    return;
  }
  if (mode == MODE_FWD) ring_launch_mode<MODE_FWD>(bm, bn, grid, a, st);
  else if (mode == MODE_DGRAD) ring_launch_mode<MODE_DGRAD>(bm, bn, grid, a, st);
  else if (mode == MODE_PS) ring_launch_mode<MODE_PS>(bm, bn, grid, a, st);
}

}  // namespace tdeconv
