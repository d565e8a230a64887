// Halo-tiled stride-1 convolution (bf16x6 MFMA) -- internal interface between conv_igemm.hip (the ABI
// entry points and their planners) and halo_conv.hip (the kernels).
#pragma once
#include "tde_common.h"

// Plan of one stride-1 FWD (y = conv(x, w)) or DGRAD (dx = conv(dy, flip(w)^T)) call on the halo path.
struct HaloPlan {
  int ok;
  int mode;               // 0 FWD, 1 DGRAD (of a stride-1 conv)
  int planes;             // split planes: 3 bf16 (bf16x6, math 2/3), 2 fp16 (fp16x3, math 4)
  int NW, TN;             // waves per block (pixel rows 2*NW), 16-column MFMA fragments per wave
  int HWd, HP;            // halo width (16 + KW - 1), halo pixels
  int CC, nch, SA;        // channels per chunk (multiple of 8), chunks, LDS row stride (u16)
  int swz;                // 0: padded rows; 4 / 8: rows of 4 / 8 XOR-swizzled 16-byte chunks (fp16x3)
  int steps, ntap;        // 32-deep k-steps per chunk, KH*KW
  int KH, KW, PT, PL;     // geometry of the conv as executed (DGRAD: flipped taps and pads)
  int Cv, ics, ico;       // input view: channels read, cstride, coff
  int Cred;               // reduction channels with nonzero weights (FWD: w_cin, DGRAD: K)
  int Ncols, ocs, oco;    // output columns and view
  int ncolt, NcolsP;      // column tiles of 16*TN, padded column count of the split weights
  int gx, gy, gz;         // grid
  size_t wbytes;          // split-weight planes in the workspace
  size_t lds_bytes;
  int nparts;             // BN statistics partials (one per pixel tile)
};

// mode 0 FWD / 1 DGRAD of the conv described by d; math = current conv math.  Returns false when the
// call should take the implicit-GEMM path.
bool halo_plan(const tde_conv_desc_t& d, int mode, int math, HaloPlan& hp);

// Weight split (one launch; skipped when d.w_split[hp.mode] holds the pre-split weights) + conv (one launch).  ws: >= hp.wbytes of 16-byte aligned workspace;
// bnp: fp64 BN partials [hp.nparts][2][Ncols] or null.  bias / relu: folded-BN inference epilogue
// (out = relu?(conv + bias[col]); accumulate 0), null / 0 for a plain conv.
void halo_launch(const HaloPlan& hp, const tde_conv_desc_t& d, const float* in, const float* w, float* out,
                 int accumulate, void* ws, double* bnp, hipStream_t st, const float* bias = nullptr,
                 int relu = 0);

// The weight splits of n (plan, layer) pairs in one launch (tde_conv2d_split_weights): outs[i] >= hps[i].wbytes.
void halo_wprep_batch(int n, const HaloPlan* hps, const tde_conv_desc_t* const* ds, const float* const* ws,
                      void* const* outs, hipStream_t st);

// Halo-tiled filter gradient (halo_wgrad.hip) of a stride-1 (fp16x3 also stride-2) conv with K <= 32 output
// channels at high resolution: partial dW per (pixel chunk, kernel row) on MFMA, then a fixed-order chunk reduce.
struct HwgPlan {
  int ok;
  int f16;                // fp16x3 kernel (math 4): CF / NF / nitems = (kw, cf) items / CPS, KPS in fp16 elements
  int S;                  // stride (2: the fp16x3 kernel's parity planes)
  int CF, NF, nitems;     // 16-channel input / output fragments, (kw, cf, nf) items per block
  int CPS, KPS;           // LDS row strides (floats)
  int ntw, chunks;        // 128-pixel segments per output row, pixel chunks (grid x; grid y = KH)
  long ntiles;
  size_t lds_bytes, part_bytes;
};
bool hwg_plan(const tde_conv_desc_t& d, HwgPlan& hp, int math);
// dw (+)= dL/dW from x (view of d) and dy (y view of d); ws >= hp.part_bytes (16-byte aligned).
void hwg_launch(const HwgPlan& hp, const tde_conv_desc_t& d, const float* x, const float* dy, float* dw,
                int accumulate, void* ws, hipStream_t st);
