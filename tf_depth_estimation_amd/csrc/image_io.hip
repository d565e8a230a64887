// Input pipeline, device half: the per-sample image work of
// imageselect_Dataloader_optflow.py:104-133,216-233 for a whole batch in one launch --
//   image_seq = to_float(resize_images(decode_jpeg(file), [resizedheight, resizedwidth * nframes]))
//   tgt_image = image_seq[:, 0:W], src_image_1 = image_seq[:, W:2W]   (unpack_image_sequence)
// The JPEG decode runs on the host (imageselect_Dataloader_optflow.DataLoader, PIL / libjpeg); this kernel
// takes the packed uint8 HWC images of the batch (any size per image, one H2D copy), applies TF-1's
// resize_images default (ResizeMethod.BILINEAR, align_corners=False: src = dst * in/out, lower =
// floor, upper = min(lower + 1, in - 1), lerp in float32 in TF's order top / bottom / blend) and writes
// each frame straight into its NHWC float view (e.g. the training program's padded input buffer).
//
// HBM-bound: per output pixel 4 taps x 3 bytes gathered (cached: neighbouring outputs share taps) and
// 12 bytes written.  One thread per output pixel of the [out_h, nframes * out_w] resized strip; FMA
// contraction is off in the arithmetic (HIP's __fmul_rn / __fadd_rn are plain operators that
// -ffp-contract=fast still fuses) and the scale is a correctly rounded division: the result is bit-identical
// to the float32 restatement in oracle/dataloader.py.
#include "tde_common.h"

namespace {

struct Tap {
  int lo, hi;
  float l;
};

// TF-1 resize_bilinear_op.cc compute_interpolation_weights: in = i * scale, lower = (int64)in,
// upper = min(lower + 1, in_size - 1), lerp = in - lower
__device__ __forceinline__ Tap tap(int o, float scale, int n_in) {
#pragma clang fp contract(off)
  Tap t;
  const float in = (float)o * scale;
  t.lo = (int)in;
  t.hi = min(t.lo + 1, n_in - 1);
  t.l = in - (float)t.lo;
  return t;
}

__device__ __forceinline__ float blend(float a, float b, float l) {   // a + (b - a) * l, unfused
#pragma clang fp contract(off)
  return a + (b - a) * l;
}

__global__ void __launch_bounds__(256) resize_unpack_kernel(const tde_image_batch_t a) {
  const int OWt = a.out_w * a.nframes;
  const int per_img = a.out_h * OWt;
  const int total = per_img * a.B;                  // < 2^31 (checked on the host): 32-bit index math
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int b = i / per_img;
    const int r = i - b * per_img;
    const int oy = r / OWt, ox = r - oy * OWt;
    const int h = a.src_hw[2 * b], w = a.src_hw[2 * b + 1];
    const unsigned char* img = a.src + a.src_off[b];
    // CalculateResizeScale(in, out, align_corners=false) = in / (float)out, correctly rounded (a plain '/'
    // may compile to the approximate reciprocal sequence)
    const Tap ty = tap(oy, __fdiv_rn((float)h, (float)a.out_h), h);
    const Tap tx = tap(ox, __fdiv_rn((float)w, (float)OWt), w);
    const unsigned char* p00 = img + ((long)ty.lo * w + tx.lo) * 3;
    const unsigned char* p01 = img + ((long)ty.lo * w + tx.hi) * 3;
    const unsigned char* p10 = img + ((long)ty.hi * w + tx.lo) * 3;
    const unsigned char* p11 = img + ((long)ty.hi * w + tx.hi) * 3;
    const int f = ox / a.out_w, x = ox - f * a.out_w;
    float* o = a.out[f] + ((long)(b * a.out_h + oy) * a.out_w + x) * a.out_cstride[f] + a.out_coff[f];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float top = blend((float)p00[c], (float)p01[c], tx.l);
      const float bot = blend((float)p10[c], (float)p11[c], tx.l);
      o[c] = blend(top, bot, ty.l);
    }
  }
}

}  // namespace

extern "C" {

int tde_image_resize_unpack(const tde_image_batch_t* a, void* stream) {
  tde_clear_error();
  TDE_CHECK_ARG(a && a->B > 0 && a->out_h > 0 && a->out_w > 0 && a->nframes >= 1 && a->nframes <= TDE_MAX_FRAMES);
  TDE_CHECK_ARG(a->src && a->src_off && a->src_hw);
  for (int f = 0; f < a->nframes; ++f)
    TDE_CHECK_ARG(a->out[f] && a->out_coff[f] >= 0 && a->out_coff[f] + 3 <= a->out_cstride[f]);
  const long total = (long)a->B * a->out_h * a->out_w * a->nframes;
  TDE_CHECK_ARG(total < (1L << 31));
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(resize_unpack_kernel, dim3((int)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), *a);
  return tde_launch_status();
}

}  // extern "C"
