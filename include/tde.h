/*
 * tde.h -- C ABI of the MI355X-native hot path of wrlife/tf_depth_estimation.
 *
 * The reference has no FFI: its hot path is a TensorFlow-1 graph built by Python functions
 * (SURVEY.md §8b).  This ABI exports the kernels that replace the TF ops those functions emit;
 * each entry point names the reference call site it stands in for.  The PyTorch-ROCm host layer
 * (tf_depth_estimation_amd/) binds it with ctypes and exposes the reference's Python signatures
 * (`disp_net`, `depth_net`, `projective_inverse_warp`, ...).
 *
 * Conventions
 *   - All tensors are fp32, NHWC, in caller-owned device memory (no allocation inside).
 *   - An activation operand is a *channel view*: element (n,h,w,c) of a view with pixel stride
 *     `cstride` and channel offset `coff` lives at ptr[((n*H+h)*W+w)*cstride + coff + c].  This is
 *     how skip-concats (tf.concat(..., axis=3), nets_optflow_depth.py:106-141) are fused: producers
 *     write straight into their channel slice of the consumer's input buffer.
 *   - Weights keep the TF checkpoint layout: conv [KH][KW][Cin][Cout],
 *     conv2d_transpose [KH][KW][Cout][Cin].
 *   - `stream` is a hipStream_t passed as void*.  Every call is stream-ordered, never synchronises
 *     the host and is safe to capture in a hipGraph.  Re-entrant across streams.
 *   - Return value: TDE_OK (0) or a negative tde_status.
 *   - `ws` / `ws_bytes`: caller-provided device workspace; size it with the *_workspace_size query.
 *     One workspace per stream (calls on one stream reuse it in order).
 */
#ifndef TDE_H_
#define TDE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDE_ABI_VERSION 10

/* An operand bound (tde_conv_desc_t.*_absmax, tde_bn_bwd dz_absmax) is an array of this many floats whose
 * maximum is the bound: producers raise one slot per workgroup (atomic max), consumers read all. */
#define TDE_BOUND_SLOTS 16

typedef enum {
  TDE_OK = 0,
  TDE_ERR_ARG = -1,        /* bad pointer / alignment / shape */
  TDE_ERR_WORKSPACE = -2,  /* ws_bytes smaller than the query */
  TDE_ERR_HIP = -3,        /* kernel launch failed */
  TDE_ERR_UNSUPPORTED = -4
} tde_status;

/* Geometry of one conv layer, always expressed as a FORWARD conv x[N,H,W,C] -> y[N,OH,OW,K]
 * with TF 'SAME' padding (pad_top/pad_left are TF's pad_before).  For conv2d_transpose layers the
 * descriptor is that of the *virtual* forward conv whose Conv2DBackpropInput the deconv is:
 * x = deconv output [N,2h,2w,Cout], y = deconv input [N,h,w,Cin], K = Cin, C = Cout. */
typedef struct {
  int N, H, W, C;          /* x; C may include zero pad channels (C % 4 == 0) */
  int OH, OW, K;           /* y */
  int KH, KW, stride, pad_top, pad_left;
  int w_cin;               /* input channels of the weight tensor (<= C); rows ci >= w_cin are zero */
  int x_cstride, x_coff;   /* channel view of x (and of dx) */
  int y_cstride, y_coff;   /* channel view of y (and of dy) */
  /* Optional operand bounds for conv math 4 (fp16x3; ignored by the other modes): device pointers to
   * TDE_BOUND_SLOTS floats whose maximum is >= max|.| of the operand read through the x view, the y view,
   * and of the weights (a single bound: slot 0, the others 0).  The split
   * scales an operand by 2^(14 - e) (e = frexp exponent of its bound) so it fits fp16 with full precision
   * down to 2^-16 of the bound.  NULL: x / y operands are split unscaled (full precision for
   * 2^-3 <= |v| < 2^15: activations, images) and weights by 2^8 (|w| < 256).  Gradient operands (dy of a
   * conv, dy_big of a deconv) must carry a bound -- tde_bn_bwd writes one (dz_absmax). */
  const float* x_absmax;
  const float* y_absmax;
  const float* w_absmax;
  /* Optional pre-split weights: w_split[0] for the forward conv (tde_conv2d_fwd / _fwd_bn / _fwd_bias_act),
   * w_split[1] for its data gradient (tde_conv2d_bwd_data / tde_conv2d_bwd), each written by
   * tde_conv2d_split_weights for THESE weights under the current conv math.  NULL: a call that needs a
   * split makes it itself (one extra launch per call). */
  const void* w_split[2];
} tde_conv_desc_t;

int tde_abi_version(void);
const char* tde_status_string(int status);

/* Host-side CRC-32C (Castagnoli) of n bytes, continuing from `crc` (0 to start); the checksum of the
 * TF tensor-bundle checkpoint format (BundleEntryProto.crc32c, table block trailers) behind
 * tf.train.Saver (batch_prediction.py:49-55, split_training.py:147-202), used by
 * tf_depth_estimation_amd/checkpoint.py.  No device work; callable without a GPU. */
uint32_t tde_crc32c(const void* data, size_t n, uint32_t crc);

/* ---------------------------------------------------------------- MFMA implicit-GEMM convs
 * slim.conv2d (no bias; the BN that follows owns the shift), nets_optflow_depth.py:88-101,107-142
 * -> TF Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter.
 * Requires C, K, cstrides and coffs to be multiples of 4 (16-byte vectors). */
/* Process-wide conv arithmetic (set before graph capture; not per-stream):
 *   0 = exact fp32 MFMA (v_mfma_f32_16x16x4_f32; bit-for-bit an fp32 fma chain);
 *   1 = bf16x3: each fp32 operand split into bf16 hi + lo, products hi*hi + hi*lo + lo*hi on
 *       v_mfma_f32_16x16x32_bf16 with fp32 accumulation (~2^-16 relative per product, 5.3x rate);
 *       does NOT meet the 1e-4 output bar (opt-in only);
 *   2 = bf16x6: exact three-way bf16 split x = hi + mid + lo of both operands, the six product terms
 *       of order <= 2^-14 on v_mfma_f32_16x16x32_bf16, fp32 accumulation (dropped terms < 2^-21 of
 *       |x*y|), split once at LDS staging;
 *   3 = bf16x6 split per fragment in registers (fp32 LDS image); tiles narrower than 64 columns run
 *       mode 0.  Held to the same parity bars as mode 0;
 *   4 = fp16x3: each operand scaled by a power of two (see x_absmax above) and split into fp16 hi + lo
 *       (11 + 11 significant bits), products hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_f16 with fp32
 *       accumulation (<= ~3 * 2^-22 relative per product), half the MFMAs of bf16x6.  DEFAULT. */
int tde_set_conv_math(int mode);
int tde_get_conv_math(void);
/* Measurement hook (no reference counterpart: bench.py's roofline timing).  Arms the calling thread's pair of
 * device timestamp slots for the NEXT conv entry call (any tde_conv2d_* / tde_deconv2d_* compute function): a
 * one-wave kernel writes the 100 MHz real-time counter into *stamp_begin right before the call's first
 * conv-family kernel and into *stamp_end right after its last (split-K reduce included, BatchNorm launches of a
 * fused call excluded), so inside a stream capture the stamps time the kernels where the graph replays them.
 * (NULL, NULL) disarms.  Returns the number of stamps the previous arming launched. */
int tde_conv_span_arm(unsigned long long* stamp_begin, unsigned long long* stamp_end);
/* Diagnostic timeline (probe/step_timeline.py): one one-wave kernel on `stream` that writes the device's 100 MHz
 * real-time counter into *slot when the stream reaches it (inside a capture: when the replayed graph does). */
int tde_stamp(unsigned long long* slot, void* stream);
size_t tde_conv2d_workspace_size(const tde_conv_desc_t* d, int op /*0 fwd,1 bwd_data,2 bwd_filter*/);
/* Weight pre-split (the halo-tiled stride-1 path keeps the layer's weights as split fp16 / bf16 tiles): bytes of the split image op & 1 (0: the FWD GEMM's, read by a conv's forward; 1: the DGRAD GEMM's, read by
 * a conv's data gradient) of layer d needs under the current conv math; add 2 to op when d is a deconv's virtual
 * conv (its forward reads image 1, its data gradient image 0), so the size is that of the image the calls of that
 * role read.  0 = that call takes no split weights (then leave d->w_split[op & 1] NULL).  tde_conv2d_split_weights writes
 * n such images (outs[i], 256-byte aligned, >= the size) in ONE launch -- e.g. every layer of a network
 * once per step, then each conv call skips its own split launch. */
size_t tde_conv2d_split_weights_size(const tde_conv_desc_t* d, int op);
int tde_conv2d_split_weights(int n, const tde_conv_desc_t* const* descs, const int* ops,
                             const float* const* weights, void* const* outs, void* stream);
int tde_conv2d_fwd(const tde_conv_desc_t* d, const float* x, const float* w, float* y,
                   int accumulate, void* ws, size_t ws_bytes, void* stream);
int tde_conv2d_bwd_data(const tde_conv_desc_t* d, const float* dy, const float* w, float* dx,
                        int accumulate, void* ws, size_t ws_bytes, void* stream);
int tde_conv2d_bwd_filter(const tde_conv_desc_t* d, const float* x, const float* dy, float* dw,
                          int accumulate, void* ws, size_t ws_bytes, void* stream);

/* conv + training-mode batch norm + ReLU in one call: slim.conv2d / conv2d_transpose with
 * normalizer_fn=batch_norm (arg_scope nets_optflow_depth.py:82-87; same semantics as
 * tde_bn_fwd_train).  z = conv(x) is written densely (the backward needs it); the BN pass reads the
 * conv's split-K partials directly (no separate reduce launch), computes the batch statistics (fp64,
 * fixed order), updates moving_mean / moving_var (both NULL: no update) and writes
 * y = relu?((z - mean) * invstd + beta) into the channel view (y, y_cstride, y_coff). */
typedef struct {
  const float* beta;
  float eps, decay;
  int bessel;
  float* moving_mean; float* moving_var;
  float* save_mean; float* save_invstd;
  float* y; int y_cstride, y_coff;
  int relu;
  int groups;              /* row groups (0 or 1: one), see tde_bn_fwd_train */
  double* sums;            /* SyncBN phase 1 (non-NULL): write the per-group fp64 (sum z, sum z^2) [groups][2][C]
                              from the conv's own statistics partials and stop -- no statistics, moving averages
                              or y (see tde_bn_sums / tde_bn_fwd_from_sums) */
} tde_bn_train_t;
/* z dense [N*OH*OW][K] (y_cstride == K, y_coff == 0 in d).  Workspace: tde_conv2d_workspace_size(d, 3). */
int tde_conv2d_fwd_bn(const tde_conv_desc_t* d, const float* x, const float* w, float* z,
                      const tde_bn_train_t* bn, void* ws, size_t ws_bytes, void* stream);

/* Both backward GEMMs of one conv layer (TF's Conv2DBackpropInput + Conv2DBackpropFilter of one
 * slim.conv2d): dx (+)= dL/dx and dw (+)= dL/dw from dy, horizontally fused into one launch (the two are
 * independent; at the deep levels neither fills the chip alone), then the split-K reductions.
 * Workspace: tde_conv2d_bwd_workspace_size(d). */
size_t tde_conv2d_bwd_workspace_size(const tde_conv_desc_t* d);
int tde_conv2d_bwd(const tde_conv_desc_t* d, const float* x, const float* dy, const float* w, float* dx,
                   int accumulate_dx, float* dw, int accumulate_dw, void* ws, size_t ws_bytes,
                   void* stream);

/* slim.conv2d_transpose (stride 2, SAME), nets_optflow_depth.py:103,109,114,119,126,133,140.
 * `d` is the virtual forward conv (see above); x = deconv input, y = deconv output.
 *   fwd       : y_big  = Conv2DBackpropInput(x_small)     (weights [KH][KW][Cout][Cin])
 *   bwd_data  : dx_small = Conv2D(dy_big)
 *   bwd_filter: dW = Conv2DBackpropFilter(dy_big, x_small) */
size_t tde_deconv2d_workspace_size(const tde_conv_desc_t* d, int op);
int tde_deconv2d_fwd(const tde_conv_desc_t* d, const float* x_small, const float* w, float* y_big,
                     int accumulate, void* ws, size_t ws_bytes, void* stream);
/* deconv backward: dx_small (+)= Conv2D(dy_big), dw (+)= Conv2DBackpropFilter(dy_big, x_small), one
 * fused launch (see tde_conv2d_bwd).  Workspace: tde_deconv2d_bwd_workspace_size(d). */
size_t tde_deconv2d_bwd_workspace_size(const tde_conv_desc_t* d);
int tde_deconv2d_bwd(const tde_conv_desc_t* d, const float* dy_big, const float* x_small, const float* w,
                     float* dx_small, int accumulate_dx, float* dw, int accumulate_dw, void* ws,
                     size_t ws_bytes, void* stream);
/* deconv forward + BN + ReLU: z_big dense [N*H*W][C] (x_cstride == C, x_coff == 0); workspace op 3. */
int tde_deconv2d_fwd_bn(const tde_conv_desc_t* d, const float* x_small, const float* w, float* z_big,
                        const tde_bn_train_t* bn, void* ws, size_t ws_bytes, void* stream);

/* Inference path with batch norm folded into the conv (batch_prediction.py:41-44,
 * batch_prediction_optflow.py: disp_net(x, is_training=False), then sess.run per image; replaces the
 * conv -> FusedBatchNorm(is_training=False) -> Relu triple of slim.conv2d / conv2d_transpose,
 * nets_optflow_depth.py:82-87).  w / bias from tde_bn_fold; y = relu?(conv(x, w) + bias[col]) written
 * straight into the output channel view (conv: d's y view; deconv: d's x view, the virtual conv's
 * input).  One launch per layer (plus the split-K reduce when planned), no pre-BN tensor. */
int tde_conv2d_fwd_bias_act(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias,
                            int relu, float* y, void* ws, size_t ws_bytes, void* stream);
int tde_deconv2d_fwd_bias_act(const tde_conv_desc_t* d, const float* x_small, const float* w,
                              const float* bias, int relu, float* y_big, void* ws, size_t ws_bytes,
                              void* stream);
int tde_deconv2d_bwd_data(const tde_conv_desc_t* d, const float* dy_big, const float* w,
                          float* dx_small, int accumulate, void* ws, size_t ws_bytes, void* stream);
int tde_deconv2d_bwd_filter(const tde_conv_desc_t* d, const float* dy_big, const float* x_small,
                            float* dw, int accumulate, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- few-channel heads
 * slim.conv2d(..., normalizer_fn=None, activation_fn=sigmoid|None) with bias: disp heads
 * (nets_optflow_depth.py:122-144: DISP_SCALING*sigmoid(.) [+MIN_DISP]), flow heads (nets_depth.py:169-191),
 * mask heads (nets_optflow_depth.py:193-198), pose/pred 1x1 (:181) and the 3-channel linear disp heads of
 * nets.py:122-144.  K in {1, 2, 3, 6}.
 * act: 0 linear (y = z), 1 y = scale*sigmoid(z) + offset.  Backward takes y (not z). */
size_t tde_head_workspace_size(const tde_conv_desc_t* d);
int tde_head_fwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* bias,
                 float* y, int act, float scale, float offset, void* stream);
int tde_head_bwd(const tde_conv_desc_t* d, const float* x, const float* w, const float* y,
                 const float* dy, float* dx, int accumulate_dx, float* dw, float* dbias,
                 int accumulate_dw, int act, float scale, float offset, void* ws, size_t ws_bytes,
                 void* stream);

/* ---------------------------------------------------------------- batch norm (+ReLU)
 * slim.batch_norm(center=True, scale=False, epsilon=1e-3) -> TF FusedBatchNorm(+Grad)
 * (arg_scope nets_optflow_depth.py:82-87).  z is the dense conv output [M][C] (M = N*H*W);
 * y is a channel view (y_cstride, y_coff).  Training normalises with the biased batch variance and
 * updates moving_mean/moving_var in place (v -= (v - batch) * (1 - decay)); `bessel` selects the
 * FusedBatchNorm n/(n-1) correction of the variance fed to the moving average.
 * groups G (1..8, G | M): the M rows are G equal consecutive row groups, each normalised over its OWN rows --
 * the G calls of one shared-variable network on different images (train_depth_then_cam_lr.py:130-136: disp_net
 * on the left and on the right image, separate BN batches) batched into one launch.  save_mean / save_invstd
 * are then [G][C], the moving averages take G updates in group order, and the backward's dbeta is the sum of
 * the groups' (in group order; the first overwrites unless accumulate_dbeta). */
size_t tde_bn_workspace_size(int M, int C);
int tde_bn_fwd_train(int M, int C, int groups, const float* z, const float* beta, float eps, float decay,
                     int bessel, float* moving_mean, float* moving_var, float* save_mean,
                     float* save_invstd, float* y, int y_cstride, int y_coff, int relu,
                     void* ws, size_t ws_bytes, void* stream);
int tde_bn_fwd_infer(int M, int C, const float* z, const float* beta, float eps,
                     const float* moving_mean, const float* moving_var, float* y, int y_cstride,
                     int y_coff, int relu, void* stream);
/* Fold inference BN (beta only, scale=False; eps) into the preceding conv's weights:
 * w_out = w * rsqrt(mv + eps)[k], bias_out[k] = beta[k] - mm[k] * rsqrt(mv + eps)[k] (fp64 math).
 * layout 0: conv [taps][cin][K]; layout 1: conv2d_transpose [taps][K][cin].  w_out != w. */
int tde_bn_fold(int taps, int cin, int K, int layout, const float* w, const float* moving_mean,
                const float* moving_var, const float* beta, float eps, float* w_out, float* bias_out,
                void* stream);
/* dz = d(BN+ReLU)/dz given dy (view); dbeta = sum(dy * relu'); accumulate_dbeta adds to dbeta.
 * dz_absmax (nullable): TDE_BOUND_SLOTS device floats whose max is raised to max|dz| (atomic max; the caller
 * zeroes them first) -- the bound of dz as the gradient operand of the conv backward in conv math 4
 * (tde_conv_desc_t.y_absmax). */
int tde_bn_bwd(int M, int C, int groups, const float* z, const float* save_mean, const float* save_invstd,
               const float* beta, const float* dy, int dy_cstride, int dy_coff, float* dz,
               float* dbeta, int accumulate_dbeta, int relu, float* dz_absmax, void* ws, size_t ws_bytes,
               void* stream);

/* BN-free conv / conv2d_transpose layers with bias + ReLU (the BN-free disp_net of
 * nets_optflow_depth_pairtest.py:76-147: normalizer_fn commented out at :83-84, so slim.conv2d adds biases):
 * forward = tde_conv2d_fwd_bias_act / tde_deconv2d_fwd_bias_act with the trained weights and biases; backward:
 * dz = dy * relu'(y) written dense [M][C] (y, dy are channel views of the layer's output and its gradient),
 * dbias (+)= sum_rows dz (fp64, fixed order), dz_absmax as tde_bn_bwd.  Workspace: tde_bn_workspace_size(M, C). */
int tde_bias_relu_bwd(int M, int C, const float* y, int y_cstride, int y_coff, const float* dy, int dy_cstride,
                      int dy_coff, int relu, float* dz, float* dbias, int accumulate_dbias, float* dz_absmax,
                      void* ws, size_t ws_bytes, void* stream);

/* SyncBN (BatchNorm over the batch of ALL data-parallel replicas), in two phases around
 * the caller's ONE all-reduce of `sums` (fp64 [groups][2][C]; M rows = `groups` equal row groups, each its own
 * BatchNorm batch as in tde_bn_fwd_train):
 *   forward : tde_bn_sums(mode 0), or the conv itself (tde_conv2d_fwd_bn / tde_deconv2d_fwd_bn with
 *             tde_bn_train_t.sums) -> sums = (sum z, sum z^2) per group over this replica's rows; all-reduce;
 *             tde_bn_fwd_from_sums(M, C, groups, M_total, ...) = tde_bn_fwd_train semantics over M_total rows per
 *             group, in ONE launch (statistics computed from the sums in the apply pass; block 0 publishes them
 *             and the moving averages, groups in order).
 *   backward: tde_bn_sums(mode 1) -> (sum g, sum g*xhat), g = dy * relu'(y), into `sums` and (optional) the same
 *             values into `sums_copy` (the local copy); all-reduce `sums` (global); tde_bn_bwd_from_sums: dz from
 *             the global means, dbeta from the LOCAL sum g (the data-parallel gradient average divides the summed
 *             dbeta by the replica count), one launch.
 * Replaces slim.batch_norm's moments over the single-device batch (nets_optflow_depth.py:82-87) with
 * moments over the global batch (the reference's own semantics at global batch 64 on one device). */
int tde_bn_sums(int M, int C, int groups, const float* z, const float* dy, int dy_cstride, int dy_coff,
                const float* save_mean, const float* save_invstd, const float* beta, int relu, int mode,
                double* sums, double* sums_copy, void* ws, size_t ws_bytes, void* stream);
int tde_bn_fwd_from_sums(int M, int C, int groups, long M_total, const float* z, const double* sums,
                         const float* beta, float eps, float decay, int bessel, float* moving_mean, float* moving_var,
                         float* save_mean, float* save_invstd, float* y, int y_cstride, int y_coff, int relu,
                         void* stream);
int tde_bn_bwd_from_sums(int M, int C, int groups, long M_total, const float* z, const float* save_mean,
                         const float* save_invstd, const float* beta, const float* dy, int dy_cstride, int dy_coff,
                         const double* global_sums, const double* local_sums, float* dz, float* dbeta,
                         int accumulate_dbeta, int relu, float* dz_absmax, void* stream);

/* ---------------------------------------------------------------- legacy resizes
 * resize_like -> tf.image.resize_nearest_neighbor (nets_optflow_depth.py:11-16),
 * tf.image.resize_bilinear of the disparity (nets_optflow_depth.py:124,131,138),
 * tf.image.resize_area pyramids (train_depth_then_cam_lr.py:227-232).  align_corners=False. */
int tde_resize_nearest_fwd(int N, int H, int W, int C, const float* x, int x_cstride, int x_coff,
                           int OH, int OW, float* y, int y_cstride, int y_coff, void* stream);
int tde_resize_nearest_bwd(int N, int H, int W, int C, float* dx, int dx_cstride, int dx_coff,
                           int accumulate, int OH, int OW, const float* dy, int dy_cstride,
                           int dy_coff, void* stream);
int tde_resize_bilinear_fwd(int N, int H, int W, int C, const float* x, int x_cstride, int x_coff,
                            int OH, int OW, float* y, int y_cstride, int y_coff, void* stream);
int tde_resize_bilinear_bwd(int N, int H, int W, int C, float* dx, int dx_cstride, int dx_coff,
                            int accumulate, int OH, int OW, const float* dy, int dy_cstride,
                            int dy_coff, void* stream);
int tde_resize_area_fwd(int N, int H, int W, int C, const float* x, int OH, int OW, float* y,
                        void* stream);

/* ---------------------------------------------------------------- input pipeline (device half)
 * imageselect_Dataloader_optflow.py:104-133,216-233 (read_images_from_disk + unpack_image_sequence):
 * to_float(tf.image.resize_images(decode_jpeg(file), [out_h, out_w * nframes])) -- BILINEAR,
 * align_corners=False, TF-1 legacy coordinates -- cut into nframes frames of [out_h, out_w] (frame 0 =
 * tgt_image, 1 = src_image_1), each written into an NHWC float view (3 channels at out_coff[f] of
 * out_cstride[f]).  Input: the batch's decoded uint8 HWC RGB images packed in device memory, image b at byte
 * src_off[b] with size src_hw[2b] x src_hw[2b+1] (both arrays in device memory).  Results are bit-identical
 * to the float32 restatement (no FMA contraction). */
#define TDE_MAX_FRAMES 4
typedef struct {
  int B, out_h, out_w, nframes;
  const unsigned char* src;
  const long long* src_off;
  const int* src_hw;
  float* out[TDE_MAX_FRAMES];
  int out_cstride[TDE_MAX_FRAMES];
  int out_coff[TDE_MAX_FRAMES];
} tde_image_batch_t;
int tde_image_resize_unpack(const tde_image_batch_t* args, void* stream);

/* ---------------------------------------------------------------- inference pre / post-processing (ABI 10)
 * The OpenCV steps of batch_prediction.py:62,72-73 on the GPU, restated from OpenCV 4.x's scalar reference code
 * (cv2 is a pip dependency of the reference, not vendored; parity unpinned -- oracle/cv_ops.py restates the same):
 *   I = cv2.resize(I, (224, 224), interpolation=cv2.INTER_AREA)   (:62, replaces the host cv2 call)
 * src uint8 [B,H,W,C] (C <= 4, dense) -> [B,OH,OW,C]: dst_u8 (dense) and / or dst_f32 (float of the same values,
 * pixel stride f32_cstride: e.g. the network's padded input buffer); true area averaging when both scales are >= 1
 * (integer scales: the box mean), OpenCV's area-emulating fixed-point linear path otherwise. */
int tde_resize_area_u8(int B, int H, int W, int C, const uint8_t* src, int OH, int OW, uint8_t* dst_u8,
                       float* dst_f32, int f32_cstride, void* stream);
/*   z = cv2.resize(pred[0][0,:,:,0], (image_width, image_height), interpolation=cv2.INTER_CUBIC)   (:72)
 * one channel (channel s_coff of a view with pixel stride s_cstride, e.g. a disparity output) [B,H,W] ->
 * dense float [B,OH,OW]; bicubic A = -0.75, edge taps replicated. */
int tde_resize_cubic_f32(int B, int H, int W, const float* src, int s_cstride, int s_coff, int OH, int OW,
                         float* dst, void* stream);
/*   z = cv2.bilateralFilter(z, 9, 75, 75)   (:73)
 * dense float [B,H,W] -> [B,H,W] (src != dst), each image filtered on its own: circular window of radius d/2,
 * spatial weights exp(-r^2 / 2 sigma_space^2), colour weights from a 4096-bin exp table over the image's value
 * range, BORDER_REFLECT_101; a constant image is copied.  ws: tde_bilateral_workspace_size(B) bytes. */
size_t tde_bilateral_workspace_size(int B);
int tde_bilateral_f32(int B, int H, int W, const float* src, float* dst, int d, double sigma_color,
                      double sigma_space, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- loss head
 * Fused forward+backward of the scalar loss terms: each call ADDS weight*term to loss[0] (a
 * device fp64 accumulator) and ADDS d(weight*term)/d(pred) into grad (same view layout as pred).
 *
 * compute_smooth_loss (train_depth_then_cam_lr.py:59-68) of pred (recip=0) or of 1/pred (recip=1):
 * mean|dx2| + mean|dxdy| + mean|dydx| + mean|dy2| over one channel c of a view. */
int tde_loss_smooth2(int N, int H, int W, const float* pred, int cstride, int coff, int recip,
                     float weight, double* loss, float* grad, int g_cstride, int g_coff,
                     void* stream);
/* mean|nf(label - pred)| (train_depth_only.py:183-184; replace_nonfinite when nonfinite=1,
 * train_depth_then_cam_lr.py:241-243).  label is dense [N,H,W,1]; pred is a 1-channel view. */
/* DeMoN scale-invariant-gradient loss of compute_loss_single_depth (my_losses.py:78-82, used by
 * split_training*.py:117): sig = lmbspecialops.scale_invariant_gradient per delta d (host arrays deltas /
 * weights, <= 8): w_d (f(p+d) - f(p)) / (|f(p+d)| + |f(p)| + sig_epsilon) along x and y (0 where p+d
 * leaves the image), channels concatenated (depthmotionnet.v2.losses.scale_invariant_gradient); then
 * pointwise_l2_loss(sig(pred), sig(label), epsilon) = mean_p sqrt(sum_c nf(diff_c)^2 + epsilon), label
 * under stop_gradient.  label dense [N,H,W,1] (NaN holes allowed); pred a 1-channel view.
 * lmbspecialops / DeMoN are not vendored in the reference: restated, parity unpinned. */
int tde_loss_sig_l2(int N, int H, int W, const float* pred, int cstride, int coff, const float* label,
                    int ndeltas, const int* deltas, const float* weights, float sig_epsilon, float epsilon,
                    float weight, double* loss, float* grad, int g_cstride, int g_coff, void* stream);
int tde_loss_l1(int N, int H, int W, const float* pred, int cstride, int coff, const float* label,
                int nonfinite, float weight, double* loss, float* grad, int g_cstride, int g_coff,
                void* stream);

/* The per-scale smooth + depth-L1 terms of every scale in ONE launch (train_depth_only.py:160-187;
 * the same terms inside train_depth_then_cam_lr.py:216-243, refine_depth.py:185-213):
 *   loss_smooth += sum_s smooth_w[s] * compute_smooth_loss(pred_s or 1/pred_s)
 *   loss_l1     += sum_s l1_w[s] * mean|nf(resize_area(label, 2^-s) - pred_s)|
 * pred_s / grad_s are 1-channel views at (H >> s, W >> s); label is the full-resolution [N,H,W,1]
 * (area-downsampled on the fly, H and W divisible by 2^s).  A zero weight disables a term.
 * grad_accumulate = 0 WRITES every grad_s pixel (no zeroed buffer needed), 1 adds. */
#define TDE_MAX_SCALES 4
typedef struct {
  int N, H, W, nscales;
  const float* pred[TDE_MAX_SCALES]; int pred_cs[TDE_MAX_SCALES], pred_co[TDE_MAX_SCALES];
  float* grad[TDE_MAX_SCALES]; int g_cs[TDE_MAX_SCALES], g_co[TDE_MAX_SCALES];
  float smooth_w[TDE_MAX_SCALES];
  int recip;
  const float* label;
  int nonfinite;
  float l1_w[TDE_MAX_SCALES];
  double* loss_smooth; double* loss_l1;
  int grad_accumulate;
} tde_depth_loss_t;
int tde_loss_depth_pyramid(const tde_depth_loss_t* args, void* stream);
/* n <= TDE_PYR_MULTI_MAX independent tde_loss_depth_pyramid calls (config 4's four disparity maps) in ONE launch:
 * same results as n calls when their grad views are disjoint (the loss sums are fp64 atomics either way). */
#define TDE_PYR_MULTI_MAX 4
int tde_loss_depth_pyramid_multi(const tde_depth_loss_t* args, int n, void* stream);

/* ---------------------------------------------------------------- projective warp loss head
 * Fused forward + hand-derived backward of the per-scale self-supervised terms of
 * train_depth_then_cam_lr.py:253-340 (config 4), train_optflow_combine.py:178-198 (config 3) and
 * refine_depth.py:200-212 (config 5) over utils_lr.py:151-366 (pixel2cam, cam2pixel,
 * projective_inverse_warp, bilinear_sampler) and :369-458 (consistent_depth_loss):
 *   coords: (u,v,z) = cam2pixel(P @ pixel2cam(1/disp, Kinv))  or  grid + flow (optflow_warp, :258-274)
 *   photo  : photo_w  * mean_{pix,3ch}(|bilinear(img_src,(u,v)) - img_tgt| * w_pix),
 *            w_pix = softmax(logits)[1] (exp mask), wmask (data) or 1
 *   exp    : exp_w    * mean_pix(CE(logits, [0,1]))               (compute_exp_reg_loss, :87-91)
 *   consist: consist_w* mean_pix(|z - bilinear(1/disp_other,(u,v))| * softmax(logits)[1])
 * loss[0..2] += (photo, exp, consist); gradients are ADDED into g_disp / g_flow / g_logits (same views
 * as the inputs), scattered with float atomics (or, with det_ws, deterministically) into g_other, and reduced
 * per batch element into
 * g_P[b][12] = dL/dP (fp64, +=), from which tde_pose_grad chains to the 6-DoF pose vector. */
typedef struct {
  int B, H, W;
  const float* disp; int disp_cs, disp_co;          /* projective mode: target disparity view */
  const float* flow; int flow_cs, flow_co;          /* flow mode (disp == NULL) */
  const float* P;                                    /* [B][12] rows 0..2 of K4 @ T */
  const float* Kinv;                                 /* [B][9] */
  const float* img_src;                              /* [B,H,W,3] dense, sampled */
  const float* img_tgt;                              /* [B,H,W,3] dense */
  const float* wmask;                                /* optional [B,H,W] photometric weight */
  const float* logits; int logit_cs, logit_co;       /* optional 2-channel explainability logits */
  const float* disp_other; int other_cs, other_co;   /* optional consistency source disparity */
  float photo_w, exp_w, consist_w;
  double* loss;                                      /* [3] */
  float* g_disp; float* g_flow; float* g_logits; float* g_other;
  double* g_P;                                       /* [B][12] or NULL (pose is data) */
  /* Deterministic mode (NULL: off): a device workspace of >= tde_warp_loss_det_workspace_size(B, H, W) bytes.
   * The g_other scatter then runs as 64-bit fixed-point integer atomics (associative: the same sum in any
   * order, scaled from max(1/disp_other)^2 so no pixel can overflow) added into g_other once, and the loss
   * parts / g_P leave each block as partials summed in block order -- run-to-run bit-identical results, at
   * the cost of 3 more launches.  The fixed-point sums are exact to ~2^-40 of the largest possible one. */
  void* det_ws;
  size_t det_ws_bytes;
} tde_warp_loss_t;
int tde_warp_loss(const tde_warp_loss_t* args, void* stream);
size_t tde_warp_loss_det_workspace_size(int B, int H, int W);
/* n <= TDE_WARP_MULTI_MAX tde_warp_loss calls in ONE launch (the per-scale calls of one direction of
 * train_depth_then_cam_lr.py:253-340: 8 launches per step become 2).  The calls must write disjoint
 * g_disp / g_logits views (those are plain +=; the g_other / loss / g_P sums are atomics as in tde_warp_loss),
 * must all have det_ws == NULL and either all or none compute g_P.  Results equal n tde_warp_loss calls up to
 * the float-atomic order. */
#define TDE_WARP_MULTI_MAX 8
int tde_warp_loss_multi(const tde_warp_loss_t* args, int n, void* stream);

/* Forward-only projective_inverse_warp (utils_lr.py:222-256) / bilinear_sampler (:276-366): coords from
 * depth (or 1/disp when depth_is_disp) through P and Kinv, or given coords_in [B,H,W,2] when depth is
 * NULL.  Any output may be NULL: out [B,H,W,C] (samples img [B,Hs,Ws,C]), coords [B,H,W,2],
 * flow_x/flow_y = coords - grid (depth_optflow, :472-489), wmask [B,H,W], z [B,H,W]. */
int tde_warp_fwd(int B, int H, int W, int C, const float* depth, int depth_is_disp, const float* P,
                 const float* Kinv, const float* coords_in, const float* img, int Hs, int Ws, float* out,
                 float* coords, float* flow_x, float* flow_y, float* wmask, float* z, void* stream);

/* pose_vec2mat(vec,'angleaxis') (utils_lr.py:106-149; NaN at r = 0 as in the reference) or a given 4x4
 * (format='matrix'), then P = (K4 @ T)[0:3] (:245-251) and Kinv = matrix_inverse(K) (:165).
 * T may be NULL.  K is [B][9]. */
int tde_pose_prep(int B, const float* pose_vec, const float* pose_mat, const float* K, float* T,
                  float* P, float* Kinv, void* stream);
/* n <= TDE_WARP_MULTI_MAX independent tde_pose_prep calls (every scale and direction of the config-4 loss) in
 * ONE launch; same arguments per job, same results. */
typedef struct {
  int B;
  const float* pose_vec; const float* pose_mat; const float* K;
  float* T; float* P; float* Kinv;
} tde_pose_prep_t;
int tde_pose_prep_multi(const tde_pose_prep_t* jobs, int n, void* stream);
/* ---- reference-named geometry ops with their backward (the un-fused utils_lr.py path; the host layer
 * tf_depth_estimation_amd/utils_lr.py wraps them as autograd functions).
 * pose_vec2mat(vec, format) (utils_lr.py:106-149): vec [B][6] (tx,ty,tz,rx,ry,rz) -> T [B][16];
 * format 0 'angleaxis' (Rodrigues, :77-103, NaN at r = 0), 1 'eular' (euler2mat, :26-75, angles clipped
 * to [-pi,pi]), 2 'test' (identity, zero translation). */
int tde_pose_vec2mat(int B, const float* vec, int format, float* T, void* stream);
/* dvec (+)= d<dT, T(vec)>/dvec ('eular': zero outside the clip range, as tf.clip_by_value). */
int tde_pose_vec2mat_bwd(int B, const float* vec, int format, const float* dT, float* dvec, int accumulate,
                         void* stream);
/* bilinear_sampler backward (utils_lr.py:276-366) of tde_warp_fwd's given-coords mode:
 * d_img += scatter of w*d_out (float atomics; zero it first), d_coords [B,H,W,2] = d_out . dout/dcoords
 * + d_wmask . dwmask/dcoords (d_out / d_wmask may be NULL). */
int tde_sampler_bwd(int B, int H, int W, int C, const float* coords, const float* img, int Hs, int Ws,
                    const float* d_out, const float* d_wmask, float* d_img, float* d_coords, void* stream);
/* backward of (coords, z) = cam2pixel(P, pixel2cam(depth, meshgrid, Kinv)) (utils_lr.py:151-194,
 * :240-251): d_depth (+)= ..., gP [B][12] += dL/dP (fp64).  Intrinsics are data (no gradient, as at every
 * reference call site). */
int tde_cam_coords_bwd(int B, int H, int W, const float* depth, const float* P, const float* Kinv,
                       const float* d_coords, const float* d_z, float* d_depth, int accumulate, double* gP,
                       void* stream);
/* dT [B][16] = d/dT of P = (K4 @ T)[0:3] given gP [B][12] (row 3 of dT = 0). */
int tde_pose_dp_to_dt(int B, const float* K, const double* gP, float* dT, void* stream);
/* d loss / d pose_vec from gP [nscales][B][12] (each scale's K_s at K + b*k_stride_b + 9*s) plus an
 * optional direct dL/dT [B][16]; Rodrigues backward. */
int tde_pose_grad(int B, int nscales, const float* pose_vec, const float* K, long k_stride_b,
                  const double* gP, const float* gT_extra, float* g_pose_vec, int accumulate,
                  void* stream);
/* n <= TDE_WARP_MULTI_MAX tde_pose_grad jobs in ONE launch, each optionally followed by the backward of
 * pose_avg = reduce_mean(pose_pred, [1, 2]) (nets_optflow_depth.py:183-186; tde_spatial_mean_bwd with C = 6):
 * dpose [B][hw] rows of dpose_cstride floats, channels 0..5 (+)= g_pose_vec / hw.  Same results as tde_pose_grad
 * followed by tde_spatial_mean_bwd per job (config 4's two directions: 4 launches become 1). */
typedef struct {
  int B, nscales;
  const float* pose_vec; const float* K; long k_stride_b;
  const double* gP; const float* gT_extra;
  float* g_pose_vec; int accumulate;
  float* dpose; int hw, dpose_cstride, dpose_accumulate;   /* dpose NULL: no spatial-mean backward */
} tde_pose_grad_t;
int tde_pose_grad_spread(const tde_pose_grad_t* jobs, int n, void* stream);
/* Config 4 cam loss (train_depth_then_cam_lr.py:278-286): w*mean((T_gt-T_lr)^2) +
 * w*mean((inv(T_gt)-T_rl)^2); loss += value, gT_lr/gT_rl += gradients. */
int tde_cam_loss(int B, const float* gt_vec, const float* T_lr, const float* T_rl, float weight,
                 double* loss, float* gT_lr, float* gT_rl, void* stream);

/* ---------------------------------------------------------------- optimizer
 * tf.train.AdamOptimizer (train_depth_then_cam_lr.py:413-417), TF epsilon-hat form, one launch over
 * a flat parameter buffer.  `step` is a device counter (incremented on device by tde_adam_step_begin)
 * so a captured graph replays correctly.  lr_t = lr*sqrt(1-b2^t)/(1-b1^t). */
int tde_adam_step_begin(float* step, void* stream);
/* grad_scale multiplies the gradient as it is read (1: as stored; 1/world: the data-parallel mean of a summed
 * gradient -- the captured exchange all-reduces with SUM, which RCCL skips at one rank, ABI 9). */
int tde_adam_update(size_t n, float* param, const float* grad, float* m, float* v,
                    const float* step, float lr, float beta1, float beta2, float eps, float grad_scale,
                    void* stream);

/* ---------------------------------------------------------------- utilities */
int tde_fill(size_t n, float* x, float value, void* stream);
int tde_scale(size_t n, float* x, float alpha, void* stream);   /* x *= alpha (DP gradient mean) */
int tde_zero_bytes(size_t bytes, void* p, void* stream);
/* pose_avg = tf.reduce_mean(pose_pred, [1, 2]) (nets_optflow_depth.py:183): x [N,HW,C] (pixel stride
 * x_cstride) -> y [N,C], and its gradient (dx (+)= dy/HW). */
int tde_spatial_mean_fwd(int N, int HW, int C, const float* x, int x_cstride, float* y, void* stream);
int tde_spatial_mean_bwd(int N, int HW, int C, float* dx, int dx_cstride, int accumulate, const float* dy,
                         void* stream);
/* Copy a dense [M][C] tensor into a channel view (or back when `to_view`=0). */
int tde_copy_view(int M, int C, const float* src, int s_cstride, int s_coff, float* dst,
                  int d_cstride, int d_coff, int accumulate, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TDE_H_ */
