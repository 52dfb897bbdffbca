/*
 * libhulkkp — C ABI of the MI355X-native keypoint-heatmap CNN hot path.
 *
 * Replaces the device work the reference hands to PyTorch/cuDNN implicitly
 * (reference: vainaviv/hulk-keypoints, Python only, no FFI of its own —
 * SURVEY §8(b)).  Each entry point cites the reference code whose device work
 * it performs.  The Python host layer (hulk-keypoints_amd/hkp/) binds these
 * with ctypes and re-exposes the reference's own call surface
 * (KeypointsGauss, gauss_2d_batch, Prediction, train.py forward/fit).
 *
 * Conventions
 *   - extern "C", plain pointers and sizes; no torch or C++ types cross it.
 *   - Activations are NHWC fp32, conv weights KRSC ([Cout][R][S][Cin]) fp32,
 *     except the stem, which reads the reference's NCHW image and OIHW weight.
 *   - The caller owns and allocates every buffer (device pointers).  The
 *     library never allocates, never synchronises; every launch goes on the
 *     stream argument (a hipStream_t; NULL = legacy default stream).
 *   - Return: 0 ok; <0 bad argument (see hkp_last_error()); >0 a hipError_t.
 *   - All reductions are deterministic (fixed order, no float atomics), so
 *     results are bitwise reproducible run to run.
 */
#ifndef HULKKP_H
#define HULKKP_H

#include <stddef.h>
#include <stdint.h>

#include "hkp_jpeg.h"   /* hkpj_geom: the host half of the hybrid JPEG decode */

#ifdef __cplusplus
extern "C" {
#endif

#define HKP_OK 0
#define HKP_ERR_BAD_ARG (-1)
#define HKP_ERR_UNSUPPORTED (-2)

#define HKP_LAYOUT_NHWC 0
#define HKP_LAYOUT_NCHW 1

#define HKP_LOSS_BCE 0
#define HKP_LOSS_MSE 1

typedef void* hkp_stream_t;

/* thread-local message of the last failing call on this thread */
const char* hkp_last_error(void);
/* "hulkkp <version> gfx950" */
const char* hkp_version(void);

/* ---------------------------------------------------------------- conv ---- */
typedef struct hkp_conv_desc {
    int32_t n, h, w, c;             /* input batch, height, width, channels            */
    int32_t k, r, s;                /* output channels, filter height, filter width    */
    int32_t stride, pad, dilation;  /* symmetric                                        */
    int32_t in_layout;              /* HKP_LAYOUT_NHWC, or HKP_LAYOUT_NCHW (stem only)  */
    int32_t tile;                   /* x3 / fp16 conv tile policy, HKP_TILE_* (0: the
                                       planner).  Per call — no process-global state */
} hkp_conv_desc;

/* Tile policies of the packed-operand convs (hkp_conv2d_fwd_x3 / _fwd_f16 /
 * _bwd_data_x3 / _bwd_data_x3_strided).  AUTO: fewest rounds of blocks over the
 * CUs weighted by the measured per-column cost of each tile width (256x256,
 * 256x128, 256x64), data-parallel or stream-K (with a workspace).  The others
 * force one kernel body (for tests and tuning; outputs agree to fp32 summation
 * order): NO_SK never stream-K; SK stream-K wherever a tile split helps;
 * 256 = 256x256 16x16x32 (Cout % 256 == 0); 128_MF16 / 128_MF32 = 256x128 with
 * 16x16x32 / 32x32x16 MFMAs; 64_PAIR = 256x64, two blocks per CU. */
#define HKP_TILE_AUTO 0
#define HKP_TILE_NO_SK 1
#define HKP_TILE_SK 2
#define HKP_TILE_256 3
#define HKP_TILE_128_MF16 4
#define HKP_TILE_128_MF32 5
#define HKP_TILE_64_PAIR 6
#define HKP_TILE_RESERVED_7 7         /* retired: the persistent conv (measured slower */
#define HKP_TILE_RESERVED_8 8         /* than the one-tile grid); rejected with HKP_ERR_ARG */
#define HKP_TILE_256_TAIL 9           /* 256x256; tiles past the last full round as split-K segments */
#define HKP_TILE_HALO 10              /* 8x32-pixel halo tiles (stride-1 3x3, pad = dil = 1, Ho%8 = Wo%32 = 0;
                                         the default there under AUTO and 256_TAIL when the
                                         input has 64 channels) */
#define HKP_TILE_AUTO_A3 12           /* the round-4 planner: AUTO without its plain-fp16 DUO
                                         choices (K-depth 64, 128-wide outputs) */
#define HKP_TILE_256_A3 11            /* 256x256 on the A3 body (A ring 3 stages deep, B ring 2: an A
                                         line has two K-steps to land) + the split-K tail of 9 */
#define HKP_TILE_DUO 13               /* plain fp16 (hkp_conv2d_fwd_f16 / _f16_bn) only: 256x128 tiles,
                                         two 4-wave blocks per CU (one block's fill and epilogue
                                         beside the other's K loop); Cout % 128 == 0; other
                                         operand layouts plan as AUTO */
#define HKP_TILE_RESERVED_14 14      /* retired: the persistent A3 body (measured slower on every shape,
                                         round 5); rejected with HKP_ERR_BAD_ARG */
#define HKP_TILE_192_A3 15            /* packed operands (x3 forward / dgrad), Cout % 256 == 0: the A3
                                         body on 192 x 256 tiles (one partial round of 256-row
                                         tiles on many fewer tiles than CUs); its BN partials are
                                         per 96-row tile: hkp_bn_finalize(..., tile_rows = 96, ...)
                                         over ceil(M / 96) tiles.  Other shapes plan as AUTO */
#define HKP_TILE_160_A3 16            /* the same on 160 x 256 tiles (waves 2 x 4; 160 x 128 where
                                         Cout % 256 != 0, Cout % 128 == 0), BN partials per 80-row
                                         tile (tile_rows = 80) */

/* output spatial size: (h + 2*pad - dilation*(r-1) - 1)/stride + 1 */
int hkp_conv_out_hw(const hkp_conv_desc* d, int32_t* ho, int32_t* wo);

/* number of BatchNorm statistic tiles the conv epilogue emits; the
 * stat_partials buffer holds tiles * k * 2 floats */
int64_t hkp_conv_stat_tiles(const hkp_conv_desc* d);

/* y[n,ho,wo,k] = sum_{r,s,c} x[n, ho*st-pad+r*dil, wo*st-pad+s*dil, c] * w[k,r,s,c]
 * (zero padding, no bias) on fp32 MFMA (v_mfma_f32_32x32x2_f32).
 * Replaces: conv3x3 src/resnet.py:20-37 (BasicBlock :45,48; Bottleneck :80),
 *           1x1 convs src/resnet.py:77,86 and downsample :184-188,
 *           stem conv src/resnet.py:137,199 (in_layout NCHW, w OIHW).
 * If stat_partials != NULL the epilogue also writes per-tile per-channel
 * (sum, sum of squared deviations from the tile mean) for train-mode BN. */
int hkp_conv2d_fwd(const hkp_conv_desc* d, const float* x, const float* w, float* y,
                   float* stat_partials, hkp_stream_t stream);

/* The f16x3 conv of the main path (same conv and epilogue as hkp_conv2d_fwd;
 * fp32-class accuracy) on operands pre-split into the "packed split" layout:
 * per pixel (weights: per output channel and filter tap) and per 32-channel
 * group one 128-B line [hi 32 | lo 32] (fp16 bit patterns), hi = f16(v),
 * lo = f16(v - hi); the conv sums hi*hi + hi*lo + lo*hi in fp32.
 *   x_split[n*h*w][c/32][64]   written by hkp_bn_apply / hkp_bn_relu_maxpool with
 *                              split_passes = 3 (v = the activation),
 *   w_split[k][r*s][c/32][64]  written by hkp_weight_pack_x3 from KRSC fp32, each
 *                              output channel scaled by a power of two (max|w| ->
 *                              [2^13, 2^14)); w_inv_scale[k] = the inverse, which
 *                              the conv applies to its output.
 * Needs c % 32 == 0 and k % 64 == 0.  Replaces the same convs as hkp_conv2d_fwd. */
int hkp_weight_pack_x3(int32_t k, int32_t rsc, int32_t c, const float* w, uint16_t* w_split, float* w_inv_scale,
                       hkp_stream_t stream);
int hkp_conv2d_fwd_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                      const float* w_inv_scale, float* y, float* stat_partials, void* sk_workspace,
                      int64_t sk_ws_bytes, hkp_stream_t stream);
/* Stream-K workspace of the x3 convs (hkp_conv2d_fwd_x3, hkp_conv2d_bwd_data_x3,
 * hkp_conv2d_bwd_data_x3_strided; nullable: then every launch is one tile per
 * block).  With it, a launch whose tiles fill the CUs poorly (e.g. 300 tiles on
 * 256 CUs) splits tiles x K-steps evenly over one block per CU and sums each split
 * tile's fp32 segments in fixed segment order (deterministic).  Its first 64 KiB
 * are arrival counters that must be ZERO before the first call; every call
 * leaves them zero (allocate once, zeroed, per stream: calls on one workspace
 * must not run concurrently).  Size: hkp_conv_x3_sk_workspace_bytes(). */
int64_t hkp_conv_x3_sk_workspace_bytes(void);
/* hkp_conv2d_fwd_x3 with a chosen subset of the three f16x3 products (inference
 * precision modes between config C4's plain fp16 and f16x3; same operands,
 * outputs and workspace).  products: HKP_X3_ALL = hkp_conv2d_fwd_x3;
 * HKP_X3_W16 = hi_x*hi_w + lo_x*hi_w (the weights rounded to fp16 after their
 * per-channel power-of-two scale, the activation kept to ~2^-22); HKP_X3_X16 =
 * hi_x*hi_w + hi_x*lo_w (the activation rounded to fp16, the weights kept).
 * Two fp16 MFMAs per 32 channels instead of three.  Replaces the same convs as
 * hkp_conv2d_fwd_x3 (src/resnet.py:20-37,77,86,184-188). */
#define HKP_X3_ALL 3
#define HKP_X3_W16 2
#define HKP_X3_X16 4
int hkp_conv2d_fwd_x3_products(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                               const float* w_inv_scale, int32_t products, float* y, float* stat_partials,
                               void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream);
/* Inference: hkp_conv2d_fwd_x3 whose input is the producer conv's raw output,
 * with the producer's train-mode BN + ReLU applied in the conv itself — the
 * bn_apply pass between a BasicBlock's / Bottleneck's inner convs
 * (src/resnet.py:46-48 / 80-86: relu(bn1(conv1 x)) feeding conv2) disappears.
 * x_raw: fp32 NHWC [n][h][w][c]; in_scale_shift: [2c] scale | shift from
 * hkp_bn_finalize (or hkp_bn_finalize_ranks) of that output; the A operand is
 * relu(x * scale + shift) with bn_apply's arithmetic (two roundings), split as
 * hkp_bn_apply(split = 3) would write it — so y is bit-identical to hkp_bn_apply
 * followed by hkp_conv2d_fwd_x3 with the same d->tile and workspace.  Runs
 * where that unfused launch runs the halo-tile body (stride-1 3x3, pad = dil =
 * 1, Ho % 8 == 0, Wo % 32 == 0) — the kernel hkp_conv_kernel_name names for
 * HKP_KOP_FWD_X3, with "_bnin" before "_kernel"; other launches return
 * HKP_ERR_BAD_ARG. */
int hkp_conv2d_fwd_x3_bnin(const hkp_conv_desc* d, const float* x_raw, const float* in_scale_shift,
                           const uint16_t* w_split, const float* w_inv_scale, float* y, float* stat_partials,
                           void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream);
/* The plain-fp16 form (config C4): x_raw_f16 is the producer's fp16 output,
 * relu(x * scale + shift) rounded to fp16 as hkp_bn_apply_f16 writes it; the
 * halo-tile body only. */
int hkp_conv2d_fwd_f16_bnin(const hkp_conv_desc* d, const uint16_t* x_raw_f16, const float* in_scale_shift,
                            const uint16_t* w_f16, const float* w_inv_scale, uint16_t* y_f16, float* stat_partials,
                            void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream);
/* Plain-fp16 conv (BASELINE config C4, "fp16 with MFMA"): the same LDS-DMA
 * kernel family as hkp_conv2d_fwd_x3 with one fp16 product per MAC (fp32
 * accumulation).  x_f16: NHWC fp16 [n][h][w][c] (a producer's split_passes = 1
 * output); w_f16: KRSC fp16 written by hkp_weight_pack_f16 (each output channel
 * scaled by a power of two, max|w| -> [2^13, 2^14); w_inv_scale[k] the inverse).
 * Output y_f16: fp16 NHWC (autocast semantics; the tile is staged in LDS and
 * written as whole 16-B row chunks); BN partials from the fp32 accumulators.
 * Needs c % 64 == 0 and k % 64 == 0.  Stream-K workspace as hkp_conv2d_fwd_x3. */
int hkp_weight_pack_f16(int32_t k, int32_t rsc, const float* w, uint16_t* w_f16, float* w_inv_scale,
                        hkp_stream_t stream);
int hkp_conv2d_fwd_f16(const hkp_conv_desc* d, const uint16_t* x_f16, const uint16_t* w_f16,
                       const float* w_inv_scale, uint16_t* y_f16, float* stat_partials, void* sk_workspace,
                       int64_t sk_ws_bytes, hkp_stream_t stream);
/* The plain-fp16 conv with the output's train-mode BN apply fused into its
 * epilogue (config C4's Bottleneck tail, src/resnet.py:106-110: bn3, + residual,
 * ReLU): out_f16 = [relu](y*scale + shift [+ res | + res*rscale + rshift]) on the
 * fp16-rounded conv output y — hkp_bn_apply_f16's arithmetic, so the result is
 * what hkp_conv2d_fwd_f16 + hkp_bn_apply_f16 give with the same scale_shift [2k].
 * y is never written.  res_f16 [n*ho*wo][k] (nullable), res_scale_shift [2k]
 * (nullable: raw residual).  The scale/shift must be known before the conv:
 * eval-mode BN, or train-mode statistics from the input's second moments
 * (hkp_gram_f16 + hkp_bn_from_gram, 1x1 convs).  Stream-K workspace as
 * hkp_conv2d_fwd_x3. */
int hkp_conv2d_fwd_f16_bn(const hkp_conv_desc* d, const uint16_t* x_f16, const uint16_t* w_f16,
                          const float* w_inv_scale, const float* scale_shift, const uint16_t* res_f16,
                          const float* res_scale_shift, int32_t relu, uint16_t* out_f16, void* sk_workspace,
                          int64_t sk_ws_bytes, hkp_stream_t stream);
/* Train-mode BN statistics of a 1x1 conv's output y = W a without a pass over y
 * (replaces the batch statistics of bn3, src/resnet.py:106-108, for
 * hkp_conv2d_fwd_f16_bn): hkp_gram_f16 reduces the fp16 input a [m][c] (c % 64
 * == 0, c <= 2048) to its mean mu [c] and second moments E = a^T a / m [c][c]
 * (fp64; fp32 MFMA partials over row splits of <= 16 k rows, merged in fp64 in
 * fixed order; workspace hkp_gram_f16_workspace_bytes(m, c)); hkp_bn_from_gram
 * takes, per output channel k of the packed fp16 weight w_f16 [k][c] (x
 * w_inv_scale[k], hkp_weight_pack_f16 — the weights the conv multiplies with),
 * mean = w.mu and var = w^T E w - mean^2 (fp64), and writes hkp_bn_finalize's
 * outputs from them
 * (scale_shift, mean_invstd (nullable), running stats with the unbiased
 * variance, num_batches_tracked += 1); workspace hkp_bn_from_gram_workspace_bytes(k,
 * c) (per-column-block partial sums, merged in fixed order). */
int64_t hkp_gram_f16_workspace_bytes(int64_t m, int32_t c);
int hkp_gram_f16(int64_t m, int32_t c, const uint16_t* a, double* mean, double* second, void* workspace,
                 int64_t ws_bytes, hkp_stream_t stream);
int64_t hkp_bn_from_gram_workspace_bytes(int32_t k, int32_t c);
int hkp_bn_from_gram(int32_t k, int32_t c, int64_t count, const double* mean, const double* second,
                     const uint16_t* w_f16, const float* w_inv_scale, const float* gamma, const float* beta,
                     float momentum, float eps, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float* scale_shift, float* mean_invstd, void* workspace,
                     int64_t ws_bytes, hkp_stream_t stream);
/* The kernel a launch with descriptor d runs — its template name as rocprofv3
 * reports it (e.g. "conv_x3_kernel<256, false, false, 16, false, 3>"), for
 * profiling / roofline attribution.  op: HKP_KOP_*; stream_k_ok: whether the
 * call passes a stream-K workspace.  Writes at most len bytes (NUL-terminated);
 * returns the name's length, or < 0 on bad args. */
#define HKP_KOP_FWD_X3 0
#define HKP_KOP_DGRAD_X3 1
#define HKP_KOP_FWD_F16 2
#define HKP_KOP_STEM_X3 3
#define HKP_KOP_WGRAD_X3 4
#define HKP_KOP_FWD_X3_W16 5   /* hkp_conv2d_fwd_x3_products(HKP_X3_W16) */
#define HKP_KOP_FWD_X3_X16 6   /* hkp_conv2d_fwd_x3_products(HKP_X3_X16) */
#define HKP_KOP_STEM_X3_IMAGE 7     /* hkp_conv2d_fwd_stem_x3_image, fp32 NCHW image */
#define HKP_KOP_STEM_X3_IMAGE_U8 8  /* hkp_conv2d_fwd_stem_x3_image, uint8 NHWC batch */
int32_t hkp_conv_kernel_name(const hkp_conv_desc* d, int32_t op, int32_t stream_k_ok, char* buf, int32_t len);
/* Rows per BN statistic tile of a packed forward conv (op HKP_KOP_FWD_X3 / _W16 /
 * _X16) with this descriptor: 96 with d->tile == HKP_TILE_192_A3 (k % 256 == 0), 80
 * with HKP_TILE_160_A3 (k % 128 == 0), else 128 (hkp_conv_stat_tiles' tiles).  stat_partials then holds
 * ceil(M / rows) * k * 2 floats, and hkp_bn_finalize / _ws / hkp_bn_stats take
 * tile_rows = rows (src/resnet.py:46,49: the statistics are the same). */
int32_t hkp_conv_x3_stat_tile_rows(const hkp_conv_desc* d, int32_t op);

/* (The A/B instruments — hkp_debug_* — are not part of this library: they exist only
 * in the tools build, include/hulkkp_ab.h.) */

/* ----------------------------------------------------------- batchnorm ---- */
/* Train-mode BatchNorm2d statistics (src/resnet.py:46,49,78,85,87,139,187;
 * nn.BatchNorm2d defaults eps=1e-5, momentum=0.1): merges the conv's tile
 * partials in fp64 (Chan), writes scale_shift = [gamma*invstd | beta - mean*scale],
 * mean_invstd = [mean | invstd] (nullable), and updates the running stats
 * (unbiased variance; nullable) and num_batches_tracked (nullable, +1). */
int hkp_bn_finalize(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                    const float* gamma, const float* beta, float momentum, float eps,
                    float* running_mean, float* running_var, int64_t* num_batches_tracked,
                    float* scale_shift, float* mean_invstd, hkp_stream_t stream);

/* The same statistics in two levels for long tile lists (tiles > 128): chunks of
 * 128 tiles reduced by [C/64][chunks] blocks into a caller-allocated fp64
 * workspace of hkp_bn_finalize_workspace_bytes(c, tiles) bytes, then merged per
 * channel in fixed order (Chan at both levels).  Same outputs and argument
 * meaning as hkp_bn_finalize (src/resnet.py:46,49,78,85,87,139,187); the two
 * forms agree to fp64 summation order. */
int64_t hkp_bn_finalize_workspace_bytes(int32_t c, int64_t tiles);
int hkp_bn_finalize_ws(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                       const float* gamma, const float* beta, float momentum, float eps,
                       float* running_mean, float* running_var, int64_t* num_batches_tracked,
                       float* scale_shift, float* mean_invstd, void* workspace, int64_t ws_bytes,
                       hkp_stream_t stream);

/* SyncBN for data-parallel ranks (caveat D5: train-mode BN makes a
 * shard's outputs depend on the shard; torch.nn.SyncBatchNorm's forward
 * statistics).  hkp_bn_stats: this rank's per-channel statistics from its conv
 * tile partials, written as stats = [mean[c] | M2[c] | count] (2c+1 fp64) —
 * the merge of hkp_bn_finalize (workspace == NULL) or hkp_bn_finalize_ws
 * (workspace of hkp_bn_finalize_workspace_bytes) without the scale/shift.  The
 * caller all-gathers the blocks in rank order into stats[nranks][2c+1], and
 * hkp_bn_finalize_ranks merges them in fixed rank order (Chan:
 * mean = sum n_r mean_r / N, M2 = sum M2_r + n_r (mean_r - mean)^2) into the same
 * outputs as hkp_bn_finalize over the global batch (running stats with the global
 * count's unbiased variance, num_batches_tracked += 1).  Identical bytes on every
 * rank.  Replaces the batch statistics of nn.BatchNorm2d.forward
 * (src/resnet.py:46,49,78,85,87,139,187) for a batch sharded over ranks. */
int hkp_bn_stats(int32_t c, int64_t count, int64_t tiles, int32_t tile_rows, const float* partials,
                 double* stats, void* workspace, int64_t ws_bytes, hkp_stream_t stream);
int hkp_bn_finalize_ranks(int32_t c, int32_t nranks, const double* stats, const float* gamma, const float* beta,
                          float momentum, float eps, float* running_mean, float* running_var,
                          int64_t* num_batches_tracked, float* scale_shift, float* mean_invstd,
                          hkp_stream_t stream);

/* Eval-mode BN parameters from running statistics (the reference never uses
 * them; offered as an option). */
int hkp_bn_eval_params(int32_t c, const float* gamma, const float* beta, const float* running_mean,
                       const float* running_var, float eps, float* scale_shift, float* mean_invstd,
                       hkp_stream_t stream);

/* out = [relu]( y*scale + shift  [+ res | + res*rscale + rshift] ), NHWC [m][c].
 * Replaces the bn→relu / bn→(+residual)→relu tails of BasicBlock
 * (src/resnet.py:57-67) and Bottleneck (:96-110). res may be NULL;
 * res_scale_shift NULL means the residual is added raw.  res_split (instead of res;
 * c % 32 == 0): the raw residual read from its packed split, hi + lo (the block
 * input a producer wrote split-only: inference keeps the residual stream as an
 * fp16 pair with a 22-bit significand instead of fp32).
 * out_split (nullable; needs c % 32 == 0): the same values also written as the
 * next conv's operand — split_passes = 1: fp16 plane [m][c] for
 * hkp_conv2d_fwd_f16; split_passes = 3: the packed split layout
 * [m][c/32][hi32|lo32] (hi = f16(out), lo = f16(out-hi)) for
 * hkp_conv2d_fwd_x3.  out may be NULL when out_split is given (an activation
 * only a conv consumes).  hkp_bn_relu_maxpool takes the same optional split. */
int hkp_bn_apply(int64_t m, int32_t c, const float* y, const float* scale_shift, const float* res,
                 const float* res_scale_shift, const uint16_t* res_split, int32_t relu, float* out,
                 uint16_t* out_split, int32_t split_passes, hkp_stream_t stream);

/* Plain-fp16 path (BASELINE config C4; autocast semantics): out (fp16) =
 * [relu](y*scale + shift [+ res | + res*rscale + rshift]) for an fp16 conv output
 * y [m][c] (hkp_conv2d_fwd_f16), fp16 residual res (the block input, or with
 * res_scale_shift the downsample conv's fp16 y); the arithmetic is fp32.  out32
 * (nullable): the same values in fp32 (the block feeding the head).  c % 8 == 0. */
int hkp_bn_apply_f16(int64_t m, int32_t c, const uint16_t* y, const float* scale_shift, const uint16_t* res,
                     const float* res_scale_shift, int32_t relu, uint16_t* out, float* out32, hkp_stream_t stream);

/* Stem tail: maxpool3x3/s2/p1( relu( y*scale + shift ) ), NHWC
 * (src/resnet.py:139-141, 200-202). Output [n, (h-1)/2+1, (w-1)/2+1, c].
 * route (nullable; training): per output element the window tap 0..8 (r*3+s)
 * of its first maximum — the pixel max_pool2d's backward routes the gradient
 * to — or 255 when the maximum is <= 0 (the ReLU derivative there is 0). */
int hkp_bn_relu_maxpool(int32_t n, int32_t h, int32_t w, int32_t c, const float* y,
                        const float* scale_shift, float* out, uint16_t* out_split, int32_t split_passes,
                        uint8_t* route, hkp_stream_t stream);

/* ---------------------------------------------------------------- head ---- */
/* K-channel 1x1 scoring conv + bias (src/resnet_dilated.py:16 sliced to the K
 * rows src/model.py:21 keeps): feat NHWC [n,hw,c] → lowres [n,k,hw]. */
int hkp_head_fc(int32_t n, int32_t hw, int32_t c, int32_t k, const float* feat, const float* w,
                const float* bias, float* lowres, hkp_stream_t stream);

/* Inference tail: the last block's BN apply (+ residual, ReLU — hkp_bn_apply /
 * hkp_bn_apply_f16's arithmetic) fused with hkp_head_fc, so the final feature
 * map is never written (src/resnet.py:110-112 / :68-69 of the last block, then
 * src/resnet_dilated.py:16 sliced to the K rows src/model.py:21 keeps).
 * y [n*hw][c] fp32 (y_f16 = 0) or fp16 (y_f16 = 1); res_kind 0: none, 1: raw
 * residual of y's dtype, 2: residual * rscale + rshift (res_scale_shift [2c]),
 * 3: packed split raw residual (fp32 y only); w [k][c], bias [k] →
 * lowres [n][k][hw].  Needs c % 512 == 0, c <= 2048, k <= 16.  fp16 y with
 * k <= 8 (config C4): the fp32 apply's result enters the head rounded to fp16,
 * against fp16-rounded head rows, fp32 accumulation (autocast's ReLU output and
 * 1x1 conv; MFMA). */
int hkp_bn_apply_head(int32_t n, int32_t hw, int32_t c, int32_t k, int32_t y_f16, const void* y,
                      const float* scale_shift, const void* res, const float* res_scale_shift, int32_t res_kind,
                      const float* w, const float* bias, float* lowres, hkp_stream_t stream);

/* bilinear align_corners=True upsample [n,k,h,w] → [n,k,H,W]
 * (src/resnet_dilated.py:27) + sigmoid (src/model.py:21; skipped when
 * apply_sigmoid == 0, the raw Resnet34_8s.forward output), NCHW output (nullable),
 * and the per-(n,k) argmax (src/prediction.py:46, first index wins) as
 * int32 (y, x) pairs in argmax_yx [n*k*2] (nullable).  argmax_ws: workspace of
 * hkp_upsample_argmax_ws_bytes(n,k,H,W) bytes (one key per 1024-pixel block per
 * plane; reduced in fixed order, no atomics), required when argmax_yx != NULL. */
int64_t hkp_upsample_argmax_ws_bytes(int32_t n, int32_t k, int32_t H, int32_t W);
int hkp_upsample_sigmoid(int32_t n, int32_t k, int32_t h, int32_t w, int32_t H, int32_t W,
                         int32_t apply_sigmoid, const float* lowres, float* heat, uint64_t* argmax_ws, int32_t* argmax_yx,
                         hkp_stream_t stream);

/* On-GPU visualisation (Prediction.plot, src/prediction.py:40-66):
 * per heatmap plane cv2.normalize NORM_MINMAX → .astype(uint8) (double scale /
 * shift, truncation), JET colour map (BGR; analytic — OpenCV's LUT is not in
 * this image, so cv2-pixel parity is unpinned), cv2.addWeighted(img, 0.65, map,
 * 0.35, 0) (rounded, saturated), a black filled radius-4 disc at argmax_yx as
 * cv2.circle's midpoint rasteriser draws it, tiled into the reference's grid:
 * planes k < K/2 stacked in column 0, the rest in column 1 — out
 * [n][H*K/2][2W][3] uint8 (K = 1: [n][H][W][3]; other odd K rejected, as the
 * reference's hconcat of unequal columns fails).  heat NCHW [n,k,H,W] fp32,
 * img_nhwc [n,H,W,3] uint8 BGR, argmax_yx [n,k,2] int32 (hkp_upsample_sigmoid),
 * minmax_ws [n*k*2] floats of workspace. */
int hkp_heat_overlay(int32_t n, int32_t k, int32_t H, int32_t W, const float* heat, const uint8_t* img_nhwc,
                     const int32_t* argmax_yx, float* minmax_ws, uint8_t* out, hkp_stream_t stream);

/* Soft-argmax per heatmap plane, the reference's Prediction.expectation
 * (src/prediction.py:31-38) with its axis mix-up fixed: p = softmax(beta * h)
 * over the plane (beta = 1: the reference's softmax), out_xy[n][k] = (sum p*x,
 * sum p*y) as fp32 from fp64 sums in fixed order (deterministic). */
int hkp_soft_argmax(int32_t n, int32_t k, int32_t H, int32_t W, float beta, const float* heat, float* out_xy,
                    hkp_stream_t stream);

/* Gaussian target (src/dataset.py:36-44): out[n,k,H,W] (fp64) =
 * (double) expf( -((x-u)^2 + (y-v)^2) / (2 sigma^2) ) computed in fp32;
 * uv [n,k,2] fp32 (u = column, v = row). */
int hkp_gauss_target(int32_t n, int32_t k, int32_t H, int32_t W, float sigma, const float* uv,
                     double* out, hkp_stream_t stream);

/* ============================================================ backward ==== */
/* Everything loss.backward() (train.py:35) runs through the reference's
 * modules, as hand-written kernels.  d = the FORWARD conv descriptor. */

/* w_flip[c][r][s][k] = w[k][R-1-r][S-1-s][c]: the dgrad weight (KRSC in → CRSK-flipped out). */
int hkp_conv_weight_flip(const hkp_conv_desc* d, const float* w, float* w_flip, hkp_stream_t stream);

/* dx[n,h,w,c] = sum over taps/k of dy * w (+ add[n,h,w,c], nullable: fuses the
 * residual-branch gradient sum): backward-data of hkp_conv2d_fwd (NHWC convs;
 * strided convs take the transposed-loader path).  w_flip from hkp_conv_weight_flip. */
int hkp_conv2d_bwd_data(const hkp_conv_desc* d, const float* dy, const float* w_flip, const float* add, float* dx,
                        hkp_stream_t stream);

/* max |x| as an IEEE bit pattern in amax_bits[0] (non-negative floats order like
 * their bits): the power-of-two gradient scale of the f16x3 backward convs
 * (dy_amax_bits of hkp_conv2d_bwd_data_x3 / _filter_x3 and hkp_split_pack_x3)
 * when no BN backward bound is at hand.  n % 4 == 0. */
int hkp_absmax(int64_t n, const float* x, uint32_t* amax_bits, hkp_stream_t stream);

/* The stem conv (7x7, stride 2, pad 3, NCHW input with C <= 4; src/resnet.py:137,199)
 * on the f16x3 path: hkp_stem_pack_x3 writes the image as zero-padded NHWC4 fp16
 * planes [2][n][2*ho+6][2*wo+6][4] (hi, then lo; hkp_stem_pack_x3_elems halves),
 * hkp_stem_weight_pack_x3 the OIHW weight as [k][7][hi32|lo32] (k*7*64 halves,
 * per-output-channel power-of-two scale, inverse in w_inv_scale[k]),
 * hkp_conv2d_fwd_stem_x3 = hkp_conv2d_fwd on them (NHWC fp32 y + BN partials). */
int64_t hkp_stem_pack_x3_elems(const hkp_conv_desc* d);
int hkp_stem_pack_x3(const hkp_conv_desc* d, const float* x_nchw, uint16_t* x_split, hkp_stream_t stream);
/* Device data path: the same planes straight from the uint8 batch
 * cv2.imread gives — img_nhwc [n][h][w][c] (BGR, c = d->c = 3), x = u8 / 255 in
 * fp32 exactly as ToTensor (src/dataset.py:16,71): 3 B per pixel read instead of
 * 12, and no fp32 image in HBM or over PCIe. */
int hkp_stem_pack_x3_u8(const hkp_conv_desc* d, const uint8_t* img_nhwc, uint16_t* x_split, hkp_stream_t stream);
/* ToTensor on the device: uint8 [n][h][w][c] → fp32 NCHW / 255 (the training path's
 * stem wgrad operand, and any consumer that wants the reference's tensor). */
int hkp_images_u8_to_nchw(int32_t n, int32_t h, int32_t w, int32_t c, const uint8_t* img_nhwc, float* x_nchw,
                          hkp_stream_t stream);
int hkp_stem_weight_pack_x3(int32_t k, int32_t c, const float* w_oihw, uint16_t* w_split, float* w_inv_scale,
                            hkp_stream_t stream);
int hkp_conv2d_fwd_stem_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* w_split,
                           const float* w_inv_scale, float* y, float* stat_partials, hkp_stream_t stream);
/* The stem straight from the image where the patch body takes the shape (output
 * height % 8 == 0, width % 32 == 0, d->tile != HKP_TILE_64_PAIR: hkp_stem_x3_image_ok
 * returns 1): the fp32 NCHW image (image_u8 = 0) or the uint8 NHWC batch (1), split
 * in LDS per 8x32-pixel tile with hkp_stem_pack_x3's arithmetic — the same y and
 * partials bit for bit, without writing or reading the packed planes. */
int32_t hkp_stem_x3_image_ok(const hkp_conv_desc* d);
int hkp_conv2d_fwd_stem_x3_image(const hkp_conv_desc* d, const void* image, int32_t image_u8, const uint16_t* w_split,
                                 const float* w_inv_scale, float* y, float* stat_partials, hkp_stream_t stream);

/* f16x3 backward on packed split operands (the layout of hkp_conv2d_fwd_x3):
 *   hkp_split_pack_x3:       x * 2^e → packed split [n/c][c/32][64]; 2^e from
 *                            amax_bits (max|x| as from hkp_absmax; NULL: 2^0) puts
 *                            max|x|*2^e in [2^13, 2^14) — gradients far below
 *                            fp16's normal range keep fp32-class accuracy.
 *   hkp_weight_flip_pack_x3: KRSC w → packed flipped [c][r][s][k/32][64] (dgrad
 *                            operand), per-row power-of-two scale, inverse in
 *                            wf_inv_scale[c].
 *   hkp_conv2d_bwd_data_x3:  dx = conv(dy, flipped w) + add for stride-1 convs,
 *                            dy_split packed with the scale of dy_amax_bits;
 *                            needs Cin % 64 == 0, Cout % 32 == 0.
 *   hkp_conv2d_bwd_filter_x3: dw (KRSC) from x_split (forward operand) and dy_split;
 *                            split-K over output pixels into `workspace`
 *                            (hkp_conv_bwd_filter_x3_workspace bytes), fixed-order
 *                            reduce; needs Cout % 64 == 0, Cin % 32 == 0.  Here
 *                            d->tile is the number of CUs the grid should occupy
 *                            (0: the planner's split count, which fills whole
 *                            rounds of all CUs; a wgrad sharing the GPU with a
 *                            dgrad may take fewer): splits = max(1, tile / tiles).
 *                            3x3 stride-1 pad-1 convs with Cin, Cout in {64, 128},
 *                            Ho % 4 == 0 and Wo % 16 == 0 run the halo body
 *                            (wgrad_x3_halo_kernel: 64 Cout x 9 taps x 64 Cin per
 *                            block, 4x16-pixel patches staged once for every tap);
 *                            tile == -1 keeps the tiled body for them.
 * Replace the same cuDNN backward calls as hkp_conv2d_bwd_data / _filter. */
int hkp_split_pack_x3(int64_t n, int32_t c, const float* x, const uint32_t* amax_bits, uint16_t* x_split,
                      hkp_stream_t stream);
int hkp_weight_flip_pack_x3(const hkp_conv_desc* d, const float* w, uint16_t* wf_split, float* wf_inv_scale,
                            hkp_stream_t stream);
int hkp_conv2d_bwd_data_x3(const hkp_conv_desc* d, const uint16_t* dy_split, const uint16_t* wf_split,
                           const float* wf_inv_scale, const uint32_t* dy_amax_bits, const float* add, float* dx,
                           void* sk_workspace, int64_t sk_ws_bytes, hkp_stream_t stream);
/* Strided (stride 2, dilation 1) backward-data on the f16x3 path: dx is computed
 * per output phase (py, px) as a stride-1 conv of dy with that phase's taps
 * (phase_split[py*2+px] = kind-2 packs of hkp_weight_pack_x3_batch, inverse
 * scales phase_inv_scale[..]) written to dx pixels (2a+py, 2b+px); a phase no tap
 * reaches (NULL entry; e.g. the odd pixels of a 1x1 stride-2 downsample) gets
 * dx = add (or 0).  d = the forward descriptor; needs Cin % 64 == 0, Cout % 32 == 0.
 * hkp_phase_taps: taps of phase `phase` along an axis of r taps (0: none, -1: bad args). */
int32_t hkp_phase_taps(int32_t r, int32_t pad, int32_t stride, int32_t phase);
int hkp_conv2d_bwd_data_x3_strided(const hkp_conv_desc* d, const uint16_t* dy_split,
                                   const uint16_t* const* phase_split, const float* const* phase_inv_scale,
                                   const uint32_t* dy_amax_bits, const float* add, float* dx, void* sk_workspace,
                                   int64_t sk_ws_bytes, hkp_stream_t stream);
/* Batched weight packing for a training step (one launch pair for a whole
 * network instead of one hkp_weight_pack_x3 / hkp_weight_flip_pack_x3 per conv;
 * outputs bit-identical to those).  jobs: host array; kind 0 = forward pack
 * (out = w_split [k][rs][c/32][64], inv_scale [k]; needs c % 32 == 0), kind 1 =
 * flipped dgrad pack (out = wf_split [c][rs][k/32][64], inv_scale [c]; needs
 * c % 64 == 0, k % 32 == 0), kind 2 = output phase `phase` (= py*2 + px) of a
 * stride-2 conv's dgrad operand (fields r, s, pad; out = [c][R2][S2][k/32][64]
 * with R2/S2 = hkp_phase_taps(r|s, pad, 2, py|px); inv_scale [c] = kind 1's) for
 * hkp_conv2d_bwd_data_x3_strided; w is KRSC fp32 [k][rs][c].  workspace:
 * hkp_weight_pack_x3_batch_ws_bytes(njobs, jobs) bytes (per-channel column
 * maxima of the flip jobs). */
typedef struct hkp_pack_job {
    const float* w;
    uint16_t* out;
    float* inv_scale;
    int32_t kind, k, rs, c;
    int32_t r, s, pad, phase;   /* kind 2 only */
} hkp_pack_job;
int64_t hkp_weight_pack_x3_batch_ws_bytes(int32_t njobs, const hkp_pack_job* jobs);
int hkp_weight_pack_x3_batch(int32_t njobs, const hkp_pack_job* jobs, void* workspace, int64_t ws_bytes,
                             hkp_stream_t stream);
int64_t hkp_conv_bwd_filter_x3_workspace(const hkp_conv_desc* d);
int hkp_conv2d_bwd_filter_x3(const hkp_conv_desc* d, const uint16_t* x_split, const uint16_t* dy_split,
                             const uint32_t* dy_amax_bits, float* dw, void* workspace, int64_t ws_bytes,
                             hkp_stream_t stream);

/* dw (KRSC, or OIHW for the stem) = sum over pixels of dy x im2col(x); split-K over
 * pixels into `workspace`, reduced in fixed order.  accumulate != 0 adds into dw. */
int64_t hkp_conv_bwd_filter_workspace(const hkp_conv_desc* d);
int hkp_conv2d_bwd_filter(const hkp_conv_desc* d, const float* x, const float* dy, float* dw, int32_t accumulate,
                          void* workspace, int64_t ws_bytes, hkp_stream_t stream);

/* Train-mode BatchNorm backward, three launches:
 *   reduce:   dz = g * (out_mask > 0) (out_mask NULL: dz = g), optionally stored to dz;
 *             partials[tiles][c][2] = (sum dz, sum dz*(y-mean)); tiles = hkp_bn_bwd_tiles(m);
 *             maxima (nullable) [tiles][c][2] = (max|dz|, max|y-mean|), and then
 *             dy_bound_bits (nullable) is zeroed for finalize
 *   finalize: dgamma = invstd*sum dz*(y-mean), dbeta = sum dz (nullable), coef[3c];
 *             with maxima: dy_amax_bits receives an upper bound of max|dy|,
 *             (max|dz| + |mean dz| + max|y-mean|*|k|) * |invstd*gamma|; without:
 *             dy_amax_bits (nullable) is reset to 0 for apply's exact max
 *   apply:    dy = ((dz - sum dz/m) - (y-mean)*invstd^2*sum dz*(y-mean)/m) * invstd*gamma
 *             dy_split (nullable): dy written as the packed f16x3 split of dy*2^e,
 *             2^e = the power of two of the bound in dy_amax_bits — the gradient
 *             operand of the x3 backward convs, with no hkp_split_pack_x3 pass and
 *             dy (fp32) optional; else dy_amax_bits (nullable) gets the exact max|dy|.
 * mean_invstd is what hkp_bn_finalize produced in the forward. */
/* The ReLU mask: out_mask (the BN+ReLU output, > 0), or relu_ss = the forward's
 * [scale | shift] of this BN — the mask is then recomputed from y exactly as
 * hkp_bn_apply made it (round(round(y*scale) + shift) > 0), so an inner BN's fp32
 * activation is not read back; both NULL: no ReLU. */
int64_t hkp_bn_bwd_tiles(int64_t m);
int hkp_bn_bwd_reduce(int64_t m, int32_t c, const float* g, const float* out_mask, const float* relu_ss,
                      const float* y, const float* mean_invstd, float* dz, float* partials, float* maxima,
                      uint32_t* dy_bound_bits, hkp_stream_t stream);
int hkp_bn_bwd_finalize(int32_t c, int64_t m, const float* partials, const float* maxima, const float* mean_invstd,
                        const float* gamma, float* dgamma, float* dbeta, float* coef, uint32_t* dy_amax_bits,
                        hkp_stream_t stream);
/* SyncBN backward (torch SyncBatchNorm: sum_dy and sum_dy_xmu over all ranks).
 * hkp_bn_bwd_stats: in place of hkp_bn_bwd_finalize's outputs, this rank's
 * per-channel [S = sum dz | D = sum dz*(y-mean) | max|dz| | max|y-mean| | m]
 * (4c+1 fp64; the maxima are 0 when maxima == NULL).  The caller all-gathers the
 * blocks in rank order into stats[nranks][4c+1]; hkp_bn_bwd_finalize_ranks sums
 * them in fixed rank order and writes hkp_bn_bwd_finalize's outputs: coef from
 * the global sums and count, dgamma/dbeta from this rank's block `own`, the
 * dy-split scale bound (has_maxima) from own maxima.  One rank: the same bits as
 * hkp_bn_bwd_finalize.  Replaces the backward of nn.BatchNorm2d in train mode
 * (src/resnet.py:46,49,78,85,87,139,187) for a batch sharded over ranks. */
int hkp_bn_bwd_stats(int32_t c, int64_t m, const float* partials, const float* maxima, const float* mean_invstd,
                     double* stats, hkp_stream_t stream);
int hkp_bn_bwd_finalize_ranks(int32_t c, int32_t nranks, const double* stats, const double* own, int32_t has_maxima,
                              const float* mean_invstd, const float* gamma, float* dgamma, float* dbeta, float* coef,
                              uint32_t* dy_amax_bits, hkp_stream_t stream);
int hkp_bn_bwd_apply(int64_t m, int32_t c, const float* g, const float* out_mask, const float* relu_ss,
                     const float* y, const float* mean_invstd, const float* coef, float* dy, uint32_t* dy_amax_bits,
                     uint16_t* dy_split, hkp_stream_t stream);

/* ----------------------------------------------------------- optimizer ---- */
/* Fused multi-tensor Adam with L2 weight decay (replaces the
 * optim.Adam(lr, weight_decay) step of train.py:36,79 — torch/optim/adam.py's
 * multi-tensor path, amsgrad/maximize off): for every element of every tensor
 *   g = g + wd*p;  m = m + (1-b1)*(g-m);  v = v*b2 + (1-b2)*g*g;
 *   p = p + neg_step_size * m / (sqrt(v)/bias_correction2_sqrt + eps)
 * with one_minus_beta1/2 = 1-b1, 1-b2, neg_step_size = -lr/(1-b1^step) and
 * bias_correction2_sqrt = sqrt(1-b2^step) computed by the caller in double (as
 * torch does with its Python-float scalars).  p, m, v updated in place; g read only. */
typedef struct hkp_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t n;
} hkp_adam_tensor;
int hkp_adam_step(int32_t ntensors, const hkp_adam_tensor* tensors, float beta2, float one_minus_beta1,
                  float one_minus_beta2, float eps, float weight_decay, float neg_step_size,
                  float bias_correction2_sqrt, hkp_stream_t stream);

/* Stem: backward of maxpool3x3/s2/p1(relu(y*scale+shift)) → dz = dL/d(BN output)
 * [n,h,w,c], ReLU mask applied (src/resnet.py:200-202; ATen's first-max window
 * rule): each window's dpool goes to the tap the forward recorded in `route`
 * (hkp_bn_relu_maxpool), summed per pixel over its windows in (ho, wo) order. */
int hkp_maxpool_bwd(int32_t n, int32_t h, int32_t w, int32_t c, const float* dpool, const uint8_t* route, float* dz,
                    hkp_stream_t stream);

/* Loss over the heatmaps (train.py:21,25; MSE train.py:13) in fp64: loss (device
 * double), dheat = dL/dheat as fp32 (nullable).  Target: dense fp64 `target`
 * [n,k,H,W], or NULL to recompute the Gaussian from uv/sigma (dataset.py:36-44).
 * workspace: hkp_heat_loss_workspace() bytes. */
int64_t hkp_heat_loss_workspace(void);
int hkp_heat_loss(int32_t n, int32_t k, int32_t H, int32_t W, int32_t loss_kind, const float* heat,
                  const double* target, const float* uv, float sigma, double* loss, float* dheat, void* workspace,
                  hkp_stream_t stream);

/* dlow = upsample-adjoint( dheat * (1-heat) * heat ) (sigmoid backward fused;
 * heat NULL = dheat is already the pre-sigmoid gradient): a row gather into
 * `workspace` (hkp_head_bwd_workspace bytes: [n*k][H][w] floats), then a column
 * gather — the direct double sum's loop order, so the same bits. */
int64_t hkp_head_bwd_workspace(int32_t n, int32_t k, int32_t w, int32_t H);
int hkp_head_bwd(int32_t n, int32_t k, int32_t h, int32_t w, int32_t H, int32_t W, const float* dheat,
                 const float* heat, float* dlow, void* workspace, int64_t ws_bytes, hkp_stream_t stream);

/* fc (K used rows) backward: dfeat NHWC [n,hw,c], dw [k][c], db [k]. */
int64_t hkp_head_fc_bwd_workspace(int32_t n, int32_t hw, int32_t c, int32_t k);
int hkp_head_fc_bwd(int32_t n, int32_t hw, int32_t c, int32_t k, const float* dlow, const float* feat,
                    const float* w, float* dfeat, float* dw, float* db, void* workspace, int64_t ws_bytes,
                    hkp_stream_t stream);

/* ----------------------------------------------------------- JPEG ---- */
/* Device half of the hybrid JPEG decode (hkp_jpeg.h; replaces cv2.imread,
 * src/dataset.py:71): n images of one geometry g (hkpj_probe), coefs = int16
 * [n][g->nblocks][64] and qt = uint16 [n][g->ncomp][64] from hkpj_decode, on
 * the device → out_bgr = uint8 [n][H][W][3] BGR, bit-identical to
 * libjpeg-turbo's default decode (islow IDCT, fancy upsampling).  planes:
 * workspace of n * hkp_jpeg_planes_bytes(g) bytes (the IDCT'd component
 * planes).  hkp_jpeg_planes_bytes returns -1 for a geometry the kernels do not
 * take. */
int64_t hkp_jpeg_planes_bytes(const hkpj_geom* g);
int hkp_jpeg_reconstruct(int32_t n, const hkpj_geom* g, const int16_t* coefs, const uint16_t* qt, uint8_t* planes,
                         int64_t planes_bytes, uint8_t* out_bgr, hkp_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* HULKKP_H */
