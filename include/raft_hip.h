/*
 * raft_hip.h — C-ABI of the MI355X-native RAFT inference path (libraft_hip.so).
 *
 * Plain pointers, sizes and a hipStream_t (passed as void*).  No allocation
 * happens inside any entry point (callers own every buffer, including the
 * workspaces whose sizes the *_workspace_floats queries return), nothing
 * synchronises the host, so every call is legal inside hipStreamBeginCapture
 * (hipGraph capture).  Every entry point returns 0 on success, a positive
 * hipError_t from the launch, or a negative RAFT_E_* argument error; the
 * message of the last failure on the calling thread is raft_hip_last_error().
 *
 * All device buffers are fp32.  "NHWC rows" means pixel-major rows of `ld`
 * floats: element (pixel m, channel c) lives at ptr[m * ld + c], with pixel
 * m = (b * H + y) * W + x.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   raft_alt_corr_forward   <- alt_cuda_corr.forward   (alt_cuda_corr/correlation.cpp:23-33,
 *                                                      correlation_kernel.cu:260-286)
 *   raft_alt_corr_backward  <- alt_cuda_corr.backward  (alt_cuda_corr/correlation.cpp:36-48,
 *                                                      correlation_kernel.cu:288-324)
 *   raft_corr_build         <- CorrBlock.__init__ + CorrBlock.corr (core/corr.py:25-54, 96-127)
 *   raft_corr_lookup        <- CorrBlock.__call__ + bilinear_sampler (core/corr.py:56-94,
 *                                                      core/utils/utils.py:57-71)
 *   raft_corr_lookup_conv   <- corr_fn(coords1) + BasicMotionEncoder.convc1 / convf1
 *                              (core/raft.py:219, core/update.py:185-205)
 *   raft_conv2d             <- nn.Conv2d + fused activations / GRU gates of
 *                              core/update.py:6-325 and core/extractor.py:6-267
 *   raft_instnorm_*         <- nn.InstanceNorm2d in core/extractor.py (norm_fn='instance')
 *   raft_convex_upsample    <- RAFT.upsample_flow (core/raft.py:112-142)
 *   raft_upflow8            <- upflow8 (core/utils/utils.py:80-82)
 *   raft_prep_images        <- RAFT.forward normalisation 2*(x/255)-1 (core/raft.py:164-169)
 *   raft_avgpool2_nhwc      <- F.avg_pool2d(x, 2, stride=2) in AlternateCorrBlock (core/corr.py:157-161)
 *   raft_pad_replicate      <- InputPadder.pad (core/utils/utils.py:7-24, F.pad mode='replicate')
 *   raft_bilinear_sample    <- bilinear_sampler (core/utils/utils.py:57-71)
 *   raft_forward_interpolate <- forward_interpolate (core/utils/utils.py:26-54; scipy griddata 'nearest')
 */
#ifndef RAFT_HIP_H_
#define RAFT_HIP_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAFT_HIP_ABI_VERSION 18

/* Negative return codes (argument errors, raised before any launch). */
#define RAFT_E_INVALID (-1)   /* bad size / null pointer / unsupported shape */
#define RAFT_E_ALIGN (-2)     /* pointer or leading dimension not aligned as required */

typedef void* raft_stream_t;  /* hipStream_t; NULL = the legacy default stream */

int raft_hip_abi_version(void);
const char* raft_hip_arch(void);        /* offload arch the library was built for ("gfx950") */
const char* raft_hip_last_error(void);  /* message of the last failure on this thread ("" if none) */
/* first 16 hex digits of the sha256 of the sources the library was built from (csrc/Makefile
 * SRC_HASH: the .hip files in SRCS order, the csrc .hpp headers and include/raft_hip.h); the loader
 * refuses a library whose hash differs from the sources beside it (a stale prebuilt .so) */
const char* raft_hip_source_hash(void);
/* Launch-span timing (bench / profiling): after raft_debug_launch_span(1) every
 * raft_corr_lookup_conv launch takes the next of 256 slots and records the realtime counter
 * (100 MHz) at its first work-group's start and at its last work-group's end, after that
 * work-group's stores completed; raft_debug_launch_span_read copies n values (slot k: [2k] start,
 * [2k+1] end).  raft_debug_launch_span(0) clears the slots and stops numbering.  Valid for eager
 * launches from one host thread on one device only: a launch enqueued while its stream is being
 * captured takes no slot (a graph would replay the slot it baked in). */
int raft_debug_launch_span(int enable);
int raft_debug_launch_span_read(unsigned long long* host, int n);
/* Debug (tests only): fill the LDS of every CU with all-ones words (NaN as fp32, f16 and bf16) by
 * kernels that take a CU's whole 160 KiB each; no global memory is touched.  A kernel launched next
 * on the stream that reads LDS it did not write then sees NaN: the parity tests run every launch of
 * a forward behind it and require the bit-identical, finite result (round 3's conv_stem K-padding
 * read was such a bug). */
int raft_debug_fill_lds_nan(raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * All-pairs correlation pyramid (CorrBlock)
 *
 * fmap1, fmap2: NHWC rows [B*H*W][ld] (channels 0..C-1 used, C % 4 == 0, 16-B aligned).
 * pyramid: num_levels levels stored back to back, H_0 = H, H_{l+1} = floor(H_l / 2)
 *   (same for W).  Every query pixel's level-l map is stored in 4x4 TILES:
 *   TH_l = ceil(H_l/4), TW_l = ceil(W_l/4), map size S_l = TH_l*TW_l*16 floats,
 *   element (y, x) at ((y>>2)*TW_l + (x>>2))*16 + (y&3)*4 + (x&3), padding = 0;
 *   the map of query pixel p of batch b starts at pyramid + off_l + (b*H*W + p)*S_l,
 *   off_l = B*H*W * sum_{j<l} S_j.  (64-B tiles = the HBM read granule: a
 *   radius-4 window touches ~10.6 tiles instead of ten straddling row runs.)
 * Level 0 = <fmap1[p], fmap2[q]> / sqrt_c (a division, as core/corr.py:127);
 * level l+1 = 2x2 average pool (floor) of level l.  16-byte aligned buffers.
 * --------------------------------------------------------------------------- */
size_t raft_corr_pyramid_floats(int B, int H, int W, int num_levels);
int raft_corr_build(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C,
                    int num_levels, float sqrt_c, float* pyramid, raft_stream_t stream);
/* The same with the GEMM arithmetic chosen: RAFT_PREC_FP32 (raft_corr_build: f32
 * MFMA) or RAFT_PREC_F16X3 (both fmaps split into f16 hi + lo at staging,
 * hi*hi + lo*hi + hi*lo with fp32 accumulation: ~2^-22 relative per product,
 * 5x the MFMA rate).  The RAFT forward uses F16X3 unless conv_precision="fp32". */
int raft_corr_build_prec(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C,
                         int num_levels, float sqrt_c, int precision, float* pyramid, raft_stream_t stream);
/* raft_corr_build_prec with a workspace (the forward's build): in RAFT_PREC_F16X3 with C % 16 == 0,
 * 64 <= C <= 1024, both fmaps are split once into f16 hi | lo maps in ws and the volume is built on
 * 256 x 256 tiles (one fp32 accumulator chain for hi*hi, lo*hi, hi*lo; same ~2^-22 relative
 * accuracy); otherwise it is raft_corr_build_prec.  ws: >= raft_corr_build_ws_bytes(B, H, W, C)
 * bytes, 16-byte aligned; ws == NULL, or fmaps / pyramid / ws off 16-B alignment, also take
 * raft_corr_build_prec (ws_bytes may then be 0).  RAFT_CORR_BUILD4=0: always raft_corr_build_prec.
 * (Argument order since ABI 15: ..., pyramid, ws, ws_bytes, stream.) */
size_t raft_corr_build_ws_bytes(int B, int H, int W, int C);
/* The workspace raft_corr_build_ws needs for its 256 x 256 kernel at this shape and precision, or 0 when that
 * call would take raft_corr_build_prec's kernel (not f16x3, C not a multiple of 16 in [64, 1024], maps past
 * 2^31 bytes, or RAFT_CORR_BUILD4=0): callers size the workspace from it instead of restating the rule. */
size_t raft_corr_build_ws_bytes_prec(int B, int H, int W, int C, int precision);
int raft_corr_build_ws(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C,
                       int num_levels, float sqrt_c, int precision, float* pyramid, void* ws, size_t ws_bytes,
                       raft_stream_t stream);
/* Row-major copy of one level, out [B*H*W][H_l][W_l] (the reference's corr_pyramid[l]). */
int raft_corr_pyramid_level(const float* pyramid, int B, int H, int W, int num_levels, int level,
                            float* out, raft_stream_t stream);

/* Radius-r bilinear window lookup of every level (CorrBlock.__call__).
 * coords: (x, y) per query pixel; coords_layout 0 = NHWC [B*H*W][2],
 *         1 = NCHW [B][2][H][W] (the reference's tensor as it stands).
 * out: out_layout 0 = NHWC rows [B*H*W][out_ld], channel lvl*(2r+1)^2 + ix*(2r+1) + iy;
 *      out_layout 1 = NCHW [B][L*(2r+1)^2][H][W] (out_ld ignored).
 * flow_out (optional, may be NULL): NHWC rows [B*H*W][flow_ld] receive
 *      coords - coords_grid (the RAFT loop's `flow`, core/raft.py:222).
 * range_flag (optional, may be NULL): set to 1 when an output exceeds RAFT_RANGE_LIMIT in
 *      magnitude (see the f16x3 range guard below). */
int raft_corr_lookup(const float* pyramid, int B, int H, int W, int num_levels, int radius,
                     const float* coords, int coords_layout, float* out, int out_ld, int out_layout,
                     float* flow_out, int flow_ld, int* range_flag, raft_stream_t stream);
/* raft_corr_lookup and, in the same launch, the motion encoder's first flow conv
 * (BasicMotionEncoder.convf1, core/update.py:186,205): f1_out rows [B*H*W][f1_out_ld]
 * (16-B aligned, ld % 4 == 0) = relu(conv7x7(flow) + f1_bias), flow = coords - coords_grid
 * with zero padding, as the reference's F.relu(self.convf1(flow)).  The convf1 work-groups
 * run on the VALU beside the lookup's memory-bound waves instead of as a launch of their own.
 * f1_weight: [f1_n/32][k*k][2][32] fp32 (16-B aligned), element ((g*k*k + dy*k + dx)*2 + ci)*32 + j
 * = weight[32g + j][ci][dy][dx] of the OIHW tensor; f1_k = 7, f1_n % 32 == 0.  Products are
 * exact fp32; f1_precision RAFT_PREC_F16 / RAFT_PREC_BF16 rounds the flow operand to that
 * type (round the weights the same way, as the MFMA kernels' operands).  f1_range_flag:
 * the range guard of the output (it feeds the split-precision convf2), or NULL.  The lookup
 * outputs are bit-identical to raft_corr_lookup's. */
int raft_corr_lookup_convf1(const float* pyramid, int B, int H, int W, int num_levels, int radius,
                            const float* coords, int coords_layout, float* out, int out_ld, int out_layout,
                            float* flow_out, int flow_ld, int* range_flag, const float* f1_weight,
                            const float* f1_bias, int f1_n, int f1_k, int f1_precision, float* f1_out,
                            int f1_out_ld, int* f1_range_flag, raft_stream_t stream);
/* The same convf1 alone (the alternate-correlation loop, whose lookup launch has no room
 * for it): f1_out = relu(conv7x7(coords - coords_grid) + f1_bias), arguments as above. */
int raft_convf1_flow(const float* coords, int coords_layout, int B, int H, int W, const float* f1_weight,
                     const float* f1_bias, int f1_n, int f1_k, int f1_precision, float* f1_out, int f1_out_ld,
                     int* f1_range_flag, raft_stream_t stream);

/* The lookup fused with the motion encoder's first convs (RAFT-full: radius 4, 4 levels), ONE
 * launch per iteration of the all-pairs loop (core/corr.py:56-94 + core/update.py:185-205):
 *   c1_out rows [B*H*W][c1_out_ld] = relu(convc1(corr) + c1_bias), convc1 = the 1x1 324 -> 256 conv
 *   over the lookup's 324 channels (channel order of raft_corr_lookup); the correlation rows never
 *   leave the work-group (LDS), so they are not an output;
 *   f1_out rows [B*H*W][f1_out_ld] = relu(convf1(flow) + f1_bias), convf1 the 7x7 2 -> 128 conv of
 *   flow = coords - coords_grid (zero padding), f1_k = 7;
 *   flow_out (optional): as raft_corr_lookup.
 * Both convs in `precision` (RAFT_PREC_F16X3 / F16 / BF16: the arithmetic of raft_conv2d).
 * coords: NHWC [B*H*W][2].  c1_weight / f1_weight: raft_lookup_conv_pack_weight's output for the
 * split form (raft_conv2d_split_weight_prec, `precision`) of the conv's packed weight (convc1
 * [256][352] RAFT_CONV_VEC, convf1 [128][128] RAFT_CONV_GATHER), 16-B aligned.  range_flag: raised
 * by a lookup tap above RAFT_RANGE_LIMIT (the split convc1 input); c1_range_flag / f1_range_flag:
 * by the convc1 / convf1 outputs (split convc2 / convf2 inputs).  Returns RAFT_E_INVALID for any
 * other radius / level count / channel count (the caller then runs raft_corr_lookup_convf1 +
 * raft_conv2d). */
int raft_corr_lookup_conv(const float* pyramid, int B, int H, int W, int num_levels, int radius,
                          const float* coords, float* flow_out, int flow_ld, int* range_flag, int precision,
                          const void* c1_weight, const float* c1_bias, int c1_n, float* c1_out, int c1_out_ld,
                          int* c1_range_flag, const void* f1_weight, const float* f1_bias, int f1_n, int f1_k,
                          float* f1_out, int f1_out_ld, int* f1_range_flag, raft_stream_t stream);
/* convc1's split weight [n_pad][k_pad] (k_pad % 32 == 0) -> raft_corr_lookup_conv's fragment order:
 * [k_pad/32][n/32][4][64] x 16 B, element (j, s, t, lane) = 8 halves of split row 32s + lane%32,
 * K-step j, quad (t/2)*4 + 2*(lane/32) + t%2; out holds raft_lookup_conv_weight_floats(n, k_pad)
 * floats (16-B aligned). */
size_t raft_lookup_conv_weight_floats(int n, int k_pad);
int raft_lookup_conv_pack_weight(const void* split_weight, int n_pad, int k_pad, int n, void* out,
                                 raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * On-the-fly ("alternate") correlation — the alt_cuda_corr plugin.
 *
 * fmap1 [B][H1][W1][C], fmap2 [B][H2][W2][C] (NHWC, contiguous),
 * coords [B][N][H1][W1][2] (x, y in fmap2 pixels).
 * corr [B][N][(2r+1)^2][H1][W1], channel iy + (2r+1)*ix, every element
 * written (no pre-zeroing needed), divided by `scale_div` (1.0f = the
 * reference's unscaled output; sqrtf(C) = AlternateCorrBlock's / sqrt(dim),
 * core/corr.py:198).
 * --------------------------------------------------------------------------- */
int raft_alt_corr_forward(const float* fmap1, const float* fmap2, const float* coords, float* corr,
                          int B, int H1, int W1, int H2, int W2, int C, int N, int radius, float scale_div,
                          raft_stream_t stream);
/* Arithmetic of the alternate lookups: RAFT_PREC_FP32 = exact fp32 products on the VALU (the
 * reference kernel's arithmetic; raft_alt_corr_forward, the plugin's entry point, always uses
 * it); any other value = the fp32-accurate f16x3 box GEMM on MFMA where it applies (r = 4,
 * C % 32 == 0, C <= 256; exact only while |fmap| < 65504: the RAFT forward's range guard covers
 * it), exact fp32 elsewhere.  raft_alt_corr_lookup_nhwc / raft_alt_corr_lookup_levels below
 * are the _prec forms with RAFT_PREC_F16X3. */
int raft_alt_corr_forward_prec(const float* fmap1, const float* fmap2, const float* coords, float* corr,
                               int B, int H1, int W1, int H2, int W2, int C, int N, int radius, float scale_div,
                               int precision, raft_stream_t stream);

/* Same computation, NHWC output: out rows [B*H1*W1][out_ld] at channel
 * offset already applied by the caller; coords_layout as raft_corr_lookup
 * (coordinates are divided by coord_div before use: 2**level in RAFT);
 * range_flag as raft_corr_lookup. */
int raft_alt_corr_lookup_nhwc(const float* fmap1, const float* fmap2, const float* coords, int coords_layout,
                              float coord_div, float* out, int out_ld, int B, int H1, int W1, int H2, int W2,
                              int C, int radius, float scale_div, float* flow_out, int flow_ld,
                              int* range_flag, raft_stream_t stream);
int raft_alt_corr_lookup_nhwc_prec(const float* fmap1, const float* fmap2, const float* coords, int coords_layout,
                                   float coord_div, float* out, int out_ld, int B, int H1, int W1, int H2, int W2,
                                   int C, int radius, float scale_div, float* flow_out, int flow_ld,
                                   int* range_flag, int precision, raft_stream_t stream);
/* All L levels of AlternateCorrBlock.__call__ (core/corr.py:163-198, the L calls of
 * alt_cuda_corr.forward of :176-186) as one call: level l reads fmap2_levels[l] (NHWC,
 * h2s[l] x w2s[l]) with the coordinates divided by 2^l and writes output channels
 * l*(2r+1)^2 .. of each NHWC row; flow_out as raft_alt_corr_lookup_nhwc (written once).  RAFT's
 * case (r = 4, C % 32 == 0, C <= 256) is ONE launch whose work-groups stage their fmap1 tile
 * once for every level; otherwise L launches of raft_alt_corr_lookup_nhwc.  Results equal the
 * L separate calls.  The pointer / size arrays are read on the host during the call. */
int raft_alt_corr_lookup_levels(const float* fmap1, const float* const* fmap2_levels, const int* h2s,
                                const int* w2s, int L, const float* coords, int coords_layout, float* out,
                                int out_ld, int B, int H1, int W1, int C, int radius, float scale_div,
                                float* flow_out, int flow_ld, int* range_flag, raft_stream_t stream);
int raft_alt_corr_lookup_levels_prec(const float* fmap1, const float* const* fmap2_levels, const int* h2s,
                                     const int* w2s, int L, const float* coords, int coords_layout, float* out,
                                     int out_ld, int B, int H1, int W1, int C, int radius, float scale_div,
                                     float* flow_out, int flow_ld, int* range_flag, int precision,
                                     raft_stream_t stream);

/* Gradients of raft_alt_corr_forward (unscaled), replacing correlation_kernel.cu:122-256:
 * every output is written (no pre-zeroing) and bit-identical run to run.  fmap1_grad is
 * a gather over each query's taps; fmap2_grad inverts the (query, tap) -> fmap2 pixel map
 * (a stable sort of the queries by window origin, then a gather per fmap2 pixel) instead
 * of the reference's float atomics; coords_grad is the true gradient through the bilinear
 * weights (the reference leaves it zero, correlation_kernel.cu:307).  workspace: at least
 * raft_alt_corr_backward_workspace_floats(...) floats, 256-byte aligned.  C % 4 == 0,
 * C <= 1024, radius <= 32 (the forward's range). */
int raft_alt_corr_backward(const float* fmap1, const float* fmap2, const float* coords, const float* corr_grad,
                           float* fmap1_grad, float* fmap2_grad, float* coords_grad,
                           int B, int H1, int W1, int H2, int W2, int C, int N, int radius,
                           float* workspace, size_t workspace_floats, raft_stream_t stream);
size_t raft_alt_corr_backward_workspace_floats(int B, int H1, int W1, int H2, int W2, int C, int N, int radius);

/* 2x2 / stride-2 average pool (floor), NHWC contiguous [B][H][W][C] -> [B][H/2][W/2][C]. */
int raft_avgpool2_nhwc(const float* in, float* out, int B, int H, int W, int C, raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * Convolution as implicit GEMM on MFMA, NHWC.
 * M = batch*out_h*out_w pixels, N = out channels, K = taps x input channels.
 * The input is a virtual concat of up to two NHWC row sources (seg 0, then
 * seg 1), which is how torch.cat([...], dim=1) of the reference is elided.
 *
 * Packed weights (see raft_conv2d_packed_shape):
 *   mode RAFT_CONV_VEC    (every segment's channel count % 4 == 0, seg0 % 32 == 0
 *                          when seg 1 is used): w[n_pad][KH*KW][c_pad],
 *                          c_pad = roundup(c0 + c1, 32), zero padded;
 *   mode RAFT_CONV_GATHER (small inputs, e.g. 2- or 3-channel):
 *                          w[n_pad][k_pad], k = (ky*KW + kx)*(c0+c1) + c,
 *                          k_pad = roundup(KH*KW*(c0+c1), 32), zero padded;
 *   n_pad = roundup(N, 64).
 *
 * Arithmetic (params.precision):
 *   RAFT_PREC_FP32   v_mfma_f32_32x32x2_f32 on the fp32 packed weight.
 *   RAFT_PREC_F16X3  fp32-accurate split: every operand x = hi + lo/2048 with
 *                    hi = f16(x), lo = f16((x - hi) * 2048); products
 *                    hi*hi + (hi*lo + lo*hi)/2048 on v_mfma_f32_32x32x16_f16
 *                    with fp32 accumulation (the lo*lo term, 2^-22 relative,
 *                    is dropped).  Weight: the split form of the packed
 *                    weight (raft_conv2d_split_weight), same byte size.
 *   RAFT_PREC_F16    one f16 product (hi*hi), fp32 accumulation: the mixed-
 *                    precision mode (reference: autocast, core/raft.py:156);
 *                    uses the same split weight.
 *   RAFT_PREC_BF16   one bf16 product, fp32 accumulation, on v_mfma_f32_32x32x16_bf16
 *                    (bf16 mixed precision: the reference under a bf16 autocast;
 *                    fp32's exponent range).  Weight: raft_conv2d_split_weight_prec
 *                    with RAFT_PREC_BF16 (32 bf16 hi then 32 bf16 lo per K-step).
 * N <= 4 convolutions always take the fp32 packed weight (VALU kernel).
 * --------------------------------------------------------------------------- */
#define RAFT_CONV_VEC 0
#define RAFT_CONV_GATHER 1

#define RAFT_PREC_FP32 0
#define RAFT_PREC_F16X3 1
#define RAFT_PREC_F16 2
#define RAFT_PREC_BF16 3

/* epilogues: v = acc + bias[n] */
#define RAFT_EPI_LINEAR 0         /* out = alpha * v                                          */
#define RAFT_EPI_RELU 1           /* out = relu(v)                                            */
#define RAFT_EPI_RESID_RELU 2     /* out = relu(aux0[m,n] + relu(v))    (ResidualBlock tail) */
#define RAFT_EPI_GRU_ZR 3         /* n <  split: out[m,n] = sigmoid(v) (z); split % 32 == 0      */
                                  /* n >= split: out1[m,n-split] = sigmoid(v)*aux0[m,n-split] (r*h) */
#define RAFT_EPI_GRU_Q 4          /* q = tanh(v); out[m,n] = (1-aux1[m,n])*aux0[m,n] + aux1[m,n]*q */
#define RAFT_EPI_TANH_RELU 5      /* n < split: out[m,n] = tanh(v); else out1[m,n-split] = relu(v); split % 32 == 0 */
#define RAFT_EPI_ADD_TO_OUT 6     /* out[m,n] = out[m,n] + v   (coords1 += delta_flow)         */

typedef struct raft_conv2d_params {
  const float* in0; int in0_ld; int in0_c;  /* seg 0: NHWC rows, first channel at in0 */
  const float* in1; int in1_ld; int in1_c;  /* seg 1 (in1_c = 0: unused) */
  int batch, in_h, in_w;
  int out_h, out_w;
  int kh, kw, stride_h, stride_w, pad_h, pad_w;
  int mode;                                 /* RAFT_CONV_VEC / RAFT_CONV_GATHER */
  const float* weight;                      /* packed, see above */
  const float* bias;                        /* [N] or NULL */
  int n;                                    /* output channels N */
  float* out; int out_ld;
  int epilogue; float alpha; int split;
  const float* aux0; int aux0_ld;
  const float* aux1; int aux1_ld;
  float* out1; int out1_ld;
  const float* add0; int add0_ld;           /* optional addend rows: v = acc + bias[n] + add0[m,n]
                                               (a precomputed partial sum, e.g. the GRU's
                                               iteration-invariant context term) */
  int precision;                            /* RAFT_PREC_* (weight format follows it) */
  int* range_flag;                          /* optional (NULL = off): set to 1 when an output
                                               exceeds RAFT_RANGE_LIMIT in magnitude */
  float* stats_part; int stats_ld;          /* optional (NULL = off): InstanceNorm partial statistics
                                               of the output, see raft_conv2d_stats_slots */
  const float* in_norm; int in_norm_relu;   /* optional (NULL = off): the conv reads
                                               act((seg0 - mean[b][c]) * rstd[b][c]) instead of seg 0,
                                               in_norm = [batch][in0_c][2] {mean, rstd} (the output of
                                               raft_instnorm_stats / _merge), act = relu if
                                               in_norm_relu; zero padding stays zero.  Only where
                                               raft_conv2d_in_norm_ok says so. */
  const void* weight_s;                     /* optional (NULL = off), RAFT_PREC_F16X3 only: the
                                               column-scaled split of the same weight
                                               (raft_conv2d_split_weight_scaled).  With it, multi-
                                               round stride-1 3x3 convs run on 256-pixel x 64-
                                               column tiles whose three products share one
                                               accumulator; without it they keep the 128-pixel
                                               tiles.  Same results to fp32 rounding. */
} raft_conv2d_params;

/* f16x3 range guard.  RAFT_PREC_F16X3 splits every activation x as hi = f16(x), which is
 * only exact for |x| < 65504: a larger conv input would silently become inf.  Producers
 * whose outputs feed a split-precision conv (conv epilogues, the correlation lookups) can
 * raise a device flag when any output exceeds RAFT_RANGE_LIMIT = 2^15 (NaN does not raise
 * it: a NaN input propagates as in fp32); the caller checks the flag after the forward and
 * re-runs it with RAFT_PREC_FP32 (or raises).  Producers with bounded outputs need no flag:
 * InstanceNorm outputs (|x| <= sqrt(H*W)), the prepared images (|x| <= 1) and the GRU
 * epilogues (sigmoid / tanh blends of |h| <= 1); neither do convs whose outputs only feed
 * fp32 consumers (the raw convs of an InstanceNorm encoder, the flow head's first conv). */
#define RAFT_RANGE_LIMIT 32768.0f

/* InstanceNorm statistics from the conv epilogue (core/extractor.py norm_fn='instance': the
 * raw conv output's per-(image, channel) mean and variance without a pass over it).  With
 * p->stats_part set, every wave of the conv writes, per output channel n, the (count, mean, M2)
 * of its <= 32 output pixels (M2 = sum of squared deviations from that mean) as 4 floats at
 * stats_part[((slot * stats_ld) + n) * 4 ..], slot = image * slots_per_image + s, s <
 * slots_per_image; raft_instnorm_merge combines them (Chan's formula in double, fixed order).
 * Only for convs with the linear epilogue (alpha 1, no add0) and more than 4 outputs (VEC) that run
 * on the halo, stem or (since round 5: the strided encoder convs) 64x64-tile GEMM kernel, whose
 * tiles then hold one image's rows each: raft_conv2d_stats_slots returns slots_per_image for such a
 * conv and 0 otherwise (raft_conv2d then rejects stats_part). */
int raft_conv2d_stats_slots(const raft_conv2d_params* p);
/* Tile rows of the halo kernel's launch of this conv: 8 (128-pixel tiles), 16 (the multi-round
 * 256-pixel tiles), 0 when the halo kernel does not run it (inspection / tests). */
int raft_conv2d_halo_tile_rows(const raft_conv2d_params* p);
/* Tiles each work-group of the halo kernel's launch of this conv runs back to back (1, or
 * ceil(tiles / CUs) for a launch of more tiles than CUs: the loaders run on into the next tile while
 * the compute waves store the last one), 0 when the halo kernel does not run it (inspection / tests). */
int raft_conv2d_halo_tiles_per_wg(const raft_conv2d_params* p);
/* 1 when the conv can apply its input's InstanceNorm in its loaders (in_norm above: the halo
 * kernel's 3x3 convs over <= 256 channels), else 0. */
int raft_conv2d_in_norm_ok(const raft_conv2d_params* p);
int raft_instnorm_merge(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps,
                        float* stats, raft_stream_t stream);
/* raft_instnorm_merge over many slots, spread over the CUs: level 1 sums groups of 32 slots per
 * channel relative to slot 0's mean (coalesced 1-KiB slot rows, no division), level 2 combines the
 * groups in order (deterministic).  ws: raft_instnorm_merge_ws_floats(slots_per_image, B, C) floats,
 * 8-byte aligned; the same {mean, rstd} as raft_instnorm_merge to double rounding. */
size_t raft_instnorm_merge_ws_floats(int slots_per_image, int B, int C);
int raft_instnorm_merge_ws(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps, void* ws,
                           float* stats, raft_stream_t stream);
/* raft_instnorm_merge_ws as ONE launch: the level-1 block of a (64-channel group, image) whose
 * group sums land last (an agent-scope counter per group and image) runs level 2, in level 2's
 * order: the same statistics bit for bit, one kernel boundary fewer.  counters:
 * raft_instnorm_merge_counters(B, C) ints, zero before the first call; every call leaves them zero
 * (so a captured graph replays).  ws as raft_instnorm_merge_ws. */
size_t raft_instnorm_merge_counters(int B, int C);
int raft_instnorm_merge_fused(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps, void* ws,
                              int* counters, float* stats, raft_stream_t stream);

/* Packed weight geometry for a conv (n_pad, k_pad in floats per row). */
int raft_conv2d_packed_shape(int mode, int n, int kh, int kw, int cin, int* n_pad, int* k_pad);
int raft_conv2d(const raft_conv2d_params* p, raft_stream_t stream);
/* Two convs with no data dependence between them (core/update.py:276-285: convc2 of the corr
 * branch beside convf2 of the flow branch), results identical to raft_conv2d(p0) then
 * raft_conv2d(p1).  When both are halo-kernel convs of one shape class and precision, their
 * tiles run side by side in ONE launch: the pair fills CUs that either alone leaves idle at
 * one frame pair, with no second stream (a cross-stream fork/join costs a graph ~7 us per
 * edge on ROCm).  Each conv keeps the tile rows raft_conv2d would pick for it
 * (raft_conv2d_halo_tile_rows), so the bits match also with weight_s set; convs that pick
 * different rows are not co-launched.  Otherwise, or when one reads what the other writes, or both write a common
 * element (column ranges of their output rows meet), the two run in order. */
int raft_conv2d_pair(const raft_conv2d_params* p0, const raft_conv2d_params* p1, raft_stream_t stream);
/* Loader waves of the halo kernel's one-tile f16x3 3x3 / 1x5 / 5x1 convs (the update block at one frame
 * pair): 4 (a 512-thread work-group) or 8 (768 threads: each loader issues half the weight DMAs
 * and stages half of each patch); the same results bit for bit.  Default 8 (RAFT_HALO_NL8=0: 4).
 * Returns the previous count; other values only query.  Process-wide; plans capture launches, so
 * set it before building / capturing a plan. */
int raft_conv2d_set_halo_loaders(int nl);
/* The compute waves per SIMD of the same convs when their N tile is 64 columns: 2 (default; the K-split form:
 * waves w and w + 4 take the even / odd K-steps of one 32 x 64 block, their partial sums meet in LDS and each
 * stores half the columns; 4 loader waves, 768 threads) or 1.  The two forms sum the K-steps in different orders
 * (results within fp32 rounding of each other; each deterministic).  Returns the previous count; other values
 * only query.  Process-wide; set it before building / capturing a plan.  (Engine-level knob; no reference
 * counterpart.) */
int raft_conv2d_set_halo_ks(int ks);
/* fp32 packed weight [n_pad][k_pad] -> split form for RAFT_PREC_F16X3 / F16:
 * per row and 32-wide K-step, 32 f16 hi then 32 f16 lo (lo scaled by 2048);
 * out holds n_pad*k_pad*4 bytes, like the input. */
int raft_conv2d_split_weight(const float* w, void* out, int n_pad, int k_pad, raft_stream_t stream);
/* Column-scaled f16x3 split (raft_conv2d_params.weight_s): per output row n a power of two
 * S_n = 2^(14 - e_n), e_n = the binary exponent of max_k |w[n][k]| (so |w * S_n| < 2^14; S_n = 1 for
 * a zero row), then per K-step 32 f16 hi = f16(w S_n) and 32 f16 lo = f16(w S_n - hi), both at
 * the scale S_n, followed by the n_pad floats 1 / S_n.  hi*hi + hi*lo + lo*hi then sum in one
 * fp32 chain and the epilogue multiplies by 1 / S_n (exact).  out holds
 * raft_conv2d_split_scaled_bytes(n_pad, k_pad) bytes, 16-byte aligned. */
size_t raft_conv2d_split_scaled_bytes(int n_pad, int k_pad);
int raft_conv2d_split_weight_scaled(const float* w, void* out, int n_pad, int k_pad, raft_stream_t stream);
/* The split form for a given precision: RAFT_PREC_F16X3 / RAFT_PREC_F16 as above;
 * RAFT_PREC_BF16: per row and K-step 32 bf16 hi = bf16(x) then 32 bf16 lo = bf16(x - hi). */
int raft_conv2d_split_weight_prec(const float* w, void* out, int n_pad, int k_pad, int precision,
                                  raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * InstanceNorm2d (affine=False, eps): statistics per (image, channel) over
 * the image's hw pixels; stats[(b*C + c)*2 + {0,1}] = {mean, 1/sqrt(var+eps)}.
 * --------------------------------------------------------------------------- */
size_t raft_instnorm_workspace_floats(int B, int HW, int C);
int raft_instnorm_stats(const float* x, int ld, int B, int HW, int C, float eps, float* stats,
                        float* workspace, raft_stream_t stream);
/* out = act( norm(x) + resid ) where resid = 0 (resid NULL), raw resid rows, or
 * norm(resid) with its own stats (resid_stats != NULL); relu_mode: 0 none, 1 relu(norm(x)),
 * 2 relu(resid + relu(norm(x)))  (ResidualBlock tail). */
/* nn.GroupNorm (core/extractor.py:23-25: ResidualBlock / BottleneckBlock with norm_fn='group', the
 * blocks' default): per (image, group of C/G consecutive channels) mean and 1/sqrt(var + eps) over the
 * group's channels x HW pixels (double, deterministic), written per (image, channel) as
 * stats[b][c] = {mean, rstd} of c's group — the layout raft_instnorm_apply reads.  C % G == 0. */
int raft_groupnorm_stats(const float* x, int ld, int B, int HW, int C, int G, float eps, float* stats,
                         raft_stream_t stream);
/* raft_instnorm_apply with a per-channel affine: v = (x - mean) * rstd * gamma[c] + beta[c]
 * (gamma / beta NULL = 1 / 0); the residual likewise with resid_gamma / resid_beta. */
int raft_norm_apply_affine(const float* x, int ld, const float* stats, const float* gamma, const float* beta,
                           const float* resid, int resid_ld, const float* resid_stats, const float* resid_gamma,
                           const float* resid_beta, int relu_mode, float* out, int out_ld, int B, int HW, int C,
                           raft_stream_t stream);
int raft_instnorm_apply(const float* x, int ld, const float* stats, const float* resid, int resid_ld,
                        const float* resid_stats, int relu_mode, float* out, int out_ld,
                        int B, int HW, int C, raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * Small elementwise / layout kernels of RAFT.forward
 * --------------------------------------------------------------------------- */
/* images NCHW [B][3][H][W] in 0..255 -> NHWC rows [2B*H*W][3]: img1 batch then img2, 2*(x/255)-1 */
int raft_prep_images(const float* img1, const float* img2, float* out, int B, int H, int W,
                     raft_stream_t stream);
/* coords NHWC [B*H*W][2] = coords_grid (+ flow_init NCHW [B][2][H][W] if not NULL) */
int raft_init_coords(float* coords, const float* flow_init, int B, int H, int W, raft_stream_t stream);
/* flow_low NCHW [B][2][H][W] = coords - coords_grid */
int raft_flow_from_coords(const float* coords, float* flow, int B, int H, int W, raft_stream_t stream);
/* convex upsample of flow = coords - grid with mask rows [B*H*W][mask_ld] (576 used)
 * -> NCHW [B][2][8H][8W] */
int raft_convex_upsample(const float* coords, const float* mask, int mask_ld, float* flow_up,
                         int B, int H, int W, raft_stream_t stream);
/* 8 * bilinear(align_corners=True) x8 upsample of flow = coords - grid -> NCHW [B][2][8H][8W] */
int raft_upflow8(const float* coords, float* flow_up, int B, int H, int W, raft_stream_t stream);
/* NCHW [B][C][H][W] <-> NHWC rows [B*H*W][ld] */
int raft_nchw_to_nhwc(const float* in, float* out, int out_ld, int B, int C, int H, int W, raft_stream_t stream);
int raft_nhwc_to_nchw(const float* in, int in_ld, float* out, int B, int C, int H, int W, raft_stream_t stream);

/* ---------------------------------------------------------------------------
 * Caller-side helpers (demo.py / evaluate.py around RAFT.forward), NCHW fp32
 * --------------------------------------------------------------------------- */
/* replicate padding: in [NC][H][W] -> out [NC][H+top+bottom][W+left+right] */
int raft_pad_replicate(const float* in, float* out, int NC, int H, int W, int top, int bottom, int left, int right,
                       raft_stream_t stream);
/* bilinear_sampler: img [N][C][H][W], coords [N][Ho][Wo][2] pixel (x, y) -> out [N][C][Ho][Wo]
 * (grid_sample, align_corners=True, zero padding; a non-finite position gives NaN, as the
 * reference on a 1-px axis); mask (optional) [N][Ho][Wo] = 1 where -1 < grid < 1 on both axes. */
int raft_bilinear_sample(const float* img, const float* coords, float* out, float* mask, int N, int C, int H, int W,
                         int Ho, int Wo, raft_stream_t stream);
/* forward_interpolate: flow [B][2][H][W] -> out [B][2][H][W]; every grid point takes the flow of
 * the nearest (fp64 Euclidean) forward-moved point (x + dx, y + dy) strictly inside
 * (0, W) x (0, H); ties -> the lowest source index; no valid point -> 0.  An all-pairs search,
 * for the 1/8-resolution flow of the warm start: H*W <= RAFT_FI_MAX_POINTS (else RAFT_E_INVALID). */
#define RAFT_FI_MAX_POINTS 65536
int raft_forward_interpolate(const float* flow, float* out, int B, int H, int W, raft_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RAFT_HIP_H_ */
