/*
 * libfvc — MI355X (gfx950) C-ABI for the DVC P-frame encode/decode hot path.
 *
 * Every entry point is `extern "C"`, takes plain pointers + sizes + a hipStream_t, never
 * allocates, never throws, and returns 0 on success or a negative code
 * (-hipError_t, or FVC_E*). Device pointers are caller-owned (torch tensors in the Python
 * host layer); calls are stream-ordered and reentrant: the library keeps no mutable state
 * between calls (launch policy such as the CU reserve and status flags such as the
 * split-precision overflow flag are arguments), so concurrent calls on different streams or
 * host threads do not interact.
 *
 * Activation layout inside the codec is NHWC fp32 with the channel count padded to a
 * multiple of 4 ("cp"; pad channels are written as zeros). Frames at the module boundary
 * are NCHW fp32, exactly as the reference forward takes them.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   conv/deconv .......... nn.Conv2d / nn.ConvTranspose2d of DVC/subnet/{endecoder,analysis*,
 *                          synthesis*}.py (ATen conv2d / conv_transpose2d)
 *   warp ................. endecoder.py:52-67 torch_warp / :116-119 flow_warp (grid_sample)
 *   upsample ............. endecoder.py:173-184 bilinearupsacling(2)  (upsample_bilinear2d)
 *   avgpool .............. endecoder.py:345-346, :272,274               (avg_pool2d)
 *   gdn .................. DVC/subnet/GDN.py:63-93
 *   bits ................. DVC/net.py:121-205 (Laplace + BitEstimator estimates)
 *   indexes .............. compressai GaussianConditional.build_indexes (entropy_models.py:82,90)
 *   rans ................. compressai RansEncoder/RansDecoder.{encode,decode}_with_indexes
 *                          (pybind11, called from entropy_models.py:82-93)
 *   pmf_to_quantized_cdf . compressai._CXX.pmf_to_quantized_cdf (EntropyModel._pmf_to_cdf)
 */
#ifndef FVC_H_
#define FVC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* fvc_stream_t; /* == hipStream_t */

enum {
  FVC_OK = 0,
  FVC_EINVAL = -1000,  /* bad shape / argument */
  FVC_ENOSPC = -1001,  /* output capacity too small */
  FVC_ECORRUPT = -1002 /* malformed bitstream */
};

/* conv input transform applied while staging the input tile */
enum { FVC_IN_NONE = 0, FVC_IN_RELU = 1, FVC_IN_ABS = 2, FVC_IN_ROUND = 3 };
/* activation after bias */
enum { FVC_ACT_NONE = 0, FVC_ACT_RELU = 1, FVC_ACT_LRELU = 2 /* slope 0.1 */ };
/* transform after the residual add */
enum { FVC_POST_NONE = 0, FVC_POST_EXP = 1 };

int fvc_version(void);
int fvc_device_arch_ok(void); /* 1 if device 0 is gfx950 */

/* ------------------------------------------------------------------ convolutions
 * y = post( act(conv(in_op(x)) + bias) + res )
 * conv:   nn.Conv2d(cin, cout, k, stride, padding=k//2)              -> out h/stride x w/stride
 * deconv: nn.ConvTranspose2d(cin, cout, k, stride, padding=k//2,
 *                            output_padding=stride-1)                 -> out h*stride x w*stride
 * Weights come in the reference layout (conv OIHW, deconv IOHW) on the HOST and are packed
 * once by fvc_conv_pack_weight into the kernel's k-block layout (copy the pack to device).
 * res may be NULL. x: [b][h][w][cp_in]; y: [b][ho][wo][cp_out]; res like y.
 */
size_t fvc_conv_wpack_floats(int cin, int cout, int ksize, int stride, int transposed);
int fvc_conv_pack_weight(const float* w_host, float* wpack_host, int cin, int cout, int ksize,
                         int stride, int transposed);
int fvc_conv2d_nhwc_f32(const float* x, const float* wpack, const float* bias, const float* res,
                        float* y, int batch, int h, int w, int cin, int cout, int ksize, int stride,
                        int in_op, int act, int post_op, fvc_stream_t stream);
int fvc_deconv2d_nhwc_f32(const float* x, const float* wpack, const float* bias,
                          const float* res, float* y, int batch, int h, int w, int cin, int cout,
                          int ksize, int stride, int in_op, int act, int post_op,
                          fvc_stream_t stream);

/* Split-precision variant ("fp16 x3", fvc_conv_x3.hip): same math and arguments, computed on the
 * fp16 matrix cores with every fp32 operand split into hi + lo*2^-11 halves and three MFMAs per
 * product (fp32-level accuracy, ~1e-6 relative). Taken for layers with cin padded to a multiple
 * of 8 and cout > 4 (fvc_conv_x3_supported). The pack is fp16 pairs plus a per-layer output
 * scale osc = 2^-kw (weights are pre-scaled by 2^kw). Activations must stay below 65000 in
 * magnitude: a launch that stages a larger (or non-finite) value ORs 1 into *overflow_flag
 * (a caller-owned device int; NULL = unchecked) and its output must be recomputed on the fp32
 * kernels (the Python layer does this, net.py). cu_reserve (>= 0): CUs the persistent grid
 * leaves to kernels of other streams (capped at half the CUs). A pipelined caller (encoder +
 * coder + decoder streams in flight, fastvideocodec_amd/gop.py) passes it so that a conv block
 * never waits for a CU held by a long-running rANS chain, which would double that launch's
 * time; 0 = the whole GPU. sched (may be NULL): caller-owned device scratch of sched_len ints,
 * zero before the first launch, used and left zeroed by each launch (launches sharing it must
 * be ordered, e.g. one buffer per stream): with at least 1 + (N-groups x batch) ints, blocks take
 * work items from per-group counters, so a block that starts late (its CU busy with another
 * stream's kernel) takes fewer tiles instead of stretching the launch; otherwise each block of
 * the persistent grid walks a fixed run. */
int fvc_conv_x3_supported(int cin, int cout, int ksize, int stride, int transposed);
size_t fvc_conv_x3_wpack_bytes(int cin, int cout, int ksize, int stride, int transposed);
/* Layout id (nonzero) of the pack fvc_conv_x3_pack_weight writes for this geometry under the
 * current configuration, 0 if the x3 path does not take it. The FVC_DX / FVC_X3_PT / FVC_X3_CIN4 /
 * FVC_X3_CC / FVC_X3_SMALLN switches are read at pack and at launch time: record the id with the
 * pack and compare before launching (the Python layer refuses a mismatch). */
unsigned fvc_conv_x3_layout_id(int cin, int cout, int ksize, int stride, int transposed);
int fvc_conv_x3_pack_weight(const float* w_host, void* wpack_host, float* osc_out, int cin,
                            int cout, int ksize, int stride, int transposed);
int fvc_conv2d_nhwc_x3(const float* x, const void* wpack, float osc, const float* bias,
                       const float* res, float* y, int batch, int h, int w, int cin, int cout,
                       int ksize, int stride, int in_op, int act, int post_op, int cu_reserve,
                       int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream);
int fvc_deconv2d_nhwc_x3(const float* x, const void* wpack, float osc, const float* bias,
                         const float* res, float* y, int batch, int h, int w, int cin, int cout,
                         int ksize, int stride, int in_op, int act, int post_op, int cu_reserve,
                         int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream);
/* 1 if fvc_deconv2d_nhwc_x3 / _x3_tap run this transposed geometry on the all-classes kernel
 * (stride 2, 64 / 96 / 128 input and 64 / 128 output channels: the four output-parity classes of a
 * tile from one staged full-channel input tile; its pack is the x3 pack with one channel chunk).
 * The environment variable FVC_DX=0 (read at pack and at launch time) keeps such layers on the
 * per-class path of conv_x3_kernel. */
int fvc_deconv_x3_all_classes(int cin, int cout, int ksize, int stride);
/* Fused producer + tap partials of a cout <= 4 consumer (the pair nn.Conv2d(c->128/64) ->
 * nn.Conv2d(128/64->2/3): synthesis_mv.py:41-43 deconv7 -> deconv8, endecoder.py:278-279
 * Warp_net conv5 -> conv6): the producer conv / transposed conv runs as fvc_*_x3 (in_op none,
 * act, res; post none) but instead of its output y it writes
 *   P [batch][Ho][Wo][pcp] = tap_w [np][cout] . y   per output pixel   (np <= pcp <= 32)
 * i.e. the 1x1 first half of the consumer's tap-partial form, which fvc_tap_gather_nhwc then
 * sums into the consumer's output. tap_wpack from fvc_x3_tap_pack_weight (host), np = k*k*cout'
 * rows t*cout' + co. fvc_conv_x3_tap_supported says whether a geometry takes this path. */
int fvc_conv_x3_tap_supported(int cin, int cout, int ksize, int stride, int transposed, int pcp);
size_t fvc_x3_tap_wpack_bytes(int np, int cin);
int fvc_x3_tap_pack_weight(const float* w_host, void* wpack_host, float* osc_out, int np, int cin);
int fvc_conv2d_nhwc_x3_tap(const float* x, const void* wpack, float osc, const float* bias,
                           const float* res, float* P, int batch, int h, int w, int cin, int cout,
                           int ksize, int stride, int act, const void* tap_wpack, float tap_osc,
                           int pcp, int cu_reserve, int* overflow_flag, int* sched, int sched_len,
                           fvc_stream_t stream);
/* y = fvc_conv2d_nhwc_x3(x, stride 1, in_op none, post none) and pool = avg_pool2d(y, 2)
 * [batch][h/2][w/2][cp] in the same launch (Warp_net's ResBlock output feeding F.avg_pool2d,
 * endecoder.py:272,274; bit-identical to fvc_avgpool2_nhwc of y). */
int fvc_conv_x3_pool_supported(int cin, int cout, int ksize);
int fvc_conv2d_nhwc_x3_pool(const float* x, const void* wpack, float osc, const float* bias,
                            const float* res, float* y, float* pool, int batch, int h, int w, int cin,
                            int cout, int ksize, int act, int cu_reserve, int* overflow_flag, int* sched,
                            int sched_len, fvc_stream_t stream);
int fvc_deconv2d_nhwc_x3_tap(const float* x, const void* wpack, float osc, const float* bias,
                             const float* res, float* P, int batch, int h, int w, int cin, int cout,
                             int ksize, int stride, int act, const void* tap_wpack, float tap_osc,
                             int pcp, int cu_reserve, int* overflow_flag, int* sched, int sched_len,
                             fvc_stream_t stream);
/* Winograd F(2x2,3x3) split-precision conv for the 64 -> 64-channel 3x3 stride-1 pad-1 layers
 * (Warp_net ResBlocks, endecoder.py:228-296; same contract as fvc_conv2d_nhwc_x3 with cin = cout =
 * 64, in_op none / relu, act, res; pool != NULL additionally writes avg_pool2d(y, 2) as
 * fvc_conv2d_nhwc_x3_pool: [batch][h/2][w/2][64], floor sizes). The transformed weights U = G g G^T (computed in double,
 * split fp16 hi/lo) come from fvc_conv_wino_pack_weight (host, fvc_conv_wino_wpack_bytes() bytes,
 * w OIHW [64][64][3][3]). sched: >= 2 ints, zero between launches (shared with the x3 kernels). */
int fvc_conv_wino_supported(int cin, int cout, int ksize, int stride, int transposed);
size_t fvc_conv_wino_wpack_bytes(void);
int fvc_conv_wino_pack_weight(const float* w_host, void* wpack_host, float* osc_out);
int fvc_conv2d_nhwc_wino(const float* x, const void* wpack, float osc, const float* bias,
                         const float* res, float* y, float* pool, int batch, int h, int w, int in_op,
                         int act, int cu_reserve, int* overflow_flag, int* sched, int sched_len,
                         fvc_stream_t stream);
/* The same Winograd conv (in_op none / relu, act; no residual, pool or tap epilogue) reading
 * X = skip + upsample(low, 2x, bilinear, align_corners=True) instead of a materialised input:
 * Warp_net's c3_u = c1 + up(c3) and c4_u = c0 + up(c4) feeding ResBlock conv1
 * (endecoder.py:288-293; replaces F.interpolate + add + the conv's input read). skip / xsum:
 * [batch][h][w][64], low: [batch][h/2][w/2][64] (h, w even). X is formed in the kernel's LDS
 * staging and also written to xsum (every pixel, bit-identical to fvc_upsample2x_add_nhwc with
 * align_corners = 1, scale 1), which the ResBlock's conv2 reads as its residual. */
int fvc_conv2d_nhwc_wino_up(const float* skip, const float* low, float* xsum, const void* wpack,
                            float osc, const float* bias, float* y, int batch, int h, int w,
                            int in_op, int act, int cu_reserve, int* overflow_flag, int* sched,
                            int sched_len, fvc_stream_t stream);
/* The same Winograd conv (in_op none, act, res) fused with the next layer's tap partials, as
 * fvc_conv2d_nhwc_x3_tap: instead of y it writes P [batch][h][w][pcp] = T . y per pixel (Warp_net
 * conv5.conv2 -> conv6, endecoder.py:278-279: 27 partials of the 64 -> 3 3x3 conv), which
 * fvc_tap_gather_nhwc sums into the consumer's output. T [np <= 32][64] (rows t*cout' + co) is
 * packed by fvc_wino_tap_pack_weight (host, fvc_wino_tap_wpack_bytes(np) bytes; pcp = np rounded
 * up to 4). */
size_t fvc_wino_tap_wpack_bytes(int np);
int fvc_wino_tap_pack_weight(const float* w_host, void* wpack_host, float* osc_out, int np);
int fvc_conv2d_nhwc_wino_tap(const float* x, const void* wpack, float osc, const float* bias,
                             const float* res, float* P, int batch, int h, int w, int act,
                             const void* tap_wpack, float tap_osc, int pcp, int cu_reserve,
                             int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream);
/* The 128 -> 128 3x3 stride-1 layers (MV analysis/synthesis conv2/4/6/8, analysis_mv.py:58-66,
 * synthesis_mv.py:59-79; in_op none / relu, act, no residual) as four 64 -> 64 Winograd quarters
 * of the same kernel on 128-channel pixels: per output half the first input half's sum goes into
 * y's half, then the second input half adds bias and that partial sum before the activation.
 * wpack: fvc_conv_wino128_wpack_bytes() bytes from fvc_conv_wino128_pack_weight (w OIHW
 * [128][128][3][3]); osc4: the four quarter scales (host floats). */
int fvc_conv_wino128_supported(int cin, int cout, int ksize, int stride, int transposed);
size_t fvc_conv_wino128_wpack_bytes(void);
int fvc_conv_wino128_pack_weight(const float* w_host, void* wpack_host, float* osc4_out);
int fvc_conv2d_nhwc_wino128(const float* x, const void* wpack, const float* osc4_host, const float* bias,
                            float* y, int batch, int h, int w, int in_op, int act, int cu_reserve,
                            int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream);

/* Winograd-rows F(2,7) split-precision conv for SpyNet's 7x7 stride-1 pad-3 layers (MEBasic,
 * endecoder.py:142-169: conv2 32 -> 64, conv3 64 -> 32, conv4 32 -> 16; replaces the same
 * torch.nn.Conv2d forwards as fvc_conv2d_nhwc_x3). One launch covers 32 input channels and
 * 16 * nt (nt 1 or 2) output channels: x points at input channel ci0 (pixel pitch xp floats),
 * y at output channel co0 (pitch yp), bias at bias + co0. mode 0: y = act(conv + bias); mode 1:
 * y = conv (first 32-channel input half of a 64-channel layer, bias unused); mode 2:
 * y = act(conv + bias + y) (the second half). upack: fvc_conv_wr7_wpack_bytes(nt) bytes from
 * fvc_conv_wr7_pack_weight (host; w OIHW [cout][cin][7][7], the block ci0 .. ci0+31 x
 * co0 .. co0+16nt-1), osc from the same call. sched: >= 2 ints, zero between launches. */
int fvc_conv_wr7_supported(int cin, int cout, int ksize, int stride, int transposed);
size_t fvc_conv_wr7_wpack_bytes(int nt);
int fvc_conv_wr7_pack_weight(const float* w_host, int cin, int cout, int ci0, int co0, int nt,
                             void* wpack_host, float* osc_out);
int fvc_conv2d_nhwc_wr7(const float* x, int xp, const void* upack, int nt, float osc, const float* bias,
                        float* y, int yp, int batch, int h, int w, int mode, int act, int cu_reserve,
                        int* overflow_flag, int* sched, int sched_len, fvc_stream_t stream);

/* Split-precision direct conv for the small-input stems (fvc_conv_stem.hip; replaces ATen conv2d
 * for DVC/subnet/endecoder.py:253 Warp_net feature_ext 3x3 6->64, analysis_mv.py:19 mvEncoder conv1
 * 3x3 s2 2->128, analysis.py:15 resEncoder conv1 5x5 s2 3->64): 1 <= cin <= 8 on a 4-float (cin <= 4)
 * or 8-float pixel, cout 64 / 128, 3x3 s1 / s2 or 5x5 s2, padding k/2, bias + act (none / ReLU /
 * LeakyReLU 0.1). wpack: fvc_conv_stem_wpack_bytes(cin, cout, k) bytes from fvc_conv_stem_pack_weight
 * (host; w OIHW). Numerics as fvc_conv2d_nhwc_x3; overflow_flag as there. */
int fvc_conv_stem_supported(int cin, int cout, int ksize, int stride, int transposed);
size_t fvc_conv_stem_wpack_bytes(int cin, int cout, int ksize);
int fvc_conv_stem_pack_weight(const float* w_host, int cin, int cout, int ksize, void* wpack_host,
                              float* osc_out);
int fvc_conv2d_nhwc_stem(const float* x, const void* wpack, float osc, const float* bias, float* y,
                         int batch, int h, int w, int cin, int cout, int ksize, int stride, int act,
                         int* overflow_flag, fvc_stream_t stream);

/* ------------------------------------------------------------------ layout / resampling */
int fvc_nchw_to_nhwc(const float* src, float* dst, int batch, int c, int h, int w, int cp,
                     fvc_stream_t stream);
/* clamp01: also clamp to [0,1] (the decoder's final recon.clamp(0,1), net.py:105) */
int fvc_nhwc_to_nchw(const float* src, float* dst, int batch, int c, int h, int w, int cp,
                     int clamp01, fvc_stream_t stream);
/* 2x2 mean, src h x w (even) -> h/2 x w/2 */
int fvc_avgpool2_nhwc(const float* src, float* dst, int batch, int h, int w, int cp,
                      fvc_stream_t stream);
/* backward bilinear warp, border padding (torch_warp), im/out [b][h][w][cp], flow [b][h][w][4] */
int fvc_warp_nhwc(const float* im, const float* flow, float* out, int batch, int h, int w, int cp,
                  fvc_stream_t stream);
/* out = skip + upsample2x(src) ; src h x w -> 2h x 2w ; align_corners 0/1 ; scale multiplies
 * the upsampled value (SpyNet uses 2.0, ac=0); skip may be NULL */
int fvc_upsample2x_add_nhwc(const float* src, const float* skip, float* out, int batch, int h,
                            int w, int cp, int align_corners, float scale, fvc_stream_t stream);
/* SpyNet level input (endecoder.py:352-354): flow_up = 2*up2(flow_prev) (flow_prev may be NULL
 * = zeros); x8 = [im1, warp(im2, flow_up), flow_up]; im1/im2 [b][h][w][4], flow [b][h][w][4],
 * x8 [b][h][w][8] */
int fvc_spynet_assemble(const float* im1, const float* im2, const float* flow_prev,
                        float* flow_up, float* x8, int batch, int h, int w, fvc_stream_t stream);
/* motion compensation input (net.py:64-68): warpframe = warp(ref, mv); x8 = [warpframe, ref, 0, 0] */
int fvc_mc_assemble(const float* ref, const float* mv, float* warpframe, float* x8, int batch,
                    int h, int w, fvc_stream_t stream);
/* out = a - b elementwise over n floats */
int fvc_sub_f32(const float* a, const float* b, float* out, size_t n, fvc_stream_t stream);

/* cout <= 4 conv (stride 1) / transposed conv (stride 2) as a tap-partial GEMM: P [batch,h,w,pcp]
 * holds, per input pixel, sum_ci x * w for every tap t = ky*ksize+kx and output channel co at
 * channel t*cout+co (a 1x1 fvc_conv2d_nhwc_x3 with cout' = ksize^2 * cout); this sums the taps
 * reaching each output pixel, adds bias, applies act / res / post_op, writes y [.., 4] (pad = 0).
 * Replaces the same nn.Conv2d / nn.ConvTranspose2d forwards as fvc_conv2d_nhwc_* for the 2- and
 * 3-channel output layers (DVC/subnet/endecoder.py:279,295 Warp_net.conv6; synthesis_mv.py:43
 * deconv8; synthesis.py:26,57 deconv4). */
int fvc_tap_gather_nhwc(const float* P, int pcp, const float* bias, const float* res, float* y, int batch,
                        int h, int w, int cout, int ksize, int stride, int transposed, int act, int post_op,
                        fvc_stream_t stream);

/* ------------------------------------------------------------------ GDN (GDN.py:63-93)
 * beta/gamma are the effective (bounded, reparametrised) parameters: gamma[i*c + j] */
int fvc_gdn_nhwc(const float* x, float* y, const float* beta, const float* gamma, int batch,
                 int h, int w, int c, int inverse, fvc_stream_t stream);
/* GDN / IGDN of x (64 channels) followed by the next layer's 1x1 tap-partial GEMM: P [b][h][w][pcp]
 * = tap_w . y with y never written (resDecoder igdn3 -> deconv4, synthesis.py:26,57); tap_wpack
 * is ntiles concatenated fvc_x3_tap_pack_weight packs of 32 rows each (cin = 64), tap_osc
 * (host, ntiles floats) their scales; |y| >= 65000 ORs 1 into *overflow_flag. */
int fvc_gdn_tap_nhwc(const float* x, float* P, const float* beta, const float* gamma,
                     const void* tap_wpack, const float* tap_osc, int ntiles, int pcp, int batch,
                     int h, int w, int c, int inverse, int* overflow_flag, fvc_stream_t stream);

/* ------------------------------------------------------------------ reductions
 * Deterministic (fixed-order, no atomics) two-pass reductions; ws must hold
 * fvc_reduce_ws_doubles() doubles. Results are written to device doubles. */
size_t fvc_reduce_ws_doubles(void);
/* clipped = clamp(recon,0,1) as NCHW [b][3][h][w]; out4 = {sum (recon-in)^2, sum (warp-in)^2,
 * sum (pred-in)^2, sum (clipped-in)^2} over b*3*h*w elements (all inputs NHWC cp=4): DVC's
 * mse/warp/inter losses use the unclipped recon (net.py:103-116), RLVC's img_loss / PSNR the
 * clipped Y1_com (models.py:1019,1033-1034) */
int fvc_recon_finalize(const float* recon, const float* input, const float* warpframe,
                       const float* prediction, float* clipped_nchw, double* out4, double* ws,
                       int batch, int h, int w, fvc_stream_t stream);
/* bits of round(feature) under Laplace(0, clamp(sigma,1e-5,1e10)) (net.py:121-151) */
int fvc_bits_laplace(const float* feature, const float* sigma, double* out1, double* ws,
                     int batch, int h, int w, int c, int cp, fvc_stream_t stream);
/* bits of round(v) under the per-channel BitEstimator (net.py:153-205); params [11][c]:
 * h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4 */
int fvc_bits_factorized(const float* v, const float* params, double* out1, double* ws,
                        int batch, int h, int w, int c, int cp, fvc_stream_t stream);

/* ------------------------------------------------------------------ entropy coding
 * Symbol streams are channel-major: stream (b, ch) holds round(lat[b,:,:,ch]) in raster
 * order. Each stream is coded independently and is byte-identical to compressai's
 * RansEncoder.encode_with_indexes on that sequence (precision 16, bypass 4 bits). */
int fvc_latent_to_symbols(const float* lat, int32_t* sym, int batch, int h, int w, int c, int cp,
                          fvc_stream_t stream);
int fvc_symbols_to_latent(const int32_t* sym, float* lat, int batch, int h, int w, int c, int cp,
                          fvc_stream_t stream);
/* GaussianConditional.build_indexes over a scale table; output channel-major like symbols */
int fvc_build_indexes(const float* sigma, const float* scale_table, int n_scales, int32_t* idx,
                      int batch, int h, int w, int c, int cp, fvc_stream_t stream);
/* per-channel table index for factorized latents: idx[b][ch][i] = ch */
int fvc_channel_indexes(int32_t* idx, int batch, int hw, int c, fvc_stream_t stream);
/* Elementwise over n values of any contiguous layout (the compressai-framed API, NCHW):
 * EntropyModel.quantize(x, "symbols", means): sym = round_half_even(x - means) (means may be NULL);
 * EntropyModel.dequantize: out = sym + means; GaussianConditional.build_indexes on a flat array. */
int fvc_quantize_symbols(const float* x, const float* means, int32_t* sym, size_t n, fvc_stream_t stream);
int fvc_dequantize_symbols(const int32_t* sym, const float* means, float* out, size_t n,
                           fvc_stream_t stream);
int fvc_build_indexes_flat(const float* scales, const float* scale_table, int n_scales, int32_t* idx,
                           size_t n, fvc_stream_t stream);

/* host: compressai pmf_to_quantized_cdf; cdf_out has n+1 entries. */
int fvc_pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf_out);

/* Device rANS over nstreams independent streams. Stream s codes symbols
 * [sym_off[s], sym_off[s+1]) (nsymbols in total) with tables indexes[i]; cdfs is
 * [ntables][cdf_stride] int32, cdf_sizes/offsets per table (compressai _quantized_cdf /
 * _cdf_length / _offset). ws: fvc_rans_encode_ws_bytes(nsymbols) bytes of scratch.
 * Encode writes stream s downward into words[word_off[s] .. word_off[s+1]) and its length
 * (in 32-bit words, counted from the END of its region) into nwords[s] (-1 = no space); the
 * stream's bytes are the last nwords[s] words of its region, little-endian. */
size_t fvc_rans_encode_ws_bytes(int64_t nsymbols);
int fvc_rans_encode(const int32_t* symbols, const int32_t* indexes, const int64_t* sym_off,
                    int nstreams, int64_t nsymbols, const int32_t* cdfs, int cdf_stride,
                    const int32_t* cdf_sizes, const int32_t* offsets, void* ws, uint32_t* words,
                    const int64_t* word_off, int32_t* nwords, fvc_stream_t stream);
/* Pack encoded regions into one contiguous buffer: out[pack_off[s] ..] = last nwords[s] words
 * of region s; pack_off is [nstreams+1] (exclusive scan of nwords, computed on device).
 * status (device int, may be NULL) = 0, or FVC_ENOSPC if any stream ran out of space (such a
 * stream packs as empty; the caller must not ship the result). */
int fvc_rans_pack(const uint32_t* words, const int64_t* word_off, const int32_t* nwords,
                  int nstreams, int64_t* pack_off, uint32_t* out, int32_t* status,
                  fvc_stream_t stream);
/* Decode tables, built once per table set (fvc_rans_lut_bytes(ntables, cdf_stride) bytes): per
 * table a 128-bucket cum -> {first, last candidate symbol, start|freq of the first} map and a
 * start|freq<<16 word per symbol. The decoder copies the tables its streams use into LDS (a
 * decoded symbol then costs one LDS read in most buckets) and reads the rest from L2. */
size_t fvc_rans_lut_bytes(int ntables, int cdf_stride);
int fvc_rans_build_lut(const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes, int ntables,
                       void* lut, fvc_stream_t stream);
/* Decode: stream s reads packed words starting at pack_off[s]; status[s] = 0 or FVC_ECORRUPT.
 * Output identical to compressai RansDecoder.decode_with_indexes per stream. */
/* streams_per_block (1..64, 0 = 64): a block decodes that many streams, one lane each. Fewer
 * streams per block keep every stream's tables in the block's LDS cache (no lane waits on L2 per
 * symbol: lower latency), more leave CUs free for concurrent kernels (higher pipelined throughput):
 * the GOP pipeline passes 64, latency-bound decodes 16. */
int fvc_rans_decode(const uint32_t* packed, const int64_t* pack_off, const int32_t* indexes,
                    const int64_t* sym_off, int nstreams, int ntables, int cdf_stride,
                    const int32_t* cdf_sizes, const int32_t* offsets, const void* lut,
                    int32_t* symbols, int32_t* status, int streams_per_block, fvc_stream_t stream);

/* ------------------------------------------------------------------ I-frame codec
 * Replaces the reference's BPG I-frame (models.py:412-429 I_compression: bpgenc/bpgdec through
 * os.system; the binaries are absent). Integer pipeline, encoder == decoder bit for bit:
 * rct_fwd: x [b][3][h][w] in [0,1] -> q = clamp(rint(255 x), 0, 255) -> JPEG 2000 RCT planes
 *          (Y, U, V) int32 [b][3][h][w]; rct_inv: the inverse, back to k/255 floats.
 * dwt53:   `levels` levels of the reversible LeGall 5/3 lifting wavelet over `planes` planes of
 *          h x w (rows then columns; Mallat layout), in place; tmp is scratch of the same size;
 *          h, w multiples of 2^levels. inverse = 1 undoes it exactly.
 * quant:   dead-zone quantisation (step q >= 1) of every coefficient outside the level-L LL
 *          band; inverse = 1 reconstructs sign(v) (|v| q + q/2).
 * block_index: per (plane, bs x bs block) the Laplace scale-table index of the block's mean
 *          |coefficient| (compressai build_indexes semantics) into bidx (uint8), expanded to a
 *          per-coefficient int32 index for the range coder; expand_index does the expansion
 *          alone (decoder side). */
int fvc_iframe_rct_fwd(const float* x, int32_t* coeff, int batch, int h, int w, fvc_stream_t stream);
int fvc_iframe_rct_inv(const int32_t* coeff, float* x, int batch, int h, int w, fvc_stream_t stream);
int fvc_iframe_dwt53(int32_t* coeff, int32_t* tmp, int planes, int h, int w, int levels, int inverse,
                     fvc_stream_t stream);
int fvc_iframe_quant(int32_t* coeff, int planes, int h, int w, int levels, int q, int inverse,
                     fvc_stream_t stream);
int fvc_iframe_block_index(const int32_t* coeff, const float* scale_table, int n_scales, uint8_t* bidx,
                           int32_t* idx, int planes, int h, int w, int bs, fvc_stream_t stream);
int fvc_iframe_expand_index(const uint8_t* bidx, int32_t* idx, int planes, int h, int w, int bs,
                            fvc_stream_t stream);

/* ------------------------------------------------------------------ RLVC path
 * gdn_nhwc_cai: compressai.layers.GDN (models.py:23; RLVC Coder2D, models.py:529-538), C in
 *   {64, 128}: y = x * rsqrt(beta + gamma . x^2), inverse: y = x * sqrt(...); beta/gamma effective.
 * lstm_gates: ConvLSTM cell update (entropy_models.py:367-378) from the 4 gate conv outputs.
 * rpm_scale: exp(max(sigma, -7)) / 10 (entropy_models.py:61-62).
 * eb_forward: compressai EntropyBottleneck (filters 3,3,3,3) eval forward: x_hat = round(x - med)
 *   + med and the sum of clamp(-log2(likelihood + 1e-5), 0, 50) (get_estimate_bits,
 *   entropy_models.py:74-78); params [C][58] = softplus(matrices), biases, tanh(factors).
 * gc_forward: compressai GaussianConditional with means: x_hat = round(x - mu) + mu and the bits
 *   sum under N(mu, max(scale, 0.11)). */
int fvc_gdn_nhwc_cai(const float* x, float* y, const float* beta, const float* gamma, int batch, int h, int w,
                     int c, int inverse, fvc_stream_t stream);
int fvc_lstm_gates(const float* gj, const float* gi, const float* gf, const float* go, const float* c_prev,
                   float* c_out, float* h_out, size_t n, float forget_bias, fvc_stream_t stream);
int fvc_rpm_scale(const float* in, float* out, size_t n, fvc_stream_t stream);
int fvc_eb_forward(const float* x, const float* params, const float* medians, float* xhat, double* out1,
                   double* ws, int batch, int h, int w, int c, int cp, fvc_stream_t stream);
int fvc_gc_forward(const float* x, const float* scale, const float* mu, float* xhat, double* out1, double* ws,
                   int batch, int h, int w, int c, int cp, fvc_stream_t stream);

/* ------------------------------------------------------------------ torchac-compatible coder
 * Replaces torchac.encode_float_cdf / decode_float_cdf (third-party, absent), which DVC's
 * calrealbits mode calls with 2*mxrange bins per element (DVC/net.py:123-138, 155-168, 183-195).
 * Device (stream-ordered): CDF rows / symbol bounds in torchac's int16 normalisation
 * (round(cdf * (2^16 - (Lp-1))) + k, as uint16), elements in NCHW order; latents are NHWC with
 * cp padded channels. status (device int) |= 1 for a symbol outside [0, Lp-2] (torchac's
 * check_input_bounds). Host (synchronous, CPU memory): the sequential arithmetic coder over
 * [lo, hi) bounds (encode: FVC_ENOSPC if cap is too small; fvc_torchac_max_bytes(n) always
 * fits) and its decoder over uint16 rows (rows == NULL: element i uses row i; else rows[i] < nrows). */
int fvc_torchac_normalize(const float* cdf, int64_t nrows, int Lp, int needs_normalization, uint16_t* out,
                          fvc_stream_t stream);
int fvc_torchac_rows_bounds(const uint16_t* rows, const int16_t* sym, int64_t n, int Lp, uint32_t* lo,
                            uint32_t* hi, int* status, fvc_stream_t stream);
int fvc_torchac_laplace_rows(const float* sigma, int batch, int h, int w, int c, int cp, int mxrange,
                             uint16_t* rows, fvc_stream_t stream);
int fvc_torchac_laplace_bounds(const float* x, const float* sigma, int batch, int h, int w, int c, int cp,
                               int mxrange, uint32_t* lo, uint32_t* hi, int* status, fvc_stream_t stream);
int fvc_torchac_bitest_table(const float* params, int c, int mxrange, uint16_t* table, fvc_stream_t stream);
int fvc_torchac_table_bounds(const float* x, const uint16_t* table, int batch, int h, int w, int c, int cp,
                             int mxrange, uint32_t* lo, uint32_t* hi, int* status, fvc_stream_t stream);
size_t fvc_torchac_max_bytes(int64_t n);
int fvc_torchac_encode(const uint32_t* lo, const uint32_t* hi, int64_t n, uint8_t* out, size_t cap,
                       size_t* out_len);
int fvc_torchac_decode(const uint16_t* cdf, int Lp, const int32_t* rows, int64_t nrows, int64_t n,
                       const uint8_t* in, size_t len, int16_t* sym);

#ifdef __cplusplus
}
#endif
#endif /* FVC_H_ */
