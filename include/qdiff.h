/*
 * libqdiff — C ABI of the MI355X (gfx950) quantized-diffusion denoising path.
 *
 * The reference (maani3/Quantization---Diffusion-Models) has no FFI: its boundary is the
 * nn.Module swap of quantize/quantizer.py:517,533 that replaces every nn.Linear / nn.Conv2d of
 * the UNet with WxAxLinear / WxAxConv2d (quantize/fake_quant.py:170-398), whose forward calls
 * F.linear / F.conv2d on fp16 fake-quantized operands.  The Python host package mirrors those
 * module classes (same names, from_float keywords, buffers and errors) and calls the entry
 * points below; each entry point cites the reference computation it replaces.
 *
 * Conventions
 *   - Plain pointers to caller-allocated DEVICE memory; fp16 tensors are IEEE binary16.
 *   - `stream` is a hipStream_t passed as void*; every call is stream-ordered, enqueues work
 *     only (no host sync, no allocation), and is capturable into a hipGraph.
 *   - Return 0 on success, QD_ERR_ARG on a bad argument (nothing launched), or the hipError_t
 *     of a failed launch.  qd_last_error() returns a static message for the last failure.
 *   - Activations of the fused UNet path are NHWC ([N, H, W, C], C fastest) == token layout
 *     [N, H*W, C]; the drop-in modules also accept NCHW.
 */
#ifndef QDIFF_H
#define QDIFF_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QD_OK 0
#define QD_ERR_ARG 1000

/* granularities (fake_quant.py names) */
#define QD_GRAN_PER_TOKEN 0    /* quantize_activation_per_token_absmax   fake_quant.py:108-118 */
#define QD_GRAN_PER_CHANNEL 1  /* quantize_activation_per_channel_absmax fake_quant.py:123-131 */
#define QD_GRAN_PER_TENSOR 2   /* quantize_activation_per_tensor_absmax  fake_quant.py:157-167 */
#define QD_GRAN_PER_GROUP 3    /* quantize_activation_per_channel_group_absmax :133-153 */
/* qd_act_absmax only: OR into `gran` when `amax` is known to hold zeros already (a pooled
 * buffer zeroed once per step with qd_fill_zero); the call then skips its own zero-fill. */
#define QD_GRAN_ZEROED 0x100

#define QD_LAYOUT_NCHW 0
#define QD_LAYOUT_NHWC 1

/* weight storage formats of the GEMM B operand */
#define QD_WFMT_F16 0   /* dequantized fp16 (the reference's own buffer format) */
#define QD_WFMT_I8 1    /* int8 codes [N][K] + fp16 scales [N][K/group] */
#define QD_WFMT_I4 2    /* int4 codes packed 8/dword along K (qd_pack_int4 layout) + scales */

int qd_version(void);
const char* qd_last_error(void);
int qd_device_arch(char* buf, int len); /* writes gcnArchName of the current device */
/* p[0:n) = 0.0f with a kernel (never a memset node: graph-capture safe). */
int qd_fill_zero(float* p, long n, void* stream);

/* ---------------- activation fake-quant ---------------------------------------------- */
/* Reduction pass: amax[...] = max |x| over the granularity's reduction set.  `amax` is fp32,
 * sized N*C (per_channel), rows (per_token), 1 (per_tensor), N*C*(H/g)*(W/g) (per_group);
 * it is zeroed by the call.  x is [n, c, h, w] in `layout` (per_token: rows = n*h*w... see
 * qd_act_fakequant). */
int qd_act_absmax(const void* x, int layout, int n, int c, int h, int w, int gran, int group,
                  float* amax, void* stream);
/* Full quantize->dequantize of an activation tensor (both passes), y may alias x.
 * Replaces quantize_activation_{per_token,per_channel,per_tensor,per_channel_group}_absmax
 * (fake_quant.py:108-167).  per_token: x is viewed as [n*h*w... rows = n, cols = c] i.e. pass
 * (n = rows, c = cols, h = w = 1).  per_group: NCHW only, `group` already shrunk by the host
 * rule of fake_quant.py:138-139.  `amax_ws` is an fp32 workspace of the qd_act_absmax size. */
int qd_act_fakequant(const void* x, void* y, int layout, int n, int c, int h, int w, int gran,
                     int group, int n_bits, float* amax_ws, void* stream);
/* Quantize with a precomputed amax (second pass only).  For NHWC per_channel, group > 0 means
 * only the first `group` channels are real (the rest is zero channel padding, copied as is). */
int qd_act_apply(const void* x, void* y, int layout, int n, int c, int h, int w, int gran,
                 int group, int n_bits, const float* amax, void* stream);

/* quantize_activation_per_channel_absmax (fake_quant.py:123-131) of the NHWC channel concat
 * [x (c1) | x2 (c2)] -> y [n, hw, c1 + c2]: the UNet skip concat feeding a quantized conv,
 * materialised only in its quantized form.  amax: fp32 [n*(c1+c2)] workspace (zeroed by the
 * call unless amax_zeroed). */
int qd_act_quant_cat_nhwc(const void* x, int c1, const void* x2, int c2, int n, int hw, int n_bits,
                          float* amax, int amax_zeroed, void* y, void* stream);
/* qd_act_quant_cat_nhwc's apply pass with the per-(n, c) maxima of [x | x2] already known
 * (amax [n*(c1+c2)], e.g. qd_groupnorm_xamax over the same concat): no column-max pass. */
int qd_act_apply_cat_nhwc(const void* x, int c1, const void* x2, int c2, int n, int hw, int n_bits,
                          const float* amax, void* y, void* stream);
/* NHWC per_channel fake-quant (qd_act_absmax + qd_act_apply, fake_quant.py:123-131) of a SMALL tensor
 * in one launch, one workgroup per sample: x, y [n][hw][c] (y may alias x), channels >= c_valid
 * (c_valid > 0) copied as is; same bits as the two passes.  qd_act_fq_small_ok(hw, c) (returns 0/1,
 * no status): c % 8 == 0, c / 8 a power of two, hw * c / 8 <= 4096 (the UNet's conv_in latent). */
int qd_act_fq_small_ok(int hw, int c);
int qd_act_fq_small_nhwc(const void* x, void* y, int n, int hw, int c, int c_valid, int n_bits, void* stream);

/* ---------------- weight fake-quant (offline, on device) ----------------------------- */
/* Row-group absmax RTN of quantize_weight_absmax / _per_channel_ / _per_tensor_
 * (fake_quant.py:21-105).  w is [rows, cols] fp16 (a 4-D conv weight is [Co*Ci*kh, kw]);
 * groups of `group` consecutive elements along cols (group == cols for per_channel;
 * per_tensor: group = rows*cols with rows = 1).  Any of codes (int8 [rows, cols]),
 * scales (fp16 [rows, cols/group]) and w_dq (fp16 [rows, cols]) may be NULL.  n_bits in
 * [2, 16] as the reference accepts any width; codes must be NULL above 8 bits. */
int qd_weight_quant(const void* w, int rows, int cols, int group, int n_bits, int8_t* codes,
                    void* scales, void* w_dq, void* stream);
/* pack int8 codes q in [-8, 7] to int4, 8 per little-endian dword along cols (cols % 8 == 0):
 * in the dword of codes k = 8i .. 8i + 7, nibble j holds q(8i + 2j) + 8 and nibble j + 4 holds
 * q(8i + 2j + 1) + 8, so (w >> 4j) & 0x000F000F | 0x64006400 is the fp16 pair (1024 + c, 1024 + c')
 * of two consecutive k (the GEMM's packed dequant).  `packed` 4-B aligned. */
int qd_pack_int4(const int8_t* codes, int rows, int cols, uint8_t* packed, void* stream);
/* conv weight [Co][Ci][kh][kw] -> GEMM B layout [Co][kh][kw][Ci_pad] (zero-padded Ci). */
int qd_conv_weight_khwc(const void* w, int co, int ci, int kh, int kw, int ci_pad, void* out,
                        void* stream);

/* ---------------- GEMMs (fp16 MFMA, fp32 accumulate) --------------------------------- */
/* Epilogue flags */
#define QD_EPI_BIAS 1        /* + bias[N] (fp16), then round to fp16 (F.linear/F.conv2d out) */
#define QD_EPI_RESIDUAL 2    /* out = half(y + residual[M, N]) */
#define QD_EPI_AMAX 4        /* per-(sample, col) amax of the rounded y into amax[M/rows_per_sample][N]
                                (zeroed by the call itself, then atomically max-reduced) */
#define QD_EPI_AMAX_ZEROED 16 /* with QD_EPI_AMAX: amax already holds zeros (pooled, zeroed once
                                 per step); the call skips its own zero-fill launch */
#define QD_EPI_GEGLU 8       /* B holds [hidden; gate] halves (N = 2*I): out[M, I] = h * gelu(g) */
#define QD_EPI_GELU_TANH 32  /* out = half(gelu_tanh(half(y + bias))): diffusers GELU(approximate="tanh")
                                (SD3 FeedForward net.0) applied to the rounded projection output;
                                no residual / amax / GEGLU with it */
#define QD_EPI_AMAX_POST 64  /* with QD_EPI_AMAX | QD_EPI_RESIDUAL: the amax is of the FINAL output
                                half(half(y + bias) + residual) - the per-(sample, channel) input amax
                                of the quantized conv that consumes it (fake_quant.py:125 reduction),
                                so no separate column-max pass; never split-K or ping-pong tiles */
#define QD_EPI_CADD 128      /* int8 conv (qd_conv2d_i8): out = half(out + cadd[n * cadd_ld + col]), one
                                fp16 vector per (sample, column) after the residual - the diffusers
                                ResnetBlock2D time-embedding add of conv1's output */
#define QD_EPI_GNSTATS 256   /* int8 conv (qd_conv2d_i8): GroupNorm statistics of the FINAL output over
                                64-row slots of each sample into gn_part[M / 64][N] float4 = (slot mean,
                                sum of squared deviations from it, min, max), fp32 - the consuming
                                GroupNorm (qd_groupnorm_part) needs no statistics pass over the
                                tensor; rows_per_sample % 64 == 0, never ping-pong tiles */
#define QD_EPI_LN 512        /* (set by qd_linear_ln / qd_linear_i8_ln) */
#define QD_EPI_SILU 1024     /* qd_linear_fwd GEMV shapes only (M <= 4): out = half(silu(out)) after the
                                bias / residual rounding - the diffusers TimestepEmbedding act and
                                the UNet's silu(temb), bit-identical to qd_silu on the output */
#define QD_EPI_ROWREP 2048   /* qd_linear_fwd GEMV shapes with M == 1, no residual: the output row is
                                stored to rows 0 .. rows_per_sample - 1 of y (stride ldy) - a batch whose
                                rows share one input (the CFG batch's time embedding: every row embeds
                                the same timestep) computed once, every row bit-identical */

/* y[M, N] = x[M, K] . W[N, K]^T (+ epilogue).  WxAxLinear.forward's F.linear
 * (fake_quant.py:223) with the dequant of the stored codes fused into the B-tile staging.
 * wfmt: QD_WFMT_*; wscale [N][K/group] fp16 for I8/I4.  wscale_t (I4 only, optional, 16-B
 * aligned): the same scales as [K/group][N]; with it the int4 codes also run in the LDS-DMA /
 * ping-pong families (qd_gemm_force 110..117, 300..304), dequantized from LDS per fragment with the
 * register tile's rounding (bit-identical results).  lda/ldy in elements.
 * rows_per_sample: sample boundary for QD_EPI_AMAX (multiple of 32).
 * M <= 4 without AMAX / GEGLU runs a weight-stream GEMV (same dequant and epilogue rounding; v_dot2
 * fp32 accumulation instead of the MFMA's, so only the summation order differs from the tile GEMM);
 * QD_EPI_SILU requires such a shape. */
int qd_linear_fwd(const void* x, int M, int K, int lda, const void* w, int wfmt,
                  const void* wscale, const void* wscale_t, int group, const void* bias,
                  const void* residual, void* y, int N, int ldy, int epi, float* amax,
                  int rows_per_sample, float* ws, long ws_elems, void* stream);

/* Tuning / test knob (process-global, not thread-safe): force the GEMM kernel family of every
 * following qd_linear_fwd / qd_conv2d_fwd.  -1 = planner's choice (default); 0..3 = the
 * register-staged tiles 128x160, 128x128, 128x64, 64x64; 100 + i = LDS-DMA variant i (F16
 * weights; packed int4 with wscale_t: the BK-32 variants 110..117 and ping-pong 300..304; other
 * quantized formats keep the planner's register-staged choice); 200..203 the fp16 halo conv (BN 160 /
 * 128, lock-step / split-phase), 204 / 205 the split-phase halo conv on 128-pixel tiles (images
 * <= 32 wide; forceable only, no tuner candidate).  int8 (qd_linear_i8 / qd_conv2d_i8):
 * 110..117 LDS-DMA, 130..134 ping-pong, 140..149 halo conv, 150 / 151 the fused GEGLU + codes kernel,
 * 160..167 / 170..177 persistent LDS-DMA linears (2 / 4 tiles per block), 190..192 A-stationary
 * linears.  + 1000 * s: explicit split-K count s (1 = unsplit).  Every int8 choice gives the same bits. */
int qd_gemm_force(int variant);
/* Measurement knob: on != 0 routes every GEMM / conv epilogue through the LDS C tile (the default,
 * 0, stores straight from the MFMA fragments wherever the epilogue allows; same output bits). */
int qd_gemm_epi_lds(int on);

/* Measurement knob (process-global): rows per thread of the streaming GroupNorm statistics /
 * apply passes (qd_groupnorm*, 0 = the built-in rule).  Changes the workspace size, so query
 * qd_groupnorm_workspace after setting it. */
int qd_gn_geom_force(int stats_rows_per_thread, int apply_rows_per_thread);

/* fp32 elements of split-K workspace the GEMM plans for this shape (0: runs unsplit).  Pass
 * at least that much as (ws, ws_elems) to qd_linear_fwd / qd_conv2d_fwd (conv: M = N*Ho*Wo,
 * K = kh*kw*Ci_pad, rows_per_sample = Ho*Wo); with less (or NULL) the call runs unsplit.
 * group: the int4 group size the qd_linear_fwd call passes (QD_WFMT_I4 with wscale_t; else 0),
 * so the queried plan is the launch's plan. */
long qd_gemm_workspace(int M, int N, int K, int wfmt, int group, int rows_per_sample, int epi);

/* NHWC implicit-GEMM Conv2d: y[N, Ho, Wo, Co] = conv(x[N, H, W, Ci], W[Co][kh][kw][Ci_pad]).
 * WxAxConv2d.forward's F.conv2d (fake_quant.py:339); groups = dilation = 1.
 * x channel stride is Ci_pad (>= Ci, multiple of 8, padded channels zero).
 * upsample2x != 0: x is the pre-upsample tensor [N, H/2, W/2, Ci] read with nearest
 * indexing (diffusers Upsample2D interpolate + conv fused).  QD_EPI_AMAX: per-(n, co) amax of
 * the rounded output into amax[N][Co] (zeroed by the call). */
int qd_conv2d_fwd(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt, int co,
                  int kh, int kw, int stride, int pad, int upsample2x, const void* bias,
                  const void* residual, void* y, int epi, float* amax, float* ws, long ws_elems,
                  void* stream);

/* Conv output fake-quant + fused adds (the q_y = output_quant(y) of fake_quant.py:340 followed
 * by the diffusers residual / temb add): out = half(fq(y; amax[n][c]) + res) with res either a
 * full [N, HW, C] tensor (`residual`), or a per-(n, c) vector (`chan_add` [N][chan_add_ld], the
 * time embedding projection; chan_add_ld <= 0 means C), or none.  n_bits == 0 disables the
 * quantization. */
int qd_fq_finalize(const void* y, const float* amax, int n, int hw, int c, int n_bits,
                   const void* residual, const void* chan_add, int chan_add_ld, void* out,
                   void* stream);
/* Measurement knobs (sweep scripts only; process-wide, not thread-safe): the per-channel column-max
 * launch geometry (min_blocks / max_rows_per_thread, <= 0: the defaults 128 / 64) and the attention
 * kernel choice (0: heuristic; 1-6 the 16x16x32 k_attn configurations, 7 / 8 the 32x32x16 kernel
 * with 4 / 8 waves (8: the staggered form the heuristic runs), 9 the 8-wave kernel unstaggered). */
int qd_colmax_geom_force(int min_blocks, int max_rows_per_thread);
int qd_attn_force(int cfg);
/* qd_conv2d_fwd (epi = QD_EPI_AMAX [| QD_EPI_AMAX_ZEROED | QD_EPI_BIAS]) followed by
 * qd_fq_finalize(y, amax, ..., n_bits, residual, chan_add, chan_add_ld, out = y): when the plan splits
 * K and a sample's Ho*Wo rows (<= 256, a multiple of 32) fit one reduction block, the split-K
 * reduction finalizes the output itself (column maxima in LDS, no atomics, no finalize launch);
 * otherwise the two launches run.  y = the final output, amax = the per-(n, co) maxima; bit-identical
 * to the two calls either way.  xamax (optional, [N][Co] fp32): the final output's per-(n, co)
 * max |y| - the per_channel input amax of the conv that consumes it (= qd_act_absmax of y). */
int qd_conv2d_fq(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt, int co, int kh, int kw,
                 int stride, int pad, int upsample2x, const void* bias, int n_bits, const void* residual,
                 const void* chan_add, int chan_add_ld, void* y, int epi, float* amax, float* xamax, float* ws,
                 long ws_elems, void* stream);

/* ---------------- int8-MFMA W8A8 mode ------------------------------------------------ */
/* The reference's W8A8 is fake-quant (fp16 F.linear / F.conv2d on dequantized operands,
 * fake_quant.py:223, 339) with granularities that vary along K (conv weights per (Co, Ci, kh),
 * activations per (n, c): fake_quant.py:86-93, 123-131), so an integer dot product cannot
 * reproduce it.  This mode re-granularizes to what factors out of the dot product and computes
 * on v_mfma_i32_16x16x64_i8: weights per output channel, activations per token (linear) or per
 * sample (conv), codes from the reference's RTN recipe (fake_quant.py:44-46: s = half(half(amax)
 * / 127), q = rint(half(x / s))), exact int32 sums, then y = half(((float)acc * sa) * sw + bias)
 * and the same epilogue flags as the fp16 GEMM.  Tolerance vs the fake-quant path: DESIGN.md. */
/* int8 codes of each row of x [rows][ldx] (c values, dynamic per token) -> y [rows][ldy],
 * scales[rows] fp32 (the fp16 scale widened). */
int qd_quant_rows_i8(const void* x, long rows, int c, int ldx, int8_t* y, int ldy, float* scales, void* stream);
/* int8 codes of n samples of per_sample contiguous values each (one scale per sample: the
 * conv-input granularity of this mode) -> y, scales[n]; amax_ws fp32 [n] workspace, zeroed by the
 * call unless amax_zeroed (a pooled buffer zeroed once per step). */
int qd_quant_samples_i8(const void* x, int n, long per_sample, int8_t* y, float* scales, float* amax_ws,
                        int amax_zeroed, void* stream);
/* qd_quant_samples_i8 with the per-(sample, channel) amax of x [n][rows][c] already reduced by its
 * producer (a GEMM's QD_EPI_AMAX | QD_EPI_AMAX_POST epilogue): the sample's scale is the max over
 * amax_nc[n][0..c) - the same value, codes and scales as qd_quant_samples_i8. */
int qd_quant_samples_i8_amax(const void* x, int n, long per_sample, const float* amax_nc, int c, int8_t* y,
                             float* scales, void* stream);
/* y[M, N] = (x_i8[M, K] . w_i8[N, K]^T) * sa[m] * sw[n] (+ epilogue), K % 64 == 0, lda % 16 == 0;
 * sa fp32 [M], sw fp32 [N] (16-B aligned).  Epilogue flags / rows_per_sample / workspace as
 * qd_linear_fwd (workspace size: qd_gemm_i8_workspace).  qd_gemm_force 110..113 picks the tile. */
int qd_linear_i8(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                 const void* bias, const void* residual, void* y, int N, int ldy, int epi, float* amax,
                 int rows_per_sample, float* ws, long ws_elems, void* stream);
/* int8-MFMA mode, diffusers FeedForward at the SD1.5 64x64 level: the GEGLU projection (w [N][K] codes
 * with rows interleaved in 16-row [hidden | gate] blocks, fp32 per-row scales sw, fp16 bias) of
 * per-token codes x / sa, GEGLU, and the per-token int8 codes y8 [M, N / 2] (ldy8) + fp32 scales
 * sa8 [M] of its output - ff.net.2's input - in ONE launch; the fp16 GEGLU output never reaches
 * memory.  Bit-identical to qd_linear_i8(..., QD_EPI_GEGLU) followed by qd_quant_rows_i8.  Replaces
 * ff.net.0 + ff.net.2's input quantization (reference: diffusers GEGLU around quantize/
 * fake_quant.py:223's F.linear).  Shapes: qd_linear_i8_geglu_q_ok(K, N) (K 320, N 2560). */
int qd_linear_i8_geglu_q_ok(int K, int N);
int qd_linear_i8_geglu_q(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                         const void* bias, int N, int8_t* y8, int ldy8, float* sa8, void* stream);

/* Row-complete LayerNorm epilogue (diffusers BasicTransformerBlock: attn.to_out + residual ->
 * norm2 / norm3): y = the qd_linear_fwd / qd_linear_i8 output with QD_EPI_RESIDUAL (epi must
 * hold it; no amax / GEGLU / GELU-tanh), AND LayerNorm(y) over each row (gamma / beta fp16 [N],
 * eps) in the same launch - one block owns whole rows (N == 320: the 128 x 320 tiles, unsplit), so
 * the LayerNorm reads the final tile from LDS instead of a second pass over y.  ln_y8 == NULL:
 * ln_y [M][N] fp16 = qd_layernorm's value; else ln_y8 [M][N] int8 + ln_sa8 [M] fp32 = qd_layernorm_i8's
 * codes and scales (the consumer linear's per-token operand).  Bit-identical to the unfused
 * qd_linear_fwd / qd_linear_i8 + qd_layernorm(_i8) sequence (same per-lane chunk sums and lane
 * butterfly as the grouped-row LayerNorm).  Returns QD_ERR_ARG for any other N (callers fall back). */
int qd_linear_ln(const void* x, int M, int K, int lda, const void* w, int wfmt, const void* wscale,
                 const void* wscale_t, int group, const void* bias, const void* residual, void* y, int N, int ldy,
                 int epi, const void* ln_gamma, const void* ln_beta, float ln_eps, void* ln_y, int8_t* ln_y8,
                 float* ln_sa8, float* ws, long ws_elems, void* stream);
int qd_linear_i8_ln(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                    const void* bias, const void* residual, void* y, int N, int ldy, int epi, const void* ln_gamma,
                    const void* ln_beta, float ln_eps, void* ln_y, int8_t* ln_y8, float* ln_sa8, void* stream);
/* 1 when qd_linear_ln / qd_linear_i8_ln take this N (a row-complete tile exists), else 0. */
int qd_linear_ln_ok(int N);
/* NHWC implicit-GEMM conv on int8 codes: x_i8 [N, H, W, Ci_pad] (Ci_pad % 64 == 0), one scale
 * per sample sa[N]; w_i8 [Co][kh][kw][Ci_pad], sw[Co]; geometry / epilogue as qd_conv2d_fwd.
 * QD_EPI_CADD: + cadd[n * cadd_ld + co] after the residual (cadd_ld <= 0: Co; 16-B aligned rows).  QD_EPI_GNSTATS:
 * the consumer GroupNorm's slot statistics of the final output into gn_part [N*Ho*Wo / 64][Co]
 * float4 (Ho*Wo % 64 == 0; for qd_groupnorm_part). */
int qd_conv2d_i8(const void* x, const float* sa, int n, int h, int w, int ci, int ci_pad, const void* wt,
                 const float* sw, int co, int kh, int kw, int stride, int pad, int upsample2x, const void* bias,
                 const void* residual, void* y, int epi, float* amax, const void* cadd, int cadd_ld,
                 float* gn_part, float* ws, long ws_elems, void* stream);
/* fp32 elements of split-K workspace qd_linear_i8 / qd_conv2d_i8 plan for this shape (K = codes
 * per row; conv: M = N*Ho*Wo, K = kh*kw*Ci_pad, rows_per_sample = Ho*Wo). */
long qd_gemm_i8_workspace(int M, int N, int K, int rows_per_sample, int epi);
/* qd_groupnorm / qd_groupnorm_fq_in whose output is written as the int8 codes of the conv that
 * consumes it (one scale per sample, scales[n] fp32) instead of fp16: the fp16 GroupNorm(+SiLU)
 * value is formed exactly as qd_groupnorm does, then coded (= qd_quant_samples_i8 of it) in the
 * same pass.  x2 (concat) and in_amax / cadd (virtual finalized input) as the fp16 entry points;
 * ws: qd_groupnorm_workspace(). */
int qd_groupnorm_i8(const void* x, const void* x2, int c1, const float* in_amax, int in_bits, const void* cadd,
                    int cadd_ld, int n, int hw, int c, int groups, float eps, const void* gamma, const void* beta,
                    int silu, int8_t* y8, float* scales, float* ws, void* stream);
/* GroupNorm(+SiLU) of x [N, hw, C] (fp16 NHWC) from the slot statistics its producer wrote
 * (qd_conv2d_i8 with QD_EPI_GNSTATS: part [N * hw / 64][C] float4, hw % 64 == 0): no statistics
 * pass.  x2 (optional): the input is the channel concat x [.., c1] | x2 [.., c - c1] (the UNet
 * skip concat, never materialised), part2 the second source's slot statistics.  y8 + scales:
 * int8 codes, one scale per sample (as qd_groupnorm_i8); else fp16 y.  xamax (int8 output only,
 * optional): the per-(n, c) max |input| [N][C] (for qd_quant_samples_i8_cat).
 * ws: qd_groupnorm_workspace(). */
int qd_groupnorm_part(const float* part, const void* x, const float* part2, const void* x2, int c1, int n, int hw,
                      int c, int groups, float eps, const void* gamma, const void* beta, int silu, void* y,
                      int8_t* y8, float* scales, float* xamax, float* ws, void* stream);
/* Per-sample int8 codes (qd_quant_samples_i8 semantics) of the channel concat x [N, rows, c1] |
 * x2 [N, rows, c - c1] written to y [N, rows, c], the sample scale from the per-(n, c) maxima
 * amax_nc [N][C] (e.g. qd_groupnorm_part's xamax): no concat copy, no amax pass. */
int qd_quant_samples_i8_cat(const void* x, const void* x2, int c1, int c, int n, long rows, const float* amax_nc,
                            int8_t* y, float* scales, void* stream);
/* qd_layernorm with per-row int8 output (= qd_quant_rows_i8 of the fp16 LayerNorm output). */
int qd_layernorm_i8(const void* x, int rows, int c, float eps, const void* gamma, const void* beta, int8_t* y8,
                    float* scales, void* stream);

/* ---------------- normalisation / activations (diffusers UNet ops, fp16 I/O) --------- */
/* GroupNorm(groups, eps, affine) on NHWC [N, HW, C] (+ SiLU) (+ per-(n, c) fake-quant of the
 * result with q_bits, i.e. the input quant of the conv that consumes it, fused because a
 * per-(n, c) amax is reduced deterministically across the slab's row chunks).  x may be two
 * tensors concatenated along C: x2 != NULL -> channels [0, c1) from x (row stride c1), [c1, c)
 * from x2 (row stride c - c1); c1 and c multiples of 8.  ws: qd_groupnorm_workspace() fp32. */
int qd_groupnorm(const void* x, const void* x2, int c1, int n, int hw, int c, int groups,
                 float eps, const void* gamma, const void* beta, int silu, int q_bits,
                 void* y, float* ws, void* stream);
/* qd_groupnorm (q_bits > 0) that also writes xamax [n*c] = max |x| per (sample, channel) of the
 * input x | x2 (from the statistics pass's channel extremes; exact): the up blocks' skip-concat
 * shortcut quant then needs no column-max pass of its own (qd_act_apply_cat_nhwc). */
int qd_groupnorm_xamax(const void* x, const void* x2, int c1, int n, int hw, int c, int groups,
                       float eps, const void* gamma, const void* beta, int silu, int q_bits,
                       void* y, float* xamax, float* ws, void* stream);
/* qd_groupnorm on the finalized output of the conv that feeds it, recomputed on the fly from
 * the raw conv output y_raw [N, HW, C]: x = half(fq(y_raw; in_amax[n][c], in_bits) + cadd[n][c])
 * (in_bits 0: no quantization; cadd [N][cadd_ld] may be NULL) - the q_y = output_quant(y) of
 * fake_quant.py:340 and the diffusers time-embedding add of ResnetBlock2D, without writing
 * that tensor (qd_fq_finalize semantics). */
int qd_groupnorm_fq_in(const void* y_raw, const float* in_amax, int in_bits, const void* cadd, int cadd_ld,
                       int n, int hw, int c, int groups, float eps, const void* gamma, const void* beta,
                       int silu, int q_bits, void* y, float* ws, void* stream);
/* GroupNorm (+SiLU)(+output fake-quant) of x = half(fq(y_raw; in_amax, in_bits) + residual) (or
 * + cadd[n * cadd_ld + c], the time-embedding add) - a conv output whose output quant
 * (fake_quant.py:340) and add are pending - whose statistics pass also writes x to x_out (the
 * block output the later consumers read; for conv1 -> norm2 a scratch the apply pass re-reads
 * instead of recomputing the fake-quant), so the separate finalize pass disappears.  x_out must
 * not alias y_raw / residual; residual and cadd are exclusive. */
int qd_groupnorm_fin(const void* y_raw, const float* in_amax, int in_bits, const void* residual, const void* cadd,
                     int cadd_ld, void* x_out, int n, int hw, int c, int groups, float eps, const void* gamma,
                     const void* beta, int silu, int q_bits, void* y, float* ws, void* stream);
/* fp32 elements of the qd_groupnorm workspace for this shape. */
int qd_groupnorm_workspace(int n, int hw, int c, int groups);
/* LayerNorm over the last dim C of [rows, C]. */
int qd_layernorm(const void* x, int rows, int c, float eps, const void* gamma, const void* beta,
                 void* y, void* stream);
/* LayerNorm of a conv output whose per-(sample, channel) output fake-quant is pending
 * (Transformer2DModel proj_in -> BasicTransformerBlock norm1): t_out = fq(x; amax[n][c], n_bits)
 * (qd_fq_finalize arithmetic, the block's residual stream) and y = LayerNorm(t_out) in one pass.
 * rows_per_sample % 4 == 0 (row r belongs to sample r / rows_per_sample); C <= 2048. */
int qd_layernorm_fq(const void* x, const float* amax, int n_bits, int rows, int rows_per_sample, int c,
                    float eps, const void* gamma, const void* beta, void* t_out, void* y, void* stream);
/* GEGLU (diffusers): h[M, 2I] -> out[M, I] = h[:, :I] * gelu(h[:, I:]). */
int qd_geglu(const void* h, int m, int inner, void* out, void* stream);
/* out = silu(x) elementwise (count elements). */
int qd_silu(const void* x, void* y, int64_t count, void* stream);
/* out = a + b (fp16) */
int qd_add(const void* a, const void* b, void* y, int64_t count, void* stream);
/* NHWC channel concat: out[M, c1+c2] = [a | b] */
int qd_concat_c(const void* a, int c1, const void* b, int c2, int64_t m, void* out, void* stream);
/* layout transposes for the drop-in NCHW modules */
int qd_nchw_to_nhwc(const void* x, int n, int c, int hw, int c_pad, void* y, void* stream);
int qd_nhwc_to_nchw(const void* x, int n, int c, int hw, int c_pad, void* y, void* stream);

/* ---------------- attention ----------------------------------------------------------- */
/* softmax(Q K^T * scale) V per (batch, head); Q [B, Sq, ldq] with head h at columns
 * [h*D, h*D + D), same for K/V/O.  The SDPA of diffusers AttnProcessor2_0 (fp16 I/O, fp32
 * softmax/accumulation). */
int qd_attention(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                 int ldo, int b, int heads, int sq, int skv, int d, float scale, void* stream);
/* head_dim d: a multiple of 8 up to 512 (d > 256: the VAE mid block's single 512-wide head).
 * Causal self-attention (transformers CLIPAttention with the causal mask; sq == skv == s):
 * query i attends keys 0..i. */
int qd_attention_causal(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                        int ldo, int b, int heads, int s, int d, float scale, void* stream);

/* ---------------- time embedding / scheduler ---------------------------------------- */
/* diffusers Timesteps(dim, flip_sin_to_cos, downscale_freq_shift) on timesteps[step_idx[0]]
 * for b rows: out[b, dim] fp16. `timesteps` fp32 device array, `step_idx` int32 device scalar.
 * flip_sin_to_cos | 2: row r embeds timesteps[r] instead (SDXL add_time_proj of the time_ids). */
int qd_timestep_embedding(const float* timesteps, const int* step_idx, int b, int dim,
                          int flip_sin_to_cos, float shift, void* out, void* stream);
/* CFG + DDIM step (eta = 0) on fp16 latents [B, L]: eps = u + g*(c - u) from the UNet output
 * [2B, L] (uncond first), x_{t-1} = sqrt(a_prev) * x0 + sqrt(1 - a_prev) * eps,
 * x0 = (x - sqrt(1-a_t) eps)/sqrt(a_t).  alphas: fp32 [steps] a_t, [steps] a_prev; the
 * step index is read from and then incremented in `step_idx` (graph-replayable).
 * Also writes the next UNet input [2B, L] (latents duplicated, NHWC with c_pad channels). */
int qd_cfg_ddim_step(void* latents, const void* unet_out, int b, int64_t l, float guidance,
                     const float* alpha_t, const float* alpha_prev, int* step_idx,
                     void* next_in, int c, int c_pad, void* stream);
/* CFG + PNDMScheduler.step with skip_prk_steps (PLMS; SD1.5's own scheduler_config) on fp16
 * latents [B, L]: the linear multistep of the last <= 4 noise predictions (device ring `ets`,
 * 4 * B * L fp16) and the step-1 re-evaluation (`cur`, B * L fp16), then
 * prev = sqrt(a_prev / a_t) x - (a_prev - a_t) eps' / (a_t sqrt(1 - a_prev) + sqrt(a_t (1 - a_t) a_prev)).
 * alpha_t / alpha_prev: fp32 [steps + 1] host tables (scheduler.pndm_tables); step index read
 * from and incremented in `step_idx`; next_in as qd_cfg_ddim_step. */
int qd_cfg_pndm_step(void* latents, const void* unet_out, int b, int64_t l, float guidance, const float* alpha_t,
                     const float* alpha_prev, int* step_idx, void* ets, void* cur, void* next_in, int c, int c_pad,
                     void* stream);
/* CFG + EulerDiscreteScheduler.step (epsilon, s_churn 0; the SDXL pipeline's scheduler) on fp16
 * latents [B, L]: sample in fp32, x0 = x - sigma*eps, x += (x - x0)/sigma * (sigma_next - sigma);
 * writes the next UNet input [2B, L] = latents / dscale[i + 1] (scale_model_input).  sigmas,
 * dscale fp32 [steps + 1]; step index read from and incremented in `step_idx`. */
int qd_cfg_euler_discrete_step(void* latents, const void* unet_out, int b, int64_t l, float guidance,
                               const float* sigmas, const float* dscale, int* step_idx, void* next_in, int c,
                               int c_pad, void* stream);
/* latents = half(latents * mul); next_in[0..n) = next_in[n..2n) = half(latents / div) when
 * next_in != NULL (EulerDiscrete init_noise_sigma scaling + the first scale_model_input). */
int qd_scale_latents(void* latents, int64_t n, float mul, float div, void* next_in, int c, int c_pad,
                     void* stream);

/* ---------------- fp8 (e4m3) activations: SD3.5's W4A8-fp8 mode ------------------------
 * (quantize(..., fp8_act=True) with a 4-bit, group-128 config: BASELINE config C5's "fp8
 * activations on CDNA4"; the reference has no fp8 path - stated-tolerance parity)
 * Per-token activation codes: s[r] = max(amax_r, 1e-5) / 448 (f32), y = e4m3(x / s) (RNE). */
int qd_quant_rows_fp8(const void* x, long rows, int c, int ldx, void* y, int ldy, float* scales, void* stream);
/* W4 codes (int8 [N, K], -8..7) -> e4m3 bytes w8 [N, K] (exact), group scales fp16 [N, K/group] ->
 * fp32 gs [K/group][N] (transposed for the GEMM's per-stage scale row). */
int qd_fp8_weight(const int8_t* codes, const void* scales, int n, int k, int group, void* w8, float* gs,
                  void* stream);
/* y[M, N] = half(sa[m] * sum_g gs[g][n] * (x8[m, g] . w8[n, g]) + bias) [GELU-tanh] [+ residual]:
 * x8 e4m3 [M, lda], w8 e4m3 [N, K], K % 128 == 0 (one 128-code group per
 * v_mfma_scale_f32_16x16x128_f8f6f4), epi: QD_EPI_BIAS | QD_EPI_RESIDUAL | QD_EPI_GELU_TANH. */
int qd_linear_fp8(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* gs,
                  const void* bias, const void* residual, void* y, int N, int ldy, int epi, void* stream);

/* ---------------- text encoder (CLIP) / VAE decoder ---------------------------------- */
/* The models around the denoising loop: the reference's pipelines call them through diffusers
 * (models/StableDiffusion1_x.py:19-33 component discovery; base.py:848 pipeline call, whose
 * output_type decides whether the VAE decodes; quantTextEncoder / quantVAE (decoder only,
 * StableDiffusion1_x.py:58-67) swap their layers like the UNet's).
 * out[r, :] = half(tok[ids[r], :] + pos[r % seq, :]) - CLIPTextEmbeddings (ids int64 device,
 * range-checked by the caller; c % 8 == 0). */
int qd_embed_tokens(const int64_t* ids, int64_t rows, int seq, const void* tok, int64_t vocab, const void* pos,
                    int c, void* out, void* stream);
/* CLIP MLP activation, elementwise: kind 0 quick_gelu = x * sigmoid(1.702 x) (three fp16
 * roundings, as the Half ops), kind 1 exact-erf gelu. */
int qd_clip_act(const void* x, void* y, int64_t count, int kind, void* stream);
/* y[i, :] = x[idx[i], :] (rows of c fp16, row stride ldx; idx int64 device) - pooled EOS rows. */
int qd_gather_rows(const void* x, int64_t ldx, int64_t rows_x, const int64_t* idx, int n, int c, void* y,
                   void* stream);
/* VAE decode input: y = half(x / scale) [then half(y + shift) if has_shift], NHWC latents with c
 * of cin_pad channels -> NHWC with cout_pad channels (the rest zero). */
int qd_vae_prescale(const void* x, int64_t pix, int cin_pad, int c, float scale, float shift, int has_shift,
                    int cout_pad, void* y, void* stream);
/* VaeImageProcessor.postprocess of the decoder output y (NHWC, c of c_pad channels):
 * v = clamp(half(half(y / 2) + 0.5), 0, 1) -> out_nchw fp16 [n, c, h, w] and/or
 * out_u8 [n, h, w, c] = rint(v * 255) (either may be NULL, not both). */
int qd_vae_postprocess(const void* y, int n, int64_t hw, int c_pad, int c, void* out_nchw, void* out_u8,
                       void* stream);

/* ---------------- calibration (SmoothQuant) ------------------------------------------ */
/* Mean_Max_Activation_Hook (utils/calib_data.py:105-124): per-channel max |x| of x[rows, C]
 * for one forward call, accumulated into sum[C] (fp32) for the later mean over calls
 * (StableDiffusion1_x.py:104-112).  amax_out (fp16 [C]) optional: this call's values. */
int qd_channel_absmax_accum(const void* x, int64_t rows, int c, float* amax_ws, float* sum,
                            void* amax_out, void* stream);
/* smooth_ln_fcs scales (quantizer_SQ.py:416-424): s = clamp(a^alpha / w^(1-alpha), 1e-5) in
 * fp16 op order, a = act_mean (fp16 [C]), w = max over the nfc weight matrices [Ni][C] of
 * max_k |W[k][c]| clamp 1e-5.  Applies ln.w /= s, ln.b /= s (ln_b may be NULL),
 * W_i *= s in place.  fc_w / fc_rows are HOST arrays of nfc device pointers / row counts;
 * wmax_ws is an fp32 [C] workspace. */
int qd_smooth_fold(void* ln_w, void* ln_b, void* const* fc_w, const int* fc_rows, int nfc, int c,
                   const void* act_mean, float alpha, float* wmax_ws, void* scales_out,
                   void* stream);

/* ---------------- self-tests (test infrastructure) ---------------------------------- */
/* Exhaustive check of the reciprocal shortcut used by every fake-quant apply kernel against the
 * IEEE-division form (all fp16 scales): counts[0] = reciprocal errors > 1 ulp, counts[1] =
 * differing fake-quant results at the values around every quantization midpoint, counts[2] =
 * differing f16 quotients over every finite fp16 x (device int[3]). */
int qd_selftest_recip(int* counts, void* stream);

/* ---------------- SD3 / SD3.5 MMDiT -------------------------------------------------------
 * The diffusers SD3Transformer2DModel ops the reference runs around its WxAxLinear layers
 * (models/StableDiffusion3_5.py:37-45 hands the transformer to the quantizer swap,
 * quantize/quantizer.py:491-533; the model itself is third-party diffusers code).  fp16 in/out,
 * each torch op computed in fp32 and rounded to fp16 once. */
/* AdaLayerNormZero / AdaLayerNormContinuous apply (LayerNorm without affine, eps):
 * y = half(half(half(LN(x)) * half(1 + scale[b])) + shift[b]), x / y [rows, c],
 * b = row / tokens_per_sample; shift / scale [B, mod_ld] (column slices of the adaLN linear). */
int qd_adaln_modulate(const void* x, long rows, int c, int tokens_per_sample, float eps, const void* shift,
                      const void* scale, int mod_ld, void* y, void* stream);
/* JointTransformerBlock gated residual: out = half(x + half(gate[b] * y)); y row stride y_ld,
 * gate [B, gate_ld], b = row / tokens_per_sample.  out may alias x. */
int qd_gated_residual(const void* x, const void* y, int y_ld, const void* gate, int gate_ld, long rows, int c,
                      int tokens_per_sample, void* out, void* stream);
/* diffusers RMSNorm(head_dim) (Attention.norm_q / norm_k / norm_added_q / norm_added_k), in place
 * over each d-wide head of `rows` rows: half(half(x * rsqrt(mean(x^2) + eps)) * w).  Row r lives
 * at x + ((r / rows_per_group) * group_stride + r % rows_per_group) * ld (rows_per_group <= 0:
 * contiguous rows).  d in {16, 32, 64, 128}. */
int qd_rmsnorm_heads(void* x, long rows, int heads, int d, int ld, long rows_per_group, long group_stride,
                     const void* weight, float eps, void* stream);
/* F.gelu(x, approximate="tanh") (FeedForward activation_fn="gelu-approximate"); n % 8 == 0. */
int qd_gelu_tanh(const void* x, void* y, int64_t n, void* stream);
/* PatchEmbed position add: out[b, s, :] = half(x[b, s, :] + pos[s, :]), pos [s, c] (cropped). */
int qd_add_pos(const void* x, const void* pos, int b, long s, int c, void* out, void* stream);
/* Grouped strided row copy: dst row ((r / rows_per_group) * group_stride + r % rows_per_group)
 * (stride dst_ld) = src row r (stride src_ld), `cols` halves; builds the joint [x; context]
 * q|k|v sequence of JointAttnProcessor2_0 (torch.cat along the sequence). */
int qd_copy_rows(const void* src, int src_ld, void* dst, int dst_ld, long rows, int cols, long rows_per_group,
                 long group_stride, void* stream);
/* SD3Transformer2DModel unpatchify: tokens [B, h*w, p*p*c] -> NHWC [B, h*p, w*p, c]. */
int qd_unpatchify(const void* tokens, int b, int h, int w, int p, int c, void* out, void* stream);
/* CFG + FlowMatchEulerDiscreteScheduler.step on fp16 latents [B, L]: v = u + g*(c - u) from the
 * model output [2B, L] (uncond first), x += (sigma[i+1] - sigma[i]) * v with sample.to(float32)
 * semantics; sigmas fp32 [steps + 1]; i read from and then incremented in `step_idx`.  Also
 * writes the next model input [2B, L] (latents duplicated) when next_in != NULL. */
int qd_cfg_euler_step(void* latents, const void* model_out, int b, int64_t l, float guidance, const float* sigmas,
                      int* step_idx, void* next_in, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QDIFF_H */
