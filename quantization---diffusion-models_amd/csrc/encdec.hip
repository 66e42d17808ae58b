// Text encoder (CLIP) and VAE decoder ops around the denoising loop: token + position
// embedding gather, the CLIP MLP activations, row gather (pooled EOS token), and the VAE's
// latent rescale in / image postprocess out.  Everything else the two models run (LayerNorm,
// GroupNorm+SiLU, linears, implicit-GEMM convs with fused nearest upsampling, attention - causal
// for CLIP, one 512-wide head for the VAE mid block) is the UNet's kernels.
// All fp16 ops follow torch-CPU Half semantics: each op computed in fp32, rounded to fp16 once.
#include "common.h"

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
static int grid1(long count, int per_block = 256) { return (int)((count + per_block - 1) / per_block); }

// transformers CLIPTextEmbeddings.forward: token_embedding(input_ids) + position_embedding(
// position_ids), an fp16 + fp16 add.  8 channels per thread.  Ids were range-checked on the host;
// the clamp only keeps a bad id from reading outside the table.
__global__ void k_embed_tokens(const int64_t* __restrict__ ids, long rows, int seq, const f16* __restrict__ tok,
                               const f16* __restrict__ pos, int c, long vocab, f16* __restrict__ out) {
  const int per_row = c >> 3;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * per_row) return;
  const long r = e / per_row;
  const int c8 = (int)(e - r * per_row) * 8;
  long id = ids[r];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const f16x8 a = *reinterpret_cast<const f16x8*>(tok + id * c + c8);
  const f16x8 b = *reinterpret_cast<const f16x8*>(pos + (long)(r % seq) * c + c8);
  f16x8 y;
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = (f16)((float)a[j] + (float)b[j]);
  *reinterpret_cast<f16x8*>(out + r * c + c8) = y;
}

extern "C" int qd_embed_tokens(const int64_t* ids, int64_t rows, int seq, const void* tok, int64_t vocab,
                               const void* pos, int c, void* out, void* stream) {
  QD_REQUIRE(ids && tok && pos && out, "null pointer");
  QD_REQUIRE(c % 8 == 0 && c > 0 && seq > 0 && vocab > 0, "embedding width must be a multiple of 8");
  if (rows == 0) return 0;
  k_embed_tokens<<<grid1(rows * (c / 8)), 256, 0, S(stream)>>>(ids, rows, seq, (const f16*)tok, (const f16*)pos,
                                                               c, vocab, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// CLIP MLP activation (transformers ACT2FN):
//   kind 0 "quick_gelu": input * torch.sigmoid(1.702 * input) - three Half ops, three roundings
//     (the sigmoid's exp is libm's on the CPU: results agree within 1 fp16 ulp, almost always exactly)
//   kind 1 "gelu": F.gelu (exact erf), one rounding
__global__ void k_clip_act(const f16* __restrict__ x, f16* __restrict__ y, long count, int kind) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  const float v = (float)x[e];
  if (kind == 0) {
    // the f32 product must round to f32 before the f16 conversion (the CPU's two roundings):
    // without the barrier the backend folds mul + cvt into one mixed-precision v_fma_mix with a
    // single rounding, which differs on f32 ties (1 fp16 ulp of t, ~0.4 % of the sigmoid)
    float p = 1.702f * v;
    asm volatile("" : "+v"(p));
    const float t = (float)(f16)p;
    // sigmoid in f64, rounded to f32 then f16: the correctly rounded value the CPU's f32
    // 1 / (1 + exp(-t)) lands on except within an ulp of an fp16 rounding boundary
    const float s = (float)(f16)(float)(1.0 / (1.0 + exp(-(double)t)));
    y[e] = (f16)(v * s);
  } else {
    y[e] = (f16)gelu_f(v);
  }
}

extern "C" int qd_clip_act(const void* x, void* y, int64_t count, int kind, void* stream) {
  QD_REQUIRE(x && y, "null pointer");
  QD_REQUIRE(kind == 0 || kind == 1, "kind: 0 quick_gelu, 1 gelu");
  if (count == 0) return 0;
  k_clip_act<<<grid1(count), 256, 0, S(stream)>>>((const f16*)x, (f16*)y, count, kind);
  QD_CHECK_LAUNCH();
  return 0;
}

// y[i] = x[idx[i]] for rows of c fp16 (the pooled EOS row of every prompt).
__global__ void k_gather_rows(const f16* __restrict__ x, long ldx, const int64_t* __restrict__ idx, int n, int c,
                              long rows_x, f16* __restrict__ y) {
  const int per_row = c >> 3;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)n * per_row) return;
  const int i = (int)(e / per_row), c8 = (int)(e % per_row) * 8;
  long r = idx[i];
  r = r < 0 ? 0 : (r >= rows_x ? rows_x - 1 : r);
  *reinterpret_cast<f16x8*>(y + (long)i * c + c8) = *reinterpret_cast<const f16x8*>(x + r * ldx + c8);
}

extern "C" int qd_gather_rows(const void* x, int64_t ldx, int64_t rows_x, const int64_t* idx, int n, int c, void* y,
                              void* stream) {
  QD_REQUIRE(x && idx && y, "null pointer");
  QD_REQUIRE(c % 8 == 0 && ldx % 8 == 0 && ldx >= c, "row width / stride must be multiples of 8");
  if (n == 0) return 0;
  k_gather_rows<<<grid1((long)n * (c / 8)), 256, 0, S(stream)>>>((const f16*)x, ldx, idx, n, c, rows_x, (f16*)y);
  QD_CHECK_LAUNCH();
  return 0;
}

// VAE decode input (the pipelines' `latents / vae.config.scaling_factor` [`+ shift_factor`, SD3]):
// NHWC latents with c valid of cin_pad channels -> NHWC [.., cout_pad], channels >= c zero.
__global__ void k_vae_prescale(const f16* __restrict__ x, long pix, int cin_pad, int c, float scale, float shift,
                               int has_shift, int cout_pad, f16* __restrict__ y) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= pix * cout_pad) return;
  const long p = e / cout_pad;
  const int ch = (int)(e - p * cout_pad);
  float v = 0.f;
  if (ch < c) {
    v = (float)(f16)((float)x[p * cin_pad + ch] / scale);
    if (has_shift) {
      // torch casts a Python-number addend to the tensor's dtype (div keeps the f32 scalar):
      // half(shift), then the f32 sum rounded once (the barrier keeps it from folding, see k_clip_act)
      float t = v + (float)(f16)shift;
      asm volatile("" : "+v"(t));
      v = (float)(f16)t;
    }
  }
  y[e] = (f16)v;
}

extern "C" int qd_vae_prescale(const void* x, int64_t pix, int cin_pad, int c, float scale, float shift, int has_shift,
                               int cout_pad, void* y, void* stream) {
  QD_REQUIRE(x && y, "null pointer");
  QD_REQUIRE(c > 0 && c <= cin_pad && c <= cout_pad && scale != 0.f, "bad channel counts / scale");
  if (pix == 0) return 0;
  k_vae_prescale<<<grid1(pix * cout_pad), 256, 0, S(stream)>>>((const f16*)x, pix, cin_pad, c, scale, shift, has_shift,
                                                              cout_pad, (f16*)y);
  QD_CHECK_LAUNCH();
  return 0;
}

// VaeImageProcessor.postprocess: denormalize (image / 2 + 0.5).clamp(0, 1) as Half ops ->
// out_nchw fp16 [n, c, h, w] ("pt"), and/or out_u8 [n, h, w, c] = round(float(v) * 255)
// (numpy_to_pil: (images * 255).round().astype("uint8"), float32 with round-half-even).
__global__ void k_vae_postprocess(const f16* __restrict__ y, int n, long hw, int c_pad, int c,
                                  f16* __restrict__ out_nchw, uint8_t* __restrict__ out_u8) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)n * hw * c) return;
  const long p = e / c;               // pixel (n, h, w)
  const int ch = (int)(e - p * c);
  const long b = p / hw, q = p - b * hw;
  float v = (float)(f16)((float)y[p * c_pad + ch] / 2.0f);
  v = (float)(f16)(v + 0.5f);
  v = fminf(fmaxf(v, 0.f), 1.f);
  if (out_nchw) out_nchw[(b * c + ch) * hw + q] = (f16)v;
  if (out_u8) out_u8[e] = (uint8_t)__builtin_rintf(v * 255.0f);
}

extern "C" int qd_vae_postprocess(const void* y, int n, int64_t hw, int c_pad, int c, void* out_nchw, void* out_u8,
                                  void* stream) {
  QD_REQUIRE(y && (out_nchw || out_u8), "null pointer");
  QD_REQUIRE(c > 0 && c <= c_pad, "bad channel counts");
  if ((long)n * hw == 0) return 0;
  k_vae_postprocess<<<grid1((long)n * hw * c), 256, 0, S(stream)>>>((const f16*)y, n, hw, c_pad, c, (f16*)out_nchw,
                                                                   (uint8_t*)out_u8);
  QD_CHECK_LAUNCH();
  return 0;
}
