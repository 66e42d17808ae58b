// SD3 / SD3.5 MMDiT ops (diffusers SD3Transformer2DModel / JointTransformerBlock, restated; the
// reference runs them through the third-party diffusers model with WxAxLinear swapped in, see
// models/StableDiffusion3_5.py:37-45, quantize/quantizer.py:491-533), fp16 I/O with fp16
// op-boundary rounding (each torch op computed in fp32, rounded to fp16 once):
//   k_adaln         AdaLayerNormZero / AdaLayerNormContinuous apply:
//                   y = half(half(half(LN(x)) * half(1 + scale[b])) + shift[b])
//   k_gated_add     x + gate * y  (the gate_msa / gate_mlp residuals): half(x + half(g * y))
//   k_rmsnorm_heads diffusers RMSNorm(head_dim) on q / k in place: half(half(x * rsqrt(mean x^2 + eps)) * w)
//   k_gelu_tanh     F.gelu(approximate="tanh") (FeedForward "gelu-approximate")
//   k_add_pos       PatchEmbed: half(tokens + pos[s])
//   k_copy_rows     grouped strided row copy (stream outputs into the joint q|k|v buffer)
//   k_unpatchify    tokens [B, h*w, p*p*C] -> NHWC latents [B, h*p, w*p, C]
//   k_cfg_euler     CFG combine + FlowMatchEulerDiscreteScheduler.step
#include "common.h"

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
static int grid1(long count, int per_block = 256) { return (int)((count + per_block - 1) / per_block); }

// row r of a grouped row set: groups of `rpg` consecutive rows, group g starting at row g * gstride
static __device__ __forceinline__ long grouped_row(long r, long rpg, long gstride) {
  const long g = r / rpg;
  return g * gstride + (r - g * rpg);
}

// ---------------------------------------------------------------------------------------
// LayerNorm (no affine, eps) + modulation; one wave per row, lane owns 8-channel chunks.
// shift / scale: [B][mod_ld] (column slices of the adaLN projection output), b = row / tps.
template <int PER>
__global__ void __launch_bounds__(256) k_adaln(const f16* __restrict__ x, long rows, int c, int tps, float eps,
                                               const f16* __restrict__ shift, const f16* __restrict__ scale,
                                               int mod_ld, f16* __restrict__ y) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int chunks = c >> 3;
  const long b = row / tps;
  f16x8 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + i * 64;
    v[i] = *reinterpret_cast<const f16x8*>(x + row * c + (j < chunks ? j : 0) * 8);
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) QD_PIN(v[i]);
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (lane + i * 64 >= chunks) v[i] = (f16x8){};
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)v[i][e];
  const float mean = wave_sum(s) / (float)c;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
    if (lane + i * 64 < chunks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = (float)v[i][e] - mean;
        q = fmaf(a, a, q);
      }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)c + eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + i * 64;
    if (j < chunks) {
      const f16x8 sh = *reinterpret_cast<const f16x8*>(shift + b * mod_ld + j * 8);
      const f16x8 sc = *reinterpret_cast<const f16x8*>(scale + b * mod_ld + j * 8);
      f16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const f16 h = (f16)(((float)v[i][e] - mean) * rstd);
        const f16 one_sc = (f16)(1.0f + (float)sc[e]);
        const f16 m = (f16)((float)h * (float)one_sc);
        o[e] = (f16)((float)m + (float)sh[e]);
      }
      *reinterpret_cast<f16x8*>(y + row * c + j * 8) = o;
    }
  }
}

extern "C" int qd_adaln_modulate(const void* x, long rows, int c, int tokens_per_sample, float eps,
                                 const void* shift, const void* scale, int mod_ld, void* y, void* stream) {
  QD_REQUIRE(x && shift && scale && y, "null pointer");
  QD_REQUIRE(c % 8 == 0 && c > 0 && c <= 8192 && mod_ld % 8 == 0 && tokens_per_sample > 0, "bad adaLN shape");
  if (rows == 0) return 0;
  const int per = (c / 8 + 63) / 64;
  const dim3 g(grid1(rows, 4));
  hipStream_t st = S(stream);
#define QD_ADALN(P)                                                                                          \
  k_adaln<P><<<g, 256, 0, st>>>((const f16*)x, rows, c, tokens_per_sample, eps, (const f16*)shift,           \
                                (const f16*)scale, mod_ld, (f16*)y)
  if (per <= 1) QD_ADALN(1);
  else if (per <= 2) QD_ADALN(2);
  else if (per <= 4) QD_ADALN(4);
  else if (per <= 8) QD_ADALN(8);
  else QD_ADALN(16);
#undef QD_ADALN
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
__global__ void k_gated_add(const f16* __restrict__ x, const f16* __restrict__ yv, int y_ld,
                            const f16* __restrict__ gate, int gate_ld, long rows, int c, int tps,
                            f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // 8-channel chunk index
  const int cc = c >> 3;
  if (e >= rows * cc) return;
  const long row = e / cc;
  const int ch = (int)(e - row * cc) * 8;
  const f16x8 a = *reinterpret_cast<const f16x8*>(x + row * c + ch);
  const f16x8 b = *reinterpret_cast<const f16x8*>(yv + row * y_ld + ch);
  const f16x8 g = *reinterpret_cast<const f16x8*>(gate + (row / tps) * gate_ld + ch);
  f16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (f16)((float)a[j] + (float)(f16)((float)g[j] * (float)b[j]));
  *reinterpret_cast<f16x8*>(out + row * c + ch) = o;
}

extern "C" int qd_gated_residual(const void* x, const void* y, int y_ld, const void* gate, int gate_ld, long rows,
                                 int c, int tokens_per_sample, void* out, void* stream) {
  QD_REQUIRE(x && y && gate && out, "null pointer");
  if (y_ld <= 0) y_ld = c;
  QD_REQUIRE(c % 8 == 0 && gate_ld % 8 == 0 && y_ld % 8 == 0 && tokens_per_sample > 0, "bad gated residual shape");
  if (rows == 0) return 0;
  k_gated_add<<<grid1(rows * (c / 8)), 256, 0, S(stream)>>>((const f16*)x, (const f16*)y, y_ld, (const f16*)gate,
                                                            gate_ld, rows, c, tokens_per_sample, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// RMSNorm over each head (in place): one 8-channel chunk per lane, a head = D/8 consecutive lanes
// (reduction by shuffles within the group).  Row r lives at grouped_row(r, rpg, gstride) * ld.
template <int D>
__global__ void __launch_bounds__(256) k_rmsnorm_heads(f16* __restrict__ x, long rows, int heads, int ld, long rpg,
                                                       long gstride, const f16* __restrict__ w, float eps) {
  constexpr int G = D / 8;  // lanes per head
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = rows * heads * G;
  const bool ok = e < total;
  const long eh = ok ? e : total - 1;
  const long rh = eh / G;
  const int lg = (int)(eh - rh * G);
  const long row = rh / heads;
  const int h = (int)(rh - row * heads);
  f16* p = x + grouped_row(row, rpg, gstride) * ld + h * D + lg * 8;
  const f16x8 v = *reinterpret_cast<const f16x8*>(p);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s = fmaf((float)v[j], (float)v[j], s);
#pragma unroll
  for (int o = 1; o < G; o <<= 1) s += __shfl_xor(s, o, 64);
  const float rs = 1.0f / sqrtf(s / (float)D + eps);
  const f16x8 wv = *reinterpret_cast<const f16x8*>(w + lg * 8);
  f16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = (f16)((float)(f16)((float)v[j] * rs) * (float)wv[j]);
  if (ok) *reinterpret_cast<f16x8*>(p) = out;
}

extern "C" int qd_rmsnorm_heads(void* x, long rows, int heads, int d, int ld, long rows_per_group,
                                long group_stride, const void* weight, float eps, void* stream) {
  QD_REQUIRE(x && weight, "null pointer");
  QD_REQUIRE(ld % 8 == 0 && ld >= heads * d, "bad leading dim");
  if (rows_per_group <= 0) {
    rows_per_group = rows > 0 ? rows : 1;
    group_stride = rows_per_group;
  }
  QD_REQUIRE(group_stride >= rows_per_group, "bad row grouping");
  if (rows * heads == 0) return 0;
  hipStream_t st = S(stream);
  const long threads = rows * heads * (d / 8);
  const dim3 g(grid1(threads));
#define QD_RMS(DD)                                                                                           \
  k_rmsnorm_heads<DD><<<g, 256, 0, st>>>((f16*)x, rows, heads, ld, rows_per_group, group_stride,            \
                                         (const f16*)weight, eps)
  switch (d) {
    case 16: QD_RMS(16); break;
    case 32: QD_RMS(32); break;
    case 64: QD_RMS(64); break;
    case 128: QD_RMS(128); break;
    default: return qd_set_error(QD_ERR_ARG, "rmsnorm_heads: head_dim must be 16, 32, 64 or 128");
  }
#undef QD_RMS
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// torch gelu(approximate="tanh"): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))) (common.h)
__global__ void k_gelu_tanh(const f16* __restrict__ x, f16* __restrict__ y, long n8) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n8) return;
  const f16x8 v = reinterpret_cast<const f16x8*>(x)[e];
  f16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (f16)gelu_tanh_f((float)v[j]);
  reinterpret_cast<f16x8*>(y)[e] = o;
}

extern "C" int qd_gelu_tanh(const void* x, void* y, int64_t n, void* stream) {
  QD_REQUIRE(x && y && n % 8 == 0, "gelu_tanh: n must be a multiple of 8");
  if (n == 0) return 0;
  k_gelu_tanh<<<grid1(n / 8), 256, 0, S(stream)>>>((const f16*)x, (f16*)y, n / 8);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
__global__ void k_add_pos(const f16* __restrict__ x, const f16* __restrict__ pos, long total_chunks, long s_c,
                          f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= total_chunks) return;
  const long off = e * 8;
  const f16x8 a = *reinterpret_cast<const f16x8*>(x + off);
  const f16x8 p = *reinterpret_cast<const f16x8*>(pos + off % s_c);
  f16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (f16)((float)a[j] + (float)p[j]);
  *reinterpret_cast<f16x8*>(out + off) = o;
}

extern "C" int qd_add_pos(const void* x, const void* pos, int b, long s, int c, void* out, void* stream) {
  QD_REQUIRE(x && pos && out && c % 8 == 0, "bad args");
  const long chunks = (long)b * s * c / 8;
  if (chunks == 0) return 0;
  k_add_pos<<<grid1(chunks), 256, 0, S(stream)>>>((const f16*)x, (const f16*)pos, chunks, s * c, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// dst[grouped_row(r) * dst_ld + c] = src[r * src_ld + c] for c < cols (16-B chunks)
__global__ void k_copy_rows(const f16* __restrict__ src, int src_ld, f16* __restrict__ dst, int dst_ld, long rows,
                            int cols, long rpg, long gstride) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const int cc = cols >> 3;
  if (e >= rows * cc) return;
  const long r = e / cc;
  const int c = (int)(e - r * cc) * 8;
  *reinterpret_cast<f16x8*>(dst + grouped_row(r, rpg, gstride) * dst_ld + c) =
      *reinterpret_cast<const f16x8*>(src + r * src_ld + c);
}

extern "C" int qd_copy_rows(const void* src, int src_ld, void* dst, int dst_ld, long rows, int cols,
                            long rows_per_group, long group_stride, void* stream) {
  QD_REQUIRE(src && dst && cols % 8 == 0 && src_ld % 8 == 0 && dst_ld % 8 == 0, "bad copy_rows args");
  if (rows_per_group <= 0) {
    rows_per_group = rows > 0 ? rows : 1;
    group_stride = rows_per_group;
  }
  QD_REQUIRE(group_stride >= rows_per_group, "bad row grouping");
  if (rows * cols == 0) return 0;
  k_copy_rows<<<grid1(rows * (cols / 8)), 256, 0, S(stream)>>>((const f16*)src, src_ld, (f16*)dst, dst_ld, rows,
                                                               cols, rows_per_group, group_stride);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// tokens [B][h*w][p*p*C] (feature (pi*p + qi)*C + ch) -> NHWC [B][h*p][w*p][C]
// (diffusers: reshape(B, h, w, p, p, C) -> einsum "nhwpqc->nchpwq")
__global__ void k_unpatchify(const f16* __restrict__ t, int h, int w, int p, int c, long total,
                             f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // over output elements
  if (e >= total) return;
  const int ch = (int)(e % c);
  long r = e / c;
  const int X = (int)(r % (w * p));
  r /= (w * p);
  const int Y = (int)(r % (h * p));
  const long n = r / (h * p);
  const int hi = Y / p, pi = Y - hi * p, wi = X / p, qi = X - wi * p;
  out[e] = t[((n * h + hi) * w + wi) * (long)(p * p * c) + (pi * p + qi) * c + ch];
}

extern "C" int qd_unpatchify(const void* tokens, int b, int h, int w, int p, int c, void* out, void* stream) {
  QD_REQUIRE(tokens && out && p > 0 && c > 0, "bad args");
  const long total = (long)b * h * p * w * p * c;
  if (total == 0) return 0;
  k_unpatchify<<<grid1(total), 256, 0, S(stream)>>>((const f16*)tokens, h, w, p, c, total, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// CFG + FlowMatchEulerDiscreteScheduler.step (diffusers op order, torch Half semantics as the
// oracle evaluates them):
//   v    = u + g * (c - u)                     (fp16 ops; g a python float)
//   dsig = sigma[i + 1] - sigma[i]             (fp32 0-d tensor; a 0-d tensor times a half tensor
//                                               is rounded to half first, as in k_cfg_ddim)
//   prev = half(float(x) + float(half(half(dsig) * v)))   (sample.to(float32) + the fp16 product)
// latents [B, L]; model output [2B, L] (uncond first); next_in = [prev; prev].
__global__ void k_cfg_euler(f16* __restrict__ lat, const f16* __restrict__ mo, int b, long l, float g,
                            const float* __restrict__ sig, const int* __restrict__ step_idx,
                            f16* __restrict__ next_in) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)b * l) return;
  const int si = step_idx[0];
  const long bi = e / l, off = e - bi * l;
  const float u = (float)mo[bi * l + off];
  const float cc = (float)mo[((long)b + bi) * l + off];
  const f16 diff = (f16)(cc - u);
  const f16 gd = (f16)(g * (float)diff);
  const f16 v = (f16)(u + (float)gd);
  const float dsig = (float)(f16)(sig[si + 1] - sig[si]);
  const f16 t = (f16)(dsig * (float)v);
  const f16 out = (f16)((float)lat[e] + (float)t);
  lat[e] = out;
  if (next_in) {
    next_in[e] = out;
    next_in[(long)b * l + e] = out;
  }
}

__global__ void k_euler_step_inc(int* step_idx) {
  if (threadIdx.x == 0) step_idx[0] += 1;
}

extern "C" int qd_cfg_euler_step(void* latents, const void* model_out, int b, int64_t l, float guidance,
                                 const float* sigmas, int* step_idx, void* next_in, void* stream) {
  QD_REQUIRE(latents && model_out && sigmas && step_idx, "null pointer");
  hipStream_t st = S(stream);
  if ((long)b * l > 0)
    k_cfg_euler<<<grid1((long)b * l), 256, 0, st>>>((f16*)latents, (const f16*)model_out, b, l, guidance, sigmas,
                                                    step_idx, (f16*)next_in);
  k_euler_step_inc<<<1, 64, 0, st>>>(step_idx);
  QD_CHECK_LAUNCH();
  return 0;
}
