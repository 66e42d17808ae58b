// UNet elementwise / normalisation kernels (diffusers ops the reference runs in fp16 on CPU):
// GroupNorm(+SiLU)(+fused per-(n,c) act fake-quant), LayerNorm, GEGLU, SiLU, add, channel
// concat, NCHW<->NHWC, Timesteps embedding, CFG + DDIM step.
//
// Op-boundary rounding follows PyTorch-CPU Half: each torch op computes in fp32 and rounds
// its output to fp16 (GroupNorm output, then SiLU output, then the fake-quant chain).
#include "common.h"

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
static int grid1(long count, int per_block = 256) { return (int)((count + per_block - 1) / per_block); }

// ---------------------------------------------------------------------------------------
// GroupNorm on NHWC [N, HW, C] (+ SiLU) (+ fused per-(n,c) fake-quant of the output).
//
// The input is "virtual" (GnIn): either x itself, or x | x2 concatenated along C (the UNet's
// skip concat, never materialised), or the finalized output of the conv that feeds it,
// x = half(fq(y; amax[n][c]) + cadd[n][c]) (fake_quant.py:340 output quant + the diffusers
// time-embedding add), recomputed on the fly from the raw conv output so the finalize pass and
// its tensor never exist (ResnetBlock2D conv1 -> norm2).
//
// Three stream-ordered kernels, all deterministic (fixed-order reductions, max is exact).  The
// two streaming passes share one geometry: block (bx, by), thread (tx, ty) owns the 8-channel
// 16-B chunk blockIdx.x * bx + tx of sample blockIdx.y and rows ty, ty + by, ... of row range
// blockIdx.z: fully coalesced 16-B accesses, per-channel state in registers.
//   1. k_gn_stats   per-channel shifted sums (shift = the group's first element) and min / max
//                   -> LDS reduction over ty -> partial[n][z][c] (s1, s2, min, max)
//   2. k_gn_coeff   per (n, c): group mean / rstd from the partials in fixed order ->
//                   scale = rstd*gamma, bias = beta - scale*mean (torch CPU GroupNorm form);
//                   [q_bits] the exact per-(n,c) amax of the output from the channel's min / max
//                   (monotonicity argument below); the rare channels it cannot bound are
//                   scanned by the same block (the input quant of the consuming conv:
//                   fake_quant.py:125 reduction)
//   3. k_gn_apply   y = fq(silu(half(x*a + b)))
// ---------------------------------------------------------------------------------------
struct GnIn {
  const f16* x;
  const f16* x2;     // channels [c1, c) (row stride c - c1) or null
  int c1;
  const float* amax; // virtual input: per-(n, c) amax of the raw conv output (null: none)
  int qmax;          // ... and its fake-quant qmax (0: no quantization)
  const f16* cadd;   // ... + cadd[n * cadd_ld + c] (null: none)
  int cadd_ld;
  const f16* res;    // ... + res[row][c] (the block's residual; null: none) - XF 2: the statistics
  f16* xout;         // pass writes the finalized input x to xout, which the apply pass then reads
};

// per-channel input transform state of one 8-channel chunk of sample n
struct GnXf {
  float s[8];
  double rs[8];
  float ca[8];
};

__device__ __forceinline__ void gn_xf_init(const GnIn& in, int c, long n, int ch, GnXf& t) {
  if (in.qmax > 0) {
    fq_scales8(in.amax + n * c + ch, in.qmax, t.s, t.rs);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      t.s[j] = 0.f;
      t.rs[j] = 0.0;
    }
  }
  f16x8 ca = {};
  if (in.cadd) ca = *reinterpret_cast<const f16x8*>(in.cadd + n * in.cadd_ld + ch);
#pragma unroll
  for (int j = 0; j < 8; ++j) t.ca[j] = (float)ca[j];
}

// XF: 0 plain source(s); 1 finalize transform (output quant if in.qmax > 0, + cadd if set:
// a zero cadd adds +0, which leaves every fp16 value - including -0 - bit-identical... except
// -0 + +0 = +0; the callers pass cadd only when the reference adds it)
__device__ __forceinline__ f16x8 gn_raw8(const GnIn& in, int c, long row, int ch) {
  const f16* p = ch < in.c1 ? in.x + row * in.c1 + ch : in.x2 + row * (c - in.c1) + (ch - in.c1);
  return *reinterpret_cast<const f16x8*>(p);
}

// XF 2: output quant (if in.qmax) then + the residual row chunk r
__device__ __forceinline__ f16x8 gn_fin8(const GnIn& in, f16x8 v, const GnXf& t, f16x8 r) {
  const bool q = in.qmax > 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f16 o = v[j];
    if (q) o = fq_apply_r((float)o, t.s[j], t.rs[j]);
    v[j] = to_f16((float)o + (float)r[j]);
  }
  return v;
}

template <int XF>
__device__ __forceinline__ f16x8 gn_xf8(const GnIn& in, f16x8 v, const GnXf& t) {
  if constexpr (XF == 1) {
    const bool q = in.qmax > 0, a = in.cadd != nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f16 o = v[j];
      if (q) o = fq_apply_r((float)o, t.s[j], t.rs[j]);
      if (a) o = to_f16((float)o + t.ca[j]);
      v[j] = o;
    }
  }
  return v;
}

// Compile-time-flag forms of gn_xf8<1> / gn_fin8 for the statistics pass (same operations, so the
// same bits): without the per-element uniform branches on in.qmax / in.cadd the 8 channels'
// conversion chains interleave instead of issuing one dependent chain at a time.
template <bool Q, bool A>
__device__ __forceinline__ f16x8 gn_xf8c(f16x8 v, const GnXf& t) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f16 o = v[j];
    if constexpr (Q) o = fq_apply_r((float)o, t.s[j], t.rs[j]);
    if constexpr (A) o = to_f16((float)o + t.ca[j]);
    v[j] = o;
  }
  return v;
}

template <bool Q>
__device__ __forceinline__ f16x8 gn_fin8c(f16x8 v, const GnXf& t, f16x8 r) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f16 o = v[j];
    if constexpr (Q) o = fq_apply_r((float)o, t.s[j], t.rs[j]);
    v[j] = to_f16((float)o + (float)r[j]);
  }
  return v;
}

template <int XF>
__device__ __forceinline__ f16x8 gn_load8(const GnIn& in, int c, long row, int ch, const GnXf& t) {
  const f16* p = ch < in.c1 ? in.x + row * in.c1 + ch : in.x2 + row * (c - in.c1) + (ch - in.c1);
  f16x8 v = *reinterpret_cast<const f16x8*>(p);
  if constexpr (XF == 1) {
    const bool q = in.qmax > 0, a = in.cadd != nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f16 o = v[j];
      if (q) o = fq_apply_r((float)o, t.s[j], t.rs[j]);
      if (a) o = to_f16((float)o + t.ca[j]);
      v[j] = o;
    }
  }
  return v;
}

// single element (coefficient kernel: shifts and the fallback scan)
__device__ __forceinline__ float gn_load1(const GnIn& in, int c, long n, long row, int ch) {
  const f16* p = ch < in.c1 ? in.x + row * in.c1 + ch : in.x2 + row * (c - in.c1) + (ch - in.c1);
  f16 v = *p;
  if (in.qmax > 0) {
    const float s = fq_scale(in.amax[n * c + ch], in.qmax);
    v = fq_apply_r((float)v, s, rcp_exact(s));
  }
  if (in.cadd) v = to_f16((float)v + (float)in.cadd[n * in.cadd_ld + ch]);
  if (in.res) v = to_f16((float)v + (float)in.res[row * c + ch]);
  return (float)v;
}

struct GnGeom {
  int bx, by, gx, z, rpb;  // apply pass
  int bys, zs, rpbs;       // stats pass: 256-thread blocks, up to 16 rows per thread
};
// measurement knob (qd_gn_geom_force): rows per thread of the statistics / apply passes, 0 = the
// rule below
static int g_gn_srpt = 0, g_gn_arpt = 0;
extern "C" int qd_gn_geom_force(int stats_rows_per_thread, int apply_rows_per_thread) {
  g_gn_srpt = stats_rows_per_thread > 0 ? stats_rows_per_thread : 0;
  g_gn_arpt = apply_rows_per_thread > 0 ? apply_rows_per_thread : 0;
  return 0;
}

static GnGeom gn_geom(int n, int hw, int c) {
  GnGeom g;
  const int chunks = c / 8;
  g.bx = std::min(chunks, 256);
  g.by = 256 / g.bx;
  g.gx = (chunks + g.bx - 1) / g.bx;
  // >= 4 rows per thread: the per-thread setup (coefficients, fake-quant scales) is amortised over
  // 4 rows (2 rows per thread, the earlier rule's choice for grids under 2048 blocks, measured 5-9 %
  // slower on every SD1.5 streaming shape: profiles/r03w_gn_geom_sweep.log)
  g.rpb = g.by * 4;
  while ((long)g.gx * n * ((hw + g.rpb - 1) / g.rpb) > 8192) g.rpb *= 2;
  if (g_gn_arpt) g.rpb = g.by * g_gn_arpt;
  g.z = (hw + g.rpb - 1) / g.rpb;
  // stats: 8 loads in flight per thread, 16 rows per thread while the grid keeps >= 512 blocks
  g.bys = g.by;
  g.rpbs = g.bys * 16;
  while (g.rpbs > g.bys * 8 && (long)g.gx * n * ((hw + g.rpbs - 1) / g.rpbs) < 256) g.rpbs /= 2;
  if (g_gn_srpt) g.rpbs = g.bys * g_gn_srpt;
  g.zs = (hw + g.rpbs - 1) / g.rpbs;
  return g;
}

__device__ __forceinline__ float gn_out(float xv, float2 k, int silu) {
  f16 o = to_f16(fmaf(xv, k.x, k.y));
  if (silu) o = to_f16(silu_f((float)o));
  return (float)o;
}

// F: the input transform's flags, fixed at compile time (GN_FQ output quant, GN_FA + cadd, GN_FR
// + residual; the host maps in.qmax / in.cadd / in.res onto them)
constexpr int GN_FQ = 1, GN_FA = 2, GN_FR = 4;

template <int XF, int F = 0>
__global__ void __launch_bounds__(256) k_gn_stats(GnIn in, int hw, int c, int cg, int rows_per_block,
                                                  float4* __restrict__ part, float* __restrict__ amax_n) {
  constexpr bool FQ = (F & GN_FQ) != 0, FA = (F & GN_FA) != 0, FR = XF == 2 && (F & GN_FR) != 0;
  // rows per batch, all loads issued before any use (memory-level parallelism); the residual form
  // holds two tiles per row, so it batches 4 rows (VGPR budget: more waves per SIMD instead)
  constexpr int UB = FR ? 4 : 8;
  __shared__ float2 red[256][8];
  const int tx = threadIdx.x, ty = threadIdx.y, bx = blockDim.x, by = blockDim.y;
  const int chunk = blockIdx.x * bx + tx;
  const bool active = chunk * 8 < c;
  const int ch = chunk * 8;
  const long n = blockIdx.y;

  const int r0 = blockIdx.z * rows_per_block, r1 = min(hw, r0 + rows_per_block);
  float s1[8], s2[8], sh[8], mn[8], mx[8];
  GnXf xf;
  if (active) gn_xf_init(in, c, n, ch, xf);
  // the shift of channel ch + j is its group's first element; with >= 8 channels per group the
  // chunk spans at most two groups, so two (transformed) loads serve all 8 channels
  const int f0 = ch / cg * cg, f7 = (ch + 7) / cg * cg;
  float sh0 = 0.f, sh7 = 0.f;
  if (active && cg >= 8) {
    sh0 = gn_load1(in, c, n, n * hw, f0);
    sh7 = gn_load1(in, c, n, n * hw, f7);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] = s2[j] = 0.f;
    mn[j] = INFINITY;
    mx[j] = -INFINITY;
    sh[j] = !active ? 0.f : cg >= 8 ? ((ch + j) / cg * cg == f0 ? sh0 : sh7) : gn_load1(in, c, n, n * hw, (ch + j) / cg * cg);
  }
  // (Issuing the first row batch before this setup, and a two-register-set ping-pong that keeps
  // batch b + 1 in flight while batch b is reduced, measured no faster and cost a wave per SIMD:
  // profiles/r06i_gn_stats_variants.log.)
  if (active) {
    for (int rb = r0 + ty; rb < r1; rb += UB * by) {
      f16x8 v[UB];
      // unconditional loads (row clamped): a guarded load makes hipcc wait per load
#pragma unroll
      for (int u = 0; u < UB; ++u) v[u] = gn_raw8(in, c, n * hw + min(rb + u * by, r1 - 1), ch);
      f16x8 rr[UB];
      if constexpr (FR) {
#pragma unroll
        for (int u = 0; u < UB; ++u) rr[u] = *reinterpret_cast<const f16x8*>(in.res + (n * hw + min(rb + u * by, r1 - 1)) * c + ch);
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) QD_PIN(v[u]);
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        if (rb + u * by >= r1) break;
        f16x8 w;
        if constexpr (XF == 2) {
          if constexpr (FR) w = gn_fin8c<FQ>(v[u], xf, rr[u]);
          else w = gn_xf8c<FQ, FA>(v[u], xf);
          *reinterpret_cast<f16x8*>(in.xout + (n * hw + rb + u * by) * c + ch) = w;
        } else if constexpr (XF == 1) {
          w = gn_xf8c<FQ, FA>(v[u], xf);
        } else {
          w = v[u];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = (float)w[j];
          const float a = xv - sh[j];
          s1[j] += a;
          s2[j] = fmaf(a, a, s2[j]);
          mn[j] = fminf(mn[j], xv);
          mx[j] = fmaxf(mx[j], xv);
        }
      }
    }
  }
  const int t = ty * bx + tx;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = make_float2(s1[j], s2[j]);
  __syncthreads();
  if (ty == 0 && active)
    for (int k = 1; k < by; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 o = red[k * bx + tx][j];
        s1[j] += o.x;
        s2[j] += o.y;
      }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = make_float2(mn[j], mx[j]);
  __syncthreads();
  if (ty == 0 && active) {
    for (int k = 1; k < by; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 o = red[k * bx + tx][j];
        mn[j] = fminf(mn[j], o.x);
        mx[j] = fmaxf(mx[j], o.y);
      }
    float4* dst = part + ((n * gridDim.z + blockIdx.z) * c + ch);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = make_float4(s1[j], s2[j], mn[j], mx[j]);
  }
}

// largest |silu| of any input: silu(-1.2785) = -0.27846; a |half(silu(.))| >= this bound can only
// come from the positive branch, where the rounded GN+SiLU output is non-decreasing in z
constexpr float SILU_NEG_BOUND = 0.2786f;

// One block per (n, group): group mean / rstd from the partials (fixed thread -> partial map,
// fixed reduction tree: deterministic).  MODE 0: k_gn_stats' per-channel shifted sums; MODE 1: the
// 64-row slot moments (mean, M2, min, max) a producing int8 conv's epilogue wrote (gemm.hip
// QD_EPI_GNSTATS), merged in one pass as shifted sums about the group's first slot mean
// (sum (x - K) = 64 sum (mean_i - K), sum (x - K)^2 = sum (M2_i + 64 (mean_i - K)^2)).  Then per channel the affine coefficients and - when the
// output is fake-quantized - its exact amax from the channel's min / max input:
// out = half([silu](half(x * a + b))) is monotone in x on each side of silu's minimum, so
// max |out| is |out(x_min)| or |out(x_max)| except when SiLU is on and both extremes map below
// the bound above; the block then scans those (rare) channels' rows itself.
// MODE 1 with a concatenated input (x | x2 along C, GnIn.c1): channels [0, c1) read their slots
// from part ([n][Z][c1]), channels [c1, c) from part2 ([n][Z][c - c1]) - each source's own producer
// wrote them.  xamax (quant): the per-(n, c) max |x| of the INPUT from the channel extremes (the
// input quant of a conv that reads the same input, e.g. the up blocks' skip-concat shortcut).
template <int MODE>
__global__ void __launch_bounds__(256) k_gn_coeff(const float4* __restrict__ part, GnIn in, int hw, int c, int cg,
                                                  int Z, float eps, const f16* __restrict__ gamma,
                                                  const f16* __restrict__ beta, int silu, int quant,
                                                  float2* __restrict__ coef, float* __restrict__ amax,
                                                  float* __restrict__ amax_n,
                                                  const float4* __restrict__ part2 = nullptr,
                                                  float* __restrict__ xamax = nullptr) {
  __shared__ float red[2][4];
  __shared__ float stat[2];
  __shared__ int nflag;
  __shared__ int flagged[1024];
  __shared__ int cmin[1024], cmax[1024];  // per-channel min / max as order-preserving ints
  __shared__ float fmx[4];
  const int groups = c / cg;
  const int ni = blockIdx.x / groups, g0 = (blockIdx.x % groups) * cg;
  const int t = threadIdx.x;
  // the affine parameters of the thread's first channel, loaded before the partials pass (their
  // latency hides under it instead of following the group statistics)
  const float gm0 = t < cg ? (float)gamma[g0 + t] : 0.f, bt0 = t < cg ? (float)beta[g0 + t] : 0.f;
  // MODE 0's shift (the group's first element), likewise issued up front by the thread that uses it
  const float shift0 = MODE == 0 && t == 0 ? gn_load1(in, c, ni, (long)ni * hw, g0) : 0.f;
  if (t == 0) nflag = 0;
  for (int j = t; j < cg; j += 256) {
    cmin[j] = 0x7fffffff;
    cmax[j] = (int)0x80000000;
  }
  __syncthreads();
  // one pass over the (z, channel) partials: group sums in registers, channel extremes by LDS
  // integer min / max of the order-preserving image of the float (exact, order-independent)
  // partial of (slot z, channel g0 + j): one [n][Z][c] array, or the concat's two sources (MODE 1)
  const int c1 = MODE == 1 ? in.c1 : c;
  auto pv = [&](int z, int j) {
    const int ch = g0 + j;
    return ch < c1 ? part[((long)ni * Z + z) * c1 + ch] : part2[((long)ni * Z + z) * (c - c1) + (ch - c1)];
  };
  // MODE 1: one pass of shifted sums over the slots (shift K1 = the group's first slot mean):
  // sum over rows of (x - K1) = 64 sum (mean_i - K1), of (x - K1)^2 = sum (M2_i + 64 (mean_i - K1)^2)
  // - then MODE 0's finalisation with the shift K1
  const float K1 = MODE == 1 ? pv(0, 0).x : 0.f;
  float s1 = 0.f, s2 = 0.f;
  // PF partials per thread in flight before the first is used (one memory round trip instead of
  // one per 256 partials); the per-thread accumulation order is unchanged (e ascending)
  constexpr int PF = 4;
  const int ne = Z * cg;
  for (int e0 = t; e0 < ne; e0 += 256 * PF) {
    float4 v[PF];
    int jj[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const int e = min(e0 + 256 * k, ne - 1);
      const int z = e / cg;
      jj[k] = e - z * cg;
      v[k] = pv(z, jj[k]);
    }
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (e0 + 256 * k >= ne) break;
      if constexpr (MODE == 0) {
        s1 += v[k].x;
        s2 += v[k].y;
      } else {
        const float d = v[k].x - K1;
        s1 += 64.0f * d;
        s2 += v[k].y + 64.0f * (d * d);
      }
      if (quant) {
        const int a = __float_as_int(v[k].z), b = __float_as_int(v[k].w);
        atomicMin(&cmin[jj[k]], a ^ ((a >> 31) & 0x7fffffff));
        atomicMax(&cmax[jj[k]], b ^ ((b >> 31) & 0x7fffffff));
      }
    }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if ((t & 63) == 0) {
    red[0][t >> 6] = s1;
    red[1][t >> 6] = s2;
  }
  __syncthreads();
  if (t == 0) {
    const float S1 = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const float S2 = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const float cnt = (float)cg * (float)hw;
    const float m = S1 / cnt;                        // mean of the shifted values
    const float var = fmaxf(S2 / cnt - m * m, 0.f);  // population variance
    stat[0] = m + (MODE == 0 ? shift0 : K1);
    stat[1] = 1.0f / sqrtf(var + eps);
  }
  __syncthreads();
  float gmx = 0.f;  // the thread's max over its channels' output amax (amax_n below)
  for (int j = t; j < cg; j += 256) {
    const int ch = g0 + j;
    const long i = (long)ni * c + ch;
    const float sc = stat[1] * (j == t ? gm0 : (float)gamma[ch]);
    const float2 k = make_float2(sc, fmaf(-sc, stat[0], j == t ? bt0 : (float)beta[ch]));
    coef[i] = k;
    if (!quant) continue;
    const int ia = cmin[j], ib = cmax[j];
    const float mn = __int_as_float(ia ^ ((ia >> 31) & 0x7fffffff));
    const float mx = __int_as_float(ib ^ ((ib >> 31) & 0x7fffffff));
    if (xamax) xamax[i] = fmaxf(fabsf(mn), fabsf(mx));
    const float lo = fabsf(gn_out(mn, k, silu)), hi = fabsf(gn_out(mx, k, silu));
    const float top = fabsf(gn_out(sc >= 0.f ? mx : mn, k, silu));  // largest z
    if (!silu) {
      amax[i] = fmaxf(lo, hi);
      gmx = fmaxf(gmx, fmaxf(lo, hi));
    } else if (top >= SILU_NEG_BOUND) {
      amax[i] = top;
      gmx = fmaxf(gmx, top);
    } else {
      flagged[atomicAdd(&nflag, 1)] = j;
    }
  }
  __syncthreads();
  // fallback: a full max |out| scan of each flagged channel by the whole block (fixed order of
  // channels is irrelevant: max is exact)
  for (int f = 0; f < nflag; ++f) {
    const int ch = g0 + flagged[f];
    const long i = (long)ni * c + ch;
    const float2 k = coef[i];
    float m = 0.f;
    for (int r = t; r < hw; r += 256) m = fmaxf(m, fabsf(gn_out(gn_load1(in, c, ni, (long)ni * hw + r, ch), k, silu)));
    m = wave_max(m);
    if ((t & 63) == 0) fmx[t >> 6] = m;
    __syncthreads();
    if (t == 0) {
      const float a = fmaxf(fmaxf(fmx[0], fmx[1]), fmaxf(fmx[2], fmx[3]));
      amax[i] = a;
      gmx = fmaxf(gmx, a);
    }
    __syncthreads();
  }
  if (amax_n) {
    // int8 output: this (n, group)'s max over its channels into amax_n[n][group] - from the
    // registers that wrote amax above (the scanned channels' values sit with thread 0), not a
    // re-read of amax; the apply pass takes the max over the groups (no same-address atomics:
    // they serialise across blocks)
    float m = wave_max(gmx);
    if ((t & 63) == 0) fmx[t >> 6] = m;
    __syncthreads();
    if (t == 0) amax_n[blockIdx.x] = fmaxf(fmaxf(fmx[0], fmx[1]), fmaxf(fmx[2], fmx[3]));
  }
}

// block (bx, by): thread (tx, ty) owns channel chunk blockIdx.x * bx + tx (8 channels, 16 B) of
// sample blockIdx.y and rows ty, ty + by, ... of its row range: the per-channel coefficients
// and fake-quant scales are loaded / computed once per thread, rows stream through.
// The two sources are both multiples of 8 channels wide (host check).
// int8 output (the int8-MFMA mode's conv input, one scale per sample): codes
// rint(half(out / s_n)) with s_n = half(half(max_c amax[n][c]) / 127) written to y8, s_n to sa8[n]
template <int XF, int SILU, bool Q, bool I8 = false>
__global__ void __launch_bounds__(256) k_gn_apply(GnIn in, int hw, int c, int rows_per_block,
                                                  const float2* __restrict__ coef, int qmax,
                                                  const float* __restrict__ amax, f16* __restrict__ y,
                                                  const float* __restrict__ amax_n = nullptr,
                                                  int8_t* __restrict__ y8 = nullptr, float* __restrict__ sa8 = nullptr) {
  const int chunk = blockIdx.x * blockDim.x + threadIdx.x;
  const long n = blockIdx.y;
  float s8 = 0.f;
  double r8 = 0.0;
  if constexpr (I8) {
    // amax_n[n][g] (qmax carries the group count here, <= 64): max over the sample's groups - one
    // load per lane of the block's first wave (always full: blocks hold >= 64 threads) and a wave
    // reduction (max is exact), handed to the block through LDS, instead of qmax loads per thread
    // (a partial last wave's shuffles would read inactive lanes)
    __shared__ float smx;
    const int flat = threadIdx.y * blockDim.x + threadIdx.x;
    if (flat < 64) {
      float m = flat < qmax ? amax_n[n * qmax + flat] : 0.f;
      m = wave_max(m);
      if (flat == 0) smx = m;
    }
    __syncthreads();
    s8 = fq_scale(smx, 127);
    r8 = rcp_exact(s8);
    if (chunk == 0 && blockIdx.z == 0 && threadIdx.y == 0) sa8[n] = s8;
  }
  if (chunk * 8 >= c) return;
  const int ch = chunk * 8;
  const int r0 = blockIdx.z * rows_per_block, r1 = min(hw, r0 + rows_per_block);
  float2 k[8];
  float sq[8];
  double rq[8];
  GnXf xf;
  gn_xf_init(in, c, n, ch, xf);
  {
    const float4* cp = reinterpret_cast<const float4*>(coef + n * c + ch);
    const float4 k0 = cp[0], k1 = cp[1], k2 = cp[2], k3 = cp[3];
    k[0] = make_float2(k0.x, k0.y); k[1] = make_float2(k0.z, k0.w);
    k[2] = make_float2(k1.x, k1.y); k[3] = make_float2(k1.z, k1.w);
    k[4] = make_float2(k2.x, k2.y); k[5] = make_float2(k2.z, k2.w);
    k[6] = make_float2(k3.x, k3.y); k[7] = make_float2(k3.z, k3.w);
  }
  if constexpr (Q) {
    fq_scales8(amax + n * c + ch, qmax, sq, rq);
  }
  const int by = blockDim.y;
  for (int rb = r0 + threadIdx.y; rb < r1; rb += 4 * by) {
    f16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = gn_raw8(in, c, n * hw + min(rb + u * by, r1 - 1), ch);
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + u * by >= r1) break;
      const f16x8 w = gn_xf8<XF>(in, v[u], xf);
      if constexpr (I8) {
        unsigned lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float val = gn_out((float)w[j], k[j], SILU);
          const f16 tq = (f16)(float)((double)val * r8);
          const unsigned q = (unsigned)(uint8_t)(int8_t)__builtin_rintf((float)tq);
          if (j < 4) lo |= q << (8 * j);
          else hi |= q << (8 * (j - 4));
        }
        *reinterpret_cast<uint2*>(y8 + (n * hw + rb + u * by) * c + ch) = make_uint2(lo, hi);
        continue;
      }
      f16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = gn_out((float)w[j], k[j], SILU);
        if constexpr (Q) o[j] = fq_apply_r(val, sq[j], rq[j]);
        else o[j] = (f16)val;
      }
      *reinterpret_cast<f16x8*>(y + (n * hw + rb + u * by) * c + ch) = o;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Single-kernel GroupNorm for the small UNet levels (hw <= 256): one block per (sample, set of
// G groups whose channels form whole 16-B octets) does statistics, coefficients, the output
// amax and the apply, reading its slice twice (the second time from L2) instead of three
// stream-ordered launches whose fixed costs dominate there (8x8, 16x16: 17-20 us for a 1-5 MB
// tensor vs a 3 us copy; at 32x32 the 3-launch path's wider grid wins).  Same arithmetic as k_gn_stats / k_gn_coeff / k_gn_apply
// (shifted sums, the group's first element as the shift, monotone amax with the scan
// fallback); only the fp32 summation order of the group sums differs.
// ---------------------------------------------------------------------------------------
constexpr int GNF_CW = 128;  // max channels per block (16 octets)

template <int XF, int SILU, bool Q>
__global__ void __launch_bounds__(256) k_gn_fused(GnIn in, int hw, int c, int cg, int G, float eps,
                                                  const f16* __restrict__ gamma, const f16* __restrict__ beta,
                                                  int qmax, f16* __restrict__ y) {
  __shared__ float4 red[256][8];   // per thread and channel (s1, s2, min, max)
  __shared__ float4 chs[GNF_CW];   // per channel (S1, S2, min, max) of the block's slice
  __shared__ float2 gst[16];       // per group (mean, rstd)
  __shared__ float2 kco[GNF_CW];   // per channel (scale, bias)
  __shared__ float amx[GNF_CW];
  __shared__ int flagged[GNF_CW];
  __shared__ int nflag;
  __shared__ float fmx[4];
  const int CW = G * cg, CPP = CW / 8, PS = 256 / CPP;
  const int t = threadIdx.x;
  const int o = t % CPP, p0 = t / CPP;
  const bool active = p0 < PS;
  const int c0 = blockIdx.x * CW, ch = c0 + o * 8;
  const long n = blockIdx.y;
  if (t == 0) nflag = 0;

  GnXf xf;
  float s1[8], s2[8], sh[8], mn[8], mx[8];
  if (active) gn_xf_init(in, c, n, ch, xf);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] = s2[j] = 0.f;
    mn[j] = INFINITY;
    mx[j] = -INFINITY;
    sh[j] = active ? gn_load1(in, c, n, n * hw, (ch + j) / cg * cg) : 0.f;
  }
  if (active) {
    for (int rb = p0; rb < hw; rb += 8 * PS) {
      f16x8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = gn_raw8(in, c, n * hw + min(rb + u * PS, hw - 1), ch);
#pragma unroll
      for (int u = 0; u < 8; ++u) QD_PIN(v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (rb + u * PS >= hw) break;
        const f16x8 w = gn_xf8<XF>(in, v[u], xf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = (float)w[j];
          const float a = xv - sh[j];
          s1[j] += a;
          s2[j] = fmaf(a, a, s2[j]);
          mn[j] = fminf(mn[j], xv);
          mx[j] = fmaxf(mx[j], xv);
        }
      }
    }
  }
  // per-channel totals over the PS threads of each octet: one thread per channel, fixed order
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = make_float4(s1[j], s2[j], mn[j], mx[j]);
  __syncthreads();
  if (t < CW) {
    const int oc = t >> 3, j = t & 7;
    float4 a = red[oc][j];
    for (int k = 1; k < PS; ++k) {
      const float4 v = red[k * CPP + oc][j];
      a.x += v.x;
      a.y += v.y;
      a.z = fminf(a.z, v.z);
      a.w = fmaxf(a.w, v.w);
    }
    chs[t] = a;
  }
  __syncthreads();
  if (t < G) {
    float S1 = 0.f, S2 = 0.f;
    for (int j = 0; j < cg; ++j) {
      S1 += chs[t * cg + j].x;
      S2 += chs[t * cg + j].y;
    }
    const float cnt = (float)cg * (float)hw;
    const float m = S1 / cnt;
    const float var = fmaxf(S2 / cnt - m * m, 0.f);
    gst[t] = make_float2(m + gn_load1(in, c, n, n * hw, c0 + t * cg), 1.0f / sqrtf(var + eps));
  }
  __syncthreads();
  if (t < CW) {
    const int cc = c0 + t;
    const float2 st = gst[t / cg];
    const float sc = st.y * (float)gamma[cc];
    const float2 k = make_float2(sc, fmaf(-sc, st.x, (float)beta[cc]));
    kco[t] = k;
    if (Q) {
      const float4 e = chs[t];
      const float lo = fabsf(gn_out(e.z, k, SILU)), hi = fabsf(gn_out(e.w, k, SILU));
      const float top = fabsf(gn_out(sc >= 0.f ? e.w : e.z, k, SILU));
      if (!SILU) amx[t] = fmaxf(lo, hi);
      else if (top >= SILU_NEG_BOUND) amx[t] = top;
      else flagged[atomicAdd(&nflag, 1)] = t;
    }
  }
  __syncthreads();
  if (Q) {
    for (int f = 0; f < nflag; ++f) {  // rare: a full max |out| scan of the channel
      const int cl = flagged[f];
      const float2 k = kco[cl];
      float m = 0.f;
      for (int r = t; r < hw; r += 256) m = fmaxf(m, fabsf(gn_out(gn_load1(in, c, n, n * hw + r, c0 + cl), k, SILU)));
      m = wave_max(m);
      if ((t & 63) == 0) fmx[t >> 6] = m;
      __syncthreads();
      if (t == 0) amx[cl] = fmaxf(fmaxf(fmx[0], fmx[1]), fmaxf(fmx[2], fmx[3]));
      __syncthreads();
    }
  }
  if (!active) return;
  float2 k[8];
  float sq[8];
  double rq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k[j] = kco[o * 8 + j];
    if (Q) {
      sq[j] = fq_scale(amx[o * 8 + j], qmax);
      rq[j] = rcp_exact(sq[j]);
    }
  }
  // XF 2: this block's statistics pass wrote its rows of x to xout (visible after the barriers)
  for (int rb = p0; rb < hw; rb += 4 * PS) {
    f16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = gn_raw8(in, c, n * hw + min(rb + u * PS, hw - 1), ch);
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + u * PS >= hw) break;
      const f16x8 w = gn_xf8<XF>(in, v[u], xf);
      f16x8 out;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = gn_out((float)w[j], k[j], SILU);
        if constexpr (Q) out[j] = fq_apply_r(val, sq[j], rq[j]);
        else out[j] = (f16)val;
      }
      *reinterpret_cast<f16x8*>(y + (n * hw + rb + u * PS) * c + ch) = out;
    }
  }
}

// groups per fused block: the fewest whole groups spanning whole octets (0: not fused)
static int gn_fused_groups(int n, int hw, int c, int groups) {
  if (hw > 256) return 0;
  const int cg = c / groups;
  for (int G = 1; G <= 16 && G * cg <= GNF_CW; ++G) {
    if (groups % G || (G * cg) % 8) continue;
    return G;
  }
  return 0;
}

extern "C" int qd_groupnorm_workspace(int n, int hw, int c, int groups) {
  const GnGeom g = gn_geom(n, hw, c);
  return 4 * n * g.zs * c + 2 * n * c + n * c + n * c;  // partials (float4), coef (float2), amax, spare
}

static int run_groupnorm(const GnIn& in, int n, int hw, int c, int groups, float eps, const void* gamma,
                         const void* beta, int silu, int q_bits, void* y, float* ws, hipStream_t st,
                         int8_t* y8 = nullptr, float* sa8 = nullptr, float* xamax = nullptr) {
  QD_REQUIRE(in.x && gamma && beta && (y || y8) && ws, "null pointer");
  QD_REQUIRE(!y8 || (sa8 && q_bits == 0), "int8 output: scales needed, no fake-quant bits");
  QD_REQUIRE(groups > 0 && c % groups == 0, "groups must divide C");
  QD_REQUIRE(c % 8 == 0, "GroupNorm needs C % 8 == 0");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0, "workspace must be 16-B aligned");
  QD_REQUIRE(q_bits == 0 || (q_bits >= 2 && q_bits <= 16), "bad q_bits");
  QD_REQUIRE(c / groups <= 1024, "GroupNorm supports at most 1024 channels per group");
  if ((long)n * hw == 0) return 0;
  const int cg = c / groups;
  const GnGeom g = gn_geom(n, hw, c);
  float4* part = reinterpret_cast<float4*>(ws);
  float2* coef = reinterpret_cast<float2*>(part + (long)n * g.zs * c);
  float* amax = reinterpret_cast<float*>(coef + (long)n * c);
  float* amax_n = y8 ? amax + (long)n * c : nullptr;  // per-(n, group) maxima in the spare n * c floats
  const int qmax = q_bits ? (1 << (q_bits - 1)) - 1 : 0;
  // XF 2: the finalized input x (output quant + residual, or + temb) is written to in.xout by the
  // statistics pass and read back by the apply pass
  const bool fin = in.xout != nullptr;
  QD_REQUIRE(!fin || (!in.x2 && !(in.res && in.cadd) && !y8), "materialised input: no concat / int8 output, residual or temb");
  const bool xf = !fin && (in.qmax > 0 || in.cadd);
  // (the residual-input form always takes the streaming passes: its statistics pass writes x)
  QD_REQUIRE(!xamax || q_bits > 0 || y8, "the input amax comes from the quantized output's channel extremes");
  // (xamax: the three-pass form, whose coefficient kernel reduces the channel extremes)
  if (const int G = y8 || fin || xamax ? 0 : gn_fused_groups(n, hw, c, groups)) {
    const dim3 gf(groups / G, n);
#define QD_GN_FUSED(XFV, SV, QV)                                                                               \
  k_gn_fused<XFV, SV, QV><<<gf, 256, 0, st>>>(in, hw, c, cg, G, eps, (const f16*)gamma, (const f16*)beta, qmax, \
                                              (f16*)y)
    switch ((xf ? 4 : 0) | (silu ? 2 : 0) | (qmax > 0 ? 1 : 0)) {
      case 0: QD_GN_FUSED(0, 0, false); break;
      case 1: QD_GN_FUSED(0, 0, true); break;
      case 2: QD_GN_FUSED(0, 1, false); break;
      case 3: QD_GN_FUSED(0, 1, true); break;
      case 4: QD_GN_FUSED(1, 0, false); break;
      case 5: QD_GN_FUSED(1, 0, true); break;
      case 6: QD_GN_FUSED(1, 1, false); break;
      default: QD_GN_FUSED(1, 1, true); break;
    }
#undef QD_GN_FUSED
    QD_CHECK_LAUNCH();
    return 0;
  }
  const dim3 gs(g.gx, n, g.zs), bs(g.bx, g.bys);
  {
    const int f = (in.qmax > 0 ? GN_FQ : 0) | (in.cadd ? GN_FA : 0) | (in.res ? GN_FR : 0);
#define QD_GN_STATS(XFV, FV) k_gn_stats<XFV, FV><<<gs, bs, 0, st>>>(in, hw, c, cg, g.rpbs, part, amax_n)
    if (fin) {
      switch (f) {  // (the residual and cadd forms exclude each other: host check above)
        case 0: QD_GN_STATS(2, 0); break;
        case GN_FQ: QD_GN_STATS(2, GN_FQ); break;
        case GN_FA: QD_GN_STATS(2, GN_FA); break;
        case GN_FQ | GN_FA: QD_GN_STATS(2, GN_FQ | GN_FA); break;
        case GN_FR: QD_GN_STATS(2, GN_FR); break;
        default: QD_GN_STATS(2, GN_FQ | GN_FR); break;
      }
    } else if (xf) {
      QD_REQUIRE(!in.res, "the residual input form is the materialising statistics pass");
      switch (f) {
        case GN_FQ: QD_GN_STATS(1, GN_FQ); break;
        case GN_FA: QD_GN_STATS(1, GN_FA); break;
        default: QD_GN_STATS(1, GN_FQ | GN_FA); break;
      }
    } else {
      QD_GN_STATS(0, 0);
    }
#undef QD_GN_STATS
  }
  // (the coefficient stage recomputes its shift / fallback elements from the raw sources; the
  // apply pass reads the materialised x)
  k_gn_coeff<0><<<n * groups, 256, 0, st>>>(part, in, hw, c, cg, g.zs, eps, (const f16*)gamma, (const f16*)beta,
                                            silu, qmax > 0 || y8, coef, amax, amax_n, nullptr, xamax);
  const dim3 ga(g.gx, n, g.z), ba(g.bx, g.by);
  if (fin) {
    const GnIn inx{in.xout, nullptr, c, nullptr, 0, nullptr, 0, nullptr, nullptr};
    if (silu && qmax > 0) k_gn_apply<0, 1, true><<<ga, ba, 0, st>>>(inx, hw, c, g.rpb, coef, qmax, amax, (f16*)y);
    else if (silu) k_gn_apply<0, 1, false><<<ga, ba, 0, st>>>(inx, hw, c, g.rpb, coef, qmax, amax, (f16*)y);
    else if (qmax > 0) k_gn_apply<0, 0, true><<<ga, ba, 0, st>>>(inx, hw, c, g.rpb, coef, qmax, amax, (f16*)y);
    else k_gn_apply<0, 0, false><<<ga, ba, 0, st>>>(inx, hw, c, g.rpb, coef, qmax, amax, (f16*)y);
    QD_CHECK_LAUNCH();
    return 0;
  }
  if (y8) {  // (the qmax argument carries the group count of amax_n[n][group])
    QD_REQUIRE(groups <= 64, "int8 output: at most 64 groups (one per lane of the apply pass's reduction)");
    if (xf && silu) k_gn_apply<1, 1, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, sa8);
    else if (xf) k_gn_apply<1, 0, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, sa8);
    else if (silu) k_gn_apply<0, 1, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, sa8);
    else k_gn_apply<0, 0, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, sa8);
    QD_CHECK_LAUNCH();
    return 0;
  }
#define QD_GN_APPLY(XFV, SV, QV) \
  k_gn_apply<XFV, SV, QV><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, qmax, amax, (f16*)y)
  const int sel = (xf ? 4 : 0) | (silu ? 2 : 0) | (qmax > 0 ? 1 : 0);
  switch (sel) {
    case 0: QD_GN_APPLY(0, 0, false); break;
    case 1: QD_GN_APPLY(0, 0, true); break;
    case 2: QD_GN_APPLY(0, 1, false); break;
    case 3: QD_GN_APPLY(0, 1, true); break;
    case 4: QD_GN_APPLY(1, 0, false); break;
    case 5: QD_GN_APPLY(1, 0, true); break;
    case 6: QD_GN_APPLY(1, 1, false); break;
    default: QD_GN_APPLY(1, 1, true); break;
  }
#undef QD_GN_APPLY
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_groupnorm(const void* x, const void* x2, int c1, int n, int hw, int c, int groups,
                            float eps, const void* gamma, const void* beta, int silu, int q_bits,
                            void* y, float* ws, void* stream) {
  if (x2) QD_REQUIRE(c1 % 8 == 0 && c1 > 0 && c1 < c, "bad concat split (must be a multiple of 8)");
  else c1 = c;
  GnIn in{(const f16*)x, (const f16*)x2, c1, nullptr, 0, nullptr, 0, nullptr, nullptr};
  return run_groupnorm(in, n, hw, c, groups, eps, gamma, beta, silu, q_bits, y, ws, S(stream));
}

// qd_groupnorm (q_bits > 0) that also writes xamax[n * c + ch] = max |input| of each (sample, channel)
// of x | x2, from the statistics pass's channel extremes: the input quant of the skip-concat shortcut
// without its own column-max pass (qd_act_apply_cat_nhwc)
extern "C" int qd_groupnorm_xamax(const void* x, const void* x2, int c1, int n, int hw, int c, int groups,
                                  float eps, const void* gamma, const void* beta, int silu, int q_bits,
                                  void* y, float* xamax, float* ws, void* stream) {
  QD_REQUIRE(xamax && q_bits > 0, "xamax output needs a quantized GroupNorm output");
  if (x2) QD_REQUIRE(c1 % 8 == 0 && c1 > 0 && c1 < c, "bad concat split (must be a multiple of 8)");
  else c1 = c;
  GnIn in{(const f16*)x, (const f16*)x2, c1, nullptr, 0, nullptr, 0, nullptr, nullptr};
  return run_groupnorm(in, n, hw, c, groups, eps, gamma, beta, silu, q_bits, y, ws, S(stream), nullptr, nullptr,
                       xamax);
}

extern "C" int qd_groupnorm_i8(const void* x, const void* x2, int c1, const float* in_amax, int in_bits,
                               const void* cadd, int cadd_ld, int n, int hw, int c, int groups, float eps,
                               const void* gamma, const void* beta, int silu, int8_t* y8, float* scales, float* ws,
                               void* stream) {
  QD_REQUIRE(y8 && scales, "null pointer");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(y8) & 7) == 0, "y8 must be 8-B aligned");
  if (x2) {
    QD_REQUIRE(c1 % 8 == 0 && c1 > 0 && c1 < c && !in_amax && !cadd, "bad concat split / concat with fq_in");
  } else {
    c1 = c;
  }
  QD_REQUIRE(in_bits == 0 || (in_bits >= 2 && in_bits <= 16 && in_amax), "bad input quant bits / amax");
  if (cadd_ld <= 0) cadd_ld = c;
  QD_REQUIRE(!cadd || (cadd_ld >= c && cadd_ld % 8 == 0), "bad cadd leading dim");
  GnIn in{(const f16*)x, (const f16*)x2, c1, in_amax, in_bits ? (1 << (in_bits - 1)) - 1 : 0, (const f16*)cadd, cadd_ld,
          nullptr, nullptr};
  return run_groupnorm(in, n, hw, c, groups, eps, gamma, beta, silu, 0, nullptr, ws, S(stream), y8, scales);
}

extern "C" int qd_groupnorm_fq_in(const void* y_raw, const float* in_amax, int in_bits, const void* cadd,
                                  int cadd_ld, int n, int hw, int c, int groups, float eps, const void* gamma,
                                  const void* beta, int silu, int q_bits, void* y, float* ws, void* stream) {
  QD_REQUIRE(in_bits == 0 || (in_bits >= 2 && in_bits <= 16 && in_amax), "bad input quant bits / amax");
  if (cadd_ld <= 0) cadd_ld = c;
  QD_REQUIRE(!cadd || (cadd_ld >= c && cadd_ld % 8 == 0), "bad cadd leading dim");
  GnIn in{(const f16*)y_raw, nullptr, c, in_amax, in_bits ? (1 << (in_bits - 1)) - 1 : 0, (const f16*)cadd, cadd_ld,
          nullptr, nullptr};
  return run_groupnorm(in, n, hw, c, groups, eps, gamma, beta, silu, q_bits, y, ws, S(stream));
}

extern "C" int qd_groupnorm_fin(const void* y_raw, const float* in_amax, int in_bits, const void* residual,
                                const void* cadd, int cadd_ld, void* x_out, int n, int hw, int c, int groups,
                                float eps, const void* gamma, const void* beta, int silu, int q_bits, void* y,
                                float* ws, void* stream) {
  QD_REQUIRE(y_raw && x_out, "null pointer");
  QD_REQUIRE(!(residual && cadd), "residual or temb add, not both");
  QD_REQUIRE(in_bits == 0 || (in_bits >= 2 && in_bits <= 16 && in_amax), "bad input quant bits / amax");
  QD_REQUIRE(x_out != y_raw && x_out != residual, "x_out must not alias the sources (other blocks still read them)");
  if (cadd_ld <= 0) cadd_ld = c;
  QD_REQUIRE(!cadd || (cadd_ld >= c && cadd_ld % 8 == 0), "bad cadd leading dim");
  GnIn in{(const f16*)y_raw, nullptr, c, in_amax, in_bits ? (1 << (in_bits - 1)) - 1 : 0, (const f16*)cadd, cadd_ld,
          (const f16*)residual, (f16*)x_out};
  return run_groupnorm(in, n, hw, c, groups, eps, gamma, beta, silu, q_bits, y, ws, S(stream));
}

// GroupNorm(+SiLU) whose statistics a producing int8 conv already reduced in its epilogue
// (gemm.hip QD_EPI_GNSTATS: part[n * hw / 64 + slot][c] = 64-row slot moments of x): the
// coefficient kernel merges the slots (k_gn_coeff<1>), the apply pass streams x once - two
// launches and one read of x instead of three launches and two reads.  y8: int8 codes with one
// scale per sample (the int8-MFMA mode's conv input, = qd_quant_samples_i8 of the fp16 output);
// else the fp16 output y (no output fake-quant: the test / diagnostic form).
extern "C" int qd_groupnorm_part(const float* part, const void* x, const float* part2, const void* x2, int c1,
                                 int n, int hw, int c, int groups, float eps, const void* gamma, const void* beta,
                                 int silu, void* y, int8_t* y8, float* scales, float* xamax, float* ws,
                                 void* stream) {
  QD_REQUIRE(part && x && gamma && beta && ws && (y || (y8 && scales)), "null pointer");
  if (x2) {
    QD_REQUIRE(part2 && c1 % 8 == 0 && c1 > 0 && c1 < c && (reinterpret_cast<uintptr_t>(part2) & 15) == 0,
               "concat: second source's slot statistics, c1 % 8 == 0");
  } else {
    c1 = c;
  }
  QD_REQUIRE(!xamax || y8, "the input amax is produced with the int8 output");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(part) & 15) == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0,
             "partials / workspace must be 16-B aligned");
  QD_REQUIRE(!y8 || (reinterpret_cast<uintptr_t>(y8) & 7) == 0, "y8 must be 8-B aligned");
  QD_REQUIRE(hw % 64 == 0 && hw > 0, "slot statistics need hw % 64 == 0");
  QD_REQUIRE(groups > 0 && c % groups == 0 && c % 8 == 0 && c / groups <= 1024, "bad channel grouping");
  if (n == 0) return 0;
  hipStream_t st = S(stream);
  const int cg = c / groups;
  const GnGeom g = gn_geom(n, hw, c);
  float2* coef = reinterpret_cast<float2*>(ws);
  float* amax = reinterpret_cast<float*>(coef + (long)n * c);
  float* amax_n = y8 ? amax + (long)n * c : nullptr;
  const GnIn in{(const f16*)x, (const f16*)x2, c1, nullptr, 0, nullptr, 0, nullptr, nullptr};
  k_gn_coeff<1><<<n * groups, 256, 0, st>>>(reinterpret_cast<const float4*>(part), in, hw, c, cg, hw / 64, eps,
                                            (const f16*)gamma, (const f16*)beta, silu, y8 != nullptr, coef, amax,
                                            amax_n, reinterpret_cast<const float4*>(part2), xamax);
  const dim3 ga(g.gx, n, g.z), ba(g.bx, g.by);
  QD_REQUIRE(!y8 || groups <= 64, "int8 output: at most 64 groups (one per lane of the apply pass's reduction)");
  if (y8) {  // (the qmax argument carries the group count of amax_n[n][group])
    if (silu) k_gn_apply<0, 1, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, scales);
    else k_gn_apply<0, 0, false, true><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, groups, amax, nullptr, amax_n, y8, scales);
  } else {
    if (silu) k_gn_apply<0, 1, false><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, 0, amax, (f16*)y);
    else k_gn_apply<0, 0, false><<<ga, ba, 0, st>>>(in, hw, c, g.rpb, coef, 0, amax, (f16*)y);
  }
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// LayerNorm over the last dim (diffusers BasicTransformerBlock norm1/2/3, torch CPU Half
// semantics: fp32 mean / biased variance, y = half((x - mean) * rstd * gamma + beta)).
// One wave per row, R rows per wave with every row's 16-B loads issued before any reduction
// (enough bytes in flight per CU to stream at HBM rate even for C = 320 rows of 640 B); lane l
// owns the 8-channel chunks l, l + 64, ... of the row.
// ---------------------------------------------------------------------------------------
// I8: int8 output with one scale per row (the int8-MFMA mode's linear input, per token):
// codes rint(half(out / s)), s = half(half(max |out|) / 127) -> y8, s -> sa8[row]
template <int PER, int R, bool I8 = false>  // 8-channel chunks per lane, rows per wave
__global__ void __launch_bounds__(256) k_layernorm(const f16* __restrict__ x, long rows, int c, float eps,
                                                   const f16* __restrict__ gamma,
                                                   const f16* __restrict__ beta, f16* __restrict__ y,
                                                   int8_t* __restrict__ y8 = nullptr, float* __restrict__ sa8 = nullptr) {
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  const int lane = threadIdx.x & 63;
  const int chunks = c >> 3;
  f16x8 v[R][PER];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = lane + i * 64;
      v[r][i] = (row0 + r < rows && j < chunks) ? *reinterpret_cast<const f16x8*>(x + (row0 + r) * c + j * 8)
                                                : (f16x8){};
    }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (row0 + r >= rows) break;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)v[r][i][e];
    const float mean = wave_sum(s) / (float)c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      if (lane + i * 64 < chunks) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = (float)v[r][i][e] - mean;
          q = fmaf(a, a, q);
        }
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)c + eps);
    if constexpr (I8) {
      f16x8 o[PER];
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = lane + i * 64;
        o[i] = (f16x8){};
        if (j < chunks) {
          const f16x8 g = *reinterpret_cast<const f16x8*>(gamma + j * 8);
          const f16x8 b = *reinterpret_cast<const f16x8*>(beta + j * 8);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            o[i][e] = to_f16(fmaf(((float)v[r][i][e] - mean) * rstd, (float)g[e], (float)b[e]));
            m = fmaxf(m, fabsf((float)o[i][e]));
          }
        }
      }
      const float s = fq_scale(wave_max(m), 127);
      const double rs = rcp_exact(s);
      if (lane == 0) sa8[row0 + r] = s;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = lane + i * 64;
        if (j < chunks) {
          unsigned lo = 0, hi = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const f16 tq = (f16)(float)((double)(float)o[i][e] * rs);
            const unsigned qv = (unsigned)(uint8_t)(int8_t)__builtin_rintf((float)tq);
            if (e < 4) lo |= qv << (8 * e);
            else hi |= qv << (8 * (e - 4));
          }
          *reinterpret_cast<uint2*>(y8 + (row0 + r) * c + j * 8) = make_uint2(lo, hi);
        }
      }
      continue;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = lane + i * 64;
      if (j < chunks) {
        const f16x8 g = *reinterpret_cast<const f16x8*>(gamma + j * 8);
        const f16x8 b = *reinterpret_cast<const f16x8*>(beta + j * 8);
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = to_f16(fmaf(((float)v[r][i][e] - mean) * rstd, (float)g[e], (float)b[e]));
        *reinterpret_cast<f16x8*>(y + (row0 + r) * c + j * 8) = o;
      }
    }
  }
}

template <int PER, bool I8 = false>
static void launch_ln(const f16* x, long rows, int c, float eps, const f16* g, const f16* b, f16* y, hipStream_t st,
                      int8_t* y8 = nullptr, float* sa8 = nullptr) {
  // rows per wave: ~2 KB of loads in flight per wave, while the grid still fills the chip
  int r = std::max(1, 2048 / (c * 2));
  while (r > 1 && (rows + 4L * r - 1) / (4L * r) < 1024) r >>= 1;
  if (r >= 4) k_layernorm<PER, 4, I8><<<(int)((rows + 15) / 16), 256, 0, st>>>(x, rows, c, eps, g, b, y, y8, sa8);
  else if (r >= 2) k_layernorm<PER, 2, I8><<<(int)((rows + 7) / 8), 256, 0, st>>>(x, rows, c, eps, g, b, y, y8, sa8);
  else k_layernorm<PER, 1, I8><<<(int)((rows + 3) / 4), 256, 0, st>>>(x, rows, c, eps, g, b, y, y8, sa8);
}

// ---------------------------------------------------------------------------------------
// Grouped-row LayerNorm (every C = 8 * LPR * P with LPR in {8..64} lanes per row, P <= 5 16-B
// chunks per lane: SD's 320 / 640 / 1280 / 2560, CLIP's 768 / 1280): a wave holds 64 / LPR rows at
// once, lane l of a row owning chunks l, l + LPR, ... (coalesced), so all 64 lanes carry data
// (the one-row-per-wave kernel above leaves 24 of 64 lanes idle at C 320) and 64 / LPR rows' loads
// are in flight per wave.  Sums: each lane's P x 8 values in order, then a butterfly over the row's
// LPR lanes.  MODE 0: fp16 out; 1: int8 codes + one scale per row (the int8-MFMA mode's linear
// input); 2: the input is a conv output with its per-(sample, channel) output fake-quant pending -
// t = fq(y) is written (the residual stream) and LayerNorm(t) (qd_layernorm_fq).  The three modes
// share the arithmetic, so LN-fq == finalize + LN and LN-int8 == LN + per-row quant bit for bit.
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int LPR>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int LPR, int P, int MODE>
__global__ void __launch_bounds__(256) k_ln_rows(const f16* __restrict__ x, long rows, int c, float eps,
                                                 const f16* __restrict__ gamma, const f16* __restrict__ beta,
                                                 f16* __restrict__ y, int8_t* __restrict__ y8, float* __restrict__ sa8,
                                                 int iters, int rps, const float* __restrict__ amax, int qmax,
                                                 f16* __restrict__ t_out) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, lr = lane % LPR, rw = lane / LPR;
  const long wrow0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW * iters;
  // MODE 2: the sample's C scales s and 1/s, computed once per block into LDS (a block's rows lie in
  // one sample: host check rps % (4 * RPW * iters) == 0); held in registers they would cost 120 VGPRs
  extern __shared__ double lds_fq[];
  if constexpr (MODE == 2) {
    const long n = (long)blockIdx.x * 4 * RPW * iters / rps;
    float* ssc = reinterpret_cast<float*>(lds_fq + c);
    for (int j = threadIdx.x; j < c / 8; j += 256) {
      float s8[8];
      double r8[8];
      fq_scales8(amax + n * c + j * 8, qmax, s8, r8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        lds_fq[j * 8 + e] = r8[e];
        ssc[j * 8 + e] = s8[e];
      }
    }
    __syncthreads();
  }
  if (wrow0 >= rows) return;
  f16x8 g[P], b[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    g[i] = *reinterpret_cast<const f16x8*>(gamma + (lr + i * LPR) * 8);
    b[i] = *reinterpret_cast<const f16x8*>(beta + (lr + i * LPR) * 8);
  }
  for (int it = 0; it < iters; ++it) {
    const long row = wrow0 + (long)it * RPW + rw;
    const bool ok = row < rows;
    f16x8 v[P];
#pragma unroll
    for (int i = 0; i < P; ++i)
      v[i] = ok ? *reinterpret_cast<const f16x8*>(x + row * c + (lr + i * LPR) * 8) : (f16x8){};
    if constexpr (MODE == 2) {
      const float* ssc = reinterpret_cast<const float*>(lds_fq + c);
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int ch = (lr + i * LPR) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = fq_apply_r((float)v[i][e], ssc[ch + e], lds_fq[ch + e]);
        if (ok) *reinterpret_cast<f16x8*>(t_out + row * c + (lr + i * LPR) * 8) = v[i];
      }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)v[i][e];
    const float mean = group_sum<LPR>(s) / (float)c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = (float)v[i][e] - mean;
        q = fmaf(a, a, q);
      }
    const float rstd = 1.0f / sqrtf(group_sum<LPR>(q) / (float)c + eps);
    f16x8 o[P];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[i][e] = to_f16(fmaf(((float)v[i][e] - mean) * rstd, (float)g[i][e], (float)b[i][e]));
        if (MODE == 1) m = fmaxf(m, fabsf((float)o[i][e]));
      }
    if constexpr (MODE == 1) {
      const float s8 = fq_scale(group_max<LPR>(m), 127);
      const double r8 = rcp_exact(s8);
      if (ok && lr == 0) sa8[row] = s8;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        unsigned lo = 0, hi = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const f16 tq = (f16)(float)((double)(float)o[i][e] * r8);
          const unsigned qv = (unsigned)(uint8_t)(int8_t)__builtin_rintf((float)tq);
          if (e < 4) lo |= qv << (8 * e);
          else hi |= qv << (8 * (e - 4));
        }
        if (ok) *reinterpret_cast<uint2*>(y8 + row * c + (lr + i * LPR) * 8) = make_uint2(lo, hi);
      }
    } else {
#pragma unroll
      for (int i = 0; i < P; ++i)
        if (ok) *reinterpret_cast<f16x8*>(y + row * c + (lr + i * LPR) * 8) = o[i];
    }
  }
}

// (LPR, P) of the grouped-row kernel for C, or LPR = 0 (the one-row-per-wave kernels)
static void ln_rows_geom(int c, int& lpr, int& per) {
  lpr = per = 0;
  if (c % 8) return;
  const int ch = c / 8;
  for (int l = 8; l <= 64; l *= 2)
    if (ch % l == 0 && ch / l <= 5) {
      lpr = l;
      per = ch / l;
      return;
    }
}
template <int MODE>
static bool launch_ln_rows(const f16* x, long rows, int c, float eps, const f16* g, const f16* b, f16* y, int8_t* y8,
                           float* sa8, int rps, const float* amax, int qmax, f16* t_out, hipStream_t st) {
  int lpr, per;
  ln_rows_geom(c, lpr, per);
  if (!lpr) return false;
  const int rpw = 64 / lpr;
  int iters = 1;  // more rows per wave while the grid keeps >= 1024 blocks
  while (iters < 4 && (rows + 4L * rpw * iters * 2 - 1) / (4L * rpw * iters * 2) >= 1024) iters *= 2;
  if (MODE == 2) {
    while (iters > 1 && rps % (4 * rpw * iters)) iters >>= 1;
    if (rps % (4 * rpw)) return false;
  }
  const int grid = (int)((rows + 4L * rpw * iters - 1) / (4L * rpw * iters));
  const size_t lds = MODE == 2 ? (size_t)c * 12 : 0;
#define QD_LNR(L, PP)                                                                                          \
  if (lpr == L && per == PP) {                                                                                 \
    k_ln_rows<L, PP, MODE><<<grid, 256, lds, st>>>(x, rows, c, eps, g, b, y, y8, sa8, iters, rps, amax, qmax, t_out); \
    return true;                                                                                               \
  }
  QD_LNR(8, 5) QD_LNR(16, 5) QD_LNR(32, 3) QD_LNR(32, 4) QD_LNR(32, 5) QD_LNR(64, 2) QD_LNR(64, 4) QD_LNR(64, 5)
#undef QD_LNR
  return false;
}

// LayerNorm of a conv output whose per-(sample, channel) output fake-quant is still pending
// (Transformer2DModel proj_in -> BasicTransformerBlock norm1): t = fq(y; amax[n][c]) is written
// (the block's residual stream, k_finalize's arithmetic) and LayerNorm(t) (k_layernorm's) in the
// same pass, so the finalize launch and its re-read disappear.  A wave owns RPW consecutive rows
// of one sample (rows_per_sample % RPW == 0), all their loads issued together: its lanes'
// fake-quant scales are computed once per RPW rows (16 rows per wave: too few waves in flight).
constexpr int LNFQ_RPW = 4;
template <int PER, int R>
__global__ void __launch_bounds__(256) k_fq_layernorm(const f16* __restrict__ x, long rows, int c, int rps,
                                                      const float* __restrict__ amax, int qmax, float eps,
                                                      const f16* __restrict__ gamma, const f16* __restrict__ beta,
                                                      f16* __restrict__ t_out, f16* __restrict__ y) {
  const long rbeg = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * LNFQ_RPW;
  if (rbeg >= rows) return;
  const long rend = rbeg + LNFQ_RPW < rows ? rbeg + LNFQ_RPW : rows;
  const long n = rbeg / rps;
  const int lane = threadIdx.x & 63;
  const int chunks = c >> 3;
  float sc[PER][8];
  double rs[PER][8];
  f16x8 g[PER], b[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + i * 64;
    if (j < chunks) {
      fq_scales8(amax + n * c + j * 8, qmax, sc[i], rs[i]);
      g[i] = *reinterpret_cast<const f16x8*>(gamma + j * 8);
      b[i] = *reinterpret_cast<const f16x8*>(beta + j * 8);
    }
  }
  for (long row0 = rbeg; row0 < rend; row0 += R) {
    f16x8 v[R][PER];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = lane + i * 64;
        v[r][i] = (row0 + r < rend && j < chunks) ? *reinterpret_cast<const f16x8*>(x + (row0 + r) * c + j * 8)
                                                  : (f16x8){};
      }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (row0 + r >= rend) break;
      // t = fq(y): the finalized value, stored as the residual stream
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = lane + i * 64;
        if (j < chunks) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[r][i][e] = fq_apply_r((float)v[r][i][e], sc[i][e], rs[i][e]);
          *reinterpret_cast<f16x8*>(t_out + (row0 + r) * c + j * 8) = v[r][i];
        }
      }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += (float)v[r][i][e];
      const float mean = wave_sum(s) / (float)c;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        if (lane + i * 64 < chunks) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float a = (float)v[r][i][e] - mean;
            q = fmaf(a, a, q);
          }
        }
      }
      const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)c + eps);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int j = lane + i * 64;
        if (j < chunks) {
          f16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = to_f16(fmaf(((float)v[r][i][e] - mean) * rstd, (float)g[i][e], (float)b[i][e]));
          *reinterpret_cast<f16x8*>(y + (row0 + r) * c + j * 8) = o;
        }
      }
    }
  }
}

extern "C" int qd_layernorm_fq(const void* x, const float* amax, int n_bits, int rows, int rows_per_sample, int c,
                               float eps, const void* gamma, const void* beta, void* t_out, void* y, void* stream) {
  QD_REQUIRE(x && amax && gamma && beta && t_out && y, "null pointer");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "bad n_bits");
  QD_REQUIRE(c % 8 == 0 && c <= 2048, "LayerNorm-fq needs C % 8 == 0, C <= 2048");
  QD_REQUIRE(rows_per_sample > 0 && rows_per_sample % LNFQ_RPW == 0 && rows % rows_per_sample == 0,
             "LayerNorm-fq needs rows_per_sample % 4 == 0 and whole samples");
  QD_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(t_out) |
               reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
               reinterpret_cast<uintptr_t>(amax)) & 15) == 0, "LayerNorm-fq operands must be 16-B aligned");
  if (rows == 0) return 0;
  const int per = (c / 8 + 63) / 64;
  const int grid = (int)((rows + 4L * LNFQ_RPW - 1) / (4L * LNFQ_RPW));
  const int qm = (1 << (n_bits - 1)) - 1;
  hipStream_t st = S(stream);
  const f16 *xp = (const f16*)x, *g = (const f16*)gamma, *b = (const f16*)beta;
  if (launch_ln_rows<2>(xp, rows, c, eps, g, b, (f16*)y, nullptr, nullptr, rows_per_sample, amax, qm, (f16*)t_out, st)) {
    QD_CHECK_LAUNCH();
    return 0;
  }
#define QD_LNFQ(P, RR) \
  k_fq_layernorm<P, RR><<<grid, 256, 0, st>>>(xp, rows, c, rows_per_sample, amax, qm, eps, g, b, (f16*)t_out, (f16*)y)
  if (per <= 1) QD_LNFQ(1, 4);
  else if (per <= 2) QD_LNFQ(2, 4);
  else QD_LNFQ(4, 2);
#undef QD_LNFQ
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_layernorm_i8(const void* x, int rows, int c, float eps, const void* gamma, const void* beta,
                               int8_t* y8, float* scales, void* stream) {
  QD_REQUIRE(x && gamma && beta && y8 && scales, "null pointer");
  QD_REQUIRE(c % 8 == 0 && c <= 4096, "LayerNorm needs C % 8 == 0, C <= 4096");
  QD_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta)) &
              15) == 0 && (reinterpret_cast<uintptr_t>(y8) & 7) == 0, "LayerNorm operands must be aligned");
  if (rows == 0) return 0;
  const int per = (c / 8 + 63) / 64;
  hipStream_t st = S(stream);
  const f16 *xp = (const f16*)x, *g = (const f16*)gamma, *b = (const f16*)beta;
  if (launch_ln_rows<1>(xp, rows, c, eps, g, b, nullptr, y8, scales, 0, nullptr, 0, nullptr, st)) {
    QD_CHECK_LAUNCH();
    return 0;
  }
  if (per <= 1) launch_ln<1, true>(xp, rows, c, eps, g, b, nullptr, st, y8, scales);
  else if (per <= 2) launch_ln<2, true>(xp, rows, c, eps, g, b, nullptr, st, y8, scales);
  else if (per <= 3) launch_ln<3, true>(xp, rows, c, eps, g, b, nullptr, st, y8, scales);
  else if (per <= 4) launch_ln<4, true>(xp, rows, c, eps, g, b, nullptr, st, y8, scales);
  else launch_ln<8, true>(xp, rows, c, eps, g, b, nullptr, st, y8, scales);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_layernorm(const void* x, int rows, int c, float eps, const void* gamma,
                            const void* beta, void* y, void* stream) {
  QD_REQUIRE(x && gamma && beta && y, "null pointer");
  QD_REQUIRE(c % 8 == 0 && c <= 4096, "LayerNorm needs C % 8 == 0, C <= 4096");
  QD_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gamma) |
               reinterpret_cast<uintptr_t>(beta)) & 15) == 0, "LayerNorm operands must be 16-B aligned");
  if (rows == 0) return 0;
  const int per = (c / 8 + 63) / 64;
  hipStream_t st = S(stream);
  const f16 *xp = (const f16*)x, *g = (const f16*)gamma, *b = (const f16*)beta;
  f16* yp = (f16*)y;
  if (launch_ln_rows<0>(xp, rows, c, eps, g, b, yp, nullptr, nullptr, 0, nullptr, 0, nullptr, st)) {
    QD_CHECK_LAUNCH();
    return 0;
  }
  if (per <= 1) launch_ln<1>(xp, rows, c, eps, g, b, yp, st);
  else if (per <= 2) launch_ln<2>(xp, rows, c, eps, g, b, yp, st);
  else if (per <= 3) launch_ln<3>(xp, rows, c, eps, g, b, yp, st);
  else if (per <= 4) launch_ln<4>(xp, rows, c, eps, g, b, yp, st);
  else launch_ln<8>(xp, rows, c, eps, g, b, yp, st);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// GEGLU, SiLU, add, concat, layout transposes
// ---------------------------------------------------------------------------------------
__global__ void k_geglu(const f16* __restrict__ h, long m, int inner, f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // index into out (pairs)
  const long total = m * inner / 2;
  if (e >= total) return;
  const long row = (2 * e) / inner;
  const int col = (int)((2 * e) % inner);
  const __half2 a = *reinterpret_cast<const __half2*>(h + row * 2 * inner + col);
  const __half2 g = *reinterpret_cast<const __half2*>(h + row * 2 * inner + inner + col);
  const f16 g0 = (f16)gelu_f(__low2float(g)), g1 = (f16)gelu_f(__high2float(g));
  const f16 o0 = (f16)(__low2float(a) * (float)g0), o1 = (f16)(__high2float(a) * (float)g1);
  f16* dst = out + row * inner + col;
  dst[0] = o0;
  dst[1] = o1;
}

extern "C" int qd_geglu(const void* h, int m, int inner, void* out, void* stream) {
  QD_REQUIRE(h && out && inner % 2 == 0, "bad geglu args");
  const long total = (long)m * inner / 2;
  if (total == 0) return 0;
  k_geglu<<<grid1(total), 256, 0, S(stream)>>>((const f16*)h, m, inner, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

__global__ void k_silu(const f16* __restrict__ x, f16* __restrict__ y, long count) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e < count) y[e] = to_f16(silu_f((float)x[e]));
}

extern "C" int qd_silu(const void* x, void* y, int64_t count, void* stream) {
  QD_REQUIRE(x && y, "null pointer");
  if (count == 0) return 0;
  k_silu<<<grid1(count), 256, 0, S(stream)>>>((const f16*)x, (f16*)y, count);
  QD_CHECK_LAUNCH();
  return 0;
}

__global__ void k_add(const f16* __restrict__ a, const f16* __restrict__ b, f16* __restrict__ y, long count) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e < count) y[e] = (f16)((float)a[e] + (float)b[e]);
}

extern "C" int qd_add(const void* a, const void* b, void* y, int64_t count, void* stream) {
  QD_REQUIRE(a && b && y, "null pointer");
  if (count == 0) return 0;
  k_add<<<grid1(count), 256, 0, S(stream)>>>((const f16*)a, (const f16*)b, (f16*)y, count);
  QD_CHECK_LAUNCH();
  return 0;
}

// 16-B chunks (c1, c2 multiples of 8)
__global__ void k_concat(const f16* __restrict__ a, int c1, const f16* __restrict__ b, int c2, long m,
                         f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const int cc = (c1 + c2) >> 3;
  if (e >= m * cc) return;
  const long r = e / cc;
  const int ch = (int)(e - r * cc) * 8;
  const f16* src = ch < c1 ? a + r * c1 + ch : b + r * c2 + ch - c1;
  *reinterpret_cast<f16x8*>(out + e * 8) = *reinterpret_cast<const f16x8*>(src);
}

extern "C" int qd_concat_c(const void* a, int c1, const void* b, int c2, int64_t m, void* out, void* stream) {
  QD_REQUIRE(a && b && out, "null pointer");
  QD_REQUIRE(c1 % 8 == 0 && c2 % 8 == 0, "concat needs both widths to be multiples of 8");
  if (m == 0) return 0;
  k_concat<<<grid1(m * ((c1 + c2) / 8)), 256, 0, S(stream)>>>((const f16*)a, c1, (const f16*)b, c2, m, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// 64x64 tiled transpose through LDS: [N][C][HW] <-> [N][HW][Cp]
__global__ void k_nchw_to_nhwc(const f16* __restrict__ x, int c, int hw, int cp, f16* __restrict__ y) {
  __shared__ f16 tile[64][65];
  const int n = blockIdx.z;
  const int c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
  const f16* xs = x + (long)n * c * hw;
  f16* ys = y + (long)n * hw * cp;
  for (int i = threadIdx.y; i < 64; i += 4) {
    const int ch = c0 + i, p = p0 + threadIdx.x;
    tile[i][threadIdx.x] = (ch < c && p < hw) ? xs[(long)ch * hw + p] : (f16)0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 64; i += 4) {
    const int p = p0 + i, ch = c0 + threadIdx.x;
    if (p < hw && ch < cp) ys[(long)p * cp + ch] = tile[threadIdx.x][i];
  }
}

__global__ void k_nhwc_to_nchw(const f16* __restrict__ x, int c, int hw, int cp, f16* __restrict__ y) {
  __shared__ f16 tile[64][65];
  const int n = blockIdx.z;
  const int c0 = blockIdx.y * 64, p0 = blockIdx.x * 64;
  const f16* xs = x + (long)n * hw * cp;
  f16* ys = y + (long)n * c * hw;
  for (int i = threadIdx.y; i < 64; i += 4) {
    const int p = p0 + i, ch = c0 + threadIdx.x;
    tile[i][threadIdx.x] = (p < hw && ch < c) ? xs[(long)p * cp + ch] : (f16)0.f;
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 64; i += 4) {
    const int ch = c0 + i, p = p0 + threadIdx.x;
    if (ch < c && p < hw) ys[(long)ch * hw + p] = tile[threadIdx.x][i];
  }
}

extern "C" int qd_nchw_to_nhwc(const void* x, int n, int c, int hw, int c_pad, void* y, void* stream) {
  QD_REQUIRE(x && y && c_pad >= c, "bad args");
  if ((long)n * hw == 0) return 0;
  dim3 grid((hw + 63) / 64, (c_pad + 63) / 64, n);
  k_nchw_to_nhwc<<<grid, dim3(64, 4), 0, S(stream)>>>((const f16*)x, c, hw, c_pad, (f16*)y);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_nhwc_to_nchw(const void* x, int n, int c, int hw, int c_pad, void* y, void* stream) {
  QD_REQUIRE(x && y && c_pad >= c, "bad args");
  if ((long)n * hw == 0) return 0;
  dim3 grid((hw + 63) / 64, (c + 63) / 64, n);
  k_nhwc_to_nchw<<<grid, dim3(64, 4), 0, S(stream)>>>((const f16*)x, c, hw, c_pad, (f16*)y);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// diffusers Timesteps / get_timestep_embedding (max_period 10000, scale 1)
// ---------------------------------------------------------------------------------------
__global__ void k_temb(const float* __restrict__ ts, const int* __restrict__ step_idx, int b, int dim,
                       int flip, float shift, f16* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int half_dim = dim / 2;
  if (i >= b * half_dim) return;
  const int row = i / half_dim, k = i % half_dim;
  // flip bit 1: row r embeds ts[r] (SDXL add_time_proj over the flattened time_ids)
  const float t = (flip & 2) ? ts[row] : ts[step_idx ? step_idx[0] : 0];
  flip &= 1;
  const float ex = (-9.210340371976184f * (float)k) / ((float)half_dim - shift);  // -ln(1e4)*k/(h-s)
  const float arg = t * expf(ex);
  const float sv = sinf(arg), cv = cosf(arg);
  f16* o = out + (long)row * dim;
  if (flip) {
    o[k] = (f16)cv;
    o[half_dim + k] = (f16)sv;
  } else {
    o[k] = (f16)sv;
    o[half_dim + k] = (f16)cv;
  }
}

extern "C" int qd_timestep_embedding(const float* timesteps, const int* step_idx, int b, int dim,
                                     int flip_sin_to_cos, float shift, void* out, void* stream) {
  QD_REQUIRE(timesteps && out && dim % 2 == 0, "bad args");
  k_temb<<<grid1((long)b * dim / 2), 256, 0, S(stream)>>>(timesteps, step_idx, b, dim, flip_sin_to_cos,
                                                          shift, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// CFG combine + DDIM step (eta = 0), diffusers op order with fp16 rounding per torch op:
//   eps  = u + g * (c - u)                       pipeline_stable_diffusion.py (CFG)
//   x0   = (x - sqrt(1 - a_t) * eps) / sqrt(a_t) DDIMScheduler.step
//   prev = sqrt(a_prev) * x0 + sqrt(1 - a_prev) * eps
// torch-CPU Half semantics, measured (tests/test_gpu_kernels.py pins them against torch):
//   python-float * half  -> half(float(g) * x)            (scalar kept in fp32)
//   0-d fp32 tensor * half -> half(float(half(s)) * x)    (scalar first cast to fp16)
//   half / 0-d fp32 tensor -> half(x / s)                 (scalar kept in fp32)
// latents / unet_out are NHWC with c_pad channel stride (only c used); next_in = [x; x].
// ---------------------------------------------------------------------------------------
__global__ void k_cfg_ddim(f16* __restrict__ lat, const f16* __restrict__ uo, int b, long l, float g,
                           const float* __restrict__ at, const float* __restrict__ ap,
                           const int* __restrict__ step_idx, f16* __restrict__ next_in, int c, int cp) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // over b * l (l = pixels * cp)
  if (e >= (long)b * l) return;
  const int ch = e % cp;
  const int si = step_idx[0];
  const float a_t = at[si], a_p = ap[si];
  f16 out;
  if (ch < c) {
    const long bi = e / l, off = e % l;
    const float u = (float)uo[bi * l + off];
    const float cc = (float)uo[((long)b + bi) * l + off];
    const f16 diff = (f16)(cc - u);
    const f16 gd = (f16)(g * (float)diff);
    const f16 eps = (f16)(u + (float)gd);
    const float sb = (float)(f16)sqrtf(1.0f - a_t);   // beta_prod_t ** 0.5 (0-d tensor, cast for *)
    const float sa = sqrtf(a_t);                      // alpha_prod_t ** 0.5 (divisor, fp32)
    const f16 t1 = (f16)(sb * (float)eps);
    const f16 t2 = (f16)((float)lat[e] - (float)t1);
    const f16 x0 = (f16)((float)t2 / sa);
    const float sd = (float)(f16)sqrtf(1.0f - a_p);
    const float sp = (float)(f16)sqrtf(a_p);
    const f16 dir = (f16)(sd * (float)eps);
    const f16 t3 = (f16)(sp * (float)x0);
    out = (f16)((float)t3 + (float)dir);
  } else {
    out = (f16)0.f;
  }
  lat[e] = out;
  if (next_in) {
    next_in[e] = out;
    next_in[(long)b * l + e] = out;
  }
}

__global__ void k_step_inc(int* step_idx) { step_idx[0] += 1; }

// ---------------------------------------------------------------------------------------
// CFG combine + PNDMScheduler.step with skip_prk_steps (the PLMS branch, step_plms) - the SD1.5
// checkpoint's own scheduler (scheduler_config.json), which the reference's generate() runs
// (models/base.py:848).  The multistep history ets (<= 4 past noise predictions) lives in a
// device ring of 4 [B, L] slots, cur_sample in one more; the branch is taken from the device step
// counter, so one graph replays every step.  Host tables give per step the (possibly shifted)
// timestep's alpha_t and the previous one's alpha_prev (counter 1 re-evaluates the first step:
// timestep + ratio -> timestep).  Op order / torch-CPU Half scalar semantics as k_cfg_ddim:
//   i == 0 : ets = [e]; mo = e; cur = x
//   i == 1 : mo = (e + ets[-1]) / 2; x = cur                      (ets unchanged)
//   i >= 2 : ets.append(e) (last 4 kept); len 2: (3 e1 - e0) / 2; len 3: (23 e2 - 16 e1 + 5 e0) / 12;
//            len 4: (1 / 24) * (55 e3 - 59 e2 + 37 e1 - 9 e0)
//   prev = sc * x - (a_prev - a_t) * mo / denom,  sc = (a_prev / a_t) ** 0.5,
//   denom = a_t * (1 - a_prev) ** 0.5 + (a_t * (1 - a_t) * a_prev) ** 0.5      (0-d fp32 scalars)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ f16 h_mul(float s, f16 x) { return (f16)(s * (float)x); }
__device__ __forceinline__ f16 h_sub(f16 a, f16 b) { return (f16)((float)a - (float)b); }
__device__ __forceinline__ f16 h_add(f16 a, f16 b) { return (f16)((float)a + (float)b); }

__global__ void k_cfg_pndm(f16* __restrict__ lat, const f16* __restrict__ uo, int b, long l, float g,
                           const float* __restrict__ at, const float* __restrict__ ap,
                           const int* __restrict__ step_idx, f16* __restrict__ ets, f16* __restrict__ cur,
                           f16* __restrict__ next_in, int c, int cp) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // over b * l
  const long bl = (long)b * l;
  if (e >= bl) return;
  const int ch = e % cp;
  const int si = step_idx[0];
  f16 out = (f16)0.f;
  if (ch < c) {
    const long bi = e / l, off = e % l;
    const float u = (float)uo[bi * l + off];
    const float cc = (float)uo[((long)b + bi) * l + off];
    const f16 gd = (f16)(g * (float)(f16)(cc - u));
    const f16 eps = (f16)(u + (float)gd);
    f16 x = lat[e], mo;
    if (si == 0) {
      ets[e] = eps;
      cur[e] = x;
      mo = eps;
    } else if (si == 1) {
      mo = (f16)((float)h_add(eps, ets[e]) / 2.0f);
      x = cur[e];
    } else {
      const int k = si - 1;  // append index of this step's eps (step 0 was append 0)
      ets[(long)(k & 3) * bl + e] = eps;
      const f16 e1 = eps;
      const f16 e0 = ets[(long)((k - 1) & 3) * bl + e];
      if (si == 2) {
        mo = (f16)((float)h_sub(h_mul(3.f, e1), e0) / 2.0f);
      } else if (si == 3) {
        const f16 em = ets[(long)((k - 2) & 3) * bl + e];  // ets[-3]
        // (23 * e[-1] - 16 * e[-2] + 5 * e[-3]) / 12
        mo = (f16)((float)h_add(h_sub(h_mul(23.f, e1), h_mul(16.f, e0)), h_mul(5.f, em)) / 12.0f);
      } else {
        const f16 em = ets[(long)((k - 2) & 3) * bl + e], en = ets[(long)((k - 3) & 3) * bl + e];
        const f16 sum = h_sub(h_add(h_sub(h_mul(55.f, e1), h_mul(59.f, e0)), h_mul(37.f, em)), h_mul(9.f, en));
        mo = h_mul((float)(1.0 / 24.0), sum);
      }
    }
    const float a_t = at[si], a_p = ap[si];
    const float sc = (float)(f16)sqrtf(a_p / a_t);                        // 0-d * half: scalar -> fp16
    const float denom = a_t * sqrtf(1.0f - a_p) + sqrtf(a_t * (1.0f - a_t) * a_p);
    const f16 t1 = (f16)(sc * (float)x);
    const f16 t2 = (f16)((float)(f16)(a_p - a_t) * (float)mo);
    const f16 t3 = (f16)((float)t2 / denom);                               // half / 0-d: scalar fp32
    out = (f16)((float)t1 - (float)t3);
  }
  lat[e] = out;
  if (next_in) {
    next_in[e] = out;
    next_in[bl + e] = out;
  }
}

extern "C" int qd_cfg_pndm_step(void* latents, const void* unet_out, int b, int64_t l, float guidance,
                                const float* alpha_t, const float* alpha_prev, int* step_idx, void* ets, void* cur,
                                void* next_in, int c, int c_pad, void* stream) {
  QD_REQUIRE(latents && unet_out && alpha_t && alpha_prev && step_idx && ets && cur, "null pointer");
  QD_REQUIRE(c_pad >= c && l % c_pad == 0, "bad channel padding");
  hipStream_t st = S(stream);
  k_cfg_pndm<<<grid1((long)b * l), 256, 0, st>>>((f16*)latents, (const f16*)unet_out, b, l, guidance, alpha_t,
                                                 alpha_prev, step_idx, (f16*)ets, (f16*)cur, (f16*)next_in, c, c_pad);
  k_step_inc<<<1, 1, 0, st>>>(step_idx);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// CFG + EulerDiscreteScheduler.step (epsilon prediction, s_churn = 0) and the next step's
// scale_model_input, in diffusers' op order with the torch-CPU scalar semantics above:
//   eps   = u + g * (c - u)                                (fp16 ops)
//   x     = float(latents)                                 (sample.to(float32))
//   pred  = x - float(half(half(sigma) * eps))             (0-d sigma_hat first operand: fp16)
//   deriv = (x - pred) / sigma ; prev = x + deriv * (sigma_next - sigma)    (fp32)
//   lat   = half(prev) ; next_in = half(float(lat) / dscale[i + 1]) for both CFG halves
// dscale[i] = (sigma_i ** 2 + 1) ** 0.5 (fp32, host table: scale_model_input's divisor).
// ---------------------------------------------------------------------------------------
__global__ void k_cfg_euler_discrete(f16* __restrict__ lat, const f16* __restrict__ uo, int b, long l, float g,
                                     const float* __restrict__ sig, const float* __restrict__ dsc,
                                     const int* __restrict__ step_idx, f16* __restrict__ next_in, int c, int cp) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)b * l) return;
  const int ch = e % cp;
  const int si = step_idx[0];
  f16 out = (f16)0.f;
  if (ch < c) {
    const long bi = e / l, off = e % l;
    const float u = (float)uo[bi * l + off];
    const float cc = (float)uo[((long)b + bi) * l + off];
    const f16 diff = (f16)(cc - u);
    const f16 gd = (f16)(g * (float)diff);
    const f16 eps = (f16)(u + (float)gd);
    const float sigma = sig[si];
    const float x = (float)lat[e];
    const float pred = x - (float)(f16)((float)(f16)sigma * (float)eps);
    const float deriv = (x - pred) / sigma;
    const float prev = x + deriv * (sig[si + 1] - sigma);
    out = (f16)prev;
  }
  lat[e] = out;
  if (next_in) {
    const f16 sc = ch < c ? (f16)((float)out / dsc[si + 1]) : (f16)0.f;
    next_in[e] = sc;
    next_in[(long)b * l + e] = sc;
  }
}

extern "C" int qd_cfg_euler_discrete_step(void* latents, const void* unet_out, int b, int64_t l, float guidance,
                                          const float* sigmas, const float* dscale, int* step_idx, void* next_in,
                                          int c, int c_pad, void* stream) {
  QD_REQUIRE(latents && unet_out && sigmas && dscale && step_idx, "null pointer");
  QD_REQUIRE(c_pad >= c && l % c_pad == 0, "bad channel padding");
  hipStream_t st = S(stream);
  k_cfg_euler_discrete<<<grid1((long)b * l), 256, 0, st>>>((f16*)latents, (const f16*)unet_out, b, l, guidance,
                                                           sigmas, dscale, step_idx, (f16*)next_in, c, c_pad);
  k_step_inc<<<1, 1, 0, st>>>(step_idx);
  QD_CHECK_LAUNCH();
  return 0;
}

// x = half(float(x) * mul) then (optional) y = half(float(x) / div) into both CFG halves of y:
// EulerDiscrete prepare_latents (latents * init_noise_sigma, a 0-d fp32 second operand) and the
// first step's scale_model_input.  Channels >= c (padding) stay zero.
__global__ void k_scale_latents(f16* __restrict__ x, long n, float mul, float div, long half_off,
                                f16* __restrict__ y, int c, int cp) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const bool ok = (e % cp) < c;
  const f16 v = ok ? (f16)((float)x[e] * mul) : (f16)0.f;
  x[e] = v;
  if (y) {
    const f16 s = ok ? (f16)((float)v / div) : (f16)0.f;
    y[e] = s;
    y[half_off + e] = s;
  }
}

extern "C" int qd_scale_latents(void* latents, int64_t n, float mul, float div, void* next_in, int c, int c_pad,
                                void* stream) {
  QD_REQUIRE(latents && c_pad >= c && n % c_pad == 0, "bad args");
  if (n == 0) return 0;
  k_scale_latents<<<grid1(n), 256, 0, S(stream)>>>((f16*)latents, n, mul, div, n, (f16*)next_in, c, c_pad);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_cfg_ddim_step(void* latents, const void* unet_out, int b, int64_t l, float guidance,
                                const float* alpha_t, const float* alpha_prev, int* step_idx,
                                void* next_in, int c, int c_pad, void* stream) {
  QD_REQUIRE(latents && unet_out && alpha_t && alpha_prev && step_idx, "null pointer");
  QD_REQUIRE(c_pad >= c && l % c_pad == 0, "bad channel padding");
  hipStream_t st = S(stream);
  k_cfg_ddim<<<grid1((long)b * l), 256, 0, st>>>((f16*)latents, (const f16*)unet_out, b, l, guidance,
                                                 alpha_t, alpha_prev, step_idx, (f16*)next_in, c, c_pad);
  k_step_inc<<<1, 1, 0, st>>>(step_idx);
  QD_CHECK_LAUNCH();
  return 0;
}
