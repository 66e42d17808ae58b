// Fake-quant GEMMs on CDNA4 MFMA: the F.linear / F.conv2d of WxAxLinear / WxAxConv2d
// (quantize/fake_quant.py:223, 339) as ONE tiled kernel family.
//
//   C[M, N] = A[M, K] . B[N, K]^T, fp16 operands, fp32 accumulation (v_mfma_f32_16x16x32_f16)
//
// A operand: LINEAR    - activations [M][lda] (K contiguous)
//            CONV      - implicit im2col of an NHWC activation, K ordered (kh, kw, ci); rows are
//                        output pixels (n, oh, ow).  Ci_pad % 64 == 0: a 64-deep K step lies in
//                        one filter tap, decoded once per step in scalar registers.
//            CONV_ANY  - same, any Ci_pad (per-chunk decode; the 4-channel conv_in)
//            Padding / stride / nearest-2x upsample are resolved in the A address (no im2col).
// B operand: the quantized weight [N][K]: fp16 (dequantized), or int8 / packed-int4 codes +
//            fp16 group scales, dequantized in registers while staging into LDS
//            (w = half(q * s), bit-identical to the reference's stored buffer).
// Epilogue:  + bias, round to fp16 (the fp16 output of F.linear / F.conv2d), [+ residual],
//            [per-(sample, col) amax for the conv output fake-quant: lane-shuffle reduction
//            then one atomic per column per wave tile].
//
// Structure (MI355X): 256 threads = 2 x 2 waves, block tile BM x BN x 64, wave tile
// (BM/2) x (BN/2).  Each wave computes C^T tiles (MFMA A = weight fragment, B = activation
// fragment), so a lane ends with 4 consecutive output columns of one row (8-B bias vectors,
// column amax by 16-lane shuffles); the fp16 tile is then re-read from LDS in 16-B row chunks
// for fully coalesced residual loads and stores.  All global operand loads are raw buffer loads whose invalid
// chunks (rows past M/N, halo of the conv, K tail) carry an offset >= 2^31 and read zero:
// the staging path has no branches and the next K step's loads stay in flight while the
// current step's MFMAs run (register-staged, LDS double-buffered, one barrier per step).
// LDS 16-B chunks XOR-swizzled by (row & 7).  Blocks are remapped so each XCD gets a
// contiguous run of tiles (L2 reuse).  Small-M shapes split K (fp32 partial slabs in a caller
// workspace + a fixed-order reduction kernel that runs the same epilogue: deterministic).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

enum { AM_LINEAR = 0, AM_CONV = 1, AM_CONV_ANY = 2 };

struct GemmArgs {
  const f16* a;
  int lda;
  const void* b;
  const f16* bscale;
  const f16* bscale_t;  // the same group scales as [K / group][N] (int4 LDS-DMA families), or null
  int group;
  const f16* bias;
  const f16* res;
  f16* y;
  int ldy;
  float* amax;
  int rows_per_sample;
  int M, N, K;
  // conv geometry
  int H, W, Hs, Ws, Cip, Ho, Wo, kh, kw, stride, pad, ups;  // H, W: logical (post-upsample) input
  int epi;
  // split-K
  float* part;
  int splits, kps;  // K per split (multiple of 64)
  unsigned a_bytes, b_bytes;
  // int8 x int8 path (qd_linear_i8 / qd_conv2d_i8): A and B are int8 codes addressed through a
  // "half view" (K, lda and Cip halved: two codes per fp16 slot), so the LDS-DMA loaders move
  // them unchanged; the MFMA is v_mfma_i32_16x16x64_i8 and the int32 sums are scaled in the
  // epilogue: y = half(((float)acc * sa[row]) * sw[col] + bias).  Split-K slabs hold the int32
  // partial sums (exact), so every tile / split choice gives bit-identical outputs.
  const float* sa;  // activation scale per row (sa_rps == 0) or per sa_rps consecutive rows
  int sa_rps;
  const float* sw;  // weight scale per output column (16-B aligned)
  int i8;
  // fp8 path (qd_linear_fp8, SD3.5's W4A8-fp8 mode): A = per-token e4m3 activation codes, B = the
  // W4 codes as e4m3 (integers -8..7, exact), both through the half view; one 128-code K group
  // per LDS stage = one v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales); the group's fp32
  // weight scales gs[k / 128][n] ride in the stage (LDS-DMA) and scale the MFMA result before it
  // is added to the accumulator; the row's activation scale sa[m] multiplies the sum.
  const float* gs;
  int f8;
  // GroupNorm-statistics epilogue (QD_EPI_GNSTATS) and the per-(sample, column) add (QD_EPI_CADD):
  // the int8-MFMA mode's producing convs hand their consumer GroupNorm (norm.hip k_gn_coeff<1>) the
  // moments of each 64-row slot of the final output, gnp[slot][col] = (mean, M2, min, max)
  const f16* cadd;
  int cadd_ld;
  float* gnp;
  // block order (tile_of): 0 = split fastest, then N tiles (one XCD's blocks share A rows); 1 = M
  // tiles fastest (one XCD's blocks share a weight slice) - set by the host when the weights are
  // the larger operand (the low UNet levels: 1280 x 11520 weights against 2048 x 1280 activations)
  int mfast;
  // row-complete LayerNorm epilogue (QD_EPI_LN; BN == N tiles, unsplit, residual path): LayerNorm of
  // each final output row read back from the LDS tile - fp16 into ln_y [M][N], or the int8 codes
  // ln_y8 [M][N] + per-row scales ln_sa8 [M] (norm.hip k_ln_rows MODE 0 / 1 arithmetic)
  const f16* ln_g;
  const f16* ln_b;
  float ln_eps;
  f16* ln_y;
  int8_t* ln_y8;
  float* ln_sa8;
  // conv output fake-quant + residual / per-sample add fused into the split-K reduction
  // (qd_conv2d_fq): requested with fq_qmax > 0; run_gemm sets fq_done when its plan split K and
  // the reduction finalized the output (else the caller launches qd_fq_finalize)
  int fq_qmax;
  const f16* fq_cadd;
  int fq_cadd_ld;
  int fq_done;
  float* fq_xamax;  // optional: the finalized output's per-(n, c) max |x| (its consumer conv's amax)
  // epilogue form (measurement knob qd_gemm_epi_direct): 0 = stores straight from the MFMA fragments
  // (permlane16 pairs -> 16-B stores) wherever the epilogue allows it; 1 = always through the LDS C tile
  int epi_lds;
  // persistent int8 LDS-DMA linears (qd_gemm_force 160+ / 170+): the launch's block count; each block
  // runs logical tiles bid, bid + grid, ... and stages the next tile's first K steps under the
  // current tile's epilogue whenever that epilogue stores straight from the fragments (no LDS)
  int pgrid;
  // A-stationary int8 linears (k_gemm_as_i8): N-tile ranges per A panel
  int as_nsplit;
};

constexpr int BK = 64;
constexpr unsigned OOB = 0x80000000u;

// block (XCD-remapped index wg) -> (M tile, N tile, K split); see GemmArgs::mfast
__device__ __forceinline__ void tile_of(const GemmArgs& p, int wg, int nbm, int nbn, int& bm, int& bn, int& split) {
  if (p.mfast) {
    bm = wg % nbm;
    const int r = wg / nbm;
    split = r % p.splits;
    bn = r / p.splits;
  } else {
    const int tile = wg / p.splits;
    split = wg - tile * p.splits;
    bm = tile / nbn;
    bn = tile - bm * nbn;
  }
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f16x8 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ int4 bload_i4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// ---- A staging ------------------------------------------------------------------------
// thread t stages rows (t >> 3) + 32 j, 16-B chunk t & 7 of the 64-deep K step
template <int BM, int AMODE>
struct ALoader {
  static constexpr int CH = BM * BK / 8 / 256;
  f16x8 r[CH];
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[CH];   // LINEAR: byte offset of the row (OOB if row >= M)
  int pix[CH];           // CONV: n * Hs * Ws (-1 if row >= M)
  int ih0[CH], iw0[CH];
  // CONV: scalar decode of the current K step: filter tap (ky, kx), first channel ci0
  int ky, kx, ci0;

  __device__ void init(const GemmArgs& p, int m0, int kbeg) {
    rs = rsrc(p.a, p.a_bytes);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int m = m0 + (t >> 3) + 32 * j;
      const bool ok = m < p.M;
      if (AMODE == AM_LINEAR) {
        rowoff[j] = ok ? (unsigned)m * (unsigned)p.lda * 2u : OOB;
      } else {
        const int mm = ok ? m : 0;
        const int ow = mm % p.Wo, oh = (mm / p.Wo) % p.Ho, n = mm / (p.Wo * p.Ho);
        pix[j] = ok ? n * p.Hs * p.Ws : -1;
        ih0[j] = oh * p.stride - p.pad;
        iw0[j] = ow * p.stride - p.pad;
      }
    }
    if (AMODE == AM_CONV) {
      const int kpos = kbeg / p.Cip;
      ci0 = kbeg - kpos * p.Cip;
      ky = kpos / p.kw;
      kx = kpos - ky * p.kw;
    }
  }

  __device__ __forceinline__ unsigned conv_off(const GemmArgs& p, int j, int kyy, int kxx, int ci) const {
    const int ih = ih0[j] + kyy, iw = iw0[j] + kxx;
    const bool ok = pix[j] >= 0 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
    return ok ? (unsigned)((pix[j] + sh * p.Ws + sw) * p.Cip + ci) * 2u : OOB;
  }

  __device__ void load(const GemmArgs& p, int k0) {
    const int kc = (threadIdx.x & 7) * 8;
    if (AMODE == AM_LINEAR) {
      const unsigned ko = k0 + kc < p.K ? (unsigned)(k0 + kc) * 2u : OOB;
#pragma unroll
      for (int j = 0; j < CH; ++j) r[j] = bload(rs, rowoff[j] + ko);
    } else if (AMODE == AM_CONV) {
#pragma unroll
      for (int j = 0; j < CH; ++j) r[j] = bload(rs, conv_off(p, j, ky, kx, ci0 + kc));
      // advance the scalar decode to the next K step (Cip % 64 == 0)
      ci0 += BK;
      if (ci0 == p.Cip) {
        ci0 = 0;
        if (++kx == p.kw) {
          kx = 0;
          ++ky;
        }
      }
    } else {
      const int k = k0 + kc;
      const int kpos = k / p.Cip, ci = k - kpos * p.Cip;
      const int kyy = kpos / p.kw, kxx = kpos - kyy * p.kw;
#pragma unroll
      for (int j = 0; j < CH; ++j) r[j] = bload(rs, k < p.K ? conv_off(p, j, kyy, kxx, ci) : OOB);
    }
  }

  __device__ void store(f16* lds) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CH; ++j) *reinterpret_cast<f16x8*>(lds + swz((t >> 3) + 32 * j, t & 7)) = r[j];
  }
};

// ---- B staging ------------------------------------------------------------------------
template <int BN, int BFMT>
struct BLoader;

template <int BN>
struct BLoader<BN, QD_WFMT_F16> {
  static constexpr int CH = BN * BK / 8 / 256;
  f16x8 r[CH];
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[CH];
  __device__ void init(const GemmArgs& p, int n0) {
    rs = rsrc(p.b, p.b_bytes);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int n = n0 + (t >> 3) + 32 * j;
      rowoff[j] = n < p.N ? (unsigned)n * (unsigned)p.K * 2u : OOB;
    }
  }
  __device__ void load(const GemmArgs& p, int k0) {
    const int k = k0 + (threadIdx.x & 7) * 8;
    const unsigned ko = k < p.K ? (unsigned)k * 2u : OOB;
#pragma unroll
    for (int j = 0; j < CH; ++j) r[j] = bload(rs, rowoff[j] + ko);
  }
  __device__ void store(f16* lds) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CH; ++j) *reinterpret_cast<f16x8*>(lds + swz((t >> 3) + 32 * j, t & 7)) = r[j];
  }
};

// int8 codes: a 16-B load = 16 codes = 2 LDS chunks; thread -> (row (t >> 2) + 64 j, quarter t & 3)
template <int BN>
struct BLoader<BN, QD_WFMT_I8> {
  static constexpr int LOADS = (BN * BK / 16 + 255) / 256;
  int4 r[LOADS];
  float s[LOADS];
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[LOADS];
  int srow[LOADS];
  __device__ void init(const GemmArgs& p, int n0) {
    rs = rsrc(p.b, p.b_bytes);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int n = n0 + (t >> 2) + 64 * j;
      rowoff[j] = n < p.N ? (unsigned)n * (unsigned)p.K : OOB;
      srow[j] = (n < p.N ? n : p.N - 1) * (p.K / p.group);
    }
  }
  __device__ void load(const GemmArgs& p, int k0) {
    const int k = k0 + (threadIdx.x & 3) * 16;  // K % 64 == 0 for quantized weights
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      r[j] = bload_i4(rs, rowoff[j] + (unsigned)k);
      s[j] = (float)p.bscale[srow[j] + k / p.group];
    }
  }
  __device__ void store(f16* lds) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 2) + 64 * j;
      if (BN % 64 != 0 && row >= BN) continue;
      const int q = t & 3;
      const int w[4] = {r[j].x, r[j].y, r[j].z, r[j].w};
      f16x8 lo, hi;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int b0 = (int)(int8_t)((w[e >> 2] >> ((e & 3) * 8)) & 0xff);
        const int b1 = (int)(int8_t)((w[2 + (e >> 2)] >> ((e & 3) * 8)) & 0xff);
        lo[e] = (f16)((float)b0 * s[j]);
        hi[e] = (f16)((float)b1 * s[j]);
      }
      *reinterpret_cast<f16x8*>(lds + swz(row, 2 * q)) = lo;
      *reinterpret_cast<f16x8*>(lds + swz(row, 2 * q + 1)) = hi;
    }
  }
};

// packed int4 (low nibble = even k): a 16-B load = 32 codes = 4 LDS chunks; thread -> (row, half)
template <int BN>
struct BLoader<BN, QD_WFMT_I4> {
  static constexpr int LOADS = (BN * BK / 32 + 255) / 256;
  int4 r[LOADS];
  float s[LOADS];
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[LOADS];
  int srow[LOADS];
  __device__ void init(const GemmArgs& p, int n0) {
    rs = rsrc(p.b, p.b_bytes);
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int n = n0 + (t >> 1) + 128 * j;
      rowoff[j] = n < p.N ? (unsigned)n * (unsigned)(p.K / 2) : OOB;
      srow[j] = (n < p.N ? n : p.N - 1) * (p.K / p.group);
    }
  }
  __device__ void load(const GemmArgs& p, int k0) {
    const int k = k0 + (threadIdx.x & 1) * 32;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      r[j] = bload_i4(rs, rowoff[j] + (unsigned)(k / 2));
      s[j] = (float)p.bscale[srow[j] + k / p.group];
    }
  }
  __device__ void store(f16* lds) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 1) + 128 * j;
      if (BN % 128 != 0 && row >= BN) continue;
      const int hq = t & 1;
      const int w[4] = {r[j].x, r[j].y, r[j].z, r[j].w};
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // pair-interleaved offset-binary nibbles (qd_pack_int4)
          const int q = (int)(((unsigned)w[cc] >> ((e & 1) * 16 + (e >> 1) * 4)) & 0xf) - 8;
          o[e] = (f16)((float)q * s[j]);
        }
        *reinterpret_cast<f16x8*>(lds + swz(row, 4 * hq + cc)) = o;
      }
    }
  }
};

// ---- shared epilogue pieces ---------------------------------------------------------------
// column amax of 4 columns over the 16 rows held by lanes fr = 0..15 of a lane group
__device__ __forceinline__ float rowgroup_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x2e __attribute__((ext_vector_type(2)));

__device__ __forceinline__ i32x8 f8_operand(f16x8 lo, f16x8 hi) {
  const i32x4 a = __builtin_bit_cast(i32x4, lo), b = __builtin_bit_cast(i32x4, hi);
  return (i32x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// int8 path: C^T fragments of int32 sums -> scaled fp32 (or the raw int32 bits for a split-K slab)
template <int TM, int TN, bool SPLIT>
__device__ __forceinline__ void i8_scale(const GemmArgs& p, const i32x4 (&acc)[TM][TN], f32x4 (&out)[TM][TN], int m0,
                                         int n0, int wm0, int wn0) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (SPLIT) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) out[i][j] = __builtin_bit_cast(f32x4, acc[i][j]);
  } else {
    float sa[TM];
    if (p.sa_rps && p.sa_rps % (TM * 16) == 0) {
      // per-sample scales (conv): the wave tile's rows lie in one sample - one scalar index
      const float s = p.sa[min(m0 + wm0, p.M - 1) / p.sa_rps];
#pragma unroll
      for (int i = 0; i < TM; ++i) sa[i] = s;
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = min(m0 + wm0 + i * 16 + fr, p.M - 1);
        sa[i] = p.sa[p.sa_rps ? m / p.sa_rps : m];
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + j * 16 + fq * 4;
      const f32x4 sw = n < p.N ? *reinterpret_cast<const f32x4*>(p.sw + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[i][j][r] = ((float)acc[i][j][r] * sa[i]) * sw[r];
    }
  }
}

// ---- shared epilogue ----------------------------------------------------------------------
// acc[i][j]: C^T fragment (rows n = n0 + wn0 + 16j + 4fq + r, column m = m0 + wm0 + 16i + fr).
// LDS halves the epilogue needs: the [BM][BN + 8] fp16 C tile + the per-wave-row column-max
// slots of the amax combine (WGM x BN floats, WGM <= 8)
constexpr int epi_lds_halves(int bm, int bn) { return bm * (bn + 8) + 16 * bn; }

// grouped-row LayerNorm geometry of a row of BN columns (norm.hip ln_rows_geom): LPR lanes per row,
// P 16-B chunks per lane (lane l owns chunks l, l + LPR, ...); 0 = no such geometry
constexpr int ln_lpr(int bn) {
  return bn % 8 ? 0 : (bn / 8) % 8 == 0 && bn / 64 <= 5 ? 8 : (bn / 8) % 16 == 0 && bn / 128 <= 5 ? 16 :
                      (bn / 8) % 32 == 0 && bn / 256 <= 5 ? 32 : (bn / 8) % 64 == 0 && bn / 512 <= 5 ? 64 : 0;
}
constexpr int ln_per(int bn) { return ln_lpr(bn) ? bn / 8 / ln_lpr(bn) : 0; }

// CONV: a conv kernel's epilogue (no GEGLU / GELU-tanh: those are linear-only, compiled out);
// DIRECT: the direct-store path is compiled in (kernels whose epilogues always take the LDS path - the
// int8 halo conv's GroupNorm slot statistics - leave it out: its registers would spill there)
// whether gemm_epilogue stores straight from the fragments (see there): the tile shapes whose pair
// loop fits the register budget (TN 8: spills), and the epilogues that need no row-complete / slot
// view of the tile (plain, bias, residual, pre-residual amax, GEGLU at TN % 4 == 0, GELU-tanh)
template <int TM, int TN, bool DIRECT>
constexpr bool epi_direct_ok() { return DIRECT && TN >= 2 && TN <= 5 && TM * ((TN + 1) / 2) <= 20; }
// the post-residual amax in the direct path (column maxima of the final fp16 values kept packed,
// TN / 2 + 1 f16x8 registers per lane): the tiles of at most 20 fragments only
template <int TM, int TN, bool DIRECT, bool DPOSTK>
constexpr bool epi_dpost_ok() { return DPOSTK && epi_direct_ok<TM, TN, DIRECT>() && TM * TN <= 20; }
template <int BN, int TM, int TN, bool CONV, bool DIRECT, bool DPOSTK = false>
__device__ __forceinline__ bool epi_direct(const GemmArgs& p) {
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
  const bool geglu = !CONV && (p.epi & QD_EPI_GEGLU) != 0;
  const bool gtanh = !CONV && (p.epi & QD_EPI_GELU_TANH) != 0;
  const bool post = has_res && do_amax && (p.epi & QD_EPI_AMAX_POST) && !geglu && !gtanh;
  const bool gn = (p.epi & QD_EPI_GNSTATS) && p.gnp && !geglu && !gtanh;
  const bool ln = BN == 320 && (p.epi & QD_EPI_LN) && !geglu && !gtanh;
  const bool cadd = (p.epi & QD_EPI_CADD) && p.cadd && !geglu && !gtanh;
  return epi_direct_ok<TM, TN, DIRECT>() && !p.epi_lds && !gn && !ln && !cadd &&
         (!post || epi_dpost_ok<TM, TN, DIRECT, DPOSTK>()) && (!geglu || TN % 4 == 0);
}

template <int BM, int BN, int NT, int TM, int TN, bool SPLIT, int LDSH, bool CONV = false, bool DIRECT = true,
          bool DPOSTK = false>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& p, f32x4 (&acc)[TM][TN], f16* smem, int m0, int n0,
                                              int wm0, int wn0, int split) {
  static_assert(SPLIT || epi_lds_halves(BM, BN) <= LDSH, "epilogue LDS exceeds the kernel's buffer");
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (SPLIT) {
    // fp32 partial slab [split][M][N]
    float* part = p.part + (long)split * p.M * p.N;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + j * 16 + fq * 4;
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm0 + i * 16 + fr;
        if (m < p.M) *reinterpret_cast<f32x4*>(part + (long)m * p.N + n) = acc[i][j];
      }
    }
  } else {
    // (1) fragments: h = half(acc + bias) -> per-column amax (pre-residual, the conv output the
    //     reference fake-quantizes) and an fp16 C tile in LDS (the K loop ended on a barrier);
    // (2) coalesced: 16-B row chunks of the tile (+ residual) -> y.
    constexpr int LP = BN + 8;  // LDS row pitch (halves)
    f16* ct = smem;
    const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
    const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
    const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
    const bool geglu = !CONV && (p.epi & QD_EPI_GEGLU) != 0;
    const bool gtanh = !CONV && (p.epi & QD_EPI_GELU_TANH) != 0;
    // post-residual amax: the residual is added to the fragments (8-B loads per lane) before the
    // column maxes, and the coalesced pass below stores the tile as it stands
    const bool post = has_res && do_amax && (p.epi & QD_EPI_AMAX_POST) && !geglu && !gtanh;
    // GroupNorm slot statistics / per-(sample, column) add of the final output: cadd is added to
    // the fragments (the tile lies in one sample: rows_per_sample % BM == 0, host; a residual then
    // goes there first), the coalesced pass adds the residual and writes the final tile back to
    // LDS, and the slot moments are reduced from there
    const bool gn = (p.epi & QD_EPI_GNSTATS) && p.gnp && !geglu && !gtanh;
    // row-complete LayerNorm (host: BN == N, n0 == 0, residual, no amax): the final tile is written
    // back to LDS by the coalesced pass like the GroupNorm slots' and normalised row by row from there
    constexpr bool LN_OK = BN == 320 && ln_lpr(BN) != 0;  // (the tiles ln_var plans; others compile it out)
    const bool ln = LN_OK && (p.epi & QD_EPI_LN) && !geglu && !gtanh;
    const bool cadd = (p.epi & QD_EPI_CADD) && p.cadd && !geglu && !gtanh;
    const bool fres = post || (has_res && cadd);
    const f16* const cadd_row = cadd ? p.cadd + (long)(min(m0, p.M - 1) / p.rows_per_sample) * p.cadd_ld : nullptr;
    // amax: the WGM wave rows of the block combine their column maxes in LDS first when the
    // block's rows lie in one sample, so each (sample, column) address takes one atomic per
    // block instead of one per wave row (same-line atomic chains bound this epilogue)
    constexpr int WM = TM * 16, WGM = BM / WM;
    static_assert(WGM <= 8, "column-max slots");
    float* const cmx = reinterpret_cast<float*>(ct + BM * LP);
    const bool blk_amax = do_amax && !geglu && WGM > 1 && p.rows_per_sample % BM == 0;
    const unsigned ybytes = (unsigned)min((long)p.M * p.ldy * 2, 2147483647L);
    const __amdgpu_buffer_rsrc_t yrs = rsrc(p.y, ybytes);
    // (the LDS path's fres forms load their residual in the fragment layout; the direct path - post
    // included - through this descriptor)
    const bool rdesc = has_res && (!fres || (DPOSTK && epi_direct<BN, TM, TN, CONV, DIRECT, DPOSTK>(p)));
    const __amdgpu_buffer_rsrc_t rrs = rsrc(rdesc ? p.res : p.y, rdesc ? ybytes : 0u);
    // the residual tile of the coalesced pass is loaded first, all NR chunks per thread in flight
    // while the fragments go to LDS (a 2-deep load / add / store loop left the epilogue waiting on
    // HBM latency NR / 2 times)
    constexpr int CPR16 = BN / 8, NR = (BM * CPR16 + NT - 1) / NT;
    // direct stores (no LDS C tile): the epilogues that need no row-complete / slot view of the tile
    // (plain, bias, residual, pre-residual amax, GEGLU, GELU-tanh) store each lane's fragments
    // themselves: fragments j, j + 1 (4 columns each, rows fr) are paired by one v_permlane16_swap per
    // dword, after which lane (fr, fq) holds 8 consecutive columns 16 (fq & 1) + 8 (fq >> 1) of the
    // pair - one 16-B store (or residual load) per lane and pair, 16 rows x 64 B per instruction.
    // Same arithmetic per element as the LDS pass below, so the output bits are identical.
    // (an odd TN's last fragment stores its 4 columns as one 8-B store per lane)
    constexpr bool DIRECT_OK = epi_direct_ok<TM, TN, DIRECT>();
    const bool direct = epi_direct<BN, TM, TN, CONV, DIRECT, DPOSTK>(p);
    const bool pre_res = has_res && !fres && !geglu && !direct;
    // post-residual amax: the residual in the fragments' layout (4 consecutive columns of one row
    // per lane and fragment), all TM x TN 8-B loads issued before any is used
    constexpr bool PF_POST = TM * TN <= 20;  // (register budget: the 4 x 5 fragment tiles and smaller)
    f16x4 rf[PF_POST ? TM : 1][PF_POST ? TN : 1];
    if (PF_POST && fres && !(DPOSTK && direct)) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 16 + fq * 4;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int m = m0 + wm0 + i * 16 + fr;
          if constexpr (PF_POST)
            rf[i][j] = (m < p.M && n < p.N) ? *reinterpret_cast<const f16x4*>(p.res + (long)m * p.ldy + n) : f16x4{};
        }
      }
    }
    // (the direct path's residual fragments share this array: one private array fewer keeps the
    // promote-alloca budget for the accumulators and operand staging)
    constexpr int NRQ = NR > TM * (TN / 2 + (TN & 1)) ? NR : TM * (TN / 2 + (TN & 1));
    f16x8 rq[NRQ];
    if (pre_res) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int e = (int)threadIdx.x + i * NT;
        const int row = e / CPR16, n = n0 + (e - row * CPR16) * 8;
        const bool ok = (BM * CPR16 % NT == 0 || e < BM * CPR16) && m0 + row < p.M && n < p.N;
        rq[i] = bload(rrs, ok ? ((unsigned)(m0 + row) * (unsigned)p.ldy + (unsigned)n) * 2u : OOB);
      }
    }
    // column-max commit of fragment column group j (cm: this lane's 4 column maxima over its rows)
    auto amax_commit = [&](int j, float (&cm)[4]) {
      const int nl = wn0 + j * 16 + fq * 4;
      const int n = n0 + nl;
#pragma unroll
      for (int r = 0; r < 4; ++r) cm[r] = rowgroup_max(cm[r]);
      const int row0 = m0 + wm0;
      if (blk_amax) {
        if (fr == 0) *reinterpret_cast<f32x4*>(cmx + (wm0 / WM) * BN + nl) = (f32x4){cm[0], cm[1], cm[2], cm[3]};
      } else if (fr == 0 && n < p.N && row0 < p.M) {
        float* a = p.amax + (long)(row0 / p.rows_per_sample) * p.N + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) atomic_max_pos(a + r, cm[r]);
      }
    };
    if constexpr (DIRECT_OK) {
      if (direct) {
        constexpr int NJ = TN / 2;
        const int cpart = 16 * (fq & 1) + 8 * (fq >> 1);
        const bool gg = geglu;
        // output columns of pair jp: GEGLU pairs OUTPUT fragments (2 gemm fragments each: hidden | gate)
        const int ocol0 = gg ? ((n0 + wn0) >> 1) : n0 + wn0;
        const int oN = gg ? (p.N >> 1) : p.N;
        const int npair = gg ? NJ / 2 : NJ;
        constexpr bool TAIL = TN & 1;  // (never with GEGLU: TN % 4 == 0 there)
        // residual fragments of row block i are loaded two row blocks ahead (all TM x NJ at once would
        // hold 64 VGPRs beside the 256 x 128 tile's 128 accumulators and spill)
        constexpr int NJT = NJ + (TAIL ? 1 : 0);  // rq[i * NJT + jp]: pair jp of row block i (jp == NJ: the tail)
        auto load_res = [&](int i) {
          {
            const int m = m0 + wm0 + i * 16 + fr;
#pragma unroll
            for (int jp = 0; jp < NJ; ++jp) {
              const int n = ocol0 + 32 * jp + cpart;
              rq[i * NJT + jp] = bload(rrs, (jp < npair && m < p.M && n < oN) ? ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u : OOB);
            }
            if constexpr (TAIL) {
              const int n = n0 + wn0 + (TN - 1) * 16 + fq * 4;
              const f16x4 t = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(
                  rrs, (m < p.M && n < p.N) ? (int)(((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u) : (int)OOB, 0, 0));
              rq[i * NJT + NJ] = (f16x8){t[0], t[1], t[2], t[3], (f16)0, (f16)0, (f16)0, (f16)0};
            }
          }
        };
        // prefetch distance in row blocks (the 256 x 128 tiles' 32 fragments leave room for one)
        constexpr int PFD = TM * TN >= 32 || DPOSTK ? 1 : 2;  // (DPOSTK: room for the packed column maxima)
        if (has_res) {
#pragma unroll
          for (int i = 0; i < PFD && i < TM; ++i) load_res(i);
        }
        // the bias per fragment column (h = half(acc + bias), the LDS pass's f32 add), then this lane's
        // column maxima of h per column group (no per-row arrays: register pressure)
        // (the bias widened to f32 once per column group, not once per row block: the per-row-block
        // sched_barrier below keeps the compiler from hoisting the conversions itself)
        f32x4 bq[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn0 + j * 16 + fq * 4;
          const f16x4 b = (has_bias && n < p.N) ? *reinterpret_cast<const f16x4*>(p.bias + n) : f16x4{};
#pragma unroll
          for (int r = 0; r < 4; ++r) bq[j][r] = (float)b[r];
        }
        auto frag16 = [&](int i, int j) {
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = (f16)(acc[i][j][r] + bq[j][r]);
          return h;
        };
        if (do_amax && !gg && !post) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 16 + fq * 4;
            float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const bool ok = m0 + wm0 + i * 16 + fr < p.M && n < p.N;
              const f16x4 h = frag16(i, j);
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (ok) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
            }
            amax_commit(j, cm);
          }
        }
        // GEGLU output fragment: half(h * half(gelu(g))) of gemm fragments j | j + 1
        auto geglu_frag = [&](int i, int j) {
          const f16x4 hv = frag16(i, j), gv = frag16(i, j + 1);
          f16x4 o;
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 g2 = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
            o[r] = (f16)((float)hv[r] * (float)(f16)g2.x);
            o[r + 1] = (f16)((float)hv[r + 1] * (float)(f16)g2.y);
          }
          return o;
        };
        auto plain_frag = [&](int i, int j) {
          f16x4 o = frag16(i, j);
          if (gtanh) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (f16)gelu_tanh_f((float)o[r]);
          }
          return o;
        };
        // post-residual amax: |final| column maxima of this lane's rows, packed fp16 (max of fp16 values
        // is exact, so the f32 maxima of the LDS path come out bit-identical): pair jp's 8 columns in
        // pm[jp], the odd tail's 4 in pmt
        constexpr bool DPOST = epi_dpost_ok<TM, TN, DIRECT, DPOSTK>();
        f16x8 pm[DPOST ? (NJ > 0 ? NJ : 1) : 1];
        f16x4 pmt = {};
        if constexpr (DPOST) {
#pragma unroll
          for (int jp = 0; jp < NJ; ++jp) pm[jp] = f16x8{};
        }
        // pair (a | b) -> 16-B store (+ residual: RES, a compile-time copy of has_res - the row loop is
        // instantiated for both, so no per-element select; POST: the post-residual column maxima) at
        // output column n of row m
        auto store_pair = [&](auto res_c, auto post_c, int i, int jp, f16x4 fa, f16x4 fb, int m, bool row_ok) {
          constexpr bool RES = decltype(res_c)::value;
          constexpr bool POST = DPOST && decltype(post_c)::value;
          u32x4 w;
          {
            const u32x2 a = __builtin_bit_cast(u32x2, fa), b = __builtin_bit_cast(u32x2, fb);
            const auto s0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
            w = (u32x4){s0[0], s1[0], s0[1], s1[1]};
          }
          const int n = ocol0 + 32 * jp + cpart;
          if constexpr (RES) {
            f16x8 v = __builtin_bit_cast(f16x8, w);
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[i * NJT + jp][r]);
            w = __builtin_bit_cast(u32x4, v);
          }
          if constexpr (POST) {
            if (row_ok && n < oN)
              pm[jp] = __builtin_elementwise_max(pm[jp], __builtin_bit_cast(f16x8, w & 0x7fff7fffu));
          }
          const unsigned off = ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u;
#ifdef QD_ABLATE_EPI_STORES  // diagnostic build: the direct epilogue's stores dropped (values kept live)
          asm volatile("" ::"v"(w), "v"(off));
#else
          __builtin_amdgcn_raw_buffer_store_b128(w, yrs, (row_ok && n < oN) ? (int)off : (int)OOB, 0, 0);
#endif
        };
        auto rows = [&](auto res_c, auto post_c) {
          constexpr bool RES = decltype(res_c)::value;
          constexpr bool POST = DPOST && decltype(post_c)::value;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            if (RES && i + PFD < TM) load_res(i + PFD);
            const int m = m0 + wm0 + i * 16 + fr;
            const bool row_ok = m < p.M;
            if constexpr (TN % 4 == 0 && !POST) {
              if (gg) {
#pragma unroll
                for (int jp = 0; jp < TN / 4; ++jp)
                  store_pair(res_c, post_c, i, jp, geglu_frag(i, 4 * jp), geglu_frag(i, 4 * jp + 2), m, row_ok);
                continue;
              }
            }
#pragma unroll
            for (int jp = 0; jp < NJ; ++jp)
              store_pair(res_c, post_c, i, jp, plain_frag(i, 2 * jp), plain_frag(i, 2 * jp + 1), m, row_ok);
            if constexpr (TAIL) {
              f16x4 v = plain_frag(i, TN - 1);
              if constexpr (RES) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = (f16)((float)v[r] + (float)rq[i * NJT + NJ][r]);
              }
              const int n = n0 + wn0 + (TN - 1) * 16 + fq * 4;
              if constexpr (POST) {
                if (row_ok && n < p.N)
                  pmt = __builtin_elementwise_max(
                      pmt, __builtin_bit_cast(f16x4, __builtin_bit_cast(u32x2, v) & 0x7fff7fffu));
              }
              const unsigned off = ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u;
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), yrs,
                                                    (row_ok && n < p.N) ? (int)off : (int)OOB, 0, 0);
            }
            // one row block at a time: the scheduler may not pull later blocks' conversions / swaps up
            // (their temporaries beside the live accumulators spill)
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        if (DPOST && post) {
          rows(std::true_type{}, std::true_type{});
          if constexpr (DPOST) {
            // the lane's maxima over its 16-row groups (lanes fr = 0..15 of each fq), then lane fr == 0
            // commits them in the fragment column order of amax_commit
            auto red = [&](unsigned u) {
#pragma unroll
              for (int o = 1; o < 16; o <<= 1) {
                const unsigned t = (unsigned)__shfl_xor((int)u, o, 64);
                u = __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(f16x2e, u),
                                                                           __builtin_bit_cast(f16x2e, t)));
              }
              return u;
            };
            const int row0 = m0 + wm0;
            auto commit = [&](int nl, float v) {
              if (blk_amax) cmx[(wm0 / WM) * BN + nl] = v;
              else if (n0 + nl < p.N && row0 < p.M)
                atomic_max_pos(p.amax + (long)(row0 / p.rows_per_sample) * p.N + n0 + nl, v);
            };
#pragma unroll
            for (int jp = 0; jp < NJ; ++jp) {
              u32x4 u = __builtin_bit_cast(u32x4, pm[jp]);
#pragma unroll
              for (int r = 0; r < 4; ++r) u[r] = red(u[r]);
              const f16x8 h = __builtin_bit_cast(f16x8, u);
              if (fr == 0) {
#pragma unroll
                for (int e = 0; e < 8; ++e) commit(wn0 + 32 * jp + cpart + e, (float)h[e]);
              }
            }
            if constexpr (TAIL) {
              u32x2 u = __builtin_bit_cast(u32x2, pmt);
              u[0] = red(u[0]);
              u[1] = red(u[1]);
              const f16x4 h = __builtin_bit_cast(f16x4, u);
              if (fr == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) commit(wn0 + (TN - 1) * 16 + fq * 4 + r, (float)h[r]);
              }
            }
          }
        } else if (has_res) {
          rows(std::true_type{}, std::false_type{});
        } else {
          rows(std::false_type{}, std::false_type{});
        }
        if (do_amax && !gg && blk_amax) {
          __syncthreads();
          for (int c = threadIdx.x; c < BN; c += NT) {
            float mm = cmx[c];
#pragma unroll
            for (int w = 1; w < WGM; ++w) mm = fmaxf(mm, cmx[w * BN + c]);
            if (n0 + c < p.N && m0 < p.M) atomic_max_pos(p.amax + (long)(m0 / p.rows_per_sample) * p.N + n0 + c, mm);
          }
        }
        return;
      }
    }
    {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn0 + j * 16 + fq * 4;
        const int n = n0 + nl;
        const bool col_ok = n < p.N;  // N % 8 == 0: a lane's 4 columns are all in or all out
        f16x4 bq = {}, cv = {};
        if (has_bias && col_ok) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
        if (cadd && col_ok) cv = *reinterpret_cast<const f16x4*>(cadd_row + n);
        float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ml = wm0 + i * 16 + fr;
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = (f16)(acc[i][j][r] + (float)bq[r]);
          if (fres) {
            const bool ok = m0 + ml < p.M && col_ok;
            if (ok) {
              f16x4 rv;
              if constexpr (PF_POST) rv = rf[i][j];
              else rv = *reinterpret_cast<const f16x4*>(p.res + (long)(m0 + ml) * p.ldy + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)rv[r]);
            }
          }
          if (cadd) {
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)cv[r]);
          }
          if (do_amax) {  // (uniform) the column maxes only when an amax is reduced
            const bool ok = m0 + ml < p.M && col_ok;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (ok) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
          }
          *reinterpret_cast<f16x4*>(ct + ml * LP + nl) = h;
        }
        // rows of this wave tile lie in one sample (rows_per_sample % WM == 0, host check); rows past
        // M contribute 0 (cm starts at 0, `ok` excludes them)
        if (do_amax && !geglu) amax_commit(j, cm);
      }
    }
    __syncthreads();
    if (blk_amax) {
      for (int c = threadIdx.x; c < BN; c += NT) {
        float m = cmx[c];
#pragma unroll
        for (int w = 1; w < WGM; ++w) m = fmaxf(m, cmx[w * BN + c]);
        if (n0 + c < p.N && m0 < p.M) atomic_max_pos(p.amax + (long)(m0 / p.rows_per_sample) * p.N + n0 + c, m);
      }
    }
    // output tile: BN columns (BN / 2 with GEGLU) starting at n0 (n0 / 2).  GEGLU: weight rows
    // are interleaved in 16-row blocks [hidden 16 | gate 16] (BN % 32 == 0), so output columns
    // 16b + j of the tile read h = tile[32b + j], g = tile[32b + 16 + j]; diffusers GEGLU on the
    // fp16 projection outputs: out = half(h * half(gelu(g))).
    // 16-B chunks per output row are a compile-time constant in each branch (no runtime
    // division); stores / residual loads are 32-bit-offset buffer ops (rows past M fall off the
    // end of the buffer range and are dropped / read 0).
    static_assert(BN % 32 == 0 || BN % 16 == 0, "tile width");
    // GroupNorm slot statistics from the final tile in LDS: thread -> (64-row slot, 8-channel
    // chunk, row phase k of G): rows k, k + G, ... of the slot, shifted by the slot's first row
    // (no cancellation), then the G phases summed by lane shuffles (G consecutive lanes)
    auto gn_slots = [&]() {
      constexpr int SL = BM / 64, NPAIR = SL * CPR16;
      constexpr int G0 = NT / NPAIR >= 64 ? 64 : NT / NPAIR >= 32 ? 32 : NT / NPAIR >= 16 ? 16 :
                         NT / NPAIR >= 8 ? 8 : NT / NPAIR >= 4 ? 4 : NT / NPAIR >= 2 ? 2 : 1;
      static_assert(BM % 64 == 0 && NPAIR * G0 <= NT, "slot geometry");
      const int t = threadIdx.x;
      if (t >= NPAIR * G0) return;
      const int pr = t / G0, k = t - pr * G0;
      const int s = pr / CPR16, c = pr - s * CPR16;
      const int row0 = s * 64, n = n0 + c * 8;
      const f16x8 sh = *reinterpret_cast<const f16x8*>(ct + row0 * LP + c * 8);
      float s1[8], s2[8], mn[8], mx[8];
      // min / max on the fp16 values themselves (exact; packed f16 pairs), sums in f32
      f16x8 mn8 = sh, mx8 = sh;
#pragma unroll
      for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
#pragma unroll 4
      for (int rr = k; rr < 64; rr += G0) {
        const f16x8 v = *reinterpret_cast<const f16x8*>(ct + (row0 + rr) * LP + c * 8);
        mn8 = __builtin_elementwise_min(mn8, v);
        mx8 = __builtin_elementwise_max(mx8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = (float)v[j] - (float)sh[j];
          s1[j] += a;
          s2[j] += a * a;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mn[j] = (float)mn8[j];
        mx[j] = (float)mx8[j];
      }
#pragma unroll
      for (int o = G0 / 2; o > 0; o >>= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1[j] += __shfl_xor(s1[j], o, 64);
          s2[j] += __shfl_xor(s2[j], o, 64);
          mn[j] = fminf(mn[j], __shfl_xor(mn[j], o, 64));
          mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], o, 64));
        }
      if (k == 0 && n < p.N && m0 + row0 < p.M) {
        float4* dst = reinterpret_cast<float4*>(p.gnp) + (long)((m0 + row0) / 64) * p.N + n;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          dst[j] = make_float4((float)sh[j] + s1[j] * (1.0f / 64.0f), s2[j] - s1[j] * s1[j] * (1.0f / 64.0f), mn[j], mx[j]);
      }
    };
    // LayerNorm rows from the final tile in LDS: a wave takes 64 / LPR rows at a time, LPR lanes per
    // row, lane lr owning chunks lr, lr + LPR, ... - k_ln_rows' lane map, sums and butterflies, so
    // the output is bit-identical to the separate LayerNorm launch over y
    auto ln_rows = [&]() {
      constexpr int LPR = LN_OK ? ln_lpr(BN) : 8, P = LN_OK ? ln_per(BN) : 1, RPW = 64 / LPR, NWV = NT / 64;
      const int wv = threadIdx.x >> 6, lr = lane % LPR, rw = lane / LPR;
      f16x8 g[P], b[P];
#pragma unroll
      for (int i = 0; i < P; ++i) {
        g[i] = *reinterpret_cast<const f16x8*>(p.ln_g + (lr + i * LPR) * 8);
        b[i] = *reinterpret_cast<const f16x8*>(p.ln_b + (lr + i * LPR) * 8);
      }
      const float inv_c = (float)BN;
      for (int r0 = wv * RPW; r0 < BM; r0 += NWV * RPW) {
        const int row = r0 + rw;
        const long m = (long)m0 + row;
        const bool ok = m < p.M;
        f16x8 v[P];
#pragma unroll
        for (int i = 0; i < P; ++i) v[i] = *reinterpret_cast<const f16x8*>(ct + row * LP + (lr + i * LPR) * 8);
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) sm += (float)v[i][e];
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
        const float mean = sm / inv_c;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float a = (float)v[i][e] - mean;
            q = fmaf(a, a, q);
          }
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
        const float rstd = 1.0f / sqrtf(q / inv_c + p.ln_eps);
        f16x8 o8[P];
        float mx = 0.f;
#pragma unroll
        for (int i = 0; i < P; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            o8[i][e] = to_f16(fmaf(((float)v[i][e] - mean) * rstd, (float)g[i][e], (float)b[i][e]));
            mx = fmaxf(mx, fabsf((float)o8[i][e]));
          }
        if (p.ln_y8) {
#pragma unroll
          for (int o = LPR / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
          const float s8 = fq_scale(mx, 127);
          const double r8 = rcp_exact(s8);
          if (ok && lr == 0) p.ln_sa8[m] = s8;
#pragma unroll
          for (int i = 0; i < P; ++i) {
            unsigned lo = 0, hi = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const f16 tq = (f16)(float)((double)(float)o8[i][e] * r8);
              const unsigned qv = (unsigned)(uint8_t)(int8_t)__builtin_rintf((float)tq);
              if (e < 4) lo |= qv << (8 * e);
              else hi |= qv << (8 * (e - 4));
            }
            if (ok) *reinterpret_cast<uint2*>(p.ln_y8 + m * BN + (lr + i * LPR) * 8) = make_uint2(lo, hi);
          }
        } else {
#pragma unroll
          for (int i = 0; i < P; ++i)
            if (ok) *reinterpret_cast<f16x8*>(p.ln_y + m * BN + (lr + i * LPR) * 8) = o8[i];
        }
      }
    };
    if (pre_res) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int e = (int)threadIdx.x + i * NT;
        const int row = e / CPR16, c = e - row * CPR16;
        const int n = n0 + c * 8;
        if ((BM * CPR16 % NT == 0 || e < BM * CPR16) && n < p.N) {
          const unsigned off = ((unsigned)(m0 + row) * (unsigned)p.ldy + (unsigned)n) * 2u;
          f16x8 v = *reinterpret_cast<const f16x8*>(ct + row * LP + c * 8);
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[i][r]);
          if (gn || ln) *reinterpret_cast<f16x8*>(ct + row * LP + c * 8) = v;  // (this thread's own element)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, m0 + row < p.M ? (int)off : (int)OOB, 0, 0);
        }
      }
      if (gn || ln) __syncthreads();
      if (gn) gn_slots();
      if constexpr (LN_OK) {
        if (ln) ln_rows();
      }
      return;
    }
    auto pass2 = [&](auto cpr_c, auto geglu_c) {
      constexpr int CPR = decltype(cpr_c)::value;
      constexpr bool GG = decltype(geglu_c)::value;
      const int on0 = GG ? n0 >> 1 : n0, oN = GG ? p.N >> 1 : p.N;
#pragma unroll 2
      for (int e = threadIdx.x; e < BM * CPR; e += NT) {
        const int row = e / CPR, c = e - row * CPR;
        const int n = on0 + c * 8;
        if (n < oN) {
          const unsigned off = ((unsigned)(m0 + row) * (unsigned)p.ldy + (unsigned)n) * 2u;
          f16x8 v;
          if constexpr (GG) {
            const int tc = (c >> 1) * 32 + (c & 1) * 8;
            const f16x8 hv = *reinterpret_cast<const f16x8*>(ct + row * LP + tc);
            const f16x8 gv = *reinterpret_cast<const f16x8*>(ct + row * LP + tc + 16);
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
              const f32x2 gg = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
              v[r] = (f16)((float)hv[r] * (float)(f16)gg.x);
              v[r + 1] = (f16)((float)hv[r + 1] * (float)(f16)gg.y);
            }
          } else {
            v = *reinterpret_cast<const f16x8*>(ct + row * LP + c * 8);
            if (gtanh) {
#pragma unroll
              for (int r = 0; r < 8; ++r) v[r] = (f16)gelu_tanh_f((float)v[r]);
            }
          }
          if (has_res && !fres) {
            const f16x8 rq = bload(rrs, m0 + row < p.M ? off : OOB);
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[r]);
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, m0 + row < p.M ? (int)off : (int)OOB, 0, 0);
        }
      }
    };
    if (geglu) pass2(std::integral_constant<int, BN / 16>{}, std::true_type{});
    else pass2(std::integral_constant<int, BN / 8>{}, std::false_type{});
    if (gn) {
      __syncthreads();
      gn_slots();
    }
  }
}

// The direct-store epilogue in two phases for the persistent DMA kernels: direct_outputs forms every
// 16-B store word of the wave tile (bias, GELU-tanh / GEGLU, permlane16 pairing, residual add - the
// same per-element arithmetic as gemm_epilogue's direct path, so the same bits) with every load it
// needs (bias, residual) issued AND consumed first; direct_stores then only stores.  Between the two
// the kernel issues the next tile's DMA: no load younger than that DMA is waited for (a counted
// vmcnt on an ordinary load would wait for the older DMA too), so the DMA runs under the stores.
template <int TM, int TN>
__device__ __forceinline__ void direct_outputs(const GemmArgs& p, const f32x4 (&acc)[TM][TN], int m0, int n0, int wm0,
                                               int wn0, u32x4 (&wo)[TM][TN / 2 + (TN & 1)]) {
  constexpr int NJ = TN / 2, NJT = NJ + (TN & 1);
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool gg = (p.epi & QD_EPI_GEGLU) != 0;
  const bool gtanh = (p.epi & QD_EPI_GELU_TANH) != 0;
  const int cpart = 16 * (fq & 1) + 8 * (fq >> 1);
  const int ocol0 = gg ? ((n0 + wn0) >> 1) : n0 + wn0;
  const int oN = gg ? (p.N >> 1) : p.N;
  const int npair = gg ? NJ / 2 : NJ;
  const unsigned ybytes = (unsigned)min((long)p.M * p.ldy * 2, 2147483647L);
  const __amdgpu_buffer_rsrc_t rrs = rsrc(has_res ? p.res : p.y, has_res ? ybytes : 0u);
  f16x8 rq[TM][NJT];
  if (has_res) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm0 + i * 16 + fr;
#pragma unroll
      for (int jp = 0; jp < NJ; ++jp) {
        const int n = ocol0 + 32 * jp + cpart;
        rq[i][jp] = bload(rrs, (jp < npair && m < p.M && n < oN) ? ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u : OOB);
      }
      if constexpr ((TN & 1) != 0) {
        const int n = n0 + wn0 + (TN - 1) * 16 + fq * 4;
        const f16x4 t = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(
            rrs, (m < p.M && n < p.N) ? (int)(((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u) : (int)OOB, 0, 0));
        rq[i][NJ] = (f16x8){t[0], t[1], t[2], t[3], (f16)0, (f16)0, (f16)0, (f16)0};
      }
    }
  }
  f16x4 bq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn0 + j * 16 + fq * 4;
    bq[j] = (has_bias && n < p.N) ? *reinterpret_cast<const f16x4*>(p.bias + n) : f16x4{};
  }
  auto frag16 = [&](int i, int j) {
    f16x4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (f16)(acc[i][j][r] + (float)bq[j][r]);
    return h;
  };
  auto geglu_frag = [&](int i, int j) {
    const f16x4 hv = frag16(i, j), gv = frag16(i, j + 1);
    f16x4 o;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      const f32x2 g2 = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
      o[r] = (f16)((float)hv[r] * (float)(f16)g2.x);
      o[r + 1] = (f16)((float)hv[r + 1] * (float)(f16)g2.y);
    }
    return o;
  };
  auto plain_frag = [&](int i, int j) {
    f16x4 o = frag16(i, j);
    if (gtanh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (f16)gelu_tanh_f((float)o[r]);
    }
    return o;
  };
  auto pair = [&](int i, int jp, f16x4 fa, f16x4 fb) {
    const u32x2 a = __builtin_bit_cast(u32x2, fa), b = __builtin_bit_cast(u32x2, fb);
    const auto s0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
    u32x4 w = (u32x4){s0[0], s1[0], s0[1], s1[1]};
    if (has_res) {
      f16x8 v = __builtin_bit_cast(f16x8, w);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[i][jp][r]);
      w = __builtin_bit_cast(u32x4, v);
    }
    return w;
  };
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if constexpr (TN % 4 == 0) {
      if (gg) {
#pragma unroll
        for (int jp = 0; jp < TN / 4; ++jp) wo[i][jp] = pair(i, jp, geglu_frag(i, 4 * jp), geglu_frag(i, 4 * jp + 2));
#pragma unroll
        for (int jp = TN / 4; jp < NJT; ++jp) wo[i][jp] = (u32x4){0u, 0u, 0u, 0u};
        continue;
      }
    }
#pragma unroll
    for (int jp = 0; jp < NJ; ++jp) wo[i][jp] = pair(i, jp, plain_frag(i, 2 * jp), plain_frag(i, 2 * jp + 1));
    if constexpr ((TN & 1) != 0) {
      f16x4 v = plain_frag(i, TN - 1);
      if (has_res) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (f16)((float)v[r] + (float)rq[i][NJ][r]);
      }
      const u32x2 t = __builtin_bit_cast(u32x2, v);
      wo[i][NJ] = (u32x4){t.x, t.y, 0u, 0u};
    }
  }
}

// direct_outputs without a residual, the bias fragments already loaded (the A-stationary kernel
// loads them ahead of its DMA): the same per-element arithmetic
template <int TM, int TN>
__device__ __forceinline__ void direct_outputs_pre(const GemmArgs& p, const f32x4 (&acc)[TM][TN], const f16x4 (&bq)[TN],
                                                   int m0, int n0, int wm0, int wn0,
                                                   u32x4 (&wo)[TM][TN / 2 + (TN & 1)]) {
  constexpr int NJ = TN / 2, NJT = NJ + (TN & 1);
  const bool gg = (p.epi & QD_EPI_GEGLU) != 0;
  const bool gtanh = (p.epi & QD_EPI_GELU_TANH) != 0;
  auto frag16 = [&](int i, int j) {
    f16x4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (f16)(acc[i][j][r] + (float)bq[j][r]);
    return h;
  };
  auto geglu_frag = [&](int i, int j) {
    const f16x4 hv = frag16(i, j), gv = frag16(i, j + 1);
    f16x4 o;
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      const f32x2 g2 = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
      o[r] = (f16)((float)hv[r] * (float)(f16)g2.x);
      o[r + 1] = (f16)((float)hv[r + 1] * (float)(f16)g2.y);
    }
    return o;
  };
  auto plain_frag = [&](int i, int j) {
    f16x4 o = frag16(i, j);
    if (gtanh) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (f16)gelu_tanh_f((float)o[r]);
    }
    return o;
  };
  auto pair = [&](f16x4 fa, f16x4 fb) {
    const u32x2 a = __builtin_bit_cast(u32x2, fa), b = __builtin_bit_cast(u32x2, fb);
    const auto s0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
    return (u32x4){s0[0], s1[0], s0[1], s1[1]};
  };
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if constexpr (TN % 4 == 0) {
      if (gg) {
#pragma unroll
        for (int jp = 0; jp < TN / 4; ++jp) wo[i][jp] = pair(geglu_frag(i, 4 * jp), geglu_frag(i, 4 * jp + 2));
#pragma unroll
        for (int jp = TN / 4; jp < NJT; ++jp) wo[i][jp] = (u32x4){0u, 0u, 0u, 0u};
        continue;
      }
    }
#pragma unroll
    for (int jp = 0; jp < NJ; ++jp) wo[i][jp] = pair(plain_frag(i, 2 * jp), plain_frag(i, 2 * jp + 1));
    if constexpr ((TN & 1) != 0) {
      const u32x2 t = __builtin_bit_cast(u32x2, plain_frag(i, TN - 1));
      wo[i][NJ] = (u32x4){t.x, t.y, 0u, 0u};
    }
  }
}

// the stores of direct_outputs' words; returns the number of store instructions this wave issued
template <int TM, int TN>
__device__ __forceinline__ int direct_stores(const GemmArgs& p, const u32x4 (&wo)[TM][TN / 2 + (TN & 1)], int m0, int n0,
                                             int wm0, int wn0) {
  constexpr int NJ = TN / 2;
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const bool gg = (p.epi & QD_EPI_GEGLU) != 0;
  const int cpart = 16 * (fq & 1) + 8 * (fq >> 1);
  const int ocol0 = gg ? ((n0 + wn0) >> 1) : n0 + wn0;
  const int oN = gg ? (p.N >> 1) : p.N;
  const int npair = gg ? NJ / 2 : NJ;
  const unsigned ybytes = (unsigned)min((long)p.M * p.ldy * 2, 2147483647L);
  const __amdgpu_buffer_rsrc_t yrs = rsrc(p.y, ybytes);
  int nst = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm0 + i * 16 + fr;
    const bool row_ok = m < p.M;
#pragma unroll
    for (int jp = 0; jp < NJ; ++jp) {
      if (jp >= npair) continue;  // (wave-uniform: GEGLU halves the pairs)
      const int n = ocol0 + 32 * jp + cpart;
      const unsigned off = ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u;
      __builtin_amdgcn_raw_buffer_store_b128(wo[i][jp], yrs, (row_ok && n < oN) ? (int)off : (int)OOB, 0, 0);
      ++nst;
    }
    if constexpr ((TN & 1) != 0) {
      const int n = n0 + wn0 + (TN - 1) * 16 + fq * 4;
      const unsigned off = ((unsigned)m * (unsigned)p.ldy + (unsigned)n) * 2u;
      __builtin_amdgcn_raw_buffer_store_b64((u32x2){wo[i][NJ][0], wo[i][NJ][1]}, yrs,
                                            (row_ok && n < p.N) ? (int)off : (int)OOB, 0, 0);
      ++nst;
    }
  }
  return nst;
}

// ---- kernel -----------------------------------------------------------------------------
template <int BM, int BN, int AMODE, int BFMT, bool SPLIT>
__global__ void __launch_bounds__(256, 2) k_gemm(GemmArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ASZ = BM * BK, BSZ = BN * BK;
  __shared__ __attribute__((aligned(16))) f16 smem[2 * (ASZ + BSZ)];

  // XCD-aware bijective remap of the linear block id (MI355X_MICROARCH: blocks b, b+8 share an XCD)
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int ntile = nbm * nbn;
  const int nwg = ntile * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int bm, bn, split;
  tile_of(p, wg, nbm, nbn, bm, bn, split);
  const int m0 = bm * BM, n0 = bn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * WM, wn0 = (wid & 1) * WN;
  const int fr = lane & 15, fq = lane >> 4;

  ALoader<BM, AMODE> al;
  BLoader<BN, BFMT> bl;
  al.init(p, m0, kbeg);
  bl.init(p, n0);

  // acc[i][j]: C^T tile (rows n = n0 + wn0 + 16j + 4fq + r, column m = m0 + wm0 + 16i + fr)
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  al.load(p, kbeg);
  bl.load(p, kbeg);
  al.store(smem);
  bl.store(smem + ASZ);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      al.load(p, kbeg + (kt + 1) * BK);
      bl.load(p, kbeg + (kt + 1) * BK);
    }
    const f16* As = smem + cur * (ASZ + BSZ);
    const f16* Bs = As + ASZ;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(As + swz(wm0 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f16x8*>(Bs + swz(wn0 + j * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      f16* nx = smem + (cur ^ 1) * (ASZ + BSZ);
      al.store(nx);
      bl.store(nx + ASZ);
    }
    __syncthreads();
  }

  gemm_epilogue<BM, BN, 256, TM, TN, SPLIT, 2 * (ASZ + BSZ), AMODE != AM_LINEAR>(p, acc, smem, m0, n0, wm0, wn0, split);
}

// ---- LDS-DMA variant ----------------------------------------------------------------------
// Operands go HBM/L2 -> LDS directly (buffer_load_dwordx4 ... lds): no staging registers, no
// ds_write, and the loads of the next ST-1 K steps stay in flight across the per-step barrier
// (counted vmcnt + raw s_barrier; __syncthreads would drain them).  A wave-instruction writes
// 64 x 16 B lane-linearly = 8 LDS rows of 128 B; the XOR swizzle is applied on the SOURCE side
// (lane l of the row group loads K chunk (l & 7) ^ (row & 7)), so fragments are read with the
// same swz() as the register-staged kernel.  OOB chunks (rows past M/N, conv halo, K tail)
// carry offsets >= 2^31 and land as zeros.  F16 B operand only (the reference's dequantized
// buffer); quantized codes use the register-staged kernel, which dequantizes while staging.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, f16* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, (int)voff, 0, 0, 0);
}

// LDS stage layout of the DMA kernels: rows of BKT halves (BKT = 64: 8 chunks of 16 B,
// 128-B rows, chunk ^= row & 7;  BKT = 32: 4 chunks, 64-B rows, chunk ^= (row >> 1) & 3) -
// both conflict-free for the 16-row ds_read_b128 fragment reads.
template <int BKT>
__device__ __forceinline__ int swz_t(int row, int chunk) {
  if constexpr (BKT == 64) return row * 64 + ((chunk ^ (row & 7)) << 3);
  else return row * 32 + ((chunk ^ ((row >> 1) & 3)) << 3);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// thread (wave w, lane l), load slot j: wave-instruction g = j * NW + w covers rows 8g..8g+7;
// lane l -> row 8g + (l >> 3), LDS chunk l & 7 holding K chunk (l & 7) ^ (l >> 3).
template <int BM, int NT, int AMODE, int BKT>
struct ADma {
  static constexpr int NW = NT / 64;
  static constexpr int CPR = BKT / 8;    // 16-B chunks per LDS row
  static constexpr int RPW = 64 / CPR;   // rows per wave-instruction (1 KB)
  static constexpr int L = BM * CPR / NT;
  static_assert(BM * CPR % NT == 0, "A tile rows must split evenly over the wave-instructions");
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[L];
  int pix[L], ih0[L], iw0[L];
  int ky, kx, ci0, gc;

  __device__ void init(const GemmArgs& p, int m0, int kbeg, int wid) {
    rs = rsrc(p.a, p.a_bytes);
    const int lane = threadIdx.x & 63;
    gc = BKT == 64 ? ((lane & 7) ^ (lane >> 3)) * 8 : ((lane & 3) ^ ((lane >> 3) & 3)) * 8;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int m = m0 + (j * NW + wid) * RPW + lane / CPR;
      const bool ok = m < p.M;
      if (AMODE == AM_LINEAR) {
        rowoff[j] = ok ? (unsigned)m * (unsigned)p.lda * 2u : OOB;
      } else {
        const int mm = ok ? m : 0;
        const int ow = mm % p.Wo, oh = (mm / p.Wo) % p.Ho, n = mm / (p.Wo * p.Ho);
        pix[j] = ok ? n * p.Hs * p.Ws : -1;
        ih0[j] = oh * p.stride - p.pad;
        iw0[j] = ow * p.stride - p.pad;
      }
    }
    if (AMODE == AM_CONV) {
      const int kpos = kbeg / p.Cip;
      ci0 = kbeg - kpos * p.Cip;
      ky = kpos / p.kw;
      kx = kpos - ky * p.kw;
    }
  }
  __device__ __forceinline__ unsigned conv_off(const GemmArgs& p, int j, int kyy, int kxx, int ci) const {
    const int ih = ih0[j] + kyy, iw = iw0[j] + kxx;
    const bool ok = pix[j] >= 0 && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
    return ok ? (unsigned)((pix[j] + sh * p.Ws + sw) * p.Cip + ci) * 2u : OOB;
  }
  __device__ void issue(const GemmArgs& p, int k0, f16* sa, int wid) {
    if (AMODE == AM_LINEAR) {
      const unsigned ko = k0 + gc < p.K ? (unsigned)(k0 + gc) * 2u : OOB;
#pragma unroll
      for (int j = 0; j < L; ++j) glds16(rs, sa + (j * NW + wid) * RPW * BKT, rowoff[j] + ko);
    } else if (AMODE == AM_CONV) {
#pragma unroll
      for (int j = 0; j < L; ++j) glds16(rs, sa + (j * NW + wid) * RPW * BKT, conv_off(p, j, ky, kx, ci0 + gc));
      ci0 += BKT;
      if (ci0 == p.Cip) {
        ci0 = 0;
        if (++kx == p.kw) {
          kx = 0;
          ++ky;
        }
      }
    } else {
      const int k = k0 + gc;
      const int kpos = k / p.Cip, ci = k - kpos * p.Cip;
      const int kyy = kpos / p.kw, kxx = kpos - kyy * p.kw;
#pragma unroll
      for (int j = 0; j < L; ++j)
        glds16(rs, sa + (j * NW + wid) * RPW * BKT, k < p.K ? conv_off(p, j, kyy, kxx, ci) : OOB);
    }
  }
};

template <int BN, int NT, int BKT>
struct BDma {
  // BN / RPW row groups over NW waves; when they do not split evenly the first G % NW waves
  // issue one wave-instruction more (wave-uniform guard; the per-wave count feeds vmcnt)
  static constexpr int NW = NT / 64;
  static constexpr int CPR = BKT / 8;
  static constexpr int RPW = 64 / CPR;
  static constexpr int G = BN / RPW;
  static constexpr int L = (G + NW - 1) / NW;
  static_assert(BN % RPW == 0, "B tile rows in whole wave-instruction groups");
  __amdgpu_buffer_rsrc_t rs;
  unsigned rowoff[L];
  int gc;
  __device__ static int count(int wid) { return G / NW + (wid < G % NW ? 1 : 0); }
  __device__ void init(const GemmArgs& p, int n0, int wid) {
    rs = rsrc(p.b, p.b_bytes);
    const int lane = threadIdx.x & 63;
    gc = BKT == 64 ? ((lane & 7) ^ (lane >> 3)) * 8 : ((lane & 3) ^ ((lane >> 3) & 3)) * 8;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int n = n0 + (j * NW + wid) * RPW + lane / CPR;
      rowoff[j] = n < p.N ? (unsigned)n * (unsigned)p.K * 2u : OOB;
    }
  }
  __device__ void issue(const GemmArgs& p, int k0, f16* sb, int wid) {
    const unsigned ko = k0 + gc < p.K ? (unsigned)(k0 + gc) * 2u : OOB;
#pragma unroll
    for (int j = 0; j < L; ++j)
      if (G % NW == 0 || j * NW + wid < G) glds16(rs, sb + (j * NW + wid) * RPW * BKT, rowoff[j] + ko);
  }
};

// ---- packed-int4 B operand in the LDS-DMA families ------------------------------------------
// The codes go HBM -> LDS as they are stored (qd_pack_int4: BKT / 2 bytes per row and K step, so
// one 1-KB DMA wave-instruction moves 2048 / BKT weight rows: a quarter of the fp16 operand's
// bytes), followed in the stage by the step's group-scale row s[k0 / group][n0 .. n0 + BN) (fp16,
// one piece, from the [K / group][N] copy; group % BKT == 0).  BKT 64 rows hold two 16-B chunks,
// swapped on rows with bit 3 set (the DMA source is permuted, as the fp16 stages' XOR swizzle), so
// the 16 rows x 4 dwords a fragment read touches are bank-conflict free.  A lane's B fragment
// (row r, k = 32ks + 8fq .. + 7) is one ds_read_b32 of codes + its row's scale, dequantized in
// registers (w4_frag); half(q * s) is the reference's dequantized weight, so every int4 variant
// gives the fp16-buffer GEMM's bits.
template <int BN, int NT, int BKT>
struct BDma4 {
  static constexpr int NW = NT / 64;
  static constexpr int RB = BKT / 2;           // code bytes per row and stage
  static constexpr int RPP = 1024 / RB;        // rows per 1-KB piece
  static constexpr int G = (BN + RPP - 1) / RPP;
  static constexpr int L = (G + NW - 1) / NW;
  static constexpr int CODE_H = G * 512;       // halves of the code region (whole pieces)
  static constexpr int SZ = CODE_H + 512;      // + the scale row piece
  static constexpr int SW = NW - 1;            // the wave that DMAs the scale row
  __amdgpu_buffer_rsrc_t rs, srs;
  unsigned rowoff[L];
  unsigned soff;
  __device__ static int count(int wid) { return G / NW + (wid < G % NW ? 1 : 0) + (wid == SW ? 1 : 0); }
  __device__ void init(const GemmArgs& p, int n0, int wid) {
    rs = rsrc(p.b, p.b_bytes);
    srs = rsrc(p.bscale_t, (unsigned)((p.K / p.group) * p.N * 2));
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int r = (j * NW + wid) * RPP + lane * 16 / RB;  // RB / 16 lanes per row
      const int n = n0 + r;
      // BKT 64: lane pair (2r', 2r' + 1) fills row r' chunks 0 / 1 with K halves (0, 1) ^ (r' >> 3 & 1)
      const unsigned ch = BKT == 64 ? (unsigned)(((lane & 1) ^ ((r >> 3) & 1)) * 16) : 0u;
      rowoff[j] = (r < BN && n < p.N) ? (unsigned)n * (unsigned)(p.K / 2) + ch : OOB;
    }
    soff = (lane * 8 < BN && n0 + lane * 8 < p.N) ? (unsigned)(n0 + lane * 8) * 2u : OOB;
  }
  __device__ void issue(const GemmArgs& p, int k0, f16* sb, int wid) {
    const unsigned ko = (unsigned)(k0 / 2);
#pragma unroll
    for (int j = 0; j < L; ++j)
      if (G % NW == 0 || j * NW + wid < G) glds16(rs, sb + (j * NW + wid) * 512, rowoff[j] + ko);
    if (wid == SW) glds16(srs, sb + CODE_H, soff == OOB ? OOB : soff + (unsigned)(k0 / p.group) * (unsigned)p.N * 2u);
  }
};

typedef f16 f16x2v __attribute__((ext_vector_type(2)));
// B fragment of row `row`, k = 32ks + 8fq .. + 7 of the stage, from an int4 stage.  Per dword of
// 8 offset-binary codes (pairs of consecutive k in nibbles j / j + 4): the pair in nibble 0 / 4
// OR'd into fp16 0x6400 is (1024 + c, 1024 + c'); the pair in nibble 1 / 5 lands on mantissa bits
// 4..7 and with 0x5400 is (64 + c, 64 + c') (ulp 1/16 there: c counts whole units); the same two
// masks on w >> 8 give pairs 2 and 3.  Subtracting 1032 / 72 leaves (q, q') exactly, and one
// v_pk_mul_f16 by (s, s) rounds q * s once: 1 shift + 4 and-or + 4 sub + 4 mul per 8 weights.
__device__ __forceinline__ f16x8 w4_dq8(unsigned w, f16 s, unsigned m64, unsigned m54) {
  const f16x2v s2 = {s, s};
  const f16x2v o1032 = {(f16)1032.f, (f16)1032.f}, o72 = {(f16)72.f, (f16)72.f};
  const unsigned w8 = w >> 8;
  const f16x2v q0 = __builtin_bit_cast(f16x2v, (w & 0x000F000Fu) | m64) - o1032;
  const f16x2v q1 = __builtin_bit_cast(f16x2v, (w & 0x00F000F0u) | m54) - o72;
  const f16x2v q2 = __builtin_bit_cast(f16x2v, (w8 & 0x000F000Fu) | m64) - o1032;
  const f16x2v q3 = __builtin_bit_cast(f16x2v, (w8 & 0x00F000F0u) | m54) - o72;
  const f16x2v v0 = q0 * s2, v1 = q1 * s2, v2 = q2 * s2, v3 = q3 * s2;
  return (f16x8){v0[0], v0[1], v1[0], v1[1], v2[0], v2[1], v3[0], v3[1]};
}
template <int BKT>
__device__ __forceinline__ f16x8 w4_frag(const f16* sb, int row, int ks, int fq, int code_h, unsigned m64,
                                         unsigned m54) {
  constexpr int RB = BKT / 2;
  const int ch = BKT == 64 ? ((ks ^ ((row >> 3) & 1)) << 4) : 0;
  const unsigned w = *reinterpret_cast<const unsigned*>(reinterpret_cast<const char*>(sb) + row * RB + ch + fq * 4);
  return w4_dq8(w, sb[code_h + row], m64, m54);
}

// the two magics in VGPRs (opaque to constant folding), so each mask-and-or is one v_and_or_b32
// with the mask as its single literal
__device__ __forceinline__ void w4_magics(unsigned& m64, unsigned& m54) {
  asm volatile("v_mov_b32 %0, 0x64006400" : "=v"(m64));
  asm volatile("v_mov_b32 %0, 0x54005400" : "=v"(m54));
}

// vmcnt of a value the caller's unrolling makes a compile-time constant (folds to one s_waitcnt)
__device__ __forceinline__ void wait_vm_c(int n) {
  if (n <= 0) wait_vm<0>();
  else if (n == 1) wait_vm<1>();
  else if (n == 2) wait_vm<2>();
  else if (n == 3) wait_vm<3>();
  else if (n == 4) wait_vm<4>();
  else if (n == 5) wait_vm<5>();
  else if (n == 6) wait_vm<6>();
  else if (n == 7) wait_vm<7>();
  else if (n == 8) wait_vm<8>();
  else if (n == 9) wait_vm<9>();
  else if (n == 10) wait_vm<10>();
  else wait_vm<0>();
}

#define QD_VM_CASE(n) \
  case n:             \
    wait_vm<n>();     \
    break;
// vmcnt with a wave-uniform runtime count (immediate operand: one case per value)
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    QD_VM_CASE(0) QD_VM_CASE(1) QD_VM_CASE(2) QD_VM_CASE(3) QD_VM_CASE(4) QD_VM_CASE(5) QD_VM_CASE(6)
    QD_VM_CASE(7) QD_VM_CASE(8) QD_VM_CASE(9) QD_VM_CASE(10) QD_VM_CASE(11) QD_VM_CASE(12)
    QD_VM_CASE(13) QD_VM_CASE(14) QD_VM_CASE(15) QD_VM_CASE(16) QD_VM_CASE(17) QD_VM_CASE(18)
    QD_VM_CASE(19) QD_VM_CASE(20) QD_VM_CASE(21) QD_VM_CASE(22) QD_VM_CASE(23) QD_VM_CASE(24)
    QD_VM_CASE(25) QD_VM_CASE(26) QD_VM_CASE(27) QD_VM_CASE(28) QD_VM_CASE(29) QD_VM_CASE(30)
    QD_VM_CASE(31) QD_VM_CASE(32)
    default: wait_vm<0>(); break;
  }
}
#undef QD_VM_CASE

// PIPE 0: per K step  wait(own loads of tile k) -> barrier -> issue tile k+ST-1 -> read + MFMA.
// PIPE 1 (ST >= 3): the barrier sits between the two K=32 halves of a step, and the fragments
//   of the next half are read while the current half's MFMAs run:
//     MFMA(k, half 0) | read(k, half 1)  -> wait(tile k+1) -> barrier -> issue tile k+2 ->
//     MFMA(k, half 1) | read(k+1, half 0)
//   (the stage written after the barrier held tile k-1, whose last reads precede it).
constexpr int dma_lds_halves(int bm, int bn, int st, int bkt = 64) {
  return st * (bm + bn) * bkt > epi_lds_halves(bm, bn) ? st * (bm + bn) * bkt : epi_lds_halves(bm, bn);
}
// fp8 stages carry the group-scale row (BN fp32, one 1-KB DMA wave-instruction) after the B tile
constexpr int F8_SCL = 512;  // halves
constexpr int dma_lds_halves_f8(int bm, int bn, int st) {
  return st * ((bm + bn) * 64 + F8_SCL) > epi_lds_halves(bm, bn) ? st * ((bm + bn) * 64 + F8_SCL) : epi_lds_halves(bm, bn);
}
// minimum waves per SIMD for __launch_bounds__: (blocks that fit the 160 KB LDS) x waves / 4
constexpr int dma_waves_per_eu(int bm, int bn, int st, int nt, int bkt = 64) {
  return (163840 / (2 * dma_lds_halves(bm, bn, st, bkt))) * nt / 256 > 0
             ? (163840 / (2 * dma_lds_halves(bm, bn, st, bkt))) * nt / 256
             : 1;
}

// int4 B stages: A tile + the BDma4 code pieces and scale row
constexpr int w4_stage_halves(int bm, int bn, int bkt) {
  return bm * bkt + ((bn + 2048 / bkt - 1) / (2048 / bkt)) * 512 + 512;
}
constexpr int dma_lds_halves_w4(int bm, int bn, int st, int bkt) {
  return st * w4_stage_halves(bm, bn, bkt) > epi_lds_halves(bm, bn) ? st * w4_stage_halves(bm, bn, bkt) : epi_lds_halves(bm, bn);
}
// (at most 2 waves per SIMD: the smaller int4 stages would admit 3 blocks, whose 170-register cap
// spills the 128 x 160 tile's accumulators + prefetched residual)
constexpr int dma_waves_per_eu_w4(int bm, int bn, int st, int nt, int bkt) {
  return (163840 / (2 * dma_lds_halves_w4(bm, bn, st, bkt))) * nt / 256 > 2
             ? 2
             : (163840 / (2 * dma_lds_halves_w4(bm, bn, st, bkt))) * nt / 256 > 0
                   ? (163840 / (2 * dma_lds_halves_w4(bm, bn, st, bkt))) * nt / 256
                   : 1;
}

// PERSIST (int8 linears, lock-step pipeline, unsplit; the template also builds for fp16 weights, whose
// persistent tiles measured no faster on any SD shape - profiles/r05q_sweep_f16.log): a grid of p.pgrid blocks; block b runs the
// logical tiles b, b + grid, ... (XCD-remapped like the one-tile grid).  After a tile's K loop the
// first ST-1 K steps of the block's next tile are issued into the (now free) stages BEFORE the tile's
// epilogue when that epilogue touches no LDS (direct stores, no column amax), so the next tile's
// L2 -> LDS traffic runs under this tile's scaling, conversions and output stores; the next tile's
// first K step then waits for every outstanding memory op (its DMA is older than the stores).  The
// register cap is half the one-tile kernel's occupancy (the tile loop keeps the next tile's DMA
// state and the loop-invariant lane coordinates live through the epilogue: at the one-tile cap the
// 128 x 160 tile spills ~50 VGPRs).
template <int BM, int BN, int WGM, int WGN, int ST, int PIPE, int BKT, int AMODE, bool SPLIT, bool I8 = false,
          bool F8 = false, bool W4 = false, bool PERSIST = false, bool DPOSTK = false>
__global__ void __launch_bounds__(64 * WGM * WGN,
                                  W4        ? dma_waves_per_eu_w4(BM, BN, ST, 64 * WGM * WGN, BKT)
                                  : PERSIST ? (dma_waves_per_eu(BM, BN, ST, 64 * WGM * WGN, BKT) / 2 > 0
                                                   ? dma_waves_per_eu(BM, BN, ST, 64 * WGM * WGN, BKT) / 2 : 1)
                                            : dma_waves_per_eu(BM, BN, ST, 64 * WGM * WGN, BKT))
    k_gemm_dma(GemmArgs p) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ASZ = BM * BKT;
  constexpr int SSZ = W4 ? ASZ + BDma4<BN, NT, BKT>::SZ : (BM + BN) * BKT + (F8 ? F8_SCL : 0);
  constexpr int LDSZ = W4 ? dma_lds_halves_w4(BM, BN, ST, BKT) : F8 ? dma_lds_halves_f8(BM, BN, ST) : dma_lds_halves(BM, BN, ST, BKT);
  constexpr int KSUB = BKT / 32;  // 32-deep MFMA slices per stage
  static_assert(PIPE == 0 || (ST >= 3 && BKT == 64), "split-phase pipeline needs >= 3 stages of 64");
  static_assert(!I8 || (BKT == 32 && PIPE == 0), "int8: one 64-code MFMA k-slice per 64-B LDS row");
  static_assert(!F8 || (BKT == 64 && PIPE == 0 && !SPLIT && BN * 4 <= 1024),
                "fp8: one 128-code group per 128-B LDS row, no split-K, the scale row in one DMA piece");
  static_assert(!W4 || (!I8 && !F8 && PIPE == 0 && AMODE == AM_LINEAR && BN <= 512),
                "int4: lock-step pipeline, linear A operand, one scale piece");
  static_assert(!PERSIST || (!F8 && !W4 && PIPE == 0 && AMODE == AM_LINEAR && !SPLIT),
                "persistent: int8 / fp16 linears, lock-step pipeline, unsplit");
  using AL = ADma<BM, NT, AMODE, BKT>;
  using BL = std::conditional_t<W4, BDma4<BN, NT, BKT>, BDma<BN, NT, BKT>>;
  __shared__ __attribute__((aligned(16))) f16 smem[LDSZ];

  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int ntile = nbm * nbn;
  const int nwg = ntile * p.splits;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  auto xmap = [&](int b) {  // (logical) block index -> XCD-contiguous tile index
    const int xcd = b & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  };
  int lt = blockIdx.x;
  int bm, bn, split;
  tile_of(p, xmap(lt), nbm, nbn, bm, bn, split);
  int m0 = bm * BM, n0 = bn * BN;
  int kbeg = split * p.kps;
  int kend = min(p.K, kbeg + p.kps);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int per = AL::L + BL::count(wid) + (F8 && wid == 0 ? 1 : 0);  // this wave's loads per K step

  AL al;
  BL bl;
  al.init(p, m0, kbeg, wid);
  bl.init(p, n0, wid);
  // fp8: wave 0 DMAs the stage's group-scale row gs[k / 128][n0 .. n0 + BN) (4 floats per lane)
  const __amdgpu_buffer_rsrc_t srs = rsrc(F8 ? (const void*)p.gs : p.b, F8 ? (unsigned)(((p.K + 63) / 64) * p.N * 4) : 0u);
  unsigned soff = OOB;
  if constexpr (F8) {
    const int nn = n0 + lane * 4;
    soff = (lane * 4 < BN && nn < p.N) ? (unsigned)nn * 4u : OOB;
  }
  auto issue_scale = [&](int k0, f16* stage) {
    if constexpr (F8) {
      if (wid == 0) glds16(srs, stage + ASZ + BN * BKT, soff == OOB ? OOB : soff + (unsigned)(k0 / 64) * (unsigned)p.N * 4u);
    }
  };

  f32x4 acc[TM][TN];
  i32x4 iacc[I8 ? TM : 1][I8 ? TN : 1];
  // the first ST-1 K steps of the tile whose K range starts at kb (nks steps)
  auto prologue = [&](int kb, int nks) {
#pragma unroll
    for (int s = 0; s < ST - 1; ++s) {
      if (s < nks) {
        al.issue(p, kb + s * BKT, smem + s * SSZ, wid);
        bl.issue(p, kb + s * BKT, smem + s * SSZ + ASZ, wid);
        issue_scale(kb + s * BKT, smem + s * SSZ);
      }
    }
  };
  int nk = (kend - kbeg + BKT - 1) / BKT;
  prologue(kbeg, nk);
  bool drain = false;  // (PERSIST) a later tile: its first K step waits for its stage past the stores
  int nst = 0;         // (PERSIST) store instructions the previous tile's epilogue issued after the DMA
  for (;;) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if constexpr (I8) iacc[i][j] = (i32x4){0, 0, 0, 0};
    }
  unsigned m64 = 0, m54 = 0;
  if constexpr (W4) w4_magics(m64, m54);
  // (PERSIST: the fragment addresses are re-derived per tile from an opaque copy of the lane
  // coordinates - hoisted out of the tile loop they stay live through every epilogue and spill)
  int frl = fr, fql = fq;
  if constexpr (PERSIST) asm volatile("" : "+v"(frl), "+v"(fql));
  auto read_frags = [&](const f16* As, int ks, f16x8 (&af)[TM], f16x8 (&bf)[TN]) {
    const f16* Bs = As + ASZ;
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(As + swz_t<BKT>(wm0 + i * 16 + frl, ks * 4 + fql));
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (W4) bf[j] = w4_frag<BKT>(Bs, wn0 + j * 16 + frl, ks, fql, BDma4<BN, NT, BKT>::CODE_H, m64, m54);
      else bf[j] = *reinterpret_cast<const f16x8*>(Bs + swz_t<BKT>(wn0 + j * 16 + frl, ks * 4 + fql));
    }
  };
  auto mfmas = [&](const f16x8 (&af)[TM], const f16x8 (&bf)[TN]) {
#ifdef QD_ABLATE_NO_MFMA  // diagnostic build: staging + fragment reads only (values kept live)
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bf[j]));
#else
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (I8)
          iacc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, bf[j]),
                                                             __builtin_bit_cast(i32x4, af[i]), iacc[i][j], 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
      }
#endif
  };
  auto sync = [&](int ahead) {  // own loads of the awaited tile landed, `ahead` later tiles in flight
    wait_vm_rt(ahead * per);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if constexpr (PIPE == 0) {
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (PERSIST && kt == 0 && drain) {
        // younger than this tile's first stage: its next ST-2 stages and the previous tile's stores
        // (counted in issue order with the DMA; nst = 0 after an LDS-tile epilogue)
        wait_vm_rt(min(ST - 2, nk - 1) * per + nst);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      } else {
        sync(min(ST - 2, nk - 1 - kt));
      }
      if (kt + ST - 1 < nk) {
        int nx = cur + ST - 1;
        if (nx >= ST) nx -= ST;
        al.issue(p, kbeg + (kt + ST - 1) * BKT, smem + nx * SSZ, wid);
        bl.issue(p, kbeg + (kt + ST - 1) * BKT, smem + nx * SSZ + ASZ, wid);
        issue_scale(kbeg + (kt + ST - 1) * BKT, smem + nx * SSZ);
      }
      if constexpr (F8) {
        // the stage's two 16-B chunks per row (fq, fq + 4) form the 32-code operand; A and B take
        // them in the same order, so the MFMA sums the stage's 128 codes exactly once each
        f16x8 a0[TM], b0[TN], a1[TM], b1[TN];
        read_frags(smem + cur * SSZ, 0, a0, b0);
        read_frags(smem + cur * SSZ, 1, a1, b1);
        const float* sg = reinterpret_cast<const float*>(smem + cur * SSZ + ASZ + BN * BKT);
        f32x4 sgv[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) sgv[j] = *reinterpret_cast<const f32x4*>(sg + wn0 + j * 16 + fq * 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const i32x8 bop = f8_operand(a0[i], a1[i]);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const f32x4 t = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                f8_operand(b0[j], b1[j]), bop, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0, 127, 0, 127);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(t[r], sgv[j][r], acc[i][j][r]);
          }
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KSUB; ++ks) {
          f16x8 af[TM], bf[TN];
          read_frags(smem + cur * SSZ, ks, af, bf);
          mfmas(af, bf);
        }
      }
      if (++cur == ST) cur = 0;
    }
  } else {
    f16x8 a0[TM], b0[TN], a1[TM], b1[TN];
    if (nk > 0) {
      sync(min(ST - 2, nk - 1));
      read_frags(smem, 0, a0, b0);
    }
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      int nxt = cur + 1;
      if (nxt == ST) nxt = 0;
      read_frags(smem + cur * SSZ, 1, a1, b1);
      mfmas(a0, b0);
      if (kt + 1 < nk) {
        sync(min(ST - 3, nk - 2 - kt));  // tile kt+1 landed everywhere; tile kt-1 fully read
        if (kt + ST - 1 < nk) {
          int nx = cur + ST - 1;
          if (nx >= ST) nx -= ST;
          al.issue(p, kbeg + (kt + ST - 1) * BKT, smem + nx * SSZ, wid);
          bl.issue(p, kbeg + (kt + ST - 1) * BKT, smem + nx * SSZ + ASZ, wid);
        }
        read_frags(smem + nxt * SSZ, 0, a0, b0);
      }
      mfmas(a1, b1);
      cur = nxt;
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (I8) i8_scale<TM, TN, SPLIT>(p, iacc, acc, m0, n0, wm0, wn0);
  if constexpr (F8) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float s = p.sa[min(m0 + wm0 + i * 16 + fr, p.M - 1)];
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] *= s;
    }
  }
  if constexpr (PERSIST) {
    const int ln = lt + (int)gridDim.x;
    const bool more = ln < nwg;
    int m0n = 0, n0n = 0, kbn = 0, ken = 0, bmn = 0, bnn = 0, spn = 0;
    if (more) {
      tile_of(p, xmap(ln), nbm, nbn, bmn, bnn, spn);
      m0n = bmn * BM;
      n0n = bnn * BN;
      kbn = spn * p.kps;
      ken = min(p.K, kbn + p.kps);
    }
    const int nkn = (ken - kbn + BKT - 1) / BKT;
    // a direct-store epilogue with no column maxima: every output word is formed (its loads
    // consumed) before the next tile's DMA is issued, then only stored
    const bool early = more && epi_direct<BN, TM, TN, false, true>(p) && !((p.epi & QD_EPI_AMAX) && p.amax);
    nst = 0;
    if constexpr (epi_direct_ok<TM, TN, true>()) {
      if (early) {
        u32x4 wo[TM][TN / 2 + (TN & 1)];
        direct_outputs<TM, TN>(p, acc, m0, n0, wm0, wn0, wo);
        al.init(p, m0n, kbn, wid);
        bl.init(p, n0n, wid);
        prologue(kbn, nkn);
        // the first K step's counted wait (wait_vm_rt(... + nst) above) assumes exactly the nst
        // stores below are younger than the DMA just issued: pin that issue order against both the
        // IR (memory clobber) and the machine scheduler (sched_barrier 0: nothing crosses)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        nst = direct_stores<TM, TN>(p, wo, m0, n0, wm0, wn0);
      }
    }
    if (!early) gemm_epilogue<BM, BN, NT, TM, TN, SPLIT, LDSZ, false>(p, acc, smem, m0, n0, wm0, wn0, split);
    if (!more) break;
    if (!early) {
      __syncthreads();  // the epilogue's LDS C tile / column maxima are read
      al.init(p, m0n, kbn, wid);
      bl.init(p, n0n, wid);
      prologue(kbn, nkn);
    }
    lt = ln;
    m0 = m0n;
    n0 = n0n;
    split = spn;
    kbeg = kbn;
    kend = ken;
    nk = nkn;
    drain = true;
  } else {
    gemm_epilogue<BM, BN, NT, TM, TN, SPLIT, LDSZ, AMODE != AM_LINEAR, true, DPOSTK>(p, acc, smem, m0, n0, wm0, wn0,
                                                                                     split);
    break;
  }
  }
}

// ---- A-stationary int8 linear (qd_gemm_force 190-192; round 5) ------------------------------
// For short K (K = KC codes, 320 or 640) and wide N the one-tile kernels restream the A rows once per
// N tile: at M 32768 N 2560 K 320 a CU moves 1.2 MB of operands at the ~25 GB/s per CU its LDS-DMA
// ring sustains inside a GEMM.  Here a block (8 waves, WGM x WGN, wave tile 64 x BN/WGN)
// keeps its BM x KC A panel in LDS for all of its N tiles (loaded once) and streams only the weight
// rows through a RING-deep ring that runs continuously across the tiles - W step g = (tile g / NK,
// k-step g % NK) - so a tile's epilogue runs while the next tile's first stages land.  Per CU at that
// shape: 80 KB of A + 400 KB of W.  The epilogue is the two-phase direct store (direct_outputs /
// direct_stores: plain, bias, GEGLU at TN 4); its scale / bias loads are issued at the top of the
// tile's last step, before that step's DMA, so waiting for them never waits for younger DMA; the
// stores are counted into the next waits (vmcnt counts loads, stores and LDS-DMA in issue order).
// Every step issues the same DMA (past the last step: a dummy piece into a scratch slot), so every
// count is exact.  Exact int32 sums, the i8_scale / epilogue arithmetic: the same bits as every
// other int8 variant.
template <int BM, int BN, int KC, int RING>
__global__ void __launch_bounds__(512, 1) k_gemm_as_i8(GemmArgs p) {
  constexpr int NT = 512, NW = 8, WGM = BM / 64, WGN = NW / WGM;
  constexpr int WN = BN / WGN, TM = 4, TN = WN / 16, NK = KC / 64;
  constexpr int ASZ = BM * 32, BSZ = BN * 32;  // halves per A / W stage (64-B rows)
  static_assert(BM % 64 == 0 && NW % WGM == 0 && WN % 16 == 0 && KC % 64 == 0 && RING >= 3, "A-stationary tile");
  static_assert(epi_direct_ok<TM, TN, true>(), "A-stationary: direct-store epilogue tiles only");
  static_assert(NK >= RING - 1, "one store batch pending at a time");
  using AL = ADma<BM, NT, AM_LINEAR, 32>;
  using BL = BDma<BN, NT, 32>;
  static_assert((BN / 16) % NW == 0, "the same number of 16-row W pieces per wave and step");
  constexpr int PW = BN / 16 / NW;  // W pieces per wave and step
  __shared__ __attribute__((aligned(16))) f16 smem[NK * ASZ + (RING + 1) * BSZ];
  f16* const apanel = smem;
  f16* const ring = smem + NK * ASZ;
  f16* const scratch = ring + RING * BSZ;  // the dummy pieces past the last step

  const int npanel = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int nsplit = p.as_nsplit;
  const int nwg = npanel * nsplit;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int panel = wg / nsplit, part = wg - panel * nsplit;
  const int tper = (ntn + nsplit - 1) / nsplit;
  const int t0 = part * tper, ntile = min(ntn, t0 + tper) - t0;
  if (ntile <= 0) return;  // (block-uniform)
  const int m0 = panel * BM;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * 64, wn0 = (wid % WGN) * WN;
  const int fr = lane & 15, fq = lane >> 4;

  AL al;
  al.init(p, m0, 0, wid);
#pragma unroll
  for (int s = 0; s < NK; ++s) al.issue(p, s * 32, apanel + s * ASZ, wid);
  BL bl;
  int btile = -1;
  const int T = ntile * NK;
  // W step g -> ring slot g % RING (steps >= T: a dummy piece into the scratch slot)
  auto issue_w = [&](int g) {
    const int gg = g < T ? g : T - 1;
    const int j = gg / NK, s = gg - j * NK;
    if (j != btile) {
      bl.init(p, (t0 + j) * BN, wid);
      btile = j;
    }
    bl.issue(p, s * 32, g < T ? ring + (g % RING) * BSZ : scratch, wid);
  };
#pragma unroll
  for (int g = 0; g < RING - 1; ++g) issue_w(g);

  i32x4 iacc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) iacc[i][j] = (i32x4){0, 0, 0, 0};
  int nst = 0, store_after = -1;  // store instructions of the last epilogue, issued after W step store_after
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  for (int g = 0; g < T; ++g) {
    const int j = g / NK, s = g - j * NK;
    const int n0 = (t0 + j) * BN;
    // own pieces of step g landed; younger: the next RING-2 steps' pieces (+ the stores issued after
    // step store_after, when g <= store_after)
    wait_vm_rt((RING - 2) * PW + (g <= store_after ? nst : 0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    float sa[TM];
    f32x4 sw[TN];
    f16x4 bq[TN];
    if (s == NK - 1) {  // the epilogue's operands, before this step's DMA (waiting for them then
                        // waits for older pieces only)
#pragma unroll
      for (int i = 0; i < TM; ++i) sa[i] = p.sa[min(m0 + wm0 + i * 16 + fr, p.M - 1)];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int n = n0 + wn0 + jj * 16 + fq * 4;
        sw[jj] = n < p.N ? *reinterpret_cast<const f32x4*>(p.sw + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
        bq[jj] = (has_bias && n < p.N) ? *reinterpret_cast<const f16x4*>(p.bias + n) : f16x4{};
      }
      asm volatile("" ::: "memory");
    }
    issue_w(g + RING - 1);
    {
      const f16* As = apanel + s * ASZ;
      const f16* Bs = ring + (g % RING) * BSZ;
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(As + swz_t<32>(wm0 + i * 16 + fr, fq));
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) bf[jj] = *reinterpret_cast<const f16x8*>(Bs + swz_t<32>(wn0 + jj * 16 + fr, fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
          iacc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, bf[jj]),
                                                              __builtin_bit_cast(i32x4, af[i]), iacc[i][jj], 0, 0, 0);
    }
    if (s == NK - 1) {
      f32x4 acc[TM][TN];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][jj][r] = ((float)iacc[i][jj][r] * sa[i]) * sw[jj][r];
          iacc[i][jj] = (i32x4){0, 0, 0, 0};
        }
      u32x4 wo[TM][TN / 2 + (TN & 1)];
      direct_outputs_pre<TM, TN>(p, acc, bq, m0, n0, wm0, wn0, wo);
      nst = direct_stores<TM, TN>(p, wo, m0, n0, wm0, wn0);
      store_after = g + RING - 1;
    }
  }
  wait_vm<0>();  // (the dummy pieces land in this block's LDS before it exits)
}

// ---- ping-pong GEMM (256 x BN tile, 8 waves, BK 32, 4-stage LDS-DMA ring) ----------------
// 8 waves = 2 (M halves) x 4 (N quarters); wave tile 128 x BN/4.  The two M-half wave groups
// run one barrier apart ("ping-pong"): each SIMD hosts one wave of each group, and between two
// consecutive workgroup barriers one group issues its MFMAs while the other issues its LDS
// fragment reads and its share of the LDS-DMA prefetch, so the matrix pipe is fed by one group
// while the other waits on memory.  A K-tile (32 deep) is two phases per wave:
//   phase a: read A frags 0-3 + all B frags, issue A loads of K-tile kt+2 | MFMAs (i 0-3)
//   phase b: read A frags 4-7, wait for K-tile kt+1, issue B loads of kt+2  | MFMAs (i 4-7)
// each phase = [ds_reads, DMA issue] s_barrier lgkmcnt(0) [MFMAs] s_barrier.
// Hazards (phase p of a wave of group g sits between barriers 2p+g-1 .. 2p+g+1):
//  RAW: K-tile t is waited for (own counted vmcnt) in phase b of t-1, before that phase's first
//       barrier, and read in phase a of t or later, i.e. after a barrier every wave of both groups
//       passed after its wait;
//  WAR: K-tile t+2 overwrites the stage of t-2, whose last reads (phase b of t-2) retired before
//       barrier 4t-4 at the latest; the overwrite is issued after barrier 4t-1.
// The 256-row tile halves the L2->LDS bytes per flop of the 128-row DMA tiles, the staging rate
// that bounds them.
constexpr int pp_lds_halves(int bn) {
  return 4 * (256 + bn) * 32 > 128 * (bn + 8) ? 4 * (256 + bn) * 32 : 128 * (bn + 8);
}

// I8: the int8-MFMA mode's operands through the same half view (a 32-half K-tile = one 64-code
// v_mfma_i32_16x16x64_i8 slice, the fragment reads unchanged); the int32 sums live in the fp32
// accumulator registers (bit-cast) and are scaled by sa[m] * sw[n] before the epilogue, or go
// to the split-K slab as int32 bits (k_splitk_reduce's i8 path) - the k_gemm_dma<I8> arithmetic.
// W4: packed-int4 B stages (BDma4: code pieces + the group-scale row), dequantized per fragment
template <int BN, int WGM, int AMODE, bool SPLIT, bool I8 = false, bool W4 = false>
__global__ void __launch_bounds__(512, 2) k_gemm_pp(GemmArgs p) {
  constexpr int BM = 256, BK = 32, NT = 512;
  constexpr int WGN = 8 / WGM;                      // wave grid WGM x WGN (2x4 or 4x2)
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16, TH = TM / 2;  // TH m-frags per phase
  constexpr int ASZ = BM * BK, SSZ = W4 ? ASZ + BDma4<BN, NT, BK>::SZ : (BM + BN) * BK;
  static_assert(WN % 16 == 0 && TM % 2 == 0 && (WGM == 2 || WGM == 4), "wave tile");
  static_assert(!W4 || (!I8 && AMODE == AM_LINEAR), "int4 B: linear A operand");
  using AL = ADma<BM, NT, AMODE, BK>;
  using BL = std::conditional_t<W4, BDma4<BN, NT, BK>, BDma<BN, NT, BK>>;
  __shared__ __attribute__((aligned(16))) f16 smem[4 * SSZ > 128 * (BN + 8) ? 4 * SSZ : 128 * (BN + 8)];

  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int ntile = nbm * nbn;
  const int nwg = ntile * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int bm, bn, split;
  tile_of(p, wg, nbm, nbn, bm, bn, split);
  const int m0 = bm * BM, n0 = bn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / WGN, wc = wid - wr * WGN;
  const int grp = wid >> 2;  // ping-pong group = M half (waves w and w + 4 share a SIMD)
  const int wm0 = wr * WM, wn0 = wc * WN;
  const int fr = lane & 15, fq = lane >> 4;

  AL al;
  BL bl;
  al.init(p, m0, kbeg, wid);
  bl.init(p, n0, wid);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  // prologue: K-tiles 0 and 1 in flight, wait for 0
  if (nk > 0) {
    al.issue(p, kbeg, smem, wid);
    bl.issue(p, kbeg, smem + ASZ, wid);
  }
  if (nk > 1) {
    al.issue(p, kbeg + BK, smem + SSZ, wid);
    bl.issue(p, kbeg + BK, smem + SSZ + ASZ, wid);
    wait_vm_rt(AL::L + BL::count(wid));
  } else {
    wait_vm<0>();
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 runs one barrier behind
  asm volatile("" ::: "memory");

  f16x8 af[TH], bf[TN];
  unsigned m64 = 0, m54 = 0;
  if constexpr (W4) w4_magics(m64, m54);
  auto mfma_block = [&](int ih) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TH; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (I8)
          acc[ih * TH + i][j] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, bf[j]), __builtin_bit_cast(i32x4, af[i]),
                                                          __builtin_bit_cast(i32x4, acc[ih * TH + i][j]), 0, 0, 0));
        else
          acc[ih * TH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[ih * TH + i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto bar = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  for (int kt = 0; kt < nk; ++kt) {
    const f16* As = smem + (kt & 3) * SSZ;
    const f16* Bs = As + ASZ;
    const bool pre = kt + 2 < nk;
    f16* nxt = smem + ((kt + 2) & 3) * SSZ;
    // ---- phase a
#pragma unroll
    for (int i = 0; i < TH; ++i) af[i] = *reinterpret_cast<const f16x8*>(As + swz_t<BK>(wm0 + i * 16 + fr, fq));
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (W4) bf[j] = w4_frag<BK>(Bs, wn0 + j * 16 + fr, 0, fq, BDma4<BN, NT, BK>::CODE_H, m64, m54);
      else bf[j] = *reinterpret_cast<const f16x8*>(Bs + swz_t<BK>(wn0 + j * 16 + fr, fq));
    }
    if (pre) al.issue(p, kbeg + (kt + 2) * BK, nxt, wid);
    bar();
    mfma_block(0);
    bar();
    // ---- phase b
#pragma unroll
    for (int i = 0; i < TH; ++i)
      af[i] = *reinterpret_cast<const f16x8*>(As + swz_t<BK>(wm0 + (TH + i) * 16 + fr, fq));
    if (kt + 1 < nk) {
      if (pre) wait_vm_rt(AL::L);
      else wait_vm<0>();
    }
    if (pre) bl.issue(p, kbeg + (kt + 2) * BK, nxt + ASZ, wid);
    bar();
    mfma_block(1);
    bar();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
  const bool geglu = (p.epi & QD_EPI_GEGLU) != 0;
  const bool gtanh = (p.epi & QD_EPI_GELU_TANH) != 0;
  if constexpr (SPLIT) {
    float* part = p.part + (long)split * p.M * p.N;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn0 + j * 16 + fq * 4;
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm0 + i * 16 + fr;
        if (m < p.M) *reinterpret_cast<f32x4*>(part + (long)m * p.N + n) = acc[i][j];
      }
    }
    return;
  }
  // epilogue in two 128-row passes (one per wave group) through a [128][BN + 8] fp16 LDS tile:
  // h = half(acc + bias) -> per-column amax (rows_per_sample % WM == 0) -> (+GEGLU) (+residual)
  constexpr int LP = BN + 8;
  f16* ct = smem;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (grp == pass) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn0 + j * 16 + fq * 4;
        const int n = n0 + nl;
        const bool col_ok = n < p.N;
        f16x4 bq = {};
        if (has_bias && col_ok) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
        f32x4 sw = {};
        if (I8 && col_ok) sw = *reinterpret_cast<const f32x4*>(p.sw + n);
        float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ml = wm0 - pass * 128 + i * 16 + fr;  // row within this pass's 128
          const bool ok = m0 + pass * 128 + ml < p.M && col_ok;
          float sa = 0.f;
          if constexpr (I8) {  // int32 sum -> (q * sa[m]) * sw[n], as i8_scale
            const int m = min(m0 + pass * 128 + ml, p.M - 1);
            sa = p.sa[p.sa_rps ? m / p.sa_rps : m];
          }
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = I8 ? ((float)__builtin_bit_cast(i32x4, acc[i][j])[r] * sa) * sw[r] : acc[i][j][r];
            h[r] = (f16)(v + (float)bq[r]);
            if (ok) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
          }
          *reinterpret_cast<f16x4*>(ct + ml * LP + nl) = h;
        }
        if (do_amax && !geglu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) cm[r] = rowgroup_max(cm[r]);
          const int row0 = m0 + wm0;
          if (fr == 0 && col_ok && row0 < p.M) {
            float* a = p.amax + (long)(row0 / p.rows_per_sample) * p.N + n;
#pragma unroll
            for (int r = 0; r < 4; ++r) atomic_max_pos(a + r, cm[r]);
          }
        }
      }
    }
    __syncthreads();
    const int cpr = geglu ? BN / 16 : BN / 8;
    const int on0 = geglu ? n0 >> 1 : n0, oN = geglu ? p.N >> 1 : p.N;
    const int mb = m0 + pass * 128;
#pragma unroll 2
    for (int e = threadIdx.x; e < 128 * cpr; e += NT) {
      const int row = e / cpr, c = e - row * cpr;
      const int m = mb + row, n = on0 + c * 8;
      if (m < p.M && n < oN) {
        f16x8 v;
        if (geglu) {
          const int tc = (c >> 1) * 32 + (c & 1) * 8;
          const f16x8 hv = *reinterpret_cast<const f16x8*>(ct + row * LP + tc);
          const f16x8 gv = *reinterpret_cast<const f16x8*>(ct + row * LP + tc + 16);
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            const f32x2 gg = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
            v[r] = (f16)((float)hv[r] * (float)(f16)gg.x);
            v[r + 1] = (f16)((float)hv[r + 1] * (float)(f16)gg.y);
          }
        } else {
          v = *reinterpret_cast<const f16x8*>(ct + row * LP + c * 8);
          if (gtanh) {
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = (f16)gelu_tanh_f((float)v[r]);
          }
        }
        if (has_res) {
          const f16x8 rq = *reinterpret_cast<const f16x8*>(p.res + (long)m * p.ldy + n);
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[r]);
        }
        *reinterpret_cast<f16x8*>(p.y + (long)m * p.ldy + n) = v;
      }
    }
    if (pass == 0) __syncthreads();
  }
}

// ---- halo-reuse implicit-GEMM conv (3x3, stride 1, pad 1) ----------------------------------
// A block owns 256 output pixels = RB = 256 / W whole image rows of one image (W in {16, 32,
// 64}) x BN output channels.  K is walked chunk-major: for each 64-channel chunk of the input
// the (RB + 2) x (W + 2) halo of those rows is staged in LDS ONCE (LDS-DMA, zero halo from OOB
// offsets) and all 9 filter taps read their shifted A fragments from it; only the 9 weight
// tiles stream per chunk.  The implicit-GEMM kernels above re-load every A row for each tap
// (9x the activation bytes); for the SD1.5 64x64 convs this cuts the L2->LDS traffic per block
// ~2.8x - the load pipeline, not the MFMAs, bounds those kernels (ablation: DESIGN.md).
// Halo chunk c+1 is staged under chunk c's taps, 1/8 of its rows per tap step; weight tiles are
// double-buffered one tap ahead.  Summation order over K differs from the tap-major kernels
// (chunk-major), so its outputs may differ from theirs in the last fp16 bit.
#ifndef QD_HALO_ABL  // diagnostic builds only (scripts/halo_ablate.sh): 1 no MFMA, 2 no weight DMA in the
#define QD_HALO_ABL 0  // K loop, 4 no halo DMA in the K loop, 8 no barrier / wait (results are garbage);
#endif                 // int8 halo conv also: 16 no fragment reads in the K loop, 32 no epilogue
constexpr int HALO_ROWS_MAX = 400;  // (RB + 2) * (W + 2) <= 396 for W in {16, 32, 64}

template <int BN>
__global__ void __launch_bounds__(512, 2) k_conv_halo(GemmArgs p) {
  constexpr int BM = 256, NT = 512, NW = 8, WGN = 2;
  constexpr int WM = 64, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int HSZ = HALO_ROWS_MAX * BK;  // halves per halo buffer
  constexpr int BSZ = BN * BK;
  constexpr int LDSZ = 2 * HSZ + 2 * BSZ > epi_lds_halves(BM, BN) ? 2 * HSZ + 2 * BSZ : epi_lds_halves(BM, BN);
  constexpr int HG = HALO_ROWS_MAX / 8;                     // halo wave-instruction groups (max)
  constexpr int HL = (HG + NW - 1) / NW;                    // per wave
  static_assert(HL <= 8, "halo rows must stage within the 8 tap steps of a chunk");
  using BL = BDma<BN, NT, 64>;
  __shared__ __attribute__((aligned(16))) f16 smem[LDSZ];
  f16* const halo0 = smem;
  f16* const bring = smem + 2 * HSZ;

  const int W = p.W, RB = BM / W, W2 = W + 2;
  const int hrows = (RB + 2) * W2;
  const int nbm = p.M / BM, nbn = p.N / BN;
  const int ntile = nbm * nbn, nwg = ntile * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int bm, bn, split;
  tile_of(p, wg, nbm, nbn, bm, bn, split);
  const int m0 = bm * BM, n0 = bn * BN;
  const int img = m0 / (p.Ho * p.Wo), oh0 = (m0 - img * p.Ho * p.Wo) / W;
  const int c_beg = split * p.kps, c_end = c_beg + p.kps;  // 64-channel chunks of this split

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int fr = lane & 15, fq = lane >> 4;

  // halo staging: wave-instruction g covers halo rows 8g .. 8g+7 (lane -> row 8g + (lane >> 3),
  // LDS chunk lane & 7 holding K chunk (lane & 7) ^ (lane >> 3)); slot j of this wave is g = 8j + wid
  const __amdgpu_buffer_rsrc_t ars = rsrc(p.a, p.a_bytes);
  const int gc = ((lane & 7) ^ (lane >> 3)) * 8;
  unsigned hoff[HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    const int hr = (j * NW + wid) * 8 + (lane >> 3);
    const int hy = hr / W2, hx = hr - hy * W2;
    const int ih = oh0 - 1 + hy, iw = hx - 1;
    const bool ok = hr < hrows && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
    hoff[j] = ok ? (unsigned)(((img * p.Hs + sh) * p.Ws + sw) * p.Cip + gc) * 2u : OOB;
  }
  auto halo_issue = [&](int j, int chunk, f16* hb) {
    if (j * NW + wid < (hrows + 7) / 8) glds16(ars, hb + (j * NW + wid) * 8 * BK, hoff[j] + (unsigned)(chunk * BK * 2));
  };
  auto halo_cnt = [&](int j) { return (j < HL && j * NW + wid < (hrows + 7) / 8) ? 1 : 0; };

  BL bl;
  bl.init(p, n0, wid);
  const int bcnt = BL::count(wid);
  // weight tile of (tap t, chunk c): K offset t * Cip + c * 64 ([Co][kh][kw][Cip] layout)
  auto b_issue = [&](int s, f16* dst) {
    const int c = c_beg + s / 9, t = s - (s / 9) * 9;
    bl.issue(p, t * p.Cip + c * BK, dst, wid);
  };

  // per-lane halo row of each A fragment row (tap (0, 0)); tap (ky, kx) adds ky * W2 + kx
  int hr0[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wm0 + i * 16 + fr;
    const int r = ml / W, x = ml - r * W;
    hr0[i] = r * W2 + x;
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = (c_end - c_beg) * 9;
  // prologue: the first chunk's whole halo, then the first weight tile
#pragma unroll
  for (int j = 0; j < HL; ++j) halo_issue(j, c_beg, halo0);
  b_issue(0, bring);

  for (int s = 0; s < nsteps; ++s) {
    const int cl = s / 9, t = s - cl * 9;
    // own loads of weight tile s landed (halo rows issued after it in step s-1 may stay in flight)
    if (!(QD_HALO_ABL & 8)) {
      wait_vm_rt(t >= 1 && cl + 1 < c_end - c_beg ? halo_cnt(t - 1) : 0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (!(QD_HALO_ABL & 2))
      if (s + 1 < nsteps) b_issue(s + 1, bring + ((s + 1) & 1) * BSZ);
    if (!(QD_HALO_ABL & 4))
      if (t < 8 && cl + 1 < c_end - c_beg) halo_issue(t, c_beg + cl + 1, halo0 + ((cl + 1) & 1) * HSZ);
    const f16* hb = halo0 + (cl & 1) * HSZ;
    const f16* Bs = bring + (s & 1) * BSZ;
    const int ky = t / 3, kx = t - ky * 3;
    const int tap = ky * W2 + kx;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(hb + swz(hr0[i] + tap, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f16x8*>(Bs + swz(wn0 + j * 16 + fr, ks * 4 + fq));
      if (QD_HALO_ABL & 1) {
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bf[j]));
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (p.splits > 1) gemm_epilogue<BM, BN, NT, TM, TN, true, LDSZ, true>(p, acc, smem, m0, n0, wm0, wn0, split);
  else gemm_epilogue<BM, BN, NT, TM, TN, false, LDSZ, true>(p, acc, smem, m0, n0, wm0, wn0, split);
}

// ---- split-phase halo conv (variants 202 / 203) -------------------------------------------
// The halo conv's tile and K order with its LDS reads taken off the MFMAs' critical path.
// Ablation of the lock-step kernel (64x64 320->320, scripts/halo_ablate.py): 66.5 us; without
// MFMAs 42.3; without DMA and barriers (LDS reads + MFMAs only) still 56.1; reads alone 26.5 -
// the fragment reads and the MFMAs serialise (every wave reads its fragments right after the
// step's barrier and waits for them).  Here the barrier sits between the two 32-deep halves of a
// tap step and each half's fragments are read under the other half's MFMAs:
//   read(s, half 1) | MFMA(s, half 0) -> wait(tile s+1 [+ next chunk's halo]) -> barrier ->
//   issue tile s+2 (into the slot of s-1) + a halo row group -> read(s+1, half 0) | MFMA(s, half 1)
// which needs a 3-deep weight ring (halo double buffer 100 KB + 3 x 20 KB = the whole 160 KB).
// The 9 taps of a chunk are unrolled, so the ring slot (step % 3 == tap % 3) and the tap's
// halo offset are compile-time constants (immediate ds_read offsets, few address VALU ops).
// Hazards: tile s+1 is waited for (own vmcnt) before barrier s and read after it; tile s+2
// overwrites the slot of s-1, whose last reads fed MFMA(s-1, half 1) before barrier s; halo rows
// of chunk c+1 go into chunk c-1's buffer after barrier (c, tap 0), after the last reads of chunk
// c-1 (MFMA(c-1, tap 8, half 1)).  Same K order as the lock-step kernel: identical bits.
// BM 128 (variants 204 / 205, W <= 32): 4 waves (2 x 2) on 128-pixel tiles.  At 32x32 x 640 channels
// (CFG batch 8) the 256-pixel tiles make 32 x 5 = 160 tiles for 256 CUs; 128 x 160 tiles make 256.
template <int BM>
constexpr int halo2_rows() { return BM == 256 ? HALO_ROWS_MAX : 208; }  // (RB + 2) * (W + 2): 204 at W 32, 180 at W 16

template <int BN, int BM = 256>
__global__ void __launch_bounds__(2 * BM, 1) k_conv_halo2(GemmArgs p) {
  constexpr int NT = 2 * BM, NW = NT / 64, WGN = 2;
  constexpr int WM = 64, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  static_assert((NW / WGN) * WM == BM, "wave grid");
  constexpr int HSZ = halo2_rows<BM>() * BK;
  constexpr int BSZ = BN * BK;
  constexpr int LDSZ = 2 * HSZ + 3 * BSZ > epi_lds_halves(BM, BN) ? 2 * HSZ + 3 * BSZ : epi_lds_halves(BM, BN);
  static_assert(LDSZ * 2 <= 163840, "halo + weight ring exceed the 160 KB of LDS");
  constexpr int HG = halo2_rows<BM>() / 8;
  constexpr int HL = (HG + NW - 1) / NW;
  static_assert(HL <= 8, "halo rows must stage within the 8 tap steps of a chunk");
  using BL = BDma<BN, NT, 64>;
  __shared__ __attribute__((aligned(16))) f16 smem[LDSZ];
  f16* const halo0 = smem;
  f16* const bring = smem + 2 * HSZ;

  const int W = p.W, RB = BM / W, W2 = W + 2;
  const int hrows = (RB + 2) * W2;
  const int nbm = p.M / BM, nbn = p.N / BN;
  const int ntile = nbm * nbn, nwg = ntile * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int bm, bn, split;
  tile_of(p, wg, nbm, nbn, bm, bn, split);
  const int m0 = bm * BM, n0 = bn * BN;
  const int img = m0 / (p.Ho * p.Wo), oh0 = (m0 - img * p.Ho * p.Wo) / W;
  const int c_beg = split * p.kps, nch = p.kps;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int fr = lane & 15, fq = lane >> 4;

  const __amdgpu_buffer_rsrc_t ars = rsrc(p.a, p.a_bytes);
  const int gc = ((lane & 7) ^ (lane >> 3)) * 8;
  unsigned hoff[HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    const int hr = (j * NW + wid) * 8 + (lane >> 3);
    const int hy = hr / W2, hx = hr - hy * W2;
    const int ih = oh0 - 1 + hy, iw = hx - 1;
    const bool ok = hr < hrows && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
    hoff[j] = ok ? (unsigned)(((img * p.Hs + sh) * p.Ws + sw) * p.Cip + gc) * 2u : OOB;
  }
  const int hgroups = (hrows + 7) / 8;
  BL bl;
  bl.init(p, n0, wid);
  const int bcnt = BL::count(wid);
  // the tap offset in halo rows depends on the runtime image width: ky * W2 + kx
  int hr0[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wm0 + i * 16 + fr;
    const int r = ml / W, x = ml - r * W;
    hr0[i] = r * W2 + x;
  }
  // B fragment offsets (halves) within a ring slot, per half
  int bofs[2][TN];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < TN; ++j) bofs[ks][j] = swz(wn0 + j * 16 + fr, ks * 4 + fq);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nsteps = nch * 9;
  // prologue: chunk 0's halo, weight tiles 0 and 1; wait for the halo and tile 0
#pragma unroll
  for (int j = 0; j < HL; ++j)
    if (j * NW + wid < hgroups) glds16(ars, halo0 + (j * NW + wid) * 8 * BK, hoff[j] + (unsigned)(c_beg * BK * 2));
  bl.issue(p, c_beg * BK, bring, wid);
  if (nsteps > 1) bl.issue(p, p.Cip + c_beg * BK, bring + BSZ, wid);
  wait_vm_rt(nsteps > 1 ? bcnt : 0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  f16x8 a0[TM], b0[TN], a1[TM], b1[TN];
  // fragment reads in the order the next half's MFMAs (i-major) consume them: A0, B0..B4, A1..A3
  auto read_a1 = [&](const f16* hb, int tap, int ks, int i, f16x8& af) {
    int h = hr0[i];
    asm volatile("" : "+v"(h));  // keep the per-tap address math here (hoisted: 72 VGPRs, spills)
    af = *reinterpret_cast<const f16x8*>(hb + swz(h + tap, ks * 4 + fq));
  };
  auto read_frags = [&](const f16* hb, int tap, int slot, int ks, f16x8 (&af)[TM], f16x8 (&bf)[TN]) {
    read_a1(hb, tap, ks, 0, af[0]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f16x8*>(bring + slot * BSZ + bofs[ks][j]);
#pragma unroll
    for (int i = 1; i < TM; ++i) read_a1(hb, tap, ks, i, af[i]);
  };
  auto mfmas = [&](const f16x8 (&af)[TM], const f16x8 (&bf)[TN]) {
    if (QD_HALO_ABL & 1) {
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bf[j]));
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
  };
  // one fragment read per two MFMAs: the reads of the next half go out under this half's MFMAs
  // (left to itself the scheduler clusters them and waits for them right before their use)
  auto interleave = [&]() {
#pragma unroll
    for (int k = 0; k < TM + TN; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
    }
    __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - 2 * (TM + TN), 0);
  };
  read_frags(halo0, 0, 0, 0, a0, b0);
#pragma nounroll
  for (int cl = 0; cl < nch; ++cl) {
    const f16* hb = halo0 + (cl & 1) * HSZ;
    f16* const hnext = halo0 + ((cl + 1) & 1) * HSZ;
    const bool more = cl + 1 < nch;
    const int s0 = cl * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t % 3;
      read_frags(hb, ky * W2 + kx, t % 3, 1, a1, b1);
      mfmas(a0, b0);
      interleave();
      if (t < 8 || more) {
        // own loads of tile s+1 landed (issued in the middle of step s-1, followed only by
        // that step's halo row group); at a chunk's last tap also the next chunk's halo
        if (!(QD_HALO_ABL & 8)) {
          wait_vm_rt(t >= 1 && t < 8 && t - 1 < HL && more && (t - 1) * NW + wid < hgroups ? 1 : 0);
          asm volatile("" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        const int s2 = s0 + t + 2;  // weight tile s + 2: tap (t + 2) % 9 of chunk cl + (t + 2) / 9
        if (!(QD_HALO_ABL & 2) && s2 < nsteps) bl.issue(p, ((t + 2) % 9) * p.Cip + (c_beg + cl + (t + 2) / 9) * BK, bring + ((t + 2) % 3) * BSZ, wid);
        if (!(QD_HALO_ABL & 4) && t < HL && more && t * NW + wid < hgroups)
          glds16(ars, hnext + (t * NW + wid) * 8 * BK, hoff[t] + (unsigned)((c_beg + cl + 1) * BK * 2));
        if (t < 8) read_frags(hb, ((t + 1) / 3) * W2 + (t + 1) % 3, (t + 1) % 3, 0, a0, b0);
        else read_frags(hnext, 0, 0, 0, a0, b0);
      }
      mfmas(a1, b1);
      interleave();
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (p.splits > 1) gemm_epilogue<BM, BN, NT, TM, TN, true, LDSZ, true>(p, acc, smem, m0, n0, wm0, wn0, split);
  else gemm_epilogue<BM, BN, NT, TM, TN, false, LDSZ, true>(p, acc, smem, m0, n0, wm0, wn0, split);
}

// ---- int8 halo conv (int8-MFMA mode, qd_gemm_force 140 / 141) -------------------------------
// The halo conv's tile (256 output pixels = whole image rows x BN channels, 8 waves, wave tile
// 64 x BN/2) and K order (64-channel chunk major, the 9 taps inside a chunk) on int8 codes in the
// "half view" (two codes per fp16 slot, p.Cip = Ci_pad / 2).  A chunk is 64 codes = one 64-B LDS
// row per halo pixel / weight row, so one 16-B fragment read is the i32x4 operand of one
// v_mfma_i32_16x16x64_i8: half the LDS bytes per MFMA flop of the fp16 halo kernels, twice their
// MFMA rate.  What bounds a kernel of this shape is instruction issue (an MFMA holds its SIMD's
// issue for half of its 16 cycles; the rest must carry the reads, the DMA and the bookkeeping of
// both waves), so the K loop is built to issue almost nothing but MFMAs and fragment reads:
//  * W is a template parameter and the halo is stored with a row pitch of W2P = roundup(W + 2, 8)
//    pixels: the XOR swizzle of an A fragment row (row >> 1 & 3) then depends only on (lane, kx),
//    so every fragment read is one per-(kx) base VGPR + a compile-time immediate offset - no
//    address VALU in the loop (the B fragments likewise, the ring slot being tap % 3);
//  * every wave issues the same DMA instructions each step (the surplus halo / weight groups of
//    the uneven wave split load out-of-range offsets into a scratch LDS slot), so every vmcnt is a
//    compile-time constant, and the K offsets of a step ride in the scalar soffset;
//  * the MFMAs of step s start before its barrier: phase 1 (fragment rows 0..TM/2-1) -> wait(own
//    loads of tile s+1 [+ the next chunk's halo at a chunk's last tap]) -> barrier -> DMA tile s+2
//    into the slot of s-1 (read in step s-2, consumed by MFMA(s-1) before this barrier) + one halo
//    group of chunk c+1 into chunk c-1's buffer (last read in step (c-1, 7)) -> phase 2 (rows
//    TM/2..TM-1) with the fragment reads of step s+1 interleaved one per MFMA.
// Exact int32 sums: identical bits to every other int8 variant (k_gemm_dma<I8>, k_gemm_pp<I8>).
__device__ __forceinline__ void glds16s(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, (int)voff, soff, 0, 0);
}
typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) const f16x8 lds_f16x8_t;
// 32-bit LDS byte offset of a __shared__ object, and a 16-B read at one (constant parts of the
// offset fold into the ds_read_b128 immediate)
__device__ __forceinline__ int lds_addr(const void* p) { return (int)(uintptr_t)(lds_char_t*)p; }
__device__ __forceinline__ f16x8 lds_read16(int addr) { return *(lds_f16x8_t*)(uintptr_t)(unsigned)addr; }

// BM 256: 8 waves (4 x 2), one block per CU - the grid at the 64x64 level is a single wave of
// 256 tiles whose epilogues all run at the same time; BM 128 (round 4): 4 waves (2 x 2) and two
// blocks per CU (LDS <= 80 KB each), so one block's epilogue runs beside the other's K loop;
// BM 64 (round 4, W 8 only): 2 waves, one 8x8 image per tile - the 8x8 level, whose 512-row
// GEMMs otherwise run as split-K implicit GEMMs re-reading each input pixel 9 times
template <int BN, int W, int RING, int BM = 256>
__global__ void __launch_bounds__(2 * BM, BM == 256 ? 1 : 2) k_conv_halo_i8(GemmArgs p) {
  constexpr int NT = 2 * BM, NW = NT / 64, WGN = 2;
  constexpr int WM = 64, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int RB = BM / W;                  // image rows per tile
  constexpr int W2P = (W + 2 + 7) / 8 * 8;    // halo row pitch in pixels (multiple of 8)
  constexpr int RS = 64;                      // bytes per LDS row: one 64-code chunk
  constexpr int HROWS = (RB + 2) * W2P;
  constexpr int HG = (HROWS + 15) / 16;       // 16-row halo DMA groups
  constexpr int HL = (HG + NW - 1) / NW;      // halo DMA slots per wave (uniform)
  constexpr int G = BN / 16;                  // 16-row weight DMA groups
  constexpr int BL = (G + NW - 1) / NW;       // weight DMA slots per wave (uniform)
  constexpr int HB = HROWS * RS, BB = BN * RS, SCR = 1024;
  constexpr int LOOPB = 2 * HB + RING * BB + SCR;
  constexpr int EPIB = epi_lds_halves(BM, BN) * 2;
  constexpr int LDSB = LOOPB > EPIB ? LOOPB : EPIB;
  static_assert(LDSB * (BM == 256 ? 1 : 2) <= 163840, "halo + weight ring exceed the 160 KB of LDS");
  static_assert(BM == 256 || BM == 128 || BM == 64, "tile rows");
  // the next chunk's halo groups (taps 0 .. HL-1) must be older than the weight tile a chunk's
  // last tap waits for (issued at tap 10 - RING); the previous chunk's last taps issue none
  static_assert(RING >= 3 && HL >= 1 && HL <= 10 - RING, "halo staging vs weight ring depth");
  // W 8 (the 8x8 level): a 16-pixel fragment spans two image rows, so a lane's pixel is
  // (row fr / W, column fr % W); BM 64 (one image per tile: the halo is one image's rows)
  static_assert((W % 16 == 0 || (W == 8 && BM == 64)) && 64 % W == 0 && WN % 8 == 0, "tile geometry");
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  char* const halo = smem;
  char* const ring = smem + 2 * HB;
  char* const scratch = smem + 2 * HB + RING * BB;

  const int nbm = p.M / BM, nbn = p.N / BN;
  const int ntile = nbm * nbn, nwg = ntile * p.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int bm, bn, split;
  tile_of(p, wg, nbm, nbn, bm, bn, split);
  const int m0 = bm * BM, n0 = bn * BN;
  const int img = m0 / (p.Ho * W), oh0 = (m0 - img * p.Ho * W) / W;
  const int c_beg = split * p.kps, nch = p.kps;  // 64-code chunks of this split

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int fr = lane & 15, fq = lane >> 4;

  // DMA lane map (1 KB per wave-instruction = 16 rows of 64 B): lane -> row (lane >> 2) of the
  // group, LDS chunk lane & 3 holding K chunk (lane & 3) ^ ((row >> 1) & 3)
  const int gcl = (lane & 3) ^ ((lane >> 3) & 3);
  const __amdgpu_buffer_rsrc_t ars = rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t brs = rsrc(p.b, p.b_bytes);
  unsigned hoff[HL];
  char* hdst[HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    const int g = j * NW + wid;
    const int r = g * 16 + (lane >> 2);
    const int hy = r / W2P, hx = r - hy * W2P;
    const int ih = oh0 - 1 + hy, iw = hx - 1;
    const bool ok = g < HG && r < HROWS && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)W;
    const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
    hoff[j] = ok ? (unsigned)((((img * p.Hs + sh) * p.Ws + sw) * p.Cip + gcl * 8) * 2) : OOB;
    hdst[j] = g < HG ? halo + g * 16 * RS : scratch;  // + the buffer offset of the chunk
  }
  unsigned boff[BL];
  int bdst[BL];
#pragma unroll
  for (int j = 0; j < BL; ++j) {
    const int g = j * NW + wid;
    const int n = n0 + g * 16 + (lane >> 2);
    boff[j] = g < G ? (unsigned)(((long)n * p.K + gcl * 8) * 2) : OOB;
    bdst[j] = g < G ? g * 16 * RS : -1;
  }
  const int nsteps = nch * 9;
  // weight tile of step s = (chunk c, tap t) -> ring slot s % RING; K offset (bytes) in soffset;
  // the steps past the end re-load the last tile (into a slot nobody reads again)
  auto b_issue = [&](int s, int slot) {
    const int ss = s < nsteps ? s : nsteps - 1;
    const int c = c_beg + ss / 9, t = ss - (ss / 9) * 9;
    const int soff = (t * p.Cip + c * 32) * 2;
#pragma unroll
    for (int j = 0; j < BL; ++j) glds16s(brs, bdst[j] >= 0 ? ring + slot * BB + bdst[j] : scratch, boff[j], soff);
  };
  auto h_issue = [&](int j, int chunk, int buf) {
    glds16s(ars, hdst[j] == scratch ? scratch : hdst[j] + buf * HB, hoff[j], chunk * RS);
  };

  // fragment addresses: A of (tap ky,kx), fragment i = abase[buf][kx] + ((ky + 16i / W) * W2P + 16i % W) * RS
  int abase[2][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int px = (fr / W) * W2P + fr % W + kx;  // the lane's halo pixel (fr < W for W >= 16)
    const int lo = px * RS + ((fq ^ ((px >> 1) & 3)) << 4);
    abase[0][kx] = lds_addr(halo) + (wm0 / W) * W2P * RS + lo;
    abase[1][kx] = abase[0][kx] + HB;
  }
  const int bbase = lds_addr(ring) + (wn0 + fr) * RS + ((fq ^ ((fr >> 1) & 3)) << 4);

  i32x4 iacc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) iacc[i][j] = (i32x4){0, 0, 0, 0};

  // prologue: chunk 0's halo and weight tiles 0 .. RING-2; wait for the halo and tile 0
#pragma unroll
  for (int j = 0; j < HL; ++j) h_issue(j, c_beg, 0);
#pragma unroll
  for (int u = 0; u < RING - 1; ++u) b_issue(u, u);
  wait_vm<BL * (RING - 2)>();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  f16x8 a0[TM], b0[TN], a1[TM], b1[TN];
  // reads of step (tap t, ring slot `slot`, halo buffer hbuf) in the order phase 1 / 2 consume them
  auto read_frags = [&](int hbuf, int t, int slot, f16x8 (&af)[TM], f16x8 (&bf)[TN], int k) {
    if (QD_HALO_ABL & 16) return;  // diagnostic build: no fragment reads in the K loop
    // k-th read of the step: B0..B(TN-1) first (phase 1 uses all columns), then A0..A(TM-1)
    const int ky = t / 3, kx = t % 3;
    if (k < TN) bf[k] = lds_read16(bbase + slot * BB + k * 16 * RS);
    else {
      const int i = k - TN;
      af[i] = lds_read16(abase[hbuf][kx] + ((ky + 16 * i / W) * W2P + (16 * i) % W) * RS);
    }
  };
  auto mfma = [&](int i, int j, const f16x8 (&af)[TM], const f16x8 (&bf)[TN]) {
    if (QD_HALO_ABL & 1) {  // diagnostic build: operands kept live, no MFMA
      asm volatile("" ::"v"(af[i]), "v"(bf[j]));
      return;
    }
    iacc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, bf[j]),
                                                       __builtin_bit_cast(i32x4, af[i]), iacc[i][j], 0, 0, 0);
  };
  // halo instructions issued (after tile s+1) in steps s-RING+2 .. s-1: taps t-RING+2 .. t-1 < HL
  auto hwin = [](int t) {
    int n = 0;
    for (int k = 1; k <= RING - 2; ++k) n += (t - k >= 0 && t - k < HL) ? 1 : 0;
    return n;
  };
  // one step: fragments of step s in (ca, cb); reads of step s+1 into (na, nb).  The A fragments
  // of step s+1 come from the current chunk's halo (landed and published at the previous chunk's
  // last barrier) except at a chunk's last tap, so they are read in phase 1, before the barrier;
  // the B fragments (weight tile s+1) after it - the LDS reads spread over both phases.
  auto step = [&](int cl, int t, f16x8 (&ca)[TM], f16x8 (&cb)[TN], f16x8 (&na)[TM], f16x8 (&nb)[TN]) {
    const int s = cl * 9 + t;
    const bool next = t < 8 || cl + 1 < nch;
    const int nbuf = t < 8 ? (cl & 1) : ((cl + 1) & 1), nt = t < 8 ? t + 1 : 0;
    const int nslot = 9 % RING == 0 ? (t + 1) % RING : (s + 1) % RING;
    // phase 1: rows 0 .. TM/2-1, then the A reads of step s+1 within a chunk (their registers
    // overlap the fragments phase 1 has just consumed)
#pragma unroll
    for (int i = 0; i < TM / 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(i, j, ca, cb);
    if (t < 8) {
#pragma unroll
      for (int i = 0; i < TM; ++i) read_frags(nbuf, nt, nslot, na, nb, TN + i);
    }
    int k = 0;
    if (next) {
      // own loads of tile s+1 landed (issued in step s-RING+2); younger: the tiles s+2 .. s+RING-2
      // and the halo groups of the steps since (taps t-RING+2 .. t-1 of this chunk, if < HL)
      if (!(QD_HALO_ABL & 8)) {
        wait_vm_c(BL * (RING - 3) + hwin(t));
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      if (!(QD_HALO_ABL & 2))
        b_issue(s + RING - 1, RING % 9 == 0 || 9 % RING == 0 ? (t + RING - 1) % RING : (s + RING - 1) % RING);
      if (!(QD_HALO_ABL & 4) && t < HL) h_issue(t, c_beg + cl + 1, (cl + 1) & 1);
      // phase 2: rows TM/2 .. TM-1, the B reads of step s+1 (+ its A reads at a chunk's last tap)
      constexpr int NR2 = TN + TM;
      const int nr = t < 8 ? TN : NR2;
      k = 0;
#pragma unroll
      for (int i = TM / 2; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (k < nr) {
            read_frags(nbuf, nt, nslot, na, nb, k);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          }
          ++k;
          mfma(i, j, ca, cb);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        }
#pragma unroll
      for (; k < nr; ++k) read_frags(nbuf, nt, nslot, na, nb, k);
    } else {
#pragma unroll
      for (int i = TM / 2; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma(i, j, ca, cb);
    }
  };
#pragma unroll
  for (int k = 0; k < TM + TN; ++k) read_frags(0, 0, 0, a0, b0, k);
#pragma nounroll
  for (int cl = 0; cl < nch; ++cl) {
    step(cl, 0, a0, b0, a1, b1);
    step(cl, 1, a1, b1, a0, b0);
    step(cl, 2, a0, b0, a1, b1);
    step(cl, 3, a1, b1, a0, b0);
    step(cl, 4, a0, b0, a1, b1);
    step(cl, 5, a1, b1, a0, b0);
    step(cl, 6, a0, b0, a1, b1);
    step(cl, 7, a1, b1, a0, b0);
    step(cl, 8, a0, b0, a1, b1);
    // 9 steps per chunk: the next chunk's first fragments are in set 1
#pragma unroll
    for (int i = 0; i < TM; ++i) a0[i] = a1[i];
#pragma unroll
    for (int j = 0; j < TN; ++j) b0[j] = b1[j];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  f32x4 acc[TM][TN];
  f16* const esm = reinterpret_cast<f16*>(smem);
  if (QD_HALO_ABL & 32) {  // diagnostic build: no epilogue (one store keeps the sums live)
    int v = 0;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) v ^= iacc[i][j][0] ^ iacc[i][j][3];
    if (v == 0x7fffffff) p.y[threadIdx.x] = (f16)1.f;
    return;
  }
  if (p.splits > 1) {
    i8_scale<TM, TN, true>(p, iacc, acc, m0, n0, wm0, wn0);
    gemm_epilogue<BM, BN, NT, TM, TN, true, LDSB / 2, true, false>(p, acc, esm, m0, n0, wm0, wn0, split);
  } else {
    i8_scale<TM, TN, false>(p, iacc, acc, m0, n0, wm0, wn0);
    gemm_epilogue<BM, BN, NT, TM, TN, false, LDSB / 2, true, false>(p, acc, esm, m0, n0, wm0, wn0, split);
  }
}

template <int BN, int RING, int BM = 256>
static void launch_halo_i8(const GemmArgs& p, hipStream_t st) {
  const int nwg = (p.M / BM) * (p.N / BN) * p.splits;
  if constexpr (BM == 64) {
    k_conv_halo_i8<BN, 8, RING, 64><<<nwg, 128, 0, st>>>(p);
  } else {
    if (p.W == 64) k_conv_halo_i8<BN, 64, RING, BM><<<nwg, 2 * BM, 0, st>>>(p);
    else if (p.W == 32) k_conv_halo_i8<BN, 32, RING, BM><<<nwg, 2 * BM, 0, st>>>(p);
    else k_conv_halo_i8<BN, 16, RING, BM><<<nwg, 2 * BM, 0, st>>>(p);
  }
}

// halo kernel applicability: 3x3 / stride 1 / pad 1, 64-channel chunks, whole-row bm-pixel tiles
static bool halo_ok(const GemmArgs& p, int bn, int chunk = 64, int bm = 256) {
  const bool w_ok = bm == 64 ? (p.W == 8 && p.H == 8 && chunk == 32) : (p.W == 16 || p.W == 32 || p.W == 64);
  // the fp16 split-phase kernel's 128-pixel tiles stage at most halo2_rows<128>() halo rows
  if (chunk == 64 && bm == 128 && (bm / std::max(p.W, 1) + 2) * (p.W + 2) > halo2_rows<128>()) return false;
  return p.kh == 3 && p.kw == 3 && p.stride == 1 && p.pad == 1 && p.Cip % chunk == 0 && p.N % bn == 0 && w_ok &&
         p.Ho == p.H && p.Wo == p.W && p.H % (bm / p.W) == 0 && (p.rows_per_sample % 64 == 0);
}

// split-K reduction + epilogue: block = 4*RPT rows x 256 columns (64 column quads x 4 row
// groups of RPT rows; RPT small enough that the launch has >= ~512 blocks - the slab read is
// latency-bound, not bandwidth-bound, at the small M that splits K); slabs summed in split order
// (deterministic: every RPT gives identical results); the RPT rows of a thread are loaded
// together per split.  amax: one atomic per column per 4*RPT rows (rows_per_sample % 16 == 0),
// of h = half(sum + bias), or - QD_EPI_AMAX_POST - of the final half(h + residual) (the post-residual
// amax of an explicitly split plan: the GEMM's own epilogue then only writes the slabs).
template <int RPT>
__global__ void __launch_bounds__(256) k_splitk_reduce(GemmArgs p) {
  __shared__ float red[4][256];
  const int cq = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + cq * 4;
  const int mb = blockIdx.y * (4 * RPT);
  const bool col_ok = n < p.N;
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
  const bool gtanh = (p.epi & QD_EPI_GELU_TANH) != 0;
  const bool post = do_amax && has_res && (p.epi & QD_EPI_AMAX_POST);
  f16x4 bq = {};
  if (has_bias && col_ok) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
  float cm[4] = {0.f, 0.f, 0.f, 0.f};
  if (col_ok) {
    const long mn = (long)p.M * p.N;
    f32x4 s[RPT];
    long off[RPT];
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
      const int m = min(mb + rg * RPT + rr, p.M - 1);  // clamped: rows >= M are computed, not stored
      off[rr] = (long)m * p.N + n;
      s[rr] = *reinterpret_cast<const f32x4*>(p.part + off[rr]);
    }
    if (p.i8) {
      // int32 partial sums (exact, any split order), then the int8 path's scaling
      i32x4 si[RPT];
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) si[rr] = __builtin_bit_cast(i32x4, s[rr]);
      for (int k = 1; k < p.splits; ++k) {
        i32x4 t[RPT];
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) t[rr] = *reinterpret_cast<const i32x4*>(p.part + k * mn + off[rr]);
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) si[rr] += t[rr];
      }
      const f32x4 sw = *reinterpret_cast<const f32x4*>(p.sw + n);
#pragma unroll
      for (int rr = 0; rr < RPT; ++rr) {
        const int m = min(mb + rg * RPT + rr, p.M - 1);
        const float sa = p.sa[p.sa_rps ? m / p.sa_rps : m];
#pragma unroll
        for (int r = 0; r < 4; ++r) s[rr][r] = ((float)si[rr][r] * sa) * sw[r];
      }
    } else {
      for (int k = 1; k < p.splits; ++k) {
        f32x4 t[RPT];
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) t[rr] = *reinterpret_cast<const f32x4*>(p.part + k * mn + off[rr]);
#pragma unroll
        for (int rr = 0; rr < RPT; ++rr) s[rr] += t[rr];
      }
    }
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) {
      const int m = mb + rg * RPT + rr;
      if (m >= p.M) break;
      f16x4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = (f16)(s[rr][r] + (float)bq[r]);
        if (!post) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
      }
      if (gtanh) {
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)gelu_tanh_f((float)h[r]);
      }
      if (has_res) {
        const f16x4 rq = *reinterpret_cast<const f16x4*>(p.res + (long)m * p.ldy + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)rq[r]);
      }
      if (post) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
      }
      *reinterpret_cast<f16x4*>(p.y + (long)m * p.ldy + n) = h;
    }
  }
  if (!do_amax) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[rg][cq * 4 + r] = cm[r];
  __syncthreads();
  if (rg == 0 && col_ok && mb < p.M) {
    float* a = p.amax + (long)(mb / p.rows_per_sample) * p.N + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = fmaxf(fmaxf(red[0][cq * 4 + r], red[1][cq * 4 + r]), fmaxf(red[2][cq * 4 + r], red[3][cq * 4 + r]));
      atomic_max_pos(a + r, v);
    }
  }
}

// split-K reduction fused with the conv output fake-quant and the residual / per-sample add
// (qd_conv2d_fq; the low UNet levels, whose convs split K): block = one sample's rows (RPT * 32 =
// rows_per_sample <= 256) x 32 columns, thread = 4 columns x RPT rows (8 column quads x 32 row
// groups, rows rg + 32 rr).  h = half(sum of the slabs in split order + bias) exactly as
// k_splitk_reduce; the column maxima of h over the sample (the QD_EPI_AMAX value, also written to
// amax) are reduced in LDS with no atomics, then x = half(fq(h) + residual) or half(fq(h) + cadd)
// with k_finalize's arithmetic: bit-identical to k_splitk_reduce + qd_fq_finalize.
template <int RPT>
__global__ void __launch_bounds__(256) k_splitk_reduce_fq(GemmArgs p) {
  __shared__ float red[32][33];  // [row group][column]
  __shared__ float scs[32];
  __shared__ double scr[32];
  const int cq = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int nl = cq * 4, n = blockIdx.x * 32 + nl;  // N % 32 == 0 (host)
  const long mb = (long)blockIdx.y * p.rows_per_sample;
  const long mn = (long)p.M * p.N;
  f16x4 bq = {};
  if ((p.epi & QD_EPI_BIAS) && p.bias) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
  f32x4 s[RPT];
  long off[RPT];
#pragma unroll
  for (int rr = 0; rr < RPT; ++rr) {
    off[rr] = (mb + rg + rr * 32) * p.N + n;
    s[rr] = *reinterpret_cast<const f32x4*>(p.part + off[rr]);
  }
  for (int k = 1; k < p.splits; ++k) {
    f32x4 t[RPT];
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) t[rr] = *reinterpret_cast<const f32x4*>(p.part + k * mn + off[rr]);
#pragma unroll
    for (int rr = 0; rr < RPT; ++rr) s[rr] += t[rr];
  }
  f16x4 h[RPT];
  float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int rr = 0; rr < RPT; ++rr)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      h[rr][r] = (f16)(s[rr][r] + (float)bq[r]);
      cm[r] = fmaxf(cm[r], fabsf((float)h[rr][r]));
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[rg][nl + r] = cm[r];
  __syncthreads();
  if (threadIdx.x < 32) {
    float m = 0.f;
    for (int g = 0; g < 32; ++g) m = fmaxf(m, red[g][threadIdx.x]);
    const float sc = fq_scale(m, p.fq_qmax);
    scs[threadIdx.x] = sc;
    scr[threadIdx.x] = rcp_exact(sc);
    if (p.amax) p.amax[(long)blockIdx.y * p.N + blockIdx.x * 32 + threadIdx.x] = m;
  }
  __syncthreads();
  const bool has_res = p.res != nullptr;
  f16x4 ca = {};
  if (!has_res && p.fq_cadd) ca = *reinterpret_cast<const f16x4*>(p.fq_cadd + (long)blockIdx.y * p.fq_cadd_ld + n);
#pragma unroll
  for (int rr = 0; rr < RPT; ++rr) {
    const long m = mb + rg + rr * 32;
    f16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = fq_apply_r((float)h[rr][r], scs[nl + r], scr[nl + r]);
    if (has_res) {
      const f16x4 rq = *reinterpret_cast<const f16x4*>(p.res + m * p.ldy + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (f16)((float)o[r] + (float)rq[r]);
    } else if (p.fq_cadd) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (f16)((float)o[r] + (float)ca[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) cm[r] = fmaxf(rr ? cm[r] : 0.f, fabsf((float)o[r]));
    *reinterpret_cast<f16x4*>(p.y + m * p.ldy + n) = o;
  }
  if (p.fq_xamax) {  // (uniform) the consumer's amax of the final output, the same LDS reduction
#pragma unroll
    for (int r = 0; r < 4; ++r) red[rg][nl + r] = cm[r];
    __syncthreads();
    if (threadIdx.x < 32) {
      float m = 0.f;
      for (int g = 0; g < 32; ++g) m = fmaxf(m, red[g][threadIdx.x]);
      p.fq_xamax[(long)blockIdx.y * p.N + blockIdx.x * 32 + threadIdx.x] = m;
    }
  }
}

// whether k_splitk_reduce_fq takes this plan's output (whole samples of <= 256 rows per block)
static int fq_rpt(const GemmArgs& p) {
  if (p.fq_qmax <= 0 || p.i8 || p.N % 32 || p.ldy != p.N || p.rows_per_sample <= 0 || p.M % p.rows_per_sample) return 0;
  const int r = p.rows_per_sample % 32 ? 0 : p.rows_per_sample / 32;
  return r == 1 || r == 2 || r == 4 || r == 8 ? r : 0;
}

// split-K reduction + epilogue with the GroupNorm slot statistics (QD_EPI_GNSTATS) and the
// per-(sample, column) add (QD_EPI_CADD): block = one 64-row slot x 64 columns; thread (cq, rg)
// owns 4 columns x rows 4 rg .. 4 rg + 3 (16 column quads x 16 row groups).  Slabs summed in split
// order (int32 for the int8 path: exact); h = half(s + bias) [+ residual] [+ cadd]; the thread's
// 4-row moments (two passes over registers) are merged over the 16 row groups in fixed order
// (Chan: mean = sum of means / 16, M2 = sum M2 + 4 sum (mean_g - mean)^2).
__global__ void __launch_bounds__(256) k_splitk_reduce_gn(GemmArgs p) {
  __shared__ float4 red[16][64];  // [row group][column]
  const int cq = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int nl = cq * 4, n = blockIdx.x * 64 + nl;
  const int mb = blockIdx.y * 64;
  const bool col_ok = n < p.N;
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool cadd = (p.epi & QD_EPI_CADD) && p.cadd;
  float v[4][4];  // [row][col]
  if (col_ok) {
    const long mn = (long)p.M * p.N;
    f32x4 s[4];
    long off[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      off[rr] = (long)(mb + rg * 4 + rr) * p.N + n;  // M % 64 == 0 (host check)
      s[rr] = *reinterpret_cast<const f32x4*>(p.part + off[rr]);
    }
    if (p.i8) {
      i32x4 si[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) si[rr] = __builtin_bit_cast(i32x4, s[rr]);
      for (int k = 1; k < p.splits; ++k) {
        i32x4 t[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) t[rr] = *reinterpret_cast<const i32x4*>(p.part + k * mn + off[rr]);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) si[rr] += t[rr];
      }
      const f32x4 sw = *reinterpret_cast<const f32x4*>(p.sw + n);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int m = mb + rg * 4 + rr;
        const float sa = p.sa[p.sa_rps ? m / p.sa_rps : m];
#pragma unroll
        for (int r = 0; r < 4; ++r) s[rr][r] = ((float)si[rr][r] * sa) * sw[r];
      }
    } else {
      for (int k = 1; k < p.splits; ++k) {
        f32x4 t[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) t[rr] = *reinterpret_cast<const f32x4*>(p.part + k * mn + off[rr]);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) s[rr] += t[rr];
      }
    }
    f16x4 bq = {}, cv = {};
    if (has_bias) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
    if (cadd) cv = *reinterpret_cast<const f16x4*>(p.cadd + (long)(mb / p.rows_per_sample) * p.cadd_ld + n);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = mb + rg * 4 + rr;
      f16x4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = (f16)(s[rr][r] + (float)bq[r]);
      if (has_res) {
        const f16x4 rq = *reinterpret_cast<const f16x4*>(p.res + (long)m * p.ldy + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)rq[r]);
      }
      if (cadd) {
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)cv[r]);
      }
      *reinterpret_cast<f16x4*>(p.y + (long)m * p.ldy + n) = h;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[rr][r] = (float)h[r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // this thread's 4-row moments of column r
      const float mean = (((v[0][r] + v[1][r]) + v[2][r]) + v[3][r]) * 0.25f;
      const float d0 = v[0][r] - mean, d1 = v[1][r] - mean, d2 = v[2][r] - mean, d3 = v[3][r] - mean;
      red[rg][nl + r] = make_float4(mean, ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3,
                                    fminf(fminf(v[0][r], v[1][r]), fminf(v[2][r], v[3][r])),
                                    fmaxf(fmaxf(v[0][r], v[1][r]), fmaxf(v[2][r], v[3][r])));
    }
  }
  __syncthreads();
  if (threadIdx.x < 64 && blockIdx.x * 64 + (int)threadIdx.x < p.N) {
    const int c = threadIdx.x;
    float sm = 0.f, mn = INFINITY, mx = -INFINITY;
#pragma unroll
    for (int g = 0; g < 16; ++g) sm += red[g][c].x;
    const float mean = sm * (1.0f / 16.0f);
    float m2 = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 e = red[g][c];
      const float d = e.x - mean;
      m2 += e.y + 4.0f * (d * d);
      mn = fminf(mn, e.z);
      mx = fmaxf(mx, e.w);
    }
    reinterpret_cast<float4*>(p.gnp)[(long)blockIdx.y * p.N + blockIdx.x * 64 + c] = make_float4(mean, m2, mn, mx);
  }
}

// ---- int8 GEGLU projection + per-token int8 codes of its output (int8-MFMA mode) -------------
// diffusers FeedForward's GEGLU (ff.net.0: proj -> hidden * gelu(gate)) followed by ff.net.2's
// per-token input quantization as ONE launch on a row-complete tile: a block owns BM = 64 token
// rows and ALL N = 2H interleaved projection rows, so the row max of the GEGLU output - the
// per-token scale - is found in-block and the fp16 GEGLU output never reaches HBM (the two-launch
// path writes it and the row quantizer reads it back: 2 x 84 MB per 64x64-level call at CFG 8).
//   * A (the block's 64 x K codes, K = 64 KS) stays in registers: wave (wm, wn) of the 2 x 4 wave
//     grid holds rows 32 wm .. +31 as TM = 2 x KS fragments of v_mfma_i32_16x16x64_i8;
//   * the projection streams through a 3-slot LDS-DMA ring in chunks of 128 rows = 4 interleave
//     blocks [hidden 16 | gate 16] = 64 GEGLU outputs, as KS K-step slabs of 128 x 64 B (BDma,
//     BKT 32: the int8 "half view"); wave wn takes block wn: fragment j = 0 hidden, 1 gate, C^T
//     layout as k_gemm_dma's int8 tiles; the fp32 weight scales and the bias sit in LDS;
//   * per chunk: h, g = half(((float)acc sa[m]) sw[n] + bias) and half(h half(gelu(g))) -
//     gemm_epilogue's GEGLU arithmetic - kept as fp16 in registers (NCH x 8 values per lane);
//   * after the last chunk: the row max over each lane's values, its lane groups (shuffles) and
//     the 4 waves sharing the rows (LDS), s = fq_scale(max, 127), codes q_i8 - k_quant_rows_g's
//     arithmetic - staged through LDS into 16-B row stores.
// Bit-identical to linear_i8(..., geglu=True) followed by quant_rows_i8 (tests/test_gpu_int8.py).
__device__ __forceinline__ int8_t q_i8g(float x, float s, double rs) {  // (quant.hip q_i8)
  const f16 t = (f16)(float)((double)x * rs);
  return (int8_t)__builtin_rintf((float)t);
}

// WGM = 1: 4 waves (one per SIMD, the whole 512-register file: the packed GEGLU outputs of the 64
// rows, NCH x 16 VGPRs); WGM = 2: 8 waves, two per SIMD (32 rows each, NCH x 8 VGPRs of outputs).
// Wave (wm, wn) takes rows 64 / WGM * wm .. and interleave block wn of each chunk.
template <int KS, int NCH, int WGM>
__global__ void __launch_bounds__(256 * WGM, 1) k_geglu_i8q(GemmArgs p, int8_t* __restrict__ y8, int ldy8,
                                                           float* __restrict__ sa8) {
  constexpr int BM = 64, NT = 256 * WGM, CH = 128, TM = 4 / WGM, SLAB = CH * 32, CHUNK = KS * SLAB;
  constexpr int NOUT = NCH * 64;               // GEGLU outputs per row
  constexpr int CP = NOUT + 16;                // code-tile row pitch (bytes): 16 rows x 4 B conflict-free
  constexpr int RING = 3 * CHUNK;              // halves
  constexpr int ASZ = KS * BM * 32;            // the A tile: KS slabs of 64 rows x 64 B
  static_assert(BM * CP <= RING * 2, "code tile fits the ring");
  __shared__ __attribute__((aligned(16))) f16 smem[RING + ASZ + NCH * CH * 3 + 2 * 4 * BM];
  f16* const As = smem + RING;
  float* const swl = reinterpret_cast<float*>(smem + RING + ASZ);             // [N] fp32 weight scales
  f16* const bl16 = smem + RING + ASZ + NCH * CH * 2;                          // [N] bias
  float* const rmx = reinterpret_cast<float*>(smem + RING + ASZ + NCH * CH * 3);  // [4][BM] row maxima
  const int m0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3, r0 = wm * 16 * TM;

  for (int n = threadIdx.x; n < NCH * CH; n += NT) {
    swl[n] = p.sw[n];
    bl16[n] = p.bias ? p.bias[n] : (f16)0.f;
  }
  // the block's A tile into LDS (64-B slab rows, the ring's swizzle)
  const __amdgpu_buffer_rsrc_t ars = rsrc(p.a, p.a_bytes);
  for (int e = threadIdx.x; e < BM * KS * 4; e += NT) {
    const int row = e / (KS * 4), rem = e - row * (KS * 4), ks = rem >> 2, ch = rem & 3;
    const int m = m0 + row;
    const f16x8 v = bload(ars, m < p.M ? (unsigned)m * (unsigned)p.lda * 2u + (unsigned)(ks * 64 + ch * 16) : OOB);
    *reinterpret_cast<f16x8*>(As + ks * BM * 32 + swz_t<32>(row, ch)) = v;
  }
  float sam[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) sam[i] = p.sa[min(m0 + r0 + i * 16 + fr, p.M - 1)];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  BDma<CH, NT, 32> bl;
  auto issue_chunk = [&](int c, f16* dst) {
    bl.init(p, c * CH, wid);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) bl.issue(p, ks * 32, dst + ks * SLAB, wid);
  };
  constexpr int PER = BDma<CH, NT, 32>::L;  // DMA instructions per wave and K slab
  issue_chunk(0, smem);
  issue_chunk(1, smem + CHUNK);

  unsigned vlo[NCH][TM], vhi[NCH][TM];  // packed fp16 GEGLU outputs: columns 4fq + {0, 1} | {2, 3}
  f16x2v m2[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) m2[i] = (f16x2v){(f16)0.f, (f16)0.f};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) wait_vm<KS * PER>();
    else wait_vm<0>();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 2 < NCH) issue_chunk(c + 2, smem + ((c + 2) % 3) * CHUNK);
    const f16* Bs = smem + (c % 3) * CHUNK;
    i32x4 iacc[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) iacc[i][j] = (i32x4){0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      f16x8 bf[2], af[TM];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = *reinterpret_cast<const f16x8*>(Bs + ks * SLAB + swz_t<32>(wn * 32 + j * 16 + fr, fq));
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8*>(As + ks * BM * 32 + swz_t<32>(r0 + i * 16 + fr, fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          iacc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, bf[j]),
                                                             __builtin_bit_cast(i32x4, af[i]), iacc[i][j], 0, 0, 0);
    }
    const int nl = c * CH + wn * 32 + fq * 4;
    const f32x4 sw0 = *reinterpret_cast<const f32x4*>(swl + nl), sw1 = *reinterpret_cast<const f32x4*>(swl + nl + 16);
    const f16x4 b0 = *reinterpret_cast<const f16x4*>(bl16 + nl), b1 = *reinterpret_cast<const f16x4*>(bl16 + nl + 16);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      f16x4 hv, gv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hv[r] = (f16)((((float)iacc[i][0][r] * sam[i]) * sw0[r]) + (float)b0[r]);
        gv[r] = (f16)((((float)iacc[i][1][r] * sam[i]) * sw1[r]) + (float)b1[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const f32x2 g2 = gelu2_f((f32x2){(float)gv[r], (float)gv[r + 1]});
        const f16x2v o = {(f16)((float)hv[r] * (float)(f16)g2.x), (f16)((float)hv[r + 1] * (float)(f16)g2.y)};
        if (r == 0) vlo[c][i] = __builtin_bit_cast(unsigned, o);
        else vhi[c][i] = __builtin_bit_cast(unsigned, o);
        m2[i] = __builtin_elementwise_max(m2[i], __builtin_elementwise_abs(o));
      }
      // pin the chunk's outputs here: left alone the compiler sinks this pure VALU math past the
      // later chunks' barriers and keeps every chunk's accumulators alive (hundreds of registers)
      asm volatile("" : "+v"(vlo[c][i]), "+v"(vhi[c][i]));
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float m = fmaxf((float)m2[i][0], (float)m2[i][1]);
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    if (fq == 0) rmx[wn * BM + r0 + i * 16 + fr] = m;
  }
  __syncthreads();  // (also: every wave's last ring reads are done - the code tile reuses the ring)
  char* const ct = reinterpret_cast<char*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rl = r0 + i * 16 + fr;
    const float m = fmaxf(fmaxf(rmx[rl], rmx[BM + rl]), fmaxf(rmx[2 * BM + rl], rmx[3 * BM + rl]));
    const float s = fq_scale(m, 127);
    const double rs = rcp_exact(s);
    if (wn == 0 && fq == 0 && m0 + rl < p.M) sa8[m0 + rl] = s;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      unsigned w = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f16x2v pr = __builtin_bit_cast(f16x2v, r < 2 ? vlo[c][i] : vhi[c][i]);
        w |= (unsigned)(uint8_t)q_i8g((float)pr[r & 1], s, rs) << (8 * r);
      }
      *reinterpret_cast<unsigned*>(ct + rl * CP + c * 64 + wn * 16 + fq * 4) = w;
    }
  }
  __syncthreads();
  constexpr int C16 = NOUT / 16;
  for (int e = threadIdx.x; e < BM * C16; e += NT) {
    const int row = e / C16, cc = e - row * C16;
    if (m0 + row < p.M)
      *reinterpret_cast<uint4*>(y8 + (long)(m0 + row) * ldy8 + cc * 16) = *reinterpret_cast<const uint4*>(ct + row * CP + cc * 16);
  }
}

// ---- tile / split selection (host) ----------------------------------------------------------
// kind 0: register-staged k_gemm (any weight format); kind 1: LDS-DMA k_gemm_dma (F16 weights)
struct Plan {
  int kind, bm, bn, var, splits, kps;
  int pdiv = 0;  // persistent int8 DMA linears: tiles per block (grid = tiles / pdiv)
};

// LDS-DMA variants: tile, wave grid, LDS stages
struct DmaVar {
  int bm, bn, wgm, wgn, st, pipe;
  double eff;
  int bkt = 64;
};
static constexpr DmaVar kDmaC[] = {
    {128, 160, 2, 2, 2, 0, 1.00},  // 0: 2 blocks / CU
    {128, 320, 2, 4, 2, 0, 1.00},  // 1
    {256, 128, 4, 2, 3, 0, 1.00},  // 2
    {256, 256, 2, 4, 2, 0, 1.00},  // 3
    {128, 128, 2, 2, 2, 0, 0.95},  // 4: 2 blocks / CU
    {128, 64, 2, 2, 3, 0, 0.80},   // 5
    {256, 160, 4, 2, 3, 1, 1.00},  // 6: split-phase
    {256, 128, 4, 2, 3, 1, 1.00},  // 7: split-phase
    {128, 160, 2, 2, 3, 1, 1.00},  // 8: split-phase, 1 block / CU
    {256, 160, 4, 2, 3, 0, 1.00},  // 9
    {128, 160, 2, 2, 4, 0, 1.00, 32},  // 10: BK 32, 4 stages (3 in flight), 2 blocks / CU
    {128, 128, 2, 2, 4, 0, 1.00, 32},  // 11: BK 32, 4 stages, 2 blocks / CU
    {128, 320, 2, 4, 4, 0, 1.00, 32},  // 12: BK 32, 4 stages, 1 block / CU
    {256, 256, 2, 4, 4, 0, 1.00, 32},  // 13: BK 32, 4 stages, 1 block / CU
    {128, 64, 2, 2, 4, 0, 1.00, 32},   // 14: BK 32, 4 stages, small-M / short-K shapes
    {64, 64, 2, 2, 4, 0, 1.00, 32},    // 15: BK 32, 4 stages, small-M / short-K shapes
    // short-K, large-N tiles with 2 blocks / CU (4 waves, 64 x 128 / 128 x 64 wave tiles): one block's
    // epilogue (GELU VALU, output stores) can run beside the other block's MFMAs
    {128, 256, 2, 2, 3, 0, 1.00, 32},  // 16
    {256, 128, 2, 2, 3, 0, 1.00, 32},  // 17
    // row-complete LayerNorm epilogue (QD_EPI_LN, N = 320): 64-row tiles, 4 waves, 72 KB - two blocks
    // per CU, so one block's epilogue (residual, y, LayerNorm) runs beside the other's K loop
    {64, 320, 1, 4, 3, 0, 1.00, 32},   // 18
};
static int g_epi_lds = 0;  // measurement knob (qd_gemm_epi_lds): 1 = every epilogue through the LDS C tile
extern "C" int qd_gemm_epi_lds(int on) {
  g_epi_lds = on ? 1 : 0;
  return 0;
}
static int g_force = -1;  // tuning knob (qd_gemm_force): -1 auto, 0..3 register tiles, 100 + i DMA variant i
static int g_split = 0;   // with a forced DMA / ping-pong / halo variant: exact split-K count (0 = the fit rule)

// split s (1 = unsplit) of a forced variant's plan when it is valid for the shape (else the rule's)
static bool forced_split(int nsteps, int s_min_steps, int& sp) {
  if (g_split <= 0) return false;
  if (g_split == 1) {
    sp = 1;
    return true;
  }
  if (nsteps % g_split != 0 || nsteps / g_split < s_min_steps) return false;
  sp = g_split;
  return true;
}

extern "C" int qd_gemm_force(int variant) {
  const int v = variant >= 1000 ? variant % 1000 : variant, sp = variant >= 1000 ? variant / 1000 : 0;
  QD_REQUIRE(v == -1 || (v >= 0 && v < 4) ||
                 (v >= 100 && v < 100 + (int)(sizeof(kDmaC) / sizeof(kDmaC[0]))) || (v >= 200 && v <= 205) || (v >= 300 && v <= 304) || (v >= 120 && v <= 123) ||
                 (v >= 130 && v <= 134) || (v >= 140 && v <= 151) || (v >= 160 && v <= 167) || (v >= 170 && v <= 177) ||
                 (v >= 190 && v <= 192),
             "qd_gemm_force: -1, 0..3, 100 + DMA variant (int8: 110..117, fp8: 120..123), 200-205 halo conv, "
             "300-304 ping-pong (int8: 130-134, int8 halo conv 140-149, fused GEGLU codes 150 / 151, persistent "
             "int8 DMA linears 160-167 / 170-177: variants 10-17 with 2 / 4 tiles per block, A-stationary int8 "
             "linears 190-192); + 1000 * s: "
             "split-K count s (1 = unsplit)");
  QD_REQUIRE(sp <= 32, "qd_gemm_force: split count above 32");
  g_force = v;
  g_split = sp;
  return 0;
}

// Cost model (seconds): a CU runs ~4 TFLOP/s of this kernel with 2 resident blocks, ~3 with
// one; tile efficiency eff; a launch takes ceil(blocks / 512) rounds of 2 blocks per CU.
// Splits add the fp32 slab round trip (~5 TB/s) and one reduction launch.
// w4: packed-int4 weights with transposed scales - the ping-pong and BK-32 LDS-DMA variants run
// them through BDma4 (quant_w alone admits only the register-staged tiles)
static Plan plan_gemm(int M, int N, int K, bool quant_w, int rows_per_sample, bool amax, bool geglu = false,
                      bool post = false, int w4g = 0) {
  const bool w4 = w4g > 0;  // int4 group size when the codes can take the DMA / ping-pong families
  struct T {
    int bm, bn;
    double eff;
  } tiles[] = {{128, 160, 1.00}, {128, 128, 0.97}, {128, 64, 0.80}, {64, 64, 0.60}};
  Plan best{0, 64, 64, 0, 1, K};
  double best_t = 1e300;
  for (int ti = 0; ti < 4; ++ti) {
    const T& t = tiles[ti];
    if (g_force >= 0 && g_force != ti) continue;
    if (t.bn == 160 && N % 160 != 0) continue;  // 160-wide tiles only where they fit N exactly
    if (amax && rows_per_sample % (t.bm / 2) != 0) continue;
    if (quant_w && t.bn == 160) continue;        // int staging maps are built for BN % 64 == 0
    const long tiles_mn = (long)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn);
    for (int s = 1; s <= 32; ++s) {
      // split K into s equal runs of whole 64-deep steps, each >= 8 steps
      if (s > 1 && (K % 64 != 0 || (K / 64) % s != 0 || K / s < 512 || geglu || post)) continue;
      const long blocks = tiles_mn * s;
      const double blk = 2.0 * t.bm * t.bn * ((double)K / s) / t.eff;  // flop of one block
      double tm = blocks <= 256 ? blk / 3e12 : (double)((blocks + 511) / 512) * 2.0 * blk / 4e12;
      if (s > 1) tm += 8.0 * M * N * s / 5e12 + 3e-6;
      if (tm < best_t * 0.98) {
        best_t = tm;
        best = {0, t.bm, t.bn, 0, s, K / s};
      }
    }
  }
  if (g_force >= 200 && g_force <= 205 && !quant_w && !geglu && K % 576 == 0) {
    // halo conv (applicability is checked at launch; the split only needs the chunk count):
    // 200 / 201 BN 160 / 128 lock-step, 202 / 203 the same tiles split-phase, 204 / 205 split-phase
    // on 128-pixel tiles (4 waves)
    const int bn = (g_force & 1) ? 128 : 160, bm = g_force >= 204 ? 128 : 256;
    if (N % bn == 0 && M % bm == 0) {
      const long tiles_mn = (long)(M / bm) * (N / bn);
      const int nc = K / 576;
      best = {2, bm, bn, g_force >= 202 ? 1 : 0, 1, nc};
      int fsp;
      if (forced_split(nc, 1, fsp)) {
        best.splits = fsp;
        best.kps = nc / fsp;
      } else {
        for (int sp = 2; sp <= nc; ++sp) {
          if (nc % sp != 0) continue;
          if (tiles_mn * sp > 256) break;
          best.splits = sp;
          best.kps = nc / sp;
        }
      }
    }
  } else if (g_force >= 300 && g_force <= 304 && (!quant_w || w4) && !post) {  // (own epilogue: no post-residual amax)
    // ping-pong 256 x {256, 320, 192} tiles (2x4 waves, wave rows 128) and 256 x {160, 128}
    // (4x2 waves, wave rows 64); amax needs whole-sample wave tiles
    static const int kBn[] = {256, 320, 192, 160, 128};
    const int bnp = kBn[g_force - 300];
    if (!amax || rows_per_sample % (bnp >= 192 ? 128 : 64) == 0) {
      best = {3, 256, bnp, 0, 1, K};
      const long tiles_mn = (long)((M + 255) / 256) * ((N + bnp - 1) / bnp);
      int fsp;
      if (!geglu && K % 32 == 0 && forced_split(K / 32, 8, fsp)) {
        best.splits = fsp;
        best.kps = K / fsp;
      } else {
        for (int sp = 2; sp <= 32 && !geglu && K % 32 == 0; ++sp) {
          if ((K / 32) % sp != 0 || K / sp < 512) continue;
          if (tiles_mn * sp > 256L) break;
          best.splits = sp;
          best.kps = K / sp;
        }
      }
    }
  } else if (g_force >= 100 && g_force < 118 &&  // (118: the LayerNorm epilogue's tile, ln_var only)
             (!quant_w || (w4 && w4g % kDmaC[g_force - 100].bkt == 0 && kDmaC[g_force - 100].pipe == 0))) {
    const DmaVar& d = kDmaC[g_force - 100];
    // an explicit split reduces the amax in its reduction kernel: only an unsplit tile needs every
    // wave's rows in one sample
    int fs0 = 0;
    const bool fsplit = !geglu && K % 64 == 0 && forced_split(K / 64, 4, fs0) && fs0 > 1;
    const bool ok = (fsplit || !amax || rows_per_sample % (d.bm / d.wgm) == 0) && (!geglu || d.bn % 32 == 0);
    if (ok) {
      best = {1, d.bm, d.bn, g_force - 100, 1, K};
      // split K (whole 64-deep steps, >= 8 per split) while the blocks fit one resident round
      const long tiles_mn = (long)((M + d.bm - 1) / d.bm) * ((N + d.bn - 1) / d.bn);
      const int by_lds = 163840 / (2 * dma_lds_halves(d.bm, d.bn, d.st, d.bkt)), by_waves = 2048 / (64 * d.wgm * d.wgn);
      const int per_cu = std::max(1, std::min(by_lds, by_waves));
      int fsp;
      if (!geglu && K % 64 == 0 && forced_split(K / 64, 4, fsp)) {
        best.splits = fsp;
        best.kps = K / fsp;
      } else {
        for (int sp = 2; sp <= 32 && !geglu && !post && K % 64 == 0; ++sp) {
          if ((K / 64) % sp != 0 || K / sp < 512) continue;
          if (tiles_mn * sp > 256L * per_cu) break;
          best.splits = sp;
          best.kps = K / sp;
        }
      }
    }
  }
  return best;
}

template <int BM, int BN, int AMODE, bool SPLIT>
static void launch_fmt(const GemmArgs& p, int fmt, hipStream_t st) {
  const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * p.splits;
  if (fmt == QD_WFMT_F16) k_gemm<BM, BN, AMODE, QD_WFMT_F16, SPLIT><<<nwg, 256, 0, st>>>(p);
  else if constexpr (BN != 160 && AMODE == AM_LINEAR) {
    if (fmt == QD_WFMT_I8) k_gemm<BM, BN, AMODE, QD_WFMT_I8, SPLIT><<<nwg, 256, 0, st>>>(p);
    else k_gemm<BM, BN, AMODE, QD_WFMT_I4, SPLIT><<<nwg, 256, 0, st>>>(p);
  }
}

// the post-residual amax epilogue (QD_EPI_AMAX_POST with its amax and residual): the 128 x 160 linear
// tiles (fp16 variant 0, int8 variant 10) run it in the direct-store path of their own instantiation
// (DPOSTK), so the other epilogues' register allocation does not carry the packed column maxima
static bool epi_post_direct(const GemmArgs& p) {
  return (p.epi & QD_EPI_AMAX_POST) && (p.epi & QD_EPI_AMAX) && p.amax && (p.epi & QD_EPI_RESIDUAL) && p.res &&
         !(p.epi & (QD_EPI_GEGLU | QD_EPI_GELU_TANH | QD_EPI_GNSTATS | QD_EPI_LN | QD_EPI_CADD)) && !p.epi_lds &&
         p.pgrid <= 0;
}

template <int V, int AMODE, bool SPLIT>
static void launch_dma_v(const GemmArgs& p, hipStream_t st) {
  constexpr DmaVar d = kDmaC[V];
  const int nwg = ((p.M + d.bm - 1) / d.bm) * ((p.N + d.bn - 1) / d.bn) * p.splits;
  if constexpr (AMODE == AM_LINEAR && !SPLIT && V == 0) {
    if (epi_post_direct(p)) {
      k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AMODE, false, false, false, false, false, true>
          <<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
      return;
    }
  }
  k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AMODE, SPLIT><<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
}

template <int V, bool SPLIT>
static void launch_dma_w4_v(const GemmArgs& p, hipStream_t st) {
  constexpr DmaVar d = kDmaC[V];
  const int nwg = ((p.M + d.bm - 1) / d.bm) * ((p.N + d.bn - 1) / d.bn) * p.splits;
  k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AM_LINEAR, SPLIT, false, false, true>
      <<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
}

template <int AMODE, bool SPLIT>
static void launch_dma(const GemmArgs& p, int var, hipStream_t st, int fmt = QD_WFMT_F16) {
  if constexpr (AMODE == AM_LINEAR) {
    if (fmt == QD_WFMT_I4) {
      switch (var) {
        case 0: launch_dma_w4_v<0, SPLIT>(p, st); break;
        case 1: launch_dma_w4_v<1, SPLIT>(p, st); break;
        case 2: launch_dma_w4_v<2, SPLIT>(p, st); break;
        case 3: launch_dma_w4_v<3, SPLIT>(p, st); break;
        case 4: launch_dma_w4_v<4, SPLIT>(p, st); break;
        case 5: launch_dma_w4_v<5, SPLIT>(p, st); break;
        case 9: launch_dma_w4_v<9, SPLIT>(p, st); break;
        case 10: launch_dma_w4_v<10, SPLIT>(p, st); break;
        case 11: launch_dma_w4_v<11, SPLIT>(p, st); break;
        case 12: launch_dma_w4_v<12, SPLIT>(p, st); break;
        case 13: launch_dma_w4_v<13, SPLIT>(p, st); break;
        case 14: launch_dma_w4_v<14, SPLIT>(p, st); break;
        case 16: launch_dma_w4_v<16, SPLIT>(p, st); break;
        case 17: launch_dma_w4_v<17, SPLIT>(p, st); break;
        default: launch_dma_w4_v<15, SPLIT>(p, st); break;
      }
      return;
    }
  }
  switch (var) {
    case 0: launch_dma_v<0, AMODE, SPLIT>(p, st); break;
    case 1: launch_dma_v<1, AMODE, SPLIT>(p, st); break;
    case 2: launch_dma_v<2, AMODE, SPLIT>(p, st); break;
    case 3: launch_dma_v<3, AMODE, SPLIT>(p, st); break;
    case 4: launch_dma_v<4, AMODE, SPLIT>(p, st); break;
    case 5: launch_dma_v<5, AMODE, SPLIT>(p, st); break;
    case 6: launch_dma_v<6, AMODE, SPLIT>(p, st); break;
    case 7: launch_dma_v<7, AMODE, SPLIT>(p, st); break;
    case 8: launch_dma_v<8, AMODE, SPLIT>(p, st); break;
    case 9: launch_dma_v<9, AMODE, SPLIT>(p, st); break;
    case 10: launch_dma_v<10, AMODE, SPLIT>(p, st); break;
    case 11: launch_dma_v<11, AMODE, SPLIT>(p, st); break;
    case 12: launch_dma_v<12, AMODE, SPLIT>(p, st); break;
    case 13: launch_dma_v<13, AMODE, SPLIT>(p, st); break;
    case 14: launch_dma_v<14, AMODE, SPLIT>(p, st); break;
    case 16: launch_dma_v<16, AMODE, SPLIT>(p, st); break;
    case 17: launch_dma_v<17, AMODE, SPLIT>(p, st); break;
    case 18:
      if constexpr (AMODE == AM_LINEAR && !SPLIT) launch_dma_v<18, AMODE, SPLIT>(p, st);
      break;
    default: launch_dma_v<15, AMODE, SPLIT>(p, st); break;
  }
}

template <int AMODE, bool SPLIT>
static void launch_tile(const GemmArgs& p, const Plan& pl, int fmt, hipStream_t st) {
  if (pl.kind == 3) {
    const int nwg = ((p.M + 255) / 256) * ((p.N + pl.bn - 1) / pl.bn) * p.splits;
    if constexpr (AMODE == AM_LINEAR) {
      if (fmt == QD_WFMT_I4) {
        if (pl.bn == 256) k_gemm_pp<256, 2, AMODE, SPLIT, false, true><<<nwg, 512, 0, st>>>(p);
        else if (pl.bn == 320) k_gemm_pp<320, 2, AMODE, SPLIT, false, true><<<nwg, 512, 0, st>>>(p);
        else if (pl.bn == 192) k_gemm_pp<192, 2, AMODE, SPLIT, false, true><<<nwg, 512, 0, st>>>(p);
        else if (pl.bn == 160) k_gemm_pp<160, 4, AMODE, SPLIT, false, true><<<nwg, 512, 0, st>>>(p);
        else k_gemm_pp<128, 4, AMODE, SPLIT, false, true><<<nwg, 512, 0, st>>>(p);
        return;
      }
    }
    if (pl.bn == 256) k_gemm_pp<256, 2, AMODE, SPLIT><<<nwg, 512, 0, st>>>(p);
    else if (pl.bn == 320) k_gemm_pp<320, 2, AMODE, SPLIT><<<nwg, 512, 0, st>>>(p);
    else if (pl.bn == 192) k_gemm_pp<192, 2, AMODE, SPLIT><<<nwg, 512, 0, st>>>(p);
    else if (pl.bn == 160) k_gemm_pp<160, 4, AMODE, SPLIT><<<nwg, 512, 0, st>>>(p);
    else k_gemm_pp<128, 4, AMODE, SPLIT><<<nwg, 512, 0, st>>>(p);
  } else if (pl.kind == 2) {
    const int nwg = (p.M / pl.bm) * (p.N / pl.bn) * p.splits;
    if (pl.var == 1 && pl.bm == 128) {
      if (pl.bn == 160) k_conv_halo2<160, 128><<<nwg, 256, 0, st>>>(p);
      else k_conv_halo2<128, 128><<<nwg, 256, 0, st>>>(p);
    } else if (pl.var == 1) {
      if (pl.bn == 160) k_conv_halo2<160><<<nwg, 512, 0, st>>>(p);
      else k_conv_halo2<128><<<nwg, 512, 0, st>>>(p);
    } else {
      if (pl.bn == 160) k_conv_halo<160><<<nwg, 512, 0, st>>>(p);
      else k_conv_halo<128><<<nwg, 512, 0, st>>>(p);
    }
  } else if (pl.kind == 1) launch_dma<AMODE, SPLIT>(p, pl.var, st, fmt);
  else if (pl.bm == 128 && pl.bn == 160) launch_fmt<128, 160, AMODE, SPLIT>(p, fmt, st);
  else if (pl.bm == 128 && pl.bn == 128) launch_fmt<128, 128, AMODE, SPLIT>(p, fmt, st);
  else if (pl.bm == 128) launch_fmt<128, 64, AMODE, SPLIT>(p, fmt, st);
  else launch_fmt<64, 64, AMODE, SPLIT>(p, fmt, st);
}

// ---- skinny-M GEMV (M <= 4) ------------------------------------------------------------
// The SD3 stacked adaLN projection (M = CFG batch 2, N = 1.1 M rows of int4 codes, K 2432) and
// the per-step time-embedding linears are weight-stream (HBM) bound: a 64x64 MFMA tile wastes
// 62 of its 64 rows and reaches ~1 TB/s.  Here each wave owns 4 consecutive output rows at a
// time (grid-stride), its lanes stride over 32-element k chunks (16 B of int4 codes, 32 B of
// int8, 64 B of fp16 per chunk and row, 4 rows' loads in flight), the activation chunks a lane
// needs stay in registers for the whole kernel, and a butterfly reduces each (row, m) dot.
// Dequant is the tile loaders' half(q * s) and the epilogue rounds like gemm_epilogue
// (half(acc + bias) -> GELU-tanh -> + residual); only the fp32 summation order differs.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x2 __attribute__((ext_vector_type(2)));

template <int BFMT>
struct GemvChunk {
  static constexpr int NV = BFMT == QD_WFMT_F16 ? 4 : BFMT == QD_WFMT_I8 ? 2 : 1;  // 16-B loads
  i32x4 v[NV];
  float s;
  __device__ __forceinline__ void load(const GemmArgs& p, long n, int c) {
    const int k0 = c * 32;
    const i32x4* src;
    if constexpr (BFMT == QD_WFMT_F16) src = reinterpret_cast<const i32x4*>((const f16*)p.b + n * p.K + k0);
    else if constexpr (BFMT == QD_WFMT_I8) src = reinterpret_cast<const i32x4*>((const int8_t*)p.b + n * p.K + k0);
    else src = reinterpret_cast<const i32x4*>((const uint8_t*)p.b + n * (p.K / 2) + k0 / 2);
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = __builtin_nontemporal_load(src + q);
    s = BFMT == QD_WFMT_F16 ? 0.f : (float)p.bscale[n * (p.K / p.group) + k0 / p.group];
  }
  // weight k0 + e as the tile GEMM's fp16 operand
  __device__ __forceinline__ void decode(f16 (&w)[32]) const {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int wd[4] = {v[q][0], v[q][1], v[q][2], v[q][3]};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if constexpr (BFMT == QD_WFMT_F16) {
          w[q * 8 + 2 * d] = __builtin_bit_cast(f16, (unsigned short)(wd[d] & 0xffff));
          w[q * 8 + 2 * d + 1] = __builtin_bit_cast(f16, (unsigned short)((unsigned)wd[d] >> 16));
        } else if constexpr (BFMT == QD_WFMT_I8) {
#pragma unroll
          for (int e = 0; e < 4; ++e) w[q * 16 + d * 4 + e] = (f16)((float)(int)(int8_t)((wd[d] >> (8 * e)) & 0xff) * s);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int q = (int)(((unsigned)wd[d] >> ((e & 1) * 16 + (e >> 1) * 4)) & 0xf) - 8;
            w[d * 8 + e] = (f16)((float)q * s);
          }
        }
      }
    }
  }
};

// one 32-element k chunk of one weight row against the lane's activation slot j
template <int BFMT, int MM, int CPL>
__device__ __forceinline__ void gemv_dot(const GemvChunk<BFMT>& ch, const f16x8 (&a)[MM][CPL][4], int j,
                                         float (&out)[MM]) {
    if constexpr (BFMT == QD_WFMT_I4) {
      // packed decode: c | 0x6400 is the fp16 1024 + c = 1024 + q + 8, minus 1032 = q exactly;
      // v_pk_mul_f16 by s rounds q * s (exact in fp32) once, as the tile loader's
      // half((float)q * s).  Lanes of a pair are k = 8d + 2t and 8d + 2t + 1 (qd_pack_int4).
      const f16 sh = (f16)ch.s;
      const f16x2 s2 = {sh, sh};
      const f16x2 off = {(f16)1032.f, (f16)1032.f};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const unsigned u = (unsigned)ch.v[0][d];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f16x2 q2 = __builtin_bit_cast(f16x2, ((u >> (4 * t)) & 0x000F000Fu) | 0x64006400u) - off;
          const f16x2 w2 = q2 * s2;
#pragma unroll
          for (int m = 0; m < MM; ++m) {
            const f16x2 a2 = {a[m][j][d][2 * t], a[m][j][d][2 * t + 1]};
            out[m] = __builtin_amdgcn_fdot2(a2, w2, out[m], false);
          }
        }
      }
      return;
    }
    f16 w[32];
    ch.decode(w);
#pragma unroll
    for (int e = 0; e < 32; e += 2) {
      const f16x2 w2 = {w[e], w[e + 1]};
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        const f16x2 a2 = {a[m][j][e >> 3][e & 7], a[m][j][e >> 3][(e & 7) + 1]};
        out[m] = __builtin_amdgcn_fdot2(a2, w2, out[m], false);   // v_dot2_f32_f16
      }
    }
}

template <int BFMT, int MM, int CPL>
__global__ void __launch_bounds__(256) k_gemv(GemmArgs p) {
  constexpr int R = 4;
  const int lane = threadIdx.x & 63;
  const int nch = p.K / 32;
  f16x8 a[MM][CPL][4];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[m][j][q] = (m < p.M && c < nch) ? *reinterpret_cast<const f16x8*>(p.a + (long)m * p.lda + c * 32 + q * 8)
                                           : f16x8{};
      }
    }
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool gtanh = (p.epi & QD_EPI_GELU_TANH) != 0;
  const bool silu = (p.epi & QD_EPI_SILU) != 0;
  const int reps = (p.epi & QD_EPI_ROWREP) ? p.rows_per_sample : 1;
  const long nwaves = (long)gridDim.x * 4;
  for (long n0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R; n0 < p.N; n0 += nwaves * R) {
    float acc[R][MM];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MM; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = lane + 64 * j;
      if (c < nch) {
        GemvChunk<BFMT> ch[R];
#pragma unroll
        for (int r = 0; r < R; ++r) ch[r].load(p, n0 + r, c);   // N % 8 == 0: n0 + r < N
#pragma unroll
        for (int r = 0; r < R; ++r) {
          gemv_dot<BFMT, MM, CPL>(ch[r], a, j, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        float v = acc[r][m];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == r * MM + m && m < p.M) {
          const long n = n0 + r;
          f16 h = (f16)(v + (has_bias ? (float)p.bias[n] : 0.f));
          if (gtanh) h = (f16)gelu_tanh_f((float)h);
          if (has_res) h = (f16)((float)h + (float)p.res[(long)m * p.ldy + n]);
          if (silu) h = to_f16(silu_f((float)h));   // = k_silu on the rounded output
          p.y[(long)m * p.ldy + n] = h;
          for (int q = 1; q < reps; ++q) p.y[(long)q * p.ldy + n] = h;   // QD_EPI_ROWREP (M == 1)
        }
      }
  }
}

// chunks per lane the register-resident activation allows (0: not a GEMV shape)
// (M 5..8 - SD1.5's CFG-batch-8 time-embedding projections - was measured on an 8-row form of this
// kernel and left on the tile GEMM: 16.5 / 16.2 / 49.2 us against 12.8 / 18.8 / 20.6 us for
// 320 -> 1280, 1280 -> 1280 and the stacked 1280 -> 20160 projection, profiles/r06c_*: every wave
// re-reads the whole 8 x K activation, 20 KB per 4 weight rows at N 20160)
static int gemv_cpl(const GemmArgs& p) {
  if (p.M < 1 || p.M > 4 || (p.epi & (QD_EPI_AMAX | QD_EPI_GEGLU)) || p.K % 32) return 0;
  const int cpl = (p.K / 32 + 63) / 64;
  const int mm = p.M <= 2 ? 2 : 4;
  const int cap = mm == 2 ? 4 : 2;   // MM * CPL * 16 activation VGPRs <= 128
  return cpl <= cap ? (cpl <= 1 ? 1 : cpl <= 2 ? 2 : 4) : 0;
}

template <int BFMT, int MM>
static void launch_gemv_cpl(const GemmArgs& p, int cpl, int nwg, hipStream_t st) {
  if (cpl == 1) k_gemv<BFMT, MM, 1><<<nwg, 256, 0, st>>>(p);
  else if (cpl == 2) k_gemv<BFMT, MM, 2><<<nwg, 256, 0, st>>>(p);
  else if constexpr (MM == 2) k_gemv<BFMT, MM, 4><<<nwg, 256, 0, st>>>(p);
}

template <int BFMT>
static void launch_gemv_fmt(const GemmArgs& p, int cpl, hipStream_t st) {
  // one 4-row group per wave per pass; cap the grid at 8 waves per SIMD-slot's worth of CUs
  const long groups = (p.N + 3) / 4;
  const int nwg = (int)std::min<long>((groups + 3) / 4, 256L * 16);
  if (p.M <= 2) launch_gemv_cpl<BFMT, 2>(p, cpl, nwg, st);
  else launch_gemv_cpl<BFMT, 4>(p, cpl, nwg, st);
}

static void launch_gemv(const GemmArgs& p, int fmt, int cpl, hipStream_t st) {
  if (fmt == QD_WFMT_F16) launch_gemv_fmt<QD_WFMT_F16>(p, cpl, st);
  else if (fmt == QD_WFMT_I8) launch_gemv_fmt<QD_WFMT_I8>(p, cpl, st);
  else launch_gemv_fmt<QD_WFMT_I4>(p, cpl, st);
}

// M-fastest block order when the weight operand's bytes outweigh the activation operand's
// (GemmArgs::mfast; wbytes / abytes: bytes per element of each, in the K the GemmArgs carry)
static int block_order(const GemmArgs& p, bool linear, double wbytes, double abytes) {  // (convs: linear false)
  return (double)p.N * p.K * wbytes > (double)p.M * (linear ? p.K : p.Cip) * abytes ? 1 : 0;
}

static long split_ws_elems(const Plan& pl, int M, int N) { return pl.splits > 1 ? (long)pl.splits * M * N : 0; }

// row-complete LayerNorm epilogue (QD_EPI_LN): an LDS-DMA variant whose tile is the whole row -
// 64 x 320 (variant 18, two blocks per CU) or 128 x 320 (fp16: variant 1, two 64-deep stages, or
// 12, four 32-deep; int8: 12); a forced variant (qd_gemm_force 100 + v) is taken when it is one of
// them; -1 = no row-complete tile for N
static int ln_var(int N, bool i8) {
  if (N != 320) return -1;
  const int fv = g_force - 100;
  if (fv == 18 || fv == 12 || (!i8 && fv == 1)) return fv;
  return 18;
}

template <int AMODE>
static void run_gemm(GemmArgs& p, int fmt, float* ws, long ws_elems, hipStream_t st) {
  if (p.epi & QD_EPI_LN) {  // (host checks: F16 weights, N with a row-complete tile)
    p.splits = 1;
    p.kps = p.K;
    p.mfast = 0;
    launch_dma<AMODE, false>(p, ln_var(p.N, false), st, fmt);
    return;
  }
  const bool post = (p.epi & QD_EPI_AMAX_POST) != 0;
  const int w4g = fmt == QD_WFMT_I4 && p.bscale_t != nullptr && AMODE == AM_LINEAR ? p.group : 0;
  Plan pl = plan_gemm(p.M, p.N, p.K, fmt != QD_WFMT_F16, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0,
                      (p.epi & QD_EPI_GEGLU) != 0, post, w4g);
  if (pl.kind == 2 && (AMODE != AM_CONV || !halo_ok(p, pl.bn, 64, pl.bm))) {  // halo conv not applicable
    const int f = g_force;
    g_force = -1;
    pl = plan_gemm(p.M, p.N, p.K, fmt != QD_WFMT_F16, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0,
                   (p.epi & QD_EPI_GEGLU) != 0, post);
    g_force = f;
  }
  if (pl.kind == 2 && (!ws || ws_elems < split_ws_elems(pl, p.M, p.N)) && pl.splits > 1) {
    pl.splits = 1;  // halo split is over 64-channel chunks
    pl.kps = p.K / 576;
  }
  if (pl.kind != 2 && (AMODE == AM_CONV_ANY || !ws || ws_elems < split_ws_elems(pl, p.M, p.N))) {
    if (pl.splits > 1) {  // no room for slabs: best unsplit plan
      pl.splits = 1;
      pl.kps = p.K;
      if (pl.kind == 1 && (p.epi & QD_EPI_AMAX) && p.rows_per_sample % (kDmaC[pl.var].bm / kDmaC[pl.var].wgm) != 0) {
        const int f = g_force, sp = g_split;  // the explicitly split tile needs whole-sample wave rows unsplit
        g_force = -1;
        g_split = 0;
        pl = plan_gemm(p.M, p.N, p.K, fmt != QD_WFMT_F16, p.rows_per_sample, true, (p.epi & QD_EPI_GEGLU) != 0, post,
                       w4g);
        g_force = f;
        g_split = sp;
        pl.splits = 1;
        pl.kps = p.K;
      }
    }
  }
  p.splits = pl.splits;
  p.kps = pl.kps;
  // (convs only: with the rule on the linears too, SD3.5-L ran 3.8 % slower end to end - its
  // small-M context-stream projections, int4 or fp16 buffer alike - profiles/r04p_ab_mfast_sd35.log)
  p.mfast = AMODE == AM_LINEAR ? 0 : block_order(p, false, 2.0, 2.0);
  if (pl.splits == 1) {
    launch_tile<AMODE, false>(p, pl, fmt, st);
  } else {
    p.part = ws;
    launch_tile<AMODE, true>(p, pl, fmt, st);
    const int gx = (p.N + 255) / 256;
    if (const int r = fq_rpt(p)) {
      const dim3 g(p.N / 32, p.M / p.rows_per_sample);
      if (r == 1) k_splitk_reduce_fq<1><<<g, 256, 0, st>>>(p);
      else if (r == 2) k_splitk_reduce_fq<2><<<g, 256, 0, st>>>(p);
      else if (r == 4) k_splitk_reduce_fq<4><<<g, 256, 0, st>>>(p);
      else k_splitk_reduce_fq<8><<<g, 256, 0, st>>>(p);
      p.fq_done = 1;
    } else if ((long)gx * ((p.M + 15) / 16) >= 512) {
      k_splitk_reduce<4><<<dim3(gx, (p.M + 15) / 16), 256, 0, st>>>(p);
    } else {
      k_splitk_reduce<1><<<dim3(gx, (p.M + 3) / 4), 256, 0, st>>>(p);
    }
  }
}

static int check_common(const GemmArgs& p, int fmt) {
  QD_REQUIRE(p.a && p.b && p.y, "null pointer");
  QD_REQUIRE(p.M >= 0 && p.N > 0 && p.K > 0, "bad GEMM shape");
  QD_REQUIRE(p.K % 8 == 0, "K must be a multiple of 8");
  QD_REQUIRE(p.N % 8 == 0 && p.ldy % 8 == 0, "N and ldy must be multiples of 8");
  QD_REQUIRE(fmt == QD_WFMT_F16 || fmt == QD_WFMT_I8 || fmt == QD_WFMT_I4, "bad weight format");
  if (fmt != QD_WFMT_F16) {
    QD_REQUIRE(p.bscale && p.group > 0 && p.K % p.group == 0, "bad weight scales / group");
    QD_REQUIRE(p.group % 32 == 0, "quantized weights need group % 32 == 0");
    QD_REQUIRE(p.K % 64 == 0, "quantized weights need K % 64 == 0");
  }
  QD_REQUIRE(!(p.epi & QD_EPI_RESIDUAL) || p.res, "residual epilogue without residual");
  QD_REQUIRE(!(p.epi & QD_EPI_AMAX) || (p.amax && p.rows_per_sample > 0 && p.rows_per_sample % 64 == 0),
             "amax epilogue needs rows_per_sample % 64 == 0");
  QD_REQUIRE(!(p.epi & QD_EPI_GEGLU) || (!(p.epi & (QD_EPI_AMAX | QD_EPI_RESIDUAL)) && p.N % 32 == 0),
             "GEGLU epilogue: N % 32 == 0, no residual / amax");
  QD_REQUIRE(!(p.epi & QD_EPI_GELU_TANH) || !(p.epi & (QD_EPI_AMAX | QD_EPI_RESIDUAL | QD_EPI_GEGLU)),
             "GELU-tanh epilogue: no residual / amax / GEGLU");
  QD_REQUIRE(!(p.epi & QD_EPI_AMAX_POST) || ((p.epi & QD_EPI_AMAX) && (p.epi & QD_EPI_RESIDUAL) &&
                                             !(p.epi & (QD_EPI_GEGLU | QD_EPI_GELU_TANH))),
             "post-residual amax needs QD_EPI_AMAX | QD_EPI_RESIDUAL, no GEGLU / GELU-tanh");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(p.y) & 15) == 0, "y must be 16-B aligned");
  QD_REQUIRE((double)p.M * p.ldy * 2 < 2147483648.0, "output exceeds the 2 GiB buffer-addressing range");
  QD_REQUIRE(!p.bias || (reinterpret_cast<uintptr_t>(p.bias) & 7) == 0, "bias must be 8-B aligned");
  QD_REQUIRE(!p.res || (reinterpret_cast<uintptr_t>(p.res) & 15) == 0, "residual must be 16-B aligned");
  const double wbytes = (double)p.N * p.K * (fmt == QD_WFMT_F16 ? 2 : fmt == QD_WFMT_I8 ? 1 : 0.5);
  QD_REQUIRE(wbytes < 2147483648.0, "weight exceeds the 2 GiB buffer-addressing range");
  return 0;
}

extern "C" long qd_gemm_workspace(int M, int N, int K, int wfmt, int group, int rows_per_sample, int epi) {
  // the launch's own plan: an int4 weight plans its LDS-DMA stages with its group (qd_linear_fwd
  // with wscale_t), so the slab size queried here is the one that launch uses
  const Plan pl = plan_gemm(M, N, K, wfmt != QD_WFMT_F16, rows_per_sample, (epi & QD_EPI_AMAX) != 0,
                            (epi & QD_EPI_GEGLU) != 0, (epi & QD_EPI_AMAX_POST) != 0,
                            wfmt == QD_WFMT_I4 ? group : 0);
  return split_ws_elems(pl, M, N);
}

struct LnArgs {
  const void *g, *b;
  float eps;
  void* y;
  int8_t* y8;
  float* sa8;
};

static int check_ln(const GemmArgs& p, const LnArgs& ln) {
  QD_REQUIRE(ln_var(p.N, false) >= 0, "row-complete LayerNorm epilogue: no tile for this N (qd_linear_ln_ok)");
  QD_REQUIRE((p.epi & QD_EPI_RESIDUAL) && !(p.epi & (QD_EPI_AMAX | QD_EPI_GEGLU | QD_EPI_GELU_TANH)),
             "row-complete LayerNorm epilogue: residual, no amax / GEGLU / GELU-tanh");
  QD_REQUIRE(p.ldy == p.N, "row-complete LayerNorm epilogue: dense output (ldy == N)");
  QD_REQUIRE(ln.g && ln.b && (reinterpret_cast<uintptr_t>(ln.g) & 15) == 0 && (reinterpret_cast<uintptr_t>(ln.b) & 15) == 0,
             "LayerNorm gamma / beta: 16-B aligned fp16 [N]");
  QD_REQUIRE(ln.y8 ? (ln.sa8 && (reinterpret_cast<uintptr_t>(ln.y8) & 7) == 0)
                   : (ln.y && (reinterpret_cast<uintptr_t>(ln.y) & 15) == 0),
             "LayerNorm output: ln_y (16-B aligned fp16) or ln_y8 (8-B aligned) + ln_sa8");
  return 0;
}

static void set_ln(GemmArgs& p, const LnArgs& ln) {
  p.epi |= QD_EPI_LN;
  p.ln_g = (const f16*)ln.g;
  p.ln_b = (const f16*)ln.b;
  p.ln_eps = ln.eps;
  p.ln_y = (f16*)ln.y;
  p.ln_y8 = ln.y8;
  p.ln_sa8 = ln.sa8;
}

extern "C" int qd_linear_ln_ok(int N) { return ln_var(N, false) >= 0 ? 1 : 0; }

static int linear_fwd(const void* x, int M, int K, int lda, const void* w, int wfmt, const void* wscale,
                      const void* wscale_t, int group, const void* bias, const void* residual, void* y, int N,
                      int ldy, int epi, float* amax, int rows_per_sample, float* ws, long ws_elems, void* stream,
                      const LnArgs* ln) {
  QD_REQUIRE(!(epi & QD_EPI_LN), "QD_EPI_LN is set by qd_linear_ln");
  GemmArgs p{};
  p.epi_lds = g_epi_lds;
  p.a = (const f16*)x;
  p.lda = lda;
  p.b = w;
  p.bscale = (const f16*)wscale;
  p.bscale_t = wfmt == QD_WFMT_I4 ? (const f16*)wscale_t : nullptr;
  QD_REQUIRE(!p.bscale_t || (reinterpret_cast<uintptr_t>(wscale_t) & 15) == 0, "wscale_t must be 16-B aligned");
  p.group = group;
  p.bias = (const f16*)bias;
  p.res = (const f16*)residual;
  p.y = (f16*)y;
  p.ldy = ldy;
  p.amax = amax;
  p.rows_per_sample = rows_per_sample;
  p.M = M;
  p.N = N;
  p.K = K;
  p.epi = epi;
  int rc = check_common(p, wfmt);
  if (rc) return rc;
  if (ln) {
    QD_REQUIRE(wfmt == QD_WFMT_F16, "row-complete LayerNorm epilogue: fp16 weights (the dequantized buffer)");
    if ((rc = check_ln(p, *ln))) return rc;
    set_ln(p, *ln);
  }
  QD_REQUIRE(lda >= K && lda % 8 == 0 && ldy >= ((epi & QD_EPI_GEGLU) ? N / 2 : N), "bad leading dimensions");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-B aligned");
  QD_REQUIRE((double)M * lda * 2 < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (M == 0) return 0;
  p.a_bytes = (unsigned)((long)(M - 1) * lda * 2 + (long)K * 2);
  p.b_bytes = (unsigned)(wfmt == QD_WFMT_F16 ? (long)N * K * 2 : wfmt == QD_WFMT_I8 ? (long)N * K : (long)N * K / 2);
  if ((epi & QD_EPI_AMAX) && !(epi & QD_EPI_AMAX_ZEROED))  // stream-ordered, graph-capturable
    qd_zero_f32(amax, (size_t)((M + rows_per_sample - 1) / rows_per_sample) * N, S(stream));
  const int cpl = ln ? 0 : gemv_cpl(p);
  QD_REQUIRE(!(epi & QD_EPI_SILU) || cpl, "SiLU epilogue: GEMV shapes only (M <= 4, no amax / GEGLU)");
  QD_REQUIRE(!(epi & QD_EPI_ROWREP) || (cpl && M == 1 && rows_per_sample >= 1 && !(epi & QD_EPI_RESIDUAL) &&
                                        (double)rows_per_sample * ldy * 2 < 2147483648.0),
             "row-replicating epilogue: GEMV shapes with M == 1, rows_per_sample >= 1 output rows, no residual");
  if (cpl) launch_gemv(p, wfmt, cpl, S(stream));
  else run_gemm<AM_LINEAR>(p, wfmt, ws, ws_elems, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_linear_fwd(const void* x, int M, int K, int lda, const void* w, int wfmt,
                             const void* wscale, const void* wscale_t, int group, const void* bias,
                             const void* residual, void* y, int N, int ldy, int epi, float* amax,
                             int rows_per_sample, float* ws, long ws_elems, void* stream) {
  return linear_fwd(x, M, K, lda, w, wfmt, wscale, wscale_t, group, bias, residual, y, N, ldy, epi, amax,
                    rows_per_sample, ws, ws_elems, stream, nullptr);
}

extern "C" int qd_linear_ln(const void* x, int M, int K, int lda, const void* w, int wfmt, const void* wscale,
                            const void* wscale_t, int group, const void* bias, const void* residual, void* y, int N,
                            int ldy, int epi, const void* ln_gamma, const void* ln_beta, float ln_eps, void* ln_y,
                            int8_t* ln_y8, float* ln_sa8, float* ws, long ws_elems, void* stream) {
  const LnArgs ln{ln_gamma, ln_beta, ln_eps, ln_y, ln_y8, ln_sa8};
  return linear_fwd(x, M, K, lda, w, wfmt, wscale, wscale_t, group, bias, residual, y, N, ldy, epi, nullptr, 0, ws,
                    ws_elems, stream, &ln);
}

struct FqArgs {
  int n_bits;
  const void* residual;
  const void* cadd;
  int cadd_ld;
  float* xamax;
};

// ---- narrow-output 3x3 conv (Co <= 16: the UNet / VAE conv_out) ----------------------------------
// A 64-wide tile GEMM idles 15/16 of its MFMA columns and re-reads the input 9x at N = 8 (SD1.5's
// conv_out, 320 -> 4 (+4 pad) at 64x64, CFG batch 8: 40 us in k_gemm<64, 64> for 0.75 GFLOP and a 21 MB
// input).  Here a block owns 2 output rows x 64 pixels x every output channel: per 64-channel input
// chunk the 4 x 66-pixel halo and the chunk's [9 taps][16 co][64] weights are staged into LDS once
// (register-staged, double-buffered, one barrier per chunk) and each wave runs 2 pixel groups of 16
// as C^T = W . X^T on v_mfma_f32_16x16x32_f16 (A = weight fragment, shared by both groups).  Blocks are
// XCD-remapped so one XCD walks consecutive row pairs (the 2 halo rows two neighbouring tiles share
// stay in that XCD's L2).  Epilogue: + bias, fp16 rounding, the per-(n, co) amax of the rounded output
// (shuffles -> LDS -> one atomic per channel per block) - the F.conv2d of fake_quant.py:339 with the
// input of its output fake-quant.  K order: (64-channel chunk, tap, channel) - an fp32 summation order
// of its own, like the split-K / halo plans.  Requires 3x3, stride 1, pad 1, no upsample, Ci_pad % 64
// == 0, Co <= 16, Co % 4 == 0, W % 64 == 0, epilogue BIAS / AMAX only.
constexpr int NC_W = 64;                        // output pixels per tile row
constexpr int NC_HP = NC_W + 2;                 // halo pixels per row
constexpr int NC_ACT = 4 * NC_HP * 64;          // halo elements per chunk (4 rows x 66 px x 64 ch)
constexpr int NC_WT = 9 * 16 * 64;              // weight elements per chunk
constexpr int NC_AP = (4 * NC_HP * 8 + 255) / 256;  // 16-B activation pieces per thread
constexpr int NC_WP = (9 * 16 * 8) / 256 + 1;       // 16-B weight pieces per thread (1152 / 256 -> 5)

__global__ void __launch_bounds__(256) k_conv_narrow(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) f16 sm[2 * (NC_ACT + NC_WT)];
  __shared__ float red[4][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int segs = p.W / NC_W, rpairs = (p.H + 1) / 2;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int seg = wg % segs, rp = (wg / segs) % rpairs, n = wg / (segs * rpairs);
  const int r0 = 2 * rp, x0 = seg * NC_W;
  const int Cip = p.Cip, nch = Cip / 64;

  const __amdgpu_buffer_rsrc_t ars = rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.b, p.b_bytes);
  // staging maps: activation piece q -> (halo row, halo px, 16-B chunk); weight piece -> (tap, co, chunk)
  unsigned aoff[NC_AP];
  int adst[NC_AP];
#pragma unroll
  for (int i = 0; i < NC_AP; ++i) {
    const int q = tid + 256 * i;
    const int row = q / (NC_HP * 8), rem = q % (NC_HP * 8), px = rem >> 3, c = rem & 7;
    const int ih = r0 - 1 + row, iw = x0 - 1 + px;
    const bool ok = q < 4 * NC_HP * 8 && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
    aoff[i] = ok ? (unsigned)((((long)n * p.H + ih) * p.W + iw) * Cip + c * 8) * 2u : OOB;
    const int hp = row * NC_HP + px;  // linear halo pixel: the swizzle key of the fragment reads
    adst[i] = q < 4 * NC_HP * 8 ? hp * 64 + ((c ^ (hp & 7)) << 3) : -1;
  }
  unsigned woff[NC_WP];
  int wdst[NC_WP];
#pragma unroll
  for (int i = 0; i < NC_WP; ++i) {
    const int q = tid + 256 * i;
    const int tap = q / 128, co = (q >> 3) & 15, c = q & 7;
    const bool ok = q < 9 * 16 * 8 && co < p.N;
    woff[i] = ok ? (unsigned)(((long)co * 9 + tap) * Cip + c * 8) * 2u : OOB;
    wdst[i] = q < 9 * 16 * 8 ? NC_ACT + (tap * 16 + co) * 64 + ((c ^ (co & 7)) << 3) : -1;
  }
  f16x8 ast[NC_AP], wst[NC_WP];
  auto load = [&](int ch) {
    const unsigned ca = (unsigned)ch * 128u;  // 64 channels x 2 B
#pragma unroll
    for (int i = 0; i < NC_AP; ++i) ast[i] = bload(ars, aoff[i] == OOB ? OOB : aoff[i] + ca);
#pragma unroll
    for (int i = 0; i < NC_WP; ++i) wst[i] = bload(wrs, woff[i] == OOB ? OOB : woff[i] + ca);
  };
  auto store = [&](f16* buf) {
#pragma unroll
    for (int i = 0; i < NC_AP; ++i)
      if (adst[i] >= 0) *reinterpret_cast<f16x8*>(buf + adst[i]) = ast[i];
#pragma unroll
    for (int i = 0; i < NC_WP; ++i)
      if (wdst[i] >= 0) *reinterpret_cast<f16x8*>(buf + wdst[i]) = wst[i];
  };

  // wave w: pixel groups 2w, 2w + 1 = (tile row g >> 2, pixels 16 (g & 3) + 0..15)
  const int fr = lane & 15, fq = lane >> 4;
  int bsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int g = 2 * wid + j;
    bsrc[j] = (g >> 2) * NC_HP + 16 * (g & 3) + fr;  // halo pixel of tap (0, 0)
  }
  f32x4 acc[2] = {};
  load(0);
  store(sm);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    f16* cur = sm + (ch & 1) * (NC_ACT + NC_WT);
    if (ch + 1 < nch) load(ch + 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap % 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c16 = 4 * ks + fq;
        const f16x8 wf = *reinterpret_cast<const f16x8*>(cur + NC_ACT + (tap * 16 + fr) * 64 + ((c16 ^ (fr & 7)) << 3));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int hp = bsrc[j] + dy * NC_HP + dx;
          const f16x8 xf = *reinterpret_cast<const f16x8*>(cur + hp * 64 + ((c16 ^ (hp & 7)) << 3));
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf, xf, acc[j], 0, 0, 0);
        }
      }
    }
    if (ch + 1 < nch) store(sm + ((ch + 1) & 1) * (NC_ACT + NC_WT));
    __syncthreads();
  }
  // epilogue: lane holds channels 4 fq + r of pixel fr of each group
  const bool amax = (p.epi & QD_EPI_AMAX) != 0;
  const int co0 = 4 * fq;
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if ((p.epi & QD_EPI_BIAS) && p.bias && co0 < p.N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (float)p.bias[co0 + r];
  }
  float m[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int g = 2 * wid + j;
    const int oh = r0 + (g >> 2), ow = x0 + 16 * (g & 3) + fr;
    if (oh < p.H) {  // (odd H: the second row of the last pair lies outside)
      f16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        o[r] = (f16)(acc[j][r] + bv[r]);
        m[r] = fmaxf(m[r], fabsf((float)o[r]));   // channels >= N: zero weights and bias, o = 0
      }
      if (co0 < p.N) *reinterpret_cast<f16x4*>(p.y + (((long)n * p.H + oh) * p.W + ow) * p.ldy + co0) = o;
    }
  }
  if (amax) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m[r] = fmaxf(m[r], __shfl_xor(m[r], o, 64));
      if (fr == 0) red[wid][co0 + r] = m[r];
    }
    __syncthreads();
    if (tid < p.N) {
      const float v = fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid]));
      atomic_max_pos(p.amax + (long)n * p.N + tid, v);
    }
  }
}

static bool narrow_conv_ok(const GemmArgs& p) {
  return p.kh == 3 && p.kw == 3 && p.stride == 1 && p.pad == 1 && !p.ups && p.Cip % 64 == 0 && p.N <= 16 &&
         p.N % 4 == 0 && p.ldy == p.N && p.W % NC_W == 0 && !(p.epi & ~(QD_EPI_BIAS | QD_EPI_AMAX | QD_EPI_AMAX_ZEROED));
}

static int conv_fwd(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt, int co, int kh, int kw,
                    int stride, int pad, int upsample2x, const void* bias, const void* residual, void* y, int epi,
                    float* amax, float* ws, long ws_elems, void* stream, const FqArgs* fq) {
  GemmArgs p{};
  p.epi_lds = g_epi_lds;
  const int H = upsample2x ? 2 * h : h, W = upsample2x ? 2 * w : w;
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  p.a = (const f16*)x;
  p.lda = 0;
  p.b = wt;
  p.bias = (const f16*)bias;
  p.res = (const f16*)residual;
  p.y = (f16*)y;
  p.ldy = co;
  p.amax = amax;
  p.rows_per_sample = Ho * Wo;
  p.M = n * Ho * Wo;
  p.N = co;
  p.K = kh * kw * ci_pad;
  p.H = H;
  p.W = W;
  p.Hs = h;
  p.Ws = w;
  p.Cip = ci_pad;
  p.Ho = Ho;
  p.Wo = Wo;
  p.kh = kh;
  p.kw = kw;
  p.stride = stride;
  p.pad = pad;
  p.ups = upsample2x;
  p.epi = epi;
  int rc = check_common(p, QD_WFMT_F16);
  if (rc) return rc;
  QD_REQUIRE(ci_pad % 8 == 0 && ci_pad >= ci, "ci_pad must be a multiple of 8 and >= ci");
  QD_REQUIRE(stride >= 1 && pad >= 0 && Ho > 0 && Wo > 0, "bad conv geometry");
  QD_REQUIRE(!upsample2x || stride == 1, "upsample fusion needs stride 1");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-B aligned");
  QD_REQUIRE((double)n * h * w * ci_pad * 2 < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (p.M == 0) return 0;
  p.a_bytes = (unsigned)((long)n * h * w * ci_pad * 2);
  p.b_bytes = (unsigned)((long)co * p.K * 2);
  if ((epi & QD_EPI_AMAX) && !(epi & QD_EPI_AMAX_ZEROED))  // stream-ordered, graph-capturable
    qd_zero_f32(amax, (size_t)n * co, S(stream));
  if (fq) {  // the finalize's operands ride with the reduction (fq_rpt decides at the split plan)
    p.fq_qmax = (1 << (fq->n_bits - 1)) - 1;
    p.res = (const f16*)fq->residual;
    p.fq_cadd = (const f16*)fq->cadd;
    p.fq_cadd_ld = fq->cadd_ld > 0 ? fq->cadd_ld : co;
    p.fq_xamax = fq->xamax;
  }
  if (narrow_conv_ok(p)) {
    // Co <= 16 (conv_out): one block per 2 x 64 output pixels; any fused finalize runs as its own pass
    k_conv_narrow<<<n * ((Ho + 1) / 2) * (Wo / NC_W), 256, 0, S(stream)>>>(p);
  } else if (kh == 1 && kw == 1 && stride == 1 && pad == 0 && !upsample2x) {
    // a pointwise conv IS a GEMM over the NHWC pixel rows (x [N*H*W][Ci_pad]): no tap decode
    p.lda = ci_pad;
    run_gemm<AM_LINEAR>(p, QD_WFMT_F16, ws, ws_elems, S(stream));
  } else if (ci_pad % 64 == 0) {
    run_gemm<AM_CONV>(p, QD_WFMT_F16, ws, ws_elems, S(stream));
  } else {
    run_gemm<AM_CONV_ANY>(p, QD_WFMT_F16, ws, ws_elems, S(stream));
  }
  QD_CHECK_LAUNCH();
  if (fq && !p.fq_done) {  // unsplit plan: the GEMM reduced the amax, the finalize is its own pass
    const int rc2 = qd_fq_finalize(y, amax, n, Ho * Wo, co, fq->n_bits, fq->residual, fq->cadd, fq->cadd_ld, y, stream);
    if (rc2 || !fq->xamax) return rc2;
    return qd_act_absmax(y, QD_LAYOUT_NHWC, n, co, Ho, Wo, QD_GRAN_PER_CHANNEL, 0, fq->xamax, stream);
  }
  return 0;
}

extern "C" int qd_conv2d_fwd(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt,
                             int co, int kh, int kw, int stride, int pad, int upsample2x,
                             const void* bias, const void* residual, void* y, int epi, float* amax,
                             float* ws, long ws_elems, void* stream) {
  return conv_fwd(x, n, h, w, ci, ci_pad, wt, co, kh, kw, stride, pad, upsample2x, bias, residual, y, epi, amax, ws,
                  ws_elems, stream, nullptr);
}

extern "C" int qd_conv2d_fq(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt, int co, int kh,
                            int kw, int stride, int pad, int upsample2x, const void* bias, int n_bits,
                            const void* residual, const void* chan_add, int chan_add_ld, void* y, int epi, float* amax,
                            float* xamax, float* ws, long ws_elems, void* stream) {
  QD_REQUIRE((epi & QD_EPI_AMAX) && amax && !(epi & (QD_EPI_RESIDUAL | QD_EPI_AMAX_POST)),
             "qd_conv2d_fq: epi = QD_EPI_AMAX [| QD_EPI_AMAX_ZEROED | QD_EPI_BIAS], the residual is an argument");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "qd_conv2d_fq: 2 <= n_bits <= 16");
  // one add per output: the split-K reduction applies either the residual or the channel add
  QD_REQUIRE(!(residual && chan_add), "qd_conv2d_fq: residual and chan_add are mutually exclusive");
  QD_REQUIRE(!residual || (reinterpret_cast<uintptr_t>(residual) & 15) == 0, "residual must be 16-B aligned");
  QD_REQUIRE(!chan_add || ((reinterpret_cast<uintptr_t>(chan_add) & 15) == 0 && (chan_add_ld <= 0 || chan_add_ld >= co)),
             "chan_add: 16-B aligned rows, ld >= Co");
  const FqArgs fq{n_bits, residual, chan_add, chan_add_ld, xamax};
  return conv_fwd(x, n, h, w, ci, ci_pad, wt, co, kh, kw, stride, pad, upsample2x, bias, nullptr, y, epi, amax, ws,
                  ws_elems, stream, &fq);
}

// ---- int8 x int8 GEMM / conv (the int8-MFMA W8A8 mode) --------------------------------------
// The reference's W8A8 is fake-quant (fp16 F.linear / F.conv2d on dequantized values,
// fake_quant.py:223, 339); its granularities (conv weights per (Co, Ci, kh), activations per
// (n, c)) vary along the reduction, so no integer dot product reproduces it.  This mode
// re-granularizes to what factors out of an integer dot: weights per output channel (conv: over
// (kh, kw, Ci); linear: over K), activations per token (linear) or per sample (conv), codes from
// the reference's own RTN recipe, and runs v_mfma_i32_16x16x64_i8 (2x the fp16 MFMA rate) on the
// LDS-DMA pipeline with 64-B rows (one 64-code MFMA k-slice per stage).  Exact int32
// accumulation: every variant / split gives the same bits.
template <int V, int AMODE, bool SPLIT>
static void launch_i8_v(const GemmArgs& p, hipStream_t st) {
  constexpr DmaVar d = kDmaC[V];
  static_assert(d.bkt == 32 && d.pipe == 0, "int8 variants use the 64-B row layout");
  if constexpr (AMODE == AM_LINEAR && !SPLIT && V >= 10 && V <= 17 && V != 12 && V != 13) {
    if (p.pgrid > 0) {
      k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AMODE, false, true, false, false, true>
          <<<p.pgrid, 64 * d.wgm * d.wgn, 0, st>>>(p);
      return;
    }
  }
  const int nwg = ((p.M + d.bm - 1) / d.bm) * ((p.N + d.bn - 1) / d.bn) * p.splits;
  if constexpr (AMODE == AM_LINEAR && !SPLIT && V == 10) {
    if (epi_post_direct(p)) {
      k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AMODE, false, true, false, false, false, true>
          <<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
      return;
    }
  }
  k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AMODE, SPLIT, true><<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
}

// int8 ping-pong 256 x BN (qd_gemm_force 130 + i, BN = kPpBn[i])
static constexpr int kPpBn[] = {256, 320, 192, 160, 128};

template <int AMODE, bool SPLIT>
static void launch_pp_i8(const GemmArgs& p, int bn, hipStream_t st) {
  const int nwg = ((p.M + 255) / 256) * ((p.N + bn - 1) / bn) * p.splits;
  if (bn == 256) k_gemm_pp<256, 2, AMODE, SPLIT, true><<<nwg, 512, 0, st>>>(p);
  else if (bn == 320) k_gemm_pp<320, 2, AMODE, SPLIT, true><<<nwg, 512, 0, st>>>(p);
  else if (bn == 192) k_gemm_pp<192, 2, AMODE, SPLIT, true><<<nwg, 512, 0, st>>>(p);
  else if (bn == 160) k_gemm_pp<160, 4, AMODE, SPLIT, true><<<nwg, 512, 0, st>>>(p);
  else k_gemm_pp<128, 4, AMODE, SPLIT, true><<<nwg, 512, 0, st>>>(p);
}

template <int AMODE, bool SPLIT>
static void launch_i8(const GemmArgs& p, int var, hipStream_t st) {
  switch (var) {
    case 10: launch_i8_v<10, AMODE, SPLIT>(p, st); break;
    case 12: launch_i8_v<12, AMODE, SPLIT>(p, st); break;
    case 13: launch_i8_v<13, AMODE, SPLIT>(p, st); break;
    case 14: launch_i8_v<14, AMODE, SPLIT>(p, st); break;
    case 15: launch_i8_v<15, AMODE, SPLIT>(p, st); break;
    case 16: launch_i8_v<16, AMODE, SPLIT>(p, st); break;
    case 17: launch_i8_v<17, AMODE, SPLIT>(p, st); break;
    case 18:
      if constexpr (AMODE == AM_LINEAR && !SPLIT) launch_i8_v<18, AMODE, SPLIT>(p, st);
      break;
    default: launch_i8_v<11, AMODE, SPLIT>(p, st); break;
  }
}

// variant: qd_gemm_force 110..117 (DMA variants 10-17, the 64-B-row family), else a default by
// N; K (in the half view) splits into runs of whole 32-slot steps while the blocks fit one round
// post: post-residual amax epilogue - the lock-step DMA tiles only (the ping-pong epilogue
// reduces before its residual add); split only on an explicit split count (a tuner candidate:
// k_splitk_reduce takes the post-residual amax), never by the heuristic below, so tuned unsplit
// entries keep their plan
// gn: GroupNorm-statistics / per-(sample, column) add epilogue - lock-step DMA tiles that lie in
// one sample (rows_per_sample % BM == 0), or the halo conv; split-K plans reduce through
// k_splitk_reduce_gn (64-row blocks)
// A-stationary int8 linears (k_gemm_as_i8, qd_gemm_force 190 + c): tile BM x BN, K = KC codes
struct AsCfg {
  int bm, bn, kc, ring;
};
static constexpr AsCfg kAsC[] = {{256, 128, 320, 4}, {128, 256, 640, 3}, {128, 128, 640, 4}};

// the LDS-DMA variant an UNSPLIT int8 GEMM runs for the requested one: amax epilogues need every
// wave's rows in one sample, GroupNorm-statistics / channel-add epilogues every block's
static int i8_unsplit_var(int var, int rows_per_sample, bool amax, bool gn) {
  if (amax && rows_per_sample % (kDmaC[var].bm / kDmaC[var].wgm) != 0) var = 11;
  if (gn && rows_per_sample % kDmaC[var].bm != 0) var = rows_per_sample % 128 == 0 ? 11 : 15;  // tile in one sample
  return var;
}

static Plan plan_i8(int M, int N, int Kh, int rows_per_sample, bool amax, bool geglu, bool post = false,
                    bool gn = false) {
  if (g_force >= 190 && g_force <= 192) {
    // plain / bias / GEGLU (TN 4 tiles) epilogues, unsplit; the residual / LDS-form checks are in run_i8
    const AsCfg& c = kAsC[g_force - 190];
    const int tn = c.bn / (8 / (c.bm / 64)) / 16;
    if (Kh * 2 == c.kc && !amax && !post && !gn && (!geglu || tn % 4 == 0)) return Plan{4, c.bm, c.bn, g_force - 190, 1, Kh};
  }
  if (g_force >= 140 && g_force <= 149 && !geglu && Kh % 288 == 0) {
    // int8 halo conv (applicability checked at launch): 140 BN 160 / 141 BN 128 (3-slot weight
    // ring), 142 / 143 / 144 BN 160 with 4 / 5 / 6 slots (256-pixel tiles); 145 / 146 / 147:
    // 128-pixel tiles, two blocks per CU - BN 160 with 4 / 3 slots, BN 128 with 3; 148 / 149: one
    // 8x8 image per tile (64 pixels), BN 160 / 128, 3 slots; K splits over whole 64-code chunks
    // while the blocks fit one resident round
    const int bn = g_force == 141 || g_force == 147 || g_force == 149 ? 128 : 160;
    const int bm = g_force >= 148 ? 64 : g_force >= 145 ? 128 : 256;
    if (N % bn == 0 && M % bm == 0) {
      const long tiles_mn = (long)(M / bm) * (N / bn);
      const int nc = Kh / 288;
      Plan pl{2, bm, bn, g_force - 140, 1, nc};
      int fsp;
      if (forced_split(nc, 1, fsp)) {  // explicit split count (tuner candidate)
        pl.splits = fsp;
        pl.kps = nc / fsp;
        return pl;
      }
      for (int sp = 2; sp <= nc; ++sp) {
        if (nc % sp != 0) continue;
        if (tiles_mn * sp > 256L * (bm == 256 ? 1 : bm == 128 ? 2 : 3)) break;
        pl.splits = sp;
        pl.kps = nc / sp;
      }
      return pl;
    }
  }
  if (g_force >= 130 && g_force <= 134 && !post && !gn) {
    // ping-pong: wave rows 128 (BN >= 192) or 64 must lie in one sample for the amax epilogue
    const int bnp = kPpBn[g_force - 130];
    if (!amax || rows_per_sample % (bnp >= 192 ? 128 : 64) == 0) {
      Plan pl{3, 256, bnp, 0, 1, Kh};
      const long tiles_mn = (long)((M + 255) / 256) * ((N + bnp - 1) / bnp);
      int fsp;
      if (!geglu && Kh % 32 == 0 && forced_split(Kh / 32, 8, fsp)) {
        pl.splits = fsp;
        pl.kps = Kh / fsp;
        return pl;
      }
      for (int sp = 2; sp <= 32 && !geglu && Kh % 32 == 0; ++sp) {
        if ((Kh / 32) % sp != 0 || Kh / sp < 256) continue;
        if (tiles_mn * sp > 256L) break;
        pl.splits = sp;
        pl.kps = Kh / sp;
      }
      return pl;
    }
  }
  int var = N % 160 == 0 ? 10 : 11;
  if (g_force >= 110 && g_force <= 117) var = g_force - 100;
  int pdiv = 0;
  if (g_force >= 160 && g_force <= 177 && g_force % 10 <= 7) {
    var = 10 + g_force % 10;
    pdiv = g_force < 170 ? 2 : 4;
  }
  int fsp;
  // a split-K plan reduces the amax / GroupNorm statistics / channel add in its reduction kernel (64-row
  // blocks), so only an unsplit tile needs whole-sample rows: with an explicit split the requested tile
  // stands (the 8x8 level's GroupNorm convs otherwise all collapse to 64-row tiles, each re-reading the
  // whole weight once per 64 rows)
  const bool fsplit = g_force >= 110 && !geglu && !pdiv && Kh % 32 == 0 && forced_split(Kh / 32, 8, fsp) && fsp > 1;
  if (!fsplit) var = i8_unsplit_var(var, rows_per_sample, amax, gn);
  if (geglu && kDmaC[var].bn % 32 != 0) var = 11;
  const DmaVar& d = kDmaC[var];
  Plan pl{1, d.bm, d.bn, var, 1, Kh};
  if (pdiv && var != 12 && var != 13) {  // persistent: unsplit
    pl.pdiv = pdiv;
    return pl;
  }
  const long tiles_mn = (long)((M + d.bm - 1) / d.bm) * ((N + d.bn - 1) / d.bn);
  const int by_lds = 163840 / (2 * dma_lds_halves(d.bm, d.bn, d.st, d.bkt)), by_waves = 2048 / (64 * d.wgm * d.wgn);
  const int per_cu = std::max(1, std::min(by_lds, by_waves));
  if (g_force >= 110 && !geglu && Kh % 32 == 0 && forced_split(Kh / 32, 8, fsp)) {
    pl.splits = fsp;
    pl.kps = Kh / fsp;
    return pl;
  }
  for (int sp = 2; sp <= 32 && !geglu && !post && Kh % 32 == 0; ++sp) {
    if ((Kh / 32) % sp != 0 || Kh / sp < 256) continue;
    if (tiles_mn * sp > 256L * per_cu) break;
    pl.splits = sp;
    pl.kps = Kh / sp;
  }
  return pl;
}

static bool epi_gn(int epi) { return (epi & (QD_EPI_GNSTATS | QD_EPI_CADD)) != 0; }

template <int AMODE>
static void run_i8(GemmArgs& p, float* ws, long ws_elems, hipStream_t st) {
  if (p.epi & QD_EPI_LN) {
    p.splits = 1;
    p.kps = p.K;
    p.mfast = 0;
    launch_i8<AMODE, false>(p, ln_var(p.N, true), st);
    return;
  }
  const bool post = (p.epi & QD_EPI_AMAX_POST) != 0, gn = epi_gn(p.epi);
  Plan pl = plan_i8(p.M, p.N, p.K, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0, (p.epi & QD_EPI_GEGLU) != 0, post,
                    gn);
  if (pl.kind == 4 && (AMODE != AM_LINEAR || ((p.epi & QD_EPI_RESIDUAL) && p.res) || p.epi_lds)) {
    const int f = g_force;  // A-stationary tile not applicable (residual, the LDS-form knob, a conv)
    g_force = -1;
    pl = plan_i8(p.M, p.N, p.K, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0, (p.epi & QD_EPI_GEGLU) != 0, post, gn);
    g_force = f;
  }
  if (pl.kind == 2 && (AMODE != AM_CONV || !halo_ok(p, pl.bn, 32, pl.bm))) {  // int8 halo conv not applicable
    const int f = g_force;
    g_force = -1;
    pl = plan_i8(p.M, p.N, p.K, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0, (p.epi & QD_EPI_GEGLU) != 0, post, gn);
    g_force = f;
  }
  if (pl.splits > 1 && (!ws || ws_elems < split_ws_elems(pl, p.M, p.N))) {
    pl.splits = 1;
    pl.kps = pl.kind == 2 ? p.K / 288 : p.K;
    if (pl.kind == 1) {  // unsplit after all: the tile must hold whole-sample rows again
      pl.var = i8_unsplit_var(pl.var, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0, gn);
      pl.bm = kDmaC[pl.var].bm;
      pl.bn = kDmaC[pl.var].bn;
    }
  }
  p.splits = pl.splits;
  p.kps = pl.kps;
  p.mfast = AMODE == AM_LINEAR ? 0 : block_order(p, false, 1.0, 1.0);  // int8 codes on both sides (half view)
  p.pgrid = 0;
  if (AMODE == AM_LINEAR && pl.kind == 1 && pl.splits == 1 && pl.pdiv) {
    const long tiles = (long)((p.M + pl.bm - 1) / pl.bm) * ((p.N + pl.bn - 1) / pl.bn);
    const long g = (tiles + pl.pdiv - 1) / pl.pdiv;
    p.pgrid = (int)std::min(tiles, (g + 7) / 8 * 8);  // (a multiple of 8: logical tiles keep their XCD)
  }
  auto halo = [&]() {  // the kernel reads p.splits itself (int32 slabs when split)
    if (pl.var == 2) launch_halo_i8<160, 4>(p, st);
    else if (pl.var == 3) launch_halo_i8<160, 5>(p, st);
    else if (pl.var == 4) launch_halo_i8<160, 6>(p, st);
    else if (pl.var == 5) launch_halo_i8<160, 4, 128>(p, st);
    else if (pl.var == 6) launch_halo_i8<160, 3, 128>(p, st);
    else if (pl.var == 7) launch_halo_i8<128, 3, 128>(p, st);
    else if (pl.var == 8) launch_halo_i8<160, 3, 64>(p, st);
    else if (pl.var == 9) launch_halo_i8<128, 3, 64>(p, st);
    else if (pl.bn == 160) launch_halo_i8<160, 3>(p, st);
    else launch_halo_i8<128, 3>(p, st);
  };
  if constexpr (AMODE == AM_LINEAR) {
    if (pl.kind == 4) {
      const int npanel = (p.M + pl.bm - 1) / pl.bm, ntn = (p.N + pl.bn - 1) / pl.bn;
      p.as_nsplit = std::max(1, std::min(ntn, (256 + npanel / 2) / npanel));  // one block per CU
      const int grid = npanel * p.as_nsplit;
      if (pl.var == 0) k_gemm_as_i8<256, 128, 320, 4><<<grid, 512, 0, st>>>(p);
      else if (pl.var == 1) k_gemm_as_i8<128, 256, 640, 3><<<grid, 512, 0, st>>>(p);
      else k_gemm_as_i8<128, 128, 640, 4><<<grid, 512, 0, st>>>(p);
      return;
    }
  }
  if (pl.splits == 1) {
    if (pl.kind == 2) halo();
    else if (pl.kind == 3) launch_pp_i8<AMODE, false>(p, pl.bn, st);
    else launch_i8<AMODE, false>(p, pl.var, st);
  } else {
    p.part = ws;
    if (pl.kind == 2) halo();
    else if (pl.kind == 3) launch_pp_i8<AMODE, true>(p, pl.bn, st);
    else launch_i8<AMODE, true>(p, pl.var, st);
    const int gx = (p.N + 255) / 256;
    if (gn) k_splitk_reduce_gn<<<dim3((p.N + 63) / 64, p.M / 64), 256, 0, st>>>(p);
    else if ((long)gx * ((p.M + 15) / 16) >= 512) k_splitk_reduce<4><<<dim3(gx, (p.M + 15) / 16), 256, 0, st>>>(p);
    else k_splitk_reduce<1><<<dim3(gx, (p.M + 3) / 4), 256, 0, st>>>(p);
  }
}

static int check_i8(const GemmArgs& p) {
  QD_REQUIRE(p.a && p.b && p.y && p.sa && p.sw, "null pointer");
  QD_REQUIRE(p.M >= 0 && p.N > 0 && p.K > 0, "bad GEMM shape");
  QD_REQUIRE(p.N % 8 == 0 && p.ldy % 8 == 0, "N and ldy must be multiples of 8");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(p.sw) & 15) == 0, "sw must be 16-B aligned");
  QD_REQUIRE(!(p.epi & QD_EPI_RESIDUAL) || p.res, "residual epilogue without residual");
  QD_REQUIRE(!(p.epi & QD_EPI_AMAX) || (p.amax && p.rows_per_sample > 0 && p.rows_per_sample % 64 == 0),
             "amax epilogue needs rows_per_sample % 64 == 0");
  QD_REQUIRE(!(p.epi & QD_EPI_GEGLU) || (!(p.epi & (QD_EPI_AMAX | QD_EPI_RESIDUAL)) && p.N % 32 == 0),
             "GEGLU epilogue: N % 32 == 0, no residual / amax");
  QD_REQUIRE(!(p.epi & QD_EPI_GELU_TANH) || !(p.epi & (QD_EPI_AMAX | QD_EPI_RESIDUAL | QD_EPI_GEGLU)),
             "GELU-tanh epilogue: no residual / amax / GEGLU");
  QD_REQUIRE(!(p.epi & QD_EPI_AMAX_POST) || ((p.epi & QD_EPI_AMAX) && (p.epi & QD_EPI_RESIDUAL) &&
                                             !(p.epi & (QD_EPI_GEGLU | QD_EPI_GELU_TANH))),
             "post-residual amax needs QD_EPI_AMAX | QD_EPI_RESIDUAL, no GEGLU / GELU-tanh");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(p.y) & 15) == 0, "y must be 16-B aligned");
  QD_REQUIRE((double)p.M * p.ldy * 2 < 2147483648.0, "output exceeds the 2 GiB buffer-addressing range");
  QD_REQUIRE(!p.bias || (reinterpret_cast<uintptr_t>(p.bias) & 7) == 0, "bias must be 8-B aligned");
  QD_REQUIRE(!p.res || (reinterpret_cast<uintptr_t>(p.res) & 15) == 0, "residual must be 16-B aligned");
  QD_REQUIRE((double)p.N * p.K * 2 < 2147483648.0, "weight exceeds the 2 GiB buffer-addressing range");
  if (epi_gn(p.epi)) {
    QD_REQUIRE(!(p.epi & (QD_EPI_AMAX | QD_EPI_GEGLU | QD_EPI_GELU_TANH)),
               "GroupNorm-statistics / per-sample add epilogue: no amax / GEGLU / GELU-tanh");
    QD_REQUIRE(p.rows_per_sample > 0 && p.rows_per_sample % 64 == 0 && p.M % 64 == 0 && p.ldy == p.N,
               "GroupNorm-statistics / per-sample add epilogue: rows per sample % 64 == 0, dense output");
    QD_REQUIRE(!(p.epi & QD_EPI_GNSTATS) || (p.gnp && (reinterpret_cast<uintptr_t>(p.gnp) & 15) == 0),
               "gn_part must be a 16-B aligned buffer of M / 64 x N float4");
    QD_REQUIRE(!(p.epi & QD_EPI_CADD) || (p.cadd && p.cadd_ld >= p.N && p.cadd_ld % 8 == 0 &&
                                          (reinterpret_cast<uintptr_t>(p.cadd) & 15) == 0),
               "cadd must be a 16-B aligned [n][cadd_ld >= N] fp16 array, cadd_ld % 8 == 0");
  }
  return 0;
}

extern "C" long qd_gemm_i8_workspace(int M, int N, int K, int rows_per_sample, int epi) {
  const Plan pl = plan_i8(M, N, K / 2, rows_per_sample, (epi & QD_EPI_AMAX) != 0, (epi & QD_EPI_GEGLU) != 0,
                          (epi & QD_EPI_AMAX_POST) != 0, epi_gn(epi));
  return split_ws_elems(pl, M, N);
}

static int linear_i8(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                     const void* bias, const void* residual, void* y, int N, int ldy, int epi, float* amax,
                     int rows_per_sample, float* ws, long ws_elems, void* stream, const LnArgs* ln) {
  QD_REQUIRE(!(epi & QD_EPI_LN), "QD_EPI_LN is set by qd_linear_i8_ln");
  QD_REQUIRE(K % 64 == 0 && K > 0, "int8 GEMM needs K % 64 == 0");
  QD_REQUIRE(lda >= K && lda % 16 == 0, "int8 GEMM needs lda >= K, lda % 16 == 0");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0,
             "x and w must be 16-B aligned");
  GemmArgs p{};
  p.epi_lds = g_epi_lds;
  p.a = (const f16*)x;
  p.lda = lda / 2;
  p.b = w;
  p.bias = (const f16*)bias;
  p.res = (const f16*)residual;
  p.y = (f16*)y;
  p.ldy = ldy;
  p.amax = amax;
  p.rows_per_sample = rows_per_sample;
  p.M = M;
  p.N = N;
  p.K = K / 2;
  p.epi = epi;
  p.sa = sa;
  p.sa_rps = 0;
  p.sw = sw;
  p.i8 = 1;
  int rc = check_i8(p);
  if (rc) return rc;
  if (ln) {
    if ((rc = check_ln(p, *ln))) return rc;
    set_ln(p, *ln);
  }
  QD_REQUIRE(ldy >= ((epi & QD_EPI_GEGLU) ? N / 2 : N), "bad ldy");
  QD_REQUIRE((double)M * lda < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (M == 0) return 0;
  p.a_bytes = (unsigned)((long)(M - 1) * lda + K);
  p.b_bytes = (unsigned)((long)N * K);
  if ((epi & QD_EPI_AMAX) && !(epi & QD_EPI_AMAX_ZEROED))
    qd_zero_f32(amax, (size_t)((M + rows_per_sample - 1) / rows_per_sample) * N, S(stream));
  run_i8<AM_LINEAR>(p, ws, ws_elems, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_linear_i8(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                            const void* bias, const void* residual, void* y, int N, int ldy, int epi, float* amax,
                            int rows_per_sample, float* ws, long ws_elems, void* stream) {
  return linear_i8(x, sa, M, K, lda, w, sw, bias, residual, y, N, ldy, epi, amax, rows_per_sample, ws, ws_elems,
                   stream, nullptr);
}

// int8 GEGLU projection + per-token codes of its output (k_geglu_i8q): x [M, K] codes (lda), sa [M],
// w [N][K] codes with rows interleaved in 16-row [hidden | gate] blocks (as qd_linear_i8's GEGLU
// epilogue), sw [N] fp32, bias [N] fp16 -> y8 [M, N / 2] codes (ldy8) + sa8 [M]: bit-identical to
// qd_linear_i8(..., QD_EPI_GEGLU) followed by qd_quant_rows_i8.  Shapes: K = 320, N = 2560 (SD1.5's
// 64x64-level feed-forward); qd_linear_i8_geglu_q_ok tells.
extern "C" int qd_linear_i8_geglu_q_ok(int K, int N) { return K == 320 && N == 2560 ? 1 : 0; }

extern "C" int qd_linear_i8_geglu_q(const void* x, const float* sa, int M, int K, int lda, const void* w,
                                    const float* sw, const void* bias, int N, int8_t* y8, int ldy8, float* sa8,
                                    void* stream) {
  QD_REQUIRE(qd_linear_i8_geglu_q_ok(K, N), "qd_linear_i8_geglu_q: K = 320, N = 2560 only");
  QD_REQUIRE(x && sa && w && sw && y8 && sa8, "null pointer");
  QD_REQUIRE(lda >= K && lda % 16 == 0 && ldy8 >= N / 2 && ldy8 % 16 == 0, "lda / ldy8: >= the row, multiples of 16");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(y8) & 15) == 0 && (reinterpret_cast<uintptr_t>(sw) & 15) == 0,
             "x, w, y8, sw must be 16-B aligned");
  QD_REQUIRE(!bias || (reinterpret_cast<uintptr_t>(bias) & 7) == 0, "bias must be 8-B aligned");
  QD_REQUIRE((double)M * lda < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (M <= 0) return 0;
  GemmArgs p{};
  p.a = (const f16*)x;
  p.lda = lda / 2;
  p.b = w;
  p.bias = (const f16*)bias;
  p.M = M;
  p.N = N;
  p.K = K / 2;
  p.sa = sa;
  p.sw = sw;
  p.i8 = 1;
  p.a_bytes = (unsigned)((long)(M - 1) * lda + K);
  p.b_bytes = (unsigned)((long)N * K);
  // 8 waves, two per SIMD (the default, 150); 151: 4 waves with the whole register file (slower:
  // 110 vs 83 us at M 32768, profiles/r05h_geglu_q_bench.log - one wave per SIMD hides nothing)
  if (g_force == 151) k_geglu_i8q<5, 20, 1><<<(M + 63) / 64, 256, 0, S(stream)>>>(p, y8, ldy8, sa8);
  else k_geglu_i8q<5, 20, 2><<<(M + 63) / 64, 512, 0, S(stream)>>>(p, y8, ldy8, sa8);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_linear_i8_ln(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* sw,
                               const void* bias, const void* residual, void* y, int N, int ldy, int epi,
                               const void* ln_gamma, const void* ln_beta, float ln_eps, void* ln_y, int8_t* ln_y8,
                               float* ln_sa8, void* stream) {
  const LnArgs ln{ln_gamma, ln_beta, ln_eps, ln_y, ln_y8, ln_sa8};
  return linear_i8(x, sa, M, K, lda, w, sw, bias, residual, y, N, ldy, epi, nullptr, 0, nullptr, 0, stream, &ln);
}

extern "C" int qd_conv2d_i8(const void* x, const float* sa, int n, int h, int w, int ci, int ci_pad, const void* wt,
                            const float* sw, int co, int kh, int kw, int stride, int pad, int upsample2x,
                            const void* bias, const void* residual, void* y, int epi, float* amax,
                            const void* cadd, int cadd_ld, float* gn_part, float* ws, long ws_elems, void* stream) {
  QD_REQUIRE(ci_pad % 64 == 0 && ci_pad >= ci, "int8 conv needs ci_pad % 64 == 0");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(wt) & 15) == 0,
             "x and w must be 16-B aligned");
  GemmArgs p{};
  p.epi_lds = g_epi_lds;
  const int H = upsample2x ? 2 * h : h, W = upsample2x ? 2 * w : w;
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  p.a = (const f16*)x;
  p.b = wt;
  p.bias = (const f16*)bias;
  p.res = (const f16*)residual;
  p.y = (f16*)y;
  p.ldy = co;
  p.amax = amax;
  p.rows_per_sample = Ho * Wo;
  p.M = n * Ho * Wo;
  p.N = co;
  p.K = kh * kw * ci_pad / 2;
  p.H = H;
  p.W = W;
  p.Hs = h;
  p.Ws = w;
  p.Cip = ci_pad / 2;
  p.Ho = Ho;
  p.Wo = Wo;
  p.kh = kh;
  p.kw = kw;
  p.stride = stride;
  p.pad = pad;
  p.ups = upsample2x;
  p.epi = epi;
  p.sa = sa;
  p.sa_rps = Ho * Wo;  // one activation scale per sample
  p.sw = sw;
  p.i8 = 1;
  p.cadd = (const f16*)cadd;
  p.cadd_ld = cadd_ld > 0 ? cadd_ld : co;
  p.gnp = gn_part;
  int rc = check_i8(p);
  if (rc) return rc;
  QD_REQUIRE(stride >= 1 && pad >= 0 && Ho > 0 && Wo > 0, "bad conv geometry");
  QD_REQUIRE(!upsample2x || stride == 1, "upsample fusion needs stride 1");
  QD_REQUIRE((double)n * h * w * ci_pad < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (p.M == 0) return 0;
  p.a_bytes = (unsigned)((long)n * h * w * ci_pad);
  p.b_bytes = (unsigned)((long)co * kh * kw * ci_pad);
  if ((epi & QD_EPI_AMAX) && !(epi & QD_EPI_AMAX_ZEROED)) qd_zero_f32(amax, (size_t)n * co, S(stream));
  if (kh == 1 && kw == 1 && stride == 1 && pad == 0 && !upsample2x) {
    p.lda = ci_pad / 2;
    run_i8<AM_LINEAR>(p, ws, ws_elems, S(stream));
  } else {
    run_i8<AM_CONV>(p, ws, ws_elems, S(stream));
  }
  QD_CHECK_LAUNCH();
  return 0;
}

// ---- fp8 x fp8 GEMM (SD3.5's W4A8-fp8 mode, qd_linear_fp8) -------------------------------------
// A: per-token e4m3 activation codes, B: W4 codes as e4m3 with per-(group of 128, column) fp32
// scales gs[K / 128][N]; v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales: 2x the fp16 MFMA
// rate) per 128-code group, the group scale applied to the MFMA result, the token scale in the
// epilogue.  LDS-DMA variants with 128-B rows (BK 64 in the half view), no split-K.
static constexpr int kF8Var[] = {0, 2, 4, 9};  // qd_gemm_force 120 + i (no 256x256: it spills with the group-scale FMAs)

template <int V>
static void launch_f8_v(const GemmArgs& p, hipStream_t st) {
  constexpr DmaVar d = kDmaC[V];
  static_assert(d.bkt == 64 && d.pipe == 0, "fp8 variants use the 128-B row layout");
  const int nwg = ((p.M + d.bm - 1) / d.bm) * ((p.N + d.bn - 1) / d.bn);
  k_gemm_dma<d.bm, d.bn, d.wgm, d.wgn, d.st, d.pipe, d.bkt, AM_LINEAR, false, false, true>
      <<<nwg, 64 * d.wgm * d.wgn, 0, st>>>(p);
}

static int plan_f8(int N) {
  if (g_force >= 120 && g_force <= 123) return kF8Var[g_force - 120];
  return N % 160 == 0 ? 0 : 4;
}

extern "C" int qd_linear_fp8(const void* x, const float* sa, int M, int K, int lda, const void* w, const float* gs,
                             const void* bias, const void* residual, void* y, int N, int ldy, int epi, void* stream) {
  QD_REQUIRE(x && sa && w && gs && y, "null pointer");
  QD_REQUIRE(K % 128 == 0 && K > 0, "fp8 GEMM needs K % 128 == 0 (one 128-code weight group per step)");
  QD_REQUIRE(lda >= K && lda % 16 == 0, "fp8 GEMM needs lda >= K, lda % 16 == 0");
  QD_REQUIRE(M >= 0 && N > 0 && N % 8 == 0 && ldy % 8 == 0 && ldy >= N, "N / ldy must be multiples of 8, ldy >= N");
  QD_REQUIRE(!(epi & (QD_EPI_AMAX | QD_EPI_GEGLU)), "fp8 GEMM: no amax / GEGLU epilogue");
  QD_REQUIRE(!(epi & QD_EPI_GELU_TANH) || !(epi & QD_EPI_RESIDUAL), "GELU-tanh epilogue: no residual");
  QD_REQUIRE(!(epi & QD_EPI_RESIDUAL) || residual, "residual epilogue without residual");
  QD_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(gs) |
               reinterpret_cast<uintptr_t>(y)) & 15) == 0, "x, w, gs, y must be 16-B aligned");
  QD_REQUIRE(!bias || (reinterpret_cast<uintptr_t>(bias) & 7) == 0, "bias must be 8-B aligned");
  QD_REQUIRE(!residual || (reinterpret_cast<uintptr_t>(residual) & 15) == 0, "residual must be 16-B aligned");
  QD_REQUIRE((double)N * K < 2147483648.0 && (double)M * lda < 2147483648.0,
             "operands exceed the 2 GiB buffer-addressing range");
  if (M == 0) return 0;
  GemmArgs p{};
  p.epi_lds = g_epi_lds;
  p.a = (const f16*)x;
  p.lda = lda / 2;
  p.b = w;
  p.bias = (const f16*)bias;
  p.res = (const f16*)residual;
  p.y = (f16*)y;
  p.ldy = ldy;
  p.M = M;
  p.N = N;
  p.K = K / 2;
  p.epi = epi;
  p.sa = sa;
  p.gs = gs;
  p.f8 = 1;
  p.splits = 1;
  p.kps = p.K;
  p.a_bytes = (unsigned)((long)(M - 1) * lda + K);
  p.b_bytes = (unsigned)((long)N * K);
  hipStream_t st = S(stream);
  switch (plan_f8(N)) {
    case 0: launch_f8_v<0>(p, st); break;
    case 2: launch_f8_v<2>(p, st); break;
    case 9: launch_f8_v<9>(p, st); break;
    default: launch_f8_v<4>(p, st); break;
  }
  QD_CHECK_LAUNCH();
  return 0;
}
