// Fake-quant GEMMs on CDNA4 MFMA: the F.linear / F.conv2d of WxAxLinear / WxAxConv2d
// (quantize/fake_quant.py:223, 339) as ONE tiled kernel family.
//
//   C[M, N] = A[M, K] . B[N, K]^T, fp16 operands, fp32 accumulation (v_mfma_f32_16x16x32_f16)
//
// A operand: LINEAR  - activations [M][lda] (K contiguous)
//            CONV    - implicit im2col of an NHWC activation, K ordered (kh, kw, ci); rows are
//                      output pixels (n, oh, ow); padding / stride / nearest-2x upsample are
//                      resolved in the A-tile address computation (no im2col buffer).
// B operand: the quantized weight [N][K]: fp16 (dequantized), or int8 / packed-int4 codes +
//            fp16 group scales, dequantized in registers while staging into LDS
//            (w = half(q * s), bit-identical to the reference's stored buffer).
// Epilogue:  + bias, round to fp16 (the fp16 output of F.linear / F.conv2d), [+ residual],
//            [per-(sample, col) amax for the conv output fake-quant: wave-shuffle reduction
//            then one atomic per column per 64 rows].
//
// Tiling: 256 threads = 4 waves (2 x 2), block tile BM x BN x 64, wave tile (BM/2) x (BN/2) in
// 16x16 MFMA tiles.  LDS double-buffered, register-staged; 16-B chunks XOR-swizzled by
// (row & 7) so the ds_read_b128 fragment reads of 16 rows hit distinct bank slots.
// Blocks are remapped so each XCD (blockIdx % 8 group) gets a contiguous run of tiles that
// share A rows (L2 reuse; speed only, never correctness).
#include "common.h"

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

enum { AM_LINEAR = 0, AM_CONV = 1 };

struct GemmArgs {
  const f16* a;
  int lda;
  const void* b;
  const f16* bscale;
  int group;
  const f16* bias;
  const f16* res;
  f16* y;
  int ldy;
  float* amax;
  int rows_per_sample;
  int M, N, K;
  // conv geometry
  int H, W, Cin, Cip, Ho, Wo, kh, kw, stride, pad, ups;  // H, W: logical (post-upsample) input
  int epi;
};

constexpr int BK = 64;

template <int BM, int BN>
struct Smem {
  f16 a[2][BM * BK];
  f16 b[2][BN * BK];
};

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// ---- A staging ------------------------------------------------------------------------
template <int BM, int AMODE>
struct ALoader {
  static constexpr int CHUNKS = BM * BK / 8 / 256;  // 16-B chunks per thread
  f16x8 r[CHUNKS];
  // per-row precomputed geometry
  int row_ok[CHUNKS];
  long row_base[CHUNKS];  // LINEAR: element offset of the row; CONV: n * Hs * Ws * Cip
  int ih0[CHUNKS], iw0[CHUNKS];

  __device__ void init(const GemmArgs& p, int m0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CHUNKS; ++j) {
      const int row = (t >> 3) + 32 * j;
      const int m = m0 + row;
      row_ok[j] = m < p.M;
      const int mm = row_ok[j] ? m : 0;
      if (AMODE == AM_LINEAR) {
        row_base[j] = (long)mm * p.lda;
        ih0[j] = iw0[j] = 0;
      } else {
        const int ow = mm % p.Wo;
        const int oh = (mm / p.Wo) % p.Ho;
        const int n = mm / (p.Wo * p.Ho);
        const int Hs = p.ups ? p.H >> 1 : p.H, Ws = p.ups ? p.W >> 1 : p.W;
        row_base[j] = (long)n * Hs * Ws * p.Cip;
        ih0[j] = oh * p.stride - p.pad;
        iw0[j] = ow * p.stride - p.pad;
      }
    }
  }

  // k0: first k of the tile.  fast conv path: Cip % 64 == 0 -> the tile lies in one (kh, kw).
  __device__ void load(const GemmArgs& p, int k0) {
    // every chunk of this thread sits at the same k (only the row differs): decode once.
    const int k = k0 + (threadIdx.x & 7) * 8;
    const bool k_ok = k < p.K;
    if (AMODE == AM_LINEAR) {
#pragma unroll
      for (int j = 0; j < CHUNKS; ++j) {
        f16x8 v = {};
        if (row_ok[j] && k_ok) v = *reinterpret_cast<const f16x8*>(p.a + row_base[j] + k);
        r[j] = v;
      }
    } else {
      const int kpos = k / p.Cip;
      const int ci = k - kpos * p.Cip;
      const int ky = kpos / p.kw, kx = kpos - ky * p.kw;
      const int Ws = p.ups ? p.W >> 1 : p.W;
#pragma unroll
      for (int j = 0; j < CHUNKS; ++j) {
        f16x8 v = {};
        const int ih = ih0[j] + ky, iw = iw0[j] + kx;
        if (row_ok[j] && k_ok && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) {
          const int sh = p.ups ? ih >> 1 : ih, sw = p.ups ? iw >> 1 : iw;
          v = *reinterpret_cast<const f16x8*>(p.a + row_base[j] + ((long)sh * Ws + sw) * p.Cip + ci);
        }
        r[j] = v;
      }
    }
  }

  __device__ void store(f16* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CHUNKS; ++j) {
      const int row = (t >> 3) + 32 * j;
      *reinterpret_cast<f16x8*>(lds + swz(row, t & 7)) = r[j];
    }
  }
};

// ---- B staging ------------------------------------------------------------------------
template <int BN, int BFMT>
struct BLoader;

template <int BN>
struct BLoader<BN, QD_WFMT_F16> {
  static constexpr int CHUNKS = BN * BK / 8 / 256;
  f16x8 r[CHUNKS];
  __device__ void load(const GemmArgs& p, int n0, int k0) {
    const int t = threadIdx.x;
    const f16* B = (const f16*)p.b;
#pragma unroll
    for (int j = 0; j < CHUNKS; ++j) {
      const int row = (t >> 3) + 32 * j;
      const int n = n0 + row, k = k0 + (t & 7) * 8;
      f16x8 v = {};
      if (n < p.N && k < p.K) v = *reinterpret_cast<const f16x8*>(B + (long)n * p.K + k);
      r[j] = v;
    }
  }
  __device__ void store(f16* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < CHUNKS; ++j) {
      const int row = (t >> 3) + 32 * j;
      *reinterpret_cast<f16x8*>(lds + swz(row, t & 7)) = r[j];
    }
  }
};

// int8 codes: a 16-B load = 16 codes = 2 LDS chunks; thread -> (row, 16-code quarter)
template <int BN>
struct BLoader<BN, QD_WFMT_I8> {
  static constexpr int LOADS = BN * BK / 16 / 256;  // >= 1 for BN >= 64
  static_assert(LOADS >= 1, "BN too small for I8 staging");
  int4 r[LOADS];
  float s[LOADS];
  __device__ void load(const GemmArgs& p, int n0, int k0) {
    const int t = threadIdx.x;
    const int8_t* B = (const int8_t*)p.b;
    const int gpr = p.K / p.group;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 2) + 64 * j;
      const int n = n0 + row, k = k0 + (t & 3) * 16;
      int4 v = {0, 0, 0, 0};
      float sc = 0.f;
      if (n < p.N && k < p.K) {
        v = *reinterpret_cast<const int4*>(B + (long)n * p.K + k);
        sc = (float)p.bscale[(long)n * gpr + k / p.group];
      }
      r[j] = v;
      s[j] = sc;
    }
  }
  __device__ void store(f16* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 2) + 64 * j;
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
  __device__ void load(const GemmArgs& p, int n0, int k0) {
    const int t = threadIdx.x;
    const uint8_t* B = (const uint8_t*)p.b;
    const int gpr = p.K / p.group;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 1) + 128 * j;
      const int n = n0 + row, k = k0 + (t & 1) * 32;
      int4 v = {0, 0, 0, 0};
      float sc = 0.f;
      if (row < BN && n < p.N && k < p.K) {
        v = *reinterpret_cast<const int4*>(B + ((long)n * p.K + k) / 2);
        sc = (float)p.bscale[(long)n * gpr + k / p.group];
      }
      r[j] = v;
      s[j] = sc;
    }
  }
  __device__ void store(f16* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < LOADS; ++j) {
      const int row = (t >> 1) + 128 * j;
      if (row >= BN) continue;
      const int hq = t & 1;
      const int w[4] = {r[j].x, r[j].y, r[j].z, r[j].w};
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int nib = (w[cc] >> (4 * e)) & 0xf;
          const int q = nib >= 8 ? nib - 16 : nib;
          o[e] = (f16)((float)q * s[j]);
        }
        *reinterpret_cast<f16x8*>(lds + swz(row, 4 * hq + cc)) = o;
      }
    }
  }
};

// ---- kernel -----------------------------------------------------------------------------
template <int BM, int BN, int AMODE, int BFMT>
__global__ void __launch_bounds__(256, 2) k_gemm(GemmArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  __shared__ Smem<BM, BN> sm;

  // XCD-aware bijective remap of the linear block id (MI355X_MICROARCH: blocks b, b+8 share an XCD)
  const int nbm = (p.M + BM - 1) / BM, nbn = (p.N + BN - 1) / BN;
  const int nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int bm = wg / nbn, bn = wg % nbn;
  const int m0 = bm * BM, n0 = bn * BN;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * WM, wn0 = (wid & 1) * WN;

  ALoader<BM, AMODE> al;
  BLoader<BN, BFMT> bl;
  al.init(p, m0);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  al.load(p, 0);
  bl.load(p, n0, 0);
  al.store(sm.a[0]);
  bl.store(sm.b[0]);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      al.load(p, (kt + 1) * BK);
      bl.load(p, n0, (kt + 1) * BK);
    }
    const f16* As = sm.a[cur];
    const f16* Bs = sm.b[cur];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const f16x8*>(As + swz(wm0 + i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *reinterpret_cast<const f16x8*>(Bs + swz(wn0 + j * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      al.store(sm.a[cur ^ 1]);
      bl.store(sm.b[cur ^ 1]);
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + r ----
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn0 + j * 16 + fr;
    const bool col_ok = col < p.N;
    const float bv = (has_bias && col_ok) ? (float)p.bias[col] : 0.f;
    float cmax = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm0 + i * 16 + fq * 4 + r;
        if (row < p.M && col_ok) {
          f16 h = (f16)(acc[i][j][r] + bv);
          cmax = fmaxf(cmax, fabsf((float)h));
          if (has_res) h = (f16)((float)h + (float)p.res[(long)row * p.ldy + col]);
          p.y[(long)row * p.ldy + col] = h;
        }
      }
    }
    if (do_amax) {
      // rows of this wave tile: [m0 + wm0, m0 + wm0 + WM) lie in one sample (rows_per_sample % WM == 0)
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      const int row0 = m0 + wm0;
      if (fq == 0 && col_ok && row0 < p.M)
        atomic_max_pos(&p.amax[(long)(row0 / p.rows_per_sample) * p.N + col], cmax);
    }
  }
}

template <int BM, int BN, int AMODE>
static void launch_fmt(const GemmArgs& p, int fmt, hipStream_t st) {
  const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  if (fmt == QD_WFMT_F16) k_gemm<BM, BN, AMODE, QD_WFMT_F16><<<nwg, 256, 0, st>>>(p);
  else if (fmt == QD_WFMT_I8) k_gemm<BM, BN, AMODE, QD_WFMT_I8><<<nwg, 256, 0, st>>>(p);
  else k_gemm<BM, BN, AMODE, QD_WFMT_I4><<<nwg, 256, 0, st>>>(p);
}

template <int AMODE>
static void launch_gemm(const GemmArgs& p, int fmt, hipStream_t st) {
  // tile choice: N-waste first, then enough workgroups to fill 256 CUs
  const long blocks128 = (long)((p.M + 127) / 128) * ((p.N + 127) / 128);
  if (p.N % 128 == 0 && blocks128 >= 256) launch_fmt<128, 128, AMODE>(p, fmt, st);
  else if (p.M >= 4096 || p.N <= 64) launch_fmt<128, 64, AMODE>(p, fmt, st);
  else launch_fmt<64, 64, AMODE>(p, fmt, st);
}

static int check_common(const GemmArgs& p, int fmt) {
  QD_REQUIRE(p.a && p.b && p.y, "null pointer");
  QD_REQUIRE(p.M >= 0 && p.N > 0 && p.K > 0, "bad GEMM shape");
  QD_REQUIRE(p.K % 8 == 0, "K must be a multiple of 8");
  QD_REQUIRE(fmt == QD_WFMT_F16 || fmt == QD_WFMT_I8 || fmt == QD_WFMT_I4, "bad weight format");
  if (fmt != QD_WFMT_F16) {
    QD_REQUIRE(p.bscale && p.group > 0 && p.K % p.group == 0, "bad weight scales / group");
    QD_REQUIRE(p.group % 32 == 0, "quantized weights need group % 32 == 0");
    QD_REQUIRE(p.K % 64 == 0, "quantized weights need K % 64 == 0");
  }
  QD_REQUIRE(!(p.epi & QD_EPI_RESIDUAL) || p.res, "residual epilogue without residual");
  QD_REQUIRE(!(p.epi & QD_EPI_AMAX) || (p.amax && p.rows_per_sample > 0 && p.rows_per_sample % 64 == 0),
             "amax epilogue needs rows_per_sample % 64 == 0");
  QD_REQUIRE(!(p.epi & QD_EPI_GEGLU), "GEGLU epilogue not available in this build");
  return 0;
}

extern "C" int qd_linear_fwd(const void* x, int M, int K, int lda, const void* w, int wfmt,
                             const void* wscale, int group, const void* bias, const void* residual,
                             void* y, int N, int ldy, int epi, float* amax, int rows_per_sample,
                             void* stream) {
  GemmArgs p{};
  p.a = (const f16*)x;
  p.lda = lda;
  p.b = w;
  p.bscale = (const f16*)wscale;
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
  QD_REQUIRE(lda >= K && lda % 8 == 0 && ldy >= N, "bad leading dimensions");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-B aligned");
  if (M == 0) return 0;
  if (epi & QD_EPI_AMAX)  // amax is zeroed by the call (stream-ordered, graph-capturable)
    qd_zero_f32(amax, (size_t)((M + rows_per_sample - 1) / rows_per_sample) * N, S(stream));
  launch_gemm<AM_LINEAR>(p, wfmt, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_conv2d_fwd(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt,
                             int co, int kh, int kw, int stride, int pad, int upsample2x,
                             const void* bias, const void* residual, void* y, int epi, float* amax,
                             void* stream) {
  GemmArgs p{};
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
  p.Cin = ci;
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
  if (p.M == 0) return 0;
  if (epi & QD_EPI_AMAX)  // amax is zeroed by the call (stream-ordered, graph-capturable)
    qd_zero_f32(amax, (size_t)n * co, S(stream));
  launch_gemm<AM_CONV>(p, QD_WFMT_F16, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}
