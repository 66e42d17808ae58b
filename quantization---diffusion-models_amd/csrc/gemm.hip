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

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

enum { AM_LINEAR = 0, AM_CONV = 1, AM_CONV_ANY = 2 };

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
  int H, W, Hs, Ws, Cip, Ho, Wo, kh, kw, stride, pad, ups;  // H, W: logical (post-upsample) input
  int epi;
  // split-K
  float* part;
  int splits, kps;  // K per split (multiple of 64)
  unsigned a_bytes, b_bytes;
};

constexpr int BK = 64;
constexpr unsigned OOB = 0x80000000u;

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

// ---- shared epilogue pieces ---------------------------------------------------------------
// column amax of 4 columns over the 16 rows held by lanes fr = 0..15 of a lane group
__device__ __forceinline__ float rowgroup_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
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
  const int tile = wg / p.splits, split = wg - tile * p.splits;
  const int bm = tile / nbn, bn = tile - bm * nbn;
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
    const bool geglu = (p.epi & QD_EPI_GEGLU) != 0;
    if (geglu) {
      // weight rows interleaved in 16-row blocks [hidden 16 | gate 16]: fragment tiles j (hidden)
      // and j + 1 (gate) hold the same 16 output columns.  diffusers GEGLU: out =
      // half(h * half(gelu(g))) on the fp16 projection outputs h, g.
      // (TN is even for every tile the planner allows with GEGLU: BN in {64, 128})
#pragma unroll
      for (int j = 0; j + 1 < TN; j += 2) {
        const int nl = wn0 + j * 16 + fq * 4;
        const int n = n0 + nl;
        f16x4 bh = {}, bg = {};
        if (has_bias && n < p.N) {
          bh = *reinterpret_cast<const f16x4*>(p.bias + n);
          bg = *reinterpret_cast<const f16x4*>(p.bias + n + 16);
        }
        const int ol = (wn0 >> 1) + j * 8 + fq * 4;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ml = wm0 + i * 16 + fr;
          f16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const f16 h = (f16)(acc[i][j][r] + (float)bh[r]);
            const f16 g = (f16)(acc[i][j + 1][r] + (float)bg[r]);
            o[r] = (f16)((float)h * (float)(f16)gelu_f((float)g));
          }
          *reinterpret_cast<f16x4*>(ct + ml * LP + ol) = o;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wn0 + j * 16 + fq * 4;
        const int n = n0 + nl;
        const bool col_ok = n < p.N;  // N % 8 == 0: a lane's 4 columns are all in or all out
        f16x4 bq = {};
        if (has_bias && col_ok) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
        float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ml = wm0 + i * 16 + fr;
          const bool ok = m0 + ml < p.M && col_ok;
          f16x4 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = (f16)(acc[i][j][r] + (float)bq[r]);
            if (ok) cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
          }
          *reinterpret_cast<f16x4*>(ct + ml * LP + nl) = h;
        }
        if (do_amax) {
          // rows of this wave tile lie in one sample (rows_per_sample % WM == 0, host check)
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
    // output tile: BN columns (BN / 2 with GEGLU) starting at n0 (n0 / 2)
    const int cpr = geglu ? BN / 16 : BN / 8;
    const int on0 = geglu ? n0 >> 1 : n0, oN = geglu ? p.N >> 1 : p.N;
#pragma unroll 2
    for (int e = threadIdx.x; e < BM * cpr; e += 256) {
      const int row = e / cpr, c = e - row * cpr;
      const int m = m0 + row, n = on0 + c * 8;
      if (m < p.M && n < oN) {
        f16x8 v = *reinterpret_cast<const f16x8*>(ct + row * LP + c * 8);
        if (has_res) {
          const f16x8 rq = *reinterpret_cast<const f16x8*>(p.res + (long)m * p.ldy + n);
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = (f16)((float)v[r] + (float)rq[r]);
        }
        *reinterpret_cast<f16x8*>(p.y + (long)m * p.ldy + n) = v;
      }
    }
  }
}

// split-K reduction + epilogue: block = 64 rows x 256 columns (64 column quads x 4 row groups
// of 16 rows); slabs summed in split order (deterministic); amax: one atomic per column per
// 64 rows (rows_per_sample % 64 == 0).
__global__ void __launch_bounds__(256) k_splitk_reduce(GemmArgs p) {
  __shared__ float red[4][256];
  const int cq = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + cq * 4;
  const int mb = blockIdx.y * 64;
  const bool col_ok = n < p.N;
  const bool has_bias = (p.epi & QD_EPI_BIAS) && p.bias;
  const bool has_res = (p.epi & QD_EPI_RESIDUAL) && p.res;
  const bool do_amax = (p.epi & QD_EPI_AMAX) && p.amax;
  f16x4 bq = {};
  if (has_bias && col_ok) bq = *reinterpret_cast<const f16x4*>(p.bias + n);
  float cm[4] = {0.f, 0.f, 0.f, 0.f};
  if (col_ok) {
    for (int rr = 0; rr < 16; ++rr) {
      const int m = mb + rg * 16 + rr;
      if (m >= p.M) break;
      f32x4 s = *reinterpret_cast<const f32x4*>(p.part + (long)m * p.N + n);
      for (int k = 1; k < p.splits; ++k) s += *reinterpret_cast<const f32x4*>(p.part + ((long)k * p.M + m) * p.N + n);
      f16x4 h;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = (f16)(s[r] + (float)bq[r]);
        cm[r] = fmaxf(cm[r], fabsf((float)h[r]));
      }
      if (has_res) {
        const f16x4 rq = *reinterpret_cast<const f16x4*>(p.res + (long)m * p.ldy + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) h[r] = (f16)((float)h[r] + (float)rq[r]);
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

// ---- tile / split selection (host) ----------------------------------------------------------
struct Plan {
  int bm, bn, splits, kps;
};

// Cost model (seconds): a CU runs ~4 TFLOP/s of this kernel with 2 resident blocks, ~3 with
// one; tile efficiency eff; a launch takes ceil(blocks / 512) rounds of 2 blocks per CU.
// Splits add the fp32 slab round trip (~5 TB/s) and one reduction launch.
static Plan plan_gemm(int M, int N, int K, bool quant_w, int rows_per_sample, bool amax, bool geglu = false) {
  struct T {
    int bm, bn;
    double eff;
  } tiles[] = {{128, 160, 1.00}, {128, 128, 0.97}, {128, 64, 0.80}, {64, 64, 0.60}};
  Plan best{64, 64, 1, K};
  double best_t = 1e300;
  for (const T& t : tiles) {
    if (t.bn == 160 && N % 160 != 0) continue;  // 160-wide tiles only where they fit N exactly
    if (amax && rows_per_sample % (t.bm / 2) != 0) continue;
    if (quant_w && t.bn == 160) continue;        // int staging maps are built for BN % 64 == 0
    if (geglu && t.bn == 160) continue;          // GEGLU pairs 16-column fragments: WN % 32 == 0
    const long tiles_mn = (long)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn);
    for (int s = 1; s <= 16; s *= 2) {
      if (s > 1 && (K % (64 * s) != 0 || K / s < 512 || geglu)) break;
      const long blocks = tiles_mn * s;
      const double blk = 2.0 * t.bm * t.bn * ((double)K / s) / t.eff;  // flop of one block
      double tm = blocks <= 256 ? blk / 3e12 : (double)((blocks + 511) / 512) * 2.0 * blk / 4e12;
      if (s > 1) tm += 8.0 * M * N * s / 5e12 + 3e-6;
      if (tm < best_t * 0.98) {
        best_t = tm;
        best = {t.bm, t.bn, s, K / s};
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

template <int AMODE, bool SPLIT>
static void launch_tile(const GemmArgs& p, const Plan& pl, int fmt, hipStream_t st) {
  if (pl.bm == 128 && pl.bn == 160) launch_fmt<128, 160, AMODE, SPLIT>(p, fmt, st);
  else if (pl.bm == 128 && pl.bn == 128) launch_fmt<128, 128, AMODE, SPLIT>(p, fmt, st);
  else if (pl.bm == 128) launch_fmt<128, 64, AMODE, SPLIT>(p, fmt, st);
  else launch_fmt<64, 64, AMODE, SPLIT>(p, fmt, st);
}

static long split_ws_elems(const Plan& pl, int M, int N) { return pl.splits > 1 ? (long)pl.splits * M * N : 0; }

template <int AMODE>
static void run_gemm(GemmArgs& p, int fmt, float* ws, long ws_elems, hipStream_t st) {
  Plan pl = plan_gemm(p.M, p.N, p.K, fmt != QD_WFMT_F16, p.rows_per_sample, (p.epi & QD_EPI_AMAX) != 0,
                      (p.epi & QD_EPI_GEGLU) != 0);
  if (AMODE == AM_CONV_ANY || !ws || ws_elems < split_ws_elems(pl, p.M, p.N)) {
    if (pl.splits > 1) {  // no room for slabs: best unsplit plan
      pl.splits = 1;
      pl.kps = p.K;
    }
  }
  p.splits = pl.splits;
  p.kps = pl.kps;
  if (pl.splits == 1) {
    launch_tile<AMODE, false>(p, pl, fmt, st);
  } else {
    p.part = ws;
    launch_tile<AMODE, true>(p, pl, fmt, st);
    dim3 g((p.N + 255) / 256, (p.M + 63) / 64);
    k_splitk_reduce<<<g, 256, 0, st>>>(p);
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
  QD_REQUIRE((reinterpret_cast<uintptr_t>(p.y) & 15) == 0, "y must be 16-B aligned");
  QD_REQUIRE(!p.bias || (reinterpret_cast<uintptr_t>(p.bias) & 7) == 0, "bias must be 8-B aligned");
  QD_REQUIRE(!p.res || (reinterpret_cast<uintptr_t>(p.res) & 15) == 0, "residual must be 16-B aligned");
  const double wbytes = (double)p.N * p.K * (fmt == QD_WFMT_F16 ? 2 : fmt == QD_WFMT_I8 ? 1 : 0.5);
  QD_REQUIRE(wbytes < 2147483648.0, "weight exceeds the 2 GiB buffer-addressing range");
  return 0;
}

extern "C" long qd_gemm_workspace(int M, int N, int K, int wfmt, int rows_per_sample, int epi) {
  const Plan pl = plan_gemm(M, N, K, wfmt != QD_WFMT_F16, rows_per_sample, (epi & QD_EPI_AMAX) != 0,
                            (epi & QD_EPI_GEGLU) != 0);
  return split_ws_elems(pl, M, N);
}

extern "C" int qd_linear_fwd(const void* x, int M, int K, int lda, const void* w, int wfmt,
                             const void* wscale, int group, const void* bias, const void* residual,
                             void* y, int N, int ldy, int epi, float* amax, int rows_per_sample,
                             float* ws, long ws_elems, void* stream) {
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
  QD_REQUIRE(lda >= K && lda % 8 == 0 && ldy >= ((epi & QD_EPI_GEGLU) ? N / 2 : N), "bad leading dimensions");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-B aligned");
  QD_REQUIRE((double)M * lda * 2 < 2147483648.0, "activation exceeds the 2 GiB buffer-addressing range");
  if (M == 0) return 0;
  p.a_bytes = (unsigned)((long)(M - 1) * lda * 2 + (long)K * 2);
  p.b_bytes = (unsigned)(wfmt == QD_WFMT_F16 ? (long)N * K * 2 : wfmt == QD_WFMT_I8 ? (long)N * K : (long)N * K / 2);
  if ((epi & QD_EPI_AMAX) && !(epi & QD_EPI_AMAX_ZEROED))  // stream-ordered, graph-capturable
    qd_zero_f32(amax, (size_t)((M + rows_per_sample - 1) / rows_per_sample) * N, S(stream));
  run_gemm<AM_LINEAR>(p, wfmt, ws, ws_elems, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_conv2d_fwd(const void* x, int n, int h, int w, int ci, int ci_pad, const void* wt,
                             int co, int kh, int kw, int stride, int pad, int upsample2x,
                             const void* bias, const void* residual, void* y, int epi, float* amax,
                             float* ws, long ws_elems, void* stream) {
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
  if (ci_pad % 64 == 0) run_gemm<AM_CONV>(p, QD_WFMT_F16, ws, ws_elems, S(stream));
  else run_gemm<AM_CONV_ANY>(p, QD_WFMT_F16, ws, ws_elems, S(stream));
  QD_CHECK_LAUNCH();
  return 0;
}
