// Flash-style attention forward for the UNet's self / cross attention
// (diffusers AttnProcessor2_0 -> F.scaled_dot_product_attention, fp16 I/O, fp32 softmax).
//
// Workgroup = 4 waves = 64 query rows of one (batch, head); each wave owns 16 rows.
//   S = Q K^T  : v_mfma_f32_16x16x32_f16, K-dim = head_dim padded to 32 (Q frags in VGPRs,
//                K tile [64 kv][DP] in LDS, XOR-swizzled 16-B chunks)
//   online softmax in fp32 (row max / sum via 16-lane shuffles), P -> fp16 -> LDS
//   O += P V   : V tile stored transposed in LDS ([d][kv]) so the B fragment is a 16-B read.
// Q/K/V/O rows are token-major with head h at columns [h*D, h*D + D) (the to_q/to_k/to_v
// Linear outputs as they are), so no head split/merge copies exist.
#include "common.h"

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int KV_T = 64;

__device__ __forceinline__ int kswz(int row, int chunk, int rowchunks) {
  // XOR the low 3 bits of the chunk index (rows hold a multiple of 8 chunks)
  return row * rowchunks * 8 + (((chunk & ~7) | ((chunk & 7) ^ (row & 7))) << 3);
}

template <int DP, int DV>  // DP: head dim padded to 32 (QK^T K-dim); DV: head dim padded to 16
__global__ void __launch_bounds__(256) k_attn(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                              int ldk, const f16* __restrict__ v, int ldv,
                                              f16* __restrict__ o, int ldo, int heads, int sq, int skv,
                                              int d, float scale_log2) {
  constexpr int KCH = (DP / 8 + 7) / 8 * 8;  // chunks per K row in LDS (multiple of 8)
  constexpr int TNO = DV / 16;
  __shared__ f16 ks[KV_T * KCH * 8];
  __shared__ f16 vt[DV * KV_T];
  __shared__ f16 ps[4][16 * KV_T];

  const int bh = blockIdx.y;
  const int b = bh / heads, h = bh % heads;
  const int q0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  const f16* qb = q + (long)b * sq * ldq + h * d;
  const f16* kb = k + (long)b * skv * ldk + h * d;
  const f16* vb = v + (long)b * skv * ldv + h * d;
  f16* ob = o + (long)b * sq * ldo + h * d;

  // Q fragments: row q0 + wid*16 + fr, d = ks*32 + 8*fq .. +8
  f16x8 qf[DP / 32];
  {
    const int qrow = q0 + wid * 16 + fr;
#pragma unroll
    for (int s = 0; s < DP / 32; ++s) {
      const int dd = s * 32 + 8 * fq;
      f16x8 val = {};
      if (qrow < sq && dd < d) val = *reinterpret_cast<const f16x8*>(qb + (long)qrow * ldq + dd);
      qf[s] = val;
    }
  }

  f32x4 oacc[TNO];
#pragma unroll
  for (int j = 0; j < TNO; ++j) oacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mrow[r] = -INFINITY;
    lrow[r] = 0.f;
  }

  const int dchunks = d / 8;  // d % 8 == 0
  for (int kv0 = 0; kv0 < skv; kv0 += KV_T) {
    __syncthreads();  // previous tile fully consumed
    // ---- stage K [64][KCH*8] (zero-padded) and V^T [DV][64] ----
    for (int i = threadIdx.x; i < KV_T * KCH; i += 256) {
      const int row = i / KCH, c = i % KCH;
      f16x8 val = {};
      if (kv0 + row < skv && c < dchunks) val = *reinterpret_cast<const f16x8*>(kb + (long)(kv0 + row) * ldk + c * 8);
      *reinterpret_cast<f16x8*>(ks + kswz(row, c, KCH)) = val;
    }
    for (int i = threadIdx.x; i < KV_T * (DV / 8); i += 256) {
      const int row = i / (DV / 8), c = i % (DV / 8);  // row = kv, c = d chunk
      f16x8 val = {};
      if (kv0 + row < skv && c < dchunks) val = *reinterpret_cast<const f16x8*>(vb + (long)(kv0 + row) * ldv + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int dd = c * 8 + e;  // V^T row
        vt[dd * KV_T + ((((row >> 3) ^ (dd & 7)) << 3) | (row & 7))] = val[e];
      }
    }
    __syncthreads();

    // ---- S = Q K^T (16 x 64 per wave) ----
    f32x4 sacc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DP / 32; ++s) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(ks + kswz(j * 16 + fr, s * 4 + fq, KCH));
        sacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qf[s], kf, sacc[j], 0, 0, 0);
      }
    }
    // ---- online softmax (rows fq*4 + r, cols j*16 + fr) ----
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = kv0 + j * 16 + fr < skv;
        const float sv = ok ? sacc[j][r] * scale_log2 : -INFINITY;
        sacc[j][r] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mnew = fmaxf(mrow[r], mx);
      alpha[r] = exp2f(mrow[r] - mnew);
      mrow[r] = mnew;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float pv = exp2f(sacc[j][r] - mnew);
        sacc[j][r] = pv;
        sum += pv;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      lrow[r] = lrow[r] * alpha[r] + sum;
    }
#pragma unroll
    for (int j = 0; j < TNO; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) oacc[j][r] *= alpha[r];
    // ---- P -> LDS (fp16) as [16 q][64 kv], chunk-swizzled ----
    f16* pw = ps[wid];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = fq * 4 + r, col = j * 16 + fr;
        pw[row * KV_T + ((((col >> 3) ^ (row & 7)) << 3) | (col & 7))] = (f16)sacc[j][r];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes visible
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int pc = s * 4 + fq;
      const f16x8 pf = *reinterpret_cast<const f16x8*>(pw + fr * KV_T + ((pc ^ (fr & 7)) << 3));
#pragma unroll
      for (int j = 0; j < TNO; ++j) {
        const int dd = j * 16 + fr;
        const f16x8 vf = *reinterpret_cast<const f16x8*>(vt + dd * KV_T + ((pc ^ (dd & 7)) << 3));
        oacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pf, vf, oacc[j], 0, 0, 0);
      }
    }
  }
  // ---- epilogue ----
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qrow = q0 + wid * 16 + fq * 4 + r;
    if (qrow >= sq) continue;
    const float inv = 1.0f / lrow[r];
#pragma unroll
    for (int j = 0; j < TNO; ++j) {
      const int dd = j * 16 + fr;
      if (dd < d) ob[(long)qrow * ldo + dd] = (f16)(oacc[j][r] * inv);
    }
  }
}

template <int DP, int DV>
static void launch(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                   int ldo, int b, int heads, int sq, int skv, int d, float scale, hipStream_t st) {
  dim3 grid((sq + 63) / 64, b * heads);
  k_attn<DP, DV><<<grid, 256, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o,
                                       ldo, heads, sq, skv, d, scale * 1.4426950408889634f);
}

extern "C" int qd_attention(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                            void* o, int ldo, int b, int heads, int sq, int skv, int d, float scale,
                            void* stream) {
  QD_REQUIRE(q && k && v && o, "null pointer");
  QD_REQUIRE(d % 8 == 0 && d > 0 && d <= 256, "head_dim must be a multiple of 8 in (0, 256]");
  QD_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0, "leading dims must be multiples of 8");
  QD_REQUIRE(skv > 0, "empty key sequence");
  if ((long)b * heads * sq == 0) return 0;
  hipStream_t st = S(stream);
  if (d <= 32) launch<32, 32>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 48) launch<64, 48>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 64) launch<64, 64>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 80) launch<96, 80>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 96) launch<96, 96>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 128) launch<128, 128>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else if (d <= 160) launch<160, 160>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  else launch<256, 256>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, st);
  QD_CHECK_LAUNCH();
  return 0;
}
