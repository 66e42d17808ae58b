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

#include <cstdlib>
#include <type_traits>

using namespace qd;

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int KV_T = 64;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// V^T fragment through the gfx950 LDS transpose read: each 16-lane group gathers a 4-row x
// 16-column block of the row-major V tile and lane i receives column i (one head-dim index)
// of the 4 rows (4 consecutive keys).
__device__ __forceinline__ f16x4 tr_read(const f16* p) {
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
  return __builtin_bit_cast(f16x4, r);
}

// raw v_max3 / v_max (no canonicalising v_max x, x in front, which fmaxf brings)
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float maxf_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// max with the value of lane l ^ 32 / l ^ 16 (v_permlane32_swap / v_permlane16_swap)
__device__ __forceinline__ float xmax32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return maxf_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return maxf_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// LDS row stride (elements) of the row-major V tile: an odd multiple of 8 dwords, so the
// 8 consecutive rows one 32-lane half reads with ds_read_b64_tr_b16 hit 8 disjoint bank octets.
constexpr int v_stride(int dv) { return ((dv / 2 / 8) & 1) ? dv : dv + 16; }

// Swapped-operand flash attention (S^T = K Q^T, O^T = V^T P^T), 16x16x32 f16 MFMA.
//   * NW waves x 16 queries; a lane owns ONE query (column lane&15 of every accumulator), so
//     the softmax row max is 16 in-register maxes + 2 cross-group shuffles and the
//     online-softmax rescale is one scalar per lane, skipped (wave-uniformly) whenever no
//     lane's running max grew.
//   * P^T leaves the S^T accumulator straight into the B operand of the PV MFMA (k order
//     permuted to the accumulator's: kv = 32s + 16(j>>2) + 4g + (j&3)); V^T comes from the
//     row-major V tile with ds_read_b64_tr_b16 in that same k order.  P never touches LDS.
//   * The softmax denominator rides in the PV MFMA: V tile column d (head-dim padding,
//     DV > d) holds 1.0, so O^T row d accumulates sum(P) with the same fp16 P and the same
//     rescales as the numerator - no per-element VALU sum.
//   * K/V tiles register-staged and double-buffered in LDS (tile loop unrolled x2 so every
//     LDS address is a per-lane base + immediate); the next tile's loads are in flight while
//     the current one is computed; one barrier per tile.
//   * NQ query groups of 16 per wave: every K / V^T fragment read from LDS feeds NQ MFMAs, and
//     every staged K/V tile serves NW * 16 * NQ queries (LDS-read and L2->CU traffic per FLOP
//     both / NQ; at head_dim 40 both bound the NQ = 1 loop).
template <int DP, int DV, int NB, int NW, int NQ, bool CAUSAL = false>
__global__ void __launch_bounds__(NW * 64) k_attn(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                              int ldk, const f16* __restrict__ v, int ldv,
                                              f16* __restrict__ o, int ldo, int heads, int sq, int skv,
                                              int d, float scale_log2) {
  constexpr int KCH = DP / 8;                  // 16-B chunks per K row (QK^T depth DP)
  constexpr int KCHP = (KCH + 7) / 8 * 8;      // padded so the XOR swizzle stays in the row
  constexpr int VST = v_stride(DV);
  constexpr int KSZ = KV_T * KCHP * 8, VSZ = KV_T * VST;
  constexpr int VCH = DV / 8;
  constexpr int NT = NW * 64;
  constexpr int NKL = (KV_T * KCH + NT - 1) / NT, NVL = (KV_T * VCH + NT - 1) / NT;
  constexpr int TD = DV / 16;
  __shared__ __attribute__((aligned(16))) f16 smem[NB * (KSZ + VSZ)];

  // XCD-aware bijective remap: the q-blocks of one (batch, head) run on one XCD (blocks b and
  // b + 8 share an XCD), so that head's K/V stays in that XCD's L2 while they stream it.
  constexpr int QB = NW * 16 * NQ;                  // queries per block
  const int nqb = (sq + QB - 1) / QB;                // q-blocks per (batch, head)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int bh = wg / nqb;
  const int b = bh / heads, h = bh % heads;
  const int q0 = (wg - bh * nqb) * QB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;

  const f16* qb = q + (long)b * sq * ldq + h * d;
  const f16* kb = k + (long)b * skv * ldk + h * d;
  const f16* vb = v + (long)b * skv * ldv + h * d;
  f16* ob = o + (long)b * sq * ldo + h * d;
  const int dchunks = d >> 3;

  // B operand of S^T: Q[q = q0 + 16*(NQ*wid + g) + fr][dd = 32s + 8fq .. +8], pre-multiplied by
  // scale * log2(e) (one fp16 rounding per element), so the MFMA chain - seeded with -m, the
  // lane's running max - leaves the exponent s * scale * log2(e) - m ready for exp2: no per-score
  // fma in the loop (the softmax VALU issue bounds this kernel at head_dim 40).
  f16x8 qf[NQ][DP / 32];
#pragma unroll
  for (int g = 0; g < NQ; ++g) {
    const int qrow = q0 + (wid * NQ + g) * 16 + fr;
#pragma unroll
    for (int s = 0; s < DP / 32; ++s) {
      const int c = s * 4 + fq;
      f16x8 val = {};
      if (qrow < sq && c < dchunks) val = *reinterpret_cast<const f16x8*>(qb + (long)qrow * ldq + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) val[e] = (f16)((float)val[e] * scale_log2);
      qf[g][s] = val;
    }
  }

  // Padding of both tile buffers, written once: K chunks >= d/8 are zero; V columns >= d are
  // zero except column d = 1.0 (the denominator row of O^T).  Tile stores never touch them.
  for (int i = tid; i < NB * KV_T * KCHP; i += NT) {
    const int bf = i / (KV_T * KCHP), row = (i / KCHP) % KV_T, c = i % KCHP;
    if (c >= dchunks) *reinterpret_cast<f16x8*>(smem + bf * (KSZ + VSZ) + row * KCHP * 8 + ((c ^ (row & 7)) << 3)) = f16x8{};
  }
  for (int i = tid; i < NB * KV_T * (VST - d); i += NT) {
    const int bf = i / (KV_T * (VST - d)), row = (i / (VST - d)) % KV_T, col = d + i % (VST - d);
    smem[bf * (KSZ + VSZ) + KSZ + row * VST + col] = (f16)(col == d ? 1.0f : 0.0f);
  }

  // K/V tile loads: raw buffer loads; rows past skv fall off the end of the buffer and read 0.
  const unsigned kbytes = (unsigned)(((long)(skv - 1) * ldk + d) * 2);
  const unsigned vbytes = (unsigned)(((long)(skv - 1) * ldv + d) * 2);
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)kb, 0, kbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vb, 0, vbytes, 0x00020000);
  unsigned koff[NKL], voff[NVL];
  int kdst[NKL], vdst[NVL];  // LDS element offset within a buffer, -1 = padding chunk (skip)
#pragma unroll
  for (int i = 0; i < NKL; ++i) {
    const int e = tid + i * NT, row = e / KCH, c = e % KCH;
    const bool ok = e < KV_T * KCH && c < dchunks;
    koff[i] = (unsigned)(row * ldk + c * 8) * 2u;
    kdst[i] = ok ? row * KCHP * 8 + ((c ^ (row & 7)) << 3) : -1;
  }
#pragma unroll
  for (int i = 0; i < NVL; ++i) {
    const int e = tid + i * NT, row = e / VCH, c = e % VCH;
    const bool ok = e < KV_T * VCH && c < dchunks;
    voff[i] = (unsigned)(row * ldv + c * 8) * 2u;
    vdst[i] = ok ? KSZ + row * VST + c * 8 : -1;
  }
  f16x8 kst[NKL], vst[NVL];
  auto load_tile = [&](int kv0) {
    const unsigned ks0 = (unsigned)(kv0 * ldk) * 2u, vs0 = (unsigned)(kv0 * ldv) * 2u;
#pragma unroll
    for (int i = 0; i < NKL; ++i)
      kst[i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(krs, (int)(koff[i] + ks0), 0, 0));
#pragma unroll
    for (int i = 0; i < NVL; ++i)
      vst[i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(vrs, (int)(voff[i] + vs0), 0, 0));
  };
  auto store_tile = [&](f16* base) {
#pragma unroll
    for (int i = 0; i < NKL; ++i)
      if (kdst[i] >= 0) *reinterpret_cast<f16x8*>(base + kdst[i]) = kst[i];
#pragma unroll
    for (int i = 0; i < NVL; ++i)
      if (vdst[i] >= 0) *reinterpret_cast<f16x8*>(base + vdst[i]) = vst[i];
  };

  f32x4 oacc[NQ][TD];
  float mrow[NQ];    // running max of this lane's queries (log2 domain); 0 until the first tile sets it
  f32x4 mneg[NQ];    // -mrow broadcast: the seed accumulator of the S^T chain
  bool first = true; // the first tile always moves the max (wave-uniform)
#pragma unroll
  for (int g = 0; g < NQ; ++g) {
#pragma unroll
    for (int j = 0; j < TD; ++j) oacc[g][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    mrow[g] = 0.f;
    mneg[g] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  // per-lane LDS read offsets (elements, within a buffer)
  int kread[4][DP / 32];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < DP / 32; ++s) {
      const int row = j * 16 + fr, c = s * 4 + fq;
      kread[j][s] = row * KCHP * 8 + ((c ^ (row & 7)) << 3);
    }
  const int vread = KSZ + (fq * 4 + (fr >> 2)) * VST + (fr & 3) * 4;

  const int ntiles = (skv + KV_T - 1) / KV_T;
  auto tile = [&](const f16* ks, int kv0) {
    // ---- S^T[kv][q] = K Q^T: tile jt holds kv = 16jt + 4fq + r for query fr ----
    // ---- S'^T = K (c Q)^T - m: tile jt holds kv = 16jt + 4fq + r for query fr, log2 domain ----
    f32x4 sacc[NQ][4];
#pragma unroll
    for (int s = 0; s < DP / 32; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(ks + kread[j][s]);
#pragma unroll
        for (int g = 0; g < NQ; ++g)
          sacc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[g][s], s == 0 ? mneg[g] : sacc[g][j], 0, 0, 0);
      }
    if (kv0 + KV_T > skv) {
#pragma unroll
      for (int g = 0; g < NQ; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kv0 + j * 16 + fq * 4 + r >= skv) sacc[g][j][r] = -INFINITY;
    }
    // causal (CLIP text encoder): key kv is visible to query q iff kv <= q; key 0 is in the
    // first tile, so every query's running max is finite after it
    if (CAUSAL && kv0 + KV_T - 1 > q0) {
#pragma unroll
      for (int g = 0; g < NQ; ++g) {
        const int qrow = q0 + (wid * NQ + g) * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kv0 + j * 16 + fq * 4 + r > qrow) sacc[g][j][r] = -INFINITY;
      }
    }
    // ---- online softmax per query group (log2 domain) ----
    f16x8 pf[NQ][2];
#pragma unroll
    for (int g = 0; g < NQ; ++g) {
      // 16 scores -> one max as a depth-3 tree of three-input maxes (a serial chain stalls on each
      // dependency), then across the 4 lane groups holding the query's other keys with the
      // gfx950 permlane swaps (VALU, no LDS round trip as a ds_bpermute shuffle would take)
      float mx;
      {
        const f32x4* a = sacc[g];
        const float m0 = max3f(a[0][0], a[0][1], a[0][2]), m1 = max3f(a[0][3], a[1][0], a[1][1]);
        const float m2 = max3f(a[1][2], a[1][3], a[2][0]), m3 = max3f(a[2][1], a[2][2], a[2][3]);
        const float m4 = max3f(a[3][0], a[3][1], a[3][2]);
        mx = maxf_raw(max3f(m0, m1, m2), max3f(m3, m4, a[3][3]));
      }
      mx = xmax32(mx);
      mx = xmax16(mx);
      // deferred rescale: the running max is only moved when some lane's max grew by more than
      // 8 (log2 domain; mx is already relative to it), so P stays <= 2^8 (exact in fp16's range,
      // same relative rounding) and the O / denominator rescale is skipped on almost every tile
      // after the first.  The decision precedes this tile's exponentials, so nothing at the old
      // scale is pending; a moved max shifts this tile's exponents by the growth d.
      if (first || __any(mx > 8.0f)) {  // wave-uniform; lanes that did not grow get d = 0, alpha = 1
        const float d = first ? mx : fmaxf(mx, 0.f);
        if (!first) {  // (O is still zero on the first tile, where exp2(-d) may overflow)
          const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int j = 0; j < TD; ++j) oacc[g][j] *= alpha;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) sacc[g][j] -= d;
        mrow[g] += d;
        mneg[g] = (f32x4){-mrow[g], -mrow[g], -mrow[g], -mrow[g]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pf[g][j >> 1][(j & 1) * 4 + r] = (f16)__builtin_amdgcn_exp2f(sacc[g][j][r]);
    }
    first = false;
    // ---- O^T[d][q] += V^T P^T ----
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < TD; ++j) {
        const f16* vp = ks + vread + s * 32 * VST + j * 16;
        const f16x4 lo = tr_read(vp);
        const f16x4 hi = tr_read(vp + 16 * VST);
        const f16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int g = 0; g < NQ; ++g) oacc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[g][s], oacc[g][j], 0, 0, 0);
      }
  };

  load_tile(0);
  __syncthreads();  // padding writes above
  store_tile(smem);
  __syncthreads();
  if constexpr (NB == 2) {
    f16* const b0 = smem;
    f16* const b1 = smem + KSZ + VSZ;
    for (int t = 0; t < ntiles; t += 2) {
      if (t + 1 < ntiles) load_tile((t + 1) * KV_T);
      tile(b0, t * KV_T);
      if (t + 1 >= ntiles) break;
      store_tile(b1);
      __syncthreads();
      if (t + 2 < ntiles) load_tile((t + 2) * KV_T);
      tile(b1, (t + 1) * KV_T);
      if (t + 2 >= ntiles) break;
      store_tile(b0);
      __syncthreads();
    }
  } else {
    for (int t = 0; t < ntiles; ++t) {
      tile(smem, t * KV_T);
      if (t + 1 < ntiles) {
        load_tile((t + 1) * KV_T);
        __syncthreads();
        store_tile(smem);
        __syncthreads();
      }
    }
  }
  // ---- epilogue: lane holds O^T rows 16j + 4fq + r of query fr; row d holds sum(P) ----
  const int dj = d >> 4, dg = (d & 15) >> 2, dr = d & 3;  // (tile, lane group, reg) of row d
#pragma unroll
  for (int g = 0; g < NQ; ++g) {
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < TD; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j == dj && r == dr) lsum = oacc[g][j][r];
    lsum = __shfl(lsum, dg * 16 + fr, 64);
    const int qrow = q0 + (wid * NQ + g) * 16 + fr;
    if (qrow < sq) {
      const float inv = 1.0f / lsum;
#pragma unroll
      for (int j = 0; j < TD; ++j) {
        const int dd = j * 16 + fq * 4;
        if (dd < d) {
          f16x4 w;
#pragma unroll
          for (int r = 0; r < 4; ++r) w[r] = (f16)(oacc[g][j][r] * inv);
          *reinterpret_cast<f16x4*>(ob + (long)qrow * ldo + dd) = w;
        }
      }
    }
  }
}

// 32x32x16 form of the swapped-operand kernel for narrow heads (d = DP - 8: SD1.5's d = 40).
// The 16x16x32 kernel above is VALU-issue bound at d = 40: per 64-key tile a wave issues 28 MFMAs
// (each holds the SIMD's issue for 8 cycles), two cross-lane max reductions and 32 exponentials for
// its 32 queries.  Here a wave owns 32 queries as the 32 columns of v_mfma_f32_32x32x16 accumulators:
//   * S^T = K Q^T in 2 (key blocks) x DP/16 MFMAs: 6 at DP = 48 instead of 16 (QK^T depth 48, not 64);
//   * the running max rides in the QK^T MFMA: K column d (depth padding) is 1.0 and Q column d holds
//     -m, the lane's running max rounded to fp16 (every shift m_new - m_old between two fp16 values is
//     exact in fp32, so P = exp2(s - m) and the O rescales stay consistent); no seed registers;
//   * a lane holds 32 scores of ONE query (its partner lane l ^ 32 the other 32), so the online
//     softmax needs one in-register max tree; the cross-lane max (v_permlane32_swap) runs only on
//     the rare tiles that move the running max (wave-uniform test on the lane maxima = the same
//     decision as on the query maxima); the first tile is peeled (it always sets the max);
//   * P^T leaves the accumulator as the B operand of O^T += V^T P^T with no lane movement (registers
//     8s..8s+7 of key block jb = k-step s; element j of lane half h is key 32jb + 16s + 8(j>>2) + 4h
//     + (j&3)), V^T comes from the row-major V tile with ds_read_b64_tr_b16 in that k order;
//   * O^T rows d..DV-1 of the last 32-row block are padding except row d = sum(P) (V column d = 1.0).
// Per wave and 64-key tile: 6 + 2 * DV/32 MFMAs (14 at d = 40 vs 28), 6 ds_read_b128 + 8 * DV/32
// transposed reads, 32 v_exp_f32 + 16 packs as before.
constexpr int v_stride32(int dv) { return (dv + 31) / 64 * 64 + 32; }  // 16 x odd dwords per row

// STAG (8 waves): a half-tile stagger between the two waves that share a SIMD (waves w and w + 4;
// MI355X_MICROARCH "Two waves per SIMD", item 9).  The late half (waves 4-7) runs the softmax + PV of
// tile t - 1 and THEN the QK^T of tile t in the interval between barriers t and t + 1, so on every SIMD
// one wave's QK^T MFMAs meet its partner's exp / pack VALU instead of the partners issuing the same
// phase in lock step.  Its scores stay in registers across the barrier; V tiles get a third LDS buffer
// (tile t - 1's V is still read while tile t + 1 is staged).  Per query the same operations in the same
// order as the unstaggered kernel: bit-identical output.
template <int D, int DP, int DV, int NB, int NW, bool STAG = false>
__global__ void __launch_bounds__(NW * 64) k_attn32(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                                int ldk, const f16* __restrict__ v, int ldv,
                                                f16* __restrict__ o, int ldo, int heads, int sq, int skv,
                                                float scale_log2) {
  static_assert(DP % 16 == 0 && DV % 32 == 0 && NB == 2, "k_attn32 shapes");
  static_assert(!STAG || NW == 8, "the stagger pairs waves w and w + 4 of an 8-wave block");
  constexpr int d = D;                      // head_dim; depth d is the running-max column
  constexpr int CD = D / 8;                 // data chunks per row; chunk CD holds the ones column
  static_assert(D % 8 == 0 && DP >= D + 8 && D < DV, "k_attn32 head geometry");
  constexpr int KS = DP / 16;               // QK^T k-steps of 16
  constexpr int KCH = DP / 8;               // 16-B chunks per staged K / V row
  // K rows padded to an odd number of 16-B chunks (no swizzle): the 16 rows a ds_read_b128 lane group
  // reads (rows {0-3, 12-15, 20-27} + 32jb of one chunk) fall on 16 distinct 16-B bank slots
  constexpr int KCHP = KCH | 1;
  constexpr int VST = v_stride32(DV);
  constexpr int KSZ = KV_T * KCHP * 8, VSZ = KV_T * VST;
  constexpr int NVB = STAG ? 3 : 2;         // V tile buffers (K: always 2)
  constexpr int NT = NW * 64;
  constexpr int NL = (KV_T * CD + NT - 1) / NT;  // staged chunks per thread (d / 8 per row)
  constexpr int DB = DV / 32;               // 32-row O^T blocks
  __shared__ __attribute__((aligned(16))) f16 smem[2 * KSZ + NVB * VSZ];
  f16* const kbuf = smem;                   // K tile t in kbuf + (t & 1) * KSZ
  f16* const vbuf = smem + 2 * KSZ;         // V tile t in vbuf + (t % NVB) * VSZ

  constexpr int QB = NW * 32;
  const int nqb = (sq + QB - 1) / QB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int bh = wg / nqb;
  const int b = bh / heads, h = bh % heads;
  const int q0 = (wg - bh * nqb) * QB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lr = lane & 31, lh = lane >> 5, fr = lane & 15;
  const bool late = STAG && wid >= NW / 2;

  const f16* qb = q + (long)b * sq * ldq + h * d;
  const f16* kb = k + (long)b * skv * ldk + h * d;
  const f16* vb = v + (long)b * skv * ldv + h * d;
  f16* ob = o + (long)b * sq * ldo + h * d;
  const int qrow = q0 + wid * 32 + lr;

  // B operand of S^T: Q[qrow][16ks + 8lh .. +8] * scale * log2(e); the last chunk of lane half 1
  // is the padding chunk d / 8 whose element 0 carries -m
  f16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int c = 2 * s + lh;
    f16x8 val = {};
    if (qrow < sq && c < CD) val = *reinterpret_cast<const f16x8*>(qb + (long)qrow * ldq + c * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) val[e] = (f16)((float)val[e] * scale_log2);
    qf[s] = val;
  }

  // padding, written once: K chunk d/8 = {1, 0, ..}, further chunks 0; V column d = 1.0, columns > d 0
  for (int i = tid; i < 2 * KV_T * (KCHP - CD); i += NT) {
    const int np = KCHP - CD;
    const int bf = i / (KV_T * np), row = (i / np) % KV_T, c = CD + i % np;
    f16x8 z = {};
    if (c == CD) z[0] = (f16)1.0f;
    *reinterpret_cast<f16x8*>(kbuf + bf * KSZ + row * KCHP * 8 + c * 8) = z;
  }
  for (int i = tid; i < NVB * KV_T * (VST - d); i += NT) {
    const int bf = i / (KV_T * (VST - d)), row = (i / (VST - d)) % KV_T, col = d + i % (VST - d);
    vbuf[bf * VSZ + row * VST + col] = (f16)(col == d ? 1.0f : 0.0f);
  }

  const unsigned kbytes = (unsigned)(((long)(skv - 1) * ldk + d) * 2);
  const unsigned vbytes = (unsigned)(((long)(skv - 1) * ldv + d) * 2);
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)kb, 0, kbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)vb, 0, vbytes, 0x00020000);
  unsigned koff[NL], voff[NL];
  int kdst[NL], vdst[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = tid + i * NT, row = e / CD, c = e % CD;
    const bool ok = e < KV_T * CD;
    koff[i] = (unsigned)(row * ldk + c * 8) * 2u;
    voff[i] = (unsigned)(row * ldv + c * 8) * 2u;
    kdst[i] = ok ? row * KCHP * 8 + c * 8 : -1;
    vdst[i] = ok ? row * VST + c * 8 : -1;
  }
  // two register staging sets: tile t + 2 is loaded while tile t is computed and stored to LDS
  // after tile t + 1, so an L2 round trip has two tiles of compute to land in
  f16x8 kst[2][NL], vst[2][NL];
  auto load_tile = [&](int set, int kv0) {
    const unsigned ks0 = (unsigned)(kv0 * ldk) * 2u, vs0 = (unsigned)(kv0 * ldv) * 2u;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      kst[set][i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(krs, (int)(koff[i] + ks0), 0, 0));
      vst[set][i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(vrs, (int)(voff[i] + vs0), 0, 0));
    }
  };
  auto store_tile = [&](int set, f16* kbase, f16* vbase) {
#pragma unroll
    for (int i = 0; i < NL; ++i)
      if (kdst[i] >= 0) {
        *reinterpret_cast<f16x8*>(kbase + kdst[i]) = kst[set][i];
        *reinterpret_cast<f16x8*>(vbase + vdst[i]) = vst[set][i];
      }
  };

  f32x16 oacc[DB];
#pragma unroll
  for (int j = 0; j < DB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[j][r] = 0.f;
  float mrow = 0.f;  // running max (log2 domain), an fp16 value; -mrow sits in qf[CD / 2][0] of lane half CD & 1

  int kread[2][KS];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int row = jb * 32 + lr, c = 2 * s + lh;
      kread[jb][s] = row * KCHP * 8 + c * 8;
    }
  // 16-lane group g = lane >> 4 reads rows 4lh + (0..3) (+8 for elements 4..7) x columns 16(g & 1) + 0..15
  const int vread = (4 * lh + (fr >> 2)) * VST + 16 * ((lane >> 4) & 1) + (fr & 3) * 4;

  const int ntiles = (skv + KV_T - 1) / KV_T;
  // S'^T = K (c Q)^T - m of the 64-key tile at ks (kv0 = its first key), keys past skv -> -inf
  auto qk = [&](const f16* ks, int kv0, f32x16 (&sacc)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const f16x8 kf = *reinterpret_cast<const f16x8*>(ks + kread[jb][s]);
        sacc[jb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], s == 0 ? f32x16{} : sacc[jb], 0, 0, 0);
      }
    if (kv0 + KV_T > skv) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kv0 + jb * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh >= skv) sacc[jb][r] = -INFINITY;
    }
  };
  // online softmax of one tile's scores -> P (fp16, the PV MFMA's B operand) and O^T += V^T P^T from
  // the tile's V at vs (a software-pipelined form - QK^T of tile t + 1 issued before the softmax of
  // tile t, three LDS buffers - measured 339 vs 250 us: its 165 VGPRs leave one 8-wave block per CU)
  f16x8 pf[2][2];
  auto softmax = [&](f32x16 (&sacc)[2], auto first_tag) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first_tag)::value;
    // lane max of the 32 scores: a depth-4 tree of three-input maxes
    float lmx;
    {
      const f32x16& a = sacc[0];
      const f32x16& c = sacc[1];
      const float t0 = max3f(a[0], a[1], a[2]), t1 = max3f(a[3], a[4], a[5]), t2 = max3f(a[6], a[7], a[8]);
      const float t3 = max3f(a[9], a[10], a[11]), t4 = max3f(a[12], a[13], a[14]), t5 = max3f(a[15], c[0], c[1]);
      const float t6 = max3f(c[2], c[3], c[4]), t7 = max3f(c[5], c[6], c[7]), t8 = max3f(c[8], c[9], c[10]);
      const float t9 = max3f(c[11], c[12], c[13]), t10 = maxf_raw(c[14], c[15]);
      lmx = max3f(max3f(t0, t1, t2), max3f(t3, t4, t5), max3f(max3f(t6, t7, t8), t9, t10));
    }
    // deferred rescale as in k_attn (threshold 8, log2 domain); the first tile always sets the max
    if (FIRST || __any(lmx > 8.0f)) {
      const float mx = xmax32(lmx);  // the query max relative to mrow (lanes l, l ^ 32)
      const float mnew = (float)(f16)fminf(mrow + (FIRST ? mx : fmaxf(mx, 0.f)), 60000.f);
      const float dd = mnew - mrow;  // exact: both fp16 values
      if (!FIRST) {
        const float alpha = __builtin_amdgcn_exp2f(-dd);
#pragma unroll
        for (int j = 0; j < DB; ++j) oacc[j] *= alpha;
      }
      sacc[0] -= dd;
      sacc[1] -= dd;
      mrow = mnew;
      if (lh == (CD & 1)) qf[CD / 2][0] = (f16)(-mnew);
    }
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) pf[jb][s][e] = (f16)__builtin_amdgcn_exp2f(sacc[jb][8 * s + e]);
  };
  auto pv = [&](const f16* vs) __attribute__((always_inline)) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < DB; ++j) {
          const f16* vp = vs + vread + (32 * jb + 16 * s) * VST + 32 * j;
          const f16x4 lo = tr_read(vp);
          const f16x4 hi = tr_read(vp + 8 * VST);
          const f16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          oacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[jb][s], oacc[j], 0, 0, 0);
        }
  };

  {
    using T = std::true_type;
    using F = std::false_type;
    f32x16 sacc[2];
    // tile t (K at kt, V at vt): the early half (all waves when !STAG) runs QK^T, softmax and PV of
    // tile t; the late half runs the PV of tile t - 1 (V at vp, P from the previous interval), then
    // QK^T and softmax of tile t, whose P it keeps across the barrier (16 VGPRs: fewer than the
    // 32 fp32 scores, so the stagger keeps two 8-wave blocks per CU)
    auto run = [&](int t, const f16* kt, const f16* vt, const f16* vp, auto first_tag) __attribute__((always_inline)) {
      if (!late) {
        qk(kt, t * KV_T, sacc);
        softmax(sacc, first_tag);
        pv(vt);
      } else {
        if (t > 0) pv(vp);
        qk(kt, t * KV_T, sacc);
        softmax(sacc, first_tag);
      }
    };
    auto vof = [&](int t) { return vbuf + (NVB == 2 ? (t & 1) : t % 3) * VSZ; };
    // one barrier per tile; K double-buffered, V in NVB buffers; register staging sets alternate
    // (tile t in set t & 1, loaded two tiles ahead: unconditional loads - past the last tile they
    // read zeros off the buffer's end - so every path has the same loads in flight)
    load_tile(0, 0);
    __syncthreads();  // padding writes above
    store_tile(0, kbuf, vbuf);
    __syncthreads();
    load_tile(1, KV_T);
    load_tile(0, 2 * KV_T);
    run(0, kbuf, vbuf, nullptr, T{});
    int t = 1;
    for (; t + 1 < ntiles; t += 2) {  // tiles t (K buffer 1 / set 1) and t + 1 (K buffer 0 / set 0)
      store_tile(1, kbuf + KSZ, vof(t));
      __syncthreads();
      load_tile(1, (t + 2) * KV_T);
      run(t, kbuf + KSZ, vof(t), vof(t - 1), F{});
      store_tile(0, kbuf, vof(t + 1));
      __syncthreads();
      load_tile(0, (t + 3) * KV_T);
      run(t + 1, kbuf, vof(t + 1), vof(t), F{});
    }
    if (t < ntiles) {  // odd tail
      store_tile(1, kbuf + KSZ, vof(t));
      __syncthreads();
      run(t, kbuf + KSZ, vof(t), vof(t - 1), F{});
    }
    if (late) pv(vof(ntiles - 1));  // the late half's last PV (no barrier follows: that V stays put)
  }
  // ---- epilogue: lane holds O^T rows 32j + 8(r>>2) + 4lh + (r&3) of query qrow; row d = sum(P) ----
  constexpr int dj = d >> 5, dw = d & 31, dh = (dw >> 2) & 1, drr = (dw & 3) + 4 * (dw >> 3);
  const float lsum = __shfl(oacc[dj][drr], lr + 32 * dh, 64);
  if (qrow < sq) {
    const float inv = 1.0f / lsum;
#pragma unroll
    for (int j = 0; j < DB; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * j + 8 * g + 4 * lh;
        if (dd < d) {
          f16x4 w;
#pragma unroll
          for (int r = 0; r < 4; ++r) w[r] = (f16)(oacc[j][4 * g + r] * inv);
          *reinterpret_cast<f16x4*>(ob + (long)qrow * ldo + dd) = w;
        }
      }
  }
}

// measurement knob (qd_attn_force, benchmark sweeps only): 1 (8x2), 2 (8x1), 3 (4x1), 5 (4x2) of
// k_attn; 6 = k_attn (heuristic) instead of k_attn32 at d = 40 / 80; 7 / 8 = k_attn32 with 4 / 8
// waves (8: staggered); 9 = k_attn32, 8 waves without the stagger; 0: heuristic
static int g_attn_cfg = 0;
extern "C" int qd_attn_force(int cfg) {
  g_attn_cfg = cfg > 0 ? cfg : 0;
  return 0;
}
static int attn_forced() { return g_attn_cfg; }

template <int D, int DP, int DV>
static void launch32(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                     int ldo, int b, int heads, int sq, int skv, float scale, hipStream_t st) {
  const float sl2 = scale * 1.4426950408889634f;
  const int forced = attn_forced();
  // 8 waves (256 queries share each staged K / V tile) while the grid keeps >= 512 blocks
  if (forced == 8 || forced == 9 || (forced != 7 && (long)((sq + 255) / 256) * b * heads >= 512)) {
    // the stagger pays on long key sequences (SD1.5 64x64 self-attention: 254 -> 247 / 261 -> 257 us in
    // alternating rounds, profiles/r06b_attn_ab.log) and costs on 2-tile ones (77-token cross-attention
    // 21.5 -> 22.9 us: the late half's extra interval is not hidden)
    if (forced == 9 || (forced != 8 && skv < 512))  // the unstaggered 8-wave kernel
      k_attn32<D, DP, DV, 2, 8, false><<<((sq + 255) / 256) * b * heads, 512, 0, st>>>(
          (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, sl2);
    else
      k_attn32<D, DP, DV, 2, 8, true><<<((sq + 255) / 256) * b * heads, 512, 0, st>>>(
          (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, sl2);
  } else {
    k_attn32<D, DP, DV, 2, 4><<<((sq + 127) / 128) * b * heads, 256, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, sl2);
  }
}

template <int DP, int DV>
static void launch(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                   int ldo, int b, int heads, int sq, int skv, int d, float scale, int causal, hipStream_t st) {
  constexpr int NB = DP <= 96 ? 2 : 1;
  const float sl2 = scale * 1.4426950408889634f;
  if (causal) {
    // CLIP text encoder (77 tokens): one compile-time-causal instantiation per head width
    k_attn<DP, DV, NB, 4, 1, true><<<((sq + 63) / 64) * b * heads, 256, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  }
  if constexpr (DP > 256) {
    // wide heads (the VAE mid-block's single 512-channel head): 4 waves x 16 queries, one
    // 64-key K tile (64 KB) + V tile (66 KB) in LDS, O^T accumulators mostly in AGPRs
    k_attn<DP, DV, 1, 4, 1><<<((sq + 63) / 64) * b * heads, 256, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  } else {
  const int forced = attn_forced();
  if (forced == 1) {
    k_attn<DP, DV, NB, 8, 2><<<((sq + 255) / 256) * b * heads, 512, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  }
  if (forced == 2) {
    k_attn<DP, DV, NB, 8, 1><<<((sq + 127) / 128) * b * heads, 512, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  }
  if (forced == 5) {
    k_attn<DP, DV, NB, 4, 2><<<((sq + 127) / 128) * b * heads, 256, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  }
  if (forced == 3) {
    k_attn<DP, DV, NB, 4, 1><<<((sq + 63) / 64) * b * heads, 256, 0, st>>>(
        (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, sq, skv, d, sl2);
    return;
  }
  // long sequences: 8 waves x 2 query groups (256 queries) share each staged K/V tile while the
  // grid still holds >= 2 blocks per CU; then 8 x 1 (128 queries); 4 x 1 on short ones.
  // head_dim 49..64 (SD3.5 / SDXL): 4 waves x 2 groups (accumulators partly in AGPRs, 2 blocks
  // per CU) - scripts/attn_sweep.sh: 626 -> 543 us on SD3.5-L's joint attention, 272 -> 234 us
  // on SDXL's 64x64 level; at head_dim 40 (SD1.5) 8 x 2 stays ahead (304 vs 370 us).
  if (sq >= 512 && DV > 80 && DV <= 112) {
    // head_dim 65-96 (SD1.5's 32x32 level, d = 80): 8 waves x 2 query groups even below 512 blocks
    // (scripts/attn_bench.py: 43.7 -> 36-38 us at b 8, 1024 tokens, 8 heads; profiles/r02w_attn.log)
    const int grid = ((sq + 255) / 256) * b * heads;
    k_attn<DP, DV, NB, 8, 2><<<grid, 512, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv,
                                                  (f16*)o, ldo, heads, sq, skv, d, sl2);
  } else if (sq >= 512 && DV > 48 && DV <= 80) {
    const int grid = ((sq + 127) / 128) * b * heads;
    k_attn<DP, DV, NB, 4, 2><<<grid, 256, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv,
                                                  (f16*)o, ldo, heads, sq, skv, d, sl2);
  } else if (sq >= 512 && DP <= 96 && (long)((sq + 255) / 256) * b * heads >= 512) {
    const int grid = ((sq + 255) / 256) * b * heads;
    k_attn<DP, DV, NB, 8, 2><<<grid, 512, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv,
                                                  (f16*)o, ldo, heads, sq, skv, d, sl2);
  } else if (sq >= 512) {
    const int grid = ((sq + 127) / 128) * b * heads;
    k_attn<DP, DV, NB, 8, 1><<<grid, 512, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv,
                                                  (f16*)o, ldo, heads, sq, skv, d, sl2);
  } else {
    const int grid = ((sq + 63) / 64) * b * heads;
    k_attn<DP, DV, NB, 4, 1><<<grid, 256, 0, st>>>((const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv,
                                                  (f16*)o, ldo, heads, sq, skv, d, sl2);
  }
  }
}

static int attention_impl(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                          int ldo, int b, int heads, int sq, int skv, int d, float scale, int causal, void* stream) {
  QD_REQUIRE(q && k && v && o, "null pointer");
  QD_REQUIRE(d % 8 == 0 && d > 0 && d <= 512, "head_dim must be a multiple of 8 in (0, 512]");
  QD_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0,
             "leading dims must be multiples of 8 (q, k, v) and 4 (o)");
  QD_REQUIRE(skv > 0, "empty key sequence");
  QD_REQUIRE(!causal || skv == sq, "causal attention needs sq == skv");
  if ((long)b * heads * sq == 0) return 0;
  hipStream_t st = S(stream);
  const int c = causal;
  // DP: QK^T depth (multiple of 32 >= d); DV: PV rows, a multiple of 16 > d (row d = denominator)
  // the 32x32x16 kernel (QK^T depth: head dims + the running-max column, PV rows: head dims + the
  // denominator row, both rounded up) at head_dim 40 / 80 (at 64 - DP 80, DV 96 - it measured
  // slower than k_attn: profiles/r04m_attn_ab.log); qd_attn_force 1-6 select k_attn, 7 / 8 force
  // k_attn32 with 4 / 8 waves
  const int fc = attn_forced();
  if (!c && (fc == 0 || fc == 7 || fc == 8 || fc == 9) && (d == 40 || d == 80)) {
    if (d == 40) launch32<40, 48, 64>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, scale, st);
    else launch32<80, 96, 96>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, scale, st);
    QD_CHECK_LAUNCH();
    return 0;
  }
  if (d <= 32) launch<32, 48>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 40) launch<64, 48>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 56) launch<64, 64>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 64) launch<64, 80>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 72) launch<96, 80>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 88) launch<96, 96>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 96) launch<96, 112>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 120) launch<128, 128>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 128) launch<128, 144>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 152) launch<160, 160>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 160) launch<160, 176>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 248) launch<256, 256>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else if (d <= 256) launch<256, 272>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  else launch<512, 528>(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, c, st);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_attention(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                            void* o, int ldo, int b, int heads, int sq, int skv, int d, float scale,
                            void* stream) {
  return attention_impl(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, sq, skv, d, scale, 0, stream);
}

extern "C" int qd_attention_causal(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                   void* o, int ldo, int b, int heads, int s, int d, float scale, void* stream) {
  return attention_impl(q, ldq, k, ldk, v, ldv, o, ldo, b, heads, s, s, d, scale, 1, stream);
}
