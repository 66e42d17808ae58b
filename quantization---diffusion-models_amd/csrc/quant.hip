// Fake-quant kernels: activation / weight absmax RTN (quantize/fake_quant.py:21-167),
// the conv-output finalize pass, SmoothQuant calibration reductions and the SQ fold
// (utils/calib_data.py:105-124, quantizer_SQ.py:395-431).
//
// Bit-exactness: every kernel reproduces the reference's fp16 op-boundary rounding (common.h);
// tests/test_gpu_quant.py compares them bit-for-bit with tests/golden/fake_quant_golden.npz.
#include "common.h"

#include <cstdlib>

#include <atomic>
#include <cstring>

using namespace qd;

static thread_local char g_err[256] = "";
extern "C" int qd_set_error(int code, const char* msg) {
  std::strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
  return code;
}
extern "C" const char* qd_last_error(void) { return g_err; }
extern "C" int qd_version(void) { return 1; }
extern "C" int qd_device_arch(char* buf, int len) {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess)
    return qd_set_error(QD_ERR_ARG, "no HIP device");
  std::strncpy(buf, p.gcnArchName, len - 1);
  buf[len - 1] = 0;
  return 0;
}

static inline int qmax_of(int bits) { return (1 << (bits - 1)) - 1; }

__global__ void k_zero_f32(float* __restrict__ p, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

void qd_zero_f32(float* p, size_t n, hipStream_t st) {
  if (n == 0) return;
  k_zero_f32<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(p, n);
}

extern "C" int qd_fill_zero(float* p, long n, void* stream) {
  QD_REQUIRE(p || n == 0, "null pointer");
  QD_REQUIRE(n >= 0, "negative size");
  if (n) qd_zero_f32(p, (size_t)n, reinterpret_cast<hipStream_t>(stream));
  QD_CHECK_LAUNCH();
  return 0;
}

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------------------
// amax reductions
// ---------------------------------------------------------------------------------------

// NHWC per-(n, c) column max over rows.  block (bx, by), bx * by <= 256: x = 8-channel chunk
// (bx = min(chunks, 64): no idle lanes at C = 320), y = row lane, 8 row loads in flight per
// thread.  grid (ceil(chunks / bx), n, row_splits).  requires c % 8 == 0.
// x2 != null: channels [c1, c) come from x2 (row stride c - c1), [0, c1) from x (row stride c1)
__global__ void __launch_bounds__(256) k_colmax_nhwc(const f16* __restrict__ x, const f16* __restrict__ x2, int c1,
                                                     int hw, int c, int rows_per_split, float* __restrict__ amax) {
  __shared__ float red[256][8];
  const int bx = blockDim.x, by = blockDim.y;
  const int chunk = blockIdx.x * bx + threadIdx.x;
  const int n = blockIdx.y;
  const int r0 = blockIdx.z * rows_per_split;
  const int r1 = min(hw, r0 + rows_per_split);
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = 0.f;
  if (chunk * 8 < c) {
    const int ch = chunk * 8;
    const bool first = x2 == nullptr || ch < c1;
    const int ld = x2 == nullptr ? c : (first ? c1 : c - c1);
    const f16* base = first ? x + (size_t)n * hw * ld + ch : x2 + (size_t)n * hw * ld + (ch - c1);
    for (int rb = r0 + threadIdx.y; rb < r1; rb += 8 * by) {
      f16x8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f16x8*>(base + (size_t)min(rb + by * u, r1 - 1) * ld);
#pragma unroll
      for (int u = 0; u < 8; ++u) QD_PIN(v[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (rb + by * u >= r1) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf((float)v[u][j]));
      }
    }
  }
  const int t = threadIdx.y * bx + threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = m[j];
  __syncthreads();
  if (threadIdx.y == 0 && chunk * 8 < c) {
    for (int k = 1; k < by; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], red[k * bx + threadIdx.x][j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) atomic_max_pos(&amax[(size_t)n * c + chunk * 8 + j], m[j]);
  }
}

// launch geometry of k_colmax_nhwc: up to 64 rows per thread while the grid keeps >= 128
// blocks.  Each block ends in one atomic max per channel, and same-address device atomics
// serialise (per-XCD L2s: they resolve beyond L2), so the row splits per sample - the atomic
// chain length per address - are kept short: measured (rocprofv3, scripts/colmax_sweep.sh)
// 16.4 -> 8.4 us at [8, 64x64, 320] and 16.4 -> 5.2 us at [8, 16x16, 1280] against the old
// >= 512-block geometry.  qd_colmax_geom_force: the sweep's override (measurement knob).
static int g_colmax_minblk = 128, g_colmax_maxrpt = 64;
extern "C" int qd_colmax_geom_force(int min_blocks, int max_rows_per_thread) {
  g_colmax_minblk = min_blocks > 0 ? min_blocks : 128;
  g_colmax_maxrpt = max_rows_per_thread > 0 ? max_rows_per_thread : 64;
  return 0;
}

static void colmax_launch(const f16* x, const f16* x2, int c1, int n, long hw, int c, float* amax, hipStream_t st) {
  const int minblk = g_colmax_minblk, maxrpt = g_colmax_maxrpt;
  const int chunks = c / 8;
  const int bx = chunks < 64 ? chunks : 64, by = 256 / bx;
  const int gx = (chunks + bx - 1) / bx;
  long rps = (long)by * maxrpt;
  while (rps > by && (long)gx * n * ((hw + rps - 1) / rps) < minblk) rps /= 2;
  k_colmax_nhwc<<<dim3(gx, n, (unsigned)((hw + rps - 1) / rps)), dim3(bx, by), 0, st>>>(x, x2, c1, (int)hw, c,
                                                                                      (int)rps, amax);
}

// contiguous-row max: one wave per row of length len (NCHW per-(n,c) rows, per-token rows).
__global__ void __launch_bounds__(256) k_rowmax(const f16* __restrict__ x, long rows, int len,
                                                float* __restrict__ amax) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const f16* p = x + row * len;
  float m = 0.f;
  if ((len & 7) == 0 && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
    for (int i = lane * 8; i < len; i += 512) {
      f16x8 v = *reinterpret_cast<const f16x8*>(p + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)v[j]));
    }
  } else {
    for (int i = lane; i < len; i += 64) m = fmaxf(m, fabsf((float)p[i]));
  }
  m = wave_max(m);
  if (lane == 0) amax[row] = m;
}

// global max |x| (per-tensor); one atomic per block.
__global__ void __launch_bounds__(256) k_tensormax(const f16* __restrict__ x, long count,
                                                   float* __restrict__ amax) {
  __shared__ float red[4];
  float m = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < count; i += (long)gridDim.x * 256)
    m = fmaxf(m, fabsf((float)x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// per (n, c, g x g patch) max, NCHW.  one thread per patch.
__global__ void k_patchmax(const f16* __restrict__ x, int nc, int h, int w, int g,
                           float* __restrict__ amax) {
  const int gh = h / g, gw = w / g;
  const long pid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pid >= (long)nc * gh * gw) return;
  const int pw = pid % gw;
  const int ph = (pid / gw) % gh;
  const long ch = pid / ((long)gw * gh);
  const f16* base = x + ch * h * w + (long)ph * g * w + (long)pw * g;
  float m = 0.f;
  for (int i = 0; i < g; ++i)
    for (int j = 0; j < g; ++j) m = fmaxf(m, fabsf((float)base[(long)i * w + j]));
  amax[pid] = m;
}

// ---------------------------------------------------------------------------------------
// apply passes
// ---------------------------------------------------------------------------------------

// NHWC per-channel apply: 8 channels per thread (c % 8 == 0).
// channel-chunk x rows geometry (as the GroupNorm passes): thread (tx, ty) owns the 8-channel
// chunk blockIdx.x * bx + tx of sample blockIdx.y, rows ty, ty + by, ... of row range blockIdx.z;
// the per-channel fake-quant scales (and their f64 reciprocals) are computed once per thread.
struct CrGeom {
  int bx, by, gx, z, rpb;
};
static CrGeom cr_geom(int n, long hw, int c) {
  CrGeom g;
  const int chunks = c / 8;
  g.bx = chunks < 256 ? chunks : 256;
  g.by = 256 / g.bx;
  g.gx = (chunks + g.bx - 1) / g.bx;
  // >= 4 rows per thread: the per-thread fake-quant scale setup (two amax loads, 8 f64
  // reciprocals) is amortised over 4 rows, as in the GroupNorm apply (profiles/r03z_*)
  g.rpb = g.by * 4;
  while ((long)g.gx * n * ((hw + g.rpb - 1) / g.rpb) > 8192) g.rpb *= 2;
  g.z = (int)((hw + g.rpb - 1) / g.rpb);
  return g;
}

__global__ void __launch_bounds__(256) k_apply_nhwc(const f16* __restrict__ x, const f16* __restrict__ x2, int c1,
                                                    f16* __restrict__ y, int hw, int c, int c_valid, int qmax,
                                                    int rows_per_block, const float* __restrict__ amax) {
  const int chunk = blockIdx.x * blockDim.x + threadIdx.x;
  if (chunk * 8 >= c) return;
  const int ch = chunk * 8;
  const bool first = x2 == nullptr || ch < c1;
  const int ld = x2 == nullptr ? c : (first ? c1 : c - c1);
  const f16* src = first ? x + ch : x2 + (ch - c1);
  const long n = blockIdx.y;
  const int r0 = blockIdx.z * rows_per_block, r1 = min(hw, r0 + rows_per_block);
  float sc[8];
  double rs[8];
  fq_scales8(amax + n * c + ch, qmax, sc, rs);
  const int by = blockDim.y;
  for (int rb = r0 + threadIdx.y; rb < r1; rb += 4 * by) {
    f16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f16x8*>(src + (n * hw + min(rb + u * by, r1 - 1)) * ld);
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + u * by >= r1) break;
      f16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = ch + j < c_valid ? fq_apply_r((float)v[u][j], sc[j], rs[j]) : v[u][j];
      *reinterpret_cast<f16x8*>(y + (n * hw + rb + u * by) * c + ch) = o;
    }
  }
}

// generic apply with a scale index computed per element:
//   mode 0: idx = e / div            (NCHW per-channel: div = hw; per-token: div = cols)
//   mode 1: idx = 0                  (per-tensor)
//   mode 2: NCHW g x g patches       (per-group)
__global__ void __launch_bounds__(256) k_apply_generic(const f16* __restrict__ x, f16* __restrict__ y,
                                                       long count, int mode, long div, int h,
                                                       int w, int g, int qmax,
                                                       const float* __restrict__ amax) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  long idx;
  if (mode == 0) {
    idx = e / div;
  } else if (mode == 1) {
    idx = 0;
  } else {
    const int ww = e % w;
    const int hh = (e / w) % h;
    const long ch = e / ((long)w * h);
    idx = (ch * (h / g) + hh / g) * (w / g) + ww / g;
  }
  y[e] = fq_apply((float)x[e], fq_scale(amax[idx], qmax));
}

// per-token in one kernel: wave per row, amax then apply (row re-read hits L1/L2).
__global__ void __launch_bounds__(256) k_per_token(const f16* __restrict__ x, f16* __restrict__ y,
                                                   long rows, int cols, int qmax) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const f16* p = x + row * cols;
  f16* q = y + row * cols;
  float m = 0.f;
  for (int i = lane; i < cols; i += 64) m = fmaxf(m, fabsf((float)p[i]));
  m = wave_max(m);
  const float s = fq_scale(m, qmax);
  for (int i = lane; i < cols; i += 64) q[i] = fq_apply((float)p[i], s);
}

static int grid1(long count, int per_block = 256) { return (int)((count + per_block - 1) / per_block); }

static int launch_absmax(const void* x, int layout, int n, int c, int h, int w, int gran, int group,
                         float* amax, hipStream_t st) {
  const long hw = (long)h * w;
  const bool zeroed = (gran & QD_GRAN_ZEROED) != 0;
  gran &= ~QD_GRAN_ZEROED;
  if (gran == QD_GRAN_PER_CHANNEL) {
    if (!zeroed) qd_zero_f32(amax, (size_t)n * c, st);
    if (layout == QD_LAYOUT_NHWC) {
      QD_REQUIRE(c % 8 == 0, "per_channel NHWC needs C % 8 == 0");
      colmax_launch((const f16*)x, nullptr, c, n, hw, c, amax, st);
    } else {
      const long rows = (long)n * c;
      k_rowmax<<<grid1(rows, 4), 256, 0, st>>>((const f16*)x, rows, (int)hw, amax);
    }
  } else if (gran == QD_GRAN_PER_TOKEN) {
    const long rows = (long)n * hw;  // rows of length c (caller passes h = w = 1 normally)
    k_rowmax<<<grid1(rows, 4), 256, 0, st>>>((const f16*)x, rows, c, amax);
  } else if (gran == QD_GRAN_PER_TENSOR) {
    if (!zeroed) qd_zero_f32(amax, 1, st);
    const long count = (long)n * c * hw;
    k_tensormax<<<(int)std::min<long>(2048, grid1(count)), 256, 0, st>>>((const f16*)x, count, amax);
  } else if (gran == QD_GRAN_PER_GROUP) {
    QD_REQUIRE(layout == QD_LAYOUT_NCHW, "per_group needs NCHW");
    QD_REQUIRE(group > 0 && h % group == 0 && w % group == 0, "per_group: group must divide H and W");
    const long patches = (long)n * c * (h / group) * (w / group);
    k_patchmax<<<grid1(patches), 256, 0, st>>>((const f16*)x, n * c, h, w, group, amax);
  } else {
    return qd_set_error(QD_ERR_ARG, "unknown granularity");
  }
  QD_CHECK_LAUNCH();
  return 0;
}

static int launch_apply(const void* x, void* y, int layout, int n, int c, int h, int w, int gran,
                        int group, int bits, const float* amax, hipStream_t st) {
  QD_REQUIRE(bits >= 2 && bits <= 16, "n_bits must be in [2, 16]");
  const int qm = qmax_of(bits);
  const long hw = (long)h * w;
  const long count = (long)n * c * hw;
  if (count == 0) return 0;
  if (gran == QD_GRAN_PER_CHANNEL && layout == QD_LAYOUT_NHWC) {
    QD_REQUIRE(c % 8 == 0, "per_channel NHWC needs C % 8 == 0");
    const int c_valid = group > 0 ? std::min(group, c) : c;
    const CrGeom g = cr_geom(n, hw, c);
    k_apply_nhwc<<<dim3(g.gx, n, g.z), dim3(g.bx, g.by), 0, st>>>((const f16*)x, nullptr, c, (f16*)y, (int)hw, c,
                                                                   c_valid, qm, g.rpb, amax);
  } else if (gran == QD_GRAN_PER_CHANNEL) {
    k_apply_generic<<<grid1(count), 256, 0, st>>>((const f16*)x, (f16*)y, count, 0, hw, h, w, 1, qm, amax);
  } else if (gran == QD_GRAN_PER_TOKEN) {
    k_apply_generic<<<grid1(count), 256, 0, st>>>((const f16*)x, (f16*)y, count, 0, c, h, w, 1, qm, amax);
  } else if (gran == QD_GRAN_PER_TENSOR) {
    k_apply_generic<<<grid1(count), 256, 0, st>>>((const f16*)x, (f16*)y, count, 1, 1, h, w, 1, qm, amax);
  } else if (gran == QD_GRAN_PER_GROUP) {
    QD_REQUIRE(layout == QD_LAYOUT_NCHW, "per_group needs NCHW");
    QD_REQUIRE(group > 0 && h % group == 0 && w % group == 0, "per_group: group must divide H and W");
    k_apply_generic<<<grid1(count), 256, 0, st>>>((const f16*)x, (f16*)y, count, 2, 1, h, w, group, qm, amax);
  } else {
    return qd_set_error(QD_ERR_ARG, "unknown granularity");
  }
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_act_absmax(const void* x, int layout, int n, int c, int h, int w, int gran,
                             int group, float* amax, void* stream) {
  QD_REQUIRE(x && amax, "null pointer");
  QD_REQUIRE(n >= 0 && c >= 0 && h >= 0 && w >= 0, "negative shape");
  if ((long)n * c * h * w == 0) return 0;
  return launch_absmax(x, layout, n, c, h, w, gran, group, amax, S(stream));
}

extern "C" int qd_act_apply(const void* x, void* y, int layout, int n, int c, int h, int w, int gran,
                            int group, int n_bits, const float* amax, void* stream) {
  QD_REQUIRE(x && y && amax, "null pointer");
  return launch_apply(x, y, layout, n, c, h, w, gran, group, n_bits, amax, S(stream));
}

extern "C" int qd_act_fakequant(const void* x, void* y, int layout, int n, int c, int h, int w,
                                int gran, int group, int n_bits, float* amax_ws, void* stream) {
  QD_REQUIRE(x && y, "null pointer");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "n_bits must be in [2, 16]");
  QD_REQUIRE(n >= 0 && c >= 0 && h >= 0 && w >= 0, "negative shape");
  if ((long)n * c * h * w == 0) return 0;
  hipStream_t st = S(stream);
  if (gran == QD_GRAN_PER_TOKEN) {
    const long rows = (long)n * h * w;
    k_per_token<<<grid1(rows, 4), 256, 0, st>>>((const f16*)x, (f16*)y, rows, c, qmax_of(n_bits));
    QD_CHECK_LAUNCH();
    return 0;
  }
  QD_REQUIRE(amax_ws, "amax workspace required");
  int rc = launch_absmax(x, layout, n, c, h, w, gran, group, amax_ws, st);
  if (rc) return rc;
  return launch_apply(x, y, layout, n, c, h, w, gran, group, n_bits, amax_ws, st);
}

// ---------------------------------------------------------------------------------------
// weight quantization (offline)
// ---------------------------------------------------------------------------------------

// one wave per group of g consecutive elements
__global__ void __launch_bounds__(256) k_weight_group(const f16* __restrict__ w, long groups, int g,
                                                      int qmax, int8_t* __restrict__ codes,
                                                      f16* __restrict__ scales, f16* __restrict__ wdq) {
  const long gid = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gid >= groups) return;
  const f16* p = w + gid * g;
  float m = 0.f;
  for (int i = lane; i < g; i += 64) m = fmaxf(m, fabsf((float)p[i]));
  m = wave_max(m);
  const float s = fq_scale(m, qmax);
  if (scales && lane == 0) scales[gid] = (f16)s;
  for (int i = lane; i < g; i += 64) {
    const f16 t = (f16)((float)p[i] / s);
    const float q = __builtin_rintf((float)t);
    if (codes) codes[gid * g + i] = (int8_t)q;
    if (wdq) wdq[gid * g + i] = (f16)(q * s);
  }
}

// per-tensor (single huge group): amax from a separate reduction
__global__ void __launch_bounds__(256) k_weight_tensor_apply(const f16* __restrict__ w, long count,
                                                             int qmax, const float* __restrict__ amax,
                                                             int8_t* __restrict__ codes,
                                                             f16* __restrict__ scales,
                                                             f16* __restrict__ wdq) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const float s = fq_scale(amax[0], qmax);
  if (e == 0 && scales) scales[0] = (f16)s;
  if (e >= count) return;
  const f16 t = (f16)((float)w[e] / s);
  const float q = __builtin_rintf((float)t);
  if (codes) codes[e] = (int8_t)q;
  if (wdq) wdq[e] = (f16)(q * s);
}

extern "C" int qd_weight_quant(const void* w, int rows, int cols, int group, int n_bits,
                               int8_t* codes, void* scales, void* w_dq, void* stream) {
  QD_REQUIRE(w, "null weight");
  // the reference's quantize_weight_* accept any width (fake_quant.py:21-105); integer codes
  // exist only up to 8 bits, wider widths produce the dequantized fp16 weight only
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "weight n_bits must be in [2, 16]");
  QD_REQUIRE(n_bits <= 8 || !codes, "integer codes need n_bits <= 8 (pass codes = NULL for wider widths)");
  QD_REQUIRE(rows >= 0 && cols > 0 && group > 0, "bad shape");
  const long count = (long)rows * cols;
  if (count == 0) return 0;
  hipStream_t st = S(stream);
  if (group >= (1 << 16) || (long)group > cols) {
    QD_REQUIRE((long)group == count, "a group longer than a row must be the whole tensor");
    // per-tensor: reduce then apply.  amax workspace = first 4 bytes of a small buffer
    float* ws = nullptr;
    hipError_t e = hipMallocAsync((void**)&ws, sizeof(float), st);
    if (e != hipSuccess) return qd_set_error((int)e, "workspace alloc");
    qd_zero_f32(ws, 1, st);
    k_tensormax<<<(int)std::min<long>(2048, grid1(count)), 256, 0, st>>>((const f16*)w, count, ws);
    k_weight_tensor_apply<<<grid1(count), 256, 0, st>>>((const f16*)w, count, qmax_of(n_bits), ws,
                                                        codes, (f16*)scales, (f16*)w_dq);
    (void)hipFreeAsync(ws, st);
    QD_CHECK_LAUNCH();
    return 0;
  }
  QD_REQUIRE(cols % group == 0, "group must divide cols (apply the shrink rule on the host)");
  const long groups = count / group;
  k_weight_group<<<grid1(groups, 4), 256, 0, st>>>((const f16*)w, groups, group, qmax_of(n_bits),
                                                   codes, (f16*)scales, (f16*)w_dq);
  QD_CHECK_LAUNCH();
  return 0;
}

// Packed int4 GEMM operand: per 8-code word (k = 8i .. 8i + 7, one little-endian dword) nibble j
// holds c(8i + 2j) and nibble j + 4 holds c(8i + 2j + 1), j = 0..3, with c = q + 8 (offset binary).
// Then ((w >> 4j) & 0x000F000F) | 0x64006400 is the fp16 pair (1024 + c(2j), 1024 + c(2j + 1)):
// two codes in k order per 2 VALU, the MFMA fragment's own element order.
__global__ void k_pack_int4(const int8_t* __restrict__ codes, long words, uint32_t* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= words) return;
  const int8_t* c = codes + 8 * i;
  uint32_t w = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w |= (uint32_t)((c[2 * j] + 8) & 0xF) << (4 * j);
    w |= (uint32_t)((c[2 * j + 1] + 8) & 0xF) << (4 * j + 16);
  }
  out[i] = w;
}

extern "C" int qd_pack_int4(const int8_t* codes, int rows, int cols, uint8_t* packed, void* stream) {
  QD_REQUIRE(codes && packed, "null pointer");
  QD_REQUIRE(cols % 8 == 0, "int4 packing needs cols % 8 == 0");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(packed) & 3) == 0, "packed int4 buffer must be 4-B aligned");
  const long words = (long)rows * cols / 8;
  if (words == 0) return 0;
  k_pack_int4<<<grid1(words), 256, 0, S(stream)>>>(codes, words, reinterpret_cast<uint32_t*>(packed));
  QD_CHECK_LAUNCH();
  return 0;
}

__global__ void k_conv_w_khwc(const f16* __restrict__ w, int co, int ci, int kh, int kw, int cip,
                              f16* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)co * kh * kw * cip;
  if (e >= total) return;
  const int c = e % cip;
  const int x = (e / cip) % kw;
  const int y = (e / ((long)cip * kw)) % kh;
  const long o = e / ((long)cip * kw * kh);
  out[e] = c < ci ? w[((o * ci + c) * kh + y) * kw + x] : (f16)0.f;
}

extern "C" int qd_conv_weight_khwc(const void* w, int co, int ci, int kh, int kw, int ci_pad,
                                   void* out, void* stream) {
  QD_REQUIRE(w && out, "null pointer");
  QD_REQUIRE(ci_pad >= ci, "ci_pad < ci");
  const long total = (long)co * kh * kw * ci_pad;
  if (total == 0) return 0;
  k_conv_w_khwc<<<grid1(total), 256, 0, S(stream)>>>((const f16*)w, co, ci, kh, kw, ci_pad, (f16*)out);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// conv-output finalize: out = half(fq(y) + residual | + chan_add[n][c])
// ---------------------------------------------------------------------------------------
// Q / RES / CADD: the output fake-quant, the residual add and the per-(n, c) add as compile-time flags
// (the host maps qmax > 0 / res / cadd onto them): no per-element uniform branch, so the 8 channels'
// conversion chains interleave (as k_gn_stats<XF, F>).  RES and CADD exclude each other.
template <bool Q, bool RES, bool CADD>
__global__ void __launch_bounds__(256) k_finalize(const f16* __restrict__ y, const float* __restrict__ amax,
                                                  int hw, int c, int qmax, int rows_per_block,
                                                  const f16* __restrict__ res,
                                                  const f16* __restrict__ cadd, int cadd_ld,
                                                  f16* __restrict__ out) {
  const int chunk = blockIdx.x * blockDim.x + threadIdx.x;
  if (chunk * 8 >= c) return;
  const int ch = chunk * 8;
  const long n = blockIdx.y;
  const int r0 = blockIdx.z * rows_per_block, r1 = min(hw, r0 + rows_per_block);
  float sc[8];
  double rs[8];
  f16x8 ca = {};
  if constexpr (CADD) ca = *reinterpret_cast<const f16x8*>(cadd + n * cadd_ld + ch);
  if constexpr (Q) fq_scales8(amax + n * c + ch, qmax, sc, rs);
  const int by = blockDim.y;
  for (int rb = r0 + threadIdx.y; rb < r1; rb += 4 * by) {
    f16x8 v[4], rr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long e = (n * hw + min(rb + u * by, r1 - 1)) * c + ch;
      v[u] = *reinterpret_cast<const f16x8*>(y + e);
      if constexpr (RES) rr[u] = *reinterpret_cast<const f16x8*>(res + e);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      QD_PIN(v[u]);
      if constexpr (RES) QD_PIN(rr[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb + u * by >= r1) break;
      const long e = (n * hw + rb + u * by) * c + ch;
      f16x8 o = v[u];
      if constexpr (Q) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fq_apply_r((float)v[u][j], sc[j], rs[j]);
      }
      if constexpr (RES) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (f16)((float)o[j] + (float)rr[u][j]);
      } else if constexpr (CADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (f16)((float)o[j] + (float)ca[j]);
      }
      *reinterpret_cast<f16x8*>(out + e) = o;
    }
  }
}

extern "C" int qd_fq_finalize(const void* y, const float* amax, int n, int hw, int c, int n_bits,
                              const void* residual, const void* chan_add, int chan_add_ld, void* out,
                              void* stream) {
  QD_REQUIRE(y && out, "null pointer");
  if (chan_add_ld <= 0) chan_add_ld = c;
  QD_REQUIRE(!chan_add || (chan_add_ld >= c && chan_add_ld % 8 == 0 && (reinterpret_cast<uintptr_t>(chan_add) & 15) == 0),
             "chan_add: 16-B aligned rows, ld >= c, ld % 8 == 0");
  QD_REQUIRE(c % 8 == 0, "finalize needs C % 8 == 0");
  QD_REQUIRE(n_bits == 0 || (amax && n_bits >= 2 && n_bits <= 16), "bad n_bits / amax");
  if ((long)n * hw * c == 0) return 0;
  const CrGeom g = cr_geom(n, hw, c);
  const dim3 gr(g.gx, n, g.z), bl(g.bx, g.by);
  const int qm = n_bits ? qmax_of(n_bits) : 0;
#define QD_FIN(QV, RV, CV)                                                                                    \
  k_finalize<QV, RV, CV><<<gr, bl, 0, S(stream)>>>((const f16*)y, amax, hw, c, qm, g.rpb, (const f16*)residual, \
                                                   (const f16*)chan_add, chan_add_ld, (f16*)out)
  const bool q = qm > 0;
  if (residual) {  // (a residual takes precedence over chan_add, as before)
    if (q) QD_FIN(true, true, false);
    else QD_FIN(false, true, false);
  } else if (chan_add) {
    if (q) QD_FIN(true, false, true);
    else QD_FIN(false, false, true);
  } else {
    if (q) QD_FIN(true, false, false);
    else QD_FIN(false, false, false);
  }
#undef QD_FIN
  QD_CHECK_LAUNCH();
  return 0;
}

// Self-test of the fq_apply_r / rcp_exact shortcut against the IEEE division form fq_apply:
// every non-negative finite fp16 scale s, and for each s the fp16 values x next to every
// quantization midpoint (k + 1/2) s, |k| <= 130, plus the midpoint images themselves.
// counts[0] = scales whose rcp_exact differs from 1 / (double)s by more than 1 f64 ulp,
// counts[1] = (s, x) pairs whose fake-quant results differ, counts[2] = (s, x) pairs over ALL
// finite fp16 x whose f16 quotients differ.  Test infrastructure only.
__global__ void k_selftest_recip(int* counts) {
  const unsigned short sb = (unsigned short)(blockIdx.x);
  const f16 sh = __builtin_bit_cast(f16, sb);
  const float s = (float)sh;
  if ((sb & 0x8000u) || __builtin_isnan(s) || __builtin_isinf(s)) return;  // scales are >= +0 (fq_scale)
  const double r = rcp_exact(s), e = 1.0 / (double)s;
  if (threadIdx.x == 0 && s > 0.f) {
    const double ulp = __builtin_fabs(e) * 2.220446049250313e-16;
    if (__builtin_fabs(r - e) > ulp) atomicAdd(&counts[0], 1);
  }
  int bad = 0;
  for (int k = (int)threadIdx.x - 130; k <= 130; k += blockDim.x) {
    const f16 mid = (f16)(((float)k + 0.5f) * s);
    const unsigned short mb = __builtin_bit_cast(unsigned short, mid);
    for (int dlt = -2; dlt <= 2; ++dlt) {
      const f16 x = __builtin_bit_cast(f16, (unsigned short)(mb + dlt));
      const float xf = (float)x;
      if (__builtin_isnan(xf) || __builtin_isinf(xf)) continue;
      const f16 a = fq_apply(xf, s), b = fq_apply_r(xf, s, r);
      if (__builtin_bit_cast(unsigned short, a) != __builtin_bit_cast(unsigned short, b) &&
          !(__builtin_isnan((float)a) && __builtin_isnan((float)b)))
        ++bad;
    }
  }
  if (bad) atomicAdd(&counts[1], bad);
  // every finite fp16 x: the f16 quotient of the shortcut == half(IEEE f32 x / s)
  int badq = 0;
  for (int xb = threadIdx.x; xb < 65536; xb += blockDim.x) {
    const float xf = (float)__builtin_bit_cast(f16, (unsigned short)xb);
    if (__builtin_isnan(xf) || __builtin_isinf(xf)) continue;
    const f16 a = (f16)(xf / s), b = (f16)(float)((double)xf * r);
    if (__builtin_bit_cast(unsigned short, a) != __builtin_bit_cast(unsigned short, b) &&
        !(__builtin_isnan((float)a) && __builtin_isnan((float)b)))
      ++badq;
  }
  if (badq) atomicAdd(&counts[2], badq);
}

extern "C" int qd_selftest_recip(int* counts, void* stream) {
  QD_REQUIRE(counts, "null pointer");
  hipStream_t st = S(stream);
  qd_zero_f32(reinterpret_cast<float*>(counts), 3, st);  // int 0 == f32 +0 bits
  k_selftest_recip<<<65536, 64, 0, st>>>(counts);
  QD_CHECK_LAUNCH();
  return 0;
}

// Per-(n, c) fake-quant of the channel concat [x | x2] (NHWC), written as one tensor: the
// UNet skip concat feeding a quantized conv_shortcut, materialised only in quantized form.
extern "C" int qd_act_quant_cat_nhwc(const void* x, int c1, const void* x2, int c2, int n, int hw, int n_bits,
                                     float* amax, int amax_zeroed, void* y, void* stream) {
  QD_REQUIRE(x && x2 && y && amax, "null pointer");
  QD_REQUIRE(c1 % 8 == 0 && c2 % 8 == 0 && c1 > 0 && c2 > 0, "concat widths must be multiples of 8");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "bad n_bits");
  const int c = c1 + c2;
  if ((long)n * hw == 0) return 0;
  hipStream_t st = S(stream);
  if (!amax_zeroed) qd_zero_f32(amax, (size_t)n * c, st);
  colmax_launch((const f16*)x, (const f16*)x2, c1, n, hw, c, amax, st);
  const CrGeom g = cr_geom(n, hw, c);
  k_apply_nhwc<<<dim3(g.gx, n, g.z), dim3(g.bx, g.by), 0, st>>>((const f16*)x, (const f16*)x2, c1, (f16*)y, hw, c,
                                                                 c, qmax_of(n_bits), g.rpb, amax);
  QD_CHECK_LAUNCH();
  return 0;
}

// quantize_activation_per_channel_absmax (fake_quant.py:123-131) of a SMALL NHWC tensor in one launch:
// one 1024-thread block per sample holds the sample in registers (<= 4 rows of 8 channels per thread),
// reduces the per-channel max in LDS (fixed tree, exact) and applies the fake-quant from the same
// registers.  The UNet's conv_in input (the [2B, 64, 64, 8] latent) took a column-max pass (13.6 us:
// 16-deep atomic chains per channel at 4096 rows x 1 chunk) + an apply pass (5.4 us).  Same bits as the
// two passes (max is exact; fq_scale / fq_apply_r as k_apply_nhwc).  chunks = c / 8 a power of two.
constexpr int FQS_T = 1024, FQS_RPT = 4;
__global__ void __launch_bounds__(FQS_T) k_fq_small_nhwc(const f16* __restrict__ x, f16* __restrict__ y, int hw, int c,
                                                         int c_valid, int qmax) {
  __shared__ __attribute__((aligned(16))) float red[FQS_T][8];
  const int chunks = c >> 3, t = threadIdx.x;
  const int chunk = t & (chunks - 1), rl = t / chunks, rstride = FQS_T / chunks;
  const long n = blockIdx.x;
  const f16* src = x + n * hw * c + chunk * 8;
  f16x8 v[FQS_RPT];
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = 0.f;
#pragma unroll
  for (int u = 0; u < FQS_RPT; ++u) {
    const int row = rl + u * rstride;
    v[u] = row < hw ? *reinterpret_cast<const f16x8*>(src + (long)row * c) : f16x8{};
  }
#pragma unroll
  for (int u = 0; u < FQS_RPT; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf((float)v[u][j]));
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t][j] = m[j];
  __syncthreads();
  for (int s = rstride >> 1; s >= 1; s >>= 1) {  // rows rl, rl + s of the same chunk
    if (rl < s)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[t][j] = fmaxf(red[t][j], red[t + s * chunks][j]);
    __syncthreads();
  }
  float sc[8];
  double rs[8];
  fq_scales8(&red[chunk][0], qmax, sc, rs);
  f16* dst = y + n * hw * c + chunk * 8;
#pragma unroll
  for (int u = 0; u < FQS_RPT; ++u) {
    const int row = rl + u * rstride;
    if (row >= hw) break;
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = chunk * 8 + j < c_valid ? fq_apply_r((float)v[u][j], sc[j], rs[j]) : v[u][j];
    *reinterpret_cast<f16x8*>(dst + (long)row * c) = o;
  }
}

extern "C" int qd_act_fq_small_ok(int hw, int c) {
  const int chunks = c / 8;
  return (c % 8 == 0 && chunks >= 1 && chunks <= FQS_T && (chunks & (chunks - 1)) == 0 &&
          (long)hw * chunks <= (long)FQS_T * FQS_RPT && hw > 0) ? 1 : 0;
}

extern "C" int qd_act_fq_small_nhwc(const void* x, void* y, int n, int hw, int c, int c_valid, int n_bits,
                                    void* stream) {
  QD_REQUIRE(x && y, "null pointer");
  QD_REQUIRE(qd_act_fq_small_ok(hw, c), "qd_act_fq_small_nhwc: c / 8 a power of two, hw * c / 8 <= 4096 (qd_act_fq_small_ok)");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "bad n_bits");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0,
             "x / y must be 16-B aligned");
  if (n == 0) return 0;
  k_fq_small_nhwc<<<n, FQS_T, 0, S(stream)>>>((const f16*)x, (f16*)y, hw, c, c_valid > 0 ? c_valid : c,
                                            qmax_of(n_bits));
  QD_CHECK_LAUNCH();
  return 0;
}

// qd_act_quant_cat_nhwc's apply pass with the per-(n, c) maxima of [x | x2] given (amax [n][c1 + c2],
// e.g. from qd_groupnorm_xamax over the same concat): no column-max pass
extern "C" int qd_act_apply_cat_nhwc(const void* x, int c1, const void* x2, int c2, int n, int hw, int n_bits,
                                     const float* amax, void* y, void* stream) {
  QD_REQUIRE(x && x2 && y && amax, "null pointer");
  QD_REQUIRE(c1 % 8 == 0 && c2 % 8 == 0 && c1 > 0 && c2 > 0, "concat widths must be multiples of 8");
  QD_REQUIRE(n_bits >= 2 && n_bits <= 16, "bad n_bits");
  const int c = c1 + c2;
  if ((long)n * hw == 0) return 0;
  const CrGeom g = cr_geom(n, hw, c);
  k_apply_nhwc<<<dim3(g.gx, n, g.z), dim3(g.bx, g.by), 0, S(stream)>>>((const f16*)x, (const f16*)x2, c1, (f16*)y,
                                                                        hw, c, c, qmax_of(n_bits), g.rpb, amax);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// SmoothQuant calibration + fold
// ---------------------------------------------------------------------------------------
__global__ void k_accum_sum(const float* __restrict__ amax, int c, float* __restrict__ sum,
                            f16* __restrict__ amax_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= c) return;
  if (sum) sum[i] += amax[i];
  if (amax_out) amax_out[i] = (f16)amax[i];
}

extern "C" int qd_channel_absmax_accum(const void* x, int64_t rows, int c, float* amax_ws, float* sum,
                                       void* amax_out, void* stream) {
  QD_REQUIRE(x && amax_ws, "null pointer");
  QD_REQUIRE(c % 8 == 0, "channel absmax needs C % 8 == 0");
  QD_REQUIRE(rows > 0 && rows < (1L << 31), "bad rows");
  hipStream_t st = S(stream);
  int rc = launch_absmax(x, QD_LAYOUT_NHWC, 1, c, (int)rows, 1, QD_GRAN_PER_CHANNEL, 0, amax_ws, st);
  if (rc) return rc;
  k_accum_sum<<<grid1(c), 256, 0, st>>>(amax_ws, c, sum, (f16*)amax_out);
  QD_CHECK_LAUNCH();
  return 0;
}

// column |W| max of a [rows][c] fp16 matrix into wmax (atomic), c % 8 == 0 not required.
__global__ void k_colabsmax(const f16* __restrict__ w, int rows, int c, float* __restrict__ wmax) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= c) return;
  const int r0 = blockIdx.y * 64, r1 = min(rows, r0 + 64);
  float m = 0.f;
  for (int r = r0; r < r1; ++r) m = fmaxf(m, fabsf((float)w[(long)r * c + col]));
  atomic_max_pos(&wmax[col], m);
}

__global__ void k_smooth_scales(const float* __restrict__ wmax, const f16* __restrict__ act, int c,
                                float ea, float eb, f16* __restrict__ scales, f16* __restrict__ lnw,
                                f16* __restrict__ lnb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= c) return;
  const float cl = clamp_min_f16();
  const float ws = fmaxf(wmax[i], cl);  // exact fp16 value
  // pow in f64, rounded to f32 then fp16: torch's Half pow(Scalar) result on these inputs
  // (oracle/fake_quant_np.py smooth_scales, pinned to the reference's smooth_ln_fcs golden);
  // an f32 powf differs from it by 1 fp16 ulp on a few channels
  const f16 num = (f16)(float)pow((double)(float)act[i], (double)ea);
  const f16 den = (f16)(float)pow((double)ws, (double)eb);
  const float s = fmaxf((float)(f16)((float)num / (float)den), cl);
  scales[i] = (f16)s;
  lnw[i] = (f16)((float)lnw[i] / s);
  if (lnb) lnb[i] = (f16)((float)lnb[i] / s);
}

__global__ void k_scale_cols(f16* __restrict__ w, long count, int c, const f16* __restrict__ s) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  w[e] = (f16)((float)w[e] * (float)s[e % c]);
}

extern "C" int qd_smooth_fold(void* ln_w, void* ln_b, void* const* fc_w, const int* fc_rows, int nfc,
                              int c, const void* act_mean, float alpha, float* wmax_ws,
                              void* scales_out, void* stream) {
  QD_REQUIRE(ln_w && fc_w && fc_rows && act_mean && wmax_ws && scales_out, "null pointer");
  QD_REQUIRE(nfc > 0 && c > 0, "bad shape");
  hipStream_t st = S(stream);
  qd_zero_f32(wmax_ws, (size_t)c, st);
  for (int i = 0; i < nfc; ++i) {
    QD_REQUIRE(fc_w[i] && fc_rows[i] > 0, "bad fc");
    dim3 grid((c + 255) / 256, (fc_rows[i] + 63) / 64);
    k_colabsmax<<<grid, 256, 0, st>>>((const f16*)fc_w[i], fc_rows[i], c, wmax_ws);
  }
  // exponents are rounded to fp16 first, as torch's Half pow(Scalar) does (oracle note)
  const float ea = (float)(f16)alpha;
  const float eb = (float)(f16)(1.0f - alpha);
  k_smooth_scales<<<grid1(c), 256, 0, st>>>(wmax_ws, (const f16*)act_mean, c, ea, eb, (f16*)scales_out,
                                            (f16*)ln_w, (f16*)ln_b);
  for (int i = 0; i < nfc; ++i) {
    const long count = (long)fc_rows[i] * c;
    k_scale_cols<<<grid1(count), 256, 0, st>>>((f16*)fc_w[i], count, c, (const f16*)scales_out);
  }
  QD_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// int8 activation codes for the int8-MFMA W8A8 mode (qd_linear_i8 / qd_conv2d_i8)
// ---------------------------------------------------------------------------------------
// The reference's RTN recipe (fake_quant.py:108-131), keeping the integer instead of the
// dequantized value: s = half(half(max(amax, 1e-5)) / 127), q = rint(half(x / s)); the scale is
// stored widened to fp32 for the GEMM epilogue.  |q| <= 127 by construction.
__device__ __forceinline__ int8_t q_i8(float x, float s, double rs) {
  const f16 t = (f16)(float)((double)x * rs);  // == (f16)(x / s), fq_apply_r argument (common.h)
  return (int8_t)__builtin_rintf((float)t);
}

// per row (dynamic per-token): one wave per row, R rows per wave, the row held in registers
// (PER 16-B chunks per lane, all rows' loads issued before any reduction): one HBM read + one
// 1-B/element write, no second pass over the row
template <int PER, int R>
__global__ void __launch_bounds__(256) k_quant_rows_i8(const f16* __restrict__ x, long rows, int c, int ldx,
                                                       int8_t* __restrict__ y, int ldy, float* __restrict__ sa) {
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  const int lane = threadIdx.x & 63;
  const int chunks = c >> 3;
  f16x8 v[R][PER];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = lane + i * 64;
      v[r][i] = (row0 + r < rows && j < chunks) ? *reinterpret_cast<const f16x8*>(x + (row0 + r) * ldx + j * 8)
                                                : (f16x8){};
    }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (row0 + r >= rows) break;
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf((float)v[r][i][e]));
    const float s = fq_scale(wave_max(m), 127);
    const double rs = rcp_exact(s);
    if (lane == 0) sa[row0 + r] = s;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = lane + i * 64;
      if (j < chunks) {
        unsigned lo = 0, hi = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo |= (unsigned)(uint8_t)q_i8((float)v[r][i][e], s, rs) << (8 * e);
          hi |= (unsigned)(uint8_t)q_i8((float)v[r][i][4 + e], s, rs) << (8 * e);
        }
        *reinterpret_cast<uint2*>(y + (row0 + r) * ldy + j * 8) = make_uint2(lo, hi);
      }
    }
  }
}

template <int PER>
static void launch_rows_i8(const f16* x, long rows, int c, int ldx, int8_t* y, int ldy, float* sa, hipStream_t st) {
  int r = std::max(1, 2048 / (c * 2));
  while (r > 1 && (rows + 4L * r - 1) / (4L * r) < 1024) r >>= 1;
  if (r >= 4) k_quant_rows_i8<PER, 4><<<(int)((rows + 15) / 16), 256, 0, st>>>(x, rows, c, ldx, y, ldy, sa);
  else if (r >= 2) k_quant_rows_i8<PER, 2><<<(int)((rows + 7) / 8), 256, 0, st>>>(x, rows, c, ldx, y, ldy, sa);
  else k_quant_rows_i8<PER, 1><<<(int)((rows + 3) / 4), 256, 0, st>>>(x, rows, c, ldx, y, ldy, sa);
}

// grouped rows (every C = 8 * LPR * P, LPR in {8..64} lanes per row, P <= 5 16-B chunks per lane:
// SD's 320 / 640 / 1280 / 2560): a wave holds 64 / LPR rows at once, lane l of a row owning chunks
// l, l + LPR, ... (all 64 lanes carry data; the one-row-per-wave kernel above leaves 24 of 64 idle
// at C 320), IT row groups per wave with every load issued before the first reduction.  The row max
// is order-free, so the codes and scales equal k_quant_rows_i8's bit for bit.
template <int LPR, int P, int IT>
__global__ void __launch_bounds__(256) k_quant_rows_g(const f16* __restrict__ x, long rows, int c, int ldx,
                                                      int8_t* __restrict__ y, int ldy, float* __restrict__ sa) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, lr = lane % LPR, rw = lane / LPR;
  const long wrow0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW * IT;
  f16x8 v[IT][P];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const long row = wrow0 + (long)it * RPW + rw;
#pragma unroll
    for (int i = 0; i < P; ++i)
      v[it][i] = row < rows ? *reinterpret_cast<const f16x8*>(x + row * ldx + (lr + i * LPR) * 8) : (f16x8){};
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const long row = wrow0 + (long)it * RPW + rw;
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < P; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf((float)v[it][i][e]));
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    const float s = fq_scale(m, 127);
    const double rs = rcp_exact(s);
    if (row < rows) {
      if (lr == 0) sa[row] = s;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        unsigned lo = 0, hi = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo |= (unsigned)(uint8_t)q_i8((float)v[it][i][e], s, rs) << (8 * e);
          hi |= (unsigned)(uint8_t)q_i8((float)v[it][i][4 + e], s, rs) << (8 * e);
        }
        *reinterpret_cast<uint2*>(y + row * ldy + (lr + i * LPR) * 8) = make_uint2(lo, hi);
      }
    }
  }
}

static bool launch_rows_g(const f16* x, long rows, int c, int ldx, int8_t* y, int ldy, float* sa, hipStream_t st) {
  const int ch = c / 8;
  int lpr = 0, per = 0;
  for (int l = 8; l <= 64 && !lpr; l *= 2)
    if (ch % l == 0 && ch / l <= 5) {
      lpr = l;
      per = ch / l;
    }
  if (!lpr) return false;
  const long rpw = 64 / lpr;
  // two row groups per wave while the grid keeps >= 1024 blocks
  const bool two = (rows + 4 * rpw * 2 - 1) / (4 * rpw * 2) >= 1024;
  const int grid = (int)((rows + 4 * rpw * (two ? 2 : 1) - 1) / (4 * rpw * (two ? 2 : 1)));
#define QD_QRG(L, PP)                                                                                   \
  if (lpr == L && per == PP) {                                                                          \
    if (two) k_quant_rows_g<L, PP, 2><<<grid, 256, 0, st>>>(x, rows, c, ldx, y, ldy, sa);               \
    else k_quant_rows_g<L, PP, 1><<<grid, 256, 0, st>>>(x, rows, c, ldx, y, ldy, sa);                   \
    return true;                                                                                        \
  }
  QD_QRG(8, 5) QD_QRG(16, 5) QD_QRG(32, 3) QD_QRG(32, 5) QD_QRG(64, 5)
#undef QD_QRG
  return false;
}

extern "C" int qd_quant_rows_i8(const void* x, long rows, int c, int ldx, int8_t* y, int ldy, float* scales,
                                void* stream) {
  QD_REQUIRE(x && y && scales, "null pointer");
  QD_REQUIRE(c % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ldx >= c && ldy >= c, "c, ldx, ldy must be multiples of 8");
  QD_REQUIRE(c <= 8192, "row quantization supports c <= 8192");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0, "alignment");
  if (rows <= 0) return 0;
  const int per = (c / 8 + 63) / 64;
  const f16* xp = (const f16*)x;
  hipStream_t st = S(stream);
  if (launch_rows_g(xp, rows, c, ldx, y, ldy, scales, st)) {
    QD_CHECK_LAUNCH();
    return 0;
  }
  if (per <= 1) launch_rows_i8<1>(xp, rows, c, ldx, y, ldy, scales, st);
  else if (per <= 2) launch_rows_i8<2>(xp, rows, c, ldx, y, ldy, scales, st);
  else if (per <= 4) launch_rows_i8<4>(xp, rows, c, ldx, y, ldy, scales, st);
  else if (per <= 8) launch_rows_i8<8>(xp, rows, c, ldx, y, ldy, scales, st);
  else launch_rows_i8<16>(xp, rows, c, ldx, y, ldy, scales, st);
  QD_CHECK_LAUNCH();
  return 0;
}

// per sample (conv input): amax over the sample's per_sample values, then the codes
__global__ void __launch_bounds__(256) k_sample_absmax(const f16* __restrict__ x, long per_sample,
                                                       float* __restrict__ amax) {
  __shared__ float red[4];
  const long n = blockIdx.y;
  const f16* p = x + n * per_sample;
  float m = 0.f;
  const long stride = (long)gridDim.x * 2048;
  // 4 independent 16-B loads in flight per thread per iteration (clamped, not guarded)
  for (long i0 = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i0 < per_sample; i0 += 4 * stride) {
    f16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f16x8*>(p + min(i0 + u * stride, per_sample - 8));
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)v[u][j]));  // clamped re-reads are harmless for a max
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(amax + n, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// c > 0: amax holds the per-(sample, channel) maxima of x [n][rows][c] (reduced by its producer's
// GEMM epilogue); every block takes the sample's max over them (exact: the same scale as the
// per-sample reduction)
__global__ void __launch_bounds__(256) k_sample_apply_i8(const f16* __restrict__ x, long per_sample,
                                                         const float* __restrict__ amax, int8_t* __restrict__ y,
                                                         float* __restrict__ sa, int c = 0) {
  const long n = blockIdx.y;
  float an;
  if (c > 0) {
    __shared__ float red[4];
    float m = 0.f;
    for (int j = threadIdx.x; j < c; j += 256) m = fmaxf(m, amax[n * c + j]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    an = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  } else {
    an = amax[n];
  }
  const float s = fq_scale(an, 127);
  const double rs = rcp_exact(s);
  if (blockIdx.x == 0 && threadIdx.x == 0) sa[n] = s;
  const f16* p = x + n * per_sample;
  int8_t* q = y + n * per_sample;
  // 4 independent 16-B loads in flight per thread per iteration (clamped, not guarded; the stores
  // are guarded) instead of one dependent load per iteration
  const long stride = (long)gridDim.x * 2048;
  for (long i0 = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i0 < per_sample; i0 += 4 * stride) {
    f16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f16x8*>(p + min(i0 + u * stride, per_sample - 8));
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * stride;
      if (i >= per_sample) break;
      unsigned lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo |= (unsigned)(uint8_t)q_i8((float)v[u][j], s, rs) << (8 * j);
        hi |= (unsigned)(uint8_t)q_i8((float)v[u][4 + j], s, rs) << (8 * j);
      }
      *reinterpret_cast<uint2*>(q + i) = make_uint2(lo, hi);
    }
  }
}

// per-sample codes of the concat x | x2 (8-channel chunks never straddle: c1 % 8 == 0), the sample
// max over amax[n][0..c) - k_sample_apply_i8's arithmetic, one pass, no concat copy
__global__ void __launch_bounds__(256) k_cat_apply_i8(const f16* __restrict__ x, const f16* __restrict__ x2, int c1,
                                                      int c, long rows, const float* __restrict__ amax,
                                                      int8_t* __restrict__ y, float* __restrict__ sa) {
  const long n = blockIdx.y;
  __shared__ float red[4];
  float m = 0.f;
  for (int j = threadIdx.x; j < c; j += 256) m = fmaxf(m, amax[n * c + j]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  const float s = fq_scale(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), 127);
  const double rs = rcp_exact(s);
  if (blockIdx.x == 0 && threadIdx.x == 0) sa[n] = s;
  const int cc = c / 8, c2 = c - c1;
  const long chunks = rows * cc;
  // 4 chunks' loads in flight per thread per iteration (chunk index clamped, stores guarded)
  const long stride = (long)gridDim.x * 256;
  for (long e0 = (long)blockIdx.x * 256 + threadIdx.x; e0 < chunks; e0 += 4 * stride) {
    f16x8 v[4];
    long row[4];
    int chs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long e = min(e0 + u * stride, chunks - 1);
      const long r = e / cc;
      chs[u] = (int)(e - r * cc) * 8;
      row[u] = n * rows + r;
      v[u] = *reinterpret_cast<const f16x8*>(chs[u] < c1 ? x + row[u] * c1 + chs[u] : x2 + row[u] * c2 + (chs[u] - c1));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) QD_PIN(v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + u * stride >= chunks) break;
      unsigned lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo |= (unsigned)(uint8_t)q_i8((float)v[u][j], s, rs) << (8 * j);
        hi |= (unsigned)(uint8_t)q_i8((float)v[u][4 + j], s, rs) << (8 * j);
      }
      *reinterpret_cast<uint2*>(y + row[u] * c + chs[u]) = make_uint2(lo, hi);
    }
  }
}

extern "C" int qd_quant_samples_i8_cat(const void* x, const void* x2, int c1, int c, int n, long rows,
                                       const float* amax_nc, int8_t* y, float* scales, void* stream) {
  QD_REQUIRE(x && x2 && amax_nc && y && scales, "null pointer");
  QD_REQUIRE(c1 > 0 && c1 < c && c1 % 8 == 0 && c % 8 == 0, "concat split: multiples of 8 channels");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(x2) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(y) & 7) == 0,
             "alignment");
  if ((long)n * rows == 0) return 0;
  const long ch = (rows * (c / 8) + 255) / 256;
  const int gx = (int)std::min<long>(std::max<long>(1, 1024 / n), ch);
  k_cat_apply_i8<<<dim3(gx, n), 256, 0, S(stream)>>>((const f16*)x, (const f16*)x2, c1, c, rows, amax_nc, y, scales);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_quant_samples_i8_amax(const void* x, int n, long per_sample, const float* amax_nc, int c,
                                        int8_t* y, float* scales, void* stream) {
  QD_REQUIRE(x && amax_nc && y && scales, "null pointer");
  QD_REQUIRE(c > 0 && per_sample % c == 0 && per_sample % 8 == 0, "per_sample must be rows * c, a multiple of 8");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0, "alignment");
  if ((long)n * per_sample == 0) return 0;
  const long ch = (per_sample / 8 + 255) / 256;  // 2048-element blocks per sample
  const int gx = (int)std::min<long>(std::max<long>(1, 1024 / n), ch);
  k_sample_apply_i8<<<dim3(gx, n), 256, 0, S(stream)>>>((const f16*)x, per_sample, amax_nc, y, scales, c);
  QD_CHECK_LAUNCH();
  return 0;
}

extern "C" int qd_quant_samples_i8(const void* x, int n, long per_sample, int8_t* y, float* scales, float* amax_ws,
                                   int amax_zeroed, void* stream) {
  QD_REQUIRE(x && y && scales && amax_ws, "null pointer");
  QD_REQUIRE(per_sample % 8 == 0, "per-sample size must be a multiple of 8");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0, "alignment");
  if ((long)n * per_sample == 0) return 0;
  hipStream_t st = S(stream);
  if (!amax_zeroed) qd_zero_f32(amax_ws, (size_t)n, st);
  const long ch = (per_sample / 8 + 255) / 256;  // 2048-element blocks per sample
  const int gx = (int)std::min<long>(std::max<long>(1, 1024 / n), ch);
  const int gxa = (int)std::min<long>(std::max<long>(1, 512 / n), (ch + 3) / 4);  // 4 loads per thread
  k_sample_absmax<<<dim3(gxa, n), 256, 0, st>>>((const f16*)x, per_sample, amax_ws);
  k_sample_apply_i8<<<dim3(gx, n), 256, 0, st>>>((const f16*)x, per_sample, amax_ws, y, scales);
  QD_CHECK_LAUNCH();
  return 0;
}

// ---- fp8 (e4m3) activation codes per token (SD3.5's W4A8-fp8 mode) ---------------------------
// s = max(amax, 1e-5) / 448 (f32), code = e4m3(x / s) with round-to-nearest-even (|x / s| <= 448:
// no saturation case); scales fp32 [rows]
template <int PER>
__global__ void __launch_bounds__(256) k_quant_rows_f8(const f16* __restrict__ x, long rows, int c, int ldx,
                                                       uint8_t* __restrict__ y, int ldy, float* __restrict__ sa) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int chunks = c >> 3;
  if (row >= rows) return;
  f16x8 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + i * 64;
    v[i] = j < chunks ? *reinterpret_cast<const f16x8*>(x + row * ldx + j * 8) : (f16x8){};
  }
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf((float)v[i][e]));
  const float s = fmaxf(wave_max(m), 1e-5f) / 448.0f;
  if (lane == 0) sa[row] = s;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int j = lane + i * 64;
    if (j < chunks) {
      unsigned w[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int pk = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[i][4 * h] / s, (float)v[i][4 * h + 1] / s, 0, false);
        pk = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[i][4 * h + 2] / s, (float)v[i][4 * h + 3] / s, pk, true);
        w[h] = (unsigned)pk;
      }
      *reinterpret_cast<uint2*>(y + row * ldy + j * 8) = make_uint2(w[0], w[1]);
    }
  }
}

extern "C" int qd_quant_rows_fp8(const void* x, long rows, int c, int ldx, void* y, int ldy, float* scales,
                                 void* stream) {
  QD_REQUIRE(x && y && scales, "null pointer");
  QD_REQUIRE(c % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ldx >= c && ldy >= c, "c, ldx, ldy must be multiples of 8");
  QD_REQUIRE(c <= 16384, "row quantization supports c <= 16384");
  QD_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 7) == 0, "alignment");
  if (rows <= 0) return 0;
  const int per = (c / 8 + 63) / 64;
  const f16* xp = (const f16*)x;
  uint8_t* yp = (uint8_t*)y;
  const int grid = (int)((rows + 3) / 4);
  hipStream_t st = S(stream);
  if (per <= 1) k_quant_rows_f8<1><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  else if (per <= 2) k_quant_rows_f8<2><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  else if (per <= 4) k_quant_rows_f8<4><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  else if (per <= 8) k_quant_rows_f8<8><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  else if (per <= 16) k_quant_rows_f8<16><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  else k_quant_rows_f8<32><<<grid, 256, 0, st>>>(xp, rows, c, ldx, yp, ldy, scales);
  QD_CHECK_LAUNCH();
  return 0;
}

// W4 codes (int8 [N, K], values -8..7) -> e4m3 bytes (exact: small integers), and the group scales
// fp16 [N, K / g] -> fp32 transposed [K / g][N] (the fp8 GEMM's gs operand)
__global__ void k_codes_to_fp8(const int8_t* __restrict__ q, long count, uint8_t* __restrict__ y) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  y[e] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32((float)q[e], 0.f, 0, false) & 0xff);
}

__global__ void k_scales_t(const f16* __restrict__ s, int n, int ng, float* __restrict__ gs) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)n * ng) return;
  const int g = (int)(e / n), col = (int)(e - (long)g * n);
  gs[e] = (float)s[(long)col * ng + g];
}

extern "C" int qd_fp8_weight(const int8_t* codes, const void* scales, int n, int k, int group, void* w8, float* gs,
                             void* stream) {
  QD_REQUIRE(codes && scales && w8 && gs, "null pointer");
  QD_REQUIRE(group > 0 && k % group == 0, "group must divide K");
  const long cnt = (long)n * k;
  if (cnt == 0) return 0;
  hipStream_t st = S(stream);
  k_codes_to_fp8<<<(int)((cnt + 255) / 256), 256, 0, st>>>(codes, cnt, (uint8_t*)w8);
  const long sc = (long)n * (k / group);
  k_scales_t<<<(int)((sc + 255) / 256), 256, 0, st>>>((const f16*)scales, n, k / group, gs);
  QD_CHECK_LAUNCH();
  return 0;
}
