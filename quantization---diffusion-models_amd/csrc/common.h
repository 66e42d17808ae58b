// Shared device helpers for libqdiff (gfx950 / CDNA4, wave64).
//
// Numerics contract (pinned by tests/golden/*.npz): every fake-quant op
// is an fp16 op computed in fp32 and rounded to fp16 once (round-to-nearest-even), exactly as
// PyTorch-CPU Half arithmetic does in the reference (quantize/fake_quant.py:44-46, 72, 114-117).
// Division must be the IEEE-correct fp32 divide (hipcc default; never build with -ffast-math).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/qdiff.h"

typedef _Float16 f16;
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define QD_WAVE 64

// Keep a batch of loads issued back to back: hipcc sinks a load into the (guarded) block that
// consumes it and waits for it there, serialising a row batch; an empty asm that "uses" each
// loaded value right after the batch pins the loads in front of it (one vmcnt wait each).
#define QD_PIN(x) asm volatile("" ::"v"(x))

namespace qd {

// half(1e-5): the fp16 image of clamp_(min=1e-5) (no fp16 lies strictly between 1e-5 and it).
__device__ __forceinline__ float clamp_min_f16() { return (float)(f16)1e-5f; }

// f32 -> f16 with the f32 value materialised first.  Left alone, the backend folds the producing
// fma / mul into v_fma_mixlo_f16, which rounds the exact result to f16 once instead of to f32 and
// then to f16 (torch's op-boundary rounding); the two differ when the f32 rounding moves the value
// onto or across an f16 rounding midpoint (measured: 1 GroupNorm output in 655k moved by 1 ulp).
__device__ __forceinline__ f16 to_f16(float x) {
  asm volatile("" : "+v"(x));
  return (f16)x;
}

// s = half( half(max(amax, 1e-5)) / qmax )     fake_quant.py:44-46, 114-116, 127-129
__device__ __forceinline__ float fq_scale(float amax, int qmax) {
  float a = fmaxf(amax, clamp_min_f16());
  return (float)(f16)(a / (float)qmax);
}

// y = half( rint(half(x / s)) * s )            fake_quant.py:72, 117, 130
__device__ __forceinline__ f16 fq_apply(float x, float s) {
  f16 t = (f16)(x / s);
  float q = __builtin_rintf((float)t);
  return (f16)(q * s);
}

// fq_apply with the division replaced by a product with rs = 1.0 / (double)s (computed once per
// channel).  Exact: x and s are fp16 values, so x / s either terminates within 11 significant
// bits (then the f64 product, off by <= 2^-52 relative, rounds to it exactly) or lies >= ~2^-36
// (relative) away from every f32 rounding midpoint, far outside the f64 product's error; the f32
// rounding - and hence the fp16 one - equals that of the IEEE f32 quotient.  s == 0 (16-bit
// quant of an all-zero channel) gives rs = inf and the same inf / NaN as the division.
__device__ __forceinline__ f16 fq_apply_r(float x, float s, double rs) {
  f16 t = (f16)(float)((double)x * rs);
  float q = __builtin_rintf((float)t);
  return (f16)(q * s);
}

// rs for fq_apply_r: 1 / (double)s from the hardware f64 reciprocal estimate and two Newton
// steps (relative error <= ~2^-52, the bound the fq_apply_r argument allows, instead of the
// ~30-instruction IEEE f64 division).  s == 0 -> +inf, as the division.
__device__ __forceinline__ double rcp_exact(float s) {
  const double d = (double)s;
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
  r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
  return s == 0.f ? __builtin_inf() : r;
}

// fq_scale with the fp32 division by qmax replaced by an f64 product with rq ~ 1 / qmax (relative
// error <= 2^-50; rcp_exact((float)qmax)): bit-identical for every odd qmax (all 2^(b-1) - 1).  With
// x = a / qmax in the binade [2^e, 2^(e+1)), a (an fp32 >= 2^e) is a multiple of 2^(e-24), as is
// qmax * M for any fp32 rounding midpoint M (an odd multiple of 2^(e-24)); so |x - M| >= 2^(e-24) / qmax
// >= 2^-40 x unless a = qmax * M, impossible for odd qmax (an odd multiple of 2^(e-24) of at least 25
// significant bits).  The f64 product therefore rounds to the fp32 quotient, then to the same fp16.
__device__ __forceinline__ float fq_scale_rq(float amax, double rq) {
  const float a = fmaxf(amax, clamp_min_f16());
  return (float)(f16)(float)((double)a * rq);
}

// Per-channel fake-quant state of 8 consecutive channels: two 16-B amax loads issued together
// (a per-element conditional load would make hipcc serialise them), then s and 1/s; the 8 scale
// divisions by qmax as one reciprocal and 8 f64 products (fq_scale_rq: ~30 VALU instead of ~80).
// amax8 must be 16-B aligned (channel offsets are multiples of 8).
__device__ __forceinline__ void fq_scales8(const float* amax8, int qmax, float (&s)[8], double (&rs)[8]) {
  const float4 a0 = reinterpret_cast<const float4*>(amax8)[0];
  const float4 a1 = reinterpret_cast<const float4*>(amax8)[1];
  const float a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const double rq = rcp_exact((float)qmax);
  const bool odd = (qmax & 1) != 0;  // (uniform; an even qmax keeps the division)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = odd ? fq_scale_rq(a[j], rq) : fq_scale(a[j], qmax);
    rs[j] = rcp_exact(s[j]);
  }
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// non-negative float max through the uint image (valid for +0 and positive finite/inf)
__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// x * sigmoid(x) with the hardware reciprocal (1 ulp) instead of the IEEE division sequence: the
// GroupNorm+SiLU+fake-quant apply pass is VALU-bound; the fp16-rounded result stays within the
// GroupNorm / SiLU test tolerances (1 fp16 ulp)
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// exact-erf GELU as torch's F.gelu(approximate='none'): 0.5 * x * (1 + erf(x / sqrt 2)) in fp32 in
// torch's operation order, so its cancellation in 1 + erf for x << 0 is reproduced.  erf comes
// from the branch-free complementary fit erfc(z) = t exp(-z^2 + P(t)), t = 1 / (1 + z / 2)
// (Numerical Recipes "erfcc", fractional error < 1.2e-7 for z >= 0): ~17 VALU ops with two
// transcendentals instead of the library erff's ~25 plus a divergent branch.  The GEGLU epilogue
// is VALU-bound on the UNet's short-K (K = 320) projections.  Against erff the fp16-rounded GELU
// moves by 1 ulp on 193 of 3e6 inputs (numpy emulation over [-12, 12] + N(0, 9) samples).
__device__ __forceinline__ float gelu_f(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = t * __builtin_amdgcn_exp2f(fmaf(-z, z, p) * 1.44269504088896341f);  // erfc(z)
  const float er = 1.0f - e;                                                         // erf(z)
  return 0.5f * x * (1.0f + (x >= 0.f ? er : -er));
}

// gelu_f on two values with packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes'
// worth per instruction; the two transcendentals stay scalar): the same IEEE operations in the
// same order per element, so the results equal gelu_f's bit for bit, at ~2/3 of its issue cost
// (the GEGLU epilogue of the K = 320 projections is VALU-bound).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2_f(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  const f32x2 d = __builtin_elementwise_fma((f32x2)(0.5f), z, (f32x2)(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = (f32x2)(0.17087277f);
  p = __builtin_elementwise_fma(p, t, (f32x2)(-0.82215223f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(1.48851587f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(-1.13520398f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(0.27886807f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(-0.18628806f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(0.09678418f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(0.37409196f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(1.00002368f));
  p = __builtin_elementwise_fma(p, t, (f32x2)(-1.26551223f));
  const f32x2 q = __builtin_elementwise_fma(-z, z, p) * 1.44269504088896341f;
  const f32x2 ex = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 er = 1.0f - t * ex;
  const f32x2 ser = {x.x >= 0.f ? er.x : -er.x, x.y >= 0.f ? er.y : -er.y};
  return 0.5f * x * (1.0f + ser);
}

// tanh-approximate GELU, torch's F.gelu(approximate='tanh') = 0.5 x (1 + tanh(u)),
// u = sqrt(2/pi) (x + 0.044715 x^3), evaluated as the identical x / (1 + exp(-2u)): one hardware
// exp + one reciprocal instead of the library tanhf (fp32 result within a few ulp, so the fp16
// output equals torch's except when the value sits within ~1e-6 of an fp16 rounding boundary).
// exp(-2u) -> inf for x << 0 gives -0, as torch; exp -> 0 for x >> 0 gives x.
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * u));
}

}  // namespace qd

#define QD_CHECK_LAUNCH()                                              \
  do {                                                                 \
    hipError_t _e = hipGetLastError();                                 \
    if (_e != hipSuccess) return qd_set_error((int)_e, hipGetErrorString(_e)); \
  } while (0)

#define QD_REQUIRE(cond, msg)                                          \
  do {                                                                 \
    if (!(cond)) return qd_set_error(QD_ERR_ARG, msg);                 \
  } while (0)

extern "C" int qd_set_error(int code, const char* msg);

// Zero an fp32 workspace with a kernel node, never hipMemsetAsync: memset nodes captured into a
// hipGraph were observed (ROCm 7.x runtime bundled with torch) to race with the following
// kernel on replay, leaving atomic-max targets unzeroed/zeroed late ("graph capture").
void qd_zero_f32(float* p, size_t n, hipStream_t st);
