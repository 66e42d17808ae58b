// Store cache policy probe (measurement only, not part of the library): does a streaming kernel that
// writes B bytes finish sooner when its stores are write-through (sc1: the line leaves the XCD's L2)
// or non-temporal (nt) instead of plain (the line stays dirty in L2 and is written back at the
// kernel boundary)?  Back-to-back launches of a 16-B-per-lane copy / a copy + a tiny dependent kernel,
// HIP events around each sequence.
//   hipcc -O3 --offload-arch=gfx950 scripts/store_policy_bench.hip -o scripts/store_policy_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ void __launch_bounds__(256) k_copy(const v4i* __restrict__ x, v4i* __restrict__ y, long n16, int bytes) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n16) return;
  const v4i v = x[i];
  if constexpr (AUX < 0) {
    y[i] = v;
  } else {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, bytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(i * 16), 0, AUX);
  }
}

// per-row column sum (a GroupNorm-statistics-like read-only pass) to see read-after-write cost
__global__ void __launch_bounds__(256) k_tiny(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

template <int AUX>
static float run(const v4i* x, v4i* y, long n16, int bytes, int* flag, int reps, bool tiny) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)((n16 + 255) / 256);
  for (int w = 0; w < 3; ++w) k_copy<AUX><<<grid, 256>>>(x, y, n16, bytes);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) {
    k_copy<AUX><<<grid, 256>>>(x, y, n16, bytes);
    if (tiny) k_tiny<<<1, 64>>>(flag);
  }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1e3f / reps;
}

// a dependent chain: buffer i -> buffer i + 1 (mod 4), every launch reading what the previous wrote
template <int AUX>
static float chain(v4i* const* b, long n16, int bytes, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = (int)((n16 + 255) / 256);
  for (int w = 0; w < 4; ++w) k_copy<AUX><<<grid, 256>>>(b[w & 3], b[(w + 1) & 3], n16, bytes);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) k_copy<AUX><<<grid, 256>>>(b[r & 3], b[(r + 1) & 3], n16, bytes);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1e3f / reps;
}

int main() {
  const long sizes[] = {5L << 20, 10L << 20, 21L << 20, 42L << 20, 84L << 20};
  int* flag;
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(flag, 0, 4));
  for (long bytes : sizes) {
    v4i *x, *y;
    CK(hipMalloc(&x, bytes));
    CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 1, bytes));
    const long n16 = bytes / 16;
    for (int tiny = 0; tiny < 2; ++tiny) {
      const int reps = 200;
      const float tp = run<-1>(x, y, n16, (int)bytes, flag, reps, tiny);
      const float t1 = run<16>(x, y, n16, (int)bytes, flag, reps, tiny);
      const float tn = run<2>(x, y, n16, (int)bytes, flag, reps, tiny);
      const float tp2 = run<-1>(x, y, n16, (int)bytes, flag, reps, tiny);
      printf("%6.1f MB copy%s: plain %7.2f us (%5.2f TB/s)  sc1 %7.2f us (%5.2f TB/s)  nt %7.2f us  plain again %7.2f us\n",
             bytes / 1048576.0, tiny ? " + tiny" : "       ", tp, 2.0 * bytes / tp * 1e-6, t1, 2.0 * bytes / t1 * 1e-6, tn, tp2);
    }
    CK(hipFree(x));
    CK(hipFree(y));
    v4i* b[4];
    for (int i = 0; i < 4; ++i) {
      CK(hipMalloc(&b[i], bytes));
      CK(hipMemset(b[i], 1, bytes));
    }
    for (int rep = 0; rep < 2; ++rep) {
      const float cp = chain<-1>(b, n16, (int)bytes, 200), c1 = chain<16>(b, n16, (int)bytes, 200), cn = chain<2>(b, n16, (int)bytes, 200);
      printf("%6.1f MB chain (4 buffers, each launch reads the last one's output): plain %7.2f us  sc1 %7.2f us  nt %7.2f us\n",
             bytes / 1048576.0, cp, c1, cn);
    }
    for (int i = 0; i < 4; ++i) CK(hipFree(b[i]));
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
