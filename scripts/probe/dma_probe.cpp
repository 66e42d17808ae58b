// L2 -> LDS streaming rate of the LDS-DMA (buffer_load ... lds) lock-step ring the GEMM kernels use,
// with no MFMA / epilogue: per K step  wait(own loads of stage s, counted vmcnt) -> s_barrier ->
// issue stage s + RING - 1.  One wave-instruction moves 1 KB = (1024 / R) rows x R bytes of a row-major
// source with row pitch P (R = 64: the int8 half-view stages, R = 128: the fp16 BK-64 stages).
// Source either shared by every block (an L2-resident weight) or distinct per block (HBM / MALL).
// usage: ./dma_probe   (prints one line per configuration: GB/s per CU, chip TB/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 6: wait_vm<6>(); break;
    case 8: wait_vm<8>(); break;
    case 10: wait_vm<10>(); break;
    case 12: wait_vm<12>(); break;
    case 16: wait_vm<16>(); break;
    case 20: wait_vm<20>(); break;
    case 24: wait_vm<24>(); break;
    case 32: wait_vm<32>(); break;
    default: wait_vm<0>(); break;
  }
}

// STAGE bytes per stage (multiple of NT * 16), RING stages, rows of R bytes at pitch P
template <int NT, int STAGE, int RING, int R>
__global__ void __launch_bounds__(NT) k_stream(const char* src, long per_block_bytes, int pitch, int shared_src,
                                               int steps, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char smem[STAGE * RING];
  constexpr int PER = STAGE / (NT * 16);  // wave-instructions per thread per stage
  constexpr int RPI = 1024 / R;           // rows per wave-instruction
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const char* base = src + (shared_src ? 0 : (long)blockIdx.x * per_block_bytes);
  const unsigned bytes = (unsigned)(shared_src ? per_block_bytes : per_block_bytes);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
  // stage s covers K columns [s * R, (s + 1) * R) of rows 0 .. STAGE / R - 1 (wrapping over the source)
  const int rows = STAGE / R;
  const int ncolblk = pitch / R;
  auto issue = [&](int s, int slot) {
    const int cb = s % ncolblk, rb = (s / ncolblk) * rows;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int inst = j * (NT / 64) + wid;          // wave-instruction index in the stage
      const int row = inst * RPI + lane / (R / 16);  // row of this lane
      const int chunk = lane % (R / 16);
      const long off = ((long)(rb + row) * pitch + cb * R + chunk * 16) % (long)per_block_bytes;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(smem + slot * STAGE + inst * 1024), 16, (int)off, 0,
                                               0, 0);
    }
  };
  for (int s = 0; s < RING - 1; ++s) issue(s, s);
  int slot = 0;
  for (int s = 0; s < steps; ++s) {
    const int ahead = min(RING - 2, steps - 1 - s);
    wait_vm_rt(ahead * PER);
    __builtin_amdgcn_s_barrier();
    if (s + RING - 1 < steps) issue(s + RING - 1, (s + RING - 1) % RING);
    if (++slot == RING) slot = 0;
  }
  wait_vm<0>();
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = *(unsigned*)(smem + (threadIdx.x * 16) % (STAGE * RING));
}

template <int NT, int STAGE, int RING, int R>
void run(const char* src, unsigned* sink, int blocks_per_cu, int shared, int pitch, long per_block, int steps) {
  const int grid = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) k_stream<NT, STAGE, RING, R><<<grid, NT>>>(src, per_block, pitch, shared, steps, sink);
  hipEventRecord(e0);
  const int iters = 20;
  for (int i = 0; i < iters; ++i) k_stream<NT, STAGE, RING, R><<<grid, NT>>>(src, per_block, pitch, shared, steps, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / iters;
  const double bytes_cu = (double)STAGE * steps * blocks_per_cu;
  printf("NT %3d stage %5d ring %d R %3d pitch %4d blocks/CU %d src %-8s: %7.1f us  %6.1f GB/s per CU  %5.2f TB/s\n", NT,
         STAGE, RING, R, pitch, blocks_per_cu, shared ? "shared" : "distinct", us, bytes_cu / us / 1e3,
         bytes_cu * 256 / us / 1e6);
}

int main() {
  char* src;
  unsigned* sink;
  const long total = 512L << 20;
  hipMalloc(&src, total);
  hipMemset(src, 1, total);
  hipMalloc(&sink, 4096 * 4);
  const int steps = 400;
  // the shared 800 KB weight (2560 rows x 320 codes): every block streams it
  for (int shared = 1; shared >= 0; --shared) {
    const long pb = shared ? 2560L * 320 : (total / 1024);  // distinct: <= 4 blocks per CU stay inside the buffer
    run<256, 16384, 3, 64>(src, sink, 2, shared, 320, pb, steps);
    run<256, 16384, 4, 64>(src, sink, 2, shared, 320, pb, steps);
    run<256, 16384, 3, 128>(src, sink, 2, shared, 640, pb, steps);
    run<256, 24576, 3, 64>(src, sink, 2, shared, 320, pb, steps);
    run<256, 8192, 4, 64>(src, sink, 2, shared, 320, pb, steps);
    run<256, 8192, 6, 64>(src, sink, 2, shared, 320, pb, steps);
    run<512, 32768, 3, 64>(src, sink, 1, shared, 320, pb, steps);
    run<512, 40960, 3, 64>(src, sink, 1, shared, 320, pb, steps);
    run<512, 16384, 6, 64>(src, sink, 1, shared, 320, pb, steps);
    run<512, 32768, 4, 128>(src, sink, 1, shared, 640, pb, steps);
    run<256, 8192, 3, 64>(src, sink, 4, shared, 320, pb, steps);
  }
  return 0;
}
