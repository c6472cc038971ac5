// Achievable dense fp16 MFMA rate on this GPU under sustained load (the real ceiling the split
// kernels run against: the chip's clock drops under MFMA-heavy load). Each wave keeps NACC
// independent v_mfma_f32_32x32x16_f16 accumulator chains busy; WPS waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_peak tools/mfma_peak.hip && tools/bin/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(int iters, float* out) {
  f16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(threadIdx.x * 1e-3f + i);
    b[i] = (_Float16)(blockIdx.x * 1e-3f - i);
  }
  f32x16 acc[NACC];
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[j], 0, 0, 0);
  }
  float s = 0.f;
  for (int j = 0; j < NACC; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  if (s == 12345.f) out[threadIdx.x] = s;  // keep the work
}

template <int NACC>
void run(int blocks_per_cu, int cus) {
  float* out;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  const int iters = 20000, blocks = blocks_per_cu * cus;
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, 200, out);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(256), 0, 0, iters, out);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 16 * (double)NACC * iters * 4 /*waves*/ * blocks;
  printf("NACC %d, %d blocks/CU (%d waves/SIMD): %.3f ms, %.1f TFLOP/s dense fp16 (%.3f of 2500)\n", NACC,
         blocks_per_cu, blocks_per_cu, ms, flops / ms / 1e9, flops / ms / 1e9 / 2500.0);
  (void)hipFree(out);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int cus = p.multiProcessorCount;
  run<4>(1, cus);
  run<4>(2, cus);
  run<8>(1, cus);
  run<8>(2, cus);
  run<4>(4, cus);
  return 0;
}
