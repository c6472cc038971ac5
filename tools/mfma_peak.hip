// Achievable dense fp16 MFMA rate on this GPU under sustained load (the real ceiling the split
// kernels run against: the chip's clock drops under MFMA-heavy load, and by how much depends on the
// data and on the MFMA shape, MI355X_MICROARCH.md "DVFS give-back" (7)). Each wave keeps NACC
// independent accumulator chains busy on random fp16 operands (four operand registers per chain, so the
// data toggles every instruction); WPS waves per SIMD. Both shapes the split kernels can use:
// v_mfma_f32_32x32x16_f16 (32 cycles) and v_mfma_f32_16x16x32_f16 (16 cycles), same FLOP per cycle.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_peak tools/mfma_peak.hip && tools/bin/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline float rnd(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return (float)(x & 0xffff) * (1.f / 32768.f) - 1.f;
}

template <int NACC, bool S16>
__global__ void __launch_bounds__(256) mfma_loop(int iters, float* out) {
  f16x8 a[4], b[4];
  for (int v = 0; v < 4; ++v)
    for (int i = 0; i < 8; ++i) {
      a[v][i] = (_Float16)rnd(threadIdx.x * 977u + blockIdx.x * 131071u + v * 8 + i);
      b[v][i] = (_Float16)rnd(threadIdx.x * 613u + blockIdx.x * 524287u + v * 8 + i + 1000003u);
    }
  typedef typename std::conditional<S16, f32x4, f32x16>::type acc_t;
  constexpr int R = S16 ? 4 : 16;
  constexpr int NA = S16 ? 2 * NACC : NACC;  // same accumulator registers, same FLOP per iteration
  acc_t acc[NA];
  for (int j = 0; j < NA; ++j)
    for (int r = 0; r < R; ++r) acc[j][r] = 0.f;
  for (int it = 0; it < iters; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        if constexpr (S16) {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[j & 3], b[(j + u) & 3], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(j + 1) & 3], b[(j + u + 2) & 3], acc[j], 0, 0, 0);
        } else {
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[j & 3], b[(j + u) & 3], acc[j], 0, 0, 0);
        }
      }
  }
  float s = 0.f;
  for (int j = 0; j < NA; ++j)
    for (int r = 0; r < R; ++r) s += acc[j][r];
  if (s == 12345.f) out[threadIdx.x] = s;  // keep the work
}

template <int NACC, bool S16>
void run(int blocks_per_cu, int cus) {
  float* out;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  const int iters = 40000, blocks = blocks_per_cu * cus;
  hipLaunchKernelGGL((mfma_loop<NACC, S16>), dim3(blocks), dim3(256), 0, 0, 2000, out);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipDeviceSynchronize();
  float best = 0.f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((mfma_loop<NACC, S16>), dim3(blocks), dim3(256), 0, 0, iters, out);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // per iteration and chain: one 32x32x16 (32768 flop) or two 16x16x32 on each of 2 chains (4 x 16384)
    const double flops = 2.0 * 32 * 32 * 16 * (double)NACC * iters * 4 /*waves*/ * blocks;
    const float tf = flops / ms / 1e9;
    if (tf > best) best = tf;
  }
  printf("%s NACC %d, %d waves/SIMD: %.1f TFLOP/s dense fp16 (%.3f of 2500)\n", S16 ? "16x16x32" : "32x32x16", NACC,
         blocks_per_cu, best, best / 2500.0);
  (void)hipFree(out);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int cus = p.multiProcessorCount;
  for (int pass = 0; pass < 2; ++pass) {
    run<4, false>(1, cus);
    run<4, true>(1, cus);
    run<4, false>(2, cus);
    run<4, true>(2, cus);
    run<8, false>(2, cus);
    run<8, true>(2, cus);
  }
  return 0;
}
