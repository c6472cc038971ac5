// Probe of ds_read_b64_tr_b16 semantics (tools/probe/tr16_probe.hip): LDS holds element value = 1000 * row + col
// over a [32][272] fp16 image (as attn_block3_kernel's key-chunk image); every lane reads with the
// attn_block3_kernel PV addressing and the result is printed for lanes 0..63 (expected per the documented
// mechanism: lane i of group g receives column 16 ot + i of rows 4 g .. 4 g + 3).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16x4_t lds_tr16(const _Float16* p) {
  typedef __fp16 hv4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
  typedef __attribute__((address_space(3))) hv4 lds_hv4;
  const hv4 r = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hv4*)(p));
  return __builtin_bit_cast(f16x4_t, r);
}

__global__ void probe(float* out, int ot) {
  __shared__ __attribute__((aligned(16))) _Float16 img[32 * 272];
  for (int i = threadIdx.x; i < 32 * 272; i += 64) {
    const int r = i / 272, c = i % 272;
    img[i] = (_Float16)(float)((r % 32) * 64 + (c % 64));   // exact in fp16 (< 2048)
  }
  __syncthreads();
  const int lane = threadIdx.x, l16 = lane & 15, q = lane >> 4;
  const _Float16* pt = img + (4 * q + (l16 >> 2)) * 272 + 4 * (l16 & 3);
  const f16x4_t lo = lds_tr16(pt + 16 * ot);
  const f16x4_t hi = lds_tr16(pt + 16 * 272 + 16 * ot);
  for (int e = 0; e < 4; ++e) {
    out[lane * 8 + e] = (float)lo[e];
    out[lane * 8 + 4 + e] = (float)hi[e];
  }
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 8 * sizeof(float));
  float h[64 * 8];
  int bad = 0;
  for (int ot = 0; ot < 2; ++ot) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, ot);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int lane = 0; lane < 64; ++lane) {
      const int l16 = lane & 15, q = lane >> 4;
      for (int e = 0; e < 8; ++e) {
        const int key = e < 4 ? 4 * q + e : 16 + 4 * q + (e - 4);
        const int col = 16 * ot + l16;
        const float want = key * 64 + col;
        if (h[lane * 8 + e] != want) {
          if (bad < 12) printf("ot %d lane %d e %d got %g (row %d col %d) want %g (row %d col %d)\n", ot, lane, e,
                               h[lane * 8 + e], (int)h[lane * 8 + e] / 64, (int)h[lane * 8 + e] % 64, want, key, col);
          ++bad;
        }
      }
    }
  }
  printf("tr16 probe: %d mismatches\n", bad);
  for (int lane = 0; lane < 20; ++lane) {
    printf("lane %2d:", lane);
    for (int e = 0; e < 8; ++e) printf(" (%d,%d)", (int)h[lane * 8 + e] / 64, (int)h[lane * 8 + e] % 64);
    printf("\n");
  }
  return bad ? 1 : 0;
}
