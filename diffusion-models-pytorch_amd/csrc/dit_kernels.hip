// Small bandwidth-bound kernels of the DiT denoiser (models/dit/model.py):
//   * LayerNorm row statistics for the fused LN + adaLN-modulate GEMM prologue
//     (DiTBlock norm1 / norm2, FinalLayer norm_final: eps 1e-6, no affine);
//   * patchify (PatchEmbed's Conv2d k = s = p as a GEMM input) and unpatchify.
#include "dm_common.h"
#include "dm_kernels.h"
#include "split16.h"

namespace dm {

namespace {

// One 64-lane wavefront per row. fp64 accumulation of the mean, then of the
// squared deviations (two passes over the row, the second from L1/L2).
__global__ void __launch_bounds__(256) row_stats_kernel(const float* __restrict__ x, long rows, int D, float eps,
                                                        float2* __restrict__ stats) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* row = x + (size_t)r * D;
  const int D4 = D >> 2;
  double s = 0.0;
  for (int i = lane; i < D4; i += 64) {
    const float4 v = reinterpret_cast<const float4*>(row)[i];
    s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double mean = s / D;
  double q = 0.0;
  for (int i = lane; i < D4; i += 64) {
    const float4 v = reinterpret_cast<const float4*>(row)[i];
    const double a = v.x - mean, b = v.y - mean, c = v.z - mean, d = v.w - mean;
    q += a * a + b * b + c * c + d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  if (lane == 0) {
    const float var = (float)(q / D);
    stats[r] = make_float2((float)mean, 1.0f / sqrtf(var + eps));
  }
}

// row_stats + the LayerNorm + adaLN-modulate prologue of the GEMM that reads the row + the fp16x2 split:
// the row's pre-split A image for linear_k32 (linear_presplit_a's layout and expressions: the float
// statistics the GEMM prologue would use, ((v - mean) * rstd) * (1 + scale) + shift, times 2^ea).
// One wave per row; the statistics exactly as row_stats_kernel, then a third pass by 8-channel groups.
__global__ void __launch_bounds__(256) row_stats_split_kernel(const float* __restrict__ x, long rows, int D, float eps,
                                                              float2* __restrict__ stats, const float* ln_shift,
                                                              const float* ln_scale, int ln_pitch, int ln_rows,
                                                              int split_ea, _Float16* __restrict__ out, int* range_flag) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* row = x + (size_t)r * D;
  const int D4 = D >> 2;
  double s = 0.0;
  for (int i = lane; i < D4; i += 64) {
    const float4 v = reinterpret_cast<const float4*>(row)[i];
    s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double mean = s / D;
  double q = 0.0;
  for (int i = lane; i < D4; i += 64) {
    const float4 v = reinterpret_cast<const float4*>(row)[i];
    const double a = v.x - mean, b = v.y - mean, c = v.z - mean, d = v.w - mean;
    q += a * a + b * b + c * c + d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float var = (float)(q / D);
  const float2 lns = make_float2((float)mean, 1.0f / sqrtf(var + eps));
  if (lane == 0 && stats) stats[r] = lns;
  const float apow = ldexpf(1.f, split_ea);
  const size_t mo = (size_t)(r / ln_rows) * ln_pitch;
  bool bad = false;
  for (int g8 = lane; g8 < D / 8; g8 += 64) {
    const int c = 8 * g8;
    f4 v0 = *reinterpret_cast<const f4*>(row + c), v1 = *reinterpret_cast<const f4*>(row + c + 4);
    const f4 s0 = *reinterpret_cast<const f4*>(ln_scale + mo + c), s1 = *reinterpret_cast<const f4*>(ln_scale + mo + c + 4);
    const f4 h0 = *reinterpret_cast<const f4*>(ln_shift + mo + c), h1 = *reinterpret_cast<const f4*>(ln_shift + mo + c + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = ((v0[e] - lns.x) * lns.y) * (1.0f + s0[e]) + h0[e];
      v1[e] = ((v1[e] - lns.x) * lns.y) * (1.0f + s1[e]) + h1[e];
    }
    f16x8 pc[2];
    Split<2>::split(v0 * apow, v1 * apow, pc, bad);
    _Float16* dst = out + (size_t)r * 2 * D + (c / 32) * 64 + ((c % 32) / 8) * 8;
    *reinterpret_cast<f16x8*>(dst) = pc[0];
    *reinterpret_cast<f16x8*>(dst + 32) = pc[1];
  }
  if (bad && range_flag) *range_flag = 1;
}

// The same, with the row held in registers (D <= 1280: at most 5 float4 per lane): one global read of the
// row instead of three dependent passes (the kernel was latency-bound at 44 us for 2 x 75 MB at DiT-XL/2's
// 2B = 64). Same sums in the same order (lane l: float4 l, l + 64, ...), same expressions: bit-identical.
__global__ void __launch_bounds__(256) row_stats_split_reg_kernel(const float* __restrict__ x, long rows, int D,
                                                                  float eps, float2* __restrict__ stats,
                                                                  const float* ln_shift, const float* ln_scale,
                                                                  int ln_pitch, int ln_rows, int split_ea,
                                                                  _Float16* __restrict__ out, int* range_flag) {
  constexpr int NV = 5;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* row = x + (size_t)r * D;
  const int D4 = D >> 2;
  f4 v[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = lane + 64 * u;
    v[u] = i < D4 ? reinterpret_cast<const f4*>(row)[i] : f4{0.f, 0.f, 0.f, 0.f};
  }
  const size_t mo = (size_t)(r / ln_rows) * ln_pitch;
  f4 sc[NV], sh[NV];  // this lane's modulation, loaded with the row
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = min(lane + 64 * u, D4 - 1);
    sc[u] = *reinterpret_cast<const f4*>(ln_scale + mo + 4 * i);
    sh[u] = *reinterpret_cast<const f4*>(ln_shift + mo + 4 * i);
  }
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < NV; ++u)
    if (lane + 64 * u < D4) s += (double)v[u][0] + (double)v[u][1] + (double)v[u][2] + (double)v[u][3];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double mean = s / D;
  double q = 0.0;
#pragma unroll
  for (int u = 0; u < NV; ++u)
    if (lane + 64 * u < D4) {
      const double a = v[u][0] - mean, b = v[u][1] - mean, c = v[u][2] - mean, d = v[u][3] - mean;
      q += a * a + b * b + c * c + d * d;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float var = (float)(q / D);
  const float2 lns = make_float2((float)mean, 1.0f / sqrtf(var + eps));
  if (lane == 0 && stats) stats[r] = lns;
  const float apow = ldexpf(1.f, split_ea);
  bool bad = false;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = lane + 64 * u;
    if (i >= D4) continue;
    f4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = ((v[u][e] - lns.x) * lns.y) * (1.0f + sc[u][e]) + sh[u][e];
    f16x4 h, l;
    Split<2>::split4(y * apow, h, l, bad);
    const int c = 4 * i;
    _Float16* dst = out + (size_t)r * 2 * D + (c / 32) * 64 + ((c % 32) / 8) * 8 + (c % 8);
    *reinterpret_cast<f16x4*>(dst) = h;
    *reinterpret_cast<f16x4*>(dst + 32) = l;
  }
  if (bad && range_flag) *range_flag = 1;
}

__global__ void patchify_kernel(const float* __restrict__ x, int B, int C, int H, int W, int p,
                                float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * C * H * W;
  if (e >= total) return;
  // e enumerates the NCHW input; scatter into the [token][c * p * p + pr * p + qc] layout
  const int xx = e % W;
  long r = e / W;
  const int yy = r % H;
  r /= H;
  const int c = r % C;
  const int b = r / C;
  const int w = W / p, h = H / p;
  const long tok = ((long)b * h + yy / p) * w + xx / p;
  out[tok * (C * p * p) + c * p * p + (yy % p) * p + (xx % p)] = x[e];
}

__global__ void unpatchify_kernel(const float* __restrict__ x, int B, int C, int H, int W, int p,
                                  float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * C * H * W;
  if (e >= total) return;
  // e enumerates the NCHW output (einsum 'nhwpqc->nchpwq', dit/model.py:229-231)
  const int xx = e % W;
  long r = e / W;
  const int yy = r % H;
  r /= H;
  const int c = r % C;
  const int b = r / C;
  const int w = W / p, h = H / p;
  const long tok = ((long)b * h + yy / p) * w + xx / p;
  out[e] = x[tok * (p * p * C) + ((yy % p) * p + (xx % p)) * C + c];
}

}  // namespace

int row_stats(const float* x, long rows, int D, float eps, float2* stats, hipStream_t st) {
  DM_REQUIRE(D % 4 == 0 && rows > 0, "row_stats: D must be a multiple of 4");
  const long blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(row_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, D, eps, stats);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int row_stats_split(const float* x, long rows, int D, float eps, float2* stats, const float* ln_shift,
                    const float* ln_scale, int ln_pitch, int ln_rows, int split_ea, _Float16* out, int* range_flag,
                    hipStream_t st) {
  DM_REQUIRE(D % 64 == 0 && rows > 0 && ln_pitch % 4 == 0 && ln_rows > 0 &&
                 (reinterpret_cast<uintptr_t>(ln_shift) & 15) == 0 && (reinterpret_cast<uintptr_t>(ln_scale) & 15) == 0,
             "row_stats_split: D % 64 == 0 and 16-byte aligned modulation rows");
  const long blocks = (rows + 3) / 4;
  if (D <= 1280)
    hipLaunchKernelGGL(row_stats_split_reg_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, D, eps, stats,
                       ln_shift, ln_scale, ln_pitch, ln_rows, split_ea, out, range_flag);
  else
    hipLaunchKernelGGL(row_stats_split_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, D, eps, stats,
                       ln_shift, ln_scale, ln_pitch, ln_rows, split_ea, out, range_flag);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int patchify(const float* x, int B, int C, int H, int W, int p, float* out, hipStream_t st) {
  DM_REQUIRE(H % p == 0 && W % p == 0, "patchify: image size must be divisible by the patch size");
  const long total = (long)B * C * H * W;
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, B, C, H, W, p,
                     out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int unpatchify(const float* x, int B, int C, int H, int W, int p, float* out, hipStream_t st) {
  DM_REQUIRE(H % p == 0 && W % p == 0, "unpatchify: image size must be divisible by the patch size");
  const long total = (long)B * C * H * W;
  hipLaunchKernelGGL(unpatchify_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, B, C, H, W, p,
                     out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
