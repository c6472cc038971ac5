// GroupNorm for NHWC (channel-pitched) activations.
//
// Reference semantics: torch.nn.GroupNorm(G, C, eps=1e-5) as used by
// models/unet.py:14,23,116 and models/modules.py:82 (SiLU applied afterwards in
// the ResBlock / last_conv Sequentials, not in the attention block).
//
// Two kernels, both HBM-bound:
//   gn_partial : one pass over the tensor; per (image, pixel-chunk, group)
//                partial {sum, sum of squares} accumulated in fp64
//                (stable variance without a second pass; fp32 data).
//   gn_apply   : reduces the partials of its image to mean / rstd, builds the
//                per-channel affine  y = x * scale + shift  (ATen's order:
//                scale = rstd * gamma, shift = -scale * mean + beta), optional
//                per-(b, c) modulation  y * (1 + ys) + yb  (AdaGN / ADM
//                scale-shift norm), optional SiLU, and writes the output view.
// The partial layout [B][nchunk][G] (double2) is shared with producers that
// emit GN partials from their epilogue.
#include <algorithm>

#include "dm_common.h"
#include "dm_kernels.h"

namespace dm {

namespace {

constexpr int kMaxC = 4096;

__global__ void gn_partial_kernel(const float* __restrict__ x, int HW, int C, int pitch,
                                  int G, int pix_per_chunk, int nchunk,
                                  double2* __restrict__ part) {
  extern __shared__ double smem_d[];  // [PY][C] sums, then [PY][C] sumsq
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int C4 = C >> 2;
  const int PY = blockDim.x / C4;
  const int t = threadIdx.x;
  const int c4 = t % C4, py = t / C4;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
  const int p_beg = chunk * pix_per_chunk;
  const int p_end = min(HW, p_beg + pix_per_chunk);
  if (py < PY) {
    const float* base = x + (size_t)b * HW * pitch + 4 * c4;
    // four pixels' loads in flight before their (in-order) accumulation: the loop otherwise keeps
    // one 16-B load per thread outstanding and runs latency-bound
    auto acc4 = [&](const float4 v) {
      s0 += v.x; s1 += v.y; s2 += v.z; s3 += v.w;
      q0 += (double)v.x * v.x; q1 += (double)v.y * v.y;
      q2 += (double)v.z * v.z; q3 += (double)v.w * v.w;
    };
    int p = p_beg + py;
    for (; p + 3 * PY < p_end; p += 4 * PY) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(base + (size_t)(p + u * PY) * pitch);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc4(v[u]);
    }
    for (; p < p_end; p += PY) acc4(*reinterpret_cast<const float4*>(base + (size_t)p * pitch));
    double* S = smem_d;
    double* Q = smem_d + PY * C;
    S[py * C + 4 * c4 + 0] = s0; S[py * C + 4 * c4 + 1] = s1;
    S[py * C + 4 * c4 + 2] = s2; S[py * C + 4 * c4 + 3] = s3;
    Q[py * C + 4 * c4 + 0] = q0; Q[py * C + 4 * c4 + 1] = q1;
    Q[py * C + 4 * c4 + 2] = q2; Q[py * C + 4 * c4 + 3] = q3;
  }
  __syncthreads();
  // column reduction over PY rows -> row 0
  for (int c = t; c < C; c += blockDim.x) {
    double a = 0, q = 0;
    for (int r = 0; r < PY; ++r) { a += smem_d[r * C + c]; q += smem_d[PY * C + r * C + c]; }
    smem_d[c] = a;
    smem_d[PY * C + c] = q;
  }
  __syncthreads();
  const int cpg = C / G;
  for (int g = t; g < G; g += blockDim.x) {
    double a = 0, q = 0;
    for (int j = 0; j < cpg; ++j) { a += smem_d[g * cpg + j]; q += smem_d[PY * C + g * cpg + j]; }
    part[((size_t)b * nchunk + chunk) * G + g] = make_double2(a, q);
  }
}

__global__ void gn_apply_kernel(const float* __restrict__ x, int HW, int C, int pitch,
                                int G, const double2* __restrict__ part, int nchunk, float eps,
                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                const float* __restrict__ mod_scale, const float* __restrict__ mod_shift,
                                int mod_pitch, int act, int pix_per_block,
                                float* __restrict__ y, int y_pitch) {
  extern __shared__ float smem_f[];  // scale[C], shift[C], mean[G], rstd[G]
  float* sc = smem_f;
  float* sh = smem_f + C;
  float* mu = smem_f + 2 * C;
  float* rs = smem_f + 2 * C + G;
  const int b = blockIdx.y;
  const int t = threadIdx.x;
  const int cpg = C / G;
  const double n = (double)HW * cpg;
  for (int g = t; g < G; g += blockDim.x) {
    double a = 0, q = 0;
    for (int k = 0; k < nchunk; ++k) {
      double2 v = part[((size_t)b * nchunk + k) * G + g];
      a += v.x; q += v.y;
    }
    double m = a / n;
    double var = q / n - m * m;
    if (var < 0) var = 0;
    mu[g] = (float)m;
    rs[g] = (float)(1.0 / sqrt(var + (double)eps));
  }
  __syncthreads();
  for (int c = t; c < C; c += blockDim.x) {
    const int g = c / cpg;
    float s = rs[g] * (gamma ? gamma[c] : 1.0f);
    sc[c] = s;
    sh[c] = -s * mu[g] + (beta ? beta[c] : 0.0f);
  }
  __syncthreads();
  const int C4 = C >> 2;
  const int PY = blockDim.x / C4;
  const int c4 = t % C4, py = t / C4;
  if (py >= PY) return;
  const int p_beg = blockIdx.x * pix_per_block;
  const int p_end = min(HW, p_beg + pix_per_block);
  const float4 s4 = *reinterpret_cast<const float4*>(sc + 4 * c4);
  const float4 h4 = *reinterpret_cast<const float4*>(sh + 4 * c4);
  float4 ms = make_float4(0, 0, 0, 0), mb = make_float4(0, 0, 0, 0);
  if (mod_scale) ms = *reinterpret_cast<const float4*>(mod_scale + (size_t)b * mod_pitch + 4 * c4);
  if (mod_shift) mb = *reinterpret_cast<const float4*>(mod_shift + (size_t)b * mod_pitch + 4 * c4);
  const float* xb = x + (size_t)b * HW * pitch + 4 * c4;
  float* yb = y + (size_t)b * HW * y_pitch + 4 * c4;
  for (int p = p_beg + py; p < p_end; p += PY) {
    float4 v = *reinterpret_cast<const float4*>(xb + (size_t)p * pitch);
    float o[4] = {v.x * s4.x + h4.x, v.y * s4.y + h4.y, v.z * s4.z + h4.z, v.w * s4.w + h4.w};
    if (mod_scale) {
      o[0] = o[0] * (1.0f + ms.x); o[1] = o[1] * (1.0f + ms.y);
      o[2] = o[2] * (1.0f + ms.z); o[3] = o[3] * (1.0f + ms.w);
    }
    if (mod_shift) { o[0] += mb.x; o[1] += mb.y; o[2] += mb.z; o[3] += mb.w; }
    if (act == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = silu_f(o[i]);
    }
    *reinterpret_cast<float4*>(yb + (size_t)p * y_pitch) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// part [B][nchunk][G] -> per-(image, channel) affine: scale = rstd * gamma,
// shift = -scale * mean + beta (the exact arithmetic of gn_apply_kernel), so a
// consumer can apply the norm inside its own operand load.
__global__ void gn_finalize_kernel(const double2* __restrict__ part, int B, int nchunk, int G, int C, double n,
                                   float eps, const float* __restrict__ gamma, const float* __restrict__ beta,
                                   const float* __restrict__ mod_scale, const float* __restrict__ mod_shift,
                                   int mod_pitch, float* __restrict__ scale, float* __restrict__ shift) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * C) return;
  const int b = idx / C, c = idx - (idx / C) * C;
  const int cpg = C / G, g = c / cpg;
  double a = 0, q = 0;
  for (int k = 0; k < nchunk; ++k) {
    const double2 v = part[((size_t)b * nchunk + k) * G + g];
    a += v.x;
    q += v.y;
  }
  const double m = a / n;
  double var = q / n - m * m;
  if (var < 0) var = 0;
  const float mu = (float)m;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  float sc = rs * (gamma ? gamma[c] : 1.0f);
  float sh = -sc * mu + (beta ? beta[c] : 0.0f);
  if (mod_scale) {
    // AdaGN / scale-shift norm: (x * sc + sh) * (1 + ys) + yb  (modules.py:114-123)
    const float f = 1.0f + mod_scale[(size_t)b * mod_pitch + c];
    sc = sc * f;
    sh = sh * f + (mod_shift ? mod_shift[(size_t)b * mod_pitch + c] : 0.0f);
  }
  scale[idx] = sc;
  shift[idx] = sh;
}

// Wide maps (more than kGnWideChunks chunk partials per image: ADM's 64^2 .. 256^2 maps, up to 1024): one
// thread per (image, channel) walking every chunk serially left B * C threads with ~1k dependent fp64
// loads each (134 us per launch at B = 4, 256^2). Here 32 lanes of a wave reduce one (image, group) --
// chunk k on lane k % 32, then a fixed shuffle tree -- and the group's channels take the result: the
// same expressions from the totals on, a different (fixed) fp64 summation order.
constexpr int kGnWideChunks = 64;
__global__ void __launch_bounds__(256) gn_finalize_wide_kernel(const double2* __restrict__ part, int B, int nchunk,
                                                               int G, int C, double n, float eps,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               const float* __restrict__ mod_scale,
                                                               const float* __restrict__ mod_shift, int mod_pitch,
                                                               float* __restrict__ scale, float* __restrict__ shift) {
  const int lane = threadIdx.x & 31;
  const int bg = blockIdx.x * 8 + (threadIdx.x >> 5);   // (image, group)
  if (bg >= B * G) return;
  const int b = bg / G, g = bg - b * G;
  double a = 0, q = 0;
  for (int k = lane; k < nchunk; k += 32) {
    const double2 v = part[((size_t)b * nchunk + k) * G + g];
    a += v.x;
    q += v.y;
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 32);
    q += __shfl_xor(q, o, 32);
  }
  const double m = a / n;
  double var = q / n - m * m;
  if (var < 0) var = 0;
  const float mu = (float)m;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  const int cpg = C / G;
  for (int j = lane; j < cpg; j += 32) {
    const int c = g * cpg + j;
    const size_t idx = (size_t)b * C + c;
    float sc = rs * (gamma ? gamma[c] : 1.0f);
    float sh = -sc * mu + (beta ? beta[c] : 0.0f);
    if (mod_scale) {
      const float f = 1.0f + mod_scale[(size_t)b * mod_pitch + c];
      sc = sc * f;
      sh = sh * f + (mod_shift ? mod_shift[(size_t)b * mod_pitch + c] : 0.0f);
    }
    scale[idx] = sc;
    shift[idx] = sh;
  }
}

inline int gn_block_threads(int C) {
  int C4 = C / 4;
  int t = C4 > 256 ? C4 : 256;
  t = (t + 63) / 64 * 64;
  return t;
}

}  // namespace

// GroupNorm partials of a channel concat [h | skip] from its two slices' partials, each emitted by its producer
// with its own group count over its own channels (Gh over Ch, Gs over Cs: the consumer's G, or 4-channel units
// when the concat's groups straddle the slice boundary -- the 384 = 256 + 128 concats of the CIFAR UNet): concat
// group j sums the slice groups inside its channel range, h's then skip's, in channel order (gn_concat_ok
// checks that no slice group straddles a concat group). Replaces a gn_partial pass over the concat.
__global__ void gn_concat_stats_kernel(const double2* __restrict__ ph, const double2* __restrict__ ps, long n, int G,
                                       int cpg, int Ch, int cph, int Gh, int cps, int Gs,
                                       double2* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long bk = i / G;  // (image, chunk)
  const int j = (int)(i - bk * G);
  const int c_lo = j * cpg, c_hi = c_lo + cpg;
  double s1 = 0.0, s2 = 0.0;
  for (int c = c_lo; c < min(c_hi, Ch); c += cph) {
    const double2 v = ph[bk * Gh + c / cph];
    s1 += v.x;
    s2 += v.y;
  }
  for (int c = max(c_lo, Ch); c < c_hi; c += cps) {
    const double2 v = ps[bk * Gs + (c - Ch) / cps];
    s1 += v.x;
    s2 += v.y;
  }
  out[i] = make_double2(s1, s2);
}

int gn_num_chunks(int HW) { return ceil_div(HW, kGnPixPerChunk); }

bool gn_concat_ok(int Ch, int Gh, int Cs, int Gs, int G) {
  const int C = Ch + Cs;
  if (G <= 0 || Gh <= 0 || Gs <= 0 || C % G != 0 || Ch % Gh != 0 || Cs % Gs != 0) return false;
  const int cpg = C / G, cph = Ch / Gh, cps = Cs / Gs;
  for (int j = 0; j < G; ++j) {
    const int lo = j * cpg, hi = lo + cpg;
    if (lo < Ch && (lo % cph != 0 || std::min(hi, Ch) % cph != 0)) return false;
    if (hi > Ch && ((std::max(lo, Ch) - Ch) % cps != 0 || (hi - Ch) % cps != 0)) return false;
  }
  return true;
}

int gn_concat_stats(const double2* ph, int Ch, int Gh, const double2* ps, int Cs, int Gs, int B, int HW, int G,
                    double2* out, hipStream_t st) {
  DM_REQUIRE(gn_concat_ok(Ch, Gh, Cs, Gs, G), "gn_concat_stats: the slices' groups must tile the concat's groups");
  const long n = (long)B * gn_num_chunks(HW) * G;
  hipLaunchKernelGGL(gn_concat_stats_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ph, ps, n, G,
                     (Ch + Cs) / G, Ch, Ch / Gh, Gh, Cs / Gs, Gs, out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int gn_partial(const View& x, int G, double2* part, hipStream_t st) {
  DM_REQUIRE(x.C % 4 == 0 && x.pitch % 4 == 0, "GroupNorm needs C and pitch multiple of 4");
  DM_REQUIRE(x.C % G == 0, "GroupNorm: C must be divisible by groups");
  DM_REQUIRE(x.C <= kMaxC, "GroupNorm: C too large");
  DM_REQUIRE((reinterpret_cast<uintptr_t>(x.p) & 15) == 0, "GroupNorm: input must be 16-byte aligned");
  const int HW = x.H * x.W;
  const int nchunk = gn_num_chunks(HW);
  const int threads = gn_block_threads(x.C);
  DM_REQUIRE(threads <= 1024, "GroupNorm: too many channels");
  const int PY = threads / (x.C / 4);
  size_t smem = (size_t)2 * PY * x.C * sizeof(double);
  DM_REQUIRE(smem <= 64 * 1024, "GroupNorm: LDS budget");
  dim3 grid(nchunk, x.B);
  hipLaunchKernelGGL(gn_partial_kernel, grid, dim3(threads), smem, st, x.p, HW, x.C, x.pitch, G,
                     kGnPixPerChunk, nchunk, part);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int gn_finalize(const View& x, int G, const double2* part, float eps, const float* gamma, const float* beta,
                float* scale, float* shift, hipStream_t st, const float* mod_scale, const float* mod_shift,
                int mod_pitch) {
  DM_REQUIRE(x.C % G == 0, "GroupNorm finalize: C must be divisible by groups");
  const int HW = x.H * x.W;
  const int n = x.B * x.C;
  if (gn_num_chunks(HW) > kGnWideChunks) {
    hipLaunchKernelGGL(gn_finalize_wide_kernel, dim3(ceil_div(x.B * G, 8)), dim3(256), 0, st, part, x.B,
                       gn_num_chunks(HW), G, x.C, (double)HW * (x.C / G), eps, gamma, beta, mod_scale, mod_shift,
                       mod_pitch, scale, shift);
    DM_LAUNCH_CHECK();
    return DM_OK;
  }
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, part, x.B, gn_num_chunks(HW), G,
                     x.C, (double)HW * (x.C / G), eps, gamma, beta, mod_scale, mod_shift, mod_pitch, scale, shift);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int gn_apply(const View& x, int G, const double2* part, int nchunk, float eps, const float* gamma,
             const float* beta, const float* mod_scale, const float* mod_shift, int mod_pitch,
             int act, const View& y, hipStream_t st) {
  DM_REQUIRE(x.C == y.C && x.B == y.B && x.H == y.H && x.W == y.W, "GroupNorm apply: shape mismatch");
  DM_REQUIRE(x.C % 4 == 0 && y.pitch % 4 == 0 && x.pitch % 4 == 0, "GroupNorm apply: alignment");
  DM_REQUIRE((reinterpret_cast<uintptr_t>(y.p) & 15) == 0, "GroupNorm apply: output must be 16-byte aligned");
  DM_REQUIRE(mod_pitch % 4 == 0, "GroupNorm apply: modulation pitch");
  const int HW = x.H * x.W;
  const int threads = gn_block_threads(x.C);
  const int ppb = 64;
  dim3 grid(ceil_div(HW, ppb), x.B);
  size_t smem = (size_t)(2 * x.C + 2 * G) * sizeof(float);
  hipLaunchKernelGGL(gn_apply_kernel, grid, dim3(threads), smem, st, x.p, HW, x.C, x.pitch, G, part,
                     nchunk, eps, gamma, beta, mod_scale, mod_shift, mod_pitch, act, ppb, y.p, y.pitch);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
