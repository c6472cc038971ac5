// Folded single-head self-attention block for 16 x 16 maps of 256 channels (the CIFAR-10 UNet's stage-1
// blocks, models/modules.py:77-102): y = x + proj(softmax(s q k^T) v) with q / k / v / proj 1x1 convs of
// GroupNorm(x), computed as
//
//   T = xn A + w            A = s Wq^T Wk, w = s Wk^T bq          (query side, per token: 256 x 256)
//   S_ij = T_i . xn_j       (= s q_i . k_j minus terms constant along the key j, which softmax cancels:
//                            s xn_i^T Wq^T bk and s bq . bk)
//   y_i = x_i + sum_j P_ij g_j,   g_j = Wg xn_j + cb,   Wg = Wp Wv, cb = Wp bv + bp   (sum_j P_ij = 1)
//
// The folded matrices are products of the block's own weights, formed once in float64 (attn_fold_kernel)
// and rounded to fp32; g is a plain static-weight GEMM (linear_k32 with the GroupNorm prologue, writing
// g^T as the fp16x2 v-plane [B][2][C][L]); this kernel does T, S, softmax, P g and the residual for 128
// query tokens of one image. Per image that is 4 GEMMs of 256^3 (T, S, g, Pg) instead of the reference's
// 6 (q, k, v, S, Pv, proj): 134 instead of 201 MFLOP, no q / k / v planes in HBM.
//
// Work-group = (image, 128 query tokens), 4 waves of 32 queries, one wave per SIMD (up to 512 VGPR+AGPR:
// the wave keeps T's split pieces (128 registers) next to S (128), then P's pieces next to O (128 each)).
// Every contraction is C^T = A B^T-style with the 256-row operand (At rows c', the keys' xn rows, g^T rows
// d) staged per 32-deep k-step through LDS in the fragment-image layout of split_conv_weights (shared by
// the four waves, double buffered, loads two k-steps ahead in registers), and the wave's 32 query columns
// as the B operand from registers: v_mfma_f32_16x16x32_f16, fp16x2 products a1b0 + a0b1 + a0b0.
// The accumulators of one contraction are the next one's B operand directly: accumulator rows 4q + r of
// tiles (2ks, 2ks + 1) are k-step ks's lane-group q elements, i.e. the contraction index is permuted
// (k = 8q + e  <->  row 4q + (e & 3) + 16 (e >> 2)); the staged A images (keys' xn by channel, g^T by key)
// apply the same permutation when they are written, so no register shuffles.
//
// Scales (exact powers of two): xn x 2^ex, At / Wg rows by split_conv_weights' row scales, T per query by
// 2^eT (max |T| in [2^13, 2^14)), P x 2^14, g x 2^eg (the GEMM's plane epilogue).
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"

namespace dm {

namespace {

constexpr int kBL = 256;            // tokens (16 x 16)
constexpr int kBC = 256;            // channels
constexpr int kBQ = 128;            // query tokens per work-group
constexpr int kStepH = 16384;       // fp16 elements of one staged k-step image (256 rows x 32 k x 2 pieces)
constexpr int kOP = kBC + 4;        // fp32 pitch of the epilogue staging rows

typedef float fq __attribute__((ext_vector_type(4)));

// fragment-image offset (fp16 elements) of (row, lane group q, piece p) in a staged k-step, + e0
__device__ __forceinline__ int img_off(int row, int q, int p) {
  return (q >> 1) * 8192 + (row >> 5) * 1024 + p * 512 + (q & 1) * 256 + (row & 31) * 8;
}

__device__ __forceinline__ void split8(const float (&x)[8], f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const _Float16 h0 = (_Float16)x[e];
    hi[e] = h0;
    lo[e] = (_Float16)(x[e] - (float)h0);
  }
}

__device__ __forceinline__ void split4(const f4 x, f16x4& hi, f16x4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 h0 = (_Float16)x[e];
    hi[e] = h0;
    lo[e] = (_Float16)(x[e] - (float)h0);
  }
}

__device__ __forceinline__ void mma3(const f16x8 (&a)[2], const f16x8 (&b)[2], fq& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], acc, 0, 0, 0);
}

// One k-step of a 256-row x 32-column contraction: acc[t][qt] += A(tile t) B[qt] over 16 row tiles, the
// A fragments read from the staged image `img`, one tile ahead of its MFMAs.
__device__ __forceinline__ void kstep(const _Float16* img, int l16, int q, const f16x8 (&b)[2][2], fq (&acc)[16][2]) {
  const int base = (q >> 1) * 8192 + (q & 1) * 256 + l16 * 8;
  f16x8 a[2][2];
  auto rd = [&](int t, f16x8 (&dst)[2]) {
    const int o = base + (t >> 1) * 1024 + (t & 1) * 128;
    dst[0] = *reinterpret_cast<const f16x8*>(img + o);
    dst[1] = *reinterpret_cast<const f16x8*>(img + o + 512);
  };
  rd(0, a[0]);
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (t + 1 < 16) rd(t + 1, a[(t + 1) & 1]);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) mma3(a[t & 1], b[qt], acc[t][qt]);
  }
}

}  // namespace

// The folded weights of one attention block, float64 sums rounded once to fp32 (attn_block.hip header):
// at[c'][c] = s sum_d Wk[d][c'] Wq[d][c], w[c'] = s sum_d Wk[d][c'] bq[d], wg[d][c] = sum_e Wp[d][e] Wv[e][c],
// cb[d] = sum_e Wp[d][e] bv[e] + bp[d]. wqkv = [Wq; Wk; Wv] ([3C][C]), bqkv = [bq; bk; bv].
__global__ void attn_fold_kernel(const float* __restrict__ wqkv, const float* __restrict__ bqkv,
                                 const float* __restrict__ wp, const float* __restrict__ bp, int C, double s,
                                 float* __restrict__ at, float* __restrict__ w, float* __restrict__ wg,
                                 float* __restrict__ cb) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long CC = (long)C * C;
  const float* Wq = wqkv;
  const float* Wk = wqkv + CC;
  const float* Wv = wqkv + 2 * CC;
  if (id < CC) {  // at[c'][c]
    const int r = (int)(id / C), c = (int)(id % C);
    double acc = 0.0;
    for (int d = 0; d < C; ++d) acc += (double)Wk[(size_t)d * C + r] * (double)Wq[(size_t)d * C + c];
    at[id] = (float)(s * acc);
  } else if (id < 2 * CC) {  // wg[d][c]
    const long j = id - CC;
    const int d = (int)(j / C), c = (int)(j % C);
    double acc = 0.0;
    for (int e = 0; e < C; ++e) acc += (double)wp[(size_t)d * C + e] * (double)Wv[(size_t)e * C + c];
    wg[j] = (float)acc;
  } else if (id < 2 * CC + C) {  // w[c']
    const int r = (int)(id - 2 * CC);
    double acc = 0.0;
    for (int d = 0; d < C; ++d) acc += (double)Wk[(size_t)d * C + r] * (double)bqkv[d];
    w[r] = (float)(s * acc);
  } else if (id < 2 * CC + 2 * C) {  // cb[d]
    const int d = (int)(id - 2 * CC - C);
    double acc = 0.0;
    for (int e = 0; e < C; ++e) acc += (double)wp[(size_t)d * C + e] * (double)bqkv[2 * C + e];
    cb[d] = (float)(acc + (double)bp[d]);
  }
}

namespace {

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) attn_block_kernel(AttnBlockArgs a) {
  // LDS: two staged k-step images (64 KB) during the contractions; the epilogue's O rows (130 KB) after
  __shared__ __attribute__((aligned(16))) float lds[kBQ * kOP];
  __shared__ __attribute__((aligned(16))) float tab[2][kBC];   // GroupNorm scale / shift of the image
  static_assert(2 * kStepH * 2 <= kBQ * kOP * 4, "two k-step images fit the epilogue region");
  _Float16* stg = reinterpret_cast<_Float16*>(lds);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int b = bid >> 1, qh = bid & 1;
  const float* xb = a.x + (size_t)b * kBL * a.x_pitch;
  const int qrow0 = qh * kBQ + wave * 32;          // this wave's first query token
  const float xs = ldexpf(1.f, a.ex);
  bool bad = false;

  for (int i = t; i < kBC; i += 256) {
    tab[0][i] = a.gsc[(size_t)b * kBC + i];
    tab[1][i] = a.gsh[(size_t)b * kBC + i];
  }

  // ------------------------------------------------------------------ staging (8 x 16 B per thread per k-step)
  f4 rg[2][8];
  // At image rows (a verbatim copy of the k-step's two 16-slices of split_conv_weights' image)
  auto load_at = [&](int kk, f4 (&r)[8]) {
    const f4* src = reinterpret_cast<const f4*>(a.at_img + (size_t)kk * kStepH);
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = src[t + 256 * u];
  };
  auto store_at = [&](int buf, const f4 (&r)[8]) {
    f4* dst = reinterpret_cast<f4*>(stg + buf * kStepH);
#pragma unroll
    for (int u = 0; u < 8; ++u) dst[t + 256 * u] = r[u];
  };
  // the keys' x rows, channels 32 ks + 4 u .. + 3 (u = g + 4 hi): lane group g, lanes 8 hi .. + 7 hold 8
  // consecutive keys; slot s = 0 .. 7 of this wave covers keys 64 wave + 8 s ..
  const int kg = lane >> 4, khi = (lane >> 3) & 1, kkey = lane & 7;
  auto load_keys = [&](int ks, f4 (&r)[8]) {
    const int u = kg + 4 * khi;
#pragma unroll
    for (int s = 0; s < 8; ++s)
      r[s] = *reinterpret_cast<const f4*>(xb + (size_t)(64 * wave + 8 * s + kkey) * a.x_pitch + 32 * ks + 4 * u);
  };
  auto store_keys = [&](int ks, int buf, const f4 (&r)[8]) {
    const int u = kg + 4 * khi;
    const int c = 32 * ks + 4 * u;
    const f4 sc = *reinterpret_cast<const f4*>(&tab[0][c]), sh = *reinterpret_cast<const f4*>(&tab[1][c]);
    _Float16* img = stg + buf * kStepH;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      f4 v = r[s];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (v[e] * sc[e] + sh[e]) * xs;
      bad |= fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))) > 65504.f;
      f16x4 hi, lo;
      split4(v, hi, lo);
      const int key = 64 * wave + 8 * s + kkey;
      const int o = img_off(key, kg, 0) + 4 * khi;
      *reinterpret_cast<f16x4*>(img + o) = hi;
      *reinterpret_cast<f16x4*>(img + o + 512) = lo;
    }
  };
  // g^T rows d (the v-plane [2][C][L] of this image), keys 32 ks + 8 u' .. + 7 (u' = 2 hi + g1, piece g0)
  const _Float16* gb = a.g_plane + (size_t)b * 2 * kBC * kBL;
  const int gu = 2 * khi + (kg & 1), gp = kg >> 1;
  auto load_g = [&](int ks, f4 (&r)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
      r[s] = *reinterpret_cast<const f4*>(gb + ((size_t)gp * kBC + 64 * wave + 8 * s + kkey) * kBL + 32 * ks + 8 * gu);
  };
  auto store_g = [&](int buf, const f4 (&r)[8]) {
    // keys 8 u' .. + 3 -> lane group 2 (u' & 1), e0 = 4 (u' >> 1); keys 8 u' + 4 .. + 7 -> lane group + 1
    _Float16* img = stg + buf * kStepH;
    const int q0 = 2 * (gu & 1), e0 = 4 * (gu >> 1);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int d = 64 * wave + 8 * s + kkey;
      const f4 v = r[s];
      *reinterpret_cast<float2*>(img + img_off(d, q0, gp) + e0) = make_float2(v[0], v[1]);
      *reinterpret_cast<float2*>(img + img_off(d, q0 + 1, gp) + e0) = make_float2(v[2], v[3]);
    }
  };

  fq acc[16][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = fq{0.f, 0.f, 0.f, 0.f};
  };

  // ------------------------------------------------------------------ 1. T^T = At xn^T (+ w)
  // B operand: the wave's queries (lane l16 of tile qt), channels 32 kk + 8 q .. + 7, GroupNorm'd and split
  f4 rx[2][2][2];   // [set][qt][half]
  auto load_xq = [&](int kk, f4 (&r)[2][2]) {
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float* p = xb + (size_t)(qrow0 + 16 * qt + l16) * a.x_pitch + 32 * kk + 8 * q;
      r[qt][0] = *reinterpret_cast<const f4*>(p);
      r[qt][1] = *reinterpret_cast<const f4*>(p + 4);
    }
  };
  auto xq_frag = [&](int kk, const f4 (&r)[2][2], f16x8 (&bf)[2][2]) {
    const int c = 32 * kk + 8 * q;
    const f4 s0 = *reinterpret_cast<const f4*>(&tab[0][c]), s1 = *reinterpret_cast<const f4*>(&tab[0][c + 4]);
    const f4 h0 = *reinterpret_cast<const f4*>(&tab[1][c]), h1 = *reinterpret_cast<const f4*>(&tab[1][c + 4]);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (r[qt][0][e] * s0[e] + h0[e]) * xs;
        v[4 + e] = (r[qt][1][e] * s1[e] + h1[e]) * xs;
      }
      float m = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
      bad |= m > 65504.f;
      split8(v, bf[qt][0], bf[qt][1]);
    }
  };

  zero_acc();
  load_at(0, rg[0]);
  load_at(1, rg[1]);
  load_xq(0, rx[0]);
  load_xq(1, rx[1]);
  store_at(0, rg[0]);
  __syncthreads();   // tab and the first image
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    if (kk + 2 < 8) load_at(kk + 2, rg[kk & 1]);
    f16x8 bf[2][2];
    xq_frag(kk, rx[kk & 1], bf);
    if (kk + 2 < 8) load_xq(kk + 2, rx[kk & 1]);
    kstep(stg + (kk & 1) * kStepH, l16, q, bf, acc);
    if (kk + 1 < 8) store_at((kk + 1) & 1, rg[(kk + 1) & 1]);
    __syncthreads();
  }
  // keys' rows for the S contraction: first two k-steps in flight during the T epilogue
  load_keys(0, rg[0]);
  load_keys(1, rg[1]);

  // T = acc * rowscale * 2^-ex + w; per query the exponent eT with max |T| 2^eT in [2^13, 2^14)
  f16x8 tp[8][2][2];   // [k-step][qt][piece]: T's split pieces as the S contraction's B operand
  float tun[2];        // 2^-(ex + eT) per query tile
  {
    const float xun = ldexpf(1.f, -a.ex);
    float mx[2] = {0.f, 0.f};
#pragma unroll
    for (int ct = 0; ct < 16; ++ct) {
      const f4 rs = *reinterpret_cast<const f4*>(a.at_rowscale + 16 * ct + 4 * q);
      const f4 wv = *reinterpret_cast<const f4*>(a.w + 16 * ct + 4 * q);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[ct][qt][r] * (rs[r] * xun) + wv[r];
          acc[ct][qt][r] = v;
          mx[qt] = fmaxf(mx[qt], fabsf(v));
        }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float m = fmaxf(mx[qt], __shfl_xor(mx[qt], 16));
      m = fmaxf(m, __shfl_xor(m, 32));
      int E = 0;
      (void)frexpf(m, &E);
      const int eT = m > 0.f ? 14 - E : 0;
      const float sc = ldexpf(1.f, eT);
      tun[qt] = ldexpf(1.f, -(a.ex + eT));
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[2 * ks][qt][e] * sc;
          v[4 + e] = acc[2 * ks + 1][qt][e] * sc;
        }
        split8(v, tp[ks][qt][0], tp[ks][qt][1]);
      }
    }
  }

  // ------------------------------------------------------------------ 2. S^T = xn_keys T^T
  store_keys(0, 0, rg[0]);
  __syncthreads();
  zero_acc();
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    if (ks + 2 < 8) load_keys(ks + 2, rg[ks & 1]);
    kstep(stg + (ks & 1) * kStepH, l16, q, tp[ks], acc);
    if (ks + 1 < 8) store_keys(ks + 1, (ks + 1) & 1, rg[(ks + 1) & 1]);
    __syncthreads();
  }
  load_g(0, rg[0]);
  load_g(1, rg[1]);

  // ------------------------------------------------------------------ 3. softmax over the keys (per query lane)
  // S = acc 2^-(ex + eT); p = exp2(S log2 e - max) on the hardware exp2 (scale folded into one FMA), P = p / sum
  f16x8 pp[8][2][2];   // [k-step][qt][piece]: P x 2^14 as the Pg contraction's B operand
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float sl2 = tun[qt] * 1.4426950408889634f;
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 16; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) m = fmaxf(m, acc[kt][qt][r]);
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    const float mb = -m * sl2;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 16; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[kt][qt][r], sl2, mb));
        acc[kt][qt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 16384.f / sum;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * ks][qt][e] * inv;
        v[4 + e] = acc[2 * ks + 1][qt][e] * inv;
      }
      split8(v, pp[ks][qt][0], pp[ks][qt][1]);
    }
  }

  // ------------------------------------------------------------------ 4. O^T = g^T P^T
  store_g(0, rg[0]);
  __syncthreads();
  zero_acc();
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    if (ks + 2 < 8) load_g(ks + 2, rg[ks & 1]);
    kstep(stg + (ks & 1) * kStepH, l16, q, pp[ks], acc);
    if (ks + 1 < 8) store_g((ks + 1) & 1, rg[(ks + 1) & 1]);
    __syncthreads();
  }
  if (bad && a.range_flag) *a.range_flag = 1;

  // ------------------------------------------------------------------ 5. y = x + O, GroupNorm statistics
  // O rows to LDS ([128 queries][C] fp32): lane (l16, q) holds d = 16 dt + 4 q .. + 3 of query 16 qt + l16
  const float oun = ldexpf(1.f, -(a.eg + 14));
#pragma unroll
  for (int dt = 0; dt < 16; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      *reinterpret_cast<fq*>(lds + (wave * 32 + 16 * qt + l16) * kOP + 16 * dt + 4 * q) = acc[dt][qt] * oun;
  __syncthreads();
  // wave (chunk c = 64 rows, column half h): lane = 4 channels of one row, two rows per pass
  const int ch = wave >> 1, chalf = wave & 1;
  const int c4 = lane & 31, rsub = lane >> 5;
  const int col = 128 * chalf + 4 * c4;
  const int tok0 = qh * kBQ + 64 * ch;
  double gs[4] = {0.0, 0.0, 0.0, 0.0}, gq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int i = 0; i < 32; ++i) {
    const int row = 64 * ch + 2 * i + rsub;          // work-group-local query row
    const int tok = tok0 + 2 * i + rsub;
    const f4 o = *reinterpret_cast<const f4*>(lds + row * kOP + col);
    const f4 xr = *reinterpret_cast<const f4*>(xb + (size_t)tok * a.x_pitch + col);
    const f4 yv = xr + o;
    *reinterpret_cast<f4*>(a.y + ((size_t)b * kBL + tok) * a.y_pitch + col) = yv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gs[e] += (double)yv[e];
      gq[e] += (double)yv[e] * yv[e];
    }
  }
  if (a.gn_part) {
    double s = gs[0] + gs[1] + gs[2] + gs[3], qq = gq[0] + gq[1] + gq[2] + gq[3];
    s += __shfl_xor(s, 32);
    qq += __shfl_xor(qq, 32);
    const int cpg = kBC / a.gn_G;   // 4 .. 32 channels: cpg / 4 lanes
    for (int o = 1; o < cpg / 4; o <<= 1) {
      s += __shfl_xor(s, o);
      qq += __shfl_xor(qq, o);
    }
    if (rsub == 0 && (c4 % (cpg / 4)) == 0)
      a.gn_part[((size_t)b * (kBL / 64) + (tok0 >> 6)) * a.gn_G + col / cpg] = make_double2(s, qq);
  }
}

}  // namespace

bool attn_block_ok(int L, int C, int heads) { return L == kBL && C == kBC && heads == 1; }

int attn_fold(const float* wqkv, const float* bqkv, const float* wproj, const float* bproj, int C, double scale,
              float* at, float* w, float* wg, float* cb, hipStream_t st) {
  DM_REQUIRE(C > 0 && wqkv && bqkv && wproj && bproj && at && w && wg && cb, "attention fold: null argument");
  const long n = 2L * C * C + 2L * C;
  hipLaunchKernelGGL(attn_fold_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wqkv, bqkv, wproj, bproj,
                     C, scale, at, w, wg, cb);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int attn_block(const AttnBlockArgs& a, hipStream_t st) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  DM_REQUIRE(a.B > 0 && a.x && a.y && a.gsc && a.gsh && a.at_img && a.at_rowscale && a.w && a.g_plane,
             "attention block: null argument");
  DM_REQUIRE(a.x_pitch % 4 == 0 && a.y_pitch % 4 == 0 && al16(a.x) && al16(a.y) && al16(a.gsc) && al16(a.gsh) &&
                 al16(a.at_img) && al16(a.at_rowscale) && al16(a.w) && al16(a.g_plane),
             "attention block: 16-byte aligned rows");
  DM_REQUIRE(!a.gn_part || (a.gn_G > 0 && kBC % a.gn_G == 0 && kBC / a.gn_G >= 4 && kBC / a.gn_G <= 32 &&
                            ((kBC / a.gn_G) & (kBC / a.gn_G - 1)) == 0),
             "attention block: GroupNorm statistics need groups of 4, 8, 16 or 32 channels");
  hipLaunchKernelGGL(attn_block_kernel, dim3(a.B * (kBL / kBQ)), dim3(256), 0, st, a);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
