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
// and rounded to fp32. (Round 4's first form computed g with a separate static-weight GEMM into an fp16x2 plane;
// variant 3 below moved the projection after the key pass -- the values are xn itself -- and variant 4, the
// default, runs variant 3's arithmetic on 8 waves; the g-plane form was removed in round 5.)
//
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

#ifdef DM_K32_STAMPS
// Diagnostic build only (tools/ab_stamps.py): per work-group, wave 0's s_memtime at the phase boundaries and
// s_memrealtime at start / end, kept in scalar registers and written to this buffer at the end (no scheduling
// barriers and no stores at the boundaries, so the stamped build keeps the product kernel's registers: round 4's
// per-boundary stores spilled it).
__device__ unsigned long long g_ab_stamps[4096][10];
#define AB_DECL unsigned long long ab_t[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define AB_STAMP(k) (ab_t[k] = __builtin_amdgcn_s_memtime())
#define AB_RSTAMP(k) (ab_t[k] = __builtin_amdgcn_s_memrealtime())
#define AB_FLUSH                                                                         \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                           \
      for (int k_ = 0; k_ < 10; ++k_) g_ab_stamps[blockIdx.x][k_] = ab_t[k_];             \
  } while (0)
#else
#define AB_DECL do {} while (0)
#define AB_STAMP(k) do {} while (0)
#define AB_RSTAMP(k) do {} while (0)
#define AB_FLUSH do {} while (0)
#endif

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
// A fragments read from the staged image `img`, one tile ahead of its MFMAs. mid(t) runs after tile t's
// MFMAs are issued: the staging of later k-steps (global loads, LDS stores into the other image, the
// GroupNorm + split VALU work) placed between MFMAs, so one wave per SIMD keeps its matrix pipe fed.
template <class MID>
__device__ __forceinline__ void kstep(const _Float16* img, int l16, int q, const f16x8 (&b)[2][2], fq (&acc)[16][2],
                                      MID&& mid) {
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
    mid(t);
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

// ======================================================================================================
// Variant 3 (default): no g GEMM. The values are xn itself and the folded projection comes after:
//   y_i = x_i + Wg (sum_j P_ij xn_j) + cb        (sum_j P_ij = 1)
// so per work-group: T (At xn_q^T), then ONE pass over the keys in chunks of 32 -- S^T for the chunk, an
// online softmax update (running maximum / sum per query, the O accumulators rescaled), O^T += xn_K^T P^T --
// then Y^T = Wg' O^T and the residual. Per image and query half 4 GEMMs of 128 x 256 x 256 (T, S, P xn, Wg O):
// the g GEMM kernel and its fp16x2 plane (67 MB written, read twice at B = 256) are gone, and the keys' x rows
// are staged once for S and P xn together.
//
// The keys' chunk image holds 32 keys x 256 channels (two fp16 pieces, 544-B rows: conflict-free for both
// the 16x16x32 A-operand row reads of S and the ds_read_b64_tr_b16 transposed reads of P xn). Its channel
// order is the accumulator permutation pi within every 32 channels (storage position 32 g + 8 q + e holds
// channel 32 g + 4 q + (e & 3) + 16 (e >> 2)), so T's accumulators are S's B operand as they lie; O^T's rows
// come out in storage order, and Wg' = Wg with its columns permuted by pi o pi within 32-groups (made at the
// fold) takes them as they lie as the B operand of the projection.
constexpr int kKP = 272;            // fp16 pitch of a key row of one piece (544 B = 136 dwords: 8 mod 64)
constexpr int kKPiece = 32 * kKP;   // one piece of a key-chunk image
constexpr int kKImg = 2 * kKPiece;  // fp16 elements of a key-chunk image (34 KB)

typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));

// ds_read_b64_tr_b16 (gfx950): lane 4 q' + p of each 16-lane group addresses row q' of a 4-row block, columns
// 4 p .. 4 p + 3; lane i of the group receives column i of the 4 rows (cdna_hip_programming.md T10)
__device__ __forceinline__ f16x4_t lds_tr16(const _Float16* p) {
  typedef __fp16 hv4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
  typedef __attribute__((address_space(3))) hv4 lds_hv4;
  const hv4 r = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_hv4*)(p));
  return __builtin_bit_cast(f16x4_t, r);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) attn_block3_kernel(AttnBlockArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kBQ * kOP];
  __shared__ __attribute__((aligned(16))) float tab[2][kBC];
  static_assert(2 * kKImg * 2 <= kBQ * kOP * 4, "two key-chunk images fit the epilogue region");
  _Float16* stg = reinterpret_cast<_Float16*>(lds);
  AB_DECL;
  AB_RSTAMP(8);
  AB_STAMP(0);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int b = bid >> 1, qh = bid & 1;
  const float* xb = a.x + (size_t)b * kBL * a.x_pitch;
  const int qrow0 = qh * kBQ + wave * 32;
  const float xs = ldexpf(1.f, a.ex);
  bool bad = false;
  for (int i = t; i < kBC; i += 256) {
    tab[0][i] = a.gsc[(size_t)b * kBC + i];
    tab[1][i] = a.gsh[(size_t)b * kBC + i];
  }

  f4 rg[2][8];
  // weight images (At, Wg'): verbatim copies of split_conv_weights' k-step regions
  auto load_w = [&](const _Float16* img, int kk, int s, f4& r) {
    r = reinterpret_cast<const f4*>(img + (size_t)kk * kStepH)[t + 256 * s];
  };
  auto store_w = [&](int buf, int s, const f4& r) { reinterpret_cast<f4*>(stg + buf * kStepH)[t + 256 * s] = r; };
  // key chunk kc = keys 32 kc .. + 31, all channels. Slot s = 32-channel group s; lane: run krun of 4 channels,
  // key kkey3 (a 16-lane group covers keys {k0, k0 + 2} x 8 runs: conflict-free 8-B LDS stores; a wave
  // instruction reads 8 whole 128-B row pieces)
  const int krun = lane & 7, kk2 = (lane >> 3) & 1, kgrp = lane >> 4;
  const int kkey3 = 8 * wave + 4 * (kgrp >> 1) + 2 * kk2 + (kgrp & 1);   // 0 .. 31 within the chunk
  auto load_k = [&](int kc, int s, f4& r) {
    r = *reinterpret_cast<const f4*>(xb + (size_t)(32 * kc + kkey3) * a.x_pitch + 32 * s + 4 * krun);
  };
  auto store_k = [&](int buf, int s, const f4& r) {
    const int c = 32 * s + 4 * krun;
    const f4 sc = *reinterpret_cast<const f4*>(&tab[0][c]), sh = *reinterpret_cast<const f4*>(&tab[1][c]);
    f4 v = r;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (v[e] * sc[e] + sh[e]) * xs;
    bad |= fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))) > 65504.f;
    f16x4 hi, lo;
    split4(v, hi, lo);
    // channels 4 krun .. + 3 of the 32-group -> storage positions 8 (krun & 3) + 4 (krun >> 2) ..
    _Float16* dst = stg + buf * kKImg + kkey3 * kKP + 32 * s + 8 * (krun & 3) + 4 * (krun >> 2);
    *reinterpret_cast<f16x4*>(dst) = hi;
    *reinterpret_cast<f16x4*>(dst + kKPiece) = lo;
  };

  fq acc[16][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = fq{0.f, 0.f, 0.f, 0.f};
  };

  // ------------------------------------------------------------------ 1. T^T = At xn_q^T (+ w)
  f4 rx[2][2][2];
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
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    load_w(a.at_img, 0, u, rg[0][u]);
    load_w(a.at_img, 1, u, rg[1][u]);
  }
  load_xq(0, rx[0]);
  load_xq(1, rx[1]);
#pragma unroll
  for (int u = 0; u < 8; ++u) store_w(0, u, rg[0][u]);
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    f16x8 bf[2][2];
    xq_frag(kk, rx[kk & 1], bf);
    if (kk + 2 < 8) load_xq(kk + 2, rx[kk & 1]);
    kstep(stg + (kk & 1) * kStepH, l16, q, bf, acc, [&](int tt) {
      if (tt < 8) {
        if (kk + 2 < 8) load_w(a.at_img, kk + 2, tt, rg[kk & 1][tt]);
      } else if (kk + 1 < 8) {
        store_w((kk + 1) & 1, tt - 8, rg[(kk + 1) & 1][tt - 8]);
      }
    });
    __syncthreads();
  }
  AB_STAMP(1);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    load_k(0, u, rg[0][u]);
    load_k(1, u, rg[1][u]);
  }
  f16x8 tp[8][2][2];
  float tun[2];
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
  AB_STAMP(2);

  // ------------------------------------------------------------------ 2. one pass over the keys (chunks of 32)
  // S^T chunk [2 key tiles][qt] = xn_chunk T^T; online softmax; O^T [16 storage tiles][qt] += xn_chunk^T P^T
#pragma unroll
  for (int u = 0; u < 8; ++u) store_k(0, u, rg[0][u]);
  __syncthreads();
  zero_acc();   // O^T accumulators
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  const float sl2[2] = {tun[0] * 1.4426950408889634f, tun[1] * 1.4426950408889634f};
#pragma unroll
  for (int kc = 0; kc < 8; ++kc) {
    const _Float16* img = stg + (kc & 1) * kKImg;
    // S^T: A = the chunk's key rows (tile kt: keys 16 kt + l16), k = storage positions 32 ks + 8 q ..
    fq sacc[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) sacc[kt][qt] = fq{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const _Float16* pr = img + (16 * kt + l16) * kKP + 32 * ks + 8 * q;
        f16x8 av[2];
        av[0] = *reinterpret_cast<const f16x8*>(pr);
        av[1] = *reinterpret_cast<const f16x8*>(pr + kKPiece);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) mma3(av, tp[ks][qt], sacc[kt][qt]);
      }
      // staging between the S MFMAs: the loads of chunk kc + 2 (this thread's slots)
      if (kc + 2 < 8) load_k(kc + 2, ks, rg[kc & 1][ks]);
    }
    // online softmax of the chunk (per query lane; the 4 lane groups q hold 8 of its 32 keys each)
    f16x8 pp[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = fmaxf(fmaxf(fmaxf(sacc[0][qt][0], sacc[0][qt][1]), fmaxf(sacc[0][qt][2], sacc[0][qt][3])),
                       fmaxf(fmaxf(sacc[1][qt][0], sacc[1][qt][1]), fmaxf(sacc[1][qt][2], sacc[1][qt][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float m_new = fmaxf(m_run[qt], mx * sl2[qt]);
      const float corr = __builtin_amdgcn_exp2f(m_run[qt] - m_new);
      m_run[qt] = m_new;
      float ls = 0.f, v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[0][qt][e], sl2[qt], -m_new));
        v[4 + e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[1][qt][e], sl2[qt], -m_new));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ls += v[e];
        v[e] *= 16384.f;
      }
      l_run[qt] = l_run[qt] * corr + ls;
      split8(v, pp[qt][0], pp[qt][1]);
      // (a wave-uniform skip of this rescale when no running maximum moved made the compiler spill 2.2 KB
      // per lane: the accumulators live in AGPRs, and the branch forced copies of all of them)
      if (kc > 0) {
#pragma unroll
        for (int ot = 0; ot < 16; ++ot) acc[ot][qt] *= corr;
      }
    }
    // O^T += xn_chunk^T P^T: A rows = storage positions 16 ot + l16 (transposed reads of the key rows), k = the
    // chunk's keys in P's accumulator permutation (lane group q: keys 4 q .. + 3, then 16 + 4 q .. + 3)
    {
      const _Float16* pt = img + (4 * q + (l16 >> 2)) * kKP + 4 * (l16 & 3);
#pragma unroll
      for (int ot = 0; ot < 16; ++ot) {
        f16x8 av[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4_t lo4 = lds_tr16(pt + p * kKPiece + 16 * ot);
          const f16x4_t hi4 = lds_tr16(pt + p * kKPiece + 16 * kKP + 16 * ot);
          av[p] = f16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        }
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) mma3(av, pp[qt], acc[ot][qt]);
        // the stores of chunk kc + 1 (into the other image) between the P xn MFMAs
        if (ot >= 8 && kc + 1 < 8) store_k((kc + 1) & 1, ot - 8, rg[(kc + 1) & 1][ot - 8]);
      }
    }
    __syncthreads();
  }
  AB_STAMP(3);
  // Wg' images of the projection: the first two k-steps in flight during the O finalize
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    load_w(a.wg_img, 0, u, rg[0][u]);
    load_w(a.wg_img, 1, u, rg[1][u]);
  }
  // O x 2^ex = acc / (2^14 l) (the staged keys carry xn x 2^ex; rows in storage order) -> split pieces as the
  // projection's B operand
  f16x8 op[8][2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = l_run[qt] + __shfl_xor(l_run[qt], 16);
    l += __shfl_xor(l, 32);
    const float sc = 1.f / (16384.f * l);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * ks][qt][e] * sc;
        v[4 + e] = acc[2 * ks + 1][qt][e] * sc;
      }
      split8(v, op[ks][qt][0], op[ks][qt][1]);
    }
  }
  AB_STAMP(4);

  // ------------------------------------------------------------------ 3. Y^T = Wg' O^T
#pragma unroll
  for (int u = 0; u < 8; ++u) store_w(0, u, rg[0][u]);
  __syncthreads();
  zero_acc();
  const int ch = wave >> 1, chalf = wave & 1;
  const int c4 = lane & 31, rsub = lane >> 5;
  const int col = 128 * chalf + 4 * c4;
  const int tok0 = qh * kBQ + 64 * ch;
  auto load_res = [&](int i, f4& r) {
    r = *reinterpret_cast<const f4*>(xb + (size_t)(tok0 + 2 * i + rsub) * a.x_pitch + col);
  };
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    kstep(stg + (kk & 1) * kStepH, l16, q, op[kk], acc, [&](int tt) {
      if (tt < 8) {
        if (kk + 2 < 8) load_w(a.wg_img, kk + 2, tt, rg[kk & 1][tt]);
        else load_res(8 * (kk - 6) + tt, rg[kk & 1][tt]);   // residual rows 0 .. 15
      } else if (kk + 1 < 8) {
        store_w((kk + 1) & 1, tt - 8, rg[(kk + 1) & 1][tt - 8]);
      }
    });
    __syncthreads();
  }
  f4 xr2[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) load_res(16 + i, xr2[i]);
  if (bad && a.range_flag) *a.range_flag = 1;
  AB_STAMP(5);

  // ------------------------------------------------------------------ 4. y = x + Y + cb, GroupNorm statistics
  const float yun = ldexpf(1.f, -a.ex);
#pragma unroll
  for (int dt = 0; dt < 16; ++dt) {
    const f4 rs = *reinterpret_cast<const f4*>(a.wg_rowscale + 16 * dt + 4 * q);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      *reinterpret_cast<fq*>(lds + (wave * 32 + 16 * qt + l16) * kOP + 16 * dt + 4 * q) = acc[dt][qt] * (rs * yun);
  }
  __syncthreads();
  const f4 cb4 = *reinterpret_cast<const f4*>(a.cb + col);
  double gs[4] = {0.0, 0.0, 0.0, 0.0}, gq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int tok = tok0 + 2 * i + rsub;
    const f4 o = *reinterpret_cast<const f4*>(lds + (64 * ch + 2 * i + rsub) * kOP + col);
    const f4 xr = i < 8 ? rg[0][i & 7] : i < 16 ? rg[1][i & 7] : xr2[i & 15];
    const f4 yv = xr + (o + cb4);
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
    const int cpg = kBC / a.gn_G;
    for (int o = 1; o < cpg / 4; o <<= 1) {
      s += __shfl_xor(s, o);
      qq += __shfl_xor(qq, o);
    }
    if (rsub == 0 && (c4 % (cpg / 4)) == 0)
      a.gn_part[((size_t)b * (kBL / 64) + (tok0 >> 6)) * a.gn_G + col / cpg] = make_double2(s, qq);
  }
  AB_STAMP(6);
  AB_RSTAMP(9);
  AB_FLUSH;
}

// ---- variant 4: attn_block3_kernel's algorithm with 8 waves of 16 queries (512 threads, 128 queries per
// work-group, one work-group per CU, two waves per SIMD). Per wave half the state of variant 3 (T pieces 64,
// O / Y accumulators 64 registers, 4 staging slots per thread instead of 8), so two waves fit a SIMD and one
// wave's LDS / L2 waits, softmax and staging overlap the other's MFMAs, where variant 3's single wave per SIMD
// left its matrix pipe idle through them (0.27 of the fp16x2 issue peak). The A operands (At / Wg' rows, the
// keys' xn) are read once per 16 queries instead of per 32: 171 B/clk/CU of ds_read_b128 at the full MFMA rate,
// within the LDS's 256. Same fragment images, staging layouts, accumulator permutations and scales as variant
// 3; every output element's MFMA sequence is variant 3's, so the two give the same bits.
template <class MID>
__device__ __forceinline__ void kstep1(const _Float16* img, int l16, int q, const f16x8 (&b)[2], fq (&acc)[16],
                                       MID&& mid) {
  const int base = (q >> 1) * 8192 + (q & 1) * 256 + l16 * 8;
  f16x8 a[3][2];
  auto rd = [&](int t, f16x8 (&dst)[2]) {
    const int o = base + (t >> 1) * 1024 + (t & 1) * 128;
    dst[0] = *reinterpret_cast<const f16x8*>(img + o);
    dst[1] = *reinterpret_cast<const f16x8*>(img + o + 512);
  };
  rd(0, a[0]);
  rd(1, a[1]);
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (t + 2 < 16) rd(t + 2, a[(t + 2) % 3]);
    mma3(a[t % 3], b, acc[t]);
    mid(t);
  }
}

// NWV = 8 waves of 16 queries per work-group (variant 4: 128 queries, one work-group per CU; the 4-wave form on
// 64-query work-groups and the software-pipelined / read-ahead key passes measured neutral or negative and were
// removed in round 5). (A wave-uniform skip of the O rescale when no running maximum moved spills 572 B per lane
// here, as in variant 3.)
template <int NWV>
__global__ void __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) attn_block4_kernel(AttnBlockArgs a) {
  constexpr int NT = NWV * 64, QB = 16 * NWV, NS = 2048 / NT;   // threads, queries, staging slots per thread
  // staging register sets: 2 (loads two k-steps / key chunks ahead) with 4 slots per thread, 1 (one ahead) with 8
  constexpr int RD = NS == 4 ? 2 : 1;
  constexpr int LDSF = QB * kOP > kKImg ? QB * kOP : kKImg;     // floats: epilogue rows / two key-chunk images
  static_assert(2 * kStepH <= 2 * LDSF && 2 * kKImg <= 2 * LDSF, "staging fits");
  __shared__ __attribute__((aligned(16))) float lds[LDSF];
  __shared__ __attribute__((aligned(16))) float tab[2][kBC];
  _Float16* stg = reinterpret_cast<_Float16*>(lds);
  AB_DECL;
  AB_RSTAMP(8);
  AB_STAMP(0);

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int b = bid / (kBL / QB), qh = bid - b * (kBL / QB);
  const float* xb = a.x + (size_t)b * kBL * a.x_pitch;
  const int qrow0 = qh * QB + wave * 16;   // this wave's 16 queries
  const float xs = ldexpf(1.f, a.ex);
  bool bad = false;
  if (a.gin_part) {  // gn_finalize (gn.hip) for this image's channels, same expressions
    const int cpg = kBC / a.gin_G;
    const double n = (double)kBL * cpg;
    for (int c = t; c < kBC; c += NT) {
      const int g = c / cpg;
      double s1 = 0, s2 = 0;
      for (int k = 0; k < a.gin_nchunk; ++k) {
        const double2 v = a.gin_part[((size_t)b * a.gin_nchunk + k) * a.gin_G + g];
        s1 += v.x;
        s2 += v.y;
      }
      const double m = s1 / n;
      double var = s2 / n - m * m;
      if (var < 0) var = 0;
      const float mu = (float)m;
      const float rs = (float)(1.0 / sqrt(var + (double)a.gin_eps));
      const float sc = rs * (a.gin_gamma ? a.gin_gamma[c] : 1.0f);
      tab[0][c] = sc;
      tab[1][c] = -sc * mu + (a.gin_beta ? a.gin_beta[c] : 0.0f);
    }
  } else {
    for (int i = t; i < kBC; i += NT) {
      tab[0][i] = a.gsc[(size_t)b * kBC + i];
      tab[1][i] = a.gsh[(size_t)b * kBC + i];
    }
  }

  f4 rg[RD][NS];
  // weight images (At, Wg'): verbatim copies of split_conv_weights' k-step regions, NS x 16 B per thread
  auto load_w = [&](const _Float16* img, int kk, int s, f4& r) {
    r = reinterpret_cast<const f4*>(img + (size_t)kk * kStepH)[t + NT * s];
  };
  auto store_w = [&](int buf, int s, const f4& r) { reinterpret_cast<f4*>(stg + buf * kStepH)[t + NT * s] = r; };
  // key chunk kc: variant 3's key / run mapping on wave & 3; with 8 waves, waves 0-3 take the 32-channel
  // groups 0-3 and waves 4-7 groups 4-7 (slot u = group 4 (wave >> 2) + u); with 4 waves every thread all 8
  const int krun = lane & 7, kk2 = (lane >> 3) & 1, kgrp = lane >> 4;
  const int kkey3 = 8 * (wave & 3) + 4 * (kgrp >> 1) + 2 * kk2 + (kgrp & 1);
  const int sg0 = NWV == 8 ? 4 * (wave >> 2) : 0;
  // staging slot of the mid-step callbacks: NS = 4 at even tiles / key steps, NS = 8 at every one
  constexpr int SD = 8 / NS;
  auto load_k = [&](int kc, int u, f4& r) {
    r = *reinterpret_cast<const f4*>(xb + (size_t)(32 * kc + kkey3) * a.x_pitch + 32 * (sg0 + u) + 4 * krun);
  };
  auto store_k = [&](int buf, int u, const f4& r) {
    const int s = sg0 + u, c = 32 * s + 4 * krun;
    const f4 sc = *reinterpret_cast<const f4*>(&tab[0][c]), sh = *reinterpret_cast<const f4*>(&tab[1][c]);
    f4 v = r;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (v[e] * sc[e] + sh[e]) * xs;
    bad |= fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))) > 65504.f;
    f16x4 hi, lo;
    split4(v, hi, lo);
    _Float16* dst = stg + buf * kKImg + kkey3 * kKP + 32 * s + 8 * (krun & 3) + 4 * (krun >> 2);
    *reinterpret_cast<f16x4*>(dst) = hi;
    *reinterpret_cast<f16x4*>(dst + kKPiece) = lo;
  };

  fq acc[16];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fq{0.f, 0.f, 0.f, 0.f};
  };

  // ------------------------------------------------------------------ 1. T^T = At xn_q^T (+ w)
  f4 rx[2][2];
  auto load_xq = [&](int kk, f4 (&r)[2]) {
    const float* p = xb + (size_t)(qrow0 + l16) * a.x_pitch + 32 * kk + 8 * q;
    r[0] = *reinterpret_cast<const f4*>(p);
    r[1] = *reinterpret_cast<const f4*>(p + 4);
  };
  auto xq_frag = [&](int kk, const f4 (&r)[2], f16x8 (&bf)[2]) {
    const int c = 32 * kk + 8 * q;
    const f4 s0 = *reinterpret_cast<const f4*>(&tab[0][c]), s1 = *reinterpret_cast<const f4*>(&tab[0][c + 4]);
    const f4 h0 = *reinterpret_cast<const f4*>(&tab[1][c]), h1 = *reinterpret_cast<const f4*>(&tab[1][c + 4]);
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (r[0][e] * s0[e] + h0[e]) * xs;
      v[4 + e] = (r[1][e] * s1[e] + h1[e]) * xs;
    }
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
    bad |= m > 65504.f;
    split8(v, bf[0], bf[1]);
  };
  zero_acc();
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    load_w(a.at_img, 0, u, rg[0][u]);
    if (RD == 2) load_w(a.at_img, 1, u, rg[RD - 1][u]);
  }
  load_xq(0, rx[0]);
  load_xq(1, rx[1]);
#pragma unroll
  for (int u = 0; u < NS; ++u) store_w(0, u, rg[0][u]);
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    f16x8 bf[2];
    xq_frag(kk, rx[kk & 1], bf);
    if (kk + 2 < 8) load_xq(kk + 2, rx[kk & 1]);
    kstep1(stg + (kk & 1) * kStepH, l16, q, bf, acc, [&](int tt) {
      if (tt % SD) return;
      if (tt < 8) {
        if (kk + RD < 8) load_w(a.at_img, kk + RD, tt / SD, rg[(kk + RD) % RD][tt / SD]);
      } else if (kk + 1 < 8) {
        store_w((kk + 1) & 1, (tt - 8) / SD, rg[(kk + 1) % RD][(tt - 8) / SD]);
      }
    });
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    load_k(0, u, rg[0][u]);
    if (RD == 2) load_k(1, u, rg[RD - 1][u]);
  }
  AB_STAMP(1);
  f16x8 tp[8][2];
  float tun;
  {
    const float xun = ldexpf(1.f, -a.ex);
    float mx = 0.f;
#pragma unroll
    for (int ct = 0; ct < 16; ++ct) {
      const f4 rs = *reinterpret_cast<const f4*>(a.at_rowscale + 16 * ct + 4 * q);
      const f4 wv = *reinterpret_cast<const f4*>(a.w + 16 * ct + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[ct][r] * (rs[r] * xun) + wv[r];
        acc[ct][r] = v;
        mx = fmaxf(mx, fabsf(v));
      }
    }
    float m = fmaxf(mx, __shfl_xor(mx, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    int E = 0;
    (void)frexpf(m, &E);
    const int eT = m > 0.f ? 14 - E : 0;
    const float sc = ldexpf(1.f, eT);
    tun = ldexpf(1.f, -(a.ex + eT));
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * ks][e] * sc;
        v[4 + e] = acc[2 * ks + 1][e] * sc;
      }
      split8(v, tp[ks][0], tp[ks][1]);
    }
  }

  AB_STAMP(2);
  // ------------------------------------------------------------------ 2. one pass over the keys (chunks of 32)
#pragma unroll
  for (int u = 0; u < NS; ++u) store_k(0, u, rg[0][u]);
  __syncthreads();
  zero_acc();   // O^T accumulators
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = tun * 1.4426950408889634f;
#pragma unroll
  for (int kc = 0; kc < 8; ++kc) {
    const _Float16* img = stg + (kc & 1) * kKImg;
    fq sacc[2] = {fq{0.f, 0.f, 0.f, 0.f}, fq{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const _Float16* pr = img + (16 * kt + l16) * kKP + 32 * ks + 8 * q;
        f16x8 av[2];
        av[0] = *reinterpret_cast<const f16x8*>(pr);
        av[1] = *reinterpret_cast<const f16x8*>(pr + kKPiece);
        mma3(av, tp[ks], sacc[kt]);
      }
      if (kc + RD < 8 && ks % SD == 0) load_k(kc + RD, ks / SD, rg[(kc + RD) % RD][ks / SD]);
    }
    f16x8 pp[2];
    {
      float mx = fmaxf(fmaxf(fmaxf(sacc[0][0], sacc[0][1]), fmaxf(sacc[0][2], sacc[0][3])),
                       fmaxf(fmaxf(sacc[1][0], sacc[1][1]), fmaxf(sacc[1][2], sacc[1][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float m_new = fmaxf(m_run, mx * sl2);
      const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
      m_run = m_new;
      float ls = 0.f, v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[0][e], sl2, -m_new));
        v[4 + e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[1][e], sl2, -m_new));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ls += v[e];
        v[e] *= 16384.f;
      }
      l_run = l_run * corr + ls;
      split8(v, pp[0], pp[1]);
      if (kc > 0) {
#pragma unroll
        for (int ot = 0; ot < 16; ++ot) acc[ot] *= corr;
      }
    }
    {
      const _Float16* pt = img + (4 * q + (l16 >> 2)) * kKP + 4 * (l16 & 3);
#pragma unroll
      for (int ot = 0; ot < 16; ++ot) {
        f16x8 av[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const f16x4_t lo4 = lds_tr16(pt + p * kKPiece + 16 * ot);
          const f16x4_t hi4 = lds_tr16(pt + p * kKPiece + 16 * kKP + 16 * ot);
          av[p] = f16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        }
        mma3(av, pp, acc[ot]);
        if (ot >= 8 && ot % SD == 0 && kc + 1 < 8) store_k((kc + 1) & 1, (ot - 8) / SD, rg[(kc + 1) % RD][(ot - 8) / SD]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < NS; ++u) {
    load_w(a.wg_img, 0, u, rg[0][u]);
    if (RD == 2) load_w(a.wg_img, 1, u, rg[RD - 1][u]);
  }
  
  AB_STAMP(3);
  // O x 2^ex = acc / (2^14 l) (the staged keys carry xn x 2^ex), rows in storage order -> the projection's B
  f16x8 op[8][2];
  {
    float l = l_run + __shfl_xor(l_run, 16);
    l += __shfl_xor(l, 32);
    const float sc = 1.f / (16384.f * l);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[2 * ks][e] * sc;
        v[4 + e] = acc[2 * ks + 1][e] * sc;
      }
      split8(v, op[ks][0], op[ks][1]);
    }
  }

  AB_STAMP(4);
  // ------------------------------------------------------------------ 3. Y^T = Wg' O^T
#pragma unroll
  for (int u = 0; u < NS; ++u) store_w(0, u, rg[0][u]);
  __syncthreads();
  zero_acc();
  // output pass mapping: wave -> (64-token chunk ch, 64-column quarter cq); lane -> 4 columns, row of 4
  const int ch = wave >> 2, cq = wave & 3;
  const int c4 = lane & 15, rsub = lane >> 4;
  const int col = 64 * cq + 4 * c4;
  const int tok0 = qh * QB + 64 * ch;
  auto load_res = [&](int i, f4& r) {
    r = *reinterpret_cast<const f4*>(xb + (size_t)(tok0 + 4 * i + rsub) * a.x_pitch + col);
  };
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    kstep1(stg + (kk & 1) * kStepH, l16, q, op[kk], acc, [&](int tt) {
      if (tt % SD) return;
      if (tt < 8) {
        if (kk + RD < 8) load_w(a.wg_img, kk + RD, tt / SD, rg[(kk + RD) % RD][tt / SD]);
        else load_res(NS * (kk + RD - 8) + tt / SD, rg[(kk + RD) % RD][tt / SD]);   // residual rows 0 .. RD NS - 1
      } else if (kk + 1 < 8) {
        store_w((kk + 1) & 1, (tt - 8) / SD, rg[(kk + 1) % RD][(tt - 8) / SD]);
      }
    });
    __syncthreads();
  }
  constexpr int NX = 16 - RD * NS;   // residual rows loaded after the loop
  f4 xr2[NX > 0 ? NX : 1];
#pragma unroll
  for (int i = 0; i < NX; ++i) load_res(RD * NS + i, xr2[i]);
  if (bad && a.range_flag) *a.range_flag = 1;

  AB_STAMP(5);
  // ------------------------------------------------------------------ 4. y = x + Y + cb, GroupNorm statistics
  const float yun = ldexpf(1.f, -a.ex);
#pragma unroll
  for (int dt = 0; dt < 16; ++dt) {
    const f4 rs = *reinterpret_cast<const f4*>(a.wg_rowscale + 16 * dt + 4 * q);
    *reinterpret_cast<fq*>(lds + (wave * 16 + l16) * kOP + 16 * dt + 4 * q) = acc[dt] * (rs * yun);
  }
  __syncthreads();
  const f4 cb4 = *reinterpret_cast<const f4*>(a.cb + col);
  double gs[4] = {0.0, 0.0, 0.0, 0.0}, gq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int tok = tok0 + 4 * i + rsub;
    const f4 o = *reinterpret_cast<const f4*>(lds + (64 * ch + 4 * i + rsub) * kOP + col);
    const f4 xr = i < NS ? rg[0][i % NS] : i < RD * NS ? rg[RD - 1][i % NS] : xr2[(i - RD * NS) % (NX > 0 ? NX : 1)];
    const f4 yv = xr + (o + cb4);
    *reinterpret_cast<f4*>(a.y + ((size_t)b * kBL + tok) * a.y_pitch + col) = yv;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gs[e] += (double)yv[e];
      gq[e] += (double)yv[e] * yv[e];
    }
  }
  if (a.gn_part) {
    double s = gs[0] + gs[1] + gs[2] + gs[3], qq = gq[0] + gq[1] + gq[2] + gq[3];
    s += __shfl_xor(s, 16);
    qq += __shfl_xor(qq, 16);
    s += __shfl_xor(s, 32);
    qq += __shfl_xor(qq, 32);
    const int cpg = kBC / a.gn_G;
    for (int o = 1; o < cpg / 4; o <<= 1) {
      s += __shfl_xor(s, o);
      qq += __shfl_xor(qq, o);
    }
    if (rsub == 0 && (c4 % (cpg / 4)) == 0)
      a.gn_part[((size_t)b * (kBL / 64) + (tok0 >> 6)) * a.gn_G + col / cpg] = make_double2(s, qq);
  }
  AB_STAMP(6);
  AB_RSTAMP(9);
  AB_FLUSH;
}

__device__ __forceinline__ int pi32(int m) { return 4 * (m >> 3) + (m & 3) + 16 * ((m >> 2) & 1); }

// Wg' = Wg with its columns permuted by pi o pi within every 32 columns (attn_block3_kernel's projection)
__global__ void attn_perm_cols_kernel(const float* __restrict__ wg, float* __restrict__ wgp, int C) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)C * C) return;
  const int d = (int)(id / C), k = (int)(id % C);
  wgp[id] = wg[(size_t)d * C + (k & ~31) + pi32(pi32(k & 31))];
}

// dst[k][n] = src[n][k] (C x C): the small-map block's operands, read a row of k per step by 256 threads
__global__ void attn_transpose_kernel(const float* __restrict__ src, float* __restrict__ dst, int C) {
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= (long)C * C) return;
  const int k = (int)(id / C), n = (int)(id % C);
  dst[id] = src[(size_t)n * C + k];
}

// ======================================================================================================
// Small maps: the single-head block on a 4 x 4 map of 256 channels (the CIFAR UNet's middle block,
// models/unet.py:97-99 -> models/modules.py:77-102), L = 16 tokens. The same folded form as variant 3/4,
//   T = xn At^T + w,  S = T xn^T,  P = softmax(S),  y = x + Wg (P xn) + cb,
// but at L = 16 the block is 2.1 M multiply-adds per image (the unfolded qkv / S / PV / proj launches took
// 88 us per forward at B = 256, five launches with a q / k / v buffer between them): one work-group of 512
// threads per image, fp32 throughout (no operand split), everything in LDS. The two C x C products run on
// v_mfma_f32_16x16x4f32 (exact fp32 products, fp32 sums; wave w owns 32 channels x the 16 tokens; At^T and Wg^T
// transposed at the fold so a K step reads 16 consecutive floats per row; on the vector ALUs they took 54 us per
// launch), S / the softmax run on 16 lanes per query row, P xn on thread (n, h) = channel n x tokens 8 h .. + 7,
// and the epilogue emits the consumer's GroupNorm partials (one 64-pixel chunk per image).
constexpr int kSL = 16;          // tokens of the small map
constexpr int kSTP = kBC + 4;    // fp32 pitch of the T rows

__global__ void __launch_bounds__(512) attn_small_kernel(AttnBlockArgs a) {
  __shared__ __attribute__((aligned(16))) float xnt[kBC][kSL];   // xn^T [channel][token]
  __shared__ __attribute__((aligned(16))) float tt[kSL * kSTP];  // T [token][kSTP], then O^T [channel][token]
  __shared__ __attribute__((aligned(16))) float pm[kSL][kSL];    // S partial sums, then P
  __shared__ __attribute__((aligned(16))) float tab[2][kBC];
  __shared__ double csum[2][kBC];
  const int b = blockIdx.x, t = threadIdx.x;
  const int n = t & (kBC - 1), h = t >> 8, r0 = 8 * h;
  const float* xb = a.x + (size_t)b * kSL * a.x_pitch;
  // x rows of this thread (kept for the residual), loaded while the GroupNorm affine is formed
  float xv[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) xv[r] = xb[(size_t)(r0 + r) * a.x_pitch + n];
  if (t < kBC) {
    if (a.gin_part) {  // gn_finalize (gn.hip), the expressions of attn_block4_kernel's in-kernel finalize
      const int cpg = kBC / a.gin_G, g = t / cpg;
      const double cnt = (double)kSL * cpg;
      double s1 = 0, s2 = 0;
      for (int k = 0; k < a.gin_nchunk; ++k) {
        const double2 v = a.gin_part[((size_t)b * a.gin_nchunk + k) * a.gin_G + g];
        s1 += v.x;
        s2 += v.y;
      }
      const double m = s1 / cnt;
      double var = s2 / cnt - m * m;
      if (var < 0) var = 0;
      const float mu = (float)m;
      const float rs = (float)(1.0 / sqrt(var + (double)a.gin_eps));
      const float sc = rs * (a.gin_gamma ? a.gin_gamma[t] : 1.0f);
      tab[0][t] = sc;
      tab[1][t] = -sc * mu + (a.gin_beta ? a.gin_beta[t] : 0.0f);
    } else {
      tab[0][t] = a.gsc[(size_t)b * kBC + t];
      tab[1][t] = a.gsh[(size_t)b * kBC + t];
    }
  }
  __syncthreads();
  {
    const float sc = tab[0][n], sh = tab[1][n];
    f4 v0, v1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v0[r] = xv[r] * sc + sh;
      v1[r] = xv[4 + r] * sc + sh;
    }
    *reinterpret_cast<f4*>(&xnt[n][r0]) = v0;
    *reinterpret_cast<f4*>(&xnt[n][r0 + 4]) = v1;
  }
  __syncthreads();
  // D[i][n] = sum_k tok[k][i] wt[k][n] on v_mfma_f32_16x16x4f32 (fp32 products and sums): wave w takes the column
  // tiles nt = 2 w, 2 w + 1 (16 channels each) for all 16 tokens; lane l supplies A[l % 16][k0 + l / 16] (tok, LDS) and
  // B[k0 + l / 16][16 nt + l % 16] (wt, global, 8 K steps ahead in registers) and holds D[4 (l / 16) + e][16 nt + l % 16]
  const int lane = t & 63, wave = t >> 6, lc = lane & 15, lk = lane >> 4;
  auto product = [&](const float* tok, const float* __restrict__ wt, f4 (&d)[2]) {
    d[0] = f4{0.f, 0.f, 0.f, 0.f};
    d[1] = d[0];
    const float* wl = wt + (size_t)lk * kBC + 32 * wave + lc;
    float bc[8][2], bn[8][2];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) bc[u][jt] = wl[(size_t)(4 * u) * kBC + 16 * jt];
    for (int k0 = 0; k0 < kBC; k0 += 32) {
      if (k0 + 32 < kBC) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) bn[u][jt] = wl[(size_t)(k0 + 32 + 4 * u) * kBC + 16 * jt];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float av = tok[(k0 + 4 * u + lk) * kSL + lc];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) d[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bc[u][jt], d[jt], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) bc[u][jt] = bn[u][jt];
    }
  };
  f4 dacc[2];
  // T[i][n] = sum_k xn[i][k] At[n][k] + w[n]
  product(&xnt[0][0], a.at_t, dacc);
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int nn = 32 * wave + 16 * jt + lc;
    const float wn_ = a.w[nn];
#pragma unroll
    for (int e = 0; e < 4; ++e) tt[(4 * lk + e) * kSTP + nn] = dacc[jt][e] + wn_;
  }
  __syncthreads();
  // S[i][j] = T_i . xn_j: thread (i, j) of the 256, k half h; the halves added in LDS
  {
    const int i = (t & 255) >> 4, j = t & 15, kb = 128 * h;
    float s = 0.f;
#pragma unroll 4
    for (int k = kb; k < kb + 128; k += 4) {
      const f4 tv = *reinterpret_cast<const f4*>(&tt[i * kSTP + k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) s = fmaf(tv[e], xnt[k + e][j], s);
    }
    if (h == 1) pm[i][j] = s;
    __syncthreads();
    if (h == 0) {
      s += pm[i][j];
      // softmax over the 16 lanes of row i
      float m = s;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
      const float e = expf(s - m);
      float z = e;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) z += __shfl_xor(z, o);
      pm[i][j] = e / z;
    }
  }
  __syncthreads();
  // O^T[n][i] = sum_j P[i][j] xn[j][n] (over T's rows: T is dead)
  {
    float xc[kSL];
#pragma unroll
    for (int j = 0; j < kSL; j += 4) {
      const f4 v = *reinterpret_cast<const f4*>(&xnt[n][j]);
#pragma unroll
      for (int e = 0; e < 4; ++e) xc[j + e] = v[e];
    }
    f4 o0, o1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float o = 0.f;
#pragma unroll
      for (int j = 0; j < kSL; ++j) o = fmaf(pm[r0 + r][j], xc[j], o);
      if (r < 4) o0[r] = o; else o1[r - 4] = o;
    }
    *reinterpret_cast<f4*>(&tt[n * kSL + r0]) = o0;
    *reinterpret_cast<f4*>(&tt[n * kSL + r0 + 4]) = o1;
  }
  __syncthreads();
  // y[i][n] = x[i][n] + (sum_k O[i][k] Wg[n][k] + cb[n])
  product(tt, a.wg_t, dacc);
  float* yb = a.y + (size_t)b * kSL * a.y_pitch;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const int nn = 32 * wave + 16 * jt + lc;
    const float cbn = a.cb[nn];
    double gs = 0.0, gq = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = 4 * lk + e;
      const float v = xb[(size_t)row * a.x_pitch + nn] + (dacc[jt][e] + cbn);
      yb[(size_t)row * a.y_pitch + nn] = v;
      gs += (double)v;
      gq += (double)v * v;
    }
    if (a.gn_part) {  // column sums over the 16 tokens, then the groups' cpg columns in order (below)
      gs += __shfl_xor(gs, 16);
      gq += __shfl_xor(gq, 16);
      gs += __shfl_xor(gs, 32);
      gq += __shfl_xor(gq, 32);
      if (lk == 0) {
        csum[0][nn] = gs;
        csum[1][nn] = gq;
      }
    }
  }
  if (a.gn_part) {  // one 64-pixel chunk per image
    __syncthreads();
    const int cpg = kBC / a.gn_G;
    if (t < a.gn_G) {
      double s1 = 0.0, s2 = 0.0;
      for (int c = t * cpg; c < (t + 1) * cpg; ++c) {
        s1 += csum[0][c];
        s2 += csum[1][c];
      }
      a.gn_part[(size_t)b * a.gn_G + t] = make_double2(s1, s2);
    }
  }
}

}  // namespace

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_ab_stamps(void* host, int nblocks) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ab_stamps), (size_t)nblocks * 10 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

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

int attn_perm_cols(const float* wg, float* wgp, int C, hipStream_t st) {
  DM_REQUIRE(wg && wgp && C % 32 == 0, "attention fold: column permutation needs C % 32 == 0");
  const long n = (long)C * C;
  hipLaunchKernelGGL(attn_perm_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wg, wgp, C);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

bool attn_small_ok(int L, int C, int heads) { return L == kSL && C == kBC && heads == 1; }

int attn_transpose(const float* src, float* dst, int C, hipStream_t st) {
  DM_REQUIRE(src && dst && C > 0, "attention fold: null argument");
  const long n = (long)C * C;
  hipLaunchKernelGGL(attn_transpose_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst, C);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int attn_small(const AttnBlockArgs& a, hipStream_t st) {
  DM_REQUIRE(a.B > 0 && a.x && a.y && a.x != a.y && (a.gin_part || (a.gsc && a.gsh)) && a.at_t && a.w && a.wg_t && a.cb,
             "small-map attention block: null or in-place argument");
  DM_REQUIRE(!a.gin_part || (a.gin_G > 0 && kBC % a.gin_G == 0 && a.gin_nchunk > 0),
             "small-map attention block: the in-kernel GroupNorm finalize needs groups dividing 256 channels");
  DM_REQUIRE(!a.gn_part || (a.gn_G > 0 && kBC % a.gn_G == 0 && kBC / a.gn_G >= 4 && kBC / a.gn_G <= 64 &&
                            ((kBC / a.gn_G) & (kBC / a.gn_G - 1)) == 0),
             "small-map attention block: GroupNorm statistics need groups of 4 .. 64 channels (a power of two)");
  hipLaunchKernelGGL(attn_small_kernel, dim3(a.B), dim3(512), 0, st, a);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int attn_block(const AttnBlockArgs& a, hipStream_t st) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  DM_REQUIRE(a.variant == 3 || a.variant == 4, "attention block: variant 3 or 4");
  DM_REQUIRE(!a.gin_part || (a.variant >= 4 && a.gin_G > 0 && kBC % a.gin_G == 0 && a.gin_nchunk > 0),
             "attention block: in-kernel GroupNorm finalize needs variant 4 and groups dividing 256 channels");
  DM_REQUIRE(a.B > 0 && a.x && a.y && (a.gin_part || (a.gsc && a.gsh)) && a.at_img && a.at_rowscale && a.w &&
                 a.wg_img && a.wg_rowscale && a.cb,
             "attention block: null argument");
  DM_REQUIRE(a.x_pitch % 4 == 0 && a.y_pitch % 4 == 0 && al16(a.x) && al16(a.y) &&
                 (a.gin_part || (al16(a.gsc) && al16(a.gsh))) &&
                 al16(a.at_img) && al16(a.at_rowscale) && al16(a.w) &&
                 al16(a.wg_img) && al16(a.wg_rowscale) && al16(a.cb),
             "attention block: 16-byte aligned rows");
  DM_REQUIRE(!a.gn_part || (a.gn_G > 0 && kBC % a.gn_G == 0 && kBC / a.gn_G >= 4 && kBC / a.gn_G <= 32 &&
                            ((kBC / a.gn_G) & (kBC / a.gn_G - 1)) == 0),
             "attention block: GroupNorm statistics need groups of 4, 8, 16 or 32 channels");
  if (a.variant == 4)
    hipLaunchKernelGGL(attn_block4_kernel<8>, dim3(a.B * (kBL / 128)), dim3(512), 0, st, a);
  else
    hipLaunchKernelGGL(attn_block3_kernel, dim3(a.B * (kBL / kBQ)), dim3(256), 0, st, a);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
