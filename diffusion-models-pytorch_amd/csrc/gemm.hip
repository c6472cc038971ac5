// Batched fp32 MFMA GEMM: C[z][m][n] = act( sum_k (alpha * A[z][m][k]) * (b_scale * B[z](k, n)) + bias[n] )
//
// Used for the small dense contractions of the denoisers:
//   * nn.Linear layers (time MLP models/unet.py:64-69, ResBlock proj :18-21)
//     with B = weight [N][K] ("BT" layout) and optional SiLU epilogue;
//   * the attention contractions of SelfAttentionBlock (models/modules.py:96-97):
//       S = (q * scale)^T k   -> A = q rows (alpha = scale), B = k rows [n][k]
//       O = attn v^T         -> A = attn rows, B = v stored [k][n] ("BN")
// Batch index z = z1 * Z2 + z2 with independent strides for both levels
// (image, head).
#include <cmath>
#include <cstring>
#include <type_traits>
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"

namespace dm {

namespace {

// SPLIT (GemmArgs::split = 2): the LDS tiles hold fp16x2 pieces instead of fp32 values. A 32-deep
// row of the fp32 tile (144 B with its pitch) holds the same 32 k as two 16-deep slices of
// [2 lane groups][hi, lo][8] fp16 (128 B) in the same 144 B, so the stage geometry is unchanged.
constexpr int kLDK16 = 2 * kLDK;  // fp16 elements per LDS row

template <int BM, int BN, int WM, int WN, bool B_KN, bool SPLIT = false>
__global__ void __launch_bounds__(256, 2)
gemm_kernel(GemmArgs g) {
  using Cfg = TileCfg<BM, BN, WM, WN>;
  __shared__ __attribute__((aligned(16))) float lds[Cfg::LDS_FLOATS];
  const float a_pow = SPLIT ? ldexpf(1.f, g.split_ea) : 1.f;
  const float b_pow = SPLIT ? ldexpf(1.f, g.split_eb) : 1.f;
  bool bad = false;
  // fp16 offset of k (0..31) in a split row: slice k / 16, lane group (k % 16) / 8, element k % 8
  auto split_off = [](int k) { return (k >> 4) * 32 + ((k >> 3) & 1) * 16 + (k & 7); };

  // batched (Z > 1): XCD-aware order, so the tiles of one batch entry (which share its A rows and
  // B columns) run on one XCD and share its L2 instead of being dealt round-robin over the 8 L2s,
  // each fetching the shared operands from HBM again (attention S / PV microbenchmark -11 %; a
  // single large GEMM keeps the plain order, which measured faster)
  const int nxy = gridDim.x;
  const int flat = blockIdx.z * nxy + blockIdx.x;
  const int lin = gridDim.z > 1 ? xcd_remap_p(flat, nxy * gridDim.z) : flat;
  const int z = lin / nxy, bx = lin - (lin / nxy) * nxy;
  const int z1 = z / g.Z2, z2 = z - (z / g.Z2) * g.Z2;
  const float* A = g.A + (size_t)z1 * g.a_s1 + (size_t)z2 * g.a_s2;
  const float* Bm = g.Bm + (size_t)z1 * g.b_s1 + (size_t)z2 * g.b_s2;
  float* C = g.C + (size_t)z1 * g.c_s1 + (size_t)z2 * g.c_s2;

  const int nN = ceil_div(g.N, BN);
  const int mt = bx / nN, nt = bx % nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave / Cfg::NWN, wn = wave % Cfg::NWN;
  const int lc4 = t & 7, lrow = t >> 3;

  // "BN" loader geometry: BK rows of k, BN/4 float4 per row.
  constexpr int KN_C4 = BN / 4;
  constexpr int KN_ROWS_PER_PASS = Cfg::NT / KN_C4;
  constexpr int KN_ITERS = (kBK + KN_ROWS_PER_PASS - 1) / KN_ROWS_PER_PASS;
  static_assert(!B_KN || (Cfg::NT % KN_C4 == 0), "BN loader geometry");

  const int nk = ceil_div(g.K, kBK);
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // Branch-free loaders: rows/columns outside the problem read a clamped, valid
  // address and are zeroed when written to LDS (after the MFMA work), so the
  // next slice's loads stay in flight across the current slice's MFMAs.
  const float* arow[Cfg::A_ITERS];
  bool a_ok[Cfg::A_ITERS];
  int a_img[Cfg::A_ITERS];
  float2 a_ln[Cfg::A_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::A_ITERS; ++i) {
    const int m = m0 + lrow + i * Cfg::ROWS_PER_PASS;
    a_ok[i] = m < g.M;
    const int mc = min(m, g.M - 1);
    arow[i] = A + (size_t)mc * g.lda + 4 * lc4;
    a_img[i] = g.pro_scale ? (z1 * g.M + mc) / g.pro_rows : (g.ln_stats ? mc / g.ln_rows : 0);
    a_ln[i] = g.ln_stats ? g.ln_stats[mc] : make_float2(0.f, 1.f);
  }
  const float* brow[B_KN ? 1 : Cfg::B_ITERS];
  bool b_ok[B_KN ? 1 : Cfg::B_ITERS];
  if constexpr (!B_KN) {
#pragma unroll
    for (int j = 0; j < Cfg::B_ITERS; ++j) {
      const int n = n0 + lrow + j * Cfg::ROWS_PER_PASS;
      b_ok[j] = n < g.N;
      brow[j] = Bm + (size_t)min(n, g.N - 1) * g.ldb + 4 * lc4;
    }
  }
  // SPLIT with the [k][n] B layout: each thread loads a 4 (k) x 4 (n) block (rows 4 kq .. 4 kq + 3,
  // columns 4 n4 ..) and stores it transposed as 4 rows of 4 consecutive k per piece (ds_write_b64),
  // instead of 2-byte scatter stores; lanes kq = t % 8 of one n4 hit distinct banks
  constexpr bool KN4 = B_KN && SPLIT;
  constexpr int KN4_THREADS = 2 * BN;  // (kBK / 4) x (BN / 4)
  static_assert(!KN4 || (kBK == 32 && KN4_THREADS <= Cfg::NT), "KN4 loader geometry");
  const int kq = t & 7, n4k = t >> 3;
  // SPLIT ([n][k] B): two register sets, tiles loaded two K steps ahead (a step's MFMAs alone do not cover the
  // load latency at K = 256); set index = K step parity, a compile-time constant (loop unrolled by 2)
  constexpr int NSET = SPLIT && !B_KN ? 2 : 1;  // (the [k][n] loader's second set spilled)
  f4 ra[NSET][Cfg::A_ITERS];
  f4 rb[NSET][KN4 ? 4 : B_KN ? KN_ITERS : Cfg::B_ITERS];
  bool kn_ok[B_KN ? KN_ITERS : 1];
  int ld_k[NSET];

  // K tail: B reads the zero page (mfma_tile.h kZeroPage) so those products vanish; A reads a
  // clamped, finite column. Rows >= M / columns >= N read clamped data and are never stored.
  auto load_tile = [&](int kt, auto set_c) {
    constexpr int S = decltype(set_c)::value;
    const int k = kt * kBK + 4 * lc4;
    const bool k_ok = k < g.K;
    ld_k[S] = k_ok ? k : 0;
    const int kofs = ld_k[S] - 4 * lc4;
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i) ra[S][i] = *reinterpret_cast<const f4*>(arow[i] + kofs);
    if constexpr (!B_KN) {
#pragma unroll
      for (int j = 0; j < Cfg::B_ITERS; ++j)
        rb[S][j] = *reinterpret_cast<const f4*>(k_ok ? brow[j] + kofs : kZeroPage);
    } else if constexpr (KN4) {
      const int n = min(n0 + 4 * min(n4k, BN / 4 - 1), g.N - 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = kt * kBK + 4 * kq + r;
        rb[S][r] = *reinterpret_cast<const f4*>(kk < g.K ? Bm + (size_t)kk * g.ldb + n : kZeroPage);
      }
    } else {
      const int n4 = t % KN_C4, kr = t / KN_C4;
      const int n = min(n0 + 4 * n4, g.N - 4);
#pragma unroll
      for (int j = 0; j < KN_ITERS; ++j) {
        const int kk = kt * kBK + kr + j * KN_ROWS_PER_PASS;
        kn_ok[j] = (kr + j * KN_ROWS_PER_PASS < kBK);
        rb[S][j] = *reinterpret_cast<const f4*>(kk < g.K ? Bm + (size_t)kk * g.ldb + n : kZeroPage);
      }
    }
  };

  auto store_tile = [&](int buf, auto set_c) {
    constexpr int S = decltype(set_c)::value;
    float* As = lds + buf * Cfg::STAGE;
    float* Bs = As + Cfg::A_ELEMS;
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i) {
      f4 v = ra[S][i];
      if (g.pro_scale) {  // fused GroupNorm (no activation): x * scale[img][k] + shift[img][k]
        const f4 sc = *reinterpret_cast<const f4*>(g.pro_scale + (size_t)a_img[i] * g.K + ld_k[S]);
        const f4 sh = *reinterpret_cast<const f4*>(g.pro_shift + (size_t)a_img[i] * g.K + ld_k[S]);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = v[q] * sc[q] + sh[q];
      }
      if (g.ln_stats) {  // LayerNorm (no affine) + modulate x * (1 + scale) + shift
        const f4 sc = *reinterpret_cast<const f4*>(g.ln_scale + (size_t)a_img[i] * g.ln_pitch + ld_k[S]);
        const f4 sh = *reinterpret_cast<const f4*>(g.ln_shift + (size_t)a_img[i] * g.ln_pitch + ld_k[S]);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ((v[q] - a_ln[i].x) * a_ln[i].y) * (1.0f + sc[q]) + sh[q];
      }
      if (g.alpha != 1.0f) v = v * g.alpha;
      if constexpr (SPLIT) {
        f16x4 hi, lo;
        Split<2>::split4(v * a_pow, hi, lo, bad);
        _Float16* dst = reinterpret_cast<_Float16*>(As) + (lrow + i * Cfg::ROWS_PER_PASS) * kLDK16 + split_off(4 * lc4);
        *reinterpret_cast<f16x4*>(dst) = hi;
        *reinterpret_cast<f16x4*>(dst + 8) = lo;
      } else {
        *reinterpret_cast<f4*>(As + (lrow + i * Cfg::ROWS_PER_PASS) * kLDK + 4 * lc4) = v;
      }
    }
    if constexpr (!B_KN) {
#pragma unroll
      for (int j = 0; j < Cfg::B_ITERS; ++j) {
        const f4 v = (g.b_scale != 0.0f && g.b_scale != 1.0f) ? rb[S][j] * g.b_scale : rb[S][j];
        if constexpr (SPLIT) {
          f16x4 hi, lo;
          Split<2>::split4(v * b_pow, hi, lo, bad);
          _Float16* dst = reinterpret_cast<_Float16*>(Bs) + (lrow + j * Cfg::ROWS_PER_PASS) * kLDK16 +
                          split_off(4 * lc4);
          *reinterpret_cast<f16x4*>(dst) = hi;
          *reinterpret_cast<f16x4*>(dst + 8) = lo;
        } else {
          *reinterpret_cast<f4*>(Bs + (lrow + j * Cfg::ROWS_PER_PASS) * kLDK + 4 * lc4) = v;
        }
      }
    } else if constexpr (KN4) {
      if (t < KN4_THREADS) {
        _Float16* Bh = reinterpret_cast<_Float16*>(Bs);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f4 col = {rb[S][0][q], rb[S][1][q], rb[S][2][q], rb[S][3][q]};  // k = 4 kq .. 4 kq + 3 of column q
          f16x4 hi, lo;
          Split<2>::split4(col * b_pow, hi, lo, bad);
          _Float16* dst = Bh + (4 * n4k + q) * kLDK16 + split_off(4 * kq);
          *reinterpret_cast<f16x4*>(dst) = hi;
          *reinterpret_cast<f16x4*>(dst + 8) = lo;
        }
      }
    } else {
      const int n4 = t % KN_C4, kr = t / KN_C4;
#pragma unroll
      for (int j = 0; j < KN_ITERS; ++j) {
        const int kk = kr + j * KN_ROWS_PER_PASS;
        if (kn_ok[j]) {
          const f4 v = rb[S][j];
          if constexpr (SPLIT) {
            f16x4 hi, lo;
            Split<2>::split4(v * b_pow, hi, lo, bad);
            _Float16* Bh = reinterpret_cast<_Float16*>(Bs);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              Bh[(4 * n4 + q) * kLDK16 + split_off(kk)] = hi[q];
              Bh[(4 * n4 + q) * kLDK16 + split_off(kk) + 8] = lo[q];
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) Bs[(4 * n4 + q) * kLDK + kk] = v[q];
          }
        }
      }
    }
  };

  f16v acc[Cfg::TM][Cfg::TN];
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute_tile = [&](int buf) {
    const float* As = lds + buf * Cfg::STAGE;
    const float* Bs = As + Cfg::A_ELEMS;
    if constexpr (SPLIT) {
      const _Float16* Ah = reinterpret_cast<const _Float16*>(As);
      const _Float16* Bh = reinterpret_cast<const _Float16*>(Bs);
      const int l_r = lane & 31, l_h = lane >> 5;
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        f16x8 av[Cfg::TM][2], bv[Cfg::TN][2];
#pragma unroll
        for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            av[i][q] = *reinterpret_cast<const f16x8*>(Ah + (wm * WM + i * 32 + l_r) * kLDK16 + sl * 32 + l_h * 16 + q * 8);
#pragma unroll
        for (int j = 0; j < Cfg::TN; ++j)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            bv[j][q] = *reinterpret_cast<const f16x8*>(Bh + (wn * WN + j * 32 + l_r) * kLDK16 + sl * 32 + l_h * 16 + q * 8);
#pragma unroll
        for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
          for (int j = 0; j < Cfg::TN; ++j) Split<2>::mma(av[i], bv[j], acc[i][j]);
      }
    } else {
      mfma_slice<Cfg::TM, Cfg::TN>(As, Bs, wm * WM, wn * WN, lane, acc);
    }
  };
  const std::integral_constant<int, 0> set0{};
  const std::integral_constant<int, 1> set1{};
  load_tile(0, set0);
  store_tile(0, set0);
  if constexpr (NSET == 2) {
    if (nk > 1) load_tile(1, set1);
    __syncthreads();
    // step kt: set (kt & 1) held tile kt (already in LDS) and receives tile kt + 2; the other set
    // holds tile kt + 1, stored after this step's MFMAs
    auto step = [&](int kt, auto cur, auto nxt) {
      if (kt + 2 < nk) load_tile(kt + 2, cur);
      compute_tile(decltype(cur)::value);
      if (kt + 1 < nk) store_tile(decltype(nxt)::value, nxt);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, set0, set1);
      if (kt + 1 < nk) step(kt + 1, set1, set0);
    }
  } else {
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load_tile(kt + 1, set0);
      compute_tile(buf);
      if (kt + 1 < nk) store_tile(buf ^ 1, set0);
      __syncthreads();
    }
  }
  if constexpr (SPLIT) {
    if (bad && g.range_flag) *g.range_flag = 1;
    const float unscale = ldexpf(1.f, -(g.split_ea + g.split_eb));  // exact
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= unscale;
  }

  // Epilogue: residual / gate loads of a column group issued branch-free (clamped rows) before
  // any store, so their latencies overlap.
  const int lr = lane & 31, lh = lane >> 5;
  const bool emit = WM == 64 && g.gn_part != nullptr;
  const int wrow0 = m0 + wm * WM;
#pragma unroll
  for (int j = 0; j < Cfg::TN; ++j) {
    const int n = n0 + wn * WN + j * 32 + lr;
    const int nc = min(n, g.N - 1);
    double gs = 0.0, gq = 0.0;
    const float bn = g.bias ? g.bias[nc] : 0.f;
    float rsd[Cfg::TM][16], gt[Cfg::TM][16];
    if (g.res) {
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = min(m0 + wm * WM + i * 32 + acc_row(r, lh), g.M - 1);
          rsd[i][r] = g.res[(size_t)(g.res_mod > 0 ? m % g.res_mod : m) * g.ld_res + nc];
          gt[i][r] = g.gate ? g.gate[(size_t)(m / g.gate_rows) * g.gate_pitch + nc] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + acc_row(r, lh);
        if (m >= g.M) continue;
        float v = acc[i][j][r];
        if (g.bias) v = v + bn;
        if (g.res) v = g.gate ? rsd[i][r] + gt[i][r] * v : v + rsd[i][r];
        if (g.act == 1) v = silu_f(v);
        else if (g.act == 2) v = gelu_tanh_f(v);
        if (n < g.N) C[(size_t)m * g.ldc + n] = v;
        if (emit) {
          gs += (double)v;
          gq += (double)v * v;
        }
      }
    }
    if (emit) {
      const int cpg = g.N / g.gn_G;
      const int nchunk = (g.gn_hw + 63) / 64;
      const int bb = wrow0 / g.gn_hw, ch = (wrow0 - bb * g.gn_hw) / 64;
      gn_emit_group(gs, gq, lr, lh, cpg, n < g.N && wrow0 < g.M,
                    g.gn_part + ((size_t)bb * nchunk + ch) * g.gn_G + n / cpg);
    }
  }
}

template <int BM, int BN, int WM, int WN>
int launch_gemm(const GemmArgs& g, hipStream_t st) {
  using Cfg = TileCfg<BM, BN, WM, WN>;
  dim3 grid(ceil_div(g.M, BM) * ceil_div(g.N, BN), 1, g.Z1 * g.Z2);
  if (g.split == 2) {
    if (g.b_kn)
      hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, true, true>), grid, dim3(Cfg::NT), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, false, true>), grid, dim3(Cfg::NT), 0, st, g);
  } else if (g.b_kn) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, true>), grid, dim3(Cfg::NT), 0, st, g);
  } else {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, false>), grid, dim3(Cfg::NT), 0, st, g);
  }
  DM_LAUNCH_CHECK();
  return DM_OK;
}

// Skinny fp32 linear, C[m][n] = act(sum_k A[m][k] W[n][k] + bias[n]) for M of a batch (the time MLP and the
// ResBlocks' temb projections, models/unet.py:64-69 / :18-21: M = B rows, K <= 512). gemm_kernel's 64 x 64 tiles
// give 32 blocks for M = 256, N = 512, each walking K alone (15-33 us per launch); here a block is 8 rows x 16 outputs:
// the 8 A rows staged in LDS once (read back as broadcasts: straight from memory, the 16 lane groups' identical A
// addresses each cost the CU's address unit a full pass, 4x the W traffic), 16 lanes per output splitting K (lane l
// takes k = 4 l + 64 i .. + 3, a 256-B coalesced W segment per 16 lanes), each lane holding the 8 rows' partial sums,
// then a 16-lane tree (xor 8, 4, 2, 1). Per row the sums depend on K only, not on M or the grid: batch-invariant as
// the plans require.
constexpr int kRowsR = 8, kRowsKMax = 512;
template <int ACT>
__global__ void __launch_bounds__(256) linear_rows_kernel(GemmArgs g) {
  constexpr int R = kRowsR;
  __shared__ __attribute__((aligned(16))) f4 as[R * kRowsKMax / 4];
  const int t = threadIdx.x, l = t & 15;
  const int n = blockIdx.x * 16 + (t >> 4), m0 = blockIdx.y * R;
  const int nc = min(n, g.N - 1);
  const int K4 = g.K / 4;
  for (int i = t; i < R * K4; i += 256) {
    const int r = i / K4, k = i - r * K4;
    as[i] = reinterpret_cast<const f4*>(g.A + (size_t)min(m0 + r, g.M - 1) * g.lda)[k];
  }
  const f4* w = reinterpret_cast<const f4*>(g.Bm + (size_t)nc * g.ldb);
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
  __syncthreads();
#pragma unroll 2
  for (int k = l; k < K4; k += 16) {
    const f4 wv = w[k];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const f4 av = as[r * K4 + k];
      acc[r] = fmaf(av.x, wv.x, acc[r]);
      acc[r] = fmaf(av.y, wv.y, acc[r]);
      acc[r] = fmaf(av.z, wv.z, acc[r]);
      acc[r] = fmaf(av.w, wv.w, acc[r]);
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] += __shfl_xor(acc[r], o);
  if (n >= g.N) return;
  const float bn = g.bias ? g.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (l != r || m0 + r >= g.M) continue;
    float v = acc[r];
    if (g.bias) v = v + bn;
    if (ACT == 1) v = silu_f(v);
    g.C[(size_t)(m0 + r) * g.ldc + n] = v;
  }
}

}  // namespace

bool linear_rows_ok(const GemmArgs& g) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return g.M > 0 && g.N > 0 && g.K > 0 && g.K % 4 == 0 && g.K <= kRowsKMax && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
         al16(g.A) && al16(g.Bm) && g.Z1 == 1 && g.Z2 == 1 && !g.b_kn && g.split == 0 && !g.ws && !g.as &&
         !g.pro_scale && !g.ln_stats && !g.res && !g.gate && !g.gn_part && g.alpha == 1.0f &&
         (g.b_scale == 0.0f || g.b_scale == 1.0f) && (g.act == 0 || g.act == 1);
}

int linear_rows(const GemmArgs& g, hipStream_t st) {
  DM_REQUIRE(linear_rows_ok(g) && g.C, "linear_rows: fp32 [n][k] weights, 16-byte aligned rows, no prologue / residual");
  dim3 grid((unsigned)ceil_div(g.N, 16), (unsigned)ceil_div(g.M, kRowsR));
  if (g.act == 1)
    hipLaunchKernelGGL(linear_rows_kernel<1>, grid, dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL(linear_rows_kernel<0>, grid, dim3(256), 0, st, g);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int gemm_batched(const GemmArgs& g, hipStream_t st) {
  DM_REQUIRE(g.M > 0 && g.N > 0 && g.K > 0, "gemm: empty problem");
  if (g.ws) return linear_k32(g, st);  // pre-split static weights (linear_k32.hip)
  DM_REQUIRE(g.K % 4 == 0 && g.lda % 4 == 0 && g.ldb % 4 == 0, "gemm: K and leading dims must be multiples of 4");
  DM_REQUIRE(!g.b_kn || g.N % 4 == 0, "gemm: N must be a multiple of 4 for the [k][n] B layout");
  DM_REQUIRE((reinterpret_cast<uintptr_t>(g.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(g.Bm) & 15) == 0,
             "gemm: operands must be 16-byte aligned");
  DM_REQUIRE(g.Z1 >= 1 && g.Z2 >= 1 && (long)g.Z1 * g.Z2 <= 65535, "gemm: batch out of range");
  DM_REQUIRE(!g.pro_scale || (g.pro_shift && g.pro_rows > 0 && !g.b_kn), "gemm: A prologue needs scale, shift, rows");
  DM_REQUIRE(g.b_scale == 0.0f || !g.b_kn, "gemm: B scaling needs the [n][k] B layout");
  DM_REQUIRE(!g.ln_stats || (g.ln_scale && g.ln_shift && g.ln_rows > 0 && g.ln_pitch % 4 == 0 && !g.pro_scale &&
                             g.Z1 == 1 && g.Z2 == 1),
             "gemm: LayerNorm-modulate prologue needs stats, scale/shift tables and rows per image");
  DM_REQUIRE(!g.gate || (g.res && g.gate_rows > 0), "gemm: gated residual needs the residual and rows per image");
  DM_REQUIRE(g.split == 0 || (g.split == 2 && std::abs(g.split_ea) <= 100 && std::abs(g.split_eb) <= 100),
             "gemm: split must be 0 (fp32) or 2 (fp16x2) with power-of-two scales 2^-100 .. 2^100");
  DM_REQUIRE(!g.gn_part || (gemm_pick(g) == 0 && g.Z1 == 1 && g.Z2 == 1 && g.gn_hw % 64 == 0 && g.gn_G > 0 &&
                            g.N % g.gn_G == 0 && 32 % (g.N / g.gn_G) == 0),
             "gemm: GroupNorm statistics need 128-row tiles, whole 64-pixel chunks and groups within 32 columns");
  if (gemm_pick(g) == 0) return launch_gemm<128, 128, 64, 64>(g, st);
  return launch_gemm<64, 64, 32, 32>(g, st);
}

int gemm_pick(const GemmArgs& g) {
  const long M = g.pick_M > 0 ? g.pick_M : g.M, Z = g.pick_Z > 0 ? g.pick_Z : (long)g.Z1 * g.Z2;
  const long tiles128 = ((M + 127) / 128) * ceil_div(g.N, 128) * Z;
  return (M >= 128 && g.N >= 128 && tiles128 >= 512) ? 0 : 1;
}

std::string gemm_label(const GemmArgs& g) {
  if (g.ws) {
    return std::string("linear_k32_kernel<") + (g.as ? "3>" : g.pro_scale ? "1>" : g.ln_stats ? "2>" : "0>");
  }
  std::string s = gemm_pick(g) == 0 ? "gemm_kernel<128,128,64,64" : "gemm_kernel<64,64,32,32";
  return s + (g.b_kn ? ",true" : ",false") + (g.split == 2 ? ",true>" : ",false>");
}

namespace {
__global__ void absmax_kernel(const float* x, size_t n, unsigned* out) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));  // non-negative floats order as uints
}
}  // namespace

int split_weight_exponent(const float* x, size_t n) {
  unsigned* d = nullptr;
  unsigned h = 0;
  if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return 0;
  (void)hipMemset(d, 0, sizeof(unsigned));
  hipLaunchKernelGGL(absmax_kernel, dim3(256), dim3(256), 0, nullptr, x, n, d);
  (void)hipMemcpy(&h, d, sizeof(unsigned), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  float m;
  std::memcpy(&m, &h, sizeof m);
  if (!(m > 0.f) || !std::isfinite(m)) return 0;
  int ex;
  std::frexp(m, &ex);
  return std::min(std::max(14 - ex, -100), 100);
}

}  // namespace dm
