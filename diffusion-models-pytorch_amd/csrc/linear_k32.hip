// Static-weight GEMM C = prologue(A) W^T (+ bias, residual / gated residual, activation) on the fp16x2
// split matrix cores with K = 32 steps on v_mfma_f32_16x16x32_f16 -- the token GEMMs of DiT (qkv, proj,
// fc1, fc2, final layer: models/dit/model.py:118-142) and other static-weight linears. The weights are
// split ONCE at plan build (split_conv_weights, taps 1: conv_patch3's fragment images with per-row
// power-of-two scales) instead of on every load as gemm.hip's SPLIT path does (16-18 VALU per MFMA there).
//
// Numerics as everywhere on the fp16x2 path: an fp32 operand x = h0 + h1 (h0 = fp16(x), h1 = fp16(x - h0)),
// a*w = a1w0 + a0w1 + a0w0 into one fp32 accumulator; activations scaled by 2^split_ea before the split,
// weights by their row scale, both undone exactly in the epilogue. |scaled activation| > 65504 raises
// range_flag (the caller re-runs in fp32 / bf16x3).
//
// Block 128 x 128, four waves of 128 x 32 (8 x 2 tiles of 16 x 16). K is staged 64 channels at a time
// (two K = 32 steps per barrier), double-buffered in LDS as rows of [step][piece][4 k-groups][8] fp16 with
// a 288-B pitch (18 x 16-B slots: the 16-row fragment reads are conflict free, searched offline); the
// prologue (GroupNorm affine, or LayerNorm + adaLN modulate with per-row statistics) is applied on the
// way into LDS with its per-(image, channel) tables staged per K stage. B fragments from L2 into a 2-deep
// register ring. Epilogue staged through LDS so every lane stores 16 B. A launch whose last round of tiles is
// at most half full splits those tiles over K (the split-K tail: GemmArgs::sk_*, linear_k32 below).
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"

namespace dm {

namespace {

#ifdef DM_K32_STAMPS
// Diagnostic build only (tools/linear_stamps.py): per block of launches with K == g_lin_stamp_k (a device
// symbol the tool sets), wave 0's s_memtime at the start, after the prologue, after the K loop and at the
// end, plus s_memrealtime start / end. Written to this buffer only.
__device__ unsigned long long g_lin_stamps[65536][8];
__device__ int g_lin_stamp_k;
#define LIN_STAMP(k)                                                                                         \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536 && g.K == g_lin_stamp_k) g_lin_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define LIN_RSTAMP(k)                                                                                        \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536 && g.K == g_lin_stamp_k) g_lin_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define LIN_STAMP(k) do {} while (0)
#define LIN_RSTAMP(k) do {} while (0)
#endif

constexpr int kLP = 144;   // LDS row pitch in fp16 (288 B) of one 64-channel stage
constexpr int kLBM = 128;  // block rows
constexpr int kLGM = 4;    // M tiles per group of the tile order

// PRO: 0 none, 1 GroupNorm affine (pro_scale / pro_shift [img][K]), 2 LayerNorm + modulate, 3 pre-split A
// (GemmArgs::as: no conversion on the way into LDS -- the split of A costs VALU work once per N tile
// otherwise, which with K = 256 (the UNet's qkv) left the MFMAs idle most of the K loop).
// Wave tiles WM x WN = 128 x 32 (each wave all 128 rows from LDS, its own 32 weight columns: every B
// fragment fetched once per block, half the L2 traffic of 64 x 64 wave tiles, where each weight fragment is
// loaded by both row waves).
// One 32 x WN slab (acc * rowscale * 2^-ea, no bias yet) of the qkv projection -> the attention operand
// planes: q * alpha * 2^ea and k * b_scale * 2^eb as [B][heads][2][L][Dh], v * 2^ev transposed as
// [B][heads][2][Dh][L] (plane 0 = fp16(x), plane 1 = fp16(x - plane 0)), 16-B stores. The slab's columns lie
// in one of q / k / v (3C and C are multiples of 32; with the legacy per-head [q; k; v] order Dh is), but with
// a head dim that 32 does not divide (DiT's 72, or 80, at L = 64) they span two heads: every 8-column group is
// located on its own (Dh % 8 == 0, linear_k32_ok).
template <int WN>
__device__ __forceinline__ void plane_slab(const GemmArgs& g, const float* st, int EP, int row0, int col0, int lane,
                                           f4 bias4, bool& bad) {
  if (col0 >= g.N) return;
  const int Dh = g.ap_Dh, C = g.ap_heads * Dh;
  auto locate = [&](int col, int& part, int& h, int& d) {
    if (g.ap_vonly) {
      part = 2;
      h = col / Dh;
      d = col - h * Dh;
    } else if (g.ap_legacy) {
      h = col / (3 * Dh);
      part = (col - h * 3 * Dh) / Dh;
      d = col - h * 3 * Dh - part * Dh;
    } else {
      part = col / C;
      h = (col - part * C) / Dh;
      d = col - part * C - h * Dh;
    }
  };
  int part, h0, d0;
  locate(col0, part, h0, d0);
  const float scale = part == 0 ? g.ap_alpha : part == 1 ? g.ap_bscale : 1.f;
  const bool use_scale = part == 0 ? g.ap_alpha != 1.0f : part == 1 && g.ap_bscale != 0.0f && g.ap_bscale != 1.0f;
  const float pw = ldexpf(1.f, part == 0 ? g.ap_ea : part == 1 ? g.ap_eb : g.ap_ev);
  const size_t plane = (size_t)g.ap_L * Dh;
  auto split8 = [&](const float (&x)[8], f16x8& hi, f16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float y = (use_scale ? x[e] * scale : x[e]) * pw;
      const _Float16 h0 = (_Float16)y;
      hi[e] = h0;
      lo[e] = (_Float16)(y - (float)h0);
      bad |= fabsf(y) > 65504.f;
    }
  };
  const float* bias = g.bias ? g.bias + col0 : nullptr;
  if (part < 2) {  // q / k: 8 consecutive d of one token per item
    _Float16* dst = part == 0 ? g.ap_q : g.ap_k;
    constexpr int G8 = WN / 8;
    for (int it = lane; it < 32 * G8; it += 64) {
      const int row = it / G8, c8 = it - row * G8;
      const int m = row0 + row;
      if (m >= g.M) continue;
      int pt, h, d;
      locate(col0 + 8 * c8, pt, h, d);
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = st[row * EP + 8 * c8 + e] + (bias ? bias[8 * c8 + e] : 0.f);
      f16x8 hi, lo;
      split8(x, hi, lo);
      const int b = m / g.ap_L, tok = m - b * g.ap_L;
      _Float16* p = dst + ((size_t)b * g.ap_heads + h) * 2 * plane + (size_t)tok * Dh + d;
      *reinterpret_cast<f16x8*>(p) = hi;
      *reinterpret_cast<f16x8*>(p + plane) = lo;
    }
  } else {  // v: 8 consecutive tokens of one d per item
    for (int it = lane; it < WN * 4; it += 64) {
      const int col = it % WN, r8 = it / WN;
      const int m = row0 + 8 * r8;  // tokens m .. m + 7 lie in one image (L % 8 == 0)
      if (m >= g.M) continue;
      int pt, h, d;
      locate(col0 + col, pt, h, d);
      float x[8];
      const float bc = bias ? bias[col] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = st[(8 * r8 + e) * EP + col] + bc;
      f16x8 hi, lo;
      split8(x, hi, lo);
      const int b = m / g.ap_L, tok = m - b * g.ap_L;
      _Float16* p = g.ap_v + ((size_t)b * g.ap_heads + h) * 2 * plane + (size_t)d * g.ap_L + tok;
      *reinterpret_cast<f16x8*>(p) = hi;
      *reinterpret_cast<f16x8*>(p + plane) = lo;
    }
  }
}

// The whole 128 x 128 block tile (acc * rowscale * 2^-ea in LDS as [128][TP] fp32) -> the attention operand
// planes, with every 16 consecutive threads storing 256 contiguous bytes of a plane: q / k rows of 8
// consecutive d per thread (16 threads per token), v as 4 columns x 8 tokens per thread (16 threads per
// d row of the tile's 128 tokens) -- instead of the per-wave slabs' 64-B row pieces and 512-B strided v
// stores. The tile's rows lie in one image (L % 128 == 0); per 8-column group one of q / k / v and one head.
__device__ __forceinline__ void plane_block(const GemmArgs& g, const float* tile, int TP, int m0, int n0, int t,
                                            bool& bad) {
  const int Dh = g.ap_Dh, C = g.ap_heads * Dh;
  const size_t plane = (size_t)g.ap_L * Dh;
  auto col_map = [&](int col, int& part, int& h, int& d) {
    if (g.ap_vonly) {
      part = 2;
      h = col / Dh;
      d = col - h * Dh;
    } else if (g.ap_legacy) {
      h = col / (3 * Dh);
      part = (col - h * 3 * Dh) / Dh;
      d = col - h * 3 * Dh - part * Dh;
    } else {
      part = col / C;
      h = (col - part * C) / Dh;
      d = col - part * C - h * Dh;
    }
  };
  auto split8 = [&](int part, const float (&x)[8], f16x8& hi, f16x8& lo) {
    const float scale = part == 0 ? g.ap_alpha : part == 1 ? g.ap_bscale : 1.f;
    const bool use_scale = part == 0 ? g.ap_alpha != 1.0f : part == 1 && g.ap_bscale != 0.0f && g.ap_bscale != 1.0f;
    const float pw = ldexpf(1.f, part == 0 ? g.ap_ea : part == 1 ? g.ap_eb : g.ap_ev);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float y = (use_scale ? x[e] * scale : x[e]) * pw;
      const _Float16 h0 = (_Float16)y;
      hi[e] = h0;
      lo[e] = (_Float16)(y - (float)h0);
      bad |= fabsf(y) > 65504.f;
    }
  };
  const int b = m0 / g.ap_L, tok0 = m0 - b * g.ap_L;
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  {  // q / k: item (row, 8-column group), 16 groups per row; a thread keeps its column group
    const int c8 = t & 15, col = n0 + 8 * c8;
    int part, h, d;
    col_map(min(col, g.N - 1), part, h, d);
    if (col < g.N && part < 2) {
      const f4 b0 = g.bias ? *reinterpret_cast<const f4*>(g.bias + col) : zero4;
      const f4 b1 = g.bias ? *reinterpret_cast<const f4*>(g.bias + col + 4) : zero4;
      _Float16* base = (part == 0 ? g.ap_q : g.ap_k) + ((size_t)b * g.ap_heads + h) * 2 * plane + (size_t)tok0 * Dh + d;
#pragma unroll 2
      for (int row = t >> 4; row < 128; row += 16) {
        if (m0 + row >= g.M) break;
        const f4 v0 = *reinterpret_cast<const f4*>(tile + row * TP + 8 * c8) + b0;
        const f4 v1 = *reinterpret_cast<const f4*>(tile + row * TP + 8 * c8 + 4) + b1;
        const float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        f16x8 hi, lo;
        split8(part, x, hi, lo);
        _Float16* p = base + (size_t)row * Dh;
        *reinterpret_cast<f16x8*>(p) = hi;
        *reinterpret_cast<f16x8*>(p + plane) = lo;
      }
    }
  }
  // v: item (4-column group, 8-token group), 16 token groups per column group
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int it = t + 256 * k;
    const int r8 = it & 15, cq = it >> 4, col = n0 + 4 * cq;
    if (col >= g.N || m0 + 8 * r8 >= g.M) continue;  // M % 8 == 0 (L % 128 == 0)
    int part, h, d;
    col_map(col, part, h, d);
    if (part != 2) continue;
    const f4 bc = g.bias ? *reinterpret_cast<const f4*>(g.bias + col) : zero4;
    f4 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = *reinterpret_cast<const f4*>(tile + (8 * r8 + e) * TP + 4 * cq);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = v[e][c] + bc[c];
      f16x8 hi, lo;
      split8(2, x, hi, lo);
      _Float16* p = g.ap_v + ((size_t)b * g.ap_heads + h) * 2 * plane + (size_t)(d + c) * g.ap_L + tok0 + 8 * r8;
      *reinterpret_cast<f16x8*>(p) = hi;
      *reinterpret_cast<f16x8*>(p + plane) = lo;
    }
  }
}

// linear_presplit_a: one thread per 8 consecutive channels (one k-group of one K = 32 step) of a row:
// the linear_k32 prologue's expressions (finish_a), the split, piece 0 at [m][kk][0][kg], piece 1 at [m][kk][1][kg].
template <int PRO>
__global__ void __launch_bounds__(256) presplit_a_kernel(GemmArgs g, void* out_) {  // (void*: a demangled name)
  _Float16* out = reinterpret_cast<_Float16*>(out_);
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int per_row = g.K / 8;
  if (i >= (long)g.M * per_row) return;
  const int m = (int)(i / per_row), c = (int)(i - (long)m * per_row) * 8;
  const float* a = g.A + (size_t)m * g.lda + c;
  f4 v0 = *reinterpret_cast<const f4*>(a), v1 = *reinterpret_cast<const f4*>(a + 4);
  if (PRO == 1) {
    const size_t o = (size_t)(m / g.pro_rows) * g.K + c;
    const f4 s0 = *reinterpret_cast<const f4*>(g.pro_scale + o), s1 = *reinterpret_cast<const f4*>(g.pro_scale + o + 4);
    const f4 h0 = *reinterpret_cast<const f4*>(g.pro_shift + o), h1 = *reinterpret_cast<const f4*>(g.pro_shift + o + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = v0[e] * s0[e] + h0[e];
      v1[e] = v1[e] * s1[e] + h1[e];
    }
  } else if (PRO == 2) {
    const float2 lns = g.ln_stats[m];
    const size_t o = (size_t)(m / g.ln_rows) * g.ln_pitch + c;
    const f4 s0 = *reinterpret_cast<const f4*>(g.ln_scale + o), s1 = *reinterpret_cast<const f4*>(g.ln_scale + o + 4);
    const f4 h0 = *reinterpret_cast<const f4*>(g.ln_shift + o), h1 = *reinterpret_cast<const f4*>(g.ln_shift + o + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = ((v0[e] - lns.x) * lns.y) * (1.0f + s0[e]) + h0[e];
      v1[e] = ((v1[e] - lns.x) * lns.y) * (1.0f + s1[e]) + h1[e];
    }
  }
  if (g.alpha != 1.0f) {
    v0 = v0 * g.alpha;
    v1 = v1 * g.alpha;
  }
  const float apow = ldexpf(1.f, g.split_ea);
  bool bad = false;
  f16x8 pc[2];
  Split<2>::split(v0 * apow, v1 * apow, pc, bad);
  _Float16* dst = out + (size_t)m * 2 * g.K + (c / 32) * 64 + ((c % 32) / 8) * 8;
  *reinterpret_cast<f16x8*>(dst) = pc[0];
  *reinterpret_cast<f16x8*>(dst + 32) = pc[1];
  if (bad && g.range_flag) *g.range_flag = 1;
}

// 128 x 128 blocks of four 128 x 32 wave tiles (the 8-wave 128 x 256 and the 128 x 64 forms measured -2 % and -7 %
// on DiT-XL/2 and were removed in round 5)
template <int PRO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) linear_k32_kernel(GemmArgs g) {
  constexpr int WM = 128, WN = 32, NW = 4;
  constexpr int BM = kLBM, BN = 32 * NW * WM / BM * WN / 32, TM = WM / 16, TN = WN / 16, WD = 2, NWN = BN / WN;
  static_assert((BM / WM) * NWN == NW, "one wave tile per wave");
  static_assert(NW == 4 || PRO == 3, "8 waves: pre-split A only");
  constexpr int NT = NW * 64, RS = NT / 16, NU = BM / RS;   // PRO 3 loader: row step, rows per thread
  constexpr int STAGE = BM * kLP;  // fp16 elements per buffer
  __shared__ __attribute__((aligned(16))) _Float16 abuf[2 * STAGE];
  // prologue tables of three K stages (staged two stages ahead): [stage % 3][image of the tile][scale, shift][ch]
  __shared__ __attribute__((aligned(16))) float tab[3][2][2][64];

  LIN_RSTAMP(5);
  LIN_STAMP(0);
  const int M = g.M, N = g.N, K = g.K;
  // Grouped tile order: consecutive tiles (one XCD, xcd_remap_p) sweep all N tiles for a group of kLGM M
  // tiles, M fastest, so the group's kLGM blocks of one weight tile run together and fetch it from the
  // memory side once per group instead of once per M tile (DiT-XL/2 qkv: 16 MB of split weights re-read
  // for each of 128 M tiles otherwise); the group's A tiles stay in the XCD's L2 during the sweep.
  const int nN = ceil_div(N, BN), nM = ceil_div(M, BM);
  // Split-K tail (g.sk_S > 1): blocks sk_tdp .. sk_tdp + tail * S - 1 take the tiles of the last, partial
  // round, S blocks per tile, each a contiguous 1 / S of the K stages; S consecutive logical blocks of one
  // XCD share a tile (the reducer reads same-XCD slabs). The tiles before sk_tdp run whole, as without.
  // (a function of the block index, evaluated again after the K loop rather than kept live across it: the
  // loop holds all 256 VGPRs)
  auto sk_place = [&](int bx, int& bid_, int& slice_) {
    if (g.sk_S > 1 && bx >= g.sk_tdp) {
      const int v = xcd_remap_p(bx - g.sk_tdp, (int)gridDim.x - g.sk_tdp);
      bid_ = g.sk_tdp + v / g.sk_S;
      slice_ = v - (v / g.sk_S) * g.sk_S;
    } else {
      bid_ = xcd_remap_p(bx, g.sk_S > 1 ? g.sk_tdp : (int)gridDim.x);
      slice_ = 0;
    }
  };
  int bid, slice;
  sk_place((int)blockIdx.x, bid, slice);
  const int sk_S = g.sk_S > 1 && (int)blockIdx.x >= g.sk_tdp ? g.sk_S : 1;
  const int sbeg = slice * (K / 64) / sk_S;  // first K stage (64 channels) of this block
  const int tgrp = bid / (kLGM * nN), gm0 = tgrp * kLGM, gsz = min(kLGM, nM - gm0);
  const int r = bid - tgrp * (kLGM * nN);
  const int nt = r / gsz, mt = gm0 + (r - nt * gsz);
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / NWN, wn = wave % NWN;
  const int l16 = lane & 15, q = lane >> 4;

  constexpr bool TABS = PRO == 1 || PRO == 2;
  const int rows_img = PRO == 1 ? g.pro_rows : PRO == 2 ? g.ln_rows : 1;  // rows per image >= 128
  const int img0 = TABS ? m0 / rows_img : 0;
  // PRO 3 A loader: 16-B slot a3s = t & 15 (8 fp16 of one piece and k-group) of the stage's 256-B row span
  // in tile rows a3r + 16 u, u = 0 .. 7 -- every wave instruction reads 4 whole row spans (8 cache lines)
  // instead of 16 B of 64 different lines, as a row-half per thread did: those A refills cost 25 % of the
  // DiT GEMMs' time (an ablation build without A refills; fc1 / fc2 at 2B = 64: 663 -> 512 us). The in-GEMM prologues (PRO 0-2,
  // fp32 A) keep the row-half mapping: the same remap spills them past 256 VGPRs.
  const int a3s = t & 15, a3r = t >> 4;
  const f4* asp = PRO == 3 ? reinterpret_cast<const f4*>(g.as) + a3s + 16 * sbeg : nullptr;
  const size_t a3pitch = (size_t)K / 4;  // f4 per pre-split row
  const int lrow = t >> 1, lh = t & 1;  // PRO 0-2 loader: row, 32-channel half of the stage (= K32 step)
  const int am = min(m0 + lrow, M - 1);  // rows >= M: clamped, never stored
  const float* asrc = g.A + (size_t)am * g.lda + 32 * lh + 64 * sbeg;
  const int aimg = TABS ? am / rows_img - img0 : 0;  // 0 or 1
  const float2 lns = PRO == 2 ? g.ln_stats[am] : make_float2(0.f, 1.f);
  const float apow = ldexpf(1.f, g.split_ea);
  f4 ra[2][PRO == 3 ? NU : 8];  // A rows of two stages in flight (stage s in ra[s & 1])
  f4 rt;  // threads 0 .. 63: one f4 of a stage's tables
  const int ti = t >> 4, tk = (t & 15) * 4;  // table loader: (image, scale | shift) pair ti, channels tk
  auto load_a = [&](f4 (&dst)[PRO == 3 ? NU : 8], int st) {
    // whole tiles (the usual case) address their rows linearly from one per-lane base; the last, partial
    // tile clamps each row
    if constexpr (PRO == 3) {  // slot a3s of the stage's 256 B in NU rows
      if (m0 + kLBM <= M) {
        const f4* b0 = asp + (size_t)(m0 + a3r) * a3pitch + 16 * st;
#pragma unroll
        for (int u = 0; u < NU; ++u) dst[u] = b0[(size_t)(RS * u) * a3pitch];
      } else {
#pragma unroll
        for (int u = 0; u < NU; ++u) dst[u] = asp[(size_t)min(m0 + a3r + RS * u, M - 1) * a3pitch + 16 * st];
      }
    } else {
      const float* p = asrc + 64 * st;
#pragma unroll
      for (int u = 0; u < 8; ++u) dst[u] = *reinterpret_cast<const f4*>(p + 4 * u);
    }
  };
  auto load_tab = [&](int st) {
    if (TABS && t < 64) {
      const int im = min(img0 + (ti >> 1), (M - 1) / rows_img);
      const int kk = 64 * (sbeg + st) + tk;
      if (PRO == 1)
        rt = *reinterpret_cast<const f4*>(((ti & 1) ? g.pro_shift : g.pro_scale) + (size_t)im * K + kk);
      else
        rt = *reinterpret_cast<const f4*>(((ti & 1) ? g.ln_shift : g.ln_scale) + (size_t)im * g.ln_pitch + kk);
    }
  };
  auto store_tab = [&](int buf) {
    if (TABS && t < 64) *reinterpret_cast<f4*>(&tab[buf][ti >> 1][ti & 1][tk]) = rt;
  };
  bool bad = false;
  // prologue + split + LDS store of this thread's 32 channels (tables of the stage in tab[buf])
  auto finish_a = [&](const f4 (&src)[PRO == 3 ? NU : 8], int buf, int tb) {
    if constexpr (PRO == 3) {
      _Float16* d3 = abuf + buf * STAGE + a3r * kLP + a3s * 8;
#pragma unroll
      for (int u = 0; u < NU; ++u) *reinterpret_cast<f4*>(d3 + RS * u * kLP) = src[u];
      return;
    } else {
    _Float16* dst = abuf + buf * STAGE + lrow * kLP + lh * 64;
#pragma unroll
    for (int u = 0; u < 8; u += 2) {  // k-group u / 2: channels 8 (u / 2) .. + 7 of the step
      f4 v0 = src[u], v1 = src[u + 1];
      if (TABS) {
        const float* sc = &tab[tb][aimg][0][32 * lh + 4 * u];
        const float* sh = &tab[tb][aimg][1][32 * lh + 4 * u];
        const f4 s0 = *reinterpret_cast<const f4*>(sc), s1 = *reinterpret_cast<const f4*>(sc + 4);
        const f4 h0 = *reinterpret_cast<const f4*>(sh), h1 = *reinterpret_cast<const f4*>(sh + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (PRO == 1) {  // GroupNorm affine, as gemm.hip's prologue
            v0[e] = v0[e] * s0[e] + h0[e];
            v1[e] = v1[e] * s1[e] + h1[e];
          } else {  // LayerNorm (no affine) + modulate, as gemm.hip's prologue
            v0[e] = ((v0[e] - lns.x) * lns.y) * (1.0f + s0[e]) + h0[e];
            v1[e] = ((v1[e] - lns.x) * lns.y) * (1.0f + s1[e]) + h1[e];
          }
        }
      }
      if (g.alpha != 1.0f) {
        v0 = v0 * g.alpha;
        v1 = v1 * g.alpha;
      }
      f16x8 pc[2];
      Split<2>::split(v0 * apow, v1 * apow, pc, bad);
      *reinterpret_cast<f16x8*>(dst + (u >> 1) * 8) = pc[0];       // piece 0 at slot 8 s + q
      *reinterpret_cast<f16x8*>(dst + 32 + (u >> 1) * 8) = pc[1];  // piece 1 at slot 8 s + 4 + q
    }
    }
  };

  // ---- B: fragment images [16-slice][32-col group][piece][lane group][32][8]; K32 step kk reads
  // 16-slices 2 kk + (q >> 1), lane group q & 1
  const int ngrp = ceil_div(N, 32);
  const size_t sl = (size_t)ngrp * 1024;
  const _Float16* wbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + l16;
    const int grp = min(col >> 5, ngrp - 1);
    wbase[j] = reinterpret_cast<const _Float16*>(g.ws) + (size_t)((q >> 1) + 4 * sbeg) * sl + (size_t)grp * 1024 +
               ((q & 1) * 32 + (col & 31)) * 8;
  }
  f16x8 bq[WD][TN][2];
  auto load_b = [&](f16x8 (&dst)[TN][2], int kk) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) dst[j][p] = *reinterpret_cast<const f16x8*>(wbase[j] + (size_t)(2 * kk) * sl + p * 512);
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf, int s, const f16x8 (&bv)[TN][2]) {
    const _Float16* As = abuf + buf * STAGE + (wm * WM + l16) * kLP + s * 64 + q * 8;
    f16x8 av[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + i * 16 * kLP + p * 32);
    // all of the step's A fragment reads issued before its first MFMA (they return in order, so MFMA i waits
    // for reads 0 .. 2i + 1 only); left to itself the compiler recycles two registers and waits on each read
    // behind 2-4 MFMAs (SQ_WAIT_INST_ANY 58 % of wave cycles, MFMA busy 40 %). Not with the in-GEMM
    // prologues (PRO 1 / 2): their tables and split leave no room for 16 fragments (scratch spills).
    if (PRO == 0 || PRO == 3) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][1], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][0], acc[i][j], 0, 0, 0);
      }
  };

  const int nst = (slice + 1) * (K / 64) / sk_S - sbeg, nkk = 2 * nst;  // this block's K stages and steps
#pragma unroll
  for (int d = 0; d < WD; ++d) load_b(bq[d], min(d, nkk - 1));
  load_a(ra[0], 0);
  load_a(ra[1], min(1, nst - 1));
  load_tab(0);
  store_tab(0);
  load_tab(min(1, nst - 1));
  store_tab(1);
  __syncthreads();
  finish_a(ra[0], 0, 0);
  __syncthreads();
  LIN_STAMP(1);
  // One barrier per stage. Stage st: the A rows of stage st + 2 (into the registers stage st's rows
  // left) and the tables of stage st + 2 are loaded before step 0 -- two stages of MFMAs to land (K = 256
  // GEMMs have 4 stages: one stage did not cover the load latency); after step 1 the tables go to LDS
  // and stage st + 1 is finished into the other buffer (its tables were stored a stage earlier).
  auto stage = [&](int st, f4 (&cur)[PRO == 3 ? NU : 8], f4 (&nxt)[PRO == 3 ? NU : 8]) {
    load_a(cur, min(st + 2, nst - 1));
    load_tab(min(st + 2, nst - 1));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int kk = 2 * st + s;
      compute(st & 1, s, bq[s]);
      load_b(bq[s], min(kk + WD, nkk - 1));
      __builtin_amdgcn_sched_barrier(0);
    }
    store_tab((st + 2) % 3);
    finish_a(nxt, (st + 1) & 1, (st + 1) % 3);
    __syncthreads();
  };
  for (int st = 0; st < nst; st += 2) {
    stage(st, ra[0], ra[1]);
    if (st + 1 < nst) stage(st + 1, ra[1], ra[0]);
  }
  LIN_STAMP(2);
  if (g.sk_S > 1 && (int)blockIdx.x >= g.sk_tdp) {
    const int sk_S = g.sk_S;
    int bx = (int)blockIdx.x, bid, slice;
    asm volatile("" : "+s"(bx));  // recomputed here, not carried through the loop
    sk_place(bx, bid, slice);
    // Split-K hand-off (cdna_hip_programming.md §5 'In-launch split-K reduction', its write-through form):
    // every slice stores its accumulators as a 64-KB slab in register order with sc1 (write-through) 16-B
    // buffer stores, 1 KB per wave instruction, drains them (every wave), and one lane draws a ticket -- no
    // release fence, whose L2 write-back of every dirty line of the XCD cost more than the tail saved; the
    // block drawing S - 1 resets the counter, acquires, and sums the S slabs in slice order (its own from
    // memory too: the same sum whichever block arrives last, so the result is deterministic), then runs the
    // epilogue. Nobody waits: no residency assumption.
    const int tt = bid - g.sk_tdp;
    constexpr int SLAB = NW * TM * TN * 64;  // f4 per slab
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(g.sk_ws, 0, g.sk_cap * 65536, 0x00020000);
    const int sbyte = (((tt * sk_S + slice) * SLAB) + wave * (TM * TN * 64) + lane) * 16;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, sbyte + (i * TN + j) * 1024,
                                               0, 16 /* sc1 */);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(&tab[0][0][0][0]);  // (the tables are dead after the K loop)
    if (t == 0) {
      const unsigned tk = __hip_atomic_fetch_add(g.sk_cnt + tt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = tk == (unsigned)(sk_S - 1);
      if (is_last) {
        __hip_atomic_store(g.sk_cnt + tt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = is_last;
    }
    __syncthreads();
    if (!*last) {
      if (bad && g.range_flag) *g.range_flag = 1;
      return;
    }
    const f4* s0 = reinterpret_cast<const f4*>(g.sk_ws) + (size_t)tt * sk_S * SLAB + wave * (TM * TN * 64) + lane;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = s0[(i * TN + j) * 64];
    for (int s = 1; s < sk_S; ++s) {
      f4 v[TM][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) v[i][j] = s0[(size_t)s * SLAB + (i * TN + j) * 64];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] += v[i][j];
    }
  }
  // ---- epilogue: per 32-row slab of the wave's 64 rows, acc * rowscale * 2^-ea to LDS ([32][68] fp32),
  // then 4 consecutive columns per lane: bias, residual / gated residual, activation, 16-B store
  constexpr int EP = WN + 4, LPR = WN / 4, RPI = 64 / LPR;
  float* stg = reinterpret_cast<float*>(abuf) + wave * 32 * EP;
  const float unscale = ldexpf(1.f, -g.split_ea);
  float cs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) cs[j] = g.ws_rowscale[min(n0 + wn * WN + j * 16 + l16, N - 1)] * unscale;
  const int c4 = lane % LPR, rsub = lane / LPR;
  const int ncol = n0 + wn * WN + 4 * c4;
  const bool c_ok = ncol < N;  // N % 4 == 0
  const int nc = c_ok ? ncol : 0;
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const f4 bias4 = g.bias ? *reinterpret_cast<const f4*>(g.bias + nc) : zero4;
  if (NW == 4 && g.ap_q && g.ap_L % BM == 0) {  // attention planes from the whole block tile (the loop ended on a barrier)
    constexpr int TP = BN + 4;
    static_assert(NW != 4 || BM * TP * 4 <= 2 * STAGE * 2, "block tile fits the stage buffers");
    float* tile = reinterpret_cast<float*>(abuf);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) tile[(wm * WM + 16 * i + 4 * q + r) * TP + wn * WN + 16 * j + l16] = acc[i][j][r] * cs[j];
    __syncthreads();
    plane_block(g, tile, TP, m0, n0, t, bad);
    if (bad && g.range_flag) *g.range_flag = 1;
    LIN_STAMP(3);
    LIN_RSTAMP(6);
    return;
  }
#pragma unroll
  for (int h = 0; h < WM / 32; ++h) {
#pragma unroll
    for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[((i - 2 * h) * 16 + 4 * q + r) * EP + j * 16 + l16] = acc[i][j][r] * cs[j];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's slab is visible to its reads
    __builtin_amdgcn_wave_barrier();
    const int row0 = m0 + wm * WM + 32 * h;
    if (g.ap_q) {  // attention operand planes (conv_patch3.hip attn_plane_epilogue's expressions)
      plane_slab<WN>(g, stg, EP, row0, n0 + wn * WN, lane, bias4, bad);
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    f4 rs4[32 / RPI], gt4[32 / RPI];
    if (g.res) {
#pragma unroll
      for (int it = 0; it < 32 / RPI; ++it) {
        const int m = min(row0 + it * RPI + rsub, M - 1);
        rs4[it] = *reinterpret_cast<const f4*>(g.res + (size_t)(g.res_mod > 0 ? m % g.res_mod : m) * g.ld_res + nc);
        gt4[it] = g.gate ? *reinterpret_cast<const f4*>(g.gate + (size_t)(m / g.gate_rows) * g.gate_pitch + nc) : zero4;
      }
    }
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int row = it * RPI + rsub;
      const int m = row0 + row;
      f4 v = *reinterpret_cast<const f4*>(stg + row * EP + 4 * c4);
      if (g.bias) v = v + bias4;
      if (g.res) v = g.gate ? rs4[it] + gt4[it] * v : v + rs4[it];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (g.act == 1) v[e] = silu_f(v[e]);
        else if (g.act == 2) v[e] = gelu_tanh_f(v[e]);
      }
      if (g.c_split) {  // linear_presplit_a's expressions (alpha 1), 4 columns = half a k-group
        const float cp = ldexpf(1.f, g.c_split_ea);
        f16x4 h0, h1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y = v[e] * cp;
          const _Float16 a0 = (_Float16)y;
          h0[e] = a0;
          h1[e] = (_Float16)(y - (float)a0);
          bad |= fabsf(y) > 65504.f;
        }
        if (m < M && c_ok) {
          _Float16* d = g.c_split + (size_t)m * 2 * N + (ncol >> 5) * 64 + (ncol & 31);
          *reinterpret_cast<f16x4*>(d) = h0;
          *reinterpret_cast<f16x4*>(d + 32) = h1;
        }
      } else if (m < M && c_ok) {
        *reinterpret_cast<f4*>(g.C + (size_t)m * g.ldc + ncol) = v;
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next slab reuses the region
  }
  if (bad && g.range_flag) *g.range_flag = 1;
  LIN_STAMP(3);
  LIN_RSTAMP(6);
}

}  // namespace

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_lin_stamps(void* host, int nblocks, int k) {
  if (!host) return hipMemcpyToSymbol(HIP_SYMBOL(g_lin_stamp_k), &k, sizeof(int)) == hipSuccess ? 0 : -2;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lin_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

bool linear_k32_ok(const GemmArgs& g) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!(g.ws && g.ws_rowscale && g.split == 2 && g.Z1 == 1 && g.Z2 == 1 && !g.b_kn && g.b_scale == 0.0f)) return false;
  if (g.K % 64 != 0 || g.N % 4 != 0 || g.lda % 4 != 0 || g.ldc % 4 != 0 || !al16(g.A) || !al16(g.C)) return false;
  if (g.bias && !al16(g.bias)) return false;
  if (g.res && (g.ld_res % 4 != 0 || !al16(g.res))) return false;
  if (g.gate && (g.gate_pitch % 4 != 0 || !al16(g.gate))) return false;
  if (g.gn_part) return false;
  if (g.pro_scale && (g.pro_rows < kLBM || !al16(g.pro_scale) || !al16(g.pro_shift))) return false;
  if (g.ln_stats && (g.ln_rows < kLBM || g.ln_pitch % 4 != 0 || !al16(g.ln_scale) || !al16(g.ln_shift))) return false;
  if (g.pro_scale && g.ln_stats) return false;
  if (g.as && (g.pro_scale || g.ln_stats || (reinterpret_cast<uintptr_t>(g.as) & 15) != 0)) return false;
  if (g.c_split && (g.N % 64 != 0 || g.ap_q || (reinterpret_cast<uintptr_t>(g.c_split) & 15) != 0)) return false;
  if (g.ap_vonly && (!g.ap_q || g.ap_legacy)) return false;
  // attention planes: 8-column groups of one head (plane_slab / plane_block), q / k / v never inside one slab
  if (g.ap_q && (g.ap_Dh % 8 != 0 || (g.ap_heads * g.ap_Dh) % 32 != 0 || (g.ap_legacy && g.ap_Dh % 32 != 0)))
    return false;
  return true;
}

int linear_presplit_a(const GemmArgs& g, _Float16* out, hipStream_t st) {
  DM_REQUIRE(g.K % 64 == 0 && g.lda % 4 == 0 && (reinterpret_cast<uintptr_t>(g.A) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(out) & 15) == 0 && !(g.pro_scale && g.ln_stats),
             "linear_presplit_a: K % 64 == 0 and 16-byte aligned rows");
  const long n = (long)g.M * (g.K / 8);
  const int blocks = (int)((n + 255) / 256);
  if (g.pro_scale)
    hipLaunchKernelGGL(presplit_a_kernel<1>, dim3(blocks), dim3(256), 0, st, g, (void*)out);
  else if (g.ln_stats)
    hipLaunchKernelGGL(presplit_a_kernel<2>, dim3(blocks), dim3(256), 0, st, g, (void*)out);
  else
    hipLaunchKernelGGL(presplit_a_kernel<0>, dim3(blocks), dim3(256), 0, st, g, (void*)out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

namespace {
struct LinSlots {
  int per_cu = 0, cus = 0;
};
const LinSlots& lin_slots() {
  static const LinSlots s = [] {
    LinSlots r;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&r.per_cu, linear_k32_kernel<3>, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&r.cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      r = LinSlots{};
    }
    return r;
  }();
  return s;
}
}  // namespace

int linear_k32_slots() { return lin_slots().per_cu * lin_slots().cus; }

namespace {
// The split-K tail's ways S for a GEMM of `tiles` 128 x 128 tiles and K / 64 stages with room for `cap` slices
// (1: no split), on this device's slots (see linear_k32 below).
int sk_ways(int tiles, int nst, int cap) {
  const int P = linear_k32_slots(), cus = lin_slots().cus;
  if (nst < 2 || P <= 0) return 1;
  const int tail = tiles % P;
  // (the tail's first block index a multiple of 8: sk_place's XCD-aware remap then keeps a tile's slices on one
  // XCD under round-robin placement -- speed only; correctness rests on the write-through slab stores and the
  // reducer's agent-scope acquire, which hold across XCDs too)
  if (tail <= 0 || 2 * tail > P || (tiles - tail) % 8 != 0) return 1;
  int S = 1;
  while (2 * S <= 8 && 2 * S <= nst && tail * 2 * S <= cus && tail * 2 * S <= cap) S *= 2;
  return S;
}
}  // namespace

int linear_k32(const GemmArgs& g_in, hipStream_t st) {
  DM_REQUIRE(linear_k32_ok(g_in), "linear_k32: needs pre-split weights, K % 64 == 0, 16-byte aligned 4-column rows");
  GemmArgs g = g_in;
  const int tiles = ceil_div(g.M, kLBM) * ceil_div(g.N, 128);
  int blocks = tiles;
  g.sk_S = 1;
  g.sk_tdp = 0;
  // Split-K of the last, partial round: with T tiles on P resident blocks (2 per CU) the last round holds
  // T % P tiles and leaves the rest of the chip idle (DiT-XL/2's N = 1152 GEMMs at 2B = 64: 1152 tiles = 2.25
  // rounds of 512). When that tail is at most half a round, its tiles are split S ways over K (S a power of
  // two, S <= the K stages) with tail * S <= the CU count: one block per CU, 1 / S of the K loop each. (Filling
  // both slots of every CU measured slower: on DiT-XL/2 C5 S = 2 +1.5 %, S = 4 -0.6 % against no split; the
  // tail's unsplit tiles already run one per CU, at a CU's whole issue rate.) Those tiles' sums are re-associated (slice partials summed in slice
  // order): not bit-identical to the whole-K tile, so a row's result depends on whether its tile is in the
  // tail (DM_LIN_SK=0: every tile whole).
  if (g.sk_ws && g.sk_cnt) {  // (the slots are queried at plan build)
    const int S = sk_ways(tiles, g.K / 64, g.sk_cap);
    if (S > 1) {
      g.sk_S = S;
      g.sk_tdp = tiles - tiles % linear_k32_slots();
      blocks = g.sk_tdp + (tiles - g.sk_tdp) * S;
      note_launch("linear_k32_sk");
    }
  }
  if (g.as)
    hipLaunchKernelGGL(linear_k32_kernel<3>, dim3(blocks), dim3(256), 0, st, g);
  else if (g.pro_scale)
    hipLaunchKernelGGL(linear_k32_kernel<1>, dim3(blocks), dim3(256), 0, st, g);
  else if (g.ln_stats)
    hipLaunchKernelGGL(linear_k32_kernel<2>, dim3(blocks), dim3(256), 0, st, g);
  else
    hipLaunchKernelGGL(linear_k32_kernel<0>, dim3(blocks), dim3(256), 0, st, g);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm

/* Test hook (tests/test_gpu_r5.py): one linear_k32 launch on weights W [N][K] split here, A fp32 rows (presplit 0:
 * in-GEMM split, with the GroupNorm affine of pro_scale / pro_shift [M / pro_rows][K] when given; 1: through
 * linear_presplit_a, PRO 3), C = A W^T (+ bias, + res), 2^ea on A; sk 1 with the split-K tail's workspace (the
 * kernel decides whether the shape has a tail to split), 0 without. Synchronous; allocates and frees its buffers. */
/* Test hook: the split-K tail's ways (1: no split) linear_k32 chooses on this device for an M x N x K GEMM with the
 * workspace dm_debug_linear_k32 gives it (one slice per resident block), and the device's resident blocks and CUs. */
extern "C" int dm_debug_linear_k32_split(int M, int N, int K, int* S, int* slots, int* cus) {
  using namespace dm;
  if (M <= 0 || N <= 0 || K <= 0 || K % 64) { set_error("bad GEMM shape"); return DM_ERR_ARG; }
  const int P = linear_k32_slots();
  if (S) *S = P > 0 ? sk_ways(ceil_div(M, kLBM) * ceil_div(N, 128), K / 64, P) : 1;
  if (slots) *slots = P;
  if (cus) *cus = lin_slots().cus;
  return DM_OK;
}

extern "C" int dm_debug_linear_k32(const float* A, int lda, const float* W, const float* bias, const float* res,
                                   int ld_res, const float* pro_scale, const float* pro_shift, int pro_rows, float* C,
                                   int ldc, int M, int N, int K, int ea, int presplit, int sk, void* stream) {
  using namespace dm;
  refresh_toggles();
  hipStream_t st = (hipStream_t)stream;
  void* ws = nullptr;
  _Float16* as = nullptr;
  float* skw = nullptr;
  unsigned* skc = nullptr;
  int rc = DM_OK;
  auto fail = [&](const char* m) {
    set_error(m);
    return DM_ERR_HIP;
  };
  do {
    if (hipMalloc(&ws, split_conv_weights_bytes(1, N, K, 2)) != hipSuccess) { rc = fail("alloc"); break; }
    if ((rc = split_conv_weights(W, 1, N, K, K, 1, 2, ws, st)) != DM_OK) break;
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K; g.Z1 = 1; g.Z2 = 1;
    g.A = A; g.lda = lda; g.C = C; g.ldc = ldc; g.alpha = 1.f;
    g.bias = bias; g.res = res; g.ld_res = ld_res;
    g.pro_scale = pro_scale; g.pro_shift = pro_shift; g.pro_rows = pro_rows;
    g.split = 2; g.split_ea = ea;
    g.ws = ws; g.ws_rowscale = split_conv_rowscale(ws, 1, N, K);
    if (presplit) {
      if (hipMalloc(&as, (size_t)M * K * 4) != hipSuccess) { rc = fail("alloc"); break; }
      if ((rc = linear_presplit_a(g, as, st)) != DM_OK) break;
      g.as = as;
      g.pro_scale = g.pro_shift = nullptr;
    }
    if (sk) {
      const int slots = linear_k32_slots();
      if (slots <= 0) { rc = fail("no occupancy"); break; }
      if (hipMalloc(&skw, (size_t)slots * 65536) != hipSuccess || hipMalloc(&skc, (size_t)slots * 4) != hipSuccess ||
          hipMemsetAsync(skc, 0, (size_t)slots * 4, st) != hipSuccess) { rc = fail("alloc"); break; }
      g.sk_ws = skw; g.sk_cnt = skc; g.sk_cap = slots;
    }
    if ((rc = linear_k32(g, st)) != DM_OK) break;
    if (hipStreamSynchronize(st) != hipSuccess) rc = fail("sync");
  } while (false);
  (void)hipStreamSynchronize(st);
  if (ws) (void)hipFree(ws);
  if (as) (void)hipFree(as);
  if (skw) (void)hipFree(skw);
  if (skc) (void)hipFree(skc);
  return rc;
}
