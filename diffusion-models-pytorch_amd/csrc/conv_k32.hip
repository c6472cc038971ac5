// 3x3 stride-1 convolution on the fp16x2 split matrix cores with 32-channel K steps:
// v_mfma_f32_16x16x32_f16 instead of conv_patch3.hip's v_mfma_f32_32x32x16_f16.
//
// Same numerics as conv_patch3.hip's fp16x2 variant (models/unet.py:16,26 convolve in fp32): every
// fp32 operand x = h0 + h1 (h0 = fp16(x), h1 = fp16(x - h0)), a*w = a1w0 + a0w1 + a0w0 issued as three
// MFMAs into one fp32 accumulator, weights scaled per output channel by a power of two that the
// epilogue undoes. What changes is the MFMA shape and with it the loop structure:
//
// * Shape. 16x16x32 and 32x32x16 take the same cycles per FLOP, but on random operands the chip holds
//   a higher clock under 16x16x32 (tools/mfma_peak.hip on MI355X: 1.87 vs 1.70 PF dense fp16,
//   MI355X_MICROARCH.md "DVFS give-back" (7)).
// * K per barrier. One chunk is 32 input channels: each of the 9 taps is one K = 32 step (48 MFMAs
//   per wave for a 64 x 64 wave tile), so a chunk is twice the matrix work of conv_patch3's 16-channel
//   chunk per barrier, and the next chunk's patch loads have twice as long to land.
//
// Operands. A (activations): per chunk the (TH + 2) x (W + 2) input patch is loaded once, GroupNorm +
// SiLU'd (tables in LDS), split and stored in LDS as rows of [piece][4 k-groups][8 fp16] with a
// 160-B pitch (10 x 16-B slots: the ds_read_b128 lane groups of a 16-row fragment are conflict free,
// the ds_write_b128 of the loader 2-way); all 9 taps read shifted fragments from it. Lane (r, q) of
// a 16x16x32 MFMA reads row r, k-group q (channels 8q .. 8q+7 of the chunk). B (weights): the fp16x2
// fragment images split_conv_weights already builds for conv_patch3 ([16-deep slice][32-column
// group][piece][2 lane groups][32][8]); lane (r, q) of column group j reads column r of the 16, k-group
// q & 1 of 16-slice (2c + (q >> 1)) * 9 + tap -- k = 8q + e of the 32-deep step, the same relabelling
// as A. Loaded from L2 into a 2-deep register ring, no LDS stage.
//
// Tiles: 128 x BN blocks (BN 128 or 64) of 4 waves, 64 x WN wave tiles, whole image rows of 32-, 16- or
// 8-pixel-wide maps (8^2 maps: two images per tile; each lane addresses its own patch row, so a 16-pixel
// fragment may span image rows). LDS: 2 x 208 x 160 B patch buffers + 9 KiB of GroupNorm tables
// = 74 KiB -> two blocks per CU.
#include <cstdlib>
#include <string>

#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"
#include "conv_epilogue.h"

namespace dm {

namespace {

constexpr int BM_K32 = 128;   // block rows (output pixels)
constexpr int kC = 32;          // input channels per chunk = K of one tap's MFMA step
constexpr int kRowH = 80;       // LDS row pitch in fp16: 160 B; [piece][k-group][8] (piece at +32)
constexpr int kMaxP = 208;      // patch pixels: 32^2 maps 6 x 34, 16^2 maps 10 x 18, 8^2 maps 2 x 10 x 10
constexpr int kMaxPW = 392;     // 512-thread wide-map tiles: 3 x 130 (128-pixel row segments), 4 x 66 (64^2 maps)
constexpr int kTab = 2048;      // GroupNorm table floats (per image of the tile: its channels' scales, then the shifts)
constexpr int kTabBig = 8192;   // variant 8: up to 2048 input channels of two images (one block per CU)
constexpr int kStats = 128;     // (image, group) pairs of the in-kernel finalize


#ifdef DM_K32_STAMPS
// Diagnostic build only (-DDM_K32_STAMPS, tools/k32_stamps.py): per block, wave 0's s_memtime at the
// kernel start, after the prologue, after the main loop, before and after the epilogue, and
// s_memrealtime at the start and the end. Written to this buffer only; no output reads them.
__device__ unsigned long long g_k32_stamps[65536][8];
#define K32_STAMP(k)                                                                        \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_k32_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define K32_RSTAMP(k)                                                                       \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_k32_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define K32_STAMP(k) do {} while (0)
#define K32_RSTAMP(k) do {} while (0)
#endif

// KSPLIT: split-K over 32-channel chunks for maps of <= 16 pixels (64-row tiles of 4 images): raw partial
// sums to kpart [ksplit][M][Cout], the epilogue in conv_splitk_reduce (conv_patch.hip), as conv_patch3.
// SUB: the sub-pixel form of nearest-2x + 3x3 (models/modules.py:60-63; conv_patch3 MODE 2): per output
// parity (py, px) a 2x2-tap conv of the low-res input with pre-combined weights (repack_subpixel), tiles
// over low-res pixels, the epilogue scattering row (iy, ix) to output pixel (2 iy + py, 2 ix + px).
// NT threads per block (256, or 512 for the 128-pixel row-segment tiles of the wide maps: 8 waves of 64 x 32
// in one block per CU, each weight fragment loaded by two waves instead of by four 64 x 128 blocks' waves),
// MAXP patch pixels per buffer.
// S2: the stride-2 3x3 (Downsample, models/modules.py:70-72): 64-pixel output tiles of whole output rows, a
// (2 TH + 1) x (2 Wo + 2) input patch whose columns are stored parity-split (even input columns -1 + 2 u' at
// u', odd ones after them), so the 16 lanes of a fragment -- consecutive output columns -- read consecutive
// patch pixels for every tap, as in the stride-1 patch (conflict-free ds_read_b128).
// T2D: 2-D tiles of wide maps (ADM's 64^2 .. 256^2): a 128-row tile is TH = 4 output rows x TW = 32 columns,
// the GEMM row index m enumerating pixels tile by tile (t2d_pixel), so the patch is the 32^2 maps' 6 x 34 and the
// kernel runs as variant 1 does there; the epilogue, the shortcut segment and the GroupNorm chunks (64 rows of
// one tile: a disjoint cover of the image) map m back to the pixel.
template <int BM, int BN, int WM, int WN, bool PRO, bool KSPLIT, bool SUB = false, int NT = 256, int MAXP = kMaxP,
          int TABF = kTab, bool S2 = false, bool T2D = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) conv_k32_kernel(ConvArgs a, PatchGeom g) {
  constexpr int NWN = BN / WN;
  static_assert((BM / WM) * NWN == NT / 64, "one wave per 64 threads");
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int SROWS = NT / 4;                       // patch pixels per loader pass (4 threads per pixel)
  constexpr int PJ = (MAXP + SROWS - 1) / SROWS;      // loader passes
  static_assert(PJ == 4, "the main loop stages passes 0-1 and 2-3");
  constexpr int PATCH = MAXP * kRowH;
  constexpr int NTAP = SUB ? 4 : 9, WD = 2, CPI = 2;  // B ring depth; chunks per loop iteration (slot = compile-time)
  __shared__ __attribute__((aligned(16))) _Float16 patch[2 * PATCH];
  __shared__ __attribute__((aligned(16))) float gtab[PRO ? TABF : 4];
  __shared__ float gstat[PRO ? 2 * kStats : 2];

  const int Ho = SUB ? a.Hin : a.Hout, Wo = SUB ? a.Win : a.Wout;  // the tiled (GEMM-row) resolution
  const int M = a.B * Ho * Wo, N = a.Cout;
  const int nN = ceil_div(N, BN);
  int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  int split = 0;
  if (KSPLIT) {
    const int per_split = gridDim.x / a.ksplit;
    split = bid / per_split;
    bid -= split * per_split;
  }
  int par = 0;
  if (SUB) {
    const int per_par = ceil_div(M, BM) * nN;
    par = bid / per_par;
    bid -= par * per_par;
  }
  const int py = par >> 1, px = par & 1;
  // tile order: N tiles fastest (the blocks of one M tile share its patch in L2; the N-slow order measured -0.6 %)
  const int mt = bid / nN, nt = bid - (bid / nN) * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HWo = Ho * Wo;
  const int b0 = m0 / HWo;
  // row-segment tiles (64 pixels of a wider row): x0 > 0; 2-D tiles: tile (m0 - b0 HWo) / BM of the image
  const int tl2 = (m0 - b0 * HWo) / BM, ntx2 = Wo / g.TW;
  const int y0 = T2D ? (tl2 / ntx2) * g.TH : (m0 - b0 * HWo) / Wo;
  const int x0 = T2D ? (tl2 - (tl2 / ntx2) * ntx2) * g.TW : (m0 - b0 * HWo) - y0 * Wo;

  K32_RSTAMP(5);
  K32_STAMP(0);
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave / NWN, wn = wave % NWN;
  const int l16 = lane & 15, q = lane >> 4;
  const int srow = t >> 2, sq = t & 3;  // loader: pixel slot, 8-channel quarter of the chunk

  // ---- patch loader geometry: pixel p = srow + SROWS j of the TB x PH x PW patch
  const float* psrc[PJ];
  bool pok[PJ];
  int pimg[PJ];
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const int PHW = g.PH * g.PW;
    const int p = srow + SROWS * j;
    const int img = p / PHW;
    const int rem = p - img * PHW;
    const int pr = rem / g.PW, pc = rem - (rem / g.PW) * g.PW;
    const int b = b0 + img;
    // S2: patch row pr = input row 2 y0 - 1 + pr; patch column pc = parity-split input column
    const int u2 = pc <= g.TW ? 2 * pc : 2 * (pc - g.TW - 1) + 1;
    const int iy = S2 ? 2 * y0 - 1 + pr : y0 - 1 + pr, ix = S2 ? u2 - 1 : x0 + pc - 1;
    const bool ok = p < g.P && b < a.B && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
    pok[j] = ok;
    const int bc = min(b, a.B - 1);
    pimg[j] = bc;
    const int iyc = min(max(iy, 0), a.Hin - 1), ixc = min(max(ix, 0), a.Win - 1);
    psrc[j] = (ok || PRO) ? a.x1 + ((size_t)(bc * a.Hin + iyc) * a.Win + ixc) * a.x1_pitch + 8 * sq
                          : kZeroPage + 8 * sq;
  }

  // ---- B operand: conv_patch3's fp16x2 fragment images, 16-column halves of the 32-column groups
  const int ngrp = ceil_div(N, 32);
  const size_t sl = (size_t)ngrp * 1024;  // fp16 elements per 16-deep slice
  const _Float16* wbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + l16;
    const int grp = min(col >> 5, ngrp - 1);  // columns >= N: clamped / zero padding, never stored
    wbase[j] = reinterpret_cast<const _Float16*>(a.ws) + (size_t)par * (a.K / 16) * sl + (size_t)grp * 1024 +
               ((q & 1) * 32 + (col & 31)) * 8;
  }
  const size_t qoff = (size_t)(q >> 1) * NTAP * sl;  // k-groups 2, 3: the chunk's second 16-slice of the tap
  // step kt = c * 9 + tap of the main segment: 16-slices 2c * 9 + tap (+ 9 for k-groups 2, 3)
  auto slice_off = [&](int kt) { return (size_t)(kt + (kt / NTAP) * NTAP) * sl + qoff; };
  f16x8 bq[WD][TN][2];
  auto load_b = [&](f16x8 (&dst)[TN][2], size_t off) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) dst[j][p] = *reinterpret_cast<const f16x8*>(wbase[j] + off + p * 512);
  };

  // ---- A-fragment patch rows of this lane (row l16 of each 16-row tile)
  int fy[TM], fx[TM], fimg[TM];
  const int tile_rows = g.TH * g.TW;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = wm * WM + i * 16 + l16;
    fimg[i] = ml / tile_rows;
    const int rem = ml - fimg[i] * tile_rows;
    fy[i] = rem / g.TW;
    fx[i] = rem - fy[i] * g.TW;
  }

  // patch registers of two loader passes: passes 0, 1 and 2, 3 of the next chunk take turns
  f4 rp[2][2];
  auto load_patch = [&](int chunk, int j0) {
    const int co = chunk * kC;
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j) {
      rp[j & 1][0] = *reinterpret_cast<const f4*>(psrc[j] + co);
      rp[j & 1][1] = *reinterpret_cast<const f4*>(psrc[j] + co + 4);
    }
  };
  const bool pro_silu = !a.pro_nosilu;
  // input-channel chunks of this block (a K split: its share of them)
  const int nchunks_all = a.Cin1 / kC;
  const int c_begin = KSPLIT ? split * nchunks_all / a.ksplit : 0;
  const int c_end = KSPLIT ? (split + 1) * nchunks_all / a.ksplit : nchunks_all;
  // GroupNorm tables: [image of the tile][channel of the block's chunks] scales, then the shifts
  const int tab_img0 = b0;
  const int tab_n = PRO ? min(b0 + g.TB, a.B) - b0 : 0;
  const int tab_c0 = c_begin * kC, tab_c = (c_end - c_begin) * kC;
  // GroupNorm + SiLU of passes j0, j0 + 1 (tables from LDS), then split and store them into buffer buf
  // (padding stays exactly 0: applied after the transform)
  bool bad = false;
  auto finish_patch = [&](int chunk, int j0, int buf) {
    _Float16* dst = patch + buf * PATCH;
    const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = j0; j < j0 + 2; ++j) {
      if (PRO) {
        const float* ts = gtab + min(pimg[j] - tab_img0, tab_n - 1) * tab_c + chunk * kC - tab_c0 + 8 * sq;
        f4 sc[2], sh[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          sc[h] = *reinterpret_cast<const f4*>(ts + 4 * h);
          sh[h] = *reinterpret_cast<const f4*>(ts + tab_n * tab_c + 4 * h);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = rp[j & 1][h][e] * sc[h][e] + sh[h][e];
            rp[j & 1][h][e] = pro_silu ? silu_fast(v) : v;
          }
      }
      const int p = srow + SROWS * j;
      if (p < MAXP) {
        f16x8 pc[2];
        const bool z = PRO && !pok[j];
        Split<2>::split(z ? zero4 : rp[j & 1][0], z ? zero4 : rp[j & 1][1], pc, bad);
        *reinterpret_cast<f16x8*>(dst + p * kRowH + sq * 8) = pc[0];
        *reinterpret_cast<f16x8*>(dst + p * kRowH + 32 + sq * 8) = pc[1];
      }
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // one K = 32 step: A rows at LDS element offsets abase[i] (lane's k-group included), B in registers
  auto compute = [&](const _Float16* As, const int (&abase)[TM], const f16x8 (&bv)[TN][2]) {
    f16x8 av[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + abase[i] + p * 32);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][1], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][0], acc[i][j], 0, 0, 0);
      }
  };
  // A row offsets of tap (ky, kx) for the lane's row of tile i
  auto a_off = [&](int i, int ky, int kx) {
    if (S2) return ((fimg[i] * g.PH + 2 * fy[i] + ky) * g.PW + (kx & 1) * (g.TW + 1) + fx[i] + (kx >> 1)) * kRowH + q * 8;
    return ((fimg[i] * g.PH + fy[i] + ky) * g.PW + fx[i] + kx) * kRowH + q * 8;
  };
  // One tap of the main loop. a0 holds tile 0's fragment of this tap on entry (read ahead) and, for
  // taps 0 .. 7, tile 0's fragment of the next tap on exit, so a tap never opens on an LDS-read wait.
  f16x8 a0[2];
  auto tap_y = [&](int tap) { return SUB ? py + (tap >> 1) : tap / 3; };
  auto tap_x = [&](int tap) { return SUB ? px + (tap & 1) : tap % 3; };
  auto read_a0 = [&](int tap, int pbuf) {
    const _Float16* As = patch + pbuf * PATCH + a_off(0, tap_y(tap), tap_x(tap));
    a0[0] = *reinterpret_cast<const f16x8*>(As);
    a0[1] = *reinterpret_cast<const f16x8*>(As + 32);
  };
  auto compute_tap = [&](int tap, int pbuf, const f16x8 (&bv)[TN][2]) {
    const _Float16* As = patch + pbuf * PATCH;
    f16x8 av[TM][2];
    av[0][0] = a0[0];
    av[0][1] = a0[1];
#pragma unroll
    for (int i = 1; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        av[i][p] = *reinterpret_cast<const f16x8*>(As + a_off(i, tap_y(tap), tap_x(tap)) + p * 32);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][1], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][0], acc[i][j], 0, 0, 0);
      }
      if (i == TM - 2 && tap + 1 < NTAP) read_a0(tap + 1, pbuf);
    }
  };

  const int kt_begin = c_begin * NTAP, kt_end = c_end * NTAP;
#pragma unroll
  for (int d = 0; d < WD; ++d) load_b(bq[d], slice_off(min(kt_begin + d, kt_end - 1)));
  // the first chunk's patch (all four passes) is in flight while the GroupNorm tables are built
  load_patch(c_begin, 0);
  f4 rq[2][2];
#pragma unroll
  for (int j = 2; j < 4; ++j) {
    rq[j & 1][0] = *reinterpret_cast<const f4*>(psrc[j] + tab_c0);
    rq[j & 1][1] = *reinterpret_cast<const f4*>(psrc[j] + tab_c0 + 4);
  }
  if (PRO) {
    if (a.gin_part) {
      // gn_finalize (gn.hip) for the tile's images, same expressions (conv_patch3.hip's in-kernel finalize).
      // The per-channel affine (and AdaGN modulation) of this thread's table entries is loaded first, with
      // the statistics partials, so the prologue waits for one round trip, not two.
      const int G = a.gin_G, cpg = a.Cin1 / G;
      constexpr int TU = TABF / 2 / NT;  // table entries per thread
      float gam[TU], bet[TU], fms[TU], fmb[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int i = min(t + NT * u, tab_n * tab_c - 1);
        const int bi = i / tab_c, c = tab_c0 + i - (i / tab_c) * tab_c;
        gam[u] = a.gin_gamma ? a.gin_gamma[c] : 1.0f;
        bet[u] = a.gin_beta ? a.gin_beta[c] : 0.0f;
        const size_t mo = (size_t)(tab_img0 + bi) * a.gin_mp + c;
        fms[u] = a.gin_ms ? a.gin_ms[mo] : 0.0f;
        fmb[u] = a.gin_mb ? a.gin_mb[mo] : 0.0f;
      }
      for (int i = t; i < tab_n * G; i += NT) {
        const int b = tab_img0 + i / G, gg = i - (i / G) * G;
        double s1 = 0, s2 = 0;
#pragma unroll 4
        for (int k = 0; k < a.gin_nchunk; ++k) {
          const double2 v = a.gin_part[((size_t)b * a.gin_nchunk + k) * G + gg];
          s1 += v.x;
          s2 += v.y;
        }
        const double mu = s1 / a.gin_n;
        double var = s2 / a.gin_n - mu * mu;
        if (var < 0) var = 0;
        gstat[2 * i] = (float)mu;
        gstat[2 * i + 1] = (float)(1.0 / sqrt(var + (double)a.gin_eps));
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int i = t + NT * u;
        if (i < tab_n * tab_c) {
          const int bi = i / tab_c, c = tab_c0 + i - (i / tab_c) * tab_c;
          const int si = 2 * (bi * G + c / cpg);
          const float mu = gstat[si], rs = gstat[si + 1];
          float sc = rs * gam[u];
          float sh = -sc * mu + bet[u];
          if (a.gin_ms) {
            const float f = 1.0f + fms[u];
            sc = sc * f;
            sh = sh * f + fmb[u];
          }
          gtab[i] = sc;
          gtab[tab_n * tab_c + i] = sh;
        }
      }
    } else {
      for (int i = t; i < tab_n * tab_c; i += NT) {
        const int bi = i / tab_c, c = tab_c0 + i - (i / tab_c) * tab_c;
        gtab[i] = a.pro_scale[(size_t)(tab_img0 + bi) * a.Cin1 + c];
        gtab[tab_n * tab_c + i] = a.pro_shift[(size_t)(tab_img0 + bi) * a.Cin1 + c];
      }
    }
    __syncthreads();
  }
  finish_patch(c_begin, 0, c_begin & 1);
  rp[0][0] = rq[0][0];
  rp[0][1] = rq[0][1];
  rp[1][0] = rq[1][0];
  rp[1][1] = rq[1][1];
  finish_patch(c_begin, 2, c_begin & 1);
  __syncthreads();
  K32_STAMP(1);
  // One barrier per chunk (double-buffered patch; the other buffer is free once every wave has passed
  // the previous chunk's barrier). The next chunk's patch goes in two halves: passes 0, 1 loaded at tap
  // 0 and finished (GroupNorm + SiLU, split, LDS store) at tap 2, passes 2, 3 loaded at tap 3 and
  // finished at tap 5 -- each load has two taps (96 MFMAs) to land.
  for (int c0 = c_begin; c0 < c_end; c0 += CPI) {
#pragma unroll
    for (int cc = 0; cc < CPI; ++cc) {
      const int c = c0 + cc;
      if (c >= c_end) break;
      const int cn = min(c + 1, c_end - 1);  // after the last chunk: reloaded into an unused buffer
#pragma unroll
      for (int tap = 0; tap < NTAP; ++tap) {
        const int kt = c * NTAP + tap;
        const int slot = (cc * NTAP + tap) % WD;
        // passes 0, 1: loaded at tap 0, finished at F1; passes 2, 3: loaded at L2, finished at F2
        constexpr int F1 = SUB ? 1 : 2, L2 = SUB ? 2 : 3, F2 = SUB ? 3 : 5;
        if (tap == 0 || tap == L2) {
          load_patch(cn, tap == 0 ? 0 : 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (tap == 0) read_a0(0, c & 1);
        compute_tap(tap, c & 1, bq[slot]);
        load_b(bq[slot], slice_off(min(kt + WD, kt_end - 1)));
        __builtin_amdgcn_sched_barrier(0);  // keep the refill WD taps ahead
        if (tap == F1 || tap == F2) finish_patch(cn, tap == F1 ? 0 : 2, (c + 1) & 1);
      }
      __syncthreads();
    }
  }

  K32_STAMP(2);
  // ---- segment 2: 1x1 product of x2 (the ResBlock shortcut), K = Cin2 in 32-channel steps, un-pipelined
  if constexpr (BM >= SROWS) {  // (the stride-2 tiles take no second segment)
  if (a.Cin2 > 0 && (!KSPLIT || split == a.ksplit - 1)) {
    constexpr int RJ = BM / SROWS;  // staging passes of SROWS rows
    const size_t s2 = (size_t)(NTAP * a.Cin1 / 16) * sl + (size_t)(q >> 1) * sl;  // 16-slices 9 Cin1/16 + 2 c2 + (q>>1)
    int abase[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) abase[i] = (wm * WM + i * 16 + l16) * kRowH + q * 8;
    const float* xsrc[RJ];
#pragma unroll
    for (int j = 0; j < RJ; ++j)
      xsrc[j] = a.x2 + (T2D ? t2d_pixel(min(m0 + srow + SROWS * j, M - 1), HWo, Wo, g.TH, g.TW)
                            : (size_t)min(m0 + srow + SROWS * j, M - 1)) * a.x2_pitch + 8 * sq;
    for (int c2 = 0; c2 < a.Cin2 / kC; ++c2) {
      f4 r[RJ][2];
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        r[j][0] = *reinterpret_cast<const f4*>(xsrc[j] + c2 * kC);
        r[j][1] = *reinterpret_cast<const f4*>(xsrc[j] + c2 * kC + 4);
      }
      load_b(bq[0], s2 + (size_t)(2 * c2) * sl);
#pragma unroll
      for (int j = 0; j < RJ; ++j) {  // rows >= M hold clamped data: never stored
        f16x8 pc[2];
        Split<2>::split(r[j][0], r[j][1], pc, bad);
        const int row = srow + SROWS * j;
        *reinterpret_cast<f16x8*>(patch + row * kRowH + sq * 8) = pc[0];
        *reinterpret_cast<f16x8*>(patch + row * kRowH + 32 + sq * 8) = pc[1];
      }
      __syncthreads();
      compute(patch, abase, bq[0]);
      __syncthreads();
    }
  }
  }
  if (bad && a.range_flag) *a.range_flag = 1;
  K32_STAMP(3);

  // ---- epilogue, staged through LDS so every lane stores 16 B: per 32 of the wave's WM rows, the
  // accumulators (lane (l16, q) holds column l16 of each 16-column tile, rows 4q .. 4q+3 of each 16-row
  // tile) go to this wave's region of the (now free) patch buffers as a [32][WN + 4] fp32 tile with the
  // row scale undone; then each lane reads 4 consecutive columns of a row (LPR lanes per row), adds bias,
  // per-image row vector and residual (16-B loads) and stores 16 B. GroupNorm statistics of the stored
  // values: every 64 of the wave's rows are one 64-pixel chunk of one image (HW % 64 == 0).
  typedef StagedEpilogue<WN> Epi;
  float* st = reinterpret_cast<float*>(patch) + wave * 32 * Epi::EP;
  const int wrow0 = m0 + wm * WM;
  Epi epi(a, M, HWo, b0, (HWo % BM) == 0, n0 + wn * WN, lane);
  if (SUB) epi.sub(Wo, a.Hout, a.Wout, py, px);
  if (T2D) epi.t2d(Wo, g.TH, g.TW);
  float cs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) cs[j] = a.ws_rowscale[min(n0 + wn * WN + j * 16 + l16, N - 1)];
#pragma unroll
  for (int h = 0; h < WM / 32; ++h) {
#pragma unroll
    for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[((i - 2 * h) * 16 + 4 * q + r) * Epi::EP + j * 16 + l16] = acc[i][j][r] * cs[j];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are visible to its reads
    __builtin_amdgcn_wave_barrier();
    if (KSPLIT)
      epi.rows_raw(st, wrow0 + 32 * h, a.kpart + (size_t)split * M * N, N);
    else
      epi.rows(st, wrow0 + 32 * h);
    __builtin_amdgcn_wave_barrier();  // the next slab's writes reuse the region
    if (!KSPLIT && a.gn_part && (h & 1)) epi.emit(wrow0 + 32 * (h - 1));
  }
  if constexpr (!KSPLIT && WM == 32) {
    if (a.gn_part) {  // 64-row tiles: the block's 64 rows are one chunk, held by the two row waves
      double s, q;
      epi.quad_sums(s, q);
      double* xr = reinterpret_cast<double*>(patch) + 6144;  // past the slabs (48 KiB in)
      if (wm == 1 && lane < Epi::LPR) {
        xr[(wn * Epi::LPR + lane) * 2] = s;
        xr[(wn * Epi::LPR + lane) * 2 + 1] = q;
      }
      __syncthreads();
      if (wm == 0) {
        s += xr[(wn * Epi::LPR + lane % Epi::LPR) * 2];
        q += xr[(wn * Epi::LPR + lane % Epi::LPR) * 2 + 1];
        epi.store_quads(s, q, m0);
      }
    }
  }
  K32_STAMP(4);
  K32_RSTAMP(6);
}

// ---- Small maps (<= 16 pixels: the 4x4 level at B = 256, M = 4096). The split-K tiles above give each CU a
// 64 x 128 tile for half of K, 32 x 64 wave tiles (24 MFMAs per 8 B-fragment loads per tap) and a second
// launch to reduce the partials. Here a block owns a whole 64 x 64 output tile (256 blocks for 4096 x 256)
// and splits K inside: waves (grp, wn), grp = wave >> 1 takes the input-channel chunks [0, h) or [h, nch)
// (h = nch / 2; the ResBlock shortcut's chunks likewise), wn = wave & 1 the 32-column half, so each wave has
// a 64 x 32 tile: 24 MFMAs per 4 B-fragment loads, every weight fragment loaded once per block. Per loop
// iteration the two groups compute chunks i and h + i from their own double-buffered patch images (4 x 144
// pixels x 160 B = 90 KiB: one block per CU) while all four waves load and finish the next pair. The two
// partial tiles meet in LDS as (p0 * s) + (p1 * s) -- the split-K reduction's expression, with its chunk
// ranges: the same bits as the two-launch path -- and the epilogue emits the consumer's GroupNorm
// statistics per image (the image is the whole 64-pixel-or-less chunk), as conv_splitk_reduce_gn did.
constexpr int kSP = 144;      // patch pixels: 4 images of 4 x 4 with their halo (4 x 6 x 6)
constexpr int kTabS = 4096;   // GroupNorm tables: 4 images x 512 channels x (scale, shift)
constexpr int kStatsS = 4 * 64;

// NW = 8 (default): 8 waves, (grp, wn, wm): each wave a 32 x 32 tile (TM = 2), two waves per SIMD, so one wave's
// LDS / L2 waits overlap the other's MFMAs (the 4-wave form waited on each tap's fragment reads with its matrix
// pipe idle). Every output element's MFMA sequence and K split are those of NW = 4: bit-identical results.
template <bool PRO, int NW>
__global__ void __launch_bounds__(NW * 64) conv_k32s_kernel(ConvArgs a, PatchGeom g) {
  constexpr int NT = NW * 64, SR = NT / 4;   // threads; loader rows per pass ((pixel, quarter) items)
  constexpr int BM = 64, BN = 64, TM = NW == 8 ? 2 : 4, TN = 2, WD = 2;
  constexpr int PJ = (2 * kSP + SR - 1) / SR;  // loader passes over the pair's 2 x 144 items: 5 (NW 4) / 3 (NW 8)
  constexpr int PATCH = kSP * kRowH;
  // one LDS array: [group][buffer] patch images, then the GroupNorm tables and statistics
  __shared__ __attribute__((aligned(16))) _Float16 patch[4 * PATCH];
  __shared__ __attribute__((aligned(16))) float gtab[PRO ? kTabS : 4];
  __shared__ float gstat[PRO ? 2 * kStatsS : 2];

  const int Ho = a.Hout, Wo = a.Wout, HWo = Ho * Wo;
  const int M = a.B * HWo, N = a.Cout;
  const int nN = ceil_div(N, BN);
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int mt = bid / nN, nt = bid - (bid / nN) * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int b0 = m0 / HWo;  // tiles hold whole images (HWo divides 64)

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int grp = NW == 8 ? wave >> 2 : wave >> 1, wn = NW == 8 ? (wave >> 1) & 1 : wave & 1;
  const int wm = NW == 8 ? wave & 1 : 0;   // row half (NW 8)
  const int l16 = lane & 15, q = lane >> 4;
  const int srow = t >> 2, sq = t & 3;
  const int nch = a.Cin1 / kC, h = nch / 2;
  const int n2 = a.Cin2 / kC, h2 = n2 / 2;

  // ---- loader: pass j covers item p = srow + SR j of the pair's 2 x 144 (pixel, quarter) items; p < 144 is
  // group 0's chunk, the rest group 1's
  const float* psrc[PJ];
  bool pok[PJ];
  int pimg[PJ];
  const int PHW = g.PH * g.PW;
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const int p = srow + SR * j;
    const int pg = p >= kSP ? 1 : 0, pp = p - pg * kSP;
    const int img = pp / PHW;
    const int rem = pp - img * PHW;
    const int pr = rem / g.PW, pc = rem - (rem / g.PW) * g.PW;
    const int b = b0 + img;
    const int iy = pr - 1, ix = pc - 1;
    const bool ok = p < 2 * kSP && pp < g.P && b < a.B && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
    pok[j] = ok;
    const int bc = min(b, a.B - 1);
    pimg[j] = bc;
    const int iyc = min(max(iy, 0), a.Hin - 1), ixc = min(max(ix, 0), a.Win - 1);
    psrc[j] = (ok || PRO) ? a.x1 + ((size_t)(bc * a.Hin + iyc) * a.Win + ixc) * a.x1_pitch + 8 * sq + (pg ? h * kC : 0)
                          : kZeroPage + 8 * sq;
  }

  // ---- B: fragment images, the wave's 32 columns
  const int ngrp = ceil_div(N, 32);
  const size_t sl = (size_t)ngrp * 1024;
  const _Float16* wbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * 32 + j * 16 + l16;
    const int cg = min(col >> 5, ngrp - 1);
    wbase[j] = reinterpret_cast<const _Float16*>(a.ws) + (size_t)cg * 1024 + ((q & 1) * 32 + (col & 31)) * 8;
  }
  const size_t qoff = (size_t)(q >> 1) * 9 * sl;
  auto slice_off = [&](int kt) { return (size_t)(kt + (kt / 9) * 9) * sl + qoff; };
  f16x8 bq[WD][TN][2];
  auto load_b = [&](f16x8 (&dst)[TN][2], size_t off) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) dst[j][p] = *reinterpret_cast<const f16x8*>(wbase[j] + off + p * 512);
  };

  // ---- A-fragment patch rows of this lane
  int fy[TM], fx[TM], fimg[TM];
  const int tile_rows = g.TH * g.TW;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = (wm * TM + i) * 16 + l16;
    fimg[i] = ml / tile_rows;
    const int rem = ml - fimg[i] * tile_rows;
    fy[i] = rem / g.TW;
    fx[i] = rem - fy[i] * g.TW;
  }

  f4 rp[2][2];
  auto load_patch = [&](int i, int j0, int j1) {  // passes j0 .. j1 - 1 of pair i
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      rp[j & 1][0] = *reinterpret_cast<const f4*>(psrc[j] + i * kC);
      rp[j & 1][1] = *reinterpret_cast<const f4*>(psrc[j] + i * kC + 4);
    }
  };
  const bool pro_silu = !a.pro_nosilu;
  const int tab_n = PRO ? min(b0 + g.TB, a.B) - b0 : 0;
  const int tab_c = a.Cin1;
  bool bad = false;
  auto finish_patch = [&](int i, int j0, int j1, int buf) {
    const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      const int p = srow + SR * j;
      const int pg = p >= kSP ? 1 : 0, pp = p - pg * kSP;
      if (PRO) {
        const float* ts = gtab + min(pimg[j] - b0, tab_n - 1) * tab_c + (pg ? h + i : i) * kC + 8 * sq;
        f4 sc[2], sh[2];
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          sc[e2] = *reinterpret_cast<const f4*>(ts + 4 * e2);
          sh[e2] = *reinterpret_cast<const f4*>(ts + tab_n * tab_c + 4 * e2);
        }
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = rp[j & 1][e2][e] * sc[e2][e] + sh[e2][e];
            rp[j & 1][e2][e] = pro_silu ? silu_fast(v) : v;
          }
      }
      if (p < 2 * kSP) {
        f16x8 pc[2];
        const bool z = PRO && !pok[j];
        Split<2>::split(z ? zero4 : rp[j & 1][0], z ? zero4 : rp[j & 1][1], pc, bad);
        _Float16* dst = patch + (pg * 2 + buf) * PATCH + pp * kRowH;
        *reinterpret_cast<f16x8*>(dst + sq * 8) = pc[0];
        *reinterpret_cast<f16x8*>(dst + 32 + sq * 8) = pc[1];
      }
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  auto a_off = [&](int i, int ky, int kx) {
    return ((fimg[i] * g.PH + fy[i] + ky) * g.PW + fx[i] + kx) * kRowH + q * 8;
  };
  auto compute_tap = [&](int tap, int pbuf, const f16x8 (&bv)[TN][2]) {
    const _Float16* As = patch + pbuf * PATCH;
    f16x8 av[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + a_off(i, tap / 3, tap % 3) + p * 32);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][1], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bv[j][0], acc[i][j], 0, 0, 0);
      }
  };

  // ---- prologue: the first pair's patch loads in flight while the GroupNorm tables are built
  const int c0w = grp ? h : 0;  // this wave's first chunk
#pragma unroll
  for (int d = 0; d < WD; ++d) load_b(bq[d], slice_off(c0w * 9 + d));
  f4 rq[PJ][2];
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    rq[j][0] = *reinterpret_cast<const f4*>(psrc[j]);
    rq[j][1] = *reinterpret_cast<const f4*>(psrc[j] + 4);
  }
  if (PRO) {
    if (a.gin_part) {  // gn_finalize for the tile's images (conv_k32_kernel's in-kernel finalize)
      const int G = a.gin_G, cpg = a.Cin1 / G;
      for (int i = t; i < tab_n * G; i += NT) {
        const int b = b0 + i / G, gg = i - (i / G) * G;
        double s1 = 0, s2 = 0;
        for (int k = 0; k < a.gin_nchunk; ++k) {
          const double2 v = a.gin_part[((size_t)b * a.gin_nchunk + k) * G + gg];
          s1 += v.x;
          s2 += v.y;
        }
        const double mu = s1 / a.gin_n;
        double var = s2 / a.gin_n - mu * mu;
        if (var < 0) var = 0;
        gstat[2 * i] = (float)mu;
        gstat[2 * i + 1] = (float)(1.0 / sqrt(var + (double)a.gin_eps));
      }
      __syncthreads();
      for (int i = t; i < tab_n * tab_c; i += NT) {
        const int bi = i / tab_c, c = i - (i / tab_c) * tab_c;
        const int si = 2 * (bi * G + c / cpg);
        const float mu = gstat[si], rs = gstat[si + 1];
        float sc = rs * (a.gin_gamma ? a.gin_gamma[c] : 1.0f);
        float sh = -sc * mu + (a.gin_beta ? a.gin_beta[c] : 0.0f);
        if (a.gin_ms) {
          const size_t mo = (size_t)(b0 + bi) * a.gin_mp + c;
          const float f = 1.0f + a.gin_ms[mo];
          sc = sc * f;
          sh = sh * f + a.gin_mb[mo];
        }
        gtab[i] = sc;
        gtab[tab_n * tab_c + i] = sh;
      }
    } else {
      for (int i = t; i < tab_n * tab_c; i += NT) {
        const int bi = i / tab_c, c = i - (i / tab_c) * tab_c;
        gtab[i] = a.pro_scale[(size_t)(b0 + bi) * a.Cin1 + c];
        gtab[tab_n * tab_c + i] = a.pro_shift[(size_t)(b0 + bi) * a.Cin1 + c];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < PJ; j += 2) {
    rp[0][0] = rq[j][0];
    rp[0][1] = rq[j][1];
    if (j + 1 < PJ) {
      rp[1][0] = rq[j + 1][0];
      rp[1][1] = rq[j + 1][1];
    }
    finish_patch(0, j, min(j + 2, PJ), 0);
  }
  __syncthreads();

  // ---- main loop: pair i = chunks i (group 0) and h + i (group 1); the next pair's passes 0-1 loaded at
  // tap 0 and finished at tap 2, 2-3 at taps 3 / 5, 4 at taps 6 / 8; one barrier per pair
  for (int i0 = 0; i0 < h; i0 += 2) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int i = i0 + cc;
      if (i >= h) break;
      const int in = min(i + 1, h - 1);
      const int buf = i & 1;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kt = (c0w + i) * 9 + tap;
        const int slot = (cc * 9 + tap) % WD;
        // the pair's loader passes in three phases (taps 0 / 3 / 6 load, 2 / 5 / 8 finish): passes 0-1, 2-3, 4
        // (NW 4) or 0, 1, 2 (NW 8)
        constexpr int P0[3] = {0, NW == 8 ? 1 : 2, NW == 8 ? 2 : 4}, P1[3] = {NW == 8 ? 1 : 2, NW == 8 ? 2 : 4, PJ};
        if (tap == 0 || tap == 3 || tap == 6) {
          load_patch(in, P0[tap / 3], P1[tap / 3]);
          __builtin_amdgcn_sched_barrier(0);
        }
        compute_tap(tap, grp * 2 + buf, bq[slot]);
        load_b(bq[slot], slice_off(min(kt + WD, (c0w + h) * 9 - 1)));
        __builtin_amdgcn_sched_barrier(0);
        if (tap == 2 || tap == 5 || tap == 8) finish_patch(in, P0[tap / 3], P1[tap / 3], (i + 1) & 1);
      }
      __syncthreads();
    }
  }

  // ---- segment 2: the ResBlock shortcut (1x1 of x2), chunks [0, h2) and [h2, n2) split over the groups,
  // un-pipelined: per step each group's 64 x 32 row tile into its buffer 0
  if (n2 > 0) {
    int abase[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) abase[i] = ((wm * TM + i) * 16 + l16) * kRowH + q * 8;
    const size_t s2 = (size_t)(9 * a.Cin1 / 16) * sl + (size_t)(q >> 1) * sl;
    for (int c2 = 0; c2 < n2 - h2; ++c2) {
      // loader: item (group jg, row, quarter sq): NW 4 -- both groups per thread; NW 8 -- group srow >> 6
      constexpr int SJ = NW == 8 ? 1 : 2;
      const int lrow = srow & 63;
      f4 r[SJ][2];
#pragma unroll
      for (int j = 0; j < SJ; ++j) {
        const int jg = NW == 8 ? (srow >> 6) : j;
        const int cj = jg ? h2 + c2 : min(c2, max(h2 - 1, 0));
        const float* xs = a.x2 + (size_t)min(m0 + lrow, M - 1) * a.x2_pitch + 8 * sq + cj * kC;
        r[j][0] = *reinterpret_cast<const f4*>(xs);
        r[j][1] = *reinterpret_cast<const f4*>(xs + 4);
      }
      const int cw = grp ? h2 + c2 : c2;
      const bool active = cw < (grp ? n2 : h2);
      load_b(bq[0], s2 + (size_t)(2 * min(cw, n2 - 1)) * sl);
#pragma unroll
      for (int j = 0; j < SJ; ++j) {
        const int jg = NW == 8 ? (srow >> 6) : j;
        f16x8 pc[2];
        Split<2>::split(r[j][0], r[j][1], pc, bad);
        _Float16* dst = patch + (jg * 2) * PATCH + lrow * kRowH;
        *reinterpret_cast<f16x8*>(dst + sq * 8) = pc[0];
        *reinterpret_cast<f16x8*>(dst + 32 + sq * 8) = pc[1];
      }
      __syncthreads();
      if (active) {
        const _Float16* As = patch + (grp * 2) * PATCH;
        f16x8 av[TM][2];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + abase[i] + p * 32);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][1], bq[0][j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bq[0][j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i][0], bq[0][j][0], acc[i][j], 0, 0, 0);
          }
      }
      __syncthreads();
    }
  }
  if (bad && a.range_flag) *a.range_flag = 1;

  // ---- the two partial tiles through LDS ([group][64][68] fp32, raw accumulators), then each wave takes
  // rows 32 grp .. + 31 of its 32 columns: v = p0 * s + p1 * s, bias, per-image row vector, residual, store,
  // and the GroupNorm statistics of each of the slab's two 16-row images
  constexpr int PTP = BN + 4;
  float* part = reinterpret_cast<float*>(patch);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        part[(grp * 64 + (wm * TM + i) * 16 + 4 * q + r) * PTP + wn * 32 + j * 16 + l16] = acc[i][j][r];
  __syncthreads();
  constexpr int LPR = 8, RPI = 8;  // lanes per row (4 columns each), rows per wave instruction
  const int c4 = lane % LPR, rsub = lane / LPR;
  const int ncol = n0 + wn * 32 + 4 * c4;
  const bool c_ok = ncol < N;
  const int nc = c_ok ? ncol : 0;
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const f4 s4 = {a.ws_rowscale[nc], a.ws_rowscale[nc + 1], a.ws_rowscale[nc + 2], a.ws_rowscale[nc + 3]};
  const f4 bias4 = a.bias ? *reinterpret_cast<const f4*>(a.bias + nc) : zero4;
  // rows of this wave: 32 (NW 4: slab grp) or 16 (NW 8: slab 2 grp + wm)
  constexpr int WR = 128 / NW;
  const int row0 = NW == 8 ? 16 * (2 * grp + wm) : 32 * grp;
  double gs[2] = {0.0, 0.0}, gq[2] = {0.0, 0.0};
  f4 rs4[WR / RPI];
  if (a.res) {
#pragma unroll
    for (int it = 0; it < WR / RPI; ++it) {
      const int m = min(m0 + row0 + it * RPI + rsub, M - 1);
      rs4[it] = *reinterpret_cast<const f4*>(a.res + (size_t)m * a.res_pitch + nc);
    }
  }
#pragma unroll
  for (int it = 0; it < WR / RPI; ++it) {
    const int row = row0 + it * RPI + rsub;
    const int m = m0 + row;
    const f4 p0 = *reinterpret_cast<const f4*>(part + row * PTP + wn * 32 + 4 * c4);
    const f4 p1 = *reinterpret_cast<const f4*>(part + (64 + row) * PTP + wn * 32 + 4 * c4);
    f4 v = p0 * s4 + p1 * s4;
    if (a.bias) v = v + bias4;
    if (a.rowvec) v = v + *reinterpret_cast<const f4*>(a.rowvec + (size_t)(min(m, M - 1) / HWo) * a.rowvec_pitch + nc);
    if (a.res) v = v + rs4[it];
    if (m < M && c_ok) *reinterpret_cast<f4*>(a.y + (size_t)m * a.y_pitch + ncol) = v;
    if (a.gn_part && m < M) {
      const int hh = (it * RPI) / 16;  // the slab's first or second 16-row image (HWo = 16)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gs[hh] += (double)v[e];
        gq[hh] += (double)v[e] * v[e];
      }
    }
  }
  if (a.gn_part) {  // per image of the slab: over the row lanes, then the group's 4-channel quads
    const int cpg = N / a.gn_G;
#pragma unroll
    for (int hh = 0; hh < WR / 16; ++hh) {
      double s = gs[hh], qq = gq[hh];
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        s += __shfl_xor(s, o);
        qq += __shfl_xor(qq, o);
      }
      for (int o = 1; o < cpg / 4; o <<= 1) {
        s += __shfl_xor(s, o);
        qq += __shfl_xor(qq, o);
      }
      const int m = m0 + row0 + 16 * hh;
      if (rsub == 0 && (c4 % (cpg / 4)) == 0 && c_ok && m < M)
        a.gn_part[(size_t)(m / HWo) * a.gn_G + ncol / cpg] = make_double2(s, qq);
    }
  }
}

}  // namespace

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_k32_stamps(void* host, int nblocks) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_k32_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

// Variants: 1 = 128 x 128 tiles, 2 = 128 x 64 (whole K), 3 = 64 x 64 and 4 = 64 x 128 split-K tiles,
// 5 = 64 x 128 tiles of one image row or 64-pixel row segment (ADM's 64^2 .. 256^2 maps), 6 = the small-map
// kernel (64 x 64 tiles of four 4 x 4 images, K split in two inside the block; the plan's ksplit = 2),
// 7 = 512-thread 128 x 128 tiles of 64 x 32 wave tiles (wide maps), 8 = variant 1 / its sub-pixel form with a
// 32 KB GroupNorm table (inputs of up to 2048 channels at two images per tile; one block per CU), 9 = the
// stride-2 downsample (64 x 128 tiles of 8 waves of 32 x 32 over whole output rows, one block per CU).
static bool conv_k32s_ok(const ConvArgs& a) {
  if (!(a.ws && a.ws_np == 2 && a.ws_rowscale && a.taps == 9 && a.stride == 1 && a.upsample == 0)) return false;
  if (a.ksplit != 2 || a.Hout * a.Wout != 16 || a.Hin != a.Hout || a.Win != a.Wout) return false;
  const int nch = a.Cin1 / kC;
  if (a.Cin1 % kC != 0 || nch < 2 || nch % 2 != 0 || a.Cin2 % kC != 0 || a.K != 9 * a.Cin1 + a.Cin2) return false;
  if (a.Cout % 64 != 0) return false;
  PatchGeom g;
  if (!conv_patch_geom(a, 64, g) || g.P > kSP || g.TB > 4) return false;
  if ((a.pro_scale || a.gin_part) && 2 * g.TB * a.Cin1 > kTabS) return false;
  if (a.gin_part && g.TB * a.gin_G > kStatsS) return false;
  if (a.gn_part && (a.gn_G <= 0 || a.Cout % a.gn_G != 0 || (a.Cout / a.gn_G) % 4 != 0 || a.Cout / a.gn_G > 32))
    return false;
  return staged_epilogue_ok(a) || (a.gn_part && a.Cout % 4 == 0);
}

static bool t2d_geom(const ConvArgs& a, PatchGeom& g);

int conv_k32_variant_ok(const ConvArgs& a, int v) {
  if (v == 6 || v == 12) return conv_k32s_ok(a) ? 1 : 0;
  if (v == 11) {  // 64-row tiles of one <= 64-pixel image (8^2 maps), 4 waves of 32 x 64
    if (!(a.ws && a.ws_np == 2 && a.ws_rowscale && a.taps == 9 && a.stride == 1 && a.upsample == 0)) return 0;
    if (a.Cin1 < kC || a.Cin1 % kC != 0 || a.Cin2 % kC != 0 || a.ksplit > 1 || a.K != 9 * a.Cin1 + a.Cin2) return 0;
    if (a.Hout * a.Wout != 64 || a.Wout % 8 != 0) return 0;
    PatchGeom g;
    if (!conv_patch_geom(a, 64, g) || g.P > kMaxP || g.TB != 1) return 0;
    if (a.pro_scale && 2 * a.Cin1 > kTab) return 0;
    if (a.gin_part && a.gin_G > kStats) return 0;
    return staged_epilogue_ok(a) ? 1 : 0;
  }
  if (v == 10) {
    if (!(a.ws && a.ws_np == 2 && a.ws_rowscale)) return 0;
    if (a.Cin1 < kC || a.Cin1 % kC != 0 || a.Cin2 % kC != 0 || a.ksplit > 1) return 0;
    if (a.upsample == 2 ? (a.Cin2 != 0 || a.K != 4 * a.Cin1) : a.K != 9 * a.Cin1 + a.Cin2) return 0;
    PatchGeom g;
    if (!t2d_geom(a, g)) return 0;
    if (a.pro_scale && 2 * a.Cin1 > kTab) return 0;
    if (a.gin_part && a.gin_G > kStats) return 0;
    return staged_epilogue_ok(a) ? 1 : 0;
  }
  if (v == 9) {
    if (!(a.ws && a.ws_np == 2 && a.ws_rowscale && a.taps == 9 && a.stride == 2 && a.upsample == 0)) return 0;
    if (a.Cin1 < kC || a.Cin1 % kC != 0 || a.Cin2 != 0 || a.ksplit > 1 || a.K != 9 * a.Cin1) return 0;
    if (a.Wout % 8 != 0) return 0;
    PatchGeom g;
    if (!conv_patch_geom(a, 64, g) || g.P > kMaxPW || g.TB > 2) return 0;
    if (a.pro_scale && 2 * g.TB * a.Cin1 > kTab) return 0;
    if (a.gin_part && g.TB * a.gin_G > kStats) return 0;
    return staged_epilogue_ok(a) ? 1 : 0;
  }
  if (v == 7) {  // 128-row tiles of 512 threads over one image's 128-pixel row segment or two 64-pixel rows
    const bool sub = a.upsample == 2;
    if (!(a.ws && a.ws_np == 2 && a.ws_rowscale && a.taps == 9 && a.stride == 1 && (a.upsample == 0 || sub))) return 0;
    if (a.Cin1 < kC || a.Cin1 % kC != 0 || a.Cin2 % kC != 0 || a.ksplit > 1) return 0;
    if (sub ? (a.Cin2 != 0 || a.K != 4 * a.Cin1) : a.K != 9 * a.Cin1 + a.Cin2) return 0;
    // or whole rows of up to two images of a narrower map (8^2 .. 32^2: 8 waves per CU where 256 blocks of 4
    // waves leave one wave per SIMD)
    const int wt = sub ? a.Win : a.Wout;
    const bool wide = wt >= 64 && (wt > 128 ? wt % 128 == 0 : 128 % wt == 0);
    const bool narrow = wt < 64 && wt % 8 == 0 && 128 % wt == 0;
    if (!wide && !narrow) return 0;
    PatchGeom g;
    if (!conv_patch_geom(a, 128, g) || g.P > kMaxPW || g.TB > (wide ? 1 : 2)) return 0;
    if (a.pro_scale && 2 * g.TB * a.Cin1 > kTab) return 0;
    if (a.gin_part && g.TB * a.gin_G > kStats) return 0;
    return staged_epilogue_ok(a) ? 1 : 0;
  }
  const bool sub = a.upsample == 2;  // sub-pixel nearest-2x + 3x3: 4 parity convs of 4 taps
  if (!(a.ws && a.ws_np == 2 && a.ws_rowscale && a.taps == 9 && a.stride == 1 && (a.upsample == 0 || sub))) return 0;
  if (a.Cin1 < kC || a.Cin1 % kC != 0 || a.Cin2 % kC != 0) return 0;
  if (sub ? (a.Cin2 != 0 || a.K != 4 * a.Cin1) : a.K != 9 * a.Cin1 + a.Cin2) return 0;
  const bool split = v == 3 || v == 4, seg = v == 5, big = v == 8;
  if (split && sub) return 0;
  const int bm = (split || seg) ? 64 : BM_K32;
  if (split ? !(a.ksplit > 1 && a.kpart && a.ksplit <= a.Cin1 / kC) : a.ksplit > 1) return 0;
  const int wt = sub ? a.Win : a.Wout;  // tiled width
  if (seg ? (wt < 64 || wt % 64 != 0) : (wt > bm || bm % wt != 0)) return 0;
  PatchGeom g;
  if (!conv_patch_geom(a, bm, g) || g.P > kMaxP || g.TB > (split ? 4 : 2) || (seg && g.TB != 1)) return 0;
  const int nch = a.Cin1 / kC, tab_c = split ? ceil_div(nch, a.ksplit) * kC : a.Cin1;
  if (a.pro_scale && 2 * g.TB * tab_c > (big ? kTabBig : kTab)) return 0;
  if (a.gin_part && g.TB * a.gin_G > kStats) return 0;
  if (split) {  // raw partial sums with 16-byte stores
    if (a.Cout % 4 != 0 || (reinterpret_cast<uintptr_t>(a.kpart) & 15) != 0) return 0;
    return 1;
  }
  if (wt % 8 != 0) return 0;
  return staged_epilogue_ok(a) ? 1 : 0;  // the epilogue's 16-byte loads / stores of 4 consecutive channels
}

bool conv_k32_ok(const ConvArgs& a) { return conv_k32_variant_ok(a, 1) != 0; }

// Which conv_k32 variant runs this conv, 0 = none. Forced by tile 10 / 11 (128-row tiles) and 12 / 13
// (split-K 64-row tiles); otherwise it replaces conv_patch3's fp16x2 tiles for 3x3 stride-1 convs. The plan
// toggles (Toggles: DM_CONV_K32S, DM_CONV_K32S2, DM_CONV_K32T2, DM_K32_8X, DM_K32S_W4) keep the paths each form
// replaced as its test oracle.
// variant 10's geometry: 4 output rows x 32 columns per 128-row tile, a 6 x 34 patch
static bool t2d_geom(const ConvArgs& a, PatchGeom& g) {
  // tiles over the output map, or over the low-res map of the sub-pixel upsample (4 parities x 4 taps)
  const bool sub = a.upsample == 2;
  if (a.stride != 1 || a.taps != 9 || (a.upsample != 0 && !sub)) return false;
  if (sub ? (a.Hout != 2 * a.Hin || a.Wout != 2 * a.Win) : (a.Hin != a.Hout || a.Win != a.Wout)) return false;
  if (a.Win < 64 || a.Win % 32 != 0 || a.Hin % 4 != 0) return false;
  g.TB = 1;
  g.TH = 4;
  g.TW = 32;
  g.PH = 6;
  g.PW = 34;
  g.P = 204;
  return true;
}

int conv_k32_pick(const ConvArgs& a) {
  if (a.tile >= 10 && a.tile <= 20) return conv_k32_variant_ok(a, a.tile - 9) ? a.tile - 9 : 0;
  if (a.tile != 0) return 0;
  if (a.stride == 2) {  // at least one block per CU (the nominal batch keeps the choice batch-invariant)
    const long M = (long)(a.pick_B > 0 ? a.pick_B : a.B) * a.Hout * a.Wout;
    return toggles().k32_s2 && conv_k32_variant_ok(a, 9) && (M / 64) * ((a.Cout + 127) / 128) >= 256 ? 9 : 0;
  }
  // split-K convs of maps of <= 16 pixels: 64 x 128 tiles (4x4 maps at B = 256, K split 2: 32.5 us vs
  // 34.2 us for 64 x 64 and for conv_patch3's 64 x 64 split tiles)
  if (a.ksplit > 1) {
    if (toggles().k32_small && conv_k32_variant_ok(a, 6)) return toggles().k32s_w4 ? 12 : 6;
    return conv_k32_variant_ok(a, 4) ? 4 : conv_k32_variant_ok(a, 3) ? 3 : 0;
  }
  if (!conv_k32_ok(a)) {
    // maps whose whole-row 128-row tiles do not fit the patch image (64^2 .. 256^2): 128-pixel row segments /
    // two-row tiles of 8 waves, else 64-pixel rows / segments
    const int wt = a.upsample == 2 ? a.Win : a.Wout;
    if (wt >= 64 && toggles().k32_t2d && conv_k32_variant_ok(a, 10)) return 10;
    if (wt >= 64 && conv_k32_variant_ok(a, 7)) return 7;
    if (wt >= 64) return conv_k32_variant_ok(a, 5) ? 5 : 0;
    // 128-row tiles whose GroupNorm tables do not fit kTab: the big-table instantiation (one block per CU)
    const int p = conv_pick(a);
    return ((p == 3 || p == 4) && conv_k32_variant_ok(a, 8)) ? 8 : 0;
  }
  const int p = conv_pick(a);
  if (p != 3 && p != 4) return 0;
  // 8^2 maps on 64-row single-image tiles (two blocks per CU where 128 x 128 tiles give one; bit-identical):
  // C3 A/B +0.3 % / +0.25 % over two sessions' alternations; DM_K32_8X=0 keeps the 128 x 128 two-image tiles
  if (toggles().k32_8x && conv_k32_variant_ok(a, 11)) return 11;
  // 128 x 128 tiles down to one block per CU (measured on 8^2 maps at B = 256: 256 blocks of 128 x 128 beat
  // 512 of 128 x 64 by 6 %); the nominal batch (pick_B) keeps the choice batch-invariant
  const long M = (long)(a.pick_B > 0 ? a.pick_B : a.B) * a.Hout * a.Wout;
  return ((M + 127) / 128) * ((a.Cout + 127) / 128) >= 256 ? 1 : 2;
}

// rocprofv3's name of the instantiation conv2d_k32 launches (spaces removed)
std::string conv_k32_label(const ConvArgs& a, int v) {
  if (v == 6 || v == 12)
    return std::string("conv_k32s_kernel<") + (a.pro_scale || a.gin_part ? "true," : "false,") + (v == 12 ? "4>" : "8>");
  if (v == 7)
    return std::string("conv_k32_kernel<128,128,64,32,") + (a.pro_scale ? "true," : "false,") + "false," +
           (a.upsample == 2 ? "true,512>" : "false,512>");
  if (v == 8)
    return std::string("conv_k32_kernel<128,128,64,64,") + (a.pro_scale ? "true," : "false,") + "false," +
           (a.upsample == 2 ? "true,256,208,8192>" : "false,256,208,8192>");
  if (v == 9)
    return std::string("conv_k32_kernel<64,128,32,32,") + (a.pro_scale ? "true," : "false,") + "false,false,512,392,2048,true>";
  if (v == 11) return std::string("conv_k32_kernel<64,128,32,64,") + (a.pro_scale ? "true," : "false,") + "false,false>";
  if (v == 10)
    return std::string("conv_k32_kernel<128,128,64,64,") + (a.pro_scale ? "true," : "false,") + "false," +
           (a.upsample == 2 ? "true" : "false") + ",256,208,2048,false,true>";
  static const char* names[] = {"", "conv_k32_kernel<128,128,64,64,", "conv_k32_kernel<128,64,64,32,",
                                "conv_k32_kernel<64,64,32,32,", "conv_k32_kernel<64,128,32,64,",
                                "conv_k32_kernel<64,128,32,64,"};
  return std::string(names[v]) + (a.pro_scale ? "true," : "false,") + (v == 3 || v == 4 ? "true," : "false,") +
         (a.upsample == 2 ? "true>" : "false>");
}

template <int BM, int BN, int WM, int WN, bool KSPLIT, int NT = 256, int MAXP = kMaxP, int TABF = kTab, bool S2 = false,
          bool T2D = false>
static void launch_k32(const ConvArgs& a, const PatchGeom& g, hipStream_t st) {
  const bool sub = a.upsample == 2;
  const int M = sub ? a.B * a.Hin * a.Win : a.B * a.Hout * a.Wout;
  const int blocks = ceil_div(M, BM) * ceil_div(a.Cout, BN) * (KSPLIT ? a.ksplit : 1) * (sub ? 4 : 1);
  if constexpr (!KSPLIT) {
    if (sub) {
      if (a.pro_scale)
        hipLaunchKernelGGL((conv_k32_kernel<BM, BN, WM, WN, true, false, true, NT, MAXP, TABF, false, T2D>), dim3(blocks),
                           dim3(NT), 0, st, a, g);
      else
        hipLaunchKernelGGL((conv_k32_kernel<BM, BN, WM, WN, false, false, true, NT, MAXP, TABF, false, T2D>),
                           dim3(blocks), dim3(NT), 0, st, a, g);
      return;
    }
  }
  if (a.pro_scale)
    hipLaunchKernelGGL((conv_k32_kernel<BM, BN, WM, WN, true, KSPLIT, false, NT, MAXP, TABF, S2, T2D>), dim3(blocks),
                       dim3(NT), 0, st, a, g);
  else
    hipLaunchKernelGGL((conv_k32_kernel<BM, BN, WM, WN, false, KSPLIT, false, NT, MAXP, TABF, S2, T2D>), dim3(blocks),
                       dim3(NT), 0, st, a, g);
}

int conv2d_k32(const ConvArgs& a, int v, hipStream_t st) {
  DM_REQUIRE(v >= 1 && v <= 12 && conv_k32_variant_ok(a, v), "conv: shape not supported by the K = 32 split kernel");
  PatchGeom g;
  if (v == 6 || v == 12) {  // the small-map kernel: 8 waves (6), or its 4-wave form (12, one wave per SIMD)
    conv_patch_geom(a, 64, g);
    const int blocks = ceil_div(a.B * a.Hout * a.Wout, 64) * (a.Cout / 64);
    const bool pro = a.pro_scale || a.gin_part;
    if (v == 12) {
      if (pro) hipLaunchKernelGGL((conv_k32s_kernel<true, 4>), dim3(blocks), dim3(256), 0, st, a, g);
      else hipLaunchKernelGGL((conv_k32s_kernel<false, 4>), dim3(blocks), dim3(256), 0, st, a, g);
      note_launch(pro ? "conv_k32s_kernel<true,4>" : "conv_k32s_kernel<false,4>");
    } else {
      if (pro) hipLaunchKernelGGL((conv_k32s_kernel<true, 8>), dim3(blocks), dim3(512), 0, st, a, g);
      else hipLaunchKernelGGL((conv_k32s_kernel<false, 8>), dim3(blocks), dim3(512), 0, st, a, g);
      note_launch(pro ? "conv_k32s_kernel<true,8>" : "conv_k32s_kernel<false,8>");
    }
    DM_LAUNCH_CHECK();
    return DM_OK;
  }
  if (v == 10) {
    t2d_geom(a, g);
    launch_k32<128, 128, 64, 64, false, 256, kMaxP, kTab, false, true>(a, g, st);
    DM_LAUNCH_CHECK();
    return DM_OK;
  }
  conv_patch_geom(a, (v >= 3 && v <= 6) || v == 9 || v == 11 ? 64 : BM_K32, g);
  switch (v) {
    case 11: launch_k32<64, 128, 32, 64, false>(a, g, st); break;
    case 9: launch_k32<64, 128, 32, 32, false, 512, kMaxPW, kTab, true>(a, g, st); break;
    case 8: launch_k32<128, 128, 64, 64, false, 256, kMaxP, kTabBig>(a, g, st); break;
    case 7: launch_k32<128, 128, 64, 32, false, 512, kMaxPW>(a, g, st); break;
    case 1: launch_k32<128, 128, 64, 64, false>(a, g, st); break;
    case 2: launch_k32<128, 64, 64, 32, false>(a, g, st); break;
    case 3: launch_k32<64, 64, 32, 32, true>(a, g, st); break;
    case 4: launch_k32<64, 128, 32, 64, true>(a, g, st); break;
    default: launch_k32<64, 128, 32, 64, false>(a, g, st); break;
  }
  DM_LAUNCH_CHECK();
  if (v == 3 || v == 4) return conv_splitk_reduce(a, st);
  return DM_OK;
}

}  // namespace dm
