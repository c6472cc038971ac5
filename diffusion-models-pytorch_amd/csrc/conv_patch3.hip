// 3x3 convolution (stride 1, nearest-2x upsample, sub-pixel upsample) on the
// halo-patch tiling of conv_patch.hip, with the products computed by the
// bf16 matrix cores on a three-way split of every fp32 operand.
//
// Numerics (models/unet.py:16,26 — the reference convolves in fp32):
// an fp32 value x is split exactly as x = x0 + x1 + x2 with
// x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1) (round to nearest
// even; both subtractions are exact), which carries the full 24-bit
// significand. A product a*w is then the sum of the nine piece products; the
// six with combined weight >= 2^-16 relative are issued
//   a2w0 + a1w1 + a0w2 + a1w0 + a0w1 + a0w0   (smallest first)
// as v_mfma_f32_32x32x16_bf16 into one fp32 accumulator. Each bf16 x bf16
// piece product is exact in fp32; the three dropped ones are below
// 2^-25 |a w| — under half an fp32 ulp of the product. The contraction
// therefore keeps fp32 accuracy (errors of the same size as the fp32 MFMA
// path's, tests/test_gpu_conv_split.py) while the six 32x32x16 bf16
// MFMAs (6 x 32 cycles) replace eight 32x32x2 fp32 MFMAs (8 x 64 cycles) per
// 16-deep k step: 2.7x fewer matrix-core cycles.
//
// Layout: K advances in 16-deep slices. A slice row (one pixel, or one output
// channel) is 2 lane groups x 3 pieces x 8 bf16 = 96 B, stored with a 112 B
// pitch (7 x 16 B: an odd number of 16-B slots keeps the ds_read_b128 lane
// groups conflict-free). Lane (lr, lh) of a 32x32x16 MFMA reads, per piece,
// the 16 B at row lr, group lh: k = 8 lh + j of the slice for both operands.
// The weights are split once at plan build (split_conv_weights) into
// [matrix][slice][Cout][48] bf16; the input patch is split when it is staged
// in LDS (after the fused GroupNorm + SiLU prologue), once per 16-channel
// chunk, and read by all 9 (or 4) taps from there. The patch is double
// buffered, so one barrier per tap suffices. LDS per 128x128 block:
// 2 x 208 x 112 + 2 x 128 x 112 = 73.5 KiB -> two blocks per CU.
//
// fp16x2 variant (NP = 2, the default): x = h0 + h1 with h0 = fp16(x), h1 =
// fp16(x - h0), 22 significant bits; a*w = a0w0 + a0w1 + a1w0 (+ a1w1, below
// 2^-22 |a w|, dropped), three v_mfma_f32_32x32x16_f16 per 16-deep k step
// instead of six. fp16's narrow exponent is handled on the weight side by a
// per-output-channel power-of-two scale (max |w| * 2^e in [2^13, 2^14), so
// w1 stays a normal fp16 for every weight above 2^-16 of the row maximum),
// undone exactly in the epilogue; activations are split unscaled, their low
// piece keeps an absolute floor of 2^-25 (fp16 subnormals), far below the
// fp32 accumulation error of a K >= 288 contraction. Emulated over K = 1152
// SiLU(N(0,1)) x U(+-1/sqrt(K)) dot products: max 4.3e-7 / rms 6.0e-8 vs
// 3.1e-7 / 5.3e-8 for the fp32 path. An activation above 65504 (no fp16
// image) sets ConvArgs::range_flag; the forward then re-runs in bf16x3.
// LDS row: 2 lane groups x 2 pieces x 8 fp16 = 64 B, pitch 80 B (5 slots).
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "conv_epilogue.h"
#include "split16.h"

namespace dm {

namespace {

#ifdef DM_K32_STAMPS
// Diagnostic build only (tools/k32_stamps.py --kernel pw): per block of the split 1x1 conv (MODE 3), wave
// 0's s_memtime at the start, before the main loop, after it, after the epilogue; realtime start / end.
__device__ unsigned long long g_pw_stamps[65536][8];
#define PW_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (PW1 && threadIdx.x == 0 && blockIdx.x < 65536) g_pw_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define PW_RSTAMP(k)                                                                                  \
  do {                                                                                                \
    if (PW1 && threadIdx.x == 0 && blockIdx.x < 65536) g_pw_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define PW_STAMP(k) do {} while (0)
#define PW_RSTAMP(k) do {} while (0)
#endif

constexpr int kSK = 16;  // K per slice = channels per patch chunk
constexpr int kPwSlices = 2;        // MODE 3: 16-channel slices per chunk (32 channels; 4 measured no faster)
constexpr int kPwTabFloats = 10240;  // GroupNorm table capacity (40 KiB) of the LDS-staged prologue tables
constexpr int kGinStats = 512;       // (image, group) pairs of the in-kernel GroupNorm finalize

// MODE 3 qkv conv feeding the fused attention (attention.hip): this wave's WM x WN tile of y = acc * rowscale
// + bias goes to its own LDS region (fp32, pitch WN + 8), then each lane takes 8 consecutive columns of
// a row (q, k: [L][Dh] planes) or 8 consecutive rows of a column (v: [Dh][L] planes), scales and splits
// them exactly as conv_store_attn_planes / the attention GEMMs' loaders, and stores 16-B pieces.
template <int WM, int WN>
__device__ __forceinline__ void attn_plane_epilogue(const ConvArgs& a, f16v (&acc)[WM / 32][WN / 32], int M,
                                                    int wm0, int wn0, int lr, int lh, float* wl) {
  constexpr int TM = WM / 32, TN = WN / 32, PITCH = WN + 8;
  const int N = a.Cout, lane = lr + 32 * lh;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = min(wn0 + j * 32 + lr, N - 1);
    const float cs = a.ws_rowscale[n], bn = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[i][j][r] * cs;
        if (a.bias) v = v + bn;
        wl[(i * 32 + acc_row(r, lh)) * PITCH + j * 32 + lr] = v;
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are visible to its reads
  __builtin_amdgcn_wave_barrier();
  if (wn0 >= N) return;
  // the wave's columns lie in one of q / k / v (3C, C and Dh are multiples of 32) and in one head
  const int Dh = a.ap_Dh, C = a.ap_heads * Dh;
  int part, h, d0;
  if (a.ap_legacy) {
    h = wn0 / (3 * Dh);
    part = (wn0 - h * 3 * Dh) / Dh;
    d0 = wn0 - h * 3 * Dh - part * Dh;
  } else {
    part = wn0 / C;
    h = (wn0 - part * C) / Dh;
    d0 = wn0 - part * C - h * Dh;
  }
  const float scale = part == 0 ? a.ap_alpha : part == 1 ? a.ap_bscale : 1.f;
  const bool use_scale = part == 0 ? a.ap_alpha != 1.0f : part == 1 && a.ap_bscale != 0.0f && a.ap_bscale != 1.0f;
  const float pw = ldexpf(1.f, part == 0 ? a.ap_ea : part == 1 ? a.ap_eb : a.ap_ev);
  const size_t plane = (size_t)a.ap_L * Dh;
  bool bad = false;
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
  if (part < 2) {  // q / k planes [b][h][piece][token][d]: 8 consecutive d of one token per lane
    _Float16* dst = part == 0 ? a.ap_q : a.ap_k;
    constexpr int G = WN / 8;
    for (int g = lane; g < WM * G; g += 64) {
      const int row = g / G, c8 = g - row * G;
      const int m = wm0 + row;
      if (m >= M) continue;
      const f4 x0 = *reinterpret_cast<const f4*>(wl + row * PITCH + 8 * c8);
      const f4 x1 = *reinterpret_cast<const f4*>(wl + row * PITCH + 8 * c8 + 4);
      const float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      f16x8 hi, lo;
      split8(x, hi, lo);
      const int b = m / a.ap_L, tok = m - b * a.ap_L;
      _Float16* p = dst + ((size_t)b * a.ap_heads + h) * 2 * plane + (size_t)tok * Dh + d0 + 8 * c8;
      *reinterpret_cast<f16x8*>(p) = hi;
      *reinterpret_cast<f16x8*>(p + plane) = lo;
    }
  } else {  // v planes [b][h][piece][d][token]: 8 consecutive tokens of one d per lane
    for (int g = lane; g < WN * (WM / 8); g += 64) {
      const int col = g % WN, r8 = g / WN;
      const int m = wm0 + 8 * r8;   // tokens m .. m + 7 lie in one image (L % 8 == 0)
      if (m >= M) continue;
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = wl[(8 * r8 + e) * PITCH + col];
      f16x8 hi, lo;
      split8(x, hi, lo);
      const int b = m / a.ap_L, tok = m - b * a.ap_L;
      _Float16* p = a.ap_v + ((size_t)b * a.ap_heads + h) * 2 * plane + (size_t)(d0 + col) * a.ap_L + tok;
      *reinterpret_cast<f16x8*>(p) = hi;
      *reinterpret_cast<f16x8*>(p + plane) = lo;
    }
  }
  if (bad && a.range_flag) *a.range_flag = 1;
}

template <int BM, int BN, int WM, int WN, int MODE, int MAXP, bool PRO, bool KSPLIT = false, int NP = 3>
__global__ void __launch_bounds__(256)
conv_patch3_kernel(ConvArgs a, PatchGeom g) {
  typedef Split<NP> S;
  typedef typename S::elem elem;
  typedef typename S::vec vec;
  constexpr int kSRow = S::kRow, kSPitch = S::kPitch, kGrp = NP * 8;  // kGrp: elements per lane group
  constexpr int NWN = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert((BM / WM) * NWN == 4, "4 waves per block");
  constexpr bool UP = MODE == 1, SUB = MODE == 2;
  // MODE 4: stride-2 3x3 (Downsample, models/modules.py:72). The patch holds the (2 TH + 1) input rows
  // of the tile with each row's columns split by parity ([even | odd], g.PW / 2 each), so the 32 lanes
  // of a fragment (consecutive output columns) read consecutive LDS rows for every tap.
  constexpr bool S2 = MODE == 4;
  // MODE 3: 1x1 (pointwise) conv / GEMM with static weights (the attention block's qkv and proj).
  // The "patch" is the tile's own BM rows; a chunk is kPwSlices x 16 channels stored as 16-deep
  // slices per row, which the chunk's kPwSlices "taps" read.
  constexpr bool PW1 = MODE == 3;
  constexpr int NTAP = SUB ? 4 : (PW1 ? kPwSlices : 9);
  constexpr int CH = PW1 ? kPwSlices * kSK : kSK;            // input channels per chunk
  constexpr int PROW = PW1 ? kPwSlices * kSRow + 8 : kSPitch;  // LDS row pitch (an odd number of 16-B slots)
  constexpr int PATCH = MAXP * PROW;
  __shared__ __attribute__((aligned(16))) elem patch[2 * PATCH];
  // GroupNorm prologue tables (fp16x2, and MODE 3 always): the tile's (image, channel) scale / shift
  // staged in LDS once per block; per-thread global loads of them cost as many VMEM instructions as
  // the activations themselves (and in MODE 3, with no tap reuse, twice the activation bytes)
  constexpr bool LTAB = PRO && (PW1 || NP == 2);
  // MODE 3: also the plane epilogue's staging; row-segment tiles (MAXP = kPatch3Seg): one image's tables
  constexpr int GTAB = (LTAB || PW1) ? (MAXP == kPatch3Seg ? kSegTabFloats : kPwTabFloats) : 1;
  __shared__ __attribute__((aligned(16))) float gtab[GTAB];
  __shared__ float gstat[LTAB ? 2 * kGinStats : 1];  // in-kernel finalize: (mean, rstd) per (image, group)

  PW_RSTAMP(5);
  PW_STAMP(0);
  const int Ho = SUB ? a.Hin : a.Hout, Wo = SUB ? a.Win : a.Wout;
  const int M = a.B * Ho * Wo;
  const int N = a.Cout;
  const int nN = ceil_div(N, BN);
  int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int ksplit = KSPLIT ? a.ksplit : 1;
  int split = 0;
  if (KSPLIT) {
    const int per_split = gridDim.x / ksplit;
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
  const int mt = bid / nN, nt = bid - (bid / nN) * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HWo = Ho * Wo;
  const int b0 = m0 / HWo;
  const int y0 = (m0 - b0 * HWo) / Wo;
  const int x0 = (m0 - b0 * HWo) - y0 * Wo;  // row-segment tiles (g.TW < Wo); 0 for whole-row tiles

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave / NWN, wn = wave % NWN;
  const int lr = lane & 31, lh = lane >> 5;
  // staging: two threads per pixel / row, 8 channels each
  const int srow = t >> 1, shalf = t & 1;

  // ---- patch loader geometry (pixel p = srow + 128 j; MODE 3: row srow, 16-channel slice j)
  constexpr int PJ = PW1 ? kPwSlices : (MAXP + 127) / 128;
  const float* psrc[PJ];
  bool pok[PJ];
  int pimg[PJ];
  const int iy_base = UP ? (y0 >> 1) - 1 : S2 ? 2 * y0 - 1 : y0 - 1;
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    if constexpr (PW1) {
      const int m = m0 + srow;
      const int mc = min(m, M - 1);  // rows >= M: clamped, never stored
      pok[j] = m < M;
      pimg[j] = mc / HWo;
      psrc[j] = a.x1 + (size_t)mc * a.x1_pitch + kSK * j + 8 * shalf;
      continue;
    }
    const int PHW = g.PH * g.PW;
    const int p = srow + 128 * j;
    const int img = p / PHW;
    const int rem = p - img * PHW;
    const int pr = rem / g.PW, pc = rem - (rem / g.PW) * g.PW;
    const int b = b0 + img;
    const int half = g.PW >> 1;
    const int col = S2 ? 2 * (pc - (pc >= half ? half : 0)) + (pc >= half ? 1 : 0) : pc;  // input column + 1
    const int iy = iy_base + pr, ix = x0 + col - 1;
    const bool ok = p < g.P && b < a.B && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
    pok[j] = ok;
    const int bc = min(b, a.B - 1);
    pimg[j] = bc;
    const int iyc = min(max(iy, 0), a.Hin - 1), ixc = min(max(ix, 0), a.Win - 1);
    psrc[j] = (ok || PRO) ? a.x1 + ((size_t)(bc * a.Hin + iyc) * a.Win + ixc) * a.x1_pitch + 8 * shalf
                          : kZeroPage + 8 * shalf;
  }
  // ---- B operand: straight from global (L2) into MFMA fragment registers, no LDS stage. The split
  // weights are laid out per (matrix, slice, 32-column group) as [NP pieces][2 lane groups][32 lanes]
  // [8], so each (group, piece) load is one 16-B vector per lane, 1 KiB contiguous per wave.
  const int nslices = a.K / kSK;
  const int ngrp = ceil_div(N, 32);
  const size_t slice_stride = (size_t)ngrp * (NP * 512);  // elements per slice of one weight matrix
  const elem* wsrc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int grp = min((n0 + wn * WN + j * 32) >> 5, ngrp - 1);  // columns >= N: clamped, never stored
    wsrc[j] = reinterpret_cast<const elem*>(a.ws) + (size_t)par * nslices * slice_stride + (size_t)grp * (NP * 512) +
              (lh * 32 + lr) * 8;
  }
  // slices ride a register ring of WD slots, loaded WD taps ahead of their use. The one-wave-per-SIMD
  // big tiles (128 x 128 wave tiles: 48 MFMAs per tap already cover the L2 latency) keep 2 slots for
  // register room. The chunk loop runs CPI chunks per iteration so that a tap's slot index is a
  // compile-time constant once the loops are unrolled (CPI * NTAP divides by WD).
  constexpr bool BIG = TM * TN >= 8;
  constexpr int WD = BIG ? 2 : (NTAP == 9 ? 3 : 2);
  constexpr int CPI = NTAP % WD == 0 ? 1 : WD;
  vec bq[WD][TN][NP];
  auto load_b = [&](vec (&dst)[TN][NP], int kt) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < NP; ++q)
        dst[j][q] = *reinterpret_cast<const vec*>(wsrc[j] + (size_t)kt * slice_stride + q * 512);
  };

  // ---- A-fragment patch coordinates of this lane's rows
  int fy[TM], fx[TM], fimg[TM];
  const int tile_rows = PW1 ? 1 : g.TH * g.TW;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if constexpr (PW1) {
      fy[i] = fx[i] = fimg[i] = 0;
      continue;
    }
    const int ml = wm * WM + i * 32 + lr;
    fimg[i] = ml / tile_rows;
    const int rem = ml - fimg[i] * tile_rows;
    fy[i] = rem / g.TW;
    fx[i] = rem - fy[i] * g.TW;
  }

  // Patch registers of the next chunk and, with the GroupNorm prologue, their per-(image, channel)
  // scale / shift, all loaded at the chunk's first tap and consumed taps later: a global load consumed
  // right after issue would drain vmcnt (in order) through the B fragments prefetched before it.
  f4 rp[PJ][2];
  f4 rs[PJ][2][2];
  auto load_patch = [&](int chunk) {
    const int co = chunk * CH;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      rp[j][0] = *reinterpret_cast<const f4*>(psrc[j] + co);
      rp[j][1] = *reinterpret_cast<const f4*>(psrc[j] + co + 4);
    }
    if (PRO && !LTAB) {
#pragma unroll
      for (int j = 0; j < PJ; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int cc = co + 8 * shalf;
          rs[j][h][0] = *reinterpret_cast<const f4*>(a.pro_scale + (size_t)pimg[j] * a.Cin1 + cc + 4 * h);
          rs[j][h][1] = *reinterpret_cast<const f4*>(a.pro_shift + (size_t)pimg[j] * a.Cin1 + cc + 4 * h);
        }
    }
  };
  // GroupNorm + SiLU prologue on patch registers j in [j0, j1): silu(x * scale[b][c] + shift[b][c])
  // (pro_nosilu: GroupNorm alone, the attention block's norm before qkv)
  const bool pro_silu = !a.pro_nosilu;
  const int tab_img0 = m0 / HWo;
  // images of the tile (MODE 3) or of its patch
  const int tab_n = !LTAB ? 0 : PW1 ? (min(m0 + BM, M) - 1) / HWo - tab_img0 + 1 : min(b0 + g.TB, a.B) - b0;
  auto transform = [&](int chunk, int j0, int j1) {
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      if (j >= j0 && j < j1) {
        if constexpr (LTAB) {  // tables from LDS: [image][Cin] scales, then the shifts
          const float* ts = gtab + (pimg[j] - tab_img0) * a.Cin1 + chunk * CH + (PW1 ? kSK * j : 0) + 8 * shalf;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            rs[j][h][0] = *reinterpret_cast<const f4*>(ts + 4 * h);
            rs[j][h][1] = *reinterpret_cast<const f4*>(ts + tab_n * a.Cin1 + 4 * h);
          }
        }
        // MODE 3: two code paths behind a uniform branch (a select would evaluate the SiLU, 2
        // transcendentals per value, for the GroupNorm-only prologue of the attention qkv as well)
        if (!PW1) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float v = rp[j][h][q] * rs[j][h][0][q] + rs[j][h][1][q];
              rp[j][h][q] = pro_silu ? silu_fast(v) : v;
            }
        } else if (pro_silu) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) rp[j][h][q] = silu_fast(rp[j][h][q] * rs[j][h][0][q] + rs[j][h][1][q]);
        } else {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int q = 0; q < 4; ++q) rp[j][h][q] = rp[j][h][q] * rs[j][h][0][q] + rs[j][h][1][q];
        }
      }
    }
  };
  // split + store (padding stays exactly 0: applied after the transform)
  bool bad = false;
  auto store_patch = [&](int buf) {
    elem* dst = patch + buf * PATCH;
    const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int p = PW1 ? srow : srow + 128 * j;
      if (PW1 || (j * 128 < MAXP && p < MAXP)) {
        vec pc[NP];
        const bool z = PRO && !pok[j];
        S::split(z ? zero4 : rp[j][0], z ? zero4 : rp[j][1], pc, bad);
        const int col = PW1 ? j * kSRow : 0;
#pragma unroll
        for (int q = 0; q < NP; ++q)
          *reinterpret_cast<vec*>(dst + p * PROW + col + shalf * kGrp + q * 8) = pc[q];
      }
    }
  };
  f16v acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one 16-deep K slice: A rows at LDS offsets abase[i] (+ lane group), B fragments in registers
  auto compute = [&](const elem* As, const int (&abase)[TM], const vec (&bv)[TN][NP]) {
    vec av[TM][NP];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < NP; ++q) av[i][q] = *reinterpret_cast<const vec*>(As + abase[i] + q * 8);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) S::mma(av[i], bv[j], acc[i][j]);
  };
  auto compute_tap = [&](int ky, int kx, int pbuf, const vec (&bv)[TN][NP]) {
    int abase[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (PW1) {  // row of this lane, slice kx of the chunk
        abase[i] = (wm * WM + i * 32 + lr) * PROW + kx * kSRow + lh * kGrp;
        continue;
      }
      int pr, pc;
      if (S2) {  // input (2 fy + ky - 1, 2 fx + kx - 1): column parity kx & 1, index fx + kx / 2
        pr = 2 * fy[i] + ky;
        pc = (kx & 1) * (g.PW >> 1) + fx[i] + (kx >> 1);
      } else if (UP) {
        pr = ((fy[i] + ky - 1) >> 1) + 1;
        pc = ((fx[i] + kx - 1) >> 1) + 1;
      } else {
        pr = fy[i] + ky;
        pc = fx[i] + kx;
      }
      abase[i] = ((fimg[i] * g.PH + pr) * g.PW + pc) * kSPitch + lh * kGrp;
    }
    compute(patch + pbuf * PATCH, abase, bv);
  };

  const int nchunks = a.Cin1 / CH;
  const int c_begin = KSPLIT ? split * nchunks / ksplit : 0;
  const int c_end = KSPLIT ? (split + 1) * nchunks / ksplit : nchunks;
  const int kt_begin = c_begin * NTAP, kt_end = c_end * NTAP;
  // Every load in the chunk loop is unconditional (indices clamped to the last slice / chunk, the
  // surplus loads are never used): the waitcnt pass then sees one load sequence per tap and counts
  // the B ring precisely, instead of assuming a skipped refill and waiting for the newest loads.
#pragma unroll
  for (int d = 0; d < WD; ++d) load_b(bq[d], min(kt_begin + d, kt_end - 1));
  if (LTAB) {
    if (a.gin_part) {
      // gn_finalize (gn.hip) for the tile's images, same expressions: per (image, group) mean and
      // 1/sqrt(var + eps) from the chunk partials, then per channel the affine (+ modulation)
      const int G = a.gin_G, cpg = a.Cin1 / G;
      for (int i = t; i < tab_n * G; i += 256) {
        const int b = tab_img0 + i / G, gg = i - (i / G) * G;
        double s1 = 0, s2 = 0;
        for (int k = 0; k < a.gin_nchunk; ++k) {
          const double2 v = a.gin_part[((size_t)b * a.gin_nchunk + k) * G + gg];
          s1 += v.x;
          s2 += v.y;
        }
        const double m = s1 / a.gin_n;
        double var = s2 / a.gin_n - m * m;
        if (var < 0) var = 0;
        gstat[2 * i] = (float)m;
        gstat[2 * i + 1] = (float)(1.0 / sqrt(var + (double)a.gin_eps));
      }
      __syncthreads();
      for (int i = t; i < tab_n * a.Cin1; i += 256) {
        const int bi = i / a.Cin1, c = i - (i / a.Cin1) * a.Cin1;
        const int si = 2 * (bi * G + c / cpg);
        const float mu = gstat[si], rs = gstat[si + 1];
        float sc = rs * (a.gin_gamma ? a.gin_gamma[c] : 1.0f);
        float sh = -sc * mu + (a.gin_beta ? a.gin_beta[c] : 0.0f);
        if (a.gin_ms) {
          const size_t mo = (size_t)(tab_img0 + bi) * a.gin_mp + c;
          const float f = 1.0f + a.gin_ms[mo];
          sc = sc * f;
          sh = sh * f + (a.gin_mb ? a.gin_mb[mo] : 0.0f);
        }
        gtab[i] = sc;
        gtab[tab_n * a.Cin1 + i] = sh;
      }
    } else {
      for (int i = t; i < tab_n * a.Cin1; i += 256) {
        gtab[i] = a.pro_scale[(size_t)tab_img0 * a.Cin1 + i];
        gtab[tab_n * a.Cin1 + i] = a.pro_shift[(size_t)tab_img0 * a.Cin1 + i];
      }
    }
    __syncthreads();
  }
  load_patch(c_begin);
  if (PRO) transform(c_begin, 0, PJ);
  store_patch(c_begin & 1);
  __syncthreads();
  PW_STAMP(1);
  // The patch is double buffered and read by every tap of its chunk: one barrier per chunk. The patch
  // of chunk c + 1 is loaded at tap 0, GroupNorm+SiLU'd over taps T0 .. NTAP-1, split and stored at
  // the last tap into the other buffer (free: every wave passed the previous chunk's barrier).
  constexpr int T0 = NTAP == 9 ? 3 : 1;
  for (int c0 = c_begin; c0 < c_end; c0 += CPI) {
#pragma unroll
  for (int cc = 0; cc < CPI; ++cc) {
    const int c = c0 + cc;
    if (CPI > 1 && c >= c_end) break;
#pragma unroll
    for (int tap = 0; tap < NTAP; ++tap) {
      const int kt = c * NTAP + tap;
      const int slot = (cc * NTAP + tap) % WD;
      if (tap == 0) {
        load_patch(min(c + 1, c_end - 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      if (PRO && !PW1 && tap >= T0) {
        constexpr int per = (PJ + NTAP - T0 - 1) / (NTAP - T0);
        transform(min(c + 1, c_end - 1), (tap - T0) * per, tap == NTAP - 1 ? PJ : (tap - T0 + 1) * per);
      }
      if (SUB)
        compute_tap(py + (tap >> 1), px + (tap & 1), c & 1, bq[slot]);
      else if (PW1)
        compute_tap(0, tap, c & 1, bq[slot]);
      else
        compute_tap(tap / 3, tap % 3, c & 1, bq[slot]);
      load_b(bq[slot], min(kt + WD, kt_end - 1));
      __builtin_amdgcn_sched_barrier(0);  // keep the refill WD taps ahead (the scheduler sinks loads to their use)
      // MODE 3: the next chunk's prologue after the last tap's MFMAs (two taps of load latency hidden)
      if (PW1 && PRO && tap == NTAP - 1) transform(min(c + 1, c_end - 1), 0, PJ);
      if (tap == NTAP - 1) store_patch((c + 1) & 1);  // after the last chunk: an unused buffer
    }
    __syncthreads();
  }
  }

  PW_STAMP(2);
  // ---- segment 2: 1x1 product of x2 (ResBlock shortcut), K = Cin2, un-pipelined (last split).
  if (a.Cin2 > 0 && (!KSPLIT || split == ksplit - 1)) {
    const int s2base = NTAP * a.Cin1 / kSK;
    int abase[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) abase[i] = (wm * WM + i * 32 + lr) * kSPitch + lh * kGrp;
    constexpr int RJ = (BM + 127) / 128;  // staging passes of 128 rows
    const float* xsrc[RJ];
#pragma unroll
    for (int j = 0; j < RJ; ++j)
      xsrc[j] = a.x2 + (size_t)min(m0 + srow + 128 * j, M - 1) * a.x2_pitch + 8 * shalf;
    for (int c2 = 0; c2 < a.Cin2; c2 += kSK) {
      f4 r0[RJ], r1[RJ];
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        r0[j] = *reinterpret_cast<const f4*>(xsrc[j] + c2);
        r1[j] = *reinterpret_cast<const f4*>(xsrc[j] + c2 + 4);
      }
      load_b(bq[0], s2base + c2 / kSK);
#pragma unroll
      for (int j = 0; j < RJ; ++j) {
        const int row = srow + 128 * j;
        if (row < BM) {  // rows >= M hold clamped data: never stored
          vec pc[NP];
          S::split(r0[j], r1[j], pc, bad);
#pragma unroll
          for (int q = 0; q < NP; ++q)
            *reinterpret_cast<vec*>(patch + row * kSPitch + shalf * kGrp + q * 8) = pc[q];
        }
      }
      __syncthreads();
      compute(patch, abase, bq[0]);
      __syncthreads();
    }
  }

  if (NP == 2 && bad && a.range_flag) *a.range_flag = 1;
  if constexpr (PW1 && NP == 2) {
    if (a.ap_q) {  // the attention operand planes (ConvArgs::ap_*), written in 16-B pieces through LDS
      attn_plane_epilogue<WM, WN>(a, acc, M, m0 + wm * WM, n0 + wn * WN, lr, lh,
                                  wave < 2 ? reinterpret_cast<float*>(patch) + wave * WM * (WN + 8)
                                           : gtab + (wave - 2) * WM * (WN + 8));
      PW_STAMP(3);
      PW_RSTAMP(6);
      return;
    }
  }
  // fp16x2: the epilogue undoes the per-output-channel power-of-two weight scale (exact) as it reads acc
  conv_patch_epilogue<BM, BN, WM, WN, MODE, KSPLIT>(a, acc, M, HWo, Wo, m0, n0, b0, wm, wn, lr, lh, split, py, px,
                                                    NP == 2 ? a.ws_rowscale : nullptr);
}

template <int BM, int BN, int WM, int WN, int MODE, int MAXP, int NP>
void launch3_mode(const ConvArgs& a, const PatchGeom& g, int blocks, hipStream_t st) {
  if constexpr (BM > 128 || MAXP == kPatch3Seg) {  // big / segment tiles: stride 1, no split-K (caller checks)
    if constexpr (MODE <= 2 && (MAXP != kPatch3Seg || MODE != 1)) {
      if (a.pro_scale)
        hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, MODE, MAXP, true, false, NP>), dim3(blocks),
                           dim3(256), 0, st, a, g);
      else
        hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, MODE, MAXP, false, false, NP>), dim3(blocks),
                           dim3(256), 0, st, a, g);
    }
    return;
  }
  if (MODE == 0 && a.ksplit > 1) {
    if (a.pro_scale)
      hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, 0, MAXP, true, true, NP>), dim3(blocks), dim3(256), 0,
                         st, a, g);
    else
      hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, 0, MAXP, false, true, NP>), dim3(blocks), dim3(256),
                         0, st, a, g);
    return;
  }
  if (a.pro_scale)
    hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, MODE, MAXP, true, false, NP>), dim3(blocks), dim3(256), 0,
                       st, a, g);
  else
    hipLaunchKernelGGL((conv_patch3_kernel<BM, BN, WM, WN, MODE, MAXP, false, false, NP>), dim3(blocks), dim3(256),
                       0, st, a, g);
}

// MODE 3 (1x1 / static-weight GEMM), 128-row tiles, fp16x2
template <int BN, int WN>
int launch_pw(const ConvArgs& a, hipStream_t st) {
  const int M = a.B * a.Hout * a.Wout;
  const int blocks = ceil_div(M, 128) * ceil_div(a.Cout, BN);
  PatchGeom g{};
  if (a.pro_scale)
    hipLaunchKernelGGL((conv_patch3_kernel<128, BN, 64, WN, 3, 128, true, false, 2>), dim3(blocks), dim3(256), 0, st,
                       a, g);
  else
    hipLaunchKernelGGL((conv_patch3_kernel<128, BN, 64, WN, 3, 128, false, false, 2>), dim3(blocks), dim3(256), 0,
                       st, a, g);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

template <int BM, int BN, int WM, int WN, int MAXP, int NP>
int launch3(const ConvArgs& a, const PatchGeom& g, hipStream_t st) {
  const bool sub = a.upsample == 2;
  const int M = sub ? a.B * a.Hin * a.Win : a.B * a.Hout * a.Wout;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  DM_REQUIRE(ks == 1 || (!a.upsample && a.kpart && ks <= a.Cin1 / kSK),
             "conv: split-K needs a stride-1 3x3 conv, a workspace and at most one split per channel chunk");
  DM_REQUIRE(g.P <= MAXP, "conv: patch larger than the split kernel's LDS image");
  DM_REQUIRE(NP == 3 || a.ws_rowscale, "conv: fp16x2 split weights need their row scales");
  DM_REQUIRE((BM <= 128 && MAXP != kPatch3Seg) || (ks == 1 && a.stride == 1 && !(MAXP == kPatch3Seg && a.upsample == 1)),
             "conv: the big / row-segment split tiles run stride-1 convs without split-K");
  const int blocks = ceil_div(M, BM) * ceil_div(a.Cout, BN) * (sub ? 4 : 1) * ks;
  if (sub)
    launch3_mode<BM, BN, WM, WN, 2, MAXP, NP>(a, g, blocks, st);
  else if (a.stride == 2)
    launch3_mode<BM, BN, WM, WN, 4, MAXP, NP>(a, g, blocks, st);
  else if (a.upsample)
    launch3_mode<BM, BN, WM, WN, 1, MAXP, NP>(a, g, blocks, st);
  else
    launch3_mode<BM, BN, WM, WN, 0, MAXP, NP>(a, g, blocks, st);
  DM_LAUNCH_CHECK();
  if (ks > 1) return conv_splitk_reduce(a, st);
  return DM_OK;
}

// Split slice s of matrix `mat` starts at this K column of the packed fp32 weights: slice
// c16 * ntap + tap holds channels 16 c16 .. 16 c16 + 15 of that tap (packed chunk-major over
// 32-channel chunks), then the 1x1 segment's slices in order.
__device__ __forceinline__ int split_slice_k0(int s, int cin1, int ntap) {
  const int main_sl = ntap * cin1 / kSK;
  if (s < main_sl) {
    const int c16 = s / ntap, tap = s - (s / ntap) * ntap;
    return ((c16 >> 1) * ntap + tap) * 32 + (c16 & 1) * 16;
  }
  return ntap * cin1 + (s - main_sl) * kSK;
}

// fp16x2 row scales: per output channel n, 2^e with max_mat,k |w[mat][n][k]| * 2^e in [2^13, 2^14)
// (1 for an all-zero row). rowscale[n] = 2^e (applied at the split), rowscale[rows + n] = 2^-e (the
// epilogue's exact inverse). One block per row.
__global__ void split_row_scale_kernel(const float* w, int nmat, int rows, int K, float* rowscale) {
  const int n = blockIdx.x;
  float m = 0.f;
  for (int mat = 0; mat < nmat; ++mat)
    for (int k = threadIdx.x; k < K; k += blockDim.x) m = fmaxf(m, fabsf(w[((size_t)mat * rows + n) * K + k]));
  __shared__ float red[256];
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int e = 0;
    if (red[0] > 0.f) {
      int ex;
      frexpf(red[0], &ex);  // red[0] in [2^(ex-1), 2^ex)
      e = min(max(14 - ex, -126), 126);
    }
    rowscale[n] = ldexpf(1.f, e);
    rowscale[rows + n] = ldexpf(1.f, -e);
  }
}

// [nmat][rows][K] fp32 packed conv weights -> split slices in the order conv_patch3_kernel walks them,
// each slice as B-fragment images [ceil(rows / 32) column groups][NP pieces][2 lane groups][32][8]
// (rows past `rows` stay zero). One thread per (matrix, slice, row, lane group).
template <int NP>
__global__ void split_conv_weights_kernel(const float* w, int nmat, int rows, int K, int cin1, int ntap,
                                          const float* rowscale, typename Split<NP>::elem* out) {
  typedef Split<NP> S;
  const int nsl = K / kSK;
  const int ngrp = (rows + 31) / 32;
  const long total = (long)nmat * nsl * rows * 2;
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= total) return;
  const int lg = id & 1;
  long r = id >> 1;
  const int row = r % rows;
  r /= rows;
  const int s = r % nsl;
  const int mat = r / nsl;
  const float* src = w + ((size_t)mat * rows + row) * K + split_slice_k0(s, cin1, ntap) + 8 * lg;
  f4 lo = *reinterpret_cast<const f4*>(src);
  f4 hi = *reinterpret_cast<const f4*>(src + 4);
  if (NP == 2) {
    const float sc = rowscale[row];  // a power of two: exact
    lo *= sc;
    hi *= sc;
  }
  typename S::vec pc[NP];
  bool bad = false;
  S::split(lo, hi, pc, bad);
  typename S::elem* dst = out + (((size_t)mat * nsl + s) * ngrp + (row >> 5)) * (NP * 512) + (lg * 32 + (row & 31)) * 8;
#pragma unroll
  for (int q = 0; q < NP; ++q) *reinterpret_cast<typename S::vec*>(dst + q * 512) = pc[q];
}

}  // namespace

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_pw_stamps(void* host, int nblocks) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pw_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

bool conv_patch3_ok(const ConvArgs& a, int which, const PatchGeom& g) {
  if (!a.ws || a.Cin1 % kSK != 0 || a.Cin2 % kSK != 0 || a.K % kSK != 0) return false;
  if (a.stride == 2) return a.ws_np == 2 && which == 6 && g.P <= kPatchS2Max;  // MODE 4: fp16x2, 64-row tiles
  if (which == 9) {  // 128-pixel row segments: fp16x2, one image's GroupNorm tables
    if (a.ws_np != 2 || (a.pro_scale && (long)g.TB * a.Cin1 * 2 > kSegTabFloats)) return false;
    return g.P <= kPatch3Seg;
  }
  if (which == 7 || which == 8) {  // one wave per SIMD, 128 x 128 wave tiles: fp16x2 only
    if (a.ws_np != 2 || (a.pro_scale && (long)g.TB * a.Cin1 * 2 > kPwTabFloats)) return false;
    return g.P <= (which == 7 ? kPatch3Max256 : kPatch3Max512);
  }
  if (a.ws_np == 2 && a.pro_scale && (long)g.TB * a.Cin1 * 2 > kPwTabFloats) return false;  // LDS GroupNorm tables
  return g.P <= (which == 6 ? kPatch3Max64 : kPatch3Max128);
}

bool conv_pw_ok(const ConvArgs& a) {
  if (!(a.taps == 1 && a.ws && a.ws_np == 2 && a.ws_rowscale && a.stride == 1 && !a.upsample && a.Cin2 == 0 &&
        a.Cin1 % (kPwSlices * kSK) == 0 && a.K == a.Cin1 && a.Hout == a.Hin && a.Wout == a.Win && a.ksplit <= 1))
    return false;
  // the GroupNorm tables of every image a 128-row tile can touch fit the kernel's LDS table
  const int hw = a.Hout * a.Wout;
  return !a.pro_scale || (long)(127 / hw + 2) * a.Cin1 * 2 <= kPwTabFloats;
}

bool conv_lds_tables(const ConvArgs& a) {
  if (!a.pro_scale || a.ws_np != 2) return false;
  if (a.taps == 1) return conv_pw_ok(a);
  if (a.taps != 9 || conv_pick(a) < 3) return false;
  PatchGeom g;
  conv_patch_pick(a, g);
  return conv_patch3_ok(a, conv_pick(a) + 1, g);
}

int conv2d_patch3(const ConvArgs& a, int which, const PatchGeom& g, hipStream_t st) {
  if (a.gin_part) {
    const long hw = (long)a.Hout * a.Wout;
    const long imgs = a.taps == 1 ? 127 / hw + 2 : g.TB;
    DM_REQUIRE(conv_lds_tables(a) && a.gin_G > 0 && a.Cin1 % a.gin_G == 0 && imgs * a.gin_G <= kGinStats,
               "conv: in-kernel GroupNorm finalize needs the LDS-table path and <= 512 (image, group) pairs");
  }
  if (a.taps == 1) {
    DM_REQUIRE(conv_pw_ok(a), "conv: the split 1x1 path needs fp16x2 weights, stride 1, K = Cin1 % 32 == 0 and LDS room for the GroupNorm tables");
    return which == 4 ? launch_pw<128, 64>(a, st) : launch_pw<64, 32>(a, st);
  }
  if (a.stride == 2) {
    DM_REQUIRE(a.ws_np == 2 && which == 6, "conv: the split stride-2 conv runs fp16x2 on 64-row tiles");
    return launch3<64, 64, 32, 32, kPatchS2Max, 2>(a, g, st);
  }
  if (a.ws_np == 2) {
    switch (which) {
      case 9: return launch3<128, 128, 64, 64, kPatch3Seg, 2>(a, g, st);
      case 7: return launch3<256, 256, 128, 128, kPatch3Max256, 2>(a, g, st);
      case 8: return launch3<512, 128, 128, 128, kPatch3Max512, 2>(a, g, st);
      case 4: return launch3<128, 128, 64, 64, kPatch3Max128, 2>(a, g, st);
      case 5: return launch3<128, 64, 64, 32, kPatch3Max128, 2>(a, g, st);
      default: return launch3<64, 64, 32, 32, kPatch3Max64, 2>(a, g, st);
    }
  }
  switch (which) {
    case 4: return launch3<128, 128, 64, 64, kPatch3Max128, 3>(a, g, st);
    case 5: return launch3<128, 64, 64, 32, kPatch3Max128, 3>(a, g, st);
    default: return launch3<64, 64, 32, 32, kPatch3Max64, 3>(a, g, st);
  }
}

// Bytes of a split copy: the pieces (rows padded to 32-column groups), then (fp16x2) 2 x rows fp32
// row scales.
static size_t split_piece_bytes(int nmat, int rows, int K, int np) {
  return (size_t)nmat * (K / kSK) * ((rows + 31) / 32) * 32 * (np == 2 ? Split<2>::kRow : Split<3>::kRow) * 2;
}

size_t split_conv_weights_bytes(int nmat, int rows, int K, int np) {
  const size_t pieces = split_piece_bytes(nmat, rows, K, np);
  return np == 2 ? pieces + (size_t)2 * rows * sizeof(float) : pieces;
}

const float* split_conv_rowscale(const void* ws, int nmat, int rows, int K) {
  return reinterpret_cast<const float*>(static_cast<const char*>(ws) + split_piece_bytes(nmat, rows, K, 2)) + rows;
}

int split_conv_weights(const float* w, int nmat, int rows, int K, int cin1, int ntap, int np, void* out,
                       hipStream_t st) {
  DM_REQUIRE(w && out && nmat > 0 && rows > 0, "split weights: empty");
  DM_REQUIRE(np == 2 || np == 3, "split weights: kind must be 2 (fp16x2) or 3 (bf16x3)");
  DM_REQUIRE(K % kSK == 0 && cin1 % 32 == 0 && ntap * cin1 <= K && (ntap == 9 || ntap == 4 || ntap == 3 || ntap == 1),
             "split weights: K must be ntap * cin1 (+ a second segment), cin1 a multiple of 32");
  DM_REQUIRE((reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0,
             "split weights: 16-byte alignment");
  const long total = (long)nmat * (K / kSK) * rows * 2;
  const unsigned grid = (unsigned)((total + 255) / 256);
  DM_CHECK_HIP(hipMemsetAsync(out, 0, split_piece_bytes(nmat, rows, K, np), st));  // padded column groups
  if (np == 2) {
    float* rs = const_cast<float*>(split_conv_rowscale(out, nmat, rows, K)) - rows;
    hipLaunchKernelGGL(split_row_scale_kernel, dim3(rows), dim3(256), 0, st, w, nmat, rows, K, rs);
    DM_LAUNCH_CHECK();
    hipLaunchKernelGGL(split_conv_weights_kernel<2>, dim3(grid), dim3(256), 0, st, w, nmat, rows, K, cin1, ntap,
                       rs, static_cast<_Float16*>(out));
  } else {
    hipLaunchKernelGGL(split_conv_weights_kernel<3>, dim3(grid), dim3(256), 0, st, w, nmat, rows, K, cin1, ntap,
                       nullptr, static_cast<__bf16*>(out));
  }
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
