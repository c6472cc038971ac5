// Implicit-GEMM 2-D convolution on NHWC activations, fp32 MFMA.
//
// Replaces the torch.nn.Conv2d calls of the reference denoisers:
//   3x3 stride 1 pad 1   models/unet.py:16,26,72,118
//   3x3 stride 2 pad 1   models/modules.py:72      (Downsample)
//   nearest-2x + 3x3     models/modules.py:62-65   (Upsample; the 2x image is
//                                                   never materialised)
//   1x1                  models/unet.py:28 (shortcut), modules.py:83-86
//
// GEMM view: out[m][n] = sum_k A[m][k] * W[n][k]
//   m = output pixel (b, oy, ox), n = output channel,
//   k = tap * Cin1 + c over segment 1 (the conv input), then Cin2 more k for
//   an optional segment 2: a 1x1 product of a second NHWC tensor at the output
//   resolution (the ResBlock shortcut conv folded into the second conv's K
//   loop: out = conv2(h) + W_s x + b_s in one pass).
// Epilogue: + bias[n] + rowvec[b][n] (timestep-embedding projection,
// models/unet.py:41) + residual[m][n] (models/unet.py:43), stored through a
// pitched view so outputs can land inside a wider concat buffer.
//
// Loader: every thread owns A_ITERS output pixels for the whole K loop. Per
// tap it derives a source row pointer and a validity bit (zero padding);
// the loads themselves are unconditional (invalid rows read a clamped, valid
// address and are zeroed by a select), so the compiler keeps the next
// K-slice's global loads in flight across the MFMA work of the current one
// instead of draining vmcnt at exec-masked branches.
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"

namespace dm {

namespace {

enum ConvMode { CM_3X3_S1 = 0, CM_3X3_S2 = 1, CM_3X3_UP = 2, CM_1X1 = 3 };

// Bijective XCD-aware remap of the linear block id (cdna_hip_programming.md
// §5.5 T1): blocks dispatched round-robin over 8 XCDs; consecutive logical ids
// land on the same XCD so the N-tiles of one M-tile share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

template <int BM, int BN, int WM, int WN, int MODE>
__global__ void __launch_bounds__(256)
conv_igemm_kernel(ConvArgs a) {
  using Cfg = TileCfg<BM, BN, WM, WN>;
  __shared__ __attribute__((aligned(16))) float lds[Cfg::LDS_FLOATS];

  const int M = a.B * a.Hout * a.Wout;
  const int N = a.Cout;
  const int nN = ceil_div(N, BN);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / nN, nt = bid - (bid / nN) * nN;
  const int m0 = mt * BM, n0 = nt * BN;

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave / Cfg::NWN, wn = wave % Cfg::NWN;
  const int lc4 = t & 7;
  const int lrow = t >> 3;
  const int HWo = a.Hout * a.Wout;

  // Per-thread A rows: decode the output pixel once.
  int r_b[Cfg::A_ITERS], r_oy[Cfg::A_ITERS], r_ox[Cfg::A_ITERS];
  bool r_ok[Cfg::A_ITERS];
#pragma unroll
  for (int i = 0; i < Cfg::A_ITERS; ++i) {
    const int m = m0 + lrow + i * Cfg::ROWS_PER_PASS;
    r_ok[i] = m < M;
    const int mm = r_ok[i] ? m : M - 1;
    r_b[i] = mm / HWo;
    const int rem = mm - r_b[i] * HWo;
    r_oy[i] = rem / a.Wout;
    r_ox[i] = rem - r_oy[i] * a.Wout;
  }
  // B rows (output channels), clamped + validity.
  const float* wrow[Cfg::B_ITERS];
  bool w_ok[Cfg::B_ITERS];
#pragma unroll
  for (int j = 0; j < Cfg::B_ITERS; ++j) {
    const int n = n0 + lrow + j * Cfg::ROWS_PER_PASS;
    w_ok[j] = n < N;
    wrow[j] = a.w + (size_t)(w_ok[j] ? n : N - 1) * a.K + 4 * lc4;
  }

  const int taps = (MODE == CM_1X1) ? 1 : 9;
  const int nk1 = taps * (a.Cin1 / kBK);
  const int nk = nk1 + a.Cin2 / kBK;

  // Row pointers / validity for the current tap.
  const float* arow[Cfg::A_ITERS];
  bool a_ok[Cfg::A_ITERS];
  auto set_tap = [&](int tap) {
    const int ky = (MODE == CM_1X1) ? 1 : tap / 3;
    const int kx = (MODE == CM_1X1) ? 1 : tap - (tap / 3) * 3;
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i) {
      int iy, ix;
      bool ok = r_ok[i];
      if (MODE == CM_3X3_UP) {
        const int uy = r_oy[i] + ky - 1, ux = r_ox[i] + kx - 1;
        ok = ok && uy >= 0 && uy < 2 * a.Hin && ux >= 0 && ux < 2 * a.Win;
        iy = uy >> 1;
        ix = ux >> 1;
      } else if (MODE == CM_3X3_S2) {
        iy = 2 * r_oy[i] + ky - 1;
        ix = 2 * r_ox[i] + kx - 1;
        ok = ok && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
      } else {
        iy = r_oy[i] + ky - 1;
        ix = r_ox[i] + kx - 1;
        ok = ok && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
      }
      iy = min(max(iy, 0), a.Hin - 1);
      ix = min(max(ix, 0), a.Win - 1);
      a_ok[i] = ok;
      // zero padding by address (mfma_tile.h kZeroPage); rows >= M are clamped and discarded
      arow[i] = (ok || !r_ok[i]) ? a.x1 + ((size_t)(r_b[i] * a.Hin + iy) * a.Win + ix) * a.x1_pitch + 4 * lc4
                                 : kZeroPage + 4 * lc4;
    }
  };
  auto set_seg2 = [&]() {
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i) {
      const int m = min(m0 + lrow + i * Cfg::ROWS_PER_PASS, M - 1);
      a_ok[i] = r_ok[i];
      arow[i] = a.x2 + (size_t)m * a.x2_pitch + 4 * lc4;
    }
  };

  // Raw loaded registers; the zero-padding select is applied when they are
  // written to LDS (after the MFMA work), so no wait sits between the loads
  // and the compute that hides them.
  f4 ra[Cfg::A_ITERS], rb[Cfg::B_ITERS];
  bool ra_ok[Cfg::A_ITERS];
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // Loader state: K slice kt = chunk * taps + tap (chunk-major, matching the
  // packed weights), then segment 2.
  int ld_c = 0;
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i) {
      ra[i] = *reinterpret_cast<const f4*>(arow[i] + ld_c);
      ra_ok[i] = a_ok[i];
    }
#pragma unroll
    for (int j = 0; j < Cfg::B_ITERS; ++j) rb[j] = *reinterpret_cast<const f4*>(wrow[j] + kt * kBK);
    // advance to slice kt + 1 (wave-uniform control flow only)
    const int nx = kt + 1;
    if (nx < nk1) {
      const int chunk = (MODE == CM_1X1) ? nx : nx / 9;
      set_tap((MODE == CM_1X1) ? 0 : nx - chunk * 9);
      ld_c = chunk * kBK;
    } else if (nx == nk1) {
      ld_c = 0;
      set_seg2();
    } else {
      ld_c += kBK;
    }
  };

  auto store_tile = [&](int buf) {
    float* As = lds + buf * Cfg::STAGE;
    float* Bs = As + Cfg::A_ELEMS;
#pragma unroll
    for (int i = 0; i < Cfg::A_ITERS; ++i)
      *reinterpret_cast<f4*>(As + (lrow + i * Cfg::ROWS_PER_PASS) * kLDK + 4 * lc4) = ra[i];
#pragma unroll
    for (int j = 0; j < Cfg::B_ITERS; ++j)
      *reinterpret_cast<f4*>(Bs + (lrow + j * Cfg::ROWS_PER_PASS) * kLDK + 4 * lc4) = rb[j];  // rows >= N: discarded
  };

  f16v acc[Cfg::TM][Cfg::TN];
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk1 > 0) set_tap(0); else set_seg2();
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_tile(kt + 1);
    const float* As = lds + buf * Cfg::STAGE;
    const float* Bs = As + Cfg::A_ELEMS;
    mfma_slice<Cfg::TM, Cfg::TN>(As, Bs, wm * WM, wn * WN, lane, acc);
    if (more) store_tile(buf ^ 1);
    __syncthreads();
  }

  // Epilogue.
  const int lr = lane & 31, lh = lane >> 5;
  const bool block_one_image = (HWo % BM) == 0;
  const int b_blk = m0 / HWo;
#pragma unroll
  for (int j = 0; j < Cfg::TN; ++j) {
    const int n = n0 + wn * WN + j * 32 + lr;
    if (n >= N) continue;
    const float bn = a.bias ? a.bias[n] : 0.f;
    const float rv_blk = (a.rowvec && block_one_image) ? a.rowvec[(size_t)b_blk * a.rowvec_pitch + n] : 0.f;
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + acc_row(r, lh);
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (a.bias) v = v + bn;
        if (a.rowvec) v = v + (block_one_image ? rv_blk : a.rowvec[(size_t)(m / HWo) * a.rowvec_pitch + n]);
        if (a.res) v = v + a.res[(size_t)m * a.res_pitch + n];
        a.y[(size_t)m * a.y_pitch + n] = v;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
int launch_conv_tile(const ConvArgs& a, int mode, hipStream_t st) {
  using Cfg = TileCfg<BM, BN, WM, WN>;
  const int M = a.B * a.Hout * a.Wout;
  const int blocks = ceil_div(M, BM) * ceil_div(a.Cout, BN);
  switch (mode) {
    case CM_3X3_S1:
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CM_3X3_S1>), dim3(blocks), dim3(Cfg::NT), 0, st, a);
      break;
    case CM_3X3_S2:
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CM_3X3_S2>), dim3(blocks), dim3(Cfg::NT), 0, st, a);
      break;
    case CM_3X3_UP:
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CM_3X3_UP>), dim3(blocks), dim3(Cfg::NT), 0, st, a);
      break;
    default:
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, CM_1X1>), dim3(blocks), dim3(Cfg::NT), 0, st, a);
      break;
  }
  DM_LAUNCH_CHECK();
  return DM_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline int conv_mode(const ConvArgs& a) {
  if (a.taps == 1) return CM_1X1;
  if (a.upsample) return CM_3X3_UP;
  return a.stride == 2 ? CM_3X3_S2 : CM_3X3_S1;
}

}  // namespace

int conv2d_igemm(const ConvArgs& a, hipStream_t st) {
  DM_REQUIRE(a.taps == 1 || a.taps == 9, "conv: taps must be 1 or 9");
  DM_REQUIRE(a.stride == 1 || a.stride == 2, "conv: stride must be 1 or 2");
  DM_REQUIRE(!a.upsample || (a.taps == 9 && a.stride == 1), "conv: upsample needs 3x3 stride 1");
  DM_REQUIRE(a.upsample >= 0 && a.upsample <= 2, "conv: upsample must be 0, 1 (nearest) or 2 (sub-pixel)");
  DM_REQUIRE(a.Cin1 % kBK == 0 && a.Cin2 % kBK == 0, "conv: input channels must be multiples of 32");
  DM_REQUIRE(a.Cin1 + kBK <= kZeroPageFloats, "conv: too many input channels for the zero-padding page");
  DM_REQUIRE(a.Cin1 > 0, "conv: no input channels");
  DM_REQUIRE(a.K == (a.upsample == 2 ? 4 : a.taps) * a.Cin1 + a.Cin2, "conv: K mismatch");
  DM_REQUIRE(a.upsample != 2 || a.Cin2 == 0, "conv: sub-pixel upsample has no second segment");
  DM_REQUIRE(a.x1_pitch % 4 == 0 && a.y_pitch >= a.Cout && a.K % 4 == 0, "conv: pitch");
  DM_REQUIRE(aligned16(a.x1) && aligned16(a.w), "conv: operands must be 16-byte aligned");
  DM_REQUIRE(a.Cin2 == 0 || (a.x2 && aligned16(a.x2) && a.x2_pitch % 4 == 0), "conv: segment-2 operand");
  DM_REQUIRE(a.Cout > 0 && a.B > 0 && a.Hin > 0 && a.Win > 0, "conv: empty problem");
  if (a.upsample) {
    DM_REQUIRE(a.Hout == 2 * a.Hin && a.Wout == 2 * a.Win, "conv: upsample output size");
  } else if (a.taps == 9) {
    DM_REQUIRE(a.Hout == (a.Hin - 1) / a.stride + 1 && a.Wout == (a.Win - 1) / a.stride + 1,
               "conv: 3x3 output size");
  } else {
    DM_REQUIRE(a.stride == 1 && a.Hout == a.Hin && a.Wout == a.Win, "conv: 1x1 output size");
  }
  const long M = (long)a.B * a.Hout * a.Wout;
  DM_REQUIRE(M > 0 && M < (1L << 31), "conv: M out of range");
  DM_REQUIRE(a.tile >= 0 && a.tile <= 21, "conv: tile must be 0..21");
  if (a.tile == 21 || (a.tile == 0 && a.wino_ws)) {  // the Winograd F(2,3) kernel (conv_wino.hip)
    if (conv_wino_ok(a)) {
      if (!a.gn_part || conv_can_emit_gn(a)) return conv2d_wino(a, st);
      DM_REQUIRE(a.tile == 0, "conv: GroupNorm statistics need groups of 4..32 channels");
      // (automatic choice) statistics the Winograd epilogue cannot emit: the direct kernels without its weights
      ConvArgs d = a;
      d.wino_ws = nullptr;
      d.wino_rowscale = nullptr;
      return conv2d_igemm(d, st);
    }
    DM_REQUIRE(a.tile == 0, "conv: tile 21 needs Winograd weights and a shape conv_wino_kernel takes");
  }
  const int mode = conv_mode(a);
  const int pick = conv_pick(a);
  DM_REQUIRE(!a.gn_part || conv_can_emit_gn(a), "conv: GroupNorm statistics need a 128-row halo-patch tile, "
                                                 "whole 64-pixel chunks and groups within 32 channels");
  DM_REQUIRE(!a.pro_scale || (pick >= 3 && a.pro_shift && aligned16(a.pro_scale) && aligned16(a.pro_shift)),
             "conv: the GroupNorm prologue needs a halo-patch shape (3x3 stride 1 / upsample, whole-row tiles)");
  if (const int k32 = a.k32_resolved ? a.k32_resolved - 1 : conv_k32_pick(a)) return conv2d_k32(a, k32, st);
  if (pick >= 3 && a.taps == 1) return conv2d_patch3(a, pick + 1, PatchGeom{}, st);  // MODE 3 (split 1x1)
  if (pick >= 3) {
    PatchGeom g;
    conv_patch_pick(a, g);
    if (conv_patch3_ok(a, pick + 1, g)) return conv2d_patch3(a, pick + 1, g, st);
    if (pick + 1 <= 6) return conv2d_patch(a, pick + 1, g, st);
    return launch_conv_tile<128, 128, 64, 64>(a, mode, st);  // a split-only tile that does not fit
  }
  DM_REQUIRE(a.upsample != 2, "conv: the sub-pixel upsample runs on the halo-patch kernel only (shape has no "
                              "whole-row tiling)");
  switch (pick) {
    case 0: return launch_conv_tile<128, 128, 64, 64>(a, mode, st);
    case 1: return launch_conv_tile<128, 64, 64, 32>(a, mode, st);
    default: return launch_conv_tile<64, 64, 32, 32>(a, mode, st);
  }
}

// Kernel choice: 0..2 im2col tiles (128x128, 128x64, 64x64), 3..5 halo-patch
// tiles (same shapes). The patch kernel handles 3x3 stride-1 / upsample
// shapes whose tile covers whole rows; otherwise the im2col kernel, with the
// 128x128 tile when it still yields >= 2 waves of blocks over 256 CUs.
// `a.tile` 1..6 forces a configuration (tests / tuning); a forced patch tile
// falls back to im2col when the shape does not tile.
int conv_pick(const ConvArgs& a) {
  if (a.tile >= 1 && a.tile <= 3) return a.tile - 1;
  if ((a.tile == 10 || a.tile == 11) && conv_k32_ok(a)) return a.tile - 7;  // forced K = 32 split tiles (conv_k32.hip)
  if ((a.tile == 12 || a.tile == 13) && conv_k32_variant_ok(a, a.tile - 9)) return 5;  // forced K32 split-K tiles
  if (a.tile == 14 && conv_k32_variant_ok(a, 5)) return 8;  // forced K32 64-pixel row / segment tiles
  if (a.tile == 15 && conv_k32_variant_ok(a, 6)) return 5;  // forced K32 small-map kernel (in-block split-K)
  if (a.tile == 16 && conv_k32_variant_ok(a, 7)) return 8;  // forced K32 512-thread wide-map tiles
  if (a.tile == 17 && conv_k32_variant_ok(a, 8)) return 3;  // forced K32 big-table 128 x 128 tiles
  if (a.tile == 18 && conv_k32_variant_ok(a, 9)) return 5;  // forced K32 stride-2 tiles
  if (a.tile == 19 && conv_k32_variant_ok(a, 10)) return 3;  // forced K32 2-D tiles of wide maps
  if (a.tile == 20 && conv_k32_variant_ok(a, 11)) return 3;  // forced K32 64-row single-image tiles (8^2)
  if (conv_pw_ok(a)) {  // split 1x1: 128x128 tiles when they still give >= 2 blocks per CU, else 128x64
    const long M = (long)(a.pick_B > 0 ? a.pick_B : a.B) * a.Hout * a.Wout;
    return (a.Cout >= 128 && ((M + 127) / 128) * ((a.Cout + 127) / 128) >= 512) ? 3 : 4;
  }
  PatchGeom g;
  const int p = conv_patch_pick(a, g);
  if (p) return p - 1;
  if (a.tile >= 4 && a.tile <= 6) return a.tile - 4;  // a forced patch tile that does not fit: its im2col shape
  if (a.tile >= 7) return 0;                           // a forced big / segment split tile that does not fit
  const long M = (long)(a.pick_B > 0 ? a.pick_B : a.B) * a.Hout * a.Wout;
  const long b128 = ((M + 127) / 128) * ((a.Cout + 127) / 128);
  if (a.Cout >= 128 && b128 >= 512) return 0;
  const long b128x64 = ((M + 127) / 128) * ((a.Cout + 63) / 64);
  if (b128x64 >= 512) return 1;
  return 2;
}

bool conv_can_emit_gn(const ConvArgs& a) {
  // the split-K reduction emits them (conv_splitk_reduce_gn_kernel; after the 4 x 4 Winograd kernel, conv_k32s's own
  // in-block reduction): one chunk per image
  if (a.ksplit > 1)
    return !a.upsample && a.Hout * a.Wout <= kGnPixPerChunk && a.gn_G > 0 && a.Cout % a.gn_G == 0 &&
           a.Cout <= 1024;
  if ((a.tile == 0 || a.tile == 21) && conv_wino_ok(a))  // StagedEpilogue over 64-pixel chunks of one image
    return a.gn_G > 0 && a.Cout % a.gn_G == 0 && (a.Cout / a.gn_G) % 4 == 0 && a.Cout / a.gn_G <= 32;
  // the K32 stride-2 tiles: a block's 64 rows are one 64-pixel chunk (two 32-row waves per column slice)
  if (a.stride == 2 && conv_k32_pick(a) == 9)
    return (a.Hout * a.Wout) % 64 == 0 && a.gn_G > 0 && a.Cout % a.gn_G == 0 && 32 % (a.Cout / a.gn_G) == 0;
  // the K32 2-D tiles of wide maps: each wave's 64 rows are one tile's 64 pixels (a disjoint cover of the image;
  // of one parity's low-res pixels for the sub-pixel upsample)
  if (conv_k32_pick(a) == 10)
    return a.gn_G > 0 && a.Cout % a.gn_G == 0 && 32 % (a.Cout / a.gn_G) == 0 &&
           (a.upsample != 2 || (toggles().gn_fusion && (a.Cout / a.gn_G) % 4 == 0));
  const int pick = conv_pick(a);
  if (pick != 3 && pick != 4 && pick != 6 && pick != 7 && pick != 8) return false;  // waves own whole 64-row chunks
  if (conv_k32_pick(a) && a.Cout % a.gn_G == 0 && a.Cout / a.gn_G > 32) return false;  // K32: groups within 32 columns
  // the K32 sub-pixel upsample (128-row tiles, 64-row waves of one parity): chunks of 64 low-res pixels
  if (a.upsample == 2) {
    const int v = conv_k32_pick(a);
    return (v == 1 || v == 2) && toggles().gn_fusion && (a.Hin * a.Win) % 64 == 0 && a.gn_G > 0 &&
           a.Cout % a.gn_G == 0 && 32 % (a.Cout / a.gn_G) == 0 && (a.Cout / a.gn_G) % 4 == 0;
  }
  if (a.upsample || (a.ksplit > 1)) return false;
  if (a.taps == 1 && !conv_pw_ok(a)) return false;
  if ((a.Hout * a.Wout) % 64 != 0 || a.gn_G <= 0 || a.Cout % a.gn_G != 0) return false;
  const int cpg = a.Cout / a.gn_G;
  return 32 % cpg == 0;
}

// The exact kernel instantiation (matches the rocprofv3 kernel name with spaces removed).
std::string conv_label(const ConvArgs& a) {
  static const char* names[] = {"conv_igemm_kernel<128,128,64,64", "conv_igemm_kernel<128,64,64,32",
                                "conv_igemm_kernel<64,64,32,32",   "conv_patch_kernel<128,128,64,64",
                                "conv_patch_kernel<128,64,64,32",  "conv_patch_kernel<64,64,32,32",
                                "conv_patch_kernel<256,256,128,128", "conv_patch_kernel<512,128,128,128",
                                "conv_patch_kernel<128,128,64,64"};
  if ((a.tile == 0 || a.tile == 21) && conv_wino_ok(a)) return conv_wino_label(a);
  if (const int k32 = a.k32_resolved ? a.k32_resolved - 1 : conv_k32_pick(a)) return conv_k32_label(a, k32);
  const int p = conv_pick(a);
  std::string s = names[p];
  if (p < 3) s += "," + std::to_string(conv_mode(a)) + ">";  // <BM,BN,WM,WN,MODE>
  if (p >= 3 && a.taps == 1)  // split 1x1: conv_patch3_kernel<128,BN,64,WN,3,128,PRO,false,2>
    return std::string(p == 3 ? "conv_patch3_kernel<128,128,64,64,3,128," : "conv_patch3_kernel<128,64,64,32,3,128,") +
           (a.pro_scale ? "true" : "false") + ",false,2>";
  if (p >= 3) {  // <BM,BN,WM,WN,MODE,MAXP,PRO,KSPLIT>; MAXP 288 (208 split-bf16) for 128-row tiles, 160 for 64-row
    PatchGeom g;
    conv_patch_pick(a, g);
    const bool x3 = conv_patch3_ok(a, p + 1, g);
    if (x3) s.replace(0, 17, "conv_patch3_kernel");
    s += "," + std::to_string(a.stride == 2 ? 4 : a.upsample);
    s += a.stride == 2 ? ",384" : p == 5 ? ",160" : p == 6 ? ",352" : p == 7 ? ",656" : p == 8 ? ",392" :
         (x3 ? ",208" : ",288");
    s += a.pro_scale ? ",true" : ",false";
    s += a.ksplit > 1 ? ",true" : ",false";  // rocprofv3 prints the defaulted arguments too
    s += x3 ? "," + std::to_string(a.ws_np) + ">" : ">";  // <..., NP>: 3 bf16x3, 2 fp16x2
  }
  return s;
}

}  // namespace dm
