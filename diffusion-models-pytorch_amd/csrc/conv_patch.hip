// 3x3 convolution (stride 1, or nearest-2x upsample + stride 1) with the
// input halo patch staged in LDS once per 32-channel chunk.
//
// Same GEMM view and epilogue as conv.hip (models/unet.py:16,26,41,43,
// models/modules.py:62-65), but A is not re-gathered from global memory for
// every tap: a block's output tile covers TB images x TH rows x the full
// width, so its receptive field is a (TH+2) x (W+2) pixel patch per image.
// Per channel chunk the patch is loaded once (zero padding written as zeros)
// and the nine taps read shifted A fragments from it; only the weights
// stream per tap. Global/L2 traffic for A drops ~9x / (halo factor) versus
// the im2col loader, and the LDS write volume for A likewise.
//
// K order inside the packed weight matrix: k = (chunk * 9 + tap) * 32 + c
// (chunk-major), followed by an optional 1x1 segment (the ResBlock shortcut)
// of Cin2 columns, handled by a second, un-pipelined phase.
//
// MODE 2 (sub-pixel nearest-2x upsample + 3x3 conv, models/modules.py:60-65,
// adm/unet.py:119-129): an output pixel (2iy + py, 2ix + px) of the upsampled
// conv only ever sees the 2x2 low-res neighbourhood rows iy + py - 1 + {0, 1},
// cols ix + px - 1 + {0, 1}, with the 3x3 taps that land on the same source
// pixel summed. Each parity class (py, px) is therefore a 4-tap conv on the
// low-res input (taps (py + ty, px + tx) of the ordinary pad-1 low-res patch)
// with its own combined weights [4][Cout][chunk][4 taps][32]: 4/9 of the MFMA
// work of convolving the upsampled image. Blocks are split over the 4 parities;
// the epilogue scatters rows to (2iy + py, 2ix + px).
#include <algorithm>
#include <cstdlib>
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "conv_epilogue.h"

namespace dm {

namespace {

template <int BM, int BN, int WM, int WN, int MODE, int MAXP, bool PRO, bool KSPLIT = false>
__global__ void __launch_bounds__(256)
conv_patch_kernel(ConvArgs a, PatchGeom g) {
  using Cfg = TileCfg<BM, BN, WM, WN>;
  constexpr bool UP = MODE == 1, SUB = MODE == 2;
  constexpr int NTAP = SUB ? 4 : 9;
  constexpr int PATCH_FLOATS = MAXP * kLDK;
  constexpr int WSTAGE = BN * kLDK;
  __shared__ __attribute__((aligned(16))) float lds[PATCH_FLOATS + 2 * WSTAGE];
  float* patch = lds;
  float* wbuf = lds + PATCH_FLOATS;

  // GEMM rows: output pixels, or (SUB) low-res pixels of one parity class
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
  const int y0 = (m0 - b0 * HWo) / Wo;  // first output row of the tile (even for UP)

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int wm = wave / Cfg::NWN, wn = wave % Cfg::NWN;
  const int lc4 = t & 7;
  const int lrow = t >> 3;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- patch loader geometry (pixel p = lrow + 32 j)
  constexpr int PJ = (MAXP + 31) / 32;
  const int PHW = g.PH * g.PW;
  const float* psrc[PJ];
  bool pok[PJ];
  int pimg[PJ];
  const int iy_base = UP ? (y0 >> 1) - 1 : y0 - 1;
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const int p = lrow + 32 * j;
    const int img = p / PHW;
    const int rem = p - img * PHW;
    const int pr = rem / g.PW, pc = rem - (rem / g.PW) * g.PW;
    const int b = b0 + img;
    const int iy = iy_base + pr, ix = pc - 1;
    const bool ok = p < g.P && b < a.B && iy >= 0 && iy < a.Hin && ix >= 0 && ix < a.Win;
    pok[j] = ok;
    const int bc = min(b, a.B - 1);
    pimg[j] = bc;
    const int iyc = min(max(iy, 0), a.Hin - 1), ixc = min(max(ix, 0), a.Win - 1);
    // padding pixels read the zero page (PRO re-zeroes them after the transform instead)
    psrc[j] = (ok || PRO) ? a.x1 + ((size_t)(bc * a.Hin + iyc) * a.Win + ixc) * a.x1_pitch + 4 * lc4
                          : kZeroPage + 4 * lc4;
  }
  // ---- weight loader
  const float* wrow[Cfg::B_ITERS];
  bool w_ok[Cfg::B_ITERS];
#pragma unroll
  for (int j = 0; j < Cfg::B_ITERS; ++j) {
    const int n = n0 + lrow + j * Cfg::ROWS_PER_PASS;
    w_ok[j] = n < N;
    wrow[j] = a.w + ((size_t)par * N + (w_ok[j] ? n : N - 1)) * a.K + 4 * lc4;
  }

  // ---- A-fragment patch coordinates of this lane's rows
  int fy[Cfg::TM], fx[Cfg::TM], fimg[Cfg::TM];
  const int tile_rows = g.TH * Wo;
#pragma unroll
  for (int i = 0; i < Cfg::TM; ++i) {
    const int ml = wm * WM + i * 32 + lr;
    fimg[i] = ml / tile_rows;
    const int rem = ml - fimg[i] * tile_rows;
    fy[i] = rem / Wo;
    fx[i] = rem - fy[i] * Wo;
  }

  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  f4 rp[PJ], rb[Cfg::B_ITERS];
  auto load_patch = [&](int chunk) {
    const int co = chunk * kBK;
#pragma unroll
    for (int j = 0; j < PJ; ++j) rp[j] = *reinterpret_cast<const f4*>(psrc[j] + co);
  };
  // GroupNorm + SiLU prologue on patch registers j in [j0, j1): silu(x * scale[b][c] + shift[b][c]).
  // Spread over the taps of the previous chunk so the VALU work interleaves with MFMAs.
  auto transform = [&](int chunk, int j0, int j1) {
    const int cc = chunk * kBK + 4 * lc4;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      if (j >= j0 && j < j1) {
        const f4 sc = *reinterpret_cast<const f4*>(a.pro_scale + (size_t)pimg[j] * a.Cin1 + cc);
        const f4 sh = *reinterpret_cast<const f4*>(a.pro_shift + (size_t)pimg[j] * a.Cin1 + cc);
#pragma unroll
        for (int q = 0; q < 4; ++q) rp[j][q] = silu_fast(rp[j][q] * sc[q] + sh[q]);
      }
    }
  };
  // padding stays exactly 0 (applied after the transform)
  auto store_patch = [&]() {
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const int p = lrow + 32 * j;
      if (j * 32 < MAXP && p < MAXP)
        *reinterpret_cast<f4*>(patch + p * kLDK + 4 * lc4) = (!PRO || pok[j]) ? rp[j] : zero4;
    }
  };
  auto load_w = [&](int kt) {
#pragma unroll
    for (int j = 0; j < Cfg::B_ITERS; ++j) rb[j] = *reinterpret_cast<const f4*>(wrow[j] + kt * kBK);
  };
  auto store_w = [&](int buf) {
    float* Bs = wbuf + buf * WSTAGE;
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

  // One 32-deep K slice: A rows from the patch at tap (ky, kx), B from wbuf[buf].
  auto compute_tap = [&](int ky, int kx, int buf) {
    int abase[Cfg::TM];
#pragma unroll
    for (int i = 0; i < Cfg::TM; ++i) {
      int pr, pc;
      if (UP) {
        pr = ((fy[i] + ky - 1) >> 1) + 1;
        pc = ((fx[i] + kx - 1) >> 1) + 1;
      } else {
        pr = fy[i] + ky;
        pc = fx[i] + kx;
      }
      abase[i] = ((fimg[i] * g.PH + pr) * g.PW + pc) * kLDK + 4 * lh;
    }
    const float* Bs = wbuf + buf * WSTAGE;
#pragma unroll
    for (int kc = 0; kc < kBK; kc += 8) {
      f4 av[Cfg::TM], bv[Cfg::TN];
#pragma unroll
      for (int i = 0; i < Cfg::TM; ++i) av[i] = *reinterpret_cast<const f4*>(patch + abase[i] + kc);
#pragma unroll
      for (int j = 0; j < Cfg::TN; ++j)
        bv[j] = *reinterpret_cast<const f4*>(Bs + (wn * WN + j * 32 + lr) * kLDK + kc + 4 * lh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < Cfg::TM; ++i)
#pragma unroll
          for (int j = 0; j < Cfg::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s], bv[j][s], acc[i][j], 0, 0, 0);
    }
  };

  const int nchunks = a.Cin1 / kBK;
  const int c_begin = KSPLIT ? split * nchunks / ksplit : 0;
  const int c_end = KSPLIT ? (split + 1) * nchunks / ksplit : nchunks;
  load_patch(c_begin);
  load_w(c_begin * NTAP);
  if (PRO) transform(c_begin, 0, PJ);
  store_patch();
  store_w((c_begin * NTAP) & 1);
  __syncthreads();
  for (int c = c_begin; c < c_end; ++c) {
    const bool more_chunks = c + 1 < c_end;
#pragma unroll
    for (int tap = 0; tap < NTAP; ++tap) {
      const int kt = c * NTAP + tap;
      const bool more_w = (tap < NTAP - 1) || more_chunks;
      if (more_w) load_w(kt + 1);
      if (tap == 0 && more_chunks) load_patch(c + 1);
      if (PRO && tap >= 1 && more_chunks) {
        constexpr int per = (PJ + NTAP - 2) / (NTAP - 1);
        transform(c + 1, (tap - 1) * per, tap == NTAP - 1 ? PJ : tap * per);
      }
      if (SUB)
        compute_tap(py + (tap >> 1), px + (tap & 1), kt & 1);
      else
        compute_tap(tap / 3, tap % 3, kt & 1);
      if (more_w) store_w((kt + 1) & 1);
      __syncthreads();
    }
    if (more_chunks) {
      store_patch();
      __syncthreads();
    }
  }

  // ---- segment 2: 1x1 product of x2 (ResBlock shortcut), K = Cin2, un-pipelined (last split).
  if (a.Cin2 > 0 && (!KSPLIT || split == ksplit - 1)) {
    const int k2base = 9 * a.Cin1;
    float* As = patch;  // BM x kLDK fits in the patch region (P >= BM for the stride-1 geometry)
    for (int c2 = 0; c2 < a.Cin2; c2 += kBK) {
      f4 ra[Cfg::A_ITERS];
      bool rok[Cfg::A_ITERS];
#pragma unroll
      for (int i = 0; i < Cfg::A_ITERS; ++i) {
        const int m = m0 + lrow + i * Cfg::ROWS_PER_PASS;
        rok[i] = m < M;
        ra[i] = *reinterpret_cast<const f4*>(a.x2 + (size_t)min(m, M - 1) * a.x2_pitch + c2 + 4 * lc4);
      }
      load_w((k2base + c2) / kBK);
#pragma unroll
      for (int i = 0; i < Cfg::A_ITERS; ++i)
        *reinterpret_cast<f4*>(As + (lrow + i * Cfg::ROWS_PER_PASS) * kLDK + 4 * lc4) = ra[i];  // rows >= M: discarded
      store_w(0);
      __syncthreads();
      mfma_slice<Cfg::TM, Cfg::TN>(As, wbuf, wm * WM, wn * WN, lane, acc);
      __syncthreads();
    }
  }

  conv_patch_epilogue<BM, BN, WM, WN, MODE, KSPLIT>(a, acc, M, HWo, Wo, m0, n0, b0, wm, wn, lr, lh, split, py, px);
}

// Split-K reduction: y = sum_s kpart[s] (split order) + bias + rowvec + residual.
__global__ void conv_splitk_reduce_kernel(ConvArgs a) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int N = a.Cout;
  const long M = (long)a.B * a.Hout * a.Wout;
  if (e >= M * N) return;
  const long m = e / N;
  const int n = e - m * N;
  float v = a.kpart[e];
  for (int s = 1; s < a.ksplit; ++s) v = v + a.kpart[(size_t)s * M * N + e];
  if (a.bias) v = v + a.bias[n];
  if (a.rowvec) v = v + a.rowvec[(size_t)(m / ((long)a.Hout * a.Wout)) * a.rowvec_pitch + n];
  if (a.res) v = v + a.res[(size_t)m * a.res_pitch + n];
  a.y[(size_t)m * a.y_pitch + n] = v;
}

// The same reduction, one block per image, also emitting the GroupNorm statistics of the stored
// values (maps of <= 64 pixels: the image is one gn_partial chunk, layout [B][1][G]), so the
// consumer skips its gn_partial launch.
__global__ void __launch_bounds__(1024) conv_splitk_reduce_gn_kernel(ConvArgs a) {
  extern __shared__ double red_d[];  // [PG][2][Cout]
  const int b = blockIdx.x;
  const int N = a.Cout, HW = a.Hout * a.Wout;
  const long M = (long)a.B * HW;
  const int PG = max(1, (int)blockDim.x / N);  // pixel groups: thread (pg, n) sums pixels pg, pg + PG, ..
  const int t = threadIdx.x;
  for (int n0 = 0; n0 < N; n0 += blockDim.x) {
    const int n = n0 + t % min(N, (int)blockDim.x), pg = t / min(N, (int)blockDim.x);
    if (pg < PG && n < N) {
      double s1 = 0.0, s2 = 0.0;
      for (int p = pg; p < HW; p += PG) {
        const long m = (long)b * HW + p;
        const long e = m * N + n;
        float v = a.kpart[e];
        for (int s = 1; s < a.ksplit; ++s) v = v + a.kpart[(size_t)s * M * N + e];
        if (a.bias) v = v + a.bias[n];
        if (a.rowvec) v = v + a.rowvec[(size_t)b * a.rowvec_pitch + n];
        if (a.res) v = v + a.res[(size_t)m * a.res_pitch + n];
        a.y[(size_t)m * a.y_pitch + n] = v;
        s1 += (double)v;
        s2 += (double)v * v;
      }
      red_d[(size_t)pg * 2 * N + n] = s1;
      red_d[(size_t)pg * 2 * N + N + n] = s2;
    }
  }
  __syncthreads();
  const int cpg = N / a.gn_G;
  for (int g = t; g < a.gn_G; g += blockDim.x) {
    double s1 = 0.0, s2 = 0.0;
    for (int q = 0; q < PG; ++q)
      for (int j = 0; j < cpg; ++j) {
        s1 += red_d[(size_t)q * 2 * N + g * cpg + j];
        s2 += red_d[(size_t)q * 2 * N + N + g * cpg + j];
      }
    a.gn_part[(size_t)b * a.gn_G + g] = make_double2(s1, s2);
  }
}

}  // namespace

int conv_splitk_reduce(const ConvArgs& a, hipStream_t st) {
  if (a.gn_part) {
    DM_REQUIRE(a.Hout * a.Wout <= kGnPixPerChunk && a.gn_G > 0 && a.Cout % a.gn_G == 0 && a.Cout <= 1024,
               "conv: split-K GroupNorm statistics need maps of <= 64 pixels and whole groups");
    const int threads = 1024, pg = std::max(1, threads / a.Cout);
    hipLaunchKernelGGL(conv_splitk_reduce_gn_kernel, dim3(a.B), dim3(threads), (size_t)pg * 2 * a.Cout * sizeof(double),
                       st, a);
    DM_LAUNCH_CHECK();
    return DM_OK;
  }
  const long total = (long)a.B * a.Hout * a.Wout * a.Cout;
  hipLaunchKernelGGL(conv_splitk_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

namespace {

template <int BM, int BN, int WM, int WN, int MODE, int MAXP>
void launch_patch_mode(const ConvArgs& a, const PatchGeom& g, int blocks, hipStream_t st) {
  // split-K variants only for MODE 0 (small maps); the unsplit kernels keep their register budget
  if (MODE == 0 && a.ksplit > 1) {
    if (a.pro_scale)
      hipLaunchKernelGGL((conv_patch_kernel<BM, BN, WM, WN, 0, MAXP, true, true>), dim3(blocks), dim3(256), 0, st,
                         a, g);
    else
      hipLaunchKernelGGL((conv_patch_kernel<BM, BN, WM, WN, 0, MAXP, false, true>), dim3(blocks), dim3(256), 0, st,
                         a, g);
    return;
  }
  if (a.pro_scale)
    hipLaunchKernelGGL((conv_patch_kernel<BM, BN, WM, WN, MODE, MAXP, true>), dim3(blocks), dim3(256), 0, st, a, g);
  else
    hipLaunchKernelGGL((conv_patch_kernel<BM, BN, WM, WN, MODE, MAXP, false>), dim3(blocks), dim3(256), 0, st, a, g);
}

template <int BM, int BN, int WM, int WN, int MAXP>
int launch_patch(const ConvArgs& a, const PatchGeom& g, hipStream_t st) {
  const bool sub = a.upsample == 2;
  const int M = sub ? a.B * a.Hin * a.Win : a.B * a.Hout * a.Wout;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  DM_REQUIRE(ks == 1 || (!a.upsample && a.kpart && ks <= a.Cin1 / kBK),
             "conv: split-K needs a stride-1 3x3 conv, a workspace and at most one split per channel chunk");
  const int blocks = ceil_div(M, BM) * ceil_div(a.Cout, BN) * (sub ? 4 : 1) * ks;
  if (sub)
    launch_patch_mode<BM, BN, WM, WN, 2, MAXP>(a, g, blocks, st);
  else if (a.upsample)
    launch_patch_mode<BM, BN, WM, WN, 1, MAXP>(a, g, blocks, st);
  else
    launch_patch_mode<BM, BN, WM, WN, 0, MAXP>(a, g, blocks, st);
  DM_LAUNCH_CHECK();
  if (ks > 1) {
    const long total = (long)M * a.Cout;
    (void)total;
    return conv_splitk_reduce(a, st);
  }
  return DM_OK;
}

}  // namespace

// Patch geometry for a BM-row tile, or false when the shape does not tile
// (then the im2col kernel is used).
bool conv_patch_geom(const ConvArgs& a, int BM, PatchGeom& g) {
  if (a.taps != 9) return false;
  if (a.stride == 2) {  // split kernel MODE 4: output rows of 2 TH + 1 input rows, parity-split columns
    const int Ho = a.Hout, Wo = a.Wout;
    if (a.upsample || a.Cin2 || a.Hin != 2 * Ho || a.Win != 2 * Wo || Wo > BM || BM % Wo != 0) return false;
    const int rows = BM / Wo;
    if (rows <= Ho) {
      if (Ho % rows != 0) return false;
      g.TB = 1;
      g.TH = rows;
    } else {
      if (rows % Ho != 0) return false;
      g.TB = rows / Ho;
      g.TH = Ho;
    }
    g.PH = 2 * g.TH + 1;
    g.PW = 2 * (Wo + 1);
    g.P = g.TB * g.PH * g.PW;
    g.TW = Wo;
    return true;
  }
  if (a.stride != 1) return false;
  const bool sub = a.upsample == 2;  // tiles over the low-res pixels of one parity class
  const int Ho = sub ? a.Hin : a.Hout, Wo = sub ? a.Win : a.Wout;
  if (Wo > BM) {  // row segments of BM pixels: one image, one output row, BM consecutive columns
    if (Wo % BM != 0 || a.upsample == 1) return false;
    g.TB = 1;
    g.TH = 1;
    g.TW = BM;
    g.PH = 3;
    g.PW = BM + 2;
    g.P = g.PH * g.PW;
    return !(sub && a.Cin2 != 0);
  }
  g.TW = Wo;
  if (BM % Wo != 0) return false;
  const int rows = BM / Wo;  // output rows per tile (across images)
  if (rows <= Ho) {
    if (Ho % rows != 0) return false;
    g.TB = 1;
    g.TH = rows;
  } else {
    if (rows % Ho != 0) return false;
    g.TB = rows / Ho;
    g.TH = Ho;
  }
  if (a.upsample == 1) {
    if (g.TH % 2 != 0 || a.Cin2 != 0) return false;
    g.PH = g.TH / 2 + 2;
    g.PW = a.Win + 2;
  } else {
    if (sub && a.Cin2 != 0) return false;
    g.PH = g.TH + 2;
    g.PW = Wo + 2;
  }
  g.P = g.TB * g.PH * g.PW;
  if (a.Cin2 > 0 && g.P < BM) return false;
  return true;
}


int conv_patch_pick(const ConvArgs& a, PatchGeom& g) {
  if (a.stride == 2) {  // only the fp16x2 split kernel has a stride-2 mode (64-row tiles)
    if (!(a.ws && a.ws_np == 2) || (a.tile != 0 && a.tile != 6)) return 0;
    return conv_patch_geom(a, 64, g) && g.P <= kPatchS2Max ? 6 : 0;
  }
  // big-tile fp16x2 split kernels (one wave per SIMD): forced by tile 7 / 8 only (for now)
  if (a.tile == 7 || a.tile == 8) {
    if (!(a.ws && a.ws_np == 2)) return 0;
    if (a.tile == 7) return conv_patch_geom(a, 256, g) && g.P <= kPatch3Max256 ? 7 : 0;
    return conv_patch_geom(a, 512, g) && g.P <= kPatch3Max512 ? 8 : 0;
  }
  // wide maps (ADM 256^2 / 128^2): 128-pixel row segments on the fp16x2 split kernel
  {
    const bool sub = a.upsample == 2;
    const int Wo = sub ? a.Win : a.Wout;
    if (Wo > 128) {
      if (!(a.ws && a.ws_np == 2) || (a.tile != 0 && a.tile != 9)) return 0;
      return conv_patch_geom(a, 128, g) && g.P <= kPatch3Seg ? 9 : 0;
    }
  }
  // the split-bf16 kernel's LDS image holds fewer patch pixels at 128-row tiles
  const int max128 = a.ws ? kPatch3Max128 : kPatchMax128, max64 = a.ws ? kPatch3Max64 : kPatchMax64;
  if (a.tile == 4 || a.tile == 0) {
    const long M = (long)(a.pick_B > 0 ? a.pick_B : a.B) * a.Hout * a.Wout;
    const long b128 = ((M + 127) / 128) * ((a.Cout + 127) / 128);
    const long b128x64 = ((M + 127) / 128) * ((a.Cout + 63) / 64);
    if ((a.tile == 4 || (a.Cout >= 128 && b128 >= 512)) && conv_patch_geom(a, 128, g) && g.P <= max128)
      return 4;
    if (a.tile == 0 && b128x64 >= 512 && conv_patch_geom(a, 128, g) && g.P <= max128) return 5;
    // 64-pixel-wide maps (ADM 64^2): two whole rows per 128-row tile need the row-segment kernel's LDS image
    const int Wo = a.upsample == 2 ? a.Win : a.Wout;
    if (a.tile == 0 && a.ws && a.ws_np == 2 && Wo >= 64 && conv_patch_geom(a, 128, g) && g.TB == 1 &&
        g.P <= kPatch3Seg && g.P > max128)
      return 9;
    if (a.tile == 0 && conv_patch_geom(a, 64, g) && g.P <= max64) return 6;
  } else if (a.tile == 5) {
    if (conv_patch_geom(a, 128, g) && g.P <= max128) return 5;
  } else if (a.tile == 6) {
    if (conv_patch_geom(a, 64, g) && g.P <= max64) return 6;
  }
  return 0;
}

// Whether a conv can run on the split-bf16 kernel at every batch size: the 64-row tile (the
// picker's last resort) must fit, which depends on the layer shape only, so the fp32 / split choice
// of a layer never changes with B and results stay batch-invariant.
bool conv_split_eligible(const ConvArgs& a) {
  if (a.taps == 1)  // 1x1 / static-weight GEMM (MODE 3 of the split kernel)
    return a.stride == 1 && !a.upsample && a.Cin2 == 0 && a.Cin1 % 32 == 0 && a.K == a.Cin1 && a.Hout == a.Hin &&
           a.Wout == a.Win;
  if (a.taps == 9 && a.stride == 2) {  // MODE 4 of the split kernel
    PatchGeom g;
    return a.Cin1 % 32 == 0 && conv_patch_geom(a, 64, g) && g.P <= kPatchS2Max;
  }
  if (a.taps != 9 || a.stride != 1 || a.upsample == 1 || a.Cin1 % 16 != 0 || a.Cin2 % 16 != 0) return false;
  PatchGeom g;
  return conv_patch_geom(a, 64, g) && g.P <= kPatch3Max64;
}

// Whether a conv runs on the fp16x2 row-segment / wide-row split kernel (which 9) at every batch size:
// a shape-only test like conv_split_eligible.
bool conv_seg_eligible(const ConvArgs& a) {
  if (a.taps != 9 || a.stride != 1 || a.Cin1 % 16 != 0 || a.Cin2 % 16 != 0) return false;
  const int Wo = a.upsample == 2 ? a.Win : a.Wout;
  if (Wo < 64) return false;
  PatchGeom g;
  return conv_patch_geom(a, 128, g) && g.TB == 1 && g.P <= kPatch3Seg;
}

int conv2d_patch(const ConvArgs& a, int which, const PatchGeom& g, hipStream_t st) {
  switch (which) {
    case 4: return launch_patch<128, 128, 64, 64, kPatchMax128>(a, g, st);
    case 5: return launch_patch<128, 64, 64, 32, kPatchMax128>(a, g, st);
    default: return launch_patch<64, 64, 32, 32, kPatchMax64>(a, g, st);
  }
}

}  // namespace dm
