// Epilogue shared by the halo-patch convolution kernels (fp32 MFMA in
// conv_patch.hip, split-bf16 MFMA in conv_patch3.hip): both leave a wave's
// WM x WN sub-tile in the same 32x32 accumulator layout (column n on lane
// lr, row acc_row(r, lh) in register r), so the bias / temb row-vector /
// residual / GroupNorm-statistics epilogue (models/unet.py:16,26,41,43) and
// the split-K partial store are written once here.
#pragma once
#include "dm_kernels.h"
#include "mfma_tile.h"

namespace dm {

template <int BM, int BN, int WM, int WN, int MODE, bool KSPLIT>
__device__ __forceinline__ void conv_patch_epilogue(const ConvArgs& a, f16v (&acc)[WM / 32][WN / 32], int M,
                                                    int HWo, int Wo, int m0, int n0, int b0, int wm, int wn,
                                                    int lr, int lh, int split, int py, int px) {
  constexpr bool SUB = MODE == 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  const int N = a.Cout;
  // ---- split-K: raw partial sums, epilogue in conv_splitk_reduce
  if (KSPLIT) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      if (n >= N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WM + i * 32 + acc_row(r, lh);
          if (m < M) a.kpart[((size_t)split * M + m) * N + n] = acc[i][j][r];
        }
    }
    return;
  }

  // SUB rows scatter to output pixel (2iy + py, 2ix + px)
  const bool block_one_image = (HWo % BM) == 0;
  // GroupNorm statistics of the stored values (MODE 0 / 3, WM = 64: this wave's rows are one chunk)
  const bool emit = (MODE == 0 || MODE == 3) && WM == 64 && a.gn_part != nullptr;
  const int wrow0 = m0 + wm * WM;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n_raw = n0 + wn * WN + j * 32 + lr;
    const bool n_ok = n_raw < N;
    const int n = n_ok ? n_raw : N - 1;
    double gs = 0.0, gq = 0.0;
    const float bn = a.bias ? a.bias[n] : 0.f;
    const float rv_blk = (a.rowvec && block_one_image) ? a.rowvec[(size_t)b0 * a.rowvec_pitch + n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // residual rows of this 32-row group loaded branch-free (clamped) before the stores, so the
      // 16 loads overlap; 16 extra VGPRs keep the kernel at 2 waves / SIMD
      float rsd[16];
      if (a.res) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = min(m0 + wm * WM + i * 32 + acc_row(r, lh), M - 1);
          size_t mo = m;
          if (SUB) {
            const int bb = m / HWo, rr = m - bb * HWo;
            const int iy = rr / Wo, ix = rr - (rr / Wo) * Wo;
            mo = ((size_t)bb * a.Hout + 2 * iy + py) * a.Wout + 2 * ix + px;
          }
          rsd[r] = a.res[mo * a.res_pitch + n];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + acc_row(r, lh);
        if (m >= M) continue;
        size_t mo = m;
        if (SUB) {
          const int bb = m / HWo, rr = m - bb * HWo;
          const int iy = rr / Wo, ix = rr - (rr / Wo) * Wo;
          mo = ((size_t)bb * a.Hout + 2 * iy + py) * a.Wout + 2 * ix + px;
        }
        float v = acc[i][j][r];
        if (a.bias) v = v + bn;
        if (a.rowvec) v = v + (block_one_image ? rv_blk : a.rowvec[(size_t)(m / HWo) * a.rowvec_pitch + n]);
        if (a.res) v = v + rsd[r];
        if (n_ok) a.y[mo * a.y_pitch + n] = v;
        if (emit) {
          gs += (double)v;
          gq += (double)v * v;
        }
      }
    }
    if (emit) {
      const int cpg = N / a.gn_G;
      const int nchunk = (HWo + 63) / 64;
      const int bb = wrow0 / HWo, ch = (wrow0 - bb * HWo) / 64;
      gn_emit_group(gs, gq, lr, lh, cpg, n_ok && wrow0 < M,
                    a.gn_part + ((size_t)bb * nchunk + ch) * a.gn_G + n_raw / cpg);
    }
  }
}


}  // namespace dm
