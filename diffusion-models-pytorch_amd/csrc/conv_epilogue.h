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

// qkv column n of token m -> the attention operand planes (ConvArgs::ap_*), split as the attention
// GEMMs split on load (gemm.hip store_tile): q * alpha, k * b_scale (each only if != 1), times 2^e.
__device__ __forceinline__ void conv_store_attn_planes(const ConvArgs& a, int m, int n, float v) {
  const int Dh = a.ap_Dh, C = a.ap_heads * Dh;
  int part, h, d;
  if (a.ap_legacy) {
    h = n / (3 * Dh);
    const int r = n - h * 3 * Dh;
    part = r / Dh;
    d = r - part * Dh;
  } else {
    part = n / C;
    const int c = n - part * C;
    h = c / Dh;
    d = c - h * Dh;
  }
  const int b = m / a.ap_L, tok = m - b * a.ap_L;
  float x;
  if (part == 0) x = (a.ap_alpha != 1.0f ? v * a.ap_alpha : v) * ldexpf(1.f, a.ap_ea);
  else if (part == 1) x = ((a.ap_bscale != 0.0f && a.ap_bscale != 1.0f) ? v * a.ap_bscale : v) * ldexpf(1.f, a.ap_eb);
  else x = v * ldexpf(1.f, a.ap_ev);
  const _Float16 h0 = (_Float16)x;
  const _Float16 h1 = (_Float16)(x - (float)h0);
  if (fabsf(x) > 65504.f && a.range_flag) *a.range_flag = 1;
  const size_t plane = (size_t)a.ap_L * Dh, base = ((size_t)b * a.ap_heads + h) * 2 * plane;
  if (part < 2) {
    _Float16* dst = (part == 0 ? a.ap_q : a.ap_k) + base + (size_t)tok * Dh + d;
    dst[0] = h0;
    dst[plane] = h1;
  } else {
    _Float16* dst = a.ap_v + base + (size_t)d * a.ap_L + tok;
    dst[0] = h0;
    dst[plane] = h1;
  }
}

// colscale (fp16x2 split kernels): the per-output-channel power-of-two weight scale to undo, applied to
// each accumulator as it is read (exact), so the 16 x 16 accumulators of a 128 x 128 wave tile are never
// materialised scaled all at once.
// LEAN: no per-image row vector and no attention operand planes (the fused attention's proj)
template <int BM, int BN, int WM, int WN, int MODE, bool KSPLIT, bool LEAN = false>
__device__ __forceinline__ void conv_patch_epilogue(const ConvArgs& a, f16v (&acc)[WM / 32][WN / 32], int M,
                                                    int HWo, int Wo, int m0, int n0, int b0, int wm, int wn,
                                                    int lr, int lh, int split, int py, int px,
                                                    const float* colscale = nullptr) {
  constexpr bool SUB = MODE == 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  const int N = a.Cout;
  // ---- split-K: raw partial sums, epilogue in conv_splitk_reduce
  if (KSPLIT) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + lr;
      if (n >= N) continue;
      const float cs = colscale ? colscale[min(n, N - 1)] : 1.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * WM + i * 32 + acc_row(r, lh);
          if (m < M) a.kpart[((size_t)split * M + m) * N + n] = colscale ? acc[i][j][r] * cs : acc[i][j][r];
        }
    }
    return;
  }

  // SUB rows scatter to output pixel (2iy + py, 2ix + px)
  const bool block_one_image = (HWo % BM) == 0;
  // GroupNorm statistics of the stored values (MODE 0 / 3, WM a multiple of 64: this wave's rows are whole
  // 64-pixel chunks, summed per chunk in the same order at every WM)
  const bool emit = (MODE == 0 || MODE == 3) && WM % 64 == 0 && a.gn_part != nullptr;
  const int wrow0 = m0 + wm * WM;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n_raw = n0 + wn * WN + j * 32 + lr;
    const bool n_ok = n_raw < N;
    const int n = n_ok ? n_raw : N - 1;
    double gs = 0.0, gq = 0.0;
    const float bn = a.bias ? a.bias[n] : 0.f;
    const float cs = colscale ? colscale[n] : 1.f;
    const float rv_blk = (!LEAN && a.rowvec && block_one_image) ? a.rowvec[(size_t)b0 * a.rowvec_pitch + n] : 0.f;
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
        float v = colscale ? acc[i][j][r] * cs : acc[i][j][r];
        if (a.bias) v = v + bn;
        if (!LEAN && a.rowvec) v = v + (block_one_image ? rv_blk : a.rowvec[(size_t)(m / HWo) * a.rowvec_pitch + n]);
        if (a.res) v = v + rsd[r];
        if (!LEAN && MODE == 3 && a.ap_q) {
          if (n_ok) conv_store_attn_planes(a, m, n, v);
          continue;
        }
        if (n_ok) a.y[mo * a.y_pitch + n] = v;
        if (emit) {
          gs += (double)v;
          gq += (double)v * v;
        }
      }
      if (emit && (i & 1)) {  // rows i - 1, i: one 64-pixel chunk
        const int crow0 = wrow0 + (i - 1) * 32;
        const int cpg = N / a.gn_G;
        const int nchunk = (HWo + 63) / 64;
        const int bb = crow0 / HWo, ch = (crow0 - bb * HWo) / 64;
        gn_emit_group(gs, gq, lr, lh, cpg, n_ok && crow0 < M,
                      a.gn_part + ((size_t)bb * nchunk + ch) * a.gn_G + n_raw / cpg);
        gs = 0.0;
        gq = 0.0;
      }
    }
  }
}


}  // namespace dm
