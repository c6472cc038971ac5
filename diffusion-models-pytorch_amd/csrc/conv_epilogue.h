// Epilogue shared by the halo-patch convolution kernels (fp32 MFMA in
// conv_patch.hip, split-bf16 MFMA in conv_patch3.hip): both leave a wave's
// WM x WN sub-tile in the same 32x32 accumulator layout (column n on lane
// lr, row acc_row(r, lh) in register r), so the bias / temb row-vector /
// residual / GroupNorm-statistics epilogue (models/unet.py:16,26,41,43) and
// the split-K partial store are written once here.
#pragma once
#include <cstdint>
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


// T2D tiles (conv_k32.hip, conv_wino.hip on wide maps): GEMM row m -> pixel row of the NHWC tensor (image m / HWo,
// tile (m % HWo) / (TH TW) in row-major tile order, row-major inside the tile)
__device__ __forceinline__ size_t t2d_pixel(int m, int HWo, int Wo, int TH, int TW) {
  const int bb = m / HWo, rr = m - bb * HWo, tsz = TH * TW;
  const int tl = rr / tsz, r = rr - tl * tsz, ntx = Wo / TW;
  const int ty = tl / ntx, tx = tl - ty * ntx;
  const int iy = r / TW;
  return ((size_t)bb * HWo + (size_t)(ty * TH + iy) * Wo) + tx * TW + (r - iy * TW);
}

// LDS-staged epilogue (conv_k32.hip, the fused attention's proj): a wave's tile of acc * rowscale is put
// in LDS as 32-row slabs [32][WN + 4] fp32 by the kernel (in whatever MFMA layout it has), then each
// lane takes 4 consecutive output columns of a row (WN / 4 lanes per row), adds bias, per-image row
// vector and residual with 16-B loads and stores 16 B -- instead of one 4-B store per accumulator
// register (store-issue bound: 27k -> 8.5k cycles per K32 block). GroupNorm statistics of the stored
// values per 64-row chunk: per channel over the lane's rows, then across the wave's row lanes, then
// across the group's 4-channel quads (cpg = Cout / gn_G in {4, 8, 16, 32}: at most 8 quad lanes, within the
// LPR >= 8 lanes of a row for every wave width WN >= 32).
template <int WN>
struct StagedEpilogue {
  static constexpr int EP = WN + 4;     // slab pitch (floats)
  static constexpr int LPR = WN / 4;    // lanes per row
  static_assert(WN >= 32, "GroupNorm groups of up to 32 channels need >= 8 quad lanes per row");
  static constexpr int RPI = 64 / LPR;  // rows per wave instruction
  const ConvArgs& a;
  int M, HWo, b0, c4, rsub, ncol, nc;
  bool c_ok, one_image;
  int sub_w = 0, sub_ho = 0, sub_wo = 0, sub_py = 0, sub_px = 0;  // sub-pixel scatter (sub())
  int t2_wo = 0, t2_th = 0, t2_tw = 0;                             // 2-D tiles (t2d())
  f4 bias4, rv4;
  double gs[4], gq[4];

  // ncol0: the wave's first output column; b0: the tile's first image; one_image: every row of the tile
  // lies in image b0
  __device__ __forceinline__ StagedEpilogue(const ConvArgs& a_, int M_, int HWo_, int b0_, bool one_image_,
                                            int ncol0, int lane)
      : a(a_), M(M_), HWo(HWo_), b0(b0_), one_image(one_image_) {
    c4 = lane % LPR;
    rsub = lane / LPR;
    ncol = ncol0 + 4 * c4;
    c_ok = ncol < a.Cout;  // Cout % 4 == 0: the 4 columns are all valid or none
    nc = c_ok ? ncol : 0;
    const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
    bias4 = a.bias ? *reinterpret_cast<const f4*>(a.bias + nc) : zero4;
    rv4 = (a.rowvec && one_image) ? *reinterpret_cast<const f4*>(a.rowvec + (size_t)b0 * a.rowvec_pitch + nc) : zero4;
#pragma unroll
    for (int e = 0; e < 4; ++e) gs[e] = gq[e] = 0.0;
  }
  // sub-pixel upsample conv: tile row m = low-res pixel (b, iy, ix) of width w stores to output pixel
  // (b, 2 iy + py, 2 ix + px) of the ho x wo map
  __device__ __forceinline__ void sub(int w, int ho, int wo, int py, int px) {
    sub_w = w;
    sub_ho = ho;
    sub_wo = wo;
    sub_py = py;
    sub_px = px;
  }
  // 2-D tiles of wide maps: tile row m enumerates the image's TH x TW tiles in row-major order, row-major inside
  // the tile (conv_k32.hip T2D)
  __device__ __forceinline__ void t2d(int wo, int th, int tw) {
    t2_wo = wo;
    t2_th = th;
    t2_tw = tw;
  }
  __device__ __forceinline__ size_t out_row(int m) const {
    if (t2_wo) {  // (pixel of the tiled map: the output, or the sub-pixel conv's low-res map, then scattered)
      const int bb = m / HWo, rr = m - bb * HWo, tsz = t2_th * t2_tw;
      const int tl = rr / tsz, r = rr - tl * tsz, ntx = t2_wo / t2_tw;
      const int ty = tl / ntx, tx = tl - ty * ntx, ry = r / t2_tw;
      const int iy = ty * t2_th + ry, ix = tx * t2_tw + (r - ry * t2_tw);
      if (sub_w) return ((size_t)bb * sub_ho + 2 * iy + sub_py) * sub_wo + 2 * ix + sub_px;
      return (size_t)bb * HWo + (size_t)iy * t2_wo + ix;
    }
    if (!sub_w) return (size_t)m;
    const int bb = m / HWo, rr = m - bb * HWo;
    const int iy = rr / sub_w, ix = rr - iy * sub_w;
    return ((size_t)bb * sub_ho + 2 * iy + sub_py) * sub_wo + 2 * ix + sub_px;
  }
  // the slab's rows are output rows row0 .. row0 + 31 (this wave's slab written and visible)
  __device__ __forceinline__ void rows(const float* st, int row0) {
    rows_f([&](int row) { return *reinterpret_cast<const f4*>(st + row * EP + 4 * c4); }, row0);
  }
  // the same with the lane's 4 values of slab row `row` (columns 4 c4 ..) from val(row) instead of a staged slab
  template <class F>
  __device__ __forceinline__ void rows_f(F val, int row0) {
    f4 rs4[32 / RPI];
    if (a.res) {
#pragma unroll
      for (int it = 0; it < 32 / RPI; ++it) {
        const int m = min(row0 + it * RPI + rsub, M - 1);
        rs4[it] = *reinterpret_cast<const f4*>(a.res + out_row(m) * a.res_pitch + nc);
      }
    }
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int row = it * RPI + rsub;
      const int m = row0 + row;
      f4 v = val(row);
      if (a.bias) v = v + bias4;
      if (a.rowvec)
        v = v + (one_image ? rv4
                           : *reinterpret_cast<const f4*>(a.rowvec + (size_t)(min(m, M - 1) / HWo) * a.rowvec_pitch + nc));
      if (a.res) v = v + rs4[it];
      if (m < M && c_ok) *reinterpret_cast<f4*>(a.y + out_row(m) * a.y_pitch + ncol) = v;
      if (a.gn_part && m < M) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gs[e] += (double)v[e];
          gq[e] += (double)v[e] * v[e];
        }
      }
    }
  }
  // output rows in pairs (row0 + 2 i, row0 + 2 i + 1 for i < 16: a 32-row slab): val2(i, v0, v1) gives the lane's 4
  // values of both (the Winograd output transform, conv_wino.hip), then as rows()
  template <class F>
  __device__ __forceinline__ void pairs_f(F val2, int row0) {
    constexpr int IT = 16 / RPI;
    f4 rs4[IT][2];
    if (a.res) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int m = min(row0 + 2 * (it * RPI + rsub) + s, M - 1);
          rs4[it][s] = *reinterpret_cast<const f4*>(a.res + out_row(m) * a.res_pitch + nc);
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int i = it * RPI + rsub;
      f4 v[2];
      val2(i, v[0], v[1]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int m = row0 + 2 * i + s;
        if (a.bias) v[s] = v[s] + bias4;
        if (a.rowvec)
          v[s] = v[s] + (one_image ? rv4
                                   : *reinterpret_cast<const f4*>(a.rowvec + (size_t)(min(m, M - 1) / HWo) * a.rowvec_pitch + nc));
        if (a.res) v[s] = v[s] + rs4[it][s];
        if (m < M && c_ok) *reinterpret_cast<f4*>(a.y + out_row(m) * a.y_pitch + ncol) = v[s];
        if (a.gn_part && m < M) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gs[e] += (double)v[s][e];
            gq[e] += (double)v[s][e] * v[s][e];
          }
        }
      }
    }
  }
  // split-K partial sums: the slab as it stands to dst (pitch `pitch`), no bias / row vector / residual
  __device__ __forceinline__ void rows_raw(const float* st, int row0, float* dst, int pitch) {
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int row = it * RPI + rsub;
      const int m = row0 + row;
      const f4 v = *reinterpret_cast<const f4*>(st + row * EP + 4 * c4);
      if (m < M && c_ok) *reinterpret_cast<f4*>(dst + (size_t)m * pitch + ncol) = v;
    }
  }
  // this lane's 4-channel quad summed over the wave's rows so far (all 64 lanes call; resets the sums)
  __device__ __forceinline__ void quad_sums(double& s, double& q) {
    s = 0.0;
    q = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s += gs[e];
      q += gq[e];
      gs[e] = gq[e] = 0.0;
    }
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) {
      s += __shfl_xor(s, o);
      q += __shfl_xor(q, o);
    }
  }
  // statistics of the 64-row chunk starting at crow0 (all 64 lanes call; resets the sums)
  __device__ __forceinline__ void emit(int crow0) {
    double s, q;
    quad_sums(s, q);
    store_quads(s, q, crow0);
  }
  // the group sums of per-quad chunk totals s, q (valid in every lane of the quad's column) to gn_part
  __device__ __forceinline__ void store_quads(double s, double q, int crow0) {
    const int cpg = a.Cout / a.gn_G;
    for (int o = 1; o < cpg / 4; o <<= 1) {
      s += __shfl_xor(s, o);
      q += __shfl_xor(q, o);
    }
    int nchunk = (HWo + 63) / 64;
    const int bb = crow0 / HWo;
    int ch = (crow0 - bb * HWo) / 64;
    if (sub_w) {  // sub-pixel conv: the 64 low-res rows of parity (py, px) are chunk par * HWo / 64 + ch of the
      ch += (2 * sub_py + sub_px) * nchunk;  // output image (any disjoint cover of its pixels sums the same)
      nchunk *= 4;
    }
    if (rsub == 0 && (c4 % (cpg / 4)) == 0 && c_ok && crow0 < M)
      a.gn_part[((size_t)bb * nchunk + ch) * a.gn_G + ncol / cpg] = make_double2(s, q);
  }
};

// whether StagedEpilogue takes this conv's output (16-B columns, GroupNorm groups of 4, 8, 16 or 32 channels)
inline bool staged_epilogue_ok(const ConvArgs& a) {
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (a.Cout % 4 != 0 || a.y_pitch % 4 != 0 || !al16(a.y) || (a.bias && !al16(a.bias)) ||
      (a.res && (a.res_pitch % 4 != 0 || !al16(a.res))) || (a.rowvec && (a.rowvec_pitch % 4 != 0 || !al16(a.rowvec))))
    return false;
  if (a.gn_part && (a.gn_G <= 0 || a.Cout % a.gn_G != 0 || a.Cout / a.gn_G > 32 || (a.Cout / a.gn_G) % 4 != 0 ||
                    (a.Hout * a.Wout) % 64 != 0))
    return false;
  return true;
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
