// Fused self-attention core for 16 x 16 maps (L = 256 tokens): S = (alpha q) (b_scale k)^T, row softmax,
// O = P v, in one kernel, S never leaving the CU.
//
// Reference: models/modules.py:89-102 (SelfAttentionBlock: q * scale, bmm(q^T, k), softmax(-1),
// bmm(v, attn^T)), models/adm/unet.py:347-408 (QKVAttention[Legacy]: q, k each * ch^-1/4, softmax in
// fp32). The unfused path (gemm.hip S GEMM, softmax_rows, PV GEMM) writes S (B x heads x L x L fp32)
// to HBM, reads and rewrites it for the softmax and reads it again for PV: 4 x 67 MB per CIFAR block
// at B = 256. Here one block owns 32 (head dim 256) or 64 (head dim 64) query rows of one (image, head):
//   1. S [QT x L]: q rows and k rows staged through LDS as fp16x2 pieces (the split GEMM's operand
//      format and exponents, split16.h), 4 waves x (QT rows x L/4 keys), 3 MFMAs per 16-deep slice;
//   2. S -> LDS (fp32 rows), softmax per row exactly as softmax_rows (elementwise.hip): the same
//      per-lane max / expf / sum order and the same v * (1 / sum), so P is bit-identical; P is split
//      (x 2^14) in place into the A-operand layout of step 3;
//   3. O [QT x Dh] = P v: v rows staged transposed ([d][key], KN4 loader of gemm.hip), waves over
//      output columns (Dh = 256: 64 columns each; Dh = 64: 2 x 2 waves of 32 x 32).
// The operand tiles of both contractions are prefetched two k steps ahead into registers.
// Every contraction runs the same MFMA sequence in the same k order as the unfused GEMMs, so the
// output equals the unfused path bit for bit (tests/test_gpu_parity.py test_fused_attention_bit_identical).
// LDS (head dim 256, 32 query rows per block): 41 KB staging + 37 KB S / P rows -> two blocks per CU.
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"
#include "conv_epilogue.h"

namespace dm {

namespace {

constexpr int kAL = 256;             // tokens
constexpr int kAK = 32;              // k per staged tile
constexpr int kAP = 72;              // fp16 pitch of a staged 32-k row (two 16-deep slices + pad: 144 B)
constexpr int kSP = 8 * kAP / 2 + 4;  // fp32 pitch of an S row = one P row of 8 key blocks + 16 B (1168 B = 73
                                      // 16-B slots, odd: a 32-row P / O fragment read is conflict free; 1152 B
                                      // put every other row on the same slot, 8-way conflicts)


#ifdef DM_K32_STAMPS
// Diagnostic build only (tools/k32_stamps.py --attn): per block, wave 0's s_memtime at phase boundaries
// of attn_presplit_kernel and s_memrealtime at start / end. Written to this buffer only.
__device__ unsigned long long g_attn_stamps[8192][10];
#define AT_STAMP(k)                                                                                      \
  do {                                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_attn_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();  \
  } while (0)
#define AT_RSTAMP(k)                                                                                     \
  do {                                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_attn_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define AT_STAMP(k) do {} while (0)
#define AT_RSTAMP(k) do {} while (0)
#endif

__device__ __forceinline__ int split_off(int k) { return (k >> 4) * 32 + ((k >> 3) & 1) * 16 + (k & 7); }

// Softmax rows of L = 256 scores hold 4 consecutive keys per lane (4 lane .. 4 lane + 3, one 16-B LDS read),
// as softmax_rows (elementwise.hip) does for L = 256: the max, expf, the lane's sum in key order, then the
// butterfly -- the same operations in the same order, so P is bit-identical across the three paths. The
// lane's 4 P values are split and stored as one 8-B piece-0 write and one 8-B piece-1 write (was 8 2-B
// writes from keys lane + 64 u).
__device__ __forceinline__ void p_store4(_Float16* prow, int lane, const f4& p, float pp) {
  f16x4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float x = p[e] * pp;
    const _Float16 h0 = (_Float16)x;
    hi[e] = h0;
    lo[e] = (_Float16)(x - (float)h0);
  }
  const int k = 4 * lane;
  _Float16* dst = prow + (k >> 5) * kAP + split_off(k & 31);
  *reinterpret_cast<f16x4*>(dst) = hi;
  *reinterpret_cast<f16x4*>(dst + 8) = lo;
}

// QT query rows per block: 32 for DH = 256 (78 KB of LDS: two blocks per CU), 64 for DH = 64 (the PV
// wave layout needs 64 rows there). Operand tiles are prefetched two k steps ahead into registers.
template <int DH, int QT>
__global__ void __launch_bounds__(256) attn_fused_kernel(AttnArgs a) {
  static_assert((DH == 256 && QT == 32) || (DH == 64 && QT == 64), "head dims 64 / 256");
  constexpr int kAQ = QT;
  constexpr int STAGE_H = (kAQ + kAL) * kAP;      // Q + K tiles (fp16 elements)
  constexpr int VSTAGE_H = DH * kAP;              // V^T tile
  constexpr int REGION_H = STAGE_H > VSTAGE_H ? STAGE_H : VSTAGE_H;
  __shared__ __attribute__((aligned(16))) _Float16 stg[REGION_H];
  __shared__ __attribute__((aligned(16))) float sp[kAQ * kSP];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  // block -> (image, head, query tile); consecutive blocks of one (image, head) share its k / v in L2
  const int nq = kAL / kAQ;
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int qt = bid % nq, bh = bid / nq;
  const int h = bh % a.heads, b = bh / a.heads;
  const float* rows = a.qkv + (size_t)b * kAL * a.ld;
  const float* qsrc = rows + (size_t)qt * kAQ * a.ld + a.q0 + h * a.hs;
  const float* ksrc = rows + a.k0 + h * a.hs;
  const float* vsrc = rows + a.v0 + h * a.hs;
  const float pa = ldexpf(1.f, a.ea), pb = ldexpf(1.f, a.eb), pp = ldexpf(1.f, a.ep), pv = ldexpf(1.f, a.ev);
  bool bad = false;

  // ---------------------------------------------------------------- 1. S = (alpha q)(b_scale k)^T
  const int lc4 = t & 7, lrow = t >> 3;   // loader: 8 threads per 32-k row, 32 rows per pass
  f4 rq[2][kAQ / 32], rk[2][kAL / 32];    // two register sets: tiles kt and kt + 1 in flight
  auto load_s = [&](int kt, int set) {
    const int k = kt * kAK + 4 * lc4;
#pragma unroll
    for (int i = 0; i < kAQ / 32; ++i)
      rq[set][i] = *reinterpret_cast<const f4*>(qsrc + (size_t)(lrow + 32 * i) * a.ld + k);
#pragma unroll
    for (int i = 0; i < kAL / 32; ++i)
      rk[set][i] = *reinterpret_cast<const f4*>(ksrc + (size_t)(lrow + 32 * i) * a.ld + k);
  };
  auto store_s = [&](int set) {
#pragma unroll
    for (int i = 0; i < kAQ / 32; ++i) {
      f4 v = rq[set][i];
      if (a.alpha != 1.0f) v = v * a.alpha;
      f16x4 hi, lo;
      Split<2>::split4(v * pa, hi, lo, bad);
      _Float16* dst = stg + (lrow + 32 * i) * kAP + split_off(4 * lc4);
      *reinterpret_cast<f16x4*>(dst) = hi;
      *reinterpret_cast<f16x4*>(dst + 8) = lo;
    }
#pragma unroll
    for (int i = 0; i < kAL / 32; ++i) {
      const f4 v = (a.b_scale != 0.0f && a.b_scale != 1.0f) ? rk[set][i] * a.b_scale : rk[set][i];
      f16x4 hi, lo;
      Split<2>::split4(v * pb, hi, lo, bad);
      _Float16* dst = stg + (kAQ + lrow + 32 * i) * kAP + split_off(4 * lc4);
      *reinterpret_cast<f16x4*>(dst) = hi;
      *reinterpret_cast<f16x4*>(dst + 8) = lo;
    }
  };
  constexpr int SM = kAQ / 32;   // 32-row tiles of S per wave
  f16v acc[SM][2];
#pragma unroll
  for (int i = 0; i < SM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // wave w: all query rows of the tile, keys 64 w .. 64 w + 63 (2 x 32)
  constexpr int nkt = DH / kAK;   // even
  auto s_step = [&](int kt, int set) {
    store_s(set);
    __syncthreads();
    if (kt + 2 < nkt) load_s(kt + 2, set);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      f16x8 av[SM][2], bv[2][2];
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          av[i][q] = *reinterpret_cast<const f16x8*>(stg + (i * 32 + lr) * kAP + sl * 32 + lh * 16 + q * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          bv[j][q] = *reinterpret_cast<const f16x8*>(stg + (kAQ + wave * 64 + j * 32 + lr) * kAP + sl * 32 + lh * 16 +
                                                     q * 8);
#pragma unroll
      for (int i = 0; i < SM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) Split<2>::mma(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  };
  load_s(0, 0);
  load_s(1, 1);
  for (int kt = 0; kt < nkt; kt += 2) {
    s_step(kt, 0);
    s_step(kt + 1, 1);
  }
  // S rows to LDS (fp32, exact unscale)
  {
    const float unscale = ldexpf(1.f, -(a.ea + a.eb));
#pragma unroll
    for (int i = 0; i < SM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sp[(i * 32 + acc_row(r, lh)) * kSP + wave * 64 + j * 32 + lr] = acc[i][j][r] * unscale;
  }
  __syncthreads();

  // ---------------------------------------------------------------- 2. softmax rows -> P pieces in place
  for (int row = wave * (kAQ / 4); row < (wave + 1) * (kAQ / 4); ++row) {
    float* srow = sp + row * kSP;
    f4 v = *reinterpret_cast<const f4*>(srow + 4 * lane);
    float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = expf(v[e] - mx);
      sum += v[e];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
    // P row: 8 key blocks x kAP fp16 over the same bytes (this wave's read of the row came first)
    p_store4(reinterpret_cast<_Float16*>(srow), lane, v * inv, pp);
  }
  __syncthreads();

  // ---------------------------------------------------------------- 3. O = P v
  // waves: DH = 256: all rows x 64 columns each; DH = 64 (64 rows): 2 x 2 waves of 32 x 32
  constexpr int TM = DH == 256 ? kAQ / 32 : 1, TN = DH == 256 ? 2 : 1;
  const int orow0 = DH == 256 ? 0 : (wave >> 1) * 32;
  const int ocol0 = DH == 256 ? wave * 64 : (wave & 1) * 32;
  f16v oacc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][j][r] = 0.f;
  // V tile loader (gemm.hip KN4): thread -> 4 keys (4 kq ..) x 4 columns (4 n4 ..), stored transposed
  constexpr int NB = DH / 4 * 8;            // (32 / 4 key quads) x (DH / 4 column quads) blocks
  constexpr int VB = (NB + 255) / 256;       // blocks per thread
  f4 rv[2][VB][4];
  auto load_v = [&](int kb, int set) {
#pragma unroll
    for (int p = 0; p < VB; ++p) {
      const int blk = min(t + 256 * p, NB - 1);
      const int kq = blk & 7, n4 = blk >> 3;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        rv[set][p][r] = *reinterpret_cast<const f4*>(vsrc + (size_t)(kb * kAK + 4 * kq + r) * a.ld + 4 * n4);
    }
  };
  auto store_v = [&](int set) {
#pragma unroll
    for (int p = 0; p < VB; ++p) {
      const int blk = t + 256 * p;
      if (blk >= NB) continue;
      const int kq = blk & 7, n4 = blk >> 3;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f4 col = {rv[set][p][0][q], rv[set][p][1][q], rv[set][p][2][q], rv[set][p][3][q]};
        f16x4 hi, lo;
        Split<2>::split4(col * pv, hi, lo, bad);
        _Float16* dst = stg + (4 * n4 + q) * kAP + split_off(4 * kq);
        *reinterpret_cast<f16x4*>(dst) = hi;
        *reinterpret_cast<f16x4*>(dst + 8) = lo;
      }
    }
  };
  const _Float16* P = reinterpret_cast<const _Float16*>(sp);
  constexpr int PPITCH = 2 * kSP;  // fp16 elements per P row
  constexpr int nkb = kAL / kAK;   // even
  auto pv_step = [&](int kb, int set) {
    store_v(set);
    __syncthreads();
    if (kb + 2 < nkb) load_v(kb + 2, set);
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      f16x8 av[TM][2], bv[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          av[i][q] = *reinterpret_cast<const f16x8*>(P + (orow0 + i * 32 + lr) * PPITCH + kb * kAP + sl * 32 + lh * 16 +
                                                     q * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          bv[j][q] = *reinterpret_cast<const f16x8*>(stg + (ocol0 + j * 32 + lr) * kAP + sl * 32 + lh * 16 + q * 8);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Split<2>::mma(av[i], bv[j], oacc[i][j]);
    }
    __syncthreads();
  };
  load_v(0, 0);
  load_v(1, 1);
  for (int kb = 0; kb < nkb; kb += 2) {
    pv_step(kb, 0);
    pv_step(kb + 1, 1);
  }
  if (bad && a.range_flag) *a.range_flag = 1;
  const float ounscale = ldexpf(1.f, -(a.ep + a.ev));
  float* out = a.out + ((size_t)b * kAL + qt * kAQ) * a.ldo + h * DH;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(size_t)(orow0 + i * 32 + acc_row(r, lh)) * a.ldo + ocol0 + j * 32 + lr] = oacc[i][j][r] * ounscale;
}

// The attention block's output projection for one head of C = 256 channels (models/modules.py:101,
// proj 1x1 conv + residual; ADM proj_out), on the block's 64 O rows: O (wave w holds rows 0..63, columns
// 64 w ..) goes through LDS (fp32 rows, then split in place into the A-operand layout, the O rows split
// unscaled exactly as the MODE 3 conv splits its input), then each wave computes 64 rows x 64 output
// channels from the pre-split weights (the conv's B-fragment images, same slice order) and runs the
// conv epilogue (row scale, bias, residual, GroupNorm statistics): bit-identical to proj as its own launch.
__device__ __forceinline__ void attn_proj(const ConvArgs& c, f16v (&oacc)[2][2], float ounscale, float* sp, int m0,
                                          int wave, int lr, int lh, bool staged) {
  __syncthreads();  // every wave is done reading P
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sp[(i * 32 + acc_row(r, lh)) * kSP + wave * 64 + j * 32 + lr] = oacc[i][j][r] * ounscale;
  __syncthreads();
  const int lane = lr + 32 * lh;
  bool bad = false;
  for (int row = wave * 16; row < wave * 16 + 16; ++row) {
    float* srow = sp + row * kSP;
    f4 v = *reinterpret_cast<const f4*>(srow + 4 * lane);   // 256 values: 4 per lane
    _Float16* prow = reinterpret_cast<_Float16*>(srow);
    f16x4 hi, lo;
    Split<2>::split4(v, hi, lo, bad);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // the whole row is in registers before it is overwritten
    __builtin_amdgcn_wave_barrier();
    const int k = 4 * lane;
    _Float16* dst = prow + (k >> 5) * kAP + split_off(k & 31);
    *reinterpret_cast<f16x4*>(dst) = hi;
    *reinterpret_cast<f16x4*>(dst + 8) = lo;
  }
  __syncthreads();
  AT_STAMP(4);
  // 64 x 256 output tile: wave w owns columns 64 w .. 64 w + 63; K = 256 = 16 slices
  const _Float16* A = reinterpret_cast<const _Float16*>(sp);
  constexpr int PPITCH = 2 * kSP;
  const int ngrp = c.Cout / 32;
  const size_t slice_stride = (size_t)ngrp * (2 * 512);
  const _Float16* wsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    wsrc[j] = reinterpret_cast<const _Float16*>(c.ws) + (size_t)((wave * 64 + j * 32) >> 5) * (2 * 512) + (lh * 32 + lr) * 8;
  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  constexpr int RD = 4;
  f16x8 bq[RD][2][2];
  auto load_b = [&](int s, int slot) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q) bq[slot][j][q] = *reinterpret_cast<const f16x8*>(wsrc[j] + (size_t)s * slice_stride + q * 512);
  };
#pragma unroll
  for (int s = 0; s < RD; ++s) load_b(s, s);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int slot = s % RD;
    f16x8 av[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        av[i][q] = *reinterpret_cast<const f16x8*>(A + (i * 32 + lr) * PPITCH + (s >> 1) * kAP + (s & 1) * 32 + lh * 16 +
                                                   q * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) Split<2>::mma(av[i], bq[slot][j], acc[i][j]);
    load_b(min(s + RD, 15), slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (bad && c.range_flag) *c.range_flag = 1;
  AT_STAMP(5);
  const int M = c.B * c.Hout * c.Wout, HWo = c.Hout * c.Wout;
  if (!staged) {
    conv_patch_epilogue<64, 256, 64, 64, 3, false, true>(c, acc, M, HWo, c.Wout, m0, 0, m0 / HWo, 0, wave, lr, lh, 0, 0,
                                                         0, c.ws_rowscale);
    return;
  }
  // LDS-staged epilogue (16-B stores): per 32-row slab i, this wave's 32 x 64 tile of acc * rowscale
  typedef StagedEpilogue<64> Epi;
  __syncthreads();  // every wave is done reading the O rows
  float* st = sp + wave * 32 * Epi::EP;
  Epi epi(c, M, HWo, m0 / HWo, (HWo % 64) == 0, wave * 64, lr + 32 * lh);
  float cs[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) cs[j] = c.ws_rowscale[wave * 64 + j * 32 + lr];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) st[acc_row(r, lh) * Epi::EP + j * 32 + lr] = acc[i][j][r] * cs[j];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are visible to its reads
    __builtin_amdgcn_wave_barrier();
    epi.rows(st, m0 + 32 * i);
    __builtin_amdgcn_wave_barrier();
  }
  if (c.gn_part) epi.emit(m0);
}

// Pre-split operands (AttnArgs::pq / pk / pv, written by the qkv projection's epilogue): no split on the
// VALU. q is staged once in LDS; k and v^T fragments are 16-B loads per lane from L2 riding a register
// ring RD slices ahead of their use. (k / v^T as contiguous 1-KiB fragment images cut the block from
// 125.6 to 110.3 us but measured 1.6 % slower end to end -- every other kernel of the forward then ran at
// a lower clock -- so the [token][d] / [d][token] planes stay.) 64 query rows per block (75 KB of LDS for
// the S / P rows: two blocks per CU). Same MFMA sequence as the unfused GEMMs.
template <int DH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) attn_presplit_kernel(AttnArgs a) {
  static_assert(DH == 64 || DH == 256, "head dims 64 / 256");
  constexpr int QT = 64, NS = DH / 16, RD = 6;
  __shared__ __attribute__((aligned(16))) float sp[QT * kSP];
  static_assert(QT * (2 * DH + 8) * 2 <= QT * kSP * 4, "the staged q tile fits the S rows");
  AT_RSTAMP(6);
  AT_STAMP(0);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int nq = kAL / QT;
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int qt = bid % nq, bh = bid / nq;
  const size_t plane = (size_t)kAL * DH;
  const _Float16* Q = a.pq + (size_t)bh * 2 * plane + (size_t)(qt * QT) * DH;
  const _Float16* K = a.pk + (size_t)bh * 2 * plane;
  const _Float16* V = a.pv + (size_t)bh * 2 * plane;

  // ---------------------------------------------------------------- 1. S: wave w = 64 rows x keys 64 w ..
  // The block's 64 q rows are read by all four waves: staged once in LDS (over the S / P rows, free until
  // S is written), rows of [16-deep slice][piece][lane group][8] fp16 with a 16-B pad (an odd number of
  // 16-B slots: conflict-free fragment reads). k rows (64 per wave, no reuse) ride a register ring RD
  // slices ahead. Same operands and MFMA sequence as before: S is unchanged bit for bit.
  constexpr int QP = 2 * DH + 8;
  _Float16* Qs = reinterpret_cast<_Float16*>(sp);
  f16x8 rb[RD][2][2];   // [slot][tile][piece]
  auto load_k = [&](int s, int slot) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        rb[slot][i][q] =
            *reinterpret_cast<const f16x8*>(K + q * plane + (size_t)(wave * 64 + i * 32 + lr) * DH + 16 * s + 8 * lh);
  };
#pragma unroll
  for (int s = 0; s < RD; ++s) load_k(min(s, NS - 1), s);
  {
    constexpr int QCH = 64 * DH / 8;  // 16-B chunks of one piece plane of the tile
    f16x8 qv[2 * QCH / 256];
#pragma unroll
    for (int u = 0; u < 2 * QCH / 256; ++u) {
      const int c = t + 256 * u, piece = c / QCH, rem = c - piece * QCH;
      const int row = rem / (DH / 8), d8 = rem - row * (DH / 8);
      qv[u] = *reinterpret_cast<const f16x8*>(Q + piece * plane + (size_t)row * DH + 8 * d8);
    }
#pragma unroll
    for (int u = 0; u < 2 * QCH / 256; ++u) {
      const int c = t + 256 * u, piece = c / QCH, rem = c - piece * QCH;
      const int row = rem / (DH / 8), d8 = rem - row * (DH / 8);
      *reinterpret_cast<f16x8*>(Qs + row * QP + (d8 >> 1) * 32 + piece * 16 + (d8 & 1) * 8) = qv[u];
    }
  }
  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int slot = s % RD;
    f16x8 av[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q) av[i][q] = *reinterpret_cast<const f16x8*>(Qs + (i * 32 + lr) * QP + s * 32 + q * 16 + lh * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) Split<2>::mma(av[i], rb[slot][j], acc[i][j]);
    load_k(min(s + RD, NS - 1), slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();  // every wave is done reading the q tile before S overwrites it
  {
    const float unscale = ldexpf(1.f, -(a.ea + a.eb));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sp[(i * 32 + acc_row(r, lh)) * kSP + wave * 64 + j * 32 + lr] = acc[i][j][r] * unscale;
  }
  __syncthreads();
  AT_STAMP(1);

  // ---------------------------------------------------------------- 2. softmax rows -> P pieces in place
  const float pp = ldexpf(1.f, a.ep);
  // four rows at a time: independent max / sum shuffle chains overlap (per row the same operations in the
  // same order as softmax_rows, so P stays bit-identical)
  constexpr int RI = QT / 4;
  for (int row0 = wave * (QT / 4); row0 < (wave + 1) * (QT / 4); row0 += RI) {
    f4 v[RI];
    float mx[RI], sum[RI];
#pragma unroll
    for (int ri = 0; ri < RI; ++ri) {
      v[ri] = *reinterpret_cast<const f4*>(sp + (row0 + ri) * kSP + 4 * lane);
      mx[ri] = fmaxf(fmaxf(v[ri][0], v[ri][1]), fmaxf(v[ri][2], v[ri][3]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) mx[ri] = fmaxf(mx[ri], __shfl_xor(mx[ri], o));
#pragma unroll
    for (int ri = 0; ri < RI; ++ri) {
      sum[ri] = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[ri][e] = expf(v[ri][e] - mx[ri]);
        sum[ri] += v[ri][e];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int ri = 0; ri < RI; ++ri) sum[ri] += __shfl_xor(sum[ri], o);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // every row's S values are in registers before P overwrites the rows
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ri = 0; ri < RI; ++ri) {
      const float inv = 1.0f / sum[ri];
      p_store4(reinterpret_cast<_Float16*>(sp + (row0 + ri) * kSP), lane, v[ri] * inv, pp);
    }
  }
  __syncthreads();
  AT_STAMP(2);

  // ---------------------------------------------------------------- 3. O = P v
  constexpr int TM = DH == 256 ? 2 : 1, TN = DH == 256 ? 2 : 1, NK = kAL / 16;
  const int orow0 = DH == 256 ? 0 : (wave >> 1) * 32;
  const int ocol0 = DH == 256 ? wave * 64 : (wave & 1) * 32;
  const _Float16* P = reinterpret_cast<const _Float16*>(sp);
  constexpr int PPITCH = 2 * kSP;
  f16x8 rv[RD][TN][2];
  auto load_v = [&](int s, int slot) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        rv[slot][j][q] =
            *reinterpret_cast<const f16x8*>(V + q * plane + (size_t)(ocol0 + j * 32 + lr) * kAL + 16 * s + 8 * lh);
  };
  f16v oacc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][j][r] = 0.f;
#pragma unroll
  for (int s = 0; s < RD; ++s) load_v(s, s);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    const int slot = s % RD;
    f16x8 av[TM][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        av[i][q] = *reinterpret_cast<const f16x8*>(P + (orow0 + i * 32 + lr) * PPITCH + (s >> 1) * kAP + (s & 1) * 32 +
                                                   lh * 16 + q * 8);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) Split<2>::mma(av[i], rv[slot][j], oacc[i][j]);
    load_v(min(s + RD, NK - 1), slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  AT_STAMP(3);
  const float ounscale = ldexpf(1.f, -(a.ep + a.ev));
  const int h = bh % a.heads, b = bh / a.heads;
  if constexpr (DH == 256) {
    if (a.fuse_proj) {  // 4. y = x + proj(O): the MODE 3 1x1 conv on this block's 64 O rows
      attn_proj(a.proj, oacc, ounscale, sp, b * kAL + qt * QT, wave, lr, lh, a.proj_staged != 0);
      AT_STAMP(8);
      AT_RSTAMP(7);
      return;
    }
  }
  float* out = a.out + ((size_t)b * kAL + qt * QT) * a.ldo + h * DH;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(size_t)(orow0 + i * 32 + acc_row(r, lh)) * a.ldo + ocol0 + j * 32 + lr] = oacc[i][j][r] * ounscale;
}

// Flash attention on the pre-split operand planes (AttnArgs::pq / pk / pv) for the shapes the kernels above
// do not take: ADM's 32^2 (L = 1024) and 8^2 (L = 64) blocks with heads of 64 (models/adm/unet.py:347-408)
// and DiT's 16 heads of 72 over T = 256 tokens (timm Attention, oracle/dit.py:44-51). The L x L score matrix
// never leaves the CU: per 64-key block, S = (q)(k)^T, an online softmax (running row maximum and sum,
// exp2 with the log2(e) factor folded into the exact 2^-(ea + eb) unscale) and O += P v.
//
// Layout on the matrix cores (v_mfma_f32_32x32x16_f16, fp16x2 products a1 b0 + a0 b1 + a0 b0 as everywhere):
//  * S^T = K Q^T: the key on the MFMA row, the query on the lane (lane & 31), so a lane holds 32 scores of
//    ONE query row: the row maximum / sum are register reductions plus one cross-half shuffle, and the
//    running-softmax correction of the output is lane-local.
//  * O^T = V^T P^T: the S^T accumulators, exponentiated and split, are directly the B operand (P^T, query on
//    the lane) -- with the k index of a 16-key step permuted as the accumulator rows lie, (e & 3) + 8 (e >> 2)
//    + 4 lh for element e of lane half lh, which the V^T tile's LDS image reproduces (two 8-B stores per
//    16-B load), so a consistent relabelling of the contraction index and no register shuffles.
// Q stays in registers (its DHP / 16 slices, both pieces); K and V^T blocks are staged through LDS (double
// buffered, one barrier per 64 keys, loads for the next block in flight during this one's MFMAs), with row
// pitches of an odd number of 16-B slots times 4 dwords so the 32-row fragment reads are conflict free.
// Head dims below DHP (72 in an 80-deep contraction) are zero-padded in registers / LDS, never in memory.
//  * Head dims that are not a multiple of 32 (72, 80) take their last Dh % 32 rows of O^T on
//    v_mfma_f32_16x16x32_f16 (a 16-row tail, 2 x 16 queries per 32-key chunk) instead of a third 32-row tile:
//    DiT's 72 wide heads had wasted a quarter of their P V products on rows 72 .. 95. The 16x16x32 B operand
//    wants 16 queries x 4 k-groups of 8 where the S^T accumulators give 32 queries x 2 k-groups per 16-key
//    step: v_permlane32_swap + v_permlane16_swap of the two steps' pieces produce both 16-query halves
//    exactly (no LDS round trip); the V^T rows are read at the same permuted key offsets.
// O^T rows >= Dh read clamped V rows and are not stored. Each wave owns 32 queries; NW waves per block.
// Not bit-identical to the unfused path (exp2 and the online rescale round differently): within a few ulp of
// the unfused softmax (tests/test_gpu_r3.py test_flash_attention_vs_unfused).
template <int Dh, int NW>
__global__ void __launch_bounds__(NW * 64) attn_flash_kernel(AttnArgs a) {
  constexpr int DHP = (Dh + 15) / 16 * 16;   // contraction depth of S (16-deep slices)
  constexpr int KB = 64;                     // keys per block
  constexpr int NS = DHP / 16;               // 16-deep slices of the S contraction
  constexpr int KP = DHP == 80 ? 168 : DHP == 48 ? 104 : DHP == 32 ? 72 : 136;  // fp16 pitch of a K row:
                                             // 2 DHP + pad, 4 x an odd number of dwords (conflict-free reads)
  constexpr int VP = 136;                    // fp16 pitch of a V^T row (64 keys x 2 pieces + pad: 68 dwords)
  constexpr bool TAIL = Dh % 32 != 0;        // last Dh % 32 rows of O^T on a 16x16x32 tail
  static_assert(!TAIL || Dh % 32 <= 16, "16-row tail");
  constexpr int NDT = TAIL ? Dh / 32 : (DHP + 31) / 32;   // 32-row d tiles of O^T
  constexpr int KBUF = KB * KP, VBUF = DHP * VP, BUF = KBUF + VBUF;
  constexpr int NT = NW * 64;
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * BUF];
  static_assert(NW * 32 * (DHP + 1) * 4 <= 2 * BUF * 2, "output staging fits the operand buffers");

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int lr = lane & 31, lh = lane >> 5;
  const int L = a.L;
  const int nqb = L / (32 * NW);
  const int bid = xcd_remap_p(blockIdx.x, gridDim.x);
  const int qb = bid % nqb, bh = bid / nqb;
  const size_t plane = (size_t)L * Dh;
  const _Float16* Q = a.pq + (size_t)bh * 2 * plane;
  const _Float16* K = a.pk + (size_t)bh * 2 * plane;
  const _Float16* V = a.pv + (size_t)bh * 2 * plane;
  const int q0 = qb * 32 * NW + wave * 32;

  // Q^T fragments (B operand): query q0 + lr, d = 16 s + 8 lh .. + 7 of both pieces; zero beyond Dh
  f16x8 qf[NS][2];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int d = 16 * s + 8 * lh;
      if (d < Dh)
        qf[s][p] = *reinterpret_cast<const f16x8*>(Q + p * plane + (size_t)(q0 + lr) * Dh + d);
      else
        for (int e = 0; e < 8; ++e) qf[s][p][e] = (_Float16)0.f;
    }

  // loaders: K chunks (row, piece, 8 d) and V^T chunks (d row, piece, 8 keys), 16 B each, into registers
  constexpr int dh8 = Dh / 8;
  constexpr int nkc = 2 * KB * dh8, nvc = 2 * Dh * (KB / 8);
  constexpr int CK = (2 * KB * (DHP / 8) + NT - 1) / NT, CV = (2 * DHP * (KB / 8) + NT - 1) / NT;
  f4 rk[CK], rv[CV];
  auto load_blk = [&](int kb) {
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int i = min(t + NT * u, nkc - 1);
      const int p = i / (KB * dh8), r = i - p * (KB * dh8);   // r = row * dh8 + c8: contiguous in the plane
      rk[u] = *reinterpret_cast<const f4*>(K + p * plane + (size_t)kb * KB * Dh + 8 * r);
    }
#pragma unroll
    for (int u = 0; u < CV; ++u) {
      const int i = min(t + NT * u, nvc - 1);
      const int c8 = i & 7, pd = i >> 3, p = pd / Dh, d = pd - p * Dh;
      rv[u] = *reinterpret_cast<const f4*>(V + p * plane + (size_t)d * L + kb * KB + 8 * c8);
    }
  };
  auto store_blk = [&](int buf) {
    _Float16* kb_ = lds + buf * BUF;
    _Float16* vb_ = kb_ + KBUF;
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int i = t + NT * u;
      if (i >= nkc) continue;
      const int p = i / (KB * dh8), r = i - p * (KB * dh8);
      const int row = r / dh8, c8 = r - row * dh8;
      *reinterpret_cast<f4*>(kb_ + row * KP + (c8 >> 1) * 32 + p * 16 + (c8 & 1) * 8) = rk[u];
    }
#pragma unroll
    for (int u = 0; u < CV; ++u) {
      const int i = t + NT * u;
      if (i >= nvc) continue;
      const int c8 = i & 7, pd = i >> 3, p = pd / Dh, d = pd - p * Dh;
      // keys 8 c8 .. + 3 -> positions 4 (c8 & 1) .. + 3, keys + 4 .. + 7 -> 8 + 4 (c8 & 1) .. of the 16-key group
      _Float16* dst = vb_ + d * VP + (c8 >> 1) * 32 + p * 16 + (c8 & 1) * 4;
      const f4 v = rv[u];
      *reinterpret_cast<float2*>(dst) = make_float2(v[0], v[1]);
      *reinterpret_cast<float2*>(dst + 8) = make_float2(v[2], v[3]);
    }
  };
  // zero the K rows' head-dim padding (d in [Dh, DHP)) of both buffers: never written by the loader
  constexpr int per = 2 * (DHP / 8 - dh8 > 0 ? DHP / 8 - dh8 : 1);  // no padding (Dh % 32 == 0): no iterations
  for (int i = t; i < 2 * KB * 2 * (DHP / 8 - dh8); i += NT) {
    const int rowb = i / per, rem = i - rowb * per;
    const int buf = rowb / KB, row = rowb - buf * KB, p = rem & 1, c8 = dh8 + (rem >> 1);
    *reinterpret_cast<f4*>(lds + buf * BUF + row * KP + (c8 >> 1) * 32 + p * 16 + (c8 & 1) * 8) = f4{0.f, 0.f, 0.f, 0.f};
  }

  const float sl2 = ldexpf(1.f, -(a.ea + a.eb)) * 1.4426950408889634f;   // exact unscale x log2(e)
  f16v oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  // tail accumulators: [query half qh] lane (j = lane & 15, g = lane >> 4) holds O^T rows 32 NDT + 4 g .. + 3 of
  // query 16 qh + j
  f4 otail[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
  const int tq = lane & 15, tg = lane >> 4;
  float m_run = -INFINITY, l_run = 0.f;

  const int nkb = L / KB;
  load_blk(0);
  store_blk(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) load_blk(kb + 1);
    const _Float16* Kb = lds + (kb & 1) * BUF;
    const _Float16* Vb = Kb + KBUF;
    // S^T [64 keys x 32 queries] = K Q^T
    f16v sacc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[j][r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f16x8 ka[2];
#pragma unroll
        for (int p = 0; p < 2; ++p)
          ka[p] = *reinterpret_cast<const f16x8*>(Kb + (j * 32 + lr) * KP + s * 32 + p * 16 + lh * 8);
        Split<2>::mma(ka, qf[s], sacc[j]);
      }
    }
    // online softmax of this query row (lane) over the block's 64 keys (32 here, 32 in the other half-wave):
    // the running maximum m_run in the scaled (log2) domain, the max taken over the raw scores and scaled once
    // (sl2 > 0), each probability exp2(s sl2 - m) as one FMA and one exp2; the P scale 2^ep folded into the
    // exponent (l_run accumulates 2^ep p, undone at the end)
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[j][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx * sl2);
    const float corr = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    l_run *= corr;
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][r] *= corr;
    if constexpr (TAIL) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        const float c = __shfl(corr, 16 * qh + tq);
#pragma unroll
        for (int r = 0; r < 4; ++r) otail[qh][r] *= c;
      }
    }
    const float mb = (float)a.ep - m_new;
    // P^T pieces: k-step ks = 16 keys = accumulator registers 8 (ks & 1) .. + 7 of tile ks >> 1
    f16x8 pb[4][2];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[ks >> 1][8 * (ks & 1) + e], sl2, mb));
        l_run += x;
        const _Float16 h0 = (_Float16)x;
        pb[ks][0][e] = h0;
        pb[ks][1][e] = (_Float16)(x - (float)h0);
      }
    // O^T [d x 32 queries] += V^T P^T
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int drow = min(dt * 32 + lr, Dh - 1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        f16x8 va[2];
#pragma unroll
        for (int p = 0; p < 2; ++p)
          va[p] = *reinterpret_cast<const f16x8*>(Vb + drow * VP + ks * 32 + p * 16 + lh * 8);
        Split<2>::mma(va, pb[ks], oacc[dt]);
      }
    }
    if constexpr (TAIL) {
      // rows 32 NDT .. + 15 (clamped to Dh - 1: not stored), 32-key chunk c = steps 2c, 2c + 1
      const int drow = min(NDT * 32 + tq, Dh - 1);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        f16x8 va[2], pq[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          va[p] = *reinterpret_cast<const f16x8*>(Vb + drow * VP + (2 * c + (tg >> 1)) * 32 + p * 16 + (tg & 1) * 8);
          // lane (j, g) of half qh <- step 2c + (g >> 1), lane 16 qh + j + 32 (g & 1)
          const u4 x = __builtin_bit_cast(u4, pb[2 * c][p]), y = __builtin_bit_cast(u4, pb[2 * c + 1][p]);
          u4 h0, h1;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const auto s32 = __builtin_amdgcn_permlane32_swap(x[w], y[w], false, false);
            const auto s16 = __builtin_amdgcn_permlane16_swap(s32[0], s32[1], false, false);
            h0[w] = s16[0];
            h1[w] = s16[1];
          }
          pq[0][p] = __builtin_bit_cast(f16x8, h0);
          pq[1][p] = __builtin_bit_cast(f16x8, h1);
        }
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          otail[qh] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[1], pq[qh][0], otail[qh], 0, 0, 0);
          otail[qh] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[0], pq[qh][1], otail[qh], 0, 0, 0);
          otail[qh] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[0], pq[qh][0], otail[qh], 0, 0, 0);
        }
      }
    }
    if (kb + 1 < nkb) store_blk((kb + 1) & 1);
    __syncthreads();
  }

  // O = O^T / l (x 2^-(ep + ev)), staged through LDS as [32 queries][Dh + 1] fp32 rows per wave, stored as rows
  const float l_tot = l_run + __shfl_xor(l_run, 32);   // 2^ep x the softmax denominator
  const float scale = ldexpf(1.f, -a.ev) / l_tot;
  constexpr int OP = Dh + 1;
  float* st = reinterpret_cast<float*>(lds) + wave * 32 * OP;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = dt * 32 + acc_row(r, lh);
      if (d < Dh) st[lr * OP + d] = oacc[dt][r] * scale;
    }
  if constexpr (TAIL) {
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const float sq = __shfl(scale, 16 * qh + tq);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = NDT * 32 + 4 * tg + r;
        if (d < Dh) st[(16 * qh + tq) * OP + d] = otail[qh][r] * sq;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  const int h = bh % a.heads, b = bh / a.heads;
  if (a.o_split) {  // the output projection's pre-split A image: 8 columns (one k-group) per item, 2 x 16 B
    const float ps = ldexpf(1.f, a.o_split_ea);
    constexpr int ng = Dh / 8;
    bool bad = false;
    for (int i = lane; i < 32 * ng; i += 64) {
      const int q = i / ng, g8 = i - q * ng;
      const int c = h * Dh + 8 * g8;
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = st[q * OP + 8 * g8 + e] * ps;
        const _Float16 h0 = (_Float16)x;
        hi[e] = h0;
        lo[e] = (_Float16)(x - (float)h0);
        bad |= fabsf(x) > 65504.f;
      }
      _Float16* dst = a.o_split + ((size_t)b * L + q0 + q) * 2 * a.o_ld + (c >> 5) * 64 + ((c & 31) >> 3) * 8;
      *reinterpret_cast<f16x8*>(dst) = hi;
      *reinterpret_cast<f16x8*>(dst + 32) = lo;
    }
    if (bad && a.range_flag) *a.range_flag = 1;
    return;
  }
  float* out = a.out + ((size_t)b * L + q0) * a.ldo + h * Dh;
  for (int i = lane; i < 32 * Dh; i += 64) {
    const int q = i / Dh, d = i - q * Dh;
    out[(size_t)q * a.ldo + d] = st[q * OP + d];
  }
}

}  // namespace

bool attn_flash_ok(int L, int Dh) {
  return L >= 64 && L % 64 == 0 && (Dh == 32 || Dh == 64 || Dh == 72 || Dh == 80);
}

template <int DH>
static void launch_flash(const AttnArgs& a, unsigned blocks, bool nw8, hipStream_t st) {
  if (nw8) hipLaunchKernelGGL((attn_flash_kernel<DH, 8>), dim3(blocks), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((attn_flash_kernel<DH, 2>), dim3(blocks), dim3(128), 0, st, a);
}

int attn_flash(const AttnArgs& a, hipStream_t st) {
  DM_REQUIRE(attn_flash_ok(a.L, a.Dh), "flash attention: L % 64 == 0 and head dims 32, 64, 72 or 80");
  DM_REQUIRE(a.pq && a.pk && a.pv && (a.out || a.o_split) && a.B > 0 && a.heads > 0 && a.ldo % 4 == 0,
             "flash attention: needs the pre-split operand planes and an output");
  DM_REQUIRE(!a.o_split || (a.o_ld % 32 == 0 && a.o_ld >= a.heads * a.Dh &&
                            (reinterpret_cast<uintptr_t>(a.o_split) & 15) == 0),
             "flash attention: the pre-split output image needs 32-column groups, 16-byte aligned");
  DM_REQUIRE(((reinterpret_cast<uintptr_t>(a.pq) | reinterpret_cast<uintptr_t>(a.pk) |
               reinterpret_cast<uintptr_t>(a.pv)) & 15) == 0, "flash attention: 16-byte aligned planes");
  const bool nw8 = a.L % 256 == 0;
  const unsigned blocks = (unsigned)((long)a.B * a.heads * (a.L / (32 * (nw8 ? 8 : 2))));
  switch (a.Dh) {
    case 32: launch_flash<32>(a, blocks, nw8, st); break;
    case 64: launch_flash<64>(a, blocks, nw8, st); break;
    case 72: launch_flash<72>(a, blocks, nw8, st); break;
    default: launch_flash<80>(a, blocks, nw8, st); break;
  }
  DM_LAUNCH_CHECK();
  return DM_OK;
}

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_attn_stamps(void* host, int nblocks) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), (size_t)nblocks * 10 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

bool attn_fused_ok(int L, int Dh) { return L == kAL && (Dh == 64 || Dh == 256); }

int attn_fused(const AttnArgs& args, hipStream_t st) {
  if (!attn_fused_ok(args.L, args.Dh)) return attn_flash(args, st);
  AttnArgs a = args;
  a.proj_staged = a.fuse_proj && staged_epilogue_ok(a.proj) ? 1 : 0;
  DM_REQUIRE(attn_fused_ok(a.L, a.Dh), "fused attention: L must be 256 and the head dim 64 or 256");
  DM_REQUIRE((a.qkv || a.pq) && a.out && a.B > 0 && a.heads > 0 && a.ld % 4 == 0 && a.ldo % 4 == 0 &&
             (a.q0 + 0) % 4 == 0 && a.k0 % 4 == 0 && a.v0 % 4 == 0 && a.hs % 4 == 0,
             "fused attention: operands must be float4-aligned rows");
  if (a.pq) {
    DM_REQUIRE(a.pk && a.pv, "fused attention: all three operand planes");
    const dim3 grid(a.B * a.heads * (kAL / 64));
    if (a.Dh == 256)
      hipLaunchKernelGGL((attn_presplit_kernel<256>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((attn_presplit_kernel<64>), grid, dim3(256), 0, st, a);
    DM_LAUNCH_CHECK();
    return DM_OK;
  }
  if (a.Dh == 256)
    hipLaunchKernelGGL((attn_fused_kernel<256, 32>), dim3(a.B * a.heads * (kAL / 32)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((attn_fused_kernel<64, 64>), dim3(a.B * a.heads * (kAL / 64)), dim3(256), 0, st, a);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
