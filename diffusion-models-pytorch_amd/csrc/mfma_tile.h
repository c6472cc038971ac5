// fp32 MFMA block tile shared by the implicit-GEMM convolution and the
// batched GEMM kernels.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact fp32 fma chain (no TF32 /
// xf32 on gfx950), so every contraction in this library keeps the fp32
// arithmetic of the reference's torch CPU path, only the summation order
// differs.
//
// Tile geometry: a block computes BM x BN outputs with (BM/WM) x (BN/WN)
// wave64s; every wave owns a WM x WN sub-tile = TM x TN MFMA 32x32 tiles.
// K is staged through LDS in BK = 32 slices, double buffered, one barrier per
// slice. Both operands are stored K-contiguous in LDS ([row][k], pitch 36
// floats): with that pitch the ds_read_b128 lane groups of a 32-row fragment
// read are bank-conflict free.
//
// K permutation: one ds_read_b128 gives each lane 4 consecutive k values; the
// four MFMAs of an 8-wide k chunk consume component s of that vector, so MFMA
// step s of lane half h multiplies k = kc + 4h + s for BOTH operands (a
// consistent relabelling of the reduction index, exact in any order).
#pragma once
#include "dm_common.h"

namespace dm {

typedef float f4 __attribute__((ext_vector_type(4)));

// Zero padding by ADDRESS instead of by select: an out-of-range operand row
// (conv zero padding, K tail) loads from this all-zero buffer, so the loaded
// registers go to LDS unmodified. A select on loaded data lets the compiler
// hoist it next to the load and drain vmcnt(0) in front of the MFMAs of the
// current slice (observed in the ISA); an address select costs nothing there.
// Rows beyond M / columns beyond N read clamped, valid data instead: their
// results are never stored. One copy per translation unit (static), never written.
constexpr int kZeroPageFloats = 16384;

// GroupNorm statistics from an MFMA epilogue. A wave owns 64 consecutive output rows (one
// 64-pixel chunk of one image when HW % 64 == 0) and, per 32-column group j, lane (lr, lh) holds
// column n = ... + lr summed over its rows. Combine the two half-waves (lh), then the cpg lanes of
// each GroupNorm group, and let the group's first lane store {sum, sumsq}. All 64 lanes must call.
__device__ __forceinline__ void gn_emit_group(double s, double q, int lr, int lh, int cpg, bool store,
                                              double2* dst) {
  s += __shfl_xor(s, 32);
  q += __shfl_xor(q, 32);
  for (int o = 1; o < cpg; o <<= 1) {
    s += __shfl_xor(s, o);
    q += __shfl_xor(q, o);
  }
  if (store && lh == 0 && (lr % cpg) == 0) *dst = make_double2(s, q);
}
static __device__ __attribute__((aligned(16))) float kZeroPage[kZeroPageFloats];

// XCD-aware bijective block remap: consecutive logical tiles land on one XCD (shared L2).
__device__ __forceinline__ int xcd_remap_p(int bid, int nblk) {
  const int q = nblk >> 3, r = nblk & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kBK = 32;
constexpr int kLDK = kBK + 4;

template <int BM, int BN, int WM, int WN>
struct TileCfg {
  static constexpr int NWM = BM / WM;
  static constexpr int NWN = BN / WN;
  static constexpr int NT = NWM * NWN * 64;
  static constexpr int TM = WM / 32;
  static constexpr int TN = WN / 32;
  static constexpr int ROWS_PER_PASS = NT / (kBK / 4);  // rows covered by one float4 pass
  static constexpr int A_ITERS = BM / ROWS_PER_PASS;
  static constexpr int B_ITERS = BN / ROWS_PER_PASS;
  static constexpr int A_ELEMS = BM * kLDK;
  static constexpr int B_ELEMS = BN * kLDK;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;
  static constexpr int LDS_FLOATS = 2 * STAGE;
  static_assert(NT == 256, "kernels are launched with 256 threads");
  static_assert(BM % ROWS_PER_PASS == 0 && BN % ROWS_PER_PASS == 0, "tile/threads mismatch");
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be multiple of 32");
};

template <int TM, int TN>
__device__ __forceinline__ void mfma_slice(const float* __restrict__ As, const float* __restrict__ Bs,
                                           int a_row0, int b_row0, int lane, f16v (&acc)[TM][TN]) {
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int kc = 0; kc < kBK; kc += 8) {
    f4 a[TM], b[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      a[i] = *reinterpret_cast<const f4*>(As + (a_row0 + i * 32 + lr) * kLDK + kc + 4 * lh);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      b[j] = *reinterpret_cast<const f4*>(Bs + (b_row0 + j * 32 + lr) * kLDK + kc + 4 * lh);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
        }
      }
    }
  }
}

// Row (within the wave's 32x32 tile) of accumulator register r for lane half lh.
__device__ __forceinline__ int acc_row(int r, int lh) { return (r & 3) + 8 * (r >> 2) + 4 * lh; }


}  // namespace dm
