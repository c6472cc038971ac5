// Exact splits of fp32 operands into 16-bit pieces for the matrix cores, shared by the split
// convolution (conv_patch3.hip) and the split GEMM (gemm.hip). Numerics are described in
// conv_patch3.hip: Split<3> = three bf16 pieces, six products (a2b0 + a1b1 + a0b2 + a1b0 + a0b1 +
// a0b0); Split<2> = two fp16 pieces, three products (a1b0 + a0b1 + a0b0), the caller keeping both
// operands in fp16's normal range by power-of-two scales.
#pragma once
#include "dm_common.h"
#include "mfma_tile.h"

namespace dm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

// Piece format of one split variant. NP = 3: three bf16 pieces, six products; NP = 2: two fp16
// pieces, three products, operands pre-scaled by powers of two (conv_patch3.hip, gemm.hip).
template <int NP>
struct Split;

template <>
struct Split<3> {
  typedef __bf16 elem;
  typedef bf16x8 vec;
  static constexpr int kRow = 48;    // elements per slice row: 2 lane groups x 3 pieces x 8
  static constexpr int kPitch = 56;  // LDS row pitch (112 B = 7 x 16 B)
  // exact three-way split of 8 fp32 values
  __device__ static __forceinline__ void split(const f4 lo4, const f4 hi4, vec (&p)[3], bool& bad) {
    const float x[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const __bf16 b0 = (__bf16)x[e];
      const float r1 = x[e] - (float)b0;
      const __bf16 b1 = (__bf16)r1;
      const float r2 = r1 - (float)b1;
      p[0][e] = b0;
      p[1][e] = b1;
      p[2][e] = (__bf16)r2;
    }
  }
  __device__ static __forceinline__ void mma(const vec (&a)[3], const vec (&b)[3], f16v& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  }
};

template <>
struct Split<2> {
  typedef _Float16 elem;
  typedef f16x8 vec;
  static constexpr int kRow = 32;    // 2 lane groups x 2 pieces x 8
  static constexpr int kPitch = 40;  // 80 B = 5 x 16 B
  // x = h0 + h1 with h0 = fp16(x), h1 = fp16(x - h0) (the subtraction is exact); |x| > 65504 has no
  // fp16 image and raises `bad` (the forward's range flag: the caller re-runs in bf16x3)
  __device__ static __forceinline__ void split(const f4 lo4, const f4 hi4, vec (&p)[2], bool& bad) {
    const float x[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const _Float16 h0 = (_Float16)x[e];
      p[0][e] = h0;
      p[1][e] = (_Float16)(x[e] - (float)h0);
      m = fmaxf(m, fabsf(x[e]));
    }
    bad |= m > 65504.f;
  }
  // four values (one float4) -> hi / lo fp16 pieces
  __device__ static __forceinline__ void split4(const f4 x, f16x4& h, f16x4& l, bool& bad) {
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const _Float16 h0 = (_Float16)x[e];
      h[e] = h0;
      l[e] = (_Float16)(x[e] - (float)h0);
      m = fmaxf(m, fabsf(x[e]));
    }
    bad |= m > 65504.f;
  }
  __device__ static __forceinline__ void mma(const vec (&a)[2], const vec (&b)[2], f16v& acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], acc, 0, 0, 0);
  }
};

}  // namespace dm
