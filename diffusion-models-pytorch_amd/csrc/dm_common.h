// Internal helpers shared by the dm_hip kernels and the C-ABI layer.
// Not part of the public interface (see include/dm_hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "dm_hip.h"

namespace dm {

// Thread-local last-error string, surfaced through dm_last_error().
void set_error(const std::string& msg);
const char* last_error();

// Return codes of the C ABI (DM_OK, DM_ERR_*) come from the public header.

#define DM_CHECK_HIP(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::dm::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));         \
      return DM_ERR_HIP;                                                    \
    }                                                                             \
  } while (0)

#define DM_REQUIRE(cond, msg)                                                     \
  do {                                                                            \
    if (!(cond)) {                                                                \
      ::dm::set_error(std::string("argument check failed: ") + (msg));            \
      return DM_ERR_ARG;                                                    \
    }                                                                             \
  } while (0)

#define DM_LAUNCH_CHECK()                                                         \
  do {                                                                            \
    hipError_t _e = hipGetLastError();                                            \
    if (_e != hipSuccess) {                                                       \
      ::dm::set_error(std::string("kernel launch: ") + hipGetErrorString(_e));    \
      return DM_ERR_HIP;                                                    \
    }                                                                             \
  } while (0)

// NHWC activation view. Element (b, y, x, c) lives at
//   p[((b * H + y) * W + x) * pitch + c]
// `pitch` >= C lets a tensor be a channel slice of a wider buffer (zero-copy
// skip concatenation: the producer of a skip writes straight into the
// consumer's concat buffer).
struct View {
  float* p;
  int B, H, W, C;
  int pitch;
};

__host__ __device__ inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

__device__ __forceinline__ float silu_f(float v) {
  // torch CPU: x / (1 + exp(-x)), IEEE division, accurate expf.
  return v / (1.0f + expf(-v));
}

// SiLU for operand prologues that sit next to MFMA work (conv halo-patch load):
// hardware exp2 and reciprocal (v_exp_f32 / v_rcp_f32, ~1 ulp each) instead of
// the libm expf + IEEE division of silu_f — ~6 VALU ops instead of ~30, a
// relative difference of a few 1e-7 (well inside the 1e-4 parity bound).
__device__ __forceinline__ float silu_fast(float v) {
  const float e = __builtin_amdgcn_exp2f(-v * 1.4426950408889634f);
  return v * __builtin_amdgcn_rcpf(1.0f + e);
}

__device__ __forceinline__ float gelu_tanh_f(float v) {
  // torch GELU(approximate='tanh'): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float inner = k0 * (v + k1 * v * v * v);
  return 0.5f * v * (1.0f + tanhf(inner));
}

}  // namespace dm
