// Bandwidth-bound / small kernels of the denoising step:
//   * timestep sinusoidal embedding   models/modules.py:45-57 (UNet, [sin, cos])
//                                     models/adm/nn.py:103-121 (ADM, [cos, sin])
//   * row softmax (attention)         models/modules.py:96
//   * small-channel direct 3x3 convs  models/unet.py:72 (first_conv, Cin=1/3, NCHW in)
//                                     models/unet.py:118 (last_conv, Cout=1/3/6, NCHW out)
//   * NCHW <-> NHWC conversion
//   * the per-step sampler update     diffusions/ddpm.py:174-252, diffusions/ddim.py:57-77,
//                                     CFG combine ddim.py:185 / ddpm.py:343-345
// The sampler update is written op-for-op in the reference's rounding order
// and compiled with -ffp-contract=off, so with identical inputs it is
// bit-identical to the torch CPU path (coefficients come from the host,
// computed with the same torch 0-dim ops as the reference).
#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"

namespace dm {

namespace {

__global__ void timestep_embed_kernel(const int64_t* __restrict__ t, int B, int dim, int kind,
                                      const float* __restrict__ freqs, float* __restrict__ out) {
  const int half = dim / 2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * half) return;
  const int b = idx / half, i = idx - (idx / half) * half;
  const float tv = (float)t[b];
  float f;
  if (freqs) {
    // host-provided table (the reference's torch CPU expression, bit-identical on that host)
    f = freqs[i];
  } else if (kind == 0) {
    // UNet: exp(arange(half) * -(ln(1e4) / (half - 1)))
    const float c = (float)(-(log(10000.0) / (double)(half - 1)));
    f = expf((float)i * c);
  } else {
    // ADM: exp(-ln(1e4) * arange(half, f32) / half)
    const float c = (float)(-log(10000.0));
    f = expf(((float)i * c) / (float)half);
  }
  const float arg = tv * f;
  float s = sinf(arg), co = cosf(arg);
  if (kind == 0) {
    out[(size_t)b * dim + i] = s;
    out[(size_t)b * dim + half + i] = co;
  } else {
    out[(size_t)b * dim + i] = co;
    out[(size_t)b * dim + half + i] = s;
  }
}

// One wave per row, in place.
__global__ void softmax_rows_kernel(float* __restrict__ x, long rows, int L, int ld) {
  const long row = (long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float* r = x + row * ld;
  if (L == 256 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    // 4 consecutive keys per lane (one 16-B load and store): the order of the fused attention kernels'
    // softmax (attention.hip), so their P equals this one bit for bit
    f4 v = *reinterpret_cast<const f4*>(r + 4 * lane);
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
    *reinterpret_cast<f4*>(r + 4 * lane) = v * inv;
    return;
  }
  if (L <= 512) {
    // the row in registers (8 per lane): one read and one write of S instead of five passes; same
    // per-lane order of the max / exp / sum / scale as the loop below, so the same bits
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = lane + 64 * u;
      v[u] = j < L ? r[j] : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 8; ++u) mx = fmaxf(mx, v[u]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (lane + 64 * u < L) {
        v[u] = expf(v[u] - mx);
        sum += v[u];
      }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (lane + 64 * u < L) r[lane + 64 * u] = v[u] * inv;
    return;
  }
  float mx = -INFINITY;
  for (int j = lane; j < L; j += 64) mx = fmaxf(mx, r[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float sum = 0.f;
  for (int j = lane; j < L; j += 64) {
    float e = expf(r[j] - mx);
    r[j] = e;
    sum += e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  const float inv = 1.0f / sum;
  for (int j = lane; j < L; j += 64) r[j] = r[j] * inv;
}

// first conv: NCHW input with few channels -> NHWC (pitched) output.
// One block per R output rows of one image (R = 2 * 64 / W for W < 64, so a block is two 64-pixel GroupNorm
// chunks -- small_in_rows; else one row). The R + 2 input rows and the weights sit in LDS (coalesced loads). Thread t owns the
// output channel pair 2 cp, 2 cp + 1 (cp = t % (Cout / 2); its 2 x 9 Cin weights in registers) and a run of
// pixels of the block: per pixel 9 Cin packed multiply + packed add pairs (v_pk_mul_f32 / v_pk_add_f32, both
// channels from one broadcast input value) over a 3-column window whose column slots rotate (no register
// moves), then + bias; a float2 store per lane, coalesced over the channel pairs. Per output: acc from 0,
// acc + w x over (ci, ky, kx) with separately rounded products -- the reference CPU conv's arithmetic for
// this layer (a fused-multiply-add chain measured 2.6x further from the float64 trajectory on the ADM CFG
// test, whose free-running steps amplify a first-layer ulp ~10^3-fold).
// With gn_part the block also emits the consumer GroupNorm's per-chunk partials (sum, sum of squares in
// double) -- the layout of gn_partial_kernel -- so the first ResBlock and the last up-path concat skip their
// gn_partial passes.
constexpr int kSiMaxChunks = 8, kSiMaxPar = 4, kSiMaxG = 32;
typedef float fl2 __attribute__((ext_vector_type(2)));
template <int CIN>
__global__ void __launch_bounds__(256) conv3x3_small_in_kernel(const float* __restrict__ x, int H, int W, int R,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ bias, int Cout,
                                                               float* __restrict__ y, int y_pitch,
                                                               double2* __restrict__ gn_part, int G, int nchunk) {
  extern __shared__ __attribute__((aligned(16))) float smem_f[];
  constexpr int KW = CIN * 9;
  const int Wp = W + 2;
  const int nrow = CIN * (R + 2) * Wp;
  float* rows = smem_f;                                       // [CIN][R + 2][W + 2]
  float* wl = smem_f + nrow;                                  // [Cout][CIN * 9]
  double2* st = reinterpret_cast<double2*>(smem_f + ((nrow + Cout * KW + 3) & ~3));  // [par][chunk][G]
  const int b = blockIdx.y, oy0 = blockIdx.x * R;
  for (int i = threadIdx.x; i < nrow; i += blockDim.x) {
    const int ci = i / ((R + 2) * Wp);
    const int rr = (i / Wp) % (R + 2);
    const int xx = i % Wp - 1;
    const int iy = oy0 + rr - 1;
    float v = 0.f;
    if (iy >= 0 && iy < H && xx >= 0 && xx < W) v = x[(((size_t)b * CIN + ci) * H + iy) * W + xx];
    rows[i] = v;
  }
  for (int i = threadIdx.x; i < Cout * KW; i += blockDim.x) wl[i] = w[i];
  const int npair = Cout / 2;
  const int lanes_per_px = min(npair, (int)blockDim.x);
  const int px_par = blockDim.x / lanes_per_px;
  const int cpg = gn_part ? Cout / G : 2;  // channels per group; cpg / 2 lanes hold one group
  const int bchunks = (R * W) / kGnPixPerChunk;
  if (gn_part)
    for (int i = threadIdx.x; i < px_par * kSiMaxChunks * kSiMaxG; i += blockDim.x) st[i] = make_double2(0.0, 0.0);
  __syncthreads();
  // this thread's pixels: px_par groups over R rows (whole rows, or row segments when px_par > R)
  const int gI = threadIdx.x / lanes_per_px;
  int r0, r1, x0, x1;
  if (px_par >= R) {
    const int S = px_par / R, len = (W + S - 1) / S;
    r0 = gI / S;
    r1 = min(r0 + 1, R);
    x0 = (gI % S) * len;
    x1 = min(x0 + len, W);
  } else {
    // px_par groups over R rows, ceil(R / px_par) rows each (the last group may hold fewer); the leftover
    // threads of a block whose size the channel pairs do not divide (gI == px_par) get no rows
    const int RG = (R + px_par - 1) / px_par;
    r0 = min(gI * RG, R);
    r1 = min(r0 + RG, R);
    x0 = 0;
    x1 = W;
  }
  for (int cp = threadIdx.x % lanes_per_px; cp < npair; cp += lanes_per_px) {
    const int co = 2 * cp;
    fl2 wr[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) wr[k] = fl2{wl[co * KW + k], wl[(co + 1) * KW + k]};
    const fl2 bc = {bias[co], bias[co + 1]};
    double gs = 0.0, gq = 0.0;
    int cur = -1;  // chunk the (gs, gq) sums belong to
    auto flush = [&]() {  // over the group's cpg / 2 lanes, then one LDS slot per (px group, chunk, group)
      double s = gs, q = gq;
      for (int o = 1; o < cpg / 2; o <<= 1) {
        s += __shfl_xor(s, o);
        q += __shfl_xor(q, o);
      }
      if (co % cpg == 0) st[(gI * kSiMaxChunks + cur) * kSiMaxG + co / cpg] = make_double2(s, q);
      gs = gq = 0.0;
    };
    for (int r = r0; r < r1; ++r) {
      if (x0 >= x1) break;
      const int oy = oy0 + r;
      const float* rrow = rows + r * Wp;  // + (ci (R + 2) + ky) Wp + input column
      float col[3][CIN][3];               // column slots of the window, [slot][ci][ky]
      auto load_col = [&](int slot, int xx) {
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) col[slot][ci][ky] = rrow[(ci * (R + 2) + ky) * Wp + xx];
      };
      // output pixel ox with the window's left column in slot u % 3 (u = phase, compile-time after unrolling)
      auto pixel = [&](int ox, int u) {
        load_col((u + 2) % 3, ox + 2);
        fl2 acc = {0.f, 0.f};
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const float xv = col[(u + kx) % 3][ci][ky];
              acc = acc + wr[(ci * 3 + ky) * 3 + kx] * fl2{xv, xv};  // separately rounded (no contraction)
            }
        const fl2 v = acc + bc;
        *reinterpret_cast<fl2*>(y + (((size_t)b * H + oy) * W + ox) * y_pitch + co) = v;
        if (gn_part) {
          const int ch = ((oy - oy0) * W + ox) / kGnPixPerChunk;  // block-local chunk
          if (ch != cur) {
            if (cur >= 0) flush();
            cur = ch;
          }
          gs += (double)v.x;
          gs += (double)v.y;
          gq += (double)v.x * v.x;
          gq += (double)v.y * v.y;
        }
      };
      load_col(0, x0);
      load_col(1, x0 + 1);
      int ox = x0;
      for (; ox + 3 <= x1; ox += 3) {
#pragma unroll
        for (int u = 0; u < 3; ++u) pixel(ox + u, u);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (ox + u < x1) pixel(ox + u, u);
    }
    if (gn_part && cur >= 0) flush();
  }
  if (gn_part) {
    __syncthreads();
    const size_t c0 = (size_t)blockIdx.x * bchunks;
    for (int i = threadIdx.x; i < bchunks * G; i += blockDim.x) {
      const int cl = i / G, g = i - (i / G) * G;
      double s = 0.0, q = 0.0;
      for (int p = 0; p < px_par; ++p) {
        const double2 v = st[(p * kSiMaxChunks + cl) * kSiMaxG + g];
        s += v.x;
        q += v.y;
      }
      gn_part[((size_t)b * nchunk + c0 + cl) * G + g] = make_double2(s, q);
    }
  }
}

// last conv: NHWC (pitched) input -> NCHW output with few channels (Cout <= 8). Block = TH x TW output
// pixels of one image, one pixel per thread.
constexpr int kSoTW = 32, kSoTH = 8, kSoPP = (kSoTH + 2) * (kSoTW + 2);
// Last conv, pipelined form (the CIFAR / MNIST UNets' 128 -> 3 or 1 channel output conv at 32^2 / 28^2):
// 16-channel chunks (a 10 x 34 x 16 patch in 27 KB of LDS: five blocks per CU, so the B * 4 tiles of a
// B = 256 batch run in one wave of blocks instead of 1.33), the next chunk's patch loaded into registers
// while this chunk's 9 taps run (the previous form loaded, waited, then computed each 32-channel chunk), and
// output channels in pairs on packed FMAs (v_pk_fma_f32: one broadcast input value times a channel pair's
// weights; COP = Cout rounded up to even accumulators). Weights [9][Cin][COP] (zero-padded), wave-uniform
// 8-B pair loads. Summation per output over (16-channel chunk, tap, channel), one fused chain per channel as
// before (a packed FMA rounds each lane as v_fma_f32 does). The patch registers are double
// buffered: chunk c + 2's loads are issued right after chunk c's patch is stored, so each load has two
// chunks' taps to land (one chunk's 432 FMAs per thread did not cover the load latency).
constexpr int kSo2C = 16, kSo2LD = 20, kSo2PJ = (kSoPP * (kSo2C / 4) + 255) / 256, kSoMaxC = 512;
template <int CO>
__global__ void __launch_bounds__(256) conv3x3_small_out2_kernel(const float* __restrict__ x, int B, int H, int W,
                                                                 int Cin, int pitch, const float* __restrict__ wp,
                                                                 const float* __restrict__ bias,
                                                                 float* __restrict__ y,
                                                                 const float* __restrict__ pro_scale,
                                                                 const float* __restrict__ pro_shift, GnFin fin) {
  __shared__ __attribute__((aligned(16))) float patch[kSoPP * kSo2LD];
  __shared__ __attribute__((aligned(16))) float tab[2][kSoMaxC];  // fin: the image's GroupNorm affine
  const int tiles_x = ceil_div(W, kSoTW), tiles_y = ceil_div(H, kSoTH);
  const int b = blockIdx.x / (tiles_x * tiles_y);
  const int trem = blockIdx.x - b * tiles_x * tiles_y;
  const int ty0 = (trem / tiles_x) * kSoTH, tx0 = (trem % tiles_x) * kSoTW;
  const int t = threadIdx.x;
  const int py = t / kSoTW, px = t % kSoTW;
  // loader items: (patch pixel p, 4-channel quad c4) = i >> 2, i & 3, i = t + 256 j
  const float* src[kSo2PJ];
  bool ok[kSo2PJ];
#pragma unroll
  for (int j = 0; j < kSo2PJ; ++j) {
    const int i = min(t + 256 * j, kSoPP * 4 - 1);
    const int p = i >> 2, c4 = i & 3;
    const int iy = ty0 + p / (kSoTW + 2) - 1, ix = tx0 + p % (kSoTW + 2) - 1;
    ok[j] = t + 256 * j < kSoPP * 4 && iy >= 0 && iy < H && ix >= 0 && ix < W;
    src[j] = x + (((size_t)b * H + min(max(iy, 0), H - 1)) * W + min(max(ix, 0), W - 1)) * pitch + 4 * c4;
  }
  const bool gn = pro_scale || fin.part;
  f4 rva[kSo2PJ], rvb[kSo2PJ];
  auto load = [&](f4 (&rv)[kSo2PJ], int c0) {
#pragma unroll
    for (int j = 0; j < kSo2PJ; ++j) rv[j] = *reinterpret_cast<const f4*>(src[j] + c0);
  };
  auto store = [&](const f4 (&rv)[kSo2PJ], int c0) {
#pragma unroll
    for (int j = 0; j < kSo2PJ; ++j) {
      const int i = t + 256 * j;
      if (i >= kSoPP * 4) continue;
      const int p = i >> 2, c4 = i & 3;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (ok[j]) {
        v = rv[j];
        if (gn) {  // GroupNorm + SiLU of last_conv (models/unet.py:115-119), padding stays 0
          const f4 sc = fin.part ? *reinterpret_cast<const f4*>(&tab[0][c0 + 4 * c4])
                                 : *reinterpret_cast<const f4*>(pro_scale + (size_t)b * Cin + c0 + 4 * c4);
          const f4 sh = fin.part ? *reinterpret_cast<const f4*>(&tab[1][c0 + 4 * c4])
                                 : *reinterpret_cast<const f4*>(pro_shift + (size_t)b * Cin + c0 + 4 * c4);
          v.x = silu_fast(v.x * sc.x + sh.x); v.y = silu_fast(v.y * sc.y + sh.y);
          v.z = silu_fast(v.z * sc.z + sh.z); v.w = silu_fast(v.w * sc.w + sh.w);
        }
      }
      *reinterpret_cast<f4*>(patch + p * kSo2LD + 4 * c4) = v;
    }
  };
  constexpr int COP = (CO + 1) & ~1;
  fl2 acc[COP / 2];
#pragma unroll
  for (int c = 0; c < COP / 2; ++c) acc[c] = fl2{0.f, 0.f};
  auto chunk = [&](f4 (&rv)[kSo2PJ], int c0) {
    store(rv, c0);
    __syncthreads();
    if (c0 + 2 * kSo2C < Cin) load(rv, c0 + 2 * kSo2C);  // in flight during this and the next chunk's taps
#pragma unroll 3
    for (int tap = 0; tap < 9; ++tap) {
      const float* pr = patch + ((py + tap / 3) * (kSoTW + 2) + px + tap % 3) * kSo2LD;
      const float* wt = wp + ((size_t)tap * Cin + c0) * COP;  // wave-uniform
#pragma unroll
      for (int c4 = 0; c4 < kSo2C / 4; ++c4) {
        const f4 v = *reinterpret_cast<const f4*>(pr + 4 * c4);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int cp = 0; cp < COP / 2; ++cp)
            acc[cp] = __builtin_elementwise_fma(fl2{vv[q], vv[q]},
                                                *reinterpret_cast<const fl2*>(wt + (4 * c4 + q) * COP + 2 * cp), acc[cp]);
      }
    }
    __syncthreads();  // every thread is done with the patch before the next chunk overwrites it
  };
  load(rva, 0);
  if (kSo2C < Cin) load(rvb, kSo2C);
  if (fin.part) {  // gn_finalize (gn.hip) for this image, same expressions; read after the first chunk's barrier
    const int cpg = Cin / fin.G;
    for (int c = t; c < Cin; c += 256) {
      const int g = c / cpg;
      double a = 0, q = 0;
      for (int k = 0; k < fin.nchunk; ++k) {
        const double2 v = fin.part[((size_t)b * fin.nchunk + k) * fin.G + g];
        a += v.x;
        q += v.y;
      }
      const double m = a / fin.n;
      double var = q / fin.n - m * m;
      if (var < 0) var = 0;
      const float mu = (float)m;
      const float rs = (float)(1.0 / sqrt(var + (double)fin.eps));
      const float sc = rs * (fin.gamma ? fin.gamma[c] : 1.0f);
      tab[0][c] = sc;
      tab[1][c] = -sc * mu + (fin.beta ? fin.beta[c] : 0.0f);
    }
    __syncthreads();
  }
  for (int c0 = 0; c0 < Cin; c0 += 2 * kSo2C) {
    chunk(rva, c0);
    if (c0 + kSo2C < Cin) chunk(rvb, c0 + kSo2C);
  }
  const int oy = ty0 + py, ox = tx0 + px;
  if (oy < H && ox < W) {
#pragma unroll
    for (int c = 0; c < CO; ++c) y[(((size_t)b * CO + c) * H + oy) * W + ox] = acc[c / 2][c % 2] + bias[c];
  }
}

// torch [Cout][Cin][3][3] -> [9][Cin][CO] (zero-padded to CO outputs)
__global__ void small_out_pack_kernel(const float* w, int Cout, int Cin, int CO, float* wp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 9 * Cin * CO) return;
  const int co = i % CO, c = (i / CO) % Cin, tap = i / (CO * Cin);
  wp[i] = co < Cout ? w[((size_t)co * Cin + c) * 9 + tap] : 0.f;
}

__global__ void sampler_step_kernel(StepArgs s) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)s.C * s.HW;
  const long total = per * s.B;
  if (e >= total) return;
  const long b = e / per, r = e - b * per;
  const long mo = b * (long)s.Cm * s.HW + r;  // model-output index of the first C channels
  const float xt = s.xt[e];

  // predict(): model output -> (x0, eps) for one branch, reference ddpm.py:174-203
  auto predict = [&](float out, int objective, float& x0, float& eps) {
    if (objective == 0) {
      x0 = s.c_recip * xt - s.c_recipm1 * out;
    } else if (objective == 1) {
      x0 = out;
    } else {
      x0 = s.c_sa * xt - s.c_s1ma * out;
    }
    if (s.clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
    eps = (s.c_recip * xt - x0) / s.c_recipm1;
  };

  float x0, eps;
  if (s.out_u) {
    float x0c, epsc, x0u, epsu;
    predict(s.out_c[mo], s.objective, x0c, epsc);
    predict(s.out_u[mo], s.objective, x0u, epsu);
    const float comb = s.w_u * epsu + s.w_c * epsc;
    predict(comb, 0, x0, eps);  // hack_objective('pred_eps')
  } else {
    predict(s.out_c[mo], s.objective, x0, eps);
  }

  if (s.euler) {
    // euler.py:60-64 / heun.py:66-70 (first order), heun.py:89-100 (second order), reference op order
    float sample, d;
    if (s.euler == 1) {
      const float bar = s.e_st1 * xt;
      d = (bar - x0) / s.e_sig_t;
      sample = (bar + d * s.e_dsig) / s.e_sp1;
      if (s.e_dout) s.e_dout[e] = d;
    } else {
      const float barp = s.e_sp1 * xt;
      d = (barp - x0) / s.e_sig_p;
      d = (d + s.e_d1[e]) / 2.0f;
      const float bar = s.e_st1 * s.e_x1[e];
      sample = (bar + d * s.e_dsig) / s.e_sp1;
    }
    s.sample[e] = sample;
    if (s.x0_out) s.x0_out[e] = x0;
    if (s.eps_out) s.eps_out[e] = eps;
    return;
  }
  float mean, sample;
  if (s.kind == 0) {
    mean = s.m1 * x0 + s.m2 * eps;  // ddim.py:72-73
  } else {
    mean = s.m1 * x0 + s.m2 * xt;   // ddpm.py:230
  }
  float var = 0.f;
  float sd = s.std;
  if (s.var_mode == 1 && s.add_noise) {
    // learned_range, ddpm.py:240-246; learned channel comes from the cond branch
    const float lv = s.out_c[mo + per];
    const float frac = (lv + 1.0f) / 2.0f;
    const float logvar = frac * s.max_logvar + (1.0f - frac) * s.min_logvar;
    var = expf(logvar);
    sd = sqrtf(var);
  }
  if (s.add_noise) {
    const float nz = s.noise ? s.noise[e] : 0.f;
    sample = mean + sd * nz;
  } else {
    sample = mean;
  }
  s.sample[e] = sample;
  if (s.mean_out) s.mean_out[e] = mean;
  if (s.x0_out) s.x0_out[e] = x0;
  if (s.eps_out) s.eps_out[e] = eps;
  if (s.var_out) s.var_out[e] = var;
}

// Two-operand combination with scalar or per-row coefficients, each product and the final add / sub / div
// separately rounded (-ffp-contract=off), i.e. the torch float32 expressions of reference ddpm.py:
//   mode 0: c1 a + c2 b        diffuse (:164-172), pred_eps_from_v (:117-120)
//   mode 1: c1 a - c2 b        pred_x0_from_eps (:102-105), pred_x0_from_v (:112-115), get_v (:140-150)
//   mode 2: (c1 a - b) / c2    pred_eps_from_x0 (:107-110)
// Row r = e / row_elems selects c1_rows[r] / c2_rows[r] when given (per-image timesteps).
__global__ void lincomb_kernel(int mode, const float* __restrict__ a, const float* __restrict__ b,
                               float* __restrict__ out, long n, long row_elems, const float* __restrict__ c1r,
                               const float* __restrict__ c2r, float c1, float c2) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const long r = e / row_elems;
  const float k1 = c1r ? c1r[r] : c1, k2 = c2r ? c2r[r] : c2;
  const float pa = k1 * a[e];
  float v;
  if (mode == 0) {
    v = pa + k2 * b[e];
  } else if (mode == 1) {
    v = pa - k2 * b[e];
  } else {
    v = (pa - b[e]) / k2;
  }
  out[e] = v;
}

// avg-pool 2x2 / nearest-2x on NHWC views, float4 over channels, optional
// GroupNorm+SiLU prologue applied to each source pixel before pooling.
__global__ void resample2x_kernel(View x, View y, int down, const float* __restrict__ pro_scale,
                                  const float* __restrict__ pro_shift) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int C4 = y.C >> 2;
  const long total = (long)y.B * y.H * y.W * C4;
  if (e >= total) return;
  const int c4 = e % C4;
  long p = e / C4;
  const int ox = p % y.W;
  p /= y.W;
  const int oy = p % y.H;
  const int b = p / y.H;
  auto pro = [&](float4 v) {
    if (pro_scale) {
      const float4 sc = *reinterpret_cast<const float4*>(pro_scale + (size_t)b * x.C + 4 * c4);
      const float4 sh = *reinterpret_cast<const float4*>(pro_shift + (size_t)b * x.C + 4 * c4);
      v.x = silu_f(v.x * sc.x + sh.x); v.y = silu_f(v.y * sc.y + sh.y);
      v.z = silu_f(v.z * sc.z + sh.z); v.w = silu_f(v.w * sc.w + sh.w);
    }
    return v;
  };
  float4 o;
  if (down) {
    float4 s[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int iy = 2 * oy + (q >> 1), ix = 2 * ox + (q & 1);
      s[q] = pro(*reinterpret_cast<const float4*>(x.p + (((size_t)b * x.H + iy) * x.W + ix) * x.pitch + 4 * c4));
    }
    // torch avg_pool2d: row-major window sum, then / 4
    o.x = (((s[0].x + s[1].x) + s[2].x) + s[3].x) / 4.0f;
    o.y = (((s[0].y + s[1].y) + s[2].y) + s[3].y) / 4.0f;
    o.z = (((s[0].z + s[1].z) + s[2].z) + s[3].z) / 4.0f;
    o.w = (((s[0].w + s[1].w) + s[2].w) + s[3].w) / 4.0f;
  } else {
    o = pro(*reinterpret_cast<const float4*>(x.p + (((size_t)b * x.H + (oy >> 1)) * x.W + (ox >> 1)) * x.pitch +
                                             4 * c4));
  }
  *reinterpret_cast<float4*>(y.p + (((size_t)b * y.H + oy) * y.W + ox) * y.pitch + 4 * c4) = o;
}

__global__ void embed_add_silu_kernel(const float* __restrict__ temb, const int64_t* __restrict__ y,
                                      const float* __restrict__ table, int B, int D, int null_row,
                                      float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const int b = e / D, d = e - (e / D) * D;
  float v = temb[e];
  const int64_t cls = y ? y[b] : -1;
  const int64_t row = cls >= 0 ? cls : null_row;
  if (row >= 0) v = v + table[(size_t)row * D + d];
  out[e] = silu_f(v);
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int B, int C, int HW,
                                    float* __restrict__ y, int y_pitch) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * C * HW;
  if (e >= total) return;
  const long b = e / ((long)C * HW);
  const long r = e - b * C * HW;
  const int c = r / HW, p = r % HW;
  y[((size_t)b * HW + p) * y_pitch + c] = x[e];
}

__global__ void nhwc_to_nchw_kernel(const float* __restrict__ x, int B, int C, int HW, int pitch,
                                    float* __restrict__ y) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * C * HW;
  if (e >= total) return;
  const long b = e / ((long)C * HW);
  const long r = e - b * C * HW;
  const int c = r / HW, p = r % HW;
  y[e] = x[((size_t)b * HW + p) * pitch + c];
}

// [Cout][Cin][kh][kw] -> implicit-GEMM rows [Cout][ldw] at column offset col0.
// 3x3: chunk-major K order k = ((ci / 32) * 9 + tap) * 32 + ci % 32, so the
// nine taps of one 32-channel chunk are consecutive K slices (both conv
// kernels walk K this way); 1x1: k = ci.
__global__ void repack_conv_kernel(const float* __restrict__ w, int Cout, int Cin, int taps,
                                   float* __restrict__ out, int ldw, int col0) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Cout * Cin * taps;
  if (e >= total) return;
  const int co = e / ((long)Cin * taps);
  const int r = e - (long)co * Cin * taps;
  const int ci = r / taps, tap = r % taps;
  const int k = taps == 1 ? ci : ((ci >> 5) * taps + tap) * 32 + (ci & 31);
  out[(size_t)co * ldw + col0 + k] = w[e];
}

// Sub-pixel weights of "nearest-2x upsample, then 3x3 conv" (conv_patch.hip MODE 2):
// out[par][co][((ci/32) * 4 + ty * 2 + tx) * 32 + ci % 32] = sum over the 3x3 taps (ky, kx)
// that land on low-res pixel offset (ty, tx) for output parity par = (py, px):
// py = 0: ty 0 <- ky {0}, ty 1 <- ky {1, 2};  py = 1: ty 0 <- ky {0, 1}, ty 1 <- ky {2}  (same for x).
// Summed in fp64, rounded once.
__global__ void repack_subpix_kernel(const float* __restrict__ w, int Cout, int Cin, float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = 4L * Cout * Cin * 4;
  if (e >= total) return;
  const int tap = e & 3;
  long r = e >> 2;
  const int ci = r % Cin;
  r /= Cin;
  const int co = r % Cout;
  const int par = r / Cout;
  const int py = par >> 1, px = par & 1, ty = tap >> 1, tx = tap & 1;
  const int ky0 = (py == 0) ? (ty == 0 ? 0 : 1) : (ty == 0 ? 0 : 2);
  const int ky1 = (py == 0) ? (ty == 0 ? 0 : 2) : (ty == 0 ? 1 : 2);
  const int kx0 = (px == 0) ? (tx == 0 ? 0 : 1) : (tx == 0 ? 0 : 2);
  const int kx1 = (px == 0) ? (tx == 0 ? 0 : 2) : (tx == 0 ? 1 : 2);
  const float* wk = w + ((size_t)co * Cin + ci) * 9;
  double s = 0.0;
  for (int ky = ky0; ky <= ky1; ++ky)
    for (int kx = kx0; kx <= kx1; ++kx) s += (double)wk[ky * 3 + kx];
  out[((size_t)par * Cout + co) * (4 * (size_t)Cin) + ((ci >> 5) * 4 + tap) * 32 + (ci & 31)] = (float)s;
}

}  // namespace

int repack_subpixel(const float* w, int Cout, int Cin, float* out, hipStream_t st) {
  DM_REQUIRE(Cin % 32 == 0, "sub-pixel weight packing: input channels must be multiples of 32");
  const long total = 4L * Cout * Cin * 4;
  hipLaunchKernelGGL(repack_subpix_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, Cout, Cin,
                     out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int timestep_embed(const int64_t* t, int B, int dim, int kind, const float* freqs, float* out, hipStream_t st) {
  DM_REQUIRE(dim % 2 == 0 && dim >= 4, "timestep embedding: dim must be even and >= 4");
  const int n = B * (dim / 2);
  hipLaunchKernelGGL(timestep_embed_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, t, B, dim, kind, freqs, out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int softmax_rows(float* x, long rows, int L, int ld, hipStream_t st) {
  DM_REQUIRE(rows > 0 && L > 0 && ld >= L, "softmax: bad shape");
  const long blocks = (rows + 3) / 4;
  DM_REQUIRE(blocks < (1L << 31), "softmax: too many rows");
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, L, ld);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

// rows per block of the first conv: a whole 64-pixel chunk when W < 64 divides it, else one row
// Rows per block: two 64-pixel GroupNorm chunks of a narrow map (the CIFAR first conv: 4 rows of 32, 1024 blocks
// at B = 256) -- the per-block staging of the 3456 weights and the rows amortised over twice the pixels: C3 A/B
// +0.24 % over one chunk per block (3 alternations; four chunks +0.17 %)
constexpr int kSiChunksPerBlock = 2;
static int small_in_rows(int H, int W) {
  if (!(W < kGnPixPerChunk && kGnPixPerChunk % W == 0 && H % (kGnPixPerChunk / W) == 0)) return 1;
  int R = kGnPixPerChunk / W;
  for (int m = 1; m < kSiChunksPerBlock && H % (2 * R) == 0 && (2 * R * W) / kGnPixPerChunk <= kSiMaxChunks; m *= 2)
    R *= 2;
  return R;
}

bool conv3x3_small_in_can_emit(int H, int W, int Cout, int G) {
  const int R = small_in_rows(H, W);
  const int lpp = min(Cout / 2, 256);  // lanes per pixel (channel pairs); a wave's lanes share one pixel run
  const int cpg = G > 0 ? Cout / G : 0;
  return G > 0 && G <= kSiMaxG && Cout % G == 0 && cpg % 2 == 0 && cpg <= 64 && (cpg & (cpg - 1)) == 0 &&
         lpp >= 64 && 256 % lpp == 0 && (Cout / 2) % lpp == 0 && (R * W) % kGnPixPerChunk == 0 &&
         (R * W) / kGnPixPerChunk <= kSiMaxChunks && 256 / lpp <= kSiMaxPar;
}

int conv3x3_small_in(const float* x, int B, int Cin, int H, int W, const float* w, const float* bias,
                     int Cout, const View& y, hipStream_t st, double2* gn_part, int G) {
  DM_REQUIRE(Cin >= 1 && Cin <= 4, "first conv: Cin out of range (1..4)");
  DM_REQUIRE(Cout % 2 == 0 && y.pitch % 2 == 0, "first conv: Cout and the output pitch must be even");
  DM_REQUIRE(y.C == Cout && y.H == H && y.W == W && y.B == B, "first conv: output view mismatch");
  DM_REQUIRE(!gn_part || conv3x3_small_in_can_emit(H, W, Cout, G), "first conv: GroupNorm statistics shape");
  const int R = small_in_rows(H, W);
  const size_t nf = (size_t)Cin * 3 * (W + 2) + (size_t)Cin * (R - 1) * (W + 2) + (size_t)Cout * Cin * 9;
  size_t smem = ((nf + 3) & ~(size_t)3) * sizeof(float);
  if (gn_part) smem += (size_t)kSiMaxPar * kSiMaxChunks * kSiMaxG * sizeof(double2);
  DM_REQUIRE(smem <= 64 * 1024, "first conv: image too wide");
  const int nchunk = gn_num_chunks(H * W);
  dim3 grid(H / R, B);
#define DM_SI(CI) hipLaunchKernelGGL(conv3x3_small_in_kernel<CI>, grid, dim3(256), smem, st, x, H, W, R, w, bias, \
                                     Cout, y.p, y.pitch, gn_part, G, nchunk)
  switch (Cin) {
    case 1: DM_SI(1); break;
    case 2: DM_SI(2); break;
    case 3: DM_SI(3); break;
    default: DM_SI(4); break;
  }
#undef DM_SI
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int small_out_pack(const float* w, int Cout, int Cin, float* wp, hipStream_t st) {
  DM_REQUIRE(Cout >= 1 && Cout <= 8 && Cin > 0, "last conv: Cout out of range");
  const int CO = (Cout + 1) & ~1;  // conv3x3_small_out2_kernel<Cout>: channel pairs, zero-padded to even
  hipLaunchKernelGGL(small_out_pack_kernel, dim3((9 * Cin * CO + 255) / 256), dim3(256), 0, st, w, Cout, Cin, CO, wp);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int conv3x3_small_out(const View& x, const float* wp, const float* bias, int Cout, float* y, hipStream_t st,
                      const float* pro_scale, const float* pro_shift, const GnFin& fin) {
  DM_REQUIRE(Cout >= 1 && Cout <= 8, "last conv: Cout out of range");
  DM_REQUIRE(!fin.part || (!pro_scale && fin.G > 0 && x.C % fin.G == 0 && x.C <= kSoMaxC && fin.nchunk > 0),
             "last conv: in-kernel GroupNorm finalize needs groups dividing <= 512 channels");
  DM_REQUIRE(x.C % 32 == 0 && x.pitch % 4 == 0, "last conv: Cin must be a multiple of 32");
  // wp: small_out_pack's [9][Cin][Cout rounded up to even]
  DM_REQUIRE((reinterpret_cast<uintptr_t>(x.p) & 15) == 0, "last conv: input must be 16-byte aligned");
  const long tiles = (long)x.B * ceil_div(x.H, kSoTH) * ceil_div(x.W, kSoTW);
#define DM_SO2(CO)                                                                                            \
  hipLaunchKernelGGL(conv3x3_small_out2_kernel<CO>, dim3((unsigned)tiles), dim3(256), 0, st, x.p, x.B, x.H, x.W, \
                     x.C, x.pitch, wp, bias, y, pro_scale, pro_shift, fin)
  if (Cout == 1)
    DM_SO2(1);
  else if (Cout == 2)
    DM_SO2(2);
  else if (Cout == 3)
    DM_SO2(3);
  else if (Cout == 4)
    DM_SO2(4);
  else if (Cout == 5)
    DM_SO2(5);
  else if (Cout == 6)
    DM_SO2(6);
  else if (Cout == 7)
    DM_SO2(7);
  else
    DM_SO2(8);
#undef DM_SO2
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int sampler_step(const StepArgs& s, hipStream_t st) {
  DM_REQUIRE(s.xt && s.out_c && s.sample, "sampler step: null tensor");
  DM_REQUIRE(s.Cm == s.C || s.Cm == 2 * s.C, "sampler step: model output channels must be C or 2C");
  DM_REQUIRE(s.var_mode == 0 || s.Cm == 2 * s.C, "sampler step: learned_range needs 2C model channels");
  const long total = (long)s.B * s.C * s.HW;
  if (total == 0) return DM_OK;
  hipLaunchKernelGGL(sampler_step_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, s);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int lincomb(int mode, const float* a, const float* b, float* out, long n, long row_elems, const float* c1_rows,
            const float* c2_rows, float c1, float c2, hipStream_t st) {
  DM_REQUIRE(mode >= 0 && mode <= 2, "lincomb: mode must be 0, 1 or 2");
  DM_REQUIRE(a && b && out && n >= 0 && row_elems > 0, "lincomb: null tensor or bad shape");
  if (n == 0) return DM_OK;
  hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, mode, a, b, out, n,
                     row_elems, c1_rows, c2_rows, c1, c2);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int resample2x(const View& x, const View& y, int down, const float* pro_scale, const float* pro_shift,
               hipStream_t st) {
  DM_REQUIRE(x.C == y.C && x.B == y.B && x.C % 4 == 0 && x.pitch % 4 == 0 && y.pitch % 4 == 0,
             "resample: channel layout");
  if (down)
    DM_REQUIRE(y.H == x.H / 2 && y.W == x.W / 2 && x.H % 2 == 0 && x.W % 2 == 0, "resample: down size");
  else
    DM_REQUIRE(y.H == 2 * x.H && y.W == 2 * x.W, "resample: up size");
  const long total = (long)y.B * y.H * y.W * (y.C / 4);
  hipLaunchKernelGGL(resample2x_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, y, down,
                     pro_scale, pro_shift);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int embed_add_silu(const float* temb, const int64_t* y, const float* table, int B, int D, float* out,
                   hipStream_t st, int null_row) {
  const int n = B * D;
  hipLaunchKernelGGL(embed_add_silu_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, temb, y, table, B, D,
                     null_row, out);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int nchw_to_nhwc(const float* x, int B, int C, int HW, float* y, int y_pitch, hipStream_t st) {
  const long total = (long)B * C * HW;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, B, C, HW,
                     y, y_pitch);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int nhwc_to_nchw(const float* x, int B, int C, int HW, int pitch, float* y, hipStream_t st) {
  const long total = (long)B * C * HW;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, B, C, HW,
                     pitch, y);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

int repack_conv(const float* w, int Cout, int Cin, int taps, float* out, int ldw, int col0, hipStream_t st) {
  DM_REQUIRE(taps == 1 || Cin % 32 == 0, "conv weight packing: 3x3 input channels must be multiples of 32");
  const long total = (long)Cout * Cin * taps;
  hipLaunchKernelGGL(repack_conv_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, Cout, Cin,
                     taps, out, ldw, col0);
  DM_LAUNCH_CHECK();
  return DM_OK;
}

}  // namespace dm
