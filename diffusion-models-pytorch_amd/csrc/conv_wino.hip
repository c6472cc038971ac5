// 3x3 stride-1 convolution (models/unet.py:16,26: the ResBlock convs) as a Winograd F(2,3) along x and a direct
// 3-tap sum along y, on the fp16x2 split matrix cores of conv_k32.hip.
//
// Per output row y and output pixel pair (2j, 2j + 1), tap row dy and input channel c, the 1-D filter
// g = w[dy][0..2] over d = x[y + dy - 1][2j - 1 .. 2j + 2] (zero padding outside the map) is
//   V = B^T d = (d0 - d2, d1 + d2, d2 - d1, d1 - d3),  U = G g = (g0, (g0 + g1 + g2) / 2, (g0 - g1 + g2) / 2, g2),
//   y0 = m0 + m1 + m2,  y1 = m1 - m2 - m3,  m_nu = sum over (c, dy) of V_nu U_nu,
// i.e. four GEMMs (nu = 0..3) with K = 3 Cin: 12 K = 32 steps per pair and 32-channel chunk where the direct
// conv takes 9 per pixel (18 per pair) -- 2/3 of the MFMA products. U is formed once at plan build in float64
// (wino_pack_kernel) and split like every other weight (split_conv_weights, nmat = 4, ntap = 3: one power-of-two
// row scale per output channel over all four matrices); V is formed in fp32 from the GroupNorm + SiLU'd patch
// (one rounding) and split in the loader; the output transform is fp32 in the epilogue.
//
// Block: 512 threads, persistent over the 128-pixel tiles (TH = 128 / W whole rows of a W = 32 or 16 wide map: 64
// pairs) x 128 output channels of one image (its GroupNorm tables built once; the next tile's first pixels loaded
// during the epilogue). Wave w = (nu = w >> 1, ch = w & 1) computes GEMM nu for the 64 pairs x 64 channels of column
// half ch: 4 x 4 tiles of v_mfma_f32_16x16x32_f16, three per product (a1 w0 + a0 w1 + a0 w0), 48 MFMAs per
// K step as conv_k32's 64 x 64 wave tiles -- so the operand traffic per MFMA is conv_k32's, and the 8 waves
// (two per SIMD) keep the same occupancy in one block per CU.
// LDS: per 32-channel chunk the transformed patch, [nu][(TH + 2) x NP pair rows][piece][4 k-groups][8] fp16 with
// conv_k32's 160-B row pitch and the k-group bit swizzled by row (wswz below: A fragment i of tap row dy for wave
// nu = 16 consecutive rows nu NR + 16 i + dy NP, conflict-free ds_read_b128; the loader's stores at most 2-way),
// double buffered, one barrier per chunk. B: raw buffer loads from the U images, the wave-uniform part of each
// address in the scalar offset. The loader: lane j
// of a (patch row, 8-channel quarter) unit loads pixels 2j, 2j + 1, applies GroupNorm + SiLU, and takes its
// neighbours' 2j - 1 and 2j + 2 from lanes j -/+ 1 by DPP row shifts (each pixel normalised once).
// Epilogue: the 8 waves' m_nu tiles (row scale undone) into LDS, then each wave takes 32 output pixels x 64
// channels through StagedEpilogue (output transform, bias, temb row vector, residual, 16-B stores, GroupNorm
// partials of the consumer per 64-pixel chunk, the two 32-pixel halves combined in LDS).
#include <cstdlib>
#include <string>
#include <type_traits>

#include "dm_common.h"
#include "dm_kernels.h"
#include "mfma_tile.h"
#include "split16.h"
#include "conv_epilogue.h"

namespace dm {

namespace {

// the loader / tap-row / chunk lambdas are called from both roles' loop copies: always inlined (an outlined call would
// put the accumulators and the B ring in scratch)
#define DM_WINO_INL __attribute__((always_inline))

constexpr int kWC = 32;                        // input channels per chunk (K of one MFMA step)
constexpr int kWRowH = 80;                     // LDS row pitch in fp16 (160 B), as conv_k32
constexpr int kWNR = 96;                       // pair rows per nu plane at most: (TH + 2) NP = 6 x 16 / 10 x 8
constexpr int kWBuf = 4 * kWNR * kWRowH;       // fp16 per patch buffer (61440 B)

// Patch row layout: 16-B slots s = 4 piece + k-group, the k-group's low bit XORed with bit 2 of the pair row (slot s
// of row r at 16 (s ^ wswz(r)) bytes). Chosen by an offline search over the pitch and the linear XOR maps of r mod 16
// against the two access patterns (MI355X_MICROARCH.md LDS table): the A-fragment ds_read_b128 (16 rows from any
// base) stay conflict-free and the loader's ds_write_b64 (16 lanes: 16 rows of one 8-B half at W 32, 8 rows x both
// halves at W 16, 4 rows x 2 k-groups x 2 halves at W 8) go from 4-way / 2-way / 1 to 2-way (the minimum for one half)
// / 1 / 1. The piece bit is untouched, so a fragment's two pieces stay 64 B apart (one address, two offsets).
__device__ __forceinline__ int wswz(int r) { return (r >> 2) & 1; }
constexpr int kWTab = 4096;                    // GroupNorm table floats: one image, Cin <= 2048 (scales, shifts)
constexpr int kWEP = 68;                       // epilogue plane pitch (floats)
constexpr int kWSmem = 4 * 2 * 64 * kWEP * 4;     // the epilogue's m planes (139264 B), over the two patch buffers
static_assert(2 * kWBuf * 2 <= kWSmem, "patch buffers");
constexpr int kWMaxG = 32;                     // in-kernel GroupNorm finalize: groups of the input

#ifdef DM_K32_STAMPS
// Diagnostic build only (-DDM_K32_STAMPS, tools/wino_stamps.py): per block, wave 0's s_memtime at the start, after
// the prologue, after the main loop and at the end, and s_memrealtime at the start and the end, into this buffer only.
__device__ unsigned long long g_wino_stamps[65536][16];
#define W_STAMP(k)                                                                                           \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_wino_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#define W_RSTAMP(k)                                                                                          \
  do {                                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_wino_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define W_STAMP(k) do {} while (0)
#define W_RSTAMP(k) do {} while (0)
#endif

// lo[k] = fp16(x[k] - hi[k]) (hi[k] = fp16(x[k]): the difference exact) by v_fma_mixlo_f16 / v_fma_mixhi_f16: the
// fp16 operand converted and the result rounded to fp16 in the instruction, two lanes of lo per register
__device__ __forceinline__ void split_lo4(f4 x, f16x4 hi, f16x4& lo) {
  typedef unsigned int u2v __attribute__((ext_vector_type(2)));
  const u2v hp = __builtin_bit_cast(u2v, hi);
  u2v lp;
#pragma unroll
  for (int w = 0; w < 2; ++w)  // one asm per register: its two halves written by the pair (no zero-initialisation)
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(lp[w]) : "v"(hp[w]), "v"(x[2 * w]), "v"(x[2 * w + 1]));
  lo = __builtin_bit_cast(f16x4, lp);
}

// v0[k] = row_shr(e1)[k] - e1[k], v3[k] = e0[k] - row_shl(e0)[k], DPP folded into the subtractions (bound_ctrl: the
// shifted operand is 0 outside the 16-lane row). The leading s_nop 1 covers the VALU-write -> DPP-read hazard of the
// inputs (the compiler does not see DPP inside inline asm).
__device__ __forceinline__ void dpp_sub4(f4 e0, f4 e1, f4& v0, f4& v3) {
  asm("s_nop 1\n"
      "v_sub_f32_dpp %0, %8, %8 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_sub_f32_dpp %1, %9, %9 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_sub_f32_dpp %2, %10, %10 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_sub_f32_dpp %3, %11, %11 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_subrev_f32_dpp %4, %12, %12 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_subrev_f32_dpp %5, %13, %13 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_subrev_f32_dpp %6, %14, %14 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_subrev_f32_dpp %7, %15, %15 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "=&v"(v0[0]), "=&v"(v0[1]), "=&v"(v0[2]), "=&v"(v0[3]), "=&v"(v3[0]), "=&v"(v3[1]), "=&v"(v3[2]), "=&v"(v3[3])
      : "v"(e1[0]), "v"(e1[1]), "v"(e1[2]), "v"(e1[3]), "v"(e0[0]), "v"(e0[1]), "v"(e0[2]), "v"(e0[3]));
}

// x - hi[k] (hi[k] an fp16 piece of x: exact) in one v_fma_mix_f32 (the f16 operand converted in the instruction) instead
// of a conversion and a subtraction
__device__ __forceinline__ float sub_f16(float x, f16x4 hi, int k) {
  typedef unsigned int u2v __attribute__((ext_vector_type(2)));
  const u2v hp = __builtin_bit_cast(u2v, hi);
  float r;
  if (k & 1)
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp[k >> 1]), "v"(x));
  else
    asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[0,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp[k >> 1]), "v"(x));
  return r;
}

// DPP row shift by one lane (row_shr:1 = from lane - 1, row_shl:1 = from lane + 1), 0 where the source lane is
// outside the 16-lane row (bound_ctrl)
__device__ __forceinline__ float dpp_f(float v, int ctrl_shr) {
  return __builtin_bit_cast(float, ctrl_shr ? __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x111, 0xF, 0xF, true)
                                            : __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x101, 0xF, 0xF, true));
}

// PROM: input prologue -- 0 none, 1 GroupNorm affine, 2 GroupNorm affine + SiLU; SC: a shortcut segment (Cin2 > 0);
// WIDE: 2-D tiles of 4 rows x 32 columns of a map wider than 32 (ADM's 64^2 .. 256^2; W 32), the GEMM row index
// enumerating pixels tile by tile as conv_k32's T2D tiles (t2d_pixel), with the halo columns (the pixels left and
// right of the tile, GroupNorm + SiLU'd) from a small LDS edge buffer
template <int W, int PROM, bool SC, bool WIDE>
__device__ __forceinline__ void conv_wino_body(const ConvArgs& a) {
  static_assert(!WIDE || W == 32, "wide maps: 32-column tiles");
  constexpr bool PRO = PROM != 0;
  // a 128-pixel tile: 128 / W whole rows of one image (W 32, 16), two whole 8 x 8 images (W 8) or eight whole 4 x 4
  // images (W 4); per image RIMG output rows and PRI = RIMG + 2 patch rows (the halo)
  constexpr int IMGS = W == 8 ? 2 : W == 4 ? 8 : 1, RIMG = 128 / W / IMGS, PRI = RIMG + 2;
  constexpr int NP = W / 2, PR = IMGS * PRI, NR = PR * NP;
  static_assert(NR <= kWNR, "patch plane");
  // KS (the 4 x 4 maps: 64 tiles at B = 256 for 256 CUs): split-K over the input channels -- block (split, ..) takes
  // chunks and shortcut steps split * n / ksplit .. of the tile and stores its raw m-transformed partial sums to
  // kpart[split], conv_splitk_reduce adds them in split order with the epilogue (and the GroupNorm statistics)
  constexpr bool KS = W == 4;
  // loader units (patch row, 4-channel eighth of the chunk) of NP lanes, 64 / NP per wave instruction: NSET = 12
  // (W 32, W 4) / 10 (W 16, W 8) full sets over the 8 waves -- set s = w and, for the first NSET - 8 waves of one role,
  // 8 + w'
  constexpr int NSET = PR * 8 * NP / 64;
  static_assert(NSET * 64 == PR * 8 * NP && NSET > 8 && NSET <= 16, "loader sets");
  constexpr int TM = 4, TN = 4, NTAP = 3;
  constexpr int WD = 2;  // B ring depth: a refill issued behind the next chunk's pixel loads (in-order vmcnt)
                                 // is consumed WD tap rows later
  __shared__ __attribute__((aligned(16))) char smem[kWSmem];
  __shared__ __attribute__((aligned(16))) float gtab[kWTab];  // the image's GroupNorm tables (all its tiles)
  __shared__ float gstat[IMGS * 2 * kWMaxG];
  __shared__ double gxr[8 * 16 * 2];
  __shared__ __attribute__((aligned(16))) float gzero[8];  // the padding rows' table: 0 scale, 0 shift
  // WIDE: the halo columns of two chunks, [chunk & 1][patch row][left, right][32 channels] fp32, GroupNorm + SiLU'd
  __shared__ __attribute__((aligned(16))) float wedge[WIDE ? 2 * 6 * 2 * kWC : 4];
  _Float16* patch = reinterpret_cast<_Float16*>(smem);

  const int Wimg = WIDE ? a.Wout : W;  // the map's width (WIDE: a multiple of 32 tiles)
  const int ntx = Wimg / W;            // tile columns (1 unless WIDE)
  const int HW = a.Hout * Wimg;
  const int M = a.B * HW, N = a.Cout;
  const int nN = N / 128;
  // persistent blocks over the tiles of ONE image (two for 8 x 8 maps, eight for 4 x 4; their GroupNorm tables built
  // once): grid = [ksplit x] ceil(B / IMGS) x parts, block (images b0 .., part) takes tiles part * tpb .. + tpb - 1 of
  // the group's nN x (IMGS HW / 128), column halves outer
  const int nks = KS ? a.ksplit : 1;
  const int gsz = KS ? (int)gridDim.x / nks : (int)gridDim.x;  // blocks per split
  const int split = KS ? (int)blockIdx.x / gsz : 0;
  const int bidl = KS ? (int)blockIdx.x - split * gsz : (int)blockIdx.x;
  const int parts = gsz / ceil_div(a.B, IMGS);
  const int g0 = bidl / parts, part = bidl - g0 * parts;
  const int b0 = g0 * IMGS;
  const int tpb = (IMGS * HW / 128) * nN / parts;
  const int t_first = part * tpb, t_end = t_first + tpb;
  W_RSTAMP(5);
  W_STAMP(0);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nu = wave >> 1, ch = wave & 1;
  const int l16 = lane & 15, q = lane >> 4;
  const int lj = lane & (NP - 1);  // loader: pair lj of the lane's unit
  // Set s covers 16-lane rows 4 s .. 4 s + 3, unit u = row (W 32), 2 row + (lane & 15) / 8 (W 16) or 4 row +
  // (lane & 15) / 4 (W 8): patch row u / 8 -- s / 2, s (the same for the wave's lanes) or 2 s + lane / 32 -- and
  // channels 4 (u & 7) .. + 3, the same in both of a wave's sets (s and s + 8). The NSET - 8 extra sets go to waves
  // 0.. of the late role.
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int xw = wave_u - 4;
  const bool has2 = xw >= 0 && xw < NSET - 8;
  // (W 4: unit = 2 lanes, a 16-lane row one patch row's 8 channel quads, set s patch rows 4 s .. 4 s + 3)
  const int loff = NP == 16 ? 16 * (wave_u & 1) + 4 * (lane >> 4)
                 : NP == 8  ? 4 * (lane >> 3)
                 : NP == 4  ? 16 * ((lane >> 4) & 1) + 4 * ((lane >> 2) & 3)
                            : 4 * ((lane >> 1) & 7);
  // the input channels of this block: all, or (KS) chunks cb .. cb + nch - 1 and shortcut steps sb .. sb + ns - 1
  const int NCH = a.Cin1 / kWC, NSC = SC ? a.Cin2 / (2 * kWC) : 0;  // chunks, shortcut steps of the conv
  const int cb = KS ? split * NCH / nks : 0, sb = KS ? split * NSC / nks : 0;
  const int nch = KS ? (split + 1) * NCH / nks - cb : NCH;
  const int tabc = KS ? nch * kWC : a.Cin1;  // GroupNorm table channels per image (from channel cb kWC)
  int lpr[2], ltab[2];  // per set: patch row, the offset of its image's GroupNorm table
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int s_ = k ? 8 + max(xw, 0) : wave_u;
    lpr[k] = min(NP == 16 ? s_ >> 1 : NP == 8 ? s_ : NP == 4 ? 2 * s_ + (lane >> 5) : 4 * s_ + (lane >> 4), PR - 1);
    ltab[k] = IMGS == 1 ? 0 : (lpr[k] / PRI) * 2 * tabc;
  }
  // the lane's offset in a patch row group (pair row lpr NP + lj: its swizzle bit depends on the lane only -- lpr NP
  // is a multiple of 8, at W 8 of 4 with lpr's parity the lane's half-wave, at W 4 of 2 with bit 1 of lpr the lane's
  // half-wave)
  const int ldst = lj * kWRowH +
                   8 * ((loff >> 3) ^ wswz(NP == 4 ? 4 * (lane >> 5) + lj : NP == 2 ? 2 * (lane >> 4) + lj : lj)) +
                   (loff & 4);
  const float emL = lj == 0 ? 1.f : 0.f, emR = lj == NP - 1 ? 1.f : 0.f;  // (WIDE: the tile's edge lanes)
  const int Kp = NTAP * a.Cin1 + (SC ? a.Cin2 / 2 : 0);  // K of each U matrix (their stride in the image)
  const int ngrp = ceil_div(N, 32);
  const size_t sl = (size_t)ngrp * 1024;  // fp16 per 16-deep slice of the U images
  // B (the U images) by raw buffer loads: the lane's part of the address in voffset (column l16 + 16 (q & 1) of the
  // 32-column group, the 16-slice of k-groups 2, 3 for q >= 2: 3 slices on in the tap-row steps, 1 in the shortcut
  // steps), the wave-uniform rest in soffset -- no 64-bit VALU address arithmetic per refill
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.wino_ws), 0, 0x7FFFFFFF, 0x00020000);
  const int vb_lane = ((q & 1) * 32 + l16) * 16;
  const int vb_main = vb_lane + (q >> 1) * NTAP * (int)sl * 2, vb_sc = vb_lane + (q >> 1) * (int)sl * 2;
  const int nu_u = wave_u >> 1, ch_u = wave_u & 1;
  const int kt_end = nch * NTAP;

  // ---- per-tile state: the tile's rows and columns, the loader's pixel pointers, the B base
  int m0 = 0, n0 = 0;
  bool rok[2] = {false, false};
  // the set's pixel 2 lj (pixel 2 lj + 1 one pitch on; padding rows: the zero page, which covers a pitch and a row)
  const float* pp[2] = {nullptr, nullptr};
  int wcol = 0;  // bytes: the wave's nu plane and 32-column group of the tile (uniform)
  int ty = 0, tx = 0;  // the tile's row / column among the image's tiles
  // column halves outer: a block's consecutive tiles share one 128-column half of U, so the blocks of an XCD, which
  // run roughly in step, keep one half's U image in its L2 instead of both (wide maps: a block's tiles are one column
  // half of its image when parts == nN, and the XCDs alternate halves)
  const int MT = IMGS * HW / 128;  // row tiles of the image group
  auto set_tile = [&](int tile) DM_WINO_INL {
    const int mt = tile % MT, nt = tile / MT;
    m0 = b0 * HW + mt * 128;
    n0 = nt * 128;
    ty = WIDE ? mt / ntx : mt;
    tx = WIDE ? mt - ty * ntx : 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ti = IMGS == 1 ? 0 : lpr[k] / PRI, bi = b0 + ti;
      const int iy = ty * RIMG - 1 + lpr[k] - ti * PRI;
      rok[k] = iy >= 0 && iy < a.Hin && bi < a.B;  // (a group's second image past B: padding throughout)
      pp[k] = rok[k] ? a.x1 + ((size_t)(bi * a.Hin + iy) * Wimg + tx * W + 2 * lj) * a.x1_pitch + loff
                     : kZeroPage + loff;
    }
    // column n0 + ch 64 + 16 j + l16 (n0 % 128 == 0): 32-column group (n0 + ch 64) / 32 + j / 2, column
    // 16 (j & 1) + l16 of it -- one base pointer, compile-time offsets per j
    wcol = __builtin_amdgcn_readfirstlane((nu_u * (Kp / 16) * (int)sl + ((n0 + ch_u * 64) >> 5) * 1024) * 2);
  };

  // chunk c + 1's pixels: loaded a chunk ahead (right after the previous finish), finished before / after chunk c's
  // MFMAs (the ping-pong below)
  f4 rw[4];  // set k: pixels 2 lj, 2 lj + 1 in rw[2 k], rw[2 k + 1]
  auto load_raw = [&](int c) DM_WINO_INL {
    const int co = (cb + c) * kWC;
    rw[0] = *reinterpret_cast<const f4*>(pp[0] + co);
    rw[1] = *reinterpret_cast<const f4*>(pp[0] + a.x1_pitch + co);
    if (has2) {
      rw[2] = *reinterpret_cast<const f4*>(pp[1] + co);
      rw[3] = *reinterpret_cast<const f4*>(pp[1] + a.x1_pitch + co);
    }
  };
  if (t < 8) gzero[t] = 0.f;  // (visible after the prologue's barrier)
  // set k's 4 channels: GroupNorm (+ SiLU) of the lane's two pixels, the neighbours by DPP,
  // V = B^T d, split, stored into buffer buf. PROM 2: the tables hold -log2(e) (scale, shift), so z' = -log2(e) z
  // comes out of one fma and silu(z) = -ln 2 * z' / (1 + 2^z'): the loader keeps z' / (1 + 2^z') and the epilogue
  // scales by -ln 2 (exact algebra; one rounding each). Padding rows read the zero table: exactly 0. Range: a V
  // beyond fp16's range splits into an infinite piece, which every product carries into the accumulators -- the
  // epilogue's finiteness check raises the range flag.
  auto finish_set = [&](int c, int buf, int k) DM_WINO_INL {
    f4 e0 = rw[2 * k], e1 = rw[2 * k + 1];
    if (PROM) {
      const float* ts = rok[k] ? gtab + ltab[k] + 2 * (c * kWC + loff) : gzero;  // [4 scales][4 shifts]
      const f4 sc = *reinterpret_cast<const f4*>(ts), sh = *reinterpret_cast<const f4*>(ts + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float z0 = __builtin_fmaf(e0[k], sc[k], sh[k]);
        const float z1 = __builtin_fmaf(e1[k], sc[k], sh[k]);
        e0[k] = PROM == 2 ? z0 * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z0)) : z0;
        e1[k] = PROM == 2 ? z1 * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z1)) : z1;
      }
    }
    f4 vv[4];
    // V0 = x[2j - 1] - x[2j + 1] (lane j - 1's second pixel: DPP row_shr), V3 = x[2j] - x[2j + 2] (lane j + 1's first
    // pixel: row_shl), the shifted operand zero outside the 16-lane row (bound_ctrl) -- the map's padding columns
    dpp_sub4(e0, e1, vv[0], vv[3]);
    if (WIDE) {  // the tile's halo columns (zero at the map's edges): lane 0's x[-1], lane 15's x[32]
      const f4 h = *reinterpret_cast<const f4*>(wedge + ((c & 1) * 6 + lpr[k]) * 2 * kWC + (lj == 15 ? kWC : 0) + loff);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        vv[0][k] = __builtin_fmaf(emL, h[k], vv[0][k]);   // (-x[1]) + x[-1]: one rounding, as the subtraction
        vv[3][k] = __builtin_fmaf(-emR, h[k], vv[3][k]);  // x[30] - x[32]
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (NP < 16) {  // two units per DPP row: their boundary is a map edge too
        vv[0][k] = lj == 0 ? -e1[k] : vv[0][k];
        vv[3][k] = lj == NP - 1 ? e0[k] : vv[3][k];
      }
      vv[1][k] = e0[k] + e1[k];
      vv[2][k] = e1[k] - e0[k];
    }
    {
      _Float16* dst = patch + buf * kWBuf + lpr[k] * NP * kWRowH + ldst;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        f16x4 hi, lo;  // x = hi + lo, lo = fp16(x - hi) (the difference exact, one rounding to fp16)
#pragma unroll
        for (int k = 0; k < 4; ++k) hi[k] = (_Float16)vv[v][k];
        split_lo4(vv[v], hi, lo);
        *reinterpret_cast<f16x4*>(dst + v * NR * kWRowH) = hi;
        *reinterpret_cast<f16x4*>(dst + v * NR * kWRowH + 32) = lo;
      }
    }
  };

  auto finish = [&](int c, int buf) DM_WINO_INL {
    finish_set(c, buf, 0);
    if (has2) finish_set(c, buf, 1);
  };

  // ---- WIDE: the halo columns. Edge unit u = 64 ew + lane of the waves ew = 0, 1 (early role, one set each, so
  // rw[2] / rw[3] are theirs to use): patch row u / 16, side u & 1, channel quad (u / 2) & 7 -- 6 x 2 x 8 = 96
  // units per chunk. Chunk c's edges are finished a chunk before chunk c itself (its slot c & 1 published by the
  // barrier between), the raw pixels loaded a chunk before that.
  const int eu = wave_u * 64 + lane;
  const bool ew = WIDE && wave_u < 2;  // an edge wave
  const float* epx = kZeroPage;  // the edge unit's pixel (chunk 0), the zero page outside the map
  int etab = -1;                 // its GroupNorm table offset (-1: padding)
  auto set_edges = [&]() DM_WINO_INL {
    if (!ew) return;
    const int pr = eu >> 4, side = eu & 1, cq = (eu >> 1) & 7;
    const int iy = ty * RIMG - 1 + pr, ix = side ? tx * W + W : tx * W - 1;
    const bool ok = eu < 96 && iy >= 0 && iy < a.Hin && ix >= 0 && ix < Wimg;
    epx = ok ? a.x1 + ((size_t)(b0 * a.Hin + iy) * Wimg + ix) * a.x1_pitch + 4 * cq : kZeroPage;
    etab = ok ? 8 * cq : -1;
  };
  auto load_edge = [&](int c, f4& r) DM_WINO_INL {
    if (ew) r = *reinterpret_cast<const f4*>(epx + (etab >= 0 ? c * kWC : 0));
  };
  auto finish_edge = [&](int c, const f4& r) DM_WINO_INL {  // chunk c's edges into slot c & 1
    if (!ew || eu >= 96) return;
    f4 v = r;  // (PROM 0: the raw pixels; the zero page outside the map)
    if (PROM) {
      const float* ts = etab >= 0 ? gtab + 2 * c * kWC + etab : gzero;
      const f4 sc = *reinterpret_cast<const f4*>(ts), sh = *reinterpret_cast<const f4*>(ts + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float z = __builtin_fmaf(r[k], sc[k], sh[k]);
        v[k] = PROM == 2 ? z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z)) : z;  // (finish_set's)
      }
    }
    const int pr = eu >> 4, side = eu & 1, cq = (eu >> 1) & 7;
    *reinterpret_cast<f4*>(wedge + ((c & 1) * 6 + pr) * 2 * kWC + side * kWC + 4 * cq) = v;
  };

  // ---- B: the fp16x2 fragment images of U_nu (split_conv_weights, nmat 4, ntap 3), 16-column halves
  // all K steps of a tile: the 3 nch tap rows (step kt = 3 c + dy: 16-slice 6 c + dy, + 3 for k-groups 2, 3), then
  // the ns shortcut steps (16-slices 6 nch + 2 s, + 1 for k-groups 2, 3); past the end: the last step again
  // (refills nothing uses)
  const int ns = KS ? (split + 1) * NSC / nks - sb : NSC, nst = kt_end + ns, nst_g = nch + ns;  // K steps, stages
  f16x8 bq[WD][TN][2];
  auto load_b = [&](f16x8 (&dst)[TN][2], int kt) DM_WINO_INL {
    kt = __builtin_amdgcn_readfirstlane(min(kt, nst - 1));
    // branch-free (a uniform select of two VGPRs became a branch around every refill): the shortcut case only in
    // the SC kernels, its voffset by a bit blend under an all-ones / all-zeros scalar mask (KS: the block's steps
    // are the conv's main steps cb NTAP .. and shortcut steps sb ..)
    const int msc = SC ? -(int)(kt >= kt_end) : 0;
    const int kg = kt + cb * NTAP;
    const int so = wcol + (((kg + (kg / NTAP) * NTAP) & ~msc) | ((2 * NCH * NTAP + 2 * (kt - kt_end + sb)) & msc)) * (int)sl * 2;
    const int vo = SC ? (vb_main & ~msc) | (vb_sc & msc) : vb_main;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        dst[j][p] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, vo + ((j >> 1) * 1024 + (j & 1) * 128 + p * 512) * 2, so, 0));
  };

  f4 acc[TM][TN];
  // tap row dy: A fragment i = pair rows nu NR + 16 i + l16 + dy NP of buffer pbuf, the lane's k-group q (swizzled:
  // every fragment's first row is a multiple of 8 except the W 8 tap rows at 4 dy, where the swizzle bit flips)
  // (W 4: pair 16 i + l16 of the tile is pair l16 & 7 of image 2 i + l16 / 8, whose pair rows start 12 further on per
  // image: the lane's row 12 (l16 / 8) + (l16 & 7) of fragment i's 24, and its swizzle bit differs per tap row)
  const int lrow = NP == 2 ? 12 * (l16 >> 3) + (l16 & 7) : l16;
  auto aoff = [&](int r) { return (nu * NR + r) * kWRowH + 8 * (q ^ wswz(r)); };
  const int abase = aoff(lrow);
  const int abase_x = NP == 4 ? abase + 8 - 16 * ((q ^ wswz(l16)) & 1) : abase;  // (W 8, odd dy)
  const int abase_2 = NP == 2 ? aoff(lrow + 2) - 2 * kWRowH : abase;            // (W 4, dy 1)
  const int abase_4 = NP == 2 ? aoff(lrow + 4) - 4 * kWRowH : abase;            // (W 4, dy 2)
  auto arow_base = [&](int dy) DM_WINO_INL {
    if (NP == 2) return dy == 0 ? abase : dy == 1 ? abase_2 : abase_4;
    return ((dy * NP) & 4) ? abase_x : abase;
  };
  const int abase_sc = l16 * kWRowH + 8 * (q ^ wswz(l16));  // the shortcut steps' [nu][64] pair rows
  // a0: tile 0's fragment of this tap row on entry (read ahead); within a chunk, the next tap row's on exit
  f16x8 a0[2];
  auto read_a0 = [&](int dy, int pbuf) DM_WINO_INL {
    const _Float16* As = patch + pbuf * kWBuf + arow_base(dy) + dy * NP * kWRowH;
    a0[0] = *reinterpret_cast<const f16x8*>(As);
    a0[1] = *reinterpret_cast<const f16x8*>(As + 32);
  };
  // pair rows 16 i .. of the tile: image i / 2 of a W 8 tile sits 2 halo rows (2 NP pair rows) further down the patch;
  // images 2 i, 2 i + 1 of a W 4 tile 2 x 2 halo rows per earlier image pair (8 i pair rows)
  auto arow = [](int i) { return IMGS == 8 ? 8 * i : IMGS == 2 && i >= 2 ? 2 * NP : 0; };
  auto compute = [&](int dy, int pbuf, const f16x8 (&bv)[TN][2]) {
    const _Float16* As = patch + pbuf * kWBuf + arow_base(dy) + dy * NP * kWRowH;
    f16x8 av[TM][2];
    av[0][0] = a0[0];
    av[0][1] = a0[1];
#pragma unroll
    for (int i = 1; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + (i * 16 + arow(i)) * kWRowH + p * 32);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {  // (B, A): the transposed tile, lane (l16, q) = couts 4 q .. 4 q + 3 of pair l16
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bv[j][0], av[i][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bv[j][1], av[i][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bv[j][0], av[i][0], acc[i][j], 0, 0, 0);
      }
      if (i == TM - 2 && dy + 1 < NTAP) read_a0(dy + 1, pbuf);
    }
  };

  // ---- shortcut steps (the ResBlock's 1x1 of x2, a second K segment; wino_pack_kernel): step s stages, per pair p
  // and 4-channel slot ks of the 32, nu 0 x2[2p][H1], nu 3 x2[2p + 1][H1], nu 1 / 2 x2[2p][H2] +/- x2[2p + 1][H2]
  // (H1 = channels 32 s + .., H2 = Cin2 / 2 + 32 s + ..) as pair rows [nu][64] of a patch buffer
  const int sp = t >> 3, sks = t & 7;
  auto load_sc = [&](int st) DM_WINO_INL {
    // (rows past M -- a W 8 group's missing second image -- read the last pair: their outputs are not stored)
    const int srow = min(m0 + 2 * sp, M - 2);  // (WIDE: the pair's first pixel of the tiled map; pairs stay in a row)
    const float* xs =
        a.x2 + (WIDE ? t2d_pixel(srow, HW, Wimg, RIMG, W) : (size_t)srow) * a.x2_pitch + (sb + st) * kWC + 4 * sks;
    rw[0] = *reinterpret_cast<const f4*>(xs);
    rw[1] = *reinterpret_cast<const f4*>(xs + a.x2_pitch);
    rw[2] = *reinterpret_cast<const f4*>(xs + a.Cin2 / 2);
    rw[3] = *reinterpret_cast<const f4*>(xs + a.x2_pitch + a.Cin2 / 2);
  };
  auto finish_sc = [&](int buf, int h) DM_WINO_INL {  // h 0: planes 0, 3 (H1); h 1: planes 1, 2 (H2)
    _Float16* dst = patch + buf * kWBuf + sp * kWRowH + 8 * ((sks >> 1) ^ wswz(sp)) + 4 * (sks & 1);  // (swizzled)
#pragma unroll
    for (int v2 = 0; v2 < 2; ++v2) {
      const int v = h ? 1 + v2 : 3 * v2;
      const f4 x = h ? (v2 ? rw[2] - rw[3] : rw[2] + rw[3]) : rw[v2];
      f16x4 hi, lo;
#pragma unroll
      for (int k = 0; k < 4; ++k) hi[k] = (_Float16)x[k];
      split_lo4(x, hi, lo);
      *reinterpret_cast<f16x4*>(dst + v * 64 * kWRowH) = hi;
      *reinterpret_cast<f16x4*>(dst + v * 64 * kWRowH + 32) = lo;
    }
  };
  // stage g of a tile: chunk g < nch, else shortcut step g - nch
  auto load_stage = [&](int g) DM_WINO_INL {
    if (!SC || g < nch) load_raw(g);
    else load_sc(g - nch);
  };
  auto finish_stage = [&](int g, int buf) DM_WINO_INL {
    if (!SC || g < nch) {
      finish(g, buf);
    } else {
      finish_sc(buf, 0);
      finish_sc(buf, 1);
    }
  };

  // GroupNorm tables of image b0 into LDS (scale, shift per channel, [c / 4][4 scales][4 shifts], times -log2(e)
  // under SiLU); the caller's barrier publishes them
  auto build_table = [&]() DM_WINO_INL {
    if (!PRO) return;
    const int C = tabc, c0 = cb * kWC;  // (KS: the block's channels c0 .. c0 + C - 1)
#pragma unroll
    for (int im = 0; im < IMGS; ++im) {
      const int bi = min(b0 + im, a.B - 1);  // (a group's image past B: any table, its rows are padding)
      float* tab = gtab + im * 2 * C;
      if (a.gin_part) {  // gn_finalize (gn.hip) for the image, its expressions (conv_k32's in-kernel finalize)
        const int G = a.gin_G, cpg = a.Cin1 / G;  // (the conv's groups: C is the block's share under KS)
        float* st = gstat + im * 2 * kWMaxG;
        for (int i = t; i < G; i += 512) {
          double s1 = 0, s2 = 0;
#pragma unroll 4
          for (int k = 0; k < a.gin_nchunk; ++k) {  // (unrolled: the partials' loads in flight together)
            const double2 v = a.gin_part[((size_t)bi * a.gin_nchunk + k) * G + i];
            s1 += v.x;
            s2 += v.y;
          }
          const double mu = s1 / a.gin_n;
          double var = s2 / a.gin_n - mu * mu;
          if (var < 0) var = 0;
          st[2 * i] = (float)mu;
          st[2 * i + 1] = (float)(1.0 / sqrt(var + (double)a.gin_eps));
        }
        __syncthreads();
        for (int c = t; c < C; c += 512) {
          const int cg = c0 + c;
          const int si = 2 * (cg / cpg);
          const float mu = st[si], rs = st[si + 1];
          float sc = rs * (a.gin_gamma ? a.gin_gamma[cg] : 1.0f);
          float sh = -sc * mu + (a.gin_beta ? a.gin_beta[cg] : 0.0f);
          if (a.gin_ms) {
            const size_t mo = (size_t)bi * a.gin_mp + cg;
            const float f = 1.0f + a.gin_ms[mo];
            sc = sc * f;
            sh = sh * f + a.gin_mb[mo];
          }
          const int ti = 2 * c - (c & 3);
          tab[ti] = PROM == 2 ? sc * -1.4426950408889634f : sc;
          tab[ti + 4] = PROM == 2 ? sh * -1.4426950408889634f : sh;
        }
      } else {
        for (int c = t; c < C; c += 512) {
          const int ti = 2 * c - (c & 3);
          const size_t po = (size_t)bi * a.Cin1 + c0 + c;
          const float sc = a.pro_scale[po], sh = a.pro_shift[po];
          tab[ti] = PROM == 2 ? sc * -1.4426950408889634f : sc;
          tab[ti + 4] = PROM == 2 ? sh * -1.4426950408889634f : sh;
        }
      }
    }
  };

  // ---- first tile's prologue: B ring and the first chunk's pixels in flight while the GroupNorm tables are built.
  // The ring's last slot is requested after the second stage's pixels, as in the loop (pixels, then B refills): the
  // loop head's memory-counter waits, merged over the prologue and the loop's own back edge, then stay partial.
  int tile = t_first;
  set_tile(tile);
  if (WIDE) set_edges();
#pragma unroll
  for (int d = 0; d < WD - 1; ++d) load_b(bq[d], d);
  load_raw(0);
  if (WIDE) {
    load_edge(0, rw[2]);
    if (nch > 1) load_edge(1, rw[3]);
  }
  build_table();
  __syncthreads();
  if (WIDE) {  // chunks 0 and 1's halo columns (one barrier more, once per block)
    finish_edge(0, rw[2]);
    if (nch > 1) finish_edge(1, rw[3]);
    __syncthreads();
    if (nch > 2) load_edge(2, rw[2]);
  }
  finish(0, 0);
  load_stage(min(1, nst_g - 1));
  load_b(bq[WD - 1], WD - 1);
  __syncthreads();
  W_STAMP(1);
#ifdef DM_K32_STAMPS
  unsigned long long loop_cycles = 0, t_loop = 0, ew_cycles = 0, out_cycles = 0, np_cycles = 0, t_s = 0;
  int ntile_done = 0;
#define W_ACC(var)                                       \
  do {                                                   \
    const unsigned long long now = __builtin_amdgcn_s_memtime(); \
    var += now - t_s;                                    \
    t_s = now;                                           \
  } while (0)
  // per-role phases of the main loop (waves 0 and 4, the two roles of SIMD 0): first phase, second phase, barrier
  unsigned long long ph_t[4] = {0, 0, 0, 0}, ph_sum[3] = {0, 0, 0};
#define W_PH(k)                                                     \
  do {                                                              \
    ph_t[k] = __builtin_amdgcn_s_memtime();                         \
    if (k > 0) ph_sum[k - 1] += ph_t[k] - ph_t[k - 1];              \
  } while (0)
#else
#define W_ACC(var) do {} while (0)
#define W_PH(k) do {} while (0)
#endif
  // ping-pong of the two waves of each SIMD (waves w and w + 4): the early group finishes chunk c + 1 before chunk
  // c's MFMAs, the late group after them, so each wave's loader VALU runs beside its partner's MFMAs
  // (MI355X_MICROARCH.md, two waves per SIMD); each loads chunk c + 2's pixels right after its finish, a chunk ahead.
  // The two roles are separate copies of the loop (role_loop below): in one loop body with a branch per role the
  // compiler's memory-counter waits merge both load orders and wait for everything -- the early wave for the pixels
  // it has just requested before its first MFMA, the late wave for the B refills it has just issued before its finish.
  const bool late = wave >= 4;
  // ---- main loop: chunk c's three tap rows from buffer c & 1, chunk c + 1 finished into the other; one barrier
  // per chunk. Two chunks per iteration (CC: the B ring slots are compile-time), an odd last chunk after the loop --
  // not a skipped half inside it, whose path into the loop head would merge a second load order there as well
  auto chunk = [&](int c, auto cc_c, auto late_c) DM_WINO_INL {
    constexpr int CC = decltype(cc_c)::value;
    constexpr bool LATE = decltype(late_c)::value;
    // the next chunk's finish and the one after's pixel loads: skipped (a uniform branch) past the tile's last chunk
    const bool more = c + 1 < nch, more2 = c + 2 < nch;
    W_PH(0);
    if (!LATE) {
      if (more) finish(c + 1, (c + 1) & 1);
      if (more2) load_raw(c + 2);
      if (WIDE && more2) {  // (the edge waves) chunk c + 2's halo columns into slot c & 1, chunk c + 3's pixels
        finish_edge(c + 2, rw[2]);
        if (c + 3 < nch) load_edge(c + 3, rw[2]);
      }
      W_PH(1);
    }
    if (LATE) __builtin_amdgcn_s_setprio(1);  // the late role's MFMAs at priority 1 (its finish back at 0)
#pragma unroll
    for (int dy = 0; dy < NTAP; ++dy) {
      const int kt = c * NTAP + dy;
      const int slot = (CC * NTAP + dy) % WD;
      if (dy == 0) {
        read_a0(0, c & 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      compute(dy, c & 1, bq[slot]);
      load_b(bq[slot], kt + WD);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (LATE) {
      __builtin_amdgcn_s_setprio(0);
      W_PH(1);
      if (more) finish(c + 1, (c + 1) & 1);
      if (more2) load_raw(c + 2);
    }
    W_PH(2);
    __syncthreads();
    W_PH(3);
  };
  typedef std::integral_constant<int, 0> Cc0;
  typedef std::integral_constant<int, 1> Cc1;
  auto role_loop = [&](auto late_c) DM_WINO_INL {
    int c0 = 0;
    for (; c0 + 1 < nch; c0 += 2) {
      chunk(c0, Cc0{}, late_c);
      chunk(c0 + 1, Cc1{}, late_c);
    }
    if (c0 < nch) chunk(c0, Cc0{}, late_c);
  };
  // ---- the shortcut steps: stage g = nch + s from buffer g & 1, one K step each (ring slot CC, after the swap below)
  auto sc_step = [&](int st, auto cc_c, auto late_c) DM_WINO_INL {
    constexpr int CC = decltype(cc_c)::value;
    constexpr bool LATE = decltype(late_c)::value;
    const int g = nch + st, buf = g & 1;
    const bool more = st + 1 < ns, more2 = st + 2 < ns;
    if (!LATE) {
      if (more) {
        finish_sc(buf ^ 1, 0);  // stage g + 1: a shortcut step (its pixels loaded a stage ahead)
        finish_sc(buf ^ 1, 1);
      }
      if (more2) load_sc(st + 2);
    }
    const _Float16* As = patch + buf * kWBuf + nu * 64 * kWRowH + abase_sc;
    a0[0] = *reinterpret_cast<const f16x8*>(As);
    a0[1] = *reinterpret_cast<const f16x8*>(As + 32);
    __builtin_amdgcn_sched_barrier(0);
    f16x8 av[TM][2];
    av[0][0] = a0[0];
    av[0][1] = a0[1];
#pragma unroll
    for (int i = 1; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) av[i][p] = *reinterpret_cast<const f16x8*>(As + i * 16 * kWRowH + p * 32);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[CC][j][0], av[i][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[CC][j][1], av[i][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq[CC][j][0], av[i][0], acc[i][j], 0, 0, 0);
      }
    load_b(bq[CC], kt_end + st + WD);
    __builtin_amdgcn_sched_barrier(0);
    if (LATE) {
      if (more) {
        finish_sc(buf ^ 1, 0);
        finish_sc(buf ^ 1, 1);
      }
      if (more2) load_sc(st + 2);
    }
    __syncthreads();
  };
  auto sc_loop = [&](auto late_c) DM_WINO_INL {
    int s0 = 0;
    for (; s0 + 1 < ns; s0 += 2) {
      sc_step(s0, Cc0{}, late_c);
      sc_step(s0 + 1, Cc1{}, late_c);
    }
    if (s0 < ns) sc_step(s0, Cc0{}, late_c);
  };
  for (;;) {
#ifdef DM_K32_STAMPS
    t_loop = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    if (late) role_loop(std::true_type{});
    else role_loop(std::false_type{});
    // ---- the shortcut steps; the ring slot of step kt is kt & 1 (WD 2): after an odd number of tap rows the two
    // slots trade places
    if (SC && ns > 0) {
      // its first step staged here (the main loop ends with every wave past its last read of buffer nch & 1)
      load_sc(0);
      finish_sc(nch & 1, 0);
      finish_sc(nch & 1, 1);
      load_sc(min(1, ns - 1));
      __syncthreads();
      if (kt_end & 1) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const f16x8 tmp = bq[0][j][p];
            bq[0][j][p] = bq[1][j][p];
            bq[1][j][p] = tmp;
          }
      }
      if (late) sc_loop(std::true_type{});
      else sc_loop(std::false_type{});
    }
#ifdef DM_K32_STAMPS
    t_s = __builtin_amdgcn_s_memtime();
    loop_cycles += t_s - t_loop;
    ++ntile_done;
#endif

    // the output lane's row scales (couts n0 + (wave & 1) 64 + 4 (lane % 16) ..): loaded under the E stores
    const f4 cs4 = *reinterpret_cast<const f4*>(a.wino_rowscale + n0 + (wave & 1) * 64 + 4 * (lane & 15)) *
                   (PROM == 2 ? -0.6931471805599453f : 1.0f);
    // ---- epilogue: the m_nu tiles to LDS planes [nu][ch][64 pairs][kWEP] (16-B stores: the accumulators are the
    // transposed tile); the row scale (times -ln 2 under SiLU) is applied after the output transform
    float* E = reinterpret_cast<float*>(smem);
    {
      float* dst = E + (nu * 2 + ch) * 64 * kWEP + l16 * kWEP + 4 * q;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) *reinterpret_cast<f4*>(dst + i * 16 * kWEP + j * 16) = acc[i][j];
    }
    // the next tile's first pixels and B ring in flight during this tile's epilogue
    const int cm0 = m0, cn0 = n0, cb0 = b0;
    const int next = tile + 1;
    const bool has_next = next < t_end;
    if (has_next) {
      set_tile(next);
      load_raw(0);
      if (WIDE) {
        set_edges();
        load_edge(0, rw[2]);
        if (nch > 1) load_edge(1, rw[3]);
      }
#pragma unroll
      for (int d = 0; d < WD - 1; ++d) load_b(bq[d], d);
    }
    __syncthreads();
    W_ACC(ew_cycles);
    // wave (chunk k, half hf, column half cj): output pixels 64 k + 32 hf .. + 31 of the tile = pairs 32 k + 16 hf ..,
    // pixel 2 p + s of pair p: y0 = (m0 + m1) + m2, y1 = (m1 - m2) - m3
    if (KS) {  // raw partial sums (the row scale undone) to kpart[split]; the reduction adds the epilogue
      const int kq = wave >> 2, hf = (wave >> 1) & 1, cj = wave & 1;
      const int c4 = lane & 15, rsub = lane >> 4;  // 4 columns of a pair row, 4 pair rows per wave instruction
      const int px0 = 64 * kq + 32 * hf, ncol = cn0 + cj * 64 + 4 * c4;
      const float* Ec = E + cj * 64 * kWEP + 4 * c4;
      float* kp = a.kpart + (size_t)split * M * N + ncol;
      f4 fin = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int i = 4 * it + rsub, pp = (px0 >> 1) + i;
        const f4 mv0 = *reinterpret_cast<const f4*>(Ec + (0 * 2 * 64 + pp) * kWEP);
        const f4 mv1 = *reinterpret_cast<const f4*>(Ec + (1 * 2 * 64 + pp) * kWEP);
        const f4 mv2 = *reinterpret_cast<const f4*>(Ec + (2 * 2 * 64 + pp) * kWEP);
        const f4 mv3 = *reinterpret_cast<const f4*>(Ec + (3 * 2 * 64 + pp) * kWEP);
        const f4 y0 = ((mv0 + mv1) + mv2) * cs4, y1 = ((mv1 - mv2) - mv3) * cs4;
        fin += y0 + y1;
        const int m = cm0 + px0 + 2 * i;  // (m even, M even: both pixels or neither)
        if (m < M) {
          *reinterpret_cast<f4*>(kp + (size_t)m * N) = y0;
          *reinterpret_cast<f4*>(kp + (size_t)(m + 1) * N) = y1;
        }
      }
      if (!__builtin_isfinite(fin[0] + fin[1] + fin[2] + fin[3]) && a.range_flag) *a.range_flag = 1;
    } else {
      const int kq = wave >> 2, hf = (wave >> 1) & 1, cj = wave & 1;
      typedef StagedEpilogue<64> Epi;
      Epi epi(a, M, HW, cb0, IMGS == 1, cn0 + cj * 64, lane);
      if (WIDE) epi.t2d(Wimg, RIMG, W);  // (tile rows -> pixels; GroupNorm chunks = tile halves)
      const int px0 = 64 * kq + 32 * hf;
      const float* Ec = E + cj * 64 * kWEP + 4 * epi.c4;
      f4 fin = {0.f, 0.f, 0.f, 0.f};  // inf / NaN in any m (an operand past fp16's range) makes fin non-finite
      epi.pairs_f(
          [&](int i, f4& y0, f4& y1) {
            const int pp = (px0 >> 1) + i;
            const f4 mv0 = *reinterpret_cast<const f4*>(Ec + (0 * 2 * 64 + pp) * kWEP);
            const f4 mv1 = *reinterpret_cast<const f4*>(Ec + (1 * 2 * 64 + pp) * kWEP);
            const f4 mv2 = *reinterpret_cast<const f4*>(Ec + (2 * 2 * 64 + pp) * kWEP);
            const f4 mv3 = *reinterpret_cast<const f4*>(Ec + (3 * 2 * 64 + pp) * kWEP);
            y0 = ((mv0 + mv1) + mv2) * cs4;
            y1 = ((mv1 - mv2) - mv3) * cs4;
            fin += y0 + y1;
          },
          cm0 + px0);
      if (!__builtin_isfinite(fin[0] + fin[1] + fin[2] + fin[3]) && a.range_flag) *a.range_flag = 1;
      if (a.gn_part) {  // the 64-pixel chunk's two halves: the hf = 1 wave's quad sums via LDS to the hf = 0 wave
        double s, qq;
        epi.quad_sums(s, qq);
        double* xr = gxr + (kq * 2 + cj) * 16 * 2;
        if (hf == 1 && lane < Epi::LPR) {
          xr[2 * lane] = s;
          xr[2 * lane + 1] = qq;
        }
        __syncthreads();
        if (hf == 0) {
          s += xr[2 * (lane % Epi::LPR)];
          qq += xr[2 * (lane % Epi::LPR) + 1];
          epi.store_quads(s, qq, cm0 + 64 * kq);
        }
      }
    }
    W_ACC(out_cycles);
    if (!has_next) break;
    // ---- the next tile's prologue: its first chunk (the E planes are dead after this barrier; same image: same
    // GroupNorm tables, which sit outside the E planes)
    tile = next;
    if (WIDE) {  // the next tile's chunks 0 and 1 halo columns (the edge buffer lies outside the E planes)
      finish_edge(0, rw[2]);
      if (nch > 1) finish_edge(1, rw[3]);
    }
    __syncthreads();
    if (WIDE && nch > 2) load_edge(2, rw[2]);
    finish(0, 0);
    load_stage(min(1, nst_g - 1));
    load_b(bq[WD - 1], WD - 1);
    __syncthreads();
    W_ACC(np_cycles);
  }
#ifdef DM_K32_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 65536) {
    g_wino_stamps[blockIdx.x][2] = loop_cycles;
    g_wino_stamps[blockIdx.x][4] = ntile_done;
    g_wino_stamps[blockIdx.x][8] = ew_cycles;
    g_wino_stamps[blockIdx.x][9] = out_cycles;
    g_wino_stamps[blockIdx.x][10] = np_cycles;
  }
  if ((threadIdx.x == 0 || threadIdx.x == 256) && blockIdx.x < 65536) {
    const int o = threadIdx.x ? 14 : 11;
    g_wino_stamps[blockIdx.x][o] = ph_sum[0];
    g_wino_stamps[blockIdx.x][o + 1] = ph_sum[1];
    g_wino_stamps[blockIdx.x][threadIdx.x ? 7 : 13] = ph_sum[2];
  }
#endif
  W_STAMP(3);
  W_RSTAMP(6);
}

template <int W, int PROM, bool SC>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) conv_wino_kernel(ConvArgs a) {
  conv_wino_body<W, PROM, SC, false>(a);
}
// 2-D tiles of maps wider than 32 columns (4 x 32-pixel tiles, halo columns from neighbouring tiles)
template <int PROM, bool SC>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) conv_wino_wide_kernel(ConvArgs a) {
  conv_wino_body<32, PROM, SC, true>(a);
}

// U = G g per (nu, output channel, chunk, tap row, channel of the chunk) from the packed 3x3 weights [Cout][K]
// (K = 9 Cin1 chunk-major, conv_k32's order, + Cin2 of the ResBlock shortcut): [4][Cout][3 Cin1 + Cin2 / 2] in the
// same chunk-major order with 3 taps, float64 sums rounded once to fp32. The shortcut (y += Ws x2 per pixel) in the
// pair domain: with its channels in halves H1, H2, nu 0 takes Ws_H1 x2[2j] (y0 only), nu 3 -Ws_H1 x2[2j + 1] (y1 only),
// nu 1 / 2 Ws_H2 / 2 against x2[2j] +/- x2[2j + 1] (y0 = m1 + m2, y1 = m1 - m2): Cin2 / 2 more K per GEMM, balanced;
// times -log2(e) when the main segment's SiLU constant is folded into the epilogue (fold).
__global__ void wino_pack_kernel(const float* w, int Cout, int K, int Cin1, int Cin2, int fold, float* out) {
  const int Kp = 3 * Cin1 + Cin2 / 2;
  const long total = 4L * Cout * Kp;
  const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= total) return;
  const int k = id % Kp;
  const long r = id / Kp;
  const int co = r % Cout, nu = r / Cout;
  double u;
  if (k < 3 * Cin1) {
    const int c = k / (3 * kWC), rem = k - c * 3 * kWC, dy = rem / kWC, ci = rem - dy * kWC;
    const float* src = w + (size_t)co * K + (size_t)(c * 9 + dy * 3) * kWC + ci;
    const double g0 = src[0], g1 = src[kWC], g2 = src[2 * kWC];
    switch (nu) {
      case 0: u = g0; break;
      case 1: u = (g0 + g1 + g2) * 0.5; break;
      case 2: u = (g0 - g1 + g2) * 0.5; break;
      default: u = g2; break;
    }
  } else {
    const int i = k - 3 * Cin1, hh = Cin2 / 2;
    const float* src = w + (size_t)co * K + 9 * Cin1;
    u = nu == 0 ? (double)src[i] : nu == 3 ? -(double)src[i] : 0.5 * (double)src[hh + i];
    if (fold) u *= -1.4426950408889634074;  // 1 / (-ln 2)
  }
  out[id] = (float)u;
}

}  // namespace

#ifdef DM_K32_STAMPS
extern "C" int dm_debug_wino_stamps(void* host, int nblocks) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wino_stamps), (size_t)nblocks * 16 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -2;
}
#endif

bool conv_wino_shape_ok(const ConvArgs& a) {
  if (!(a.taps == 9 && a.stride == 1 && a.upsample == 0)) return false;
  if (a.Hin != a.Hout || a.Win != a.Wout) return false;
  // 32- or 16-wide maps in whole-row 128-pixel tiles; 8 x 8 maps two images per tile, 4 x 4 maps eight (split-K: 2 ..
  // Cin1 / 32 splits, their partial sums in kpart); wider maps (a multiple of 32 columns, of 4 rows) in 4 x 32 tiles
  const bool w4 = a.Wout == 4;
  if (w4 ? !(a.Hout == 4 && a.ksplit >= 2 && a.ksplit <= a.Cin1 / kWC && a.kpart &&
             (reinterpret_cast<uintptr_t>(a.kpart) & 15) == 0)
         : a.ksplit > 1)
    return false;
  const int imgs = a.Wout == 8 ? 2 : w4 ? 8 : 1;
  const bool wide = a.Wout > 32;
  if (wide ? (a.Wout % 32 != 0 || a.Hout % 4 != 0)
           : a.Wout == 8 ? a.Hout != 8
           : w4          ? false
                         : ((a.Wout != 32 && a.Wout != 16) || (a.Hout * a.Wout) % 128 != 0))
    return false;
  const int tabc = w4 ? ceil_div(a.Cin1 / kWC, a.ksplit) * kWC : a.Cin1;  // GroupNorm table channels of a block
  if (a.Cin1 < kWC || a.Cin1 % kWC != 0 || 2 * imgs * tabc > kWTab || a.Cin2 % (2 * kWC) != 0 ||
      a.K != 9 * a.Cin1 + a.Cin2)
    return false;
  if (a.x1_pitch + a.Cin1 > kZeroPageFloats) return false;  // the loader's padding rows read the zero page
  if (a.Cin2 && (!a.x2 || a.x2_pitch % 4 != 0 || (reinterpret_cast<uintptr_t>(a.x2) & 15) != 0)) return false;
  if (a.Cout % 128 != 0) return false;
  if (a.gin_part && (a.gin_G <= 0 || a.gin_G > kWMaxG || a.Cin1 % a.gin_G != 0)) return false;
  if (w4) {  // the epilogue runs in conv_splitk_reduce (its GroupNorm statistics: one chunk per image)
    ConvArgs e = a;
    e.gn_part = nullptr;
    return staged_epilogue_ok(e) && a.Cout % 4 == 0 &&
           (!a.gn_part || (a.gn_G > 0 && a.Cout % a.gn_G == 0 && a.Cout <= 1024));
  }
  return staged_epilogue_ok(a);
}

// the shortcut weights carry the SiLU fold of the epilogue iff the main segment's prologue has the SiLU
static bool wino_fold_of(const ConvArgs& a) { return (a.pro_scale || a.gin_part) && !a.pro_nosilu; }

bool conv_wino_ok(const ConvArgs& a) {
  return a.wino_ws && a.wino_rowscale && conv_wino_shape_ok(a) && (a.Cin2 == 0 || a.wino_fold == (int)wino_fold_of(a));
}

size_t wino_weights_bytes(int Cout, int Cin1, int Cin2) { return split_conv_weights_bytes(4, Cout, 3 * Cin1 + Cin2 / 2, 2); }

const float* wino_rowscale(const void* ws, int Cout, int Cin1, int Cin2) {
  return split_conv_rowscale(ws, 4, Cout, 3 * Cin1 + Cin2 / 2);
}

int wino_weights(const float* w, int Cout, int Cin1, int Cin2, int fold, void* out, hipStream_t st) {
  DM_REQUIRE(w && out && Cout > 0 && Cin1 > 0 && Cin1 % kWC == 0 && Cin2 >= 0 && Cin2 % (2 * kWC) == 0,
             "winograd weights: Cin must be a multiple of 32, the shortcut's a multiple of 64");
  const int Kp = 3 * Cin1 + Cin2 / 2;
  const long n = 4L * Cout * Kp;
  float* tmp = nullptr;  // plan-build time only: synchronous
  DM_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&tmp), n * sizeof(float)));
  hipLaunchKernelGGL(wino_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, Cout, 9 * Cin1 + Cin2,
                     Cin1, Cin2, fold, tmp);
  int rc = hipGetLastError() == hipSuccess ? DM_OK : DM_ERR_HIP;
  if (rc == DM_OK) rc = split_conv_weights(tmp, 4, Cout, Kp, Cin1, 3, 2, out, st);
  if (hipStreamSynchronize(st) != hipSuccess && rc == DM_OK) rc = DM_ERR_HIP;
  (void)hipFree(tmp);
  if (rc == DM_ERR_HIP) set_error("winograd weights: kernel launch failed");
  return rc;
}

std::string conv_wino_label(const ConvArgs& a) {
  const int prom = (a.pro_scale || a.gin_part) ? (a.pro_nosilu ? 1 : 2) : 0;
  if (a.Wout > 32) return std::string("conv_wino_wide_kernel<") + std::to_string(prom) + (a.Cin2 ? ",true>" : ",false>");
  return std::string("conv_wino_kernel<") + std::to_string(a.Wout) + "," + std::to_string(prom) + (a.Cin2 ? ",true>" : ",false>");
}

int conv2d_wino(const ConvArgs& a, hipStream_t st) {
  DM_REQUIRE(conv_wino_ok(a), "conv: shape not supported by the Winograd F(2,3) kernel");
  // persistent blocks over one image's tiles: parts per image = the smallest divisor of its tile count that gives
  // at least one block per CU (B = 256 at CIFAR size: one block per image)
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
  }
  // image groups (two 8 x 8 / eight 4 x 4 images per tile; the 4 x 4 maps split-K)
  const int imgs = a.Wout == 8 ? 2 : a.Wout == 4 ? 8 : 1, groups = ceil_div(a.B, imgs);
  const int ks = a.Wout == 4 ? a.ksplit : 1;
  const int tpi = (imgs * a.Hout * a.Wout / 128) * (a.Cout / 128);
  int parts = tpi;
  for (int p = 1; p <= tpi; ++p)
    if (tpi % p == 0 && (long)groups * p * ks >= ncu) {
      parts = p;
      break;
    }
  const int blocks = ks * groups * parts;
  const int prom = (a.pro_scale || a.gin_part) ? (a.pro_nosilu ? 1 : 2) : 0;
#define DM_WINO_LAUNCH(W_, P_)                                                                              \
  if (a.Wout == W_ && prom == P_) {                                                                         \
    if (a.Cin2) hipLaunchKernelGGL((conv_wino_kernel<W_, P_, true>), dim3(blocks), dim3(512), 0, st, a);       \
    else hipLaunchKernelGGL((conv_wino_kernel<W_, P_, false>), dim3(blocks), dim3(512), 0, st, a);             \
    note_launch(a.Cin2 ? "conv_wino_kernel<" #W_ "," #P_ ",true>" : "conv_wino_kernel<" #W_ "," #P_ ",false>"); \
  }
  DM_WINO_LAUNCH(32, 0) DM_WINO_LAUNCH(32, 1) DM_WINO_LAUNCH(32, 2)
  DM_WINO_LAUNCH(16, 0) DM_WINO_LAUNCH(16, 1) DM_WINO_LAUNCH(16, 2)
  DM_WINO_LAUNCH(8, 0) DM_WINO_LAUNCH(8, 1) DM_WINO_LAUNCH(8, 2)
  DM_WINO_LAUNCH(4, 0) DM_WINO_LAUNCH(4, 1) DM_WINO_LAUNCH(4, 2)
#undef DM_WINO_LAUNCH
#define DM_WINO_WIDE(P_)                                                                                     \
  if (a.Wout > 32 && prom == P_) {                                                                          \
    if (a.Cin2) hipLaunchKernelGGL((conv_wino_wide_kernel<P_, true>), dim3(blocks), dim3(512), 0, st, a);       \
    else hipLaunchKernelGGL((conv_wino_wide_kernel<P_, false>), dim3(blocks), dim3(512), 0, st, a);             \
    note_launch(a.Cin2 ? "conv_wino_wide_kernel<" #P_ ",true>" : "conv_wino_wide_kernel<" #P_ ",false>");         \
  }
  DM_WINO_WIDE(0) DM_WINO_WIDE(1) DM_WINO_WIDE(2)
#undef DM_WINO_WIDE
  DM_LAUNCH_CHECK();
  if (ks > 1) return conv_splitk_reduce(a, st);
  return DM_OK;
}

}  // namespace dm
