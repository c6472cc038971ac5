// Internal kernel entry points (host-side launchers). The public C ABI in
// include/dm_hip.h wraps these.
#pragma once
#include <cstdlib>
#include <string>
#include "dm_common.h"

namespace dm {

constexpr int kGnPixPerChunk = 64;

// Plan toggles: the environment, read ONCE per plan build (refresh_toggles(): the UNet / DiT plan builders and the
// direct-launch ABI entry points call it), so every decision of one plan -- and the label each op is profiled
// under -- comes from one snapshot. Each keeps the path it replaces as a test oracle / A/B arm.
constexpr int kAttnNoProj = 1, kAttnFused = 2, kAttnUnfused = 5;  // Toggles::attn oracle modes (DM_ATTN=noproj|fused|unfused)
struct Toggles {
  int conv_math = 2;          // DM_CONV_MATH=fp32|bf16x3: the conv / GEMM arithmetic (0 / 3; 2: fp16x2)
  bool range_check = true;    // DM_RANGE_CHECK=0: no per-forward range flag check (and no fp32 re-run)
  bool graph = true;          // DM_NO_GRAPH: launch the plan op by op instead of as a hipGraph
  bool wino = true;           // DM_CONV_WINO=0: the 3x3 convs of 32^2 / 16^2 maps on conv_k32 instead of conv_wino
  bool k32s_w4 = false;       // DM_K32S_W4=1: the small-map conv's 4-wave form (conv_k32 variant 12)
  bool k32_small = true;      // DM_CONV_K32S=0: split-K convs of <= 16-pixel maps as two launches (conv_k32 3 / 4)
  bool k32_s2 = true;         // DM_CONV_K32S2=0: stride-2 convs on conv_patch3 MODE 4 instead of conv_k32 variant 9
  bool k32_t2d = true;        // DM_CONV_K32T2=0: wide maps on 128-pixel row segments (variant 7), not 2-D tiles
  bool k32_8x = true;         // DM_K32_8X=0: 8^2 maps on 128 x 128 two-image tiles instead of 64-row tiles
  bool gn_fusion = true;      // DM_GN_FUSION=0: GroupNorm statistics by separate passes (no producer epilogues,
                              // no concat units, no first-conv statistics)
  int attn = 4;               // DM_ATTN: the attention path -- 4 (default) the folded single-head block on 8
                              // waves + flash / pre-split fused kernels elsewhere; 3 the folded block's 4-wave
                              // form; the unfolded oracles (no folding, no flash kernel): 0 "presplit" (q / k /
                              // v planes from the qkv epilogue, proj fused), kAttnNoProj, kAttnFused, kAttnUnfused
  bool attn_gn_launch = false;  // DM_ATTN_GNFIN=1: the folded block's GroupNorm finalize as its own launch
  bool attn_small = true;     // DM_ATTN_SMALL=0: the 4 x 4 single-head block unfolded (qkv / S / softmax / PV / proj
                              // launches) instead of attn_small_kernel
  bool dit_presplit = true;   // DM_DIT_PRESPLIT=0: DiT token GEMMs split their activations per tile
  bool lin_sk = true;         // DM_LIN_SK=0: no split-K of linear_k32's last, partial round of tiles
  bool lin_rows = true;       // DM_LIN_ROWS=0: the time MLP / temb projections on gemm_kernel instead of linear_rows
};
// The calling thread's snapshot: the innermost ToggleScope's (a plan's, while it is built, captured or replayed op by
// op), else the thread's last refresh_toggles(). Thread-local: plan builds in concurrent threads do not see each
// other's writes, and a plan's launch-time checks read the decisions of its own build, not whatever
// the environment or another call set since.
const Toggles& toggles();
void refresh_toggles();  // this thread's snapshot from the environment
const Toggles* toggle_scope_swap(const Toggles* t);
struct ToggleScope {
  const Toggles* prev;
  explicit ToggleScope(const Toggles& t) : prev(toggle_scope_swap(&t)) {}
  ~ToggleScope() { toggle_scope_swap(prev); }
  ToggleScope(const ToggleScope&) = delete;
  ToggleScope& operator=(const ToggleScope&) = delete;
};
// Launch log for tests (dm_debug_launch_log): the kernel instantiations the conv launchers issued, recorded in the
// branch that launches them
void note_launch(const char* name);

// Nominal batch of the plans' tile heuristics (ConvArgs::pick_B, GemmArgs::pick_M / pick_Z): every layer
// runs the kernel it would at B = kPickBatch, whatever B is, so each image's result is bit-identical at
// any batch size (the reference parity pinned at B = 1..2 holds at the benchmark's B). One exception, by
// design: linear_k32's split-K tail (GemmArgs::sk_*, DiT plans) re-associates the sums of the tiles in a
// launch's last partial round, so a DiT row agrees across batch sizes to fp32 re-association (DM_LIN_SK=0:
// bit for bit; tests/test_gpu_r3.py test_dit_xl2_cfg_batch64).
constexpr int kPickBatch = 256;

struct ConvArgs {
  // segment 1: NHWC input view (channel pitch x1_pitch), source resolution Hin x Win
  const float* x1;
  int x1_pitch, Cin1, Hin, Win;
  int taps;      // 1 or 9
  int stride;    // 1 or 2
  int upsample;  // nearest 2x before a 3x3 stride-1 conv
  // segment 2 (optional): 1x1 product of x2 at output resolution
  const float* x2;
  int x2_pitch, Cin2;
  // packed weights [Cout][K], K = taps * Cin1 + Cin2
  const float* w;
  int K;
  // output
  float* y;
  int y_pitch, Cout, B, Hout, Wout;
  const float* bias;    // [Cout] or null
  const float* rowvec;  // [B][rowvec_pitch] per-image additive vector or null
  int rowvec_pitch;
  const float* res;     // residual at output resolution or null
  int res_pitch;
  int tile;      // 0 auto; 1..3 force an im2col tile, 4..6 a halo-patch tile
  int pick_B;           // batch the tile heuristics assume (0: B). Plans pass a fixed one, so a layer's
                        // kernel (and its summation order) never changes with B: batch-invariant results
  // optional operand prologue on segment 1 (halo-patch kernel only):
  // x -> silu(x * pro_scale[b][c] + pro_shift[b][c]) before the product
  // (GroupNorm + SiLU of the ResBlock, fused into the conv's input load)
  const float* pro_scale;
  const float* pro_shift;
  int pro_nosilu;  // 1: the prologue is the affine alone (no SiLU)
  // optional: the kernel computes its GroupNorm prologue tables itself from gn_partial-layout statistics
  // of x1 ([B][gin_nchunk][gin_G] {sum, sumsq}), exactly as gn_finalize would (same expressions), into
  // LDS; the finalize launch is skipped. Only where conv_lds_tables() holds.
  const double2* gin_part;
  int gin_G, gin_nchunk;
  double gin_n;
  float gin_eps;
  const float *gin_gamma, *gin_beta, *gin_ms, *gin_mb;
  int gin_mp;
  // split-K over input-channel chunks (halo-patch kernel, MODE 0/1): ksplit > 1 writes raw partial
  // sums to kpart [ksplit][M][Cout] and a reduction pass sums them in split order and applies the
  // epilogue. The split count is fixed per layer shape (not per batch), so results stay batch-invariant.
  int ksplit;
  float* kpart;
  // optional GroupNorm statistics of the stored output for the consumer's GroupNorm(G) over this
  // view's Cout channels (cpg = Cout / G): per (image, 64-pixel chunk, group) {sum, sum of squares}
  // in the gn_partial layout [B][nchunk][G], so the consumer skips its gn_partial pass.
  // Used when HW % 64 == 0 and the tile's waves own 64 rows (halo-patch MODE 0, 128-row tiles).
  double2* gn_part;
  int gn_G;
  // optional split copy of w (split_conv_weights): halo-patch shapes then run conv_patch3_kernel with
  // fp32-accurate products on the 16-bit matrix cores. ws_np 3: [matrix][K / 16][Cout][48] bf16
  // (three-way bf16 split); ws_np 2: [matrix][K / 16][Cout][32] fp16 (two-way fp16 split of the
  // weights scaled by ws_rowscale[-Cout + n]; ws_rowscale[n] is the epilogue's inverse scale)
  const void* ws;
  int ws_np;
  const float* ws_rowscale;
  // optional device flag, set to 1 when an fp16x2 conv meets an activation beyond the fp16 range
  int* range_flag;
  // attention operand planes (MODE 3 qkv conv feeding attn_fused): instead of y, the epilogue writes
  // q * alpha * 2^ea and k * b_scale * 2^eb as fp16x2 planes [B][heads][2][L][Dh] and v * 2^ev
  // transposed, [B][heads][2][Dh][L] (plane 0 = fp16(x), plane 1 = fp16(x - plane 0)): the split the
  // attention GEMMs would do on load, done once by the producer. Columns: q | k | v blocks of C, or
  // per head [q; k; v] (ap_legacy, QKVAttentionLegacy).
  _Float16 *ap_q, *ap_k, *ap_v;
  int ap_L, ap_heads, ap_Dh, ap_legacy;
  float ap_alpha, ap_bscale;
  int ap_ea, ap_eb, ap_ev;
  // optional Winograd F(2,3) weights (conv_wino.hip, wino_weights): U = G g of the 3x3 taps, fp16x2 fragment
  // images of 4 matrices [Cout][3 Cin1] with their inverse row scales; set, the conv runs conv_wino_kernel
  const void* wino_ws;
  const float* wino_rowscale;
  int wino_fold;  // the shortcut segment's weights were packed with the SiLU fold (wino_weights fold = 1)
  // the K32 variant the plan resolved at build time (conv_k32_pick + 1; 0: pick at launch), so the launch and the
  // op's profile label come from one decision
  int k32_resolved;
};

// Patch-pixel capacity of the halo-patch kernels' LDS images (fp32 / split-bf16; 128- / 64-row tiles)
constexpr int kPatchMax128 = 288;
constexpr int kPatchMax64 = 160;
constexpr int kPatch3Max128 = 208;
constexpr int kPatch3Max64 = 160;
// fp16x2 split kernel, one wave per SIMD with 128 x 128 wave tiles: 256 x 256 blocks (32^2 maps: 8 rows,
// 10 x 34 patch; 16^2: one image, 18 x 18) and 512 x 128 blocks (32^2: 16 rows, 18 x 34; 16^2: two images)
constexpr int kPatch3Max256 = 352;
// fp16x2 split kernel, 128 x 128 blocks over 128-pixel row segments of wide maps (ADM 256^2 / 128^2):
// 3 x 130 patch pixels
constexpr int kPatch3Seg = 392;
constexpr int kSegTabFloats = 2048;  // its GroupNorm tables (one image, Cin <= 1024)
constexpr int kPatch3Max512 = 656;
constexpr int kPatchS2Max = 384;  // stride-2 split conv (64-row tiles): (2 TH + 1) x 2 (Wo + 1) per image (3 loader passes)

// Output tile = TB images x TH rows x full width; input patch PH x PW per image.
// Halo-patch tile geometry: TB images x TH output rows x TW output columns per tile (TW = Wo for whole
// rows; TW < Wo: row segments of wide maps, TB = TH = 1), patch PH x PW pixels per image, P in total.
struct PatchGeom {
  int TB, TH, PH, PW, P, TW;
};

struct GemmArgs {
  int M, N, K;
  int Z1, Z2;
  long pick_M;  // M and Z1 * Z2 the tile heuristic assumes (0: the actual ones); plans pass values for a
  long pick_Z;  // fixed nominal batch so the kernel choice (and GN-statistics routing) is batch-invariant
  const float* A;
  long a_s1, a_s2;
  int lda;
  const float* Bm;
  long b_s1, b_s2;
  int ldb;
  int b_kn;  // 0: B stored [n][k]; 1: B stored [k][n]
  float* C;
  long c_s1, c_s2;
  int ldc;
  float alpha;          // multiplies A elements on load (rounded per element)
  float b_scale;        // nonzero: multiplies B elements on load ([n][k] layout only; ADM q*s, k*s)
  const float* bias;    // [N] or null
  const float* res;     // residual [M][ld_res] (batch 0 layout only) or null
  int ld_res;
  int act;              // 0 none, 1 SiLU, 2 GELU(tanh)
  // optional GroupNorm affine on A elements: a[m][k] * pro_scale[img][k] + pro_shift[img][k],
  // img = (z1 * M + m) / pro_rows (rows per image); fused norm of the attention block's input
  const float* pro_scale;
  const float* pro_shift;
  int pro_rows;
  // optional LayerNorm + adaLN modulate on A elements (DiT, models/dit/model.py:19-20, 120-121):
  // a = ((a - mean[m]) * rstd[m]) * (1 + ln_scale[img][k]) + ln_shift[img][k], img = m / ln_rows
  const float2* ln_stats;
  const float* ln_scale;
  const float* ln_shift;
  int ln_pitch, ln_rows;
  // optional gated residual epilogue: C = res + gate[img][n] * (acc + bias), img = m / gate_rows
  const float* gate;
  int gate_pitch, gate_rows;
  int res_mod;          // > 0: residual row = m % res_mod (broadcast table, e.g. DiT pos_embed)
  // optional GroupNorm statistics of the output (as ConvArgs::gn_part): rows = pixels of images of
  // gn_hw pixels each (gn_hw % 64 == 0), 128-row tiles, Z1 = Z2 = 1
  double2* gn_part;
  int gn_G, gn_hw;
  // split = 2: fp16x2 products (conv_patch3.hip's split, on the fly for both operands): A elements
  // (after the prologue / alpha) are scaled by 2^split_ea, B elements (after b_scale) by 2^split_eb,
  // both exact, split into two fp16 pieces each, three v_mfma_f32_32x32x16_f16 per product; the
  // accumulator is scaled back by 2^-(ea + eb). |scaled value| > 65504 sets range_flag.
  int split;
  int split_ea, split_eb;
  // optional pre-split weights (split = 2, [n][k] B, Z = 1): split_conv_weights' fragment images of Bm with
  // their inverse row scales; such GEMMs run linear_k32 (linear_k32.hip) and split_eb is unused
  const void* ws;
  const float* ws_rowscale;
  // linear_k32 only: pre-split A (linear_presplit_a's image of the prologue'd, alpha- and 2^split_ea-scaled
  // rows, [M][K / 32][piece][4 k-groups][8] fp16); the kernel then stages it into LDS without conversion
  // (pro_scale / ln_stats must be null: they are applied by the pre-split pass)
  const _Float16* as;
  // linear_k32 only: the output (after bias / residual / activation) as the next GEMM's pre-split A image
  // ([M][N / 32][piece][4][8] fp16 of out * 2^c_split_ea, as linear_presplit_a writes it) instead of C
  _Float16* c_split;
  int c_split_ea;
  // linear_k32 only: the attention operand planes instead of C (as ConvArgs::ap_*, the qkv projection
  // feeding attn_presplit_kernel)
  _Float16 *ap_q, *ap_k, *ap_v;
  int ap_vonly;   // every column is a v column (the folded attention's g^T plane; ap_q = ap_k = ap_v)
  int ap_L, ap_heads, ap_Dh, ap_legacy;
  float ap_alpha, ap_bscale;
  int ap_ea, ap_eb, ap_ev;
  int* range_flag;
  // linear_k32 only: split-K of the tiles of the last, partial round (the tile count modulo the resident
  // blocks, when at most half a round): sk_cap slabs of 128 x 128 fp32 and one arrival counter per tile
  // (zero before the first use; the reducing block resets it), owned by the caller. sk_S / sk_tdp are set by
  // linear_k32 itself (slices per tail tile, first tail tile).
  float* sk_ws;
  unsigned* sk_cnt;
  int sk_cap;
  int sk_S, sk_tdp;
};

struct StepArgs {
  int B, C, HW, Cm;
  const float* xt;
  const float* out_c;
  const float* out_u;   // CFG uncond branch or null
  float w_u, w_c;       // (1 - s), s
  int objective;        // 0 eps, 1 x0, 2 v
  int clip;
  float c_recip, c_recipm1, c_sa, c_s1ma;
  int kind;             // 0 DDIM, 1 DDPM
  float m1, m2;
  int var_mode;         // 0 scalar std, 1 learned range
  float std;
  float min_logvar, max_logvar;
  int add_noise;
  const float* noise;
  float* sample;
  float* mean_out;
  float* x0_out;
  float* eps_out;
  float* var_out;
  int euler;            // 1: Euler / Heun first order, 2: Heun second order (dm_step_desc)
  float e_st1, e_sig_t, e_dsig, e_sp1, e_sig_p;
  const float* e_d1;
  const float* e_x1;
  float* e_dout;
};

int gn_num_chunks(int HW);
int gn_partial(const View& x, int G, double2* part, hipStream_t st);
// partials of a concat [h (Ch) | skip (Cs)] from the slices' own G-group partials (group-aligned slices)
// slice partials with their own group counts (Gh over Ch, Gs over Cs) -> the concat's G groups
bool gn_concat_ok(int Ch, int Gh, int Cs, int Gs, int G);
int gn_concat_stats(const double2* ph, int Ch, int Gh, const double2* ps, int Cs, int Gs, int B, int HW, int G,
                    double2* out, hipStream_t st);
int gn_finalize(const View& x, int G, const double2* part, float eps, const float* gamma, const float* beta,
                float* scale, float* shift, hipStream_t st, const float* mod_scale = nullptr,
                const float* mod_shift = nullptr, int mod_pitch = 0);
// NHWC resampling (models/unet_categorial_adagn.py:24-27, models/adm/unet.py:73-160):
// y = avg_pool2d(pro(x), 2) (down) or nearest-2x(pro(x)) (up); pro = optional silu(x * scale + shift)
int resample2x(const View& x, const View& y, int down, const float* pro_scale, const float* pro_shift,
               hipStream_t st);
// out[b] = silu(temb[b] + table[y[b]]) (class embedding, unet_categorial_adagn.py:172-174);
// rows with y == null or y[b] < 0 use table[null_row] (DiT's CFG null class, dit/model.py:241-242),
// or no class term when null_row < 0 (no label / CFG unconditional branch of the UNets)
int embed_add_silu(const float* temb, const int64_t* y, const float* table, int B, int D, float* out,
                   hipStream_t st, int null_row = -1);
// LayerNorm statistics (no affine): stats[r] = (mean, 1 / sqrt(var + eps)) of each D-wide row
int row_stats(const float* x, long rows, int D, float eps, float2* stats, hipStream_t st);
// row_stats + LayerNorm + adaLN modulate + fp16x2 split of each row: the pre-split A image (GemmArgs::as)
int row_stats_split(const float* x, long rows, int D, float eps, float2* stats, const float* ln_shift,
                    const float* ln_scale, int ln_pitch, int ln_rows, int split_ea, _Float16* out, int* range_flag,
                    hipStream_t st);
// DiT patch embedding input: NCHW [B][C][H][W] -> rows [B * (H/p) * (W/p)][C * p * p] (Conv2d k = s = p order)
int patchify(const float* x, int B, int C, int H, int W, int p, float* out, hipStream_t st);
// DiT unpatchify (dit/model.py:219-232): rows [B * T][p * p * C] -> NCHW [B][C][H][W]
int unpatchify(const float* x, int B, int C, int H, int W, int p, float* out, hipStream_t st);
int gn_apply(const View& x, int G, const double2* part, int nchunk, float eps, const float* gamma,
             const float* beta, const float* mod_scale, const float* mod_shift, int mod_pitch, int act,
             const View& y, hipStream_t st);
int conv2d_igemm(const ConvArgs& a, hipStream_t st);
int conv_pick(const ConvArgs& a);
// whether the conv can emit GroupNorm(gn_G) statistics of its output from the epilogue
bool conv_can_emit_gn(const ConvArgs& a);
bool conv_patch_geom(const ConvArgs& a, int BM, PatchGeom& g);
int conv_patch_pick(const ConvArgs& a, PatchGeom& g);
int conv2d_patch(const ConvArgs& a, int which, const PatchGeom& g, hipStream_t st);
// split-bf16 halo-patch kernel (conv_patch3.hip): whether it takes this shape / tile, and its launcher
bool conv_patch3_ok(const ConvArgs& a, int which, const PatchGeom& g);
// 1x1 convs / static-weight GEMMs on the fp16x2 split kernel (conv_patch3_kernel MODE 3)
bool conv_pw_ok(const ConvArgs& a);
// whether the conv stages its GroupNorm prologue tables in LDS (and so can take ConvArgs::gin_* instead
// of finalized tables)
bool conv_lds_tables(const ConvArgs& a);
bool conv_split_eligible(const ConvArgs& a);
bool conv_seg_eligible(const ConvArgs& a);
int conv2d_patch3(const ConvArgs& a, int which, const PatchGeom& g, hipStream_t st);
// fp16x2 split conv with K = 32 steps on v_mfma_f32_16x16x32_f16 (conv_k32.hip): 3x3 stride-1 MODE 0
// shapes. conv_k32_pick -> variant 1 (128 x 128 tiles), 2 (128 x 64), 3 (64 x 64 split-K), 4 (64 x 128
// split-K) or 0 (not this kernel); forced by ConvArgs::tile 10..13, else it replaces conv_patch3's
// 128-row and split-K tiles unless DM_CONV_K32=0)
bool conv_k32_ok(const ConvArgs& a);
int conv_k32_variant_ok(const ConvArgs& a, int v);
int conv_k32_pick(const ConvArgs& a);
int conv2d_k32(const ConvArgs& a, int v, hipStream_t st);
std::string conv_k32_label(const ConvArgs& a, int v);
// Winograd F(2,3)-along-x 3x3 convs (conv_wino.hip): the shapes the kernel takes (32- / 16-wide maps, 128-pixel
// tiles, Cout % 128 == 0, a ResBlock shortcut segment of Cin2 % 64 == 0), whether a conv has its weights and shape, the
// weights (U = G g, float64, then the fp16x2 split of split_conv_weights with nmat 4, ntap 3; fold: the shortcut's
// weights times -log2(e), for convs whose prologue has the SiLU), their size / row scales, launcher
bool conv_wino_shape_ok(const ConvArgs& a);
bool conv_wino_ok(const ConvArgs& a);
size_t wino_weights_bytes(int Cout, int Cin1, int Cin2);
const float* wino_rowscale(const void* ws, int Cout, int Cin1, int Cin2);
int wino_weights(const float* w, int Cout, int Cin1, int Cin2, int fold, void* out, hipStream_t st);
std::string conv_wino_label(const ConvArgs& a);
int conv2d_wino(const ConvArgs& a, hipStream_t st);
// static-weight GEMM on pre-split weights with K = 32 MFMA steps (linear_k32.hip)
bool linear_k32_ok(const GemmArgs& g);
int linear_k32(const GemmArgs& g, hipStream_t st);
// resident linear_k32 blocks of the device (blocks per CU x CUs): the split-K tail's slab capacity
int linear_k32_slots();
// the pre-split A image of g (prologue, alpha, 2^split_ea, fp16x2 split; |value| > 65504 sets range_flag)
int linear_presplit_a(const GemmArgs& g, _Float16* out, hipStream_t st);
int conv_splitk_reduce(const ConvArgs& a, hipStream_t st);
// fp32 packed conv weights [nmat][rows][K] -> split slices for conv_patch3_kernel (np 3: bf16x3,
// np 2: fp16x2 + row scales); split_conv_rowscale gives ConvArgs::ws_rowscale of an fp16x2 copy
size_t split_conv_weights_bytes(int nmat, int rows, int K, int np);
const float* split_conv_rowscale(const void* ws, int nmat, int rows, int K);
int split_conv_weights(const float* w, int nmat, int rows, int K, int cin1, int ntap, int np, void* out,
                       hipStream_t st);
std::string conv_label(const ConvArgs& a);
// DM_CONV_MATH: fp16x2 (default) -> 2, bf16x3 -> 3, fp32 -> 0 (ConvArgs::ws_np of the model's convs), from the
// plan's toggle snapshot
inline int conv_math_from_env() { return toggles().conv_math; }
int gemm_batched(const GemmArgs& g, hipStream_t st);
// skinny fp32 linear (the time MLP / temb projections): C = act(A W^T + bias), W [n][k], no prologue / residual
bool linear_rows_ok(const GemmArgs& g);
int linear_rows(const GemmArgs& g, hipStream_t st);
// exponent e with max|x| * 2^e in [2^13, 2^14) (0 for all-zero x): fp16x2 operand scale of a weight
// matrix, computed once at plan build (synchronous)
int split_weight_exponent(const float* x, size_t n);
int gemm_pick(const GemmArgs& g);
std::string gemm_label(const GemmArgs& g);
int timestep_embed(const int64_t* t, int B, int dim, int kind, const float* freqs, float* out, hipStream_t st);
int softmax_rows(float* x, long rows, int L, int ld, hipStream_t st);

// Fused attention core (attention.hip): per (image, head) S = (alpha q)(b_scale k)^T, softmax rows,
// O = P v with S kept on the CU, fp16x2 split operands (exponents ea / eb for S, ep / ev for PV, as
// the split GEMMs). q / k / v of token i, head h: qkv[(b L + i) ld + {q0, k0, v0} + h hs + d].
struct AttnArgs {
  const float* qkv;
  int ld, L, Dh, heads, B;
  int q0, k0, v0, hs;
  float alpha, b_scale;
  float* out;  // out[(b L + i) ldo + h Dh + d]
  int ldo;
  int ea, eb, ep, ev;
  int* range_flag;
  // pre-split operand planes written by the qkv conv (ConvArgs::ap_*); when set, qkv is not read
  const _Float16 *pq, *pk, *pv;
  // one head of C channels (heads == 1): the attention output projection (a 1x1 MODE 3 conv with fp16x2
  // split weights, bias, residual, GroupNorm statistics) applied by the same kernel to its O rows, so O
  // never goes to HBM (`out` unused); proj.x1 is ignored
  int fuse_proj;
  ConvArgs proj;
  int proj_staged;  // set by attn_fused: proj runs the LDS-staged 16-B epilogue (staged_epilogue_ok)
  // flash kernel only: O written as the next GEMM's pre-split A image instead of fp32 rows (linear_k32 PRO 3:
  // [B L][o_ld / 32][piece][4][8] fp16 of O * 2^o_split_ea, linear_presplit_a's expressions; head h at
  // columns h Dh ..): the output projection reads it without a split pass
  _Float16* o_split;
  int o_split_ea, o_ld;
};
bool attn_fused_ok(int L, int Dh);
int attn_fused(const AttnArgs& a, hipStream_t st);
// Folded single-head attention block (attn_block.hip): T = xn At^T + w, S = T xn^T, P = softmax(S),
// y = x + Wg' (P xn) + cb (Wg = Wp Wv), GroupNorm statistics of y.
struct AttnBlockArgs {
  const float* x;               // [B][256][x_pitch] block input (NHWC rows)
  int x_pitch;
  const float *gsc, *gsh;       // [B][256] GroupNorm affine of x (gn_finalize)
  const _Float16* at_img;       // split_conv_weights image of At [256][256] (fp16x2)
  const float* at_rowscale;     // its row-scale undo (split_conv_rowscale)
  const float* w;               // [256] T bias
  const _Float16* wg_img;       // split_conv_weights image of Wg' (Wg, columns permuted: attn_perm_cols)
  const float* wg_rowscale;
  const float* cb;              // [256] output bias Wp bv + bp
  int variant;                  // 4 (default): 8 waves of 16 queries; 3: 4 waves of 32 (bit-identical)
  float* y;                     // [B][256][y_pitch]
  int y_pitch;
  double2* gn_part;             // optional GroupNorm(gn_G) chunk partials of y
  int gn_G;
  int B, ex, eg;
  int* range_flag;
  // variant 4: the GroupNorm affine of x from its chunk partials in the kernel (gn_finalize's expressions)
  // instead of gsc / gsh, when gin_part is set
  const double2* gin_part;
  int gin_G, gin_nchunk;
  const float *gin_gamma, *gin_beta;
  float gin_eps;
  // attn_small (4 x 4 maps): At and Wg transposed, fp32 [k][n] (attn_transpose); w, cb, x, y, gin_*, gn_* as above
  const float *at_t, *wg_t;
};
bool attn_block_ok(int L, int C, int heads);
bool attn_small_ok(int L, int C, int heads);
int attn_small(const AttnBlockArgs& a, hipStream_t st);
int attn_transpose(const float* src, float* dst, int C, hipStream_t st);
// at = s Wk^T Wq, w = s Wk^T bq, wg = Wp Wv, cb = Wp bv + bp (float64 sums, fp32 results)
int attn_fold(const float* wqkv, const float* bqkv, const float* wproj, const float* bproj, int C, double scale,
              float* at, float* w, float* wg, float* cb, hipStream_t st);
int attn_block(const AttnBlockArgs& a, hipStream_t st);
// wgp = wg with its columns permuted within 32-groups as attn_block variant 3 reads its projection operand
int attn_perm_cols(const float* wg, float* wgp, int C, hipStream_t st);
// Flash attention (attention.hip attn_flash_kernel) on pre-split planes for L % 64 == 0, head dims 8 .. 80:
// ADM's L = 1024 / 64 blocks, DiT's 72-wide heads. attn_fused dispatches there for shapes it does not take.
bool attn_flash_ok(int L, int Dh);
int attn_flash(const AttnArgs& a, hipStream_t st);
// first conv; with gn_part also the GroupNorm(G) chunk partials of its output (conv3x3_small_in_can_emit)
int conv3x3_small_in(const float* x, int B, int Cin, int H, int W, const float* w, const float* bias,
                     int Cout, const View& y, hipStream_t st, double2* gn_part = nullptr, int G = 0);
bool conv3x3_small_in_can_emit(int H, int W, int Cout, int G);
// last conv weights torch [Cout][Cin][3][3] -> [9][Cin][CO], CO = Cout rounded up to even (<= 8; zero-padded)
int small_out_pack(const float* w, int Cout, int Cin, float* wp, hipStream_t st);
// the prologue GroupNorm finalized in the kernel from the chunk partials (gn_finalize's expressions), instead of
// pro_scale / pro_shift tables: part [B][nchunk][G] {sum, sumsq}, n = HW * C / G elements per group
struct GnFin {
  const double2* part = nullptr;
  int G = 0, nchunk = 0;
  double n = 0;
  float eps = 1e-5f;
  const float *gamma = nullptr, *beta = nullptr;
};
int conv3x3_small_out(const View& x, const float* wp, const float* bias, int Cout, float* y, hipStream_t st,
                      const float* pro_scale = nullptr, const float* pro_shift = nullptr, const GnFin& fin = GnFin{});
int sampler_step(const StepArgs& s, hipStream_t st);
// out = c1 a + c2 b (mode 0), c1 a - c2 b (1), (c1 a - b) / c2 (2); per-row coefficients when c*_rows given
int lincomb(int mode, const float* a, const float* b, float* out, long n, long row_elems, const float* c1_rows,
            const float* c2_rows, float c1, float c2, hipStream_t st);
int nchw_to_nhwc(const float* x, int B, int C, int HW, float* y, int y_pitch, hipStream_t st);
int nhwc_to_nchw(const float* x, int B, int C, int HW, int pitch, float* y, hipStream_t st);
int repack_conv(const float* w, int Cout, int Cin, int taps, float* out, int ldw, int col0, hipStream_t st);
// torch 3x3 weight [Cout][Cin][3][3] -> sub-pixel upsample weights [4 parities][Cout][4 * Cin]
int repack_subpixel(const float* w, int Cout, int Cin, float* out, hipStream_t st);

}  // namespace dm
