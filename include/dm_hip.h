/*
 * dm_hip — MI355X-native denoising-step engine (C ABI).
 *
 * The reference (xyfJASON/diffusion-models-pytorch) has no native code and no
 * FFI: its hot path is two Python calls inside the sampling loop,
 *
 *   model_output = model(img, t_batch, **model_kwargs)   diffusions/ddpm.py:276
 *   out = self.denoise(model_output, img, t, t_prev)     diffusions/ddpm.py:277
 *                                                        (DDIM: diffusions/ddim.py:57-86,
 *                                                         CFG:  ddim.py:176-188, ddpm.py:334-348)
 *
 * This header is the boundary that replaces both. The Python host package
 * (`diffusions.*`, `models.unet.UNet`) binds it with ctypes; any other host
 * (C, C++, a cgo/JNI stub) can bind the same symbols — see INTEGRATION.md.
 *
 * Conventions
 *   - Every tensor argument is a raw device pointer to float32 (or int64 for
 *     timesteps / labels) owned by the caller; shapes are explicit ints.
 *     Images are NCHW contiguous, exactly the reference's torch layout.
 *   - `stream` is a hipStream_t passed as void*; all calls are asynchronous on
 *     that stream (NULL = the legacy default stream).
 *   - Return value: DM_OK (0) or a negative DM_ERR_* code; the message of the
 *     last failure on the calling thread is available from dm_last_error().
 *     DM_ERR_ARG corresponds to the reference's ValueError / assertion cases.
 *   - Objects (dm_unet) are not re-entrant: one stream at a time per object.
 */
#ifndef DM_HIP_H_
#define DM_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 1 (rounds 1-4); 2: dm_conv_desc gained w_wino / w_wino_fold at its end (a caller compiled against
 * version 1 passes the shorter struct, so the library refuses a binding that expects another version) */
#define DM_ABI_VERSION 2

#define DM_OK 0
#define DM_ERR_ARG (-1)
#define DM_ERR_HIP (-2)
#define DM_ERR_STATE (-3)
#define DM_ERR_UNSUPPORTED (-4)

/* Library / error handling ------------------------------------------------ */
int dm_abi_version(void);
/* "src=<16 hex> arch=gfx950": the first 16 hex digits of sha256 over the library's sources in build order
 * (csrc/Makefile SRC_HASH), so a caller can tell which sources a prebuilt library came from. */
const char* dm_build_info(void);
const char* dm_last_error(void);

/* Denoiser: DDPM UNet ------------------------------------------------------
 * Replaces models/unet.py:46-152 (UNet.__init__ / UNet.forward) with the
 * same hyper-parameters (configs/ddpm_cifar10.yaml:16-26) and the same
 * parameter list: `params` are the reference state_dict tensors in
 * state_dict() order (328 tensors for the CIFAR-10 config), `numels` their
 * element counts (validated). Weights are copied/packed into library-owned
 * device memory at create time; the caller's tensors may be freed afterwards.
 */
#define DM_MAX_STAGES 8
typedef struct dm_unet_arch {
  int in_channels;
  int out_channels;
  int dim;
  int n_stages;
  int dim_mults[DM_MAX_STAGES];
  int use_attn[DM_MAX_STAGES];
  int num_res_blocks;
  int n_heads;          /* variant 0: heads of the stage attention blocks */
  /* variant 0: models/unet.py UNet (time-embedding add after conv1, conv down/upsample);
   * variant 1: models/unet_categorial_adagn.py UNetCategorialAdaGN (AdaGN before conv2,
   *            heads = C / attn_head_dims, ResBlock up/down when resblock_updown, class embedding) */
  int variant;
  int num_classes;      /* variants 1, 2: class-embedding rows (0 = no class embedding) */
  int attn_head_dims;   /* variant 1; variant 2: num_head_channels (<= 0: use n_heads / n_heads_up) */
  int resblock_updown;  /* variants 1, 2 */
  /* variant 2: models/adm/unet.py UNetModel (first conv to dim * dim_mults[0] channels, [cos, sin]
   * embedding, fused qkv 1x1 conv, q and k each scaled by ch^-1/4, middle attention with the stage
   * head rule). dim = model_channels, dim_mults = channel_mult, use_attn[l] = (2^l in
   * attention_resolutions). */
  int n_heads_up;       /* variant 2: num_heads_upsample (heads of up-path attention) */
  int scale_shift_norm; /* variant 2: use_scale_shift_norm (GN(h) * (1 + scale) + shift before conv2) */
  int pool_resample;    /* variant 2: conv_resample = False (avg-pool / nearest without a conv) */
  int attn_legacy;      /* variant 2: QKVAttentionLegacy (per-head [q; k; v] channel interleave) */
} dm_unet_arch;

typedef struct dm_unet dm_unet;

/* Number of parameter tensors the reference UNet with this arch registers. */
int dm_unet_param_count(const dm_unet_arch* arch, int* n_params);
int dm_unet_create(const dm_unet_arch* arch, const float* const* params, const int64_t* numels,
                   int n_params, void* stream, dm_unet** out);
/* x: [B, in_channels, H, W] f32, t: [B] int64, out: [B, out_channels, H, W] f32.
 * y: [B] int64 class labels or NULL (variants 1/2; y[b] = -1 = no class for that row, which lets
 * the conditional and unconditional CFG branches run as one 2B batch; the Python layer accepts -1
 * only from the CFG samplers and raises IndexError otherwise, as nn.Embedding does).
 * Workspace for batch B at H x W is allocated on first use and cached. */
int dm_unet_forward(dm_unet* m, const float* x, const int64_t* t, const int64_t* y, int B, int H, int W,
                    float* out, void* stream);
/* Install the sinusoid frequency table exp(-ln(1e4)/(dim/2-1) * i), i < dim/2
 * (models/modules.py:52-54). The reference evaluates it with torch's CPU exp,
 * whose last bit is host dependent; hosts pass the table they compute with
 * the same expression so the embedding matches their reference bit for bit.
 * `freqs` may be host or device memory; NULL reverts to the on-device expf. */
int dm_unet_set_time_freqs(dm_unet* m, const float* freqs, int n, void* stream);
/* Per-launch profiling of the cached plan (HIP events recorded on the launch
 * stream around every op of dm_unet_forward while enabled). enable = N > 0
 * observes every N-th forward (the events cost a few % of throughput; sampling
 * keeps the measured run representative), 0 disables. Enabling resets the
 * accumulators; dm_unet_profile_get synchronises pending events. `label`
 * names the kernel family/tile (matches the rocprof kernel name), `flops` /
 * `bytes` are the op's algorithmic work per launch. */
int dm_unet_profile(dm_unet* m, int enable);
int dm_unet_profile_count(dm_unet* m, int* n_ops);
int dm_unet_profile_get(dm_unet* m, int i, char* label, int label_len, double* flops, double* bytes,
                        double* ms_total, int64_t* launches);
/* Device bytes held by packed weights (fp32 arena + split copies) and by the plan scratch slab. */
int dm_unet_memory(const dm_unet* m, int64_t* weight_bytes, int64_t* workspace_bytes);
/* Plans are cached per forward shape (B, H, W), up to 3, least recently used evicted; they all run over
 * one scratch slab sized to the largest. dm_unet_share_workspace(a, b) makes b use a's slab too: for
 * models whose forwards never overlap (one stream, one after the other) -- UNetCombined's conditional
 * and unconditional networks (models/adm/unet_combined.py:23-25), which then hold one workspace instead
 * of two. A forward on a stream other than the previous forward's over the same scratch waits for that
 * forward first (an event wait), so forwards issued on several streams serialise instead of racing.
 * dm_unet_plan_stats: plans built so far and plans cached. */
int dm_unet_share_workspace(dm_unet* a, dm_unet* b);
int dm_unet_plan_stats(const dm_unet* m, int64_t* builds, int* cached);
/* Arithmetic of the 3x3 halo-patch convs (all fp32-accurate, models/unet.py:16,26 convolve in fp32):
 * DM_SPLIT_FP16X2 (default; env DM_CONV_MATH=fp16x2), DM_SPLIT_BF16X3 (bf16x3), 0 = fp32 MFMA (fp32).
 * An fp16x2 forward that meets an activation beyond the fp16 range (|a| > 65504) is detected on the
 * device and that forward is run again in bf16x3; the next forward is fp16x2 again (plans are cached per
 * shape and arithmetic). get reports the caller's kind. */
int dm_unet_set_conv_math(dm_unet* m, int kind);
int dm_unet_get_conv_math(const dm_unet* m, int* kind);
/* Deferred range check: with deferred != 0 a forward does not read the fp16x2 range flag (no host
 * sync per forward); the caller polls it once per sampling loop. dm_unet_range_poll synchronises
 * `stream`, reports whether any forward since the last poll met an activation beyond the fp16 range,
 * clears the flag and, if it was set, puts the model in fallback (bf16x3 forwards): the caller then re-runs
 * what it computed since the last poll (diffusions.DDPM.sample re-runs the loop from the same RNG state) and
 * ends the fallback with dm_unet_range_fallback(m, 0). dm_unet_range_stats: forwards / loops re-run in
 * bf16x3 so far, and the arithmetic the next forward runs in. */
int dm_unet_set_range_deferred(dm_unet* m, int deferred);
int dm_unet_range_poll(dm_unet* m, void* stream, int* flagged);
int dm_unet_range_fallback(dm_unet* m, int on);
int dm_unet_range_stats(const dm_unet* m, int64_t* fallbacks, int* active_math);
void dm_unet_destroy(dm_unet* m);

/* Denoiser: DiT ------------------------------------------------------------
 * Replaces models/dit/model.py:145-252 (DiT.__init__ / forward; the timm
 * PatchEmbed / Attention / Mlp blocks it builds on, timm~=0.9.12). `params` are
 * the state_dict tensors in order: pos_embed, x_embedder.proj.{weight,bias},
 * t_embedder.mlp.{0,2}.{weight,bias}, y_embedder.embedding_table.weight, then per
 * block attn.qkv, attn.proj, mlp.fc1, mlp.fc2, adaLN_modulation.1 (weight, bias
 * each), then final_layer.linear and final_layer.adaLN_modulation.1.
 */
typedef struct dm_dit_arch {
  int input_size;    /* latent H = W */
  int patch_size;
  int in_channels;
  int hidden_size;
  int depth;
  int num_heads;
  int mlp_hidden;    /* int(hidden_size * mlp_ratio) */
  int num_classes;
  int null_class;    /* 1: the embedding table has the CFG null row num_classes (class_dropout_prob > 0) */
  int learn_sigma;   /* out_channels = 2 * in_channels */
} dm_dit_arch;

typedef struct dm_dit dm_dit;

int dm_dit_param_count(const dm_dit_arch* arch, int* n_params);
int dm_dit_create(const dm_dit_arch* arch, const float* const* params, const int64_t* numels, int n_params,
                  void* stream, dm_dit** out);
/* x: [B, in_channels, S, S] f32 latents, t: [B] int64, y: [B] int64 labels or NULL (NULL / y[b] < 0 = the
 * null class, dit/model.py:241-242), out: [B, out_channels, S, S] f32. */
int dm_dit_forward(dm_dit* m, const float* x, const int64_t* t, const int64_t* y, int B, float* out, void* stream);
/* Arithmetic of the DiT token GEMMs: DM_SPLIT_FP16X2 (default, fp32-accurate products from an fp16 split
 * on the matrix cores) or 0 (fp32 MFMA; also DM_CONV_MATH=fp32|bf16x3). A forward whose operands leave
 * the fp16 range is re-run in fp32; the next forward is fp16x2 again. */
int dm_dit_set_math(dm_dit* m, int kind);
int dm_dit_get_math(const dm_dit* m, int* kind);
/* As dm_unet_set_range_deferred / dm_unet_range_poll / _range_fallback / _range_stats (the DiT's fallback
 * arithmetic is fp32). */
int dm_dit_set_range_deferred(dm_dit* m, int deferred);
int dm_dit_range_poll(dm_dit* m, void* stream, int* flagged);
int dm_dit_range_fallback(dm_dit* m, int on);
int dm_dit_range_stats(const dm_dit* m, int64_t* fallbacks, int* active_math);
/* 128-entry table exp(-ln(1e4) * i / 128) of the 256-wide frequency embedding (dit/model.py:51-54). */
int dm_dit_set_time_freqs(dm_dit* m, const float* freqs, int n, void* stream);
int dm_dit_profile(dm_dit* m, int enable);
int dm_dit_profile_count(dm_dit* m, int* n_ops);
int dm_dit_profile_get(dm_dit* m, int i, char* label, int label_len, double* flops, double* bytes,
                       double* ms_total, int64_t* launches);
int dm_dit_memory(const dm_dit* m, int64_t* weight_bytes, int64_t* workspace_bytes);
/* As dm_unet_plan_stats (plans keyed by B). */
int dm_dit_plan_stats(const dm_dit* m, int64_t* builds, int* cached);
void dm_dit_destroy(dm_dit* m);

/* Sampler update -----------------------------------------------------------
 * One elementwise pass doing predict() (ddpm.py:174-203), the optional CFG
 * combine (ddim.py:185 / ddpm.py:343-345, with the second predict under
 * hack_objective('pred_eps')), and the DDIM (ddim.py:64-77) or DDPM
 * (ddpm.py:221-252) update. All scalar coefficients are computed by the host
 * with the reference's own torch 0-dim op sequence and passed in, so the
 * result is bit-identical to the reference CPU path on identical inputs.
 */
typedef struct dm_step_desc {
  int B, C, HW;      /* image tensor [B, C, HW] */
  int Cm;            /* channels of the model output: C, or 2C with a learned variance */
  const float* xt;
  const float* model_out;        /* conditional (or only) branch, [B, Cm, HW] */
  const float* model_out_uncond; /* CFG unconditional branch or NULL */
  float w_uncond, w_cond;        /* (1 - s), s  (float32 of the python scalars) */
  int objective;                 /* 0 pred_eps, 1 pred_x0, 2 pred_v */
  int clip_denoised;
  float sqrt_recip_ac, sqrt_recipm1_ac, sqrt_ac, sqrt_one_minus_ac;
  int kind;                      /* 0 DDIM, 1 DDPM */
  float coef1, coef2;            /* DDIM: sqrt(ac_prev), sqrt(1-ac_prev-var); DDPM: mean_coef1, mean_coef2 */
  int var_mode;                  /* 0 scalar std, 1 learned_range */
  float std;                     /* sqrt(var) for var_mode 0 */
  float min_logvar, max_logvar;  /* learned_range */
  int add_noise;                 /* t != 0 */
  const float* noise;            /* [B, C, HW] or NULL (treated as zeros, e.g. DDIM eta=0) */
  float* sample;                 /* required */
  float* mean;                   /* optional outputs (NULL to skip) */
  float* pred_x0;
  float* pred_eps;
  float* var;
  /* Karras-style samplers on the VP schedule (sigma_t = sqrt((1 - ac_t) / ac_t)):
   * euler 1: EulerSampler.denoise / HeunSampler.denoise_1st_order (diffusions/euler.py:50-66,
   *          heun.py:56-77): sample = (st1*xt + (st1*xt - x0)/sig_t * dsig) / sp1, derivative -> e_dout;
   * euler 2: HeunSampler.denoise_2nd_order (heun.py:79-106) with xt = x_{t-1} and x0 predicted at
   *          t_prev: d = ((sp1*xt - x0)/sig_p + e_d1) / 2, sample = (st1*e_x1 + d*dsig) / sp1.
   * st1 = sqrt(1+sig_t^2), sp1 = sqrt(1+sig_p^2), dsig = sig_p - sig_t (host 0-dim float32 ops). */
  int euler;
  float e_st1, e_sig_t, e_dsig, e_sp1, e_sig_p;
  const float* e_d1;
  const float* e_x1;
  float* e_dout;
} dm_step_desc;

int dm_sampler_step(const dm_step_desc* d, void* stream);

/* Closed-form conversions of reference diffusions/ddpm.py, elementwise with separately rounded float32
 * products (bit-identical to the torch CPU expressions given the same coefficients):
 *   mode 0: out = c1 a + c2 b       diffuse (:152-172: sqrt(ac_t) x0 + sqrt(1 - ac_t) eps),
 *                                   pred_eps_from_v (:117-120)
 *   mode 1: out = c1 a - c2 b       pred_x0_from_eps (:102-105), pred_x0_from_v (:112-115), get_v (:140-150)
 *   mode 2: out = (c1 a - b) / c2   pred_eps_from_x0 (:107-110)
 * a, b, out: n floats; c1_rows / c2_rows: per-row coefficients (row = element / row_elems, one row per image
 * with its own timestep) or NULL for the scalars c1 / c2. */
int dm_lincomb(int mode, const float* a, const float* b, float* out, int64_t n, int64_t row_elems,
               const float* c1_rows, const float* c2_rows, float c1, float c2, void* stream);

/* Operator-level entry points (NHWC, channel-pitched views) ----------------
 * Used by the parity tests and to compose other denoisers.
 */
/* torch.nn.GroupNorm (+ optional per-image modulation y*(1+ms)+mb, + optional SiLU).
 * x, y: NHWC [B, H*W, C] with channel pitches; part: scratch of
 * dm_groupnorm_scratch_bytes() bytes. */
int64_t dm_groupnorm_scratch_bytes(int B, int HW, int G);
int dm_groupnorm_nhwc(const float* x, int x_pitch, float* y, int y_pitch, int B, int HW, int C, int G,
                      float eps, const float* gamma, const float* beta, const float* mod_scale,
                      const float* mod_shift, int mod_pitch, int silu, void* scratch, void* stream);

/* GroupNorm statistics -> per-(image, channel) affine tables scale/shift [B][C]
 * (y = x * scale + shift equals torch.nn.GroupNorm's output), for fused consumers. */
int dm_groupnorm_affine(const float* x, int x_pitch, int B, int HW, int C, int G, float eps, const float* gamma,
                        const float* beta, float* scale, float* shift, void* scratch, void* stream);

/* Pack a torch conv weight [Cout][Cin][kh][kw] into the implicit-GEMM layout
 * [Cout][ldw] at column offset col0 (k = tap * Cin + c). */
int dm_pack_conv_weight(const float* w, int Cout, int Cin, int taps, float* out, int ldw, int col0,
                        void* stream);

/* Pack a torch 3x3 weight [Cout][Cin][3][3] for the sub-pixel upsample conv (dm_conv_desc.upsample = 2):
 * out [4 output parities][Cout][4 * Cin], the 3x3 taps that read the same low-res pixel summed. */
int dm_pack_conv_weight_subpixel(const float* w, int Cout, int Cin, float* out, void* stream);

/* Split packed fp32 conv weights (nmat matrices [Cout][K] from dm_pack_conv_weight /
 * dm_pack_conv_weight_subpixel, K = taps * Cin (+ Cin2 of a second segment), taps 9, or 4 for
 * the sub-pixel form) into the 16-bit slices of dm_conv_desc.w_split:
 * dm_conv_weight_split_bytes(nmat, Cout, K, kind) bytes at `out` (16-byte aligned).
 * kind DM_SPLIT_BF16X3: exact three-way bf16 split (six piece products per product);
 * kind DM_SPLIT_FP16X2: two-way fp16 split of the weights scaled per output channel by a power
 * of two (three piece products per product; the scales follow the pieces in `out`). */
#define DM_SPLIT_FP16X2 2
#define DM_SPLIT_BF16X3 3
int64_t dm_conv_weight_split_bytes(int nmat, int Cout, int K, int kind);
int dm_pack_conv_weight_split(const float* w, int nmat, int Cout, int K, int Cin, int taps, int kind, void* out,
                              void* stream);

/* Winograd F(2,3)-along-x weights of a packed 3x3 conv (dm_pack_conv_weight, K = 9 Cin + Cin2, Cin % 32 == 0; Cin2: a
 * second 1x1 segment (the ResBlock shortcut), Cin2 % 64 == 0): U = G g per tap row (float64, one rounding), split to
 * fp16x2 fragment images of 4 matrices [Cout][3 Cin + Cin2 / 2] with per-output-channel power-of-two scales:
 * dm_conv_weight_wino_bytes(Cout, Cin, Cin2) bytes at `out`. fold = 1 for a conv whose input prologue has the SiLU
 * (dm_conv_desc pro_scale set, pro_nosilu 0) and a shortcut (its weights carry the kernel's SiLU constant). */
int64_t dm_conv_weight_wino_bytes(int Cout, int Cin, int Cin2);
int dm_pack_conv_weight_wino(const float* w, int Cout, int Cin, int Cin2, int fold, void* out, void* stream);

typedef struct dm_conv_desc {
  const float* x;  int x_pitch, Cin, Hin, Win;
  int taps, stride;
  int upsample;    /* 0 none; 1 nearest-2x then 3x3 (Hout = 2 Hin); 2 the same as sub-pixel
                      4-tap convs (weights from dm_pack_conv_weight_subpixel, K = 4 Cin) */
  const float* x2; int x2_pitch, Cin2;
  const float* w;  int K;
  float* y;        int y_pitch, Cout, B, Hout, Wout;
  const float* bias;
  const float* rowvec; int rowvec_pitch;
  const float* res; int res_pitch;
  int tile;  /* 0: automatic; 1..3 force the im2col kernel with a 128x128 / 128x64 / 64x64 tile,
                4..6 the halo-patch kernel with those tiles (tests, tuning) */
  /* optional fused GroupNorm+SiLU of the input: x -> silu(x * pro_scale[b][c] + pro_shift[b][c]),
   * [B][Cin] tables from dm_groupnorm_affine(); halo-patch shapes only (3x3 stride 1 / upsample) */
  const float* pro_scale;
  const float* pro_shift;
  /* optional split copy of w from dm_pack_conv_weight_split() of kind w_split_kind: halo-patch shapes
   * then compute their products on the 16-bit matrix cores from a split of both operands
   * (fp32-accurate); NULL keeps the fp32 MFMA kernels */
  const void* w_split;
  int w_split_kind;  /* DM_SPLIT_BF16X3 or DM_SPLIT_FP16X2 */
  int* range_flag;   /* optional device int, set to 1 when an fp16x2 conv meets |x| > 65504 */
  int pro_nosilu;    /* 1: the input prologue is x * pro_scale + pro_shift alone (no SiLU) */
  /* optional split-K of a 3x3 stride-1 conv (0 / 1: none): partial sums of ksplit input-channel
   * ranges go to kpart ([ksplit][B * Hout * Wout][Cout] floats), then one reduction applies the epilogue */
  int ksplit;
  float* kpart;
  /* optional Winograd F(2,3) weights of a 3x3 stride-1 conv from dm_pack_conv_weight_wino (needs w_split of kind
   * DM_SPLIT_FP16X2 too): 32- / 16-pixel-wide maps with Cout % 128 == 0 then run the Winograd kernel (tile 0 or
   * 21; 21 fails on any other shape) */
  const void* w_wino;
  int w_wino_fold;   /* the fold dm_pack_conv_weight_wino packed w_wino with */
} dm_conv_desc;
/* 1x1 convs (taps 1, K = Cin, Cin % 32 == 0) with DM_SPLIT_FP16X2 weights run on the split kernel
 * with the same prologue / epilogue options: the static-weight GEMMs of the attention blocks. */
int dm_conv2d_nhwc(const dm_conv_desc* d, void* stream);

typedef struct dm_gemm_desc {
  int M, N, K, Z1, Z2;
  const float* A; int64_t a_s1, a_s2; int lda;
  const float* B; int64_t b_s1, b_s2; int ldb; int b_kn;
  float* C; int64_t c_s1, c_s2; int ldc;
  float alpha;
  const float* bias;
  const float* res; int ld_res;
  int act;
  float b_scale;  /* 0: none; else multiplies B elements on load (B stored [n][k]) */
  /* split = DM_SPLIT_FP16X2: products on the fp16 matrix cores from a two-way fp16 split of both
   * operands (fp32-accurate), A scaled by 2^split_ea and B by 2^split_eb before the split (exact;
   * choose them to keep the scaled operands well inside fp16's normal range), the result scaled back.
   * |scaled element| > 65504 sets *range_flag (optional). 0 = fp32 MFMA. */
  int split, split_ea, split_eb;
  int* range_flag;
} dm_gemm_desc;
int dm_gemm(const dm_gemm_desc* d, void* stream);

int dm_softmax_rows(float* x, int64_t rows, int L, int ld, void* stream);
/* kind 0: models/modules.py SinusoidalPosEmb ([sin, cos]); kind 1: ADM timestep_embedding ([cos, sin]) */
int dm_timestep_embedding(const int64_t* t, int B, int dim, int kind, const float* freqs, float* out,
                          void* stream);

/* ---------------------------------------------------------------- data-parallel gather (comm.hip)
 * Replaces accelerate's gather of each rank's finished fold (reference scripts/sample_uncond.py:190,
 * scripts/sample_cfg.py:177: `accelerator.gather(samples)[:bs]`): an RCCL all-gather in rank order over the
 * ranks' own HIP devices (xGMI between the GPUs of a node). Bootstrap: rank 0 calls dm_comm_unique_id, the
 * caller hands the DM_COMM_UID_BYTES bytes to every rank, each rank calls dm_comm_init with the HIP device it
 * samples on current. RCCL is loaded on first use (dlopen "librccl.so.1"): DM_ERR_UNSUPPORTED without it.
 * dm_allgather_f32: recv holds nranks x count floats, rank r's send lands at recv + r x count; enqueued on
 * `stream` (asynchronous, like every launch here); send may be recv + rank x count (in place). */
#define DM_COMM_UID_BYTES 128
typedef struct dm_comm dm_comm;
int dm_comm_unique_id(void* uid);
int dm_comm_init(const void* uid, int nranks, int rank, dm_comm** comm);
int dm_comm_info(const dm_comm* comm, int* nranks, int* rank, int* device);
int dm_allgather_f32(dm_comm* comm, const float* send, float* recv, int64_t count, void* stream);
void dm_comm_destroy(dm_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* DM_HIP_H_ */
