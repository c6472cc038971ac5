// C-ABI wrappers over the kernel launchers (include/dm_hip.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include "dm_common.h"
#include "dm_kernels.h"

namespace dm {
namespace {
thread_local std::string g_last_error;
}
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

namespace {
thread_local Toggles t_toggles;                  // this thread's last refresh_toggles()
thread_local const Toggles* t_scope = nullptr;   // the innermost ToggleScope
bool env_is(const char* name, char c) {
  const char* e = std::getenv(name);
  return e && e[0] == c;
}
bool g_launch_log_on = false;
std::string g_launch_log;
}  // namespace
const Toggles& toggles() { return t_scope ? *t_scope : t_toggles; }
const Toggles* toggle_scope_swap(const Toggles* t) {
  const Toggles* prev = t_scope;
  t_scope = t;
  return prev;
}
// every environment switch of the library, read here and nowhere else (DESIGN.md §6 toggle table)
void refresh_toggles() {
  Toggles t;
  if (const char* m = std::getenv("DM_CONV_MATH")) {
    const std::string v(m);
    t.conv_math = v == "fp32" ? 0 : v == "bf16x3" ? 3 : 2;
  }
  t.range_check = !env_is("DM_RANGE_CHECK", '0');
  t.graph = std::getenv("DM_NO_GRAPH") == nullptr;
  t.wino = !env_is("DM_CONV_WINO", '0');
  t.k32s_w4 = env_is("DM_K32S_W4", '1');
  t.k32_small = !env_is("DM_CONV_K32S", '0');
  t.k32_s2 = !env_is("DM_CONV_K32S2", '0');
  t.k32_t2d = !env_is("DM_CONV_K32T2", '0');
  t.k32_8x = !env_is("DM_K32_8X", '0');
  t.gn_fusion = !env_is("DM_GN_FUSION", '0');
  if (const char* e = std::getenv("DM_ATTN")) {
    const std::string v(e);
    t.attn = v == "3" ? 3 : v == "0" || v == "presplit" ? 0 : v == "noproj" ? kAttnNoProj : v == "fused" ? kAttnFused
           : v == "unfused" ? kAttnUnfused : 4;
  }
  t.attn_gn_launch = env_is("DM_ATTN_GNFIN", '1');
  t.attn_small = !env_is("DM_ATTN_SMALL", '0');
  t.dit_presplit = !env_is("DM_DIT_PRESPLIT", '0');
  t.lin_sk = !env_is("DM_LIN_SK", '0');
  t.lin_rows = !env_is("DM_LIN_ROWS", '0');
  t_toggles = t;
}
void note_launch(const char* name) {
  if (!g_launch_log_on) return;
  g_launch_log += name;
  g_launch_log += '\n';
}
}  // namespace dm

/* Test hook: enable (1, clearing it) / disable (0) the launch log; read copies it NUL-terminated into buf. */
extern "C" int dm_debug_launch_log(int enable) {
  dm::g_launch_log_on = enable != 0;
  if (enable) dm::g_launch_log.clear();
  return DM_OK;
}
extern "C" int dm_debug_launch_log_read(char* buf, int len) {
  if (!buf || len <= 0) { dm::set_error("launch log: null buffer"); return DM_ERR_ARG; }
  const size_t n = std::min(dm::g_launch_log.size(), (size_t)len - 1);
  memcpy(buf, dm::g_launch_log.data(), n);
  buf[n] = 0;
  return (int)n;
}

using dm::View;

extern "C" int dm_abi_version(void) { return DM_ABI_VERSION; }

extern "C" const char* dm_last_error(void) { return dm::last_error(); }

#ifndef DM_SRC_HASH
#define DM_SRC_HASH "unknown"
#endif
extern "C" const char* dm_build_info(void) { return "src=" DM_SRC_HASH " arch=gfx950"; }

extern "C" int dm_sampler_step(const dm_step_desc* d, void* stream) {
  if (!d) { dm::set_error("null step descriptor"); return DM_ERR_ARG; }
  dm::StepArgs s{};
  s.B = d->B; s.C = d->C; s.HW = d->HW; s.Cm = d->Cm;
  s.xt = d->xt; s.out_c = d->model_out; s.out_u = d->model_out_uncond;
  s.w_u = d->w_uncond; s.w_c = d->w_cond;
  s.objective = d->objective; s.clip = d->clip_denoised;
  s.c_recip = d->sqrt_recip_ac; s.c_recipm1 = d->sqrt_recipm1_ac;
  s.c_sa = d->sqrt_ac; s.c_s1ma = d->sqrt_one_minus_ac;
  s.kind = d->kind; s.m1 = d->coef1; s.m2 = d->coef2;
  s.var_mode = d->var_mode; s.std = d->std;
  s.min_logvar = d->min_logvar; s.max_logvar = d->max_logvar;
  s.add_noise = d->add_noise; s.noise = d->noise;
  s.sample = d->sample; s.mean_out = d->mean; s.x0_out = d->pred_x0; s.eps_out = d->pred_eps;
  s.var_out = d->var;
  s.euler = d->euler; s.e_st1 = d->e_st1; s.e_sig_t = d->e_sig_t; s.e_dsig = d->e_dsig; s.e_sp1 = d->e_sp1;
  s.e_sig_p = d->e_sig_p; s.e_d1 = d->e_d1; s.e_x1 = d->e_x1; s.e_dout = d->e_dout;
  if (s.euler < 0 || s.euler > 2) { dm::set_error("invalid euler mode"); return DM_ERR_ARG; }
  if (s.euler == 2 && (!s.e_d1 || !s.e_x1)) { dm::set_error("Heun second order needs e_d1 and e_x1"); return DM_ERR_ARG; }
  if (s.objective < 0 || s.objective > 2) { dm::set_error("invalid objective"); return DM_ERR_ARG; }
  if (s.kind < 0 || s.kind > 1) { dm::set_error("invalid sampler kind"); return DM_ERR_ARG; }
  if (s.B < 0 || s.C <= 0 || s.HW <= 0) { dm::set_error("invalid shape"); return DM_ERR_ARG; }
  return dm::sampler_step(s, (hipStream_t)stream);
}

extern "C" int dm_lincomb(int mode, const float* a, const float* b, float* out, int64_t n, int64_t row_elems,
                          const float* c1_rows, const float* c2_rows, float c1, float c2, void* stream) {
  if (!a || !b || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (mode < 0 || mode > 2) { dm::set_error("lincomb mode must be 0, 1 or 2"); return DM_ERR_ARG; }
  if (n < 0 || row_elems <= 0) { dm::set_error("invalid shape"); return DM_ERR_ARG; }
  return dm::lincomb(mode, a, b, out, (long)n, (long)row_elems, c1_rows, c2_rows, c1, c2, (hipStream_t)stream);
}

extern "C" int64_t dm_groupnorm_scratch_bytes(int B, int HW, int G) {
  return (int64_t)B * dm::gn_num_chunks(HW) * G * (int64_t)sizeof(double2);
}

extern "C" int dm_groupnorm_nhwc(const float* x, int x_pitch, float* y, int y_pitch, int B, int HW, int C, int G,
                                 float eps, const float* gamma, const float* beta, const float* mod_scale,
                                 const float* mod_shift, int mod_pitch, int silu, void* scratch, void* stream) {
  if (!x || !y || !scratch) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (B <= 0 || HW <= 0 || C <= 0 || G <= 0) { dm::set_error("invalid shape"); return DM_ERR_ARG; }
  View vx{const_cast<float*>(x), B, HW, 1, C, x_pitch};
  View vy{y, B, HW, 1, C, y_pitch};
  hipStream_t st = (hipStream_t)stream;
  int rc = dm::gn_partial(vx, G, (double2*)scratch, st);
  if (rc) return rc;
  return dm::gn_apply(vx, G, (const double2*)scratch, dm::gn_num_chunks(HW), eps, gamma, beta, mod_scale,
                      mod_shift, mod_pitch, silu ? 1 : 0, vy, st);
}

extern "C" int dm_groupnorm_affine(const float* x, int x_pitch, int B, int HW, int C, int G, float eps,
                                   const float* gamma, const float* beta, float* scale, float* shift, void* scratch,
                                   void* stream) {
  if (!x || !scale || !shift || !scratch) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (B <= 0 || HW <= 0 || C <= 0 || G <= 0) { dm::set_error("invalid shape"); return DM_ERR_ARG; }
  View vx{const_cast<float*>(x), B, HW, 1, C, x_pitch};
  hipStream_t st = (hipStream_t)stream;
  int rc = dm::gn_partial(vx, G, (double2*)scratch, st);
  if (rc) return rc;
  return dm::gn_finalize(vx, G, (const double2*)scratch, eps, gamma, beta, scale, shift, st);
}

extern "C" int dm_pack_conv_weight(const float* w, int Cout, int Cin, int taps, float* out, int ldw, int col0,
                                   void* stream) {
  if (!w || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (Cout <= 0 || Cin <= 0 || (taps != 1 && taps != 9) || col0 + taps * Cin > ldw) {
    dm::set_error("invalid conv weight shape");
    return DM_ERR_ARG;
  }
  return dm::repack_conv(w, Cout, Cin, taps, out, ldw, col0, (hipStream_t)stream);
}

extern "C" int dm_conv2d_nhwc(const dm_conv_desc* d, void* stream) {
  dm::refresh_toggles();
  if (!d || !d->x || !d->w || !d->y) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  dm::ConvArgs a{};
  a.x1 = d->x; a.x1_pitch = d->x_pitch; a.Cin1 = d->Cin; a.Hin = d->Hin; a.Win = d->Win;
  a.taps = d->taps; a.stride = d->stride; a.upsample = d->upsample;
  a.x2 = d->x2; a.x2_pitch = d->x2_pitch; a.Cin2 = d->Cin2;
  a.w = d->w; a.K = d->K;
  a.y = d->y; a.y_pitch = d->y_pitch; a.Cout = d->Cout; a.B = d->B; a.Hout = d->Hout; a.Wout = d->Wout;
  a.bias = d->bias; a.rowvec = d->rowvec; a.rowvec_pitch = d->rowvec_pitch;
  a.res = d->res; a.res_pitch = d->res_pitch;
  a.tile = d->tile;
  a.pro_scale = d->pro_scale;
  a.pro_shift = d->pro_shift;
  a.pro_nosilu = d->pro_nosilu;
  a.ksplit = d->ksplit;
  a.kpart = d->kpart;
  a.ws = d->w_split;
  if (a.ws) {
    if (d->w_split_kind != DM_SPLIT_BF16X3 && d->w_split_kind != DM_SPLIT_FP16X2) {
      dm::set_error("conv: w_split_kind must be DM_SPLIT_BF16X3 or DM_SPLIT_FP16X2");
      return DM_ERR_ARG;
    }
    a.ws_np = d->w_split_kind;
    if (a.ws_np == DM_SPLIT_FP16X2)
      a.ws_rowscale = dm::split_conv_rowscale(a.ws, a.upsample == 2 ? 4 : 1, a.Cout, a.K);
    a.range_flag = d->range_flag;
  }
  if (d->w_wino) {
    if (!a.ws || a.ws_np != DM_SPLIT_FP16X2) {
      dm::set_error("conv: w_wino needs w_split of kind DM_SPLIT_FP16X2");
      return DM_ERR_ARG;
    }
    a.wino_ws = d->w_wino;
    a.wino_rowscale = dm::wino_rowscale(d->w_wino, a.Cout, a.Cin1, a.Cin2);
    a.wino_fold = d->w_wino_fold;
  }
  return dm::conv2d_igemm(a, (hipStream_t)stream);
}

extern "C" int64_t dm_conv_weight_wino_bytes(int Cout, int Cin, int Cin2) {
  if (Cout <= 0 || Cin <= 0 || Cin % 32 != 0 || Cin2 < 0 || Cin2 % 64 != 0) return -1;
  return (int64_t)dm::wino_weights_bytes(Cout, Cin, Cin2);
}

extern "C" int dm_pack_conv_weight_wino(const float* w, int Cout, int Cin, int Cin2, int fold, void* out, void* stream) {
  return dm::wino_weights(w, Cout, Cin, Cin2, fold, out, (hipStream_t)stream);
}

extern "C" int64_t dm_conv_weight_split_bytes(int nmat, int Cout, int K, int kind) {
  if (nmat <= 0 || Cout <= 0 || K <= 0 || K % 16 != 0) return 0;
  if (kind != DM_SPLIT_BF16X3 && kind != DM_SPLIT_FP16X2) return 0;
  return (int64_t)dm::split_conv_weights_bytes(nmat, Cout, K, kind);
}

extern "C" int dm_pack_conv_weight_split(const float* w, int nmat, int Cout, int K, int Cin, int taps, int kind,
                                         void* out, void* stream) {
  if (!w || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  return dm::split_conv_weights(w, nmat, Cout, K, Cin, taps, kind, out, (hipStream_t)stream);
}

extern "C" int dm_pack_conv_weight_subpixel(const float* w, int Cout, int Cin, float* out, void* stream) {
  if (!w || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  return dm::repack_subpixel(w, Cout, Cin, out, (hipStream_t)stream);
}

extern "C" int dm_gemm(const dm_gemm_desc* d, void* stream) {
  dm::refresh_toggles();
  if (!d || !d->A || !d->B || !d->C) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  dm::GemmArgs g{};
  g.M = d->M; g.N = d->N; g.K = d->K; g.Z1 = d->Z1; g.Z2 = d->Z2;
  g.A = d->A; g.a_s1 = d->a_s1; g.a_s2 = d->a_s2; g.lda = d->lda;
  g.Bm = d->B; g.b_s1 = d->b_s1; g.b_s2 = d->b_s2; g.ldb = d->ldb; g.b_kn = d->b_kn;
  g.C = d->C; g.c_s1 = d->c_s1; g.c_s2 = d->c_s2; g.ldc = d->ldc;
  g.alpha = d->alpha; g.bias = d->bias; g.res = d->res; g.ld_res = d->ld_res; g.act = d->act;
  g.b_scale = d->b_scale;
  g.split = d->split; g.split_ea = d->split_ea; g.split_eb = d->split_eb; g.range_flag = d->range_flag;
  return dm::gemm_batched(g, (hipStream_t)stream);
}

extern "C" int dm_softmax_rows(float* x, int64_t rows, int L, int ld, void* stream) {
  if (!x) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  return dm::softmax_rows(x, rows, L, ld, (hipStream_t)stream);
}

extern "C" int dm_timestep_embedding(const int64_t* t, int B, int dim, int kind, const float* freqs, float* out,
                                     void* stream) {
  if (!t || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (B <= 0) { dm::set_error("empty batch"); return DM_ERR_ARG; }
  return dm::timestep_embed(t, B, dim, kind, freqs, out, (hipStream_t)stream);
}
