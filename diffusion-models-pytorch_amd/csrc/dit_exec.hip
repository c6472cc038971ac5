// Native executor for the DiT denoiser (models/dit/model.py:145-252).
//
// Build time (dm_dit_create): the state_dict tensors are consumed in
// registration order and copied into one library-owned arena; the adaLN
// modulation Linear of every block and of the final layer are stacked into ONE
// [depth * 6D + 2D][D] matrix, so all modulation vectors of a forward come from
// a single GEMM over SiLU(t_emb + y_emb).
//
// Forward: tokens stay resident as one [B * T][D] fp32 matrix x, updated in
// place by the gated-residual epilogues. Per block (dit/model.py:118-122):
//   row_stats(x) -> QKV GEMM with the LayerNorm + modulate prologue
//   -> S = (q * d^-1/2) k^T -> softmax -> O = P v -> proj GEMM, x += gate_msa * (.)
//   row_stats(x) -> fc1 GEMM (LN + modulate prologue, GELU-tanh epilogue)
//   -> fc2 GEMM, x += gate_mlp * (.)
// so norm1/norm2/modulate/gate never materialise. All GEMMs are the fp32 MFMA
// kernel of gemm.hip.
#include <cmath>
#include <memory>
#include <vector>

#include <map>
#include "dm_common.h"
#include "dm_kernels.h"
#include "plan.h"

namespace dm {

namespace {

struct BlockP {
  size_t qkv_w, qkv_b, proj_w, proj_b, fc1_w, fc1_b, fc2_w, fc2_b;
};

int dit_count(const dm_dit_arch& a) { return 8 + 10 * a.depth + 4; }

int dit_validate(const dm_dit_arch* a) {
  DM_REQUIRE(a != nullptr, "arch is null");
  DM_REQUIRE(a->patch_size >= 1 && a->input_size % a->patch_size == 0, "input_size must be divisible by patch_size");
  DM_REQUIRE(a->in_channels >= 1 && (a->in_channels * a->patch_size * a->patch_size) % 4 == 0,
             "in_channels * patch_size^2 must be a multiple of 4");
  DM_REQUIRE(a->hidden_size >= 32 && a->hidden_size % 4 == 0, "hidden_size must be a multiple of 4");
  DM_REQUIRE(a->depth >= 1, "depth must be >= 1");
  DM_REQUIRE(a->num_heads >= 1 && a->hidden_size % a->num_heads == 0 && (a->hidden_size / a->num_heads) % 4 == 0,
             "hidden_size / num_heads must be a multiple of 4");
  DM_REQUIRE(a->mlp_hidden >= 4 && a->mlp_hidden % 4 == 0, "mlp hidden size must be a multiple of 4");
  DM_REQUIRE(a->num_classes >= 1, "num_classes must be >= 1");
  return DM_OK;
}

}  // namespace

struct DiTModel {
  dm_dit_arch arch;
  float* arena = nullptr;
  size_t arena_floats = 0;
  int D = 0, T = 0, OC = 0, PP = 0, ada_total = 0;
  size_t pos, xw, xb, tw1, tb1, tw2, tb2, ytab, freqs, ada_w, ada_b, fin_w, fin_b;
  bool freqs_set = false;
  std::vector<BlockP> blocks;
  // Arithmetic of the token GEMMs (qkv, attention, proj, fc1, fc2, final): 2 = fp16x2 split (gemm.hip
  // SPLIT; default unless DM_CONV_MATH=fp32|bf16x3), 0 = fp32 MFMA. A forward that raises range_flag
  // (an operand beyond the fp16 range) runs again in fp32; the next forward is fp16x2 again (plans cached
  // per (B, arithmetic)). Deferred mode: dm_dit_range_poll sets `fallback` for the caller's re-run,
  // dm_dit_range_fallback clears it. `math` is the arithmetic of the plan being built (set by get_plan).
  int base_math = conv_math_from_env() == 2 ? 2 : 0;
  bool fallback = false;
  long range_fallbacks = 0;
  int math = base_math;
  int run_math() const { return base_math == 2 && fallback ? 0 : base_math; }
  bool range_check = toggles().range_check;
  int* range_flag = nullptr;
  int* range_flag_host = nullptr;
  bool range_deferred = false;  // dm_dit_set_range_deferred / dm_dit_range_poll, as for the UNet
  std::map<const float*, int> w_exp;
  // fp16x2 fragment images of the token-GEMM weights (split_conv_weights, taps 1), built once: those GEMMs
  // run linear_k32 (K = 32 MFMA steps, no per-load split of the weights)
  std::map<const float*, void*> split_w;
  bool linear_k32_on = true;
  // linear_k32's split-K tail (GemmArgs::sk_*): one 64-KB slab per resident block and one arrival counter per
  // tile, zeroed once (each tile's reducing block resets its counter); forwards of this model's plans are
  // stream-ordered (ScratchPool::order), so one set serves them all
  float* sk_ws = nullptr;
  unsigned* sk_cnt = nullptr;
  int sk_cap = 0;

  struct Plan : PlanBase {
    int B = 0;
    int math = 0;   // the arithmetic the plan was built with
    // plan-owned staging of the caller's tensors (graph replay reads fixed pointers)
    float* x = nullptr;
    int64_t* t = nullptr;
    int64_t* y = nullptr;  // -1 rows select the null class
    float* out = nullptr;
  };
  PlanCache<Plan> plans;  // LRU over B, scratch from one pool
  size_t split_bytes = 0;  // device bytes of the split_w copies

  float* P(size_t off) const { return arena + off; }
  ~DiTModel() {
    plans.clear();
    for (auto& kv : split_w) (void)hipFree(kv.second);
    if (range_flag) (void)hipFree(range_flag);
    if (sk_ws) (void)hipFree(sk_ws);
    if (sk_cnt) (void)hipFree(sk_cnt);
    if (range_flag_host) (void)hipHostFree(range_flag_host);
    if (arena) (void)hipFree(arena);
  }
  int build_plan(Plan& pl, int B);
  int get_plan(int B, int m, Plan** out) {
    math = m;
    return plans.get([&](const Plan& p) { return p.B == B && p.math == m; }, [&](Plan& p) { return build_plan(p, B); },
                     out);
  }
};

static int dit_create(const dm_dit_arch* arch, const float* const* params, const int64_t* numels, int n_params,
                      hipStream_t st, DiTModel** out) {
  int rc = dit_validate(arch);
  if (rc) return rc;
  const dm_dit_arch a = *arch;
  DM_REQUIRE(n_params == dit_count(a), "expected " + std::to_string(dit_count(a)) + " parameter tensors, got " +
                                           std::to_string(n_params));
  refresh_toggles();  // the model's arithmetic and range check (member initialisers) from this snapshot
  auto m = std::make_unique<DiTModel>();
  m->arch = a;
  const int D = a.hidden_size, p = a.patch_size, C = a.in_channels, Hm = a.mlp_hidden;
  const int S = a.input_size / p;
  m->D = D;
  m->T = S * S;
  m->OC = a.learn_sigma ? 2 * C : C;
  m->PP = p * p;
  m->ada_total = a.depth * 6 * D + 2 * D;
  const int n_cls = a.num_classes + (a.null_class ? 1 : 0);

  // arena layout: everything 64-float aligned
  size_t size = 0;
  auto reserve = [&](int64_t n) { size_t off = size; size += ((size_t)n + 63) / 64 * 64; return off; };
  struct Copy { size_t dst; int idx; int64_t n; };
  std::vector<Copy> copies;
  int idx = 0;
  std::string err;
  auto take = [&](int64_t n, const char* what) {
    if (idx < n_params && numels[idx] != n && err.empty())
      err = "parameter " + std::to_string(idx) + " (" + what + "): expected " + std::to_string(n) + " elements, got " +
            std::to_string(numels[idx]);
    const size_t off = reserve(n);
    copies.push_back({off, idx++, n});
    return off;
  };
  auto take_at = [&](int64_t n, size_t dst, const char* what) {
    if (idx < n_params && numels[idx] != n && err.empty())
      err = "parameter " + std::to_string(idx) + " (" + what + "): expected " + std::to_string(n) + " elements, got " +
            std::to_string(numels[idx]);
    copies.push_back({dst, idx++, n});
  };

  m->pos = take((int64_t)m->T * D, "pos_embed");
  m->xw = take((int64_t)D * C * p * p, "x_embedder.proj.weight");
  m->xb = take(D, "x_embedder.proj.bias");
  m->tw1 = take((int64_t)D * 256, "t_embedder.mlp.0.weight");
  m->tb1 = take(D, "t_embedder.mlp.0.bias");
  m->tw2 = take((int64_t)D * D, "t_embedder.mlp.2.weight");
  m->tb2 = take(D, "t_embedder.mlp.2.bias");
  m->ytab = take((int64_t)n_cls * D, "y_embedder.embedding_table.weight");
  m->freqs = reserve(128);
  m->ada_w = reserve((int64_t)m->ada_total * D);
  m->ada_b = reserve(m->ada_total);
  for (int b = 0; b < a.depth; ++b) {
    BlockP bp;
    bp.qkv_w = take((int64_t)3 * D * D, "attn.qkv.weight");
    bp.qkv_b = take(3 * D, "attn.qkv.bias");
    bp.proj_w = take((int64_t)D * D, "attn.proj.weight");
    bp.proj_b = take(D, "attn.proj.bias");
    bp.fc1_w = take((int64_t)Hm * D, "mlp.fc1.weight");
    bp.fc1_b = take(Hm, "mlp.fc1.bias");
    bp.fc2_w = take((int64_t)D * Hm, "mlp.fc2.weight");
    bp.fc2_b = take(D, "mlp.fc2.bias");
    take_at((int64_t)6 * D * D, m->ada_w + (size_t)b * 6 * D * D, "adaLN_modulation.1.weight");
    take_at(6 * D, m->ada_b + (size_t)b * 6 * D, "adaLN_modulation.1.bias");
    m->blocks.push_back(bp);
  }
  m->fin_w = take((int64_t)m->PP * m->OC * D, "final_layer.linear.weight");
  m->fin_b = take(m->PP * m->OC, "final_layer.linear.bias");
  take_at((int64_t)2 * D * D, m->ada_w + (size_t)a.depth * 6 * D * D, "final_layer.adaLN_modulation.1.weight");
  take_at(2 * D, m->ada_b + (size_t)a.depth * 6 * D, "final_layer.adaLN_modulation.1.bias");
  if (!err.empty()) {
    set_error(err);
    return DM_ERR_ARG;
  }
  DM_REQUIRE(idx == n_params, "parameter count mismatch after walk");

  m->arena_floats = size;
  DM_CHECK_HIP(hipMalloc(&m->arena, size * sizeof(float)));
  for (auto& c : copies) {
    DM_REQUIRE(params[c.idx] != nullptr, "null parameter pointer");
    DM_CHECK_HIP(hipMemcpyAsync(m->arena + c.dst, params[c.idx], c.n * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  *out = m.release();
  return DM_OK;
}

int DiTModel::build_plan(Plan& pl, int B) {
  refresh_toggles();
  pl.toggles = toggles();
  ToggleScope scope(pl.toggles);
  pl.graph_enabled = toggles().graph;
  pl.B = B;
  pl.math = math;
  const dm_dit_arch& a = arch;
  const int p = a.patch_size, C = a.in_channels, S = a.input_size, Hm = a.mlp_hidden;
  const int heads = a.num_heads, Dh = D / heads;
  const long M = (long)B * T;
  DM_REQUIRE((long)B * heads <= 65535, "batch * heads too large for one attention launch");

  if (!range_flag) {
    DM_CHECK_HIP(hipMalloc(&range_flag, sizeof(int)));
    DM_CHECK_HIP(hipMemset(range_flag, 0, sizeof(int)));
    DM_CHECK_HIP(hipHostMalloc(&range_flag_host, sizeof(int)));
  }
  if (!sk_ws && toggles().lin_sk && linear_k32_slots() > 0) {
    const int slots = linear_k32_slots();
    DM_CHECK_HIP(hipMalloc(&sk_ws, (size_t)slots * 65536));
    DM_CHECK_HIP(hipMalloc(&sk_cnt, (size_t)slots * sizeof(unsigned)));
    DM_CHECK_HIP(hipMemset(sk_cnt, 0, (size_t)slots * sizeof(unsigned)));
    sk_cap = slots;
  }
  const bool sk_on = toggles().lin_sk && sk_ws;
  pl.x = pl.alloc((size_t)B * C * S * S * 4);
  pl.t = (int64_t*)pl.alloc((size_t)B * 8);
  pl.y = (int64_t*)pl.alloc((size_t)B * 8);
  pl.out = pl.alloc((size_t)B * OC * S * S * 4);
  float* e0 = pl.alloc((size_t)B * 256 * 4);
  float* e1 = pl.alloc((size_t)B * D * 4);
  float* temb = pl.alloc((size_t)B * D * 4);
  float* se = pl.alloc((size_t)B * D * 4);
  float* mods = pl.alloc((size_t)B * ada_total * 4);
  float* a0 = pl.alloc((size_t)M * C * p * p * 4);
  float* x = pl.alloc((size_t)M * D * 4);
  float2* stats = (float2*)pl.alloc((size_t)M * sizeof(float2));
  float* qkv = pl.alloc((size_t)M * 3 * D * 4);
  float* Sb = nullptr;  // score matrix of the unfused attention path (allocated on first use)
  float* Ob = pl.alloc((size_t)M * D * 4);
  float* hb = pl.alloc((size_t)M * Hm * 4);
  float* lin = pl.alloc((size_t)M * PP * OC * 4);
  if (pl.alloc_failed) { set_error("workspace allocation failed"); return DM_ERR_HIP; }

  Plan* P_ = &pl;
  DiTModel* self = this;
  auto add_gemm = [&](const GemmArgs& g) {
    const double Z = (double)g.Z1 * g.Z2;
    const double fl = 2.0 * Z * g.M * g.N * g.K;
    const double by = 4.0 * Z * ((double)g.M * g.K + (double)g.N * g.K + (double)g.M * g.N) +
                      (g.res ? 4.0 * g.M * g.N : 0.0);
    pl.add(gemm_label(g), fl, by, [=](hipStream_t st) { return gemm_batched(g, st); });
  };
  // token GEMMs on linear_k32: LayerNorm-modulate (or nothing) + fp16x2 split of A once per GEMM
  // (linear_presplit_a) instead of once per 128-column tile inside it (27 x for qkv, 36 x for fc1);
  // one buffer shared by all of them (stream-ordered). DM_DIT_PRESPLIT=0: split inside the GEMM.
  const bool presplit_on = toggles().dit_presplit;
  _Float16* as_buf = nullptr;
  size_t as_bytes = 0;
  // LayerNorm statistics for the next GEMM with the LN + modulate prologue: computed by that GEMM's
  // row_stats_split pass (statistics + prologue + split in one read of the tokens) or by row_stats
  bool stats_pending = false;
  const float ln_eps = 1e-6f;
  auto flush_stats = [&]() {
    if (!stats_pending) return;
    stats_pending = false;
    pl.add("row_stats", 0, 4.0 * M * D, [=](hipStream_t st) { return row_stats(x, M, D, ln_eps, stats, st); });
  };
  auto add_token_gemm = [&](GemmArgs g) {
    // nominal-batch decision (pick_M = T * kPickBatch): the same kernels at every B, so results are
    // batch-invariant (each image's row block of B * T tokens runs the same code)
    if (g.ws && presplit_on && g.pick_M >= 4096) {
      const size_t need = (size_t)g.M * g.K * 4;
      if (need > as_bytes) {
        as_buf = reinterpret_cast<_Float16*>(pl.alloc(need));
        as_bytes = need;
      }
      GemmArgs g2 = g;
      g2.as = as_buf;
      g2.pro_scale = g2.pro_shift = nullptr;
      g2.ln_stats = nullptr;
      if (as_buf && linear_k32_ok(g2)) {
        _Float16* buf = as_buf;
        if (g.ln_stats && stats_pending && g.A == x && g.lda == D && g.K == D && g.alpha == 1.0f) {
          stats_pending = false;
          float2* sp = stats;
          pl.add("row_stats_split", 0, 8.0 * g.M * g.K, [=](hipStream_t st) {
            return row_stats_split(g.A, g.M, g.K, ln_eps, sp, g.ln_shift, g.ln_scale, g.ln_pitch, g.ln_rows, g.split_ea,
                                   buf, g.range_flag, st);
          });
        } else {
          flush_stats();
          pl.add("linear_presplit_a", 0, 8.0 * g.M * g.K, [=](hipStream_t st) { return linear_presplit_a(g, buf, st); });
        }
        add_gemm(g2);
        return;
      }
    }
    flush_stats();
    add_gemm(g);
  };
  // fp16x2 operand exponents (unet_exec.hip split_gemm): weights by max |w|, activations fixed (2^6 for
  // LayerNorm-modulated tokens, q, k, v, attention and MLP outputs; 2^14 for softmax rows)
  auto split = [&](GemmArgs& g, int ea, size_t w, size_t wn, int eb_act) {
    if (math != 2) return;
    int eb = eb_act;
    if (wn) {
      auto it = w_exp.find(P(w));
      if (it == w_exp.end()) it = w_exp.emplace(P(w), split_weight_exponent(P(w), wn)).first;
      eb = it->second;
    }
    g.split = 2; g.split_ea = ea; g.split_eb = eb; g.range_flag = range_flag;
    // static weight [N][K]: pre-split once for linear_k32 (the gemm.hip path stays the fallback)
    if (wn && linear_k32_on && g.K % 64 == 0 && g.N % 4 == 0) {
      const float* wp = P(w);
      auto it = split_w.find(wp);
      if (it == split_w.end()) {
        void* buf = nullptr;
        const size_t nb = split_conv_weights_bytes(1, g.N, g.K, 2);
        if (hipMalloc(&buf, nb) != hipSuccess) return;
        if (split_conv_weights(wp, 1, g.N, g.K, g.K, 1, 2, buf, nullptr) != DM_OK || hipDeviceSynchronize() != hipSuccess) {
          (void)hipFree(buf);
          return;
        }
        it = split_w.emplace(wp, buf).first;
        split_bytes += nb;
      }
      g.ws = it->second;
      g.ws_rowscale = split_conv_rowscale(it->second, 1, g.N, g.K);
      if (sk_on) {
        g.sk_ws = sk_ws;
        g.sk_cnt = sk_cnt;
        g.sk_cap = sk_cap;
      }
      // with the pre-split A image (add_token_gemm) the GEMM takes no prologue: check that form
      GemmArgs probe = g;
      if (presplit_on && g.pick_M >= 4096 && !probe.c_split) {
        probe.ln_stats = nullptr;
        probe.pro_scale = probe.pro_shift = nullptr;
        probe.as = reinterpret_cast<const _Float16*>(uintptr_t(256));  // only its alignment is checked
      }
      if (!linear_k32_ok(probe)) {
        g.ws = nullptr;
        g.ws_rowscale = nullptr;
      }
    }
  };
  auto linear = [&](const float* A, int lda, long rows, size_t w, size_t bias, int N, int K, float* out, int ldc) {
    GemmArgs g{};
    g.M = (int)rows; g.N = N; g.K = K; g.Z1 = 1; g.Z2 = 1; g.pick_M = rows / B * kPickBatch;  // rows = B or B*T
    g.A = A; g.lda = lda; g.Bm = P(w); g.ldb = K; g.C = out; g.ldc = ldc; g.alpha = 1.f;
    g.bias = bias != (size_t)-1 ? P(bias) : nullptr;
    return g;
  };

  // --- conditioning: t_embedder (dit/model.py:40-64), y_embedder, c = t + y, SiLU for every adaLN
  pl.add("timestep_embed", 0, 4.0 * B * 256, [=](hipStream_t st) {
    return timestep_embed(P_->t, B, 256, 1, self->freqs_set ? self->P(self->freqs) : nullptr, e0, st);
  });
  {
    GemmArgs g = linear(e0, 256, B, tw1, tb1, D, 256, e1, D);
    g.act = 1;
    add_gemm(g);
    add_gemm(linear(e1, D, B, tw2, tb2, D, D, temb, D));
  }
  {
    const float* table = P(ytab);
    const int null_row = a.null_class ? a.num_classes : -1;
    pl.add("class_embed_silu", 0, 8.0 * B * D, [=](hipStream_t st) {
      return embed_add_silu(temb, P_->y, table, B, D, se, st, null_row);
    });
  }
  // every block's (and the final layer's) adaLN modulation in one GEMM: [B][depth * 6D + 2D]. A weight stream
  // (902 MB for DiT-XL/2 against 2B = 64 rows): on linear_k32 with the weights pre-split once, one block per
  // 128 columns streaming its K x 128 slice (the fp32 gemm_kernel took 558 us, 1.6 TB/s)
  {
    GemmArgs g = linear(se, D, B, ada_w, ada_b, ada_total, D, mods, ada_total);
    split(g, 6, ada_w, (size_t)ada_total * D, 6);
    add_gemm(g);
  }

  // --- patch embedding + pos_embed (dit/model.py:244)
  pl.add("patchify", 0, 8.0 * M * C * p * p,
         [=](hipStream_t st) { return patchify(P_->x, B, C, S, S, p, a0, st); });
  {
    GemmArgs g = linear(a0, C * p * p, M, xw, xb, D, C * p * p, x, D);
    g.res = P(pos); g.ld_res = D; g.res_mod = T;
    add_gemm(g);
  }

  auto stats_op = [&]() { stats_pending = true; };
  for (int b = 0; b < a.depth; ++b) {
    const BlockP bp = blocks[b];
    const float* mb = mods + (size_t)b * 6 * D;  // shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp
    // attention branch
    stats_op();
    GemmArgs gq = linear(x, D, M, bp.qkv_w, bp.qkv_b, 3 * D, D, qkv, 3 * D);
    gq.ln_stats = stats; gq.ln_shift = mb; gq.ln_scale = mb + D; gq.ln_pitch = ada_total; gq.ln_rows = T;
    split(gq, 6, bp.qkv_w, (size_t)3 * D * D, 0);
    // flash attention (attention.hip attn_flash_kernel): the qkv GEMM's epilogue writes q * d^-1/2, k, v as
    // the fp16x2 operand planes (over the qkv buffer: same bytes), S never leaves the CU
    const bool flash = math == 2 && gq.ws && attn_flash_ok(T, Dh) && toggles().attn != kAttnUnfused;
    _Float16* planes = reinterpret_cast<_Float16*>(qkv);
    const size_t plane_n = (size_t)M * D * 2;   // fp16 elements of one operand's two planes
    if (flash) {
      gq.ap_q = planes; gq.ap_k = planes + plane_n; gq.ap_v = planes + 2 * plane_n;
      gq.ap_L = T; gq.ap_heads = heads; gq.ap_Dh = Dh; gq.ap_legacy = 0;
      gq.ap_alpha = (float)std::pow((double)Dh, -0.5); gq.ap_bscale = 0.f;
      gq.ap_ea = 6; gq.ap_eb = 6; gq.ap_ev = 6;
    }
    add_token_gemm(gq);
    // the proj GEMM, built before the attention op: the flash kernel writes O as the proj's pre-split A image
    // only when this GEMM is the one that will read it (same predicate), else O as fp32 rows
    GemmArgs gpj = linear(Ob, D, M, bp.proj_w, bp.proj_b, D, D, x, D);
    gpj.res = x; gpj.ld_res = D; gpj.gate = mb + 2 * D; gpj.gate_pitch = ada_total; gpj.gate_rows = T;
    split(gpj, 6, bp.proj_w, (size_t)D * D, 0);
    GemmArgs gpj_as = gpj;
    gpj_as.as = reinterpret_cast<const _Float16*>(Ob);
    const bool o_presplit = flash && presplit_on && D % 32 == 0 && gpj.ws && gpj.split_ea == 6 && linear_k32_ok(gpj_as);
    if (flash) {
      AttnArgs at{};
      at.pq = planes; at.pk = planes + plane_n; at.pv = planes + 2 * plane_n;
      at.L = T; at.Dh = Dh; at.heads = heads; at.B = B;
      at.out = Ob; at.ldo = D;
      at.ea = 6; at.eb = 6; at.ep = 14; at.ev = 6;
      at.range_flag = range_flag;
      if (o_presplit) {   // O straight into the proj GEMM's pre-split A image (over Ob)
        at.o_split = reinterpret_cast<_Float16*>(Ob);
        at.o_split_ea = 6;
        at.o_ld = D;
      }
      pl.add("attn_flash_kernel<" + std::to_string(Dh) + ">", 4.0 * B * heads * (double)T * T * Dh,
             4.0 * M * (3.0 * D + D), [=](hipStream_t st) { return attn_flash(at, st); });
    } else {
      if (!Sb) Sb = pl.alloc((size_t)B * heads * T * T * 4);
      // timm Attention: qkv.reshape(B, N, 3, heads, d): q / k / v of head h at columns h*d, D + h*d, 2D + h*d
      GemmArgs gs{};
      gs.M = T; gs.N = T; gs.K = Dh; gs.Z1 = B; gs.Z2 = heads; gs.pick_Z = (long)kPickBatch * heads;
      gs.A = qkv; gs.a_s1 = (long)T * 3 * D; gs.a_s2 = Dh; gs.lda = 3 * D;
      gs.Bm = qkv + D; gs.b_s1 = (long)T * 3 * D; gs.b_s2 = Dh; gs.ldb = 3 * D;
      gs.C = Sb; gs.c_s1 = (long)heads * T * T; gs.c_s2 = (long)T * T; gs.ldc = T;
      gs.alpha = (float)std::pow((double)Dh, -0.5);
      split(gs, 6, 0, 0, 6);
      add_gemm(gs);
      const long rows = (long)B * heads * T;
      const int L = T;
      pl.add("softmax_rows", 0, 8.0 * rows * L, [=](hipStream_t st) { return softmax_rows(Sb, rows, L, L, st); });
      GemmArgs go{};
      go.M = T; go.N = Dh; go.K = T; go.Z1 = B; go.Z2 = heads; go.pick_Z = (long)kPickBatch * heads;
      go.A = Sb; go.a_s1 = (long)heads * T * T; go.a_s2 = (long)T * T; go.lda = T;
      go.Bm = qkv + 2 * D; go.b_s1 = (long)T * 3 * D; go.b_s2 = Dh; go.ldb = 3 * D; go.b_kn = 1;
      go.C = Ob; go.c_s1 = (long)T * D; go.c_s2 = Dh; go.ldc = D;
      go.alpha = 1.f;
      split(go, 14, 0, 0, 6);
      add_gemm(go);
    }
    if (o_presplit)
      add_gemm(gpj_as);   // A = the flash kernel's pre-split O image
    else
      add_token_gemm(gpj);
    // MLP branch
    stats_op();
    {
      GemmArgs g = linear(x, D, M, bp.fc1_w, bp.fc1_b, Hm, D, hb, Hm);
      g.ln_stats = stats; g.ln_shift = mb + 3 * D; g.ln_scale = mb + 4 * D; g.ln_pitch = ada_total; g.ln_rows = T;
      g.act = 2;
      split(g, 6, bp.fc1_w, (size_t)Hm * D, 0);
      GemmArgs g2 = linear(hb, Hm, M, bp.fc2_w, bp.fc2_b, D, Hm, x, D);
      g2.res = x; g2.ld_res = D; g2.gate = mb + 5 * D; g2.gate_pitch = ada_total; g2.gate_rows = T;
      split(g2, 6, bp.fc2_w, (size_t)D * Hm, 0);
      // fc1's epilogue writes GELU(h) as fc2's pre-split A image (over hb: same bytes), no split pass for fc2
      GemmArgs g1s = g, g2s = g2;
      g1s.c_split = reinterpret_cast<_Float16*>(hb);
      g1s.c_split_ea = g2.split_ea;
      g2s.as = reinterpret_cast<const _Float16*>(hb);
      if (presplit_on && g.ws && g2.ws && linear_k32_ok(g1s) && linear_k32_ok(g2s)) {
        add_token_gemm(g1s);
        add_gemm(g2s);
      } else {
        add_token_gemm(g);
        add_token_gemm(g2);
      }
    }
  }
  // --- final layer (dit/model.py:138-142) + unpatchify
  stats_op();
  {
    const float* mf = mods + (size_t)a.depth * 6 * D;  // shift, scale
    GemmArgs g = linear(x, D, M, fin_w, fin_b, PP * OC, D, lin, PP * OC);
    g.ln_stats = stats; g.ln_shift = mf; g.ln_scale = mf + D; g.ln_pitch = ada_total; g.ln_rows = T;
    split(g, 6, fin_w, (size_t)PP * OC * D, 0);
    add_token_gemm(g);
  }
  if (pl.alloc_failed) { set_error("workspace allocation failed"); return DM_ERR_HIP; }
  const int oc = OC;
  pl.add("unpatchify", 0, 8.0 * M * PP * OC,
         [=](hipStream_t st) { return unpatchify(lin, B, oc, S, S, p, P_->out, st); });
  return DM_OK;
}

}  // namespace dm

// ===========================================================================
// C ABI
// ===========================================================================
struct dm_dit {
  dm::DiTModel* m;
};

extern "C" int dm_dit_param_count(const dm_dit_arch* arch, int* n_params) {
  int rc = dm::dit_validate(arch);
  if (rc) return rc;
  if (!n_params) { dm::set_error("n_params is null"); return DM_ERR_ARG; }
  *n_params = dm::dit_count(*arch);
  return DM_OK;
}

extern "C" int dm_dit_create(const dm_dit_arch* arch, const float* const* params, const int64_t* numels,
                             int n_params, void* stream, dm_dit** out) {
  if (!out || !params || !numels) { dm::set_error("null argument"); return DM_ERR_ARG; }
  dm::DiTModel* m = nullptr;
  int rc = dm::dit_create(arch, params, numels, n_params, (hipStream_t)stream, &m);
  if (rc) return rc;
  *out = new dm_dit{m};
  return DM_OK;
}

extern "C" int dm_dit_forward(dm_dit* h, const float* x, const int64_t* t, const int64_t* y, int B, float* out,
                              void* stream) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (!x || !t || !out) { dm::set_error("null tensor"); return DM_ERR_ARG; }
  if (B <= 0) { dm::set_error("empty batch"); return DM_ERR_ARG; }
  if (static_cast<const void*>(out) == static_cast<const void*>(x)) {
    dm::set_error("out must not alias x");
    return DM_ERR_ARG;
  }
  dm::DiTModel* m = h->m;
  hipStream_t st = (hipStream_t)stream;
  const int S = m->arch.input_size;
  const size_t nx = (size_t)B * m->arch.in_channels * S * S, no = (size_t)B * m->OC * S * S;
  // at most two passes: the caller's arithmetic, then (an fp16x2 operand beyond the fp16 range) fp32
  if (const int rco = m->plans.pool->order(st)) return rco;
  // every exit after order() records the completion event, so a later forward on another stream waits for
  // whatever this one enqueued over the shared slab, even when it failed part way
  const int rc_body = [&]() -> int {
    for (int math = m->run_math();;) {
      dm::DiTModel::Plan* plp = nullptr;
      const int rc0 = m->get_plan(B, math, &plp);
      if (rc0) return rc0;
      auto& pl = *plp;
      DM_CHECK_HIP(hipMemcpyAsync(pl.x, x, nx * sizeof(float), hipMemcpyDeviceToDevice, st));
      DM_CHECK_HIP(hipMemcpyAsync(pl.t, t, (size_t)B * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
      if (y)
        DM_CHECK_HIP(hipMemcpyAsync(pl.y, y, (size_t)B * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
      else
        DM_CHECK_HIP(hipMemsetAsync(pl.y, 0xff, (size_t)B * sizeof(int64_t), st));  // -1: the null class
      const int rc = pl.run(st);
      if (rc) return rc;
      DM_CHECK_HIP(hipMemcpyAsync(out, pl.out, no * sizeof(float), hipMemcpyDeviceToDevice, st));
      if (math != 2 || !m->range_check || m->range_deferred) break;
      DM_CHECK_HIP(hipMemcpyAsync(m->range_flag_host, m->range_flag, sizeof(int), hipMemcpyDeviceToHost, st));
      DM_CHECK_HIP(hipStreamSynchronize(st));
      if (!*m->range_flag_host) break;
      DM_CHECK_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));
      m->range_fallbacks++;
      math = 0;
    }
    return DM_OK;
  }();
  const int rc_mark = m->plans.pool->mark(st);
  return rc_body ? rc_body : rc_mark;
}

extern "C" int dm_dit_set_range_deferred(dm_dit* h, int deferred) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  h->m->range_deferred = deferred != 0;
  return DM_OK;
}

extern "C" int dm_dit_range_poll(dm_dit* h, void* stream, int* flagged) {
  if (!h || !h->m || !flagged) { dm::set_error("null model / argument"); return DM_ERR_STATE; }
  dm::DiTModel* m = h->m;
  *flagged = 0;
  if (!m->range_flag) return DM_OK;
  hipStream_t st = (hipStream_t)stream;
  DM_CHECK_HIP(hipMemcpyAsync(m->range_flag_host, m->range_flag, sizeof(int), hipMemcpyDeviceToHost, st));
  DM_CHECK_HIP(hipStreamSynchronize(st));
  if (*m->range_flag_host) {
    DM_CHECK_HIP(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));
    *flagged = 1;
    if (m->base_math == 2) {  // the caller re-runs what it computed since the last poll: in fp32
      m->fallback = true;
      m->range_fallbacks++;
    }
  }
  return DM_OK;
}

extern "C" int dm_dit_range_fallback(dm_dit* h, int on) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  h->m->fallback = on != 0;
  return DM_OK;
}

extern "C" int dm_dit_range_stats(const dm_dit* h, int64_t* fallbacks, int* active) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (fallbacks) *fallbacks = h->m->range_fallbacks;
  if (active) *active = h->m->run_math();
  return DM_OK;
}

extern "C" int dm_dit_set_math(dm_dit* h, int kind) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (kind != 0 && kind != DM_SPLIT_FP16X2) { dm::set_error("DiT math must be 0 (fp32) or DM_SPLIT_FP16X2"); return DM_ERR_ARG; }
  h->m->fallback = false;
  if (kind != h->m->base_math) {
    h->m->base_math = kind;
    h->m->plans.clear();
  }
  return DM_OK;
}

extern "C" int dm_dit_get_math(const dm_dit* h, int* kind) {
  if (!h || !h->m || !kind) { dm::set_error("null model"); return DM_ERR_STATE; }
  *kind = h->m->base_math;
  return DM_OK;
}

extern "C" int dm_dit_set_time_freqs(dm_dit* h, const float* freqs, int n, void* stream) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (!freqs) {
    h->m->freqs_set = false;
    h->m->plans.invalidate_graphs();
    return DM_OK;
  }
  if (n != 128) { dm::set_error("time frequency table must have 128 entries"); return DM_ERR_ARG; }
  DM_CHECK_HIP(hipMemcpyAsync(h->m->P(h->m->freqs), freqs, 128 * sizeof(float), hipMemcpyDefault,
                              (hipStream_t)stream));
  h->m->freqs_set = true;
  h->m->plans.invalidate_graphs();
  return DM_OK;
}

extern "C" int dm_dit_profile(dm_dit* h, int enable) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (!h->m->plans.current()) { dm::set_error("no plan yet: run dm_dit_forward once first"); return DM_ERR_STATE; }
  h->m->plans.current()->profile_enable(enable);
  return DM_OK;
}

extern "C" int dm_dit_profile_count(dm_dit* h, int* n_ops) {
  if (!h || !h->m || !h->m->plans.current() || !n_ops) { dm::set_error("null model / no plan"); return DM_ERR_STATE; }
  *n_ops = (int)h->m->plans.current()->ops.size();
  return DM_OK;
}

extern "C" int dm_dit_profile_get(dm_dit* h, int i, char* label, int label_len, double* flops, double* bytes,
                                  double* ms_total, int64_t* launches) {
  if (!h || !h->m || !h->m->plans.current()) { dm::set_error("null model / no plan"); return DM_ERR_STATE; }
  return h->m->plans.current()->profile_get(i, label, label_len, flops, bytes, ms_total, launches);
}

extern "C" int dm_dit_memory(const dm_dit* h, int64_t* weight_bytes, int64_t* workspace_bytes) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  // the fp32 arena plus the pre-split fp16x2 copies of the token-GEMM weights (as dm_unet_memory counts them)
  if (weight_bytes) *weight_bytes = (int64_t)(h->m->arena_floats * sizeof(float) + h->m->split_bytes);
  if (workspace_bytes) *workspace_bytes = (int64_t)h->m->plans.pool->bytes();
  return DM_OK;
}

extern "C" int dm_dit_plan_stats(const dm_dit* h, int64_t* builds, int* cached) {
  if (!h || !h->m) { dm::set_error("null model"); return DM_ERR_STATE; }
  if (builds) *builds = h->m->plans.builds;
  if (cached) *cached = (int)h->m->plans.plans.size();
  return DM_OK;
}

extern "C" void dm_dit_destroy(dm_dit* h) {
  if (!h) return;
  (void)hipDeviceSynchronize();
  delete h->m;
  delete h;
}
