// attn_block variant 3 probe (tools/probe/attn3_probe.cpp, diagnostics only): drives dm::attn_block on one image
// with structured folded weights and compares y against a float64 host evaluation of the folded formula
//   xn = x gsc + gsh, T = xn At^T + w, P = softmax_j(T_i . xn_j), y = x + (P xn) Wg^T + cb
// cases: 0 At = 0, Wg = I (y = x + mean xn); 1 At = 0, Wg random; 2 At random, Wg = I; 3 all random.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "dm_kernels.h"

using namespace dm;
static const int L = 256, C = 256;

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error line %d\n", __LINE__); return 2; } } while (0)

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 3;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  int fails = 0;
  for (int cs = 0; cs < 4; ++cs) {
    std::vector<float> x(L * C), gsc(C), gsh(C), at(C * C, 0.f), w(C, 0.f), wg(C * C, 0.f), cb(C, 0.f);
    for (auto& v : x) v = nd(rng);
    for (int c = 0; c < C; ++c) { gsc[c] = 1.f + 0.1f * nd(rng); gsh[c] = 0.1f * nd(rng); }
    if (cs >= 2) { for (auto& v : at) v = 0.02f * nd(rng); for (auto& v : w) v = 0.1f * nd(rng); }
    if (cs == 1 || cs == 3) { for (auto& v : wg) v = 0.06f * nd(rng); for (auto& v : cb) v = 0.1f * nd(rng); }
    else for (int c = 0; c < C; ++c) wg[c * C + c] = 1.f;
    // host float64
    std::vector<double> xn(L * C), T(L * C), O(L * C), yr(L * C);
    for (int i = 0; i < L; ++i) for (int c = 0; c < C; ++c) xn[i * C + c] = (double)x[i * C + c] * gsc[c] + gsh[c];
    for (int i = 0; i < L; ++i) for (int r = 0; r < C; ++r) {
      double s = w[r];
      for (int c = 0; c < C; ++c) s += xn[i * C + c] * at[r * C + c];
      T[i * C + r] = s;
    }
    for (int i = 0; i < L; ++i) {
      std::vector<double> S(L);
      double m = -1e300;
      for (int j = 0; j < L; ++j) { double s = 0; for (int c = 0; c < C; ++c) s += T[i * C + c] * xn[j * C + c]; S[j] = s; m = std::max(m, s); }
      double l = 0; for (int j = 0; j < L; ++j) { S[j] = std::exp(S[j] - m); l += S[j]; }
      for (int c = 0; c < C; ++c) { double o = 0; for (int j = 0; j < L; ++j) o += S[j] * xn[j * C + c]; O[i * C + c] = o / l; }
    }
    for (int i = 0; i < L; ++i) for (int d = 0; d < C; ++d) {
      double s = (double)x[i * C + d] + cb[d];
      for (int c = 0; c < C; ++c) s += O[i * C + c] * wg[d * C + c];
      yr[i * C + d] = s;
    }
    // device
    float *dx, *dgsc, *dgsh, *dat, *dw, *dwg, *dwgp, *dcb, *dy; void *atimg, *wgimg; int* flag;
    const size_t nimg = split_conv_weights_bytes(1, C, C, 2);
    CK(hipMalloc(&dx, 4 * L * C)); CK(hipMalloc(&dy, 4 * L * C)); CK(hipMalloc(&dgsc, 4 * C)); CK(hipMalloc(&dgsh, 4 * C));
    CK(hipMalloc(&dat, 4 * C * C)); CK(hipMalloc(&dwg, 4 * C * C)); CK(hipMalloc(&dwgp, 4 * C * C));
    CK(hipMalloc(&dw, 4 * C)); CK(hipMalloc(&dcb, 4 * C)); CK(hipMalloc(&atimg, nimg)); CK(hipMalloc(&wgimg, nimg));
    CK(hipMalloc(&flag, 4)); CK(hipMemset(flag, 0, 4));
    CK(hipMemcpy(dx, x.data(), 4 * L * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(dgsc, gsc.data(), 4 * C, hipMemcpyHostToDevice)); CK(hipMemcpy(dgsh, gsh.data(), 4 * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(dat, at.data(), 4 * C * C, hipMemcpyHostToDevice)); CK(hipMemcpy(dwg, wg.data(), 4 * C * C, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, w.data(), 4 * C, hipMemcpyHostToDevice)); CK(hipMemcpy(dcb, cb.data(), 4 * C, hipMemcpyHostToDevice));
    if (split_conv_weights(dat, 1, C, C, C, 1, 2, atimg, nullptr) != 0 || attn_perm_cols(dwg, dwgp, C, nullptr) != 0 ||
        split_conv_weights(dwgp, 1, C, C, C, 1, 2, wgimg, nullptr) != 0) { printf("prep failed\n"); return 2; }
    CK(hipDeviceSynchronize());
    AttnBlockArgs a{};
    a.x = dx; a.x_pitch = C; a.gsc = dgsc; a.gsh = dgsh;
    a.at_img = (const _Float16*)atimg; a.at_rowscale = split_conv_rowscale(atimg, 1, C, C); a.w = dw;
    a.wg_img = (const _Float16*)wgimg; a.wg_rowscale = split_conv_rowscale(wgimg, 1, C, C); a.cb = dcb;
    a.variant = variant; a.y = dy; a.y_pitch = C; a.B = 1; a.ex = 6; a.eg = 6; a.range_flag = flag;
    if (attn_block(a, nullptr) != 0) { printf("launch failed\n"); return 2; }
    CK(hipDeviceSynchronize());
    std::vector<float> y(L * C);
    CK(hipMemcpy(y.data(), dy, 4 * L * C, hipMemcpyDeviceToHost));
    double e = 0, emax_tok[L] = {0};
    int worst = 0;
    for (int i = 0; i < L; ++i) for (int d = 0; d < C; ++d) {
      const double v = std::fabs(y[i * C + d] - yr[i * C + d]);
      emax_tok[i] = std::max(emax_tok[i], v);
      if (v > e) { e = v; worst = i * C + d; }
    }
    printf("case %d: max err %.3e at token %d ch %d (got %.5f want %.5f)\n", cs, e, worst / C, worst % C, y[worst], yr[worst]);
    printf("  per-token max err, tokens 0..15:");
    for (int i = 0; i < 16; ++i) printf(" %.1e", emax_tok[i]);
    printf("\n  tokens 128..135:");
    for (int i = 128; i < 136; ++i) printf(" %.1e", emax_tok[i]);
    printf("\n");
    if (cs == 0) {
      printf("  token 5, d: (y - x) vs O:");
      for (int d = 0; d < 40; ++d) printf(" %d:%.3f/%.3f", d, y[5 * C + d] - x[5 * C + d], O[5 * C + d]);
      printf("\n");
      // is (y - x) a permutation / sum of O columns? print the xn column means by channel
      double so = 0, sy = 0;
      for (int d = 0; d < C; ++d) { so += O[5 * C + d]; sy += y[5 * C + d] - x[5 * C + d]; }
      printf("  sum over channels: y - x %.4f, O %.4f\n", sy, so);
    }
    if (!(e < 1e-4)) ++fails;
    (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dgsc); (void)hipFree(dgsh); (void)hipFree(dat); (void)hipFree(dwg);
    (void)hipFree(dwgp); (void)hipFree(dw); (void)hipFree(dcb); (void)hipFree(atimg); (void)hipFree(wgimg); (void)hipFree(flag);
  }
  printf("attn3 probe variant %d: %d failing cases\n", variant, fails);
  return fails ? 1 : 0;
}
