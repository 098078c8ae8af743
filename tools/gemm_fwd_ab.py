#!/usr/bin/env python3
"""Where pass F of the 64-chain full-data sweep (sweep.hip: k_gemm_fwd) spends its time:
writes tools/_bin/gemm_ab_src/gemm_ab.hip -- the product sweep.hip included as is, plus an
ablation copy k_gemm_fwd_x<FAM, ABL> made by text substitution from the product kernel (bit 0:
no beta^T LDS-DMA, 1: no X LDS-DMA, 2: no tile epilogue, 3: no MFMAs; ablated arms compute
garbage and are timed only) -- and a harness that times the product pass F, the ablations and
pass B at configs[4]'s shape (d = 1000, 64 chains) on synthetic rows; builds it with hipcc.
The product source is not changed.

usage: tools/gemm_fwd_ab.py   (then on the GPU: tools/_bin/gemm_ab [rows_per_shard] [shards] [rounds])"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_bin", "gemm_ab_src")


def ablation_copy(src):
    i = src.index("template <int FAM>\n__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd(SweepArgs A) {")
    j = src.index("\n}\n", i) + 3
    k = src[i:j]
    k = k.replace("template <int FAM>\n__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd(SweepArgs A) {",
                  "template <int FAM, int ABL>\n__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd_x(SweepArgs A) {")
    old_x = "#pragma unroll\n    for (int i = 0; i < NDMA; ++i)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr,"
    assert k.count(old_x) == 1
    k = k.replace(old_x, "#pragma unroll\n    for (int i = 0; i < NDMA; ++i)\n      if constexpr (!(ABL & 2)) __builtin_amdgcn_raw_ptr_buffer_load_lds(xr,")
    old_b = "#pragma unroll\n    for (int i = 0; i < NDMA; ++i)\n      __builtin_amdgcn_raw_ptr_buffer_load_lds(br,"
    assert k.count(old_b) == 1
    k = k.replace(old_b, "#pragma unroll\n    for (int i = 0; i < NDMA; ++i)\n      if constexpr (!(ABL & 1)) __builtin_amdgcn_raw_ptr_buffer_load_lds(br,")
    old_e = "    if (kc == NKC - 1) {                                 // ---- tile epilogue"
    assert k.count(old_e) == 1
    # ABL 4: the epilogue reduced to folding the accumulators into lp (so the MFMAs stay live)
    k = k.replace(old_e, "    if ((ABL & 4) && kc == NKC - 1) {\n#pragma unroll\n      for (int c2 = 0; c2 < NCT; ++c2) gaa[c2] += acc[c2][0] + acc[c2][1] + acc[c2][2] + acc[c2][3];\n    }\n"
                         "    if (!(ABL & 4) && kc == NKC - 1) {                   // ---- tile epilogue")
    old_m = "        acc[c2] = mfma_f64(a,"
    assert k.count(old_m) == 1
    k = k.replace(old_m, "        if constexpr (!(ABL & 8)) acc[c2] = mfma_f64(a,")
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def deferred_copy(src):
    """k_gemm_fwd_d<FAM>: the product pass F with the tile's R stores issued at the top of the
    next stage (after its barrier and DMA issue) instead of at the tile's end followed by
    vmcnt(0): the stores' write latency then runs under the next stage's MFMAs and is waited for
    by the following stage's vmcnt(0) (NS = 2: every stage waits for vmcnt(0) anyway)."""
    i = src.index("template <int FAM>\n__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd(SweepArgs A) {")
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_d(SweepArgs A) {")
    old_loop = "  for (int st = 0; st < nst; ++st) {\n    const int kc = st % NKC;\n"
    assert k.count(old_loop) == 1
    k = k.replace(old_loop, "  double rdv[NCT][4];\n  int rtile = -1;\n"
                  "  auto flush_r = [&]() {\n#pragma unroll\n    for (int c2 = 0; c2 < NCT; ++c2)\n#pragma unroll\n"
                  "      for (int i = 0; i < 4; ++i)\n        *reinterpret_cast<double*>(Rimg + g5_chain_off(rtile * G5_TR + 16 * wr + lh + 4 * i, "
                  "16 * (NCT * wc + c2) + lr)) = rdv[c2][i];\n  };\n" + old_loop)
    old_issue = "    if (st + NS - 1 < nst) issue(st + NS - 1);\n"
    assert k.count(old_issue) == 1
    k = k.replace(old_issue, old_issue + "    if (kc == 0 && st > 0) flush_r();               // the previous tile's R rows\n")
    old_store = "          *reinterpret_cast<double*>(Rimg + g5_chain_off((int)grow, 16 * ct + lr)) = dv;\n"
    assert k.count(old_store) == 1
    k = k.replace(old_store, "          rdv[c2][i] = dv;\n")
    old_wait = "      __builtin_amdgcn_s_waitcnt(0xF70);                  // vmcnt(0): R stores retired before the next counted DMA wait\n"
    assert k.count(old_wait) == 1
    k = k.replace(old_wait, "      rtile = tile;\n")
    old_end = "  double lpa[NCT];\n"
    assert k.count(old_end) == 1
    k = k.replace(old_end, "  if (rtile >= 0) flush_r();\n" + old_end, 1)
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


HARNESS = r'''
#include <stdarg.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
void stk_set_error(const char* fmt, ...) { va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap); fputc('\n', stderr); }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)
using namespace stk;
int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 2000000;
  const int nsh = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  const int d = 1000, C = 64, Dp = (d + 2 + 7) / 8 * 8;
  hipStream_t st; CK(hipStreamCreate(&st));
  std::vector<double> beta(d);
  for (int j = 0; j < d; ++j) beta[j] = ((j * 37) % 19 - 9) / (9.0 * sqrt((double)d));
  double* beta_d; CK(hipMalloc(&beta_d, sizeof(double) * d));
  CK(hipMemcpy(beta_d, beta.data(), sizeof(double) * d, hipMemcpyHostToDevice));
  std::vector<ShardDev> sh(nsh);
  for (int s = 0; s < nsh; ++s) {
    double* X; int32_t* y;
    CK(hipMalloc(&X, sizeof(double) * rows * d)); CK(hipMalloc(&y, sizeof(int32_t) * rows));
    CK(stk_launch_gen_shard(X, nullptr, y, rows, d, s * rows, 20240, 0.0, beta_d, 1.0, STK_LOGREG, st));
    sh[s] = ShardDev{X, nullptr, y, nullptr, rows, d, d + 1, d + 2};
  }
  ShardDev* sh_d; CK(hipMalloc(&sh_d, sizeof(ShardDev) * nsh));
  CK(hipMemcpy(sh_d, sh.data(), sizeof(ShardDev) * nsh, hipMemcpyHostToDevice));
  std::vector<double> qh((size_t)nsh * C * Dp, 0.0);
  for (int g = 0; g < nsh * C; ++g) { qh[(size_t)g * Dp] = 0.01 * ((g % 5) - 2); for (int j = 0; j < d; ++j) qh[(size_t)g * Dp + 1 + j] = beta[j] * (0.9 + 0.002 * g); }
  double *q, *partial; CK(hipMalloc(&q, sizeof(double) * qh.size()));
  CK(hipMemcpy(q, qh.data(), sizeof(double) * qh.size(), hipMemcpyHostToDevice));
  int T, LD, G; size_t lds; stk_sweep_geometry(rows, d, &T, &LD, &G, &lds, C);
  CK(hipMalloc(&partial, sizeof(double) * (size_t)nsh * G * C * (d + 2)));
  void* wsb; CK(hipMalloc(&wsb, stk_sweep_ws_bytes(rows, d, C, nsh)));
  SweepWs ws = stk_sweep_ws(wsb, rows, d, nsh);
  SweepArgs A{sh_d, q, partial, nullptr, 0, C, Dp, G, LD, d + 2, 0, G, nullptr};
  A.qT = ws.qT; A.R = ws.R; A.Rrows = ws.Rrows;
  hipLaunchKernelGGL(k_qt_swizzle, dim3((g5_kp(d) * G5_C + 255) / 256, nsh), dim3(256), 0, st, A, d);
  CK(hipStreamSynchronize(st));
  const double flops = 2.0 * rows * nsh * (double)g5_kp(d) * C;
  // kind 0: pass F (par: computes, so checked against F), 1: pass B
  struct Arm { const char* name; const void* k; int kind; size_t lds; bool par; std::vector<float> ms; };
#define HAVE_OLD @OLD@
  // the committed pass F's LDS: its stages + its own table (round 3's residual v3 tables are
  // 1284 doubles, v4's 1024: launched with v4's size, v3's log entries fell outside the block)
  const size_t lds_old = std::max(lds, (size_t)G5_FS * g5_fstage_bytes() + @OLDTAB@ * sizeof(double));
  std::vector<Arm> arms = {{"F", (const void*)k_gemm_fwd<STK_LOGREG>, 0, lds, true, {}}};
#if HAVE_OLD
  arms.push_back(Arm{"F-old", (const void*)k_gemm_fwd_old<STK_LOGREG>, 0, lds_old, true, {}});
#endif
  if (getenv("GEMM_AB_DEFER")) arms.push_back(Arm{"F-defer", (const void*)k_gemm_fwd_d<STK_LOGREG>, 0, lds, true, {}});
  if (getenv("GEMM_AB_F8")) {
    arms.push_back(Arm{"F8-s2", (const void*)k_gemm_fwd8<STK_LOGREG, 2>, 2, gemm_fwd8_lds<STK_LOGREG, 2>(), true, {}});
    arms.push_back(Arm{"F8-s3", (const void*)k_gemm_fwd8<STK_LOGREG, 3>, 2, gemm_fwd8_lds<STK_LOGREG, 3>(), true, {}});
  }
  if (getenv("GEMM_AB_PIPE")) {
    arms.push_back(Arm{"F-pipe-pre", (const void*)k_gemm_fwd_p<STK_LOGREG, true>, 0, lds, true, {}});
    arms.push_back(Arm{"F-pipe-post", (const void*)k_gemm_fwd_p<STK_LOGREG, false>, 0, lds, true, {}});
  }
  arms.push_back(Arm{"F-w128", (const void*)k_gemm_fwd_w<STK_LOGREG, 4>, 0, gemm_fwd_w_lds<STK_LOGREG, 4>(), true, {}});
  arms.push_back(Arm{"F-w256", (const void*)k_gemm_fwd_w<STK_LOGREG, 8>, 2, gemm_fwd_w_lds<STK_LOGREG, 8>(), true, {}});
  if (getenv("GEMM_AB_TILES")) {
    arms.push_back(Arm{"F-r1k32s2", gemm_fwd_t_ptr<2, 32, 1>(), 0, gemm_fwd_t_lds<2, 32, 1>(), true, {}});
    arms.push_back(Arm{"F-r2k16s2", gemm_fwd_t_ptr<2, 16, 2>(), 0, gemm_fwd_t_lds<2, 16, 2>(), true, {}});
    arms.push_back(Arm{"F-r2k16s3", gemm_fwd_t_ptr<3, 16, 2>(), 0, gemm_fwd_t_lds<3, 16, 2>(), true, {}});
  }
  if (getenv("GEMM_AB_ABL")) {
    arms.push_back(Arm{"F-noB", (const void*)k_gemm_fwd_x<STK_LOGREG, 1>, 0, lds, false, {}});
    arms.push_back(Arm{"F-noEpi", (const void*)k_gemm_fwd_x<STK_LOGREG, 4>, 0, lds, false, {}});
    arms.push_back(Arm{"F-onlyMFMA", (const void*)k_gemm_fwd_x<STK_LOGREG, 7>, 0, lds, false, {}});
  }
  arms.push_back(Arm{"B", (const void*)k_gemm_bwd, 1, 0, false, {}});
  for (auto& a : arms) CK(hipFuncSetAttribute(a.k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int njb = (d + G5_BJB - 1) / G5_BJB;
  auto launch = [&](const Arm& a) {
    if (a.kind == 0) hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs)>(const_cast<void*>(a.k)), dim3(nsh * G), dim3(64 * G5_FW), a.lds, st, A);
    else if (a.kind == 2) hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs)>(const_cast<void*>(a.k)), dim3(nsh * G), dim3(512), a.lds, st, A);
    else hipLaunchKernelGGL(k_gemm_bwd, dim3(nsh * G * njb), dim3(64 * G5_NW), G5_BNS * g5_bstage_bytes(), st, A, njb);
  };
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  {   // parity of the arms that compute: F (and F-old) + pass B + the chunk reduction
    double *lp, *grad; CK(hipMalloc(&lp, sizeof(double) * nsh * C)); CK(hipMalloc(&grad, sizeof(double) * nsh * C * Dp));
    std::vector<std::vector<double>> res;
    std::vector<const char*> names;
    for (const Arm& a : arms) {
      if (!a.par) continue;
      names.push_back(a.name);
      CK(hipMemset(ws.R, 0xFF, sizeof(double) * (size_t)nsh * ws.Rrows * C));   // NaN: an unwritten R row shows
      launch(a);
      CK(hipGetLastError());
      hipLaunchKernelGGL(k_gemm_bwd, dim3(nsh * G * njb), dim3(64 * G5_NW), G5_BNS * g5_bstage_bytes(), st, A, njb);
      CK(stk_launch_sweep_reduce(STK_LOGREG, sh_d, 0, nsh, d, G, G, q, C, Dp, partial, nullptr, 0, lp, grad, st));
      std::vector<double> h((size_t)nsh * C * (Dp + 1));
      CK(hipMemcpy(h.data(), lp, sizeof(double) * nsh * C, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h.data() + nsh * C, grad, sizeof(double) * nsh * C * Dp, hipMemcpyDeviceToHost));
      res.push_back(h);
    }
    for (size_t k = 1; k < res.size(); ++k) {
      double lpr = 0, gr = 0, gmax = 0;
      for (int i = 0; i < nsh * C; ++i) lpr = std::max(lpr, fabs(res[k][i] - res[0][i]) / fabs(res[0][i]));
      for (size_t i = nsh * C; i < res[0].size(); ++i) gmax = std::max(gmax, fabs(res[0][i]));
      for (size_t i = nsh * C; i < res[0].size(); ++i) gr = std::max(gr, fabs(res[k][i] - res[0][i]) / gmax);
      printf("parity %s vs F: lp max rel %.3g, grad max |diff| / max|grad| %.3g (lp[0] %.6f)\n", names[k], lpr, gr, res[0][0]);
    }
  }
  printf("rows/shard %lld shards %d d %d C %d: G %d, %.1f GFLOP per pass\n", (long long)rows, nsh, d, C, G, flops / 1e9);
  for (int r = 0; r < rounds; ++r)
    for (auto& a : arms) {
      launch(a); CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st)); for (int i = 0; i < 3; ++i) launch(a); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); a.ms.push_back(ms / 3);
      printf("round %d %-10s %8.3f ms %6.1f TF\n", r, a.name, ms / 3, flops / (ms / 3) / 1e9); fflush(stdout);
    }
  for (auto& a : arms) { auto v = a.ms; std::sort(v.begin(), v.end()); printf("median %-10s %8.3f ms %6.1f TF\n", a.name, v[v.size() / 2], flops / v[v.size() / 2] / 1e9); }
  return 0;
}
'''


def old_copy(ref="HEAD"):
    """The committed (git `ref`) pass F as k_gemm_fwd_old<FAM>, for a before/after arm."""
    src = subprocess.run(["git", "-C", ROOT, "show", ref + ":stark_amd/csrc/sweep.hip"], check=True,
                         capture_output=True, text=True).stdout
    i = src.index("template <int FAM>\n__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd(SweepArgs A) {")
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_old(SweepArgs A) {")
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def old_table():
    """Doubles of the committed pass F's LDS table (the lds_bytes line of stk_sweep_geometry's C = 64 branch)."""
    ref = os.environ.get("GEMM_AB_OLD")
    if not ref:
        return "0"
    src = subprocess.run(["git", "-C", ROOT, "show", ref + ":stark_amd/csrc/sweep.hip"], check=True,
                         capture_output=True, text=True).stdout
    line = [l for l in src.splitlines() if "*lds_bytes = G5_FS * g5_fstage_bytes() +" in l][0]
    return "(" + line.split("+", 1)[1].split("*")[0].strip() + ")"


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(os.path.join(ROOT, "stark_amd", "csrc", "sweep.hip")).read()
    c = os.path.join(ROOT, "stark_amd", "csrc")
    body = ('#include "%s"\n#include "%s"\n#include "%s"\n' % (os.path.join(c, "sweep.hip"), os.path.join(c, "sweep16.hip"),
                                                          os.path.join(c, "datagen.hip"))
            + '#include "%s"\n#include "%s"\n#include "%s"\n' % (os.path.join(ROOT, "tools", "sweep_legacy.hip"), os.path.join(ROOT, "tools", "gemm_fwd_variants.hip"),
                                                  os.path.join(ROOT, "tools", "gemm_fwd_r5.hip"))
            + ablation_copy(src) + deferred_copy(src) + (old_copy(os.environ.get("GEMM_AB_OLD", "HEAD")) if os.environ.get("GEMM_AB_OLD") else "")
            + HARNESS.replace("@OLD@", "1" if os.environ.get("GEMM_AB_OLD") else "0").replace("@OLDTAB@", old_table()))
    f = os.path.join(OUT, "gemm_ab.hip")
    open(f, "w").write(body)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", f, "-o",
                    os.path.join(ROOT, "tools", "_bin", "gemm_ab")], check=True)
    print("built tools/_bin/gemm_ab")


if __name__ == "__main__":
    main()
