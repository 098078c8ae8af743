#!/usr/bin/env python3
"""Pass F of the 64-chain full-data sweep (sweep.hip: k_gemm_fwd) against its alternatives:
writes tools/_bin/gemm_ab_src/gemm_ab.hip -- the product sweep.hip included as is, round 4's
pass F frozen in tools/gemm_fwd_r4.hip -- and a harness that checks every pass F arm against
the product's (lp and gradient after pass B and the chunk reduction) and times them and pass B
at configs[4]'s shape (d = 1000, 64 chains) on synthetic rows; builds it with hipcc.
Pass B arms: tools/gemm_bwd_r5.hip (wider column blocks, fewer R re-reads).
Pass F arms: F (the product at d = 1000: 128-row tiles of 4 waves, two blocks per CU, the split
stage schedule), F-loop (the same kernel with one epilogue-part dispatch per stage, as used for
d <= 112), F-r4 (round 4: 64-row tiles, 32-column stages), geometry arms (FARM) and ablations.
Round 5's exploratory variants (8-wave 128-row tiles, pipelined epilogues on 64-row tiles,
tools/gemm_fwd_r5.hip / gemm_fwd_variants.hip) were built against round 4's sweep.hip.
The product source is not changed.

usage: tools/gemm_fwd_ab.py   (then on the GPU: tools/_bin/gemm_ab [rows_per_shard] [shards] [rounds])"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_bin", "gemm_ab_src")


def ablation_copy(src):
    """k_gemm_fwd_x<FAM, ABL>: the product pass F with parts removed by text substitution (bit 0:
    no beta^T LDS-DMA, 1: no X LDS-DMA, 2: the epilogue reduced to folding eta into the lp sum,
    3: no R stores, 4: every tile's X stages read from the chunk's first tile (L2-resident),
    5: the X stages read as one sequential stream of the same bytes, 6: no parked eta at all,
    the accumulators folded into the gradient sum at the tile's end: 64 VGPRs fewer); ablated
    arms compute garbage and are timed only."""
    head = ("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
            "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {")
    i = src.index(head)
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace(head, "template <int FAM, int ABL, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
                                "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd_x(SweepArgs A) {")
    subs = [("    xvo[i] = row * d * 8 + pc * 16;", "    xvo[i] = (ABL & 32) ? row * KCF * 8 + pc * 16 : row * d * 8 + pc * 16;"),
            ("    const int xso = tile * TR * d * 8 + kc * KCF * 8;",
             "    const int xso = (ABL & 16) ? kc * KCF * 8 : (ABL & 32) ? st * TR * KCF * 8 : tile * TR * d * 8 + kc * KCF * 8;"),
            ("for (int i = 0; i < NDB; ++i) dma16_lds(br,", "for (int i = 0; i < NDB; ++i) if constexpr (!(ABL & 1)) dma16_lds(br,"),
            ("for (int i = 0; i < NDX; ++i) dma16_lds(xr,", "for (int i = 0; i < NDX; ++i) if constexpr (!(ABL & 2)) dma16_lds(xr,"),
            ("      if (grow < rcap) *reinterpret_cast<double*>(Rimg", "      if (!(ABL & 8) && grow < rcap) *reinterpret_cast<double*>(Rimg"),
            ("        for (int i = 0; i < 4; ++i) pend[rt][c2][i] = acc[rt][c2][i] + alpha[c2];",
             "        for (int i = 0; i < 4; ++i) { if constexpr ((ABL & 64) != 0) gaa[c2] += acc[rt][c2][i]; else pend[rt][c2][i] = acc[rt][c2][i] + alpha[c2]; }"),
            ("    ptile = tile;", "    if constexpr (!(ABL & 64)) ptile = tile;"),
            ("  auto epi = [&](const int p) {", "  auto epi = [&](const int p) {\n    if constexpr ((ABL & 4) != 0) {\n      const int rt = p / NCT, c2 = p % NCT;\n"
             "      gaa[c2] += pend[rt][c2][0] + pend[rt][c2][1] + pend[rt][c2][2] + pend[rt][c2][3];\n      return;\n    }")]
    for a, b in subs:
        assert k.count(a) == 1, a
        k = k.replace(a, b)
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def early_copy(src):
    """k_gemm_fwd_e<FAM>: the product pass F with the next stage's DMA issued right after the
    barrier, before the parked tile's epilogue part and the tile's y loads (the compiler waits
    for the y loads where it uses them; the DMA'd stages keep their counted waits)."""
    head = ("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
            "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {")
    i = src.index(head)
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_e(SweepArgs A) {")
    iss = "    if (st + NS - 1 < nst) issue(st + NS - 1);\n"
    bar = "    lds_barrier();                                       // stage st landed for every wave; slot of st-1 free\n"
    assert k.count(iss) == 1 and k.count(bar) == 1
    k = k.replace(iss, "").replace(bar, bar + iss)
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def nt_copies(src):
    """k_gemm_fwd_n<FAM> / k_gemm_bwd_n<JB>: the product passes with X's LDS-DMA issued
    non-temporal (aux 2, as k_sweep16's stream: X is read once per pass); beta^T and R keep the
    default policy (re-read from L2)."""
    out = "namespace stk {\n__device__ __forceinline__ void dma16_lds_nt(__amdgpu_buffer_rsrc_t r, char* dst, int voff, int soff) {\n" \
          "  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)dst, 16, voff, soff, 0, 2);\n}\n"
    for head, name in (("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
                        "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {", ("k_gemm_fwd(", "k_gemm_fwd_n(")),
                       ("template <int JB>\n__global__ __launch_bounds__(64 * G5_BW, 2) void k_gemm_bwd(SweepArgs A, int njb) {",
                        ("k_gemm_bwd(", "k_gemm_bwd_n("))):
        i = src.index(head)
        j = src.index("\n}\n", i) + 3
        k = src[i:j].replace(name[0], name[1], 1)
        assert k.count("dma16_lds(xr,") == 1
        out += k.replace("dma16_lds(xr,", "dma16_lds_nt(xr,") + "\n"
    return out + "}  // namespace stk\n"


def spread_copy(src):
    """k_gemm_fwd_s<FAM>: the product pass F with the next stage's DMA spread over the stage's
    k-steps (the beta^T pieces and X piece 0 before k-step 0, X piece i before k-step i) instead
    of all six instructions at once before the MFMAs."""
    head = ("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
            "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {")
    i = src.index(head)
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_s(SweepArgs A) {")
    subs = [("  auto issue = [&](int st) {                            // global stage index st = tile * NKC + kc\n",
             "  auto issue_part = [&](int st, int part) {\n"
             "    const int tile = st / NKC, kc = st % NKC;\n    char* b = stg + (st % NS) * STG;\n"
             "    const int xso = tile * TR * d * 8 + kc * KCF * 8;\n"
             "    if (part == 0) {\n#pragma unroll\n      for (int i = 0; i < NDB; ++i) dma16_lds(br, b + XB + (w * NDB + i) * 1024, lane * 16, kc * KCF * 512 + (w * NDB + i) * 1024);\n    }\n"
             "    if (part < NDX) dma16_lds(xr, b + (w * NDX + part) * 1024, xvo[part], xso);\n  };\n"
             "  auto issue = [&](int st) {                            // global stage index st = tile * NKC + kc\n"),
            ("    if (st + NS - 1 < nst) issue(st + NS - 1);\n", "    const bool doiss = st + NS - 1 < nst;\n"),
            ("    for (int step = 0; step < KCF / 4; ++step) {\n      const int kk = 4 * step + lh;\n",
             "    for (int step = 0; step < KCF / 4; ++step) {\n      if (doiss) issue_part(st + NS - 1, step);\n      const int kk = 4 * step + lh;\n")]
    for a, b2 in subs:
        assert k.count(a) == 1, a
        k = k.replace(a, b2)
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def volatile_copy(src):
    """k_gemm_fwd_v<FAM>: the product pass F with its A-fragment reads volatile, so the compiler
    cannot pair a lane's two row tiles (2 KB apart) into one ds_read2st64_b64: that form is
    serviced in 16-lane groups over 32 banks, where lanes lr and lr ^ 1 of the 128-B X rows
    share a bank (2-way); as two ds_read_b64 (32-lane groups over 64 banks) they do not."""
    head = ("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
            "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {")
    i = src.index(head)
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_v(SweepArgs A) {")
    a = "        a[rt] = *reinterpret_cast<const double*>(b + r * (16 * PPR)"
    assert k.count(a) == 1
    k = k.replace(a, "        a[rt] = *reinterpret_cast<const volatile double*>(b + r * (16 * PPR)")
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


def swz2_copy(src):
    """k_gemm_fwd_z<FAM>: the product pass F with the X piece swizzle ((row >> 1) & 7) ^ ((row >> 4) & 1):
    a lane's two row tiles (rows r, r + 16) then sit a lane-dependent distance apart, so the
    compiler keeps them as two ds_read_b64 (32-lane groups over 64 banks: conflict free) instead
    of one ds_read2st64_b64 (16-lane groups over 32 banks: lanes lr, lr ^ 1 collide)."""
    head = ("template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>\n"
            "__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {")
    i = src.index(head)
    j = src.index("\n}\n", i) + 3
    k = src[i:j].replace("void k_gemm_fwd(SweepArgs A) {", "void k_gemm_fwd_z(SweepArgs A) {")
    a = "  auto swz = [](int row) { return PPR == 16 ? (row & 15) : ((row >> 1) & 7); };"
    assert k.count(a) == 1
    k = k.replace(a, "  auto swz = [](int row) { return PPR == 16 ? (row & 15) : (((row >> 1) & 7) ^ ((row >> 4) & 1)); };")
    return "namespace stk {\n" + k + "\n}  // namespace stk\n"


HARNESS = r'''
#include <stdarg.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#include <string.h>
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
  struct Arm { const char* name; const void* k; int kind; size_t lds; bool par; std::vector<float> ms; int threads; int jb = 0; };
  // the product's pass F at d = 1000: the split stage schedule (stk_launch_sweep picks it for d > 112)
  std::vector<Arm> arms = {{"F", (const void*)k_gemm_fwd<STK_LOGREG, G5_FW, 2, G5_FKC, G5_FS, 1>, 0, lds, true, {}, 64 * G5_FW}};
  arms.push_back(Arm{"F-loop", (const void*)k_gemm_fwd<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  // (alpha re-read at the park instead of held, 1 VGPR spilled instead of 4: 38.70 / 60.66 ms against
  // 38.44 / 60.39, profiles/r05as_*; its SPLIT = 3 form since removed)
  // (the parts spread over the tile, part p at stage p NKC / 8: 40.05 / 62.86 ms against the split
  // head's 39.75 / 62.15, profiles/r05ap_*; its SPLIT = 2 schedule since removed)
  // pass F geometries: NW waves x RT 16-row tiles per wave, KCF-column stages, NS-deep ring
  // (8-column stages in 4-6 deep rings, 42.7-43.5 ms against 39.5: profiles/r05ae_passF_k8_ab.log,
  // built with a (row >> 2) & 3 swizzle for 64-B rows, since removed)
#define FARM(NW, RT, KCF, NS) arms.push_back(Arm{"F-" #NW "w" #RT "r" #KCF "k" #NS "s", (const void*)k_gemm_fwd<STK_LOGREG, NW, RT, KCF, NS>, 0, \
    (size_t)NS * (16 * RT * NW * KCF * 8 + KCF * 512) + EX_TAB * 8, true, {}, 64 * NW})
  if (getenv("GEMM_AB_NT")) arms.push_back(Arm{"F-ntX", (const void*)k_gemm_fwd_n<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_VOLA")) arms.push_back(Arm{"F-volA", (const void*)k_gemm_fwd_v<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_SWZ2")) arms.push_back(Arm{"F-swz2", (const void*)k_gemm_fwd_z<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_SPREAD")) arms.push_back(Arm{"F-spread", (const void*)k_gemm_fwd_s<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_EARLY")) arms.push_back(Arm{"F-early", (const void*)k_gemm_fwd_e<STK_LOGREG>, 0, lds, true, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_ABL")) arms.push_back(Arm{"F-split-noPark", (const void*)k_gemm_fwd_x<STK_LOGREG, 64, 4, 2, 16, 3, 1>, 0, lds, false, {}, 64 * G5_FW});
  if (getenv("GEMM_AB_R5Y")) {   // round 5, call y's arms (profiles/r05y_passF_geom_*.log)
    FARM(8, 1, 32, 3);
    FARM(8, 1, 16, 4);
    FARM(8, 1, 32, 2);
    FARM(4, 2, 32, 2);
    FARM(8, 2, 16, 3);
  }
  arms.push_back(Arm{"F-r4", (const void*)k_gemm_fwd_r4<STK_LOGREG>, 0, (size_t)G4_FS * g4_fstage_bytes() + EX_TAB * 8, true, {}, 64 * G4_FW});
  if (getenv("GEMM_AB_ABL")) {
    arms.push_back(Arm{"F-noB", (const void*)k_gemm_fwd_x<STK_LOGREG, 1>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-noR", (const void*)k_gemm_fwd_x<STK_LOGREG, 8>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-noEpi", (const void*)k_gemm_fwd_x<STK_LOGREG, 12>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-noEpiB", (const void*)k_gemm_fwd_x<STK_LOGREG, 13>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-onlyMFMA", (const void*)k_gemm_fwd_x<STK_LOGREG, 15>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-noPark", (const void*)k_gemm_fwd_x<STK_LOGREG, 64>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-noPark-onlyMFMA", (const void*)k_gemm_fwd_x<STK_LOGREG, 64 + 15>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-Xtile0", (const void*)k_gemm_fwd_x<STK_LOGREG, 16>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-Xseq", (const void*)k_gemm_fwd_x<STK_LOGREG, 32>, 0, lds, false, {}, 64 * G5_FW});
    arms.push_back(Arm{"F-Xseq-noB", (const void*)k_gemm_fwd_x<STK_LOGREG, 33>, 0, lds, false, {}, 64 * G5_FW});
  }
  arms.push_back(Arm{"B", (const void*)k_gemm_bwd<256>, 3, (size_t)G5_BNS * g5_bstage_bytes(256), true, {}, 64 * G5_BW, 256});
  if (getenv("GEMM_AB_NT")) arms.push_back(Arm{"B-ntX", (const void*)k_gemm_bwd_n<256>, 3, (size_t)G5_BNS * g5_bstage_bytes(256), true, {}, 64 * G5_BW, 256});
  // round 4's pass B geometry (128-column blocks of 8 waves, 32-row stages; tools/gemm_bwd_r5.hip)
  arms.push_back(Arm{"B-r4", (const void*)k_gemm_bwd_w<128, 32, 8, 3>, 3, gemm_bwd_w_lds<128, 32, 8, 3>(), true, {}, 512, 128});
  // pass B variants (kind 3, tools/gemm_bwd_r5.hip): JB columns x RB rows per stage, NW waves, NS stages
  if (getenv("GEMM_AB_R5U")) {   // round 5, call u's arms (profiles/r05u_passB_ab_*.log)
    arms.push_back(Arm{"B-256r16w8s3", (const void*)k_gemm_bwd_w<256, 16, 8, 3>, 3, gemm_bwd_w_lds<256, 16, 8, 3>(), true, {}, 512, 256});
    arms.push_back(Arm{"B-256r16w8s2", (const void*)k_gemm_bwd_w<256, 16, 8, 2>, 3, gemm_bwd_w_lds<256, 16, 8, 2>(), true, {}, 512, 256});
    arms.push_back(Arm{"B-256r32w8s2", (const void*)k_gemm_bwd_w<256, 32, 8, 2>, 3, gemm_bwd_w_lds<256, 32, 8, 2>(), true, {}, 512, 256});
  }
  arms.push_back(Arm{"B-128r16w4s3", (const void*)k_gemm_bwd_w<128, 16, 4, 3>, 3, gemm_bwd_w_lds<128, 16, 4, 3>(), true, {}, 256, 128});
  if (getenv("GEMM_AB_R5V")) {   // round 5, call v's arms (profiles/r05v_passB_ab_*.log)
    arms.push_back(Arm{"B-128r16w4s2", (const void*)k_gemm_bwd_w<128, 16, 4, 2>, 3, gemm_bwd_w_lds<128, 16, 4, 2>(), true, {}, 256, 128});
    arms.push_back(Arm{"B-128r8w4s4", (const void*)k_gemm_bwd_w<128, 8, 4, 4>, 3, gemm_bwd_w_lds<128, 8, 4, 4>(), true, {}, 256, 128});
    arms.push_back(Arm{"B-64r16w4s3", (const void*)k_gemm_bwd_w<64, 16, 4, 3>, 3, gemm_bwd_w_lds<64, 16, 4, 3>(), true, {}, 256, 64});
  }
  if (getenv("GEMM_AB_R5W")) {   // round 5, call w's arms (profiles/r05w_passB_ab_*.log; 256r8w4s3 is now the product)
    arms.push_back(Arm{"B-256r16w4s2", (const void*)k_gemm_bwd_w<256, 16, 4, 2>, 3, gemm_bwd_w_lds<256, 16, 4, 2>(), true, {}, 256, 256});
    arms.push_back(Arm{"B-256r8w4s4", (const void*)k_gemm_bwd_w<256, 8, 4, 4>, 3, gemm_bwd_w_lds<256, 8, 4, 4>(), true, {}, 256, 256});
  }
  arms.push_back(Arm{"B-256r8w4s2", (const void*)k_gemm_bwd_w<256, 8, 4, 2>, 3, gemm_bwd_w_lds<256, 8, 4, 2>(), true, {}, 256, 256});
  for (auto& a : arms) CK(hipFuncSetAttribute(a.k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto launch = [&](const Arm& a) {
    if (a.kind == 0) hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs)>(const_cast<void*>(a.k)), dim3(nsh * G), dim3(a.threads), a.lds, st, A);
    else if (a.kind == 3) {
      const int nj = (d + a.jb - 1) / a.jb;
      hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs, int)>(const_cast<void*>(a.k)), dim3(nsh * G * nj), dim3(a.threads), a.lds, st, A, nj);
    }
  };
  const Arm* prodB = nullptr;
  for (const Arm& a : arms) if (!strcmp(a.name, "B")) prodB = &a;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  {   // parity of the arms that compute: pass F + pass B + the chunk reduction
    double *lp, *grad; CK(hipMalloc(&lp, sizeof(double) * nsh * C)); CK(hipMalloc(&grad, sizeof(double) * nsh * C * Dp));
    std::vector<std::vector<double>> res;
    std::vector<const char*> names;
    for (const Arm& a : arms) {
      if (!a.par) continue;
      names.push_back(a.name);
      CK(hipMemset(ws.R, 0xFF, sizeof(double) * (size_t)nsh * ws.Rrows * C));   // NaN: an unwritten R row shows
      if (a.kind == 3) {            // a pass B arm: after the product's pass F
        launch(arms[0]);
        launch(a);
      } else {
        launch(a);
        launch(*prodB);
      }
      CK(hipGetLastError());
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
      printf("parity %s vs F+B: lp max rel %.3g, grad max |diff| / max|grad| %.3g (lp[0] %.6f)\n", names[k], lpr, gr, res[0][0]);
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


def main():
    os.makedirs(OUT, exist_ok=True)
    c = os.path.join(ROOT, "stark_amd", "csrc")
    src = open(os.path.join(c, "sweep.hip")).read()
    body = ('#include "%s"\n#include "%s"\n#include "%s"\n#include "%s"\n'
            % (os.path.join(c, "sweep.hip"), os.path.join(c, "sweep16.hip"), os.path.join(c, "datagen.hip"),
               os.path.join(ROOT, "tools", "gemm_fwd_r4.hip"))
            + '#include "%s"\n' % os.path.join(ROOT, "tools", "gemm_bwd_r5.hip") + ablation_copy(src) + early_copy(src) + nt_copies(src) + spread_copy(src) + volatile_copy(src) + swz2_copy(src) + HARNESS)
    f = os.path.join(OUT, "gemm_ab.hip")
    open(f, "w").write(body)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", f, "-o",
                    os.path.join(ROOT, "tools", "_bin", "gemm_ab")], check=True)
    print("built tools/_bin/gemm_ab")


if __name__ == "__main__":
    main()
