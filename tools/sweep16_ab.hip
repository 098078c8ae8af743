// A/B timing of the 16-chain sweep at the bench geometry (BASELINE configs[3]: 8 shards x 1.25e7
// rows, d = 100, 16 chains; 80.4 GB per sweep; or configs[2]'s d = 50), interleaved rounds so box
// drift hits every arm, plus parity of every arm against round 3's product kernel (k_sweepe,
// residual v3) after the chunk reduction.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep16_ab.hip -o tools/_bin/sweep16_ab
// Run:   tools/_bin/sweep16_ab [rows_per_shard] [shards] [rounds] [reps] [d] [family 3=logistic 2=linear]
#include "../stark_amd/csrc/sweep.hip"
#include "sweep_variants.hip"
#include "../stark_amd/csrc/sweep16.hip"
#include "sweep16_variants.hip"
#include "sweep16_r5.hip"
#if __has_include("_bin/s16_old.hip")
#include "_bin/s16_old.hip"   // a committed k_sweep16 renamed k_sweep16_old (see the arms)
#define HAVE_S16_OLD 1
#endif
#include "../stark_amd/csrc/datagen.hip"
#include <stdarg.h>
#include <stdio.h>
#include <vector>

void stk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

using namespace stk;

struct Arm {
  const char* name;
  const void* kern;
  size_t lds;
  std::vector<float> ms;
  int G = 0;                // chunks per shard (0: the library's geometry)
};

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 12500000;
  const int nsh = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  const int reps = argc > 4 ? atoi(argv[4]) : 10;
  const int d = argc > 5 ? atoi(argv[5]) : 100;
  const int fam = argc > 6 ? atoi(argv[6]) : STK_LOGREG;
  const int C = 16, Dp = (d + 2 + 7) / 8 * 8;
  if (!(d == 100 || d == 50)) {
    fprintf(stderr, "d must be 100 or 50\n");
    return 2;
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<ShardDev> sh(nsh);
  std::vector<double> beta(d);
  for (int j = 0; j < d; ++j) beta[j] = ((j * 37) % 19 - 9) / (9.0 * sqrt((double)d));
  double* beta_d;
  CK(hipMalloc(&beta_d, sizeof(double) * d));
  CK(hipMemcpy(beta_d, beta.data(), sizeof(double) * d, hipMemcpyHostToDevice));
  for (int s = 0; s < nsh; ++s) {
    double* X;
    int32_t* yi = nullptr;
    double* yd = nullptr;
    CK(hipMalloc(&X, sizeof(double) * rows * d));
    if (fam == STK_LOGREG) CK(hipMalloc(&yi, sizeof(int32_t) * rows));
    else CK(hipMalloc(&yd, sizeof(double) * rows));
    CK(stk_launch_gen_shard(X, yd, yi, rows, d, s * rows, 20240, 0.0, beta_d, 1.0, fam, st));
    sh[s] = ShardDev{X, yd, yi, nullptr, rows, d, fam == STK_LOGREG ? d + 1 : d + 2, d + 2};
  }
  ShardDev* sh_d;
  CK(hipMalloc(&sh_d, sizeof(ShardDev) * nsh));
  CK(hipMemcpy(sh_d, sh.data(), sizeof(ShardDev) * nsh, hipMemcpyHostToDevice));
  std::vector<double> qh((size_t)nsh * C * Dp, 0.0);
  for (int g = 0; g < nsh * C; ++g) {
    qh[(size_t)g * Dp] = 0.05 * ((g % 5) - 2);                      // alpha
    for (int j = 0; j < d; ++j) qh[(size_t)g * Dp + 1 + j] = beta[j] * (0.9 + 0.01 * g);
    if (fam == STK_LINREG) qh[(size_t)g * Dp + d + 1] = 0.1 * (g % 3);   // log sigma
  }
  double *q, *partial, *lp, *grad;
  CK(hipMalloc(&q, sizeof(double) * qh.size()));
  CK(hipMemcpy(q, qh.data(), sizeof(double) * qh.size(), hipMemcpyHostToDevice));
  int T, LD, G;
  size_t lds;
  stk_sweep_geometry(rows, d, &T, &LD, &G, &lds, C);
  CK(hipMalloc(&partial, sizeof(double) * (size_t)nsh * 2048 * C * (d + 2)));   // room for G <= 2048
  CK(hipMalloc(&lp, sizeof(double) * nsh * C));
  CK(hipMalloc(&grad, sizeof(double) * nsh * C * Dp));
  CK(hipStreamSynchronize(st));
  const double bytes = (double)nsh * rows * (8.0 * d + (fam == STK_LOGREG ? 4.0 : 8.0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  SweepArgs A{sh_d, q, partial, nullptr, 0, C, Dp, G, LD, d + 2, 0, G, nullptr};
  const size_t l16 = stk_sweep16_lds_bytes(fam, d);
  // LDS of the committed kernel before beta moved to registers (its block image of beta for
  // KF < 28 beside the slots), which the legacy k_sweepe arm also fits in
  const size_t l16_old = std::max((size_t)SM_W * sweepm_slot_bytes(d) + (size_t)16 * (4 * ((d + 3) / 4) + 2) * 8 +
                                      (fam == STK_LOGREG ? EX_TAB * 8 : 0) + (size_t)SM_W * 64 * 8, l16);
  printf("rows/shard %lld shards %d d %d C %d family %d: G %d lds %zu / %zu, %.1f GB per sweep\n", (long long)rows, nsh,
         d, C, fam, G, lds, l16, bytes / 1e9);
  std::vector<Arm> arms;
#ifdef HAVE_S16_OLD
#define S16_OLD_ARM(F, KF) arms.push_back(Arm{"s16-old", (const void*)k_sweep16_old<F, KF>, l16, {}});
#else
#define S16_OLD_ARM(F, KF)
#endif
#define ARMS(F, KF, JT)                                                                        \
  arms = {{"s16", (const void*)k_sweep16<F, KF>, l16, {}},                                     \
          {"v0", (const void*)k_sweep16v<F, KF, 0>, l16, {}},                                  \
          {"dppv2", (const void*)k_sweep16v<F, KF, 128>, l16, {}},                             \
          {"dppv2-peel", (const void*)k_sweep16v<F, KF, 160>, l16, {}},                        \
          {"dppv", (const void*)k_sweep16v<F, KF, 64>, l16, {}}};                              \
  S16_OLD_ARM(F, KF)
  if (fam == STK_LOGREG) {
    if (d == 100) { ARMS(STK_LOGREG, 25, 7) } else { ARMS(STK_LOGREG, 13, 4) }
  } else {
    if (d == 100) { ARMS(STK_LINREG, 25, 7) } else { ARMS(STK_LINREG, 13, 4) }
  }
  for (auto& a : arms) CK(hipFuncSetAttribute(a.kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto launch = [&](const Arm& a) {
    SweepArgs B = A;
    B.G = B.Gs = a.G ? a.G : G;
    hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs)>(const_cast<void*>(a.kern)), dim3(nsh * B.G), dim3(256),
                       a.lds, st, B);
  };
  std::vector<std::vector<double>> res;
  for (size_t k = 0; k < arms.size(); ++k) {
    launch(arms[k]);
    CK(hipGetLastError());
    const int Gk = arms[k].G ? arms[k].G : G;
    CK(stk_launch_sweep_reduce(fam, sh_d, 0, nsh, d, Gk, Gk, q, C, Dp, partial, nullptr, 0, lp, grad, st));
    std::vector<double> h((size_t)nsh * C * (Dp + 1));
    CK(hipMemcpyAsync(h.data(), lp, sizeof(double) * nsh * C, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(h.data() + nsh * C, grad, sizeof(double) * nsh * C * Dp, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    res.push_back(h);
  }
  for (size_t k = 1; k < arms.size(); ++k) {
    double lpr = 0, gr = 0, gmax = 0;
    for (int i = 0; i < nsh * C; ++i) lpr = std::max(lpr, fabs(res[k][i] - res[0][i]) / fabs(res[0][i]));
    for (size_t i = nsh * C; i < res[0].size(); ++i) gmax = std::max(gmax, fabs(res[0][i]));
    for (size_t i = nsh * C; i < res[0].size(); ++i) gr = std::max(gr, fabs(res[k][i] - res[0][i]) / gmax);
    printf("parity %s vs %s: lp max rel %.3g, grad max |diff| / max|grad| %.3g (lp[0] %.6f)\n", arms[k].name,
           arms[0].name, lpr, gr, res[0][0]);
  }
  for (int r = 0; r < rounds; ++r) {
    for (auto& a : arms) {
      launch(a);
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) launch(a);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      a.ms.push_back(ms / reps);
      printf("round %d %-8s %8.3f ms  %7.1f GB/s  %.3f of 8 TB/s\n", r, a.name, ms / reps, bytes / (ms / reps) / 1e6,
             bytes / (ms / reps) / 1e6 / 8000.0);
      fflush(stdout);
    }
  }
  for (auto& a : arms) {
    std::vector<float> v = a.ms;
    std::sort(v.begin(), v.end());
    printf("median %-8s %8.3f ms  %.3f of 8 TB/s\n", a.name, v[v.size() / 2], bytes / v[v.size() / 2] / 1e6 / 8000.0);
  }
  return 0;
}
