// A/B of the C = 16 sweep at BASELINE configs[2]'s shape (linear regression, 8 shards x 1.25e6
// rows, d = 50, 16 chains; 4.0 GB per sweep): the product kernel for d = 50 (k_sweepm with
// compile-time KF / JT and the VALU remainder columns) against k_sweepe instantiated for d = 50
// (one 16-row slot per wave, nt DMA, raised priority around the residual), interleaved rounds,
// plus a parity check of lp / gradient after the chunk reduction.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweepe_d50.hip -o tools/_bin/sweepe_d50
// Run:   tools/_bin/sweepe_d50 [rows_per_shard] [shards] [rounds] [reps]
#include "../stark_amd/csrc/sweep.hip"
#include "../stark_amd/csrc/datagen.hip"
#include <stdarg.h>
#include <stdio.h>
#include <algorithm>
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

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 1250000;
  const int nsh = argc > 2 ? atoi(argv[2]) : 8;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  const int reps = argc > 4 ? atoi(argv[4]) : 50;
  constexpr int d = 50, C = 16, KF = 13, JT = 4;
  const int Dp = (d + 2 + 7) / 8 * 8;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<ShardDev> sh(nsh);
  std::vector<double> beta(d);
  for (int j = 0; j < d; ++j) beta[j] = ((j * 37) % 19 - 9) / (9.0 * sqrt((double)d));
  double* beta_d;
  CK(hipMalloc(&beta_d, sizeof(double) * d));
  CK(hipMemcpy(beta_d, beta.data(), sizeof(double) * d, hipMemcpyHostToDevice));
  for (int s = 0; s < nsh; ++s) {
    double *X, *y;
    CK(hipMalloc(&X, sizeof(double) * rows * d));
    CK(hipMalloc(&y, sizeof(double) * rows));
    CK(stk_launch_gen_shard(X, y, nullptr, rows, d, s * rows, 20240, 0.3, beta_d, 1.0, STK_LINREG, st));
    sh[s] = ShardDev{X, y, nullptr, nullptr, rows, d, d + 2, d + 3, 0.0, 0.0};
  }
  ShardDev* sh_d;
  CK(hipMalloc(&sh_d, sizeof(ShardDev) * nsh));
  CK(hipMemcpy(sh_d, sh.data(), sizeof(ShardDev) * nsh, hipMemcpyHostToDevice));
  std::vector<double> qh((size_t)nsh * C * Dp, 0.0);
  for (int g = 0; g < nsh * C; ++g) {
    qh[(size_t)g * Dp] = 0.3 + 0.01 * ((g % 5) - 2);                 // alpha
    for (int j = 0; j < d; ++j) qh[(size_t)g * Dp + 1 + j] = beta[j] * (0.9 + 0.01 * g);
    qh[(size_t)g * Dp + d + 1] = 0.02 * (g % 7);                       // log sigma
  }
  double *q, *partial, *lp, *grad;
  CK(hipMalloc(&q, sizeof(double) * qh.size()));
  CK(hipMemcpy(q, qh.data(), sizeof(double) * qh.size(), hipMemcpyHostToDevice));
  int T, LD, G;
  size_t lds;
  stk_sweep_geometry(rows, d, &T, &LD, &G, &lds, C);
  CK(hipMalloc(&partial, sizeof(double) * (size_t)nsh * G * C * (d + 2)));
  CK(hipMalloc(&lp, sizeof(double) * nsh * C));
  CK(hipMalloc(&grad, sizeof(double) * nsh * C * Dp));
  CK(hipStreamSynchronize(st));
  const double bytes = (double)nsh * rows * (8.0 * d + 8.0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  SweepArgs A{sh_d, q, partial, nullptr, 0, C, Dp, G, LD, d + 2, 0, G, nullptr};
  // k_sweepe's LDS: the per-wave slots, the beta image [16][4 KF + SE_BPAD], the (unused for the
  // linear family) table block, the ER / PF scratch; or the block reduction, whichever is larger
  const size_t lds_e = std::max(
      (size_t)SM_W * sweepm_slot_bytes(d) + (16 * (4 * KF + SE_BPAD) + LG_TAB + SM_W * 64 + SM_W * 32) * sizeof(double),
      ((size_t)SM_W * JT * 16 * 16 + (size_t)SM_W * 64 * 2 + (size_t)SM_W * 4 * 4 * 16) * sizeof(double));
  printf("rows/shard %lld shards %d d %d C %d: G %d LD %d lds %zu (sweepe %zu), %.2f GB per sweep\n", (long long)rows,
         nsh, d, C, G, LD, lds, lds_e, bytes / 1e9);
  struct Arm { const char* name; const void* kern; bool m; size_t lds; std::vector<float> ms; };
  std::vector<Arm> arms = {
      {"sweepm", (const void*)k_sweepm<STK_LINREG, KF, JT, 0, SM_MINB, true>, true, lds, {}},
      {"sweepe", (const void*)k_sweepe<STK_LINREG, KF, JT, 0, 1, SE_NACC, 0, 2, 1>, false, lds_e, {}},
      {"sweepe-p0", (const void*)k_sweepe<STK_LINREG, KF, JT, 0, 1, SE_NACC, 0, 2, 0>, false, lds_e, {}},
  };
  for (auto& a : arms) CK(hipFuncSetAttribute(a.kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  auto launch = [&](const Arm& a) {
    if (a.m)
      hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs, int)>(const_cast<void*>(a.kern)), dim3(nsh * G),
                         dim3(SM_W * 64), a.lds, st, A, LD);
    else
      hipLaunchKernelGGL(reinterpret_cast<void (*)(SweepArgs)>(const_cast<void*>(a.kern)), dim3(nsh * G),
                         dim3(SM_W * 64), a.lds, st, A);
  };
  std::vector<std::vector<double>> res;
  for (size_t k = 0; k < arms.size(); ++k) {
    launch(arms[k]);
    CK(hipGetLastError());
    CK(stk_launch_sweep_reduce(STK_LINREG, sh_d, 0, nsh, d, G, G, q, C, Dp, partial, nullptr, 0, lp, grad, st));
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
    printf("parity %s vs sweepm: lp max rel %.3g, grad max |diff| / max|grad| %.3g (lp[0] %.6f)\n", arms[k].name, lpr,
           gr, res[0][0]);
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
      printf("round %d %-10s %8.4f ms  %7.1f GB/s  %.3f of 8 TB/s\n", r, a.name, ms / reps, bytes / (ms / reps) / 1e6,
             bytes / (ms / reps) / 1e6 / 8000.0);
      fflush(stdout);
    }
  }
  for (auto& a : arms) {
    std::vector<float> v = a.ms;
    std::sort(v.begin(), v.end());
    printf("median %-10s %8.4f ms  %.3f of 8 TB/s\n", a.name, v[v.size() / 2], bytes / v[v.size() / 2] / 1e6 / 8000.0);
  }
  return 0;
}
