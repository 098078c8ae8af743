// Ablations of the combine's fp64 MFMA GEMM (k_mgemm, combine.hip) at the headline combine size
// (8 shards, P = 102, S = 1600): the real loaders against loaders with no memory traffic and with
// plain row-major pointers, to find what bounds the launch.
// Build: hipcc -O3 --offload-arch=gfx950 -I stark_amd/csrc tools/mgemm_micro.hip -o tools/_bin/mgemm_micro
#include "../stark_amd/csrc/combine.hip"
#include <stdio.h>
#include <vector>

struct SynthLd {             // operands from arithmetic only (no loads)
  double* out;
  int P;
  __device__ void a4(int z, int m, int k, int, double* v) const {
    for (int j = 0; j < 4; ++j) v[j] = 1e-3 * (m + 1) + 1e-6 * ((k + j) & 63) + z;
  }
  __device__ void b4(int z, int k, int n, int, double* v) const {
    for (int j = 0; j < 4; ++j) v[j] = 1e-3 * (n + 1) - 1e-6 * ((k + j) & 31) + z;
  }
  __device__ void store(int z, int m, int n, double v) const { out[((size_t)z * P + m) * P + n] = v; }
};
struct RowLd {               // Cov shape from plain row-major pointers, no centring
  const double* X;
  double* out;
  int P, S;
  __device__ void a4(int z, int m, int k, int K, double* v) const {
    for (int j = 0; j < 4; ++j) v[j] = k + j < K ? X[((size_t)z * P + m) * S + k + j] : 0.0;
  }
  __device__ void b4(int z, int k, int n, int K, double* v) const { a4(z, n, k, K, v); }
  __device__ void store(int z, int m, int n, double v) const { out[((size_t)z * P + m) * P + n] = v; }
};

template <class F>
static float timeit(F f, int reps = 50) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return 1e3f * ms / reps;   // us
}

int main() {
  const int Z = 8, P = 102, S = 1600;
  std::vector<double> h((size_t)Z * P * S);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) * 1e-3;
  double *X, *mean, *cov, *W, *out;
  int32_t* used;
  hipMalloc(&X, sizeof(double) * h.size());
  hipMalloc(&mean, sizeof(double) * Z * P);
  hipMalloc(&cov, sizeof(double) * Z * P * P);
  hipMalloc(&W, sizeof(double) * Z * P * P);
  hipMalloc(&out, sizeof(double) * (size_t)P * S * 2);
  hipMalloc(&used, sizeof(int32_t) * Z);
  hipMemcpy(X, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
  hipMemset(mean, 0, sizeof(double) * Z * P);
  hipMemset(W, 0, sizeof(double) * Z * P * P);
  std::vector<int32_t> u(Z, 1);
  hipMemcpy(used, u.data(), sizeof(int32_t) * Z, hipMemcpyHostToDevice);
  hipStream_t st = 0;
  printf("cov  CovLd   %8.2f us\n", timeit([&] { mgemm<CovLd, 1, 4, true>(CovLd{X, mean, nullptr, cov, P, S, 1.0}, P, P, S, Z, st); }));
  mgemm<CovLd, 1, 4, true>(CovLd{X, mean, nullptr, cov, P, S, 1.0 / (S - 1)}, P, P, S, Z, st);
  int32_t* status;
  hipMalloc(&status, sizeof(int32_t) * Z);
  printf("inv  spd x1  %8.2f us\n", timeit([&] { stk_launch_spd_inverse(cov, W, nullptr, P, 1, nullptr, status, st); }, 20));
  printf("inv  spd x8  %8.2f us\n", timeit([&] { stk_launch_spd_inverse(cov, W, nullptr, P, Z, used, status, st); }, 20));
  int32_t hs[8];
  hipMemcpy(hs, status, sizeof(hs), hipMemcpyDeviceToHost);
  printf("inv  status  %d %d %d %d %d %d %d %d\n", hs[0], hs[1], hs[2], hs[3], hs[4], hs[5], hs[6], hs[7]);
  printf("cov  RowLd   %8.2f us\n", timeit([&] { mgemm<RowLd, 1, 4, true>(RowLd{X, cov, P, S}, P, P, S, Z, st); }));
  printf("cov  SynthLd %8.2f us\n", timeit([&] { mgemm<SynthLd, 1, 4, true>(SynthLd{cov, P}, P, P, S, Z, st); }));
  printf("wth  WTheta  %8.2f us\n", timeit([&] { mgemm<WThetaLd, 2, 2, false>(WThetaLd{W, X, used, out, P, S}, P, S, Z * P, 1, st); }));
  printf("wth  Plain   %8.2f us\n", timeit([&] { mgemm<PlainLd, 2, 2, false>(PlainLd{W, X, out, Z * P, S, S}, P, S, Z * P, 1, st); }));
  printf("wth  Synth   %8.2f us\n", timeit([&] { mgemm<SynthLd, 2, 2, false>(SynthLd{out, S}, P, S, Z * P, 1, st); }));
  printf("sol  Plain   %8.2f us\n", timeit([&] { mgemm<PlainLd, 2, 2, false>(PlainLd{W, X, out, P, S, S}, P, S, P, 1, st); }));
  printf("empty launch %8.2f us\n", timeit([&] { hipLaunchKernelGGL(k_sum_w, dim3(1), dim3(64), 0, st, mean, 1, (size_t)1, mean + 1); }));
  return 0;
}
