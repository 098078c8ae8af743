// fp64 MFMA ceiling on gfx950 (pins the roofline the data sweep is judged against).
//
// v_mfma_f64_16x16x4_f64 back to back with NACC independent accumulators per wave, W waves
// per SIMD (W blocks of 256 threads per CU), operands random (DVFS depends on operand bits).
// Every block stamps s_memtime / s_memrealtime around its loop, so the in-kernel clock is
// measured next to the wall time: TF/s = flops / wall; cycles per MFMA per SIMD =
// clock * wall / (MFMAs per SIMD).  Diagnostic build only: the stamps go to a buffer of their
// own that nothing else reads.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mfma_ceiling.hip -o tools/_bin/mfma_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef double dbl4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(const double* src, double* sink, unsigned long long* stamps, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const double a = src[t & 4095], b = src[(t * 7 + 13) & 4095];
  dbl4 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) acc[j] = dbl4{src[(t + j) & 4095], 0.0, 0.0, 0.0};
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][3];
  if (s == 12345.678) sink[t] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// The 4x4x4 four-block form: v_mfma_f64_4x4x4_4b_f64, 512 flops per instruction, one f64
// accumulator per lane.
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma4(const double* src, double* sink, unsigned long long* stamps, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const double a = src[t & 4095], b = src[(t * 7 + 13) & 4095];
  double acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) acc[j] = src[(t + j) & 4095];
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[j], 0, 0, 0);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += acc[j];
  if (s == 12345.678) sink[t] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int NACC>
static void run4(int wps, int iters, const double* src, double* sink, unsigned long long* st, int ncu) {
  const int nb = ncu * wps;
  hipLaunchKernelGGL(k_mfma4<NACC>, dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_mfma4<NACC>, dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost));
  std::vector<double> clk(nb);
  for (int b = 0; b < nb; ++b) clk[b] = (double)h[2 * b] / (double)h[2 * b + 1] * 100.0;
  std::sort(clk.begin(), clk.end());
  const double flops = (double)nb * 4 * iters * NACC * 512.0;
  const double per_simd = (double)wps * iters * NACC;
  const double cyc = clk[nb / 2] * 1e6 * best * 1e-3 / per_simd;
  printf("mfma_f64_4x4x4_4b  waves/SIMD %d  acc %2d  %8.3f ms  %6.1f TF/s  clock %6.0f MHz  cycles/instr/SIMD %5.1f\n",
         wps, NACC, best, flops / best / 1e9, clk[nb / 2], cyc);
  fflush(stdout);
}

// fp64 VALU FMA rate: NACC independent v_fma_f64 chains per lane (operands in VGPRs), and
// the same with one operand a wave-uniform SGPR value (the beta-from-scalar-registers form).
template <int NACC, bool SOP>
__global__ __launch_bounds__(256) void k_fma(const double* src, double* sink, unsigned long long* stamps, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  double b = src[(t * 7 + 13) & 4095];
  if (SOP) b = __builtin_amdgcn_readfirstlane((int)t) == 12345 ? 1.0 : src[blockIdx.x & 4095];
  double acc[NACC];
  double a[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) { acc[j] = src[(t + j) & 4095]; a[j] = src[(t + 3 * j + 1) & 4095]; }
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = fma(a[j], b, acc[j]);
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NACC; ++j) s += acc[j];
  if (s == 12345.678) sink[t] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int NACC, bool SOP>
static void run_fma(int wps, int iters, const double* src, double* sink, unsigned long long* st, int ncu) {
  const int nb = ncu * wps;
  hipLaunchKernelGGL((k_fma<NACC, SOP>), dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_fma<NACC, SOP>), dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost));
  std::vector<double> clk(nb);
  for (int b = 0; b < nb; ++b) clk[b] = (double)h[2 * b] / (double)h[2 * b + 1] * 100.0;
  std::sort(clk.begin(), clk.end());
  const double flops = (double)nb * 256 * iters * NACC * 2.0;
  const double instr_per_simd = (double)wps * iters * NACC;
  const double cyc = clk[nb / 2] * 1e6 * best * 1e-3 / instr_per_simd;
  printf("v_fma_f64 %s  waves/SIMD %d  chains %2d  %8.3f ms  %6.1f TF/s  clock %6.0f MHz  cycles/instr/SIMD %5.2f\n",
         SOP ? "sgpr-op" : "vgpr   ", wps, NACC, best, flops / best / 1e9, clk[nb / 2], cyc);
  fflush(stdout);
}

template <int NACC>
static void run(int wps, int iters, const double* src, double* sink, unsigned long long* st, int ncu) {
  const int nb = ncu * 4 * wps / 4;   // 256-thread blocks: 4 waves each, one per SIMD
  hipLaunchKernelGGL(k_mfma<NACC>, dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_mfma<NACC>, dim3(nb), dim3(256), 0, 0, src, sink, st, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  std::vector<unsigned long long> h(2 * nb);
  CK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost));
  std::vector<double> clk(nb);
  for (int b = 0; b < nb; ++b) clk[b] = (double)h[2 * b] / (double)h[2 * b + 1] * 100.0;   // MHz (realtime = 100 MHz)
  std::sort(clk.begin(), clk.end());
  const double flops = (double)nb * 4 * iters * NACC * 2048.0;
  const double mfma_per_simd = (double)wps * iters * NACC;
  const double cyc = clk[nb / 2] * 1e6 * best * 1e-3 / mfma_per_simd;
  printf("waves/SIMD %d  acc %2d  %8.3f ms  %6.1f TF/s  clock(median) %6.0f MHz  cycles/MFMA/SIMD %5.1f  -> %.1f TF at 2400 MHz\n",
         wps, NACC, best, flops / best / 1e9, clk[nb / 2], cyc, 1024.0 * 2048.0 / cyc * 2.4e9 / 1e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  printf("%s, %d CUs\n", p.gcnArchName, ncu);
  std::vector<double> h(4096);
  unsigned s = 12345;
  for (auto& v : h) { s = s * 1103515245u + 12345u; v = ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; }
  double *src, *sink;
  unsigned long long* st;
  CK(hipMalloc(&src, sizeof(double) * 4096));
  CK(hipMemcpy(src, h.data(), sizeof(double) * 4096, hipMemcpyHostToDevice));
  CK(hipMalloc(&sink, sizeof(double) * ncu * 4 * 8 * 256));
  CK(hipMalloc(&st, sizeof(unsigned long long) * 2 * ncu * 8));
  const bool only4 = argc > 2 && argv[2][0] == '4';
  for (int w : {1, 2, 4}) {
    run4<4>(w, iters * 2, src, sink, st, ncu);
    run4<8>(w, iters * 2, src, sink, st, ncu);
  }
  if (only4) return 0;
  for (int w : {1, 2, 4}) {
    run<4>(w, iters, src, sink, st, ncu);
    run<8>(w, iters, src, sink, st, ncu);
  }
  run<16>(1, iters, src, sink, st, ncu);
  for (int w : {1, 2, 4}) {
    run_fma<8, false>(w, iters * 4, src, sink, st, ncu);
    run_fma<16, false>(w, iters * 2, src, sink, st, ncu);
    run_fma<8, true>(w, iters * 4, src, sink, st, ncu);
  }
  return 0;
}
