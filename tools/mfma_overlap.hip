// Does one wave overlap its own fp64 VALU work with its in-flight fp64 MFMAs (gfx950)?
// MODE 1: 4 independent MFMA accumulators per iteration only; 2: 64 independent v_fma_f64
// only; 3: both, interleaved by sched_group_barrier (1 MFMA : 16 VALU).
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_overlap.hip -o tools/_bin/mfma_overlap
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int MODE, int NV, int NA = 4>
__global__ __launch_bounds__(256) void k_ov(double* sink, int iters) {
  dbl4 acc[NA] = {};
  double v[NV];
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-6;
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = j * 1e-3 + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    if (MODE & 1) {
#pragma unroll
      for (int j = 0; j < NA; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    if (MODE & 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] = fma(v[j], b, a);
    }
    if (MODE == 3) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      }
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NA; ++j) s += acc[j][j & 3];
#pragma unroll
  for (int j = 0; j < NV; ++j) s += v[j];
  if (s == 12345.678) sink[blockIdx.x] = 1.0;
}

int main() {
  double* sink;
  hipMalloc(&sink, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  auto run = [&](const char* name, auto kern, int wpb, double flops_per_iter_wave) {
    const int blocks = 1024;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, sink, iters);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * wpb), 0, 0, sink, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-24s waves/blk %d  %8.3f ms  %7.1f TF (fp64 incl. both units)\n", name, wpb, ms,
           (double)blocks * wpb * iters * flops_per_iter_wave / ms / 1e9);
  };
  run("mfma only, 8 acc", k_ov<1, 16, 8>, 1, 8 * 2048.0);
  run("mfma only, 12 acc", k_ov<1, 16, 12>, 1, 12 * 2048.0);
  run("mfma only, 16 acc", k_ov<1, 16, 16>, 1, 16 * 2048.0);
  run("mfma only, 8 acc", k_ov<1, 16, 8>, 2, 8 * 2048.0);
  run("valu only 32 chains", k_ov<2, 32>, 1, 128.0 * 64 * 2);
  for (int wpb = 1; wpb <= 2; ++wpb) {
    run("mfma only", k_ov<1, 16>, wpb, 4 * 2048.0);
    run("valu only (16x4 fma)", k_ov<2, 16>, wpb, 64.0 * 64 * 2);
    run("both interleaved", k_ov<3, 16>, wpb, 4 * 2048.0 + 64.0 * 64 * 2);
    run("both, no barrier", k_ov<7, 16>, wpb, 4 * 2048.0 + 64.0 * 64 * 2);
  }
  return 0;
}
