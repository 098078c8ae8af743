// Cost of one workgroup barrier step on gfx950 (the SPD inverse's pivot loop is a chain of
// them): ITERS x {LDS read of a broadcast value, FMAs, LDS write, __syncthreads()} for 1, 4 and
// 16 waves per workgroup, one workgroup (latency), reported per iteration.
// Build: hipcc -O3 --offload-arch=gfx950 tools/barrier_micro.hip -o tools/_bin/barrier_micro
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NFMA>
__global__ void k_steps(double* out, int iters) {
  __shared__ double buf[2][1024];
  const int t = threadIdx.x;
  double a[NFMA > 0 ? NFMA : 1];
  for (int r = 0; r < (NFMA > 0 ? NFMA : 1); ++r) a[r] = t * 1e-3 + r;
  buf[0][t] = 1.0 + t * 1e-6;
  __syncthreads();
  for (int k = 0; k < iters; ++k) {
    const int cur = k & 1;
    const double p = buf[cur][k & 1023];
    const double q = buf[cur][(t + k) & 1023];
#pragma unroll
    for (int r = 0; r < NFMA; ++r) a[r] = fma(-p, q, a[r]);
    buf[cur ^ 1][t] = q * 0.999 + (NFMA > 0 ? a[0] * 1e-30 : 0.0);
    __syncthreads();
  }
  double s = 0;
  for (int r = 0; r < (NFMA > 0 ? NFMA : 1); ++r) s += a[r];
  out[t] = s;
}

template <int NFMA>
static void run(int threads, int iters, double* out) {
  hipLaunchKernelGGL(k_steps<NFMA>, dim3(1), dim3(threads), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_steps<NFMA>, dim3(1), dim3(threads), 0, 0, out, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("threads %4d  fma/thread/step %2d  %8.3f us per step\n", threads, NFMA, ms * 1e3 / iters);
}

int main() {
  double* out;
  if (hipMalloc(&out, 1024 * sizeof(double)) != hipSuccess) return 1;
  const int iters = 20000;
  for (int th : {64, 256, 1024}) {
    run<0>(th, iters, out);
    run<16>(th, iters, out);
  }
  return 0;
}
