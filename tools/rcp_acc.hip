// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp) on gfx950 against the correctly rounded 1/x, over
// u = 1 + e, e in [0, 1] (the logistic residual's denominator), in units of the last place.
// Build: hipcc -O3 --offload-arch=gfx950 tools/rcp_acc.hip -o tools/_bin/rcp_acc
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
__global__ void k(const double* x, double* r, double* r1, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double u = x[i];
    double ri = __builtin_amdgcn_rcp(u);
    r[i] = ri;
    r1[i] = fma(ri, fma(-u, ri, 1.0), ri);
  }
}
int main() {
  const int n = 1 << 24;
  std::vector<double> x(n), r(n), r1(n);
  srand(1);
  for (int i = 0; i < n; ++i) x[i] = 1.0 + (double)i / n + ((double)rand() / RAND_MAX) / n;
  double *dx, *dr, *dr1;
  hipMalloc(&dx, 8.0 * n); hipMalloc(&dr, 8.0 * n); hipMalloc(&dr1, 8.0 * n);
  hipMemcpy(dx, x.data(), 8.0 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dr, dr1, n);
  hipMemcpy(r.data(), dr, 8.0 * n, hipMemcpyDeviceToHost);
  hipMemcpy(r1.data(), dr1, 8.0 * n, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0;
  long bad0 = 0;
  for (int i = 0; i < n; ++i) {
    const long double ex = 1.0L / (long double)x[i];
    const double ulp = nextafter((double)ex, 2.0) - (double)ex;
    const double e0 = fabs((double)((long double)r[i] - ex)) / ulp, e1 = fabs((double)((long double)r1[i] - ex)) / ulp;
    m0 = fmax(m0, e0); m1 = fmax(m1, e1);
    bad0 += e0 > 1.0;
  }
  printf("v_rcp_f64 on [1, 2]: max error %.3f ulp (%ld of %d above 1 ulp); after one Newton step %.3f ulp\n", m0, bad0, n, m1);
  return 0;
}
