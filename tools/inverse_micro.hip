// Time per pivot of the combine's SPD inverse (the kernel of combine.hip, copied by the
// round-2 investigation; V is unused).
// Build: hipcc -O3 --offload-arch=gfx950 tools/inverse_micro.hip -o tools/_bin/inverse_micro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <math.h>
typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int SI_B = 8;                           // block edge
template <int V>
__global__ __launch_bounds__(256) void k_inv(const double* Min, double* Out, int P, const int32_t* used,
                                                     int32_t* status) {
  __shared__ __attribute__((aligned(16))) double rowk[2][128];
  __shared__ __attribute__((aligned(16))) double colk[2][128];
  __shared__ double dsc[128];                     // 1 / sqrt(A_ii)
  const int b = blockIdx.x, tid = threadIdx.x;
  const int bi = tid >> 4, bj = tid & 15;        // block row / column
  const int i0 = SI_B * bi, j0 = SI_B * bj;
  const double* M = Min + (size_t)b * P * P;
  double* out = Out + (size_t)b * P * P;
  if (used && !used[b]) {
    for (int i = tid; i < P * P; i += 256) out[i] = 0.0;
    if (tid == 0) status[b] = 0;
    return;
  }
  int sing = 0;
  if (tid < 128) {
    const double dii = tid < P ? M[(size_t)tid * P + tid] : 1.0;
    if (!(dii > 0.0)) sing = 1;
    dsc[tid] = dii > 0.0 ? 1.0 / sqrt(dii) : 1.0;
  }
  sing = __syncthreads_or(sing);
  if (sing) {
    if (tid == 0) status[b] = 1;
    return;
  }
  double a[SI_B][SI_B];
  double si[SI_B], sj[SI_B];
#pragma unroll
  for (int u = 0; u < SI_B; ++u) {
    si[u] = dsc[i0 + u];
    sj[u] = dsc[j0 + u];
  }
#pragma unroll
  for (int u = 0; u < SI_B; ++u)
#pragma unroll
    for (int v = 0; v < SI_B; ++v) {
      const int i = i0 + u, j = j0 + v;
      a[u][v] = (i == j) ? 1.0 : ((i < P && j < P) ? M[(size_t)i * P + j] * si[u] * sj[v] : 0.0);
    }
  if (bi == 0) {
#pragma unroll
    for (int v = 0; v < SI_B; ++v) rowk[0][j0 + v] = a[0][v];
  }
  if (bj == 0) {
#pragma unroll
    for (int u = 0; u < SI_B; ++u) colk[0][i0 + u] = (i0 + u == 0) ? a[u][0] - 1.0 : a[u][0];
  }
  __syncthreads();
  for (int k = 0; k < P; ++k) {
    const int cur = k & 1, nxt = cur ^ 1;
    double c[SI_B], r[SI_B];
    const dbl2* cp = reinterpret_cast<const dbl2*>(&colk[cur][i0]);
    const dbl2* rp = reinterpret_cast<const dbl2*>(&rowk[cur][j0]);
#pragma unroll
    for (int h = 0; h < SI_B / 2; ++h) {
      const dbl2 cv = cp[h], rv = rp[h];
      c[2 * h] = cv.x;
      c[2 * h + 1] = cv.y;
      r[2 * h] = rv.x;
      r[2 * h + 1] = rv.y;
    }
    const double piv = rowk[cur][k];
    if (!(piv > 0.0)) { sing = 1; break; }      // uniform: every thread read the same pivot
    double ip = __builtin_amdgcn_rcp(piv);      // 1/piv to the last ulp: two Newton steps
    ip = fma(ip, fma(-piv, ip, 1.0), ip);
    ip = fma(ip, fma(-piv, ip, 1.0), ip);
    const int kb = k >> 3, kv = k & 7;
#pragma unroll
    for (int v = 0; v < SI_B; ++v) r[v] = (bj == kb && v == kv) ? 1.0 + ip : r[v] * ip;
#pragma unroll
    for (int u = 0; u < SI_B; ++u)
#pragma unroll
      for (int v = 0; v < SI_B; ++v) a[u][v] = fma(-c[u], r[v], a[u][v]);   // the whole step
    // publish row and column k+1 (block-uniform tests on k)
    const int k1 = k + 1, k1b = k1 >> 3, k1u = k1 & 7;
    if (bi == k1b) {
#pragma unroll
      for (int u = 0; u < SI_B; ++u)
        if (u == k1u) {
#pragma unroll
          for (int v = 0; v < SI_B; ++v) rowk[nxt][j0 + v] = a[u][v];
        }
    }
    if (bj == k1b) {
#pragma unroll
      for (int v = 0; v < SI_B; ++v)
        if (v == k1u) {
#pragma unroll
          for (int u = 0; u < SI_B; ++u) colk[nxt][i0 + u] = (i0 + u == k1) ? a[u][v] - 1.0 : a[u][v];
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < SI_B; ++u)
#pragma unroll
    for (int v = 0; v < SI_B; ++v) {
      const int i = i0 + u, j = j0 + v;
      if (i < P && j < P) out[(size_t)i * P + j] = a[u][v] * si[u] * sj[v];
    }
  if (tid == 0) status[b] = sing;
}

template <int V>
static void run(int P, int batch, const double* M, double* O, int* st) {
  hipLaunchKernelGGL(k_inv<V>, dim3(batch), dim3(256), 0, 0, M, O, P, nullptr, st);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_inv<V>, dim3(batch), dim3(256), 0, 0, M, O, P, nullptr, st);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("V%d P %3d batch %d: %8.2f us per launch, %6.3f us per pivot\n", V, P, batch, ms * 100, ms * 100 / P);
}
int main() {
  const int P = 102;
  std::vector<double> h((size_t)8 * P * P);
  for (int b = 0; b < 8; ++b)
    for (int i = 0; i < P; ++i)
      for (int j = 0; j < P; ++j) h[(size_t)b * P * P + i * P + j] = (i == j ? 2.0 : 0.0) + 0.01 / (1 + abs(i - j));
  double *M, *O;
  int* st;
  if (hipMalloc(&M, h.size() * 8) || hipMalloc(&O, h.size() * 8) || hipMalloc(&st, 64)) return 1;
  (void)hipMemcpy(M, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  run<0>(102, 1, M, O, st);
  run<0>(102, 8, M, O, st);
  return 0;
}
