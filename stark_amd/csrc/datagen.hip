// Synthetic shards generated in HBM, so an 80 GB logistic dataset
// never crosses PCIe.  Bit-exact twin of oracle orc_gen_x / orc_gen_y_*:
//   X_ij = ((2k+1) * 2^-52 - 1) * sqrt(3), k = top 52 bits of Philox(TAG_X, row, j/2)
//   eta_i = fma chain alpha + sum_j x_ij beta_j in column order
//   logistic: y_i = 1{u_i < 1/(1+exp(-eta_i))};  linear: y_i = eta_i + sigma * N(0,1)
// Rows carry their GLOBAL index, so a shard's contents do not depend on how the
// dataset was split across GPUs.
#include "common.h"
#include <math.h>

namespace stk {

__device__ __forceinline__ double x_from_bits(uint64_t w) {
  const uint64_t k = w >> 12;
  const double v = __dsub_rn(__dmul_rn((double)(2 * k + 1), 0x1.0p-52), 1.0);
  return __dmul_rn(v, 1.7320508075688772);
}

// One workgroup per tile of T rows: generate X (coalesced stores + LDS copy), then one
// lane per row forms eta sequentially (same fma order as the oracle) and draws y.
__global__ __launch_bounds__(256) void k_gen_shard(double* X, double* yd, int32_t* yi, int64_t nrows, int d,
                                                   int64_t grow0, int T, uint64_t seed, double alpha,
                                                   const double* beta, double noise_sigma, int family) {
  extern __shared__ __attribute__((aligned(16))) double xs[];
  const int64_t r0 = (int64_t)blockIdx.x * T;
  const int rows = (int)((nrows - r0) < T ? (nrows - r0) : T);
  const int hp = (d + 1) / 2;   // Philox calls per row
  for (int i = threadIdx.x; i < rows * hp; i += blockDim.x) {
    const int r = i / hp, jp = i % hp;
    const int64_t g = grow0 + r0 + r;
    const u64x2 w = philox(seed, (uint32_t)g, (uint32_t)((uint64_t)g >> 32), (uint32_t)jp, TAG_X);
    const int j = 2 * jp;
    const double a = x_from_bits(w.a);
    double* row = X + (r0 + r) * d;
    row[j] = a;
    xs[r * d + j] = a;
    if (j + 1 < d) {
      const double b = x_from_bits(w.b);
      row[j + 1] = b;
      xs[r * d + j + 1] = b;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < rows) {
    const int r = threadIdx.x;
    const int64_t g = grow0 + r0 + r;
    double eta = alpha;
    for (int j = 0; j < d; ++j) eta = __fma_rn(xs[r * d + j], beta[j], eta);
    const u64x2 w = philox(seed, (uint32_t)g, (uint32_t)((uint64_t)g >> 32), 0u, TAG_Y);
    if (family == STK_LOGREG) {
      const double p = 1.0 / (1.0 + exp(-eta));
      yi[r0 + r] = u53(w.a) < p ? 1 : 0;
    } else {
      const double u1 = u53(w.a), u2 = u53(w.b);
      const double z0 = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
      yd[r0 + r] = eta + noise_sigma * z0;
    }
  }
}

// y in {0, 1} check of a bernoulli_logit shard (stk_model_create): *first = the first row whose
// y is neither, or INT64_MAX.  Each block takes the minimum over its rows, one atomicMin per block.
__global__ __launch_bounds__(256) void k_check_y01(const int32_t* y, int64_t n, unsigned long long* first) {
  __shared__ unsigned long long m[4];
  unsigned long long b = ~0ull >> 1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int32_t v = y[i];
    if ((v != 0 && v != 1) && (unsigned long long)i < b) b = (unsigned long long)i;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(b, o);
    b = t < b ? t : b;
  }
  if ((threadIdx.x & 63) == 0) m[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) b = m[w] < b ? m[w] : b;
    if (b != (~0ull >> 1)) atomicMin(first, b);
  }
}

__global__ void k_set_i64(int64_t* p, int64_t v) { *p = v; }

}  // namespace stk

using namespace stk;

hipError_t stk_launch_check_y01(const int32_t* y, int64_t n, int64_t* first, hipStream_t st) {
  hipLaunchKernelGGL(k_set_i64, dim3(1), dim3(1), 0, st, first, (int64_t)(~0ull >> 1));
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_check_y01, dim3((unsigned)blocks), dim3(256), 0, st, y, n,
                     reinterpret_cast<unsigned long long*>(first));
  return hipGetLastError();
}

hipError_t stk_launch_gen_shard(double* X, double* yd, int32_t* yi, int64_t nrows, int d, int64_t grow0,
                                uint64_t seed, double alpha, const double* beta, double noise_sigma, int family,
                                hipStream_t st) {
  int T = 64;
  while (T > 1 && (int64_t)T * d * 8 > 64 * 1024) T >>= 1;
  const size_t lds = (size_t)T * d * sizeof(double);
  if (const hipError_t e = allow_big_lds((const void*)k_gen_shard)) return e;
  const int64_t blocks = (nrows + T - 1) / T;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gen_shard, dim3((unsigned)blocks), dim3(256), lds, st, X, yd, yi, nrows, d, grow0, T, seed,
                     alpha, beta, noise_sigma, family);
  return hipGetLastError();
}
