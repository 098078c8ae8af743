// Consensus weighted-average combine on gfx950 (fp64).
//
// Replaces stark/stark.py:7-21 (consensus_avg: W_s = inv(np.cov(theta_s)), returns
// [sum W_s, sum W_s theta_s]) and the driver solve stark/stark.py:66-70
// (inv(sum W) . sum W theta).  General in the shard count (the reference reducer only
// works for two partitions); shards holding NaN draws are left out, the
// intent of the guard at stark/stark.py:9-10.  All sums run in shard order, so the result
// is bitwise identical however the shards were spread over GPUs.
//
// Kernels: per-row means, centring, a 16x16-tiled fp64 GEMM (LDS-staged K slices) for
// cov = Xc Xc^T * 1/(S-1), W_s theta_s and the final product, and Gauss-Jordan inversion
// with partial pivoting (one workgroup per matrix, as LAPACK getrf+getri pivot rows).
#include "common.h"
#include <math.h>

namespace stk {

__global__ __launch_bounds__(256) void k_nan_flags(const double* X, int64_t per, int32_t* used) {
  const int s = blockIdx.x;
  const double* x = X + (size_t)s * per;
  int bad = 0;
  for (int64_t i = threadIdx.x; i < per; i += blockDim.x) bad |= isnan(x[i]) ? 1 : 0;
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) used[s] = bad ? 0 : 1;
}

// mean over the S columns of row (s, a), then centred copy (numpy: X -= X.mean(axis=1)).
__global__ __launch_bounds__(256) void k_center(const double* X, double* Xc, int P, int S) {
  const int row = blockIdx.x;   // s * P + a
  const double* x = X + (size_t)row * S;
  double* xc = Xc + (size_t)row * S;
  __shared__ double red[256];
  double v = 0.0;
  for (int k = threadIdx.x; k < S; k += 256) v += x[k];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double mean = red[0] / (double)S;
  for (int k = threadIdx.x; k < S; k += 256) xc[k] = x[k] - mean;
}

// C[M x N] (ldc) = alpha * A[M x K] (lda) . op(B) + beta * C, op(B) = B[K x N] or B^T with
// B stored [N x K].  batch over blockIdx.z with strides.  16x16 threads, 16-deep K slices.
template <bool BT>
__global__ __launch_bounds__(256) void k_gemm(const double* A, const double* B, double* C, int M, int N, int K,
                                              int lda, int ldb, int ldc, double alpha, double beta, size_t sA,
                                              size_t sB, size_t sC) {
  __shared__ double As[16][17];
  __shared__ double Bs[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int row = blockIdx.y * 16 + ty, col = blockIdx.x * 16 + tx;
  A += sA * blockIdx.z;
  B += sB * blockIdx.z;
  C += sC * blockIdx.z;
  double acc = 0.0;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const int ar = blockIdx.y * 16 + ty, ak = k0 + tx;
    As[ty][tx] = (ar < M && ak < K) ? A[(size_t)ar * lda + ak] : 0.0;
    if (BT) {
      const int bn = blockIdx.x * 16 + ty, bk = k0 + tx;   // B is [N x K]
      Bs[tx][ty] = (bn < N && bk < K) ? B[(size_t)bn * ldb + bk] : 0.0;
    } else {
      const int bk = k0 + ty, bn = blockIdx.x * 16 + tx;   // B is [K x N]
      Bs[ty][tx] = (bk < K && bn < N) ? B[(size_t)bk * ldb + bn] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc += As[ty][kk] * Bs[kk][tx];
    __syncthreads();
  }
  if (row < M && col < N) {
    double* c = C + (size_t)row * ldc + col;
    *c = (beta == 0.0) ? alpha * acc : alpha * acc + beta * *c;
  }
}

// Gauss-Jordan inverse with partial pivoting of a batch of P x P matrices.  W holds the
// [P x 2P] augmented workspace per matrix; writes the inverse to Inv.  status[b] = 1 on a
// zero pivot (singular).
__global__ __launch_bounds__(1024) void k_gj_inverse(const double* Min, double* W, double* Inv, int P,
                                                     int32_t* status) {
  const int b = blockIdx.x;
  const double* M = Min + (size_t)b * P * P;
  double* A = W + (size_t)b * P * 2 * P;
  double* out = Inv + (size_t)b * P * P;
  const int tid = threadIdx.x, nt = blockDim.x, W2 = 2 * P;
  for (int i = tid; i < P * W2; i += nt) {
    const int r = i / W2, c = i % W2;
    A[i] = c < P ? M[(size_t)r * P + c] : (c - P == r ? 1.0 : 0.0);
  }
  __shared__ double sval[1024];
  __shared__ int sidx[1024];
  __shared__ int singular;
  if (tid == 0) singular = 0;
  __syncthreads();
  for (int k = 0; k < P; ++k) {
    // pivot search over rows k..P-1 (max |a_ik|, lowest index on ties)
    double best = -1.0;
    int bi = k;
    for (int i = k + tid; i < P; i += nt) {
      const double v = fabs(A[(size_t)i * W2 + k]);
      if (v > best) { best = v; bi = i; }
    }
    sval[tid] = best;
    sidx[tid] = bi;
    __syncthreads();
    for (int o = nt / 2; o > 0; o >>= 1) {
      if (tid < o) {
        const double v2 = sval[tid + o];
        const int i2 = sidx[tid + o];
        if (v2 > sval[tid] || (v2 == sval[tid] && i2 < sidx[tid])) { sval[tid] = v2; sidx[tid] = i2; }
      }
      __syncthreads();
    }
    const int piv = sidx[0];
    if (sval[0] == 0.0) { if (tid == 0) singular = 1; }
    __syncthreads();
    if (piv != k) {
      for (int c = tid; c < W2; c += nt) {
        const double t = A[(size_t)k * W2 + c];
        A[(size_t)k * W2 + c] = A[(size_t)piv * W2 + c];
        A[(size_t)piv * W2 + c] = t;
      }
    }
    __syncthreads();
    const double inv_p = 1.0 / A[(size_t)k * W2 + k];
    __syncthreads();
    for (int c = tid; c < W2; c += nt) A[(size_t)k * W2 + c] *= inv_p;
    __syncthreads();
    for (int i = tid; i < P * W2; i += nt) {
      const int r = i / W2, c = i % W2;
      if (r == k) continue;
      const double f = A[(size_t)r * W2 + k];
      if (c == k) continue;
      A[i] -= f * A[(size_t)k * W2 + c];
    }
    __syncthreads();
    for (int r = tid; r < P; r += nt)
      if (r != k) A[(size_t)r * W2 + k] = 0.0;
    __syncthreads();
  }
  for (int i = tid; i < P * P; i += nt) {
    const int r = i / P, c = i % P;
    out[i] = A[(size_t)r * W2 + P + c];
  }
  if (tid == 0) status[b] = singular;
}

// sum over used shards, in shard order: dst = sum_s src_s (n elements each)
__global__ void k_masked_sum(const double* src, const int32_t* used, int nshards, size_t n, double* dst) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double v = 0.0;
    bool any = false;
    for (int s = 0; s < nshards; ++s) {
      if (!used[s]) continue;
      const double x = src[(size_t)s * n + i];
      v = any ? v + x : x;
      any = true;
    }
    dst[i] = v;
  }
}

}  // namespace stk

using namespace stk;

hipError_t stk_launch_nan_flags(const double* X, int nshards, int64_t per, int32_t* used, hipStream_t st) {
  hipLaunchKernelGGL(k_nan_flags, dim3(nshards), dim3(256), 0, st, X, per, used);
  return hipGetLastError();
}
hipError_t stk_launch_center(const double* X, double* Xc, int rows, int P, int S, hipStream_t st) {
  hipLaunchKernelGGL(k_center, dim3(rows), dim3(256), 0, st, X, Xc, P, S);
  return hipGetLastError();
}
hipError_t stk_launch_gemm(bool bt, const double* A, const double* B, double* C, int M, int N, int K, int lda, int ldb,
                           int ldc, double alpha, double beta, int batch, size_t sA, size_t sB, size_t sC,
                           hipStream_t st) {
  dim3 grid((N + 15) / 16, (M + 15) / 16, batch);
  if (bt)
    hipLaunchKernelGGL(k_gemm<true>, grid, dim3(256), 0, st, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, sA, sB, sC);
  else
    hipLaunchKernelGGL(k_gemm<false>, grid, dim3(256), 0, st, A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, sA, sB, sC);
  return hipGetLastError();
}
hipError_t stk_launch_gj_inverse(const double* M, double* W, double* Inv, int P, int batch, int32_t* status,
                                 hipStream_t st) {
  int nt = 256;
  while (nt < 1024 && nt < 2 * P) nt *= 2;
  hipLaunchKernelGGL(k_gj_inverse, dim3(batch), dim3(nt), 0, st, M, W, Inv, P, status);
  return hipGetLastError();
}
hipError_t stk_launch_masked_sum(const double* src, const int32_t* used, int nshards, size_t n, double* dst,
                                 hipStream_t st) {
  size_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_masked_sum, dim3((unsigned)blocks), dim3(256), 0, st, src, used, nshards, n, dst);
  return hipGetLastError();
}
