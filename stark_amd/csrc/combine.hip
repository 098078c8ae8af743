// Consensus weighted-average combine on gfx950 (fp64).
//
// Replaces stark/stark.py:7-21 (consensus_avg: W_s = inv(np.cov(theta_s)), returns
// [sum W_s, sum W_s theta_s]) and the driver solve stark/stark.py:66-70
// (inv(sum W) . sum W theta).  General in the shard count (the reference reducer only
// works for two partitions); shards holding NaN draws are left out, the
// intent of the guard at stark/stark.py:9-10.  Every sum runs in a fixed order, so the
// result is bitwise identical however the shards were spread over GPUs.
//
// The whole combine is a handful of launches on one stream, no host round trip in between:
//   k_row_stats      per (shard, row): mean over the S draws (np.cov centres rows) + NaN flag
//   k_mgemm<Cov>     cov_s = (X_s - m_s)(X_s - m_s)^T / (S - 1), centring folded into the
//                    tile loads; rows of different weight blocks (lp__ alone)
//                    get 0, so the weights are block-diagonal when asked for
//   k_spd_inverse    W_s = inv(cov_s): block Gauss-Jordan on 16 x 16 tiles held in registers,
//                    fp64 MFMA updates (P <= 128), diagonal pivots -- a covariance is
//                    symmetric positive (semi)definite, where diagonal pivoting is stable
//                    (Cholesky's argument); a pivot <= P eps or NaN is reported as singular
//                    (LinAlgError).  One workgroup per shard, shards in parallel.  P > 128
//                    falls back to k_gj_inverse (partial pivoting, global memory).
//   k_sum_w          sum_s W_s in shard order (NaN shards hold W = 0)
//   k_mgemm<WTheta>  sum_s W_s theta_s as ONE GEMM with K = shards x P:
//                    [W_1 .. W_S] (P x SP) . [theta_1; ..; theta_S] (SP x S), NaN shards skipped
//   k_spd_inverse + k_mgemm<Plain>  out = inv(sum W) . sum W theta (the public stk_consensus_solve,
//                    whose sum W comes from the caller, inverts it by partial pivoting instead)
// k_mgemm: fp64 MFMA, one 16 x 16 NB output tile per block, K split over the block's waves,
// every output a fixed-order sum (cov_s only on the upper tiles, stored both ways).
#include "common.h"
#include <math.h>
#include <algorithm>
#include <utility>

namespace stk {

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef double dbl4 __attribute__((ext_vector_type(4)));

// ---- tile loaders: a4(m, k..k+3), b4(k..k+3, n) (zero past K; k % 4 == 0), store(m, n, v)
struct CovLd {               // batch = shard (blockIdx.z)
  const double* X;           // [shard][P][S]
  const double* mean;        // [shard][P]
  const int32_t* blk;        // [P] weight block of each row, or null (one block)
  double* cov;               // [shard][P][P]
  int P, S;
  double scale;
  __device__ void store(int z, int m, int n, double v) const {
    cov[((size_t)z * P + m) * P + n] = (blk && blk[m] != blk[n]) ? 0.0 : v * scale;
  }
  // 4 consecutive k of one centred row (k % 4 == 0): two 16-B loads when the row is 16-B aligned
  __device__ void row4(int z, int m, int k, int K, double* v) const {
    const double* row = X + ((size_t)z * P + m) * S;
    const double mu = mean[(size_t)z * P + m];
    if (k + 3 < K && !(S & 1)) {
      const dbl2 x0 = *reinterpret_cast<const dbl2*>(row + k), x1 = *reinterpret_cast<const dbl2*>(row + k + 2);
      v[0] = x0.x - mu;
      v[1] = x0.y - mu;
      v[2] = x1.x - mu;
      v[3] = x1.y - mu;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = k + j < K ? row[k + j] - mu : 0.0;
    }
  }
  __device__ void a4(int z, int m, int k, int K, double* v) const { row4(z, m, k, K, v); }
  __device__ void b4(int z, int k, int n, int K, double* v) const { row4(z, n, k, K, v); }
};
struct WThetaLd {            // sum_s W_s theta_s, K = nshards * P
  const double* W;           // [shard][P][P]
  const double* X;           // [shard][P][S] = [(shard, row)][S]
  const int32_t* used;       // [shard]
  double* out;               // [P][S]
  int P, S;
  __device__ void store(int, int m, int n, double v) const { out[(size_t)m * S + n] = v; }
  // k % 4 == 0; the shards of k .. k+3 follow from k's with one division per call.
  // W of a NaN shard is 0 already (k_spd_inverse), its draws are masked here
  __device__ void a4(int, int m, int k, int K, double* v) const {
    int sh = k / P, r = k - sh * P;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = k + j < K ? W[((size_t)sh * P + m) * P + r] : 0.0;
      if (++r == P) { r = 0; ++sh; }
    }
  }
  __device__ void b4(int, int k, int n, int K, double* v) const {
    int sh = k / P, r = k - sh * P;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = (k + j < K && used[sh]) ? X[(size_t)(k + j) * S + n] : 0.0;
      if (++r == P) { r = 0; ++sh; }
    }
  }
};
struct PlainLd {             // C[M x N] = A[M x K] . B[K x N], row-major
  const double* A;
  const double* B;
  double* C;
  int lda, ldb, ldc;
  __device__ void store(int, int m, int n, double v) const { C[(size_t)m * ldc + n] = v; }
  __device__ void a4(int, int m, int k, int K, double* v) const {
    const double* row = A + (size_t)m * lda;
    if (k + 3 < K && !(lda & 1)) {
      const dbl2 x0 = *reinterpret_cast<const dbl2*>(row + k), x1 = *reinterpret_cast<const dbl2*>(row + k + 2);
      v[0] = x0.x;
      v[1] = x0.y;
      v[2] = x1.x;
      v[3] = x1.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = k + j < K ? row[k + j] : 0.0;
    }
  }
  __device__ void b4(int, int k, int n, int K, double* v) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = k + j < K ? B[(size_t)(k + j) * ldb + n] : 0.0;
  }
};

// fp64 MFMA GEMM for the combine's products (v_mfma_f64_16x16x4_f64).  One block = MG_KW waves
// = one 16 x (16 NB) output tile; the waves split K into contiguous runs of 16-deep k-groups, and
// a k-group is 4 MFMAs of k = 4 where lane (r = lane & 15, g = lane >> 4) supplies k = 16 grp +
// 4 g + j to MFMA j: A(m0 + r, k) and B(k, n0 + r), so each lane's A loads are 4 consecutive k of
// one row.  The products are small (K <= a few thousand) and their operands come from L2 or the
// MALL, so the kernel is load-latency bound: a wave issues the loads of CH k-groups at once
// (4 CH (1 + NB) independent loads in flight) before their MFMAs, and 16 waves per block keep the
// chains short (<= 2 chunks at the headline size).  Then every wave parks its tile in LDS and
// the block sums the waves in wave order: each output is a fixed-order sum, independent of the
// launch.  Out-of-range m, n, k read 0.
// Blocks are placed XCD-aware: the (z, tile) work list, z-major and column-tile-major, is cut
// into 8 contiguous ranges and range x runs on XCD x (block id = x + 8 i; dispatch round-robins
// block ids over the 8 XCDs), so a shard's draws (cov_s) or a column slice of theta (sum W theta,
// the final solve) stay in one XCD's L2.
// SYM (square tiles, NB = 1): the tiles of each z are the pairs tm <= tn of a symmetric product
// and each tile is also stored transposed.
constexpr int MG_KW = 16;                         // waves per block (K split)
template <class LD, int NB, int CH, bool SYM>
__global__ __launch_bounds__(64 * MG_KW) void k_mgemm(LD L, int M, int N, int K, int tiles_m, int tiles_n,
                                                      int ntiles, int total, int per_xcd) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int item = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (item >= total) return;                      // block-uniform
  const int z = item / ntiles;
  int t = item - z * ntiles, tm, tn;
  if (SYM) {                                      // t -> (tm, tn), tm <= tn, row by row
    tm = 0;
    while (t >= tiles_m - tm) { t -= tiles_m - tm; ++tm; }
    tn = tm + t;
  } else {                                        // column-tile-major
    tn = t / tiles_m;
    tm = t - tn * tiles_m;
  }
  const int m0 = 16 * tm, n0 = 16 * NB * tn;
  const int ngrp = (K + 15) >> 4;
  const int gb = (ngrp * w) / MG_KW, ge = (ngrp * (w + 1)) / MG_KW;
  const int ma = m0 + r;
  dbl4 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int c0 = gb; c0 < ge; c0 += CH) {
    double a[CH][4], b[CH][NB][4];
#pragma unroll
    for (int h = 0; h < CH; ++h) {
      const int k = 16 * (c0 + h) + 4 * g;
      const bool live = c0 + h < ge;
      if (live && ma < M) {
        L.a4(z, ma, k, K, a[h]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[h][j] = 0.0;
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = n0 + 16 * nb + r;
        if (live && n < N) {
          L.b4(z, k, n, K, b[h][nb]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) b[h][nb][j] = 0.0;
        }
      }
    }
#pragma unroll
    for (int h = 0; h < CH; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[h][j], b[h][nb][j], acc[nb], 0, 0, 0);
  }
  __shared__ dbl4 red[MG_KW][NB][64];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) red[w][nb][lane] = acc[nb];
  __syncthreads();
  // thread t < 256: lane t & 63 of register i = t >> 6, every column tile
  if (threadIdx.x < 256) {
    const int ol = threadIdx.x & 63, i = threadIdx.x >> 6;
    const int m = m0 + (ol >> 4) + 4 * i;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      double v = red[0][nb][ol][i];
#pragma unroll
      for (int ww = 1; ww < MG_KW; ++ww) v += red[ww][nb][ol][i];
      const int n = n0 + 16 * nb + (ol & 15);
      if (m < M && n < N) {
        L.store(z, m, n, v);
        if (SYM && tm != tn) L.store(z, n, m, v);
      }
    }
  }
}

// per (shard, row): mean over S (fixed-order block sum) and a NaN flag
__global__ __launch_bounds__(256) void k_row_stats(const double* X, int S, double* mean, int32_t* rowbad) {
  const int row = blockIdx.x;
  const double* x = X + (size_t)row * S;
  __shared__ double red[256];
  double v = 0.0;
  int bad = 0;
  for (int k = threadIdx.x; k < S; k += 256) {
    const double t = x[k];
    bad |= isnan(t) ? 1 : 0;
    v += t;
  }
  red[threadIdx.x] = v;
  bad = __syncthreads_or(bad);
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    mean[row] = red[0] / (double)S;
    rowbad[row] = bad;
  }
}

// used[s] = no NaN in any of its P rows
__global__ void k_shard_used(const int32_t* rowbad, int P, int nshards, int32_t* used) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nshards) return;
  int bad = 0;
  for (int a = 0; a < P; ++a) bad |= rowbad[(size_t)s * P + a];
  used[s] = bad ? 0 : 1;
}

// Inverse of a batch of SPD P x P matrices (P <= 128): block Gauss-Jordan on 16 x 16 tiles with
// fp64 MFMA, the matrix held in REGISTERS.  One block per matrix, 8 waves; wave w owns tile
// column w of the matrix padded to NT = ceil(P / 16) tiles with an identity block, each tile in
// the MFMA D layout (lane (c, g) register i = T[g + 4i][c]).  The matrix is first equilibrated
// to unit diagonal (A = D^1/2 C D^1/2, inv(A) = D^-1/2 inv(C) D^-1/2), so every scalar pivot,
// a diagonal of a Schur complement, lies in (0, 1].  Panel kb (pivot block K = tile kb):
//   R_J = Dinv T(K, J),  T(K, J) = R_J     owner of column J != kb: 4 MFMAs
//   T(I, J) -= T(I, K) R_J                 4 MFMAs per tile
//   T(I, K) = -T(I, K) Dinv,  T(K, K) = Dinv   owner of column kb
// with Dinv = inv(T(K, K)).  An MFMA contracts 4 k-slots; call s maps slot g to k = g + 4 s, so
// its B operand is register s of a D-layout tile (R_J, T(K, J)) as is, and its A operand is lane
// (r, g) holding A[r][g + 4s].  The column block T(., K) is read in that A layout from LDS.
// Look-ahead: in panel kb the owner of column kb + 1 updates its pivot tile T(kb+1, kb+1) first,
// inverts it (16 x 16, below) while its other tiles' MFMAs are in flight, and publishes the
// updated column (negated, 4 consecutive doubles per lane) together with its Dinv into the other
// half of a double buffer -- so each panel costs ONE barrier (7 at P = 102, against one per
// pivot) and the small inverse sits on one wave's path instead of every wave's.  A symmetric
// matrix is used as its own transpose where the other layout is needed (T(K, K) read in the A
// layout, Dinv as a B operand and as the D-layout T(K, K)): rounding-level differences.
// The 16 x 16 inverse: lane (r, g) holds D[r][g + 4s] (s = 0..3); pivot k takes column k and row
// k with cross-lane shuffles and does the folded rank-1 step a_ij -= c_i r_j (c_k = a_kk - 1,
// r_k = 1 + 1/a_kk, r_j = a_kj / a_kk: Gauss-Jordan with no per-element cases; with pivots <= 1
// the folded terms do not cancel).  Shard b with used[b] == 0 (NaN draws) gets W = 0 and no
// status; status[b] = 1 when a pivot is <= P eps or NaN (a singular covariance; numpy's inv
// raises LinAlgError only on an exactly zero LU pivot and otherwise returns rounding noise).
// Row k of the tile (rk) sits in lane (k, g) of every 16-lane row: a DPP row_newbcast:k move per
// register, no LDS crossbar; the pivot a[k][k] is one lane's, read as a scalar; only column k
// (c, lane (r, k mod 4) of another row) still needs a ds_bpermute -- one per pivot instead of six.
template <int CTRL>
__device__ __forceinline__ double cb_dpp(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int L>
__device__ __forceinline__ double cb_lane(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, L);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), L);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int K>
__device__ __forceinline__ void inv16_pivot(double (&a)[4], int lr, int lg, double pmin, int& sing) {
  constexpr int kg = K & 3, ks = K >> 2;
  const double c = __shfl(a[ks], lr + 16 * kg);          // a[r][k]
  double rk[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) rk[s] = cb_dpp<0x150 + K>(a[s]);   // a[k][g + 4s]
  const double piv = cb_lane<K + 16 * kg>(a[ks]);         // a[k][k], wave-uniform
  if (!(piv > pmin)) sing = 1;
  double ip = __builtin_amdgcn_rcp(piv);
  ip = fma(ip, fma(-piv, ip, 1.0), ip);
  ip = fma(ip, fma(-piv, ip, 1.0), ip);
  const double cc = (lr == K) ? c - 1.0 : c;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const double rj = (lg + 4 * s == K) ? 1.0 + ip : rk[s] * ip;
    a[s] = fma(-cc, rj, a[s]);
  }
}
template <int... K>
__device__ __forceinline__ void inv16_all(double (&a)[4], int lr, int lg, double pmin, int& sing,
                                          std::integer_sequence<int, K...>) {
  (inv16_pivot<K>(a, lr, lg, pmin, sing), ...);
}
__device__ __forceinline__ int inv16(double (&a)[4], int lr, int lg, double pmin) {
  int sing = 0;
  inv16_all(a, lr, lg, pmin, sing, std::make_integer_sequence<int, 16>{});
  return sing;
}

template <int NT>
__global__ __launch_bounds__(512) void k_spd_inverse(const double* Min, double* Out, int P, const int32_t* used,
                                                     int32_t* status) {
  __shared__ __attribute__((aligned(16))) double pub[2][NT + 1][256];  // -T(I, K) then Dinv, A-read order
  __shared__ int32_t psing[2];
  __shared__ double dsc[128];                                           // 1 / sqrt(A_ii)
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const double* M = Min + (size_t)b * P * P;
  double* out = Out + (size_t)b * P * P;
  if (used && !used[b]) {
    for (int i = tid; i < P * P; i += 512) out[i] = 0.0;
    if (tid == 0) status[b] = 0;
    return;
  }
  // pivots of the unit-diagonal matrix lie in (0, 1]; one at the rounding level of the
  // elimination (<= P eps) means a numerically singular covariance (linearly dependent rows),
  // reported as singular.  A full-rank but strongly correlated covariance (1 - R^2 ~ 1e-12,
  // condition number ~1e12) stays above it and is inverted, as numpy's inv does
  const double pmin = P * 2.220446049250313e-16;
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
  const bool own = w < NT;
  const int jc = 16 * w + lr;                     // this lane's matrix column
  dbl4 T[NT];
#pragma unroll
  for (int I = 0; I < NT; ++I)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * I + lg + 4 * i;
      T[I][i] = (row == jc) ? 1.0 : ((own && row < P && jc < P) ? M[(size_t)row * P + jc] * dsc[row] * dsc[jc] : 0.0);
    }
  // slot I < NT: lane (c, g) register i = -T(I)[g + 4i][c] goes to row g + 4i, position
  // (c & 3) * 4 + (c >> 2), so that reader lane (r, g) finds -T(I)[r][g + 4s], s = 0..3, as 4
  // consecutive doubles; slot NT: Dinv, written by lane (r, g) in its own A layout
  auto publish = [&](double* dst, const double (&dinv)[4], int sg) {
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[I * 256 + (lg + 4 * i) * 16 + (lr & 3) * 4 + (lr >> 2)] = -T[I][i];
    dbl2* dp = reinterpret_cast<dbl2*>(dst + NT * 256 + lr * 16 + lg * 4);
    dp[0] = dbl2{dinv[0], dinv[1]};
    dp[1] = dbl2{dinv[2], dinv[3]};
    if (lane == 0) psing[(dst == &pub[0][0][0]) ? 0 : 1] = sg;
  };
  auto rd4 = [&](const double* src, double (&v)[4]) {
    const dbl2* p = reinterpret_cast<const dbl2*>(src + lr * 16 + lg * 4);
    const dbl2 x0 = p[0], x1 = p[1];
    v[0] = x0.x;
    v[1] = x0.y;
    v[2] = x1.x;
    v[3] = x1.y;
  };
  if (w == 0) {
    double d0[4] = {T[0][0], T[0][1], T[0][2], T[0][3]};   // T(0, 0), symmetric: read as A layout
    const int sg = inv16(d0, lr, lg, pmin);
    publish(&pub[0][0][0], d0, sg);
  }
  __syncthreads();
  for (int kb = 0; kb < NT; ++kb) {
    const int cur = kb & 1;
    if (psing[cur]) {
      sing = 1;
      break;                                      // block-uniform
    }
    double a[4];                                  // Dinv(kb), A layout
    rd4(&pub[cur][NT][0], a);
    if (own) {
      if (w == kb) {
#pragma unroll
        for (int I = 0; I < NT; ++I) {
          if (I == kb) {
            T[I] = dbl4{a[0], a[1], a[2], a[3]};
          } else {
            double c[4];
            rd4(&pub[cur][I][0], c);
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(c[s], a[s], acc, 0, 0, 0);
            T[I] = acc;
          }
        }
      } else {
        dbl4 tk = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int I = 0; I < NT; ++I)
          if (I == kb) tk = T[I];
        dbl4 R = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) R = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], tk[s], R, 0, 0, 0);
        if (w == kb + 1) {                        // look-ahead: the next pivot tile first, then its inverse
          double d[4];
#pragma unroll
          for (int I = 0; I < NT; ++I)
            if (I == kb + 1) {
              double c[4];
              rd4(&pub[cur][I][0], c);
#pragma unroll
              for (int s = 0; s < 4; ++s) T[I] = __builtin_amdgcn_mfma_f64_16x16x4f64(c[s], R[s], T[I], 0, 0, 0);
#pragma unroll
              for (int s = 0; s < 4; ++s) d[s] = T[I][s];
            }
          const int sg = inv16(d, lr, lg, pmin);
#pragma unroll
          for (int I = 0; I < NT; ++I) {
            if (I == kb) {
              T[I] = R;
            } else if (I != kb + 1) {
              double c[4];
              rd4(&pub[cur][I][0], c);
#pragma unroll
              for (int s = 0; s < 4; ++s) T[I] = __builtin_amdgcn_mfma_f64_16x16x4f64(c[s], R[s], T[I], 0, 0, 0);
            }
          }
          publish(&pub[cur ^ 1][0][0], d, sg);
        } else {
#pragma unroll
          for (int I = 0; I < NT; ++I) {
            if (I == kb) {
              T[I] = R;
            } else {
              double c[4];
              rd4(&pub[cur][I][0], c);
#pragma unroll
              for (int s = 0; s < 4; ++s) T[I] = __builtin_amdgcn_mfma_f64_16x16x4f64(c[s], R[s], T[I], 0, 0, 0);
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (own && !sing) {
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 16 * I + lg + 4 * i;
        if (row < P && jc < P) out[(size_t)row * P + jc] = T[I][i] * dsc[row] * dsc[jc];
      }
  }
  if (tid == 0) status[b] = sing;
}

// Gauss-Jordan inverse with partial pivoting of a batch of P x P matrices in global memory
// (P > 128).  W holds the [P x 2P] augmented workspace per matrix; status[b] = 1 on a zero
// pivot.  Shards with used[b] == 0 get W = 0.
__global__ __launch_bounds__(1024) void k_gj_inverse(const double* Min, double* W, double* Inv, int P,
                                                     const int32_t* used, int32_t* status) {
  const int b = blockIdx.x;
  const double* M = Min + (size_t)b * P * P;
  double* A = W + (size_t)b * P * 2 * P;
  double* out = Inv + (size_t)b * P * P;
  const int tid = threadIdx.x, nt = blockDim.x, W2 = 2 * P;
  if (used && !used[b]) {
    for (int i = tid; i < P * P; i += nt) out[i] = 0.0;
    if (tid == 0) status[b] = 0;
    return;
  }
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
      if (r == k || c == k) continue;
      A[i] -= A[(size_t)r * W2 + k] * A[(size_t)k * W2 + c];
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

// sum over shards, in shard order (NaN shards hold zeros): dst = sum_s src_s
__global__ void k_sum_w(const double* src, int nshards, size_t n, double* dst) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double v = src[i];
    for (int s = 1; s < nshards; ++s) v += src[(size_t)s * n + i];
    dst[i] = v;
  }
}

template <class LD, int NB, int CH, bool SYM>
static hipError_t mgemm(const LD& L, int M, int N, int K, int batch, hipStream_t st) {
  const int tiles_m = (M + 15) / 16, tiles_n = SYM ? tiles_m : (N + 16 * NB - 1) / (16 * NB);
  const int ntiles = SYM ? tiles_m * (tiles_m + 1) / 2 : tiles_m * tiles_n;
  const int total = ntiles * batch, per_xcd = (total + 7) / 8;
  hipLaunchKernelGGL((k_mgemm<LD, NB, CH, SYM>), dim3(8 * per_xcd), dim3(64 * MG_KW), 0, st, L, M, N, K, tiles_m,
                     tiles_n, ntiles, total, per_xcd);
  return hipGetLastError();
}

}  // namespace stk

using namespace stk;

static bool lds_inverse_fits(int P) { return P <= 128; }

// batched inverse of SPD matrices (workspace only for P > 128)
hipError_t stk_launch_spd_inverse(const double* M, double* Inv, double* work, int P, int batch, const int32_t* used,
                                  int32_t* status, hipStream_t st) {
  if (lds_inverse_fits(P)) {
    const int nt = (P + 15) / 16;
    switch (nt) {
#define STK_INV(N) \
  case N: hipLaunchKernelGGL(k_spd_inverse<N>, dim3(batch), dim3(512), 0, st, M, Inv, P, used, status); break;
      STK_INV(1) STK_INV(2) STK_INV(3) STK_INV(4) STK_INV(5) STK_INV(6) STK_INV(7) STK_INV(8)
#undef STK_INV
    }
  } else {
    hipLaunchKernelGGL(k_gj_inverse, dim3(batch), dim3(1024), 0, st, M, work, Inv, P, used, status);
  }
  return hipGetLastError();
}
size_t stk_spd_inverse_work_bytes(int P, int batch) {
  return lds_inverse_fits(P) ? 0 : sizeof(double) * (size_t)P * 2 * P * batch;
}

// draws X [nshards][P][S] on the device -> W [nshards][P][P], sum_w [P][P], sum_wtheta [P][S].
hipError_t stk_launch_consensus_products(const double* X, int nshards, int P, int S, const int32_t* blk, double* mean,
                                         int32_t* rowbad, int32_t* used, int32_t* status, double* cov, double* W,
                                         double* work, double* sum_w, double* sum_wtheta, hipStream_t st) {
  hipLaunchKernelGGL(k_row_stats, dim3(nshards * P), dim3(256), 0, st, X, S, mean, rowbad);
  hipLaunchKernelGGL(k_shard_used, dim3((nshards + 63) / 64), dim3(64), 0, st, rowbad, P, nshards, used);
  hipError_t e = mgemm<CovLd, 1, 4, true>(CovLd{X, mean, blk, cov, P, S, 1.0 / (double)(S - 1)}, P, P, S, nshards, st);
  if (e != hipSuccess) return e;
  e = stk_launch_spd_inverse(cov, W, work, P, nshards, used, status, st);
  if (e != hipSuccess) return e;
  const size_t pp = (size_t)P * P;
  hipLaunchKernelGGL(k_sum_w, dim3((unsigned)std::min<size_t>((pp + 255) / 256, 1024)), dim3(256), 0, st, W, nshards,
                     pp, sum_w);
  return mgemm<WThetaLd, 2, 2, false>(WThetaLd{W, X, used, sum_wtheta, P, S}, P, S, nshards * P, 1, st);
}

// out [P][S] = inv(sum_w) . sum_wtheta (inv_buf [P][P], work for P > 128)
hipError_t stk_launch_consensus_solve(const double* sum_w, const double* sum_wtheta, int P, int S, double* inv_buf,
                                      double* work, int32_t* status, double* out, hipStream_t st, bool general) {
  // general: a caller's sum W (stk_consensus_solve) need not be symmetric positive definite, so it
  // is inverted as np.linalg.inv does, by partial-pivot elimination (k_gj_inverse: singular only on
  // an exactly zero pivot, as LAPACK getrf); inside stk_consensus sum W is a sum of SPD inverses
  hipError_t e;
  if (general) {
    hipLaunchKernelGGL(k_gj_inverse, dim3(1), dim3(1024), 0, st, sum_w, work, inv_buf, P, nullptr, status);
    e = hipGetLastError();
  } else {
    e = stk_launch_spd_inverse(sum_w, inv_buf, work, P, 1, nullptr, status, st);
  }
  if (e != hipSuccess) return e;
  return mgemm<PlainLd, 2, 2, false>(PlainLd{inv_buf, sum_wtheta, out, P, S, S}, P, S, P, 1, st);
}
size_t stk_general_inverse_work_bytes(int P) { return sizeof(double) * (size_t)P * 2 * P; }
