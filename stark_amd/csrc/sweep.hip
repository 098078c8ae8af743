// Regression log-density + gradient sweeps for gfx950 (the HBM-bound hot kernel).
//
// Replaces the gradient Stan's reverse-mode autodiff computes for every leapfrog inside
// `sm.sampling` (stark/stark.py:48) for the build's regression programs
// (stark_amd/models/logistic.stan, linear.stan; oracle: orc_logreg_lpgrad / orc_linreg_lpgrad).
//
// One pass over a shard's X serves all C chains of the shard: a 256-thread workgroup
// streams a chunk of rows in tiles of T rows (T*d*8 <= 64 KB), staged through LDS with a
// register prefetch of the next tile (global_load_dwordx4 in flight while the current tile
// is computed), and for each tile computes
//   forward   eta[r][c] = alpha_c + x_r . beta_c       (S = 256/T lanes per row, xor-reduce)
//   residual  d eta[r][c] and the lp terms            (Stan's +-20 cutoff for bernoulli_logit)
//   backward  g[j][c]  += sum_r x_r[j] * d eta[r][c]  (lanes over columns, rows split RG ways)
// so X crosses HBM exactly once per leapfrog: algorithmic bytes per sweep = n*(8d + 4)
// (logreg, int32 y) or n*(8d + 8) (linreg).  Each shard is cut into G chunks that depend
// only on (n, d); per-chunk partial sums are reduced in chunk order by k_sweep_reduce, so
// results are bitwise independent of how many shards share a GPU.
#include "sweep_common.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <set>
#include <type_traits>

namespace stk {



template <int FAM, int C, int T, int JPT, int VEC>
__global__ __launch_bounds__(256) void k_sweep(SweepArgs A) {
  constexpr int NT = 256;
  constexpr int S = NT / T;        // lanes per row in the forward pass
  constexpr int NVMAX = (8192 / VEC + NT - 1) / NT;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);   // shards swept
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, LD = A.LD, tid = threadIdx.x;
  const int64_t r0 = sh.n * chunk / A.G, r1 = sh.n * (chunk + 1) / A.G;

  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* Xs = lds;                       // T * LD
  double* Bs = Xs + T * LD;               // C * LD   (beta_c)
  double* Rs = Bs + C * LD;               // T * C    (d eta)
  double* Al = Rs + T * C;                // C        (alpha_c) + C (inv sigma)

  for (int i = tid; i < C * d; i += NT) {
    const int c = i / d, j = i % d;
    Bs[c * LD + j] = A.q[(size_t)(shard * C + c) * A.Dp + 1 + j];
  }
  if (tid < C) {
    const double* qc = A.q + (size_t)(shard * C + tid) * A.Dp;
    Al[tid] = qc[0];
    Al[C + tid] = (FAM == STK_LINREG) ? exp(-qc[d + 1]) : 0.0;
  }

  // per-thread accumulators
  double gacc[JPT][C];
  double lpa[C], ga[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    lpa[c] = 0.0;
    ga[c] = 0.0;
#pragma unroll
    for (int m = 0; m < JPT; ++m) gacc[m][c] = 0.0;
  }
  const int JW = d <= 64 ? 64 : (d <= 128 ? 128 : 256);
  const int RG = NT / JW;
  const int jl = tid % JW, rg = tid / JW;
  const int fr = tid / S, fs = tid % S;   // forward mapping

  // tile staging: VEC doubles per load, element e = VEC*(tid + NT*v) of the tile
  using vec_t = typename std::conditional<VEC == 2, dbl2, double>::type;
  vec_t buf[NVMAX];
  const int64_t ntiles = (r1 - r0 + T - 1) / T;
  auto prefetch = [&](int64_t t) {
    const int64_t row_start = r0 + t * T;
    const int64_t rows = (r1 - row_start) < T ? (r1 - row_start) : T;
    const int64_t nel = rows * d;
    const gptr_t<vec_t> src = (gptr_t<vec_t>)(gp(sh.x) + row_start * d);
#pragma unroll
    for (int v = 0; v < NVMAX; ++v) {
      const int64_t e = (int64_t)VEC * (tid + NT * v);
      if (e < nel) buf[v] = src[tid + NT * v];
    }
  };
  auto stage = [&](int64_t t) {
    const int64_t row_start = r0 + t * T;
    const int64_t rows = (r1 - row_start) < T ? (r1 - row_start) : T;
    const int nel = (int)(rows * d);
    int e = VEC * tid;
    int row = e / d, col = e % d;
    const int step = VEC * NT, dq = step / d, dr = step % d;
#pragma unroll
    for (int v = 0; v < NVMAX; ++v) {
      if (e < nel) {
        if constexpr (VEC == 2) {
          *reinterpret_cast<dbl2*>(&Xs[row * LD + col]) = buf[v];
        } else {
          Xs[row * LD + col] = buf[v];
        }
      }
      e += step;
      row += dq;
      col += dr;
      if (col >= d) { col -= d; ++row; }
    }
  };

  if (ntiles > 0) prefetch(0);
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t row_start = r0 + t * T;
    const int rows = (int)((r1 - row_start) < T ? (r1 - row_start) : T);
    stage(t);
    __syncthreads();
    if (t + 1 < ntiles) prefetch(t + 1);

    // ---- forward + residual
    {
      double acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = 0.0;
      if (fr < rows) {
        const double* xr = Xs + fr * LD;
        for (int j = fs; j < d; j += S) {
          const double x = xr[j];
#pragma unroll
          for (int c = 0; c < C; ++c) acc[c] += x * Bs[c * LD + j];
        }
      }
#pragma unroll
      for (int o = S / 2; o > 0; o >>= 1)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += __shfl_xor(acc[c], o, 64);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if ((c % S) != fs) continue;
        double de = 0.0;
        if (fr < rows) {
          const int64_t row = row_start + fr;
          const double eta = Al[c] + acc[c];
          if constexpr (FAM == STK_LOGREG) {
            const double sgn = 2.0 * gp(sh.yi)[row] - 1.0;
            const double nt = sgn * eta;
            const double e = exp(-nt);
            if (nt > 20.0) { lpa[c] -= e; de = sgn * e; }
            else if (nt < -20.0) { lpa[c] += nt; de = sgn; }
            else { lpa[c] -= log1p(e); de = sgn * e / (e + 1.0); }
          } else {
            const double is = Al[C + c];
            const double z = (gp(sh.y)[row] - eta) * is;
            lpa[c] += z * z;          // linreg: sum of squares, finished in the reduce
            de = z * is;
          }
          ga[c] += de;
        }
        Rs[fr * C + c] = de;
      }
    }
    __syncthreads();

    // ---- backward: g[j][c] += x[r][j] * d eta[r][c]
    for (int r = rg; r < rows; r += RG) {
      const double* xr = Xs + r * LD;
      double rr[C];
#pragma unroll
      for (int c = 0; c < C; ++c) rr[c] = Rs[r * C + c];
#pragma unroll
      for (int m = 0; m < JPT; ++m) {
        const int j = jl + m * JW;
        if (j < d) {
          const double x = xr[j];
#pragma unroll
          for (int c = 0; c < C; ++c) gacc[m][c] += x * rr[c];
        }
      }
    }
    __syncthreads();
  }

  // ---- block reduction in a fixed order, then one partial row per chain
  double* red = lds;   // reuse: RG * C * JW*JPT  and  NT * 2C
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
#pragma unroll
  for (int m = 0; m < JPT; ++m)
#pragma unroll
    for (int c = 0; c < C; ++c) red[((size_t)rg * C + c) * (JW * JPT) + m * JW + jl] = gacc[m][c];
  __syncthreads();
  for (int i = tid; i < C * d; i += NT) {
    const int c = i / d, j = i % d;
    double v = 0.0;
    for (int g = 0; g < RG; ++g) v += red[((size_t)g * C + c) * (JW * JPT) + j];
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    red[(size_t)c * NT + tid] = lpa[c];
    red[(size_t)(C + c) * NT + tid] = ga[c];
  }
  __syncthreads();
  if (tid < 2 * C) {
    const int c = tid % C;
    const bool is_lp = tid < C;
    const double* src = red + (size_t)(is_lp ? c : C + c) * NT;
    double v = 0.0;
    for (int i = 0; i < NT; ++i) v += src[i];
    out[(size_t)c * A.PW + (is_lp ? d + 1 : 0)] = v;
  }
}

// v2 sweep for d <= 128 (T = 64-row tiles, 4 waves):
//   forward   wave w owns columns [w*d/4, (w+1)*d/4), lane = row: eta partials with beta_c[j]
//             as wave-uniform (scalar) operands -- one LDS read per 64 rows per column;
//   residual  64*C (row, chain) pairs over all 256 threads (full lanes for exp/log1p);
//   backward  wave w owns rows [16w, 16w+16), lane = column (JPT = 2), residuals broadcast.
// LDS row stride LD is odd, so lane-per-row reads and lane-per-column reads are both free of
// bank conflicts; tiles are register-prefetched one ahead (global_load_dwordx4).
template <int FAM, int C>
__global__ __launch_bounds__(256, 2) void k_sweep2(SweepArgs A) {
  constexpr int T = 64, NT = 256, JPT = 2;
  constexpr int CP = (T * C + NT - 1) / NT;       // residual pairs per thread
  constexpr int NVMAX = (T * 128 / 2 + NT - 1) / NT;
  using yv_t = typename std::conditional<FAM == STK_LOGREG, int32_t, double>::type;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, LD = A.LD, tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int64_t r0 = sh.n * chunk / A.G, r1 = sh.n * (chunk + 1) / A.G;
  const cptr_t<double> qs = cp(A.q) + (size_t)shard * C * A.Dp;   // chain c: (alpha, beta, [u])
  const gptr_t<double> X = gp(sh.x);
  const gptr_t<yv_t> Y = (gptr_t<yv_t>)(FAM == STK_LOGREG ? (const void*)sh.yi : (const void*)sh.y);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* Xs = lds;                    // T * LD
  double* Part = Xs + T * LD;          // [4][C][T] forward partials
  double* Rs = Part + 4 * C * T;       // [T][C] d eta

  const int jq = (d + 3) / 4;
  const int j0 = min(d, w * jq), j1 = min(d, j0 + jq);
  double alpha[C], inv_s[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    alpha[c] = qs[(size_t)c * A.Dp];
    inv_s[c] = (FAM == STK_LINREG) ? exp(-qs[(size_t)c * A.Dp + d + 1]) : 0.0;
  }

  double gacc[JPT][C];
  double lpa[CP], ga[CP];
#pragma unroll
  for (int i = 0; i < CP; ++i) { lpa[i] = 0.0; ga[i] = 0.0; }
#pragma unroll
  for (int m = 0; m < JPT; ++m)
#pragma unroll
    for (int c = 0; c < C; ++c) gacc[m][c] = 0.0;

  dbl2 buf[NVMAX];
  yv_t yv = 0;                         // y of row (tile start + lane): the only row this thread's residuals use
  const int64_t ntiles = (r1 - r0 + T - 1) / T;
  const int step = 2 * NT, dq = step / d, dr = step % d;
  auto issue = [&](int64_t rs) {       // prefetch X tile + y values starting at row rs
    const int64_t rws = (r1 - rs) < T ? (r1 - rs) : T;
    const int64_t nvec = rws * d / 2;
    const gptr_t<dbl2> src = (gptr_t<dbl2>)(X + rs * d);
#pragma unroll
    for (int v = 0; v < NVMAX; ++v)
      if ((int64_t)(tid + NT * v) < nvec) buf[v] = src[tid + NT * v];
    if (lane < rws) yv = Y[rs + lane];
  };

  if (ntiles > 0) issue(r0);
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t row_start = r0 + t * T;
    const int rows = (int)((r1 - row_start) < T ? (r1 - row_start) : T);
    const yv_t ycur = yv;
    {   // stage the prefetched tile into LDS (2 x ds_write_b64: LD is odd)
      const int nel = rows * d;
      int e = 2 * tid, row = e / d, col = e % d;
#pragma unroll
      for (int v = 0; v < NVMAX; ++v) {
        if (e < nel) {
          double* dst = Xs + row * LD + col;
          dst[0] = buf[v].x;
          dst[1] = buf[v].y;
        }
        e += step;
        row += dq;
        col += dr;
        if (col >= d) { col -= d; ++row; }
      }
    }
    __syncthreads();
    if (t + 1 < ntiles) issue(row_start + T);   // next tile in flight during this tile's compute
    // ---- forward partials: lane = row, wave = column quarter; beta via scalar loads
    {
      double acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = 0.0;
      if (lane < rows) {
        const double* xr = Xs + lane * LD;
#pragma unroll 4
        for (int j = j0; j < j1; ++j) {
          const double x = xr[j];
#pragma unroll
          for (int c = 0; c < C; ++c) acc[c] = fma(x, qs[(size_t)c * A.Dp + 1 + j], acc[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) Part[(w * C + c) * T + lane] = acc[c];
    }
    __syncthreads();
    // ---- residuals: pair p = tid + NT*i -> (row p%64 = lane, chain p/64)
#pragma unroll
    for (int i = 0; i < CP; ++i) {
      const int p = tid + NT * i;
      if (p < T * C) {
        const int r = lane, c = p >> 6;
        double de = 0.0;
        if (r < rows) {
          double a = alpha[0], is = inv_s[0];
#pragma unroll
          for (int cc = 1; cc < C; ++cc)
            if (cc == c) { a = alpha[cc]; is = inv_s[cc]; }
          const double eta = a + (((Part[(0 * C + c) * T + r] + Part[(1 * C + c) * T + r]) +
                                   Part[(2 * C + c) * T + r]) + Part[(3 * C + c) * T + r]);
          if constexpr (FAM == STK_LOGREG) {
            const double sgn = 2.0 * ycur - 1.0;
            const double nt = sgn * eta;
            const double e = exp(-nt);
            if (nt > 20.0) { lpa[i] -= e; de = sgn * e; }
            else if (nt < -20.0) { lpa[i] += nt; de = sgn; }
            else { lpa[i] -= log1p(e); de = sgn * e / (e + 1.0); }
          } else {
            const double z = (ycur - eta) * is;
            lpa[i] += z * z;
            de = z * is;
          }
          ga[i] += de;
        }
        Rs[r * C + c] = de;
      }
    }
    __syncthreads();
    // ---- backward: wave w owns 16 rows, lane = column
    {
      const int rb0 = w * (T / 4), rb1 = min(rows, rb0 + T / 4);
      for (int r = rb0; r < rb1; ++r) {
        double rv[C];
#pragma unroll
        for (int c = 0; c < C; ++c) rv[c] = Rs[r * C + c];
        const double* xr = Xs + r * LD;
#pragma unroll
        for (int m = 0; m < JPT; ++m) {
          const int j = lane + 64 * m;
          if (j < d) {
            const double x = xr[j];
#pragma unroll
            for (int c = 0; c < C; ++c) gacc[m][c] = fma(x, rv[c], gacc[m][c]);
          }
        }
      }
    }
    __syncthreads();
  }

  // ---- fixed-order block reduction -> one partial row per chain
  double* red = lds;
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
#pragma unroll
  for (int m = 0; m < JPT; ++m)
#pragma unroll
    for (int c = 0; c < C; ++c) red[((w * C + c) * JPT + m) * 64 + lane] = gacc[m][c];
  __syncthreads();
  for (int i = tid; i < C * d; i += NT) {
    const int c = i / d, j = i % d, m = j >> 6, l = j & 63;
    const double v = ((red[((0 * C + c) * JPT + m) * 64 + l] + red[((1 * C + c) * JPT + m) * 64 + l]) +
                      red[((2 * C + c) * JPT + m) * 64 + l]) + red[((3 * C + c) * JPT + m) * 64 + l];
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CP; ++i) {
    red[(size_t)(2 * i) * NT + tid] = lpa[i];
    red[(size_t)(2 * i + 1) * NT + tid] = ga[i];
  }
  __syncthreads();
  if (tid < 2 * C) {          // chain c's pairs: slot i = (c*64)/NT, threads (c*64)%NT .. +63
    const int c = tid >> 1, kind = tid & 1;
    const int i = (c * 64) / NT, t0 = (c * 64) % NT;
    const double* src = red + (size_t)(2 * i + kind) * NT + t0;
    double v = 0.0;
    for (int k = 0; k < 64; ++k) v += src[k];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

// v3 sweep (even d <= 104, C <= 4): wave-private LDS-DMA rings, no barrier in the main loop.
//
// v2 holds one tile ahead in registers per block; with two blocks per CU that leaves too few
// bytes in flight (tools/sweep_micro.hip: the v2 pipeline without arithmetic reaches only
// 3.7-4.5 TB/s against 6.1 TB/s for a plain streaming read).  Here one 512-thread block per
// CU streams a chunk of 64-row tiles; wave w owns rows [8w, 8w+8) of every tile and moves
// them itself: `buffer_load_dwordx4 ... lds` (1 KiB per wave-instruction, no VGPR staging,
// no ds_write pass) into a private ring of NB 8-row slots, so while it computes sub-tile t
// its sub-tiles t+1 .. t+NB-1 are in flight (8 waves x 2 x 6.4 KB at d = 100) and it never
// waits for another wave: counted vmcnt on its own DMAs only, no s_barrier until the final
// reduction (a block-wide barrier per tile put all waves in lockstep and exposed the whole
// forward -> residual -> backward latency chain every tile).  Per sub-tile:
//   forward   8 lanes per row, lane i reads 16-B pieces i, i+8, ... of its row (ds_read_b128)
//             and keeps its beta pieces in registers for the whole launch; 3 xor steps sum
//             the row;
//   residual  lane i < C of each row group finishes chain i (Stan's bernoulli_logit cutoffs /
//             normal residual), d eta -> a per-wave LDS scratch;
//   backward  lane k = piece k (2 columns), 8 rows, d eta read as broadcasts.
// Chunks are whole tiles ([64*t0, 64*t1) rows, a function of (n, d) only) and all sums run in
// a fixed order, so the result is bitwise independent of shard placement, as for v1/v2.


constexpr int S3_T = 64;          // rows per tile
constexpr int S3_W = 8;           // waves per block
constexpr int S3_MAXP = 7;        // pieces per lane in the forward: K <= 56
constexpr int S3_KMAX = 52;       // pieces per row (d/2) handled by v3


// DPP lane exchange of a double (full-rate VALU, no LDS round trip like ds_bpermute); bound_ctrl
// zero-fills as old = 0 would, without a v_mov of the old value before each move.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Sum over each group of 8 consecutive lanes; every lane of the group gets the total:
// xor 1, xor 2 (quad_perm), then row_half_mirror (lane i <-> 7 - i) joins the two quads.
__device__ __forceinline__ double sum8(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  return v + dpp_d<0x141>(v);
}

// -log1p(exp(-x)) and its derivative weight exp(-x)/(1+exp(-x)) for |x| <= 20 (Stan's
// bernoulli_logit middle branch) with one exp, one log and one reciprocal: with u = 1 + e,
// log1p(e) = log(u) - ((u - 1) - e)/u (the rounding of u corrected to first order), and
// e/(1+e) = e * (1/u); 1/u by v_rcp_f64 + two Newton steps.
__device__ __forceinline__ void softplus_terms(double x, double* lp_term, double* w) {
  const double e = exp(-x);
  const double u = 1.0 + e;
  double r = __builtin_amdgcn_rcp(u);
  r = fma(r, fma(-u, r, 1.0), r);
  r = fma(r, fma(-u, r, 1.0), r);
  *lp_term = log(u) - ((u - 1.0) - e) * r;
  *w = e * r;
}

// One wave's ring slot: 8 rows of X (8 * 16 * K bytes) + 8 rows of y (<= 64 B), 16-B aligned.
__host__ __device__ constexpr int sweep3_slot_bytes(int K) { return 8 * 16 * K + 64; }


// ABL (micro-benchmark ablations only, tools/sweep_micro.hip; 0 in the product): bit 0 replaces
// the residual's transcendentals by a linear stand-in, bit 1 skips the backward, bit 2 the forward.
// KS, NBS: compile-time K (= d/2) and ring depth for the BASELINE shapes (d = 100, 50), so
// the DMA issue unrolls and the steady-state wait is one immediate; 0 = runtime (any d).
template <int FAM, int C, int ABL = 0, int KS = 0, int NBS = 0>
__global__ __launch_bounds__(512) void k_sweep3(SweepArgs A, int NBrt) {
  constexpr int T = S3_T, NW = S3_W;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, K = KS ? KS : (d >> 1), NB = NBS ? NBS : NBrt;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int64_t nt = (sh.n + T - 1) / T;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * T, r1 = std::min<int64_t>(sh.n, t1 * T);
  const int ntiles = (int)(t1 - t0);
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;   // y bytes per row
  const int SB = 8 * 16 * K;                        // X bytes of one wave's 8-row sub-tile
  const int SS = sweep3_slot_bytes(K);              // slot: X [0, SB), y [SB, SB + 8*YB)

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const ring = reinterpret_cast<char*>(lds) + (size_t)w * NB * SS;   // this wave's NB slots
  double* const dsc = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * NB * SS);  // [NW][8][C]

  // ---- per-lane constants: beta pieces (forward) and alpha / 1/sigma (residual)
  const double* qs = A.q + (size_t)shard * C * A.Dp;
  const int fi = lane & 7, frow = w * 8 + (lane >> 3);   // forward: lane-in-row, row in tile
  double bt[S3_MAXP][C][2];
#pragma unroll
  for (int m = 0; m < S3_MAXP; ++m) {
    const int k = fi + 8 * m;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      bt[m][c][0] = k < K ? qs[(size_t)c * A.Dp + 1 + 2 * k] : 0.0;
      bt[m][c][1] = k < K ? qs[(size_t)c * A.Dp + 2 + 2 * k] : 0.0;
    }
  }
  const int rc = fi < C ? fi : 0;                        // residual chain of this lane
  const double alpha = qs[(size_t)rc * A.Dp];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qs[(size_t)rc * A.Dp + d + 1]) : 0.0;
  __builtin_amdgcn_s_waitcnt(0xF70);                      // ordinary loads retired before the DMAs start

  // ---- DMA issue: sub-tile t of this wave = rows [64 t + 8 w, 64 t + 8 w + 8) of the chunk:
  // nx 1-KiB X pieces (the last one partial) + one size-4 piece for y; buffer descriptors cover
  // exactly the chunk, so a partial last tile reads zeros past its end instead of faulting.
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (r1 - r0) * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (r1 - r0) * YB);
  const int nx = (SB + 1023) >> 10;
  const int last_lanes = (SB - ((nx - 1) << 10)) >> 4;
  const int per_tile = nx + 1;                            // DMAs this wave issues per sub-tile
  auto issue = [&](int t) {
    char* sl = ring + (size_t)(t % NB) * SS;
    const int xoff = (t * 64 + w * 8) * 16 * K;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + j * 1024), 16, lane * 16, xoff + j * 1024, 0, 0);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, 0);
    if (lane < 2 * YB)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(sl + SB), 4, lane * 4, (t * 64 + w * 8) * YB, 0, 0);
  };

  double gacc[C][2];
  double lpa = 0.0, gaa = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) gacc[c][0] = gacc[c][1] = 0.0;

  for (int t = 0; t < NB - 1 && t < ntiles; ++t) issue(t);
  for (int t = 0; t < ntiles; ++t) {
    // own DMAs of sub-tile t retired; later sub-tiles (issued already) stay in flight
    const int later = std::min(NB - 2, ntiles - 1 - t);
    if constexpr (KS > 0) {
      constexpr int PT = ((8 * 16 * KS + 1023) >> 10) + 1;
      if (later == NBS - 2) wait_vm<(NBS - 2) * PT>();
      else wait_vmcnt(later * PT);
    } else {
      wait_vmcnt(later * per_tile);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): reads of slot t-1 are done
    __builtin_amdgcn_sched_barrier(0);
    if (t + NB - 1 < ntiles) issue(t + NB - 1);          // into slot (t-1) % NB
    const char* xs = ring + (size_t)(t % NB) * SS - (size_t)w * 8 * 16 * K;   // row r of the tile at r*16K
    const char* ys = xs + (size_t)w * 8 * 16 * K + SB - (size_t)w * 8 * YB;   // y of row r at r*YB
    const int rows = (int)std::min<int64_t>(T, r1 - r0 - (int64_t)t * T);

    // ---- forward: eta partial of row frow over this lane's pieces, then the row sum
    double acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.0;
#pragma unroll
    for (int m = 0; m < ((ABL & 4) ? 0 : S3_MAXP); ++m) {
      const int k = std::min(fi + 8 * m, K - 1);
      const dbl2 x = *reinterpret_cast<const dbl2*>(xs + ((size_t)frow * K + k) * 16);
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = fma(x.y, bt[m][c][1], fma(x.x, bt[m][c][0], acc[c]));
    }
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = sum8(acc[c]);

    // ---- residual: lane fi < C finishes chain fi of row frow
    if (fi < C) {
      double eta = acc[0];
#pragma unroll
      for (int c = 1; c < C; ++c)
        if (fi == c) eta = acc[c];
      eta += alpha;
      double de = 0.0;
      if (frow < rows) {
        if constexpr (ABL & 1) {
          const int32_t yv = *reinterpret_cast<const int32_t*>(ys + frow * 4);
          de = (2.0 * yv - 1.0) - 0.25 * eta;
          lpa -= de * de;
        } else if constexpr (FAM == STK_LOGREG) {
          const int32_t yv = *reinterpret_cast<const int32_t*>(ys + frow * 4);
          const double sgn = 2.0 * yv - 1.0;
          const double ntt = sgn * eta;
          if (ntt > 20.0) { const double e = exp(-ntt); lpa -= e; de = sgn * e; }
          else if (ntt < -20.0) { lpa += ntt; de = sgn; }
          else { double lt, wt; softplus_terms(ntt, &lt, &wt); lpa -= lt; de = sgn * wt; }
        } else {
          const double yv = *reinterpret_cast<const double*>(ys + frow * 8);
          const double z = (yv - eta) * inv_s;
          lpa += z * z;
          de = z * inv_s;
        }
        gaa += de;
      }
      dsc[(w * 8 + (lane >> 3)) * C + fi] = de;
    }

    // ---- backward: lane = piece k (columns 2k, 2k+1), the wave's 8 rows
    {
      const int k = std::min(lane, K - 1);
      const int nr = (ABL & 2) ? 0 : std::min(8, rows - w * 8);
      auto row = [&](int rr) {
        const dbl2 x = *reinterpret_cast<const dbl2*>(xs + ((size_t)(w * 8 + rr) * K + k) * 16);
        const double* dr = dsc + (w * 8 + rr) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const double dv = dr[c];
          gacc[c][0] = fma(x.x, dv, gacc[c][0]);
          gacc[c][1] = fma(x.y, dv, gacc[c][1]);
        }
      };
      if (nr == 8) {            // full sub-tile: branch-free, the compiler pipelines the reads
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) row(rr);
      } else {
        for (int rr = 0; rr < nr; ++rr) row(rr);
      }
    }
  }

  // ---- fixed-order block reduction -> one partial row per chain
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;                                    // [NW][C][64][2] then [NW][64][2]
  if (lane < K) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      red[((size_t)(w * C + c) * 64 + lane) * 2 + 0] = gacc[c][0];
      red[((size_t)(w * C + c) * 64 + lane) * 2 + 1] = gacc[c][1];
    }
  }
  double* red2 = red + (size_t)NW * C * 128;
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  for (int i = tid; i < C * d; i += NW * 64) {
    const int c = i / d, j = i % d, k = j >> 1, h = j & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww) v += red[((size_t)(ww * C + c) * 64 + k) * 2 + h];
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {          // chain c: lanes with lane % 8 == c of every wave, in (wave, lane) order
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int g = 0; g < 8; ++g) v += red2[(size_t)(ww * 64 + g * 8 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}


// v5 sweep: 64 chains of a shard, any d -- two fp64 MFMA GEMM passes (BASELINE configs[4]:
// full-data logistic regression, d = 1000, 64 chains).
//
// At d*C = 64000 neither beta (B operand, d x 64) nor the gradient accumulators fit a
// workgroup's registers, so the sweep is split at the residual:
//   pass F  eta = X . [beta_1 .. beta_64] (M = rows, N = chains, K = d), + alpha, residual
//           on the fly: d eta -> R (HBM, 512 B per row), lp and sum(d eta) per chain;
//   pass B  G = X^T . R (M = d, N = chains, K = rows) per (row chunk, column block).
// X crosses HBM twice per leapfrog (8d B per row each pass) plus R (1 KB per row), against
// 4*d*64 flop per row: 15 flop/B at d = 1000, above the fp64 balance point, so both passes
// are fp64-MFMA bound.  Both are LDS-staged GEMMs of 4 waves, two blocks
// per CU, over rings of stages moved by `buffer_load_dwordx4 ... lds`; a wave holds 2 (pass F)
// or 4 (pass B) 16-row tiles x all four 16-chain tiles, so a k-step is 2 or 4 A fragment reads
// + four B fragment reads + 8 or 16 independent v_mfma_f64_16x16x4_f64.  LDS images are
// XOR-swizzled in 16-B pieces so every fragment read is bank-conflict free: X by per-lane DMA
// source offsets, beta^T and R by their writers (k_qt_swizzle, pass F's epilogue).
constexpr int G5_C = 64;      // chains (4 MFMA N tiles)
constexpr int G5_KC = 32;     // beta^T image rows: d rounded up to this
constexpr int G5_TR = 64;     // chunk granularity in rows (R's rows: n rounded up to this)

__host__ __device__ inline int g5_kp(int d) { return (d + G5_KC - 1) / G5_KC * G5_KC; }
// byte offset of element (row r, chain c) in a 512-B-row chain image (beta^T rows k, R rows r)
__device__ __forceinline__ int g5_chain_off(int r, int c) { return r * 512 + ((((c >> 1) ^ ((r & 1) << 3))) << 4) + ((c & 1) << 3); }

// beta^T images for pass F: qT[shard][k][.] = beta_c[k] (0 for k >= d), swizzled as g5_chain_off.
__global__ __launch_bounds__(256) void k_qt_swizzle(SweepArgs A, int d) {
  const int shard = A.shard0 + blockIdx.y;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  const int KP = g5_kp(d);
  const int i = blockIdx.x * 256 + threadIdx.x;     // k * 64 + c
  if (i >= KP * G5_C) return;
  const int k = i >> 6, c = i & 63;
  const double v = k < d ? A.q[((size_t)shard * G5_C + c) * A.Dp + 1 + k] : 0.0;
  char* img = reinterpret_cast<char*>(A.qT + (size_t)shard * KP * G5_C);
  *reinterpret_cast<double*>(img + g5_chain_off(k, c)) = v;
}

// A barrier that leaves LDS-DMAs in flight: __syncthreads() makes hipcc drain vmcnt(0) first
// (an LDS-DMA is a pending LDS write on the VM counter), which would empty the stage ring at
// every stage; the counted wait before it is what orders the DMA'd data.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);                   // lgkmcnt(0): this wave's LDS accesses done
  __builtin_amdgcn_s_barrier();
}
// Pass F geometry: tiles of G5_FTR = 32 G5_FW rows, G5_FW waves of 32 rows (2 MFMA row tiles) x
// all 4 chain tiles each (8 accumulators, 64 VGPRs), 16-column stages in a 3-deep ring.
constexpr int G5_FW = 4;      // pass F: waves per block (two blocks per CU share its 160 KB of LDS)
constexpr int G5_FS = 3;      // pass F: stages in the ring
constexpr int G5_FKC = 16;    // pass F: columns per stage
constexpr int G5_FTR = 32 * G5_FW;   // pass F: rows per tile
__host__ __device__ constexpr int g5_fstage_bytes() { return G5_FTR * G5_FKC * 8 + G5_FKC * 512; }   // [X][beta^T]

// The DMA goes through a plain function: clang's host pass drops a kernel template's stub when the
// builtin's operands depend on a template parameter (undefined symbol at link, no diagnostic).
__device__ __forceinline__ void dma16_lds(__amdgpu_buffer_rsrc_t r, char* dst, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)dst, 16, voff, soff, 0, 0);
}

// Pass F: one block per (shard, chunk); the chunk's 128-row tiles one after another.  A stage
// is 16 columns of the tile's X (16 KB) and of beta^T (8 KB), so one beta^T stage feeds 128 rows
// (LDS-DMA volume 1.5 x the X bytes; round 4's 64-row tiles: 2 x).  Two blocks per CU (72 KB of
// LDS each with the exp table) overlap one block's epilogue with the other's MFMAs.  The 64
// accumulators per lane leave no room for the whole tile's epilogue at once, so it is
// pipelined: the finished tile's eta is parked, and its 8 (row tile, chain tile) parts of 4
// elements are done during the next tile.  SPLIT = 1 (the product for d > 112, NKC >= 8): the
// next tile's first 8 stages are unrolled, each carrying one part as a compile-time constant,
// then a plain loop over the rest -- no per-stage part dispatch, which cost 3-5 % (DESIGN.md
// section 3); SPLIT = 0: the parts p with p % NKC == kc at stage kc (the rest at the chunk's end).
// Waits: the LDS-DMA loads and the tile's y loads complete in issue order, so "at most the next
// stage's DMA outstanding" proves the current stage landed whatever the R stores in between do
// (a store still in flight only makes the count larger).  DESIGN.md section 3.
// (Template geometry for tools/gemm_fwd_ab.py's A/B arms: NW waves of RT 16-row tiles, KCF-column
// stages, an NS-deep ring; the product launches the defaults with SPLIT 0 or 1.)
template <int FAM, int NW = G5_FW, int RT = 2, int KCF = G5_FKC, int NS = G5_FS, int SPLIT = 0>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd(SweepArgs A) {
  constexpr int NCT = 4, TR = 16 * RT * NW;
  constexpr int XB = TR * KCF * 8, BB = KCF * 512, STG = XB + BB;
  constexpr int PPR = KCF / 2;                          // 16-B pieces per X row in the stage (8)
  constexpr int NDX = XB / 1024 / NW, NDB = BB / 1024 / NW, NPART = RT * NCT;
  constexpr int FLUSH = 64 / RT;                        // tiles per log1p flush: 256 elements per lane and chain tile
  static_assert(NDX >= 1 && NDB >= 1 && XB % (1024 * NW) == 0 && BB % (1024 * NW) == 0 && (PPR == 8 || PPR == 16),
                "pass F stage geometry");
  // X piece swizzle: 128-B rows put rows of one parity on one half of the banks, so XOR the
  // piece with (row >> 1) & 7; 256-B rows XOR it with row & 15 (every A fragment read conflict free)
  auto swz = [](int row) { return PPR == 16 ? (row & 15) : ((row >> 1) & 7); };
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, KP = (d + KCF - 1) / KCF * KCF, NKC = KP / KCF;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  // chunks are whole 64-row tiles of the shard (R's geometry, pass B's too); the last 128-row
  // tile of a chunk may cover 64 rows past it: X reads there are 0 (descriptor bound), R stores skipped
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
  const int nrows = (int)(r1 - r0);
  const int rcap = (int)((t1 - t0) * G5_TR);
  const int ntile = (rcap + TR - 1) / TR;

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const stg = reinterpret_cast<char*>(lds);      // NS stages of STG bytes
  double* const sptab = reinterpret_cast<double*>(stg + NS * STG);
  if constexpr (FAM == STK_LOGREG) exp_table_init(sptab);
  // per-lane chain constants: chain 16 c2 + lr
  const double* qb = A.q + (size_t)shard * G5_C * A.Dp;
  double alpha[NCT], inv_s[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) {
    alpha[c2] = qb[(size_t)(16 * c2 + lr) * A.Dp];
    inv_s[c2] = (FAM == STK_LINREG) ? exp(-qb[(size_t)(16 * c2 + lr) * A.Dp + d + 1]) : 0.0;
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const int KPI = g5_kp(d);                             // beta^T image rows (>= KP, zero past d)
  const __amdgpu_buffer_rsrc_t br = uniform_rsrc(A.qT + (size_t)shard * KPI * G5_C, (int64_t)KPI * G5_C * 8);
  // X stage: slot s (16 B) = row s / PPR, piece (s % PPR) ^ swz(row) of the stage's KCF columns
  int xvo[NDX];
#pragma unroll
  for (int i = 0; i < NDX; ++i) {
    const int sl = (w * NDX + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ swz(row);
    xvo[i] = row * d * 8 + pc * 16;
  }
  auto issue = [&](int st) {                            // global stage index st = tile * NKC + kc
    const int tile = st / NKC, kc = st % NKC;
    char* b = stg + (st % NS) * STG;
    const int xso = tile * TR * d * 8 + kc * KCF * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i) dma16_lds(xr, b + (w * NDX + i) * 1024, xvo[i], xso);
#pragma unroll
    for (int i = 0; i < NDB; ++i) dma16_lds(br, b + XB + (w * NDB + i) * 1024, lane * 16, kc * KCF * 512 + (w * NDB + i) * 1024);
  };
  // per chain tile: logistic lm = sum(t - |t|) - 2 sum(flushed log1p(sp)), sp = prod(1 + e) - 1
  // (residual v4, sweep_common.h); linear: lm = sum z^2
  double lm[NCT], sp[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  dbl4 acc[RT][NCT];
  double pend[RT][NCT][4];                              // the parked tile's eta
  uint32_t ybit = 0u, pybit = 0u;                       // logistic y of this lane's 8 rows of the tile, one bit each
  double yt[RT][4] = {}, pyt[RT][4] = {};               // linear y
  int ptile = -1;
  auto epi = [&](const int p) {                         // part p = (row tile p / NCT, chain tile p % NCT);
    const int rt = p / NCT, c2 = p % NCT;                // called from unrolled loops: p is a constant
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int grow = ptile * TR + 16 * RT * w + 16 * rt + lh + 4 * i;   // row of the chunk
      const bool valid = grow < nrows;
      const double eta = pend[rt][c2][i];
      double dv;
      if constexpr (FAM == STK_LOGREG) {
        double lm2 = lm[c2], sp2 = sp[c2];
        dv = -logit_resid4(eta, (pybit >> (4 * rt + i)) & 1u, sptab, lm2, sp2);
        lm[c2] = valid ? lm2 : lm[c2];
        sp[c2] = valid ? sp2 : sp[c2];
      } else {
        const double z = (pyt[rt][i] - eta) * inv_s[c2];
        lm[c2] += valid ? z * z : 0.0;
        dv = z * inv_s[c2];
      }
      dv = valid ? dv : 0.0;
      gaa[c2] += dv;
      if (grow < rcap) *reinterpret_cast<double*>(Rimg + g5_chain_off(grow, 16 * c2 + lr)) = dv;
    }
    if (FAM == STK_LOGREG && rt == RT - 1 && (ptile % FLUSH) == FLUSH - 1) {   // FLUSH tiles x 4 RT elements per lane
      lm[c2] -= 2.0 * log1p(sp[c2]);
      sp[c2] = 0.0;
    }
  };
  // One stage: wait for its DMA, barrier, the parked tile's epilogue part(s) due, the tile's y,
  // the DMA NS - 1 stages ahead, the stage's MFMAs.  part >= 0: that part; -1: none; -2: the
  // parts p with p % NKC == kc (NKC < NPART); yload: read the tile's y.  Inlined at every call
  // site with first / part / yload constant where they can be: straight-line steady-state stages.
  auto stage = [&](const int st, const int kc, const bool first, const int part, const bool yload) {
    if (first) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int c2 = 0; c2 < NCT; ++c2) acc[rt][c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDB));   // own DMAs of stage st retired
    lds_barrier();                                       // stage st landed for every wave; slot of st-1 free
    if (part >= 0 && ptile >= 0) epi(part);
    if (part == -2 && ptile >= 0) {
#pragma unroll
      for (int p = 0; p < NPART; ++p)
        if (p % NKC == kc) epi(p);
    }
    if (yload) {                                         // this tile's y (loads: in order with the DMA)
      if constexpr (FAM == STK_LOGREG) ybit = 0u;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t grow = (int64_t)(st / NKC) * TR + 16 * RT * w + 16 * rt + lh + 4 * i;
          if constexpr (FAM == STK_LOGREG) ybit |= (grow < nrows ? (uint32_t)sh.yi[r0 + grow] & 1u : 0u) << (4 * rt + i);
          else yt[rt][i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
        }
    }
    if (st + NS - 1 < nst) issue(st + NS - 1);
    const char* b = stg + (st % NS) * STG;
#pragma unroll
    for (int step = 0; step < KCF / 4; ++step) {
      const int kk = 4 * step + lh;
      double a[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = 16 * RT * w + 16 * rt + lr;
        a[rt] = *reinterpret_cast<const double*>(b + r * (16 * PPR) + (((kk >> 1) ^ swz(r)) << 4) + ((kk & 1) << 3));
      }
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const double bb = *reinterpret_cast<const double*>(b + XB + g5_chain_off(kk, 16 * c2 + lr));
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][c2] = mfma_f64(a[rt], bb, acc[rt][c2]);
      }
    }
  };
  auto park = [&](const int tile) {   // the tile's epilogue runs during the next
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2)
#pragma unroll
        for (int i = 0; i < 4; ++i) pend[rt][c2][i] = acc[rt][c2][i] + alpha[c2];
#pragma unroll
      for (int i = 0; i < 4; ++i) pyt[rt][i] = yt[rt][i];
    }
    pybit = ybit;
    ptile = tile;
  };
  if constexpr (SPLIT == 1) {
    // (NKC >= NPART: the host's choice) tile by tile, the first NPART stages of a tile each carry
    // one part of the parked tile (p a constant: no per-stage part dispatch), the rest none
    for (int tile = 0, st = 0; tile < ntile; ++tile, st += NKC) {
#pragma unroll
      for (int p = 0; p < NPART; ++p) stage(st + p, p, p == 0, p, p == NPART - 1);   // y after the last part: pend dead
      for (int kc = NPART; kc < NKC; ++kc) stage(st + kc, kc, false, -1, false);
      park(tile);
    }
  } else {
    for (int st = 0; st < nst; ++st) {
      const int kc = st % NKC;
      stage(st, kc, kc == 0, -2, kc == 0);
      if (kc == NKC - 1) park(st / NKC);
    }
  }
  if (ptile >= 0) {                                      // the last tile, and any parts NKC < 8 stages left over
#pragma unroll
    for (int p = 0; p < NPART; ++p) epi(p);
  }
  double lpa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lpa[c2] = (FAM == STK_LOGREG) ? 0.5 * lm[c2] - log1p(sp[c2]) : lm[c2];

  // ---- lp and sum(d eta) per chain: lanes lr of the 4 row groups h of the NW waves, fixed order
  __builtin_amdgcn_s_waitcnt(0xF70);
  __syncthreads();
  double* red = lds;                                     // [NW waves][64 lanes][NCT][2]
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) {
    red[((w * 64 + lane) * NCT + c2) * 2 + 0] = lpa[c2];
    red[((w * 64 + lane) * NCT + c2) * 2 + 1] = gaa[c2];
  }
  __syncthreads();
  if (tid < 2 * G5_C) {
    const int c = tid >> 1, kind = tid & 1, c2 = c >> 4, l = c & 15;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red[((ww * 64 + h * 16 + l) * NCT + c2) * 2 + kind];
    A.partial[(((size_t)shard * A.Gs + chunk) * G5_C + c) * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

// Pass B: one block per (shard, chunk, JB-column block); G[j][c] += X[r][j] R[r][c] over the
// chunk's rows, straight into the chunk's partial row (columns 1 .. d).  4 waves, two blocks per
// CU: wave w takes CTW = JB / 64 column tiles (16 columns each) x all 4 chain tiles (CTW A reads
// + 4 B reads per 4 CTW MFMAs, 16 CTW accumulators), stages of 8 rows in a 3-deep ring.
// JB = 256 (d > 128) re-reads each chunk's R from L2 once per column block: 4 x at d = 1000
// (round 4's 128-column blocks: 8 x).  Every output sums its chunk's rows in row order.
constexpr int G5_BRB = 8;     // pass B: rows per stage
constexpr int G5_BW = 4;      // pass B: waves per block
constexpr int G5_BNS = 3;     // pass B: stages in the ring
__host__ __device__ constexpr int g5_bstage_bytes(int jb) { return G5_BRB * jb * 8 + G5_BRB * 512; }
__host__ __device__ inline int g5_bjb(int d) { return d <= 64 ? 64 : d <= 128 ? 128 : 256; }
template <int JB>
__global__ __launch_bounds__(64 * G5_BW, 2) void k_gemm_bwd(SweepArgs A, int njb) {
  constexpr int NW = G5_BW, RB = G5_BRB, NS = G5_BNS;
  constexpr int CTW = JB / 16 / NW, NCT = 4, PPR = JB / 2;
  constexpr int XB = RB * JB * 8, RBB = RB * 512, STG = XB + RBB;
  constexpr int NDX = XB / 1024 / NW, NDR = RBB / 1024 / NW;   // DMA instructions per wave
  static_assert(CTW >= 1 && NDX >= 1 && NDR >= 1 && XB % (1024 * NW) == 0 && RBB % (1024 * NW) == 0 &&
                STG == g5_bstage_bytes(JB), "pass B stage geometry");
  // XCD-aware order: blocks are dealt to the 8 XCDs round-robin (blockIdx % 8), so the njb
  // column blocks of a chunk get blockIdx values of one residue -- one XCD, whose L2 then
  // serves the chunk's R rows to all of them (else each XCD re-reads R from HBM)
  const int nsc = gridDim.x / njb;
  int sc, jb;
  if ((nsc & 7) == 0) {
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    sc = x + 8 * (k / njb);
    jb = k % njb;
  } else {
    jb = blockIdx.x % njb;
    sc = blockIdx.x / njb;
  }
  const int shard = A.shard0 + sc / A.G;
  const int chunk = sc % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
  const int nrows = (int)(r1 - r0);
  const int nst = (nrows + RB - 1) / RB;
  const int j0 = jb * JB;

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const stg = reinterpret_cast<char*>(lds);      // NS stages: [X block XB][R block RBB]
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(A.R + ((size_t)shard * A.Rrows + r0) * G5_C, (int64_t)nrows * G5_C * 8);
  // X stage: slot s = row s / PPR, piece (s % PPR) ^ ((row & 1) << 3) of the block's JB columns
  // (rows 4s + lh of one lane group then sit on opposite halves of the banks)
  int xvo[NDX];
#pragma unroll
  for (int i = 0; i < NDX; ++i) {
    const int sl = (w * NDX + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ ((row & 1) << 3);
    xvo[i] = row * d * 8 + (j0 + 2 * pc) * 8;
  }
  auto issue = [&](int st) {
    char* b = stg + (st % NS) * STG;
    const int xso = st * RB * d * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i) dma16_lds(xr, b + (w * NDX + i) * 1024, xvo[i], xso);
#pragma unroll
    for (int i = 0; i < NDR; ++i) dma16_lds(rr, b + XB + (w * NDR + i) * 1024, lane * 16, st * RB * 512 + (w * NDR + i) * 1024);
  };
  dbl4 acc[CTW][NCT];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int c2 = 0; c2 < NCT; ++c2) acc[ct][c2] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  for (int st = 0; st < nst; ++st) {
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDR));
    lds_barrier();
    if (st + NS - 1 < nst) issue(st + NS - 1);
    const char* b = stg + (st % NS) * STG;
#pragma unroll
    for (int step = 0; step < RB / 4; ++step) {
      const int r = 4 * step + lh;
      double a[CTW];
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        const int jl = 16 * (w * CTW + ct) + lr;       // A row (column of X) of this lane
        a[ct] = *reinterpret_cast<const double*>(b + r * (16 * PPR) + ((((jl >> 1) ^ ((r & 1) << 3))) << 4) + ((jl & 1) << 3));
      }
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const double bb = *reinterpret_cast<const double*>(b + XB + g5_chain_off(r, 16 * c2 + lr));
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) acc[ct][c2] = mfma_f64(a[ct], bb, acc[ct][c2]);
      }
    }
  }
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * G5_C * A.PW;
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int c2 = 0; c2 < NCT; ++c2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = j0 + 16 * (w * CTW + ct) + lh + 4 * i;
        if (j < d) out[(size_t)(16 * c2 + lr) * A.PW + 1 + j] = acc[ct][c2][i];
      }
}

// Sum chunk partials in chunk order and finish the family's lp / gradient.
// grid (nshards*C, ceil(PW/64)), 1024 threads: 16 waves split the chunks (each sums its
// contiguous range in order, 8 loads in flight), then the 16 partial sums are added in wave
// order -- a fixed order that depends only on G.  (At one shard per GPU the 4-wave form was a
// chain of 32 dependent load batches per wave: 19 us per step.)
constexpr int RD_W = 16;
template <int FAM>
__global__ __launch_bounds__(64 * RD_W) void k_sweep_reduce(SweepArgs A, double* lp_out, double* g_out, int C) {
  const int gidl = blockIdx.x;              // local chain index in this launch
  const int shard = A.shard0 + gidl / C, c = gidl % C;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int o = blockIdx.y * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  __shared__ double part[RD_W][64];
  double v = 0.0;
  if (o < A.PW) {
    const int per = (A.G + RD_W - 1) / RD_W;
    const int k0 = w * per, k1 = min(A.G, k0 + per);
    const double* src = A.partial + ((size_t)shard * A.Gs * C + c) * A.PW + o;
    const size_t stride = (size_t)C * A.PW;
    int k = k0;
    for (; k + 8 <= k1; k += 8) {
      double a[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = src[(size_t)(k + i) * stride];
#pragma unroll
      for (int i = 0; i < 8; ++i) v += a[i];
    }
    for (; k < k1; ++k) v += src[(size_t)k * stride];
  }
  part[w][threadIdx.x & 63] = v;
  __syncthreads();
  if (w != 0 || o >= A.PW) return;
  double t = part[0][threadIdx.x];
#pragma unroll
  for (int i = 1; i < RD_W; ++i) t += part[i][threadIdx.x];
  const size_t gid = (size_t)shard * C + c;
  double* g = g_out + gid * A.Dp;
  const double* qc = A.q + gid * A.Dp;
  // normal(0, s) priors on alpha (q[0]) and beta (q[1..d]): lp -= pa a^2/2 + pb |b|^2/2 (Stan's
  // propto drops the constants), d/dq -= p q.  Flat (pa = pb = 0): no change, bit for bit.
  double prior_g = 0.0, prior_lp = 0.0;
  if (sh.pa != 0.0 || sh.pb != 0.0) {
    if (o == 0) prior_g = -sh.pa * qc[0];
    else if (o <= d) prior_g = -sh.pb * qc[o];
    else {
      double sb = 0.0;
      for (int j = 1; j <= d; ++j) sb = fma(qc[j], qc[j], sb);
      prior_lp = -0.5 * (sh.pa * qc[0] * qc[0] + sh.pb * sb);
    }
  }
  if (FAM == STK_LOGREG) {
    if (o == d + 1) lp_out[gid] = t + prior_lp;
    else g[o] = t + prior_g;
  } else {
    const double u = qc[d + 1];
    const double N = (double)sh.n;
    if (o == d + 1) {
      g[d + 1] = -N + t + 1.0;
      lp_out[gid] = -0.5 * t - N * u + u + prior_lp;
    } else {
      g[o] = t + prior_g;
    }
  }
}

}  // namespace stk

using namespace stk;

// Host-side geometry: depends only on (n, d, C) so reductions are identical on 1 or N GPUs.
// v3 (LDS-DMA ring) for even d <= 104 and C <= 4, v2 for other even d <= 128, else v1.
// stk_sweep_force_variant (1 | 2 | 3, 0 = by shape) is set by tools/sweep_micro.hip only: the
// library reads no environment variable to pick a kernel.
int stk_sweep_force_variant = 0;
static int sweep_forced() { return stk_sweep_force_variant; }

// Ring depth of v3: as many slots per wave as fit next to the d-eta scratch (at most 5).
static int sweep3_nb(int d, int C) {
  const size_t fixed = (size_t)S3_W * 8 * C * sizeof(double);
  const size_t per = (size_t)S3_W * sweep3_slot_bytes(d / 2);
  int nb = (int)((160 * 1024 - fixed) / per);
  return std::min(nb, 5);
}

static int sweep_variant(int64_t n, int d, int C) {
  if (C == G5_C) return (((n + 511) / 512 + G5_TR + G5_FTR) * d * 8 < ((int64_t)1 << 31)) ? 5 : 0;   // chunk bytes (+ pass F's last tile) fit a buffer descriptor
  if (C == SM_C) return (stk_sweep16_supported(d) && (n * d * 8) / 512 < ((int64_t)1 << 30)) ? 4 : 0;
  const int f = sweep_forced();
  const bool v3ok = d % 2 == 0 && d / 2 <= S3_KMAX && (C == 1 || C == 2 || C == 4) && sweep3_nb(d, C) >= 3 &&
                    (n * d * 8) / 512 < ((int64_t)1 << 30);
  const bool v2ok = d <= 128 && d % 2 == 0;
  if (f == 1) return 1;
  if (f == 2) return v2ok ? 2 : 1;
  if (v3ok) return 3;
  return v2ok ? 2 : 1;
}

void stk_sweep_geometry(int64_t n, int d, int* T, int* LD, int* G, size_t* lds_bytes, int C) {
  const int var = sweep_variant(n, d, C);
  if (var == 5) {
    const int64_t nt = (n + G5_TR - 1) / G5_TR;
    int64_t g = (nt + 3) / 4;            // >= 4 tiles of 64 rows per chunk
    if (g > 512) g = 512;
    if (g < 1) g = 1;
    *T = G5_TR;
    *LD = 0;
    *G = (int)g;
    *lds_bytes = G5_FS * g5_fstage_bytes() + EX_TAB * sizeof(double);   // pass F's (pass B sizes its own)
    return;
  }
  if (var == 4) {                       // k_sweep16 (sweep16.hip)
    const int64_t nt = (n + 63) / 64;
    int64_t g = (nt + 7) / 8;            // >= 8 tiles of 64 rows per chunk (as v3)
    if (g > 512) g = 512;
    if (g < 1) g = 1;
    *T = 64;
    *LD = 1;
    *G = (int)g;
    *lds_bytes = stk_sweep16_lds_bytes(STK_LOGREG, d);   // the larger of the two families
    return;
  }
  if (var == 3) {
    const int64_t nt = (n + S3_T - 1) / S3_T;
    int64_t g = (nt + 7) / 8;            // >= 8 tiles per chunk
    if (g > 512) g = 512;
    if (g < 1) g = 1;
    const int nb = sweep3_nb(d, C);
    *T = S3_T;
    *LD = nb;
    *G = (int)g;
    const int K = d / 2;
    const size_t ring = (size_t)S3_W * nb * sweep3_slot_bytes(K) + (size_t)S3_W * 8 * C * sizeof(double);
    const size_t red = ((size_t)S3_W * C * 128 + (size_t)S3_W * 64 * 2) * sizeof(double);
    *lds_bytes = std::max(ring, red);
    return;
  }
  int t = 64;
  while (t > 8 && (int64_t)t * d > 8192) t >>= 1;
  int64_t g = (n + (int64_t)8 * t - 1) / ((int64_t)8 * t);
  if (g > 512) g = 512;
  if (g < 1) g = 1;
  *T = t;
  *G = (int)g;
  if (var == 2) {
    *LD = d | 1;
    const size_t main = (size_t)(64 * (d | 1) + 4 * C * 64 + 64 * C) * sizeof(double);
    const size_t red = (size_t)std::max(4 * C * 2 * 64, 4 * 256) * sizeof(double);
    *lds_bytes = std::max(main, red);
    return;
  }
  const int m = (256 / t) % 32;   // LD = m (mod 32): conflict-free ds_read_b64 in the forward pass
  int ld = d;
  while ((ld % 32) != m) ++ld;
  *LD = ld;
  const int JW = d <= 64 ? 64 : (d <= 128 ? 128 : 256);
  const int JPT = (d + JW - 1) / JW;
  const size_t main = (size_t)(t * ld + C * ld + t * C + 2 * C) * sizeof(double);
  const size_t red1 = (size_t)(256 / JW) * C * JW * JPT * sizeof(double);
  const size_t red2 = (size_t)2 * C * 256 * sizeof(double);
  size_t b = main;
  if (red1 > b) b = red1;
  if (red2 > b) b = red2;
  *lds_bytes = b;
}

template <int FAM, int C, int T, int JPT, int VEC>
static hipError_t launch_sweep_t(const SweepArgs& A, int nblocks, size_t lds, hipStream_t st) {
  if (const hipError_t e = allow_big_lds((const void*)k_sweep<FAM, C, T, JPT, VEC>)) return e;
  hipLaunchKernelGGL((k_sweep<FAM, C, T, JPT, VEC>), dim3(nblocks), dim3(256), lds, st, A);
  return hipGetLastError();
}

template <int FAM, int C, int T, int JPT>
static hipError_t pick_vec(const SweepArgs& A, int d, int nblocks, size_t lds, hipStream_t st) {
  if (d % 2 == 0) return launch_sweep_t<FAM, C, T, JPT, 2>(A, nblocks, lds, st);
  return launch_sweep_t<FAM, C, T, JPT, 1>(A, nblocks, lds, st);
}

template <int FAM, int C>
static hipError_t pick_tile(const SweepArgs& A, int64_t n, int d, int T, int nblocks, size_t lds, hipStream_t st) {
  const int var = sweep_variant(n, d, C);
  if (var == 3) {
    if constexpr (C <= 4) {
      auto go = [&](auto kern) {
        if (const hipError_t e = allow_big_lds((const void*)kern)) return e;
        hipLaunchKernelGGL(kern, dim3(nblocks), dim3(512), lds, st, A, A.LD);
        return hipGetLastError();
      };
      if (d == 100 && A.LD == 3) return go(k_sweep3<FAM, C, 0, 50, 3>);
      if (d == 50 && A.LD == 5) return go(k_sweep3<FAM, C, 0, 25, 5>);
      return go(k_sweep3<FAM, C>);
    }
    return hipErrorInvalidValue;
  }
  if (var == 2) {
    if (const hipError_t e = allow_big_lds((const void*)k_sweep2<FAM, C>)) return e;
    hipLaunchKernelGGL((k_sweep2<FAM, C>), dim3(nblocks), dim3(256), lds, st, A);
    return hipGetLastError();
  }
  switch (T) {
    case 64: return pick_vec<FAM, C, 64, 1>(A, d, nblocks, lds, st);
    case 32: return pick_vec<FAM, C, 32, 1>(A, d, nblocks, lds, st);
    case 16: return pick_vec<FAM, C, 16, 2>(A, d, nblocks, lds, st);
    case 8: return pick_vec<FAM, C, 8, 4>(A, d, nblocks, lds, st);
  }
  return hipErrorInvalidValue;
}

template <int FAM>
static hipError_t pick_c(const SweepArgs& A, int64_t n, int d, int T, int nblocks, size_t lds, hipStream_t st) {
  if (A.C == SM_C) return sweep_variant(n, d, A.C) == 4 ? stk_launch_sweep16(FAM, A, d, nblocks, lds, st) : hipErrorInvalidValue;
  switch (A.C) {
    case 1: return pick_tile<FAM, 1>(A, n, d, T, nblocks, lds, st);
    case 2: return pick_tile<FAM, 2>(A, n, d, T, nblocks, lds, st);
    case 4: return pick_tile<FAM, 4>(A, n, d, T, nblocks, lds, st);
    case 8: return pick_tile<FAM, 8>(A, n, d, T, nblocks, lds, st);
  }
  return hipErrorInvalidValue;
}

bool stk_sweep_supported(int C, int d) {
  if (C == G5_C) return d >= 1 && d <= 4096;
  if (C == SM_C) return d >= 1 && d <= 128;
  if (!(C == 1 || C == 2 || C == 4 || C == 8)) return false;
  return d >= 1 && d <= 1024;
}

// Workspace bytes of the sweep for `nshards` shards of at most n_max rows (0 unless v5).
size_t stk_sweep_ws_bytes(int64_t n_max, int d, int C, int nshards) {
  if (sweep_variant(n_max, d, C) != 5) return 0;
  const int64_t rrows = (n_max + G5_TR - 1) / G5_TR * G5_TR;
  return sizeof(double) * (size_t)nshards * G5_C * ((size_t)g5_kp(d) + (size_t)rrows);
}
SweepWs stk_sweep_ws(void* base, int64_t n_max, int d, int nshards) {
  SweepWs w{};
  w.Rrows = (n_max + G5_TR - 1) / G5_TR * G5_TR;
  w.qT = reinterpret_cast<double*>(base);
  w.R = w.qT + (size_t)nshards * g5_kp(d) * G5_C;
  return w;
}

// Launch the sweep over `nsh` shards starting at shard0 (all with the same n, d geometry).
hipError_t stk_launch_sweep(int family, const ShardDev* shards_dev, int shard0, int nsh, int64_t n, int d, int T,
                            int LD, int G, int Gs, size_t lds, const double* q, int C, int Dp, double* partial,
                            const int* req_step, int step_id, int* ran, hipStream_t st, const SweepWs* ws = nullptr) {
  SweepArgs A{shards_dev, q, partial, req_step, step_id, C, Dp, G, LD, d + 2, shard0, Gs, ran};
  const int nblocks = nsh * G;
  if (sweep_variant(n, d, C) == 5) {
    if (!ws || !ws->qT || !ws->R || ws->Rrows < (n + G5_TR - 1) / G5_TR * G5_TR) return hipErrorInvalidValue;
    A.qT = ws->qT;
    A.R = ws->R;
    A.Rrows = ws->Rrows;
    const int bjb = g5_bjb(d), njb = (d + bjb - 1) / bjb;
    hipLaunchKernelGGL(k_qt_swizzle, dim3((g5_kp(d) * G5_C + 255) / 256, nsh), dim3(256), 0, st, A, d);
    // the split stage schedule needs a tile's NKC = ceil(d / 16) stages to hold its 8 epilogue parts
    const bool split = (d + G5_FKC - 1) / G5_FKC >= 8;
    auto kf = family == STK_LOGREG ? (split ? k_gemm_fwd<STK_LOGREG, G5_FW, 2, G5_FKC, G5_FS, 1> : k_gemm_fwd<STK_LOGREG>)
                                   : (split ? k_gemm_fwd<STK_LINREG, G5_FW, 2, G5_FKC, G5_FS, 1> : k_gemm_fwd<STK_LINREG>);
    if (const hipError_t e = allow_big_lds((const void*)kf)) return e;
    hipLaunchKernelGGL(kf, dim3(nblocks), dim3(64 * G5_FW), lds, st, A);
    auto kb = bjb == 64 ? k_gemm_bwd<64> : bjb == 128 ? k_gemm_bwd<128> : k_gemm_bwd<256>;
    if (const hipError_t e = allow_big_lds((const void*)kb)) return e;
    hipLaunchKernelGGL(kb, dim3(nblocks * njb), dim3(64 * G5_BW), G5_BNS * g5_bstage_bytes(bjb), st, A, njb);
    return hipGetLastError();
  }
  if (family == STK_LOGREG) return pick_c<STK_LOGREG>(A, n, d, T, nblocks, lds, st);
  if (family == STK_LINREG) return pick_c<STK_LINREG>(A, n, d, T, nblocks, lds, st);
  return hipErrorInvalidValue;
}

hipError_t stk_launch_sweep_reduce(int family, const ShardDev* shards_dev, int shard0, int nsh, int d, int G, int Gs,
                                   const double* q, int C, int Dp, double* partial, const int* req_step,
                                   int step_id, double* lp_out, double* g_out, hipStream_t st) {
  SweepArgs A{shards_dev, q, partial, req_step, step_id, C, Dp, G, 0, d + 2, shard0, Gs, nullptr};
  dim3 grid(nsh * C, (d + 2 + 63) / 64);
  if (family == STK_LOGREG)
    hipLaunchKernelGGL(k_sweep_reduce<STK_LOGREG>, grid, dim3(64 * RD_W), 0, st, A, lp_out, g_out, C);
  else
    hipLaunchKernelGGL(k_sweep_reduce<STK_LINREG>, grid, dim3(64 * RD_W), 0, st, A, lp_out, g_out, C);
  return hipGetLastError();
}
