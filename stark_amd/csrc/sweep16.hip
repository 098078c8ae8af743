// The 16-chain regression sweep (C = 16, any d <= 128): log density + gradient of the 16
// chains of a shard in ONE pass over the shard's rows, on the fp64 MFMA.
//
// Replaces the gradient Stan's reverse-mode autodiff computes for every leapfrog inside
// `sm.sampling` (stark/stark.py:48) for the regression programs (oracle: orc_logreg_lpgrad /
// orc_linreg_lpgrad).  With 16 chains sharing a shard, X . [beta_1 .. beta_16] is a dense GEMM
// (8 flop per byte of X at d = 100) and the sweep is bound by the fp64 pipe at the clock the
// chip holds under it, not by HBM: every vector instruction takes the issue slot an fp64 MFMA
// needs (tools/valu_mix.hip), so the design goal is the fewest vector instructions per row
// (DESIGN.md section 3).
//
// Workgroup = 4 waves (two workgroups per CU: two waves per SIMD).  The shard is cut into G
// chunks that depend only on (n, d); wave w owns the 16-row sub-tiles u = w, w + 4, ... of its
// chunk.  Per sub-tile:
//   DMA       16 rows of X and their y, `buffer_load_dwordx4 ... lds` (nt: X is read once per
//             sweep) into the wave's LDS slot;
//   forward   eta[16 rows][16 chains] on v_mfma_f64_16x16x4: k-step s, lane group lh = lane>>4
//             takes one column of row lane&15 (A) and beta_{lane&15} at that column (B, held in
//             registers for the whole launch: no LDS reads for it); KF = ceil(d/4) k-steps, the
//             accumulator starts at alpha;
//   release   the backward's A operands, the last <= 4 columns and y move to registers, the
//             slot takes the DMA of the next sub-tile (d <= 108 logistic, every d linear; past
//             that the slot is released after the backward: registers);
//   residual  on the MFMA output registers (lane: rows lh + 4i, chain lane&15) -- logistic:
//             logit_resid4 below; linear: z = (y - eta)/sigma;
//   backward  G[16 cols][16 chains] += X_tile^T . d_eta: the D layout of the forward is the B
//             layout of the backward (k-step s = rows 4s..4s+3 = register s), one MFMA per
//             (16-column tile, k-step); a last tile of <= 4 columns runs on the VALU (16 DPP
//             FMAs instead of 4 mostly-padding MFMAs).
// Chunk partials are summed in chunk order by k_sweep_reduce (sweep.hip): the gradient is
// bitwise independent of how many shards share a launch or which GPU runs a shard.
#include "sweep_common.h"
#include <math.h>
#include <algorithm>

namespace stk {

// exp table, logistic residual v4 (logit_resid4): sweep_common.h (shared with the 64-chain pass F)

// Geometry of k_sweep16 for a given d (host and device).
struct S16Geom {
  int KF, JT, REM, JTM;
  bool VREM;
};
__host__ __device__ constexpr S16Geom s16_geom(int KF) {
  const int JT = (KF + 3) / 4;                  // 16-column tiles covering 4 KF >= d columns
  const int REM = 4 * KF - 16 * (JT - 1);       // columns of the last tile (d has up to 3 fewer)
  const bool VREM = REM <= 4;                   // <= 4: the VALU does the last tile
  return S16Geom{KF, JT, REM, VREM ? JT - 1 : JT, VREM};
}
// Early release (PRE): the backward's A operands (4 JTM doubles) join beta (KF doubles) in
// registers.  Logistic at KF >= 28 (d > 108) would spill, so there the backward reads them from
// the slot, which is released after the backward (the next DMA's latency is then covered by the
// SIMD's other wave only).  beta in registers instead of a block image in LDS: 14.00 -> 13.84 and
// 14.24 -> 14.05 ms at d = 100 on two boxes, 7.03 -> 6.92 and 7.15 -> 7.04 ms at d = 50 linear
// (profiles/r04q_*, r04s_*).
__host__ __device__ constexpr bool s16_pre(int FAM, int KF) { return FAM == STK_LINREG || KF <= 27; }
constexpr int S16_FLUSH = 64;                   // sub-tiles between log1p flushes (4 elements each)

template <int FAM, int KF, bool PRE = s16_pre(FAM, KF), int NACC = 2>
__global__ __launch_bounds__(256, 2) void k_sweep16(SweepArgs A) {
  constexpr S16Geom g = s16_geom(KF);
  constexpr int C = SM_C, NW = SM_W, JTM = g.JTM;
  constexpr bool LOGI = FAM == STK_LOGREG;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + SM_R - 1) / SM_R;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;   // own sub-tiles u = w + NW k
  constexpr int YB = LOGI ? 4 : 8;
  const int SBX = SM_R * d * 8;
  const int SS = sweepm_slot_bytes(d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const slot = reinterpret_cast<char*>(lds) + (size_t)w * SS;
  double* const tab = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * SS);
  if constexpr (LOGI) exp_table_init(tab);
  const double* qs = A.q + (size_t)shard * C * A.Dp;
  double bf[KF];                   // beta_{lr} at the column k-step s of lane group lh takes (forward)
#pragma unroll
  for (int s = 0; s < KF; ++s) {
    const int col = (d & 1) ? lh * KF + s : (s < KF - (KF & 1) ? 8 * (s / 2) + 2 * lh + (s & 1) : 8 * (KF / 2) + lh);
    bf[s] = col < d ? qs[(size_t)lr * A.Dp + 1 + col] : 0.0;
  }
  const double alpha = qs[(size_t)lr * A.Dp];
  const double inv_s = LOGI ? 0.0 : exp(-qs[(size_t)lr * A.Dp + d + 1]);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = LOGI ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  auto issue = [&](int k) {           // 1 KiB per DMA instruction, aux = 2 (nt)
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + j * 1024), 16, lane * 16, xoff + j * 1024, 0, 2);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, 2);
    if (lane < SM_R * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(slot + SBX), 4, lane * 4, u * SM_R * YB, 0, 2);
  };

  dbl4 gacc[JTM > 0 ? JTM : 1];
#pragma unroll
  for (int t = 0; t < JTM; ++t) gacc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gv[4] = {0.0, 0.0, 0.0, 0.0};
  double lm = 0.0, sp = 0.0, ll = 0.0, ga = 0.0;   // logistic lp pieces (linear: lm = sum z^2)
  const double* xs = reinterpret_cast<const double*>(slot);
  // column of the backward's A operand in tile t: only a last MFMA tile (no VALU remainder) can
  // reach past d - 1 (VREM: 16 JTM = 4 KF - 4 <= d), so only it is clamped -- a clamp with the
  // runtime d gives every (row, tile) its own address register, held across the loop
  auto bcol = [&](int t) { return (g.VREM || t < JTM - 1) ? 16 * t + lr : std::min(16 * t + lr, d - 1); };
  const double* xrow = xs + lr * d;

  if (mine > 0) issue(0);
  for (int k = 0; k < mine; ++k) {
    __builtin_amdgcn_s_waitcnt(0xF70);                 // vmcnt(0): sub-tile k landed
    __builtin_amdgcn_sched_barrier(0);
    const int rv = std::min(SM_R, nrows - SM_R * (w + NW * k));
    // ---- forward: eta[row lh + 4i][chain lr], starting from alpha
    dbl4 ea[NACC];
    ea[0] = dbl4{alpha, alpha, alpha, alpha};
#pragma unroll
    for (int i = 1; i < NACC; ++i) ea[i] = dbl4{0.0, 0.0, 0.0, 0.0};
    if ((d & 1) == 0) {
      // even d (16-B aligned rows): k-steps 2m, 2m+1 of lane group lh take columns 8m + 2 lh and
      // 8m + 2 lh + 1, one ds_read_b128 of X per pair instead of two ds_read_b64; KF odd: the
      // last k-step takes column 8 (KF / 2) + lh.  (A/B at d = 100: 13.88 -> 13.79 ms,
      // profiles/r04c_*); odd d: k-step s of lane group lh takes column lh KF + s
#pragma unroll
      for (int m = 0; m < KF / 2; ++m) {
        const dbl2 x2 = *reinterpret_cast<const dbl2*>(xs + lr * d + 8 * m + 2 * lh);
        ea[(2 * m) % NACC] = mfma_f64(x2.x, bf[2 * m], ea[(2 * m) % NACC]);
        ea[(2 * m + 1) % NACC] = mfma_f64(x2.y, bf[2 * m + 1], ea[(2 * m + 1) % NACC]);
      }
      if constexpr (KF & 1) {
        const int col = 8 * (KF / 2) + lh;
        ea[(KF - 1) % NACC] = mfma_f64(xrow[std::min(col, d - 1)], bf[KF - 1], ea[(KF - 1) % NACC]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KF; ++s) {
        // lh KF + s <= d - 1 unless s >= KF - 3 (d >= 4 KF - 3): clamp those steps only (see bcol)
        ea[s % NACC] = mfma_f64(xrow[s < KF - 3 ? lh * KF + s : std::min(lh * KF + s, d - 1)], bf[s], ea[s % NACC]);
      }
    }
    // ---- everything else the sub-tile needs from the slot, into registers; then release it
    double xa[4][PRE && JTM > 0 ? JTM : 1];
    if constexpr (PRE) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < JTM; ++t) xa[s][t] = xs[(lh + 4 * s) * d + bcol(t)];
    }
    // the VALU last tile's X: ONE value per lane, row lh + 4 (lr >> 2), column 16 JTM + (lr & 3) --
    // the value of (row lh + 4i, column jj) is then lane 4i + jj of the lane's own DPP row
    double xv = 0.0;
    if constexpr (g.VREM) xv = xs[(lh + 4 * (lr >> 2)) * d + std::min(16 * JTM + (lr & 3), d - 1)];
    uint32_t ym[4];
    double yv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (LOGI)   // y in {0, 1}
        ym[i] = *reinterpret_cast<const uint32_t*>(slot + SBX + (lh + 4 * i) * 4);
      else
        yv[i] = *reinterpret_cast<const double*>(slot + SBX + (lh + 4 * i) * 8);
    }
    if constexpr (PRE) {
      __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0): the slot is free
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < mine) issue(k + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    dbl4 eta4 = ea[0];
#pragma unroll
    for (int i = 1; i < NACC; ++i) eta4 += ea[i];

    // ---- residual (raised wave priority: the dependent chain goes first, the partner wave's
    // MFMAs fill its gaps; +1.5 % in round 3's A/B)
    double de[4];
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(2);
    if (rv == SM_R) {                                  // full sub-tile: no masks
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (LOGI) {
          de[i] = logit_resid4(eta4[i], ym[i], tab, lm, sp);
        } else {
          const double z = (yv[i] - eta4[i]) * inv_s;
          lm = fma(z, z, lm);
          de[i] = z * inv_s;
        }
        ga += de[i];
      }
    } else {                                           // a chunk's last sub-tile
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool valid = lh + 4 * i < rv;
        double lm2 = lm, sp2 = sp, dv;
        if constexpr (LOGI) {
          dv = logit_resid4(eta4[i], ym[i], tab, lm2, sp2);
        } else {
          const double z = (yv[i] - eta4[i]) * inv_s;
          lm2 = fma(z, z, lm);
          dv = z * inv_s;
        }
        lm = valid ? lm2 : lm;
        sp = valid ? sp2 : sp;
        de[i] = valid ? dv : 0.0;
        ga += de[i];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    // ---- backward
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTM; ++t)
        gacc[t] = mfma_f64(PRE ? xa[s][t] : xs[(lh + 4 * s) * d + bcol(t)], de[s], gacc[t]);
    if constexpr (g.VREM) {
      // gv[jj] += X[lh + 4i][16 JTM + jj] * de[i] with the X value broadcast from lane 4i + jj of
      // the row by v_fmac_f64_dpp row_newbcast (DPP64): no LDS copy of the last columns, 512 B
      // instead of 8.5 KB of LDS traffic per sub-tile (A/B at d = 100: -0.8 / -1.1 % on two
      // boxes, profiles/r05j_*, r05l_*).  s_nop 1: the two wait states a VALU write of the DPP
      // source needs before the DPP read, should the register allocator copy xv
#define S16_DPP_FMAC(I, J, G) "v_fmac_f64_dpp %" #G ", %4, %" #I " row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"
      asm volatile("s_nop 1\n\t"
                   S16_DPP_FMAC(5, 0, 0) S16_DPP_FMAC(5, 1, 1) S16_DPP_FMAC(5, 2, 2) S16_DPP_FMAC(5, 3, 3)
                   S16_DPP_FMAC(6, 4, 0) S16_DPP_FMAC(6, 5, 1) S16_DPP_FMAC(6, 6, 2) S16_DPP_FMAC(6, 7, 3)
                   S16_DPP_FMAC(7, 8, 0) S16_DPP_FMAC(7, 9, 1) S16_DPP_FMAC(7, 10, 2) S16_DPP_FMAC(7, 11, 3)
                   S16_DPP_FMAC(8, 12, 0) S16_DPP_FMAC(8, 13, 1) S16_DPP_FMAC(8, 14, 2) S16_DPP_FMAC(8, 15, 3)
                   : "+v"(gv[0]), "+v"(gv[1]), "+v"(gv[2]), "+v"(gv[3])
                   : "v"(xv), "v"(de[0]), "v"(de[1]), "v"(de[2]), "v"(de[3]));
#undef S16_DPP_FMAC
    }
    if constexpr (!PRE) {
      __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0): the slot is free
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < mine) issue(k + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (LOGI) {
      if ((k % S16_FLUSH) == S16_FLUSH - 1) {
        ll += log1p(sp);
        sp = 0.0;
      }
    }
  }
  double lpa;
  if constexpr (LOGI) {   // the residual returned -dv: negate the gradient sums once
    lpa = 0.5 * lm - (ll + log1p(sp));
    ga = -ga;
#pragma unroll
    for (int t = 0; t < JTM; ++t) gacc[t] = -gacc[t];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) gv[jj] = -gv[jj];
  } else {
    lpa = lm;
  }

  // ---- fixed-order block reduction -> one partial row per chain
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;                                   // [NW][JT*16 columns][16 chains]
  constexpr int JC = g.JT * 16;
#pragma unroll
  for (int t = 0; t < JTM; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((size_t)w * JC + 16 * t + lh + 4 * i) * 16 + lr] = gacc[t][i];
  double* red2 = red + (size_t)NW * JC * 16;           // [NW][64 lanes][lp, g_alpha]
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = ga;
  double* red3 = red2 + (size_t)NW * 64 * 2;           // VREM: [NW][4 lh][4 jj][16 chains]
  if constexpr (g.VREM) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) red3[((size_t)(w * 4 + lh) * 4 + jj) * 16 + lr] = gv[jj];
  }
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  const int jv = 16 * JTM;                             // first column summed from red3
  for (int i = tid; i < C * d; i += NW * 64) {
    const int c = i / d, j = i % d;
    double v = 0.0;
    if (j < jv) {
      for (int ww = 0; ww < NW; ++ww) v += red[((size_t)ww * JC + j) * 16 + c];
    } else {
      for (int ww = 0; ww < NW; ++ww)
        for (int h = 0; h < 4; ++h) v += red3[((size_t)(ww * 4 + h) * 4 + (j - jv)) * 16 + c];
    }
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {          // chain c: lanes h*16 + c of every wave, in (wave, h) order
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

}  // namespace stk

using namespace stk;

// LDS bytes of k_sweep16 at d (the main loop's slots + table + remainder scratch, or the block
// reduction's area, whichever is larger).
size_t stk_sweep16_lds_bytes(int family, int d) {
  const int KF = (d + 3) / 4;
  const S16Geom g = s16_geom(KF);
  size_t main = (size_t)SM_W * sweepm_slot_bytes(d) + (family == STK_LOGREG ? EX_TAB * 8 : 0);
  const size_t red = ((size_t)SM_W * g.JT * 16 * 16 + (size_t)SM_W * 64 * 2 + (size_t)SM_W * 4 * 4 * 16) * 8;
  return std::max(main, red);
}

template <int FAM, int KF>
static hipError_t go16(const SweepArgs& A, int nblocks, size_t lds, hipStream_t st) {
  auto kern = k_sweep16<FAM, KF>;
  if (const hipError_t e = allow_big_lds((const void*)kern)) return e;
  hipLaunchKernelGGL(kern, dim3(nblocks), dim3(SM_W * 64), lds, st, A);
  return hipGetLastError();
}

template <int FAM>
static hipError_t launch16(const SweepArgs& A, int d, int nblocks, size_t lds, hipStream_t st) {
  switch ((d + 3) / 4) {
#define S16_CASE(K) case K: return go16<FAM, K>(A, nblocks, lds, st);
    S16_CASE(1) S16_CASE(2) S16_CASE(3) S16_CASE(4) S16_CASE(5) S16_CASE(6) S16_CASE(7) S16_CASE(8)
    S16_CASE(9) S16_CASE(10) S16_CASE(11) S16_CASE(12) S16_CASE(13) S16_CASE(14) S16_CASE(15) S16_CASE(16)
    S16_CASE(17) S16_CASE(18) S16_CASE(19) S16_CASE(20) S16_CASE(21) S16_CASE(22) S16_CASE(23) S16_CASE(24)
    S16_CASE(25) S16_CASE(26) S16_CASE(27) S16_CASE(28) S16_CASE(29) S16_CASE(30) S16_CASE(31) S16_CASE(32)
#undef S16_CASE
  }
  return hipErrorInvalidValue;
}

bool stk_sweep16_supported(int d) { return d >= 1 && d <= 128; }

hipError_t stk_launch_sweep16(int family, const SweepArgs& A, int d, int nblocks, size_t lds, hipStream_t st) {
  if (family == STK_LOGREG) return launch16<STK_LOGREG>(A, d, nblocks, lds, st);
  if (family == STK_LINREG) return launch16<STK_LINREG>(A, d, nblocks, lds, st);
  return hipErrorInvalidValue;
}
