// Round-5 measurement variants of k_sweep16 (stark_amd/csrc/sweep16.hip) for
// tools/sweep16_ab.hip: a copy of the product kernel with knobs V (bits)
//   1  NOWAIT  ablation: no vmcnt(0) before a sub-tile (reads whatever the slot holds: results are
//              garbage, the time says how much DMA latency the two waves leave exposed)
//   2  NORES   ablation: the residual replaced by one multiply (what the residual's vector
//              instructions cost)
//   4  NOXA    ablation: the backward's 24 operands are lane constants, not read from the slot
//   8  NOVREM  ablation: no VALU last tile (the last <= 4 columns' 16 FMAs and their LDS copy)
//  16  EARLYXA the backward's operand reads interleaved with the forward's MFMAs (even d), so
//              the release waits only for the last of them
//  32  PEEL    full sub-tiles in a loop without the partial-sub-tile test; the wave's last
//              sub-tile, if partial, after the loop
//  64  DPPV    the VALU last tile's X values as 4 registers per lane read from the slot before
//              the release (lane lr & 3 of each row), broadcast by v_fmac_f64_dpp row_newbcast:
//              no LDS copy and 2 KB instead of 8 KB of LDS reads per sub-tile
// 128  DPPV2   the same from ONE register per lane: X[lh + 4 (lr >> 2)][16 JTM + (lr & 3)], so the
//              value of (row lh + 4i, column jj) is lane 4i + jj of the DPP row: 512 B of LDS reads
// 256 x FPD    the forward's X pairs read FPD pairs ahead of their MFMAs
// Included after sweep16.hip (namespace stk).
namespace stk {

template <int FAM, int KF, int V, bool PRE = s16_pre(FAM, KF), int NACC = 2>
__global__ __launch_bounds__(256, 2) void k_sweep16v(SweepArgs A) {
  constexpr bool NOWAIT = V & 1, NORES = V & 2, NOXA = V & 4, NOVREM = V & 8, EARLYXA = V & 16, PEEL = V & 32;
  constexpr bool DPPV = V & 64;                 // VALU last tile from a DPP broadcast (no LDS copy)
  constexpr bool DPPV2 = V & 128;               // ... from ONE register per lane (row lh + 4 (lr >> 2), column lr & 3)
  constexpr int FPD = (V >> 8) & 7;             // forward read-ahead depth in X pairs (0: the compiler's)
  constexpr S16Geom g = s16_geom(KF);
  constexpr bool VREM = g.VREM && !NOVREM;
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
  double* const xst = tab + (LOGI ? EX_TAB : 0) + w * 64;      // the last tile's <= 4 columns x 16 rows
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
  auto step = [&](int k, auto full_tag) {
    constexpr int FULLK = decltype(full_tag)::value;   // 1: a full sub-tile, 0: may be partial (checked)
    if constexpr (!NOWAIT) __builtin_amdgcn_s_waitcnt(0xF70);   // vmcnt(0): sub-tile k landed
    __builtin_amdgcn_sched_barrier(0);
    const int rv = FULLK ? SM_R : std::min(SM_R, nrows - SM_R * (w + NW * k));
    // ---- forward: eta[row lh + 4i][chain lr], starting from alpha
    double xa[4][PRE && JTM > 0 ? JTM : 1];
    dbl4 ea[NACC];
    ea[0] = dbl4{alpha, alpha, alpha, alpha};
#pragma unroll
    for (int i = 1; i < NACC; ++i) ea[i] = dbl4{0.0, 0.0, 0.0, 0.0};
    if ((d & 1) == 0) {
      // even d (16-B aligned rows): k-steps 2m, 2m+1 of lane group lh take columns 8m + 2 lh and
      // 8m + 2 lh + 1, one ds_read_b128 of X per pair instead of two ds_read_b64; KF odd: the
      // last k-step takes column 8 (KF / 2) + lh.  (A/B at d = 100: 13.88 -> 13.79 ms,
      // profiles/r04c_*); odd d: k-step s of lane group lh takes column lh KF + s
      dbl2 xq[KF / 2 > 0 ? KF / 2 : 1];
      if constexpr (FPD > 0) {
#pragma unroll
        for (int m = 0; m < FPD && m < KF / 2; ++m) xq[m] = *reinterpret_cast<const dbl2*>(xs + lr * d + 8 * m + 2 * lh);
      }
#pragma unroll
      for (int m = 0; m < KF / 2; ++m) {
        dbl2 x2;
        if constexpr (FPD > 0) {
          if (m + FPD < KF / 2) xq[m + FPD] = *reinterpret_cast<const dbl2*>(xs + lr * d + 8 * (m + FPD) + 2 * lh);
          x2 = xq[m];
        } else {
          x2 = *reinterpret_cast<const dbl2*>(xs + lr * d + 8 * m + 2 * lh);
        }
        ea[(2 * m) % NACC] = mfma_f64(x2.x, bf[2 * m], ea[(2 * m) % NACC]);
        ea[(2 * m + 1) % NACC] = mfma_f64(x2.y, bf[2 * m + 1], ea[(2 * m + 1) % NACC]);
        if constexpr (EARLYXA && PRE) {       // the backward's operands read between the forward's MFMAs
#pragma unroll
          for (int q = 0; q < 4 * JTM; ++q)
            if (q * (KF / 2) / (4 * JTM) == m)
              xa[q / JTM][q % JTM] = NOXA ? 1e-3 * (lane + 7 * (q / JTM) + 3 * (q % JTM))
                                          : xs[(lh + 4 * (q / JTM)) * d + bcol(q % JTM)];
        }
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
    if constexpr (PRE && !(EARLYXA && (KF / 2) > 0)) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < JTM; ++t) xa[s][t] = NOXA ? 1e-3 * (lane + 7 * s + 3 * t) : xs[(lh + 4 * s) * d + bcol(t)];
    }
    double xv[4];
    double xv2 = 0.0;
    if constexpr (VREM && DPPV2) {
      xv2 = xs[(lh + 4 * (lr >> 2)) * d + std::min(16 * JTM + (lr & 3), d - 1)];
    } else if constexpr (VREM && DPPV) {   // lane (lr, lh): X[lh + 4i][16 JTM + (lr & 3)]; lanes lr = 0..3 are broadcast
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[i] = xs[(lh + 4 * i) * d + std::min(16 * JTM + (lr & 3), d - 1)];
    } else if constexpr (VREM) {
      xst[lane] = xs[(lane >> 2) * d + std::min(16 * JTM + (lane & 3), d - 1)];
    }
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
    if (FULLK || rv == SM_R) {                         // full sub-tile: no masks
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (NORES) {
          de[i] = eta4[i] * 1e-6;
          lm += (double)ym[i];
        } else if constexpr (LOGI) {
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
    if constexpr (VREM && DPPV2) {
      // gv[jj] += X[lh + 4i][16 JTM + jj] * de[i]: that X value sits in lane 4i + jj of this lane's
      // DPP row (rows lh + 4i of every chain share the row), broadcast by row_newbcast
#define S16_F(I, J, G) "v_fmac_f64_dpp %" #G ", %4, %" #I " row_newbcast:" #J " row_mask:0xf bank_mask:0xf\n\t"
      asm volatile("s_nop 1\n\t"
                   S16_F(5, 0, 0) S16_F(5, 1, 1) S16_F(5, 2, 2) S16_F(5, 3, 3)
                   S16_F(6, 4, 0) S16_F(6, 5, 1) S16_F(6, 6, 2) S16_F(6, 7, 3)
                   S16_F(7, 8, 0) S16_F(7, 9, 1) S16_F(7, 10, 2) S16_F(7, 11, 3)
                   S16_F(8, 12, 0) S16_F(8, 13, 1) S16_F(8, 14, 2) S16_F(8, 15, 3)
                   : "+v"(gv[0]), "+v"(gv[1]), "+v"(gv[2]), "+v"(gv[3])
                   : "v"(xv2), "v"(de[0]), "v"(de[1]), "v"(de[2]), "v"(de[3]));
#undef S16_F
    } else if constexpr (VREM && DPPV) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // gv[jj] += X[lh + 4i][16 JTM + jj] (lane jj of the row) * de[i]
        // s_nop 1: two wait states between any VALU write of %4 (a copy the register allocator
        // might insert) and its DPP read
        asm volatile("s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %4, %5 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %1, %4, %5 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %2, %4, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                     "v_fmac_f64_dpp %3, %4, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                     : "+v"(gv[0]), "+v"(gv[1]), "+v"(gv[2]), "+v"(gv[3])
                     : "v"(xv[i]), "v"(de[i]));
      }
    } else if constexpr (VREM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const dbl2* p = reinterpret_cast<const dbl2*>(xst + (lh + 4 * i) * 4);
        const dbl2 a0 = p[0], a1 = p[1];
        gv[0] = fma(a0.x, de[i], gv[0]);
        gv[1] = fma(a0.y, de[i], gv[1]);
        gv[2] = fma(a1.x, de[i], gv[2]);
        gv[3] = fma(a1.y, de[i], gv[3]);
      }
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
  };
  if constexpr (PEEL) {   // full sub-tiles in the loop; this wave's last one, if partial, after it
    const bool part = mine > 0 && nrows - SM_R * (w + NW * (mine - 1)) < SM_R;
    for (int k = 0; k < mine - (int)part; ++k) step(k, std::integral_constant<int, 1>{});
    if (part) step(mine - 1, std::integral_constant<int, 0>{});
  } else {
    for (int k = 0; k < mine; ++k) step(k, std::integral_constant<int, 0>{});
  }
  if constexpr (NOWAIT) __builtin_amdgcn_s_waitcnt(0xF70);    // drain the last DMA before the LDS is reused
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
