// Measurement-only variants of the 16-chain sweep k_sweep16 (stark_amd/csrc/sweep16.hip), for
// tools/sweep16_ab.hip: the same kernel with knobs
//   BREG / NACC   as the product (beta in registers + late slot release; forward accumulators)
//   LSA           (y << 31) + hi as ONE v_lshl_add_u32 per use (inline asm; the compiler otherwise
//                 shares one v_lshlrev_b32 between the two uses and adds twice: 3 instructions)
//   PB            wave priority: 0 the product (2 over the residual), 1 + a static 1 for odd blocks
//                 (the SIMD partner that loses arbitration), 2 none at all, 3 the static one only
//   PAIR          the forward's k-steps 2m, 2m+1 read columns 8m + 2 lh, +1 of X and beta as one
//                 ds_read_b128 each (needs an even d), instead of two ds_read_b64
// Included after sweep16.hip (namespace stk).
namespace stk {

__device__ __forceinline__ uint32_t lsa31(uint32_t y, uint32_t hi, bool asm_form) {
  if (!asm_form) return (y << 31) + hi;
  uint32_t r;
  asm("v_lshl_add_u32 %0, %1, 31, %2" : "=v"(r) : "v"(y), "v"(hi));
  return r;
}

template <bool LSA>
__device__ __forceinline__ double logit_resid4x(double eta, uint32_t y, const double* tab, double& lm, double& sp) {
  constexpr double MAGIC = 6755399441055744.0;            // 1.5 * 2^52
  constexpr double INV_L = 1477.3197218702985;            // 1024 / ln 2
  constexpr double L = 0.0006769015435155716;             // ln 2 / 1024
  constexpr double C2 = 0.5000000039583942, C3 = 0.16666666713444417;   // e^r on |r| <= ln2/2048 (fit)
  const uint64_t eb = __builtin_bit_cast(uint64_t, eta);
  const double s = __builtin_bit_cast(double, (eb & 0xFFFFFFFFull) | ((uint64_t)lsa31(y, (uint32_t)(eb >> 32), LSA) << 32));
  const double a = fmin_abs(s, 700.0);                    // |s| = |eta|; NaN -> 700 (the NaN stays in lm)
  const double sn = fma(-a, INV_L, MAGIC);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = sn - MAGIC;
  const double r = fma(-n, L, -a);
  const double p = fma(fma(fma(C3, r, C2), r, 1.0), r, 1.0);
  const int ke = (s > 20.0) ? -1100 : (ni >> 10);         // Stan's lower cutoff (t < -20): e = 0
  const double e = __builtin_amdgcn_ldexp(tab[ni & (EX_TAB - 1)] * p, ke);
  const double u = 1.0 + e;
  double ri = __builtin_amdgcn_rcp(u);
  ri = fma(ri, fma(-u, ri, 1.0), ri);
  const double w = e * ri;
  const uint64_t sb = __builtin_bit_cast(uint64_t, s);
  const uint32_t spos = (uint32_t)((int32_t)(sb >> 32) >> 31);   // ~0u when s < 0, i.e. t > 0
  const uint64_t dvp = __builtin_bit_cast(uint64_t, blend(spos, w, ri));   // dv/sgn
  lm += -s - fabs(s);                                     // t - |t|
  sp = fma(sp, u, e);
  return __builtin_bit_cast(double, (dvp & 0xFFFFFFFFull) | ((uint64_t)lsa31(y, (uint32_t)(dvp >> 32), LSA) << 32));   // -dv
}

template <int FAM, int KF, bool BREG = (KF >= 28), int NACC = 2, bool LSA = false, bool PAIR = false, int PB = 0>
__global__ __launch_bounds__(256, 2) void k_sweep16x(SweepArgs A) {
  constexpr S16Geom g = s16_geom(KF);
  constexpr int C = SM_C, NW = SM_W, JTM = g.JTM, KP = 4 * KF, KB = KP + 2;
  constexpr bool LOGI = FAM == STK_LOGREG;
  constexpr bool PRE = !BREG;                  // early release: backward operands into registers
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
  double* const bimg = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * SS);   // [16][KB]
  double* const tab = bimg + (BREG ? 0 : C * KB);
  double* const xst = tab + (LOGI ? EX_TAB : 0) + w * 64;      // the last tile's <= 4 columns x 16 rows
  if constexpr (LOGI) exp_table_init(tab);
  const double* qs = A.q + (size_t)shard * C * A.Dp;
  double bf[BREG ? KF : 1];
  if constexpr (BREG) {
#pragma unroll
    for (int s = 0; s < KF; ++s) {
      const int col = lh * KF + s;
      bf[s] = col < d ? qs[(size_t)lr * A.Dp + 1 + col] : 0.0;
    }
  } else {
    for (int i = tid; i < C * KP; i += NW * 64) {
      const int c = i / KP, col = i % KP;
      bimg[c * KB + col] = col < d ? qs[(size_t)c * A.Dp + 1 + col] : 0.0;
    }
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
  const double* brow = bimg + lr * KB + lh * KF;
  const double* xrow = xs + lr * d;

  if constexpr (PB == 1 || PB == 3) { if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1); }
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
    if constexpr (PAIR) {          // k-steps 2m, 2m+1 of lane group lh: columns 8m + 2lh, +1 (one b128 each)
#pragma unroll
      for (int m = 0; m < KF / 2; ++m) {
        const dbl2 xa2 = *reinterpret_cast<const dbl2*>(xs + lr * d + 8 * m + 2 * lh);
        const dbl2 b2 = *reinterpret_cast<const dbl2*>(bimg + lr * KB + 8 * m + 2 * lh);
        ea[(2 * m) % NACC] = mfma_f64(xa2.x, b2.x, ea[(2 * m) % NACC]);
        ea[(2 * m + 1) % NACC] = mfma_f64(xa2.y, b2.y, ea[(2 * m + 1) % NACC]);
      }
      if constexpr (KF & 1) {
        const int col = 8 * (KF / 2) + lh;
        ea[(KF - 1) % NACC] = mfma_f64(xrow[std::min(col, d - 1)], bimg[lr * KB + col], ea[(KF - 1) % NACC]);
      }
    } else {
#pragma unroll
    for (int s = 0; s < KF; ++s) {
      const double b = BREG ? bf[s] : brow[s];
      ea[s % NACC] = mfma_f64(xrow[std::min(lh * KF + s, d - 1)], b, ea[s % NACC]);
    }
    }
    // ---- everything else the sub-tile needs from the slot, into registers; then release it
    double xa[4][PRE && JTM > 0 ? JTM : 1];
    if constexpr (PRE) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < JTM; ++t) xa[s][t] = xs[(lh + 4 * s) * d + std::min(16 * t + lr, d - 1)];
    }
    if constexpr (g.VREM) xst[lane] = xs[(lane >> 2) * d + std::min(16 * JTM + (lane & 3), d - 1)];
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
    if constexpr (PB == 0) __builtin_amdgcn_s_setprio(2);
    if constexpr (PB == 1) { if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(3); else __builtin_amdgcn_s_setprio(2); }
    if (rv == SM_R) {                                  // full sub-tile: no masks
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (LOGI) {
          de[i] = logit_resid4x<LSA>(eta4[i], ym[i], tab, lm, sp);
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
          dv = logit_resid4x<LSA>(eta4[i], ym[i], tab, lm2, sp2);
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
    if constexpr (PB == 0) __builtin_amdgcn_s_setprio(0);
    if constexpr (PB == 1 || PB == 3) { if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1); else __builtin_amdgcn_s_setprio(0); }
    // ---- backward
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTM; ++t)
        gacc[t] = mfma_f64(PRE ? xa[s][t] : xs[(lh + 4 * s) * d + std::min(16 * t + lr, d - 1)], de[s], gacc[t]);
    if constexpr (g.VREM) {
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
