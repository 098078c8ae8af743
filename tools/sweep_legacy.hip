// Round 1-3 16-chain sweeps, kept out of libstark_hip.so for measurement tools only
// (tools/sweepe_ab.hip, tools/sweep16_ab.hip, tools/sweep_micro.hip, tools/sweepe_d50.hip):
// k_sweepm (any d <= 128, ring of slots), k_sweepe (round 3's product at d = 100 / 50, with its
// measurement knobs RV / ER / AUX / PRIO / PF / IL / FS / ABL), the residuals v1 (softplus_tab)
// and v2 (logit_resid).  The product is k_sweep16 (stark_amd/csrc/sweep16.hip).  Included after
// stark_amd/csrc/sweep.hip (namespace stk).
#pragma once
namespace stk {

// Logistic residual v3 (round 3's 16-chain sweep and pass F epilogue): round 2's v2 with fewer VALU instructions -- on gfx950 EVERY
// vector instruction (f64, f32, int, select) takes the issue slot the f64 MFMA needs
// (tools/valu_mix.hip: no class overlaps v_mfma_f64_16x16x4), so the residual's instruction
// count, not its f64 count, is what it costs.  Same quantities and cutoffs as v2:
//   Stan's lower cutoff without selects: a = min(|t| + 2^60 max(-20 - t, 0), 700) is |t| for
//   t >= -20 and 700 below, where e = exp(-700) ~ 1e-304 makes lg = e, lt = t - lg = t and
//   dv/sgn = 1/(1 + e) = 1 exactly -- Stan's (t, 1);
//   exp(-a): 256-entry 2^{j/256} table, |r| <= ln2/512, degree-4 Taylor (rel. error 4e-17), the
//   2^{n div 256} scale by v_ldexp_f64;  log1p(e): 257-entry [c_j, d_j, l_j] table (j = rint(256 e)),
//   |rl| <= 1/512, degree-4 fitted q (abs. error 1.2e-18);
//   lt = t/2 - (|t|/2 + lg) = min(t, 0) - lg with NaN kept (a NaN eta gives a NaN lp; t = +inf
//   gives NaN where Stan's upper branch gives 0 -- a point no finite beta reaches).
// About 38 vector instructions per (row, chain) against v2's ~50.
constexpr int LG3_TAB = 256 + 4 * 257;     // doubles: T[256], then [c_j, d_j, l_j, 0] for j = 0..256
__device__ void logit3_tables_init(double* tab) {
  for (int i = threadIdx.x; i < LG3_TAB; i += blockDim.x) {
    double v;
    if (i < 256) {
      v = exp2((double)i / 256.0);
    } else {
      const int j = (i - 256) >> 2, f = (i - 256) & 3;
      v = f == 0 ? 256.0 / (256 + j) : (f == 1 ? (double)j / (256 + j) : (f == 2 ? log1p((double)j / 256.0) : 0.0));
    }
    tab[i] = v;
  }
}

// v_rcp_f64 alone is good to ~2^-24 only (tools/rcp_acc.hip, profiles/r03s_rcp_acc.log: 2.6e8 ulp;
// 11 ulp after the one Newton step below).
__device__ __forceinline__ void logit_resid3(double eta, uint32_t ymask, const double* tab, double& lt, double& dv) {
  constexpr double MAGIC = 6755399441055744.0;            // 1.5 * 2^52
  constexpr double INV_L = 369.3299304675746;             // 256 / ln 2
  constexpr double L_HI = 0.0027076061742263846;          // ln2/256 to 32 significant bits: n L_HI exact
  constexpr double L_LO = -1.6409824498184568e-13;        // ln2/256 - L_HI
  constexpr double Q1 = -0.4999999999996968, Q2 = 0.33333333333269194, Q3 = -0.25000063579045223,
                   Q4 = 0.2000006787837857;               // log(1+x)/x on |x| <= 1/512 (tools: least squares)
  const double t = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, eta) ^ ((uint64_t)ymask << 32));
  const double a = fmin(fma(fmax(-20.0 - t, 0.0), 1152921504606846976.0, fabs(t)), 700.0);   // + 2^60 max(-20 - t, 0)
  const double sn = fma(-a, INV_L, MAGIC);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = sn - MAGIC;
  double r = fma(-n, L_HI, -a);
  r = fma(-n, L_LO, r);
  const double p = fma(fma(fma(fma(1.0 / 24.0, r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0);
  const double e = __builtin_amdgcn_ldexp(tab[ni & 255] * p, ni >> 8);
  const int j = (int)fma(e, 256.0, 0.5);                  // rint(256 e), e in [0, 1] (v_cvt_i32_f64 truncates)
  const double* cj = tab + 256 + 4 * j;
  const dbl2 cd = *reinterpret_cast<const dbl2*>(cj);
  const double rl = fma(e, cd.x, -cd.y);
  const double q = fma(fma(fma(fma(Q4, rl, Q3), rl, Q2), rl, Q1), rl, 1.0);
  const double lg = fma(rl, q, cj[2]);
  const double u = 1.0 + e;
  double ri = __builtin_amdgcn_rcp(u);
  ri = fma(ri, fma(-u, ri, 1.0), ri);
  const double w = e * ri;
  const uint32_t neg = (uint32_t)((int32_t)(__builtin_bit_cast(uint64_t, t) >> 32) >> 31);   // ~0u when t < 0
  const double dvp = blend(neg, ri, w);
  dv = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, dvp) ^ ((uint64_t)ymask << 32));
  lt = fma(0.5, t, fma(-0.5, fabs(t), -lg));
}


// NEWTON: one Newton step on v_rcp_f64, which alone is good to ~2^-24 only (tools/rcp_acc.hip,
// profiles/r03s_rcp_acc.log: 2.6e8 ulp; 11 ulp after the step); without it the gradient moves by
// 4e-9 relative (RV 4, measurement only).  EXP4: degree-4 Taylor exp (else a fitted degree 3,
// relative error 7e-14; RV 5, measurement only: no faster, profiles/r03s_sweepe_ab.log).
template <bool NEWTON = true, bool EXP4 = true>
__device__ __forceinline__ void logit_resid3x(double eta, uint32_t ymask, const double* tab, double& lt, double& dv) {
  constexpr double MAGIC = 6755399441055744.0;            // 1.5 * 2^52
  constexpr double INV_L = 369.3299304675746;             // 256 / ln 2
  constexpr double L_HI = 0.0027076061742263846;          // ln2/256 to 32 significant bits: n L_HI exact
  constexpr double L_LO = -1.6409824498184568e-13;        // ln2/256 - L_HI
  constexpr double Q1 = -0.4999999999996968, Q2 = 0.33333333333269194, Q3 = -0.25000063579045223,
                   Q4 = 0.2000006787837857;               // log(1+x)/x on |x| <= 1/512 (tools: least squares)
  const double t = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, eta) ^ ((uint64_t)ymask << 32));
  const double a = fmin(fma(fmax(-20.0 - t, 0.0), 1152921504606846976.0, fabs(t)), 700.0);   // + 2^60 max(-20 - t, 0)
  const double sn = fma(-a, INV_L, MAGIC);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = sn - MAGIC;
  double r = fma(-n, L_HI, -a);
  r = fma(-n, L_LO, r);
  const double p = EXP4 ? fma(fma(fma(fma(1.0 / 24.0, r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0)
                        : fma(fma(fma(0.16666667813799327, r, 0.500000038186625), r, 1.0), r, 1.0);
  const double e = __builtin_amdgcn_ldexp(tab[ni & 255] * p, ni >> 8);
  const int j = (int)fma(e, 256.0, 0.5);                  // rint(256 e), e in [0, 1] (v_cvt_i32_f64 truncates)
  const double* cj = tab + 256 + 4 * j;
  const dbl2 cd = *reinterpret_cast<const dbl2*>(cj);
  const double rl = fma(e, cd.x, -cd.y);
  const double q = fma(fma(fma(fma(Q4, rl, Q3), rl, Q2), rl, Q1), rl, 1.0);
  const double lg = fma(rl, q, cj[2]);
  const double u = 1.0 + e;
  double ri = __builtin_amdgcn_rcp(u);
  if constexpr (NEWTON) ri = fma(ri, fma(-u, ri, 1.0), ri);
  const double w = e * ri;
  const uint32_t neg = (uint32_t)((int32_t)(__builtin_bit_cast(uint64_t, t) >> 32) >> 31);   // ~0u when t < 0
  const double dvp = blend(neg, ri, w);
  dv = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, dvp) ^ ((uint64_t)ymask << 32));
  lt = fma(0.5, t, fma(-0.5, fabs(t), -lg));
}

// Table-driven softplus for the fp64-bound v4 residual (the fp64 MFMA and fp64 VALU share one
// pipe on gfx950, so every f64 instruction of the residual costs MFMA time; ocml's exp + log
// + the correction take ~105 instructions per (row, chain), this ~45).  Tables in LDS:
//   tab[0 .. 64)          T_j = 2^(j/64)
//   tab[64 + 2j], +1      c_j = 1/(1 + (j + 1/2)/128) (c_0 = 1), l_j = -log(c_j), j < 128
// exp(x): x = n ln2/64 + r, |r| <= ln2/128, e^r by degree 5 (rel. error < 4e-17), times
//         T_{n mod 64}, scaled by 2^(n div 64) (v_ldexp_f64);
// log(u): u = 2^k m, m in [1, 2), r = m c_j - 1 (|r| <= 1/128; exact for j = 0, so log(u)
//         keeps its relative accuracy as u -> 1), log(1+r) = r q(r), q of degree 6.
// Worst relative error of the softplus term over |x| <= 20: 1e-14 (numpy/mpmath check of the
// same formulas); the bar is 1e-10 (tests/test_gpu_kernels.py).
constexpr int SP_TAB = 64 + 2 * 128;
__device__ void softplus_tables_init(double* tab) {
  for (int i = threadIdx.x; i < SP_TAB; i += blockDim.x) {
    double v;
    if (i < 64) {
      v = exp2((double)i / 64.0);
    } else {
      const int j = (i - 64) >> 1;
      const double c = j == 0 ? 1.0 : 1.0 / (1.0 + (j + 0.5) / 128.0);
      v = ((i - 64) & 1) ? -log(c) : c;
    }
    tab[i] = v;
  }
}

// e = exp(-ntt); lmid = log1p(e) (Stan's middle branch); w = e / (1 + e)
__device__ __forceinline__ void softplus_tab(double ntt, const double* tab, double* e_out, double* lmid, double* w) {
  constexpr double INV_L = 92.33248261689366;              // 64 / ln 2
  constexpr double L_HI = 0.010830417275428772;            // ln2/64 rounded to 21 bits: n * L_HI is exact
  constexpr double L_LO = 7.420820373486988e-09;           // ln2/64 - L_HI
  constexpr double LN2 = 0.69314718055994530942;
  const double x = fmin(fmax(-ntt, -800.0), 800.0);
  const double n = __builtin_rint(x * INV_L);
  const int ni = (int)n;
  double r = fma(-n, L_HI, x);
  r = fma(-n, L_LO, r);
  double p = fma(fma(fma(fma(fma(1.0 / 120.0, r, 1.0 / 24.0), r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0);
  const double e = __builtin_amdgcn_ldexp(tab[ni & 63] * p, ni >> 6);
  const double u = 1.0 + e;
  const double m2 = 2.0 * __builtin_amdgcn_frexp_mant(u);
  const int k = __builtin_amdgcn_frexp_exp(u) - 1;
  const int j = (int)((uint32_t)(__builtin_bit_cast(uint64_t, m2) >> 45) & 127u);
  const dbl2 cl = *reinterpret_cast<const dbl2*>(tab + 64 + 2 * j);
  const double rl = fma(m2, cl.x, -1.0);
  double q = fma(fma(fma(fma(fma(fma(1.0 / 7.0, rl, -1.0 / 6.0), rl, 1.0 / 5.0), rl, -0.25), rl, 1.0 / 3.0), rl, -0.5), rl, 1.0);
  const double lg = fma((double)k, LN2, fma(rl, q, cl.y));
  double ri = __builtin_amdgcn_rcp(u);
  ri = fma(ri, fma(-u, ri, 1.0), ri);
  ri = fma(ri, fma(-u, ri, 1.0), ri);
  *e_out = e;
  *lmid = lg - ((u - 1.0) - e) * ri;
  *w = e * ri;
}

// Logistic residual v2 (k_sweepe): Stan's bernoulli_logit term lt and its derivative dv for
// one (row, chain) from ONE exp and ONE log1p of a = |t|, t = (2y - 1) eta:
//   e = exp(-a)                 x = -a = n ln2/128 + r, |r| <= ln2/256; e^r by degree 4 (rel. error
//                               1.2e-15), times T_{n mod 128} = 2^{(n mod 128)/128} from LDS, times
//                               2^{n div 128} added to the exponent field with an integer add (a is
//                               clamped to 700, so the result stays a normal number);
//                               n = rint(x 128/ln2) comes from the low word of fma(x, 128/ln2, 1.5 2^52);
//   lg = log1p(e)               j = rint(128 e) (the same fma trick), c_j = 128/(128 + j),
//                               d_j = j/(128 + j), l_j = log(1 + j/128): rl = e c_j - d_j (one fma,
//                               |rl| <= 1/256, exact for j = 0 so small e keeps its relative accuracy,
//                               and 1 + e is never formed), lg = l_j + rl q(rl), q of degree 5;
//   ri = 1/(1 + e)              v_rcp_f64 + one Newton step;  w = e ri.
// Then lt = min(t, 0) - lg and dv/sgn = (t < 0 ? ri : w), with Stan's lower cutoff t < -20 ->
// (lt, dv/sgn) = (t, 1) applied as a select (NaN takes that branch, so a NaN eta stays NaN).
// Stan's upper cutoff (t > 20: -exp(-t), exp(-t)) differs from the smooth expressions by
// <= e^2 <= 4.3e-18 and needs no branch.  t and dv's sign come from an XOR of the sign bit
// (ymask = 0x80000000 for y = 0).  About 30 f64 instructions per (row, chain) against ~50 for
// softplus_tab (fp64 VALU and fp64 MFMA share one pipe on gfx950).
constexpr int LG_TAB = 128 + 4 * 129;     // doubles: T[128], then [c_j, d_j, l_j, 0] for j = 0..128
__device__ void logit_tables_init(double* tab) {
  for (int i = threadIdx.x; i < LG_TAB; i += blockDim.x) {
    double v;
    if (i < 128) {
      v = exp2((double)i / 128.0);
    } else {
      const int j = (i - 128) >> 2, f = (i - 128) & 3;
      v = f == 0 ? 128.0 / (128 + j) : (f == 1 ? (double)j / (128 + j) : (f == 2 ? log1p((double)j / 128.0) : 0.0));
    }
    tab[i] = v;
  }
}


__device__ __forceinline__ void logit_resid(double eta, uint32_t ymask, const double* tab, double& lt, double& dv) {
  constexpr double MAGIC = 6755399441055744.0;            // 1.5 * 2^52
  constexpr double INV_L = 184.6649652337873;            // 128 / ln 2
  constexpr double L_HI = 0.005415212348452769;          // ln2/128 rounded to 32 significant bits: n L_HI exact
  constexpr double L_LO = -3.2819649005320973e-13;       // ln2/128 - L_HI
  const double t = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, eta) ^ ((uint64_t)ymask << 32));
  // a = min(|t|, 700): past it e = exp(-700) ~ 1e-304 stands in for exp(-a) (|lt|, |dv| error
  // < 1e-304), and n = rint(-a 128/ln2) >= -129,300 stays exact in the low word of the fma trick
  // and 2^{n div 128} a normal scale (a NaN t gives a = 700 here; the cutoff select below keeps NaN)
  const double a = fmin(fabs(t), 700.0);
  const double sn = fma(-a, INV_L, MAGIC);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = (double)ni;
  double r = fma(-n, L_HI, -a);
  r = fma(-n, L_LO, r);
  const double p = fma(fma(fma(fma(1.0 / 24.0, r, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0);
  const double tp = tab[ni & 127] * p;
  const double e = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, tp) + ((uint64_t)(int64_t)(ni >> 7) << 52));
  const double sj = fma(e, 128.0, MAGIC);
  const int j = (int)(uint32_t)__builtin_bit_cast(uint64_t, sj);
  const double* cj = tab + 128 + 4 * j;
  const dbl2 cd = *reinterpret_cast<const dbl2*>(cj);
  const double rl = fma(e, cd.x, -cd.y);
  const double q = fma(fma(fma(fma(fma(-1.0 / 6.0, rl, 0.2), rl, -0.25), rl, 1.0 / 3.0), rl, -0.5), rl, 1.0);
  const double lg = fma(rl, q, cj[2]);
  const double u = 1.0 + e;
  double ri = __builtin_amdgcn_rcp(u);
  ri = fma(ri, fma(-u, ri, 1.0), ri);
  const double w = e * ri;
  const uint32_t neg = (uint32_t)((int32_t)(__builtin_bit_cast(uint64_t, t) >> 32) >> 31);   // ~0u when t < 0 (or -0)
  const uint32_t lo = (t >= -20.0) ? 0u : ~0u;                                                 // Stan's cutoff; NaN too
  const double lts = blend(neg, t, 0.0) - lg;                                                  // min(t, 0) - lg
  lt = blend(lo, t, lts);
  const double dvp = blend(lo, 1.0, blend(neg, ri, w));
  dv = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, dvp) ^ ((uint64_t)ymask << 32));
}

// ABL (micro-benchmark ablations only): bit 0 linear residual stand-in, bit 1 no backward,
// bit 2 no forward.  KFS/JTS: compile-time KF / JT for the BASELINE shapes (0 = runtime).
template <int FAM, int KFS = 0, int JTS = 0, int ABL = 0, int MINB = SM_MINB, bool VREM = false>
__global__ __launch_bounds__(256, MINB) void k_sweepm(SweepArgs A, int NB) {
  constexpr int C = SM_C, NW = SM_W;
  constexpr int KFM = KFS ? KFS : 32, JTM = JTS ? JTS : 8;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int KF = KFS ? KFS : (d + 3) >> 2;
  const int JT = JTS ? JTS : (d + 15) >> 4;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + SM_R - 1) / SM_R;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;   // own sub-tiles u = w + NW*k
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  const int SBX = SM_R * d * 8;
  const int SS = sweepm_slot_bytes(d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const ring = reinterpret_cast<char*>(lds) + (size_t)w * NB * SS;
  double* const sptab = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * NB * SS);
  if constexpr (FAM == STK_LOGREG) {
    logit_tables_init(sptab);
    __syncthreads();
  }

  // ---- chain lr's beta fragments (B operand of the forward), alpha, 1/sigma
  const double* qc = A.q + ((size_t)shard * C + lr) * A.Dp;
  double bf[KFM];
#pragma unroll
  for (int s = 0; s < KFM; ++s) {
    const int col = lh * KF + s;
    bf[s] = (s < KF && col < d) ? qc[1 + col] : 0.0;
  }
  const double alpha = qc[0];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qc[d + 1]) : 0.0;
  __builtin_amdgcn_s_waitcnt(0xF70);                      // ordinary loads retired before the DMAs start

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  const int per_tile = nx + 1;
  auto issue = [&](int k) {
    char* sl = ring + (size_t)(k % NB) * SS;
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + j * 1024), 16, lane * 16, xoff + j * 1024, 0, 0);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, 0);
    if (lane < SM_R * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(sl + SBX), 4, lane * 4, u * SM_R * YB, 0, 0);
  };

  dbl4 gacc[JTM];
#pragma unroll
  for (int t = 0; t < JTM; ++t) gacc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double lpa = 0.0, gaa = 0.0;
  // VREM: the last column tile holds d - 16 (JT - 1) <= 4 columns (d = 100: 96..99, d = 50: 48, 49);
  // 4 MFMAs for it would be >= 75 % padding, so the VALU does them (16 FMAs per lane): gv[jj] =
  // column 16 (JT - 1) + jj, chain lr, summed over this lane's 4 rows (rows lh + 4i)
  constexpr int JTMM = VREM ? JTM - 1 : JTM;
  double gv[4] = {0.0, 0.0, 0.0, 0.0};

  // Ring of NB slots per wave: sub-tiles k+1 .. k+NB-1 are in flight while sub-tile k is
  // computed (NB = 1: the DMA of sub-tile k is issued when sub-tile k-1 is done, and the
  // other waves of the SIMD -- two blocks per CU -- cover its latency).
  for (int k = 0; k < NB - 1 && k < mine; ++k) issue(k);
  for (int k = 0; k < mine; ++k) {
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): reads of slot k-1 are done
    __builtin_amdgcn_sched_barrier(0);
    if (k + NB - 1 < mine) issue(k + NB - 1);            // into slot (k-1) % NB
    wait_vmcnt(std::max(0, std::min(NB - 2, mine - 1 - k)) * per_tile);   // own DMAs of sub-tile k retired
    __builtin_amdgcn_sched_barrier(0);
    const char* sl = ring + (size_t)(k % NB) * SS;
    const double* xs = reinterpret_cast<const double*>(sl);
    const int rv = std::min(SM_R, nrows - SM_R * (w + NW * k));

    // ---- forward: eta[row lh + 4i][chain lr] (without alpha)
    dbl4 e0 = {0.0, 0.0, 0.0, 0.0}, e1 = {0.0, 0.0, 0.0, 0.0};
    if constexpr (!(ABL & 4)) {
      const double* xrow = xs + lr * d;
#pragma unroll
      for (int s = 0; s < KFM; ++s) {
        if (s < KF) {
          const double a = xrow[std::min(lh * KF + s, d - 1)];
          if (s & 1) e1 = mfma_f64(a, bf[s], e1);
          else e0 = mfma_f64(a, bf[s], e0);
        }
      }
    }
    const dbl4 eta4 = e0 + e1;

    // ---- residual on (row lh + 4i, chain lr)
    double de[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = lh + 4 * i;
      const bool valid = row < rv;
      const double eta = eta4[i] + alpha;
      double dv, lt;
      if constexpr (ABL & 1) {
        const int32_t yv = *reinterpret_cast<const int32_t*>(sl + SBX + row * 4);
        dv = (2.0 * yv - 1.0) - 0.25 * eta;
        lt = -dv * dv;
      } else if constexpr (FAM == STK_LOGREG) {
        // Stan's bernoulli_logit: ntt > 20 -> -exp(-ntt); ntt < -20 -> ntt; else -log1p(exp(-ntt))
        const int32_t yv = *reinterpret_cast<const int32_t*>(sl + SBX + row * 4);
        logit_resid(eta, yv == 0 ? 0x80000000u : 0u, sptab, lt, dv);
      } else {
        const double yv = *reinterpret_cast<const double*>(sl + SBX + row * 8);
        const double z = (yv - eta) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[i] = dv;
    }

    // ---- backward (s outer: JT independent accumulators between dependent MFMAs)
    if constexpr (!(ABL & 2)) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int t = 0; t < JTMM; ++t) {
          if (t < JT) gacc[t] = mfma_f64(xs[(lh + 4 * s) * d + std::min(16 * t + lr, d - 1)], de[s], gacc[t]);
        }
      }
      if constexpr (VREM) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // 16-B aligned: d and 16 (JT - 1) are even; columns past d read the next row / the y
          // area and are never written out
          const dbl2* xv = reinterpret_cast<const dbl2*>(xs + (lh + 4 * i) * d + 16 * (JTM - 1));
          const dbl2 a0 = xv[0], a1 = xv[1];
          gv[0] = fma(a0.x, de[i], gv[0]);
          gv[1] = fma(a0.y, de[i], gv[1]);
          gv[2] = fma(a1.x, de[i], gv[2]);
          gv[3] = fma(a1.y, de[i], gv[3]);
        }
      }
    }
  }

  // ---- fixed-order block reduction -> one partial row per chain
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;                                   // [NW][JT*16 columns][16 chains]
  const int JC = JT * 16;
#pragma unroll
  for (int t = 0; t < JTMM; ++t) {
    if (t < JT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) red[((size_t)w * JC + 16 * t + lh + 4 * i) * 16 + lr] = gacc[t][i];
    }
  }
  double* red2 = red + (size_t)NW * JC * 16;           // [NW][64 lanes][lp, g_alpha]
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  double* red3 = red2 + (size_t)NW * 64 * 2;           // VREM: [NW][4 lh][4 jj][16 chains]
  if constexpr (VREM) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) red3[((size_t)(w * 4 + lh) * 4 + jj) * 16 + lr] = gv[jj];
  }
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  const int jv = VREM ? 16 * (JT - 1) : d;             // first column summed from red3
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

// v4e: k_sweepm for the BASELINE shapes (d = 100, 50) with an early slot release.  With one
// 16-row slot per wave (NB = 1, two blocks per CU), k_sweepm issues the DMA of sub-tile k+1
// only after sub-tile k is done, so each sub-tile's HBM latency is exposed and only the other
// wave of the SIMD can cover it (PMC: MFMA busy 56 %, f64 VALU ~15 %, the rest idle).  Here
// the backward's A operands (24 values), the remainder columns and y move to registers right
// after the forward, the slot is refilled at once, and the residual + backward run while the
// next sub-tile streams in.  beta moves from registers to LDS (one 16 x 4KF image per block)
// to pay for those registers.
#ifndef SE_NACC
#define SE_NACC 2             // forward accumulators (4: same time, more registers; 8: spills)
#endif
// beta image row stride = 4 KF + SE_BPAD doubles: at 100 doubles (200 dwords = 8 mod 64 banks)
// chains c and c + 8 of one 32-lane group hit the same banks (2-way); 102 spreads the 16 chains
// of a group over 16 distinct bank pairs, lane groups lh = 0 / 1 on the other parity
#ifndef SE_BPAD
#define SE_BPAD 2
#endif
// RV: logistic residual version, 2 = logit_resid (alpha folded into the forward's accumulator
// init, sign flips by XOR; the product), 1 = softplus_tab (kept for A/B in tools/sweep_micro.hip).
// ER: early release -- the forward's A operands (25 values per lane) are read into registers with
// everything else the sub-tile needs BEFORE the forward, so the slot is refilled while the
// forward, the residual and the backward all run (ER = 0: after the forward, round 2).
// AUX: cache-policy bits of the X / y LDS-DMA loads (2 = nt: X is streamed once per sweep, 80 GB
// against a 256 MB MALL).
// PRIO (wave issue priority, s_setprio): 1 = raised over the residual (the dependent VALU / LDS
// table chain goes first, the other wave's MFMAs fill its gaps), 2 = raised from the top of the
// sub-tile until the next DMA is issued.
// PF: L2 prefetch distance 2 -- with the DMA of sub-tile k+1 the wave also touches every 64-B
// sector of sub-tile k+2 (and its y) by 4-byte LDS-DMA loads into a 256-B dummy LDS area, so the
// sub-tile is on its way into L2 one sub-tile early and its own DMA, one iteration later, is
// served from L2: HBM latency leaves the wave's critical path without another 12.8 KB slot.
// IL: on full sub-tiles the residual and the backward run in two halves (rows 0-1, then 2-3 of the
// lane's four): half the residual's live registers, and the first half's backward MFMAs are
// independent of the second half's residual chain (same summation order: bitwise the same result).
// FS (ER = 0): the forward's operand reads and the reads of everything else the sub-tile needs
// from the slot are interleaved with the forward MFMAs two ds_reads per MFMA (sched_group_barrier),
// so the LDS latency hides behind MFMAs and the slot is free when the last forward MFMA issues.
template <int FAM, int KF, int JT, int ABL = 0, int RV = 2, int NACC = SE_NACC, int ER = 1, int AUX = 0, int PRIO = 0,
          int PF = 0, int IL = 0, int FS = 0>
__global__ __launch_bounds__(256, 2) void k_sweepe(SweepArgs A) {
  constexpr int C = SM_C, NW = SM_W, JTV = JT - 1, KP = 4 * KF, KB = KP + SE_BPAD;
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
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  const int SBX = SM_R * d * 8;
  const int SS = sweepm_slot_bytes(d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const slot = reinterpret_cast<char*>(lds) + (size_t)w * SS;
  double* const bimg = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * SS);  // [16][KB]
  double* const sptab = bimg + C * KB;
  // ER: the 4 remainder columns (16 rows x 4) of the wave's sub-tile, kept past the slot's release
  constexpr int TABN = RV >= 3 ? LG3_TAB : LG_TAB;
  double* const xst = sptab + TABN + w * 64;
  double* const pfd = sptab + TABN + NW * 64 + w * 32;       // PF: 256-B dummy per wave
  constexpr bool R2 = FAM == STK_LOGREG && RV >= 2;
  if constexpr (FAM == STK_LOGREG && RV >= 3) logit3_tables_init(sptab);
  else if constexpr (R2) logit_tables_init(sptab);
  else if constexpr (FAM == STK_LOGREG) softplus_tables_init(sptab);
  const double* qs = A.q + (size_t)shard * C * A.Dp;
  for (int i = tid; i < C * KP; i += NW * 64) {
    const int c = i / KP, col = i % KP;
    bimg[c * KB + col] = col < d ? qs[(size_t)c * A.Dp + 1 + col] : 0.0;
  }
  const double alpha = qs[(size_t)lr * A.Dp];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qs[(size_t)lr * A.Dp + d + 1]) : 0.0;
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  auto issue = [&](int k) {
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + j * 1024), 16, lane * 16, xoff + j * 1024, 0, AUX);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, AUX);
    if (lane < SM_R * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(slot + SBX), 4, lane * 4, u * SM_R * YB, 0, AUX);
  };
  // PF touches: ceil(SBX / 4096) loads of one dword per 64-B sector + one for y -- a fixed count
  // per sub-tile (every instruction has at least one active lane), so the DMA of sub-tile k is
  // waited for with a counted vmcnt that leaves the touches of sub-tile k+1 in flight
  const int npf = ((SBX + 4095) >> 12) + 1;
  auto touch = [&](int k) {
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < npf - 1; ++j)
      if (j * 4096 + lane * 64 < SBX)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)pfd, 4, lane * 64, xoff + j * 4096, 0, 0);
    if (lane == 0) __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)pfd, 4, 0, u * SM_R * YB, 0, 0);
  };

  dbl4 gacc[JTV];
#pragma unroll
  for (int t = 0; t < JTV; ++t) gacc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gv[4] = {0.0, 0.0, 0.0, 0.0};
  double lpa = 0.0, gaa = 0.0;
  const double* xs = reinterpret_cast<const double*>(slot);
  const double* brow = bimg + lr * KB + lh * KF;

  // ER = 2: the forward operands of sub-tile k+1 are read from the slot during sub-tile k's
  // backward (their DMA was issued at the top of sub-tile k), the rest of the slot at the top of
  // sub-tile k+1, which then releases it: the DMA flies during forward + residual + backward
  static_assert(ER != 2 || IL == 0, "ER = 2 keeps the unsplit backward");
  double fa2[ER == 2 ? KF : 1];
  auto load_fa2 = [&]() {
    const double* xr_ = xs + lr * d;
#pragma unroll
    for (int s = 0; s < KF; ++s) fa2[s] = xr_[std::min(lh * KF + s, d - 1)];
  };
  if (mine > 0) issue(0);
  if (PF && mine > 1) touch(1);
  if constexpr (ER == 2) {
    if (mine > 0) {
      __builtin_amdgcn_s_waitcnt(0xF70);
      __builtin_amdgcn_sched_barrier(0);
      load_fa2();
    }
  }
  for (int k = 0; k < mine; ++k) {
    if constexpr (ER == 2) {
      // sub-tile k landed at the end of the previous iteration (or in the prologue)
    } else if (PF && k + 1 < mine) {
      wait_vmcnt(npf);                                   // sub-tile k landed, the touches of k+1 may fly
    } else {
      __builtin_amdgcn_s_waitcnt(0xF70);                 // vmcnt(0): sub-tile k landed
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(2);
    const int rv = std::min(SM_R, nrows - SM_R * (w + NW * k));
    // ---- forward (ER: operands first, MFMAs after the slot is released)
    dbl4 ea[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) ea[i] = dbl4{0.0, 0.0, 0.0, 0.0};
    if constexpr (R2) ea[0] = dbl4{alpha, alpha, alpha, alpha};     // D layout: lane holds chain lr
    double fa[ER ? KF : 1];
    const double* xrow = xs + lr * d;
    if constexpr (ER == 1) {
#pragma unroll
      for (int s = 0; s < KF; ++s) fa[s] = xrow[std::min(lh * KF + s, d - 1)];
    } else if constexpr (ER == 2) {
#pragma unroll
      for (int s = 0; s < KF; ++s) fa[s] = fa2[s];
    } else if constexpr (!(ABL & 4)) {
#pragma unroll
      for (int s = 0; s < KF; ++s) ea[s % NACC] = mfma_f64(xrow[std::min(lh * KF + s, d - 1)], brow[s], ea[s % NACC]);
    }
    // ---- everything the rest of the sub-tile needs from the slot, into registers
    double xa[4][JTV];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTV; ++t) xa[s][t] = xs[(lh + 4 * s) * d + 16 * t + lr];
    dbl2 xv[4][2];
    double yv[4];
    uint32_t ym[4];
    if constexpr (ER) xst[lane] = xs[(lane >> 2) * d + 16 * JTV + (lane & 3)];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (!ER) {
        const dbl2* p = reinterpret_cast<const dbl2*>(xs + (lh + 4 * i) * d + 16 * JTV);
        xv[i][0] = p[0];
        xv[i][1] = p[1];
      }
      if constexpr (R2) {
        // y in {0, 1}: (y << 31) + 2^31 = 2^31 for y = 0, 0 for y = 1 (one v_lshl_add_u32)
        ym[i] = ((uint32_t)*reinterpret_cast<const int32_t*>(slot + SBX + (lh + 4 * i) * 4) << 31) + 0x80000000u;
      } else {
        yv[i] = (FAM == STK_LOGREG) ? (double)*reinterpret_cast<const int32_t*>(slot + SBX + (lh + 4 * i) * 4)
                                    : *reinterpret_cast<const double*>(slot + SBX + (lh + 4 * i) * 8);
      }
    }
    if constexpr (FS && !ER && !(ABL & 4)) {
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);         // 6 ds_reads ahead
#pragma unroll
      for (int s = 0; s < KF; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);       // 2 ds_reads
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): the slot is free
    __builtin_amdgcn_sched_barrier(0);
    if (k + 1 < mine) issue(k + 1);
    if (PF && k + 2 < mine) touch(k + 2);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ER && !(ABL & 4)) {
#pragma unroll
      for (int s = 0; s < KF; ++s) ea[s % NACC] = mfma_f64(fa[s], brow[s], ea[s % NACC]);
    }
    dbl4 e0 = ea[0], e1 = {0.0, 0.0, 0.0, 0.0};
    if constexpr (NACC > 1) e1 = ea[1];
#pragma unroll
    for (int i = 2; i < NACC; ++i) { if (i & 1) e1 += ea[i]; else e0 += ea[i]; }
    const dbl4 eta4 = NACC > 1 ? e0 + e1 : e0;

    // ---- residual
    double de[4];
    if constexpr (PRIO == 1) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(2);
    }
    bool bwd_done = false;
    auto bwd_rows = [&](int s0, int s1) {              // backward MFMAs + remainder columns of rows s0..s1-1
#pragma unroll
      for (int s = s0; s < s1; ++s)
#pragma unroll
        for (int t = 0; t < JTV; ++t) gacc[t] = mfma_f64(xa[s][t], de[s], gacc[t]);
#pragma unroll
      for (int i = s0; i < s1; ++i) {
        if constexpr (ER) {
          const dbl2* p = reinterpret_cast<const dbl2*>(xst + (lh + 4 * i) * 4);
          xv[i][0] = p[0];
          xv[i][1] = p[1];
        }
        gv[0] = fma(xv[i][0].x, de[i], gv[0]);
        gv[1] = fma(xv[i][0].y, de[i], gv[1]);
        gv[2] = fma(xv[i][1].x, de[i], gv[2]);
        gv[3] = fma(xv[i][1].y, de[i], gv[3]);
      }
    };
    if constexpr (R2 && !(ABL & 1)) {
      if (rv == SM_R) {                                  // full sub-tile (all but a chunk's last): no masks
#pragma unroll
        for (int h = 0; h < (IL ? 2 : 1); ++h) {
          const int i0 = IL ? 2 * h : 0, i1 = IL ? 2 * h + 2 : 4;
#pragma unroll
          for (int i = i0; i < i1; ++i) {
            double lt;
            if constexpr (RV >= 3) logit_resid3x<RV == 3, RV != 5>(eta4[i], ym[i], sptab, lt, de[i]);
            else logit_resid(eta4[i], ym[i], sptab, lt, de[i]);
            lpa += lt;
            gaa += de[i];
          }
          if constexpr (IL && !(ABL & 2)) bwd_rows(i0, i1);
        }
        bwd_done = IL;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool valid = lh + 4 * i < rv;
          double lt, dv;
          if constexpr (RV >= 3) logit_resid3x<RV == 3, RV != 5>(eta4[i], ym[i], sptab, lt, dv);
          else logit_resid(eta4[i], ym[i], sptab, lt, dv);
          dv = valid ? dv : 0.0;
          lpa += valid ? lt : 0.0;
          gaa += dv;
          de[i] = dv;
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool valid = lh + 4 * i < rv;
      const double eta = eta4[i] + alpha;
      double dv, lt;
      if constexpr (ABL & 1) {
        dv = (2.0 * yv[i] - 1.0) - 0.25 * eta;
        lt = -dv * dv;
      } else if constexpr (FAM == STK_LOGREG) {
        const double sgn = 2.0 * yv[i] - 1.0;
        const double ntt = sgn * eta;
        double e, lm, wt;
        softplus_tab(ntt, sptab, &e, &lm, &wt);
        const bool hi = ntt > 20.0, lo = ntt < -20.0;
        lt = hi ? -e : (lo ? ntt : -lm);
        dv = sgn * (hi ? e : (lo ? 1.0 : wt));
      } else {
        const double z = (yv[i] - eta) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[i] = dv;
    }
    if constexpr (PRIO == 1) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
    }
    // ---- backward
    if constexpr (ER == 2) {
      if constexpr (!(ABL & 2)) bwd_rows(0, 2);
      if (k + 1 < mine) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xF70);               // vmcnt(0): sub-tile k+1 landed
        __builtin_amdgcn_sched_barrier(0);
        load_fa2();
      }
      if constexpr (!(ABL & 2)) bwd_rows(2, 4);
    } else if constexpr (!(ABL & 2)) {
      if (!bwd_done) bwd_rows(0, 4);
    }
  }

  // ---- fixed-order block reduction (as k_sweepm with VREM)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;
  constexpr int JC = JT * 16;
#pragma unroll
  for (int t = 0; t < JTV; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((size_t)w * JC + 16 * t + lh + 4 * i) * 16 + lr] = gacc[t][i];
  double* red2 = red + (size_t)NW * JC * 16;
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  double* red3 = red2 + (size_t)NW * 64 * 2;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) red3[((size_t)(w * 4 + lh) * 4 + jj) * 16 + lr] = gv[jj];
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  const int jv = 16 * JTV;
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
  if (tid < 2 * C) {
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}


// Ring depth of k_sweepm: slots of 16 rows per wave that fit SM_MINB blocks per CU, at most 6,
// DMAs in flight <= 63 (d = 100: NB = 1, two blocks per CU).
inline int sweepm_nb(int d, int minb = SM_MINB) {
  int nb = std::min(6, (160 * 1024 / minb - LG_TAB * 8) / (SM_W * sweepm_slot_bytes(d)));
  const int pt = ((SM_R * d * 8 + 1023) >> 10) + 1;
  while (nb > 2 && (nb - 2) * pt > 63) --nb;
  return nb;
}

}  // namespace stk
