// Types and helpers shared by the regression sweeps (sweep.hip: C != 16 and the 64-chain GEMM
// passes; sweep16.hip: the 16-chain fp64-MFMA sweep) and by the measurement tools in tools/.
#pragma once
#include "common.h"

namespace stk {

typedef double dbl2 __attribute__((ext_vector_type(2)));   // loads from any address space

struct SweepArgs {
  const ShardDev* shards;
  const double* q;        // [nshards*C][Dp] evaluation points
  double* partial;        // [nshards][G][C][PW]
  const int* req_step;    // nullptr: always run
  int step_id;
  int C, Dp, G, LD, PW;
  int shard0;             // first shard of this launch
  int Gs;                 // partial-buffer stride in chunks per shard (>= G)
  int* ran;               // optional: ran[step_id & 63] = 1 when any shard swept
  double* qT;             // v5 workspace: [nshards][KP][64] swizzled beta^T images (KP = d rounded to 32)
  double* R;              // v5 workspace: [nshards][Rrows][64] residuals d eta, swizzled rows
  int64_t Rrows;          // v5: rows of R per shard (n rounded up to 64)
};

__device__ __forceinline__ void wait_vmcnt(int n) {
  // s_waitcnt encoding (gfx9): vmcnt [3:0] + [15:14], expcnt [6:4] = 7, lgkmcnt [11:8] = 15
#define STK_VMCNT(N) case N: __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0xF70); break;
  switch (n) {   // vmcnt is 6 bits on gfx950: 0..63
    STK_VMCNT(0) STK_VMCNT(1) STK_VMCNT(2) STK_VMCNT(3) STK_VMCNT(4) STK_VMCNT(5) STK_VMCNT(6)
    STK_VMCNT(7) STK_VMCNT(8) STK_VMCNT(9) STK_VMCNT(10) STK_VMCNT(11) STK_VMCNT(12) STK_VMCNT(13)
    STK_VMCNT(14) STK_VMCNT(15) STK_VMCNT(16) STK_VMCNT(17) STK_VMCNT(18) STK_VMCNT(19) STK_VMCNT(20)
    STK_VMCNT(21) STK_VMCNT(22) STK_VMCNT(23) STK_VMCNT(24) STK_VMCNT(25) STK_VMCNT(26) STK_VMCNT(27)
    STK_VMCNT(28) STK_VMCNT(29) STK_VMCNT(30) STK_VMCNT(31) STK_VMCNT(32) STK_VMCNT(33) STK_VMCNT(34)
    STK_VMCNT(35) STK_VMCNT(36) STK_VMCNT(37) STK_VMCNT(38) STK_VMCNT(39) STK_VMCNT(40) STK_VMCNT(41)
    STK_VMCNT(42) STK_VMCNT(43) STK_VMCNT(44) STK_VMCNT(45) STK_VMCNT(46) STK_VMCNT(47) STK_VMCNT(48)
    STK_VMCNT(49) STK_VMCNT(50) STK_VMCNT(51) STK_VMCNT(52) STK_VMCNT(53) STK_VMCNT(54) STK_VMCNT(55)
    STK_VMCNT(56) STK_VMCNT(57) STK_VMCNT(58) STK_VMCNT(59) STK_VMCNT(60) STK_VMCNT(61) STK_VMCNT(62)
    STK_VMCNT(63)
    default: __builtin_amdgcn_s_waitcnt(0xF70); break;   // vmcnt(0)
  }
#undef STK_VMCNT
}

template <int N>
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0xF70); }

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int SM_W = 4;                 // waves per block (one per SIMD)
constexpr int SM_R = 16;                // rows per wave sub-tile = MFMA M (forward) and K (backward)
constexpr int SM_C = 16;                // chains per launch row = MFMA N
constexpr int SM_MINB = 2;              // blocks per CU: two waves per SIMD (one wave cannot cover the slot's DMA latency)
__host__ __device__ constexpr int sweepm_slot_bytes(int d) { return SM_R * d * 8 + 128; }

__device__ __forceinline__ dbl4 mfma_f64(double a, double b, dbl4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// 64-bit select as an integer bit blend (v_bfi_b32 x 2): a C++ conditional here lets the
// compiler sink a whole arm's arithmetic into an exec-masked branch, which serialises the
// four (row, chain) pairs of a lane instead of interleaving them
__device__ __forceinline__ double blend(uint32_t m, double a, double b) {   // m = ~0u: a, 0: b
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const uint64_t mm = ((uint64_t)m << 32) | m;
  return __builtin_bit_cast(double, (ua & mm) | (ub & ~mm));
}

// exp table: T_j = 2^(j/1024), j < 1024 (8 KB of LDS per workgroup)
constexpr int EX_TAB = 1024;
__device__ void exp_table_init(double* tab) {
  for (int i = threadIdx.x; i < EX_TAB; i += blockDim.x) tab[i] = exp2((double)i / (double)EX_TAB);
}

// Logistic residual v4: Stan 2.19's bernoulli_logit term and its derivative for one (row,
// chain), t = (2y - 1) eta:
//   t > 20:   lt = -exp(-t),             dv/sgn = exp(-t)
//   t < -20:  lt = t,                    dv/sgn = 1
//   else:     lt = -log1p(exp(-t)),      dv/sgn = exp(-t) / (exp(-t) + 1)
// computed branch-free from e = exp(-|t|) as lt = min(t, 0) - log1p(e), dv/sgn = (t < 0 ?
// 1/(1+e) : e/(1+e)); above 20 the smooth form differs from Stan's by <= e^2/2 < 2.2e-18.
// The kernel works with s = -t = (1 - 2y) eta, whose sign bit is eta's plus y << 31 (one
// v_lshl_add_u32: adding 2^31 to the high word flips the sign), and returns -dv the same way;
// the kernel negates the gradient sums once at the end.
//
// The log is not taken per element.  Per lane (one chain) the kernel keeps
//   lm = sum (t - |t|)              = 2 sum min(t, 0), exact per term, a NaN eta stays NaN
//   sp = prod (1 + e) - 1           one fma per element: sp <- sp (1 + e) + e
// and adds log1p(sp) to the lane's lp every 64 sub-tiles (256 elements: 1 + sp < 2^256, and
// every step adds at most eps of relative error to 1 + sp, so log1p(sp) is off by <= 256 eps
// absolute); lp = lm/2 - sum log1p(sp).  Rows with e below eps are summed exactly (1 + e = 1,
// sp += e).  Against residual v3 this drops the table log1p (its index, two LDS reads, a degree-4
// polynomial) and the per-element lp terms: ~27 instead of ~43 vector instructions per element.
//   exp(-a), a = min(|t|, 700): n = rint(-a 1024/ln2) by the 1.5 2^52 trick, r = -a - n ln2/1024
//   (|r| <= ln2/2048; ln2/1024 rounded once: |error of r| <= n ulp(ln2/1024)/2, 1.6e-15 relative at
//   a = 20), e^r by a fitted degree-3 polynomial (relative error 9.4e-17), times T_{n mod 1024}, times
//   2^{n div 1024} by v_ldexp_f64 -- whose exponent is -1100 for t < -20, making e = 0: then
//   lt = min(t, 0) = t and dv/sgn = 1/(1 + 0) = 1 exactly, Stan's lower branch;
//   1/(1 + e): v_rcp_f64 + one Newton step (11 ulp, tools/rcp_acc.hip).
__device__ __forceinline__ double fmin_abs(double x, double c) {   // min(|x|, c), NaN x -> c
  // one v_min_f64 with the abs modifier (fmin() adds a canonicalising v_max_f64 in IEEE mode)
  double r;
  asm("v_min_f64 %0, |%1|, %2" : "=v"(r) : "v"(x), "s"(c));
  return r;
}
__device__ __forceinline__ double logit_resid4(double eta, uint32_t y, const double* tab, double& lm, double& sp) {
  constexpr double MAGIC = 6755399441055744.0;            // 1.5 * 2^52
  constexpr double INV_L = 1477.3197218702985;            // 1024 / ln 2
  constexpr double L = 0.0006769015435155716;             // ln 2 / 1024
  constexpr double C2 = 0.5000000039583942, C3 = 0.16666666713444417;   // e^r on |r| <= ln2/2048 (fit)
  const uint64_t eb = __builtin_bit_cast(uint64_t, eta);
  const double s = __builtin_bit_cast(double, (eb & 0xFFFFFFFFull) | ((uint64_t)((y << 31) + (uint32_t)(eb >> 32)) << 32));
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
  return __builtin_bit_cast(double, (dvp & 0xFFFFFFFFull) | ((uint64_t)((y << 31) + (uint32_t)(dvp >> 32)) << 32));   // -dv
}

}  // namespace stk

// The 16-chain sweep (sweep16.hip): shapes it covers, its LDS bytes, its launch.
bool stk_sweep16_supported(int d);
size_t stk_sweep16_lds_bytes(int family, int d);
hipError_t stk_launch_sweep16(int family, const stk::SweepArgs& A, int d, int nblocks, size_t lds, hipStream_t st);
