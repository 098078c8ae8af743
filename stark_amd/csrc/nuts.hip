// Batched NUTS for gfx950: one wavefront per chain, an ITERATIVE per-chain state machine.
//
// Replaces Stan's hmc_nuts_diag_e_adapt, which stark runs once per Spark partition inside
// `sm.sampling(data=data, **kwargs)` (stark/stark.py:48).  Algorithm = Stan 2.19.1
// base_nuts::transition / build_tree (restated in oracle/stark_oracle.c, which keeps the
// recursive form), rewritten so that one call advances a chain by exactly ONE leapfrog step:
//
//   consume the gradient at the point requested last step
//     -> finish the leapfrog -> leaf bookkeeping -> merge completed sub-trees (binary
//        counter over the leaf index; pending left sub-trees live on a per-level stack)
//     -> top-level multinomial / U-turn / depth checks -> maybe end the transition
//        (draw, dual averaging, Welford windows, init_stepsize probes) and start the next
//     -> half-step p, full-step q, request the gradient at the new q.
//
// A chain that finishes its transition starts the next one on the very next step, so
// chains of one wave group never idle behind each other's tree depth (the SIMD-lockstep
// problem of recursive NUTS).  Lanes hold dimensions (64 per chunk, NCH chunks), every
// scalar is wave-uniform (reductions broadcast lane 0's value), and every uniform value
// is stored by all lanes, so each lane only ever re-reads its own writes.
//
// Two drivers share the state machine:
//   k_nuts_step   split mode: the gradient comes from the data-sweep kernels (sweep.hip),
//                 one launch per leapfrog for all chains of all local shards;
//   k_nuts_fused  local models (8 schools): the gradient is computed inline and each wave
//                 loops its own chain for up to max_steps leapfrogs in ONE launch.
#include "common.h"
#include <math.h>
#include <stdlib.h>
#include <algorithm>

namespace stk {

typedef double dbl2 __attribute__((ext_vector_type(2)));


// Lane exchange of a double by DPP (VALU, a few cycles; __shfl is a ds_bpermute round trip).
// bound_ctrl: an invalid source lane reads 0 -- the old value 0 would give the same, but as an
// operand it costs a v_mov of 0 into the destination before every DPP move.
template <int CTRL>
__device__ __forceinline__ double nuts_dpp(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Lane l's double, as a wave-uniform (scalar) value.
__device__ __forceinline__ double lane_d(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// Sum over the 64 lanes with identical bits in every lane: DPP within each 16-lane row (xor 1,
// xor 2, half-mirror, mirror -- every lane of a row ends with the same row total, addition
// being commutative), then the four row totals as scalars, added in row order.  The per-
// leapfrog state machine is a chain of these; the DPP form cut 8-schools time (configs[1]).
__device__ __forceinline__ double wave_sum(double v) {
  v += nuts_dpp<0xB1>(v);
  v += nuts_dpp<0x4E>(v);
  v += nuts_dpp<0x141>(v);
  v += nuts_dpp<0x140>(v);
  return (lane_d(v, 0) + lane_d(v, 16)) + (lane_d(v, 32) + lane_d(v, 48));
}

// Sum over a segment of SEG consecutive lanes (SEG chains' worth of lanes per wave when
// chains are packed, SEG = 64 / chains per wave): SEG = 64 is wave_sum; SEG = 16 is one DPP
// row (the row total of wave_sum's first four steps); SEG = 32 adds the partner row.  For
// D <= SEG the extra rows of wave_sum only add zeros, so the packed sums are bit-identical.
template <int SEG>
__device__ __forceinline__ double seg_sum(double v) {
  if constexpr (SEG == WAVE) {
    return wave_sum(v);
  } else {
    v += nuts_dpp<0xB1>(v);
    v += nuts_dpp<0x4E>(v);
    v += nuts_dpp<0x141>(v);
    v += nuts_dpp<0x140>(v);
    if constexpr (SEG == 32) v += __shfl_xor(v, 16);
    return v;
  }
}
// Lane L of this lane's segment, broadcast to the segment: a segment of 16 is one DPP row, so
// row_newbcast (a VALU move) instead of a ds_bpermute round trip through the LDS crossbar.
template <int SEG, int L>
__device__ __forceinline__ double seg_bcast(double v) {
  if constexpr (SEG == WAVE) {
    return lane_d(v, L);
  } else if constexpr (SEG == 16) {
    static_assert(L >= 0 && L < 16, "row_newbcast selects a lane of the row");
    return nuts_dpp<0x150 + L>(v);
  } else {
    return __shfl(v, ((int)threadIdx.x & (WAVE - SEG)) + L);
  }
}

__device__ __forceinline__ double log_sum_exp2(double a, double b) {   // stan::math::log_sum_exp
  if (a == -INFINITY) return b;
  if (a == INFINITY && b == INFINITY) return INFINITY;
  if (a > b) return a + log1p(exp(b - a));
  return b + log1p(exp(a - b));
}

// ------------------------------------------------------------------ table-driven exp / log1p
// The fused 8-schools kernel is a serial chain of dependent fp64 operations per leapfrog at one
// wave per SIMD, and ocml's f64 exp is ~35 vector instructions, log1p ~130 and a log_sum_exp
// ~180; a leaf takes 1-3 exps and a merge one log_sum_exp.  With a 5 KB table in the workgroup's
// LDS (MT_N doubles, filled once per launch):
//   exp_mt(x)       x = n ln2/128 + r (n = rint(x 128/ln2) by the 1.5 2^52 trick, ln2/128 in two
//                   parts so n L_HI is exact), e^r by its degree-5 Taylor polynomial (|r| <= ln2/256:
//                   truncation 5e-19), times 2^{(n mod 128)/128} from the table, times 2^{n div 128}
//                   by v_ldexp_f64; x clamped to [-800, 800] first (0 / inf beyond), NaN kept;
//   log1p01_mt(e)   e in [0, 1]: j = rint(128 e), rl = e c_j - d_j = (e - j/128) / (1 + j/128)
//                   (|rl| <= 1/256, exact for j = 0, so a tiny e keeps its relative accuracy),
//                   log1p(e) = log1p(j/128) + log1p(rl), the latter by its degree-7 Taylor series;
// about 20 and 14 instructions, errors of 1-2 ulp (tools/nuts_math_accuracy.py).  The recursive CPU
// twin (libm) and the GPU machine then differ by ulps in log weights and acceptance probabilities,
// as they already did with ocml's: a multinomial / acceptance decision flips only when the uniform
// lies within those ulps of the threshold.
constexpr int MT_E = 128;                    // T_j = 2^(j/128)
constexpr int MT_L = 129;                    // [c_j, d_j, l_j, 0], j = 0..128
constexpr int MT_N = MT_E + 4 * MT_L;
__device__ void mt_init(double* t, int tid, int nthreads) {
  for (int i = tid; i < MT_N; i += nthreads) {
    double v;
    if (i < MT_E) {
      v = exp2((double)i / (double)MT_E);
    } else {
      const int j = (i - MT_E) >> 2, f = (i - MT_E) & 3;
      v = f == 0 ? 128.0 / (128 + j) : (f == 1 ? (double)j / (128 + j) : (f == 2 ? log1p((double)j / 128.0) : 0.0));
    }
    t[i] = v;
  }
}
// The fp64 constants of the table math (and the leaf's divergence threshold) as values the
// compiler cannot see through: it then keeps each in a VGPR pair for the whole launch instead of
// rematerialising it with two s_mov_b32 at every use (fp64 has no literal operand in VOP3, and at
// one wave per SIMD every issued instruction costs the wave 4 cycles).  Same values, same
// operations: bit-identical results.
struct MtK {
  double lo, hi, inv_l, magic, l_hi, l_lo, c5, c4, c3, f128, q7, q6, q5, q4, q3, pinf, ninf, div;
};
__device__ __forceinline__ double opq(double v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ MtK mt_consts() {
  return MtK{opq(-800.0), opq(800.0),
             opq(184.6649652337873),         // 128 / ln 2
             opq(6755399441055744.0),        // 1.5 * 2^52
             opq(0.005415212348452769),      // ln2/128 to 32 significant bits
             opq(-3.2819649005320973e-13),   // ln2/128 - L_HI
             opq(1.0 / 120.0), opq(1.0 / 24.0), opq(1.0 / 6.0), opq(128.0),
             opq(1.0 / 7.0), opq(-1.0 / 6.0), opq(0.2), opq(-0.25), opq(1.0 / 3.0),
             opq(INFINITY), opq(-INFINITY), opq(1000.0)};
}
__device__ __forceinline__ double exp_mt(double x, const double* t, const MtK& k) {
  const double xc = fmin(fmax(x, k.lo), k.hi);
  const double sn = fma(xc, k.inv_l, k.magic);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = sn - k.magic;
  double r = fma(-n, k.l_hi, xc);
  r = fma(-n, k.l_lo, r);
  const double p = fma(fma(fma(fma(fma(k.c5, r, k.c4), r, k.c3), r, 0.5), r, 1.0), r, 1.0);
  const double e = __builtin_amdgcn_ldexp(t[ni & (MT_E - 1)] * p, ni >> 7);
  return x == x ? e : x;
}
__device__ __forceinline__ double log1p01_mt(double e, const double* t, const MtK& k) {   // e in [0, 1] (NaN kept)
  const int j = (int)fma(e, k.f128, 0.5);
  const double* cj = t + MT_E + 4 * j;
  const dbl2 cd = *reinterpret_cast<const dbl2*>(cj);
  const double rl = fma(e, cd.x, -cd.y);
  const double q = fma(fma(fma(fma(fma(fma(k.q7, rl, k.q6), rl, k.q5), rl, k.q4), rl, k.q3), rl, -0.5), rl, 1.0);
  return fma(rl, q, cj[2]);
}
// log_sum_exp_mt that also returns e = exp(-|a - b|), from which the merge's and the top level's
// acceptance probabilities follow without a second exp (see NutsChain::on_leaf)
__device__ __forceinline__ double log_sum_exp_mt_e(double a, double b, const double* t, const MtK& k, double& e) {
  e = exp_mt(-fabs(a - b), t, k);
  const double r = fmax(a, b) + log1p01_mt(e, t, k);
  const double r1 = (a == k.pinf && b == k.pinf) ? k.pinf : r;
  return a == k.ninf ? b : r1;
}
// The tree's own log_sum_exp (the merge of two sub-trees' log weights, and of the trajectory's
// with a new sub-tree's): both weights are finite there -- a divergent leaf (energy error > 1000
// or NaN) stops the transition before any merge -- so log_sum_exp2's two infinite cases cannot
// occur and their selects go; exp's argument -|a - b| is <= 0, so only the lower clamp stays;
// NaN still propagates (a NaN weight gives a NaN sum, as before).  At one wave per SIMD every
// issued instruction costs the wave 4 cycles, and this runs once per merge.
__device__ __forceinline__ double log_sum_exp_mt_e_tree(double a, double b, const double* t, const MtK& k, double& e) {
  const double x = -fabs(a - b);
  const double xc = fmax(x, k.lo);
  const double sn = fma(xc, k.inv_l, k.magic);
  const int ni = (int)(uint32_t)__builtin_bit_cast(uint64_t, sn);
  const double n = sn - k.magic;
  double r = fma(-n, k.l_hi, xc);
  r = fma(-n, k.l_lo, r);
  const double p = fma(fma(fma(fma(fma(k.c5, r, k.c4), r, k.c3), r, 0.5), r, 1.0), r, 1.0);
  const double ee = __builtin_amdgcn_ldexp(t[ni & (MT_E - 1)] * p, ni >> 7);
  e = x == x ? ee : x;
  return fmax(a, b) + log1p01_mt(e, t, k);
}
__device__ __forceinline__ double log_sum_exp_mt(double a, double b, const double* t, const MtK& k) {   // as log_sum_exp2
  // branch-free: max + log1p(exp(-|a - b|)), with log_sum_exp2's two special cases as selects
  // (a = -inf with b finite needs none: exp(-inf) = 0 gives b)
  const double r = fmax(a, b) + log1p01_mt(exp_mt(-fabs(a - b), t, k), t, k);
  const double r1 = (a == k.pinf && b == k.pinf) ? k.pinf : r;
  return a == k.ninf ? b : r1;
}

// ------------------------------------------------------------------ model hooks
// 8 schools (example/schools.stan:1-18): q = (mu, log tau, eta_1..J); returns lp, writes
// grad lp.  Mirrors oracle orc_schools_lpgrad.
// y_j and 1 / sigma_j of this lane's schools (element e = k SEG + lane is school e - 2), loaded
// once per launch instead of two global loads per leapfrog (their latency was on every
// leapfrog's critical path at one wave per SIMD).  normal_lpdf as Stan Math 2.18/2.19 computes
// it: inv_sigma = 1 / sigma once, then (y - theta) * inv_sigma and the partial inv_sigma * z --
// no division per leapfrog (oracle orc_schools_lpgrad does the same arithmetic).
template <int NCH, int SEG = WAVE>
__device__ __forceinline__ void schools_data(const ShardDev& sh, double (&yc)[NCH], double (&isc)[NCH], int lane, int D) {
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int e = k * SEG + lane;
    const bool in = e >= 2 && e < D;
    yc[k] = in ? sh.y[e - 2] : 0.0;
    isc[k] = in ? 1.0 / sh.sigma[e - 2] : 1.0;
  }
}
template <int NCH, int SEG = WAVE, bool FM = false>
__device__ double schools_lpgrad(const double (&yc)[NCH], const double (&isc)[NCH], const double (&q)[NCH],
                                 double (&glp)[NCH], int lane, int D, const double* mt = nullptr,
                                 const MtK* mk = nullptr) {
  const double mu = seg_bcast<SEG, 0>(q[0]);
  const double u = seg_bcast<SEG, 1>(q[0]);
  double tau;
  if constexpr (FM) tau = exp_mt(u, mt, *mk);
  else tau = exp(u);
  double lp = 0.0, smu = 0.0, su = 0.0;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int e = k * SEG + lane;
    glp[k] = 0.0;
    if (e >= 2 && e < D) {
      const double eta = q[k];
      const double theta = mu + tau * eta;
      const double z = (yc[k] - theta) * isc[k];
      const double r = isc[k] * z;
      lp += -0.5 * eta * eta - 0.5 * z * z;
      smu += r;
      su += r * eta;
      glp[k] = -eta + tau * r;
    }
  }
  lp = seg_sum<SEG>(lp) + u;
  smu = seg_sum<SEG>(smu);
  su = seg_sum<SEG>(su);
  if (lane == 0) glp[0] = smu;
  if (lane == 1) glp[0] = tau * su + 1.0;
  return lp;
}

// Cold paths of a transition's end, out of line: their transcendentals (Box-Muller's log / sqrt /
// sin / cos, dual averaging's pow / exp / sqrt) would otherwise add their temporaries to the
// register budget of the per-leapfrog loop they are inlined into.
// (normal_at's Box-Muller with one sincos: lanes of even and odd e share a wave, so a sin / cos
// branch would run both functions under complementary masks)
__device__ __noinline__ double momentum_cold(uint64_t seed, uint32_t rid, uint32_t c1, uint32_t c2hi, uint32_t e,
                                             uint32_t tag, double im) {
  const u64x2 r = philox(seed, rid, c1, c2hi | (e >> 1), tag);
  const double rad = sqrt(-2.0 * log(u53(r.a)));
  double sn, cs;
  sincos(6.283185307179586 * u53(r.b), &sn, &cs);
  return ((e & 1) ? rad * sn : rad * cs) / sqrt(im);
}
__device__ __noinline__ double exp_cold(double x) { return exp(x); }
__device__ __noinline__ double log_cold(double x) { return log(x); }
struct DaState { double sbar, xbar, nomeps; };
__device__ __noinline__ DaState dual_averaging_cold(double cnt, double sbar, double xbar, double mu, double adapt_stat,
                                                   double t0, double delta, double gamma, double kappa) {
  adapt_stat = adapt_stat > 1 ? 1 : adapt_stat;
  const double eta = 1.0 / (cnt + t0);
  sbar = (1.0 - eta) * sbar + eta * (delta - adapt_stat);
  const double x = mu - sbar * sqrt(cnt) / gamma;
  const double x_eta = pow(cnt, -kappa);
  xbar = (1.0 - x_eta) * xbar + x_eta * x;
  return DaState{sbar, xbar, exp(x)};
}

// Constrained output row (extract() order: params, transformed params, lp__).
template <int NCH, int SEG = WAVE>
__device__ __forceinline__ void write_draw(const NutsArgs& A, const ShardDev& sh, int shard, int col, const double (&q)[NCH],
                           double lp, int lane) {
  double* out = A.draws + (size_t)shard * A.Pmax * A.S_total;
  const int D = sh.D;
  const size_t S = (size_t)A.S_total;
  if (A.family == STK_SCHOOLS) {
    const double mu = seg_bcast<SEG, 0>(q[0]);
    const double tau = exp_cold(seg_bcast<SEG, 1>(q[0]));
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int e = k * SEG + lane;
      if (e < D) out[(size_t)e * S + col] = (e == 1) ? tau : q[k];
      if (e >= 2 && e < D) out[(size_t)(D + e - 2) * S + col] = mu + tau * q[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int e = k * SEG + lane;
      if (e < D) out[(size_t)e * S + col] = (A.family == STK_LINREG && e == D - 1) ? exp_cold(q[k]) : q[k];
    }
  }
  if (lane == 0) out[(size_t)(sh.P - 1) * S + col] = lp;
}

// ------------------------------------------------------------------ the chain
// SEG: lanes per chain (64: one chain per wave; 16 / 32: 4 / 2 chains packed in a wave, each
// in its own DPP row(s), D <= SEG).  `lane` is the lane's position inside its segment.
template <int NCH, int SEG = WAVE, bool FM = false, int UT = -1, bool ZP = false>
// UT: the U-turn criterion at compile time (0: Stan 2.19, 1: Stan >= 2.23's junction checks; -1: at
// run time from A.uturn_ext) -- a run-time branch on it splits the merge loop's basic block
// (every member is force-inlined: a non-inlined constructor or method receiving `this` puts
// the whole chain object -- s[], iv[], q, p, g -- in scratch memory; 48.7 -> 26.1 us per step,
// profiles/r02q_kernel_stats.csv vs r02r_kernel_stats_global.csv)
struct NutsChain {
  const NutsArgs& A;
  const int gid, lane, shard, cidx, D;
  const uint32_t rid;   // RNG stream id (global shard * chains + chain)
  const ShardDev& sh;
  double* const vec;
  double* const stk;
  double* const stks;
  // the per-transition scalars and counters live in registers; the ones touched only at a
  // transition's end or by adaptation (cold_s / cold_i) stay in memory -- the chain's global
  // block, or its LDS image in the fused kernel -- and are read and written in place
  double* const scold;
  int* const icold;
  double s[S_COUNT];
  int iv[I_COUNT];
  double q[NCH], p[NCH], g[NCH], im[NCH];
  const double* mt = nullptr;     // FM: the fused kernel's exp / log1p table in LDS (else ocml)
  MtK mk{};                       // FM: its constants, VGPR-resident (mt_consts)
  __device__ __forceinline__ double ex(double x) const {
    if constexpr (FM) return exp_mt(x, mt, mk);
    else return exp(x);
  }
  __device__ __forceinline__ double lse(double a, double b) const {
    if constexpr (FM) return log_sum_exp_mt(a, b, mt, mk);
    else return log_sum_exp2(a, b);
  }
  uint32_t nleap = 0, ndiv = 0;   // leapfrogs / divergent draws since the last flush_counts()

  __device__ __forceinline__ NutsChain(const NutsArgs& a, int gid_, int lane_)
      : NutsChain(a, gid_, lane_, a.vec + (size_t)gid_ * V_COUNT * a.Dp,
                  a.stk + (size_t)gid_ * a.max_depth * SV_COUNT * a.Dp, a.stks + (size_t)gid_ * a.max_depth * SS_COUNT,
                  a.sc + (size_t)gid_ * S_COUNT, a.iv + (size_t)gid_ * I_COUNT) {}
  // vec_ / stk_ / stks_ / scold_ / icold_: this chain's vector block, tree stack, stack scalars
  // and cold scalars / counters (global memory, or the fused kernel's LDS image).  No null
  // defaults: a select between an LDS and a global pointer leaves a generic pointer, and every
  // access through it a flat instruction (waits on both the vector-memory and the LDS counter)
  __device__ __forceinline__ NutsChain(const NutsArgs& a, int gid_, int lane_, double* vec_, double* stk_,
                                       double* stks_, double* scold_, int* icold_)
      : A(a), gid(gid_), lane(lane_), shard(gid_ / a.C), cidx(gid_ % a.C), D(a.shards[gid_ / a.C].D),
        rid(rng_stream(a, gid_)),
        sh(a.shards[gid_ / a.C]),
        vec(vec_),
        stk(stk_),
        stks(stks_),
        scold(scold_),
        icold(icold_) {}

  static constexpr bool cold_s(int i) {
    return i == S_VS || i == S_HS || i == S_NOMEPS || i == S_DA_CNT || i == S_SBAR || i == S_XBAR || i == S_MU ||
           i == S_WFN || i == S_PH0;
  }
  static constexpr bool cold_i(int i) {
    return i == I_PROBE || i == I_PDIR || i == I_SSCALL || i == I_SSREASON || i == I_WCNT || i == I_WSIZE ||
           i == I_WNEXT;
  }
  __device__ __forceinline__ double& S(int i) { return cold_s(i) ? scold[i] : s[i]; }
  __device__ __forceinline__ int& IV(int i) { return cold_i(i) ? icold[i] : iv[i]; }

  __device__ __forceinline__ bool uext() const {
    if constexpr (UT >= 0) return UT != 0;
    else return A.uturn_ext != 0;
  }
  __device__ __forceinline__ bool ok(int k) const { return k * SEG + lane < D; }
  // ZP (the fused kernel when a chain's segment spans exactly its vectors, Dp = SEG NCH): the lanes past D hold +0 in every vector register and in every padding slot of
  // the LDS image -- momenta are drawn as 0 there, the gradient is 0 there, and q, p, rho, p_sharp,
  // the Welford sums follow from them; the tree stack starts zeroed (stk_sampler_create) -- so the
  // LDS reads need no select, the stores no exec mask and the dot products no masked adds: the
  // padding lanes contribute exact zeros.  Vector arithmetic then uses okv() instead of ok().
  __device__ __forceinline__ bool okv(int k) const {
    if constexpr (FM && ZP) return true;
    else return ok(k);
  }
  // the vector stride: ZP runs only at Dp = SEG NCH, a compile-time constant, so every vector of
  // the LDS image sits at an immediate offset from one base (no per-vector address registers)
  __device__ __forceinline__ int dp() const {
    if constexpr (FM && ZP) return SEG * NCH;
    else return A.Dp;
  }
  __device__ __forceinline__ double* vp(int v) const { return vec + (size_t)v * dp(); }
  __device__ __forceinline__ double* svp(int level, int v) const {
    return stk + ((size_t)level * (uext() ? SV_COUNT : SV_PB) + v) * dp();   // stack_vecs(A)
  }
  // FM (the fused kernel, where every vector lives in the workgroup's LDS image): the load is
  // unconditional and lanes past D select 0 -- an exec-masked load would split the basic block
  // (s_cbranch_execz) and keep the compiler from interleaving a merge's independent chains.  Lanes
  // past D read inside the image (the next vector, the stack scalars, the next chain or the table).
  __device__ __forceinline__ void ld(const double* base, double (&r)[NCH]) const {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if constexpr (FM) {
        const double v = base[k * SEG + lane];
        r[k] = okv(k) ? v : 0.0;
      } else {
        r[k] = ok(k) ? base[k * SEG + lane] : 0.0;
      }
    }
  }
  __device__ __forceinline__ void ldg(const double* base, double (&r)[NCH]) const {   // global memory: masked
#pragma unroll
    for (int k = 0; k < NCH; ++k) r[k] = ok(k) ? base[k * SEG + lane] : 0.0;
  }
  __device__ __forceinline__ void st(double* base, const double (&r)[NCH]) const {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (okv(k)) base[k * SEG + lane] = r[k];
  }
  // The trajectory's vectors (z+, z-, the sample point, rho, p_sharp, the metric and its Welford
  // sums): RV (the fused kernel in its zero-padding form) keeps them in registers for the whole
  // launch -- at one wave per SIMD nothing hides an LDS round trip, and the register file has room
  // (the tree stack, indexed by level at run time, stays in LDS).  Otherwise they live at vp(v).
  // Every vector index below is a compile-time constant after inlining (a run-time index into rv
  // would put it in scratch); the two-way choices go through vld_sel / vst_sel.
  static constexpr bool RV = FM && ZP;
  double rv[RV ? V_COUNT : 1][NCH];
  __device__ __forceinline__ void vld(int v, double (&r)[NCH]) const {
    if constexpr (RV) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) r[k] = rv[v][k];
    } else {
      ld(vp(v), r);
    }
  }
  __device__ __forceinline__ void vst(int v, const double (&r)[NCH]) {
    if constexpr (RV) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) rv[v][k] = r[k];
    } else {
      st(vp(v), r);
    }
  }
  __device__ __forceinline__ void vld_sel(bool c, int va, int vb, double (&r)[NCH]) const {   // c ? va : vb
    if constexpr (RV) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) r[k] = c ? rv[va][k] : rv[vb][k];
    } else {
      ld(vp(c ? va : vb), r);
    }
  }
  __device__ __forceinline__ void vst_sel(bool c, int va, int vb, const double (&r)[NCH]) {   // into c ? va : vb
    if constexpr (RV) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        rv[va][k] = c ? r[k] : rv[va][k];
        rv[vb][k] = c ? rv[vb][k] : r[k];
      }
    } else {
      st(vp(c ? va : vb), r);
    }
  }
  // RV: the launch's copy of the vectors in and out of the chain's global block (Dp = SEG NCH: every
  // lane of every vector, padding zeros included)
  __device__ __forceinline__ void rv_in(const double* gvec) {
    if constexpr (RV) {
#pragma unroll
      for (int v = 0; v < V_COUNT; ++v)
#pragma unroll
        for (int k = 0; k < NCH; ++k) rv[v][k] = gvec[(size_t)v * dp() + k * SEG + lane];
    }
  }
  __device__ __forceinline__ void rv_out(double* gvec) const {
    if constexpr (RV) {
#pragma unroll
      for (int v = 0; v < V_COUNT; ++v)
#pragma unroll
        for (int k = 0; k < NCH; ++k) gvec[(size_t)v * dp() + k * SEG + lane] = rv[v][k];
    }
  }

  __device__ __forceinline__ void load() {
    load_scalars();
    load_vectors();
  }
  __device__ __forceinline__ void load_scalars() {
    const double* sc = A.sc + (size_t)gid * S_COUNT;
    const int* ivp = A.iv + (size_t)gid * I_COUNT;
#pragma unroll
    for (int i = 0; i < S_COUNT; ++i)
      if (!cold_s(i)) s[i] = sc[i];
#pragma unroll
    for (int i = 0; i < I_COUNT; ++i)
      if (!cold_i(i)) iv[i] = ivp[i];
  }
  __device__ __forceinline__ void load_vectors() {
    vld(V_Q, q);
    vld(V_P, p);
    vld(V_G, g);
    vld(V_IM, im);
  }
  __device__ __forceinline__ void flush_counts() {
    if (lane == 0 && (nleap | ndiv)) {
      A.cnt[(size_t)gid * C_COUNT + C_LEAP] += nleap;
      A.cnt[(size_t)gid * C_COUNT + C_DIV] += ndiv;
    }
    nleap = ndiv = 0;
  }
  __device__ __forceinline__ void save() {
    double* sc = A.sc + (size_t)gid * S_COUNT;
    int* ivp = A.iv + (size_t)gid * I_COUNT;
#pragma unroll
    for (int i = 0; i < S_COUNT; ++i)
      if (!cold_s(i)) sc[i] = s[i];
#pragma unroll
    for (int i = 0; i < I_COUNT; ++i)
      if (!cold_i(i)) ivp[i] = iv[i];
    vst(V_Q, q);
    vst(V_P, p);
    vst(V_G, g);
  }

  __device__ __forceinline__ double kinetic(const double (&pp)[NCH]) const {   // diag_e_metric::tau
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (okv(k)) t += pp[k] * im[k] * pp[k];
    return 0.5 * seg_sum<SEG>(t);
  }
  __device__ __forceinline__ bool criterion(const double (&psm)[NCH], const double (&psp)[NCH], const double (&rho)[NCH]) const {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (okv(k)) { a += psp[k] * rho[k]; b += psm[k] * rho[k]; }
    a = seg_sum<SEG>(a);
    b = seg_sum<SEG>(b);
    return a > 0 && b > 0;
  }
  // uniforms k = 2m and 2m + 1 of a transition come from one Philox block: the odd one is kept
  // from the even one's call (u_key = the block's (iteration, m) + 1; 0 = nothing kept)
  uint64_t u_odd = 0, u_key = 0;
  // FM (the fused kernel): the transition's uniforms come from a window of 2 SEG precomputed in
  // the chain's LDS slots ub[] -- lane l of the chain computes Philox block base/2 + l, so a
  // window costs ONE Philox latency for all its 2 SEG uniforms -- and uniform() is a branch-free
  // LDS read: the sub-tree merge loop is then one basic block whose chains (the stack loads and
  // U-turn sums, the log_sum_exp / exp, the uniform) the compiler can interleave.  Same counter
  // mapping as the direct form (uniform k = element k & 1 of block k >> 1): identical draws.
  double* ub = nullptr;
  int ub_base = 0;
  __device__ __forceinline__ void fill_uniforms(int base) {   // window [base, base + 2 SEG), base even
    const uint32_t it = (uint32_t)(IV(I_ITER) + A.iter_offset);
    const u64x2 r = philox(A.seed, rid, it, (uint32_t)(base >> 1) + (uint32_t)lane, TAG_UNI);
    const dbl2 v = {u53(r.a), u53(r.b)};
    *reinterpret_cast<dbl2*>(ub + 2 * lane) = v;
    ub_base = base;
  }
  // a step takes at most max_depth + 1 uniforms (merges, the top level, the next sub-tree's direction)
  __device__ __forceinline__ void ensure_uniforms() {
    if constexpr (FM) {
      const int k = IV(I_UK);
      if (k - ub_base + A.max_depth + 2 > 2 * SEG) fill_uniforms(k & ~1);
    }
  }
  __device__ __forceinline__ double uniform() {
    if constexpr (FM) {
      const int k = IV(I_UK)++;
      return ub[k - ub_base];
    }
    const uint32_t it = (uint32_t)(IV(I_ITER) + A.iter_offset);
    const uint32_t k = (uint32_t)IV(I_UK)++;
    const uint64_t key = (((uint64_t)it << 32) | (k >> 1)) + 1;
    if ((k & 1) && key == u_key) return u53(u_odd);
    const u64x2 r = philox(A.seed, rid, it, k >> 1, TAG_UNI);
    u_odd = r.b;
    u_key = key;
    return u53((k & 1) ? r.b : r.a);
  }
  __device__ __forceinline__ void sample_momentum(uint32_t c1, uint32_t c2hi, uint32_t tag) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int e = k * SEG + lane;
      p[k] = ok(k) ? momentum_cold(A.seed, rid, c1, c2hi, (uint32_t)e, tag, im[k]) : 0.0;
    }
  }
  __device__ __forceinline__ void load_sample_point() {
    vld(V_QS, q);
    vld(V_GS, g);
    S(S_V) = S(S_VS);
  }

  // Request = the new q after begin_update_p + update_q (expl_leapfrog).
  __device__ __forceinline__ void begin_leapfrog(double eps) {
    S(S_LFEPS) = eps;
    const double he = 0.5 * eps;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      p[k] -= he * g[k];
      q[k] += eps * (im[k] * p[k]);
    }
  }
  __device__ __forceinline__ void finish_leapfrog(double lp, const double (&glp)[NCH]) {
    const double he = 0.5 * S(S_LFEPS);
    S(S_V) = -lp;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      g[k] = -glp[k];
      p[k] -= he * g[k];
    }
  }

  // ---- init_stepsize (base_hmc) as a probe sequence, one leapfrog per step
  __device__ __forceinline__ bool start_probe() {
    const double e = S(S_NOMEPS);
    if (e == 0 || e > 1e7 || isnan(e)) return false;
    IV(I_PROBE) = 0;
    IV(I_MODE) = M_PROBE;
    load_sample_point();
    sample_momentum((uint32_t)IV(I_SSCALL), 0u, TAG_SSMOM);
    S(S_PH0) = S(S_V) + kinetic(p);
    begin_leapfrog(e);
    return true;
  }

  // ---- adaptation (stepsize_adaptation, windowed var_adaptation)
  __device__ __forceinline__ void learn_stepsize(double adapt_stat) {
    S(S_DA_CNT) += 1.0;
    const DaState r = dual_averaging_cold(S(S_DA_CNT), S(S_SBAR), S(S_XBAR), S(S_MU), adapt_stat, A.t0, A.delta,
                                          A.gamma, A.kappa);
    S(S_SBAR) = r.sbar;
    S(S_XBAR) = r.xbar;
    S(S_NOMEPS) = r.nomeps;
  }
  __device__ __forceinline__ bool learn_variance() {
    const unsigned cnt = (unsigned)IV(I_WCNT);
    const unsigned nw = (unsigned)A.num_warmup;
    const bool in_window = (cnt >= A.init_buffer) && (cnt < nw - A.term_buffer) && (cnt != nw);
    double wm[NCH], wm2[NCH];
    vld(V_WM, wm);
    vld(V_WM2, wm2);
    if (in_window) {
      double qs[NCH];
      vld(V_QS, qs);
      S(S_WFN) += 1.0;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const double delta = qs[k] - wm[k];
        wm[k] += delta / S(S_WFN);
        wm2[k] += (qs[k] - wm[k]) * delta;
      }
    }
    const bool end_window = (cnt == (unsigned)IV(I_WNEXT)) && (cnt != nw);
    if (end_window) {
      // compute_next_window
      const unsigned last = nw - A.term_buffer - 1;
      if ((unsigned)IV(I_WNEXT) != last) {
        unsigned size = (unsigned)IV(I_WSIZE) * 2;
        unsigned next = cnt + size;
        if (next != last) {
          const unsigned nb = next + 2 * size;
          if (nb >= nw - A.term_buffer) next = last;
        }
        IV(I_WSIZE) = (int)size;
        IV(I_WNEXT) = (int)next;
      }
      const double n = S(S_WFN);
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        double v = im[k];
        if (n > 1) v = wm2[k] / (n - 1.0);
        im[k] = (n / (n + 5.0)) * v + 1e-3 * (5.0 / (n + 5.0));
        wm[k] = 0.0;
        wm2[k] = 0.0;
      }
      S(S_WFN) = 0.0;
      vst(V_IM, im);
    }
    vst(V_WM, wm);
    vst(V_WM2, wm2);
    IV(I_WCNT) = (int)(cnt + 1);
    return end_window;
  }

  // ---- transitions
  __device__ __forceinline__ void begin_subtree() {
    IV(I_DIR) = uniform() > 0.5 ? 1 : -1;
    const int f = IV(I_DIR) > 0;
    vld_sel(f, V_QF, V_QB, q);
    vld_sel(f, V_PF, V_PB, p);
    vld_sel(f, V_GF, V_GB, g);
    S(S_V) = f ? S(S_VF) : S(S_VB);
    IV(I_LEAF) = 0;
    begin_leapfrog(IV(I_DIR) * S(S_EPS));
  }

  __device__ __forceinline__ void start_transition() {
    IV(I_MODE) = M_TRAJ;
    S(S_EPS) = S(S_NOMEPS);   // base_hmc::sample_stepsize; jitter on its own stream (TAG_JIT)
    if (A.jitter > 0)
      S(S_EPS) *= 1.0 + A.jitter * (2.0 * uniform_at(A.seed, rid, (uint32_t)(IV(I_ITER) + A.iter_offset), 0u, TAG_JIT) - 1.0);
    IV(I_UK) = 0;
    if constexpr (FM) fill_uniforms(0);
    load_sample_point();
    sample_momentum((uint32_t)(IV(I_ITER) + A.iter_offset), 0u, TAG_MOM);
    const double H0 = S(S_V) + kinetic(p);
    S(S_H0) = H0;
    S(S_HS) = H0;
    vst(V_QF, q); vst(V_PF, p); vst(V_GF, g);
    vst(V_QB, q); vst(V_PB, p); vst(V_GB, g);
    S(S_VF) = S(S_V);
    S(S_VB) = S(S_V);
    double ps[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) ps[k] = im[k] * p[k];
    vst(V_PSP, ps);
    vst(V_PSM, ps);
    vst(V_RHO, p);
    S(S_LSW) = 0.0;
    S(S_SUMMETRO) = 0.0;
    IV(I_NLEAP) = 0;
    IV(I_DEPTH) = 0;
    IV(I_DIV) = 0;
    begin_subtree();
  }

  // After a transition (or its adaptation probes): stop, pause or go on.  Returns true
  // if a gradient request was issued.
  __device__ __forceinline__ bool continue_or_stop(int pause_at) {
    if (IV(I_ITER) >= A.total_iters) { IV(I_MODE) = M_DONE; return false; }
    if (IV(I_ITER) >= pause_at) { IV(I_MODE) = M_PAUSED; return false; }
    start_transition();
    return true;
  }

  __device__ __forceinline__ bool end_transition(int pause_at) {
    const double accept = S(S_SUMMETRO) / (double)IV(I_NLEAP);
    const int it = IV(I_ITER);
    if (it >= A.ud_first) {
      double qs[NCH];
      vld(V_QS, qs);
      st(A.udraws + ((size_t)gid * A.ud_iters + (it - A.ud_first)) * A.Dp, qs);
    }
    if (it >= A.num_warmup) {
      const int col = cidx * A.num_samples + (it - A.num_warmup);
      double qs[NCH];
      vld(V_QS, qs);
      write_draw<NCH, SEG>(A, sh, shard, col, qs, -S(S_VS), lane);
      if (lane < N_STATS) {
        double v = 0;
        switch (lane) {
          case 0: v = accept; break;
          case 1: v = S(S_EPS); break;
          case 2: v = (double)IV(I_DEPTH); break;
          case 3: v = (double)IV(I_NLEAP); break;
          case 4: v = (double)IV(I_DIV); break;
          default: v = S(S_HS); break;
        }
        A.stats[((size_t)shard * A.S_total + col) * N_STATS + lane] = v;
      }
      if (IV(I_DIV)) ++ndiv;
    }
    bool update = false;
    if (A.adapt && it < A.num_warmup) {
      learn_stepsize(accept);
      if (A.var_on) update = learn_variance();
    }
    IV(I_ITER) = it + 1;
    if (update) {
      IV(I_SSREASON) = (A.adapt && it + 1 == A.num_warmup) ? 2 : 1;
      if (start_probe()) return true;
      finish_window_update();
    } else if (A.adapt && it + 1 == A.num_warmup) {
      S(S_NOMEPS) = exp_cold(S(S_XBAR));   // complete_adaptation
    }
    return continue_or_stop(pause_at);
  }

  __device__ __forceinline__ void finish_window_update() {
    S(S_MU) = log_cold(10.0 * S(S_NOMEPS));
    S(S_DA_CNT) = 0.0;
    S(S_SBAR) = 0.0;
    S(S_XBAR) = 0.0;
    if (IV(I_SSREASON) == 2) S(S_NOMEPS) = exp_cold(S(S_XBAR));
  }

  __device__ __forceinline__ bool on_probe(double lp, const double (&glp)[NCH], int pause_at) {
    finish_leapfrog(lp, glp);
    double h = S(S_V) + kinetic(p);
    if (isnan(h)) h = INFINITY;
    const double dH = S(S_PH0) - h;
    const double l08 = log(0.8);
    bool more = true;
    if (IV(I_PROBE) == 0) {
      IV(I_PDIR) = dH > l08 ? 1 : -1;
    } else if ((IV(I_PDIR) == 1 && !(dH > l08)) || (IV(I_PDIR) == -1 && !(dH < l08))) {
      more = false;
    } else {
      S(S_NOMEPS) = IV(I_PDIR) == 1 ? 2 * S(S_NOMEPS) : 0.5 * S(S_NOMEPS);
      if (S(S_NOMEPS) > 1e7 || S(S_NOMEPS) == 0) {
        IV(I_MODE) = M_ERROR;
        load_sample_point();
        return false;
      }
    }
    if (more) {
      IV(I_PROBE) += 1;
      load_sample_point();
      sample_momentum((uint32_t)IV(I_SSCALL), (uint32_t)IV(I_PROBE) << 12, TAG_SSMOM);
      S(S_PH0) = S(S_V) + kinetic(p);
      begin_leapfrog(S(S_NOMEPS));
      return true;
    }
    IV(I_SSCALL) += 1;
    load_sample_point();
    if (IV(I_SSREASON) >= 1) finish_window_update();
    return continue_or_stop(pause_at);
  }

  __device__ __forceinline__ bool on_leaf(double lp, const double (&glp)[NCH], int pause_at) {
    finish_leapfrog(lp, glp);
    ++nleap;
    const double H0 = S(S_H0);
    double h = S(S_V) + kinetic(p);
    if constexpr (FM) {
      if (isnan(h)) h = mk.pinf;
      if ((h - H0) > mk.div) IV(I_DIV) = 1;
    } else {
      if (isnan(h)) h = INFINITY;
      if ((h - H0) > 1000.0) IV(I_DIV) = 1;
    }
    IV(I_NLEAP) += 1;
    S(S_SUMMETRO) += (H0 - h > 0) ? 1.0 : ex(H0 - h);
    // the leaf as a depth-0 sub-tree
    double c_lsw = H0 - h;
    double c_rho[NCH], c_psb[NCH], c_pse[NCH], c_q[NCH], c_g[NCH], c_pb[NCH];
    double c_V = S(S_V), c_H = h;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      c_rho[k] = p[k];
      c_psb[k] = im[k] * p[k];
      c_pse[k] = c_psb[k];
      c_q[k] = q[k];
      c_g[k] = g[k];
      c_pb[k] = p[k];
    }
    // every way out that ends the transition leaves through ONE end_transition call after the
    // tree code (a divergent leaf, a U-turn inside a merge, the top level): an inlined call
    // inside the merge loop made the loop body carry end_transition's code and registers (27
    // register copies and the structurizer's mask juggling per merge in the fused kernel's ISA)
    bool stop = IV(I_DIV) != 0;
    const int depth = IV(I_DEPTH);
    const int n = IV(I_LEAF);
    int j = 0;
    while (!stop && j < depth && ((n >> j) & 1)) {
      // merge pending left sub-tree (level j) with the just-completed right one
      const double l_lsw = stks[j * SS_COUNT + SS_LSW];
      double l_rho[NCH], l_psb[NCH];
      ld(svp(j, SV_RHO), l_rho);
      ld(svp(j, SV_PSB), l_psb);
      double lsw_sub;
      bool take_right;
      const double u = uniform();
      if constexpr (FM) {
        // exp(c_lsw - lsw_sub) = 1 / (1 + exp(l_lsw - c_lsw)): with e = exp(-|l_lsw - c_lsw|) from
        // the log_sum_exp, u < 1/(1 + e) (c >= l) or e/(1 + e) (c < l), compared without a division
        // (c_lsw > lsw_sub never holds); the same decision up to the last bits of the probability
        double e;
        lsw_sub = log_sum_exp_mt_e_tree(l_lsw, c_lsw, mt, mk, e);
        take_right = u * (1.0 + e) < (c_lsw >= l_lsw ? 1.0 : e);
      } else {
        lsw_sub = lse(l_lsw, c_lsw);
        take_right = (c_lsw > lsw_sub) || (u < ex(c_lsw - lsw_sub));
      }
      if constexpr (FM) {   // the left sub-tree's sample read unconditionally and selected: no branch
        double l_q[NCH], l_g[NCH];
        ld(svp(j, SV_Q), l_q);
        ld(svp(j, SV_G), l_g);
        const double l_V = stks[j * SS_COUNT + SS_V], l_H = stks[j * SS_COUNT + SS_H];
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          c_q[k] = take_right ? c_q[k] : l_q[k];
          c_g[k] = take_right ? c_g[k] : l_g[k];
        }
        c_V = take_right ? c_V : l_V;
        c_H = take_right ? c_H : l_H;
      } else if (!take_right) {
        ld(svp(j, SV_Q), c_q);
        ld(svp(j, SV_G), c_g);
        c_V = stks[j * SS_COUNT + SS_V];
        c_H = stks[j * SS_COUNT + SS_H];
      }
      bool junction_ok = true;
      if (uext()) {
        // Stan >= 2.23: the left half extended by the right half's first momentum, and the
        // right half extended by the left half's last momentum, must not turn either
        double l_pb[NCH], l_pe[NCH], l_pse[NCH], e1[NCH], e2[NCH];
        ld(svp(j, SV_PB), l_pb);
        ld(svp(j, SV_PE), l_pe);
        ld(svp(j, SV_PSE), l_pse);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          e1[k] = l_rho[k] + c_pb[k];
          e2[k] = c_rho[k] + l_pe[k];
          c_pb[k] = l_pb[k];
        }
        const bool ok2 = criterion(l_psb, c_psb, e1);
        const bool ok3 = criterion(l_pse, c_pse, e2);
        junction_ok = ok2 && ok3;
      }
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        c_rho[k] = l_rho[k] + c_rho[k];
        c_psb[k] = l_psb[k];
      }
      c_lsw = lsw_sub;
      const bool ok1 = criterion(l_psb, c_pse, c_rho);
      stop = !ok1 || !junction_ok;
      ++j;
    }
    if (!stop && j < depth) {
      // push the completed sub-tree as the pending left sub-tree of level j
      st(svp(j, SV_RHO), c_rho);
      st(svp(j, SV_PSB), c_psb);
      st(svp(j, SV_Q), c_q);
      st(svp(j, SV_G), c_g);
      if (uext()) {
        st(svp(j, SV_PB), c_pb);
        st(svp(j, SV_PE), p);          // its last leaf is the latest one
        st(svp(j, SV_PSE), c_pse);
      }
      stks[j * SS_COUNT + SS_LSW] = c_lsw;
      stks[j * SS_COUNT + SS_V] = c_V;
      stks[j * SS_COUNT + SS_H] = c_H;
      IV(I_LEAF) = n + 1;
      begin_leapfrog(IV(I_DIR) * S(S_EPS));
      return true;
    }
    if (!stop) {
      // the top-level sub-tree of this depth is complete and valid
      const int fwd = IV(I_DIR) > 0;
      double o_p[NCH], o_ps[NCH];     // the old trajectory's end next to the new sub-tree
      if (uext()) {
        vld_sel(fwd, V_PF, V_PB, o_p);
        vld_sel(fwd, V_PSP, V_PSM, o_ps);
      }
      vst_sel(fwd, V_QF, V_QB, q);
      vst_sel(fwd, V_PF, V_PB, p);
      vst_sel(fwd, V_GF, V_GB, g);
      // (no run-time index into the register arrays: that would move them to scratch)
      S(S_VF) = fwd ? S(S_V) : S(S_VF);
      S(S_VB) = fwd ? S(S_VB) : S(S_V);
      IV(I_DEPTH) = depth + 1;
      const double u = uniform();
      bool take;
      double lsw_new;
      if constexpr (FM) {   // one exp for both: e = exp(-|c_lsw - lsw|) is exp(c_lsw - lsw) when c_lsw <= lsw
        double e;
        lsw_new = log_sum_exp_mt_e_tree(S(S_LSW), c_lsw, mt, mk, e);
        take = c_lsw > S(S_LSW) || u < e;
      } else {
        take = c_lsw > S(S_LSW) || u < ex(c_lsw - S(S_LSW));
        lsw_new = lse(S(S_LSW), c_lsw);
      }
      double rho[NCH], psp[NCH], psm[NCH], rho_old[NCH];
      if constexpr (FM) {   // branch-free: the sample point rewritten with a select (LDS image)
        double o_q[NCH], o_g[NCH], nq[NCH], ng[NCH];
        vld(V_QS, o_q);
        vld(V_GS, o_g);
        vld(V_RHO, rho);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          nq[k] = take ? c_q[k] : o_q[k];
          ng[k] = take ? c_g[k] : o_g[k];
        }
        vst(V_QS, nq);
        vst(V_GS, ng);
        S(S_VS) = take ? c_V : S(S_VS);
        S(S_HS) = take ? c_H : S(S_HS);
      } else {
        if (take) {
          vst(V_QS, c_q);
          vst(V_GS, c_g);
          S(S_VS) = c_V;
          S(S_HS) = c_H;
        }
        vld(V_RHO, rho);
      }
      S(S_LSW) = lsw_new;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        rho_old[k] = rho[k];
        rho[k] = rho[k] + c_rho[k];
      }
      vst(V_RHO, rho);
      if constexpr (FM) {   // the end this sub-tree extends gets its p_sharp; the other end's is read
        double oth[NCH];
        vst_sel(fwd, V_PSP, V_PSM, c_pse);
        vld_sel(fwd, V_PSM, V_PSP, oth);
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          psp[k] = fwd ? c_pse[k] : oth[k];
          psm[k] = fwd ? oth[k] : c_pse[k];
        }
      } else if (fwd) {
        vst(V_PSP, c_pse);
#pragma unroll
        for (int k = 0; k < NCH; ++k) psp[k] = c_pse[k];
        vld(V_PSM, psm);
      } else {
        vst(V_PSM, c_pse);
#pragma unroll
        for (int k = 0; k < NCH; ++k) psm[k] = c_pse[k];
        vld(V_PSP, psp);
      }
      bool junction_ok = true;
      if (uext()) {
        // the new sub-tree against the old trajectory across their junction (base_nuts::transition)
        double e1[NCH], e2[NCH];
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          e1[k] = fwd ? rho_old[k] + c_pb[k] : c_rho[k] + o_p[k];
          e2[k] = fwd ? c_rho[k] + o_p[k] : rho_old[k] + c_pb[k];
        }
        const bool ok2 = fwd ? criterion(psm, c_psb, e1) : criterion(c_pse, o_ps, e1);
        const bool ok3 = fwd ? criterion(o_ps, c_pse, e2) : criterion(c_psb, psp, e2);
        junction_ok = ok2 && ok3;
      }
      stop = !junction_ok || !criterion(psm, psp, rho) || IV(I_DEPTH) >= A.max_depth;
      if (!stop) {
        begin_subtree();
        return true;
      }
    }
    return end_transition(pause_at);
  }

  // Consume the evaluation requested last step.  Returns true if a new request (at q) was issued.
  __device__ __forceinline__ bool consume(double lp, const double (&glp)[NCH], int pause_at) {
    switch (IV(I_MODE)) {
      case M_INIT: {
        S(S_V) = -lp;
#pragma unroll
        for (int k = 0; k < NCH; ++k) g[k] = -glp[k];
        vst(V_QS, q);
        vst(V_GS, g);
        S(S_VS) = S(S_V);
        IV(I_SSREASON) = 0;
        if (!A.skip_ss && start_probe()) return true;
        return continue_or_stop(pause_at);
      }
      case M_PROBE: return on_probe(lp, glp, pause_at);
      case M_TRAJ: return on_leaf(lp, glp, pause_at);
      default: return false;
    }
  }

  __device__ __forceinline__ bool resume(int pause_at) {   // PAUSED -> next transition
    if (IV(I_MODE) != M_PAUSED) return false;
    return continue_or_stop(pause_at);
  }
};

// ------------------------------------------------------------------ kernels
#ifndef STK_NUTS_FUSED4_TU
__global__ __launch_bounds__(64) void k_nuts_init(NutsArgs A, const double* init, const double* inv_metric,
                                                  double stepsize, double init_radius) {
  const int gid = blockIdx.x, lane = threadIdx.x;
  const ShardDev& sh = A.shards[gid / A.C];
  const int D = sh.D;
  double* vec = A.vec + (size_t)gid * V_COUNT * A.Dp;
  for (int v = 0; v < V_COUNT; ++v)
    for (int e = lane; e < A.Dp; e += WAVE) vec[(size_t)v * A.Dp + e] = 0.0;
  for (int e = lane; e < A.Dp; e += WAVE) {
    double q0 = 0.0, imv = 1.0;
    if (e < D) {
      q0 = init ? init[(size_t)gid * D + e]
                : -init_radius + 2.0 * init_radius * uniform_at(A.seed, rng_stream(A, gid), 0u, (uint32_t)e, TAG_INIT);
      if (inv_metric) imv = inv_metric[e];
    }
    vec[(size_t)V_Q * A.Dp + e] = q0;
    vec[(size_t)V_QS * A.Dp + e] = q0;
    vec[(size_t)V_IM * A.Dp + e] = imv;
    A.qeval[(size_t)gid * A.Dp + e] = q0;
  }
  double* sc = A.sc + (size_t)gid * S_COUNT;
  for (int i = lane; i < S_COUNT; i += WAVE) sc[i] = 0.0;
  int* ivp = A.iv + (size_t)gid * I_COUNT;
  for (int i = lane; i < I_COUNT; i += WAVE) ivp[i] = 0;
  for (int i = lane; i < C_COUNT; i += WAVE) A.cnt[(size_t)gid * C_COUNT + i] = 0;
  __syncthreads();
  if (lane == 0) {
    sc[S_NOMEPS] = stepsize;
    sc[S_EPS] = stepsize;
    sc[S_MU] = log(10.0 * stepsize);
    ivp[I_MODE] = M_INIT;
    ivp[I_WCNT] = 0;
    ivp[I_WSIZE] = (int)A.base_window;
    ivp[I_WNEXT] = (int)(A.init_buffer + A.base_window - 1);
    A.cnt[(size_t)gid * C_COUNT + C_GRAD] = 1;   // the evaluation at q0
    A.req_step[gid / A.C] = -1;
  }
}

#endif  // STK_NUTS_FUSED4_TU
template <int NCH>
__global__ __launch_bounds__(64) void k_nuts_step(NutsArgs A, int step_id, int pause_at) {
  const int gid = blockIdx.x, lane = threadIdx.x;
  NutsChain<NCH> ch(A, gid, lane);
  ch.load();
  const int mode = ch.IV(I_MODE);
  if (mode == M_DONE || mode == M_ERROR) return;
  bool req;
  if (mode == M_PAUSED) {
    if (ch.IV(I_ITER) >= pause_at) return;
    req = ch.resume(pause_at);
  } else {
    double glp[NCH];
    ch.ld(A.g_in + (size_t)gid * A.Dp, glp);
    req = ch.consume(A.lp_in[gid], glp, pause_at);
  }
  ch.save();
  ch.flush_counts();
  if (req) {
    ch.st(A.qeval + (size_t)gid * A.Dp, ch.q);
    A.req_step[ch.shard] = step_id;
    if (lane == 0) A.cnt[(size_t)gid * C_COUNT + C_GRAD] += 1;
  }
}

// The chain's vector block and tree stack live in LDS for the whole launch (copied in and
// out once): the state machine's per-leapfrog bookkeeping (z+/z-, sample point, rho, p#,
// Welford sums, the pending sub-tree stack) then costs LDS instead of L2/HBM round trips.
// CPW chains share a wave (SEG = 64 / CPW lanes each, D <= SEG): at D = 10 (8 schools) one
// chain per wave leaves 54 of 64 lanes idle, four per wave leave 24.  Every chain still runs
// its own state machine; lanes of one chain always take the same branch, and the segmented
// sums stay inside a chain's DPP row(s), so chains in other states never interfere.
template <int NCH, int CPW, int MINW = 1, int UT = 0, bool ZP = false>
__global__ __launch_bounds__(64, MINW) void k_nuts_fused_schools(NutsArgs A, int pause_at, int max_steps) {
  constexpr int SEG = WAVE / CPW;
  static_assert(CPW == 1 || NCH == 1, "packed chains hold one chunk of lanes each");
  const int seg = (int)threadIdx.x / SEG, lane = (int)threadIdx.x % SEG;
  const int gid = blockIdx.x * CPW + seg;
  const bool live = gid < A.nchains;
  extern __shared__ double fl_all[];
  const int dpk = ZP ? SEG * NCH : A.Dp;                 // ZP: Dp = SEG NCH at compile time
  const size_t nv = (size_t)V_COUNT * dpk, ns = (size_t)A.max_depth * stack_vecs(A) * dpk;
  const size_t nss = (size_t)A.max_depth * SS_COUNT;
  constexpr size_t nsc = S_COUNT + (I_COUNT + 1) / 2;   // the chain's scalars and counters
  const size_t nvl = ZP ? 0 : nv;                        // ZP: the vectors are in registers (NutsChain::RV)
  const size_t per = (nvl + ns + nss + nsc + 2 * SEG + 1) & ~(size_t)1;   // per-chain image + uniform window, even
  double* const fl = fl_all + (size_t)seg * per;
  double* const mtab = fl_all + (size_t)CPW * per;                   // exp / log1p table (MT_N doubles)
  mt_init(mtab, (int)threadIdx.x, WAVE);
  double* const lsc = fl + nvl + ns + nss;
  int* const liv = (int*)(lsc + S_COUNT);
  double* const gvec = A.vec + (size_t)gid * nv;
  double* const gstk = A.stk + (size_t)gid * A.max_depth * SV_COUNT * A.Dp;   // (allocation stride; ns used)
  double* const gstks = A.stks + (size_t)gid * nss;
  bool run = live;
  if (run) {
    const int mode0 = A.iv[(size_t)gid * I_COUNT + I_MODE];
    run = !(mode0 == M_DONE || mode0 == M_ERROR);
  }
  if (run) {
    for (size_t i = lane; i < nvl; i += SEG) fl[i] = gvec[i];
    for (size_t i = lane; i < ns; i += SEG) fl[nvl + i] = gstk[i];
    for (size_t i = lane; i < nss; i += SEG) fl[nvl + ns + i] = gstks[i];
    for (int i = lane; i < S_COUNT; i += SEG) lsc[i] = A.sc[(size_t)gid * S_COUNT + i];
    for (int i = lane; i < I_COUNT; i += SEG) liv[i] = A.iv[(size_t)gid * I_COUNT + i];
  }
  __syncthreads();
  if (run) {
    NutsChain<NCH, SEG, true, UT, ZP> ch(A, gid, lane, fl, fl + nvl, fl + nvl + ns, lsc, liv);
    ch.mt = mtab;
    ch.mk = mt_consts();
    ch.ub = fl + ((nvl + ns + nss + nsc + 1) & ~(size_t)1);   // after the chain's image, 16-B aligned: 2 SEG doubles
    ch.rv_in(gvec);
    ch.load();
    ch.fill_uniforms(ch.IV(I_UK) & ~1);                // the current transition's window (a resumed chain)
    double yc[NCH], isc[NCH];
    schools_data<NCH, SEG>(ch.sh, yc, isc, lane, ch.D);
    const int mode = ch.IV(I_MODE);
    bool req = false, go = true;
    if (mode == M_PAUSED) {
      if (ch.IV(I_ITER) >= pause_at) {
        go = false;
      } else {
        req = ch.resume(pause_at);
        if (req && lane == 0) A.cnt[(size_t)gid * C_COUNT + C_GRAD] += 1;
      }
    } else {
      ch.ldg(A.qeval + (size_t)gid * A.Dp, ch.q);  // the pending request
      req = true;
    }
    if (go) {
      int steps = 0;
      unsigned long long ngrad = 0;
      while (req && steps < max_steps) {
        double glp[NCH];
        ch.ensure_uniforms();
        const double lp = schools_lpgrad<NCH, SEG, true>(yc, isc, ch.q, glp, lane, ch.D, mtab, &ch.mk);
        ++steps;
        req = ch.consume(lp, glp, pause_at);
        if (req) ++ngrad;
      }
      ch.save();
      ch.rv_out(gvec);
      ch.flush_counts();
      if (req) ch.st(A.qeval + (size_t)gid * A.Dp, ch.q);
      if (lane == 0) A.cnt[(size_t)gid * C_COUNT + C_GRAD] += ngrad;
    } else {
      run = false;                                  // paused at its target: nothing changed
    }
  }
  __syncthreads();
  if (run) {
    for (size_t i = lane; i < nvl; i += SEG) gvec[i] = fl[i];
    for (size_t i = lane; i < ns; i += SEG) gstk[i] = fl[nvl + i];
    for (size_t i = lane; i < nss; i += SEG) gstks[i] = fl[nvl + ns + i];
    for (int i = lane; i < S_COUNT; i += SEG)
      if (NutsChain<NCH, SEG>::cold_s(i)) A.sc[(size_t)gid * S_COUNT + i] = lsc[i];
    for (int i = lane; i < I_COUNT; i += SEG)
      if (NutsChain<NCH, SEG>::cold_i(i)) A.iv[(size_t)gid * I_COUNT + i] = liv[i];
  }
}

// lp / gradient of the 8-schools density at C points of one shard (parity hook).
template <int NCH>
__global__ __launch_bounds__(64) void k_schools_lpgrad(const ShardDev* shards, int shard, const double* q, int Dp,
                                                       double* lp, double* g) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const ShardDev& sh = shards[shard];
  double qq[NCH], gl[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int e = k * WAVE + lane;
    qq[k] = e < sh.D ? q[(size_t)c * Dp + e] : 0.0;
  }
  double yc[NCH], isc[NCH];
  schools_data<NCH>(sh, yc, isc, lane, sh.D);
  const double v = schools_lpgrad<NCH>(yc, isc, qq, gl, lane, sh.D);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int e = k * WAVE + lane;
    if (e < sh.D) g[(size_t)c * Dp + e] = gl[k];
  }
  if (lane == 0) lp[c] = v;
}

}  // namespace stk

// ------------------------------------------------------------------ launchers
using namespace stk;

template <int NCH>
static hipError_t launch_step_t(const NutsArgs& A, int step_id, int pause_at, hipStream_t st) {
  hipLaunchKernelGGL(k_nuts_step<NCH>, dim3(A.nchains), dim3(64), 0, st, A, step_id, pause_at);
  return hipGetLastError();
}
template <int NCH, int CPW, int MINW = 1, int UT = 0, bool ZP = false>
static hipError_t launch_fused_zp(const NutsArgs& A, int pause_at, int max_steps, hipStream_t st) {
  constexpr int SEG = WAVE / CPW;
  size_t per = (ZP ? 0 : (size_t)V_COUNT * A.Dp) +   // ZP: the vectors are in registers (NutsChain::RV)
               (size_t)A.max_depth * stack_vecs(A) * A.Dp + (size_t)A.max_depth * SS_COUNT +
               S_COUNT + (I_COUNT + 1) / 2 + 2 * SEG;  // + the chain's uniform window
  per += per & 1;                                        // keep the table after the chains 16-B aligned
  const size_t lds = sizeof(double) * (CPW * per + MT_N);
  if (lds > 64 * 1024) {
    // the attribute is per device (allow_big_lds keys it on the current one); a failure is
    // reported as such rather than as a generic launch failure
    if (const hipError_t e = allow_big_lds((const void*)k_nuts_fused_schools<NCH, CPW, MINW, UT, ZP>)) return e;
  }
  hipLaunchKernelGGL((k_nuts_fused_schools<NCH, CPW, MINW, UT, ZP>), dim3((A.nchains + CPW - 1) / CPW), dim3(64), lds,
                     st, A, pause_at, max_steps);
  return hipGetLastError();
}
// The zero-padding form (NutsChain ZP) where a chain's segment spans its vectors: 4 chains per wave
// at Dp = 16 (8 schools, J = 8..14).  It is instantiated in its own translation unit,
// nuts_fused4.hip (this file with STK_NUTS_FUSED4_TU), so that it alone is built with LLVM's
// iterative ILP scheduler (Makefile): that experimental scheduler gains it 2-3 % but has crashed
// the compiler on other instantiations of this file.
hipError_t stk_launch_fused4_zp(const NutsArgs& A, int pause_at, int max_steps, hipStream_t st);
#ifdef STK_NUTS_FUSED4_TU
hipError_t stk_launch_fused4_zp(const NutsArgs& A, int pause_at, int max_steps, hipStream_t st) {
  return A.uturn_ext ? launch_fused_zp<1, 4, 1, 1, true>(A, pause_at, max_steps, st)
                     : launch_fused_zp<1, 4, 1, 0, true>(A, pause_at, max_steps, st);
}
#else
template <int NCH, int CPW, int MINW = 1, int UT = 0>
static hipError_t launch_fused_ut(const NutsArgs& A, int pause_at, int max_steps, hipStream_t st) {
  if constexpr (CPW == 4 && NCH == 1) {
    if (A.Dp == WAVE / CPW) return stk_launch_fused4_zp(A, pause_at, max_steps, st);
  }
  return launch_fused_zp<NCH, CPW, MINW, UT, false>(A, pause_at, max_steps, st);
}
template <int NCH, int CPW, int MINW = 1>
static hipError_t launch_fused_t(const NutsArgs& A, int pause_at, int max_steps, hipStream_t st) {
  return A.uturn_ext ? launch_fused_ut<NCH, CPW, MINW, 1>(A, pause_at, max_steps, st)
                     : launch_fused_ut<NCH, CPW, MINW, 0>(A, pause_at, max_steps, st);
}

// chains per wave of the fused 8-schools kernel: 4 for D <= 16, 2 for D <= 32, capped by the
// sampler's chains_per_wave (stk_config; 0 = no cap)
static int fused_cpw(const NutsArgs& A) {
  int c = A.Dp <= 16 ? 4 : (A.Dp <= 32 ? 2 : 1);
  if (A.cpw_cap > 0) c = std::min(c, A.cpw_cap);
  return c;
}

int stk_nch_for(int Dmax) {
  if (Dmax <= 64) return 1;
  if (Dmax <= 128) return 2;
  if (Dmax <= 256) return 4;
  if (Dmax <= 1024) return 16;
  return -1;
}

hipError_t stk_launch_nuts_init(const NutsArgs& A, const double* init, const double* inv_metric, double stepsize,
                                double init_radius, hipStream_t st) {
  hipLaunchKernelGGL(k_nuts_init, dim3(A.nchains), dim3(64), 0, st, A, init, inv_metric, stepsize, init_radius);
  return hipGetLastError();
}

hipError_t stk_launch_nuts_step(const NutsArgs& A, int nch, int step_id, int pause_at, hipStream_t st) {
  switch (nch) {
    case 1: return launch_step_t<1>(A, step_id, pause_at, st);
    case 2: return launch_step_t<2>(A, step_id, pause_at, st);
    case 4: return launch_step_t<4>(A, step_id, pause_at, st);
    case 16: return launch_step_t<16>(A, step_id, pause_at, st);
  }
  return hipErrorInvalidValue;
}

hipError_t stk_launch_nuts_fused(const NutsArgs& A, int nch, int pause_at, int max_steps, hipStream_t st) {
  if (nch == 1) {
    switch (fused_cpw(A)) {
      case 4: return launch_fused_t<1, 4>(A, pause_at, max_steps, st);
      case 2: return launch_fused_t<1, 2>(A, pause_at, max_steps, st);
      default: return launch_fused_t<1, 1>(A, pause_at, max_steps, st);
    }
  }
  if (nch == 2) return launch_fused_t<2, 1>(A, pause_at, max_steps, st);
  return hipErrorInvalidValue;
}

hipError_t stk_launch_schools_lpgrad(const ShardDev* shards, int shard, int nch, const double* q, int C, int Dp,
                                     double* lp, double* g, hipStream_t st) {
  if (nch == 1)
    hipLaunchKernelGGL(k_schools_lpgrad<1>, dim3(C), dim3(64), 0, st, shards, shard, q, Dp, lp, g);
  else if (nch == 2)
    hipLaunchKernelGGL(k_schools_lpgrad<2>, dim3(C), dim3(64), 0, st, shards, shard, q, Dp, lp, g);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
#endif  // STK_NUTS_FUSED4_TU
