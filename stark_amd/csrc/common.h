// Internal types shared by the gfx950 kernels and the C-ABI layer of libstark_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include <set>
#include <utility>
#include "philox.h"
#include "../../include/stark_hip.h"

namespace stk {

typedef __attribute__((address_space(3))) void* lds_vptr;
// Buffer descriptor built from readfirstlane'd inputs, so the compiler can prove it
// wave-uniform and keeps it in SGPRs (no waterfall loop around every buffer op).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, nb, 0x00020000);
}

constexpr int WAVE = 64;

// Pointers fetched from device structs are generic to the compiler: loads through them
// become flat_load (counted on both vmcnt and lgkmcnt, so every LDS wait drains them).
// Casting to the global address space restores global_load with independent counters.
template <class T>
using gptr_t = const __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr_t<T> gp(const T* p) { return (gptr_t<T>)p; }

// Read-only data at wave-uniform addresses through the constant address space: the
// compiler emits scalar loads (s_load, lgkmcnt) that never wait on in-flight vector loads.
template <class T>
using cptr_t = const __attribute__((address_space(4))) T*;
template <class T>
__device__ __forceinline__ cptr_t<T> cp(const T* p) { return (cptr_t<T>)p; }

// A value the compiler cannot prove wave-uniform (e.g. threadIdx.x >> 6), made uniform.
__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// One data shard resident in HBM (copied or generated once, then streamed every sweep).
struct ShardDev {
  const double* x;      // n x d row-major (regressions)
  const double* y;      // schools y / linreg y
  const int32_t* yi;    // logreg y
  const double* sigma;  // schools sigma
  int64_t n;            // rows (J for schools)
  int d;                // covariates
  int D;                // unconstrained dimension
  int P;                // output columns (params + transformed params + lp__)
  double pa, pb;        // regressions: prior precisions 1/s^2 of alpha ~ normal(0, s_a), beta ~ normal(0, s_b) (0: flat)
};

// Workspace of the two-pass (v5, 64-chain) sweep: beta^T images and the residual matrix.
struct SweepWs {
  double* qT;       // [nshards][KP][64]
  double* R;        // [nshards][Rrows][64]
  int64_t Rrows;    // rows per shard, n rounded up to 64
};

// ---- per-chain NUTS state (global memory, one block of Dp-strided vectors per chain)
enum Vec : int {
  V_Q, V_P, V_G,        // current integration point z (g = dV/dq = -grad lp)
  V_QF, V_PF, V_GF,     // z_plus  (forward end of the trajectory)
  V_QB, V_PB, V_GB,     // z_minus (backward end)
  V_QS, V_GS,           // z_sample (also the init point of init_stepsize probes)
  V_RHO, V_PSP, V_PSM,  // trajectory rho, p_sharp at the + / - ends
  V_IM,                 // diagonal inverse metric
  V_WM, V_WM2,          // Welford mean / M2
  V_COUNT
};
// pending left subtree per level; SV_PB / SV_PE / SV_PSE (its first / last momentum and last
// p_sharp) serve the Stan >= 2.23 checks across subtree junctions (nuts_criterion = 1)
enum StackVec : int { SV_RHO, SV_PSB, SV_Q, SV_G, SV_PB, SV_PE, SV_PSE, SV_COUNT };
enum Scal : int {
  S_V, S_VF, S_VB, S_VS, S_HS, S_H0, S_LSW, S_EPS, S_NOMEPS, S_SUMMETRO,
  S_DA_CNT, S_SBAR, S_XBAR, S_MU, S_WFN, S_PH0, S_LFEPS, S_COUNT
};
enum StackScal : int { SS_LSW, SS_V, SS_H, SS_COUNT };
enum IVar : int {
  I_MODE, I_ITER, I_DEPTH, I_DIR, I_LEAF, I_UK, I_NLEAP, I_DIV, I_PROBE, I_PDIR,
  I_SSCALL, I_SSREASON, I_WCNT, I_WSIZE, I_WNEXT, I_COUNT
};
enum Mode : int { M_INIT = 0, M_PROBE = 1, M_TRAJ = 2, M_PAUSED = 3, M_DONE = 4, M_ERROR = 5 };
enum Counter : int { C_GRAD, C_LEAP, C_DIV, C_COUNT };
constexpr int N_STATS = 6;

struct NutsArgs {
  int nchains, C, Dp, family;
  int max_depth, num_warmup, num_samples, total_iters;
  int adapt, var_on, skip_ss, iter_offset;
  unsigned init_buffer, term_buffer, base_window;
  double delta, gamma, kappa, t0;
  uint64_t seed;
  int S_total, Pmax;
  const ShardDev* shards;
  double* vec;      // nchains * V_COUNT * Dp
  double* stk;      // nchains * max_depth * SV_COUNT * Dp
  double* sc;       // nchains * S_COUNT
  double* stks;     // nchains * max_depth * SS_COUNT
  int* iv;          // nchains * I_COUNT
  unsigned long long* cnt;  // nchains * C_COUNT
  double* qeval;    // nchains * Dp   requested evaluation points
  double* lp_in;    // nchains        lp at the requested points
  double* g_in;     // nchains * Dp   grad lp at the requested points
  double* draws;    // nshards * Pmax * S_total   (P x S per shard, chain-major columns)
  double* stats;    // nshards * S_total * N_STATS
  double* udraws;   // nchains * ud_iters * Dp  (unconstrained draws)
  int ud_first;     // first transition index stored in udraws (num_warmup, or 0 with save_warmup)
  int ud_iters;     // transitions stored per chain
  int* req_step;    // nshards: last step index that issued a request for the shard
  const int* shard_ids;  // nullptr or global shard index per local shard (RNG stream keys)
  double jitter;         // stepsize_jitter (0: off)
  int uturn_ext;         // nuts_criterion: 1 = Stan >= 2.23 extra U-turn checks
  int cpw_cap;           // chains_per_wave cap of the fused 8-schools kernel (0: none)
};

// Stack vectors per level in use: the Stan >= 2.23 junction checks need SV_PB / SV_PE / SV_PSE,
// Stan 2.19 only the first four (the smaller stride keeps the fused 8-schools kernel's LDS
// image, and with it its occupancy, at the 2.19 size).
__host__ __device__ inline int stack_vecs(const NutsArgs& A) { return A.uturn_ext ? SV_COUNT : SV_PB; }

// RNG stream of a chain: global shard index * chains + chain.
__host__ __device__ inline uint32_t rng_stream(const NutsArgs& A, int gid) {
  const int s = gid / A.C;
  return (uint32_t)((A.shard_ids ? A.shard_ids[s] : s) * A.C + gid % A.C);
}

// Raise a kernel's dynamic-LDS limit to the CU's 160 KiB.  The attribute is per device, so it
// is set once per (current device, kernel); a failure is returned to the launch that needed it.
inline hipError_t allow_big_lds(const void* kern) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({dev, kern})) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess) done.insert({dev, kern});
  return e;
}

}  // namespace stk

// Error plumbing for the C-ABI layer.
void stk_set_error(const char* fmt, ...);
#define STK_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      stk_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
      return STK_E_HIP;                                                            \
    }                                                                              \
  } while (0)
