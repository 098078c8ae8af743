// Philox4x32-10 counter-based RNG (Salmon et al., SC'11) for gfx950 kernels and host code.
// Every random number in the sampler is a pure function of (seed, counter), so the
// 1-GPU and N-GPU runs of the same shards draw identical streams.  Stream layout
// (DESIGN.md "RNG streams"):
//   TAG_INIT  ctr = {chain_gid, 0,         i/2,               TAG}  init q_i ~ U(-R, R)
//   TAG_MOM   ctr = {chain_gid, iteration, i/2,               TAG}  momentum (Box-Muller)
//   TAG_UNI   ctr = {chain_gid, iteration, k/2,               TAG}  k-th uniform of a transition
//   TAG_SSMOM ctr = {chain_gid, ss_call,   probe<<12 | i/2,   TAG}  init_stepsize momenta
//   TAG_JIT   ctr = {chain_gid, iteration, 0,                 TAG}  stepsize jitter of a transition
//   TAG_X     ctr = {row_lo, row_hi,       j/2,               TAG}  synthetic X_ij
//   TAG_Y     ctr = {row_lo, row_hi,       0,                 TAG}  synthetic y_i noise
//   TAG_BETA  ctr = {j/2, 0, 0, TAG}                                 synthetic beta_j
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define STK_HD __host__ __device__ __forceinline__

namespace stk {

enum : uint32_t { TAG_INIT = 0x1, TAG_MOM = 0x2, TAG_UNI = 0x3, TAG_SSMOM = 0x4, TAG_JIT = 0x5,
                  TAG_X = 0x10, TAG_Y = 0x11, TAG_BETA = 0x12 };

struct u64x2 { uint64_t a, b; };

STK_HD u64x2 philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u64x2 r;
  r.a = ((uint64_t)c1 << 32) | c0;
  r.b = ((uint64_t)c3 << 32) | c2;
  return r;
}

// 53-bit uniform on (0, 1).
STK_HD double u53(uint64_t x) { return ((double)(x >> 11) + 0.5) * 0x1.0p-53; }

STK_HD double uniform_at(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t idx, uint32_t tag) {
  u64x2 r = philox(seed, c0, c1, idx >> 1, tag);
  return u53((idx & 1) ? r.b : r.a);
}

STK_HD double normal_at(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2hi, uint32_t idx, uint32_t tag) {
  u64x2 r = philox(seed, c0, c1, c2hi | (idx >> 1), tag);
  double u1 = u53(r.a), u2 = u53(r.b);
  double rad = sqrt(-2.0 * log(u1));
  double th = 6.283185307179586 * u2;
  return (idx & 1) ? rad * sin(th) : rad * cos(th);
}

}  // namespace stk
