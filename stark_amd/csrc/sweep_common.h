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

}  // namespace stk

// The 16-chain sweep (sweep16.hip): shapes it covers, its LDS bytes, its launch.
bool stk_sweep16_supported(int d);
size_t stk_sweep16_lds_bytes(int family, int d);
hipError_t stk_launch_sweep16(int family, const stk::SweepArgs& A, int d, int nblocks, size_t lds, hipStream_t st);
