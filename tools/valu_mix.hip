// Which vector instructions share gfx950's fp64 pipe with v_mfma_f64_16x16x4_f64?
//
// tools/mfma_overlap.hip showed that v_fma_f64 and the fp64 MFMA do not overlap (their times
// add).  The k_sweepe residual also issues 32-bit integer, fp32, conversion and select
// instructions; this measures, per instruction class, a VALU-only stream, an MFMA-only stream,
// and both (a) interleaved in ONE wave and (b) split over two waves of one SIMD (waves w and
// w + 4 of an 8-wave block share SIMD w).  time(both) ~ max(...) means the class runs beside
// the fp64 MFMAs; ~ sum means it competes for the same pipe.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize tools/valu_mix.hip -o tools/_bin/valu_mix
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
typedef double dbl4 __attribute__((ext_vector_type(4)));

enum Op { F64FMA, F32FMA, I32, CVT_F32_F64, CVT_F64_F32, CVT_F64_I32, CVT_I32_F64, SEL_CMP64, LDEXP64,
          RCP64, EXP32, RNDNE64, FREXP64, MOV64, F64ADD, NOP_OPS };
static const char* op_name[] = {"v_fma_f64", "v_fma_f32", "int32 add/xor/shift", "cvt_f32_f64 + and + or",
                                "cvt f32->f64->f32 + mul_f64", "cvt i32->f64->i32 + mul_f64 + add",
                                "ldexp_f64 + cvt_i32_f64 + and + or", "v_cmp_f64 + mul_f64 + 2 cndmask",
                                "v_ldexp_f64", "v_rcp_f64", "v_exp_f32", "v_rndne_f64 + add_f64",
                                "v_frexp_mant_f64 + add_f64", "int cmp + cndmask + add/shift", "v_add_f64"};

// one instruction of class OP applied to independent chain j; state kept in 64-bit registers
template <int OP>
__device__ __forceinline__ void step(double& x, float& f, int& k, double a, float af, int ai) {
  if constexpr (OP == F64FMA) x = fma(x, a, 1e-3);
  else if constexpr (OP == F64ADD) x = x + a;
  else if constexpr (OP == F32FMA) f = fmaf(f, af, 1e-3f);
  else if constexpr (OP == I32) k = (k + ai) ^ (k >> 3);
  else if constexpr (OP == CVT_F32_F64) {                            // cvt_f32_f64 + and + or
    const uint32_t u = __float_as_uint((float)x);
    x = __builtin_bit_cast(double, (uint64_t)(0x3FF00000u | (u & 0xFFFFFu)) << 32);
  }
  else if constexpr (OP == CVT_F64_F32) f = (float)((double)f * a);  // cvt pair + f64 mul
  else if constexpr (OP == CVT_F64_I32) k = (int)((double)k * a) + ai;   // cvt pair + f64 mul + add
  else if constexpr (OP == CVT_I32_F64) {                            // ldexp (x 1024) + cvt_i32_f64 + and + or
    const int t = (int)(x * 1024.0);
    x = __builtin_bit_cast(double, (uint64_t)(0x3FF00000u | ((uint32_t)t & 0xFFFFFu)) << 32);
  }
  else if constexpr (OP == SEL_CMP64) x = x > a ? x : 0.5 * x;       // cmp_f64 + mul + 2 cndmask
  else if constexpr (OP == LDEXP64) x = __builtin_amdgcn_ldexp(x, ai);
  else if constexpr (OP == RCP64) x = __builtin_amdgcn_rcp(x);
  else if constexpr (OP == EXP32) f = __builtin_amdgcn_exp2f(f);
  else if constexpr (OP == RNDNE64) x = __builtin_rint(x + a);
  else if constexpr (OP == FREXP64) x = __builtin_amdgcn_frexp_mant(x) + a;
  else if constexpr (OP == MOV64) { k = (k & 1) ? k + ai : (k >> 1); }   // lane-divergent select
}

// MODE bit 0: MFMAs (NA independent accumulators, 4 rounds per trip); bit 1: VALU (NV chains x
// 16 rounds per trip).  ROLE 0: every wave runs MODE; ROLE 1: waves 0-3 run the MFMA part of
// MODE and waves 4-7 its VALU part (one wave of each kind per SIMD)
template <int OP, int MODE, int ROLE, int NV = 8, int NA = 4>
__global__ __launch_bounds__(512) void k_mix(double* sink, int iters, double a, int ai) {
  const int w = threadIdx.x >> 6;
  const bool do_m = (MODE & 1) && (ROLE ? (w < 4) : true);
  const bool do_v = (MODE & 2) && (ROLE ? (w >= 4) : true);
  dbl4 acc[NA] = {};
  double x[NV];
  float f[NV];
  int k[NV];
  const double b = 1.0 + threadIdx.x * 1e-9;
  const float af = 0.999f;
#pragma unroll
  for (int j = 0; j < NV; ++j) { x[j] = 1.0 + j * 1e-3 + threadIdx.x * 1e-6; f[j] = 1.0f + j; k[j] = threadIdx.x + j; }
  for (int i = 0; i < iters; ++i) {
    if (do_m) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < NA; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    if (do_v) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int j = 0; j < NV; ++j) step<OP>(x[j], f[j], k[j], a, af, ai + r);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NA; ++j) s += acc[j][j & 3];
#pragma unroll
  for (int j = 0; j < NV; ++j) s += x[j] + f[j] + k[j];
  if (s == 12345.678) sink[blockIdx.x] = 1.0;
}

static hipEvent_t e0, e1;
static double* sink;

template <typename K>
static float timeit(K kern, int iters) {
  const int blocks = 256;                   // one 8-wave block per CU: two waves per SIMD
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, sink, iters, 0.999999, 3);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(512), 0, 0, sink, iters, 0.999999, 3);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

template <int OP>
static void row(int iters) {
  const float m = timeit(k_mix<OP, 1, 0>, iters);
  const float v = timeit(k_mix<OP, 2, 0>, iters);
  const float b = timeit(k_mix<OP, 3, 0>, iters);
  const float p = timeit(k_mix<OP, 3, 1>, iters);
  const float pm = timeit(k_mix<OP, 1, 1>, iters);    // the partner run's MFMA wave alone
  const float pv = timeit(k_mix<OP, 2, 1>, iters);    // its VALU wave alone
  // per SIMD per trip: 2 waves x 16 MFMA; VALU 2 waves x 128 instances
  const double cyc = 1e-3 / iters * 2.1e9;  // nominal clock for a rough per-trip cycle figure
  // serial fraction: (both - mfma) / valu; 1 = the VALU stream's time adds in full, 0 = hidden
  printf("%-34s 2 waves/SIMD: mfma %6.3f valu %6.3f both %6.3f (serial %5.2f) | 1+1 waves: mfma %6.3f valu %6.3f "
         "both %6.3f (serial %5.2f) | valu cyc/trip~%6.0f\n",
         op_name[OP], m, v, b, (b - std::max(m, v)) / std::min(m, v), pm, pv, p,
         (p - std::max(pm, pv)) / std::min(pm, pv), v * cyc);
}

int main() {
  hipMalloc(&sink, 1 << 20);
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 2000;
  printf("times in ms; 256 blocks x 8 waves, %d trips; per trip per SIMD: 32 MFMAs (64 cyc each) and/or "
         "2 x 128 VALU instances\n", iters);
  row<F64FMA>(iters);
  row<F64ADD>(iters);
  row<F32FMA>(iters);
  row<I32>(iters);
  row<CVT_F32_F64>(iters);
  row<CVT_F64_F32>(iters);
  row<CVT_F64_I32>(iters);
  row<CVT_I32_F64>(iters);
  row<SEL_CMP64>(iters);
  row<LDEXP64>(iters);
  row<RCP64>(iters);
  row<EXP32>(iters);
  row<RNDNE64>(iters);
  row<FREXP64>(iters);
  row<MOV64>(iters);
  return 0;
}
