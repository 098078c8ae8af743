// Micro-benchmark of the logistic data sweep against two ceilings on the same buffers:
//   stream   plain dwordx4 read of every shard (one contiguous chunk per workgroup, the
//            sweep's chunking), 8 loads in flight per thread: the HBM read ceiling;
//   skeleton v2's tile pipeline (register prefetch one tile ahead, LDS staging, 4 barriers
//            per tile) with the arithmetic removed;
//   sweep    the product kernel (stk_launch_sweep, variant per STARK_SWEEP=1|2|3 / shape), all
//            shards in one launch.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sweep_micro.hip -o tools/_bin/sweep_micro
// Run:   tools/_bin/sweep_micro [rows_per_shard] [shards] [d] [reps]
#include "../stark_amd/csrc/sweep.hip"
#include "sweep_variants.hip"
#include "../stark_amd/csrc/datagen.hip"
#include <stdarg.h>
#include <stdio.h>
#include <vector>

void stk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
}

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

namespace stk {

__global__ __launch_bounds__(256) void k_stream(const ShardDev* shards, int G, double* sink) {
  const int shard = blockIdx.x / G, chunk = blockIdx.x % G;
  const ShardDev sh = shards[shard];
  const int64_t n2 = sh.n * sh.d / 2;                 // dbl2 elements of the shard
  const int64_t e0 = n2 * chunk / G, e1 = n2 * (chunk + 1) / G;
  const gptr_t<dbl2> src = (gptr_t<dbl2>)gp(sh.x);
  dbl2 acc = {0.0, 0.0};
  int64_t e = e0 + threadIdx.x;
  for (; e + 7 * 256 < e1; e += 8 * 256) {
    dbl2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[e + k * 256];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  for (; e < e1; e += 256) acc += src[e];
  if (acc.x == 12345.678) sink[blockIdx.x] = acc.y;   // never true: keeps the loads
}

// fp64 MFMA issue rate: 4 independent accumulators per wave, back to back.
__global__ __launch_bounds__(256) void k_mfma_peak(double* sink, int iters) {
  dbl4 acc[4] = {};
  const double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-6;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = mfma_f64(a, b, acc[j]);
  }
  if (acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3] == 12345.678) sink[blockIdx.x] = 1.0;
}

template <int NT_ROWS>
__global__ __launch_bounds__(256, 2) void k_skeleton(SweepArgs A, double* sink) {
  constexpr int T = NT_ROWS, NT = 256;
  constexpr int NVMAX = (T * 128 / 2 + NT - 1) / NT;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, LD = A.LD, tid = threadIdx.x;
  const int64_t r0 = sh.n * chunk / A.G, r1 = sh.n * (chunk + 1) / A.G;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* Xs = lds;
  const gptr_t<double> X = gp(sh.x);
  dbl2 buf[NVMAX];
  const int64_t ntiles = (r1 - r0 + T - 1) / T;
  const int step = 2 * NT, dq = step / d, dr = step % d;
  auto issue = [&](int64_t rs) {
    const int64_t rws = (r1 - rs) < T ? (r1 - rs) : T;
    const int64_t nvec = rws * d / 2;
    const gptr_t<dbl2> src = (gptr_t<dbl2>)(X + rs * d);
#pragma unroll
    for (int v = 0; v < NVMAX; ++v)
      if ((int64_t)(tid + NT * v) < nvec) buf[v] = src[tid + NT * v];
  };
  double acc = 0.0;
  if (ntiles > 0) issue(r0);
  for (int64_t t = 0; t < ntiles; ++t) {
    const int64_t row_start = r0 + t * T;
    const int rows = (int)((r1 - row_start) < T ? (r1 - row_start) : T);
    {
      const int nel = rows * d;
      int e = 2 * tid, row = e / d, col = e % d;
#pragma unroll
      for (int v = 0; v < NVMAX; ++v) {
        if (e < nel) {
          double* dst = Xs + row * LD + col;
          dst[0] = buf[v].x;
          dst[1] = buf[v].y;
        }
        e += step;
        row += dq;
        col += dr;
        if (col >= d) { col -= d; ++row; }
      }
    }
    __syncthreads();
    if (t + 1 < ntiles) issue(row_start + T);
    acc += Xs[(tid & 63) * LD + (tid >> 6)];
    __syncthreads();
    __syncthreads();
    __syncthreads();
  }
  if (acc == 12345.678) sink[blockIdx.x] = acc;
}

// v3's DMA ring (buffer_load ... lds, counted vmcnt, raw barrier) with the arithmetic removed.
__global__ __launch_bounds__(512) void k_skel3(SweepArgs A, int NB, double* sink) {
  constexpr int T = S3_T, NW = S3_W;
  const int shard = blockIdx.x / A.G, chunk = blockIdx.x % A.G;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, K = d >> 1;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int64_t nt = (sh.n + T - 1) / T;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * T, r1 = std::min<int64_t>(sh.n, t1 * T);
  const int ntiles = (int)(t1 - t0);
  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const ring = reinterpret_cast<char*>(lds);
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (r1 - r0) * d * 8);
  const int nblk = K;
  const int lo_n = nblk / NW;
  auto issue = [&](int t) {
    const int slot = t % NB;
    for (int j = w; j < nblk; j += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(ring + ((size_t)slot * K + j) * 1024), 16, lane * 16,
                                               t * (T * 16 * K) + j * 1024, 0, 0);
  };
  double acc = 0.0;
  for (int t = 0; t < NB - 1 && t < ntiles; ++t) issue(t);
  for (int t = 0; t < ntiles; ++t) {
    const int later = std::min(NB - 2, ntiles - 1 - t);
    wait_vmcnt(later * lo_n);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NB - 1 < ntiles) issue(t + NB - 1);
    const double* xs = reinterpret_cast<const double*>(ring + (size_t)(t % NB) * K * 1024);
    acc += xs[tid];
  }
  if (acc == 12345.678) sink[blockIdx.x] = acc;
}

}  // namespace stk

int main(int argc, char** argv) {
  if (const char* e = getenv("STARK_SWEEP")) stk_sweep_force_variant = atoi(e);   // this tool only
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 12500000;
  const int nsh = argc > 2 ? atoi(argv[2]) : 4;
  const int d = argc > 3 ? atoi(argv[3]) : 100;
  const int reps = argc > 4 ? atoi(argv[4]) : 10;
  const int C = argc > 5 ? atoi(argv[5]) : 4, Dp = (d + 1 + 7) / 8 * 8;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<ShardDev> sh(nsh);
  std::vector<double> beta(d);
  for (int j = 0; j < d; ++j) beta[j] = ((j * 37) % 19 - 9) / (9.0 * sqrt((double)d));
  double* beta_d;
  CK(hipMalloc(&beta_d, sizeof(double) * d));
  CK(hipMemcpy(beta_d, beta.data(), sizeof(double) * d, hipMemcpyHostToDevice));
  for (int s = 0; s < nsh; ++s) {
    double* X;
    int32_t* y;
    CK(hipMalloc(&X, sizeof(double) * rows * d));
    CK(hipMalloc(&y, sizeof(int32_t) * rows));
    CK(stk_launch_gen_shard(X, nullptr, y, rows, d, s * rows, 20240, 0.0, beta_d, 1.0, STK_LOGREG, st));
    sh[s] = ShardDev{X, nullptr, y, nullptr, rows, d, d + 1, d + 2};
  }
  ShardDev* sh_d;
  CK(hipMalloc(&sh_d, sizeof(ShardDev) * nsh));
  CK(hipMemcpy(sh_d, sh.data(), sizeof(ShardDev) * nsh, hipMemcpyHostToDevice));
  std::vector<double> qh((size_t)nsh * C * Dp, 0.0);
  for (int g = 0; g < nsh * C; ++g)
    for (int j = 0; j < d; ++j) qh[(size_t)g * Dp + 1 + j] = beta[j] * (0.9 + 0.01 * g);
  double *q, *partial, *lp, *grad, *sink;
  CK(hipMalloc(&q, sizeof(double) * qh.size()));
  CK(hipMemcpy(q, qh.data(), sizeof(double) * qh.size(), hipMemcpyHostToDevice));
  int T, LD, G;
  size_t lds;
  stk_sweep_geometry(rows, d, &T, &LD, &G, &lds, C);
  CK(hipMalloc(&partial, sizeof(double) * (size_t)nsh * G * C * (d + 2)));
  const size_t wsb = stk_sweep_ws_bytes(rows, d, C, nsh);
  SweepWs ws{};
  if (wsb) {
    void* wp;
    CK(hipMalloc(&wp, wsb));
    ws = stk_sweep_ws(wp, rows, d, nsh);
  }
  const SweepWs* wsp = wsb ? &ws : nullptr;
  CK(hipMalloc(&lp, sizeof(double) * nsh * C));
  CK(hipMalloc(&grad, sizeof(double) * nsh * C * Dp));
  CK(hipMalloc(&sink, sizeof(double) * nsh * G));
  CK(hipStreamSynchronize(st));
  const double bytes = (double)nsh * rows * (8.0 * d + 4.0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double nbytes, auto&& launch) {
    launch();
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-10s %8.3f ms  %7.1f GB/s  %.3f of 8 TB/s\n", name, ms, nbytes / ms / 1e6, nbytes / ms / 1e6 / 8000.0);
    fflush(stdout);
  };
  printf("rows/shard %lld shards %d d %d C %d: T %d LD %d G %d lds %zu\n", (long long)rows, nsh, d, C, T, LD, G, lds);
  timeit("stream", (double)nsh * rows * 8.0 * d, [&] {
    hipLaunchKernelGGL(k_stream, dim3(nsh * G), dim3(256), 0, st, sh_d, G, sink);
  });
  SweepArgs A{sh_d, q, partial, nullptr, 0, C, Dp, G, d | 1, d + 2, 0, G, nullptr};
  hipFuncSetAttribute((const void*)k_skeleton<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if ((size_t)64 * (d | 1) * 8 <= 160 * 1024)
    timeit("skeleton", (double)nsh * rows * 8.0 * d, [&] {   // v2's register pipeline, no arithmetic
      hipLaunchKernelGGL(k_skeleton<64>, dim3(nsh * G), dim3(256), (size_t)64 * (d | 1) * 8, st, A, sink);
    });
  {
    const int K = d / 2;
    for (int nb = 2; nb <= 6; ++nb) {
      const size_t l3 = (size_t)nb * K * 1024;
      if (l3 > 160 * 1024) break;
      hipFuncSetAttribute((const void*)k_skel3, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      const int64_t nt = (rows + 63) / 64;
      int g3 = (int)std::min<int64_t>(512, (nt + 7) / 8);
      SweepArgs A3{sh_d, q, partial, nullptr, 0, C, Dp, g3, nb, d + 2, 0, g3, nullptr};
      char name[32];
      snprintf(name, sizeof name, "skel3 nb%d", nb);
      timeit(name, (double)nsh * rows * 8.0 * d, [&] {
        hipLaunchKernelGGL(k_skel3, dim3(nsh * g3), dim3(512), l3, st, A3, nb, sink);
      });
    }
  }
  if (sweep_variant(rows, d, C) == 3) {
    SweepArgs A3{sh_d, q, partial, nullptr, 0, C, Dp, G, LD, d + 2, 0, G, nullptr};
    auto abl = [&](const char* name, auto kern) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      timeit(name, bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(512), lds, st, A3, LD); });
    };
    abl("v3 generic", k_sweep3<STK_LOGREG, 4, 0>);
    abl("v3 -trans", k_sweep3<STK_LOGREG, 4, 1>);
    abl("v3 -bwd", k_sweep3<STK_LOGREG, 4, 2>);
    abl("v3 -fwd", k_sweep3<STK_LOGREG, 4, 4>);
    abl("v3 -t-b", k_sweep3<STK_LOGREG, 4, 3>);
    abl("v3 -all", k_sweep3<STK_LOGREG, 4, 7>);
  }
  if (sweep_variant(rows, d, C) == 4 && d == 100) {
    SweepArgs A4{sh_d, q, partial, nullptr, 0, C, Dp, G, LD, d + 2, 0, G, nullptr};
    auto abl = [&](const char* name, auto kern) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      timeit(name, bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(256), lds, st, A4, LD); });
    };
    abl("v4 generic", k_sweepm<STK_LOGREG, 0, 0, 0>);
    {
      const size_t le = std::max((size_t)SM_W * sweepm_slot_bytes(d) + 16 * (100 + SE_BPAD) * 8 + SP_TAB * 8, lds);
      auto ke = [&](const char* name, auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        timeit(name, bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(256), le, st, A4); });
      };
      ke("v4e", k_sweepe<STK_LOGREG, 25, 7>);
      ke("v4e -trans", k_sweepe<STK_LOGREG, 25, 7, 1>);
      ke("v4e -all", k_sweepe<STK_LOGREG, 25, 7, 7>);
    }
    {   // one block per CU, 3-slot rings
      const int nb1 = sweepm_nb(d, 1);
      SweepArgs A1 = A4;
      A1.LD = nb1;
      const size_t l1 = std::max((size_t)SM_W * nb1 * sweepm_slot_bytes(d) + SP_TAB * 8, lds);
      auto kern = k_sweepm<STK_LOGREG, 25, 7, 0, 1>;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      timeit("v4 1blk nb3", bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(256), l1, st, A1, nb1); });
    }
    abl("v4 -trans", k_sweepm<STK_LOGREG, 25, 7, 1, SM_MINB, true>);
    abl("v4 -bwd", k_sweepm<STK_LOGREG, 25, 7, 2, SM_MINB, true>);
    abl("v4 -fwd", k_sweepm<STK_LOGREG, 25, 7, 4, SM_MINB, true>);
    abl("v4 -all", k_sweepm<STK_LOGREG, 25, 7, 7, SM_MINB, true>);
    {   // k_sweepq (4x4x4 four-block MFMA), S = 8, NB = 3, two blocks per CU: ablations
      const size_t lq = sweepq_lds(8, 3, 25, d);
      auto kq = [&](const char* name, auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        timeit(name, bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(256), lq, st, A4); });
      };
      kq("q", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 0>);
      kq("q -trans", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 1>);
      kq("q -bwd", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 2>);
      kq("q -fwd", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 4>);
      kq("q -all", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 7>);
      kq("q -lds", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 8>);
      kq("q -lds-trans", k_sweepq<STK_LOGREG, 25, 8, 3, 2, 9>);
      kq("q4 -lds-trans", k_sweepq<STK_LOGREG, 25, 4, 6, 2, 9>);
    }
    {   // k_sweepx (4x4x4, rotated row groups, two register images per sub-tile)
      const size_t lx = sweepx_lds(25, d);
      auto kx = [&](const char* name, auto kern) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        timeit(name, bytes, [&] { hipLaunchKernelGGL(kern, dim3(nsh * G), dim3(256), lx, st, A4); });
      };
      kx("x", k_sweepx<STK_LOGREG, 25, 2, 0>);
      kx("x -trans", k_sweepx<STK_LOGREG, 25, 2, 1>);
      kx("x -bwd", k_sweepx<STK_LOGREG, 25, 2, 2>);
      kx("x -fwd", k_sweepx<STK_LOGREG, 25, 2, 4>);
      kx("x -all", k_sweepx<STK_LOGREG, 25, 2, 7>);
      kx("x -lds", k_sweepx<STK_LOGREG, 25, 2, 8>);
      kx("x 1blk", k_sweepx<STK_LOGREG, 25, 1, 0>);
    }
    const double fl = 4.0 * d * C * (double)rows * nsh;   // algorithmic fp64 flops of one sweep
    timeit("v4 flops", fl, [&] {
      CK(stk_launch_sweep(STK_LOGREG, sh_d, 0, nsh, rows, d, T, LD, G, G, lds, q, C, Dp, partial, nullptr, 0, nullptr, st, wsp));
    });
    printf("  (v4 flops line: 'GB/s' column = GFLOP/s of the sweep's 4*d*C flop per row)\n");
    for (int wpb = 1; wpb <= 4; wpb *= 2) {
      const int iters = 2000, blocks = 256 * 4;
      char name[32];
      snprintf(name, sizeof name, "mfma f64 w%d", wpb);
      timeit(name, (double)blocks * wpb * iters * 4 * 2048.0, [&] {
        hipLaunchKernelGGL(k_mfma_peak, dim3(blocks), dim3(64 * wpb), 0, st, sink, iters);
      });
    }
  }
  if (sweep_variant(rows, d, C) == 5) {
    const double fl = 4.0 * d * C * (double)rows * nsh;
    timeit("v5 flops", fl, [&] {
      CK(stk_launch_sweep(STK_LOGREG, sh_d, 0, nsh, rows, d, T, LD, G, G, lds, q, C, Dp, partial, nullptr, 0, nullptr, st, wsp));
    });
    printf("  (v5 flops line: 'GB/s' column = GFLOP/s of the two GEMMs, 4*d*C flop per row)\n");
  }
  timeit("sweep", bytes, [&] {
    CK(stk_launch_sweep(STK_LOGREG, sh_d, 0, nsh, rows, d, T, LD, G, G, lds, q, C, Dp, partial, nullptr, 0, nullptr, st, wsp));
  });
  timeit("sweep+red", bytes, [&] {
    CK(stk_launch_sweep(STK_LOGREG, sh_d, 0, nsh, rows, d, T, LD, G, G, lds, q, C, Dp, partial, nullptr, 0, nullptr, st, wsp));
    CK(stk_launch_sweep_reduce(STK_LOGREG, sh_d, 0, nsh, d, G, G, q, C, Dp, partial, nullptr, 0, lp, grad, st));
  });
  CK(hipStreamSynchronize(st));
  return 0;
}
