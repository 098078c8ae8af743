// Operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950, found by testing every
// assignment of the three 2-bit lane fields (block, row/col, k) against a host GEMM.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma4_layout.hip -o tools/_bin/mfma4_layout
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <array>
#include <vector>

__global__ void k_probe(const double* a, const double* b, const double* c, double* d) {
  const int l = threadIdx.x;
  d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c[l], 0, 0, 0);
}

// field order: which lane field (0: bits 0-1, 1: bits 2-3, 2: bits 4-5) holds each of three
// named indices
static int lane_of(const std::array<int, 3>& pos, int x0, int x1, int x2) {
  int l = 0;
  l |= x0 << (2 * pos[0]);
  l |= x1 << (2 * pos[1]);
  l |= x2 << (2 * pos[2]);
  return l;
}

int main() {
  std::vector<double> ha(64), hb(64), hc(64), hd(64);
  for (int l = 0; l < 64; ++l) { ha[l] = 1 + l; hb[l] = 1000 + 7 * l; hc[l] = 1e6 * (l + 1); }
  double *da, *db, *dc, *dd;
  hipMalloc(&da, 512); hipMalloc(&db, 512); hipMalloc(&dc, 512); hipMalloc(&dd, 512);
  hipMemcpy(da, ha.data(), 512, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), 512, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dc, dd);
  if (hipMemcpy(hd.data(), dd, 512, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
  printf("D[lane] for lanes 0..15:");
  for (int l = 0; l < 16; ++l) printf(" %.0f", hd[l]);
  printf("\n");
  std::vector<std::array<int, 3>> perms = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
  int found = 0;
  // A: (blk, m, k); B: (blk, n, k); C/D: (blk, m, n)
  for (auto& pa : perms)
    for (auto& pb : perms)
      for (auto& pd : perms) {
        bool ok = true;
        for (int bl = 0; bl < 4 && ok; ++bl)
          for (int m = 0; m < 4 && ok; ++m)
            for (int n = 0; n < 4 && ok; ++n) {
              double s = hc[lane_of(pd, bl, m, n)];
              for (int k = 0; k < 4; ++k) s += ha[lane_of(pa, bl, m, k)] * hb[lane_of(pb, bl, n, k)];
              if (fabs(s - hd[lane_of(pd, bl, m, n)]) > 1e-6 * fabs(s)) ok = false;
            }
        if (ok) {
          ++found;
          printf("match: A lane fields (blk,m,k) at bit-pairs (%d,%d,%d); B (blk,n,k) (%d,%d,%d); D (blk,m,n) (%d,%d,%d)\n",
                 pa[0], pa[1], pa[2], pb[0], pb[1], pb[2], pd[0], pd[1], pd[2]);
        }
      }
  printf("%d matching layouts\n", found);
  return found ? 0 : 2;
}
