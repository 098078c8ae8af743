// Pass B variants for tools/gemm_fwd_ab.py (round 5): G[j][c] += X[r][j] R[r][c] as the product's
// k_gemm_bwd (sweep.hip), but each wave takes CTW = JB / 16 / NW column tiles x all 4 chain tiles
// (CTW A reads + 4 B reads per 4 CTW MFMAs), stages of RB rows.  JB = 256 halves the R re-reads
// from L2 (one per column block: 4 instead of 8 at d = 1000).  Built only into the A/B harness.
namespace stk {

template <int JB, int RB, int NW, int NS>
__global__ __launch_bounds__(64 * NW, 8 / NW >= 1 ? 8 / NW : 1) void k_gemm_bwd_w(SweepArgs A, int njb) {
  constexpr int WC = JB / 16, CTW = WC / NW, NCT = 4, PPR = JB / 2;
  constexpr int XB = RB * JB * 8, RBB = RB * 512, STG = XB + RBB;
  constexpr int NDX = XB / 1024 / NW, NDR = RBB / 1024 / NW;
  static_assert(CTW >= 1 && WC % NW == 0 && NDX >= 1 && NDR >= 1 && XB % (1024 * NW) == 0 && RBB % (1024 * NW) == 0,
                "pass B stage geometry");
  const int nsc = gridDim.x / njb;
  int sc, jb;
  if ((nsc & 7) == 0) {
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
    sc = x + 8 * (k / njb);
    jb = k % njb;
  } else {
    jb = blockIdx.x % njb;
    sc = blockIdx.x / njb;
  }
  const int shard = A.shard0 + sc / A.G;
  const int chunk = sc % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
  const int nrows = (int)(r1 - r0);
  const int nst = (nrows + RB - 1) / RB;
  const int j0 = jb * JB;

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const stg = reinterpret_cast<char*>(lds);
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(A.R + ((size_t)shard * A.Rrows + r0) * G5_C, (int64_t)nrows * G5_C * 8);
  int xvo[NDX];
#pragma unroll
  for (int i = 0; i < NDX; ++i) {
    const int sl = (w * NDX + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ ((row & 1) << 3);
    xvo[i] = row * d * 8 + (j0 + 2 * pc) * 8;
  }
  auto issue = [&](int st) {
    char* b = stg + (st % NS) * STG;
    const int xso = st * RB * d * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i) dma16_lds(xr, b + (w * NDX + i) * 1024, xvo[i], xso);
#pragma unroll
    for (int i = 0; i < NDR; ++i) dma16_lds(rr, b + XB + (w * NDR + i) * 1024, lane * 16, st * RB * 512 + (w * NDR + i) * 1024);
  };
  dbl4 acc[CTW][NCT];
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int c2 = 0; c2 < NCT; ++c2) acc[ct][c2] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  for (int st = 0; st < nst; ++st) {
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDR));
    lds_barrier();
    if (st + NS - 1 < nst) issue(st + NS - 1);
    const char* b = stg + (st % NS) * STG;
#pragma unroll
    for (int step = 0; step < RB / 4; ++step) {
      const int r = 4 * step + lh;
      double a[CTW];
#pragma unroll
      for (int ct = 0; ct < CTW; ++ct) {
        const int jl = 16 * (w * CTW + ct) + lr;
        a[ct] = *reinterpret_cast<const double*>(b + r * (16 * PPR) + ((((jl >> 1) ^ ((r & 1) << 3))) << 4) + ((jl & 1) << 3));
      }
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const double bb = *reinterpret_cast<const double*>(b + XB + g5_chain_off(r, 16 * c2 + lr));
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct) acc[ct][c2] = mfma_f64(a[ct], bb, acc[ct][c2]);
      }
    }
  }
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * G5_C * A.PW;
#pragma unroll
  for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
    for (int c2 = 0; c2 < NCT; ++c2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = j0 + 16 * (w * CTW + ct) + lh + 4 * i;
        if (j < d) out[(size_t)(16 * c2 + lr) * A.PW + 1 + j] = acc[ct][c2][i];
      }
}

template <int JB, int RB, int NW, int NS>
constexpr size_t gemm_bwd_w_lds() { return (size_t)NS * (RB * JB * 8 + RB * 512); }

}  // namespace stk
