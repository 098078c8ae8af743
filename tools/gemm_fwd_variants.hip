// (Built against stark_amd/csrc/sweep.hip as of commit 2f88366, before round 5 moved the product's
// pass F to 128-row tiles; it does not build against the current sweep.hip.  Kept as the record of
// the arms measured in profiles/r05e-r05t and r04o.)
// A/B variants of pass F (sweep.hip: k_gemm_fwd), for tools/gemm_fwd_ab.py.  Included after
// sweep.hip inside the harness; not part of the library.
//
// k_gemm_fwd_t<FAM, NS, KCF, RT>: the product's skeleton (4 waves, two blocks per CU, LDS-DMA
// stages, residual v4 epilogue straight from the accumulators) with RT 16-row groups per wave,
// i.e. 64 RT-row tiles.  RT = 2 halves the beta^T bytes each row streams through LDS (one
// beta^T stage serves 128 rows) and reads 6 fragments per 8 MFMAs instead of 5 per 4; with
// KCF = 16 columns per stage a stage is 16 KB X + 8 KB beta^T, so 2 or 3 stages keep two blocks
// on a CU.  Chunks are cut in whole 64 RT-row tiles (pass B's chunks stay in 64-row tiles: pass B
// reads the finished R, so its chunk rows need not match; the sums over chunks are the same rows),
// so only the shard's last tile is ragged and R's rows are written unconditionally (R is padded to
// a whole tile).
namespace stk {

template <int FAM, int NS, int KCF, int RT>
__global__ __launch_bounds__(256, 2) void k_gemm_fwd_t(SweepArgs A) {
  constexpr int NW = 4, NCT = 4, TRT = 64 * RT;
  constexpr int XBt = TRT * KCF * 8, BB = KCF * 512, STG = XBt + BB;
  constexpr int PPR = KCF / 2;
  constexpr int NDX = XBt / 1024 / NW, NDB = BB / 1024 / NW;
  static_assert(NDX >= 1 && NDB >= 1, "stage geometry");
  auto swz = [](int row) { return PPR == 16 ? (row & 15) : ((row >> 1) & 7); };
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, KP = g5_kp(d), NKC = KP / KCF;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + TRT - 1) / TRT;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * TRT, r1 = std::min<int64_t>(sh.n, t1 * TRT);
  const int nrows = (int)(r1 - r0);
  const int ntile = (int)(t1 - t0);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const stg = reinterpret_cast<char*>(lds);
  double* const sptab = reinterpret_cast<double*>(stg + NS * STG);
  if constexpr (FAM == STK_LOGREG) exp_table_init(sptab);

  const double* qb = A.q + (size_t)shard * G5_C * A.Dp;
  double alpha[NCT], inv_s[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) {
    alpha[c2] = qb[(size_t)(16 * c2 + lr) * A.Dp];
    inv_s[c2] = (FAM == STK_LINREG) ? exp(-qb[(size_t)(16 * c2 + lr) * A.Dp + d + 1]) : 0.0;
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const __amdgpu_buffer_rsrc_t br = uniform_rsrc(A.qT + (size_t)shard * KP * G5_C, (int64_t)KP * G5_C * 8);
  int xvo[NDX];
#pragma unroll
  for (int i = 0; i < NDX; ++i) {
    const int sl = (w * NDX + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ swz(row);
    xvo[i] = row * d * 8 + pc * 16;
  }
  auto issue = [&](int st) {
    const int tile = st / NKC, kc = st % NKC;
    char* b = stg + (st % NS) * STG;
    const int xso = tile * TRT * d * 8 + kc * KCF * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(b + (w * NDX + i) * 1024), 16, (int)xvo[i], xso, 0, 0);   // (int): hip-clang drops the host stub for a
                                                                   // template-sized array read bare in the builtin
#pragma unroll
    for (int i = 0; i < NDB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(br, (lds_vptr)(b + XBt + (w * NDB + i) * 1024), 16, lane * 16,
                                               kc * KCF * 512 + (w * NDB + i) * 1024, 0, 0);
  };

  double lm[NCT], sp[NCT], ll[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = ll[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  dbl4 acc[RT][NCT];
  double yt[RT][4];
  uint32_t yit[RT][4];
#pragma unroll
  for (int g = 0; g < RT; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) { yt[g][i] = 0.0; yit[g][i] = 0u; }
  for (int st = 0; st < nst; ++st) {
    const int kc = st % NKC;
    if (kc == 0) {
#pragma unroll
      for (int g = 0; g < RT; ++g)
#pragma unroll
        for (int c2 = 0; c2 < NCT; ++c2) acc[g][c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDB));
    lds_barrier();
    if (st + NS - 1 < nst) issue(st + NS - 1);
    if (kc == 0) {
#pragma unroll
      for (int g = 0; g < RT; ++g) {
        const int64_t tb = (int64_t)(st / NKC) * TRT + 16 * (RT * w + g) + lh;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t grow = tb + 4 * i;
          if constexpr (FAM == STK_LOGREG) yit[g][i] = grow < nrows ? (uint32_t)sh.yi[r0 + grow] : 0u;
          else yt[g][i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
        }
      }
    }
    const char* b = stg + (st % NS) * STG;
#pragma unroll
    for (int step = 0; step < KCF / 4; ++step) {
      const int kk = 4 * step + lh;
      double a[RT];
#pragma unroll
      for (int g = 0; g < RT; ++g) {
        const int r = 16 * (RT * w + g) + lr;
        a[g] = *reinterpret_cast<const double*>(b + r * (16 * PPR) + (((kk >> 1) ^ swz(r)) << 4) + ((kk & 1) << 3));
      }
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const double bv = *reinterpret_cast<const double*>(b + XBt + g5_chain_off(kk, 16 * c2 + lr));
#pragma unroll
        for (int g = 0; g < RT; ++g) acc[g][c2] = mfma_f64(a[g], bv, acc[g][c2]);
      }
    }
    if (kc == NKC - 1) {
      const int tile = st / NKC;
#pragma unroll
      for (int g = 0; g < RT; ++g) {
#pragma unroll
        for (int c2 = 0; c2 < NCT; ++c2) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * (RT * w + g) + lh + 4 * i;
            const int64_t grow = (int64_t)tile * TRT + row;
            const bool valid = grow < nrows;
            const double eta = acc[g][c2][i] + alpha[c2];
            double dv;
            if constexpr (FAM == STK_LOGREG) {
              double lm2 = lm[c2], sp2 = sp[c2];
              dv = -logit_resid4(eta, yit[g][i], sptab, lm2, sp2);
              lm[c2] = valid ? lm2 : lm[c2];
              sp[c2] = valid ? sp2 : sp[c2];
            } else {
              const double z = (yt[g][i] - eta) * inv_s[c2];
              lm[c2] += valid ? z * z : 0.0;
              dv = z * inv_s[c2];
            }
            dv = valid ? dv : 0.0;
            gaa[c2] += dv;
            *reinterpret_cast<double*>(Rimg + g5_chain_off((int)grow, 16 * c2 + lr)) = dv;
          }
        }
      }
      if constexpr (FAM == STK_LOGREG) {
        if ((tile & (64 / RT - 1)) == 64 / RT - 1) {     // 256 elements per lane and chain tile
#pragma unroll
          for (int c2 = 0; c2 < NCT; ++c2) {
            ll[c2] += log1p(sp[c2]);
            sp[c2] = 0.0;
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xF70);
    }
  }
  double lpa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lpa[c2] = (FAM == STK_LOGREG) ? 0.5 * lm[c2] - (ll[c2] + log1p(sp[c2])) : lm[c2];
  __syncthreads();
  double* red = lds;                                     // [NW waves][64 lanes][NCT][2]
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) {
    red[((w * 64 + lane) * NCT + c2) * 2 + 0] = lpa[c2];
    red[((w * 64 + lane) * NCT + c2) * 2 + 1] = gaa[c2];
  }
  __syncthreads();
  if (tid < 2 * G5_C) {
    const int c = tid >> 1, kind = tid & 1, c2 = c >> 4, l = c & 15;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red[(((ww * 64 + h * 16 + l) * NCT + c2) * 2) + kind];
    A.partial[(((size_t)shard * A.Gs + chunk) * G5_C + c) * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

template <int NS, int KCF, int RT>
constexpr size_t gemm_fwd_t_lds() { return (size_t)NS * (64 * RT * KCF * 8 + KCF * 512) + EX_TAB * sizeof(double); }

}  // namespace stk

// the kernel's address through a typed pointer (a bare (const void*) cast of the template-id left
// hip-clang without the host stub)
template <int NS, int KCF, int RT>
const void* gemm_fwd_t_ptr() {
  void (*f)(stk::SweepArgs) = stk::k_gemm_fwd_t<STK_LOGREG, NS, KCF, RT>;
  return reinterpret_cast<const void*>(f);
}
