// (Built against stark_amd/csrc/sweep.hip as of commit 2f88366, before round 5 moved the product's
// pass F to 128-row tiles; it does not build against the current sweep.hip.  Kept as the record of
// the arms measured in profiles/r05e-r05t and r04o.)
// Round-5 measurement variant of pass F (stark_amd/csrc/sweep.hip: k_gemm_fwd) for
// tools/gemm_fwd_ab.py: 128-row tiles shared by 8 waves (one block per CU, two waves per SIMD),
// each wave 16 rows x all 64 chains -- the product's per-wave shape -- so one beta^T stage feeds
// twice the rows: the LDS-DMA volume per row drops from 2 x (X) to 1.5 x (X) (the product's two
// 4-wave blocks per CU each re-stream all of beta^T per 64 rows), and NS stages of 48 KB give a
// deeper prefetch.  Chunk row ranges stay those of 64-row tiles (pass B, the reduction and the
// placement independence are unchanged): a chunk's last 128-row tile may be half empty, and no R
// row past the chunk's 64-row-aligned end is written.
// Included after sweep.hip (namespace stk).
namespace stk {

template <int FAM, int NS>
__global__ __launch_bounds__(512, 1) void k_gemm_fwd8(SweepArgs A) {
  constexpr int NW = 8, NCT = 4, TR = 128;
  constexpr int KCF = 32, XB = TR * KCF * 8, BB = KCF * 512, STG = XB + BB;   // stage: [X 128 x KCF][beta^T KCF x 64]
  constexpr int PPR = KCF / 2;                          // 16-B pieces per X row in the stage
  constexpr int NDX = XB / 1024 / NW, NDB = BB / 1024 / NW;
  static_assert(NDX >= 1 && NDB >= 1, "pass F8 stage geometry");
  auto swz = [](int row) { return row & 15; };
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, KP = g5_kp(d), NKC = KP / KCF;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;       // the chunk geometry of 64-row tiles
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
  const int nrows = (int)(r1 - r0);
  const int rcap = (int)((t1 - t0) * G5_TR);           // R rows of this chunk
  const int ntile = (rcap + TR - 1) / TR;

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
    const int xso = tile * TR * d * 8 + kc * KCF * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(b + (w * NDX + i) * 1024), 16, xvo[i], xso, 0, 0);
#pragma unroll
    for (int i = 0; i < NDB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(br, (lds_vptr)(b + XB + (w * NDB + i) * 1024), 16, lane * 16,
                                               kc * KCF * 512 + (w * NDB + i) * 1024, 0, 0);
  };
  double lm[NCT], sp[NCT], ll[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = ll[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  dbl4 acc[NCT];
  double yt[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t yit[4] = {0u, 0u, 0u, 0u};
  for (int st = 0; st < nst; ++st) {
    const int kc = st % NKC;
    if (kc == 0) {
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) acc[c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    // own DMAs of stage st retired: the stages after it (at most NS - 2) may stay in flight; a
    // stricter wait also covers the tile's y loads issued one stage earlier
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDB));
    lds_barrier();
    if (st + NS - 1 < nst) issue(st + NS - 1);
    if (kc == (NKC > 1 ? 1 : 0)) {                       // the tile's y, a stage ahead of its epilogue
      const int64_t tb = (int64_t)(st / NKC) * TR + 16 * w + lh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t grow = tb + 4 * i;
        if constexpr (FAM == STK_LOGREG) yit[i] = grow < nrows ? (uint32_t)sh.yi[r0 + grow] : 0u;
        else yt[i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
      }
    }
    const char* b = stg + (st % NS) * STG;
    const int r = 16 * w + lr;
#pragma unroll
    for (int step = 0; step < KCF / 4; ++step) {
      const int kk = 4 * step + lh;
      const double a = *reinterpret_cast<const double*>(b + r * (16 * PPR) + (((kk >> 1) ^ swz(r)) << 4) + ((kk & 1) << 3));
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2)
        acc[c2] = mfma_f64(a, *reinterpret_cast<const double*>(b + XB + g5_chain_off(kk, 16 * c2 + lr)), acc[c2]);
    }
    if (kc == NKC - 1) {
      const int tile = st / NKC;
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * w + lh + 4 * i;
          const int grow = tile * TR + row;
          const bool valid = grow < nrows;
          const double eta = acc[c2][i] + alpha[c2];
          double dv;
          if constexpr (FAM == STK_LOGREG) {
            double lm2 = lm[c2], sp2 = sp[c2];
            dv = -logit_resid4(eta, yit[i], sptab, lm2, sp2);
            lm[c2] = valid ? lm2 : lm[c2];
            sp[c2] = valid ? sp2 : sp[c2];
          } else {
            const double z = (yt[i] - eta) * inv_s[c2];
            lm[c2] += valid ? z * z : 0.0;
            dv = z * inv_s[c2];
          }
          dv = valid ? dv : 0.0;
          gaa[c2] += dv;
          if (grow < rcap) *reinterpret_cast<double*>(Rimg + g5_chain_off(grow, 16 * c2 + lr)) = dv;
        }
      }
      if constexpr (FAM == STK_LOGREG) {
        if ((tile & 31) == 31) {                          // 32 tiles x 4 rows = 128 elements per lane
#pragma unroll
          for (int c2 = 0; c2 < NCT; ++c2) {
            ll[c2] += log1p(sp[c2]);
            sp[c2] = 0.0;
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xF70);                  // vmcnt(0): R stores retired before the next counted wait
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
      for (int h = 0; h < 4; ++h) v += red[((ww * 64 + h * 16 + l) * NCT + c2) * 2 + kind];
    A.partial[(((size_t)shard * A.Gs + chunk) * G5_C + c) * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

template <int FAM, int NS>
constexpr size_t gemm_fwd8_lds() { return (size_t)NS * (128 * 32 * 8 + 32 * 512) + EX_TAB * 8; }

// Pass F with a PIPELINED epilogue: the tile's eta (accumulators + alpha) is parked in registers at
// its last stage, and its residual / R stores / lp terms run one chain tile per stage during the
// next tile's first stages (chain tile c2 at stage kc with c2 % NKC == kc), interleaved with their
// MFMAs, instead of all 16 (row, chain) elements at the tile's end followed by vmcnt(0) -- the
// unrolled 16-element epilogue is what holds the product kernel at 229 VGPRs (83 without it) and
// what every wave of a block runs at once.  EPRE: the chain tile's residual before the stage's
// MFMAs (its R stores then have the whole stage before the next vmcnt(0)); else after them.
// Per chain tile the lp terms are added in the product's order: lp and the gradient are
// bit-identical to k_gemm_fwd's.
template <int FAM, bool EPRE>
__global__ __launch_bounds__(64 * G5_FW, 8 / G5_FW) void k_gemm_fwd_p(SweepArgs A) {
  constexpr int NW = G5_FW, NS = G5_FS, NCT = 16 / NW;
  constexpr int KCF = G5_FKC, STG = g5_fstage_bytes(), XB = STG / 2;
  constexpr int PPR = KCF / 2;
  constexpr int NDMA = (XB / 1024) / NW;
  static_assert(NDMA >= 1 && NS == 2, "pass F stage geometry");
  auto swz = [](int row) { return PPR == 16 ? (row & 15) : ((row >> 1) & 7); };
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, KP = g5_kp(d), NKC = KP / KCF;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int wr = w & 3, wc = w >> 2;
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
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
    const int ct = NCT * wc + c2;
    alpha[c2] = qb[(size_t)(16 * ct + lr) * A.Dp];
    inv_s[c2] = (FAM == STK_LINREG) ? exp(-qb[(size_t)(16 * ct + lr) * A.Dp + d + 1]) : 0.0;
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const __amdgpu_buffer_rsrc_t br = uniform_rsrc(A.qT + (size_t)shard * KP * G5_C, (int64_t)KP * G5_C * 8);
  int xvo[NDMA];
#pragma unroll
  for (int i = 0; i < NDMA; ++i) {
    const int sl = (w * NDMA + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ swz(row);
    xvo[i] = row * d * 8 + pc * 16;
  }
  auto issue = [&](int st) {
    const int tile = st / NKC, kc = st % NKC;
    char* b = stg + (st % NS) * STG;
    const int xso = tile * G5_TR * d * 8 + kc * KCF * 8;
#pragma unroll
    for (int i = 0; i < NDMA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(b + (w * NDMA + i) * 1024), 16, xvo[i], xso, 0, 0);
#pragma unroll
    for (int i = 0; i < NDMA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(br, (lds_vptr)(b + XB + (w * NDMA + i) * 1024), 16, lane * 16,
                                               kc * KCF * 512 + (w * NDMA + i) * 1024, 0, 0);
  };
  double lm[NCT], sp[NCT], ll[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = ll[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  issue(0);
  dbl4 acc[NCT];
  double pend[NCT][4];                                  // eta of the parked tile
  double yt[4] = {0.0, 0.0, 0.0, 0.0}, pyt[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t yit[4] = {0u, 0u, 0u, 0u}, pyit[4] = {0u, 0u, 0u, 0u};
  int ptile = -1;
  auto epi = [&](auto c2c) {                            // the parked tile's chain tile c2
    constexpr int c2 = decltype(c2c)::value;
    const int ct = NCT * wc + c2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * wr + lh + 4 * i;
      const int64_t grow = (int64_t)ptile * G5_TR + row;
      const bool valid = grow < nrows;
      const double eta = pend[c2][i];
      double dv;
      if constexpr (FAM == STK_LOGREG) {
        double lm2 = lm[c2], sp2 = sp[c2];
        dv = -logit_resid4(eta, pyit[i], sptab, lm2, sp2);
        lm[c2] = valid ? lm2 : lm[c2];
        sp[c2] = valid ? sp2 : sp[c2];
      } else {
        const double z = (pyt[i] - eta) * inv_s[c2];
        lm[c2] += valid ? z * z : 0.0;
        dv = z * inv_s[c2];
      }
      dv = valid ? dv : 0.0;
      gaa[c2] += dv;
      *reinterpret_cast<double*>(Rimg + g5_chain_off((int)grow, 16 * ct + lr)) = dv;
    }
    if constexpr (FAM == STK_LOGREG) {
      if ((ptile & 63) == 63) {
        ll[c2] += log1p(sp[c2]);
        sp[c2] = 0.0;
      }
    }
  };
  auto epi_stage = [&](int kc) {
    if (ptile >= 0) {
      if (0 % NKC == kc) epi(std::integral_constant<int, 0>{});
      if (NCT > 1 && 1 % NKC == kc) epi(std::integral_constant<int, 1 % NCT>{});
      if (NCT > 2 && 2 % NKC == kc) epi(std::integral_constant<int, 2 % NCT>{});
      if (NCT > 3 && 3 % NKC == kc) epi(std::integral_constant<int, 3 % NCT>{});
    }
  };
  for (int st = 0; st < nst; ++st) {
    const int kc = st % NKC;
    if (kc == 0) {
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) acc[c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    __builtin_amdgcn_s_waitcnt(0xF70);                   // vmcnt(0): stage st landed, the last R stores retired
    lds_barrier();
    if (st + 1 < nst) issue(st + 1);
    if (kc == 0) {
      const int64_t tb = (int64_t)(st / NKC) * G5_TR + 16 * wr + lh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t grow = tb + 4 * i;
        if constexpr (FAM == STK_LOGREG) yit[i] = grow < nrows ? (uint32_t)sh.yi[r0 + grow] : 0u;
        else yt[i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
      }
    }
    if constexpr (EPRE) epi_stage(kc);
    const char* b = stg + (st % NS) * STG;
    const int r = 16 * wr + lr;
#pragma unroll
    for (int step = 0; step < KCF / 4; ++step) {
      const int kk = 4 * step + lh;
      const double a = *reinterpret_cast<const double*>(b + r * (16 * PPR) + (((kk >> 1) ^ swz(r)) << 4) + ((kk & 1) << 3));
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2)
        acc[c2] = mfma_f64(a, *reinterpret_cast<const double*>(b + XB + g5_chain_off(kk, 16 * (NCT * wc + c2) + lr)), acc[c2]);
    }
    if constexpr (!EPRE) epi_stage(kc);
    if (kc == NKC - 1) {                                 // park this tile for the next tile's stages
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2)
#pragma unroll
        for (int i = 0; i < 4; ++i) pend[c2][i] = acc[c2][i] + alpha[c2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pyit[i] = yit[i];
        pyt[i] = yt[i];
      }
      ptile = st / NKC;
    }
  }
  if (ptile >= 0) {                                     // the chunk's last tile
    epi(std::integral_constant<int, 0>{});
    if constexpr (NCT > 1) epi(std::integral_constant<int, 1 % NCT>{});
    if constexpr (NCT > 2) epi(std::integral_constant<int, 2 % NCT>{});
    if constexpr (NCT > 3) epi(std::integral_constant<int, 3 % NCT>{});
  }
  double lpa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lpa[c2] = (FAM == STK_LOGREG) ? 0.5 * lm[c2] - (ll[c2] + log1p(sp[c2])) : lm[c2];
  __syncthreads();
  double* red = lds;
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) {
    red[((w * 64 + lane) * NCT + c2) * 2 + 0] = lpa[c2];
    red[((w * 64 + lane) * NCT + c2) * 2 + 1] = gaa[c2];
  }
  __syncthreads();
  if (tid < 2 * G5_C) {
    const int c = tid >> 1, kind = tid & 1, ct = c >> 4, l = c & 15, cw = ct / NCT, c2 = ct % NCT;
    double v = 0.0;
    for (int ww = 0; ww < 4; ++ww)
      for (int h = 0; h < 4; ++h) v += red[(((cw * 4 + ww) * 64 + h * 16 + l) * NCT + c2) * 2 + kind];
    A.partial[(((size_t)shard * A.Gs + chunk) * G5_C + c) * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

// Pass F with 128-row tiles on the product's 4-wave block (two blocks per CU): each wave 32 rows
// (two 16-row MFMA tiles) x all 64 chains, stages of 16 columns (X 16 KB + beta^T 8 KB) in a 3-deep
// ring -- 80 KB per block with the table, two blocks fill the CU's 160 KB -- so one beta^T stage
// feeds 128 rows (LDS-DMA volume 1.5 x the X bytes instead of 2 x) while one block's epilogue still
// overlaps the other's MFMAs.  The 64 accumulators per wave leave no room for an all-at-once
// epilogue (round 4's 128-row tiles spilled 70 VGPRs), so it is pipelined as in k_gemm_fwd_p: the
// tile's eta parked, one (row tile, chain tile) part of 4 elements per stage of the next tile.
// Waits: the LDS-DMA loads and the tile's y loads complete in issue order, so "at most the next
// stage's DMA outstanding" proves the current stage landed whatever the R stores in between do;
// the stores go out right after the barrier, a whole stage ahead of the wait that also counts them.
// The DMA goes through a plain function: clang's host pass drops a kernel template's stub when the
// builtin's operands depend on a template parameter (undefined symbol at link, no diagnostic).
__device__ __forceinline__ void dma16_lds(__amdgpu_buffer_rsrc_t r, char* dst, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_vptr)dst, 16, voff, soff, 0, 0);
}

template <int FAM, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_fwd_w(SweepArgs A) {
  constexpr int NCT = 4, RT = 2, TR = 32 * NW, KCF = 16, NS = 3;
  constexpr int XB = TR * KCF * 8, BB = KCF * 512, STG = XB + BB;
  constexpr int PPR = KCF / 2;                          // 16-B pieces per X row in the stage (8)
  constexpr int NDX = XB / 1024 / NW, NDB = BB / 1024 / NW, NPART = RT * NCT;
  static_assert(NDX == 4 && NDB >= 1 && BB % (1024 * NW) == 0, "pass Fw stage geometry");
  auto swz = [](int row) { return (row >> 1) & 7; };
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d, KP = (d + KCF - 1) / KCF * KCF, NKC = KP / KCF;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + G5_TR - 1) / G5_TR;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * G5_TR, r1 = std::min<int64_t>(sh.n, t1 * G5_TR);
  const int nrows = (int)(r1 - r0);
  const int rcap = (int)((t1 - t0) * G5_TR);
  const int ntile = (rcap + TR - 1) / TR;

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
  // beta^T rows past the image's KP (a multiple of 32) read as 0 through the descriptor bound
  const int KPI = g5_kp(d);
  const __amdgpu_buffer_rsrc_t br = uniform_rsrc(A.qT + (size_t)shard * KPI * G5_C, (int64_t)KPI * G5_C * 8);
  int xvo[NDX];
#pragma unroll
  for (int i = 0; i < NDX; ++i) {
    const int sl = (w * NDX + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ swz(row);
    xvo[i] = row * d * 8 + pc * 16;
  }
  auto issue = [&](int st) {
    const int tile = st / NKC, kc = st % NKC;
    char* b = stg + (st % NS) * STG;
    const int xso = tile * TR * d * 8 + kc * KCF * 8;
#pragma unroll
    for (int i = 0; i < NDX; ++i)
      dma16_lds(xr, b + (w * NDX + i) * 1024, xvo[i], xso);
#pragma unroll
    for (int i = 0; i < NDB; ++i)
      dma16_lds(br, b + XB + (w * NDB + i) * 1024, lane * 16, kc * KCF * 512 + (w * NDB + i) * 1024);
  };
  // lm = sum (t - |t|) - 2 sum log1p(sp) at the flushes (the flushed logs folded in: no ll registers)
  double lm[NCT], sp[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  dbl4 acc[RT][NCT];
  double pend[RT][NCT][4];
  uint32_t ybit = 0u, pybit = 0u;                       // logistic y of the tile's 8 rows per lane, one bit each
  double yt[RT][4] = {}, pyt[RT][4] = {};
  int ptile = -1;
  auto epi = [&](const int p) {                         // part p = (row tile p / NCT, chain tile p % NCT);
    const int rt = p / NCT, c2 = p % NCT;                // called from unrolled loops: p is a constant
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int grow = ptile * TR + 32 * w + 16 * rt + lh + 4 * i;
      const bool valid = grow < nrows;
      const double eta = pend[rt][c2][i];
      double dv;
      if constexpr (FAM == STK_LOGREG) {
        double lm2 = lm[c2], sp2 = sp[c2];
        dv = -logit_resid4(eta, (pybit >> (4 * rt + i)) & 1u, sptab, lm2, sp2);
        lm[c2] = valid ? lm2 : lm[c2];
        sp[c2] = valid ? sp2 : sp[c2];
      } else {
        const double z = (pyt[rt][i] - eta) * inv_s[c2];
        lm[c2] += valid ? z * z : 0.0;
        dv = z * inv_s[c2];
      }
      dv = valid ? dv : 0.0;
      gaa[c2] += dv;
      if (grow < rcap) *reinterpret_cast<double*>(Rimg + g5_chain_off(grow, 16 * c2 + lr)) = dv;
    }
    if (FAM == STK_LOGREG && rt == RT - 1) {
      if ((ptile & 31) == 31) {                          // 32 tiles x 8 elements per chain tile and lane
        lm[c2] -= 2.0 * log1p(sp[c2]);
        sp[c2] = 0.0;
      }
    }
  };
  auto epi_stage = [&](int kc) {
    if (ptile >= 0) {
#pragma unroll
      for (int p = 0; p < NPART; ++p)
        if (p % NKC == kc) epi(p);
    }
  };
  for (int st = 0; st < nst; ++st) {
    const int kc = st % NKC;
    if (kc == 0) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int c2 = 0; c2 < NCT; ++c2) acc[rt][c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * (NDX + NDB));
    lds_barrier();
    epi_stage(kc);
    if (kc == 0) {                                       // this tile's y (loads: in order with the DMA)
      if constexpr (FAM == STK_LOGREG) ybit = 0u;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t grow = (int64_t)(st / NKC) * TR + 32 * w + 16 * rt + lh + 4 * i;
          if constexpr (FAM == STK_LOGREG) ybit |= (grow < nrows ? (uint32_t)sh.yi[r0 + grow] & 1u : 0u) << (4 * rt + i);
          else yt[rt][i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
        }
    }
    if (st + NS - 1 < nst) issue(st + NS - 1);
    const char* b = stg + (st % NS) * STG;
#pragma unroll
    for (int step = 0; step < KCF / 4; ++step) {
      const int kk = 4 * step + lh;
      double a[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int r = 32 * w + 16 * rt + lr;
        a[rt] = *reinterpret_cast<const double*>(b + r * (16 * PPR) + (((kk >> 1) ^ swz(r)) << 4) + ((kk & 1) << 3));
      }
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const double bb = *reinterpret_cast<const double*>(b + XB + g5_chain_off(kk, 16 * c2 + lr));
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][c2] = mfma_f64(a[rt], bb, acc[rt][c2]);
      }
    }
    if (kc == NKC - 1) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int c2 = 0; c2 < NCT; ++c2)
#pragma unroll
          for (int i = 0; i < 4; ++i) pend[rt][c2][i] = acc[rt][c2][i] + alpha[c2];
#pragma unroll
        for (int i = 0; i < 4; ++i) pyt[rt][i] = yt[rt][i];
      }
      pybit = ybit;
      ptile = st / NKC;
    }
  }
  if (ptile >= 0) {
#pragma unroll
    for (int p = 0; p < NPART; ++p) epi(p);
  }
  double lpa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lpa[c2] = (FAM == STK_LOGREG) ? 0.5 * lm[c2] - log1p(sp[c2]) : lm[c2];
  __builtin_amdgcn_s_waitcnt(0xF70);
  __syncthreads();
  double* red = lds;
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
      for (int h = 0; h < 4; ++h) v += red[((ww * 64 + h * 16 + l) * NCT + c2) * 2 + kind];
    A.partial[(((size_t)shard * A.Gs + chunk) * G5_C + c) * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

template <int FAM, int NW = 4>
constexpr size_t gemm_fwd_w_lds() { return (size_t)3 * (32 * NW * 16 * 8 + 16 * 512) + EX_TAB * 8; }

}  // namespace stk
