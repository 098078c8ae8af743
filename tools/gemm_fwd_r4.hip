// Round 4's pass F (64-row tiles of 4 waves, 32-column stages in a double buffer, the tile's
// epilogue all at once after its last stage), frozen here as the A/B baseline of
// tools/gemm_fwd_ab.py after the product moved to 128-row tiles (stark_amd/csrc/sweep.hip).
namespace stk {
constexpr int G4_FW = 4;      // pass F: waves per block (two blocks per CU; 8 waves, one block: slower)
constexpr int G4_FS = 2;      // pass F: stages in the ring
constexpr int G4_FKC = 32;    // pass F: columns per stage (32 KB stages; 16 columns x 4 stages: slower)
__host__ __device__ constexpr int g4_fstage_bytes() { return 1024 * G4_FKC; }

// Pass F: one block per (shard, chunk); the chunk's 64-row tiles one after another.  NW waves
// (4: two blocks per CU, a double buffer; 8: one block per CU, the 4-stage ring), each with
// NCT = 16 / NW chain tiles.  With one block per CU every wave reaches the tile epilogue (the
// residual, VALU) at once and the MFMAs idle meanwhile; two blocks overlap one's epilogue with
// the other's GEMM, which measured faster for this pass.
template <int FAM>
__global__ __launch_bounds__(64 * G4_FW, 8 / G4_FW) void k_gemm_fwd_r4(SweepArgs A) {
  constexpr int NW = G4_FW, NS = G4_FS, NCT = 16 / NW;
  constexpr int KCF = G4_FKC, STG = g4_fstage_bytes(), XB = STG / 2;   // stage: [X 64 x KCF][beta^T KCF x 64]
  constexpr int PPR = KCF / 2;                          // 16-B pieces per X row in the stage
  constexpr int NDMA = (XB / 1024) / NW;                // DMA instructions per wave per operand image
  static_assert(NDMA >= 1, "pass F stage geometry");
  // X piece swizzle: 256-B rows (PPR 16) XOR the piece with row & 15; 128-B rows (PPR 8) put
  // rows of one parity on one half of the banks, so XOR with (row >> 1) & 7
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
  char* const stg = reinterpret_cast<char*>(lds);                 // NS stages of STG bytes
  double* const sptab = reinterpret_cast<double*>(stg + NS * STG);
  if constexpr (FAM == STK_LOGREG) exp_table_init(sptab);

  // per-lane chain constants: chain 16 ct + lr, ct = 2 wc + c2
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
  // X stage: slot s (16 B) = row s / PPR, piece (s % PPR) ^ swz(row) of the stage's KCF columns
  int xvo[NDMA];
#pragma unroll
  for (int i = 0; i < NDMA; ++i) {
    const int sl = (w * NDMA + i) * 64 + lane, row = sl / PPR, pc = (sl % PPR) ^ swz(row);
    xvo[i] = row * d * 8 + pc * 16;
  }
  auto issue = [&](int st) {          // global stage index st = tile * NKC + kc
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

  // per chain tile: logistic lm = sum(t - |t|), sp = prod(1 + e) - 1, ll = the flushed log1p(sp)
  // (residual v4, sweep_common.h); linear: lm = sum z^2
  double lm[NCT], sp[NCT], ll[NCT], gaa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lm[c2] = sp[c2] = ll[c2] = gaa[c2] = 0.0;
  char* const Rimg = reinterpret_cast<char*>(A.R + ((size_t)shard * A.Rrows + r0) * G5_C);
  const int nst = ntile * NKC;
  for (int s0 = 0; s0 < NS - 1 && s0 < nst; ++s0) issue(s0);
  dbl4 acc[NCT];
  double yt[4] = {0.0, 0.0, 0.0, 0.0};                  // y of this lane's 4 rows of the current tile
  uint32_t yit[4] = {0u, 0u, 0u, 0u};
  for (int st = 0; st < nst; ++st) {
    const int kc = st % NKC;
    if (kc == 0) {
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) acc[c2] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
    wait_vmcnt(std::min(NS - 2, nst - 1 - st) * 2 * NDMA);   // own DMAs of stage st retired (and the y loads)
    lds_barrier();                                       // stage st landed for every wave; slot of st-1 free
    if (st + NS - 1 < nst) issue(st + NS - 1);
    if (kc == 0) {                                       // the tile's y, needed by its epilogue: one latency per tile
      const int64_t tb = (int64_t)(st / NKC) * G5_TR + 16 * wr + lh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t grow = tb + 4 * i;
        if constexpr (FAM == STK_LOGREG) yit[i] = grow < nrows ? (uint32_t)sh.yi[r0 + grow] : 0u;
        else yt[i] = grow < nrows ? sh.y[r0 + grow] : 0.0;
      }
    }
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
    if (kc == NKC - 1) {                                 // ---- tile epilogue: residual, R, lp
      // straight from the accumulators, every (chain tile, row) unrolled: compile-time indices
      // into alpha / lm / sp, and residual v4 (one exp per element, the logs as a running
      // product per chain tile, flushed every 64 tiles = 256 elements)
      const int tile = st / NKC;
#pragma unroll
      for (int c2 = 0; c2 < NCT; ++c2) {
        const int ct = NCT * wc + c2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 16 * wr + lh + 4 * i;              // row of the tile
          const int64_t grow = (int64_t)tile * G5_TR + row;  // row of the chunk
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
          *reinterpret_cast<double*>(Rimg + g5_chain_off((int)grow, 16 * ct + lr)) = dv;
        }
      }
      if constexpr (FAM == STK_LOGREG) {
        if ((tile & 63) == 63) {
#pragma unroll
          for (int c2 = 0; c2 < NCT; ++c2) {
            ll[c2] += log1p(sp[c2]);
            sp[c2] = 0.0;
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xF70);                  // vmcnt(0): R stores retired before the next counted DMA wait
    }
  }
  double lpa[NCT];
#pragma unroll
  for (int c2 = 0; c2 < NCT; ++c2) lpa[c2] = (FAM == STK_LOGREG) ? 0.5 * lm[c2] - (ll[c2] + log1p(sp[c2])) : lm[c2];

  // ---- lp and sum(d eta) per chain: lanes lr of the 4 row groups h of the 4 waves wr, fixed order
  __syncthreads();
  double* red = lds;                                     // [NW waves][64 lanes][NCT][2]
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

}  // namespace stk
