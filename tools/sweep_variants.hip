// Measurement-only variants of the 16-chain sweep ("tried and measured"):
// k_sweepr (the next sub-tile streamed through VGPRs), k_sweepq and k_sweepx (the 4x4x4
// four-block fp64 MFMA), k_sweepw (one wave per SIMD, software-pipelined).  Each was correct
// and slower than k_sweepe; they are kept here, out of libstark_hip.so, for tools/sweep_micro.hip
// and tools/sweepe_ab.hip only (included after sweep.hip, namespace stk).
// Build: see tools/sweep_micro.hip.
#include "sweep_legacy.hip"
namespace stk {

// v4r: the v4 sub-tile computation with the NEXT sub-tile streamed through registers.
//
// In k_sweepe the next sub-tile's DMA is issued after the forward and must land before the
// next forward, i.e. within the residual + backward of one sub-tile (plus what the SIMD's
// other wave does meanwhile); under full-chip streaming the HBM latency is longer than that
// and the waves wait at vmcnt(0) (PMC: MFMA busy 56 %, f64 VALU 15 %, ~29 % idle).  Here each
// wave keeps PF sub-tiles in flight in VGPRs (global -> VGPR buffer loads, 16 B per lane per
// instruction, 1 KiB contiguous per wave-instruction): sub-tile k+1's loads are issued right
// after sub-tile k has been written into the slot, so they have a whole iteration (PF = 1) or
// two (PF = 2) to land; at the end of the iteration the wave writes them into its LDS slot
// (ds_write_b128, conflict-free: piece p at byte 16 p) and issues the next loads.  The slot
// is never shared, so the backward reads its A operands straight from the slot (no register
// copy) and the slot costs the same LDS as k_sweepe.  Arithmetic, operand layouts, sums and
// their order are exactly k_sweepe's, so the results are bitwise identical.
typedef unsigned int stk_u4 __attribute__((ext_vector_type(4)));
template <int NP>
struct SubtileRegs {                 // one 16-row sub-tile: NP 16-B pieces per lane + y
  stk_u4 x[NP];
  uint64_t y;
};
template <int FAM, int KF, int JT, int PF = 1>
__global__ __launch_bounds__(256, 2) void k_sweepr(SweepArgs A) {
  constexpr int C = SM_C, NW = SM_W, JTV = JT - 1, KP = 4 * KF;
  constexpr int D = KP;                               // d = 4 KF for the shapes this serves
  constexpr int SBX = SM_R * D * 8;                   // X bytes of a sub-tile
  constexpr int NPC = SBX / 16;                       // 16-B pieces of a sub-tile
  constexpr int NP = (NPC + 63) / 64;                 // pieces per lane
  constexpr int LASTL = NPC - 64 * (NP - 1);          // lanes holding a piece in the last round
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  static_assert(SBX % 16 == 0 && LASTL > 0 && PF >= 1 && PF <= 2, "k_sweepr geometry");
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + SM_R - 1) / SM_R;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;
  constexpr int SS = SBX + 128;

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const slot = reinterpret_cast<char*>(lds) + (size_t)w * SS;
  double* const bimg = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * SS);  // [16][KP]
  double* const sptab = bimg + C * KP;
  if constexpr (FAM == STK_LOGREG) softplus_tables_init(sptab);
  const double* qs = A.q + (size_t)shard * C * A.Dp;
  for (int i = tid; i < C * KP; i += NW * 64) {
    const int c = i / KP, col = i % KP;
    bimg[i] = qs[(size_t)c * A.Dp + 1 + col];
  }
  const double alpha = qs[(size_t)lr * A.Dp];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qs[(size_t)lr * A.Dp + D + 1]) : 0.0;
  __syncthreads();

  // rows past the chunk read as zeros (buffer range check) and are masked in the residual
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * D, (int64_t)nrows * D * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  auto load = [&](SubtileRegs<NP>& b, int k) {
    const int xoff = (w + NW * k) * SBX;
#pragma unroll
    for (int j = 0; j < NP - 1; ++j) b.x[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, lane * 16 + j * 1024, xoff, 0);
    b.x[NP - 1] = lane < LASTL ? __builtin_amdgcn_raw_buffer_load_b128(xr, lane * 16 + (NP - 1) * 1024, xoff, 0)
                               : stk_u4{0u, 0u, 0u, 0u};
    const int yoff = (w + NW * k) * SM_R * YB;
    if constexpr (YB == 4) {
      b.y = lane < SM_R ? (uint64_t)__builtin_amdgcn_raw_buffer_load_b32(yr, lane * 4, yoff, 0) : 0u;
    } else {
      b.y = 0;
      if (lane < SM_R) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(yr, lane * 8, yoff, 0);
        b.y = __builtin_bit_cast(uint64_t, v);
      }
    }
  };
  auto store = [&](const SubtileRegs<NP>& b) {
#pragma unroll
    for (int j = 0; j < NP - 1; ++j) *reinterpret_cast<stk_u4*>(slot + lane * 16 + j * 1024) = b.x[j];
    if (lane < LASTL) *reinterpret_cast<stk_u4*>(slot + lane * 16 + (NP - 1) * 1024) = b.x[NP - 1];
    if (lane < SM_R) {
      if constexpr (YB == 4) *reinterpret_cast<uint32_t*>(slot + SBX + lane * 4) = (uint32_t)b.y;
      else *reinterpret_cast<uint64_t*>(slot + SBX + lane * 8) = b.y;
    }
  };

  dbl4 gacc[JTV];
#pragma unroll
  for (int t = 0; t < JTV; ++t) gacc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gv[4] = {0.0, 0.0, 0.0, 0.0};
  double lpa = 0.0, gaa = 0.0;
  const double* xs = reinterpret_cast<const double*>(slot);
  const double* brow = bimg + lr * KP + lh * KF;

  auto compute = [&](int k) {
    const int rv = std::min(SM_R, nrows - SM_R * (w + NW * k));
    // ---- forward
    dbl4 ea[SE_NACC];
#pragma unroll
    for (int i = 0; i < SE_NACC; ++i) ea[i] = dbl4{0.0, 0.0, 0.0, 0.0};
    const double* xrow = xs + lr * D;
#pragma unroll
    for (int s = 0; s < KF; ++s) ea[s % SE_NACC] = mfma_f64(xrow[lh * KF + s], brow[s], ea[s % SE_NACC]);
    dbl4 e0 = ea[0], e1 = ea[1];
#pragma unroll
    for (int i = 2; i < SE_NACC; ++i) { if (i & 1) e1 += ea[i]; else e0 += ea[i]; }
    const dbl4 eta4 = e0 + e1;
    // ---- residual
    double de[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool valid = lh + 4 * i < rv;
      const double eta = eta4[i] + alpha;
      double dv, lt;
      if constexpr (FAM == STK_LOGREG) {
        const double yv = (double)*reinterpret_cast<const int32_t*>(slot + SBX + (lh + 4 * i) * 4);
        const double sgn = 2.0 * yv - 1.0;
        const double ntt = sgn * eta;
        double e, lm, wt;
        softplus_tab(ntt, sptab, &e, &lm, &wt);
        const bool hi = ntt > 20.0, lo = ntt < -20.0;
        lt = hi ? -e : (lo ? ntt : -lm);
        dv = sgn * (hi ? e : (lo ? 1.0 : wt));
      } else {
        const double yv = *reinterpret_cast<const double*>(slot + SBX + (lh + 4 * i) * 8);
        const double z = (yv - eta) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[i] = dv;
    }
    // ---- backward (A operands straight from the slot)
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTV; ++t) gacc[t] = mfma_f64(xs[(lh + 4 * s) * D + 16 * t + lr], de[s], gacc[t]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const dbl2* p = reinterpret_cast<const dbl2*>(xs + (lh + 4 * i) * D + 16 * JTV);
      const dbl2 a0 = p[0], a1 = p[1];
      gv[0] = fma(a0.x, de[i], gv[0]);
      gv[1] = fma(a0.y, de[i], gv[1]);
      gv[2] = fma(a1.x, de[i], gv[2]);
      gv[3] = fma(a1.y, de[i], gv[3]);
    }
  };

  if constexpr (PF == 1) {
    SubtileRegs<NP> b;
    if (mine > 0) {
      load(b, 0);
      store(b);
    }
    if (mine > 1) load(b, 1);
    for (int k = 0; k < mine; ++k) {
      compute(k);
      if (k + 1 < mine) {
        __builtin_amdgcn_sched_barrier(0);
        store(b);                                      // waits for sub-tile k+1's loads
        if (k + 2 < mine) load(b, k + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    // two sub-tiles in flight: b0 holds the even ones, b1 the odd ones
    SubtileRegs<NP> b0, b1;
    if (mine > 0) {
      load(b0, 0);
      store(b0);
    }
    if (mine > 1) load(b1, 1);
    if (mine > 2) load(b0, 2);
    for (int k = 0; k < mine; k += 2) {
      compute(k);
      if (k + 1 < mine) {
        __builtin_amdgcn_sched_barrier(0);
        store(b1);
        if (k + 3 < mine) load(b1, k + 3);
        __builtin_amdgcn_sched_barrier(0);
        compute(k + 1);
        if (k + 2 < mine) {
          __builtin_amdgcn_sched_barrier(0);
          store(b0);
          if (k + 4 < mine) load(b0, k + 4);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }

  // ---- fixed-order block reduction (as k_sweepe)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;
  constexpr int JC = JT * 16;
#pragma unroll
  for (int t = 0; t < JTV; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((size_t)w * JC + 16 * t + lh + 4 * i) * 16 + lr] = gacc[t][i];
  double* red2 = red + (size_t)NW * JC * 16;
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  double* red3 = red2 + (size_t)NW * 64 * 2;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) red3[((size_t)(w * 4 + lh) * 4 + jj) * 16 + lr] = gv[jj];
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  constexpr int jv = 16 * JTV;
  for (int i = tid; i < C * D; i += NW * 64) {
    const int c = i / D, j = i % D;
    double v = 0.0;
    if (j < jv) {
      for (int ww = 0; ww < NW; ++ww) v += red[((size_t)ww * JC + j) * 16 + c];
    } else {
      for (int ww = 0; ww < NW; ++ww)
        for (int h = 0; h < 4; ++h) v += red3[((size_t)(ww * 4 + h) * 4 + (j - jv)) * 16 + c];
    }
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? D + 1 : 0)] = v;
  }
}

// v6 (k_sweepq): the 16-chain sweep on the four-block fp64 MFMA, v_mfma_f64_4x4x4_4b_f64.
//
// On gfx950 the four-block 4x4x4 form issues every 16.5 cycles per SIMD (512 flop: 75 TF/s
// chip-wide), the same rate per flop as v_mfma_f64_16x16x4_f64 (64 cycles, 2048 flop, 78 TF/s;
// profiles/r02zd_mfma_ceiling_vgprform.log -- an earlier reading of 105 cycles was a
// micro-benchmark codegen artefact).  Lane layout (measured,
// tools/mfma4_layout.hip): A lane = m + 4 blk + 16 k, B lane = n + 4 blk + 16 k, D lane =
// n + 4 blk + 16 m.  The four blocks are the four groups of 4 chains, so with lr = lane & 15
// (chain) and lh = lane >> 4 every operand is one f64 per lane and nothing is shuffled:
//   forward   eta[4 rows][16 chains] per 4-row group g, k-step s: A = X[4g + (lane & 3)][4s + lh]
//             (the same in the four blocks: a broadcast LDS read), B = beta_lr[4s + lh] (held in
//             registers for the whole launch); D lane = eta[4g + lh][chain lr];
//   residual  on that one (row, chain) pair per lane and group;
//   backward  G[4 cols][16 chains] += X^T . d_eta per column tile t: A = X[4g + lh][4t + (lane & 3)],
//             B = the residual as it stands (the forward's D layout is the backward's B layout),
//             D lane = G[4t + lh][chain lr]: ceil(d/4) independent accumulators.
// d = 100 is 25 k-steps and 25 column tiles with no padding (the 16 x 16 form pads the
// backward to 112 columns).  Each wave streams S-row sub-tiles through a private ring of NB
// LDS slots with `buffer_load ... lds` (as v3/v4); no barrier in the main loop.  Chunks and
// the chunk-order reduction are v4's, so the gradient is bitwise independent of placement.
__device__ __forceinline__ double mfma4_f64(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__host__ __device__ constexpr int sweepq_slot_bytes(int S, int d) { return S * d * 8 + S * 8; }

// ABL (micro-benchmark ablations only): bit 0 linear residual stand-in, bit 1 no backward, bit 2
// no forward, bit 3 MFMA A operands from registers instead of LDS reads.
template <int FAM, int KF, int S, int NB, int MINB, int ABL = 0>
__global__ __launch_bounds__(256, MINB) void k_sweepq(SweepArgs A) {
  constexpr int C = SM_C, NW = SM_W, G = S / 4;
  static_assert(S % 4 == 0 && G >= 1, "sub-tile rows: a multiple of 4");
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4, l3 = lane & 3;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + S - 1) / S;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;   // own sub-tiles u = w + NW*k
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  const int SBX = S * d * 8;
  const int SS = sweepq_slot_bytes(S, d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const ring = reinterpret_cast<char*>(lds) + (size_t)w * NB * SS;
  double* const sptab = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * NB * SS);
  if constexpr (FAM == STK_LOGREG) {
    softplus_tables_init(sptab);
    __syncthreads();
  }

  // chain lr's beta at columns 4s + lh (B operand of the forward); 0 past d
  const double* qc = A.q + ((size_t)shard * C + lr) * A.Dp;
  double bq[KF];
#pragma unroll
  for (int s = 0; s < KF; ++s) bq[s] = (4 * s + lh < d) ? qc[1 + 4 * s + lh] : 0.0;
  const double alpha = qc[0];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qc[d + 1]) : 0.0;
  __builtin_amdgcn_s_waitcnt(0xF70);                      // ordinary loads retired before the DMAs start

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  const int per_tile = nx + 1;                            // DMA instructions per sub-tile
  auto issue = [&](int k) {
    char* sl = ring + (size_t)(k % NB) * SS;
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + j * 1024), 16, lane * 16, xoff + j * 1024, 0, 0);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, 0);
    if (lane < S * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(sl + SBX), 4, lane * 4, u * S * YB, 0, 0);
  };

  double gacc[KF];
#pragma unroll
  for (int t = 0; t < KF; ++t) gacc[t] = 0.0;
  double lpa = 0.0, gaa = 0.0;

  for (int k = 0; k < NB - 1 && k < mine; ++k) issue(k);
  for (int k = 0; k < mine; ++k) {
    wait_vmcnt(std::max(0, std::min(NB - 2, mine - 1 - k)) * per_tile);   // sub-tile k landed
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): reads of slot k-1 are done
    __builtin_amdgcn_sched_barrier(0);
    if (k + NB - 1 < mine) issue(k + NB - 1);            // into slot (k-1) % NB
    __builtin_amdgcn_sched_barrier(0);
    const char* sl = ring + (size_t)(k % NB) * SS;
    const double* xs = reinterpret_cast<const double*>(sl);
    const int rv = std::min(S, nrows - S * (w + NW * k));

    // ---- forward: two accumulators per 4-row group (k-steps even / odd)
    double ef[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) ef[g][0] = ef[g][1] = 0.0;
    if constexpr (!(ABL & 4)) {
#pragma unroll
      for (int s = 0; s < KF; ++s) {
        const int col = std::min(4 * s + lh, d - 1);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const double a = (ABL & 8) ? bq[(s + g) % KF] : xs[(4 * g + l3) * d + col];
          ef[g][s & 1] = mfma4_f64(a, bq[s], ef[g][s & 1]);
        }
      }
    }

    // ---- residual on (row 4g + lh, chain lr)
    double de[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int row = 4 * g + lh;
      const bool valid = row < rv;
      const double eta = (ef[g][0] + ef[g][1]) + alpha;
      double dv, lt;
      if constexpr (ABL & 1) {
        const int32_t yv = *reinterpret_cast<const int32_t*>(sl + SBX + row * 4);
        dv = (2.0 * yv - 1.0) - 0.25 * eta;
        lt = -dv * dv;
      } else if constexpr (FAM == STK_LOGREG) {
        // Stan's bernoulli_logit: ntt > 20 -> -exp(-ntt); ntt < -20 -> ntt; else -log1p(exp(-ntt))
        const int32_t yv = *reinterpret_cast<const int32_t*>(sl + SBX + row * 4);
        const double sgn = 2.0 * yv - 1.0;
        const double ntt = sgn * eta;
        double e, lm, wt;
        softplus_tab(ntt, sptab, &e, &lm, &wt);
        const bool hi = ntt > 20.0, lo = ntt < -20.0;
        lt = hi ? -e : (lo ? ntt : -lm);
        dv = sgn * (hi ? e : (lo ? 1.0 : wt));
      } else {
        const double yv = *reinterpret_cast<const double*>(sl + SBX + row * 8);
        const double z = (yv - eta) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[g] = dv;
    }

    // ---- backward: KF independent accumulators
    if constexpr (!(ABL & 2)) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double* xrow = xs + (4 * g + lh) * d;
#pragma unroll
        for (int t = 0; t < KF; ++t) {
          const double a = (ABL & 8) ? bq[(t + 3 * g) % KF] : xrow[std::min(4 * t + l3, d - 1)];
          gacc[t] = mfma4_f64(a, de[g], gacc[t]);
        }
      }
    }
  }

  // ---- fixed-order block reduction -> one partial row per chain
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;                                   // [NW][4 KF columns][16 chains]
  constexpr int JC = 4 * KF;
#pragma unroll
  for (int t = 0; t < KF; ++t) red[((size_t)w * JC + 4 * t + lh) * 16 + lr] = gacc[t];
  double* red2 = red + (size_t)NW * JC * 16;           // [NW][64 lanes][lp, g_alpha]
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  for (int i = tid; i < C * d; i += NW * 64) {
    const int c = i / d, j = i % d;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww) v += red[((size_t)ww * JC + j) * 16 + c];
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {          // chain c: lanes h*16 + c of every wave, in (wave, h) order
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}
// v7 (k_sweepx): the four-block 4x4x4 MFMA without replicated operands.
//
// k_sweepq feeds every block the same X values (block = chain group), so each LDS read serves
// one 512-flop MFMA, and the reads, not the MFMAs, set its time (profiles/r02o_micro_qabl.log:
// 20.2 ms, 15.2 ms with the reads replaced by registers).  Here a 16-row sub-tile's four row
// groups are spread over the blocks: in MFMA r block b (= chain group b, chains 4b..4b+3) takes
// row group rho_r(b), a rotation of b by r, so one MFMA covers four row groups x four chain
// groups and the four rotations cover all sixteen pairs.  A lane's operand for rotation r is its
// rotation-0 operand taken from the lane 4r places along its 16-lane row (DPP row_ror), so the
// whole sub-tile enters registers as TWO images of 25 values per lane (d = 100):
//   forward  image F[s]  lane (m, b, k) = X[4b + m][4s + k]   (A of eta = X . beta, K = cols)
//   backward image Bk[t] lane (m, b, k) = X[4b + k][4t + m]   (A of G = X^T . d_eta, K = rows)
// 50 LDS reads per 16 rows instead of 400; the slot is released as soon as both images (and
// the 16 y values) are in registers, and the next sub-tile's DMA streams in during the
// residual + backward (as v4e).  The rotation's direction is whatever the hardware's row_ror
// is: rho_r is obtained by rotating each lane's block index with the same DPP operation.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int R>
__device__ __forceinline__ double rot_blk(double v) {   // R = 0..3: block b gets block rho_R(b)'s value
  if constexpr (R == 0) return v;
  else return dpp_d<0x120 + 4 * R>(v);                   // row_ror:4R
}
template <int R>
__device__ __forceinline__ int rot_blk_i(int v) {
  if constexpr (R == 0) return v;
  else return dpp_i<0x120 + 4 * R>(v);
}

template <int FAM, int KF, int MINB, int ABL = 0>
__global__ __launch_bounds__(256, MINB) void k_sweepx(SweepArgs A) {
  constexpr int C = SM_C, NW = SM_W, S = 16;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4, l3 = lane & 3, blk = (lane >> 2) & 3;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + S - 1) / S;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  const int SBX = S * d * 8;
  const int SS = sweepm_slot_bytes(d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const slot = reinterpret_cast<char*>(lds) + (size_t)w * SS;
  double* const sptab = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * SS);
  if constexpr (FAM == STK_LOGREG) {
    softplus_tables_init(sptab);
    __syncthreads();
  }
  const double* qc = A.q + ((size_t)shard * C + lr) * A.Dp;
  double bq[KF];
#pragma unroll
  for (int s = 0; s < KF; ++s) bq[s] = (4 * s + lh < d) ? qc[1 + 4 * s + lh] : 0.0;
  const double alpha = qc[0];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qc[d + 1]) : 0.0;
  // row group of rotation r at this lane
  int rho[4];
  rho[0] = blk;
  rho[1] = rot_blk_i<1>(blk);
  rho[2] = rot_blk_i<2>(blk);
  rho[3] = rot_blk_i<3>(blk);
  __builtin_amdgcn_s_waitcnt(0xF70);

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  auto issue = [&](int k) {
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + j * 1024), 16, lane * 16, xoff + j * 1024, 0, 0);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(slot + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, 0);
    if (lane < S * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(slot + SBX), 4, lane * 4, u * S * YB, 0, 0);
  };

  double gacc[KF];
#pragma unroll
  for (int t = 0; t < KF; ++t) gacc[t] = 0.0;
  double lpa = 0.0, gaa = 0.0;
  const double* xs = reinterpret_cast<const double*>(slot);

  if (mine > 0) issue(0);
  for (int k = 0; k < mine; ++k) {
    __builtin_amdgcn_s_waitcnt(0xF70);                   // vmcnt(0): sub-tile k landed
    __builtin_amdgcn_sched_barrier(0);
    const int rv = std::min(S, nrows - S * (w + NW * k));
    // ---- forward: 8 accumulators (rotation r, k-step parity)
    double ea[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) ea[r][0] = ea[r][1] = 0.0;
    if constexpr (!(ABL & 4)) {
      const double* xf = xs + (4 * blk + l3) * d;
#pragma unroll
      for (int s = 0; s < KF; ++s) {
        const double a0 = (ABL & 8) ? bq[(s + 1) % KF] : xf[std::min(4 * s + lh, d - 1)];
        ea[0][s & 1] = mfma4_f64(a0, bq[s], ea[0][s & 1]);
        ea[1][s & 1] = mfma4_f64(rot_blk<1>(a0), bq[s], ea[1][s & 1]);
        ea[2][s & 1] = mfma4_f64(rot_blk<2>(a0), bq[s], ea[2][s & 1]);
        ea[3][s & 1] = mfma4_f64(rot_blk<3>(a0), bq[s], ea[3][s & 1]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);                   // keep the backward image's loads below the forward
    // ---- the backward image and y into registers, then the slot is free
    double xb[KF];
    {
      const double* xbr = xs + (4 * blk + lh) * d;
#pragma unroll
      for (int t = 0; t < KF; ++t) xb[t] = (ABL & 8) ? bq[(t + 2) % KF] : xbr[std::min(4 * t + l3, d - 1)];
    }
    double yv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * rho[r] + lh;
      yv[r] = (FAM == STK_LOGREG) ? (double)*reinterpret_cast<const int32_t*>(slot + SBX + row * 4)
                                  : *reinterpret_cast<const double*>(slot + SBX + row * 8);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);                  // lgkmcnt(0): the slot is free
    __builtin_amdgcn_sched_barrier(0);
    if (k + 1 < mine) issue(k + 1);
    __builtin_amdgcn_sched_barrier(0);

    // ---- residual on (row 4 rho_r + lh, chain lr)
    double de[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool valid = 4 * rho[r] + lh < rv;
      const double eta = (ea[r][0] + ea[r][1]) + alpha;
      double dv, lt;
      if constexpr (ABL & 1) {
        dv = (2.0 * yv[r] - 1.0) - 0.25 * eta;
        lt = -dv * dv;
      } else if constexpr (FAM == STK_LOGREG) {
        const double sgn = 2.0 * yv[r] - 1.0;
        const double ntt = sgn * eta;
        double e, lm, wt;
        softplus_tab(ntt, sptab, &e, &lm, &wt);
        const bool hi = ntt > 20.0, lo = ntt < -20.0;
        lt = hi ? -e : (lo ? ntt : -lm);
        dv = sgn * (hi ? e : (lo ? 1.0 : wt));
      } else {
        const double z = (yv[r] - eta) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[r] = dv;
    }
    // ---- backward: rotation r pairs block b's chains with row group rho_r(b)
    // (column tiles in groups of XTB: XTB independent accumulators between two MFMAs on the
    // same one, and only the group's rotated operands live at a time)
    if constexpr (!(ABL & 2)) {
      constexpr int XTB = 5;
#pragma unroll
      for (int t0 = 0; t0 < KF; t0 += XTB) {
#pragma unroll
        for (int t = t0; t < t0 + XTB && t < KF; ++t) gacc[t] = mfma4_f64(xb[t], de[0], gacc[t]);
#pragma unroll
        for (int t = t0; t < t0 + XTB && t < KF; ++t) gacc[t] = mfma4_f64(rot_blk<1>(xb[t]), de[1], gacc[t]);
#pragma unroll
        for (int t = t0; t < t0 + XTB && t < KF; ++t) gacc[t] = mfma4_f64(rot_blk<2>(xb[t]), de[2], gacc[t]);
#pragma unroll
        for (int t = t0; t < t0 + XTB && t < KF; ++t) gacc[t] = mfma4_f64(rot_blk<3>(xb[t]), de[3], gacc[t]);
      }
    }
  }

  // ---- fixed-order block reduction (as k_sweepq)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;
  constexpr int JC = 4 * KF;
#pragma unroll
  for (int t = 0; t < KF; ++t) red[((size_t)w * JC + 4 * t + lh) * 16 + lr] = gacc[t];
  double* red2 = red + (size_t)NW * JC * 16;
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  for (int i = tid; i < C * d; i += NW * 64) {
    const int c = i / d, j = i % d;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww) v += red[((size_t)ww * JC + j) * 16 + c];
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}
static size_t sweepx_lds(int KF, int d) {
  const size_t ring = (size_t)SM_W * sweepm_slot_bytes(d) + SP_TAB * sizeof(double);
  const size_t red = ((size_t)SM_W * 4 * KF * 16 + (size_t)SM_W * 64 * 2) * sizeof(double);
  return std::max(ring, red);
}

// LDS of k_sweepq: the rings + the softplus table, or the reduction, whichever is larger
static size_t sweepq_lds(int S, int NB, int KF, int d) {
  const size_t ring = (size_t)SM_W * NB * sweepq_slot_bytes(S, d) + SP_TAB * sizeof(double);
  const size_t red = ((size_t)SM_W * 4 * KF * 16 + (size_t)SM_W * 64 * 2) * sizeof(double);
  return std::max(ring, red);
}

// v4w (tools/sweepe_ab.hip; measured 17.6 ms against k_sweepe's 14.7 on one box, MFMA busy 48 %
// at 2.2 GHz against 71 % at 1.8: one wave per SIMD does not keep the fp64 pipe fed, as with
// k_sweepf in round 2 -- profiles/r03t_*): k_sweepe's arithmetic at ONE wave per SIMD
// (one 256-thread block per CU), software-pipelined so the wave itself keeps the fp64 pipe busy:
// two LDS slots per wave (the DMA of sub-tile k+2 is issued at the top of sub-tile k, a whole
// iteration before it is needed), beta's B fragments in registers (the wave has 512), and per
// iteration
//   phase A: the residual of sub-tile k (VALU)  interleaved with  the forward of sub-tile k+1 (MFMA)
//   phase B: the backward of sub-tile k (MFMA)  interleaved with  the reads of sub-tile k+1's
//            backward operands, y and remainder columns from its slot (LDS)
// with the backward operands double-buffered in registers by sub-tile parity.
template <int FAM, int KF, int JT, int AUX = 2, int SGB = 1>
__global__ __launch_bounds__(256, 1) void k_sweepw(SweepArgs A) {
  constexpr int C = SM_C, NW = SM_W, JTV = JT - 1;
  const int shard = A.shard0 + blockIdx.x / A.G;
  const int chunk = blockIdx.x % A.G;
  if (A.req_step && A.req_step[shard] != A.step_id - 1) return;
  if (A.ran && chunk == 0 && threadIdx.x == 0) atomicAdd(&A.ran[A.step_id & 63], 1);
  const ShardDev sh = A.shards[shard];
  const int d = sh.d;
  const int tid = threadIdx.x, lane = tid & 63, w = uniform_int(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int64_t nt = (sh.n + 63) / 64;
  const int64_t t0 = nt * chunk / A.G, t1 = nt * (chunk + 1) / A.G;
  const int64_t r0 = t0 * 64, r1 = std::min<int64_t>(sh.n, t1 * 64);
  const int nrows = (int)(r1 - r0);
  const int nsub = (nrows + SM_R - 1) / SM_R;
  const int mine = nsub > w ? (nsub - w + NW - 1) / NW : 0;
  constexpr int YB = (FAM == STK_LOGREG) ? 4 : 8;
  const int SBX = SM_R * d * 8;
  const int SS = sweepm_slot_bytes(d);

  extern __shared__ __attribute__((aligned(16))) double lds[];
  char* const slots = reinterpret_cast<char*>(lds) + (size_t)w * 2 * SS;
  double* const sptab = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + (size_t)NW * 2 * SS);
  if constexpr (FAM == STK_LOGREG) logit3_tables_init(sptab);
  const double* qc = A.q + ((size_t)shard * C + lr) * A.Dp;
  double bf[KF];
#pragma unroll
  for (int s = 0; s < KF; ++s) {
    const int col = lh * KF + s;
    bf[s] = col < d ? qc[1 + col] : 0.0;
  }
  const double alpha = qc[0];
  const double inv_s = (FAM == STK_LINREG) ? exp(-qc[d + 1]) : 0.0;
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0xF70);

  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(sh.x + r0 * d, (int64_t)nrows * d * 8);
  const void* ybase = (FAM == STK_LOGREG) ? (const void*)(sh.yi + r0) : (const void*)(sh.y + r0);
  const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(ybase, (int64_t)nrows * YB);
  const int nx = (SBX + 1023) >> 10;
  const int last_lanes = (SBX - ((nx - 1) << 10)) >> 4;
  const int per_tile = nx + 1;
  auto slot_of = [&](int k) { return slots + (size_t)(k & 1) * SS; };
  auto issue = [&](int k) {
    char* const sl = slot_of(k);
    const int u = w + NW * k;
    const int xoff = u * SBX;
    for (int j = 0; j < nx - 1; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + j * 1024), 16, lane * 16, xoff + j * 1024, 0, AUX);
    if (lane < last_lanes)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_vptr)(sl + (nx - 1) * 1024), 16, lane * 16,
                                               xoff + (nx - 1) * 1024, 0, AUX);
    if (lane < SM_R * YB / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_vptr)(sl + SBX), 4, lane * 4, u * SM_R * YB, 0, AUX);
  };

  dbl4 gacc[JTV];
#pragma unroll
  for (int t = 0; t < JTV; ++t) gacc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gv[4] = {0.0, 0.0, 0.0, 0.0};
  double lpa = 0.0, gaa = 0.0;
  // per-sub-tile operands, double-buffered by parity
  double xa[2][4][JTV];
  dbl2 xv[2][4][2];
  double yv[2][4];
  uint32_t ym[2][4];
  dbl4 eta = {0.0, 0.0, 0.0, 0.0};

  auto forward = [&](int k) {                        // eta of sub-tile k, alpha in the accumulator
    const double* xrow = reinterpret_cast<const double*>(slot_of(k)) + lr * d;
    dbl4 e0 = FAM == STK_LOGREG ? dbl4{alpha, alpha, alpha, alpha} : dbl4{0.0, 0.0, 0.0, 0.0};
    dbl4 e1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KF; ++s) {
      if (s & 1) e1 = mfma_f64(xrow[lh * KF + s], bf[s], e1);      // d == 4 KF (host-checked)
      else e0 = mfma_f64(xrow[lh * KF + s], bf[s], e0);
    }
    return e0 + e1;
  };
  auto read_rest = [&](int k, auto P) {              // backward operands, remainder columns, y
    constexpr int par = decltype(P)::value;
    const char* sl = slot_of(k);
    const double* xs = reinterpret_cast<const double*>(sl);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTV; ++t) xa[par][s][t] = xs[(lh + 4 * s) * d + 16 * t + lr];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const dbl2* pv = reinterpret_cast<const dbl2*>(xs + (lh + 4 * i) * d + 16 * JTV);
      xv[par][i][0] = pv[0];
      xv[par][i][1] = pv[1];
      if constexpr (FAM == STK_LOGREG)
        ym[par][i] = ((uint32_t)*reinterpret_cast<const int32_t*>(sl + SBX + (lh + 4 * i) * 4) << 31) + 0x80000000u;
      else
        yv[par][i] = *reinterpret_cast<const double*>(sl + SBX + (lh + 4 * i) * 8);
    }
  };

  if (mine > 0) issue(0);
  if (mine > 1) issue(1);
  if (mine > 0) {
    wait_vmcnt(mine > 1 ? per_tile : 0);
    __builtin_amdgcn_sched_barrier(0);
    eta = forward(0);
    read_rest(0, std::integral_constant<int, 0>{});
  }

  auto body = [&](int k, auto P, auto M) {
    constexpr int par = decltype(P)::value;
    constexpr int nxt = par ^ 1;
    constexpr bool more = decltype(M)::value;         // a sub-tile k+1 follows (the last one is peeled)
    __builtin_amdgcn_s_waitcnt(0xC07F);                 // lgkmcnt(0): slot k fully read (last iteration)
    __builtin_amdgcn_sched_barrier(0);
    if (k + 2 < mine) issue(k + 2);                     // into slot k's
    if constexpr (more) wait_vmcnt(k + 2 < mine ? per_tile : 0);   // sub-tile k+1 landed
    __builtin_amdgcn_sched_barrier(0);
    const int rv = std::min(SM_R, nrows - SM_R * (w + NW * k));
    // ---- phase A: residual of k, forward of k+1
    double de[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool valid = lh + 4 * i < rv;
      double lt, dv;
      if constexpr (FAM == STK_LOGREG) {
        logit_resid3(eta[i], ym[par][i], sptab, lt, dv);
      } else {
        const double z = (yv[par][i] - (eta[i] + alpha)) * inv_s;
        lt = z * z;
        dv = z * inv_s;
      }
      dv = valid ? dv : 0.0;
      lpa += valid ? lt : 0.0;
      gaa += dv;
      de[i] = dv;
    }
    dbl4 eta_n = eta;
    if constexpr (more) eta_n = forward(k + 1);
    if constexpr (SGB && more) {
#pragma unroll
      for (int s = 0; s < KF; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);   // 6 VALU
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase B: backward of k, reads of k+1's operands
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < JTV; ++t) gacc[t] = mfma_f64(xa[par][s][t], de[s], gacc[t]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gv[0] = fma(xv[par][i][0].x, de[i], gv[0]);
      gv[1] = fma(xv[par][i][0].y, de[i], gv[1]);
      gv[2] = fma(xv[par][i][1].x, de[i], gv[2]);
      gv[3] = fma(xv[par][i][1].y, de[i], gv[3]);
    }
    if constexpr (more) read_rest(k + 1, std::integral_constant<int, nxt>{});
    if constexpr (SGB && more) {
#pragma unroll
      for (int s = 0; s < 4 * JTV; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);   // 1 VALU
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    eta = eta_n;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  int k = 0;
  for (; k + 2 < mine; k += 2) {                      // pairs with a successor each
    body(k, I0{}, T_{});
    body(k + 1, I1{}, T_{});
  }
  if (k + 1 < mine) {                                 // two left: the second is the last
    body(k, I0{}, T_{});
    body(k + 1, I1{}, F_{});
  } else if (k < mine) {                              // one left
    body(k, I0{}, F_{});
  }

  // ---- fixed-order block reduction (as k_sweepe)
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __syncthreads();
  double* red = lds;
  constexpr int JC = JT * 16;
#pragma unroll
  for (int t = 0; t < JTV; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((size_t)w * JC + 16 * t + lh + 4 * i) * 16 + lr] = gacc[t][i];
  double* red2 = red + (size_t)NW * JC * 16;
  red2[(size_t)tid * 2 + 0] = lpa;
  red2[(size_t)tid * 2 + 1] = gaa;
  double* red3 = red2 + (size_t)NW * 64 * 2;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) red3[((size_t)(w * 4 + lh) * 4 + jj) * 16 + lr] = gv[jj];
  __syncthreads();
  double* out = A.partial + ((size_t)shard * A.Gs + chunk) * C * A.PW;
  const int jv = 16 * JTV;
  for (int i = tid; i < C * d; i += NW * 64) {
    const int c = i / d, j = i % d;
    double v = 0.0;
    if (j < jv) {
      for (int ww = 0; ww < NW; ++ww) v += red[((size_t)ww * JC + j) * 16 + c];
    } else {
      for (int ww = 0; ww < NW; ++ww)
        for (int h = 0; h < 4; ++h) v += red3[((size_t)(ww * 4 + h) * 4 + (j - jv)) * 16 + c];
    }
    out[(size_t)c * A.PW + 1 + j] = v;
  }
  if (tid < 2 * C) {
    const int c = tid >> 1, kind = tid & 1;
    double v = 0.0;
    for (int ww = 0; ww < NW; ++ww)
      for (int h = 0; h < 4; ++h) v += red2[(size_t)(ww * 64 + h * 16 + c) * 2 + kind];
    out[(size_t)c * A.PW + (kind == 0 ? d + 1 : 0)] = v;
  }
}

}  // namespace stk
