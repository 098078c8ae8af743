// C ABI of libstark_hip.so (declared in include/stark_hip.h).  Host-side orchestration
// only: every numeric result comes from a gfx950 kernel; there is no CPU fallback.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "common.h"
#include <cmath>

using namespace stk;

// ---- kernels' launchers (other translation units)
int stk_nch_for(int Dmax);
hipError_t stk_launch_nuts_init(const NutsArgs& A, const double* init, const double* inv_metric, double stepsize,
                                double init_radius, hipStream_t st);
hipError_t stk_launch_nuts_step(const NutsArgs& A, int nch, int step_id, int pause_at, hipStream_t st);
hipError_t stk_launch_nuts_fused(const NutsArgs& A, int nch, int pause_at, int max_steps, hipStream_t st);
hipError_t stk_launch_schools_lpgrad(const ShardDev* shards, int shard, int nch, const double* q, int C, int Dp,
                                     double* lp, double* g, hipStream_t st);
void stk_sweep_geometry(int64_t n, int d, int* T, int* LD, int* G, size_t* lds_bytes, int C);
bool stk_sweep_supported(int C, int d);
hipError_t stk_launch_sweep(int family, const ShardDev* shards_dev, int shard0, int nsh, int64_t n, int d, int T, int LD, int G,
                            int Gs, size_t lds, const double* q, int C, int Dp, double* partial, const int* req_step,
                            int step_id, int* ran, hipStream_t st, const SweepWs* ws = nullptr);
size_t stk_sweep_ws_bytes(int64_t n_max, int d, int C, int nshards);
SweepWs stk_sweep_ws(void* base, int64_t n_max, int d, int nshards);
hipError_t stk_launch_sweep_reduce(int family, const ShardDev* shards_dev, int shard0, int nsh, int d, int G, int Gs,
                                   const double* q, int C, int Dp, double* partial, const int* req_step, int step_id,
                                   double* lp_out, double* g_out, hipStream_t st);
hipError_t stk_launch_check_y01(const int32_t* y, int64_t n, int64_t* first, hipStream_t st);
hipError_t stk_launch_gen_shard(double* X, double* yd, int32_t* yi, int64_t nrows, int d, int64_t grow0,
                                uint64_t seed, double alpha, const double* beta, double noise_sigma, int family,
                                hipStream_t st);
hipError_t stk_launch_consensus_products(const double* X, int nshards, int P, int S, const int32_t* blk, double* mean,
                                         int32_t* rowbad, int32_t* used, int32_t* status, double* cov, double* W,
                                         double* work, double* sum_w, double* sum_wtheta, hipStream_t st);
size_t stk_general_inverse_work_bytes(int P);
hipError_t stk_launch_consensus_solve(const double* sum_w, const double* sum_wtheta, int P, int S, double* inv_buf,
                                      double* work, int32_t* status, double* out, hipStream_t st, bool general);
size_t stk_spd_inverse_work_bytes(int P, int batch);

// ---------------------------------------------------------------- errors
static thread_local char g_err[1024] = "";
void stk_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
#define ARG_CHECK(cond, ...)          \
  do {                                \
    if (!(cond)) {                    \
      stk_set_error(__VA_ARGS__);     \
      return STK_E_ARG;               \
    }                                 \
  } while (0)
#define RC(expr)                      \
  do {                                \
    int _rc = (expr);                 \
    if (_rc != STK_OK) return _rc;    \
  } while (0)

// ---------------------------------------------------------------- device buffers
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  int ensure(size_t bytes) {
    if (bytes <= n && p) return STK_OK;
    if (p) hipFree(p);
    p = nullptr;
    n = 0;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      p = nullptr;
      stk_set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
      return STK_E_NOMEM;
    }
    n = bytes;
    return STK_OK;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// Handles are reference counted (a model holds its context, a sampler its model), so the
// caller may destroy them in any order -- e.g. a garbage collector finalising a cycle.
struct stk_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = true;     // false: a caller's stream (stk_ctx_create_on_stream), not destroyed here
  int profiling = 0;
  int refs = 1;
  DevBuf scratch[12];
};

struct stk_model {
  int refs = 1;
  stk_ctx* ctx = nullptr;
  int family = 0;
  int nshards = 0;
  int d = 0;
  int Dmax = 0, Pmax = 0;
  std::vector<ShardDev> sh;
  std::vector<DevBuf> bufs;
  DevBuf sh_dev;
  int64_t bytes = 0;
};

struct stk_sampler {
  stk_model* m = nullptr;
  stk_config cfg{};
  NutsArgs A{};
  int nch = 1;
  int step = 0;
  int64_t steps = 0;
  int64_t sweeps = 0;
  int64_t shard_sweeps = 0;
  double sweep_ms = 0.0;
  std::vector<DevBuf> bufs;
  DevBuf partial, lp, g, ran, ws;
  SweepWs sws{};
  stk_allreduce_fn ar_fn = nullptr;   // full-data mode: rank-sum of [grad | lp] after every reduce
  void* ar_user = nullptr;
  int Gs = 1;
  struct Group { int shard0, nsh, T, LD, G; size_t lds; };
  std::vector<Group> groups;
  std::vector<hipEvent_t> ev;
  std::vector<int> iv_host;
  std::vector<unsigned long long> cnt_host;
};

extern "C" {

const char* stk_last_error(void) { return g_err; }
int stk_version(void) { return 1; }

void stk_config_default(stk_config* c) {
  memset(c, 0, sizeof(*c));
  c->num_warmup = 1000;
  c->num_samples = 1000;
  c->chains = 1;
  c->max_depth = 10;
  c->adapt_delta = 0.8;
  c->adapt_gamma = 0.05;
  c->adapt_kappa = 0.75;
  c->adapt_t0 = 10.0;
  c->stepsize = 1.0;
  c->init_radius = 2.0;
  c->adapt_init_buffer = 75;
  c->adapt_term_buffer = 50;
  c->adapt_window = 25;
  c->adapt_engaged = 1;
  c->seed = 1234;
}

// ---------------------------------------------------------------- context
int stk_ctx_create(int device, stk_ctx** out) {
  ARG_CHECK(out, "stk_ctx_create: out is NULL");
  int n = 0;
  STK_HIP_CHECK(hipGetDeviceCount(&n));
  ARG_CHECK(device >= 0 && device < n, "stk_ctx_create: device %d not in [0, %d)", device, n);
  STK_HIP_CHECK(hipSetDevice(device));
  stk_ctx* c = new stk_ctx();
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    stk_set_error("hipStreamCreate failed: %s", hipGetErrorString(e));
    return STK_E_HIP;
  }
  *out = c;
  return STK_OK;
}

int stk_ctx_create_on_stream(int device, void* stream, stk_ctx** out) {
  ARG_CHECK(out, "stk_ctx_create_on_stream: out is NULL");   // stream NULL = the device's null stream
  int n = 0;
  STK_HIP_CHECK(hipGetDeviceCount(&n));
  ARG_CHECK(device >= 0 && device < n, "stk_ctx_create_on_stream: device %d not in [0, %d)", device, n);
  STK_HIP_CHECK(hipSetDevice(device));
  stk_ctx* c = new stk_ctx();
  c->device = device;
  c->stream = (hipStream_t)stream;
  c->own_stream = false;
  *out = c;
  return STK_OK;
}

static void ctx_release(stk_ctx* c) {
  if (--c->refs > 0) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto& b : c->scratch) b.release();
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
}

int stk_ctx_destroy(stk_ctx* c) {
  if (c) ctx_release(c);
  return STK_OK;
}

int stk_ctx_sync(stk_ctx* c) {
  ARG_CHECK(c, "stk_ctx_sync: NULL context");
  STK_HIP_CHECK(hipSetDevice(c->device));
  STK_HIP_CHECK(hipStreamSynchronize(c->stream));
  return STK_OK;
}

int stk_ctx_set_profiling(stk_ctx* c, int on) {
  ARG_CHECK(c, "NULL context");
  ARG_CHECK(on >= 0, "stk_ctx_set_profiling: on must be >= 0");
  c->profiling = on;
  return STK_OK;
}

void* stk_ctx_stream(stk_ctx* c) { return c ? (void*)c->stream : nullptr; }

// ---------------------------------------------------------------- models
static int family_dims(int family, int64_t n, int d, int* D, int* P) {
  switch (family) {
    case STK_SCHOOLS: *D = (int)n + 2; *P = 2 * (int)n + 3; return STK_OK;
    case STK_LINREG: *D = d + 2; *P = d + 3; return STK_OK;
    case STK_LOGREG: *D = d + 1; *P = d + 2; return STK_OK;
  }
  stk_set_error("unknown model family %d", family);
  return STK_E_ARG;
}

static int upload(stk_model* m, const void* src, size_t bytes, void** dst) {
  m->bufs.emplace_back();
  DevBuf& b = m->bufs.back();
  RC(b.ensure(bytes));
  STK_HIP_CHECK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyDefault, m->ctx->stream));
  *dst = b.p;
  m->bytes += (int64_t)bytes;
  return STK_OK;
}

static int finish_model(stk_model* m) {
  m->Dmax = 0;
  m->Pmax = 0;
  for (auto& s : m->sh) {
    m->Dmax = std::max(m->Dmax, s.D);
    m->Pmax = std::max(m->Pmax, s.P);
  }
  RC(m->sh_dev.ensure(sizeof(ShardDev) * m->sh.size()));
  STK_HIP_CHECK(hipMemcpyAsync(m->sh_dev.p, m->sh.data(), sizeof(ShardDev) * m->sh.size(), hipMemcpyHostToDevice,
                               m->ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(m->ctx->stream));
  return STK_OK;
}

int stk_model_create(stk_ctx* ctx, int family, const stk_shard* shards, int nshards, stk_model** out) {
  ARG_CHECK(ctx && shards && out && nshards > 0, "stk_model_create: bad arguments");
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  stk_model* m = new stk_model();
  m->ctx = ctx;
  ctx->refs++;
  m->family = family;
  m->nshards = nshards;
  m->d = family == STK_SCHOOLS ? 0 : shards[0].n_cols;
  int rc = STK_OK;
  for (int s = 0; s < nshards && rc == STK_OK; ++s) {
    const stk_shard& in = shards[s];
    ShardDev sd{};
    sd.n = in.n_rows;
    sd.d = family == STK_SCHOOLS ? 0 : in.n_cols;
    if (in.n_rows <= 0) { stk_set_error("shard %d: n_rows must be positive", s); rc = STK_E_ARG; break; }
    if (family != STK_SCHOOLS && in.n_cols != m->d) {
      stk_set_error("shard %d: n_cols %d differs from shard 0 (%d)", s, in.n_cols, m->d);
      rc = STK_E_ARG;
      break;
    }
    rc = family_dims(family, in.n_rows, sd.d, &sd.D, &sd.P);
    if (rc) break;
    void* p = nullptr;
    if (family == STK_SCHOOLS) {
      if (!in.y || !in.sigma) { stk_set_error("shard %d: schools needs y and sigma", s); rc = STK_E_ARG; break; }
      if ((rc = upload(m, in.y, sizeof(double) * in.n_rows, &p))) break;
      sd.y = (const double*)p;
      if ((rc = upload(m, in.sigma, sizeof(double) * in.n_rows, &p))) break;
      sd.sigma = (const double*)p;
    } else {
      if (!in.x || in.n_cols <= 0) { stk_set_error("shard %d: regression needs x", s); rc = STK_E_ARG; break; }
      if (!stk_sweep_supported(1, in.n_cols)) { stk_set_error("n_cols %d unsupported (1..1024)", in.n_cols); rc = STK_E_ARG; break; }
      if ((rc = upload(m, in.x, sizeof(double) * in.n_rows * in.n_cols, &p))) break;
      sd.x = (const double*)p;
      if (family == STK_LOGREG) {
        if (!in.y_int) { stk_set_error("shard %d: logreg needs y_int", s); rc = STK_E_ARG; break; }
        if ((rc = upload(m, in.y_int, sizeof(int32_t) * in.n_rows, &p))) break;
        sd.yi = (const int32_t*)p;
        {   // bernoulli_logit: y in {0, 1} (the sweeps read y as a sign bit), checked on the device
            // copy by a reduction that returns the first bad row (8 bytes back, not the shard)
          DevBuf flag;
          if ((rc = flag.ensure(sizeof(int64_t)))) break;
          int64_t bad = -1;
          int32_t v = 0;
          hipError_t e = stk_launch_check_y01(sd.yi, in.n_rows, flag.as<int64_t>(), m->ctx->stream);
          if (e == hipSuccess) e = hipMemcpyAsync(&bad, flag.p, sizeof(int64_t), hipMemcpyDeviceToHost, m->ctx->stream);
          if (e == hipSuccess) e = hipStreamSynchronize(m->ctx->stream);
          if (e == hipSuccess && bad >= 0 && bad < in.n_rows)
            e = hipMemcpy(&v, sd.yi + bad, sizeof(int32_t), hipMemcpyDeviceToHost);
          flag.release();
          if (e != hipSuccess) {
            stk_set_error("shard %d: y_int check failed: %s", s, hipGetErrorString(e));
            rc = STK_E_HIP;
            break;
          }
          if (bad >= 0 && bad < in.n_rows) {
            stk_set_error("shard %d: y_int[%lld] = %d; bernoulli_logit needs 0 or 1", s, (long long)bad, v);
            rc = STK_E_ARG;
            break;
          }
        }
      } else {
        if (!in.y) { stk_set_error("shard %d: linreg needs y", s); rc = STK_E_ARG; break; }
        if ((rc = upload(m, in.y, sizeof(double) * in.n_rows, &p))) break;
        sd.y = (const double*)p;
      }
    }
    m->sh.push_back(sd);
  }
  if (rc == STK_OK) rc = finish_model(m);
  if (rc != STK_OK) {
    stk_model_destroy(m);
    return rc;
  }
  *out = m;
  return STK_OK;
}

int stk_gen_beta(uint64_t seed, int32_t d, double* beta) {
  ARG_CHECK(beta && d > 0, "stk_gen_beta: bad arguments");
  const double s = 1.0 / sqrt((double)d);
  for (int j = 0; j < d; ++j) beta[j] = normal_at(seed, (uint32_t)(j >> 1) & ~0u, 0u, 0u, (uint32_t)(j & 1), TAG_BETA) * s;
  return STK_OK;
}

int stk_model_create_synthetic(stk_ctx* ctx, int family, int nshards, int64_t rows_per_shard, int64_t row_offset,
                               int32_t n_cols, uint64_t data_seed, double alpha, const double* beta,
                               double noise_sigma, stk_model** out) {
  ARG_CHECK(ctx && out && nshards > 0 && rows_per_shard > 0 && n_cols > 0, "stk_model_create_synthetic: bad arguments");
  ARG_CHECK(family == STK_LOGREG || family == STK_LINREG, "synthetic shards exist for linreg/logreg only");
  ARG_CHECK(stk_sweep_supported(1, n_cols), "n_cols %d unsupported (1..1024)", n_cols);
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  std::vector<double> b(n_cols);
  if (beta) memcpy(b.data(), beta, sizeof(double) * n_cols);
  else stk_gen_beta(data_seed, n_cols, b.data());
  stk_model* m = new stk_model();
  m->ctx = ctx;
  ctx->refs++;
  m->family = family;
  m->nshards = nshards;
  m->d = n_cols;
  int rc = STK_OK;
  DevBuf beta_dev;
  rc = beta_dev.ensure(sizeof(double) * n_cols);
  if (rc == STK_OK && hipMemcpy(beta_dev.p, b.data(), sizeof(double) * n_cols, hipMemcpyHostToDevice) != hipSuccess) {
    stk_set_error("beta upload failed");
    rc = STK_E_HIP;
  }
  for (int s = 0; s < nshards && rc == STK_OK; ++s) {
    ShardDev sd{};
    sd.n = rows_per_shard;
    sd.d = n_cols;
    family_dims(family, rows_per_shard, n_cols, &sd.D, &sd.P);
    m->bufs.emplace_back();
    if ((rc = m->bufs.back().ensure(sizeof(double) * rows_per_shard * n_cols))) break;
    double* X = m->bufs.back().as<double>();
    m->bufs.emplace_back();
    const size_t ybytes = family == STK_LOGREG ? sizeof(int32_t) * rows_per_shard : sizeof(double) * rows_per_shard;
    if ((rc = m->bufs.back().ensure(ybytes))) break;
    void* y = m->bufs.back().p;
    m->bytes += (int64_t)(sizeof(double) * rows_per_shard * n_cols + ybytes);
    hipError_t e = stk_launch_gen_shard(X, family == STK_LINREG ? (double*)y : nullptr,
                                        family == STK_LOGREG ? (int32_t*)y : nullptr, rows_per_shard, n_cols,
                                        row_offset + (int64_t)s * rows_per_shard, data_seed, alpha,
                                        beta_dev.as<double>(), noise_sigma, family, ctx->stream);
    if (e != hipSuccess) { stk_set_error("gen_shard launch: %s", hipGetErrorString(e)); rc = STK_E_HIP; break; }
    sd.x = X;
    if (family == STK_LOGREG) sd.yi = (const int32_t*)y;
    else sd.y = (const double*)y;
    m->sh.push_back(sd);
  }
  if (rc == STK_OK) rc = finish_model(m);
  beta_dev.release();
  if (rc != STK_OK) {
    stk_model_destroy(m);
    return rc;
  }
  *out = m;
  return STK_OK;
}

static void model_release(stk_model* m) {
  if (--m->refs > 0) return;
  stk_ctx* c = m->ctx;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto& b : m->bufs) b.release();
  m->sh_dev.release();
  delete m;
  ctx_release(c);
}

int stk_model_destroy(stk_model* m) {
  if (m) model_release(m);
  return STK_OK;
}

int stk_model_info(const stk_model* m, int shard, int32_t* D, int32_t* P, int64_t* n_rows) {
  ARG_CHECK(m && shard >= 0 && shard < m->nshards, "stk_model_info: bad shard");
  if (D) *D = m->sh[shard].D;
  if (P) *P = m->sh[shard].P;
  if (n_rows) *n_rows = m->sh[shard].n;
  return STK_OK;
}

int stk_model_device_bytes(const stk_model* m, int64_t* bytes) {
  ARG_CHECK(m && bytes, "bad arguments");
  *bytes = m->bytes;
  return STK_OK;
}

int stk_model_copy_data(stk_model* m, int shard, double* x, double* y, int32_t* y_int) {
  ARG_CHECK(m && shard >= 0 && shard < m->nshards, "stk_model_copy_data: bad shard");
  STK_HIP_CHECK(hipSetDevice(m->ctx->device));
  const ShardDev& s = m->sh[shard];
  hipStream_t st = m->ctx->stream;
  if (x && s.x) STK_HIP_CHECK(hipMemcpyAsync(x, s.x, sizeof(double) * s.n * s.d, hipMemcpyDefault, st));
  if (y && s.y) STK_HIP_CHECK(hipMemcpyAsync(y, s.y, sizeof(double) * s.n, hipMemcpyDefault, st));
  if (y_int && s.yi) STK_HIP_CHECK(hipMemcpyAsync(y_int, s.yi, sizeof(int32_t) * s.n, hipMemcpyDefault, st));
  STK_HIP_CHECK(hipStreamSynchronize(st));
  return STK_OK;
}

// ---------------------------------------------------------------- lp / grad (parity hook)
int stk_log_density_grad(stk_model* m, int shard, const double* q, int32_t C, double* lp, double* grad) {
  ARG_CHECK(m && q && lp && C > 0 && shard >= 0 && shard < m->nshards, "stk_log_density_grad: bad arguments");
  stk_ctx* ctx = m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const ShardDev& s = m->sh[shard];
  const int D = s.D;
  const int Dp = (m->Dmax + 7) / 8 * 8;
  hipStream_t st = ctx->stream;
  const ShardDev* shd = m->sh_dev.as<ShardDev>();
  if (m->family == STK_SCHOOLS) {
    RC(ctx->scratch[0].ensure(sizeof(double) * (size_t)C * Dp));
    RC(ctx->scratch[1].ensure(sizeof(double) * (size_t)C));
    RC(ctx->scratch[2].ensure(sizeof(double) * (size_t)C * Dp));
    STK_HIP_CHECK(hipMemcpy2DAsync(ctx->scratch[0].p, sizeof(double) * Dp, q, sizeof(double) * D, sizeof(double) * D,
                                   C, hipMemcpyDefault, st));
    STK_HIP_CHECK(stk_launch_schools_lpgrad(shd, shard, stk_nch_for(m->Dmax), ctx->scratch[0].as<double>(), C, Dp,
                                            ctx->scratch[1].as<double>(), ctx->scratch[2].as<double>(), st));
  } else {
    int T, LD, G;
    size_t lds;
    // the chain batch the sampler's sweep uses: 64 (two-pass fp64 MFMA GEMMs) from 64 points,
    // 16 (fp64 MFMA) from 16 when d <= 128, else 4 / 2 / 1
    const int Cb = C <= 1 ? 1 : (C <= 2 ? 2 : (C >= 64 ? 64 : (C < 16 || !stk_sweep_supported(16, s.d) ? 4 : 16)));
    stk_sweep_geometry(s.n, s.d, &T, &LD, &G, &lds, Cb);
    const int PW = s.d + 2;
    const size_t wsb = stk_sweep_ws_bytes(s.n, s.d, Cb, m->nshards);
    SweepWs ws{};
    if (wsb) {
      RC(ctx->scratch[4].ensure(wsb));
      ws = stk_sweep_ws(ctx->scratch[4].p, s.n, s.d, m->nshards);
    }
    RC(ctx->scratch[0].ensure(sizeof(double) * (size_t)(m->nshards * Cb) * Dp));
    RC(ctx->scratch[1].ensure(sizeof(double) * (size_t)(m->nshards * Cb)));
    RC(ctx->scratch[2].ensure(sizeof(double) * (size_t)(m->nshards * Cb) * Dp));
    RC(ctx->scratch[3].ensure(sizeof(double) * (size_t)m->nshards * G * Cb * PW));
    for (int c0 = 0; c0 < C; c0 += Cb) {
      const int nb = std::min(Cb, C - c0);
      // the kernel reads rows shard*Cb + c of the point buffer
      double* qb = ctx->scratch[0].as<double>() + (size_t)shard * Cb * Dp;
      for (int c = 0; c < Cb; ++c) {
        const int src = c0 + std::min(c, nb - 1);
        STK_HIP_CHECK(hipMemcpyAsync(qb + (size_t)c * Dp, q + (size_t)src * D, sizeof(double) * D, hipMemcpyDefault, st));
      }
      STK_HIP_CHECK(stk_launch_sweep(m->family, shd, shard, 1, s.n, s.d, T, LD, G, G, lds, ctx->scratch[0].as<double>(), Cb,
                                     Dp, ctx->scratch[3].as<double>(), nullptr, 0, nullptr, st, wsb ? &ws : nullptr));
      STK_HIP_CHECK(stk_launch_sweep_reduce(m->family, shd, shard, 1, s.d, G, G, ctx->scratch[0].as<double>(), Cb, Dp,
                                            ctx->scratch[3].as<double>(), nullptr, 0, ctx->scratch[1].as<double>(),
                                            ctx->scratch[2].as<double>(), st));
      double* lpb = ctx->scratch[1].as<double>() + (size_t)shard * Cb;
      double* gb = ctx->scratch[2].as<double>() + (size_t)shard * Cb * Dp;
      STK_HIP_CHECK(hipMemcpyAsync(lp + c0, lpb, sizeof(double) * nb, hipMemcpyDefault, st));
      if (grad)
        STK_HIP_CHECK(hipMemcpy2DAsync(grad + (size_t)c0 * D, sizeof(double) * D, gb, sizeof(double) * Dp,
                                       sizeof(double) * D, nb, hipMemcpyDefault, st));
    }
    STK_HIP_CHECK(hipStreamSynchronize(st));
    return STK_OK;
  }
  STK_HIP_CHECK(hipMemcpyAsync(lp, ctx->scratch[1].p, sizeof(double) * C, hipMemcpyDefault, st));
  if (grad)
    STK_HIP_CHECK(hipMemcpy2DAsync(grad, sizeof(double) * D, ctx->scratch[2].p, sizeof(double) * Dp, sizeof(double) * D,
                                   C, hipMemcpyDefault, st));
  STK_HIP_CHECK(hipStreamSynchronize(st));
  return STK_OK;
}

// ---------------------------------------------------------------- sampler
static int sbuf(stk_sampler* s, size_t bytes, void** p) {
  s->bufs.emplace_back();
  RC(s->bufs.back().ensure(bytes));
  *p = s->bufs.back().p;
  return STK_OK;
}

int stk_sampler_destroy(stk_sampler* s) {
  if (!s) return STK_OK;
  stk_model* m = s->m;
  hipSetDevice(m->ctx->device);
  hipStreamSynchronize(m->ctx->stream);
  for (auto& b : s->bufs) b.release();
  s->partial.release();
  s->lp.release();
  s->g.release();
  s->ran.release();
  s->ws.release();
  for (auto e : s->ev) hipEventDestroy(e);
  delete s;
  model_release(m);
  return STK_OK;
}

int stk_sampler_create(stk_model* m, const stk_config* cfg, stk_sampler** out) {
  ARG_CHECK(m && cfg && out, "stk_sampler_create: bad arguments");
  ARG_CHECK(cfg->num_warmup >= 0 && cfg->num_samples > 0 && cfg->chains > 0, "need num_warmup>=0, num_samples>0, chains>0");
  ARG_CHECK(cfg->max_depth >= 1 && cfg->max_depth <= 30, "max_depth must be in [1, 30]");
  ARG_CHECK(cfg->adapt_delta > 0 && cfg->adapt_delta < 1, "adapt_delta must be in (0, 1)");
  ARG_CHECK(cfg->stepsize > 0, "stepsize must be positive");
  ARG_CHECK(cfg->stepsize_jitter >= 0 && cfg->stepsize_jitter <= 1, "stepsize_jitter must be in [0, 1]");
  ARG_CHECK(cfg->nuts_criterion == 0 || cfg->nuts_criterion == 1, "nuts_criterion must be 0 (Stan 2.19) or 1 (Stan >= 2.23)");
  ARG_CHECK(cfg->chains_per_wave >= 0 && cfg->chains_per_wave <= 4 && cfg->chains_per_wave != 3,
            "chains_per_wave must be 0, 1, 2 or 4");
  stk_ctx* ctx = m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const int nch = stk_nch_for(m->Dmax);
  ARG_CHECK(nch > 0, "dimension %d too large (max 1024)", m->Dmax);
  if (m->family == STK_SCHOOLS) ARG_CHECK(nch <= 2, "8-schools supports J <= 126");
  else ARG_CHECK(stk_sweep_supported(cfg->chains, m->d), "chains per shard must be 1, 2, 4, 8, 16 (d <= 128) or 64 for regressions");
  stk_sampler* s = new stk_sampler();
  s->m = m;
  m->refs++;
  s->cfg = *cfg;
  s->nch = nch;
  NutsArgs& A = s->A;
  const int nchains = m->nshards * cfg->chains;
  A.nchains = nchains;
  A.C = cfg->chains;
  A.Dp = (m->Dmax + 7) / 8 * 8;
  A.family = m->family;
  A.max_depth = cfg->max_depth;
  A.num_warmup = cfg->num_warmup;
  A.num_samples = cfg->num_samples;
  A.total_iters = cfg->num_warmup + cfg->num_samples;
  A.adapt = cfg->adapt_engaged && cfg->num_warmup > 0;
  A.skip_ss = cfg->skip_init_stepsize;
  A.iter_offset = cfg->iter_offset;
  unsigned nw = (unsigned)cfg->num_warmup, ib = (unsigned)cfg->adapt_init_buffer, tb = (unsigned)cfg->adapt_term_buffer,
           bw = (unsigned)cfg->adapt_window;
  A.var_on = A.adapt && nw >= 20;
  if (A.var_on && ib + bw + tb > nw) {   // windowed_adaptation::set_window_params, 15%/75%/10%
    ib = (unsigned)(0.15 * nw);
    tb = (unsigned)(0.1 * nw);
    bw = nw - (ib + tb);
  }
  A.init_buffer = ib;
  A.term_buffer = tb;
  A.base_window = bw;
  A.delta = cfg->adapt_delta;
  A.gamma = cfg->adapt_gamma;
  A.kappa = cfg->adapt_kappa;
  A.t0 = cfg->adapt_t0;
  A.seed = cfg->seed;
  A.jitter = cfg->stepsize_jitter;
  A.uturn_ext = cfg->nuts_criterion;
  A.cpw_cap = cfg->chains_per_wave;
  A.S_total = cfg->chains * cfg->num_samples;
  A.Pmax = m->Pmax;
  A.shards = m->sh_dev.as<ShardDev>();
  const size_t Dp = A.Dp;
  int rc = STK_OK;
  void* p;
#define ALLOC(field, type, count)                                            \
  if (rc == STK_OK && (rc = sbuf(s, sizeof(type) * (size_t)(count), &p)) == STK_OK) A.field = (type*)p;
  ALLOC(vec, double, (size_t)nchains * V_COUNT * Dp);
  ALLOC(stk, double, (size_t)nchains * cfg->max_depth * SV_COUNT * Dp);
  ALLOC(sc, double, (size_t)nchains * S_COUNT);
  ALLOC(stks, double, (size_t)nchains * cfg->max_depth * SS_COUNT);
  ALLOC(iv, int, (size_t)nchains * I_COUNT);
  ALLOC(cnt, unsigned long long, (size_t)nchains * C_COUNT);
  ALLOC(qeval, double, (size_t)nchains * Dp);
  // g_in and lp_in are one block, [nchains][Dp] then [nchains]: the unit of the full-data all-reduce
  ALLOC(g_in, double, (size_t)nchains * Dp + nchains);
  if (rc == STK_OK) A.lp_in = A.g_in + (size_t)nchains * Dp;
  ALLOC(draws, double, (size_t)m->nshards * m->Pmax * A.S_total);
  ALLOC(stats, double, (size_t)m->nshards * A.S_total * N_STATS);
  A.ud_first = cfg->save_warmup ? 0 : cfg->num_warmup;
  A.ud_iters = A.total_iters - A.ud_first;
  ALLOC(udraws, double, (size_t)nchains * A.ud_iters * Dp);
  ALLOC(req_step, int, (size_t)m->nshards);
#undef ALLOC
  double* init_dev = nullptr;
  double* im_dev = nullptr;
  if (rc == STK_OK && cfg->init) {
    // init is nshards * chains * D with per-shard D; repack to Dmax stride per chain
    std::vector<double> h((size_t)nchains * m->Dmax, 0.0);
    std::vector<double> tmp;
    size_t off = 0;
    for (int sh = 0; sh < m->nshards; ++sh) {
      const int D = m->sh[sh].D;
      for (int c = 0; c < cfg->chains; ++c) {
        tmp.resize(D);
        if (hipMemcpy(tmp.data(), cfg->init + off, sizeof(double) * D, hipMemcpyDefault) != hipSuccess) rc = STK_E_ARG;
        memcpy(&h[(size_t)(sh * cfg->chains + c) * m->Dmax], tmp.data(), sizeof(double) * D);
        off += D;
      }
    }
    // k_nuts_init reads init[gid * D(shard)] -- store each chain at gid * D_shard
    std::vector<double> packed((size_t)nchains * m->Dmax, 0.0);
    for (int gid = 0; gid < nchains; ++gid) {
      const int D = m->sh[gid / cfg->chains].D;
      memcpy(&packed[(size_t)gid * D], &h[(size_t)gid * m->Dmax], sizeof(double) * D);
    }
    if (rc == STK_OK && (rc = sbuf(s, sizeof(double) * packed.size(), &p)) == STK_OK) {
      init_dev = (double*)p;
      if (hipMemcpy(init_dev, packed.data(), sizeof(double) * packed.size(), hipMemcpyHostToDevice) != hipSuccess)
        rc = STK_E_HIP;
    }
  }
  if (rc == STK_OK && cfg->shard_ids) {
    std::vector<int32_t> ids(m->nshards);
    if (hipMemcpy(ids.data(), cfg->shard_ids, sizeof(int32_t) * m->nshards, hipMemcpyDefault) != hipSuccess) rc = STK_E_ARG;
    for (int v : ids)
      if (v < 0) rc = STK_E_ARG;
    if (rc == STK_OK && (rc = sbuf(s, sizeof(int32_t) * m->nshards, &p)) == STK_OK) {
      if (hipMemcpy(p, ids.data(), sizeof(int32_t) * m->nshards, hipMemcpyHostToDevice) != hipSuccess) rc = STK_E_HIP;
      A.shard_ids = (const int*)p;
    }
    if (rc == STK_E_ARG) stk_set_error("shard_ids: unreadable or negative");
  }
  if (rc == STK_OK && cfg->inv_metric) {
    if ((rc = sbuf(s, sizeof(double) * m->Dmax, &p)) == STK_OK) {
      im_dev = (double*)p;
      if (hipMemcpy(im_dev, cfg->inv_metric, sizeof(double) * m->Dmax, hipMemcpyDefault) != hipSuccess) rc = STK_E_HIP;
    }
  }
  if (rc == STK_OK && m->family != STK_SCHOOLS) {
    // sweep geometry, grouped by consecutive shards of equal n
    int gmax = 1;
    for (int sh = 0; sh < m->nshards;) {
      stk_sampler::Group gr{};
      gr.shard0 = sh;
      stk_sweep_geometry(m->sh[sh].n, m->d, &gr.T, &gr.LD, &gr.G, &gr.lds, cfg->chains);
      int e = sh + 1;
      while (e < m->nshards && m->sh[e].n == m->sh[sh].n) ++e;
      gr.nsh = e - sh;
      gmax = std::max(gmax, gr.G);
      s->groups.push_back(gr);
      sh = e;
    }
    s->Gs = gmax;
    rc = s->partial.ensure(sizeof(double) * (size_t)m->nshards * gmax * cfg->chains * (m->d + 2));
    int64_t nmax = 0;
    for (int sh = 0; sh < m->nshards; ++sh) nmax = std::max<int64_t>(nmax, m->sh[sh].n);
    const size_t wsb = stk_sweep_ws_bytes(nmax, m->d, cfg->chains, m->nshards);
    if (rc == STK_OK && wsb) {
      rc = s->ws.ensure(wsb);
      if (rc == STK_OK) s->sws = stk_sweep_ws(s->ws.p, nmax, m->d, m->nshards);
    }
    if (rc == STK_OK) rc = s->ran.ensure(sizeof(int) * 64);
  }
  if (rc == STK_OK) {
    hipError_t e = stk_launch_nuts_init(A, init_dev, im_dev, cfg->stepsize, cfg->init_radius, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(A.draws, 0, sizeof(double) * (size_t)m->nshards * m->Pmax * A.S_total, ctx->stream);
    // a zeroed tree stack: the fused kernel's zero-padding form relies on +0 in every padding slot
    if (e == hipSuccess)
      e = hipMemsetAsync(A.stk, 0, sizeof(double) * (size_t)nchains * cfg->max_depth * SV_COUNT * Dp, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
      stk_set_error("sampler init: %s", hipGetErrorString(e));
      rc = STK_E_HIP;
    }
  }
  if (rc != STK_OK) {
    stk_sampler_destroy(s);
    return rc;
  }
  s->iv_host.resize((size_t)nchains * I_COUNT);
  s->cnt_host.resize((size_t)nchains * C_COUNT);
  *out = s;
  return STK_OK;
}

// Read chain modes/iterations; returns true when no chain has work below pause_at.
static int poll(stk_sampler* s, int pause_at, bool* idle) {
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipMemcpyAsync(s->iv_host.data(), s->A.iv, sizeof(int) * s->iv_host.size(), hipMemcpyDeviceToHost,
                               ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  bool any = false;
  for (int c = 0; c < s->A.nchains; ++c) {
    const int mode = s->iv_host[(size_t)c * I_COUNT + I_MODE];
    const int it = s->iv_host[(size_t)c * I_COUNT + I_ITER];
    if (mode == M_INIT || mode == M_PROBE || mode == M_TRAJ) any = true;
    if (mode == M_PAUSED && it < pause_at) any = true;
  }
  *idle = !any;
  return STK_OK;
}

static int run_split_batch(stk_sampler* s, int nsteps, int pause_at) {
  stk_model* m = s->m;
  stk_ctx* ctx = m->ctx;
  hipStream_t st = ctx->stream;
  NutsArgs& A = s->A;
  const int every = ctx->profiling;            // events around the sweeps of every n-th step
  const bool prof = every > 0;
  if (prof) {
    while ((int)s->ev.size() < 2 * nsteps) {
      hipEvent_t e;
      STK_HIP_CHECK(hipEventCreate(&e));
      s->ev.push_back(e);
    }
    STK_HIP_CHECK(hipMemsetAsync(s->ran.p, 0, sizeof(int) * 64, st));
  }
  const int step0 = s->step;
  for (int k = 0; k < nsteps; ++k) {
    const int step_id = s->step;
    const bool pk = prof && step_id % every == 0;
    if (pk) STK_HIP_CHECK(hipEventRecord(s->ev[2 * k], st));
    for (const auto& gr : s->groups) {
      STK_HIP_CHECK(stk_launch_sweep(m->family, A.shards, gr.shard0, gr.nsh, m->sh[gr.shard0].n, m->d, gr.T, gr.LD, gr.G, s->Gs, gr.lds,
                                     A.qeval, A.C, A.Dp, s->partial.as<double>(), A.req_step, step_id,
                                     prof ? s->ran.as<int>() : nullptr, st, s->sws.qT ? &s->sws : nullptr));
    }
    if (pk) STK_HIP_CHECK(hipEventRecord(s->ev[2 * k + 1], st));
    for (const auto& gr : s->groups) {
      STK_HIP_CHECK(stk_launch_sweep_reduce(m->family, A.shards, gr.shard0, gr.nsh, m->d, gr.G, s->Gs, A.qeval, A.C,
                                            A.Dp, s->partial.as<double>(), A.req_step, step_id, A.lp_in, A.g_in, st));
    }
    if (s->ar_fn) {
      const int r = s->ar_fn(s->ar_user, A.g_in, (int64_t)A.nchains * (A.Dp + 1), (void*)st);
      if (r != 0) {
        stk_set_error("full-data all-reduce callback failed (%d) at step %d", r, step_id);
        return STK_E_STATE;
      }
    }
    STK_HIP_CHECK(stk_launch_nuts_step(A, s->nch, step_id, pause_at, st));
    s->step++;
    s->steps++;
  }
  if (prof) {
    int ran[64];
    STK_HIP_CHECK(hipMemcpyAsync(ran, s->ran.p, sizeof(int) * 64, hipMemcpyDeviceToHost, st));
    STK_HIP_CHECK(hipStreamSynchronize(st));
    for (int k = 0; k < nsteps; ++k) {
      if ((step0 + k) % every != 0 || !ran[(step0 + k) & 63]) continue;
      float ms = 0.f;
      STK_HIP_CHECK(hipEventElapsedTime(&ms, s->ev[2 * k], s->ev[2 * k + 1]));
      s->sweep_ms += ms;
      s->sweeps += 1;
      s->shard_sweeps += ran[(step0 + k) & 63];
    }
  }
  return STK_OK;
}

int stk_sampler_run(stk_sampler* s, int32_t target_iter, int64_t max_steps) {
  ARG_CHECK(s, "stk_sampler_run: NULL sampler");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const int pause_at = std::min(target_iter, s->A.total_iters);
  int64_t done_steps = 0;
  int batch = 4;
  for (;;) {
    bool idle = false;
    RC(poll(s, pause_at, &idle));
    if (idle) break;
    if (max_steps > 0 && done_steps >= max_steps) break;
    if (s->m->family == STK_SCHOOLS) {
      const int ms = 4096;
      STK_HIP_CHECK(stk_launch_nuts_fused(s->A, s->nch, pause_at, ms, ctx->stream));
      done_steps += ms;
      s->steps += 1;
    } else {
      int nb = batch;
      if (max_steps > 0) nb = (int)std::min<int64_t>(nb, max_steps - done_steps);
      RC(run_split_batch(s, nb, pause_at));
      done_steps += nb;
      batch = std::min(batch * 2, 64);
    }
  }
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

int stk_model_set_prior(stk_model* m, double alpha_scale, double beta_scale) {
  ARG_CHECK(m, "stk_model_set_prior: NULL model");
  ARG_CHECK(m->family == STK_LOGREG || m->family == STK_LINREG, "priors apply to the regression families");
  ARG_CHECK(alpha_scale >= 0.0 && beta_scale >= 0.0, "prior scales must be >= 0 (0 or inf: flat)");
  auto prec = [](double sc) { return (sc == 0.0 || std::isinf(sc)) ? 0.0 : 1.0 / (sc * sc); };
  for (auto& sd : m->sh) {
    sd.pa = prec(alpha_scale);
    sd.pb = prec(beta_scale);
  }
  STK_HIP_CHECK(hipSetDevice(m->ctx->device));
  STK_HIP_CHECK(hipMemcpy(m->sh_dev.p, m->sh.data(), sizeof(ShardDev) * m->sh.size(), hipMemcpyHostToDevice));
  return STK_OK;
}

int stk_sampler_grad_block(stk_sampler* s, int64_t* count) {
  ARG_CHECK(s && count, "stk_sampler_grad_block: bad arguments");
  *count = (int64_t)s->A.nchains * (s->A.Dp + 1);
  return STK_OK;
}

int stk_sampler_set_allreduce(stk_sampler* s, stk_allreduce_fn fn, void* user, double* dev_block) {
  ARG_CHECK(s, "stk_sampler_set_allreduce: NULL sampler");
  ARG_CHECK(s->m->family == STK_LOGREG,
            "full-data mode needs a purely additive log density (logistic: flat priors, no Jacobian term)");
  ARG_CHECK(s->step == 0, "stk_sampler_set_allreduce: call before the first stk_sampler_run");
  for (const auto& sd : s->m->sh)
    ARG_CHECK(sd.pa == 0.0 && sd.pb == 0.0, "full-data mode: flat priors only (a prior would be summed once per rank)");
  const size_t n = (size_t)s->A.nchains * (s->A.Dp + 1);
  if (dev_block) {
    STK_HIP_CHECK(hipSetDevice(s->m->ctx->device));
    STK_HIP_CHECK(hipMemsetAsync(dev_block, 0, sizeof(double) * n, s->m->ctx->stream));
    s->A.g_in = dev_block;
    s->A.lp_in = dev_block + (size_t)s->A.nchains * s->A.Dp;
  }
  s->ar_fn = fn;
  s->ar_user = user;
  return STK_OK;
}

int stk_sampler_info(stk_sampler* s, stk_run_info* info) {
  ARG_CHECK(s && info, "stk_sampler_info: bad arguments");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  STK_HIP_CHECK(hipMemcpyAsync(s->cnt_host.data(), s->A.cnt, sizeof(unsigned long long) * s->cnt_host.size(),
                               hipMemcpyDeviceToHost, ctx->stream));
  STK_HIP_CHECK(hipMemcpyAsync(s->iv_host.data(), s->A.iv, sizeof(int) * s->iv_host.size(), hipMemcpyDeviceToHost,
                               ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  memset(info, 0, sizeof(*info));
  info->min_iter = 1 << 30;
  for (int c = 0; c < s->A.nchains; ++c) {
    info->grad_evals += (int64_t)s->cnt_host[(size_t)c * C_COUNT + C_GRAD];
    info->leapfrogs += (int64_t)s->cnt_host[(size_t)c * C_COUNT + C_LEAP];
    info->divergent += (int32_t)s->cnt_host[(size_t)c * C_COUNT + C_DIV];
    const int mode = s->iv_host[(size_t)c * I_COUNT + I_MODE];
    info->min_iter = std::min(info->min_iter, s->iv_host[(size_t)c * I_COUNT + I_ITER]);
    if (mode == M_DONE) info->done++;
    if (mode == M_ERROR) info->errors++;
  }
  info->steps = s->steps;
  info->sweeps = s->sweeps;
  info->shard_sweeps = s->shard_sweeps;
  info->sweep_ms = s->sweep_ms;
  return STK_OK;
}

int stk_sampler_draws(stk_sampler* s, int shard, double* out, double* stats) {
  ARG_CHECK(s && shard >= 0 && shard < s->m->nshards, "stk_sampler_draws: bad shard");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const size_t S = (size_t)s->A.S_total;
  const int P = s->m->sh[shard].P;
  if (out)
    STK_HIP_CHECK(hipMemcpyAsync(out, s->A.draws + (size_t)shard * s->A.Pmax * S, sizeof(double) * P * S,
                                 hipMemcpyDefault, ctx->stream));
  if (stats)
    STK_HIP_CHECK(hipMemcpyAsync(stats, s->A.stats + (size_t)shard * S * N_STATS, sizeof(double) * S * N_STATS,
                                 hipMemcpyDefault, ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

int stk_sampler_draws_unconstrained(stk_sampler* s, int shard, double* out) {
  ARG_CHECK(s && out && shard >= 0 && shard < s->m->nshards, "bad arguments");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const int D = s->m->sh[shard].D;
  const size_t rows = (size_t)s->A.C * s->A.ud_iters;
  const double* src = s->A.udraws + (size_t)shard * rows * s->A.Dp;
  STK_HIP_CHECK(hipMemcpy2DAsync(out, sizeof(double) * D, src, sizeof(double) * s->A.Dp, sizeof(double) * D, rows,
                                 hipMemcpyDefault, ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

int stk_sampler_adaptation(stk_sampler* s, double* stepsize, double* inv_metric) {
  ARG_CHECK(s, "NULL sampler");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const int n = s->A.nchains;
  if (stepsize)
    STK_HIP_CHECK(hipMemcpy2DAsync(stepsize, sizeof(double), s->A.sc + S_NOMEPS, sizeof(double) * S_COUNT,
                                   sizeof(double), n, hipMemcpyDefault, ctx->stream));
  if (inv_metric) {
    for (int c = 0; c < n; ++c) {
      const int D = s->m->sh[c / s->A.C].D;
      STK_HIP_CHECK(hipMemcpyAsync(inv_metric + (size_t)c * s->m->Dmax,
                                   s->A.vec + ((size_t)c * V_COUNT + V_IM) * s->A.Dp, sizeof(double) * D,
                                   hipMemcpyDefault, ctx->stream));
    }
  }
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

int stk_sampler_iterations(stk_sampler* s, int32_t* iters) {
  ARG_CHECK(s && iters, "stk_sampler_iterations: bad arguments");
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  STK_HIP_CHECK(hipMemcpy2DAsync(iters, sizeof(int32_t), s->A.iv + I_ITER, sizeof(int) * I_COUNT, sizeof(int32_t),
                                 s->A.nchains, hipMemcpyDefault, ctx->stream));
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- checkpoint / resume
// Blob: StateHeader, then the device segments in state_segments() order.  The header's
// geometry hash covers everything that shapes the state or its evolution (model family and
// shard geometry, priors, every sampler setting, the RNG seed and shard ids), so a blob only
// loads into a sampler that continues the same run.
namespace {
struct StateHeader {
  char magic[8];
  uint32_t version, nsegs;
  uint64_t geometry;
  int64_t step, steps, sweeps, shard_sweeps;
  double sweep_ms;
  uint64_t seg_bytes[16];
};
struct Seg {
  void* p;
  size_t bytes;
};
const char kStateMagic[8] = {'S', 'T', 'K', 'S', 'T', 'A', 'T', 'E'};

std::vector<Seg> state_segments(const stk_sampler* s) {
  const NutsArgs& A = s->A;
  const size_t n = (size_t)A.nchains, Dp = (size_t)A.Dp, md = (size_t)A.max_depth;
  const size_t nsh = (size_t)s->m->nshards, S = (size_t)A.S_total;
  return {{A.vec, sizeof(double) * n * V_COUNT * Dp},
          {A.stk, sizeof(double) * n * md * SV_COUNT * Dp},
          {A.sc, sizeof(double) * n * S_COUNT},
          {A.stks, sizeof(double) * n * md * SS_COUNT},
          {A.iv, sizeof(int) * n * I_COUNT},
          {A.cnt, sizeof(unsigned long long) * n * C_COUNT},
          {A.qeval, sizeof(double) * n * Dp},
          {A.g_in, sizeof(double) * (n * Dp + n)},       // [grad | lp] at the pending requests
          {A.draws, sizeof(double) * nsh * s->m->Pmax * S},
          {A.stats, sizeof(double) * nsh * S * N_STATS},
          {A.udraws, sizeof(double) * n * (size_t)A.ud_iters * Dp},
          {A.req_step, sizeof(int) * nsh}};
}

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  template <class T>
  void add(const T& v) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(&v);
    for (size_t i = 0; i < sizeof(T); ++i) h = (h ^ b[i]) * 1099511628211ull;
  }
};

int state_geometry(const stk_sampler* s, uint64_t* out) {
  const NutsArgs& A = s->A;
  const stk_model* m = s->m;
  Fnv f;
  f.add(m->family), f.add(m->nshards), f.add(m->d), f.add(m->Dmax), f.add(m->Pmax);
  for (const auto& sd : m->sh) f.add(sd.n), f.add(sd.D), f.add(sd.P), f.add(sd.pa), f.add(sd.pb);
  f.add(A.nchains), f.add(A.C), f.add(A.Dp), f.add(A.max_depth), f.add(A.num_warmup), f.add(A.num_samples);
  f.add(A.adapt), f.add(A.var_on), f.add(A.skip_ss), f.add(A.iter_offset);
  f.add(A.init_buffer), f.add(A.term_buffer), f.add(A.base_window);
  f.add(A.delta), f.add(A.gamma), f.add(A.kappa), f.add(A.t0), f.add(A.seed), f.add(A.jitter);
  f.add(A.uturn_ext), f.add(A.cpw_cap), f.add(A.ud_first), f.add(A.ud_iters), f.add(s->nch);
  std::vector<int32_t> ids(m->nshards);
  for (int i = 0; i < m->nshards; ++i) ids[i] = i;
  if (A.shard_ids)
    STK_HIP_CHECK(hipMemcpy(ids.data(), A.shard_ids, sizeof(int32_t) * ids.size(), hipMemcpyDeviceToHost));
  for (int v : ids) f.add(v);
  *out = f.h;
  return STK_OK;
}
}  // namespace

extern "C" {

int stk_sampler_state_bytes(stk_sampler* s, int64_t* bytes) {
  ARG_CHECK(s && bytes, "stk_sampler_state_bytes: bad arguments");
  size_t n = sizeof(StateHeader);
  for (const Seg& g : state_segments(s)) n += g.bytes;
  *bytes = (int64_t)n;
  return STK_OK;
}

int stk_sampler_save_state(stk_sampler* s, void* buf, int64_t bytes) {
  ARG_CHECK(s && buf, "stk_sampler_save_state: bad arguments");
  int64_t need = 0;
  RC(stk_sampler_state_bytes(s, &need));
  ARG_CHECK(bytes >= need, "stk_sampler_save_state: buffer of %lld bytes, the state needs %lld", (long long)bytes,
            (long long)need);
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  const auto segs = state_segments(s);
  StateHeader h{};
  memcpy(h.magic, kStateMagic, 8);
  h.version = 1;
  h.nsegs = (uint32_t)segs.size();
  RC(state_geometry(s, &h.geometry));
  h.step = s->step;
  h.steps = s->steps;
  h.sweeps = s->sweeps;
  h.shard_sweeps = s->shard_sweeps;
  h.sweep_ms = s->sweep_ms;
  for (size_t i = 0; i < segs.size(); ++i) h.seg_bytes[i] = segs[i].bytes;
  char* out = static_cast<char*>(buf);
  memcpy(out, &h, sizeof(h));
  size_t off = sizeof(h);
  for (const Seg& g : segs) {
    STK_HIP_CHECK(hipMemcpyAsync(out + off, g.p, g.bytes, hipMemcpyDefault, ctx->stream));
    off += g.bytes;
  }
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  return STK_OK;
}

int stk_sampler_load_state(stk_sampler* s, const void* buf, int64_t bytes) {
  ARG_CHECK(s && buf, "stk_sampler_load_state: bad arguments");
  int64_t need = 0;
  RC(stk_sampler_state_bytes(s, &need));
  ARG_CHECK(bytes == need, "stk_sampler_load_state: blob of %lld bytes, this sampler's state has %lld",
            (long long)bytes, (long long)need);
  stk_ctx* ctx = s->m->ctx;
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  StateHeader h;
  memcpy(&h, buf, sizeof(h));
  const auto segs = state_segments(s);
  uint64_t geo = 0;
  RC(state_geometry(s, &geo));
  ARG_CHECK(!memcmp(h.magic, kStateMagic, 8) && h.version == 1, "stk_sampler_load_state: not a sampler state blob");
  ARG_CHECK(h.geometry == geo && h.nsegs == segs.size(),
            "stk_sampler_load_state: the state belongs to another model geometry or sampler config");
  for (size_t i = 0; i < segs.size(); ++i)
    ARG_CHECK(h.seg_bytes[i] == segs[i].bytes, "stk_sampler_load_state: segment %zu size mismatch", i);
  const char* in = static_cast<const char*>(buf) + sizeof(h);
  for (const Seg& g : segs) {
    STK_HIP_CHECK(hipMemcpyAsync(g.p, in, g.bytes, hipMemcpyDefault, ctx->stream));
    in += g.bytes;
  }
  STK_HIP_CHECK(hipStreamSynchronize(ctx->stream));
  s->step = (int)h.step;
  s->steps = h.steps;
  s->sweeps = h.sweeps;
  s->shard_sweeps = h.shard_sweeps;
  s->sweep_ms = h.sweep_ms;
  return STK_OK;
}

int stk_sample(stk_model* m, const stk_config* cfg, double* draws, double* stats, stk_run_info* info) {
  stk_sampler* s = nullptr;
  RC(stk_sampler_create(m, cfg, &s));
  int rc = stk_sampler_run(s, cfg->num_warmup + cfg->num_samples, 0);
  stk_run_info inf{};
  if (rc == STK_OK) rc = stk_sampler_info(s, &inf);
  if (rc == STK_OK && inf.errors) {
    stk_set_error("%d chain(s) stopped: step size left (0, 1e7] during init_stepsize", inf.errors);
    rc = STK_E_NUMERIC;
  }
  const size_t S = (size_t)cfg->chains * cfg->num_samples;
  for (int sh = 0; rc == STK_OK && sh < m->nshards; ++sh)
    rc = stk_sampler_draws(s, sh, draws ? draws + (size_t)sh * m->Pmax * S : nullptr,
                           stats ? stats + (size_t)sh * S * N_STATS : nullptr);
  if (info) *info = inf;
  stk_sampler_destroy(s);
  return rc;
}

int stk_transition(stk_model* m, int shard, double* q, int32_t C, uint64_t seed, int32_t iteration, double eps,
                   const double* inv_metric, int32_t max_depth, double* lp, double* stats) {
  ARG_CHECK(m && q && C > 0 && shard >= 0 && shard < m->nshards, "stk_transition: bad arguments");
  const int D = m->sh[shard].D;
  stk_config cfg;
  stk_config_default(&cfg);
  cfg.num_warmup = 0;
  cfg.num_samples = 1;
  cfg.chains = C;
  cfg.max_depth = max_depth;
  cfg.adapt_engaged = 0;
  cfg.stepsize = eps;
  cfg.seed = seed;
  cfg.skip_init_stepsize = 1;
  cfg.iter_offset = iteration;
  std::vector<double> qh((size_t)C * D);
  if (hipMemcpy(qh.data(), q, sizeof(double) * qh.size(), hipMemcpyDefault) != hipSuccess) {
    stk_set_error("stk_transition: cannot read q");
    return STK_E_ARG;
  }
  std::vector<double> init;
  for (int sh = 0; sh < m->nshards; ++sh) {
    const int Ds = m->sh[sh].D;
    for (int c = 0; c < C; ++c)
      for (int e = 0; e < Ds; ++e) init.push_back(e < D ? qh[(size_t)c * D + e] : 0.0);
  }
  cfg.init = init.data();
  std::vector<double> im;
  if (inv_metric) {
    im.assign(m->Dmax, 1.0);
    std::vector<double> tmp(D);
    if (hipMemcpy(tmp.data(), inv_metric, sizeof(double) * D, hipMemcpyDefault) != hipSuccess) return STK_E_ARG;
    std::copy(tmp.begin(), tmp.end(), im.begin());
    cfg.inv_metric = im.data();
  }
  stk_sampler* s = nullptr;
  RC(stk_sampler_create(m, &cfg, &s));
  int rc = stk_sampler_run(s, 1, 0);
  if (rc == STK_OK) rc = stk_sampler_draws_unconstrained(s, shard, qh.data());
  if (rc == STK_OK) {
    const int P = m->sh[shard].P;
    std::vector<double> dr((size_t)P * C), stv((size_t)C * N_STATS);
    rc = stk_sampler_draws(s, shard, dr.data(), stv.data());
    if (rc == STK_OK) {
      if (lp)
        for (int c = 0; c < C; ++c) lp[c] = dr[(size_t)(P - 1) * C + c];
      if (stats) memcpy(stats, stv.data(), sizeof(double) * stv.size());
      if (hipMemcpy(q, qh.data(), sizeof(double) * qh.size(), hipMemcpyDefault) != hipSuccess) rc = STK_E_HIP;
    }
  }
  stk_sampler_destroy(s);
  return rc;
}

// ---------------------------------------------------------------- consensus combine
// Device buffers of one combine (ctx scratch 8..10): the whole chain runs on the context's
// stream with one host synchronisation at the end (combine.hip header).
namespace {
struct CombineBufs {
  double *X, *mean, *cov, *W, *work, *sw, *swt, *inv, *out;
  int32_t *rowbad, *used, *status, *blk;
};
int combine_bufs(stk_ctx* ctx, int nshards, int P, int S, CombineBufs* b, bool general = false) {
  DevBuf* B = ctx->scratch;
  const size_t per = (size_t)P * S, pp = (size_t)P * P;
  const size_t wk = std::max(stk_spd_inverse_work_bytes(P, nshards), general ? stk_general_inverse_work_bytes(P) : 0);
  RC(B[8].ensure(sizeof(double) * (per * nshards + per * 2 + (size_t)P * nshards)));
  RC(B[9].ensure(sizeof(double) * (pp * nshards * 2 + pp * 2) + wk + 16));
  RC(B[10].ensure(sizeof(int32_t) * ((size_t)P * nshards + 2 * (size_t)nshards + 2 + (size_t)P) + 64));
  b->X = B[8].as<double>();
  b->swt = b->X + per * nshards;
  b->out = b->swt + per;
  b->mean = b->out + per;
  b->cov = B[9].as<double>();
  b->W = b->cov + pp * nshards;
  b->sw = b->W + pp * nshards;
  b->inv = b->sw + pp;
  b->work = b->inv + pp;
  b->rowbad = B[10].as<int32_t>();
  b->used = b->rowbad + (size_t)P * nshards;
  b->status = b->used + nshards;               // nshards + 1 (the last: the final solve)
  b->blk = b->status + nshards + 1;
  return STK_OK;
}
// host-side outcome of a products run: LinAlgError / all-NaN
int combine_check(const std::vector<int32_t>& h, int nshards, int32_t* shard_used) {
  int nused = 0;
  for (int s = 0; s < nshards; ++s) {
    if (h[s] && h[nshards + s]) {
      stk_set_error("shard %d: singular sample covariance (LinAlgError)", s);
      return STK_E_LINALG;
    }
    nused += h[s];
    if (shard_used) shard_used[s] = h[s];
  }
  if (nused == 0) {
    stk_set_error("every shard holds NaN draws");
    return STK_E_NAN;
  }
  return STK_OK;
}
// device memory ON THE CONTEXT'S DEVICE (hipMalloc / a torch cuda tensor): the combine reads the
// draws and writes the result in place instead of staging them through the context's scratch
// buffers.  Memory of another device is not used in place (the kernels would dereference it
// without peer access): it takes the staged hipMemcpyAsync(Default) path, which copies across
// devices.
bool is_device_ptr(const void* p, int device) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice && a.device == device;
}
int consensus_run(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S, const int32_t* row_block,
                  double* sum_w, double* sum_wtheta, double* out, int32_t* shard_used) {
  ARG_CHECK(ctx && draws && nshards > 0 && P > 0 && S > 1, "stk_consensus: bad arguments");
  ARG_CHECK(P <= 4096, "P = %d too large", P);
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const size_t per = (size_t)P * S;
  // A sample covariance of S draws has rank <= S - 1: with S <= p (p = the largest weight block)
  // every shard's covariance is singular.  numpy's inv then returns rounding noise of order 1/eps
  // (or raises when a pivot happens to round to exactly zero) and the reference's combine is
  // meaningless; here it is a LinAlgError, independent of rounding.
  int pmax = P;
  if (row_block) {
    std::vector<int32_t> rb(P), cnt(P, 0);
    STK_HIP_CHECK(hipMemcpy(rb.data(), row_block, sizeof(int32_t) * P, hipMemcpyDefault));
    for (int i = 0; i < P; ++i) {
      ARG_CHECK(rb[i] >= 0 && rb[i] < P, "row_block[%d] = %d out of [0, P)", i, rb[i]);
      ++cnt[rb[i]];
    }
    pmax = *std::max_element(cnt.begin(), cnt.end());
  }
  if (S <= pmax) {
    stk_set_error("%d draws give a singular sample covariance for a %d-parameter weight block (rank <= S - 1; "
                  "LinAlgError)", S, pmax);
    return STK_E_LINALG;
  }
  CombineBufs b;
  RC(combine_bufs(ctx, nshards, P, S, &b));
  const bool dev_in = is_device_ptr(draws, ctx->device), dev_out = out && is_device_ptr(out, ctx->device);
  const double* X = dev_in ? draws : b.X;
  if (!dev_in) STK_HIP_CHECK(hipMemcpyAsync(b.X, draws, sizeof(double) * per * nshards, hipMemcpyDefault, st));
  if (row_block) STK_HIP_CHECK(hipMemcpyAsync(b.blk, row_block, sizeof(int32_t) * P, hipMemcpyDefault, st));
  STK_HIP_CHECK(stk_launch_consensus_products(X, nshards, P, S, row_block ? b.blk : nullptr, b.mean, b.rowbad,
                                              b.used, b.status, b.cov, b.W, b.work, b.sw, b.swt, st));
  if (out)
    STK_HIP_CHECK(stk_launch_consensus_solve(b.sw, b.swt, P, S, b.inv, b.work, b.status + nshards,
                                             dev_out ? out : b.out, st, false));
  std::vector<int32_t> h(2 * nshards + 1, 0);
  STK_HIP_CHECK(hipMemcpyAsync(h.data(), b.used, sizeof(int32_t) * (2 * nshards + (out ? 1 : 0)), hipMemcpyDeviceToHost, st));
  STK_HIP_CHECK(hipStreamSynchronize(st));
  RC(combine_check(h, nshards, shard_used));
  if (out && h[2 * nshards]) {
    stk_set_error("singular sum of weights (LinAlgError)");
    return STK_E_LINALG;
  }
  if (sum_w) STK_HIP_CHECK(hipMemcpyAsync(sum_w, b.sw, sizeof(double) * P * P, hipMemcpyDefault, st));
  if (sum_wtheta) STK_HIP_CHECK(hipMemcpyAsync(sum_wtheta, b.swt, sizeof(double) * per, hipMemcpyDefault, st));
  if (out && !dev_out) STK_HIP_CHECK(hipMemcpyAsync(out, b.out, sizeof(double) * per, hipMemcpyDefault, st));
  if (sum_w || sum_wtheta || (out && !dev_out)) STK_HIP_CHECK(hipStreamSynchronize(st));
  return STK_OK;
}
}  // namespace

int stk_consensus_products(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S, double* sum_w,
                           double* sum_wtheta, int32_t* shard_used) {
  return consensus_run(ctx, draws, nshards, P, S, nullptr, sum_w, sum_wtheta, nullptr, shard_used);
}

int stk_consensus_solve(stk_ctx* ctx, const double* sum_w, const double* sum_wtheta, int32_t P, int32_t S,
                        double* out) {
  ARG_CHECK(ctx && sum_w && sum_wtheta && out && P > 0 && S > 0, "stk_consensus_solve: bad arguments");
  STK_HIP_CHECK(hipSetDevice(ctx->device));
  hipStream_t st = ctx->stream;
  const size_t per = (size_t)P * S;
  CombineBufs b;
  RC(combine_bufs(ctx, 1, P, S, &b, true));
  STK_HIP_CHECK(hipMemcpyAsync(b.sw, sum_w, sizeof(double) * P * P, hipMemcpyDefault, st));
  STK_HIP_CHECK(hipMemcpyAsync(b.swt, sum_wtheta, sizeof(double) * per, hipMemcpyDefault, st));
  // the caller's sum W: any invertible matrix, inverted by partial pivoting as np.linalg.inv
  STK_HIP_CHECK(stk_launch_consensus_solve(b.sw, b.swt, P, S, b.inv, b.work, b.status, b.out, st, true));
  int32_t hs = 0;
  STK_HIP_CHECK(hipMemcpyAsync(&hs, b.status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  STK_HIP_CHECK(hipMemcpyAsync(out, b.out, sizeof(double) * per, hipMemcpyDefault, st));
  STK_HIP_CHECK(hipStreamSynchronize(st));
  if (hs) {
    stk_set_error("singular sum of weights (LinAlgError)");
    return STK_E_LINALG;
  }
  return STK_OK;
}

int stk_consensus(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S, double* out,
                  int32_t* shard_used) {
  ARG_CHECK(out, "stk_consensus: out is NULL");
  return consensus_run(ctx, draws, nshards, P, S, nullptr, nullptr, nullptr, out, shard_used);
}

int stk_consensus_blocked(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S,
                          const int32_t* row_block, double* out, int32_t* shard_used) {
  ARG_CHECK(out && row_block, "stk_consensus_blocked: out / row_block is NULL");
  return consensus_run(ctx, draws, nshards, P, S, row_block, nullptr, nullptr, out, shard_used);
}

}  // extern "C"
