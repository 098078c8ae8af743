/*
 * stark_oracle.c -- CPU restatement of the stark hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library (oracle/_build/liboracle.so), and only as the checker / CPU baseline.  The
 * product path (stark_amd + libstark_hip.so) never links, imports or calls it.
 *
 * What it restates (the reference delegates all of this to third-party code, see
 * SURVEY.md section 0):
 *   - stark/stark.py:48 `sm.sampling(...)`: Stan 2.19.1 (the version bundled with the
 *     last pystan 2 release, the API generation stark/stark.py:2-4 uses) NUTS with
 *     diag_e metric and windowed adaptation (hmc_nuts_diag_e_adapt).  Restated from
 *     Stan's published algorithm: base_nuts::transition / build_tree (multinomial
 *     sampling, biased progressive top level, generalized U-turn on rho / p_sharp),
 *     expl_leapfrog, diag_e_metric, stepsize_adaptation (Nesterov dual averaging),
 *     windowed_adaptation + var_adaptation + welford_var_estimator, base_hmc::init_stepsize.
 *     Stan is not vendored under /root/reference and cannot be installed here, so the
 *     sampler is "parity unpinned" at the Stan boundary; it is
 *     pinned by exact posterior moments (tests) and by the GPU/CPU trajectory check.
 *   - the model densities of example/schools.stan:1-18 (8-schools, non-centred) and the
 *     build-defined regression programs (stark_amd/models/ logistic.stan, linear.stan), Stan log_prob with
 *     propto=true, jacobian=true.
 *   - the synthetic-input generator of SURVEY.md section 8d (Philox4x32-10 keyed inputs).
 *
 * The GPU path is an ITERATIVE per-chain state machine; this file keeps Stan's RECURSIVE
 * build_tree so the two formulations check each other.  Random numbers follow one
 * counter-based spec shared by both (documented in DESIGN.md "RNG streams"): every
 * uniform index is consumed unconditionally, so both twins draw identical numbers.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ Philox4x32-10 */
/* Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11). */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += PHILOX_W0; k1 += PHILOX_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Stream tags (counter word 3).  Same values as stark_amd/csrc/philox.h. */
enum { TAG_INIT = 0x1, TAG_MOM = 0x2, TAG_UNI = 0x3, TAG_SSMOM = 0x4, TAG_JIT = 0x5,
       TAG_X = 0x10, TAG_Y = 0x11, TAG_BETA = 0x12 };

static void philox_u64x2(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                         uint64_t* a, uint64_t* b) {
  uint32_t ctr[4] = {c0, c1, c2, c3};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  orc_philox4x32_10(ctr, key, o);
  *a = ((uint64_t)o[1] << 32) | o[0];
  *b = ((uint64_t)o[3] << 32) | o[2];
}

/* 53-bit uniform on the open interval (0,1). */
static double u53(uint64_t x) { return ((double)(x >> 11) + 0.5) * 0x1.0p-53; }

/* Box-Muller pair from one Philox call. */
static void normal_pair(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                        double* z0, double* z1) {
  uint64_t a, b;
  philox_u64x2(seed, c0, c1, c2, c3, &a, &b);
  double u1 = u53(a), u2 = u53(b);
  double r = sqrt(-2.0 * log(u1));
  double th = 6.283185307179586 * u2;
  *z0 = r * cos(th);
  *z1 = r * sin(th);
}

double orc_uniform(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t idx, uint32_t tag) {
  uint64_t a, b;
  philox_u64x2(seed, c0, c1, idx >> 1, tag, &a, &b);
  return u53((idx & 1) ? b : a);
}

double orc_normal(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2hi, uint32_t idx, uint32_t tag) {
  double z0, z1;
  normal_pair(seed, c0, c1, c2hi | (idx >> 1), tag, &z0, &z1);
  return (idx & 1) ? z1 : z0;
}

/* ------------------------------------------------------------- synthetic inputs */
/* X_ij uniform on (-sqrt3, sqrt3) from 52-bit integers (exact
 * in fp64), beta ~ N(0, 1/d), alpha = 0; y from the model.  Rows are indexed globally
 * so sharding never changes the dataset (contiguous [s*N/S, (s+1)*N/S) row blocks). */
static const double SQRT3 = 1.7320508075688772;

static double gen_x_elem(uint64_t seed, int64_t g, int j) {
  uint64_t a, b;
  philox_u64x2(seed, (uint32_t)g, (uint32_t)((uint64_t)g >> 32), (uint32_t)(j >> 1), TAG_X, &a, &b);
  uint64_t k = ((j & 1) ? b : a) >> 12;                 /* 52 bits */
  double v = (double)(2 * k + 1) * 0x1.0p-52 - 1.0;     /* exact, in (-1, 1) */
  return v * SQRT3;
}

void orc_gen_x(uint64_t seed, int64_t row0, int64_t nrows, int d, double* X) {
  for (int64_t i = 0; i < nrows; ++i)
    for (int j = 0; j < d; ++j) X[i * d + j] = gen_x_elem(seed, row0 + i, j);
}

void orc_gen_beta(uint64_t seed, int d, double* beta) {
  double s = 1.0 / sqrt((double)d);
  for (int j = 0; j < d; ++j) {
    double z0, z1;
    normal_pair(seed, (uint32_t)(j >> 1), 0, 0, TAG_BETA, &z0, &z1);
    beta[j] = ((j & 1) ? z1 : z0) * s;
  }
}

static double gen_eta(const double* x, int d, double alpha, const double* beta) {
  double acc = alpha;
  for (int j = 0; j < d; ++j) acc = fma(x[j], beta[j], acc);
  return acc;
}

/* y_i = 1{u_i < 1/(1+exp(-eta_i))}; also returns |u - p| per row in margin (may be NULL). */
void orc_gen_y_logistic(uint64_t seed, int64_t row0, int64_t nrows, int d, const double* X,
                        double alpha, const double* beta, int32_t* y, double* margin) {
  for (int64_t i = 0; i < nrows; ++i) {
    double eta = gen_eta(X + i * d, d, alpha, beta);
    double p = 1.0 / (1.0 + exp(-eta));
    int64_t g = row0 + i;
    uint64_t a, b;
    philox_u64x2(seed, (uint32_t)g, (uint32_t)((uint64_t)g >> 32), 0, TAG_Y, &a, &b);
    double u = u53(a);
    y[i] = u < p ? 1 : 0;
    if (margin) margin[i] = fabs(u - p);
  }
}

void orc_gen_y_linear(uint64_t seed, int64_t row0, int64_t nrows, int d, const double* X,
                      double alpha, const double* beta, double sigma, double* y) {
  for (int64_t i = 0; i < nrows; ++i) {
    double eta = gen_eta(X + i * d, d, alpha, beta);
    int64_t g = row0 + i;
    double z0, z1;
    normal_pair(seed, (uint32_t)g, (uint32_t)((uint64_t)g >> 32), 0, TAG_Y, &z0, &z1);
    y[i] = eta + sigma * z0;
  }
}

/* ----------------------------------------------------------- model densities */
enum { FAM_SCHOOLS = 1, FAM_LINREG = 2, FAM_LOGREG = 3 };

typedef struct {
  int family;
  int64_t n;        /* rows (J for schools) */
  int d;            /* covariates (0 for schools) */
  const double* x;  /* n x d row-major */
  const double* y;  /* schools / linreg */
  const int32_t* yi;/* logreg */
  const double* sigma; /* schools */
  double pa, pb;    /* regressions: precisions 1/s^2 of alpha ~ normal(0, s_a), beta ~ normal(0, s_b); 0 = flat */
} orc_data;

int orc_dim(const orc_data* m) {
  switch (m->family) {
    case FAM_SCHOOLS: return (int)m->n + 2;
    case FAM_LINREG: return m->d + 2;
    case FAM_LOGREG: return m->d + 1;
  }
  return -1;
}

/* 8 schools, example/schools.stan:1-18, unconstrained q = (mu, log tau, eta[1..J]).
 * eta ~ normal(0,1) (schools.stan:15), y ~ normal(theta, sigma) (:16), theta = mu + tau*eta
 * (:11-12), tau = exp(u) with log-Jacobian u (real<lower=0> tau, :7); flat mu, tau.
 * normal_lpdf's arithmetic as Stan Math 2.18/2.19 (the release pystan 2.19 ships; third-party,
 * not in the reference) does it: inv_sigma = 1 / sigma, z = (y - theta) * inv_sigma, the
 * partial wrt theta inv_sigma * z. */
double orc_schools_lpgrad(int J, const double* y, const double* sigma, const double* q, double* grad) {
  double mu = q[0], u = q[1], tau = exp(u);
  double lp = 0.0, smu = 0.0, su = 0.0;
  for (int j = 0; j < J; ++j) {
    double eta = q[2 + j];
    double theta = mu + tau * eta;
    double inv_sigma = 1.0 / sigma[j];
    double z = (y[j] - theta) * inv_sigma;
    double r = inv_sigma * z;
    lp += -0.5 * eta * eta - 0.5 * z * z;
    smu += r;
    su += r * eta;
    if (grad) grad[2 + j] = -eta + tau * r;
  }
  lp += u;
  if (grad) { grad[0] = smu; grad[1] = tau * su + 1.0; }
  return lp;
}

/* Stan 2.19 bernoulli_logit_lpmf with its +-20 cutoff on (2y-1)*eta; derivative is the
 * exact derivative of each branch.  Model: y ~ bernoulli_logit(alpha + x*beta), flat priors
 * (stark_amd/models/logistic.stan). q = (alpha, beta[1..d]). */
double orc_logreg_lpgrad(int64_t N, int d, const double* X, const int32_t* y, const double* q, double* grad) {
  double lp = 0.0;
  if (grad) memset(grad, 0, sizeof(double) * (d + 1));
  for (int64_t i = 0; i < N; ++i) {
    const double* x = X + i * d;
    double eta = q[0];
    for (int j = 0; j < d; ++j) eta += x[j] * q[1 + j];
    double sgn = 2.0 * y[i] - 1.0;
    double nt = sgn * eta;
    double e = exp(-nt);
    double de;
    if (nt > 20.0) { lp -= e; de = sgn * e; }
    else if (nt < -20.0) { lp += nt; de = sgn; }
    else { lp -= log1p(e); de = sgn * e / (e + 1.0); }
    if (grad) {
      grad[0] += de;
      for (int j = 0; j < d; ++j) grad[1 + j] += x[j] * de;
    }
  }
  return lp;
}

/* y ~ normal(alpha + x*beta, sigma), sigma = exp(u) with log-Jacobian u, flat priors
 * (stark_amd/models/linear.stan). q = (alpha, beta[1..d], log sigma). */
double orc_linreg_lpgrad(int64_t N, int d, const double* X, const double* y, const double* q, double* grad) {
  double u = q[d + 1], inv_s = exp(-u);
  double ss = 0.0;
  if (grad) memset(grad, 0, sizeof(double) * (d + 2));
  for (int64_t i = 0; i < N; ++i) {
    const double* x = X + i * d;
    double eta = q[0];
    for (int j = 0; j < d; ++j) eta += x[j] * q[1 + j];
    double z = (y[i] - eta) * inv_s;
    ss += z * z;
    if (grad) {
      double dm = z * inv_s;
      grad[0] += dm;
      for (int j = 0; j < d; ++j) grad[1 + j] += x[j] * dm;
    }
  }
  if (grad) grad[d + 1] = -(double)N + ss + 1.0;
  return -0.5 * ss - (double)N * u + u;
}

/* Stan `alpha ~ normal(0, s_a); beta ~ normal(0, s_b);` with propto=true (constants dropped):
 * lp -= (pa alpha^2 + pb |beta|^2) / 2, grad -= p q.  q = (alpha, beta[1..d], ...). */
double orc_prior_lpgrad(double pa, double pb, int d, const double* q, double* grad) {
  double sb = 0.0;
  for (int j = 1; j <= d; ++j) sb += q[j] * q[j];
  if (grad) {
    grad[0] -= pa * q[0];
    for (int j = 1; j <= d; ++j) grad[j] -= pb * q[j];
  }
  return -0.5 * (pa * q[0] * q[0] + pb * sb);
}

double orc_lpgrad(const orc_data* m, const double* q, double* grad) {
  double lp;
  switch (m->family) {
    case FAM_SCHOOLS: return orc_schools_lpgrad((int)m->n, m->y, m->sigma, q, grad);
    case FAM_LINREG: lp = orc_linreg_lpgrad(m->n, m->d, m->x, m->y, q, grad); break;
    case FAM_LOGREG: lp = orc_logreg_lpgrad(m->n, m->d, m->x, m->yi, q, grad); break;
    default: return NAN;
  }
  if (m->pa != 0.0 || m->pb != 0.0) lp += orc_prior_lpgrad(m->pa, m->pb, m->d, q, grad);
  return lp;
}

/* ------------------------------------------------------- NUTS (Stan 2.19.1) */
typedef struct { double* q; double* p; double* g; double V; double H; } ps_point; /* g = dV/dq */

typedef struct {
  int num_warmup, num_samples, max_depth;
  double adapt_delta, gamma, kappa, t0, stepsize, init_radius;
  int init_buffer, term_buffer, window, adapt_engaged;
  uint64_t seed;
  double stepsize_jitter;
  int uturn_ext;      /* 0: Stan 2.19 single criterion; 1: + the checks between subtrees (Stan >= 2.23) */
} orc_cfg;

typedef struct {
  const orc_data* m;
  int D;
  double* inv_metric;
  double eps, nom_eps, jitter;
  int max_depth;
  double max_deltaH;
  uint64_t seed;
  uint32_t gid, iter, uk;   /* uniform stream: (gid, iter, uk) */
  int divergent, depth;
  int uturn_ext;
  ps_point z;
  long n_grad;
  /* dual averaging */
  double da_counter, s_bar, x_bar, mu, delta, gamma, kappa, t0;
  /* windowed variance adaptation */
  int var_on;
  unsigned num_warmup, init_buffer, term_buffer, base_window;
  unsigned win_counter, win_size, next_window;
  double wf_n; double* wf_m; double* wf_m2;
  uint32_t ss_call;
} nuts;

static double* dalloc(int n) { return (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }
static void pt_alloc(ps_point* z, int D) { z->q = dalloc(D); z->p = dalloc(D); z->g = dalloc(D); z->V = 0; z->H = 0; }
static void pt_free(ps_point* z) { free(z->q); free(z->p); free(z->g); }
static void pt_copy(ps_point* dst, const ps_point* src, int D) {
  memcpy(dst->q, src->q, sizeof(double) * D); memcpy(dst->p, src->p, sizeof(double) * D);
  memcpy(dst->g, src->g, sizeof(double) * D); dst->V = src->V; dst->H = src->H;
}

static double log_sum_exp2(double a, double b) {   /* stan::math::log_sum_exp(double,double) */
  if (a == -INFINITY) return b;
  if (a == INFINITY && b == INFINITY) return INFINITY;
  if (a > b) return a + log1p(exp(b - a));
  return b + log1p(exp(a - b));
}

static void update_potential_gradient(nuts* s, ps_point* z) {
  z->V = -orc_lpgrad(s->m, z->q, z->g);
  for (int i = 0; i < s->D; ++i) z->g[i] = -z->g[i];
  s->n_grad++;
}

static double tau_kin(const nuts* s, const ps_point* z) {   /* diag_e_metric::tau */
  double t = 0.0;
  for (int i = 0; i < s->D; ++i) t += z->p[i] * s->inv_metric[i] * z->p[i];
  return 0.5 * t;
}
static double Hfn(const nuts* s, const ps_point* z) { return z->V + tau_kin(s, z); }

static void dtau_dp(const nuts* s, const ps_point* z, double* out) {
  for (int i = 0; i < s->D; ++i) out[i] = s->inv_metric[i] * z->p[i];
}

static void sample_p(nuts* s, ps_point* z, uint32_t c1, uint32_t c2hi, uint32_t tag) {
  for (int i = 0; i < s->D; ++i)
    z->p[i] = orc_normal(s->seed, s->gid, c1, c2hi, (uint32_t)i, tag) / sqrt(s->inv_metric[i]);
}

static double rand_uniform(nuts* s) { return orc_uniform(s->seed, s->gid, s->iter, s->uk++, TAG_UNI); }

static void evolve(nuts* s, ps_point* z, double epsilon) {    /* expl_leapfrog::evolve */
  double he = 0.5 * epsilon;
  for (int i = 0; i < s->D; ++i) z->p[i] -= he * z->g[i];                      /* begin_update_p */
  for (int i = 0; i < s->D; ++i) z->q[i] += epsilon * (s->inv_metric[i] * z->p[i]); /* update_q */
  update_potential_gradient(s, z);
  for (int i = 0; i < s->D; ++i) z->p[i] -= he * z->g[i];                      /* end_update_p */
}

static int compute_criterion(int D, const double* psm, const double* psp, const double* rho) {
  double a = 0.0, b = 0.0;
  for (int i = 0; i < D; ++i) { a += psp[i] * rho[i]; b += psm[i] * rho[i]; }
  return a > 0 && b > 0;
}

static int build_tree(nuts* s, int depth, ps_point* z_propose, double* psl, double* psr, double* rho,
                      double H0, int sign, int* n_leapfrog, double* lsw, double* sum_metro) {
  int D = s->D;
  if (depth == 0) {
    evolve(s, &s->z, sign * s->eps);
    ++*n_leapfrog;
    double h = Hfn(s, &s->z);
    if (isnan(h)) h = INFINITY;
    if ((h - H0) > s->max_deltaH) s->divergent = 1;
    *lsw = log_sum_exp2(*lsw, H0 - h);
    if (H0 - h > 0) *sum_metro += 1; else *sum_metro += exp(H0 - h);
    s->z.H = h;
    pt_copy(z_propose, &s->z, D);
    for (int i = 0; i < D; ++i) rho[i] += s->z.p[i];
    dtau_dp(s, &s->z, psl);
    memcpy(psr, psl, sizeof(double) * D);
    return !s->divergent;
  }
  double* dummy = dalloc(D);
  double* rho_left = dalloc(D);
  double* rho_right = dalloc(D);
  double lsw_left = -INFINITY, lsw_right = -INFINITY;
  int ok = build_tree(s, depth - 1, z_propose, psl, dummy, rho_left, H0, sign, n_leapfrog, &lsw_left, sum_metro);
  if (ok) {
    ps_point zr; pt_alloc(&zr, D); pt_copy(&zr, &s->z, D);
    ok = build_tree(s, depth - 1, &zr, dummy, psr, rho_right, H0, sign, n_leapfrog, &lsw_right, sum_metro);
    if (ok) {
      double lsw_sub = log_sum_exp2(lsw_left, lsw_right);
      *lsw = log_sum_exp2(*lsw, lsw_sub);
      double u = rand_uniform(s);   /* consumed unconditionally (RNG spec) */
      if (lsw_right > lsw_sub) pt_copy(z_propose, &zr, D);
      else if (u < exp(lsw_right - lsw_sub)) pt_copy(z_propose, &zr, D);
      for (int i = 0; i < D; ++i) { double r = rho_left[i] + rho_right[i]; rho_left[i] = r; rho[i] += r; }
      ok = compute_criterion(D, psl, psr, rho_left);
    }
    pt_free(&zr);
  }
  free(dummy); free(rho_left); free(rho_right);
  return ok;
}

/* Stan >= 2.23 base_nuts::build_tree: besides the U-turn test across the merged subtree,
 * two tests across the junction of the two halves (the left half extended by the first
 * momentum of the right one, and the right half extended by the last momentum of the left
 * one), which catch trajectories that turn inside a doubling -- the resonance of the single
 * criterion on near-isotropic Gaussian posteriors.  Tracks the begin / end momenta (p_beg,
 * p_end) and p_sharp at both ends of every subtree. */
static int build_tree_ext(nuts* s, int depth, ps_point* z_propose, double* ps_beg, double* ps_end, double* rho,
                          double* p_beg, double* p_end, double H0, int sign, int* n_leapfrog, double* lsw,
                          double* sum_metro) {
  int D = s->D;
  if (depth == 0) {
    evolve(s, &s->z, sign * s->eps);
    ++*n_leapfrog;
    double h = Hfn(s, &s->z);
    if (isnan(h)) h = INFINITY;
    if ((h - H0) > s->max_deltaH) s->divergent = 1;
    *lsw = log_sum_exp2(*lsw, H0 - h);
    if (H0 - h > 0) *sum_metro += 1; else *sum_metro += exp(H0 - h);
    s->z.H = h;
    pt_copy(z_propose, &s->z, D);
    dtau_dp(s, &s->z, ps_beg);
    memcpy(ps_end, ps_beg, sizeof(double) * D);
    for (int i = 0; i < D; ++i) rho[i] += s->z.p[i];
    memcpy(p_beg, s->z.p, sizeof(double) * D);
    memcpy(p_end, s->z.p, sizeof(double) * D);
    return !s->divergent;
  }
  double* p_init_end = dalloc(D); double* ps_init_end = dalloc(D); double* rho_init = dalloc(D);
  double* p_final_beg = dalloc(D); double* ps_final_beg = dalloc(D); double* rho_final = dalloc(D);
  double* ext = dalloc(D);
  double lsw_init = -INFINITY, lsw_final = -INFINITY;
  int ok = build_tree_ext(s, depth - 1, z_propose, ps_beg, ps_init_end, rho_init, p_beg, p_init_end, H0, sign,
                          n_leapfrog, &lsw_init, sum_metro);
  if (ok) {
    ps_point zr; pt_alloc(&zr, D); pt_copy(&zr, &s->z, D);
    ok = build_tree_ext(s, depth - 1, &zr, ps_final_beg, ps_end, rho_final, p_final_beg, p_end, H0, sign,
                        n_leapfrog, &lsw_final, sum_metro);
    if (ok) {
      double lsw_sub = log_sum_exp2(lsw_init, lsw_final);
      *lsw = log_sum_exp2(*lsw, lsw_sub);
      double u = rand_uniform(s);   /* consumed unconditionally (RNG spec) */
      if (lsw_final > lsw_sub) pt_copy(z_propose, &zr, D);
      else if (u < exp(lsw_final - lsw_sub)) pt_copy(z_propose, &zr, D);
      double* rho_sub = dalloc(D);
      for (int i = 0; i < D; ++i) { rho_sub[i] = rho_init[i] + rho_final[i]; rho[i] += rho_sub[i]; }
      int c1 = compute_criterion(D, ps_beg, ps_end, rho_sub);
      for (int i = 0; i < D; ++i) ext[i] = rho_init[i] + p_final_beg[i];
      int c2 = compute_criterion(D, ps_beg, ps_final_beg, ext);
      for (int i = 0; i < D; ++i) ext[i] = rho_final[i] + p_init_end[i];
      int c3 = compute_criterion(D, ps_init_end, ps_end, ext);
      ok = c1 && c2 && c3;
      free(rho_sub);
    }
    pt_free(&zr);
  }
  free(p_init_end); free(ps_init_end); free(rho_init); free(p_final_beg); free(ps_final_beg); free(rho_final);
  free(ext);
  return ok;
}

typedef struct { double accept, eps, depth, n_leapfrog, divergent, energy; } orc_stats;

/* base_nuts::transition (Stan 2.19.1).  s->z holds the start point with V and g valid. */
static void transition(nuts* s, orc_stats* st) {
  int D = s->D;
  s->eps = s->nom_eps;          /* base_hmc::sample_stepsize */
  if (s->jitter > 0)            /* own stream (TAG_JIT): the TAG_UNI indices do not move */
    s->eps *= 1.0 + s->jitter * (2.0 * orc_uniform(s->seed, s->gid, s->iter, 0, TAG_JIT) - 1.0);
  s->uk = 0;
  sample_p(s, &s->z, s->iter, 0, TAG_MOM);
  ps_point z_plus, z_minus, z_sample, z_propose;
  pt_alloc(&z_plus, D); pt_alloc(&z_minus, D); pt_alloc(&z_sample, D); pt_alloc(&z_propose, D);
  double H0 = Hfn(s, &s->z);
  s->z.H = H0;
  pt_copy(&z_plus, &s->z, D); pt_copy(&z_minus, &s->z, D);
  pt_copy(&z_sample, &s->z, D); pt_copy(&z_propose, &s->z, D);
  double* psp = dalloc(D); double* psm = dalloc(D); double* dummy = dalloc(D);
  double* rho = dalloc(D); double* rho_sub = dalloc(D);
  dtau_dp(s, &s->z, psp); memcpy(psm, psp, sizeof(double) * D);
  memcpy(rho, s->z.p, sizeof(double) * D);
  double lsw = 0.0;
  int n_leapfrog = 0; double sum_metro = 0.0;
  s->depth = 0; s->divergent = 0;
  /* Stan >= 2.23 bookkeeping: momenta / p_sharp at both ends of the backward and forward parts */
  double* p_ff = dalloc(D); double* p_fb = dalloc(D); double* p_bf = dalloc(D); double* p_bb = dalloc(D);
  double* ps_fb = dalloc(D); double* ps_bf = dalloc(D); double* rho_f = dalloc(D); double* rho_b = dalloc(D);
  double* ext = dalloc(D);
  memcpy(p_ff, s->z.p, sizeof(double) * D); memcpy(p_fb, p_ff, sizeof(double) * D);
  memcpy(p_bf, p_ff, sizeof(double) * D); memcpy(p_bb, p_ff, sizeof(double) * D);
  memcpy(ps_fb, psp, sizeof(double) * D); memcpy(ps_bf, psp, sizeof(double) * D);
  while (s->uturn_ext && s->depth < s->max_depth) {
    int valid;
    double lsw_sub = -INFINITY;
    memset(rho_f, 0, sizeof(double) * D); memset(rho_b, 0, sizeof(double) * D);
    if (rand_uniform(s) > 0.5) {
      memcpy(rho_b, rho, sizeof(double) * D);
      memcpy(p_bf, p_ff, sizeof(double) * D); memcpy(ps_bf, psp, sizeof(double) * D);
      pt_copy(&s->z, &z_plus, D);
      valid = build_tree_ext(s, s->depth, &z_propose, ps_fb, psp, rho_f, p_fb, p_ff, H0, 1, &n_leapfrog, &lsw_sub,
                             &sum_metro);
      pt_copy(&z_plus, &s->z, D);
    } else {
      memcpy(rho_f, rho, sizeof(double) * D);
      memcpy(p_fb, p_bb, sizeof(double) * D); memcpy(ps_fb, psm, sizeof(double) * D);
      pt_copy(&s->z, &z_minus, D);
      valid = build_tree_ext(s, s->depth, &z_propose, ps_bf, psm, rho_b, p_bf, p_bb, H0, -1, &n_leapfrog, &lsw_sub,
                             &sum_metro);
      pt_copy(&z_minus, &s->z, D);
    }
    if (!valid) break;
    ++s->depth;
    double u = rand_uniform(s);     /* consumed unconditionally (RNG spec) */
    if (lsw_sub > lsw) pt_copy(&z_sample, &z_propose, D);
    else if (u < exp(lsw_sub - lsw)) pt_copy(&z_sample, &z_propose, D);
    lsw = log_sum_exp2(lsw, lsw_sub);
    for (int i = 0; i < D; ++i) rho[i] = rho_b[i] + rho_f[i];
    int c1 = compute_criterion(D, psm, psp, rho);
    for (int i = 0; i < D; ++i) ext[i] = rho_b[i] + p_fb[i];
    int c2 = compute_criterion(D, psm, ps_fb, ext);
    for (int i = 0; i < D; ++i) ext[i] = rho_f[i] + p_bf[i];
    int c3 = compute_criterion(D, ps_bf, psp, ext);
    if (!(c1 && c2 && c3)) break;
  }
  free(p_ff); free(p_fb); free(p_bf); free(p_bb); free(ps_fb); free(ps_bf); free(rho_f); free(rho_b); free(ext);
  while (!s->uturn_ext && s->depth < s->max_depth) {
    memset(rho_sub, 0, sizeof(double) * D);
    int valid;
    double lsw_sub = -INFINITY;
    if (rand_uniform(s) > 0.5) {
      pt_copy(&s->z, &z_plus, D);
      valid = build_tree(s, s->depth, &z_propose, dummy, psp, rho_sub, H0, 1, &n_leapfrog, &lsw_sub, &sum_metro);
      pt_copy(&z_plus, &s->z, D);
    } else {
      pt_copy(&s->z, &z_minus, D);
      valid = build_tree(s, s->depth, &z_propose, dummy, psm, rho_sub, H0, -1, &n_leapfrog, &lsw_sub, &sum_metro);
      pt_copy(&z_minus, &s->z, D);
    }
    if (!valid) break;
    ++s->depth;
    double u = rand_uniform(s);     /* consumed unconditionally (RNG spec) */
    if (lsw_sub > lsw) pt_copy(&z_sample, &z_propose, D);
    else if (u < exp(lsw_sub - lsw)) pt_copy(&z_sample, &z_propose, D);
    lsw = log_sum_exp2(lsw, lsw_sub);
    for (int i = 0; i < D; ++i) rho[i] = rho[i] + rho_sub[i];
    if (!compute_criterion(D, psm, psp, rho)) break;
  }
  st->accept = sum_metro / (double)n_leapfrog;
  st->eps = s->eps;
  st->depth = s->depth;
  st->n_leapfrog = n_leapfrog;
  st->divergent = s->divergent;
  pt_copy(&s->z, &z_sample, D);
  st->energy = s->z.H;
  free(psp); free(psm); free(dummy); free(rho); free(rho_sub);
  pt_free(&z_plus); pt_free(&z_minus); pt_free(&z_sample); pt_free(&z_propose);
}

/* base_hmc::init_stepsize.  Returns 0, or -1 when the step size leaves (0, 1e7]. */
static int init_stepsize(nuts* s) {
  int D = s->D;
  if (s->nom_eps == 0 || s->nom_eps > 1e7 || isnan(s->nom_eps)) return 0;
  ps_point z_init; pt_alloc(&z_init, D); pt_copy(&z_init, &s->z, D);
  uint32_t probe = 0;
  int rc = 0;
  sample_p(s, &s->z, s->ss_call, probe << 12, TAG_SSMOM); ++probe;
  double H0 = Hfn(s, &s->z);
  evolve(s, &s->z, s->nom_eps);
  double h = Hfn(s, &s->z);
  if (isnan(h)) h = INFINITY;
  double dH = H0 - h;
  int direction = dH > log(0.8) ? 1 : -1;
  for (;;) {
    pt_copy(&s->z, &z_init, D);
    sample_p(s, &s->z, s->ss_call, probe << 12, TAG_SSMOM); ++probe;
    H0 = Hfn(s, &s->z);
    evolve(s, &s->z, s->nom_eps);
    h = Hfn(s, &s->z);
    if (isnan(h)) h = INFINITY;
    dH = H0 - h;
    if ((direction == 1) && !(dH > log(0.8))) break;
    else if ((direction == -1) && !(dH < log(0.8))) break;
    else s->nom_eps = direction == 1 ? 2 * s->nom_eps : 0.5 * s->nom_eps;
    if (s->nom_eps > 1e7) { rc = -1; break; }
    if (s->nom_eps == 0) { rc = -1; break; }
  }
  pt_copy(&s->z, &z_init, D);
  pt_free(&z_init);
  s->ss_call++;
  return rc;
}

static void da_restart(nuts* s) { s->da_counter = 0; s->s_bar = 0; s->x_bar = 0; }

static void learn_stepsize(nuts* s, double adapt_stat) {   /* stepsize_adaptation::learn_stepsize */
  s->da_counter += 1;
  adapt_stat = adapt_stat > 1 ? 1 : adapt_stat;
  double eta = 1.0 / (s->da_counter + s->t0);
  s->s_bar = (1.0 - eta) * s->s_bar + eta * (s->delta - adapt_stat);
  double x = s->mu - s->s_bar * sqrt(s->da_counter) / s->gamma;
  double x_eta = pow(s->da_counter, -s->kappa);
  s->x_bar = (1.0 - x_eta) * s->x_bar + x_eta * x;
  s->nom_eps = exp(x);
}

static void win_restart(nuts* s) {
  s->win_counter = 0;
  s->win_size = s->base_window;
  s->next_window = s->init_buffer + s->win_size - 1;
}

/* windowed_adaptation::set_window_params.  The short-warmup branch restarts the window
 * schedule too (the evident intent; see DESIGN.md "Adaptation"). */
static void set_window_params(nuts* s, unsigned num_warmup, unsigned init_buffer, unsigned term_buffer, unsigned base_window) {
  if (num_warmup < 20) { s->var_on = 0; return; }
  s->var_on = 1;
  s->num_warmup = num_warmup;
  if (init_buffer + base_window + term_buffer > num_warmup) {
    s->init_buffer = (unsigned)(0.15 * num_warmup);
    s->term_buffer = (unsigned)(0.1 * num_warmup);
    s->base_window = num_warmup - (s->init_buffer + s->term_buffer);
  } else {
    s->init_buffer = init_buffer; s->term_buffer = term_buffer; s->base_window = base_window;
  }
  win_restart(s);
}

static int adaptation_window(const nuts* s) {
  return (s->win_counter >= s->init_buffer) && (s->win_counter < s->num_warmup - s->term_buffer) &&
         (s->win_counter != s->num_warmup);
}
static int end_adaptation_window(const nuts* s) {
  return (s->win_counter == s->next_window) && (s->win_counter != s->num_warmup);
}
static void compute_next_window(nuts* s) {
  if (s->next_window == s->num_warmup - s->term_buffer - 1) return;
  s->win_size *= 2;
  s->next_window = s->win_counter + s->win_size;
  if (s->next_window != s->num_warmup - s->term_buffer - 1) {
    unsigned nb = s->next_window + 2 * s->win_size;
    if (nb >= s->num_warmup - s->term_buffer) s->next_window = s->num_warmup - s->term_buffer - 1;
  }
}

static int learn_variance(nuts* s, const double* q) {     /* var_adaptation::learn_variance */
  int D = s->D;
  if (adaptation_window(s)) {       /* welford_var_estimator::add_sample */
    s->wf_n += 1.0;
    for (int i = 0; i < D; ++i) {
      double delta = q[i] - s->wf_m[i];
      s->wf_m[i] += delta / s->wf_n;
      s->wf_m2[i] += (q[i] - s->wf_m[i]) * delta;
    }
  }
  if (end_adaptation_window(s)) {
    compute_next_window(s);
    double n = s->wf_n;
    if (n > 1) for (int i = 0; i < D; ++i) s->inv_metric[i] = s->wf_m2[i] / (n - 1.0);
    for (int i = 0; i < D; ++i)
      s->inv_metric[i] = (n / (n + 5.0)) * s->inv_metric[i] + 1e-3 * (5.0 / (n + 5.0));
    s->wf_n = 0; memset(s->wf_m, 0, sizeof(double) * D); memset(s->wf_m2, 0, sizeof(double) * D);
    ++s->win_counter;
    return 1;
  }
  ++s->win_counter;
  return 0;
}

/* One chain of hmc_nuts_diag_e_adapt (services/sample + util/run_adaptive_sampler).
 *   gid        global chain id (shard * chains + chain): the RNG stream key
 *   init       D unconstrained values, or NULL for uniform(-R, R)
 *   q_out      (num_warmup+num_samples) x D unconstrained draws (every transition)
 *   lp_out     (num_warmup+num_samples) lp__ values
 *   st_out     (num_warmup+num_samples) x 6 (accept, stepsize, treedepth, n_leapfrog, divergent, energy)
 *   final      1 + D: final nominal stepsize, inverse metric
 * Returns the number of gradient evaluations, or -1 on a step-size error. */
long orc_run_chain(const orc_data* m, const orc_cfg* cfg, uint32_t gid, const double* init,
                   double* q_out, double* lp_out, double* st_out, double* final) {
  nuts s; memset(&s, 0, sizeof(s));
  s.m = m; s.D = orc_dim(m); s.seed = cfg->seed; s.gid = gid;
  int D = s.D;
  s.inv_metric = dalloc(D);
  for (int i = 0; i < D; ++i) s.inv_metric[i] = 1.0;
  s.max_depth = cfg->max_depth; s.max_deltaH = 1000.0;
  s.wf_m = dalloc(D); s.wf_m2 = dalloc(D);
  pt_alloc(&s.z, D);
  for (int i = 0; i < D; ++i)
    s.z.q[i] = init ? init[i] : -cfg->init_radius + 2.0 * cfg->init_radius * orc_uniform(cfg->seed, gid, 0, (uint32_t)i, TAG_INIT);
  update_potential_gradient(&s, &s.z);
  s.nom_eps = cfg->stepsize;
  s.jitter = cfg->stepsize_jitter;
  s.uturn_ext = cfg->uturn_ext;
  s.delta = cfg->adapt_delta; s.gamma = cfg->gamma; s.kappa = cfg->kappa; s.t0 = cfg->t0;
  s.mu = log(10.0 * cfg->stepsize);
  da_restart(&s);
  int adapt = cfg->adapt_engaged && cfg->num_warmup > 0;
  set_window_params(&s, (unsigned)cfg->num_warmup, (unsigned)cfg->init_buffer, (unsigned)cfg->term_buffer, (unsigned)cfg->window);
  long rc = 0;
  if (init_stepsize(&s) < 0) rc = -1;
  int total = cfg->num_warmup + cfg->num_samples;
  for (int t = 0; t < total && rc == 0; ++t) {
    s.iter = (uint32_t)t;
    orc_stats st;
    transition(&s, &st);
    if (q_out) memcpy(q_out + (size_t)t * D, s.z.q, sizeof(double) * D);
    if (lp_out) lp_out[t] = -s.z.V;
    if (st_out) {
      double* o = st_out + (size_t)t * 6;
      o[0] = st.accept; o[1] = st.eps; o[2] = st.depth; o[3] = st.n_leapfrog; o[4] = st.divergent; o[5] = st.energy;
    }
    if (adapt && t < cfg->num_warmup) {
      learn_stepsize(&s, st.accept);
      if (s.var_on && learn_variance(&s, s.z.q)) {
        if (init_stepsize(&s) < 0) rc = -1;
        s.mu = log(10.0 * s.nom_eps);
        da_restart(&s);
      }
      if (t == cfg->num_warmup - 1) s.nom_eps = exp(s.x_bar);   /* complete_adaptation */
    }
  }
  if (final) { final[0] = s.nom_eps; memcpy(final + 1, s.inv_metric, sizeof(double) * D); }
  long ng = s.n_grad;
  free(s.inv_metric); free(s.wf_m); free(s.wf_m2); pt_free(&s.z);
  return rc < 0 ? -1 : ng;
}

/* One fixed-step-size transition from (q, inv_metric, eps) with no adaptation: the unit
 * the GPU/CPU trajectory-parity test compares.  Writes the new q, lp, stats. */
long orc_transition(const orc_data* m, uint64_t seed, uint32_t gid, uint32_t iter, int max_depth,
                    double eps, const double* inv_metric, double* q, double* lp, double* st_out, int uturn_ext) {
  nuts s; memset(&s, 0, sizeof(s));
  s.m = m; s.D = orc_dim(m); s.seed = seed; s.gid = gid; s.iter = iter;
  s.uturn_ext = uturn_ext;
  int D = s.D;
  s.inv_metric = dalloc(D); memcpy(s.inv_metric, inv_metric, sizeof(double) * D);
  s.max_depth = max_depth; s.max_deltaH = 1000.0; s.nom_eps = eps;
  pt_alloc(&s.z, D);
  memcpy(s.z.q, q, sizeof(double) * D);
  update_potential_gradient(&s, &s.z);
  orc_stats st;
  transition(&s, &st);
  memcpy(q, s.z.q, sizeof(double) * D);
  *lp = -s.z.V;
  if (st_out) { st_out[0] = st.accept; st_out[1] = st.eps; st_out[2] = st.depth; st_out[3] = st.n_leapfrog; st_out[4] = st.divergent; st_out[5] = st.energy; }
  long ng = s.n_grad;
  free(s.inv_metric); pt_free(&s.z);
  return ng;
}

/* Time-boxed gradient loop for bench.py's cpu_baseline: evaluates the logreg gradient
 * `reps` times over the given rows, returns elapsed-independent work count. */
double orc_logreg_grad_loop(int64_t N, int d, const double* X, const int32_t* y, const double* q, double* grad, int reps) {
  double acc = 0.0;
  for (int r = 0; r < reps; ++r) acc += orc_logreg_lpgrad(N, d, X, y, q, grad);
  return acc;
}
