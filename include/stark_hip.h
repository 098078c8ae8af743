/*
 * stark_hip.h -- C ABI of libstark_hip.so, the MI355X (gfx950) implementation of
 * stark's data-parallel hot path: subposterior NUTS sampling per data shard and the
 * consensus weighted-average combine.
 *
 * Each entry point replaces one reference interface (all paths under randommm/stark):
 *
 *   stk_model_create            stark/stark.py:37-39  Stark.setStanModel -> StanModel(**kw)
 *                               + stark/stark.py:46   data = callback(rows) (per partition)
 *   stk_model_create_synthetic  SURVEY.md 8d synthetic shards (bench; no host rows)
 *   stk_log_density_grad        Stan log_prob<propto=true,jacobian=true> + gradient, the
 *                               unit of work inside stark/stark.py:48 `sm.sampling`
 *   stk_sample / stk_sampler_*  stark/stark.py:48-56  `sm.sampling(data, **kw)` +
 *                               `fit.extract()` -> P x S matrix, for every local partition
 *                               (stark/stark.py:65 mapPartitions(_mcmc(...)))
 *   stk_transition              one Stan NUTS transition (parity hook, no adaptation)
 *   stk_consensus_products      stark/stark.py:7-21   consensus_avg(J) reducer body
 *   stk_consensus_solve         stark/stark.py:66-70  inv(sum W) . sum W theta
 *   stk_consensus               stark/stark.py:66-70  reduce + solve over all shards
 *   stk_consensus_blocked       the same with block-diagonal weights (lp__ in its own block)
 *
 * Conventions
 *   - Return 0 on success, a negative STK_E_* code on failure; stk_last_error() gives a
 *     thread-local message.  No entry point ever falls back to a CPU computation.
 *   - Pointer arguments may be host or device memory (HIP unified addressing); the caller
 *     keeps ownership.  The library copies shard data to the device at model creation.
 *   - A context is bound to one device and one stream and is not thread-safe.  Multi-GPU
 *     runs use one process per GPU; the host side (stark_amd) exchanges draws with
 *     torch.distributed over RCCL.
 *   - Matrices are row-major fp64.  Draw matrices are "variables by samples" (P x S), the
 *     layout stark/stark.py:56 returns.
 */
#ifndef STARK_HIP_H
#define STARK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STK_API __attribute__((visibility("default")))

typedef struct stk_ctx stk_ctx;
typedef struct stk_model stk_model;
typedef struct stk_sampler stk_sampler;

enum {
  STK_OK = 0,
  STK_E_ARG = -1,      /* invalid argument                                   */
  STK_E_HIP = -2,      /* HIP runtime error (no device, launch failure, ...)  */
  STK_E_NOMEM = -3,    /* device allocation failed                            */
  STK_E_STATE = -4,    /* call out of order                                   */
  STK_E_NUMERIC = -5,  /* step size left (0, 1e7] (Stan's init_stepsize error) */
  STK_E_NAN = -6,      /* every shard holds NaN draws (combine)               */
  STK_E_LINALG = -7    /* singular matrix in the combine (LinAlgError)        */
};

/* Model families. */
enum { STK_SCHOOLS = 1, STK_LINREG = 2, STK_LOGREG = 3 };

/* One data shard (= one Spark partition, stark/stark.py:35).
 *   schools: n_rows = J, y[J], sigma[J]                   (example/stark_ex.py:8-11)
 *   linreg : x[n_rows * n_cols] row-major, y[n_rows]
 *   logreg : x[n_rows * n_cols] row-major, y_int[n_rows] in {0, 1}                   */
typedef struct {
  int64_t n_rows;
  int32_t n_cols;
  const double* x;
  const double* y;
  const int32_t* y_int;
  const double* sigma;
} stk_shard;

/* Sampler configuration: pystan 2 `sampling()` keywords (stark/stark.py:48, defaults
 * stark/stark.py:60-64) and the Stan control block.  stk_config_default() fills Stan's
 * defaults (iter 2000 -> 1000 warmup + 1000 draws, chains 1 as stark forces, max_depth 10,
 * adapt_delta 0.8, gamma 0.05, kappa 0.75, t0 10, stepsize 1, init U(-2,2), buffers 75/50/25). */
typedef struct {
  int32_t num_warmup;
  int32_t num_samples;
  int32_t chains;            /* chains per shard */
  int32_t max_depth;
  double adapt_delta, adapt_gamma, adapt_kappa, adapt_t0;
  double stepsize;           /* initial nominal step size */
  double init_radius;        /* inits ~ U(-R, R) on the unconstrained scale */
  int32_t adapt_init_buffer, adapt_term_buffer, adapt_window;
  int32_t adapt_engaged;
  uint64_t seed;
  const double* init;        /* NULL, or nshards * chains * D unconstrained inits */
  const double* inv_metric;  /* NULL (unit), or D initial diagonal inverse metric */
  int32_t skip_init_stepsize;/* test hook: do not run base_hmc::init_stepsize */
  int32_t iter_offset;       /* test hook: RNG iteration index of the first transition */
  int32_t save_warmup;       /* also keep unconstrained warmup draws (pystan inc_warmup):
                                stk_sampler_draws_unconstrained then returns all iterations */
  const int32_t* shard_ids;  /* NULL, or the GLOBAL index of every local shard: chain c of shard s
                                draws from RNG stream shard_ids[s] * chains + c, so a shard samples
                                identically whichever GPU (and with whichever other shards) it runs */
  double stepsize_jitter;    /* Stan control stepsize_jitter in [0, 1]: every transition uses
                                stepsize * (1 + jitter * U(-1, 1)) (base_hmc::sample_stepsize) */
  int32_t nuts_criterion;    /* 0 (default): Stan 2.19.1's U-turn test across each merged subtree, as
                                the reference's pystan 2 runs it; 1: also the two tests across the
                                junction of the merged halves that Stan >= 2.23 adds (base_nuts
                                build_tree / transition), which stop the trajectories that the single
                                test lets run on near-isotropic Gaussian posteriors */
  int32_t chains_per_wave;   /* 8-schools fused kernel: chains packed per 64-lane wave, 0 (default) =
                                the most that fit (4 for D <= 16, 2 for D <= 32, else 1); 1 or 2 cap
                                it (test hook: the packing changes no bit of the draws) */
} stk_config;

typedef struct {
  int64_t grad_evals;   /* chain-gradient evaluations issued (all local chains)          */
  int64_t leapfrogs;    /* leapfrog steps inside NUTS trajectories                        */
  int64_t steps;        /* state-machine steps launched                                   */
  int64_t sweeps;       /* data-sweep launches that ran (regression families)             */
  double sweep_ms;      /* summed HIP-event time of the sweep kernel (profiling on only)  */
  int32_t divergent;    /* divergent transitions after warmup                             */
  int32_t errors;       /* chains stopped by a step-size error                            */
  int32_t min_iter;     /* fewest transitions completed by any chain                      */
  int32_t done;         /* chains that completed num_warmup + num_samples                 */
  int64_t shard_sweeps; /* shard passes inside those sweeps (bytes = shard_sweeps * n*(8d+4)) */
} stk_run_info;

STK_API const char* stk_last_error(void);
STK_API int stk_version(void);
STK_API void stk_config_default(stk_config* cfg);

/* ---- context: one device, one stream ---- */
STK_API int stk_ctx_create(int device, stk_ctx** out);
STK_API int stk_ctx_destroy(stk_ctx* ctx);
STK_API int stk_ctx_sync(stk_ctx* ctx);
/* A context on the caller's HIP stream (e.g. torch.cuda.current_stream().cuda_stream), so library
 * kernels and the caller's collectives on that stream are ordered without host syncs (NULL: the
 * null stream, which is torch's default current stream).  The stream is not destroyed with the
 * context. */
STK_API int stk_ctx_create_on_stream(int device, void* stream, stk_ctx** out);
/* HIP events around the data sweeps of every on-th split-mode step (0: off; 1: every step).
   Each event pair is a barrier on the stream: sample (e.g. 8) to keep the timing cheap. */
STK_API int stk_ctx_set_profiling(stk_ctx* ctx, int on);
STK_API void* stk_ctx_stream(stk_ctx* ctx);                /* hipStream_t of the context */

/* ---- models: stark/stark.py:37-39 + :46 ---- */
STK_API int stk_model_create(stk_ctx* ctx, int family, const stk_shard* shards, int nshards, stk_model** out);
/* Synthetic shards generated on the device: global rows
 * [row_offset + s*rows_per_shard, row_offset + (s+1)*rows_per_shard) for shard s. */
STK_API int stk_model_create_synthetic(stk_ctx* ctx, int family, int nshards, int64_t rows_per_shard,
                                       int64_t row_offset, int32_t n_cols, uint64_t data_seed,
                                       double alpha, const double* beta, double noise_sigma,
                                       stk_model** out);
STK_API int stk_gen_beta(uint64_t data_seed, int32_t n_cols, double* beta);   /* host, beta ~ N(0, 1/d) */
/* Regressions: alpha ~ normal(0, alpha_scale), beta ~ normal(0, beta_scale) (each 0 or inf = flat,
 * the default) -- the priors of a `model` block the front end recognises (stark/stark.py:37-39
 * setStanModel of such a program).  Applies to every shard, before sampling. */
STK_API int stk_model_set_prior(stk_model* m, double alpha_scale, double beta_scale);
STK_API int stk_model_destroy(stk_model* m);
STK_API int stk_model_info(const stk_model* m, int shard, int32_t* D, int32_t* P, int64_t* n_rows);
STK_API int stk_model_copy_data(stk_model* m, int shard, double* x, double* y, int32_t* y_int);
STK_API int stk_model_device_bytes(const stk_model* m, int64_t* bytes);

/* ---- log density + gradient at C points of one shard (parity hook) ---- */
STK_API int stk_log_density_grad(stk_model* m, int shard, const double* q, int32_t C, double* lp, double* grad);

/* ---- sampling: stark/stark.py:43-56 for every shard of the model ---- */
STK_API int stk_sampler_create(stk_model* m, const stk_config* cfg, stk_sampler** out);
/* Advance every chain until it has completed `target_iter` transitions (warmup counted),
 * or finished.  max_steps bounds the state-machine steps of this call (0 = no bound). */
STK_API int stk_sampler_run(stk_sampler* s, int32_t target_iter, int64_t max_steps);
STK_API int stk_sampler_info(stk_sampler* s, stk_run_info* info);
/* Draws of one shard: out[P][chains * num_samples] (chain-major columns), stats
 * [chains * num_samples][6] = accept_stat, stepsize, treedepth, n_leapfrog, divergent, energy.
 * Either pointer may be NULL. */
STK_API int stk_sampler_draws(stk_sampler* s, int shard, double* out, double* stats);
/* Unconstrained draws of one shard: out[chains][num_samples][D], or
 * out[chains][num_warmup + num_samples][D] when cfg.save_warmup is set. */
STK_API int stk_sampler_draws_unconstrained(stk_sampler* s, int shard, double* out);
STK_API int stk_sampler_adaptation(stk_sampler* s, double* stepsize, double* inv_metric);
/* Transitions completed so far by every chain (nshards * chains, shard-major). */
STK_API int stk_sampler_iterations(stk_sampler* s, int32_t* iters);
STK_API int stk_sampler_destroy(stk_sampler* s);

/* ---- checkpoint / resume of a run between stk_sampler_run calls.  The state is every chain's
 * device state (position, momentum, gradient, tree stack, adaptation windows and dual-averaging
 * scalars, Philox counters, mode and iteration), the draws and stats so far and the pending
 * evaluation requests, plus the step counters: a run saved after any stk_sampler_run call and
 * loaded into a sampler created from the same model geometry and config -- in another process,
 * on another device -- continues bit for bit as the unsplit run would (the reference has no
 * counterpart: a pystan fit cannot be resumed; SURVEY.md 8 aux "checkpoint/resume").
 * stk_sampler_state_bytes gives the size of the blob; stk_sampler_load_state refuses a blob
 * of another geometry / config (STK_E_ARG) before writing anything.  The data rows themselves
 * are not hashed (that would read the whole shard): loading into a model of the same geometry
 * built from other data is the caller's error and is not detected. */
STK_API int stk_sampler_state_bytes(stk_sampler* s, int64_t* bytes);
STK_API int stk_sampler_save_state(stk_sampler* s, void* buf, int64_t bytes);
STK_API int stk_sampler_load_state(stk_sampler* s, const void* buf, int64_t bytes);

/* ---- full-data mode (BASELINE configs[4]): ONE posterior whose rows are split over ranks.
 * Every rank builds a one-shard model of its rows and a sampler with the same config and the
 * same shard_ids (so the chains' RNG streams agree); after each step's local sweep + reduce,
 * `fn` must replace the [nchains][Dp] gradient block followed by the [nchains] log densities
 * (count = nchains * (Dp + 1) doubles, stk_sampler_grad_block) by their sum over ranks, ordered
 * on `stream` (the context's stream), and return 0.  Every rank then runs the NUTS step on
 * identical inputs, so chain states stay identical without any other exchange.  dev_block:
 * NULL (the library's block), or caller-allocated device memory of `count` doubles used in
 * its place -- e.g. a torch tensor that torch.distributed.all_reduce sums over RCCL.  Logistic
 * family with flat priors only (its log density is a pure sum over rows); call before the first run.
 * No reference counterpart (SURVEY.md 8e "full-data extension"). */
typedef int (*stk_allreduce_fn)(void* user, double* block, int64_t count, void* stream);
STK_API int stk_sampler_grad_block(stk_sampler* s, int64_t* count);
STK_API int stk_sampler_set_allreduce(stk_sampler* s, stk_allreduce_fn fn, void* user, double* dev_block);
STK_API int stk_sample(stk_model* m, const stk_config* cfg, double* draws, double* stats, stk_run_info* info);

/* One fixed-step-size NUTS transition per chain from q (C x D, updated in place), no
 * adaptation, RNG iteration index `iteration`: the unit of the GPU/CPU twin check. */
STK_API int stk_transition(stk_model* m, int shard, double* q, int32_t C, uint64_t seed, int32_t iteration,
                           double eps, const double* inv_metric, int32_t max_depth, double* lp, double* stats);

/* ---- consensus combine: stark/stark.py:7-21, 66-70 ---- */
/* draws: nshards x P x S, out: P x S (host or device memory; device buffers are read and
 * written in place, host buffers staged through the context).  shard_used[s] = 0 for shards
 * left out because of NaN draws.  Singular matrices (STK_E_LINALG, numpy's LinAlgError):
 *   - stk_consensus / _blocked / _products invert each sample covariance and sum W, which are
 *     symmetric positive (semi)definite by construction, by diagonal-pivot block Gauss-Jordan on
 *     the unit-diagonal matrix and report a pivot <= P eps or NaN as singular.  S <= p draws
 *     (p = P, or the largest row_block block) give a rank-deficient covariance (rank <= S - 1)
 *     and raise before any arithmetic; np.linalg.inv's LU usually returns a huge finite
 *     "inverse" built from rounding noise there, and raises only on an exactly zero pivot (a
 *     constant row: both raise) -- DESIGN.md section 9.  An exactly duplicated parameter row
 *     with S >> P draws is singular too: its unit-diagonal pivot is within 4.4e-16 of zero,
 *     below P eps, so it raises; numpy raises or returns ~1e34 entries depending on the
 *     rounding (tests/test_gpu_kernels.py::test_combine_duplicated_parameter_row_is_singular);
 *   - stk_consensus_solve takes the caller's sum W as ANY square matrix (symmetric or not) and
 *     inverts it as np.linalg.inv does, by partial pivoting, singular only on an exactly zero
 *     pivot. */
STK_API int stk_consensus_products(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S,
                                   double* sum_w, double* sum_wtheta, int32_t* shard_used);
STK_API int stk_consensus_solve(stk_ctx* ctx, const double* sum_w, const double* sum_wtheta, int32_t P,
                                int32_t S, double* out);
STK_API int stk_consensus(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S, double* out,
                          int32_t* shard_used);
/* stk_consensus with block-diagonal weights: row_block[a] names the weight block of row a
 * (e.g. 0 for the parameters, 1 for lp__); covariances between rows of different blocks are
 * taken as 0, so each block is combined from its own covariance. */
STK_API int stk_consensus_blocked(stk_ctx* ctx, const double* draws, int32_t nshards, int32_t P, int32_t S,
                                  const int32_t* row_block, double* out, int32_t* shard_used);

#ifdef __cplusplus
}
#endif
#endif /* STARK_HIP_H */
