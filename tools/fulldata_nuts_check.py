#!/usr/bin/env python3
"""North-star check at the headline scale against a full-data NUTS run (not a Laplace
approximation): the same synthetic rows (logistic, N = 1e8, d = 100) sampled

  (a) as 8 subposterior shards, combined by the consensus weighted average (stark/stark.py:59-71;
      lp__ in its own weight block), and
  (b) as ONE shard holding all N rows: the full-data posterior, sampled by the same GPU NUTS
      (the reference's Stan settings otherwise: diag_e, windowed adaptation).

Reported per alpha, beta, at every draw count of --eval-draws (the first n post-warmup draws of
every chain, so 250 = the bench's count and 1000 = the reference's default, iter=2000 at
stark/stark.py:60-63): z = (consensus mean - full-data mean) in full-data posterior sds and in
MCSE units.  The MCSE of the full-data mean is sd / sqrt(ESS) (Stan 2.19 multi-chain ESS); the
MCSE of the consensus mean comes from batches -- every shard's chains split into G groups, each
group set combined on its own, the variance of the G group means / G -- POOLED over the
parameters relative to the full-data sd (the estimator of tests/test_gpu_consensus.py:26-38),
so the MCSE has (G - 1) x 101 degrees of freedom instead of G - 1.  The per-parameter batch
MCSE of round 2 is kept for comparison (`per_param_batch`): with G = 4 it is a 3-dof estimate,
under which even a perfectly calibrated estimator has E[z^2] = 3 (Student t, nu / (nu - 2)).
G = 4 and G = 16 (one chain per group) are both reported; `pass` = pooled mean z^2 < 2.5, the
GPU test's bar.  Also: the consensus / full-data sd ratio and both runs against the Laplace
reference of the full data (tools/laplace.py).  The two runs share one GPU one after the other
(80 GB of rows each).  Progress goes to stderr per block of iterations and the JSON record is
rewritten to --out after each stage (partial results survive a cut-off run).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stark_amd import diagnostics, engine  # noqa: E402
from tools import laplace as L  # noqa: E402


def run(sampler, warmup, samples, block, log, tag):
    for t in range(block, warmup + samples, block):
        sampler.run(t)
        log(f"{tag}: {t}/{warmup + samples} iterations, {sampler.info()['leapfrogs']} leapfrogs")
    sampler.run(warmup + samples)


def zstats(z):
    z = np.asarray(z)
    return {"mean_z2": float((z ** 2).mean()), "max_abs_z": float(np.abs(z).max())}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=float, default=1e8)
    p.add_argument("--d", type=int, default=100)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--chains", type=int, default=16)
    p.add_argument("--warmup", type=int, default=150, help="consensus shards' warmup (the bench's)")
    p.add_argument("--full-warmup", type=int, default=300, help="full-data run's warmup")
    p.add_argument("--samples", type=int, default=1000)
    p.add_argument("--eval-draws", default="250,1000", help="draw counts per chain to evaluate at")
    p.add_argument("--groups", default="4,16", help="chain group counts for the consensus batch MCSE")
    p.add_argument("--block", type=int, default=50)
    p.add_argument("--seed", type=int, default=20240)
    p.add_argument("--jitter", type=float, default=0.5)
    p.add_argument("--nuts-criterion", choices=["stan2.19", "stan2.23"], default="stan2.23")
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "fulldata_nuts_check.json"))
    a = p.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    t0 = time.perf_counter()
    log = lambda msg: print(f"[fulldata_nuts_check {time.perf_counter() - t0:7.1f}s] {msg}", file=sys.stderr, flush=True)
    ctx = engine.Context(0)
    C, S, n = a.chains, a.samples, int(a.rows)
    rps = n // a.shards

    # ---- (a) 8 shards + consensus
    m8 = engine.Model.synthetic(ctx, "logistic", a.shards, rps, a.d, data_seed=a.seed)
    s8 = m8.sampler(num_warmup=a.warmup, num_samples=S, chains=C, seed=a.seed + 1,
                    stepsize_jitter=a.jitter, nuts_criterion=a.nuts_criterion)
    t = time.perf_counter()
    run(s8, a.warmup, S, a.block, log, "shards")
    t_cons = time.perf_counter() - t
    draws = [s8.draws(sh)[0] for sh in range(a.shards)]          # P x (C S), chain-major columns
    s8.close()
    m8.close()
    evals = [int(v) for v in a.eval_draws.split(",") if int(v) <= S]
    groups = [int(v) for v in a.groups.split(",")]

    def first(dr, n, chains):                                    # the first n draws of the given chains
        cols = np.concatenate([np.arange(c * S, c * S + n) for c in chains])
        return np.ascontiguousarray(dr[:, cols])

    cons = {}
    for n in evals:
        sel = [first(dr, n, range(C)) for dr in draws]
        comb, used = engine.consensus(sel, ctx, separate_lp=True)
        assert used.all()
        gmeans = {}
        for G in groups:
            gm = []
            for g in range(G):
                cg, _ = engine.consensus([first(dr, n, range(g * C // G, (g + 1) * C // G)) for dr in draws],
                                         ctx, separate_lp=True)
                gm.append(cg[:-1].mean(1))
            gmeans[G] = np.array(gm)
        cons[n] = {"mean": comb[:-1].mean(1), "sd": comb[:-1].std(1), "gmeans": gmeans}
    log(f"consensus done in {t_cons:.1f}s")

    rec = {"config": vars(a), "consensus_seconds": t_cons, "stage": "consensus done"}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)

    # ---- (b) the full data as one shard
    m1 = engine.Model.synthetic(ctx, "logistic", 1, rps * a.shards, a.d, data_seed=a.seed)
    s1 = m1.sampler(num_warmup=a.full_warmup, num_samples=S, chains=C, seed=a.seed + 2,
                    stepsize_jitter=a.jitter, nuts_criterion=a.nuts_criterion)
    t = time.perf_counter()
    run(s1, a.full_warmup, S, a.block, log, "full data")
    t_full = time.perf_counter() - t
    dr1, st1 = s1.draws(0)
    eps1, _ = s1.adaptation()
    info1 = s1.info()
    s1.close()
    truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
    fm = fsd_l = finfo = None
    rec["by_draws"] = {}
    for n in evals:
        x = first(dr1, n, range(C))[:-1]
        f_mean, f_sd = x.mean(1), x.std(1)
        ess_f = np.array([diagnostics.ess(x[k].reshape(C, n)) for k in range(x.shape[0])])
        rhat_f = np.array([diagnostics.split_rhat(x[k].reshape(C, n)) for k in range(x.shape[0])])
        mcse_f = f_sd / np.sqrt(ess_f)
        if fm is None:
            log(f"full-data NUTS done in {t_full:.1f}s; min ESS {ess_f.min():.0f} at {n} draws")
            fm, fc, finfo = L.laplace(m1, [0], f_mean, f_sd)
            fsd_l = np.sqrt(np.diag(fc))
        c = cons[n]
        diff = c["mean"] - f_mean
        r = {"consensus_vs_fulldata_nuts": {"in_fulldata_sd": zstats(diff / f_sd),
                                            "sd_ratio_median": float(np.median(c["sd"] / f_sd)),
                                            "sd_ratio_min_max": [float((c["sd"] / f_sd).min()),
                                                                 float((c["sd"] / f_sd).max())]},
             "in_mcse": {}}
        for G, gm in c["gmeans"].items():
            var_g = np.var(gm, axis=0, ddof=1) / G                   # per-parameter batch variance
            rel = float(np.sqrt(np.mean(var_g / f_sd ** 2)))         # pooled relative MCSE
            z_pool = diff / np.sqrt((rel * f_sd) ** 2 + mcse_f ** 2)
            z_pp = diff / np.sqrt(var_g + mcse_f ** 2)
            zp = zstats(z_pool)
            r["in_mcse"][f"G{G}"] = {"pooled": zp, "pass": bool(zp["mean_z2"] < 2.5),
                                     "pooled_rel_mcse": rel,
                                     "per_param_batch": {**zstats(z_pp), "dof": G - 1,
                                                         "calibrated_expectation": (G - 1) / (G - 3) if G > 3 else None}}
        r["fulldata_nuts"] = {"min_ess": float(ess_f.min()), "median_ess": float(np.median(ess_f)),
                              "max_split_rhat": float(rhat_f.max()),
                              "mcse_median_in_sd": float(np.median(mcse_f / f_sd))}
        r["fulldata_nuts_vs_laplace"] = {"mean_in_sd": zstats((f_mean - fm) / fsd_l),
                                         "sd_ratio_median": float(np.median(f_sd / fsd_l))}
        r["consensus_vs_laplace"] = {"mean_in_sd": zstats((c["mean"] - fm) / fsd_l),
                                     "sd_ratio_median": float(np.median(c["sd"] / fsd_l))}
        r["fulldata_nuts_vs_truth"] = zstats((f_mean - truth) / f_sd)
        rec["by_draws"][str(n)] = r
        g4 = r["in_mcse"].get(f"G{groups[0]}", {})
        log(f"{n} draws/chain: mean z2 {r['consensus_vs_fulldata_nuts']['in_fulldata_sd']['mean_z2']:.4f} (sd units), "
            + ", ".join(f"{k}: pooled {v['pooled']['mean_z2']:.2f} / per-param {v['per_param_batch']['mean_z2']:.2f}"
                        for k, v in r["in_mcse"].items()) + " (MCSE units)")
    m1.close()
    rec["fulldata_run"] = {"stepsize": [float(eps1.min()), float(np.median(eps1)), float(eps1.max())],
                           "leapfrogs_per_transition": float(st1[:, 3].mean()), "divergent": info1["divergent"],
                           "seconds": t_full}
    rec["laplace_newton_steps_in_sd"] = finfo["newton_steps_in_sd"]
    rec["elapsed_s"] = time.perf_counter() - t0
    rec["stage"] = "done"
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
