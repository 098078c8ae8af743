#!/usr/bin/env python3
"""North-star check at the headline scale against a full-data NUTS run (not a Laplace
approximation): the same synthetic rows (logistic, N = 1e8, d = 100) sampled

  (a) as 8 subposterior shards, combined by the consensus weighted average (stark/stark.py:59-71;
      lp__ in its own weight block), and
  (b) as ONE shard holding all N rows: the full-data posterior, sampled by the same GPU NUTS
      (the reference's Stan settings otherwise: diag_e, windowed adaptation).

Reported per alpha, beta: z = (consensus mean - full-data mean) in full-data posterior sds and
in MCSE units (the full-data chains' Stan 2.19 ESS and the consensus's batch MCSE: the chains of
every shard split into groups, each group combined on its own), the consensus / full-data sd
ratio, and both runs against the Laplace reference of the full data (tools/laplace.py).  The two
runs share one GPU one after the other (80 GB of rows each).  Progress goes to stderr per block of
iterations; the JSON record is written to --out and printed at the end.
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
    p.add_argument("--samples", type=int, default=250)
    p.add_argument("--groups", type=int, default=4, help="chain groups for the consensus batch MCSE")
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
    comb, used = engine.consensus(draws, ctx, separate_lp=True)
    assert used.all()
    G = a.groups
    gm = []
    for g in range(G):                                             # batch MCSE of the consensus mean
        cols = np.concatenate([np.arange(c * S, (c + 1) * S) for c in range(g * C // G, (g + 1) * C // G)])
        cg, _ = engine.consensus([d[:, cols] for d in draws], ctx, separate_lp=True)
        gm.append(cg[:-1].mean(1))
    mcse_c = np.std(gm, axis=0, ddof=1) / np.sqrt(G)
    c_mean, c_sd = comb[:-1].mean(1), comb[:-1].std(1)
    s8.close()
    m8.close()
    log(f"consensus done in {t_cons:.1f}s")

    # ---- (b) the full data as one shard
    m1 = engine.Model.synthetic(ctx, "logistic", 1, rps * a.shards, a.d, data_seed=a.seed)
    s1 = m1.sampler(num_warmup=a.full_warmup, num_samples=S, chains=C, seed=a.seed + 2,
                    stepsize_jitter=a.jitter, nuts_criterion=a.nuts_criterion)
    t = time.perf_counter()
    run(s1, a.full_warmup, S, a.block, log, "full data")
    t_full = time.perf_counter() - t
    dr1, st1 = s1.draws(0)
    x = dr1[:-1]
    f_mean, f_sd = x.mean(1), x.std(1)
    ess_f = np.array([diagnostics.ess(x[k].reshape(C, S)) for k in range(x.shape[0])])
    rhat_f = np.array([diagnostics.split_rhat(x[k].reshape(C, S)) for k in range(x.shape[0])])
    mcse_f = f_sd / np.sqrt(ess_f)
    eps1, _ = s1.adaptation()
    info1 = s1.info()
    s1.close()
    log(f"full-data NUTS done in {t_full:.1f}s; min ESS {ess_f.min():.0f}")
    fm, fc, finfo = L.laplace(m1, [0], f_mean, f_sd)
    fsd_l = np.sqrt(np.diag(fc))
    m1.close()

    z_sd = (c_mean - f_mean) / f_sd
    z_mcse = (c_mean - f_mean) / np.sqrt(mcse_f ** 2 + mcse_c ** 2)
    truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
    rec = {
        "config": vars(a),
        "consensus_vs_fulldata_nuts": {"in_fulldata_sd": zstats(z_sd), "in_mcse": zstats(z_mcse),
                                       "sd_ratio_median": float(np.median(c_sd / f_sd)),
                                       "sd_ratio_min_max": [float((c_sd / f_sd).min()), float((c_sd / f_sd).max())]},
        "fulldata_nuts_vs_laplace": {"mean_in_sd": zstats((f_mean - fm) / fsd_l),
                                     "sd_ratio_median": float(np.median(f_sd / fsd_l))},
        "consensus_vs_laplace": {"mean_in_sd": zstats((c_mean - fm) / fsd_l),
                                 "sd_ratio_median": float(np.median(c_sd / fsd_l))},
        "fulldata_nuts_vs_truth": zstats((f_mean - truth) / f_sd),
        "fulldata_nuts": {"min_ess": float(ess_f.min()), "median_ess": float(np.median(ess_f)),
                          "max_split_rhat": float(rhat_f.max()),
                          "stepsize": [float(eps1.min()), float(np.median(eps1)), float(eps1.max())],
                          "leapfrogs_per_transition": float(st1[:, 3].mean()), "divergent": info1["divergent"],
                          "seconds": t_full},
        "consensus": {"mcse_median_in_sd": float(np.median(mcse_c / f_sd)), "seconds": t_cons},
        "laplace_newton_steps_in_sd": finfo["newton_steps_in_sd"],
        "elapsed_s": time.perf_counter() - t0,
    }
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    v = rec["consensus_vs_fulldata_nuts"]
    log(f"consensus vs full-data NUTS: mean z2 {v['in_fulldata_sd']['mean_z2']:.4f} (sd units), "
        f"{v['in_mcse']['mean_z2']:.2f} (MCSE units); sd ratio {v['sd_ratio_median']:.3f}")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
