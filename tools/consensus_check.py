#!/usr/bin/env python3
"""Consensus accuracy at scale against the FULL-DATA posterior (synthetic logistic data,
SURVEY 8d): 8 subposterior shards sampled by the GPU NUTS, combined by the consensus
weighted average (stark/stark.py:59-71), compared per parameter with

  * the full-data posterior (tools/laplace.py: MAP + inverse Hessian from the GPU gradient,
    Gaussian to O(d/sqrt(N)) at N = 1e8) -- the north_star's "matching the posterior
    moments within MCSE";
  * the data-generating parameters (the truth; a property of the one fixed dataset too).

The consensus estimator's Monte Carlo standard error includes the noise of its SAMPLED
weights W_s = inv(cov(draws_s)); it is estimated by batches: the 16 chains of every shard
are split into G groups, each group is combined on its own, and mcse = sd(group means) /
sqrt(G).  Diagnostics that split the error into its sources:

  * shard z vs the shard's own Laplace mean (the sampler alone);
  * the plain average of shard means vs the full-data MAP;
  * the consensus with EXACT weights (each shard's Laplace precision) applied to the
    sampled draws vs the full-data MAP (the draws' Monte Carlo error alone);
  * the ESS of the centred squares (x - mean)^2 (how many draws the covariance really has).

Resumable: one JSON record per block of transitions is appended to --out (and a summary
line printed) as soon as it is computed, so a run cut by the lease still leaves data.
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


def chain_cut(dr, chains, ns, n):
    """First n draws of every chain of a P x (chains*ns) chain-major matrix."""
    return np.ascontiguousarray(np.concatenate([dr[:, c * ns:c * ns + n] for c in range(chains)], axis=1))


def z2(err, sd):
    z = err / sd
    return {"mean_z2": float((z ** 2).mean()), "max_abs_z": float(np.abs(z).max())}


def analyze(draws, chains, n, ctx, lap_full=None, lap_shards=None, truth=None, groups=4, lp_row=True):
    """draws: per shard a P x (chains*n) chain-major matrix (last row lp__ if lp_row).
    lap_full = (mean, cov) of the full-data posterior over the parameter rows;
    lap_shards = [(mean, cov)] per shard.  Returns a dict of accuracy figures."""
    th = [d[:-1] if lp_row else d for d in draws]
    out = {"draws_per_chain": n, "chains": chains}
    comb, _ = engine.consensus(draws, ctx, separate_lp=True) if lp_row else engine.consensus(draws, ctx)
    cm = comb[:-1].mean(1) if lp_row else comb.mean(1)
    csd = comb[:-1].std(1) if lp_row else comb.std(1)
    # batch MCSE of the consensus estimator (sampled weights included)
    gm = []
    cg = chains // groups
    for gi in range(groups):
        sel = [np.ascontiguousarray(d[:, gi * cg * n:(gi + 1) * cg * n]) for d in draws]
        cgd, _ = engine.consensus(sel, ctx, separate_lp=True) if lp_row else engine.consensus(sel, ctx)
        gm.append(cgd[:-1].mean(1) if lp_row else cgd.mean(1))
    mcse = np.std(np.array(gm), axis=0, ddof=1) / np.sqrt(groups)
    out["consensus_batch_mcse_over_sd_median"] = float(np.median(mcse / csd))
    if lp_row:
        joint, _ = engine.consensus(draws, ctx)
        jm = joint[:-1].mean(1)
    if truth is not None:
        out["vs_truth"] = {"consensus": z2(cm - truth, csd)}
        if lp_row:
            out["vs_truth"]["consensus_joint_lp"] = z2(jm - truth, csd)
        out["vs_truth"]["shards"] = [z2(t.mean(1) - truth, t.std(1)) for t in th]
    if lap_full is not None:
        fm, fc = lap_full
        fsd = np.sqrt(np.diag(fc))
        v = {"consensus": z2(cm - fm, fsd),
             "consensus_in_mcse": z2(cm - fm, mcse),
             "consensus_sd_ratio": {"median": float(np.median(csd / fsd)), "min": float((csd / fsd).min()),
                                    "max": float((csd / fsd).max())},
             "plain_average_of_shard_means": z2(np.mean([t.mean(1) for t in th], axis=0) - fm, fsd),
             "truth": z2(truth - fm, fsd) if truth is not None else None}
        if lp_row:
            v["consensus_joint_lp"] = z2(jm - fm, fsd)
        if lap_shards is not None:
            Ws = [np.linalg.inv(c) for _, c in lap_shards]
            ex = L.consensus_fixed_weights(th, Ws)
            v["consensus_exact_weights"] = z2(ex.mean(1) - fm, fsd)
            v["shards_vs_own_laplace"] = [z2(t.mean(1) - m, np.sqrt(np.diag(c))) for t, (m, c) in zip(th, lap_shards)]
            v["shard_sd_ratio_median"] = [float(np.median(t.std(1) / np.sqrt(np.diag(c))))
                                          for t, (_, c) in zip(th, lap_shards)]
        out["vs_fulldata"] = v
    # ESS of the means and of the centred squares (what the covariance estimate has), shard 0
    x = th[0]
    e1 = [diagnostics.ess(x[p].reshape(chains, n)) for p in range(x.shape[0])]
    e2 = [diagnostics.ess(((x[p] - x[p].mean()) ** 2).reshape(chains, n)) for p in range(x.shape[0])]
    out["shard0_ess"] = {"mean_min": float(np.nanmin(e1)), "mean_median": float(np.nanmedian(e1)),
                         "sq_min": float(np.nanmin(e2)), "sq_median": float(np.nanmedian(e2)),
                         "draws": chains * n}
    out["shard0_max_rhat"] = float(max(diagnostics.split_rhat(x[p].reshape(chains, n)) for p in range(x.shape[0])))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=float, default=1e8)
    p.add_argument("--d", type=int, default=100)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--chains", type=int, default=16)
    p.add_argument("--warmup", type=int, default=150)
    p.add_argument("--samples", type=int, default=250)
    p.add_argument("--block", type=int, default=50)
    p.add_argument("--seed", type=int, default=20240)
    p.add_argument("--jitter", type=float, default=0.5)
    p.add_argument("--nuts-criterion", choices=["stan2.19", "stan2.23"], default="stan2.19")
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "consensus_check.jsonl"))
    a = p.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    ctx = engine.Context(0)
    rps = int(a.rows) // a.shards
    m = engine.Model.synthetic(ctx, "logistic", a.shards, rps, a.d, data_seed=a.seed)
    s = m.sampler(num_warmup=a.warmup, num_samples=a.samples, chains=a.chains, seed=a.seed + 1,
                  stepsize_jitter=a.jitter, nuts_criterion=a.nuts_criterion)
    truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
    t0 = time.perf_counter()
    log = lambda msg: print(f"[consensus_check {time.perf_counter() - t0:7.1f}s] {msg}", file=sys.stderr, flush=True)
    for t in range(a.block, a.warmup, a.block):
        s.run(t)
        log(f"warmup {t}/{a.warmup}")
    s.run(a.warmup)
    lap_full = lap_shards = None
    shards = list(range(a.shards))
    for k in range(a.block, a.samples + 1, a.block):
        s.run(a.warmup + k)
        draws = [chain_cut(s.draws(sh)[0], a.chains, a.samples, k) for sh in shards]
        if lap_full is None:            # Laplace references, once, started from the first block
            t1 = time.perf_counter()
            pooled = np.hstack([d[:-1] for d in draws])
            sd0 = pooled.std(1) / np.sqrt(a.shards)
            lap_full = L.laplace(m, shards, pooled.mean(1), sd0)
            lap_shards = [L.laplace(m, [sh], d[:-1].mean(1), d[:-1].std(1)) for sh, d in zip(shards, draws)]
            log(f"laplace references in {time.perf_counter() - t1:.1f}s; full-data newton steps (sd) "
                f"{lap_full[2]['newton_steps_in_sd']}")
        rec = analyze(draws, a.chains, k, ctx, lap_full[:2], [x[:2] for x in lap_shards], truth)
        rec.update({"config": vars(a), "elapsed_s": time.perf_counter() - t0, "info": s.info()})
        eps, _ = s.adaptation()
        st = np.vstack([chain_cut(s.draws(sh)[1].T, a.chains, a.samples, k).T for sh in shards])
        rec["stepsize"] = {"min": float(eps.min()), "median": float(np.median(eps)), "max": float(eps.max())}
        rec["treedepth_mean"] = float(st[:, 2].mean())
        rec["leapfrogs_per_transition"] = float(st[:, 3].mean())
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
        v = rec["vs_fulldata"]
        log(f"{k} draws/chain: vs full-data z2 consensus {v['consensus']['mean_z2']:.3f} "
            f"(in mcse {v['consensus_in_mcse']['mean_z2']:.2f}), exact-weights {v['consensus_exact_weights']['mean_z2']:.3f}, "
            f"plain avg {v['plain_average_of_shard_means']['mean_z2']:.3f}, joint-lp {v['consensus_joint_lp']['mean_z2']:.3f}, "
            f"truth {v['truth']['mean_z2']:.3f}; sd ratio {v['consensus_sd_ratio']['median']:.3f}; "
            f"shard0 ess mean/sq min {rec['shard0_ess']['mean_min']:.0f}/{rec['shard0_ess']['sq_min']:.0f}")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
