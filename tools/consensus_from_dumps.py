#!/usr/bin/env python3
"""ESS/s of an 8-GPU job measured one rank at a time: BASELINE configs[3] (logistic N = 1e8,
d = 100, 8 shards x 16 chains) under the reference's sampler settings (pystan 2 = Stan 2.19.1's
criterion, stepsize_jitter 0, iter = 2000: 1000 warmup + 1000 draws), where one 8-shard launch
on one GPU does not fit a gpurun call.

Each shard k ran as `bench.py --rows 1.25e7 --shards 1 --shard-offset k --dump-draws ...`: the
rows and RNG keys of shard k of the 8-shard job, alone on one GPU -- what rank k of the 8-GPU
job runs (one shard per GPU, no data-path collective).  This script combines the
dumps as the job's consensus would (engine.consensus(separate_lp=True), restated here in numpy:
W_s = blockdiag(inv(cov(alpha, beta)), 1 / var(lp__)), theta = inv(sum W_s) sum W_s theta_s,
stark/stark.py:7-21, 66-70) and reports Stan 2.19's multi-chain ESS of the consensus (min over
alpha, beta; combined chain c = chain c of every shard) over the job's wall time = the slowest
rank's warmup + sampling.

usage: tools/consensus_from_dumps.py dump0.npz ... dump7.npz [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stark_amd import diagnostics  # noqa: E402


def block_consensus(shards):
    """shards: list of P x S arrays (last row lp__) -> P x S consensus draws."""
    P = shards[0].shape[0]
    sw = np.zeros((P, P))
    swt = np.zeros_like(shards[0])
    for th in shards:
        w = np.zeros((P, P))
        w[:-1, :-1] = np.linalg.inv(np.cov(th[:-1]))
        w[-1, -1] = 1.0 / np.var(th[-1], ddof=1)
        sw += w
        swt += w @ th
    return np.linalg.solve(sw, swt)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dumps", nargs="+")
    p.add_argument("--json", default=None)
    p.add_argument("--seed", type=int, default=20240, help="bench.py's data seed")
    a = p.parse_args()
    draws, per = {}, []
    C = n = None
    for f in a.dumps:
        z = np.load(f)          # written by bench.py (this repo), arrays only
        C, n = int(z["chains"]), int(z["draws_per_chain"])
        for sid in z["shard_ids"]:
            draws[int(sid)] = z[f"draws_{int(sid)}"]
        per.append({"file": os.path.basename(f), "shard_ids": [int(v) for v in z["shard_ids"]],
                    "t_adapt": float(z["t_adapt"]), "t_sampling": float(z["t_sampling"]),
                    "draws_per_chain": int(z["draws_per_chain"]),
                    "grad_evals": int(z["grad_evals"]), "leapfrogs_per_transition": float(z["leapfrogs_per_transition"]),
                    "divergent": int(z["divergent"])})
    # a rank stopped at a time budget (bench.py --ess-budget-s) has fewer draws per chain: the job
    # is the first n_common draws of every chain of every rank, its wall the slowest rank's
    ns = {k: v.shape[1] // C for k, v in draws.items()}
    n = min(ns.values())
    draws = {k: v.reshape(v.shape[0], C, ns[k])[:, :, :n].reshape(v.shape[0], C * n) for k, v in draws.items()}
    ids = sorted(draws)
    shards = [draws[k] for k in ids]
    comb = block_consensus(shards)

    def min_ess(x):
        return float(np.nanmin([diagnostics.ess(x[r].reshape(C, n)) for r in range(x.shape[0])]))

    wall = max(r["t_adapt"] + r["t_sampling"] for r in per)
    acc = None
    if len(ids) == 8:            # the whole job: the consensus mean against the generating parameters
        from stark_amd import engine
        d = comb.shape[0] - 2
        truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, d)])
        z = (comb[:-1].mean(1) - truth) / comb[:-1].std(1)
        acc = {"vs_generating_params": {"mean_z2": float((z ** 2).mean()), "max_abs_z": float(np.abs(z).max())}}
    ess = min_ess(comb[:-1])
    out = {"metric": "ESS/s of the consensus, configs[3] under the reference's sampler settings, 8-GPU job run one rank "
                     "at a time on one GPU",
           "shards": ids, "chains_per_shard": C, "post_warmup_draws_per_chain": n,
           "post_warmup_draws_per_chain_by_rank": {str(k): ns[k] for k in ids},
           "min_ess": ess, "job_wall_s": wall, "ess_per_sec": ess / wall,
           "subposterior_min_ess": {str(k): min_ess(draws[k][:-1]) for k in ids},
           "per_rank": per, "accuracy": acc,
           "posterior_mean_alpha_beta_first": [float(v) for v in comb[:4].mean(1)],
           "note": "wall = max over ranks of (warmup + sampling) measured on one GPU per shard (a rank stopped at a "
                   "time budget counts to its stop); the consensus of the first post_warmup_draws_per_chain draws "
                   "of every chain; consensus = "
                   "engine.consensus(separate_lp=True) restated in numpy; ESS = Stan 2.19's estimator "
                   "(stark_amd.diagnostics.ess), min over alpha, beta"}
    print(json.dumps(out))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
