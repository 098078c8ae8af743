#!/usr/bin/env python3
"""Large-scale check of the consensus path against the data-generating parameters: per-shard
subposterior means and the consensus-combined mean, each as z = (mean - truth) / sd, with
split R-hat per shard (synthetic logistic data; the truth is known exactly)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stark_amd import diagnostics, engine  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=float, default=1e7)
p.add_argument("--d", type=int, default=100)
p.add_argument("--shards", type=int, default=8)
p.add_argument("--chains", type=int, default=16)
p.add_argument("--warmup", type=int, default=300)
p.add_argument("--samples", type=int, default=300)
p.add_argument("--seed", type=int, default=20240)
p.add_argument("--jitter", type=float, default=0.5)
a = p.parse_args()
ctx = engine.Context(0)
rps = int(a.rows) // a.shards
m = engine.Model.synthetic(ctx, "logistic", a.shards, rps, a.d, data_seed=a.seed)
s = m.sampler(num_warmup=a.warmup, num_samples=a.samples, chains=a.chains, seed=a.seed + 1, stepsize_jitter=a.jitter)
total = a.warmup + a.samples
for t in list(range(50, total, 50)) + [total]:     # resumable run: a progress line per 50 transitions
    s.run(t)
    print(f"[consensus_check] {t}/{total} transitions per chain", file=sys.stderr, flush=True)
truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
draws = [s.draws(k)[0] for k in range(a.shards)]
out = {"config": vars(a), "shards": []}
for k, dr in enumerate(draws):
    x = dr[:-1]
    z = (x.mean(1) - truth) / x.std(1)
    rh = max(diagnostics.split_rhat(x[j].reshape(a.chains, -1)) for j in range(x.shape[0]))
    out["shards"].append({"max_abs_z": float(np.abs(z).max()), "mean_z2": float((z ** 2).mean()), "max_rhat": rh})
comb, used = engine.consensus(draws, ctx)
z = (comb[:-1].mean(1) - truth) / comb[:-1].std(1)
out["consensus"] = {"max_abs_z": float(np.abs(z).max()), "mean_z2": float((z ** 2).mean())}
comb_b, _ = engine.consensus(draws, ctx, separate_lp=True)     # lp__ in its own weight block
zb = (comb_b[:-1].mean(1) - truth) / comb_b[:-1].std(1)
out["consensus_separate_lp"] = {"max_abs_z": float(np.abs(zb).max()), "mean_z2": float((zb ** 2).mean())}
# is the excess in the subposteriors themselves?  mean over shards of the signed shard z,
# times sqrt(S): ~N(0, 1) per parameter when the shards' errors are independent
zsh = np.array([(dr[:-1].mean(1) - truth) / dr[:-1].std(1) for dr in draws])
zc = zsh.mean(0) * np.sqrt(len(draws))
out["shard_mean_z_times_sqrtS_mean_sq"] = float((zc ** 2).mean())
out["shard_z_corr_with_beta"] = float(np.corrcoef(zsh.mean(0)[1:], truth[1:])[0, 1])
out["consensus_err_corr_with_beta"] = float(np.corrcoef(zb[1:], truth[1:])[0, 1])
lpm = np.array([dr[-1].mean() for dr in draws])
out["lp_offsets_over_sd"] = float(lpm.std() / np.mean([dr[-1].std() for dr in draws]))
# the consensus mean vs the average of the subposterior means (should agree to within sd/sqrt(S))
sub_mean = np.mean([dr[:-1].mean(1) for dr in draws], axis=0)
out["consensus_minus_submean_over_sd"] = float(np.abs((comb[:-1].mean(1) - sub_mean) / comb[:-1].std(1)).max())
out["info"] = s.info()
print(json.dumps(out, indent=1))
