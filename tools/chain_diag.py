#!/usr/bin/env python3
"""Per-chain adaptation / tree-depth diagnostics for the bench configuration."""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stark_amd import engine  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=float, default=8e6)
p.add_argument("--d", type=int, default=100)
p.add_argument("--shards", type=int, default=8)
p.add_argument("--chains", type=int, default=4)
p.add_argument("--adapt", type=int, default=300)
p.add_argument("--samples", type=int, default=100)
p.add_argument("--init", default="random")
p.add_argument("--init-r", type=float, default=2.0)
p.add_argument("--jitter", type=float, default=0.0)
a = p.parse_args()
ctx = engine.Context(0)
rps = int(a.rows) // a.shards
m = engine.Model.synthetic(ctx, "logistic", a.shards, rps, a.d, data_seed=20240)
kw = dict(num_warmup=a.adapt, num_samples=a.samples, chains=a.chains, seed=20241, save_warmup=True,
          init_radius=a.init_r, stepsize_jitter=a.jitter)
if a.init == "zero":
    kw["init"] = np.zeros(a.shards * a.chains * (a.d + 1))
s = m.sampler(**kw)
t = time.time()
for it in range(25, a.adapt + a.samples + 25, 25):
    s.run(min(it, a.adapt + a.samples))
    print(f"{min(it, a.adapt + a.samples)} iters {time.time() - t:.1f}s leapfrogs {s.info()['leapfrogs']}", flush=True)
eps, im = s.adaptation()
beta = engine.Model.gen_beta(20240, a.d)
for sh in range(a.shards):
    d_, st = s.draws(sh)
    uq = s.unconstrained(sh)
    for c in range(a.chains):
        g = sh * a.chains + c
        depth = st[c * a.samples:(c + 1) * a.samples, 2]
        nl = st[c * a.samples:(c + 1) * a.samples, 3]
        q = uq[c]
        warm = q[:a.adapt]
        dist_w = np.abs(warm[:, 1:] - beta).max(axis=1)
        print(f"shard {sh} chain {c}: eps {eps[g]:.4g} im[min/med/max] {im[g, :a.d+1].min():.3g}/{np.median(im[g, :a.d+1]):.3g}/{im[g, :a.d+1].max():.3g} "
              f"depth mean {depth.mean():.2f} max {depth.max():.0f} nleap mean {nl.mean():.1f} "
              f"|beta-true|max at warmup it 0/50/75/100/150/end {dist_w[0]:.3g}/{dist_w[min(50,len(dist_w)-1)]:.3g}/{dist_w[min(75,len(dist_w)-1)]:.3g}/{dist_w[min(100,len(dist_w)-1)]:.3g}/{dist_w[min(150,len(dist_w)-1)]:.3g}/{dist_w[-1]:.3g}", flush=True)
