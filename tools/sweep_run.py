#!/usr/bin/env python3
"""Run exactly --steps state-machine steps of the bench configuration (each step = one data
sweep over every local shard + reduce + NUTS step), for profiling runs under rocprofv3
(--pmc passes must stay short: the step count is fixed, independent of tree depths)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stark_amd import engine  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rows", type=float, default=1e8)
p.add_argument("--d", type=int, default=100)
p.add_argument("--shards", type=int, default=8)
p.add_argument("--chains", type=int, default=4)
p.add_argument("--steps", type=int, default=6)
a = p.parse_args()
ctx = engine.Context(0)
rps = int(a.rows) // a.shards
m = engine.Model.synthetic(ctx, "logistic", a.shards, rps, a.d, data_seed=20240)
s = m.sampler(num_warmup=150, num_samples=105, chains=a.chains, seed=20241, shard_ids=list(range(a.shards)))
s.run(255, max_steps=a.steps)
print(s.info(), flush=True)
s.close()
m.close()
