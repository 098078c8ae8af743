#!/usr/bin/env python3
"""BASELINE configs[3] under the reference's sampler settings, run to completion one rank at a
time with checkpoint / resume.

The 8-GPU job (logistic N = 1e8, d = 100, one 1.25e7-row shard x 16 chains per GPU, no
data-path collective) under pystan 2's settings -- Stan 2.19.1's NUTS criterion, stepsize_jitter
0, iter = 2000: 1000 warmup + 1000 draws per chain (stark/stark.py:48, 60-63) -- has ranks that
take longer than one gpurun call.  Here rank k (shard k's rows and RNG keys, exactly what
`bench.py --rows 1.25e7 --shards 1 --shard-offset k` samples) runs on this GPU under a wall
budget; when the budget runs out the sampler state is saved (engine.Sampler.save_state: every
chain's position, momentum, tree stack, adaptation and RNG counters, the draws so far) together
with the sampling time spent, and the next call loads it and continues -- bit for bit the run
that never stopped (tests/test_gpu_nuts.py::test_run_split_across_processes_is_bit_identical).
Sampling time counts only the sampler's own run() calls (data generation and the state round
trip excluded), so a rank's time is what one GPU of the 8-GPU job spends.  A finished rank
writes bench.py's --dump-draws format; tools/consensus_from_dumps.py combines the eight.

usage: tools/refcfg_ranks.py --ranks 0,1,...,7 --budget-s 1000 --state-dir state --out-dir gpurun_out/rXX
  (a rank with a done dump in --state-dir is skipped; one with a saved state resumes from it)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ROWS, D, CHAINS, NW, NS, SEED = 12_500_000, 100, 16, 1000, 1000, 20240


def run_rank(k, ctx, budget_end, state_dir, out_dir):
    from stark_amd import engine
    done = os.path.join(state_dir, f"rank{k}.npz")
    if os.path.exists(done):
        return "done"
    model = engine.Model.synthetic(ctx, "logistic", 1, ROWS, D, data_seed=SEED, row_offset=k * ROWS)
    s = model.sampler(num_warmup=NW, num_samples=NS, chains=CHAINS, seed=SEED + 1, shard_ids=[k],
                      stepsize_jitter=0.0, nuts_criterion="stan2.19")
    st_in = os.path.join(state_dir, f"rank{k}_state.npz")
    t_adapt = t_samp = 0.0
    calls = 1
    if os.path.exists(st_in):
        z = np.load(st_in)                      # written by this script: arrays only
        s.load_state(z["state"])
        t_adapt, t_samp, calls = float(z["t_adapt"]), float(z["t_sampling"]), int(z["calls"]) + 1
    ctx.sync()
    print(f"[refcfg] rank {k}: start at transitions min {s.iterations().min()} (call {calls})", flush=True)
    last = time.monotonic()
    for target in (NW, NW + NS):
        while True:
            its = s.iterations()
            if its.min() >= target:
                break
            if time.monotonic() > budget_end:
                blob = s.save_state()
                np.savez_compressed(os.path.join(out_dir, f"rank{k}_state.npz"), state=blob, t_adapt=t_adapt,
                                    t_sampling=t_samp, calls=calls)
                print(f"[refcfg] rank {k}: budget reached at transitions min {its.min()}, state saved "
                      f"({blob.size / 1e6:.1f} MB)", flush=True)
                s.close()
                model.close()
                return "saved"
            t = time.perf_counter()
            s.run(target, max_steps=4000)
            dt = time.perf_counter() - t
            if target == NW:
                t_adapt += dt
            else:
                t_samp += dt
            if time.monotonic() - last > 30:
                last = time.monotonic()
                print(f"[refcfg] rank {k}: transitions min/median {its.min()}/{int(np.median(its))}, "
                      f"adapt {t_adapt:.0f}s sampling {t_samp:.0f}s", flush=True)
    info = s.info()
    draws, stats = s.draws(0)
    np.savez(os.path.join(out_dir, f"rank{k}.npz"), shard_ids=np.array([k]), chains=CHAINS, draws_per_chain=NS,
             t_adapt=t_adapt, t_sampling=t_samp, grad_evals=info["grad_evals"],
             leapfrogs_per_transition=float(stats[:, 3].mean()), divergent=info["divergent"], calls=calls,
             **{f"draws_{k}": draws})
    print(json.dumps({"rank": k, "t_adapt": t_adapt, "t_sampling": t_samp, "calls": calls,
                      "leapfrogs_per_transition": float(stats[:, 3].mean()), "divergent": info["divergent"]}),
          flush=True)
    s.close()
    model.close()
    return "done"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", default="0,1,2,3,4,5,6,7")
    p.add_argument("--budget-s", type=float, default=1000.0, help="wall budget of this call's sampling")
    p.add_argument("--state-dir", default=os.path.join(ROOT, "state"))
    p.add_argument("--out-dir", required=True)
    a = p.parse_args()
    os.makedirs(a.out_dir, exist_ok=True)
    from stark_amd import engine
    ctx = engine.Context(0)
    end = time.monotonic() + a.budget_s
    for k in (int(v) for v in a.ranks.split(",")):
        if run_rank(k, ctx, end, a.state_dir, a.out_dir) == "saved":
            break
    ctx.close()


if __name__ == "__main__":
    main()
