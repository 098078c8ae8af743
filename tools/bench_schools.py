#!/usr/bin/env python3
"""8-schools with 4096 parallel NUTS chains on one MI355X (BASELINE.json configs[1]).

The data are example/stark_ex.py:4-6 (J = 8, embedded here: /root/reference does not exist on
the GPU box); the program is example/schools.stan (non-centred: mu, tau, eta[J]).  All 4096
chains run Stan's defaults (1000 warmup with adaptation + 1000 draws) in the fused kernel
(k_nuts_fused_schools: one wave per chain, the O(J) gradient inline, up to 4096 leapfrogs per
launch; 4 chains share a wave at J = 8, 16 lanes each).  Reported: chain-gradient evaluations
per second over the whole run and over the sampling phase, ESS/s of the sampling phase (min
over mu, tau, eta, theta of Stan 2.19's multi-chain ESS over all 4096 chains), and a VALU
roofline line: the gradient's fp64 operations (FLOPS_PER_GRAD, counted from schools_lpgrad
in nuts.hip: 14 per school -- theta = mu + tau eta (2), z = (y - theta) / sigma (2), r = z /
sigma (1), lp += -eta^2/2 - z^2/2 (4), the three sums (3), grad eta (2) -- plus exp(tau),
the Jacobian and the two sum finishes) times gradients/s, against the 78.6 TF fp64 peak.
The NUTS bookkeeping around each gradient (kinetic energy, U-turn dot products, multinomial
log-sum-exp, Philox) is not counted: it is what bounds this kernel -- a serial chain of
dependent fp64 operations per leapfrog, latency-bound at one wave per SIMD.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FLOPS_PER_GRAD = lambda J: 14 * J + 4
FP64_PEAK_TFS = 78.6
Y = [28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0]        # example/stark_ex.py:5
SIGMA = [15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0]  # example/stark_ex.py:6


def run(chains=4096, warmup=1000, samples=1000, seed=7, chains_per_wave=0, ctx=None):
    """One 8-schools run of `chains` chains (Stan defaults: 1000 warmup + 1000 draws); returns the
    line as a dict (bench.py embeds it as its configs[1] sub-record)."""
    from stark_amd import diagnostics, engine
    own = ctx is None
    ctx = ctx or engine.Context(0)
    m = engine.Model(ctx, "schools", [{"y": np.array(Y), "sigma": np.array(SIGMA)}])
    s = m.sampler(num_warmup=warmup, num_samples=samples, chains=chains, seed=seed,
                  chains_per_wave=chains_per_wave)
    ctx.sync()
    t0 = time.perf_counter()
    s.run(warmup)
    ctx.sync()
    t1 = time.perf_counter()
    i1 = s.info()
    s.run()
    ctx.sync()
    t2 = time.perf_counter()
    i2 = s.info()
    draws, stats = s.draws(0)
    P = draws.shape[0]
    e = diagnostics.ess_matrix(draws[:-1], chains)      # drop lp__
    min_ess = float(np.nanmin(e))
    samp = t2 - t1
    line = {
        "metric": "gradient evals/sec, 8-schools 4096 NUTS chains (1 GPU)",
        "value": (i2["grad_evals"] - i1["grad_evals"]) / samp, "unit": "gradient evals/sec",
        "n_gpus": 1, "higher_is_better": True, "dtype": "f64", "data": "example/stark_ex.py 8-schools",
        "config": {"workload": "8-schools non-centred, NUTS diag_e, Stan defaults", "chains": chains,
                   "num_warmup": warmup, "num_samples": samples, "P": P},
        "grad_evals_per_sec_whole_run": i2["grad_evals"] / (t2 - t0),
        "ess_per_sec_sampling": min_ess / samp, "min_ess": min_ess,
        "ess_per_sec_whole_run": min_ess / (t2 - t0),
        "seconds": {"warmup": t1 - t0, "sampling": samp},
        "leapfrogs_per_transition": (i2["leapfrogs"] - i1["leapfrogs"]) / (chains * samples),
        "divergent": i2["divergent"], "accept_stat_mean": float(stats[:, 0].mean()),
        "posterior_mean_mu_tau": [float(draws[0].mean()), float(draws[1].mean())],
        "roofline": {"bound": "fp64 VALU (latency-bound state machine)",
                     "achieved": (i2["grad_evals"] - i1["grad_evals"]) / samp * FLOPS_PER_GRAD(len(Y)) / 1e12,
                     "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "flops_per_grad": FLOPS_PER_GRAD(len(Y))},
        "chains_per_wave": chains_per_wave or 4,
    }
    line["roofline"]["frac"] = line["roofline"]["achieved"] / FP64_PEAK_TFS
    s.close()
    m.close()
    if own:
        ctx.close()
    return line


def main():
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("--chains", type=int, default=4096)
    p.add_argument("--warmup", type=int, default=1000)
    p.add_argument("--samples", type=int, default=1000)
    p.add_argument("--seed", type=int, default=7)
    p.add_argument("--chains-per-wave", type=int, default=0, help="fused kernel packing cap (0: 4 chains per wave)")
    a = p.parse_args()
    print(json.dumps(run(a.chains, a.warmup, a.samples, a.seed, a.chains_per_wave)), flush=True)


if __name__ == "__main__":
    main()
