#!/usr/bin/env python3
"""Latency of the consensus combine at the headline size (8 shards, P = 102, S = 1600 draws,
lp__ in its own weight block) on the GPU, against the numpy restatement of the reference's
combine (oracle.consensus_combine_ref = stark/stark.py:7-21, 66-70) on one host process.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stark_amd import engine  # noqa: E402


def main():
    shards, P, S, reps = 8, 102, 1600, 20
    rng = np.random.default_rng(0)
    draws = []
    for s in range(shards):
        A = rng.normal(size=(P, P)) / np.sqrt(P)
        draws.append(rng.normal(size=(P, 1)) + (A + np.eye(P)) @ rng.normal(size=(P, S)))
    ctx = engine.Context(0)
    out = {}
    for name, kw in (("joint", {}), ("separate_lp", {"separate_lp": True})):
        engine.consensus(draws, ctx, **kw)
        t = time.perf_counter()
        for _ in range(reps):
            engine.consensus(draws, ctx, **kw)
        out[f"gpu_ms_{name}"] = 1e3 * (time.perf_counter() - t) / reps
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    t = time.perf_counter()
    for _ in range(3):
        O.consensus_combine_ref(draws)
    out["numpy_ms_joint"] = 1e3 * (time.perf_counter() - t) / 3
    out.update(shards=shards, P=P, S=S, note="host-buffer API: includes the 10.4 MB host->device copy of the draws "
                                             "and the result copy back")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
