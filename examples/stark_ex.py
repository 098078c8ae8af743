#!/usr/bin/env python3
"""The reference's example driver (example/stark_ex.py:14-30) on stark_amd.

Same program, same calls: 8 schools split into 2 partitions, one weighted (consensus) run
with iter=5000 and one naive run with n=4 (BASELINE.json configs[0]).  What
differs is only the plumbing: the Spark context becomes ``stark_amd.rdd.LocalContext`` (a
real SparkContext works too: only ``getNumPartitions()`` and ``glom().collect()`` are used
on its RDD) and each partition samples on the GPU instead of in a pystan executor.

    python examples/stark_ex.py [--seed S]            # one MI355X
    torchrun --nproc-per-node N examples/stark_ex.py  # partitions over N GPUs (RCCL)
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stark_amd import *  # noqa: E402,F401,F403  -- binds `stark`, as `from stark import *` does
from stark_amd.rdd import LocalContext  # noqa: E402

SCHOOL_DATA = list(zip(
    [28, 8, -3, 7, -1, 1, 18, 12],   # y
    [15, 10, 16, 11, 9, 11, 10, 18]))  # sigma


def prepare_school_data(data):
    return {'J': len(data),
            'y': [d[0] for d in data],
            'sigma': [d[1] for d in data]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=None, help="sampling seed (the reference sets none)")
    a = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        dist.init_process_group("nccl", device_id=torch.device("cuda", lr))
    kw = {} if a.seed is None else {"seed": a.seed}
    stanFile = os.path.join(ROOT, "stark_amd", "models", "schools.stan")
    sc = LocalContext()
    school_rdd = sc.parallelize(SCHOOL_DATA, 2)
    st = stark.Stark(sc, school_rdd, prepare_school_data)  # noqa: F405
    st.setStanModel(file=stanFile)

    ## 2 ways to distribute:
    ## + combine each subposterior, weighting according to (co)variances:
    weighted_avg = st.concensusWeight(iter=5000, **kw)
    ## + naive parallel, like running n*chains:
    dist_draws = st.distribute(n=4, **kw)
    if int(os.environ.get("RANK", "0")) == 0:
        np.set_printoptions(precision=3, threshold=40)
        print("Weighted average posterior samples:")
        print(weighted_avg)
        print("Posteriors drawn from parallel workers:")
        print(dist_draws)


if __name__ == "__main__":
    main()
