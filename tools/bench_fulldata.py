#!/usr/bin/env python3
"""Full-data HMC/NUTS throughput, BASELINE.json configs[4]: Bayesian logistic regression, d = 1000,
64 chains, fp64, rows split over the GPUs of one node with a per-leapfrog gradient all-reduce
(stark_amd/fulldata.py).

N = 1e9 x d = 1000 fp64 is 8 TB of X and does not fit a node's 8 x 288 GB of HBM, so this run
keeps --rows-per-gpu rows resident per GPU (default 2.5e7 = 200 GB; weak scaling: N = rows x
GPUs) -- DESIGN.md section 5.  A step = one leapfrog of all 64 chains = one full-data gradient
per chain: the two fp64-MFMA GEMM passes over the local rows (k_gemm_fwd / k_gemm_bwd), the
chunk reduction, the all-reduce of the [64 x (Dp+1)] block over RCCL, and one NUTS
state-machine step.  Timed: K steps after W untimed ones, from the start of sampling (a step
costs the same whatever the sampler phase, and a config-4 chain needs far more than a bench
window of full-data gradients to adapt, so ESS/s is not reported for this config).

Usage: python tools/bench_fulldata.py [--gpus N --rows-per-gpu R --steps K --warmup W]: --gpus N > 1
starts N rank processes itself with bench.py's launcher (one per GPU, before any GPU call).
bench.py runs `run()` on every rank of its own N-rank job (its configs4_fulldata sub-record).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FP64_PEAK_TFS = 78.6
HBM_PEAK_GBS = 8000.0


def run(rows, d=1000, chains=64, steps=30, warmup=3, seed=20240, init_radius=2.0, nuts_criterion="stan2.19",
        adapt_iters=0):
    """One configs[4] measurement on this process's GPU (RANK / WORLD_SIZE / LOCAL_RANK from the
    environment; the process group, if any, already initialised); returns the line (rank 0) or None."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    import torch
    import torch.distributed as dist
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    from stark_amd import engine, fulldata

    rows = int(rows)
    ctx = fulldata.context_on_torch_stream(local_rank)
    t = time.perf_counter()
    model = engine.Model.synthetic(ctx, "logistic", 1, rows, d, data_seed=seed, row_offset=rank * rows)
    ctx.sync()
    t_gen = time.perf_counter() - t
    K, W = steps, warmup
    A = adapt_iters
    nw = A if A > 0 else 1000
    total = nw + K + W + 1
    # save_warmup: the chain positions of every transition, the fingerprint compared across ranks
    fs = fulldata.FullDataSampler(model, num_warmup=nw, num_samples=total - nw, chains=chains, seed=seed + 1,
                                  stepsize_jitter=0.5 if A > 0 else 0.0, init_radius=init_radius,
                                  nuts_criterion=nuts_criterion, save_warmup=True)
    if rank == 0:
        print(f"[bench_fulldata] {world} GPU(s) x {rows} rows x d={d}: {model.device_bytes() / 1e9:.1f} GB/GPU, "
              f"generated in {t_gen:.1f}s", file=sys.stderr, flush=True)
    t_adapt = 0.0
    if A > 0:
        t = time.perf_counter()
        while True:                                   # bounded batches: a progress line per batch
            fs.run(A, max_steps=500)
            its = fs.iterations()
            if rank == 0:
                print(f"[bench_fulldata] warmup: {time.perf_counter() - t:.1f}s, transitions min/median "
                      f"{its.min()}/{int(np.median(its))} of {A}", file=sys.stderr, flush=True)
            if its.min() >= A:
                break
        t_adapt = time.perf_counter() - t
    fs.run(total, max_steps=W)

    def barrier():
        torch.cuda.synchronize(local_rank)
        if world > 1:
            dist.barrier()

    ctx.set_profiling(True)
    i0 = fs.info()
    it0 = fs.iterations()
    barrier()
    t0 = time.perf_counter()
    fs.run(total, max_steps=K)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    i1 = fs.info()
    it1 = fs.iterations()
    ess_ps, min_ess = None, None
    if A > 0 and rank == 0:
        # window transitions of every chain (ragged), ESS = min over parameters (lp__ excluded)
        # of the sum over chains of Stan's single-chain estimator
        from stark_amd import diagnostics
        dr, _ = fs.draws(0)
        per = total - nw
        done = it1 - it0
        es = np.zeros(dr.shape[0] - 1)
        for c in range(chains):
            f0 = it0[c] - nw
            if done[c] >= 4:
                seg = dr[:-1, c * per + f0: c * per + f0 + done[c]]
                es += np.array([diagnostics.ess(seg[j]) for j in range(seg.shape[0])])
        min_ess = float(np.nanmin(es)) if es.any() else None
    # every rank runs the same chains on the all-reduced gradients: their positions (warmup
    # included), step sizes and iteration counts must agree bit for bit on every rank
    import hashlib
    eps, im = fs.adaptation()
    h = hashlib.sha256()
    for arr in (fs.unconstrained(0), eps, im, it1):
        h.update(np.ascontiguousarray(arr).tobytes())
    fp = np.zeros(world)
    fp[rank] = int(h.hexdigest()[:12], 16)              # 48 bits: exact in fp64
    if world > 1:
        v = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local_rank))
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        elapsed = float(v.item())
        f = torch.from_numpy(fp).to(torch.device("cuda", local_rank))
        dist.all_reduce(f)
        fp = f.cpu().numpy()
    if min_ess:
        ess_ps = min_ess / elapsed
    nsteps = i1["steps"] - i0["steps"]
    grads = i1["grad_evals"] - i0["grad_evals"]      # chain-gradients of the full data set (same on every rank)
    sweeps = i1["sweeps"] - i0["sweeps"]
    avg_ms = (i1["sweep_ms"] - i0["sweep_ms"]) / max(sweeps, 1)   # qT image + pass F + pass B, this rank
    flops = 4.0 * d * chains * rows                    # two GEMMs over this rank's rows
    tfs = flops / (avg_ms * 1e-3) / 1e12
    hbm_bytes = rows * (2 * 8 * d + 4 + 2 * 8 * chains)   # X twice, y, R written + read once
    gbs = hbm_bytes / (avg_ms * 1e-3) / 1e9
    line = {
        "metric": "gradient evals/sec (whole node), full-data logistic regression d=1000, 64 chains",
        "value": grads / elapsed, "unit": "gradient evals/sec", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": 1e3 * elapsed / max(nsteps, 1), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (Philox in HBM, SURVEY 8d)",
        "config": {"workload": "full-data HMC/NUTS logistic regression, per-leapfrog gradient all-reduce",
                   "rows_total": rows * world, "rows_per_gpu": rows, "d": d, "chains": chains,
                   "parallelism": f"row-dp{world}", "nuts_criterion": nuts_criterion,
                   "note": "N=1e9 (8 TB) exceeds node HBM; rows per GPU resident"},
        "rows_x_chains_per_sec": grads * rows * world / elapsed,
        "ess_per_sec": ess_ps, "min_ess": min_ess, "adapt_iters": A,
        "transitions_in_window": ({"min": int((it1 - it0).min()), "median": float(np.median(it1 - it0))}
                                  if A > 0 else None),
        "roofline": {"bound": "mfma", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": tfs / FP64_PEAK_TFS, "traffic": None, "peak_measured": 78.0,
                     "frac_of_measured": tfs / 78.0,
                     "kernel": "k_gemm_fwd + k_gemm_bwd (fp64 MFMA 16x16x4, 64 chains)", "avg_launch_ms": avg_ms,
                     "algorithmic_flops_per_launch": flops,
                     "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                             "algorithmic_bytes_per_launch": hbm_bytes}},
        "setup_s": {"datagen": t_gen, "adaptation": t_adapt},
        "chains_sha16_per_rank": [f"{int(v):012x}" for v in fp],
    }
    fs.close()
    model.close()
    return line if rank == 0 else None


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); > 1 without a launcher: spawned here")
    p.add_argument("--rows-per-gpu", type=float, default=2.5e7)
    p.add_argument("--d", type=int, default=1000)
    p.add_argument("--chains", type=int, default=64)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--seed", type=int, default=20240)
    p.add_argument("--init-radius", type=float, default=2.0, help="pystan init_r (Stan default 2)")
    p.add_argument("--nuts-criterion", choices=["stan2.19", "stan2.23"], default="stan2.19")
    p.add_argument("--adapt-iters", type=int, default=0,
                   help="> 0: run Stan's warmup (untimed) first and report ESS/s of the transitions the "
                        "chains complete inside the timed window")
    a = p.parse_args()
    import bench
    refuse = bench.check_world(a.gpus, os.environ)
    if refuse:
        sys.exit(refuse)
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(bench.launch_ranks(a.gpus, sys.argv[1:], script=__file__))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # STARK_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N-rank path on one
    # GPU (ranks share devices round-robin); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("STARK_DIST_BACKEND", "nccl")
    import torch
    import torch.distributed as dist
    refuse = bench.check_devices(backend, os.environ, torch.cuda.device_count())
    if refuse:
        sys.exit(refuse)
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    line = run(a.rows_per_gpu, a.d, a.chains, a.steps, a.warmup, a.seed, a.init_radius, a.nuts_criterion,
               a.adapt_iters)
    if line is not None:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
