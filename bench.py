#!/usr/bin/env python3
"""Headline benchmark: gradient evals/s + ESS/s, Bayesian logistic regression N=1e8, d=100,
fp64, 8 subposterior shards + consensus combine (BASELINE.json configs[3], the config the
metric is quoted on; 80 GB of X fits one MI355X, so N=1 runs all 8 shards on one GPU and
N GPUs run 8/N shards each -- total work fixed, "scaling": "strong").

A "step" = one pass of the hot path over the data: ONE fused log-density+gradient sweep of
every local shard, i.e. one leapfrog of every chain (chains share a shard's sweep), followed
by the deterministic chunk reduction and one NUTS state-machine step.  Chains are never held
back by each other: each runs its own trajectories, transitions and draws.  Timeline:
  data generated in HBM (Philox, not timed) -> Stan warmup with adaptation, --adapt-iters
  transitions per chain (not timed) -> W untimed steps -> barrier+sync -> K timed steps ->
  sync+barrier.
`value` = chain-gradient evaluations of all ranks in the timed region / max-over-ranks time
(every chain evaluates one gradient per step, so = chains * K / time).
ESS/s: the transitions every chain completed inside the timed window, rank-paired across
shards (combined chain k = the chain with the k-th most window transitions of each shard,
cut to the fewest of them, so draw i of every shard is combined with draw i of the others);
the consensus combine runs on the GPU after one all-gather; ESS/s = min over non-lp__
parameters of the combined draws' ESS (sum over combined chains of Stan's single-chain
estimator) / the timed window.  ess_per_sec_equal_length: Stan's multi-chain estimator on
every chain cut to the shortest (conservative).

Usage: python bench.py [--gpus N --steps K --warmup W]; N>1 under torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6    # MI355X fp64 matrix (= vector) spec, dense
FP64_MEASURED_TFS = 46.0  # v_mfma_f64_16x16x4 back to back, 2+ waves/SIMD (tools/mfma_overlap.hip, profiles/)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--family", choices=["logistic", "linear"], default="logistic",
                   help="linear --rows 1e7 --d 50: BASELINE configs[2]")
    p.add_argument("--rows", type=float, default=1e8, help="total rows N over all shards")
    p.add_argument("--d", type=int, default=100)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--chains", type=int, default=16,
                   help="chains per shard; they share one data sweep (16: the fp64 MFMA sweep, X.[beta_1..beta_16])")
    p.add_argument("--adapt-iters", type=int, default=150,
                   help="Stan warmup iterations (>= 150: a metric window after the initial transient)")
    p.add_argument("--stepsize-jitter", type=float, default=0.5,
                   help="Stan control stepsize_jitter; breaks the trajectory-length resonance of NUTS on "
                        "this near-isotropic posterior (DESIGN.md section 4)")
    p.add_argument("--seed", type=int, default=20240)
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "sweep_pmc.json"))
    return p.parse_args()


def cpu_baseline(d, rows_per_shard, shards, seconds, family="logistic"):
    """The oracle's logistic gradient (oracle/stark_oracle.c, gcc -O2, scalar) run as the
    reference's execution model: one single-chain worker per shard, min(shards, cores)
    concurrent (Spark local[*]).  Each worker times full gradient evaluations over a bounded
    row sample and scales linearly to the shard (gradient cost is linear in rows)."""
    import multiprocessing as mp
    cores = len(os.sched_getaffinity(0))
    workers = max(1, min(shards, cores))
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        rates = pool.starmap(_cpu_worker, [(d, seconds, w, family) for w in range(workers)])
    sample_rows = rates[0][1]
    per_worker_grads = [r[0] * sample_rows / rows_per_shard for r in rates]   # full-shard grads/s
    return {"value": float(sum(per_worker_grads)), "unit": "gradient evals/sec (whole node)",
            "cores": workers, "kind": "port",
            "sample": f"oracle {'orc_logreg_lpgrad' if family == 'logistic' else 'orc_linreg_lpgrad'} "
                      f"(C, 1 thread/worker) on {sample_rows} rows x d={d} per worker, "
                      f"{seconds:.0f}s per worker, {workers} concurrent workers (one per shard, Spark local[*] model), "
                      f"scaled linearly to {rows_per_shard:.3g} rows/shard; analytic gradient (optimistic vs Stan autodiff)"}


def _cpu_worker(d, seconds, w, family="logistic"):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    rows = 100_000
    X = O.gen_x(99, w * rows, rows, d)
    beta = O.gen_beta(99, d)
    if family == "logistic":
        y, _ = O.gen_y_logistic(99, w * rows, X, 0.0, beta)
        m = O.Model(O.FAM_LOGREG, X=X, y=y)
        q = np.concatenate([[0.0], beta * 0.9])
    else:
        y = O.gen_y_linear(99, w * rows, X, 0.0, beta)
        y = y[0] if isinstance(y, tuple) else y
        m = O.Model(O.FAM_LINREG, X=X, y=y)
        q = np.concatenate([[0.0], beta * 0.9, [0.0]])
    m.lpgrad(q)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        m.lpgrad(q)
        n += 1
    return n / (time.perf_counter() - t0), rows


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # STARK_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N-rank path on one
    # GPU (ranks share devices round-robin); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("STARK_DIST_BACKEND", "nccl")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        local_rank %= torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    from stark_amd import diagnostics, engine

    assert a.shards % world == 0, "shards must divide evenly over GPUs"
    spr = a.shards // world
    rows_per_shard = int(a.rows) // a.shards
    first = rank * spr
    shard_ids = list(range(first, first + spr))
    ctx = engine.Context(local_rank)

    t = time.perf_counter()
    model = engine.Model.synthetic(ctx, a.family, spr, rows_per_shard, a.d, data_seed=a.seed,
                                   row_offset=first * rows_per_shard)
    ctx.sync()
    t_gen = time.perf_counter() - t

    A, W, K = a.adapt_iters, a.warmup, a.steps
    total = A + W + K + 1          # enough sampling iterations that no chain finishes in the window
    sampler = model.sampler(num_warmup=A, num_samples=total - A, chains=a.chains, seed=a.seed + 1,
                            shard_ids=shard_ids, stepsize_jitter=a.stepsize_jitter)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    log(f"data generated: {spr} shards x {rows_per_shard} rows x d={a.d} in {t_gen:.1f}s "
        f"({model.device_bytes() / 1e9:.1f} GB on this GPU)")
    t = time.perf_counter()
    # One run to the end of warmup, in bounded step batches for progress lines: chains move
    # independently and only wait for each other once, at iteration A.
    while True:
        sampler.run(A, max_steps=1000)
        its = sampler.iterations()
        inf = sampler.info()
        log(f"adaptation: {time.perf_counter() - t:.1f}s, transitions per chain min/median "
            f"{its.min()}/{int(np.median(its))} of {A}, leapfrogs/chain {inf['leapfrogs'] / max(1, spr * a.chains):.0f}")
        if its.min() >= A:
            break
    t_adapt = time.perf_counter() - t
    t = time.perf_counter()
    sampler.run(total, max_steps=W)
    ctx.sync()
    t_wsteps = time.perf_counter() - t
    log(f"warmup steps done; timing {K} steps")

    def barrier():
        torch.cuda.synchronize(local_rank)
        if dist:
            dist.barrier()

    nchains = spr * a.chains
    it0 = sampler.iterations()
    ctx.set_profiling(True)
    i0 = sampler.info()
    barrier()
    t0 = time.perf_counter()
    sampler.run(total, max_steps=K)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    i1 = sampler.info()
    it1 = sampler.iterations()

    grads = i1["grad_evals"] - i0["grad_evals"]
    leaps = i1["leapfrogs"] - i0["leapfrogs"]
    sweeps = i1["sweeps"] - i0["sweeps"]
    shard_sweeps = i1["shard_sweeps"] - i0["shard_sweeps"]
    sweep_ms = i1["sweep_ms"] - i0["sweep_ms"]
    done_in_window = it1 - it0                       # transitions completed per chain
    eps, _ = sampler.adaptation()
    if dist:
        v = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", local_rank))
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        elapsed = float(v.item())
        g = torch.tensor([grads, leaps], dtype=torch.float64, device=torch.device("cuda", local_rank))
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        grads, leaps = int(g[0].item()), int(g[1].item())

    # ---- draws completed inside the window -> consensus -> ESS.
    # The consensus average pairs draw i of every shard; chains are exchangeable, so combined
    # chain k joins the chain with the k-th most window transitions of every shard and keeps
    # M_k = the fewest of those (no draw is made up, chain boundaries align across shards).
    C = a.chains
    P = model.P[0]
    counts = {shard_ids[s]: done_in_window[s * C:(s + 1) * C].astype(int).tolist() for s in range(spr)}
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, counts)
        counts = {k_: v_ for dct in gathered for k_, v_ in dct.items()}
    order = {sh: np.argsort(-np.asarray(cnt), kind="stable") for sh, cnt in counts.items()}
    Mk = np.array([min(counts[sh][order[sh][k]] for sh in counts) for k in range(C)])
    local = {}
    per = total - A
    for s in range(spr):
        dr, _ = sampler.draws(s)
        sh = shard_ids[s]
        cols = []
        for k in range(C):
            c = order[sh][k]
            first = it0[s * C + c] - A               # sampling index of the chain's first window transition
            cols.append(np.arange(c * per + first, c * per + first + Mk[k]))
        local[sh] = np.ascontiguousarray(dr[:, np.concatenate(cols)]) if Mk.sum() > 0 else None
    if dist:
        allp = [None] * a.shards
        gathered = [None] * world
        dist.all_gather_object(gathered, local)
        for dct in gathered:
            for k_, v_ in dct.items():
                allp[k_] = v_
    else:
        allp = [local[k_] for k_ in range(a.shards)]

    def ess_rows(x, equal):
        """min over parameter rows of the ESS of x (P' x sum(Mk), chain segments of lengths Mk):
        equal: Stan's multi-chain estimator on every segment cut to min(Mk);
        else: sum over segments (M_k >= 4) of Stan's single-chain estimator (independent chains)."""
        off = np.concatenate([[0], np.cumsum(Mk)])
        out = []
        for p in range(x.shape[0]):
            if equal:
                m = int(Mk.min())
                out.append(diagnostics.ess(np.stack([x[p, off[k]:off[k] + m] for k in range(C)])))
            else:
                out.append(sum(diagnostics.ess(x[p, off[k]:off[k + 1]]) for k in range(C) if Mk[k] >= 4))
        return float(np.nanmin(out))

    ess_ps, min_ess, ess_eq, sub_ess, truth_check = None, None, None, None, None
    if rank == 0 and Mk.sum() > P + 1 and Mk.max() >= 4:
        sub_ess = ess_rows(allp[0][:-1], False)
        comb, used = engine.consensus(allp, ctx, separate_lp=True)
        comb_joint, _ = engine.consensus(allp, ctx)                # the reference's joint weights (lp__ in)
        min_ess = ess_rows(comb[:-1], False)                     # drop lp__
        ess_eq = ess_rows(comb[:-1], True) if Mk.min() >= 4 else None
        ess_ps = min_ess / elapsed
        # large-scale sanity of the combined posterior: the generating (alpha = 0, beta) lies
        # within a few posterior sd of the consensus mean (z ~ N(0, 1) per parameter)
        truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
        if a.family == "linear":
            truth = np.concatenate([truth, [1.0]])             # sigma
        z = (comb[:-1].mean(axis=1) - truth) / comb[:-1].std(axis=1)
        zs = (allp[0][:-1].mean(axis=1) - truth) / allp[0][:-1].std(axis=1)
        zj = (comb_joint[:-1].mean(axis=1) - truth) / comb_joint[:-1].std(axis=1)
        truth_check = {"max_abs_z": float(np.abs(z).max()), "mean_z2": float((z ** 2).mean()),
                       "subposterior_shard0_mean_z2": float((zs ** 2).mean()), "params": int(z.size),
                       "joint_lp_weights_mean_z2": float((zj ** 2).mean()),
                       "note": "consensus with lp__ in its own weight block (engine.consensus separate_lp); "
                               "joint_lp_weights_mean_z2 = the reference's joint combine (lp__ inside inv(cov), "
                               "stark/stark.py:49-56), where each shard's lp__ offset leaks into the parameters "
                               "through the sampled cross-covariances (DESIGN.md section 8)"}
    info = sampler.info()
    sampler.close()

    if rank != 0:
        model.close()
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (the data sweep)
    # C = 16: k_sweepm, X.[beta_1..beta_16] on fp64 MFMA, bound by the fp64 pipe;
    # C <= 4: k_sweep3 (VALU), bound by HBM.
    mfma = a.chains == 16
    kname = ("k_sweepe" if a.d == 100 else "k_sweepm") if mfma else "k_sweep3"
    ybytes = 4 if a.family == "logistic" else 8
    fam = "LOGREG" if a.family == "logistic" else "LINREG"
    bytes_per_shard = rows_per_shard * (8 * a.d + ybytes)   # X fp64 + y (int32 / fp64), once per sweep
    avg_ms = sweep_ms / max(sweeps, 1)
    shards_per_launch = shard_sweeps / max(sweeps, 1)
    bytes_per_launch = bytes_per_shard * shards_per_launch
    flops_per_launch = 4.0 * rows_per_shard * a.d * a.chains * shards_per_launch   # fwd + bwd GEMMs
    gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if sweeps else None
    tfs = flops_per_launch / (avg_ms * 1e-3) / 1e12 if sweeps else None
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if (tj.get("kernel") == kname and tj.get("rows_per_shard") == rows_per_shard and tj.get("d") == a.d
                    and tj.get("hbm_bytes_per_shard_sweep")):
                # PMC pass of the same shard geometry (tools/pmc_traffic.py): FETCH_SIZE x2 per
                # shard sweep, times the shards a launch swept on average
                traffic = tj["hbm_bytes_per_shard_sweep"] * shards_per_launch
        except Exception:
            traffic = None
    hbm = {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": (gbs / HBM_PEAK_GBS) if gbs else None}
    if mfma:
        roof = {"bound": "mfma", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                "frac": (tfs / FP64_PEAK_TFS) if tfs else None, "traffic": traffic,
                "kernel": f"{kname}<{fam}> (fp64 MFMA 16x16x4, {a.chains} chains)", "avg_launch_ms": avg_ms,
                "algorithmic_flops_per_launch": flops_per_launch, "algorithmic_bytes_per_launch": bytes_per_launch,
                "hbm": hbm, "fp64_measured_ceiling_tfs": FP64_MEASURED_TFS}
    else:
        roof = dict(bound="hbm", **{k: v for k, v in hbm.items()}, traffic=traffic,
                    kernel=f"k_sweep3<{fam},{a.chains}>", avg_launch_ms=avg_ms,
                    algorithmic_bytes_per_launch=bytes_per_launch)
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(a.d, rows_per_shard, a.shards, a.cpu_baseline_seconds, a.family)

    value = grads / elapsed
    line = {
        "metric": f"gradient evals/sec (whole node), {a.family} regression N={a.rows:.0e} d={a.d}".replace("e+0", "e"),
        "value": value,
        "unit": "gradient evals/sec",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": 1e3 * elapsed / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Philox in HBM, SURVEY 8d)",
        "config": {"workload": f"bayesian {a.family} regression, {a.shards} subposterior shards + consensus combine",
                   "rows": int(a.rows), "d": a.d, "shards": a.shards, "shards_per_gpu": spr,
                   "chains_per_shard": a.chains, "adapt_iters": A, "stepsize_jitter": a.stepsize_jitter,
                   "parallelism": f"shard-dp{world}"},
        "ess_per_sec": ess_ps,
        "min_ess": min_ess,
        "ess_method": "min over parameters (lp__ excluded) of the consensus draws completed in the timed window; "
                      "sum over rank-paired chains of Stan's single-chain ESS",
        "ess_per_sec_equal_length": (ess_eq / elapsed) if ess_eq else None,
        "ess_per_sec_incl_warmup": (min_ess / (t_adapt + t_wsteps + elapsed)) if min_ess else None,
        "subposterior_min_ess_shard0": sub_ess,
        "consensus_vs_generating_params": truth_check,
        "transitions_per_chain_in_window": {"min": int(done_in_window.min()), "median": float(np.median(done_in_window)),
                                            "max": int(done_in_window.max()), "used_for_ess": int(Mk.sum()),
                                            "used_equal_length": int(C * Mk.min())},
        "stepsize_per_chain": {"min": float(eps.min()), "median": float(np.median(eps)), "max": float(eps.max())},
        "leapfrogs_per_transition": float(nchains * K / max(1, done_in_window.sum())),
        "rows_x_chains_per_sec": grads * rows_per_shard / elapsed,
        "roofline": roof,
        "cpu_baseline": cpu,
        "setup_s": {"datagen": t_gen, "adaptation": t_adapt},
        "divergent": info["divergent"],
    }
    print(json.dumps(line), flush=True)
    model.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
