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
  transitions per chain -> W untimed steps -> barrier+sync -> K timed steps -> sync+barrier
  -> ESS phase: every chain runs on to the same number of post-warmup draws (--ess-draws)
  -> one all-gather of the draws -> consensus combine on the GPU -> ESS.
`value` = chain-gradient evaluations of all ranks in the timed region / max-over-ranks time
(every chain evaluates one gradient per step, so = chains * K / time).
`ess_per_sec` = min over alpha, beta of Stan 2.19's multi-chain ESS of the
consensus draws / the whole sampling wall time, adaptation included (data upload excluded).
`accuracy` compares the consensus with the full-data posterior (MAP + inverse Hessian from
the GPU gradient, tools/laplace.py) and with the data-generating parameters.

Usage: python bench.py [--gpus N --steps K --warmup W].  --gpus N > 1 without a launcher starts N
rank processes itself (one per GPU, RCCL) before any GPU call; under a
launcher (WORLD_SIZE set) --gpus must equal the world size or the run is refused.
"""
import argparse
import datetime
import hashlib
import json
import socket
import subprocess
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6    # MI355X fp64 matrix (= vector) spec, dense
FP64_MFMA_MEASURED_TFS = 78.0   # v_mfma_f64_16x16x4 back to back (64 cycles per SIMD), clock-stamped at 2.38 GHz,
                                # built with -mllvm -amdgpu-mfma-vgpr-form (tools/mfma_ceiling.hip,
                                # profiles/r02zd_mfma_ceiling_vgprform.log): the instruction the sweep issues
FP64_MFMA4_MEASURED_TFS = 75.8  # v_mfma_f64_4x4x4_4b back to back (profiles/r02zd_mfma_ceiling_vgprform.log)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks (one process per GPU).  Without a launcher, N > 1 starts N rank processes "
                        "itself; under one (torch.distributed.run), must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks, build the process group, report world size / backend / rank devices and "
                        "exit: the launcher path without sampling (CPU: STARK_DIST_BACKEND=gloo)")
    p.add_argument("--throughput-only", action="store_true",
                   help="time the K steps (sampler still in adaptation) and print the line: no ESS phase, accuracy, "
                        "second run, CPU baseline or sub-records (the chains=1 sub-record uses it)")
    p.add_argument("--deadline-s", type=float, default=500.0,
                   help="wall-time budget of the whole run: an optional phase (second criterion, sub-records) whose "
                        "expected cost would cross it is skipped and the line says so")
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--family", choices=["logistic", "linear"], default="logistic",
                   help="linear --rows 1e7 --d 50: BASELINE configs[2]")
    p.add_argument("--rows", type=float, default=1e8, help="total rows N over all shards")
    p.add_argument("--d", type=int, default=100)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--chains", type=int, default=16,
                   help="chains per shard; they share one data sweep (16: the fp64 MFMA sweep, X.[beta_1..beta_16])")
    p.add_argument("--adapt-iters", type=int, default=None,
                   help="Stan warmup iterations; default 150 for logistic (the driver's lease) and Stan's 1000 for "
                        "linear (150 leaves one 50-draw metric window inside the initial transient: DESIGN.md 4)")
    p.add_argument("--stepsize-jitter", type=float, default=0.5,
                   help="Stan control stepsize_jitter; breaks the trajectory-length resonance of NUTS on "
                        "this near-isotropic posterior (DESIGN.md section 4)")
    p.add_argument("--ess-draws", type=int, default=250,
                   help="post-warmup draws per chain for the ESS / accuracy phase (after the timed steps); "
                        "ESS/s counts the warmup too, so it rises with the draws per warmup iteration "
                        "(Stan's defaults: 1000 and 1000)")
    p.add_argument("--no-accuracy", action="store_true", help="skip the full-data Laplace reference")
    p.add_argument("--nuts-criterion", choices=["stan2.19", "stan2.23"], default="stan2.23",
                   help="stan2.23 (default): Stan's NUTS with the U-turn checks across subtree junctions "
                        "(Stan >= 2.23); stan2.19: the reference's pystan 2 NUTS, whose single test lets "
                        "trajectories resonate on this near-isotropic posterior (36 vs 11 leapfrogs per "
                        "transition, DESIGN.md section 4)")
    p.add_argument("--second-criterion", choices=["stan2.23", "stan2.19", "none"], default="none",
                   help="after the main run: a second adaptation + ESS phase on the same data with this "
                        "NUTS criterion (stan2.19: the reference's pystan 2 sampler, Stan 2.19.1), reported as "
                        "ess_second_criterion.  Off by default since round 5: the reference sampler's own settings "
                        "run in the configs2_linear sub-record (other_configs), where they fit the lease")
    p.add_argument("--second-jitter", type=float, default=0.5,
                   help="stepsize_jitter of the second run.  pystan 2's default is 0, under which the 2.19 "
                        "criterion's trajectories resonate on this near-isotropic posterior (profiles/r03i_bench.json: "
                        "164 of 250 iterations in 305 s, no ESS); 0.5 keeps the reference's criterion inside the "
                        "driver's lease")
    p.add_argument("--second-draws", type=int, default=100, help="post-warmup draws per chain of the second run")
    p.add_argument("--second-budget-s", type=float, default=330.0,
                   help="wall-time bound of the second run (warmup + draws); past it the run stops and the line "
                        "says so instead of an ESS")
    p.add_argument("--seed", type=int, default=20240)
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-schools", action="store_true",
                   help="skip the configs[1] sub-record (8-schools x 4096 chains, Stan defaults; ~2 s)")
    p.add_argument("--no-other-configs", action="store_true",
                   help="skip the configs[2] / configs[4] throughput sub-records (one GPU only; ~30 s)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "sweep_pmc.json"))
    p.add_argument("--shard-offset", type=int, default=0,
                   help="global id of this job's first shard: with --shards 1 --rows 1.25e7 and offset k, one rank "
                        "of the 8-shard job (shard k's rows and RNG keys) on this GPU (tools/consensus_from_dumps.py)")
    p.add_argument("--ess-budget-s", type=float, default=None,
                   help="(one process only) stop the post-warmup phase after this many seconds and keep the draws "
                        "every chain has by then (the line's post_warmup_draws_per_chain says how many)")
    p.add_argument("--dump-draws", default=None,
                   help="write this process's post-warmup draws per shard (npz: P x chains*draws, chain-major) and "
                        "the phase times to this path")
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
    pool = ctx.Pool(workers)
    try:
        rates = pool.starmap(_cpu_worker, [(d, seconds, w, family) for w in range(workers)])
        # close + join: the workers exit on their own (Pool.__exit__ would terminate() them, i.e.
        # SIGTERM processes that may run under a profiler's signal handler)
        pool.close()
        pool.join()
    except BaseException:
        pool.terminate()
        raise
    sample_rows = rates[0][1]
    per_worker_grads = [r[0] * sample_rows / rows_per_shard for r in rates]   # full-shard grads/s
    return {"value": float(sum(per_worker_grads)), "unit": "gradient evals/sec (whole node)",
            "cores": workers, "kind": "port",
            "sample": f"oracle {'orc_logreg_lpgrad' if family == 'logistic' else 'orc_linreg_lpgrad'} "
                      f"(C, 1 thread/worker) on {sample_rows} rows x d={d} per worker, "
                      f"{seconds:.0f}s per worker, {workers} concurrent workers (one per shard, Spark local[*] model), "
                      f"scaled linearly to {rows_per_shard:.3g} rows/shard; analytic gradient (optimistic vs Stan autodiff)"}


def cpu_combine(draws):
    """The reference's combine arithmetic on the host (oracle.consensus_combine_ref: numpy
    inv(np.cov) per shard, sums, inv(sum W) . sum W theta -- stark/stark.py:7-21, 66-70, the
    reference's own operations), timed on the same draws as the GPU combine."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    d = [np.asarray(x[:-1]) for x in draws]
    t = time.perf_counter()
    O.consensus_combine_ref(d)
    O.consensus_combine_ref([np.asarray(x[-1:]) for x in draws])
    return {"combine_ms": 1e3 * (time.perf_counter() - t),
            "combine_note": "numpy restatement of the reference combine (lp__ in its own block), 1 process"}


SCHOOLS_Y = [28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0]        # example/stark_ex.py:5
SCHOOLS_SIGMA = [15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0]  # example/stark_ex.py:6


def cpu_baseline_schools(seconds):
    """The reference's CPU path for 8 schools, timed the way example/stark_ex.py:24-26 runs it:
    pystan's single-chain NUTS (here the oracle's recursive Stan 2.19.1 twin, C) in one process
    per run, min(runs, cores) concurrent (Spark local[*]).
      weighted  concensusWeight(iter=5000): 2 runs of 2500 warmup + 2500 draws, one per
                four-school partition (stark/stark.py:59-64);
      naive     distribute(n=4): 4 full-data (J = 8) runs at iter=2000, 1000 + 1000 (the intent
                of stark/stark.py:74-85) -- the job the configs[1] GPU record scales
                to 4,096 chains.
    Each job repeats with fresh seeds for about `seconds`; gradient evals/s and ESS/s (Stan 2.19
    multi-chain ESS over the job's chains, min over mu, tau, eta, theta) per job wall time."""
    import multiprocessing as mp
    cores = len(os.sched_getaffinity(0))
    ctx = mp.get_context("spawn")
    out = {"unit": "gradient evals/sec (whole job)", "kind": "port",
           "sample": (f"oracle orc_run_chain (recursive Stan 2.19.1 NUTS twin, C, 1 thread per run), jobs repeated "
                      f"with fresh seeds for ~{seconds:.0f} s each; a job's wall time = its slowest run")}
    for job, runs, J, it in (("naive_n4", 4, 8, 2000), ("weighted_iter5000", 2, 4, 5000)):
        workers = max(1, min(runs, cores))
        pool = ctx.Pool(workers)
        try:
            res = pool.starmap(_schools_worker, [(w, J, it, seconds / 2, w >= workers // 2 and J == 4)
                                                 for w in range(workers)])
            pool.close()
            pool.join()
        except BaseException:
            pool.terminate()
            raise
        reps = min(len(r) for r in res)
        walls = [max(r[k][1] for r in res) for k in range(reps)]
        grads = [sum(r[k][0] for r in res) for k in range(reps)]
        rec = {"runs_per_job": runs, "cores": workers, "J": J, "iter": it, "jobs_timed": reps,
               "job_wall_ms_median": 1e3 * float(np.median(walls)),
               "value": float(sum(grads) / sum(walls))}
        if job == "naive_n4":
            from stark_amd import diagnostics
            ess = [float(np.nanmin(diagnostics.ess_matrix(np.hstack([r[k][2] for r in res]), workers)))
                   for k in range(reps)]
            rec["ess_per_sec"] = float(sum(ess) / sum(walls))
            rec["min_ess_median"] = float(np.median(ess))
        out[job] = rec
    out["value"] = out["naive_n4"]["value"]
    out["ess_per_sec"] = out["naive_n4"]["ess_per_sec"]
    out["cores"] = out["naive_n4"]["cores"]
    return out


def _schools_worker(w, J, it, seconds, second_half):
    """One process of a job: single-chain oracle runs on the job's data until `seconds` pass;
    per run (gradients, seconds, P x draws of mu, tau, eta, theta)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    lo = 4 if second_half else 0
    y, sig = np.array(SCHOOLS_Y[lo:lo + J]), np.array(SCHOOLS_SIGMA[lo:lo + J])
    m = O.Model(O.FAM_SCHOOLS, y=y, sigma=sig)
    out, t_all, k = [], time.perf_counter(), 0
    while time.perf_counter() - t_all < seconds or k < 2:
        t = time.perf_counter()
        r = m.run_chain(num_warmup=it // 2, num_samples=it // 2, seed=1000 + 97 * k, gid=w)
        dt = time.perf_counter() - t
        q = r["q"][it // 2:]
        tau = np.exp(q[:, 1])
        theta = q[:, :1] + tau[:, None] * q[:, 2:]
        out.append((int(r["n_grad"]), dt, np.vstack([q[:, 0], tau, q[:, 2:].T, theta.T])))
        k += 1
    return out


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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) with no launcher around it: start N ranks, one process per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1 -- what torch.distributed.run
    sets), and return the worst exit code.  This process never touches the GPU (torch is not even
    imported here); rank 0 prints the line to the inherited stdout.  A rank that fails takes the
    others down with it (they would wait in a collective).  The reference runs one partition per
    Spark executor (stark/stark.py:65)."""
    port = _free_port()
    print(f"[bench] --gpus {n}: starting {n} ranks (127.0.0.1:{port})", file=sys.stderr, flush=True)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                break
            time.sleep(0.5)
        for p in procs:
            p.wait()
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise
    return rc or max((abs(p.returncode) for p in procs), default=0)


def check_world(gpus, env):
    """None when this process may run; else the reason to refuse.  `gpus` is --gpus (None: take
    the launcher's world size), `env` the process environment."""
    if "WORLD_SIZE" not in env:
        return None
    world = int(env["WORLD_SIZE"])
    if gpus is not None and gpus != world:
        return (f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks; a {world}-rank run "
                f"is not reported as {gpus} GPUs")
    return None


def rank_devices(dist, world, rank, local_rank, dev):
    """[[rank, local device index, PCI bus id], ...] of every rank (one all-reduce)."""
    import torch
    arr = np.zeros((world, 3))
    bus = -1
    if dev is not None:
        bus = getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", -1)
    arr[rank] = (rank, local_rank if dev is not None else -1, bus)
    if dist is not None:
        t = torch.from_numpy(arr).to(dev if dev is not None and dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t)
        arr = t.cpu().numpy()
    return [[int(v) for v in row] for row in arr]


def sweep_roofline(a, rows_per_shard, sweep_ms, sweeps, shard_sweeps):
    """The roofline object of the dominant kernel (the data sweep) from the sweep events of the
    timed window (HIP events on the context's stream, every n-th step)."""
    # C = 16: k_sweep16, X.[beta_1..beta_16] on fp64 MFMA;
    # C <= 4: k_sweep3 (VALU), bound by HBM.
    mfma = a.chains == 16
    kname = "k_sweep16" if mfma else "k_sweep3"
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
        # arithmetic intensity 4 C d / (8 d + 4) = 7.96 flop/B at C = 16, d = 100: below the fp64
        # machine balance (78.6 TF / 8 TB/s = 9.8 flop/B), so the roofline that bounds the sweep is
        # HBM; the fp64-MFMA figure is reported beside it
        intensity = flops_per_launch / bytes_per_launch
        balance = FP64_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)
        mf = {"achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": (tfs / FP64_PEAK_TFS) if tfs else None,
              "peak_measured": FP64_MFMA_MEASURED_TFS,
              "peak_measured_instruction": "v_mfma_f64_16x16x4_f64 (the kernel's)",
              "frac_of_measured": (tfs / FP64_MFMA_MEASURED_TFS) if tfs else None}
        prim, sec, sec_name = (hbm, mf, "mfma") if intensity < balance else (mf, hbm, "hbm")
        roof = {"bound": "hbm" if intensity < balance else "mfma", **prim, "traffic": traffic,
                "kernel": f"{kname}<{fam}> (fp64 MFMA 16x16x4, {a.chains} chains)", "avg_launch_ms": avg_ms,
                "algorithmic_flops_per_launch": flops_per_launch, "algorithmic_bytes_per_launch": bytes_per_launch,
                "intensity_flop_per_byte": intensity, "machine_balance_flop_per_byte": balance, sec_name: sec}
    else:
        roof = dict(bound="hbm", **{k: v for k, v in hbm.items()}, traffic=traffic,
                    kernel=f"k_sweep3<{fam},{a.chains}>", avg_launch_ms=avg_ms,
                    algorithmic_bytes_per_launch=bytes_per_launch)
    return roof


def main():
    a = parse()
    refuse = check_world(a.gpus, os.environ)
    if refuse:
        sys.exit(refuse)
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if a.adapt_iters is None:
        a.adapt_iters = 150 if a.family == "logistic" else 1000
    t_start = time.perf_counter()

    def left():                        # seconds of the run's wall-time budget still unspent
        return a.deadline_s - (time.perf_counter() - t_start)

    def skipped(cost):
        return {"skipped": f"deadline: {left():.0f} s of --deadline-s {a.deadline_s:.0f} left, this record needs ~{cost} s"}

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # STARK_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N-rank path on one
    # GPU (ranks share devices round-robin); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("STARK_DIST_BACKEND", "nccl")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    ndev = torch.cuda.device_count()          # counts devices without initialising the GPU
    if backend == "nccl" and world > 1 and ndev < world:
        sys.exit(f"bench.py: {world} ranks need {world} visible GPUs (one rank per GPU), found {ndev}; "
                 "a rehearsal with ranks sharing a GPU: STARK_DIST_BACKEND=gloo")
    dist = None
    # STARK_FORCE_DIST=1: a process group even at world size 1 (exercises the RCCL collectives of
    # the N-rank path on one GPU: all-reduces, the draw all-gather, the Laplace gradient sums)
    if world > 1 or os.environ.get("STARK_FORCE_DIST") == "1":
        import torch.distributed as dist
        if ndev:
            local_rank %= ndev
            torch.cuda.set_device(local_rank)
        # ranks other than 0 wait at the final barrier while rank 0 runs the optional sub-records
        # (up to --deadline-s): a timeout well past that, not the 10-minute default
        pg_timeout = datetime.timedelta(seconds=max(1800, 3 * a.deadline_s))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)
    dev = local_rank if ndev else None
    if a.launch_check:
        devs = rank_devices(dist, world, rank, local_rank, dev)
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "world_size": world,
                              "dist_backend": dist.get_backend() if dist else None, "rank_devices": devs}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    from stark_amd import dist as sdist
    from stark_amd import engine

    assert a.shards % world == 0, "shards must divide evenly over GPUs"
    spr = a.shards // world
    rows_per_shard = int(a.rows) // a.shards
    first = a.shard_offset + rank * spr                # global id of this rank's first shard
    shard_ids = list(range(first, first + spr))
    gather_ids = list(range(rank * spr, rank * spr + spr))  # this job's shard slots (the all-gather keys)
    ctx = engine.Context(local_rank)

    t = time.perf_counter()
    model = engine.Model.synthetic(ctx, a.family, spr, rows_per_shard, a.d, data_seed=a.seed,
                                   row_offset=first * rows_per_shard)
    ctx.sync()
    t_gen = time.perf_counter() - t

    A, W, K, ND = a.adapt_iters, a.warmup, a.steps, a.ess_draws
    # every step is at most one transition per chain, so A + W + K + ND transitions always
    # cover the timed window and the fixed post-warmup draws of the ESS phase
    n_samp = W + K + ND + 1
    sampler = model.sampler(num_warmup=A, num_samples=n_samp, chains=a.chains, seed=a.seed + 1,
                            shard_ids=shard_ids, stepsize_jitter=a.stepsize_jitter, nuts_criterion=a.nuts_criterion)

    def log(msg):
        if rank == 0:
            print(f"[bench] {msg}", file=sys.stderr, flush=True)

    def barrier():
        torch.cuda.synchronize(local_rank)
        if dist:
            dist.barrier()

    def allreduce(arr, op="sum"):
        """float64 numpy array summed (or maxed) over ranks in place (RCCL / gloo)."""
        if not dist:
            return arr
        dev = sdist._device_for_backend()
        t_ = torch.from_numpy(np.ascontiguousarray(arr, np.float64)).to(dev)
        dist.all_reduce(t_, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}.get(op, dist.ReduceOp.SUM))
        arr[...] = t_.cpu().numpy()
        return arr

    log(f"data generated: {spr} shards x {rows_per_shard} rows x d={a.d} in {t_gen:.1f}s "
        f"({model.device_bytes() / 1e9:.1f} GB on this GPU)")
    t = time.perf_counter()
    # One run to the end of warmup, in bounded step batches for progress lines: chains move
    # independently and only wait for each other once, at iteration A.
    while not a.throughput_only:
        sampler.run(A, max_steps=1000)
        its = sampler.iterations()
        inf = sampler.info()
        log(f"adaptation: {time.perf_counter() - t:.1f}s, transitions per chain min/median "
            f"{its.min()}/{int(np.median(its))} of {A}, leapfrogs/chain {inf['leapfrogs'] / max(1, spr * a.chains):.0f}")
        if its.min() >= A:
            break
    t_adapt = time.perf_counter() - t
    t = time.perf_counter()
    sampler.run(A + n_samp, max_steps=W)
    ctx.sync()
    t_wsteps = time.perf_counter() - t
    log(f"warmup steps done; timing {K} steps")

    nchains = spr * a.chains
    it0 = sampler.iterations()
    # sweep events on every n-th step (each event pair is a stream barrier: ~1-2 % of a step)
    ctx.set_profiling(max(1, min(8, K // 16)))
    i0 = sampler.info()
    barrier()
    t0 = time.perf_counter()
    w0 = time.monotonic_ns()
    sampler.run(A + n_samp, max_steps=K)
    ctx.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    w1 = time.monotonic_ns()
    ctx.set_profiling(False)
    i1 = sampler.info()
    it1 = sampler.iterations()

    grads = i1["grad_evals"] - i0["grad_evals"]
    leaps = i1["leapfrogs"] - i0["leapfrogs"]
    sweeps = i1["sweeps"] - i0["sweeps"]
    shard_sweeps = i1["shard_sweeps"] - i0["shard_sweeps"]
    sweep_ms = i1["sweep_ms"] - i0["sweep_ms"]
    done_in_window = it1 - it0                       # transitions completed per chain
    if dist:
        elapsed = float(allreduce(np.array([elapsed]), "max")[0])
        grads, leaps = (int(v) for v in allreduce(np.array([grads, leaps], np.float64)))
    devs = rank_devices(dist, world, rank, local_rank, dev)
    if a.throughput_only:
        # the timed window only (the sampler still adapting: a step costs one sweep whatever the phase)
        roof = sweep_roofline(a, rows_per_shard, sweep_ms, sweeps, shard_sweeps)
        sampler.close()
        model.close()
        if rank == 0:
            print(json.dumps({
                "metric": f"gradient evals/sec (whole node), {a.family} regression N={a.rows:.0e} d={a.d}".replace("e+0", "e"),
                "value": grads / elapsed, "unit": "gradient evals/sec", "n_gpus": world, "steps": K, "warmup": W,
                "ms_per_step": 1e3 * elapsed / K, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "f64", "data": "synthetic (Philox in HBM, SURVEY 8d)",
                "config": {"workload": f"bayesian {a.family} regression, {a.shards} subposterior shards, throughput only",
                           "rows": int(a.rows), "d": a.d, "shards": a.shards, "chains_per_shard": a.chains,
                           "parallelism": f"shard-dp{world}"},
                "roofline": roof, "rank_devices": devs}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- ESS phase (not part of `value`): every chain of every rank runs on to the same
    # number of post-warmup draws, n_post = max(ND, the most any chain already has), so the
    # consensus pairs draw i of chain c of every shard (equal-length chains, Stan's
    # multi-chain estimator).  Its time counts in the ESS/s denominators.
    n_post = int(allreduce(np.array([max(ND, int(it1.max()) - A)], np.float64), "max")[0])
    assert a.ess_budget_s is None or world == 1, "--ess-budget-s: one process"
    t = time.perf_counter()
    while True:                      # bounded batches with a progress line (long phases under the 2.19 criterion)
        sampler.run(A + n_post, max_steps=2000)
        its = sampler.iterations()
        log(f"ESS phase: {time.perf_counter() - t:.1f}s, post-warmup draws per chain min {its.min() - A} of {n_post}")
        if its.min() >= A + n_post:
            break
        if a.ess_budget_s is not None and time.perf_counter() - t > a.ess_budget_s:
            n_post = int(its.min()) - A          # the draws every chain has: the phase ends here
            log(f"ESS phase stopped at the {a.ess_budget_s:.0f} s budget with {n_post} post-warmup draws per chain")
            break
    ctx.sync()
    barrier()
    t_post = time.perf_counter() - t
    info = sampler.info()
    C = a.chains
    # the draws stay in HBM: library buffer -> device tensor -> RCCL all-gather -> device combine
    dev = torch.device("cuda", local_rank) if torch.cuda.is_available() else None
    cols = np.concatenate([np.arange(c * n_samp, c * n_samp + n_post) for c in range(C)])
    cols_t = torch.as_tensor(cols, device=dev)
    local = {}
    stats = []
    for s in range(spr):
        full = sampler.draws_device(s)
        local[gather_ids[s]] = full.index_select(1, cols_t).contiguous()
        stats.append(sampler.draws(s)[1][cols])
    stats = np.vstack(stats)
    if a.dump_draws and rank == 0 and world == 1:
        np.savez(a.dump_draws, shard_ids=np.array(shard_ids), chains=C, draws_per_chain=n_post,
                 t_adapt=t_adapt, t_sampling=t_wsteps + elapsed + t_post, grad_evals=info["grad_evals"],
                 leapfrogs_per_transition=float(stats[:, 3].mean()), divergent=info["divergent"],
                 **{f"draws_{sid}": local[g].cpu().numpy() for sid, g in zip(shard_ids, gather_ids)})
        log(f"draws of shards {shard_ids} written to {a.dump_draws}")
    t = time.perf_counter()
    allp_dev = sdist.all_gather_partitions(local, a.shards, as_tensor=True)   # one all-gather (RCCL on GPUs)
    if allp_dev.is_cuda:
        torch.cuda.synchronize(allp_dev.device)
    t_gather = time.perf_counter() - t
    allp = list(allp_dev.cpu().numpy())          # host copies: Laplace start point, CPU combine, ESS
    eps, _ = sampler.adaptation()
    # full-data posterior reference (logistic, flat priors): MAP + inverse Hessian from the
    # GPU gradient summed over every shard of every rank (tools/laplace.py)
    lap = None
    if a.family == "logistic" and not a.no_accuracy:
        from tools import laplace as L
        t = time.perf_counter()
        pooled = np.hstack([x[:-1] for x in allp])
        lap = L.laplace(model, list(range(spr)), pooled.mean(1), pooled.std(1) / np.sqrt(a.shards),
                        reduce=(lambda arr: allreduce(arr)) if dist else None)
        log(f"full-data Laplace reference in {time.perf_counter() - t:.1f}s")
    second = None
    if a.second_criterion != "none" and a.second_criterion != a.nuts_criterion:
        # the same data, warmup length and shard RNG keys under another NUTS criterion / jitter
        # (default: the reference's pystan 2 sampler, Stan 2.19.1 with stepsize_jitter 0), in
        # bounded step batches under a wall-time budget
        ND2 = a.second_draws
        t = time.perf_counter()
        s2 = model.sampler(num_warmup=A, num_samples=ND2, chains=a.chains, seed=a.seed + 1, shard_ids=shard_ids,
                           stepsize_jitter=a.second_jitter, nuts_criterion=a.second_criterion)
        phase, completed = {}, True
        for target in (A, A + ND2):
            t_ph = time.perf_counter()
            while True:
                s2.run(target, max_steps=2000)
                its = s2.iterations()
                done = float(allreduce(np.array([float(its.min() >= target)]), "min")[0]) > 0
                over = float(allreduce(np.array([float(time.perf_counter() - t > a.second_budget_s
                                                         or left() < 150)]), "max")[0]) > 0
                log(f"second criterion {a.second_criterion}: {time.perf_counter() - t:.1f}s, transitions per chain "
                    f"min {its.min()} of {target}")
                if done or over:
                    break
            ctx.sync()
            barrier()
            phase[target] = time.perf_counter() - t_ph
            if not done:
                completed = False
                break
        if not completed:
            second = {"status": f"stopped at the {a.second_budget_s:.0f} s budget", "iterations_min": int(its.min()),
                      "seconds": time.perf_counter() - t}
        else:
            loc2, st2 = {}, []
            for s_ in range(spr):
                loc2[gather_ids[s_]] = s2.draws_device(s_)
                st2.append(s2.draws(s_)[1])
            allp2 = sdist.all_gather_partitions(loc2, a.shards, as_tensor=True)
            st2 = np.vstack(st2)
            second = {"allp": allp2, "t_adapt": phase[A], "t_post": phase[A + ND2], "nd": ND2,
                      "lf": float(st2[:, 3].mean()), "div": s2.info()["divergent"]}
        s2.close()
        log(f"second criterion {a.second_criterion}: {time.perf_counter() - t:.1f}s")
    lin = None
    if a.family == "linear" and not a.no_accuracy:
        # flat-prior linear regression: the full-data posterior of (alpha, beta) in closed form
        # (multivariate t) from the sufficient statistics [1 X]'[1 X], [1 X]'y, y'y, summed
        # over every shard of every rank
        k = a.d + 1
        acc = np.zeros(k * k + k + 2)
        for s_ in range(spr):
            dd = model.copy_data(s_)
            A1 = np.hstack([np.ones((dd["x"].shape[0], 1)), dd["x"]])
            acc[:k * k] += (A1.T @ A1).ravel()
            acc[k * k:k * k + k] += A1.T @ dd["y"]
            acc[-2] += dd["y"] @ dd["y"]
            acc[-1] += dd["x"].shape[0]
            del A1, dd
        allreduce(acc)
        AtA, Aty, yty, ntot = acc[:k * k].reshape(k, k), acc[k * k:k * k + k], acc[-2], acc[-1]
        mean = np.linalg.solve(AtA, Aty)
        rss = yty - 2 * mean @ Aty + mean @ AtA @ mean
        nu = ntot - k - 1
        lin = (mean, nu / (nu - 2.0) * rss / nu * np.linalg.inv(AtA))
    sampler.close()

    if rank != 0:
        model.close()
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    from stark_amd import diagnostics
    P = allp[0].shape[0]
    comb_ms = []
    for _ in range(6):      # device draws in, device result out; the first call also sizes the scratch buffers
        t = time.perf_counter()
        comb_t, used = engine.consensus(allp_dev, ctx, separate_lp=True)
        comb_ms.append(1e3 * (time.perf_counter() - t))
    comb = comb_t.cpu().numpy() if hasattr(comb_t, "cpu") else comb_t
    t = time.perf_counter()
    comb_host, _ = engine.consensus(allp, ctx, separate_lp=True)     # the host-buffer API, for comparison
    comb_host_ms = 1e3 * (time.perf_counter() - t)
    assert np.array_equal(comb_host, comb)
    comb_joint, _ = engine.consensus(allp, ctx)               # the reference's joint weights (lp__ in)

    def min_ess(x, floor=False, n=n_post):
        return float(np.nanmin([diagnostics.ess(x[p].reshape(C, n), floor=floor) for p in range(x.shape[0])]))

    ess_c = min_ess(comb[:-1])                                 # lp__ excluded
    ess_c_floor = min_ess(comb[:-1], floor=True)
    ess_s0 = min_ess(allp[0][:-1])
    t_sampling = t_wsteps + elapsed + t_post
    truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
    if a.family == "linear":
        truth = np.concatenate([truth, [1.0]])                # sigma
    csd = comb[:-1].std(1)

    def zz(err, sd):
        z = err / sd
        return {"mean_z2": float((z ** 2).mean()), "max_abs_z": float(np.abs(z).max())}

    accuracy = {"vs_generating_params": zz(comb[:-1].mean(1) - truth, csd),
                "vs_generating_params_joint_lp": zz(comb_joint[:-1].mean(1) - truth, csd)}
    if lap is not None:
        fm, fc, finfo = lap
        fsd = np.sqrt(np.diag(fc))
        accuracy["vs_fulldata_laplace"] = {
            "consensus": zz(comb[:-1].mean(1) - fm, fsd),
            "consensus_joint_lp": zz(comb_joint[:-1].mean(1) - fm, fsd),
            "sd_ratio_median": float(np.median(csd / fsd)),
            "truth": zz(truth - fm, fsd),
            "newton_steps_in_sd": finfo["newton_steps_in_sd"]}
    if lin is not None:
        fm, fc = lin
        fsd = np.sqrt(np.diag(fc))
        k = a.d + 1
        accuracy["vs_fulldata_exact"] = {
            "consensus": zz(comb[:k].mean(1) - fm, fsd),
            "consensus_joint_lp": zz(comb_joint[:k].mean(1) - fm, fsd),
            "sd_ratio_median": float(np.median(comb[:k].std(1) / fsd)),
            "truth": zz(truth[:k] - fm, fsd),
            "note": "alpha, beta vs the closed-form flat-prior posterior (multivariate t) of all N rows"}
    if second is not None and "allp" not in second:
        second_line = {"nuts_criterion": a.second_criterion, "stepsize_jitter": a.second_jitter, **second}
    elif second is not None:
        comb2_t, _ = engine.consensus(second["allp"], ctx, separate_lp=True)
        comb2 = comb2_t.cpu().numpy() if hasattr(comb2_t, "cpu") else comb2_t
        ess2 = min_ess(comb2[:-1], n=second["nd"])
        second_line = {"nuts_criterion": a.second_criterion, "stepsize_jitter": a.second_jitter,
                       "note": "the reference's NUTS criterion (pystan 2 = Stan 2.19.1's single U-turn test) on the same "
                               "data, warmup length and shard RNG keys; stepsize_jitter as stated (pystan's default 0 makes "
                               "the 2.19 trajectories resonate on this posterior and does not fit the lease)",
                       "ess_per_sec": ess2 / (second["t_adapt"] + second["t_post"]),
                       "min_ess": ess2, "min_ess_floored": min_ess(comb2[:-1], floor=True, n=second["nd"]),
                       "ess_per_sec_post_warmup": ess2 / second["t_post"], "post_warmup_draws_per_chain": second["nd"],
                       "leapfrogs_per_transition": second["lf"], "divergent": second["div"],
                       "seconds": {"adaptation": second["t_adapt"], "post_warmup_draws": second["t_post"]}}
        if lap is not None:
            second_line["vs_fulldata_laplace"] = zz(comb2[:-1].mean(1) - lap[0], np.sqrt(np.diag(lap[1])))
        if lin is not None:
            k = a.d + 1
            second_line["vs_fulldata_exact"] = zz(comb2[:k].mean(1) - lin[0], np.sqrt(np.diag(lin[1])))
    else:
        second_line = None
    accuracy["note"] = ("z = (mean - reference) / reference sd per parameter over all alpha, beta; the consensus "
                        "puts lp__ in its own weight block (engine.consensus separate_lp); *_joint_lp = the "
                        "reference's joint combine (lp__ inside inv(cov), stark/stark.py:49-56). vs_fulldata_laplace: "
                        "the full-data posterior (MAP + inverse Hessian of the GPU gradient, tools/laplace.py)")

    roof = sweep_roofline(a, rows_per_shard, sweep_ms, sweeps, shard_sweeps)
    value = grads / elapsed
    # ESS per gradient evaluation of the whole run (warmup included): the same algorithm on the
    # CPU twin (transition-identical, tests/test_gpu_nuts.py) spends the same gradients per ESS
    total_grads = info["grad_evals"] * world
    cpu = None
    if not a.no_cpu_baseline:          # rank 0 only (the other ranks returned above), at every world size
        try:
            cpu = cpu_baseline(a.d, rows_per_shard, a.shards, a.cpu_baseline_seconds, a.family)
            cpu["ess_per_sec"] = cpu["value"] * ess_c / total_grads
            cpu["ess_note"] = ("the measured CPU gradient rate x this run's ESS per gradient evaluation "
                               "(warmup included): the CPU twin runs the same NUTS transitions")
            cpu.update(cpu_combine(allp))
        except Exception as e:          # the GPU line is still printed
            cpu = {"error": repr(e)}
    schools = None
    if rank == 0 and not a.no_schools:  # BASELINE configs[1] (example/stark_ex.py 8-schools, 4096 chains)
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import bench_schools
            schools = bench_schools.run(ctx=ctx)
            schools["note"] = ("BASELINE configs[1]: 8-schools (example/stark_ex.py data, example/schools.stan) with "
                               "4096 NUTS chains, Stan defaults (1000 warmup + 1000 draws), fused kernel; run on rank 0 "
                               "after the timed window (tools/bench_schools.py)")
            if not a.no_cpu_baseline:
                schools["cpu_baseline"] = (cpu_baseline_schools(a.cpu_baseline_seconds) if left() > 40
                                           else skipped(15))
                schools["cpu_baseline"]["note"] = (
                    "the reference's CPU path for this data (example/stark_ex.py:24-26), one process per single-chain "
                    "run; ess_per_sec over the whole job (warmup included): compare with ess_per_sec_whole_run")
        except Exception as e:          # the main line is still printed
            schools = {"error": repr(e)}
    others = None
    if world == 1 and not dist and not a.no_other_configs:
        # BASELINE configs[2], configs[3] at the driver API's default chains=1, and configs[4] on
        # this GPU after the timed window (the main shards are released first: configs[4] keeps
        # 200 GB resident); each a child process running bench.py's own line, except configs[4]
        model.close()
        model = None
        others = {}
        env = {k: v for k, v in os.environ.items()
               if k not in ("STARK_FORCE_DIST", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}

        def child(args, cost, keys, extra):
            if left() < cost:
                return skipped(cost)
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=max(60, left()), env=env)
                ln = json.loads(r.stdout.strip().splitlines()[-1])
                return {**{k: ln[k] for k in keys if k in ln}, **extra(ln), "command": " ".join(["bench.py", *args])}
            except Exception as e:      # the main line is still printed
                return {"error": repr(e)}

        # configs[2] under pystan 2's own settings (stark/stark.py:48, 60-63): Stan 2.19.1's NUTS
        # criterion, stepsize_jitter 0, iter = 2000 -> 1000 warmup + 1000 draws per chain
        others["configs2_linear"] = child(
            ["--family", "linear", "--rows", "1e7", "--d", "50", "--nuts-criterion", "stan2.19",
             "--stepsize-jitter", "0", "--adapt-iters", "1000", "--ess-draws", "1000", "--steps", "300",
             "--warmup", "20", "--second-criterion", "none", "--no-schools", "--no-other-configs",
             "--cpu-baseline-seconds", str(a.cpu_baseline_seconds)] + (["--no-cpu-baseline"] if a.no_cpu_baseline else []),
            110, ("metric", "value", "unit", "ms_per_step", "steps", "roofline", "ess_per_sec", "min_ess",
                  "ess_per_sec_post_warmup", "leapfrogs_per_transition", "divergent", "stepsize_per_chain",
                  "setup_s", "cpu_baseline", "config"),
            lambda ln: {"vs_fulldata_exact": ln["accuracy"].get("vs_fulldata_exact"),
                        "note": "the reference sampler's settings (pystan 2 = Stan 2.19.1 NUTS, stepsize_jitter 0, "
                                "iter=2000: 1000 warmup + 1000 draws per chain, stark/stark.py:48, 60-63); ESS/s "
                                "over the whole sampling time, warmup included"})
        # configs[3] at the driver API's default (stark/stark.py:62-63): ONE chain per shard -> the
        # VALU k_sweep3 (HBM-bound), throughput only
        others["configs3_chains1"] = child(
            ["--chains", "1", "--throughput-only", "--steps", "200", "--warmup", "10"], 40,
            ("metric", "value", "unit", "ms_per_step", "steps", "roofline", "config"),
            lambda ln: {"note": "concensusWeight()'s default chains=1 per partition at configs[3]'s shape (8 shards x "
                                "1.25e7 rows, d = 100): one chain per shard, the sampler in adaptation (a step is one "
                                "sweep whatever the phase)"})
        if left() > 45:
            try:
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                import bench_fulldata
                others["configs4_fulldata"] = bench_fulldata.run(2.5e7, steps=10, warmup=2, seed=a.seed)
            except Exception as e:
                others["configs4_fulldata"] = {"error": repr(e)}
        else:
            others["configs4_fulldata"] = skipped(45)
    line = {
        "metric": f"gradient evals/sec (whole node), {a.family} regression N={a.rows:.0e} d={a.d}".replace("e+0", "e"),
        "value": value,
        "unit": "gradient evals/sec",
        "n_gpus": world,
        "world_size": world,
        "dist_backend": dist.get_backend() if dist else None,
        "rank_devices": devs,
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
                   "chains_per_shard": a.chains, "num_warmup": A, "post_warmup_draws_per_chain": n_post,
                   "stepsize_jitter": a.stepsize_jitter, "nuts_criterion": a.nuts_criterion,
                   "parallelism": f"shard-dp{world}"},
        "ess_per_sec": ess_c / (t_adapt + t_sampling),
        "min_ess": ess_c,
        "ess_per_sec_floored": ess_c_floor / (t_adapt + t_sampling),
        "ess_floor_note": ("*_floored: the same ESS with the tau_hat >= 1/log10(draws) bound of Stan releases after 2.19 "
                           "(ess_per_sec is Stan 2.19's estimator, which has no such bound)"),
        "ess_method": ("min over alpha, beta (lp__ excluded) of Stan 2.19's multi-chain ESS of the consensus draws "
                       f"({C} combined chains x {n_post} post-warmup draws; combined chain c = chain c of every "
                       "shard), divided by the whole sampling wall time: warmup/adaptation + the timed steps + the "
                       "post-warmup draws (SURVEY 8d; data generation excluded)"),
        "ess_per_sec_post_warmup": ess_c / t_sampling,
        "num_warmup_note": (f"num_warmup = {A} (Stan's default iter=2000 would warm up for 1000; DESIGN.md 4): "
                            "the adaptation is the dominant ESS/s cost"),
        "subposterior_min_ess_shard0": ess_s0,
        "ess_second_criterion": second_line if second_line is not None else {
            "note": "off by default (--second-criterion); the reference sampler's own settings (Stan 2.19.1 NUTS, "
                    "jitter 0, 1000 + 1000) run on configs[2] in other_configs.configs2_linear"},
        "accuracy": accuracy,
        "stepsize_per_chain": {"min": float(eps.min()), "median": float(np.median(eps)), "max": float(eps.max())},
        "treedepth_mean": float(stats[:, 2].mean()),
        "leapfrogs_per_transition": float(stats[:, 3].mean()),
        "rows_x_chains_per_sec": grads * rows_per_shard / elapsed,
        "roofline": roof,
        "cpu_baseline": cpu,
        "configs1_schools": schools,
        "other_configs": others,
        "combine": {"gpu_ms": float(np.median(comb_ms[1:])), "gpu_ms_min": min(comb_ms[1:]),
                    "gpu_ms_first_call": comb_ms[0], "host_buffers_ms": comb_host_ms, "shards": a.shards, "P": P,
                    "draws": C * n_post, "all_gather_ms": 1e3 * t_gather,
                    "draws_on_device": bool(getattr(allp_dev, "is_cuda", False)),
                    "consensus_sha16": hashlib.sha256(np.ascontiguousarray(comb).tobytes()).hexdigest()[:16],
                    "note": "engine.consensus(separate_lp=True) on the all-gathered draws where they lie (device "
                            "draws from RCCL: no host copy, the result left in HBM; a gloo rehearsal gathers on the "
                            "host); wall time of the call (median of 5 after the first); host_buffers_ms: the same "
                            "combine through host numpy buffers (H2D + D2H copies included)"},
        "setup_s": {"datagen": t_gen, "adaptation": t_adapt, "post_warmup_draws": t_post},
        "timed_window_monotonic_ns": [w0, w1],     # tools/rocpd_summary.py window: the kernel trace's dispatches in it
        "divergent": info["divergent"],
    }
    print(json.dumps(line), flush=True)
    if model is not None:
        model.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
