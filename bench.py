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

After the headline, the same process (every rank of an N-rank run) times the other BASELINE
configurations: configs[1] (8 schools x 4096 chains, rank 0: a one-GPU config), configs[2]
(linear N=1e7 d=50, 8 shards over the N ranks, the reference sampler's settings), configs[3]
at the driver API's default chains=1, and configs[4] (full-data logistic d=1000, 64 chains,
rows split over the N ranks with a per-leapfrog gradient all-reduce).  Each is a compact
sub-record; the line's keys are explained in DESIGN.md section 4 ("bench line keys") and the
headline ESS/s, min ESS and accuracy come LAST in the line (a driver that keeps the tail of
stdout keeps them).

Usage: python bench.py [--gpus N --steps K --warmup W].  --gpus N > 1 without a launcher starts N
rank processes itself (one per GPU, RCCL) before any GPU call; under a
launcher (WORLD_SIZE set) --gpus must equal the world size or the run is refused.
"""
import argparse
import datetime
import hashlib
import json
import signal
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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs = ranks (one process per GPU).  Without a launcher, N > 1 starts N rank processes "
                        "itself; under one (torch.distributed.run), must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    p.add_argument("--launch-check", action="store_true",
                   help="start the ranks, build the process group, report world size / backend / rank devices and "
                        "exit: the launcher path without sampling (CPU: STARK_DIST_BACKEND=gloo)")
    p.add_argument("--throughput-only", action="store_true",
                   help="time the K steps (sampler still in adaptation) and print the line: no ESS phase, accuracy, "
                        "CPU baseline or sub-records")
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
    p.add_argument("--ess-draws", type=int, default=1000,
                   help="post-warmup draws per chain for the ESS / accuracy phase (after the timed steps): Stan's "
                        "default num_samples (iter=2000 -> 1000 draws, stark/stark.py:60-63); ESS/s counts the "
                        "warmup too, so it rises with the draws per warmup iteration (rounds 2-5: 250)")
    p.add_argument("--no-accuracy", action="store_true", help="skip the full-data reference")
    p.add_argument("--nuts-criterion", choices=["stan2.19", "stan2.23"], default="stan2.23",
                   help="stan2.23 (default): Stan's NUTS with the U-turn checks across subtree junctions "
                        "(Stan >= 2.23); stan2.19: the reference's pystan 2 NUTS, whose single test lets "
                        "trajectories resonate on this near-isotropic posterior (36 vs 11 leapfrogs per "
                        "transition, DESIGN.md section 4)")
    p.add_argument("--second-criterion", choices=["stan2.23", "stan2.19", "none"], default="none",
                   help="after the main run: a second adaptation + ESS phase on the same data with this "
                        "NUTS criterion, reported as ess_second_criterion.  Off by default: the reference "
                        "sampler's own settings run in the configs2_linear sub-record")
    p.add_argument("--second-jitter", type=float, default=0.5, help="stepsize_jitter of the second run")
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
                   help="skip the configs[2] / configs[3] chains=1 / configs[4] sub-records")
    # sizes of the sub-records (defaults: the BASELINE configs; smaller values rehearse the path)
    p.add_argument("--cfg2-rows", type=float, default=1e7, help="configs[2] total rows (linear, d=50, 8 shards)")
    p.add_argument("--cfg2-adapt", type=int, default=1000, help="configs[2] warmup (pystan 2: iter=2000 -> 1000)")
    p.add_argument("--cfg2-draws", type=int, default=1000, help="configs[2] post-warmup draws per chain")
    p.add_argument("--cfg4-rows-per-gpu", type=float, default=2.5e7,
                   help="configs[4] rows resident per GPU (d=1000 fp64: 2.5e7 rows = 200 GB)")
    p.add_argument("--cfg4-steps", type=int, default=10)
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
    p.add_argument("--detail-json", default=None,
                   help="rank 0 also writes the uncompacted records (every sub-object of the line, in full) here")
    return p.parse_args(argv)


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
            "sample": f"oracle {'orc_logreg_lpgrad' if family == 'logistic' else 'orc_linreg_lpgrad'}, "
                      f"{sample_rows} rows x d={d} per worker, {seconds:.0f}s, {workers} workers, "
                      f"scaled to {rows_per_shard:.3g} rows/shard"}


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
    return 1e3 * (time.perf_counter() - t)


SCHOOLS_Y = [28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0]        # example/stark_ex.py:5
SCHOOLS_SIGMA = [15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0]  # example/stark_ex.py:6
SCHOOLS_JOBS = (("naive_n4", 4, 8, 2000), ("weighted_iter5000", 2, 4, 5000))


def schools_job_plan(runs, cores):
    """Waves of one CPU job: `runs` single-chain runs on min(runs, cores) worker processes,
    run w in wave w // workers.  Returns (workers, [[run ids of wave 0], [wave 1], ...])."""
    workers = max(1, min(runs, cores))
    return workers, [list(range(s, min(runs, s + workers))) for s in range(0, runs, workers)]


def cpu_baseline_schools(seconds, cores=None):
    """The reference's CPU path for 8 schools, timed the way example/stark_ex.py:24-26 runs it:
    pystan's single-chain NUTS (here the oracle's recursive Stan 2.19.1 twin, C) in one process
    per run, min(runs, cores) concurrent (Spark local[*]); with fewer cores than runs the runs
    go in waves and the job's wall time is the sum over waves of each wave's slowest run.
      weighted  concensusWeight(iter=5000): 2 runs of 2500 warmup + 2500 draws, one per
                four-school partition (stark/stark.py:59-64);
      naive     distribute(n=4): 4 full-data (J = 8) runs at iter=2000, 1000 + 1000 (the intent
                of stark/stark.py:74-85) -- the job the configs[1] GPU record scales
                to 4,096 chains.
    Each job repeats with fresh seeds for about `seconds`; gradient evals/s and ESS/s (Stan 2.19
    multi-chain ESS over the job's chains, min over mu, tau, eta, theta) per job wall time."""
    import multiprocessing as mp
    cores = cores or len(os.sched_getaffinity(0))
    ctx = mp.get_context("spawn")
    out = {"unit": "gradient evals/sec (whole job)", "kind": "port",
           "sample": f"oracle orc_run_chain (Stan 2.19.1 NUTS twin, C, 1 thread/run), jobs repeated ~{seconds:.0f} s"}
    for job, runs, J, it in SCHOOLS_JOBS:
        workers, waves = schools_job_plan(runs, cores)
        per_wave = seconds / 2 / len(waves)
        res = {}
        pool = ctx.Pool(workers)
        try:
            for wave in waves:
                # run w of the weighted job takes the four-school partition w (stark/stark.py:59-64)
                got = pool.starmap(_schools_worker, [(w, J, it, per_wave, J == 4 and w >= runs // 2) for w in wave])
                res.update(zip(wave, got))
            pool.close()
            pool.join()
        except BaseException:
            pool.terminate()
            raise
        reps = min(len(r) for r in res.values())
        walls = [sum(max(res[w][k][1] for w in wave) for wave in waves) for k in range(reps)]
        grads = [sum(res[w][k][0] for w in range(runs)) for k in range(reps)]
        rec = {"runs_per_job": runs, "runs_executed": len(res), "cores": workers, "waves": len(waves), "J": J,
               "iter": it, "jobs_timed": reps, "job_wall_ms_median": 1e3 * float(np.median(walls)),
               "value": float(sum(grads) / sum(walls))}
        if job == "naive_n4":
            from stark_amd import diagnostics
            ess = [float(np.nanmin(diagnostics.ess_matrix(np.hstack([res[w][k][2] for w in range(runs)]), runs)))
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


# ------------------------------------------------------------------ ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, script=None, grace_s=10.0):
    """`bench.py --gpus N` (N > 1) with no launcher around it: start N ranks, one process per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1 -- what torch.distributed.run
    sets), and return the worst exit code.  This process never touches the GPU (torch is not even
    imported here); rank 0 prints the line to the inherited stdout.  A rank that fails takes the
    others down with it (they would wait in a collective), and so does a SIGTERM / SIGHUP / SIGINT
    to the launcher: the ranks are terminated, then killed after `grace_s`, before it exits -- no
    rank outlives the launcher holding a GPU.  The reference runs one partition per Spark executor
    (stark/stark.py:65)."""
    port = _free_port()
    script = os.path.abspath(script or __file__)
    print(f"[bench] --gpus {n}: starting {n} ranks (127.0.0.1:{port})", file=sys.stderr, flush=True)
    procs = []

    def _stop(signum, _frame):
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, _stop) for s in (signal.SIGTERM, signal.SIGHUP)}

    def _reap():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.monotonic() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                _reap()
                break
            time.sleep(0.5)
        for p in procs:
            p.wait()
    except BaseException:
        _reap()
        raise
    finally:
        for s, h in old.items():
            signal.signal(s, h)
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


VISIBLE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def check_devices(backend, env, ndev):
    """None when every RCCL rank of this node gets a GPU of its own; else the reason to refuse.
    The ranks that share a node are LOCAL_WORLD_SIZE (default WORLD_SIZE: one node), so a
    multi-node run (world 16 = 2 x 8) needs 8 GPUs per node, not 16.  A launcher that pins one
    GPU per rank through HIP/ROCR/CUDA_VISIBLE_DEVICES leaves each rank ONE visible device (rank
    r uses its device 0).  Ranks sharing a device are the gloo rehearsal only."""
    world = int(env.get("WORLD_SIZE", "1"))
    if backend != "nccl" or world <= 1:
        return None
    local_world = int(env.get("LOCAL_WORLD_SIZE", world))
    if ndev == 0:
        return (f"bench.py: {world} RCCL ranks need one GPU each, found 0 visible GPUs; "
                "a rehearsal with ranks sharing a GPU: STARK_DIST_BACKEND=gloo")
    if ndev >= local_world or (ndev == 1 and any(env.get(k) for k in VISIBLE_VARS)):
        return None
    return (f"bench.py: {local_world} ranks on this node need {local_world} visible GPUs (one rank per GPU), "
            f"found {ndev}; a rehearsal with ranks sharing a GPU: STARK_DIST_BACKEND=gloo")


class Ranks:
    """This process's place in the job and the few host-side collectives the bench needs."""

    def __init__(self, dist, world, rank, local_rank, dev):
        self.dist, self.world, self.rank, self.local_rank, self.dev = dist, world, rank, local_rank, dev

    def allreduce(self, arr, op="sum"):
        """float64 numpy array summed (or maxed / mined) over ranks in place (RCCL / gloo)."""
        if not self.dist:
            return arr
        import torch
        from stark_amd import dist as sdist
        d = self.dist
        t_ = torch.from_numpy(np.ascontiguousarray(arr, np.float64)).to(sdist._device_for_backend())
        d.all_reduce(t_, op={"max": d.ReduceOp.MAX, "min": d.ReduceOp.MIN}.get(op, d.ReduceOp.SUM))
        arr[...] = t_.cpu().numpy()
        return arr

    def agree(self, ok):
        """True on every rank iff True on every rank (a skip decision all ranks follow)."""
        return float(self.allreduce(np.array([1.0 if ok else 0.0]), "min")[0]) > 0

    def barrier(self):
        import torch
        if self.dev is not None:
            torch.cuda.synchronize(self.local_rank)
        if self.dist:
            self.dist.barrier()

    def log(self, msg, every_s=0.0):
        """rank 0 -> stderr; every_s > 0: a progress line, printed at most once per every_s seconds
        (the driver keeps only the tail of stdout + stderr: the line must not be pushed out of it)."""
        if self.rank != 0:
            return
        now = time.monotonic()
        if every_s and now - getattr(self, "_last", -1e9) < every_s:
            return
        self._last = now
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def rank_devices(R):
    """[[rank, local device index, PCI bus id], ...] of every rank (one all-reduce)."""
    import torch
    arr = np.zeros((R.world, 3))
    bus = -1
    if R.dev is not None:
        bus = getattr(torch.cuda.get_device_properties(R.dev), "pci_bus_id", -1)
    arr[R.rank] = (R.rank, R.local_rank if R.dev is not None else -1, bus)
    R.allreduce(arr)
    return [[int(v) for v in row] for row in arr]


def sha16(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


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
    roof = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (gbs / HBM_PEAK_GBS) if gbs else None, "traffic": traffic,
            "kernel": f"{kname}<{fam}>" + (" fp64 MFMA" if mfma else f" C={a.chains}"), "avg_launch_ms": avg_ms,
            "algorithmic_bytes_per_launch": bytes_per_launch}
    if mfma:
        # arithmetic intensity 4 C d / (8 d + 4) = 7.96 flop/B at C = 16, d = 100: below the fp64
        # machine balance (78.6 TF / 8 TB/s = 9.8 flop/B), so the roofline that bounds the sweep is
        # HBM; the fp64-MFMA figure is reported beside it
        roof["mfma"] = {"achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": (tfs / FP64_PEAK_TFS) if tfs else None,
                        "frac_of_measured": (tfs / FP64_MFMA_MEASURED_TFS) if tfs else None}
    return roof


# ------------------------------------------------------------------ one consensus job
def consensus_job(a, R, ctx, left, cpu_seconds=None):
    """One subposterior-sampling + consensus job of the configuration `a` on every rank (the
    shards split over the ranks): datagen -> warmup -> W + K timed steps -> ESS phase ->
    all-gather -> combine -> ESS / accuracy.  Returns the detailed record on rank 0 (None on the
    other ranks, which return once their collectives are done)."""
    import torch
    from stark_amd import dist as sdist
    from stark_amd import engine

    world, rank = R.world, R.rank
    assert a.shards % world == 0, "shards must divide evenly over GPUs"
    spr = a.shards // world
    rows_per_shard = int(a.rows) // a.shards
    first = a.shard_offset + rank * spr                # global id of this rank's first shard
    shard_ids = list(range(first, first + spr))
    gather_ids = list(range(rank * spr, rank * spr + spr))  # this job's shard slots (the all-gather keys)
    A = a.adapt_iters if a.adapt_iters is not None else (150 if a.family == "logistic" else 1000)
    W, K, ND = a.warmup, a.steps, a.ess_draws

    t = time.perf_counter()
    model = engine.Model.synthetic(ctx, a.family, spr, rows_per_shard, a.d, data_seed=a.seed,
                                   row_offset=first * rows_per_shard)
    ctx.sync()
    t_gen = time.perf_counter() - t
    # every step is at most one transition per chain, so A + W + K + ND transitions always
    # cover the timed window and the fixed post-warmup draws of the ESS phase
    n_samp = W + K + ND + 1
    sampler = model.sampler(num_warmup=A, num_samples=n_samp, chains=a.chains, seed=a.seed + 1,
                            shard_ids=shard_ids, stepsize_jitter=a.stepsize_jitter, nuts_criterion=a.nuts_criterion)
    tag = f"{a.family} d={a.d}"
    R.log(f"{tag}: {spr} shards x {rows_per_shard} rows per rank in {t_gen:.1f}s "
          f"({model.device_bytes() / 1e9:.1f} GB on this GPU)")
    t = time.perf_counter()
    # One run to the end of warmup, in bounded step batches for progress lines: chains move
    # independently and only wait for each other once, at iteration A.
    while not a.throughput_only:
        sampler.run(A, max_steps=1000)
        its = sampler.iterations()
        R.log(f"{tag} warmup {time.perf_counter() - t:.0f}s: transitions min/median {its.min()}/{int(np.median(its))}"
              f" of {A}", every_s=30)
        if its.min() >= A:
            break
    t_adapt = time.perf_counter() - t
    t = time.perf_counter()
    sampler.run(A + n_samp, max_steps=W)
    ctx.sync()
    t_wsteps = time.perf_counter() - t

    it0 = sampler.iterations()
    # sweep events on every n-th step (each event pair is a stream barrier: ~1-2 % of a step)
    ctx.set_profiling(max(1, min(8, K // 16)))
    i0 = sampler.info()
    R.barrier()
    t0 = time.perf_counter()
    w0 = time.monotonic_ns()
    sampler.run(A + n_samp, max_steps=K)
    ctx.sync()
    R.barrier()
    elapsed = time.perf_counter() - t0
    w1 = time.monotonic_ns()
    ctx.set_profiling(False)
    i1 = sampler.info()
    it1 = sampler.iterations()

    grads = i1["grad_evals"] - i0["grad_evals"]
    sweeps = i1["sweeps"] - i0["sweeps"]
    shard_sweeps = i1["shard_sweeps"] - i0["shard_sweeps"]
    sweep_ms = i1["sweep_ms"] - i0["sweep_ms"]
    elapsed = float(R.allreduce(np.array([elapsed]), "max")[0])
    grads = int(R.allreduce(np.array([float(grads)]))[0])
    roof = sweep_roofline(a, rows_per_shard, sweep_ms, sweeps, shard_sweeps)
    rec = {"metric": f"gradient evals/sec (whole node), {a.family} regression N={a.rows:.0e} d={a.d}".replace("e+0", "e"),
           "value": grads / elapsed, "unit": "gradient evals/sec", "n_gpus": world, "steps": K, "warmup": W,
           "ms_per_step": 1e3 * elapsed / K, "roofline": roof,
           "config": {"workload": f"bayesian {a.family} regression, {a.shards} subposterior shards + consensus combine",
                      "rows": int(a.rows), "d": a.d, "shards": a.shards, "shards_per_gpu": spr,
                      "chains_per_shard": a.chains, "num_warmup": A, "stepsize_jitter": a.stepsize_jitter,
                      "nuts_criterion": a.nuts_criterion, "parallelism": f"shard-dp{world}"},
           "timed_window_monotonic_ns": [w0, w1]}
    if a.throughput_only:
        # the timed window only (the sampler still adapting: a step costs one sweep whatever the phase)
        rec["config"]["workload"] = f"bayesian {a.family} regression, {a.shards} subposterior shards, throughput only"
        sampler.close()
        model.close()
        R.barrier()
        return rec if rank == 0 else None

    # ---- ESS phase (not part of `value`): every chain of every rank runs on to the same
    # number of post-warmup draws, n_post = max(ND, the most any chain already has), so the
    # consensus pairs draw i of chain c of every shard (equal-length chains, Stan's
    # multi-chain estimator).  Its time counts in the ESS/s denominators.
    n_post = int(R.allreduce(np.array([max(ND, int(it1.max()) - A)], np.float64), "max")[0])
    assert a.ess_budget_s is None or world == 1, "--ess-budget-s: one process"
    t = time.perf_counter()
    while True:                      # bounded batches with a progress line (long phases under the 2.19 criterion)
        sampler.run(A + n_post, max_steps=2000)
        its = sampler.iterations()
        R.log(f"{tag} draws {time.perf_counter() - t:.0f}s: post-warmup min {its.min() - A} of {n_post}", every_s=30)
        if its.min() >= A + n_post:
            break
        if a.ess_budget_s is not None and time.perf_counter() - t > a.ess_budget_s:
            n_post = int(its.min()) - A          # the draws every chain has: the phase ends here
            R.log(f"ESS phase stopped at the {a.ess_budget_s:.0f} s budget with {n_post} post-warmup draws per chain")
            break
    ctx.sync()
    R.barrier()
    t_post = time.perf_counter() - t
    info = sampler.info()
    C = a.chains
    # the draws stay in HBM: library buffer -> device tensor -> RCCL all-gather -> device combine
    dev = torch.device("cuda", R.local_rank) if torch.cuda.is_available() else None
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
        R.log(f"draws of shards {shard_ids} written to {a.dump_draws}")
    t = time.perf_counter()
    allp_dev = sdist.all_gather_partitions(local, a.shards, as_tensor=True)   # one all-gather (RCCL on GPUs)
    if allp_dev.is_cuda:
        torch.cuda.synchronize(allp_dev.device)
    t_gather = time.perf_counter() - t
    allp = list(allp_dev.cpu().numpy())          # host copies: Laplace start point, CPU combine, ESS
    eps, _ = sampler.adaptation()
    divergent = int(R.allreduce(np.array([float(info["divergent"])]))[0])
    lf = float(R.allreduce(np.array([stats[:, 3].mean() / world]))[0])
    # full-data posterior reference (logistic, flat priors): MAP + inverse Hessian from the
    # GPU gradient summed over every shard of every rank (tools/laplace.py)
    fulldata = None
    if a.family == "logistic" and not a.no_accuracy:
        from tools import laplace as L
        t = time.perf_counter()
        pooled = np.hstack([x[:-1] for x in allp])
        fm, fc, finfo = L.laplace(model, list(range(spr)), pooled.mean(1), pooled.std(1) / np.sqrt(a.shards),
                                  reduce=R.allreduce if R.dist else None)
        fulldata = ("vs_fulldata_laplace", fm, np.sqrt(np.diag(fc)), a.d + 1)
        R.log(f"full-data Laplace reference in {time.perf_counter() - t:.1f}s")
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
        R.allreduce(acc)
        AtA, Aty, yty, ntot = acc[:k * k].reshape(k, k), acc[k * k:k * k + k], acc[-2], acc[-1]
        mean = np.linalg.solve(AtA, Aty)
        rss = yty - 2 * mean @ Aty + mean @ AtA @ mean
        nu = ntot - k - 1
        fulldata = ("vs_fulldata_exact", mean, np.sqrt(np.diag(nu / (nu - 2.0) * rss / nu * np.linalg.inv(AtA))), k)
    second = None
    if a.second_criterion != "none" and a.second_criterion != a.nuts_criterion:
        second = _second_run(a, R, ctx, model, shard_ids, gather_ids, A, left)
    sampler.close()
    model.close()
    if rank != 0:
        return None

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
    t_sampling = t_wsteps + elapsed + t_post
    truth = np.concatenate([[0.0], engine.Model.gen_beta(a.seed, a.d)])
    if a.family == "linear":
        truth = np.concatenate([truth, [1.0]])                # sigma
    csd = comb[:-1].std(1)

    def zz(err, sd):
        z = err / sd
        return {"mean_z2": float((z ** 2).mean()), "max_abs_z": float(np.abs(z).max())}

    accuracy = {"vs_generating_params": zz(comb[:-1].mean(1) - truth, csd)}
    if fulldata is not None:
        name, fm, fsd, k = fulldata
        accuracy[name] = {"consensus": zz(comb[:k].mean(1) - fm, fsd),
                          "consensus_joint_lp": zz(comb_joint[:k].mean(1) - fm, fsd),
                          "sd_ratio_median": float(np.median(comb[:k].std(1) / fsd)),
                          "truth": zz(truth[:k] - fm, fsd)}
    rec["config"]["post_warmup_draws_per_chain"] = n_post
    rec.update({
        "ess_per_sec": ess_c / (t_adapt + t_sampling), "min_ess": ess_c,
        "ess_per_sec_floored": min_ess(comb[:-1], floor=True) / (t_adapt + t_sampling),
        "ess_per_sec_post_warmup": ess_c / t_sampling,
        "subposterior_min_ess_shard0": min_ess(allp[0][:-1]),
        "accuracy": accuracy,
        "stepsize_median": float(np.median(eps)), "stepsize_range": [float(eps.min()), float(eps.max())],
        "treedepth_mean": float(stats[:, 2].mean()), "leapfrogs_per_transition": lf, "divergent": divergent,
        "combine": {"gpu_ms": float(np.median(comb_ms[1:])), "host_buffers_ms": comb_host_ms,
                    "all_gather_ms": 1e3 * t_gather, "P": P, "draws": C * n_post,
                    "draws_on_device": bool(getattr(allp_dev, "is_cuda", False)), "consensus_sha16": sha16(comb)},
        "setup_s": {"datagen": t_gen, "adaptation": t_adapt, "post_warmup_draws": t_post},
        "_grad_evals_total": info["grad_evals"] * world,
    })
    if second is not None:
        rec["ess_second_criterion"] = _second_record(a, ctx, second, fulldata, min_ess)
    if cpu_seconds:
        try:
            cpu = cpu_baseline(a.d, rows_per_shard, a.shards, cpu_seconds, a.family)
            # the measured CPU gradient rate x this run's ESS per gradient evaluation (warmup
            # included): the CPU twin runs the same NUTS transitions (tests/test_gpu_nuts.py)
            cpu["ess_per_sec"] = cpu["value"] * ess_c / rec["_grad_evals_total"]
            cpu["combine_ms"] = cpu_combine(allp)
            rec["cpu_baseline"] = cpu
        except Exception as e:          # the GPU line is still printed
            rec["cpu_baseline"] = {"error": repr(e)}
    return rec


def _second_run(a, R, ctx, model, shard_ids, gather_ids, A, left):
    """The same data, warmup length and shard RNG keys under another NUTS criterion / jitter,
    in bounded step batches under a wall-time budget (--second-criterion)."""
    from stark_amd import dist as sdist
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
            done = R.agree(its.min() >= target)
            over = not R.agree(not (time.perf_counter() - t > a.second_budget_s or left() < 150))
            R.log(f"second criterion {a.second_criterion}: {time.perf_counter() - t:.0f}s, transitions min "
                  f"{its.min()} of {target}", every_s=30)
            if done or over:
                break
        ctx.sync()
        R.barrier()
        phase[target] = time.perf_counter() - t_ph
        if not done:
            completed = False
            break
    if not completed:
        out = {"status": f"stopped at the {a.second_budget_s:.0f} s budget", "iterations_min": int(its.min())}
    else:
        loc2, st2 = {}, []
        for s_ in range(len(shard_ids)):
            loc2[gather_ids[s_]] = s2.draws_device(s_)
            st2.append(s2.draws(s_)[1])
        out = {"allp": sdist.all_gather_partitions(loc2, a.shards, as_tensor=True), "t_adapt": phase[A],
               "t_post": phase[A + ND2], "nd": ND2, "lf": float(np.vstack(st2)[:, 3].mean()),
               "div": s2.info()["divergent"]}
    s2.close()
    return out


def _second_record(a, ctx, second, fulldata, min_ess):
    from stark_amd import engine
    head = {"nuts_criterion": a.second_criterion, "stepsize_jitter": a.second_jitter}
    if "allp" not in second:
        return {**head, **second}
    comb2_t, _ = engine.consensus(second["allp"], ctx, separate_lp=True)
    comb2 = comb2_t.cpu().numpy()
    ess2 = min_ess(comb2[:-1], n=second["nd"])
    out = {**head, "ess_per_sec": ess2 / (second["t_adapt"] + second["t_post"]), "min_ess": ess2,
           "post_warmup_draws_per_chain": second["nd"], "leapfrogs_per_transition": second["lf"],
           "divergent": second["div"], "seconds": [second["t_adapt"], second["t_post"]]}
    if fulldata is not None:
        name, fm, fsd, k = fulldata
        z = (comb2[:k].mean(1) - fm) / fsd
        out[name + "_mean_z2"] = float((z ** 2).mean())
    return out


# ------------------------------------------------------------------ sub-records
def schools_record(ctx, cpu_seconds, left):
    """BASELINE configs[1] (example/stark_ex.py 8-schools, 4096 chains, Stan defaults) on this
    rank's GPU, with the reference example's CPU path beside it (tools/bench_schools.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_schools
    s = bench_schools.run(ctx=ctx)
    rec = {"config": "8 schools x 4096 chains, Stan defaults 1000+1000, 1 GPU",
           "leapfrogs_per_transition": s["leapfrogs_per_transition"], "divergent": s["divergent"],
           "roofline_frac_fp64": s["roofline"]["frac"], "min_ess": s["min_ess"],
           "ess_per_sec_sampling": s["ess_per_sec_sampling"], "grads_per_sec_whole_run": s["grad_evals_per_sec_whole_run"]}
    if cpu_seconds:
        if left() > 40:
            c = cpu_baseline_schools(cpu_seconds)
            rec["cpu_baseline"] = {"value": c["value"], "ess_per_sec": c["ess_per_sec"], "cores": c["cores"],
                                   "kind": c["kind"], "weighted_iter5000_value": c["weighted_iter5000"]["value"]}
        else:
            rec["cpu_baseline"] = {"skipped": "deadline"}
    rec["ess_per_sec_whole_run"] = s["ess_per_sec_whole_run"]
    rec["value"] = s["value"]
    return rec, s


def compact_consensus(rec, keep_cfg=True):
    """A consensus-job record as a compact sub-record: value (and ESS) last."""
    r = rec["roofline"]
    out = {}
    if keep_cfg:
        c = rec["config"]
        out["config"] = (f"{c['workload'].split(',')[0]} N={c['rows']:.0e} d={c['d']}, {c['shards']} shards x "
                         f"{c['chains_per_shard']} chains, {c['nuts_criterion']} jitter {c['stepsize_jitter']:g}, "
                         f"warmup {c['num_warmup']}").replace("e+0", "e")
    out.update({"n_gpus": rec["n_gpus"], "ms_per_step": rec["ms_per_step"],
                "roofline": {"frac": r["frac"], "achieved": r["achieved"], "avg_launch_ms": r["avg_launch_ms"],
                             "kernel": r["kernel"]}})
    if "min_ess" in rec:
        out["draws_per_chain"] = rec["config"]["post_warmup_draws_per_chain"]
        out["leapfrogs_per_transition"] = rec["leapfrogs_per_transition"]
        out["divergent"] = rec["divergent"]
        out["consensus_sha16"] = rec["combine"]["consensus_sha16"]
        for k, v in rec["accuracy"].items():
            if k.startswith("vs_fulldata"):
                out[k + "_mean_z2"] = v["consensus"]["mean_z2"]
        if "cpu_baseline" in rec:
            cb = rec["cpu_baseline"]
            out["cpu_baseline"] = ({k: cb[k] for k in ("value", "ess_per_sec", "cores", "kind")} if "value" in cb
                                   else cb)
        out["min_ess"] = rec["min_ess"]
        out["ess_per_sec"] = rec["ess_per_sec"]
    out["value"] = rec["value"]
    return out


def compact_fulldata(rec):
    r = rec["roofline"]
    return {"config": f"full-data logistic d={rec['config']['d']}, {rec['config']['chains']} chains, "
                      f"{rec['config']['rows_per_gpu']:.2g} rows/GPU, per-leapfrog all-reduce",
            "n_gpus": rec["n_gpus"], "ms_per_step": rec["ms_per_step"],
            "roofline": {"bound": r["bound"], "frac": r["frac"], "achieved": r["achieved"], "unit": r["unit"],
                         "avg_launch_ms": r["avg_launch_ms"]},
            "chains_sha16_per_rank": rec.get("chains_sha16_per_rank"), "value": rec["value"]}


def sub_args(a, **kw):
    d = dict(vars(a))
    d.update(dict(second_criterion="none", dump_draws=None, ess_budget_s=None, shard_offset=0,
                  throughput_only=False, no_accuracy=False))
    d.update(kw)
    return argparse.Namespace(**d)


def run_plan(a, R):
    """What each record of this run puts on each rank, built with the same collectives and skip
    decisions the run takes (--launch-check: the N-rank schedule without any GPU work)."""
    def shards_of(shards):
        assert shards % R.world == 0, "shards must divide evenly over GPUs"
        spr = shards // R.world
        got = R.allreduce(np.array([float(spr)]))[0]       # every rank's share, summed: all shards placed
        return {"n_gpus": R.world, "shards_per_gpu": spr, "shards_placed": int(got)}

    plan = {"headline": {**shards_of(a.shards), "rows_per_shard": int(a.rows) // a.shards}}
    if a.throughput_only:
        return plan
    if not a.no_schools:
        plan["configs1_schools"] = {"n_gpus": 1, "ranks": [0]}
    if not a.no_other_configs:
        if R.agree(True):
            plan["configs2_linear"] = {**shards_of(8), "rows_per_shard": int(a.cfg2_rows) // 8}
        if R.agree(True):
            plan["configs3_chains1"] = shards_of(a.shards)
        if R.agree(True):
            rows = int(a.cfg4_rows_per_gpu)
            plan["configs4_fulldata"] = {"n_gpus": R.world, "rows_per_gpu": rows,
                                         "rows_total": int(R.allreduce(np.array([float(rows)]))[0]),
                                         "exchange": "all_reduce of the [64 x (Dp+1)] block per leapfrog"}
    return plan


# ------------------------------------------------------------------ main
def main():
    a = parse()
    refuse = check_world(a.gpus, os.environ)
    if refuse:
        sys.exit(refuse)
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    t_start = time.perf_counter()

    def left():                        # seconds of the run's wall-time budget still unspent
        return a.deadline_s - (time.perf_counter() - t_start)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # c10d's per-rank rendezvous warnings would fill the stderr the driver keeps beside the line
    os.environ.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")
    # STARK_DIST_BACKEND=gloo + more ranks than GPUs: a rehearsal of the N-rank path on one
    # GPU (ranks share devices round-robin); the driver's runs use RCCL, one rank per GPU
    backend = os.environ.get("STARK_DIST_BACKEND", "nccl")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    ndev = torch.cuda.device_count()          # counts devices without initialising the GPU
    refuse = check_devices(backend, os.environ, ndev)
    if refuse:
        sys.exit(refuse)
    dist = None
    # STARK_FORCE_DIST=1: a process group even at world size 1 (exercises the RCCL collectives of
    # the N-rank path on one GPU: all-reduces, the draw all-gather, the Laplace gradient sums)
    if world > 1 or os.environ.get("STARK_FORCE_DIST") == "1":
        import torch.distributed as dist
        if ndev:
            local_rank %= ndev
            os.environ["LOCAL_RANK"] = str(local_rank)      # what stark_amd.dist and bench_fulldata read
            torch.cuda.set_device(local_rank)
        # ranks other than 0 wait in a collective while rank 0 runs its own records (the
        # combine, the CPU baselines, configs[1]): a timeout well past that, not the 10-minute default
        pg_timeout = datetime.timedelta(seconds=max(1800, 3 * a.deadline_s))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)
    R = Ranks(dist, world, rank, local_rank, local_rank if ndev else None)
    if a.launch_check:
        devs = rank_devices(R)
        plan = run_plan(a, R)
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "world_size": world,
                              "dist_backend": dist.get_backend() if dist else None, "rank_devices": devs,
                              "plan": plan}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    from stark_amd import engine
    ctx = engine.Context(local_rank)
    devs = rank_devices(R)
    cpu_s = None if a.no_cpu_baseline else a.cpu_baseline_seconds
    head = consensus_job(a, R, ctx, left, cpu_seconds=cpu_s)
    detail = {"headline": head}

    schools = others = None
    if not a.throughput_only:
        if rank == 0 and not a.no_schools:   # configs[1] is a one-GPU config: rank 0's GPU
            try:
                schools, detail["configs1_schools"] = schools_record(ctx, cpu_s, left)
            except Exception as e:          # the main line is still printed
                schools = {"error": repr(e)}
        if not a.no_other_configs:
            others = {}

            def sub(name, cost, fn):
                if not R.agree(left() > cost):
                    others[name] = {"skipped": f"deadline: {left():.0f} s of --deadline-s {a.deadline_s:.0f} left, "
                                               f"needs ~{cost} s"}
                    return
                try:
                    out = fn()
                except Exception as e:      # the main line is still printed
                    out = {"error": repr(e)}
                    R.log(f"{name}: {e!r}")
                if rank == 0:
                    others[name] = out

            def cfg2():
                # configs[2] under pystan 2's own settings (stark/stark.py:48, 60-63): Stan 2.19.1's
                # NUTS criterion, stepsize_jitter 0, iter = 2000 -> 1000 warmup + 1000 draws per chain
                s = sub_args(a, family="linear", rows=a.cfg2_rows, d=50, shards=8, chains=16,
                             nuts_criterion="stan2.19", stepsize_jitter=0.0, adapt_iters=a.cfg2_adapt,
                             ess_draws=a.cfg2_draws, steps=300, warmup=20, traffic_json="")
                r = consensus_job(s, R, ctx, left, cpu_seconds=cpu_s)
                detail["configs2_linear"] = r
                return compact_consensus(r) if r else None

            def cfg3():
                # configs[3] at the driver API's default (stark/stark.py:62-63): ONE chain per shard
                # -> the VALU k_sweep3 (HBM-bound), throughput only
                s = sub_args(a, chains=1, throughput_only=True, steps=200, warmup=10, traffic_json="")
                r = consensus_job(s, R, ctx, left)
                detail["configs3_chains1"] = r
                return compact_consensus(r, keep_cfg=False) if r else None

            def cfg4():
                # configs[4]: full-data logistic d = 1000, 64 chains, the rows split over ALL ranks,
                # the [64 x (Dp+1)] gradient block all-reduced every leapfrog (RCCL)
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                import bench_fulldata
                r = bench_fulldata.run(a.cfg4_rows_per_gpu, steps=a.cfg4_steps, warmup=2, seed=a.seed)
                detail["configs4_fulldata"] = r
                return compact_fulldata(r) if r else None

            sub("configs2_linear", 110, cfg2)
            sub("configs3_chains1", 40, cfg3)
            sub("configs4_fulldata", 45, cfg4)
    if rank == 0 and a.detail_json:
        with open(a.detail_json, "w") as f:
            json.dump(detail, f, default=float)
    if rank == 0:
        print(json.dumps(headline_line(a, head, devs, dist, schools, others)), flush=True)
    ctx.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def headline_line(a, h, devs, dist, schools, others):
    """The bench line: the contract's keys first, the ESS half of the metric LAST."""
    line = {k: h[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step")}
    line.update({"higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                 "data": "synthetic (Philox in HBM, SURVEY 8d)", "config": h["config"],
                 "world_size": h["n_gpus"], "dist_backend": dist.get_backend() if dist else None,
                 "rank_devices": devs, "roofline": h["roofline"],
                 "timed_window_monotonic_ns": h["timed_window_monotonic_ns"],
                 "keys": "DESIGN.md section 4, bench line keys"})
    if a.throughput_only:
        return line
    line["cpu_baseline"] = h.get("cpu_baseline")
    for k in ("combine", "setup_s", "stepsize_median", "stepsize_range", "treedepth_mean", "leapfrogs_per_transition",
              "divergent", "ess_second_criterion", "subposterior_min_ess_shard0", "ess_per_sec_floored",
              "ess_per_sec_post_warmup"):
        if k in h:
            line[k] = h[k]
    line["other_configs"] = others
    line["configs1_schools"] = schools
    acc = h["accuracy"]
    line["accuracy"] = {"vs_generating_params": acc["vs_generating_params"]}
    for k, v in acc.items():
        if k.startswith("vs_fulldata"):
            line["accuracy"][k] = {"consensus_joint_lp": v["consensus_joint_lp"],
                                   "sd_ratio_median": v["sd_ratio_median"], "consensus": v["consensus"]}
    line["min_ess"] = h["min_ess"]
    line["ess_per_sec"] = h["ess_per_sec"]
    return line


if __name__ == "__main__":
    main()
