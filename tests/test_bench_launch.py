"""bench.py's multi-GPU entry point: `--gpus N` with no launcher starts N
ranks itself (torch.distributed.run, before any GPU call), under a launcher of another world
size it refuses, and the line names the world size, backend and rank devices.  CPU: gloo."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "STARK_FORCE_DIST")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks():
    """--launch-check walks the run's record schedule with the same collectives and skip
    decisions the run takes: at --gpus 2 configs[2], configs[3] chains=1 and configs[4] run on
    BOTH ranks (configs[2] 8 shards as 4 + 4, configs[4] rows per GPU x 2), configs[1] on rank 0."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=180, env=_env(STARK_DIST_BACKEND="gloo"))
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["dist_backend"] == "gloo"
    assert [d[0] for d in line["rank_devices"]] == [0, 1]
    assert "starting 2 ranks" in r.stderr
    plan = line["plan"]
    assert plan["headline"] == {"n_gpus": 2, "shards_per_gpu": 4, "shards_placed": 8, "rows_per_shard": 12_500_000}
    assert plan["configs1_schools"]["ranks"] == [0]
    assert plan["configs2_linear"]["n_gpus"] == 2 and plan["configs2_linear"]["shards_placed"] == 8
    assert plan["configs3_chains1"]["n_gpus"] == 2
    c4 = plan["configs4_fulldata"]
    assert c4["n_gpus"] == 2 and c4["rows_per_gpu"] == 25_000_000 and c4["rows_total"] == 50_000_000


def test_check_devices():
    """RCCL ranks need a GPU each -- per NODE (LOCAL_WORLD_SIZE), and a launcher may pin one GPU
    per rank through *_VISIBLE_DEVICES (each rank then sees one device).  ADVICE r5."""
    sys.path.insert(0, ROOT)
    import bench
    cd = bench.check_devices
    assert cd("gloo", {"WORLD_SIZE": "4"}, 0) is None                       # the rehearsal: any devices
    assert cd("nccl", {}, 0) is None                                        # one process
    assert "found 0" in cd("nccl", {"WORLD_SIZE": "2"}, 0)
    assert cd("nccl", {"WORLD_SIZE": "8"}, 8) is None
    assert "need 8 visible GPUs" in cd("nccl", {"WORLD_SIZE": "8"}, 4)
    # two nodes of 8: world 16, 8 GPUs per node
    assert cd("nccl", {"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8"}, 8) is None
    assert cd("nccl", {"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "16"}, 8) is not None
    # one GPU visible per rank, pinned by the launcher
    assert cd("nccl", {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2", "HIP_VISIBLE_DEVICES": "1"}, 1) is None
    assert cd("nccl", {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "1"}, 1) is None
    assert cd("nccl", {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2"}, 1) is not None


SLEEPER = """import os, sys, time
open(os.path.join(sys.argv[1], "rank%s.pid" % os.environ["RANK"]), "w").write(str(os.getpid()))
time.sleep(600)
"""

LAUNCHER = """import sys
sys.path.insert(0, sys.argv[1])
import bench
sys.exit(bench.launch_ranks(2, [sys.argv[3]], script=sys.argv[2], grace_s=5))
"""


def test_launcher_sigterm_takes_the_ranks_down(tmp_path):
    """A harness `timeout` SIGTERMs the launcher: its ranks must not outlive it."""
    import signal
    import time
    (tmp_path / "sleeper.py").write_text(SLEEPER)
    (tmp_path / "launcher.py").write_text(LAUNCHER)
    p = subprocess.Popen([sys.executable, str(tmp_path / "launcher.py"), ROOT, str(tmp_path / "sleeper.py"),
                          str(tmp_path)], env=_env(), stderr=subprocess.PIPE)
    pids = []
    for _ in range(300):
        pids = [tmp_path / f"rank{r}.pid" for r in range(2)]
        if all(f.exists() and f.read_text() for f in pids):
            break
        time.sleep(0.1)
    pids = [int(f.read_text()) for f in pids]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = os.path.exists(f"/proc/{pid}") and "Z" not in open(f"/proc/{pid}/stat").read().split()[2]
        except ProcessLookupError:
            alive = False
        assert not alive, pid


def test_schools_cpu_job_runs_every_run_in_waves():
    """with fewer cores than runs the CPU job still runs all of them, in waves."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.schools_job_plan(4, 8) == (4, [[0, 1, 2, 3]])
    assert bench.schools_job_plan(4, 3) == (3, [[0, 1, 2], [3]])
    assert bench.schools_job_plan(4, 1) == (1, [[0], [1], [2], [3]])
    assert bench.schools_job_plan(2, 1) == (1, [[0], [1]])


def test_cpu_baseline_schools_on_one_core():
    """The whole job shape on one core: 4 naive runs, 2 weighted runs (both four-school
    partitions), the job wall time summed over the waves."""
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle as O
    O.build()
    out = bench.cpu_baseline_schools(0.2, cores=1)
    for job, runs in (("naive_n4", 4), ("weighted_iter5000", 2)):
        rec = out[job]
        assert rec["runs_executed"] == runs == rec["runs_per_job"] and rec["waves"] == runs and rec["cores"] == 1
        assert rec["value"] > 0 and rec["jobs_timed"] >= 2
    assert out["ess_per_sec"] > 0


def test_gpus_mismatching_world_size_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="1", RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_rccl_ranks_need_one_gpu_each():
    # the default backend is RCCL: without N visible GPUs every rank refuses (no silent sharing)
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("host has GPUs")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=180, env=_env(STARK_DIST_BACKEND="nccl"))
    assert r.returncode != 0
    assert "visible GPUs" in r.stderr


def test_check_world():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.check_world(None, {}) is None
    assert bench.check_world(8, {}) is None
    assert bench.check_world(None, {"WORLD_SIZE": "4"}) is None
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) is None
    assert "WORLD_SIZE=4" in bench.check_world(8, {"WORLD_SIZE": "4"})


@pytest.mark.gpu
@pytest.mark.timeout(500)
def test_gpus_2_gloo_rehearsal_reproduces_one_rank_consensus():
    """`bench.py --gpus 2` on one GPU (gloo rehearsal: both ranks share the device, one shard
    each) gives the 1-rank run's consensus bit for bit: shard RNG streams and the chunk-order
    reduction do not depend on placement, and the all-gather keys the shards by global id."""
    args = ["--rows", "4e5", "--shards", "2", "--d", "10", "--adapt-iters", "60", "--ess-draws", "60", "--steps", "20",
            "--warmup", "5", "--no-cpu-baseline", "--no-schools", "--no-accuracy",
            # the other configs at rehearsal sizes: configs[2] 8 x 5e3 rows, configs[4] 2e4 rows per rank
            "--cfg2-rows", "4e4", "--cfg2-adapt", "100", "--cfg2-draws", "60", "--cfg4-rows-per-gpu", "2e4",
            "--cfg4-steps", "4"]
    lines = []
    for n in (1, 2):
        r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", str(n), *args], capture_output=True, text=True,
                           timeout=240, env=_env(STARK_DIST_BACKEND="gloo"))
        assert r.returncode == 0, r.stderr[-3000:]
        lines.append(json.loads(r.stdout.strip().splitlines()[-1]))
    one, two = lines
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["dist_backend"] == "gloo"
    assert one["combine"]["consensus_sha16"] == two["combine"]["consensus_sha16"]
    assert one["min_ess"] == two["min_ess"]
    # the other configs ran on both ranks: configs[2]'s 8 shards as 4 + 4 give the 1-rank
    # consensus bit for bit; configs[4]'s two ranks (half the rows each, one all-reduce per
    # leapfrog) hold bit-identical chains
    o1, o2 = one["other_configs"], two["other_configs"]
    assert o2["configs2_linear"]["n_gpus"] == 2 and o2["configs3_chains1"]["n_gpus"] == 2
    assert o1["configs2_linear"]["consensus_sha16"] == o2["configs2_linear"]["consensus_sha16"]
    c4 = o2["configs4_fulldata"]
    assert c4["n_gpus"] == 2 and len(c4["chains_sha16_per_rank"]) == 2
    assert c4["chains_sha16_per_rank"][0] == c4["chains_sha16_per_rank"][1]
    # the ESS half of the metric closes the line (a driver keeping the tail of stdout keeps it)
    assert list(two)[-2:] == ["min_ess", "ess_per_sec"]
    assert len(r.stdout.strip().splitlines()[-1]) < 7000
