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
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=180, env=_env(STARK_DIST_BACKEND="gloo"))
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["dist_backend"] == "gloo"
    assert [d[0] for d in line["rank_devices"]] == [0, 1]
    assert "starting 2 ranks" in r.stderr


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
            "--warmup", "5", "--no-cpu-baseline", "--no-schools", "--no-other-configs", "--no-accuracy"]
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
