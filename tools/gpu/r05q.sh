#!/bin/bash
# round 5, call q: the headline configuration through bench.py's own launcher as the driver's
# 8-GPU run would start it (bench.py --gpus 8), rehearsed with gloo on this one GPU (8 ranks share
# it, one 1.25e7-row shard each), against the 1-rank run of the same arguments: same consensus
# (consensus_sha16), n_gpus / world_size / rank_devices in the line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05q
mkdir -p $O
ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-schools --no-other-configs"
timeout -k 10 400 python3 -u bench.py --gpus 1 $ARGS > $O/bench_1rank.json 2> $O/bench_1rank.err
rc=$?; echo "1 rank rc=$rc"; [ $rc -eq 0 ] || exit 4
STARK_DIST_BACKEND=gloo timeout -k 10 700 python3 -u bench.py --gpus 8 $ARGS > $O/bench_8rank.json 2> $O/bench_8rank.err
rc=$?; echo "8 ranks rc=$rc"; [ $rc -eq 0 ] || exit 5
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/r05q/bench_1rank.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/r05q/bench_8rank.json").read().strip().splitlines()[-1])
for k in ("n_gpus", "world_size", "dist_backend", "value", "ess_per_sec", "min_ess"):
    print(k, a.get(k), b.get(k))
print("consensus_sha16", a["combine"]["consensus_sha16"], b["combine"]["consensus_sha16"])
print("rank_devices", b["rank_devices"])
print("accuracy", a["accuracy"]["vs_fulldata_laplace"]["consensus"], b["accuracy"]["vs_fulldata_laplace"]["consensus"])
PY
