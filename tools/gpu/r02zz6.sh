#!/bin/bash
# round 2 re-entry: rehearsal of the driver's 8-rank bench on one GPU (gloo; the 8 ranks share
# the device, one 1.25e7-row shard each): rank -> shard mapping, the 8-way draw gather, the
# cross-rank Laplace gradient sums and rank 0's combine, at the headline shapes
set -o pipefail
mkdir -p gpurun_out/r02zz6
O=gpurun_out/r02zz6
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export STARK_DIST_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 8 --steps 50 --warmup 5 --adapt-iters 100 --ess-draws 100 --no-cpu-baseline > $O/bench_8rank.json 2> $O/bench_8rank.err
rc=$?; echo "bench 8rank rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_8rank.err; exit 2; }
python3 -c "import json; d=json.loads(open('$O/bench_8rank.json').read().strip().splitlines()[-1]); print('N8 rehearsal', d['value'], d['n_gpus'], d['config']['shards_per_gpu'], d['ess_per_sec'], d['accuracy']['vs_fulldata_laplace']['consensus'], d['combine']['all_gather_ms'])"
