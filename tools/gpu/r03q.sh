#!/bin/bash
# round 3, call q: rehearsal of the driver's 8-rank bench on one GPU (gloo; 8 ranks share the
# device, one 1.25e7-row shard each) with this round's line: second criterion, device combine,
# cpu_baseline on rank 0 at world 8
set -o pipefail
O=gpurun_out/r03q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $O
export STARK_DIST_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 8 --steps 50 --warmup 5 --adapt-iters 100 --ess-draws 100 --second-draws 30 --cpu-baseline-seconds 4 > $O/bench_8rank.json 2> $O/bench_8rank.err
rc=$?; echo "bench 8rank rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_8rank.err; exit 2; }
python3 -c "import json; d=json.loads(open('$O/bench_8rank.json').read().strip().splitlines()[-1]); print('N8 rehearsal', d['value'], d['n_gpus'], d['config']['shards_per_gpu'], d['ess_per_sec'], d['accuracy']['vs_fulldata_laplace']['consensus'], d['combine'], d['cpu_baseline'] and d['cpu_baseline']['value'], json.dumps(d['ess_second_criterion'])[:300])"
