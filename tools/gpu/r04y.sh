#!/bin/bash
# round 4, call y: the N-rank path of bench.py after this round's changes (gather keys, the
# one-GPU sub-records skipped at N > 1), rehearsed with 2 gloo ranks sharing this GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04y
mkdir -p $O
STARK_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 5 --second-criterion none --no-cpu-baseline --no-schools > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
rc=$?; echo "2-rank rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/bench_2rank_gloo.err; exit 3; }
python3 -c "import json; d=json.loads(open('$O/bench_2rank_gloo.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['ess_per_sec'], d['config']['parallelism'], d['other_configs'], d['combine']['shards'], d['accuracy']['vs_fulldata_laplace']['consensus'])"
