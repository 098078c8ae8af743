#!/bin/bash
# round 2 re-entry: bench timed window vs the kernel trace (same monotonic clock), and an N = 4
# rank rehearsal of the bench on one GPU (gloo; ranks share the device: 2 shards per rank)
set -o pipefail
mkdir -p gpurun_out/r02zt
O=gpurun_out/r02zt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 2
python3 tools/rocpd_summary.py window $O/prof/run_results.db --kernel k_sweepe --bench-json $O/bench_prof.json --json $O/window.json || exit 3
python3 tools/rocpd_summary.py stats $O/prof/run_results.db > $O/stats.csv 2>&1; head -4 $O/stats.csv
export STARK_DIST_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 100 --warmup 5 --no-cpu-baseline > $O/bench_4rank.json 2> $O/bench_4rank.err
rc=$?; echo "bench 4rank rc=$rc"; [ $rc -eq 0 ] || exit 4
python3 -c "import json; d=json.loads(open('$O/bench_4rank.json').read().strip().splitlines()[-1]); print('N4 rehearsal', d['value'], d['n_gpus'], d['ess_per_sec'], d['accuracy']['vs_fulldata_laplace']['consensus'], d['combine'])"
