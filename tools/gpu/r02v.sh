#!/bin/bash
# round 2, call v: sampled sweep events; one shard per GPU (the 8-GPU run's per-rank work) and
# the default N=1 bench line
set -o pipefail
mkdir -p gpurun_out/r02v
O=gpurun_out/r02v
timeout -k 10 300 python3 bench.py --rows 1.25e7 --shards 1 --steps 300 --warmup 20 --no-cpu-baseline --no-accuracy > $O/bench_1shard.json 2> $O/bench_1shard.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_1shard.json').read().strip().splitlines()[-1]); print('1shard', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('N1', d['value'], d['ms_per_step'], d['ess_per_sec'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
