#!/bin/bash
# round 3, call aa: refresh the secondary configs on the round-3 tree -- configs[2] linear
# (N = 1e7, d = 50, Stan's 1000 warmup, the reference's 2.19 criterion as the second run) and
# configs[4] full data (d = 1000, 64 chains, 2.5e7 rows = 200 GB on one GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 800 python3 -u bench.py --family linear --rows 1e7 --d 50 --steps 2000 --no-cpu-baseline > $O/bench_linear.json 2> $O/bench_linear.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_linear.json').read().strip().splitlines()[-1]); print('linear', d['value'], d['ess_per_sec'], d['divergent'], d['accuracy'].get('vs_fulldata_exact',{}).get('consensus'), json.dumps(d.get('ess_second_criterion'))[:300])"
timeout -k 10 400 python3 -u tools/bench_fulldata.py --rows-per-gpu 2.5e7 --steps 10 --warmup 2 > $O/fulldata_2.5e7.json 2> $O/fulldata_2.5e7.err || exit 3
cut -c1-400 $O/fulldata_2.5e7.json
