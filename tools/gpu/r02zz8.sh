#!/bin/bash
# round 2 re-entry: refresh the secondary configs on the final tree: configs[2] linear
# (N = 1e7, d = 50, Stan's 1000 warmup) and configs[1] 8-schools x 4096 chains
set -o pipefail
mkdir -p gpurun_out/r02zz8
O=gpurun_out/r02zz8
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 bench.py --family linear --rows 1e7 --d 50 --steps 2000 --no-cpu-baseline > $O/bench_linear.json 2> $O/bench_linear.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_linear.json').read().strip().splitlines()[-1]); print('linear', d['value'], d['ess_per_sec'], d['stepsize_per_chain'], d['divergent'], d['accuracy'].get('vs_fulldata_exact',{}).get('consensus'))"
timeout -k 10 300 python3 tools/bench_schools.py > $O/schools.json 2> $O/schools.err || exit 3
python3 -c "import json; d=json.loads(open('$O/schools.json').read().strip().splitlines()[-1]); print('schools', d['value'], d.get('ess_per_sec_sampling'))"
