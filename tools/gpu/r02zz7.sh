#!/bin/bash
# round 2 re-entry: the default bench line under the reference's Stan 2.19 U-turn criterion
set -o pipefail
mkdir -p gpurun_out/r02zz7
O=gpurun_out/r02zz7
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python3 bench.py --nuts-criterion stan2.19 --steps 300 --no-cpu-baseline > $O/bench_219.json 2> $O/bench_219.err || exit 2
python3 -c "import json; d=json.loads(open('$O/bench_219.json').read().strip().splitlines()[-1]); print('stan2.19', d['value'], d['ess_per_sec'], d['leapfrogs_per_transition'], d['accuracy']['vs_fulldata_laplace']['consensus'], d['setup_s'])"
