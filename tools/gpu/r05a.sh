#!/bin/bash
# round 5, call a: the bench launcher's 2-rank gloo rehearsal test, then the default bench line
# with the round-5 sub-records (schools CPU baseline, configs[2] under the reference sampler's
# settings, configs[3] at chains=1, configs[4])
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v -m gpu --timeout 500 --timeout-method thread tests/test_bench_launch.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 $O/bench.err; [ $rc -eq 0 ] || exit 5
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['frac'], r['avg_launch_ms']); print(json.dumps(d['other_configs'])[:3000]); print(json.dumps(d['configs1_schools'].get('cpu_baseline')))"
