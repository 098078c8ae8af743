#!/bin/bash
# round 3, call m: Philox block reuse for consecutive uniforms (NUTS tests, 8 schools), then the
# default bench line (second criterion stan2.19 at jitter 0.5, device-resident combine)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 python3 -u tools/bench_schools.py > $O/schools.json 2> $O/schools.err
rc=$?; echo "schools rc=$rc"; cut -c1-300 $O/schools.json; [ $rc -eq 0 ] || exit 5
timeout -k 10 700 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['bound'], r['frac'], r['avg_launch_ms'], d['combine']['gpu_ms'], json.dumps(d['ess_second_criterion'])[:600])"
