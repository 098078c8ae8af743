#!/bin/bash
# round 5, call m: k_sweep16 with the DPP VALU tail in the product -- kernel parity tests, A/B
# against the previous commit's kernel (s16-old), then the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 tools/_bin/sweep16_ab 12500000 8 7 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity s16-old|median" $O/ab_d100.log; [ $rc -eq 0 ] || exit 5
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ess_per_sec'], r['frac'], r['avg_launch_ms'], d['configs1_schools']['value'], d['other_configs']['configs2_linear']['roofline']['frac'], d['other_configs']['configs3_chains1']['roofline']['frac'])"
