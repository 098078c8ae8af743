#!/bin/bash
# round 2 re-entry: the C = 64 parity tests with pass B on 128-column blocks (library default)
set -o pipefail
mkdir -p gpurun_out/r02zz4
O=gpurun_out/r02zz4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q -x --timeout 300 --timeout-method thread -k "regression_lpgrad or prior_lpgrad or placement or reproducible or fulldata" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit 2
timeout -k 10 400 python3 tools/bench_fulldata.py --rows-per-gpu 2.5e7 --steps 10 --warmup 2 > $O/fulldata_2.5e7.json 2> $O/fulldata_2.5e7.err || exit 3
python3 -c "import json; d=json.loads(open('$O/fulldata_2.5e7.json').read().strip().splitlines()[-1]); print('fulldata 2.5e7', d['value'], d['roofline']['achieved'], d['ms_per_step'])"
