#!/bin/bash
# round 2, call u: 8-schools config 2 with the criterion-sized tree stack; GPU tests
set -o pipefail
mkdir -p gpurun_out/r02u
O=gpurun_out/r02u
timeout -k 10 300 python3 tools/bench_schools.py > $O/schools.json 2> $O/schools.err || exit 3
python3 -c "import json; d=json.loads(open('$O/schools.json').read().strip().splitlines()[-1]); print('schools', d['value'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_nuts.py tests/test_gpu_kernels.py tests/test_gpu_consensus.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest.log
