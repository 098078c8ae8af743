#!/bin/bash
# round 2, call t: 8-schools config 2 with the previous nuts.hip (non-inlined NutsChain
# constructor) vs the current one, same box; then the consensus tests
set -o pipefail
mkdir -p gpurun_out/r02t
O=gpurun_out/r02t
STARK_HIP_LIB=$PWD/tools/_bin/libstark_oldnuts.so timeout -k 10 300 python3 tools/bench_schools.py > $O/schools_old.json 2> $O/schools_old.err || exit 2
timeout -k 10 300 python3 tools/bench_schools.py > $O/schools_new.json 2> $O/schools_new.err || exit 3
for v in old new; do python3 -c "import json,sys; d=json.loads(open('$O/schools_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'])"; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_consensus.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest.log
