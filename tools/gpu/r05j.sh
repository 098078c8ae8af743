#!/bin/bash
# round 5, call j: on_leaf with ONE end_transition call site (the merge loop exits by a flag) --
# NUTS / consensus GPU tests, then the 8-schools configs[1] run against HEAD's library (base),
# alternating; then the k_sweep16 single-register DPP tail A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for v in base new base2 new2 base3 new3; do
  case $v in base*) L=$GRAFT_REPO_ROOT/tools/_bin/base_lib/libstark_hip.so;; *) L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; esac
  STARK_HIP_LIB=$L timeout -k 10 120 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  python3 -c "import json; d=json.load(open('$O/schools_$v.json')); print('$v', round(d['value']/1e6,1), 'M grads/s', round(d['ess_per_sec_sampling']/1e6,2), 'M ESS/s', d['leapfrogs_per_transition'], d['posterior_mean_mu_tau'], d['divergent'])"
done
timeout -k 10 300 tools/_bin/sweep16_ab 12500000 8 5 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "median" $O/ab_d100.log
