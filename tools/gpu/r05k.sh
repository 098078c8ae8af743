#!/bin/bash
# round 5, call k: the transition's end through ONE continue_or_stop (consume() returns a code) on top
# of call j's single end_transition site -- NUTS / consensus GPU tests; 8-schools configs[1] with
# base (before call j), new1 (call j) and new2 (this tree), alternating; the per-rank shape of the
# 8-GPU job (1 shard of 1.25e7 rows, 16 chains: k_nuts_step's share of a step) base vs new2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nuts.py tests/test_gpu_consensus.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 4
for v in base new1 new2 base2 new1b new2b; do
  case $v in base*) L=$GRAFT_REPO_ROOT/tools/_bin/base_lib/libstark_hip.so;; new1*) L=$GRAFT_REPO_ROOT/tools/_bin/new1_lib/libstark_hip.so;; *) L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; esac
  STARK_HIP_LIB=$L timeout -k 10 120 python3 -u tools/bench_schools.py > $O/schools_$v.json 2> $O/schools_$v.err || exit 5
  python3 -c "import json; d=json.load(open('$O/schools_$v.json')); print('$v', round(d['value']/1e6,1), 'M grads/s', round(d['ess_per_sec_sampling']/1e6,2), 'M ESS/s', d['leapfrogs_per_transition'], d['posterior_mean_mu_tau'], d['divergent'])"
done
for v in base new2 base2 new2b; do
  case $v in base*) L=$GRAFT_REPO_ROOT/tools/_bin/base_lib/libstark_hip.so;; *) L=$GRAFT_REPO_ROOT/stark_amd/_lib/libstark_hip.so;; esac
  STARK_HIP_LIB=$L timeout -k 10 200 python3 -u bench.py --rows 1.25e7 --shards 1 --steps 400 --warmup 20 --throughput-only > $O/rank_$v.json 2> $O/rank_$v.err || exit 6
  python3 -c "import json; d=json.loads(open('$O/rank_$v.json').read().strip().splitlines()[-1]); print('$v rank step', round(d['ms_per_step'],4), 'ms, sweep', round(d['roofline']['avg_launch_ms'],4), 'ms')"
done
