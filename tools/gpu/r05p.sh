#!/bin/bash
# round 5, call p: 8 schools x 4096 chains after the single end_transition site (167-170 VGPRs):
# 4 chains per wave (one wave per SIMD) against 2 per wave (two waves per SIMD) and 1, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05p
mkdir -p $O
for v in 4 2 1 4b 2b 1b; do
  c=${v%b}
  timeout -k 10 120 python3 -u tools/bench_schools.py --chains-per-wave $c > $O/schools_cpw$v.json 2> $O/schools_cpw$v.err || exit 5
  python3 -c "import json; d=json.load(open('$O/schools_cpw$v.json')); print('cpw $v', round(d['value']/1e6,1), 'M grads/s', round(d['ess_per_sec_sampling']/1e6,2), 'M ESS/s', d['posterior_mean_mu_tau'], d['divergent'])"
done
