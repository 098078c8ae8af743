#!/bin/bash
# round 4, call g: the fused 8-schools kernel's cycle breakdown (diagnostic stamped build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 120 python3 -u tools/bench_schools.py > $O/schools_product.json 2>&1 || exit 2
cut -c1-200 $O/schools_product.json
timeout -k 10 120 python3 -u tools/schools_stamps.py run > $O/stamps.json 2> $O/stamps.err
rc=$?; echo "stamps rc=$rc"; cat $O/stamps.json; tail -3 $O/stamps.err
