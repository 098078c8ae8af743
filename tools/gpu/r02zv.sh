#!/bin/bash
# round 2 re-entry: the 8-shard consensus against a full-data NUTS run on the same 1e8 rows
set -o pipefail
mkdir -p gpurun_out/r02zv
O=gpurun_out/r02zv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u tools/fulldata_nuts_check.py --out $O/fulldata_nuts_check.json > $O/check.json 2> $O/check.log
rc=$?; echo "rc=$rc"; tail -3 $O/check.log
