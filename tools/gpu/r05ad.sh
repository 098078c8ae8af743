#!/bin/bash
# round 5, call ad: one rank's share of the N-GPU runs on one GPU (N = 8, 4, 2: 1, 2, 4 shards of
# 1.25e7 rows), throughput only -- the per-GPU sweep efficiency the scaling curve rests on
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ad
mkdir -p $O
for s in 1 2 4; do
  rows=$(python3 -c "print($s * 12500000)")
  timeout -k 10 240 python3 bench.py --rows $rows --shards $s --throughput-only --steps 500 --warmup 20 > $O/share_$s.json 2> $O/share_$s.err
  rc=$?; echo "shards $s rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('$O/share_$s.json').read().strip().splitlines()[-1]); r=d['roofline']; print('shards', $s, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done
