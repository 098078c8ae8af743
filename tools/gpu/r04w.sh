#!/bin/bash
# round 4, call w: configs[3] under the reference's sampler settings, one rank of the 8-GPU job at
# a time (shard K alone on this GPU, its draws dumped for tools/consensus_from_dumps.py).
# usage: bash tools/gpu/r04w.sh K [K ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w
mkdir -p $O
for K in "$@"; do
  timeout -k 10 ${STEP_S:-900} python3 bench.py --rows 1.25e7 --shards 1 --shard-offset $K --nuts-criterion stan2.19 --stepsize-jitter 0 --adapt-iters 1000 --ess-draws 1000 --second-criterion none --steps 20 --warmup 5 --no-schools --no-cpu-baseline --no-accuracy ${ESS_BUDGET:+--ess-budget-s $ESS_BUDGET} --dump-draws $O/shard_$K.npz > $O/shard_$K.json 2> $O/shard_$K.err
  rc=$?; echo "shard $K rc=$rc"; grep "^\[bench\]" $O/shard_$K.err | tail -2; [ $rc -eq 0 ] || exit $rc
done
