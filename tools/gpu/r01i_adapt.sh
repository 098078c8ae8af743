#!/bin/bash
# ESS/s against the length of Stan's warmup (num_warmup 250 / 400: final metric windows
# [100, 200) / [150, 350) after the initial transient, against [75, 100) at 150).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for A in 250 400; do
  timeout -k 10 560 python -u bench.py --adapt-iters $A --no-cpu-baseline > gpurun_out/bench_adapt$A.log 2>&1
  rc=$?; echo "bench adapt $A rc=$rc"; tail -1 gpurun_out/bench_adapt$A.log | cut -c1-1600
  [ $rc -eq 0 ] || exit $rc
done
