#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 tools/_bin/sweep_micro 12500000 4 100 10 > gpurun_out/micro_d100.log 2>&1
rc=$?; echo "micro d100 rc=$rc"; cat gpurun_out/micro_d100.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/_bin/sweep_micro 25000000 4 50 10 > gpurun_out/micro_d50.log 2>&1
rc=$?; echo "micro d50 rc=$rc"; cat gpurun_out/micro_d50.log
