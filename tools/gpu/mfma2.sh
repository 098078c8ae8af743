#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/_bin/mfma_overlap > gpurun_out/overlap.log 2>&1; rc=$?; cat gpurun_out/overlap.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/sweep_micro 12500000 8 100 5 16 > gpurun_out/micro_v4b.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/micro_v4b.log
