#!/bin/bash
# Refresh the headline evidence after kernel changes: bench line, kernel trace + PMC of the bench geometry.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RUN="python3 tools/sweep_run.py --chains 16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v4b -o run -- $RUN --steps 40 > gpurun_out/prof_v4b.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_b -o run -- $RUN --steps 6 > gpurun_out/pmc_fetch_b.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma_b -o run -- $RUN --steps 6 > gpurun_out/pmc_mfma_b.log 2>&1
rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log
