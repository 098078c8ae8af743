#!/bin/bash
# rocprofv3 evidence for the v4 sweep at the bench geometry (8 shards x 1.25e7 rows x d=100, 16 chains):
# kernel trace + stats, then one PMC pass per counter group (never combined with tracing).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RUN="python3 tools/sweep_run.py --chains 16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v4 -o run -- $RUN --steps 40 > gpurun_out/prof_v4.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- $RUN --steps 6 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- $RUN --steps 6 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o run -- $RUN --steps 6 > gpurun_out/pmc_mfma.log 2>&1
rc=$?; echo "mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --adapt-iters 150 --no-cpu-baseline > gpurun_out/bench_a150.log 2>&1
rc=$?; echo "bench a150 rc=$rc"; tail -2 gpurun_out/bench_a150.log
