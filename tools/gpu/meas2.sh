#!/bin/bash
# Round-1 measurements: headline bench (configs[3]), linear (configs[2]), 8-schools x 4096 (configs[1]),
# full-data kernels (configs[4]) under rocprofv3.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/bench_schools.py > gpurun_out/bench_schools.log 2>&1
rc=$?; echo "schools rc=$rc"; tail -1 gpurun_out/bench_schools.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --family linear --rows 1e7 --d 50 --no-cpu-baseline > gpurun_out/bench_linear.log 2>&1
rc=$?; echo "linear rc=$rc"; tail -1 gpurun_out/bench_linear.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd -o run -- python3 tools/bench_fulldata.py --rows-per-gpu 1e7 --steps 10 --warmup 2 > gpurun_out/prof_fd.log 2>&1
rc=$?; echo "fd trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE -d gpurun_out/pmc_fd_mfma -o run -- python3 tools/bench_fulldata.py --rows-per-gpu 1e7 --steps 3 --warmup 1 > gpurun_out/pmc_fd_mfma.log 2>&1
rc=$?; echo "fd mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fd_fetch -o run -- python3 tools/bench_fulldata.py --rows-per-gpu 1e7 --steps 3 --warmup 1 > gpurun_out/pmc_fd_fetch.log 2>&1
rc=$?; echo "fd fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log
