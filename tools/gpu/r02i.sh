#!/bin/bash
# round 2, call i: full -m gpu suite, the driver's bench command (default: Stan >= 2.23
# criterion), PMC FETCH_SIZE / MFMA-busy passes of the sweep, kernel trace of a bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r02i_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/r02i_pytest_gpu.log; [ $rc -le 1 ] || exit 3
t0=$SECONDS; timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r02i_bench.json 2> $O/r02i_bench.err
rc=$?; echo "bench rc=$rc elapsed $((SECONDS-t0))s"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/r02i_pmc_fetch -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/r02i_pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit 4
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/r02i_pmc_mfma -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/r02i_pmc_mfma.log 2>&1
rc=$?; echo "pmc mfma rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r02i_prof_bench -o kt --output-format csv -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > $O/r02i_prof_bench.log 2>&1
echo "prof bench rc=$?"
