#!/bin/bash
# round 2, call o: k_sweepq (4x4x4 four-block fp64 MFMA) variants vs k_sweepe at the bench
# geometry, then the sweep parity tests under the fastest-looking q shape
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
VARIANTS=${VARIANTS:-q q4 q16 q16c e}
PV=${PV:-q}
for v in $VARIANTS; do
  STARK_SWEEPM=$v timeout -k 10 180 tools/_bin/sweep_micro 12500000 8 100 10 16 > $O/r02o_micro_$v.log 2>&1 || exit 2
  tail -2 $O/r02o_micro_$v.log
done
STARK_SWEEPM=$PV timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 200 --timeout-method thread -k "regression_lpgrad or prior" > $O/r02o_pytest_$PV.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/r02o_pytest_$PV.log
