#!/bin/bash
# round 2, call b: fp64 MFMA ceiling with in-kernel clock; sweep variants e / r / r2 at the
# bench geometry; parity tests on the r variant; bench with r
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 120 tools/_bin/mfma_ceiling 20000 > $O/r02b_mfma_ceiling.log 2>&1 || exit 1
for v in e r r2; do
  STARK_SWEEPM=$v timeout -k 10 180 tools/_bin/sweep_micro 12500000 8 100 10 16 > $O/r02b_micro_$v.log 2>&1 || exit 2
done
STARK_SWEEPM=r timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_nuts.py -m gpu -q --timeout 200 --timeout-method thread -k "sweep or placement or logistic or oracle" > $O/r02b_pytest_r.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit 3
STARK_SWEEPM=r timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r02b_bench_r.json 2> $O/r02b_bench_r.err
echo "bench rc=$?"
