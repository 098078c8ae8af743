#!/bin/bash
# N-rank rehearsal on one GPU (gloo, ranks share the device): full-data exchange test, the
# headline bench and the full-data bench at world size 2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts.py -m gpu -x -v --timeout 240 --timeout-method thread -k "two_ranks" > gpurun_out/pytest_2rank.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_2rank.log; [ $rc -eq 0 ] || exit $rc
export STARK_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rows 8e6 --steps 600 --adapt-iters 60 --no-cpu-baseline > gpurun_out/bench_2rank.log 2>&1
rc=$?; echo "bench 2rank rc=$rc"; tail -1 gpurun_out/bench_2rank.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 tools/bench_fulldata.py --rows-per-gpu 2e6 --steps 10 > gpurun_out/bench_fd_2rank.log 2>&1
rc=$?; echo "fd 2rank rc=$rc"; tail -1 gpurun_out/bench_fd_2rank.log
