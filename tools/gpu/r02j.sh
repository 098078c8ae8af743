#!/bin/bash
# round 2, call j: smoke, the reference example driver, N-rank rehearsals of bench.py on one
# GPU (gloo, ranks share the device): 2 and 4 ranks logistic, 2 ranks linear
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r02j_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/r02j_smoke.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 python3 examples/stark_ex.py --seed 3 > $O/r02j_example.log 2>&1
rc=$?; echo "example rc=$rc"; [ $rc -eq 0 ] || exit 3
export STARK_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --rows 1e7 --steps 50 --warmup 5 --no-cpu-baseline > $O/r02j_bench_2rank.json 2> $O/r02j_bench_2rank.err
rc=$?; echo "bench 2rank rc=$rc"; [ $rc -eq 0 ] || exit 4
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --rows 1e7 --steps 50 --warmup 5 --no-cpu-baseline > $O/r02j_bench_4rank.json 2> $O/r02j_bench_4rank.err
rc=$?; echo "bench 4rank rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --family linear --rows 1e6 --d 50 --adapt-iters 300 --steps 50 --warmup 5 --no-cpu-baseline > $O/r02j_bench_linear_2rank.json 2> $O/r02j_bench_linear_2rank.err
rc=$?; echo "linear 2rank rc=$rc"
