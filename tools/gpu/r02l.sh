#!/bin/bash
# round 2, call l: the bench's RCCL collectives on one GPU (world-1 nccl group), and the
# headline with Stan's default stepsize_jitter = 0 under the Stan >= 2.23 criterion
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out
STARK_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --rows 1e7 --steps 50 --warmup 5 > $O/r02l_bench_nccl_world1.json 2> $O/r02l_bench_nccl_world1.err
rc=$?; echo "nccl world1 rc=$rc"; [ $rc -eq 0 ] || exit 2
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --stepsize-jitter 0 --no-cpu-baseline > $O/r02l_bench_jitter0.json 2> $O/r02l_bench_jitter0.err
echo "jitter0 rc=$?"
