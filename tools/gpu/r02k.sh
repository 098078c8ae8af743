#!/bin/bash
# round 2, call k: 8-schools fused kernel PMC (instruction mix, waits), full-data configs[4]
# ESS/s under both U-turn criteria (2e6 rows, d = 1000, 64 chains), linear 2-rank rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/r02k_pmc_schools -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 200 --samples 200 > $O/r02k_pmc_schools.log 2>&1
rc=$?; echo "pmc schools rc=$rc"; [ $rc -eq 0 ] || exit 2
timeout -k 10 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $O/r02k_pmc_schools2 -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 200 --samples 200 > $O/r02k_pmc_schools2.log 2>&1
echo "pmc schools2 rc=$?"
for c in stan2.19 stan2.23; do
  timeout -k 10 400 python3 tools/bench_fulldata.py --rows-per-gpu 2e6 --adapt-iters 100 --init-radius 0.1 --steps 40 --nuts-criterion $c > $O/r02k_fulldata_$c.json 2> $O/r02k_fulldata_$c.err
  rc=$?; echo "fulldata $c rc=$rc"; [ $rc -eq 0 ] || exit 3
done
export STARK_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --family linear --rows 1e6 --adapt-iters 300 --steps 50 --warmup 5 --no-cpu-baseline > $O/r02k_bench_linear_2rank.json 2> $O/r02k_bench_linear_2rank.err
echo "linear 2rank rc=$?"
