#!/bin/bash
# round 4, call p: PMC after the round-4 changes -- pass F / pass B (gemm_ab harness: the product
# pass F, round 3's, the tile variants, pass B; medians per kernel) and the fused 8-schools kernel
# (the two passes of r03ab, same run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04p
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc_gemm -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_gemm.log 2>&1
rc=$?; echo "pmc gemm rc=$rc"; [ $rc -eq 0 ] || exit 4
python3 tools/pmc_arms.py $O/pmc_gemm/pmc_counter_collection.csv --json $O/gemm_pmc.json
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_schools -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools.log 2>&1
rc=$?; echo "pmc schools rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmc_schools2 -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools2.log 2>&1
rc=$?; echo "pmc schools2 rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 tools/schools_pmc.py $O/pmc_schools/pmc_counter_collection.csv $O/pmc_schools2/pmc_counter_collection.csv --run "tools/bench_schools.py --warmup 100 --samples 100 (4096 chains, 4 per wave), two PMC passes" --json $O/schools_pmc_r04.json | head -30
