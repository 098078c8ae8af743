#!/bin/bash
# round 3, call ab: PMC of the fused 8-schools kernel after the round-3 changes (same two passes
# and run as r03k's "before"), summarised by tools/schools_pmc.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ab
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_schools -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools.log 2>&1
rc=$?; echo "pmc schools rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmc_schools2 -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools2.log 2>&1
rc=$?; echo "pmc schools2 rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 tools/schools_pmc.py $O/pmc_schools/pmc_counter_collection.csv $O/pmc_schools2/pmc_counter_collection.csv --run "tools/bench_schools.py --warmup 100 --samples 100 (4096 chains, 4 per wave), two PMC passes" --json $O/schools_pmc_after.json | head -30
