#!/bin/bash
# round 5, call b (arms as built): k_sweep16 ablations at the bench geometry (d = 100 logistic, 8 x 1.25e7 rows):
# no vmcnt wait (exposed DMA latency), no residual (the residual's vector-instruction cost), both;
# interleaved A/B, then one SQ/GRBM PMC pass over the same arms (clock, MFMA busy, VALU share)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 300 tools/_bin/sweep16_ab 12500000 8 5 10 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "ab d100 rc=$rc"; grep -E "parity|median" $O/ab_d100.log; [ $rc -eq 0 ] || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/sweep16_ab 12500000 8 1 3 100 3 > $O/pmc_sq.log 2>&1 || exit 5
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/sweep16_pmc.json > $O/pmc_sq_summary.txt 2>&1; cat $O/pmc_sq_summary.txt
