#!/bin/bash
# round 4, call c: k_sweep16 variants (tools/sweep16_variants.hip) A/B at d = 100 and 50, plus
# their PMC (clock, MFMA busy, VALU instructions).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 5 8 100 3 > $O/ab_d100.log 2>&1
rc=$?; echo "d100 rc=$rc"; tail -9 $O/ab_d100.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 100 tools/_bin/sweep16_ab 1250000 8 5 20 50 2 > $O/ab_d50_lin.log 2>&1
rc=$?; echo "d50 lin rc=$rc"; tail -9 $O/ab_d50_lin.log; [ $rc -eq 0 ] || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/sweep16_ab 12500000 8 1 3 100 3 > $O/pmc_sq.log 2>&1 || exit 9
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/pmc.json > $O/pmc_summary.txt 2>&1; grep sweep $O/pmc_summary.txt
timeout -k 10 200 tools/_bin/sweep16_ab 12500000 8 5 8 100 3 > $O/ab_d100_2.log 2>&1
rc=$?; echo "d100 (2) rc=$rc"; tail -9 $O/ab_d100_2.log
