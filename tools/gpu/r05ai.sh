#!/bin/bash
# round 5, call ai: where pass F's waves wait, against pass B's -- SQ wait / LDS counters per arm
# (product passes, round 4's, and pass F's ablations), for the next round's work on pass F
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai
mkdir -p $O
GEMM_AB_ABL=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/gemm_wait_pmc.json | grep k_gemm
rm -rf $O/pmc_sq
