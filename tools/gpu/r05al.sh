#!/bin/bash
# round 5, call al: pass F without the parked eta (64 VGPRs fewer; the accumulators folded into the
# gradient sum) with and without its DMA, next to the earlier ablations -- times and clocks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05al
mkdir -p $O
GEMM_AB_ABL=1 timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 3 > $O/passF_nopark_ablations.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "median" $O/passF_nopark_ablations.log; [ $rc -eq 0 ] || exit $rc
GEMM_AB_ABL=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/gemm_nopark_pmc.json | grep k_gemm
rm -rf $O/pmc_sq
