#!/bin/bash
# round 5, call aj: pass F with volatile A-fragment reads (two ds_read_b64 instead of one
# ds_read2st64_b64 with 2-way bank conflicts) -- A/B at both shapes and its LDS counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aj
mkdir -p $O
timeout -k 10 300 tools/_bin/gemm_ab 2000000 8 5 > $O/passF_volA_8x2e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-volA|median F" $O/passF_volA_8x2e6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/_bin/gemm_ab 25000000 1 5 > $O/passF_volA_1x25e6.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -E "parity F-volA|median F" $O/passF_volA_1x25e6.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_sq -o pmc --output-format csv -- tools/_bin/gemm_ab 2000000 8 1 > $O/pmc_sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_arms.py $O/pmc_sq/pmc_counter_collection.csv --json $O/gemm_wait_pmc.json | grep k_gemm_fwd
rm -rf $O/pmc_sq
