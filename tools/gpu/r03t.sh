#!/bin/bash
# round 3, call t: k_sweepw (one wave per SIMD, two slots per wave, software-pipelined residual /
# forward and backward / operand reads) against the product k_sweepe, A/B at the bench geometry
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 tools/_bin/sweepe_ab 12500000 8 3 8 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log; [ $rc -eq 0 ] || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc1 -o pmc --output-format csv -- tools/_bin/sweepe_ab 12500000 8 1 1 > $O/pmc1.log 2>&1
echo "pmc rc=$?"
