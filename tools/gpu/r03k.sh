#!/bin/bash
# round 3, call k: k_sweepe residual v3 (fewer vector instructions) and the split residual /
# backward, A/B at the bench geometry, with PMC per arm
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 tools/_bin/sweepe_ab 12500000 8 3 8 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log; [ $rc -eq 0 ] || exit 3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc1 -o pmc --output-format csv -- tools/_bin/sweepe_ab 12500000 8 1 1 > $O/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
# 8 schools x 4096 chains (configs[1]): where the fused state machine's time goes
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_schools -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools.log 2>&1
rc=$?; echo "pmc schools rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH -d $O/pmc_schools2 -o pmc --output-format csv -- python3 tools/bench_schools.py --warmup 100 --samples 100 > $O/pmc_schools2.log 2>&1
rc=$?; echo "pmc schools2 rc=$rc"
