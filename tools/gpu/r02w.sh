#!/bin/bash
# round 2, call w: PMC pass on the combine's SPD inverse (what its 1.4 us per pivot is spent on)
set -o pipefail
mkdir -p gpurun_out/r02w
O=gpurun_out/r02w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/pmc1 -o run -- python3 tools/combine_bench.py > $O/combine1.json 2> $O/combine1.err || exit 2
python3 tools/rocpd_summary.py pmc $O/pmc1/run_results.db --kernel k_spd_inverse > $O/pmc1.json 2>&1; cat $O/pmc1.json | head -40
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $O/pmc2 -o run -- python3 tools/combine_bench.py > $O/combine2.json 2> $O/combine2.err || exit 3
python3 tools/rocpd_summary.py pmc $O/pmc2/run_results.db --kernel k_spd_inverse > $O/pmc2.json 2>&1; cat $O/pmc2.json | head -40
