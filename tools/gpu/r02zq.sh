#!/bin/bash
# round 2 re-entry: where k_sweepe's pipe idles (PMC: waits, LDS, VALU/MFMA activity), and the
# default bench line with the 250-draw ESS phase
set -o pipefail
mkdir -p gpurun_out/r02zq
O=gpurun_out/r02zq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc1 -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc2 -o pmc --output-format csv -- python3 tools/sweep_run.py --chains 16 --steps 6 > $O/pmc2.log 2>&1 || exit 3
echo pmc ok
timeout -k 10 500 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 4
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('N1', d['value'], d['ess_per_sec'], d['min_ess'], d['setup_s'], d['roofline']['frac'], d['accuracy']['vs_fulldata_laplace']['consensus'])"
