#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/chain_diag.py --rows 2.5e7 --adapt 300 --samples 60 > gpurun_out/diag_random.log 2>&1
rc=$?; echo "diag random rc=$rc"; grep -E "iters" gpurun_out/diag_random.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/chain_diag.py --rows 2.5e7 --adapt 300 --samples 60 --init zero > gpurun_out/diag_zero.log 2>&1
echo "diag zero rc=$?"; grep -E "iters" gpurun_out/diag_zero.log | tail -3
