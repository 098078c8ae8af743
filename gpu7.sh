cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/chain_diag.py > gpurun_out/diag_random.log 2>&1
echo "diag random rc=$?"; tail -34 gpurun_out/diag_random.log
timeout -k 10 400 python -u tools/chain_diag.py --init zero > gpurun_out/diag_zero.log 2>&1
echo "diag zero rc=$?"; grep -E "iters" gpurun_out/diag_zero.log | tail -2
