cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run smoke python -X faulthandler -u -c "import __graft_entry__ as g; g.smoke()"
run kern python -X faulthandler -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread
run nuts python -X faulthandler -u -m pytest tests/test_gpu_nuts.py -m gpu -q --timeout 200 --timeout-method thread
run all python -X faulthandler -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
