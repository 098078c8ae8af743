#!/bin/bash
# round 3, call b: VALU classes vs the fp64 MFMA pipe; k_sweepe residual v2 A/B at the bench
# geometry; the GPU kernel + touched tests; then the north_star accuracy check at N = 1e8
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 120 tools/_bin/valu_mix > $O/valu_mix.log 2>&1
rc=$?; echo "valu_mix rc=$rc"; cat $O/valu_mix.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 240 tools/_bin/sweepe_ab 12500000 8 3 10 > $O/sweepe_ab.log 2>&1
rc=$?; echo "sweepe_ab rc=$rc"; grep -E "parity|median" $O/sweepe_ab.log; [ $rc -eq 0 ] || exit 3
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_nuts.py::test_packed_schools_chains_bitwise_equal_unpacked tests/test_gpu_nuts.py::test_driver_weighted_matches_reference > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 200 python3 -u tools/fulldata_nuts_check.py --rows 1.6e6 --samples 100 --eval-draws 50,100 --groups 4 --full-warmup 100 --warmup 100 --out $O/fdcheck_small.json > $O/fdcheck_small.out 2> $O/fdcheck_small.err
rc=$?; echo "small check rc=$rc"; tail -3 $O/fdcheck_small.err; [ $rc -eq 0 ] || exit 5
timeout -k 10 800 python3 -u tools/fulldata_nuts_check.py --out $O/fulldata_nuts_check.json > $O/fdcheck.out 2> $O/fdcheck.err
rc=$?; echo "check rc=$rc"; tail -4 $O/fdcheck.err
