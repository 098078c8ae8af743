#!/bin/bash
# round 3, call a: which VALU classes share the fp64 pipe with the f64 MFMA (tools/valu_mix.hip);
# the GPU tests touched this round; then the north_star accuracy check at N = 1e8 with the pooled
# batch MCSE (small smoke first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
O=gpurun_out/r03a
timeout -k 10 120 tools/_bin/valu_mix > $O/valu_mix.log 2>&1
rc=$?; echo "valu_mix rc=$rc"; cat $O/valu_mix.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "combine" tests/test_gpu_nuts.py::test_packed_schools_chains_bitwise_equal_unpacked tests/test_gpu_nuts.py::test_driver_weighted_matches_reference > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 200 python3 -u tools/fulldata_nuts_check.py --rows 1.6e6 --samples 100 --eval-draws 50,100 --groups 4 --full-warmup 100 --warmup 100 --out $O/fdcheck_small.json > $O/fdcheck_small.out 2> $O/fdcheck_small.err
rc=$?; echo "small check rc=$rc"; tail -3 $O/fdcheck_small.err; [ $rc -eq 0 ] || exit 3
timeout -k 10 900 python3 -u tools/fulldata_nuts_check.py --out $O/fulldata_nuts_check.json > $O/fdcheck.out 2> $O/fdcheck.err
rc=$?; echo "check rc=$rc"; tail -4 $O/fdcheck.err
