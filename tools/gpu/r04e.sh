#!/bin/bash
# round 4, call e: PC sampling of the fused 8-schools kernel (where a leapfrog's cycles go).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e
mkdir -p $O
timeout -s KILL 150 rocprofv3 -L > $O/list.txt 2>&1; grep -i -B2 -A12 "pc.sampl\|PC Sampling" $O/list.txt | head -60
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d $O/ps_st -o ps --output-format csv -- python3 tools/bench_schools.py --warmup 300 --samples 300 > $O/ps_st.log 2>&1
echo "stochastic rc=$?"; tail -3 $O/ps_st.log; ls -la $O/ps_st 2>/dev/null | head
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $O/ps_ht -o ps --output-format csv -- python3 tools/bench_schools.py --warmup 300 --samples 300 > $O/ps_ht.log 2>&1
echo "host_trap rc=$?"; tail -3 $O/ps_ht.log; ls -la $O/ps_ht 2>/dev/null | head
