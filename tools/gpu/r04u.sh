#!/bin/bash
# round 4, call u: the other configurations after the sweep change -- the 8-GPU per-rank shape
# (one 1.25e7-row shard, kernel trace), configs[2] under the reference's sampler settings and
# under the default line's, configs[4] (full data, d = 1000, 64 chains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run -- python3 bench.py --rows 1.25e7 --shards 1 --steps 400 --warmup 20 --no-cpu-baseline --second-criterion none --no-schools --no-accuracy > $O/bench_1shard.json 2> $O/bench_1shard.err
rc=$?; echo "1shard rc=$rc"; [ $rc -eq 0 ] || exit 3
python3 tools/rocpd_summary.py window $O/prof1/run_results.db --kernel k_sweep16 --bench-json $O/bench_1shard.json --json $O/window_1shard.json
python3 tools/rocpd_summary.py stats $O/prof1/run_results.db > $O/stats_1shard.csv 2>&1; head -5 $O/stats_1shard.csv
rm -rf $O/prof1
timeout -k 10 300 python3 bench.py --family linear --rows 1e7 --d 50 --nuts-criterion stan2.19 --stepsize-jitter 0 --adapt-iters 1000 --ess-draws 1000 --second-criterion none --steps 20 --warmup 5 --no-schools > $O/bench_linear_refcfg.json 2> $O/bench_linear_refcfg.err
rc=$?; echo "linear refcfg rc=$rc"; [ $rc -eq 0 ] || exit 4
timeout -k 10 240 python3 bench.py --family linear --rows 1e7 --d 50 --no-schools > $O/bench_linear.json 2> $O/bench_linear.err
rc=$?; echo "linear rc=$rc"; [ $rc -eq 0 ] || exit 5
timeout -k 10 400 python3 -u tools/bench_fulldata.py --rows-per-gpu 2.5e7 --steps 10 --warmup 2 > $O/fulldata_2.5e7.json 2> $O/fulldata_2.5e7.err
rc=$?; echo "fulldata rc=$rc"; [ $rc -eq 0 ] || exit 6
python3 - <<'PY'
import json
O = "gpurun_out/r04u"
for f in ("bench_1shard", "bench_linear_refcfg", "bench_linear", "fulldata_2.5e7"):
    d = json.loads(open(f"{O}/{f}.json").read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print(f, d["value"], d.get("ms_per_step"), d.get("ess_per_sec"), r.get("frac"), r.get("avg_launch_ms"))
PY
