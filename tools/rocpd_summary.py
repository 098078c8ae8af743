#!/usr/bin/env python3
"""Summaries of rocprofv3 rocpd (.db, SQLite) outputs, for profiles/:
  stats  <db> [--csv out]                 per-kernel call count / total / average duration (us)
  window <db> --kernel K --bench-json J   average duration of kernel K's dispatches inside the
                                          bench line's timed window (timed_window_monotonic_ns;
                                          rocprofv3 stamps dispatches on the same monotonic clock):
                                          the figure bench.py's roofline.avg_launch_ms must match
  pmc    <db> --kernel K [--json out]     per-dispatch counter values of kernel K (summed over
                                          the rows of a dispatch), their median, and the derived
                                          figures: fp64 MFMA flops (MOPS_F64 x 512), MFMA busy % of
                                          SIMD cycles, HBM bytes (FETCH_SIZE x 1024 x 2 -- the gfx950
                                          halving of 16 B/lane streaming reads, MI355X_MICROARCH.md),
                                          WRITE_SIZE bytes.
"""
import argparse
import json
import sqlite3
import statistics

p = argparse.ArgumentParser()
p.add_argument("mode", choices=["stats", "pmc", "window"])
p.add_argument("--bench-json")
p.add_argument("db")
p.add_argument("--kernel", default="k_sweepm")
p.add_argument("--csv")
p.add_argument("--json")
p.add_argument("--simds", type=int, default=1024)   # 256 CUs x 4 SIMDs
p.add_argument("--xcds", type=int, default=8)      # the db's GRBM_GUI_ACTIVE is summed over the 8 XCDs
p.add_argument("--traffic-json", help="also write bench.py's traffic record (needs FETCH_SIZE)")
p.add_argument("--rows-per-shard", type=int)
p.add_argument("--d", type=int)
p.add_argument("--shards-per-gpu", type=int)
a = p.parse_args()
cur = sqlite3.connect(a.db).cursor()

if a.mode == "window":
    line = json.loads(open(a.bench_json).read().strip().splitlines()[-1])
    w0, w1 = line["timed_window_monotonic_ns"]
    rows = list(cur.execute("select start, end from kernels where name like ? order by start", (f"%{a.kernel}%",)))
    inside = [(e - s_) * 1e-6 for s_, e in rows if s_ >= w0 and e <= w1]
    out = {"kernel": a.kernel, "dispatches_total": len(rows), "window_dispatches": len(inside),
           "bench_steps": line["steps"], "window_avg_ms": statistics.mean(inside) if inside else None,
           "window_median_ms": statistics.median(inside) if inside else None,
           "bench_avg_launch_ms": line["roofline"]["avg_launch_ms"]}
    print(json.dumps(out))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
elif a.mode == "stats":
    rows = list(cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    # top_kernels durations are in microseconds
    lines = ["kernel,calls,total_ms,avg_ms,percent"] + [
        '"%s",%d,%.3f,%.4f,%.2f' % (n, c, t / 1e3, av / 1e3, pc) for n, c, t, av, pc in rows]
    txt = "\n".join(lines)
    print(txt)
    if a.csv:
        open(a.csv, "w").write(txt + "\n")
else:
    per = {}
    for did, name, cname, val, dur in cur.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
        if a.kernel not in name:
            continue
        d = per.setdefault(did, {"duration_ns": dur})
        d[cname] = d.get(cname, 0.0) + val
    med = {}
    for k in sorted({k for d in per.values() for k in d}):
        vals = [d[k] for d in per.values() if k in d]
        med[k] = statistics.median(vals)
    out = {"kernel": a.kernel, "dispatches": len(per), "median": med}
    if "SQ_INSTS_VALU_MFMA_MOPS_F64" in med:
        out["fp64_mfma_flops_per_dispatch"] = med["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
        out["mfma_busy_pct_of_simd_cycles"] = 100.0 * med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / a.xcds * a.simds)
    if "FETCH_SIZE" in med:
        out["hbm_read_bytes_per_dispatch"] = med["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in med:
        out["hbm_write_bytes_per_dispatch"] = med["WRITE_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in med:
        out["gpu_clock_ghz"] = med["GRBM_GUI_ACTIVE"] / a.xcds / med["duration_ns"]
    print(json.dumps(out, indent=1))
    if a.traffic_json and "FETCH_SIZE" in med:
        algo = a.rows_per_shard * (8 * a.d + 4) * a.shards_per_gpu
        hb = out["hbm_read_bytes_per_dispatch"]
        json.dump({"kernel": a.kernel, "rows_per_shard": a.rows_per_shard, "d": a.d, "shards_per_gpu": a.shards_per_gpu,
                   "dispatches": len(per), "fetch_size_kb_median": med["FETCH_SIZE"],
                   "correction": "x2 (gfx950 FETCH_SIZE counts half of 16B/lane streaming reads)",
                   "hbm_bytes_per_launch": hb, "algorithmic_bytes_per_launch": algo,
                   "hbm_bytes_per_shard_sweep": hb / a.shards_per_gpu, "traffic_over_algorithmic": hb / algo},
                  open(a.traffic_json, "w"), indent=1)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
