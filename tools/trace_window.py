#!/usr/bin/env python3
"""Average duration of the data-sweep kernel over the bench's timed window, from a rocprofv3
--kernel-trace CSV: the last K dispatches of the kernel are the K timed steps (bench.py
launches no sweep after its timed region).  This is the figure bench.py's roofline.avg_launch_ms
(HIP events on the context stream) must agree with; the whole-run --stats average also
counts warmup launches in which only some shards (or none) are swept.

usage: tools/trace_window.py <kernel_trace.csv> --steps K [--kernel k_sweep3]
"""
import argparse
import csv
import json

p = argparse.ArgumentParser()
p.add_argument("trace_csv")
p.add_argument("--steps", type=int, required=True)
p.add_argument("--kernel", default="k_sweep3")
a = p.parse_args()
rows = [r for r in csv.DictReader(open(a.trace_csv)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
win = rows[-a.steps:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in win]
out = {"kernel": a.kernel, "dispatches_total": len(rows), "window_dispatches": len(win),
       "window_avg_ms": sum(dur) / len(dur), "window_min_ms": min(dur), "window_max_ms": max(dur)}
print(json.dumps(out))
