#!/usr/bin/env python3
"""HBM bytes per launch of the 64-chain GEMM passes (pass F `k_gemm_fwd`, pass B `k_gemm_bwd`)
from two rocprofv3 --pmc runs of tools/_bin/gemm_ab (FETCH_SIZE, WRITE_SIZE; separate passes),
corrected as MI355X_MICROARCH.md's HBM section prescribes (FETCH_SIZE doubled for 16 B/lane
streaming reads, which is what the LDS-DMA stages are; WRITE_SIZE as counted), against each
pass's algorithmic bytes:
  pass F  reads X (8 d per row) + y (4 per row), writes R (512 per row)   [beta^T: L2-resident]
  pass B  reads X (8 d per row) + R (512 per row), writes the chunk partials
Both counters are in KB per dispatch (rocprofv3's unit for these derived metrics).

usage: tools/pmc_gemm_traffic.py <fetch.csv> <write.csv> --rows-per-shard R --shards S --d D --json out.json
"""
import argparse
import csv
import json
import statistics

p = argparse.ArgumentParser()
p.add_argument("fetch_csv")
p.add_argument("write_csv")
p.add_argument("--rows-per-shard", type=int, required=True)
p.add_argument("--shards", type=int, required=True)
p.add_argument("--d", type=int, required=True)
p.add_argument("--json", required=True)
a = p.parse_args()


def per_kernel(path, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        k = r.get("Kernel_Name", "")
        per.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
        per[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: statistics.median(v.values()) * 1024.0 for k, v in per.items()}   # KB -> bytes


fetch = per_kernel(a.fetch_csv, "FETCH_SIZE")
write = per_kernel(a.write_csv, "WRITE_SIZE")
rows = a.rows_per_shard * a.shards
G = 512
out = {"run": f"tools/_bin/gemm_ab {a.rows_per_shard} {a.shards} (d = {a.d}, 64 chains)", "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if "k_gemm_fwd" in k:
        algo_r, algo_w = rows * (8 * a.d + 4), rows * 512
    elif "k_gemm_bwd" in k:
        algo_r, algo_w = rows * (8 * a.d + 512), a.shards * G * 64 * (a.d + 2) * 8
    else:
        continue
    f = 2.0 * fetch.get(k, float("nan"))
    w = write.get(k, float("nan"))
    out["kernels"][k] = {"fetch_bytes_x2": f, "write_bytes": w, "algorithmic_read_bytes": algo_r,
                         "algorithmic_write_bytes": algo_w, "read_ratio": f / algo_r, "write_ratio": w / algo_w,
                         "total_ratio": (f + w) / (algo_r + algo_w)}
    print(f"{k}: reads {f / 1e9:.2f} GB ({f / algo_r:.3f} x), writes {w / 1e9:.2f} GB ({w / algo_w:.3f} x)")
json.dump(out, open(a.json, "w"), indent=1)
