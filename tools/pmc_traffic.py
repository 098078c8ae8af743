#!/usr/bin/env python3
"""Turn a rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) counter CSV into per-launch HBM bytes of
the data-sweep kernel, corrected as MI355X_MICROARCH.md (HBM section) prescribes: on gfx950
FETCH_SIZE counts exactly half the bytes of a wide coalesced 16 B/lane streaming read, so it
is doubled; WRITE_SIZE is exact for 16 B/lane stores (our partial-row stores are 8 B/lane and
tiny).  Writes profiles/sweep_pmc.json, which bench.py reads for roofline.traffic when its
configuration matches.

usage: tools/pmc_traffic.py <fetch_counter_collection.csv> --rows-per-shard R --d D --shards-per-gpu S
"""
import argparse
import csv
import json
import os
import statistics

p = argparse.ArgumentParser()
p.add_argument("fetch_csv")
p.add_argument("--write-csv", default=None)
p.add_argument("--rows-per-shard", type=int, required=True)
p.add_argument("--d", type=int, required=True)
p.add_argument("--shards-per-gpu", type=int, required=True)
p.add_argument("--kernel", default="k_sweep3")
p.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                             "profiles", "sweep_pmc.json"))
a = p.parse_args()


def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if a.kernel not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        vals.setdefault(r["Dispatch_Id"], 0.0)
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


fetch = per_dispatch(a.fetch_csv, "FETCH_SIZE")
algo = a.rows_per_shard * (8 * a.d + 4) * a.shards_per_gpu
# only full sweeps (every local shard swept) are comparable with the algorithmic bytes
full = [v for v in fetch if v * 1024 * 2 > 0.5 * algo]
med = statistics.median(full) * 1024 * 2 if full else None
out = {"kernel": a.kernel, "rows_per_shard": a.rows_per_shard, "d": a.d, "shards_per_gpu": a.shards_per_gpu,
       "dispatches": len(fetch), "full_sweep_dispatches": len(full), "fetch_size_kb_median": statistics.median(full) if full else None,
       "correction": "x2 (gfx950 FETCH_SIZE counts half of 16B/lane streaming reads)",
       "hbm_bytes_per_launch": med, "algorithmic_bytes_per_launch": algo,
       "hbm_bytes_per_shard_sweep": (med / a.shards_per_gpu) if med else None,
       "traffic_over_algorithmic": (med / algo) if med else None}
if a.write_csv:
    w = per_dispatch(a.write_csv, "WRITE_SIZE")
    out["write_bytes_per_launch_median"] = statistics.median(w) * 1024 if w else None
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps(out))
