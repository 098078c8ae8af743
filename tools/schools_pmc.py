#!/usr/bin/env python3
"""Summary of two rocprofv3 --pmc passes over tools/bench_schools.py for the fused 8-schools
kernel (k_nuts_fused_schools): counters summed over its dispatches, plus the derived shares
of wave cycles (SQ_* wave / busy / active counters are in quad-cycles summed over the SQs) and
per-SIMD instruction counts (1,024 SIMDs; one wave per SIMD at 4 chains per wave).

usage: tools/schools_pmc.py <pass1 counter_collection.csv> <pass2 counter_collection.csv>
                            --run "<command>" [--json out.json]
"""
import argparse
import csv
import json
from collections import defaultdict

SIMDS = 1024


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    name = None
    for r in csv.DictReader(open(path)):
        if "k_nuts_fused_schools" not in r.get("Kernel_Name", ""):
            continue
        name = r["Kernel_Name"].split("(")[0]
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    tot = defaultdict(float)
    for d in per.values():
        for k, v in d.items():
            tot[k] += v
    out = {"dispatches": len(per), "duration_ms": sum(dur.values())}
    out.update(tot)
    return name, out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("pass1")
    p.add_argument("pass2")
    p.add_argument("--run", required=True)
    p.add_argument("--json", default=None)
    a = p.parse_args()
    name, p1 = load(a.pass1)
    _, p2 = load(a.pass2)
    wc = p1.get("SQ_WAVE_CYCLES", 0.0)
    if wc:
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in p1:
                p1[k.lower() + "_frac_of_wave_cycles"] = p1[k] / wc
    if "SQ_INSTS_VALU" in p1:
        p1["valu_insts_per_simd"] = p1["SQ_INSTS_VALU"] / SIMDS
    if "SQ_INSTS_SALU" in p1:
        p1["salu_insts_per_simd"] = p1["SQ_INSTS_SALU"] / SIMDS
    if p2.get("GRBM_GUI_ACTIVE") and p2.get("duration_ms"):
        p2["clock_ghz"] = p2["GRBM_GUI_ACTIVE"] / 8 / (p2["duration_ms"] * 1e-3) / 1e9
    res = {"kernel": name, "run": a.run, "pass1": p1, "pass2": p2,
           "note": "SQ_* wave/busy/active counters in quad-cycles summed over SQs; per SIMD per run: "
                   "SQ_INSTS_VALU/1024 vector instructions; wait_any = s_waitcnt (memory) share of wave cycles"}
    s = json.dumps(res, indent=1)
    print(s)
    if a.json:
        open(a.json, "w").write(s + "\n")


if __name__ == "__main__":
    main()
