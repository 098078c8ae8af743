#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --pmc counter CSV of tools/sweepe_ab (or any run whose
kernels differ by template arguments): for every distinct kernel name, the median over its
dispatches of each counter, and the derived clock, MFMA-busy and wait fractions.

SQ_* wave / busy counters are in quad-cycles summed over the chip's SQs; GRBM_GUI_ACTIVE is
in cycles (summed over the 8 XCDs); SQ_VALU_MFMA_BUSY_CYCLES is summed over SIMDs.

usage: tools/pmc_arms.py <counter_collection.csv> [--json out.json]
"""
import argparse
import csv
import json
import re
import statistics
from collections import defaultdict

SIMDS = 1024            # 256 CUs x 4 SIMDs
XCDS = 8


def short(name):
    m = re.search(r"(k_sweepe|k_sweep16)<([^>]*)>", name)
    if m:
        return m.group(1) + "<" + m.group(2).replace(" ", "") + ">"
    return name.split("(")[0][:80]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--json", default=None)
    a = p.parse_args()
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))   # kernel -> dispatch -> counter
    dur = defaultdict(dict)
    for r in csv.DictReader(open(a.csv)):
        k = short(r.get("Kernel_Name", ""))
        d = r["Dispatch_Id"]
        per[k][d][r["Counter_Name"]] += float(r["Counter_Value"])
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    out = {}
    for k, ds in per.items():
        cnames = sorted({c for v in ds.values() for c in v})
        med = {c: statistics.median([v[c] for v in ds.values() if c in v]) for c in cnames}
        ms = statistics.median(dur[k].values()) if dur[k] else None
        rec = {"dispatches": len(ds), "duration_ms": ms, **med}
        if "GRBM_GUI_ACTIVE" in med and ms:
            rec["clock_ghz"] = med["GRBM_GUI_ACTIVE"] / XCDS / (ms * 1e-3) / 1e9
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
            rec["mfma_busy_frac"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / (med["GRBM_GUI_ACTIVE"] / XCDS)
        if "SQ_WAVE_CYCLES" in med:
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if c in med:
                    rec[c.lower() + "_frac_of_wave_cycles"] = med[c] / med["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in med and med.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_bank_conflict_frac_of_lds_cycles"] = med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"]
        if "SQ_LDS_IDX_ACTIVE" in med and "GRBM_GUI_ACTIVE" in med:
            rec["lds_active_frac"] = med["SQ_LDS_IDX_ACTIVE"] / (SIMDS / 4) / (med["GRBM_GUI_ACTIVE"] / XCDS)
        out[k] = rec
    for k, r in sorted(out.items()):
        print(k, " ".join(f"{c}={v:.4g}" for c, v in r.items() if isinstance(v, float) and ("frac" in c or c in ("clock_ghz", "duration_ms"))))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
