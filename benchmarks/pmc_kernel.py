#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 counter_collection.csv files (one pass each).

    python benchmarks/pmc_kernel.py <counter_collection.csv> [...] [--match gemm]

Sums each counter over the matching dispatches and prints derived ratios:
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs)  (per-CU MFMA pipe occupancy,
                SQ_BUSY_CYCLES counts per SE; see MI355X_MICROARCH.md for unit notes)
  wait_any    = SQ_WAIT_ANY / SQ_WAVE_CYCLES   (waves parked in s_waitcnt / barrier)
  wait_inst   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  active      = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  clock_GHz   = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time (needs --kernel-trace in that pass)
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--match", default="gemm")
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    disp = {}
    grbm_wall = 0
    name = None
    for path in a.csvs:
        has_grbm = False
        for r in csv.DictReader(open(path)):
            if not re.search(a.match, r["Kernel_Name"]):
                continue
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", ""))
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(path, r["Dispatch_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            has_grbm |= r["Counter_Name"] == "GRBM_GUI_ACTIVE"
        if has_grbm:
            grbm_wall += sum(e - s for (p, _), (s, e) in disp.items() if p == path)
    if not tot:
        print("no matching dispatches")
        return
    out = {"kernel": name, "dispatches": len(disp)}
    wc = tot.get("SQ_WAVE_CYCLES")
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if wc and c in tot:
            out[c.replace("SQ_", "").lower() + "_frac"] = round(tot[c] / wc, 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in tot and "SQ_BUSY_CYCLES" in tot:
        out["mfma_busy_per_simd_vs_sq_busy"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                     (tot["SQ_BUSY_CYCLES"] * 4 * 32), 3)
    if "SQ_LDS_BANK_CONFLICT" in tot:
        out["lds_bank_conflict_cycles"] = tot["SQ_LDS_BANK_CONFLICT"]
    if "GRBM_GUI_ACTIVE" in tot:
        out["clock_GHz"] = round(tot["GRBM_GUI_ACTIVE"] / 8 / grbm_wall, 3)
    out["raw"] = {k: v for k, v in sorted(tot.items())}
    print(out)


if __name__ == "__main__":
    main()
