"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel: MFMA busy share, LDS bank
conflict rate, wave wait shares.

    python benchmarks/pmc_summary.py gpurun_out/pmc/<run>/<name>_counter_collection.csv
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in rows:
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", ""))[:90]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
    print(f"{'kernel':90s} {'calls':>5s} {'MFMA busy/CU busy':>17s} {'LDS confl/LDS act':>17s} "
          f"{'wait_any/wave':>13s} {'wait_lds/wave':>13s}")
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CU_CYCLES", 0)):
        busy = c.get("SQ_BUSY_CU_CYCLES", 0) or 1
        # SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; SQ_BUSY_CU_CYCLES is per CU
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * busy)
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0) / (c.get("SQ_LDS_IDX_ACTIVE", 0) or 1)
        wave = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k:90s} {len(calls[k]):5d} {mfma:17.3f} {lds:17.4f} "
              f"{c.get('SQ_WAIT_ANY', 0) / wave:13.3f} {c.get('SQ_WAIT_INST_LDS', 0) / wave:13.3f}")


if __name__ == "__main__":
    main()
