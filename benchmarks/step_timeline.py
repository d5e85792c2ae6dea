"""The ordered kernel timeline of the last gap(s) between consecutive full-shard first-pass scans
of the headline (rocprofv3 kernel trace CSV): start offset from the previous scan's end, duration
and queue of every kernel that overlaps the gap -- the serial chain on the scan's queue is the
step's critical path beside the scan.

    python benchmarks/step_timeline.py <kernel_trace.csv> [--steps 2]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("void ", ""))
    return n.split("::")[-1][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 r["Queue_Id"]) for r in rows)
    scans = [k for k in ks if re.match(r"(index_scan_i8_kernel|scan_stream_kernel|scan_lq)", k[2])
             and k[1] - k[0] > 200_000]
    for s0, s1 in list(zip(scans[:-1], scans[1:]))[-a.steps:]:
        g0, g1 = s0[1], s1[0]
        print(f"== scan {s0[2]} {(s0[1] - s0[0]) / 1e3:.1f} us, gap {(g1 - g0) / 1e3:.1f} us")
        for st, en, nm, q in ks:
            if en > g0 and st < g1:
                print(f"  {(st - g0) / 1e3:8.1f} {(en - st) / 1e3:8.1f} us  q{q:>2}  {nm}")


if __name__ == "__main__":
    main()
