"""What runs between consecutive full-shard first-pass scans (the stream scan, or the round-4
LDS-ring int8 / MX-fp4 scan) of the headline (rocprofv3 kernel trace CSV): for the
gaps of the last steps, every kernel that overlaps the gap, its queue, how much of the gap it
covers, and the gap time with NO kernel running (idle).

    python benchmarks/step_gap.py <kernel_trace.csv> [--steps 5]
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("void ", ""))
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
          for r in rows]
    ks.sort()
    # the full-shard scans (a gated launch that returned at once is not one)
    scans = [k for k in ks if k[2] in ("index_scan_i8_kernel", "scan_stream_kernel")
             and k[1] - k[0] > 200_000]
    gaps = list(zip(scans[:-1], scans[1:]))[-a.steps:]
    agg = collections.defaultdict(float)
    tot_gap = tot_idle = 0.0
    for s0, s1 in gaps:
        g0, g1 = s0[1], s1[0]
        tot_gap += g1 - g0
        cover = []
        for st, en, nm, q in ks:
            lo, hi = max(st, g0), min(en, g1)
            if hi > lo:
                agg[(nm, q)] += hi - lo
                cover.append((lo, hi))
        cover.sort()
        busy, cur = 0, None
        for lo, hi in cover:
            if cur is None or lo > cur[1]:
                if cur:
                    busy += cur[1] - cur[0]
                cur = [lo, hi]
            else:
                cur[1] = max(cur[1], hi)
        if cur:
            busy += cur[1] - cur[0]
        tot_idle += (g1 - g0) - busy
    n = len(gaps)
    print(f"gap per step {tot_gap / n / 1e3:.1f} us, no kernel running {tot_idle / n / 1e3:.1f} us")
    for (nm, q), t in sorted(agg.items(), key=lambda x: -x[1])[:30]:
        print(f"  {t / n / 1e3:8.1f} us  queue {q:>3}  {nm}")


if __name__ == "__main__":
    main()
