"""Summarise a rocprofv3 database (run_results.db) of benchmarks/lat_trace.py: per forward (the
last N), the GPU span from the first kernel's start to the last kernel's end, the summed kernel
time, the idle time between kernels, and the kernels by total time.

    python benchmarks/lat_db.py <run_results.db> [--kernels-per-forward K] [--forwards 20]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--forwards", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    # forwards are separated by host syncs: split where the gap exceeds 40 us
    fw, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[1] - cur[-1][2] > 40_000:
            fw.append(cur)
            cur = [r]
        else:
            cur.append(r)
    fw.append(cur)
    last = fw[-a.forwards:]
    span = sum(f[-1][2] - f[0][1] for f in last) / len(last) / 1e3
    busy = sum(sum(r[2] - r[1] for r in f) for f in last) / len(last) / 1e3
    nk = sum(len(f) for f in last) / len(last)
    print(f"{a.db}: {len(fw)} forwards; last {len(last)}: {nk:.0f} kernels, GPU span {span:.1f} us, "
          f"kernel time {busy:.1f} us, gaps {span - busy:.1f} us ({(span - busy) / max(nk - 1, 1):.1f} us per gap)")
    agg = collections.defaultdict(float)
    for f in last:
        for n, s, e in f:
            agg[n.split("(")[0].replace("void ", "")[:70]] += (e - s) / 1e3 / len(last)
    for n, t in sorted(agg.items(), key=lambda x: -x[1])[:12]:
        print(f"  {t:8.1f} us  {n}")


if __name__ == "__main__":
    main()
