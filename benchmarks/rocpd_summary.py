"""Summarise rocprofv3 kernel timings: time per kernel name (and grid size, for a rocpd DB).

    python benchmarks/rocpd_summary.py gpurun_out/<run>/<name>_results.db [--top N]
    python benchmarks/rocpd_summary.py gpurun_out/<run>/<name>_kernel_stats.csv [--top N]
"""
import argparse
import csv
import re
import sqlite3


def _short(name: str) -> str:
    return re.sub(r"\(.*", "", name.replace("void ", ""))[:120]


def from_csv(path: str, top: int) -> None:
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows) / 1000.0
    print(f"total kernel time {total:.1f} us")
    print(f"{'calls':>6} {'total_us':>11} {'avg_us':>9} {'pct':>6}  kernel")
    for r in rows[:top]:
        print(f"{int(r['Calls']):6d} {float(r['TotalDurationNs']) / 1000:11.1f} "
              f"{float(r['AverageNs']) / 1000:9.1f} {float(r['Percentage']):6.2f}  {_short(r['Name'])}")


def from_db(path: str, top: int) -> None:
    cur = sqlite3.connect(path).cursor()
    rows = cur.execute(
        "select name, grid_x, count(*), sum(duration)/1000.0, avg(duration)/1000.0, vgpr_count, "
        "accum_vgpr_count, lds_size from kernels group by name, grid_x order by 4 desc limit ?",
        (top,)).fetchall()
    total = cur.execute("select sum(duration)/1000.0 from kernels").fetchone()[0]
    print(f"total kernel time {total:.1f} us")
    print(f"{'calls':>6} {'total_us':>11} {'avg_us':>9} {'grid_x':>8} {'vgpr':>5} {'agpr':>5} {'lds':>7}  kernel")
    for name, grid, n, tot, avg, v, acc, lds in rows:
        print(f"{n:6d} {tot:11.1f} {avg:9.1f} {grid:8d} {v:5d} {acc:5d} {lds:7d}  {_short(name)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    (from_csv if a.path.endswith(".csv") else from_db)(a.path, a.top)


if __name__ == "__main__":
    main()
