"""Summarise a rocprofv3 SQLite result (rocpd) database: time per kernel name and grid size.

    python benchmarks/rocpd_summary.py gpurun_out/<run>/<name>_results.db [--top N]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute(
        "select name, grid_x, count(*), sum(duration)/1000.0, avg(duration)/1000.0, vgpr_count, "
        "accum_vgpr_count, lds_size from kernels group by name, grid_x order by 4 desc limit ?",
        (a.top,)).fetchall()
    total = cur.execute("select sum(duration)/1000.0 from kernels").fetchone()[0]
    print(f"total kernel time {total:.1f} us")
    print(f"{'calls':>6} {'total_us':>11} {'avg_us':>9} {'grid_x':>8} {'vgpr':>5} {'agpr':>5} {'lds':>7}  kernel")
    for name, grid, n, tot, avg, v, acc, lds in rows:
        short = re.sub(r"\(.*", "", name.replace("void ", ""))[:120]
        print(f"{n:6d} {tot:11.1f} {avg:9.1f} {grid:8d} {v:5d} {acc:5d} {lds:7d}  {short}")


if __name__ == "__main__":
    main()
