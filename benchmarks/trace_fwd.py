"""Per-kernel breakdown of the forwards in a rocprofv3 database of benchmarks/lat_trace.py:
kernels per forward, GPU span, kernel time, and time per kernel name (template arguments kept).

    python benchmarks/trace_fwd.py <run_results.db> [--forwards 20]
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
    rows = list(c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x "
                          "from kernels order by start"))
    fw, cur = [], []
    for r in rows:
        if "embed_ln_kernel" in r[0]:   # a forward starts with the embedding + LayerNorm
            if cur:
                fw.append(cur)
            cur = [r]
        elif cur:
            cur.append(r)
    fw.append(cur)
    n_k = collections.Counter(len(f) for f in fw).most_common(1)[0][0]
    last = [f for f in fw if len(f) == n_k][-a.forwards:]
    span = sum(f[-1][2] - f[0][1] for f in last) / len(last) / 1e3
    busy = sum(sum(r[2] - r[1] for r in f) for f in last) / len(last) / 1e3
    print(f"{a.db}: {len(fw)} forwards; last {len(last)} of {n_k} kernels: GPU span {span:.1f} us, "
          f"kernel time {busy:.1f} us, gaps {span - busy:.1f} us")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for f in last:
        for r in f:
            name = r[0].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            agg[(name, f"{r[3] // max(r[6], 1)}x{r[4]}x{r[5]}")][0] += 1
            agg[(name, f"{r[3] // max(r[6], 1)}x{r[4]}x{r[5]}")][1] += (r[2] - r[1]) / 1e3
    for (name, grid), (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{t / len(last):8.1f} us/fwd  {n / len(last):5.1f}x  {t / n:6.2f} us  grid {grid:10s} {name}")


if __name__ == "__main__":
    main()
