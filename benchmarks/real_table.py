#!/usr/bin/env python3
"""Markdown table of a benchmarks/gpu/archive/gpu_r3_real.sh output directory: per shape and corpus, the
exact int8-pruned search (with its sampled route) against the plain bf16 emitting scan.

    python benchmarks/real_table.py gpurun_out/<dir> > profiles/<dir>/table.md
"""
import glob
import json
import os
import re
import sys


def main(d: str) -> None:
    runs = {}
    for p in glob.glob(os.path.join(d, "*.json")):
        name = os.path.basename(p)[:-5]
        m = re.match(r"(\d+)x(\d+)_(.+)_(i8|bf16)$", name)
        if not m:
            continue
        try:
            r = json.load(open(p))
        except ValueError:
            continue
        rows, nq, corpus, path = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)
        runs.setdefault((rows, nq, corpus), {})[path] = r
    print("| rows x queries (per rank) | corpus | pruned ms | plain bf16 ms | pruned / plain | "
          "batches routed to bf16 | overflowed batches | max candidates / query | exact (ids up "
          "to exact ties) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for (rows, nq, corpus) in sorted(runs, key=lambda x: (-x[0], x[2])):
        a = runs[(rows, nq, corpus)]
        i8, bf = a.get("i8"), a.get("bf16")
        if not i8 or not bf:
            continue
        ratio = i8["ms_per_step"] / bf["ms_per_step"]
        corpus_txt = (corpus.replace("clusteredc", "clustered ").replace("s0.", ", spread 0.")
                      .replace("clustered ", "clustered, ", 1))
        print(f"| {rows / 1e6:g}M x {nq} | {corpus_txt} | {i8['ms_per_step']:.2f} | "
              f"{bf['ms_per_step']:.2f} | {ratio:.2f} | {i8.get('search_dense_route_batches')} / "
              f"{i8['steps']} | {i8.get('search_overflow_batches')} | "
              f"{i8.get('search_max_candidates')} | {i8.get('verify_exact')} / "
              f"{bf.get('verify_exact')} |")


if __name__ == "__main__":
    main(sys.argv[1])
