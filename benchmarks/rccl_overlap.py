"""Do RCCL collective kernels co-reside with the full-shard scans?

Reads a rocprofv3 kernel-trace CSV of ``bench.py --opt simulate_world=N`` (the per-rank work of
the N-GPU step through a single-rank RCCL group) and reports, for every collective kernel, whether
it started while a scan kernel was running (co-resident: the scan leaves room on the CUs) or only
after a scan ended (queued behind it), with the start delay after its enqueue-order predecessor.

    python benchmarks/rccl_overlap.py <kernel_trace.csv>
"""
import argparse
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r.get("Queue_Id", "")) for r in rows)
    scans = [(s, e) for s, e, n, _ in ks
             if re.search(r"scan_stream_kernel|index_scan_i8_kernel", n) and e - s > 200_000]
    coll = [(s, e, n) for s, e, n, _ in ks if re.search(r"nccl|rccl", n, re.I)]
    # hardware queues: HIP maps streams round-robin onto GPU_MAX_HW_QUEUES queues, and kernels
    # of two streams on one queue run in FIFO order whatever their dependencies
    scan_q = {q for s, e, n, q in ks
              if re.search(r"scan_stream_kernel|index_scan_i8_kernel", n) and e - s > 200_000}
    coll_q = {q for s, e, n, q in ks if re.search(r"nccl|rccl", n, re.I)}
    inside = after = 0
    waits = []
    for s, e, n in coll:
        run = [sc for sc in scans if sc[0] <= s < sc[1]]
        if run:
            inside += 1
        else:
            after += 1
            prev = [sc for sc in scans if sc[1] <= s]
            if prev:
                waits.append((s - max(p[1] for p in prev)) / 1e3)
    out = {"scans": len(scans), "collective_kernels": len(coll),
           "started_during_a_scan": inside, "started_outside_scans": after,
           # start of each outside-scan collective after the last scan ended (a few us: it was
           # issued under the scan and waited for it)
           "start_after_scan_end_us": [round(w, 1) for w in waits],
           "collective_us": [round((e - s) / 1e3, 1) for s, e, _ in coll],
           "collective_us_mean": round(sum(e - s for s, e, _ in coll) / max(1, len(coll)) / 1e3, 2),
           "scan_hw_queues": sorted(scan_q), "collective_hw_queues": sorted(coll_q),
           "names": sorted({re.sub(r"\(.*", "", n)[:80] for _, _, n in coll})}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
