"""Per-step timeline summary of a headline kernel trace (rocprofv3 --kernel-trace CSV): mean step,
the gap from the end of one int8 scan to the start of the next (the pre-pass + post-scan critical
path), and the durations of the list-scan kernels of the last step."""
import csv, sys, statistics
def analyze(path):
    rows=list(csv.DictReader(open(path)))
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    idx=[i for i,r in enumerate(rows) if 'index_scan_i8' in r['Kernel_Name'] and int(r['End_Timestamp'])-int(r['Start_Timestamp'])>200000]  # (gated no-op launches excluded)
    pre=[]; topk=[]; steps=[]
    for a,b in zip(idx[3:-1], idx[4:]):
        t_end=int(rows[a]['End_Timestamp']); t_next=int(rows[b]['Start_Timestamp'])
        steps.append((t_next-int(rows[a]['Start_Timestamp']))/1e3)
        pre.append((t_next-t_end)/1e3)
        topk.append(sorted(round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3,1) for r in rows[a:b] if 'index_scan_topk' in r['Kernel_Name']))
    print(path, 'step', round(statistics.mean(steps),1), 'us; scan-end -> next scan', round(statistics.mean(pre),1), 'us; list scans', topk[-1])
for p in sys.argv[1:]: analyze(p)
