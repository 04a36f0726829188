"""Per-run timeline of a kernel + memory-copy trace of q6_scan (rocprofv3 csv): for each run
(from its decode kernel), the copy stream's operations as start+duration in µs, and when the
context stream's last kernel ended. Usage: python scripts/copy_timeline.py <trace dir>"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
k = list(csv.DictReader(open(next(d.glob("*kernel_trace.csv")))))
m = list(csv.DictReader(open(next(d.glob("*memory_copy_trace.csv")))))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"], r["Stream_Id"]) for r in k]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", r["Direction"], r["Stream_Id"]) for r in m]
ev.sort()
runs = [i for i, e in enumerate(ev) if e[2] == "K" and "eval_decode" in e[3]]
for j, i0 in enumerate(runs):
    s = ev[i0][0]
    end = ev[runs[j + 1]][0] if j + 1 < len(runs) else 1 << 62
    win = [e for e in ev[i0:] if e[0] < end and e[0] - s < 5e6]
    streams = sorted({e[4] for e in win})
    for st in streams:
        ops = [e for e in win if e[4] == st]
        busy = sum(e[1] - e[0] for e in ops) / 1e3
        print(f"run {j} stream {st}: {len(ops)} ops, busy {busy:.0f} us, last end {(ops[-1][1] - s) / 1e3:.0f} us")
        if st != streams[0]:
            print("   ", " ".join(f"{(e[0] - s) / 1e3:.0f}+{(e[1] - e[0]) / 1e3:.0f}" for e in ops))
