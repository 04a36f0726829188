"""HIP API calls beside the kernels and copies of one q6_scan run (rocprofv3 --hip-runtime-trace
--kernel-trace --memory-copy-trace csv): every call of 20 µs or more, and the copy stream's
operations, in µs from the run's decode kernel. Usage: python scripts/api_timeline.py <dir> <run>"""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
run = int(sys.argv[2]) if len(sys.argv) > 2 else -1
k = list(csv.DictReader(open(next(d.rglob("*kernel_trace.csv")))))
m = list(csv.DictReader(open(next(d.rglob("*memory_copy_trace.csv")))))
a = list(csv.DictReader(open(next(d.rglob("*hip_api_trace.csv")))))
dec = sorted(int(r["Start_Timestamp"]) for r in k if "eval_decode" in r["Kernel_Name"])
s = dec[run]
e = dec[run + 1] if run != -1 and run + 1 < len(dec) else s + 4_000_000
ev = []
for r in k:
    t = int(r["Start_Timestamp"])
    if s - 600_000 <= t < e:
        ev.append((t, int(r["End_Timestamp"]), f"K s{r['Stream_Id']}", r["Kernel_Name"].replace("cubit::(anonymous namespace)::", "")[:30]))
for r in m:
    t = int(r["Start_Timestamp"])
    if s - 600_000 <= t < e:
        ev.append((t, int(r["End_Timestamp"]), f"M s{r['Stream_Id']}", r["Direction"][12:]))
for r in a:
    t = int(r["Start_Timestamp"])
    dur = int(r["End_Timestamp"]) - t
    if s - 600_000 <= t < e and dur >= 20_000:
        ev.append((t, int(r["End_Timestamp"]), f"A t{r['Thread_Id'][-4:]}", r["Function"]))
ev.sort()
for t0, t1, kind, what in ev:
    print(f"{(t0 - s) / 1e3:8.0f} {(t1 - t0) / 1e3:7.1f} {kind:8s} {what}")
