"""Mean duration per kernel over the LAST k dispatches of a rocprofv3 kernel trace
(the bench's timed steps follow its warm-up), to set beside bench.py's HIP-event
kernel_ms.  Usage: python scripts/trace_mean.py PROF_DIR K"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, k = sys.argv[1], int(sys.argv[2])
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
per = defaultdict(list)
with open(f) as fh:
    for r in csv.DictReader(fh):
        per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for name, ts in sorted(per.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
    ts.sort()
    last = ts[-k:]
    mean = sum(e - s for s, e in last) / len(last) / 1e6
    print(f"{mean:.4f} ms  mean of last {len(last)} of {len(ts)}  {name[:90]}")
