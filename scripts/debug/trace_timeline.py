"""Timeline of one iteration of a (multi-stream) kernel trace: start / end of each kernel
relative to the iteration's first kernel.
python scripts/debug/trace_timeline.py PROF_DIR FIRST_KERNEL_SUBSTR [ITER_FROM_END]"""
import csv
import glob
import os
import sys

d, first = sys.argv[1], sys.argv[2]
back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""))
              for r in csv.DictReader(open(f)))
starts = [i for i, r in enumerate(rows) if first in r[2]]
i0 = starts[-back]
i1 = starts[-back + 1] if back > 1 else len(rows)
t0 = rows[i0][0]
for s, e, k, q in rows[i0:i1]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} us  q{q}  {k.split('(')[0].replace('void ', '')[:60]}")
print(f"next iteration starts at {(rows[i1][0] - t0) / 1e3:.1f} us" if i1 < len(rows) else "")
