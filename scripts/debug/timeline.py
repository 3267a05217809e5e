"""Kernel timeline of the last step in a rocprofv3 kernel trace: start / end (us) relative
to the step's first kernel.  python scripts/debug/timeline.py PROF_DIR FIRST_KERNEL_SUBSTRING"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
s0, s1 = idx[-2], idx[-1]
t0 = int(rows[s0]["Start_Timestamp"])
for r in rows[s0:s1]:
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{a / 1e3:8.1f} {b / 1e3:8.1f} {(b - a) / 1e3:7.1f} q{r.get('Queue_Id', '?')} "
          f"{r['Kernel_Name'].split('(')[0].replace('void ', '')[:48]}")
