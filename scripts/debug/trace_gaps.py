"""Per-iteration span vs busy time of a kernel trace whose iterations start with KERNEL:
python scripts/debug/trace_gaps.py PROF_DIR FIRST_KERNEL_SUBSTR [LAST_N]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, first = sys.argv[1], sys.argv[2]
last_n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))
iters, cur = [], []
for s, e, k in rows:
    if first in k and cur:
        iters.append(cur)
        cur = []
    cur.append((s, e, k))
iters.append(cur)
iters = [it for it in iters if any(first in k for _, _, k in it)][-last_n:]
per = defaultdict(list)
spans, busy = [], []
for it in iters:
    spans.append((it[-1][1] - it[0][0]) / 1e3)
    busy.append(sum(e - s for s, e, _ in it) / 1e3)
    for s, e, k in it:
        per[k.split("(")[0]].append((e - s) / 1e3)
print(f"iterations {len(iters)}: span {sum(spans)/len(spans):.1f} us, kernels busy {sum(busy)/len(busy):.1f} us, "
      f"launches/iter {len(iters[-1])}")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/len(iters):8.1f} us/iter  x{len(v)//len(iters)}  {k[:80]}")
