"""Kernel register / scratch table from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python scripts/resource_usage.py remarks.txt [name-regex]
"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cur = None
rows = []
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m:
            cur[key.split()[0]] = int(m.group(1))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if pat and not pat.search(d):
        continue
    d = re.sub(r"\(.*", "", d)
    print(f"VGPR {r.get('VGPRs', '?'):>3}  scratch {r.get('ScratchSize', '?'):>4}  occ {r.get('Occupancy', '?')}  {d}")
