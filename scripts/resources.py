"""Print per-kernel VGPR / scratch / occupancy / LDS for one csrc/*.hip file.

    python scripts/resources.py csrc/cwt.hip [regex]

Compiles for gfx950 with -Rpass-analysis=kernel-resource-usage (no GPU needed).
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]
src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-I", f"{ROOT}/wavelet-transformer_amd/csrc", "-c", src, "-o", "/tmp/_res.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?):\s*(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    if pat and not pat.search(name):
        continue
    print(f"{name[:90]:90s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize [bytes/lane]')} "
          f"occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")
