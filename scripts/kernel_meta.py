"""Register / spill / LDS table of every kernel in libwtmi.so, read from the gfx950 code
objects' metadata notes (llvm-objdump --offloading + llvm-readelf --notes; no GPU).

    python scripts/kernel_meta.py [LIB] [name-regex]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "wavelet-transformer_amd", "wtmi", "libwtmi.so")
KEYS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".vgpr_spill_count": "vgpr_spill",
        ".sgpr_spill_count": "sgpr_spill", ".private_segment_fixed_size": "scratch",
        ".group_segment_fixed_size": "lds"}


def kernel_table(lib=LIB):
    """{demangled kernel name: {vgpr, agpr, vgpr_spill, sgpr_spill, scratch, lds}}."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, os.path.join(d, "lib.so"))
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", "lib.so"], cwd=d,
                       capture_output=True, check=True)
        for f in sorted(os.listdir(d)):
            if "amdgcn" not in f:
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(d, f)],
                                   capture_output=True, text=True, check=True).stdout
            # a kernel's keys are listed alphabetically: those before ".name" (.agpr_count,
            # .group_segment_fixed_size) belong to the kernel whose name follows them
            cur, pending = None, {}
            for line in notes.splitlines():
                m = re.match(r"\s*(\.[a-z_]+):\s+(\S+)", line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2)
                if key == ".name":
                    cur = out.setdefault(val, {})
                    cur.update(pending)
                    pending = {}
                elif key in KEYS:
                    (pending if key < ".name" else cur if cur is not None else pending)[KEYS[key]] = int(val)
    names = list(out)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return {re.sub(r"\(.*", "", d): out[n] for n, d in zip(names, dem)}


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else LIB
    pat = re.compile(sys.argv[-1]) if len(sys.argv) > 1 and not sys.argv[-1].endswith(".so") else None
    for name, r in sorted(kernel_table(lib).items()):
        if pat and not pat.search(name):
            continue
        print(f"vgpr {r.get('vgpr', '?'):>3}  spill {r.get('vgpr_spill', '?'):>3}  scratch {r.get('scratch', '?'):>4}  "
              f"lds {r.get('lds', '?'):>6}  {name}")
