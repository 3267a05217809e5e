"""Per-kernel static ISA statistics of a gfx950 assembly listing (hipcc -save-temps):
VGPRs, spills, LDS and instruction counts by class, for A/B of kernel variants.
    python scripts/debug/isa_stats.py FILE.s [NAME_SUBSTRING ...]"""
import re
import sys
from collections import Counter


def kernels(text):
    meta = {}
    for b in text.split('\n  - ')[1:]:
        nm = re.search(r"\.name:\s+(\S+)", b)
        if not nm:
            continue
        g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", b) or [None, None])[1]
        meta[nm.group(1)] = (g("vgpr_count"), g("vgpr_spill_count"), g("group_segment_fixed_size"))
    bodies = {}
    for m in re.finditer(r"^(_Z\S+):[^\n]*$(.*?)^\s*s_endpgm", text, re.S | re.M):
        bodies[m.group(1)] = m.group(2)
    return meta, bodies


def main():
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    meta, bodies = kernels(text)
    for name, body in bodies.items():
        if subs and not all(s in name for s in subs):
            continue
        ins = [l.split()[0] for l in body.splitlines() if l.strip() and l.startswith("\t") and not l.strip().startswith((".", ";"))]
        c = Counter()
        for i in ins:
            if i.startswith("v_pk_"):
                c["v_pk"] += 1
            elif i.startswith("v_"):
                c["v"] += 1
            elif i.startswith("ds_"):
                c["ds"] += 1
            elif i.startswith(("buffer_", "global_", "scratch_")):
                c["vmem"] += 1
            elif i.startswith("s_"):
                c["s"] += 1
        print(name[:80], meta.get(name), dict(c))


if __name__ == "__main__":
    main()
