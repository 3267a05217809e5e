"""Per-kernel roofline of one bench config against each kernel's binding resource.

Usage: python scripts/kernel_roofline.py CONFIG TRACE_DIR FETCH_DIR WRITE_DIR VALU_DIR OUT_JSON [K]

TRACE_DIR: `rocprofv3 --kernel-trace --stats` of `bench.py --config CONFIG` (durations: mean
of the last K dispatches per kernel, the timed steps).  FETCH_DIR / WRITE_DIR: separate
`--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (HBM bytes; FETCH_SIZE doubled on gfx950,
MI355X_MICROARCH.md HBM section).  VALU_DIR: a `--pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
GRBM_GUI_ACTIVE` pass.  Per kernel (PMC values: mean per dispatch after the first):
  hbm_GBps  = HBM bytes / duration,          hbm_frac = hbm_GBps / 8000 (HBM3E peak)
  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
              (quad-cycles with a VALU instruction issuing, summed over waves, over the SIMD
              cycles of the dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles)
  bound     = whichever fraction is larger; frac = that fraction.
OUT_JSON is updated in place (one entry per config).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4


def _rows(d, pattern):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _short(name):
    return name.split("(")[0].replace("void ", "").strip()


def durations(d, k):
    per = defaultdict(list)
    for r in _rows(d, "*kernel_trace.csv"):
        per[_short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for name, ts in per.items():
        ts.sort()
        last = ts[-k:]
        out[name] = sum(e - s for s, e in last) / len(last) / 1e6
    return out


def counters(d):
    vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for r in _rows(d, "*counter_collection.csv"):
        disp = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        c = vals[_short(r["Kernel_Name"])][r["Counter_Name"]]
        c[disp] = c.get(disp, 0.0) + float(r["Counter_Value"])
    out = defaultdict(dict)
    for k, cs in vals.items():
        for cn, dv in cs.items():
            ds = sorted(dv)
            use = ds[1:] if len(ds) > 1 else ds
            out[k][cn] = sum(dv[i] for i in use) / len(use)
    return out


def main():
    cfg, tdir, fdir, wdir, vdir, out = sys.argv[1:7]
    k = int(sys.argv[7]) if len(sys.argv) > 7 else 10
    dur = durations(tdir, k)
    fetch, write, valu = counters(fdir), counters(wdir), counters(vdir)
    rows = []
    for name, ms in sorted(dur.items(), key=lambda kv: -kv[1]):
        if not name.startswith("wtmi::"):
            continue
        hbm = 2.0 * 1024.0 * fetch.get(name, {}).get("FETCH_SIZE", 0.0) + \
            1024.0 * write.get(name, {}).get("WRITE_SIZE", 0.0)
        gbs = hbm / (ms * 1e-3) / 1e9
        v = valu.get(name, {})
        grbm = v.get("GRBM_GUI_ACTIVE", 0.0)
        busy = v.get("SQ_ACTIVE_INST_VALU", 0.0) * 4.0 / (SIMDS * grbm / 8.0) if grbm else None
        hf = gbs / HBM_PEAK_GBS
        bound = "valu" if busy is not None and busy > hf else "hbm"
        rows.append({"kernel": name, "ms": round(ms, 4), "hbm_bytes": round(hbm),
                     "hbm_GBps": round(gbs, 1), "hbm_frac": round(hf, 3),
                     "valu_busy": None if busy is None else round(busy, 3),
                     "valu_insts": v.get("SQ_INSTS_VALU"),
                     "bound": bound, "frac": round(max(hf, busy or 0.0), 3)})
    data = {}
    if os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data[cfg] = {"kernels": rows, "method": __doc__.split("\n\n")[2].strip()}
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1)
    for r in rows:
        print(f"{r['ms']:8.4f} ms  {r['bound']:4s} frac {r['frac']:.3f}  hbm {r['hbm_GBps']:7.1f} GB/s  "
              f"valu {r['valu_busy']}  {r['kernel']}")


if __name__ == "__main__":
    main()
