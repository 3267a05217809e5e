"""Per-kernel roofline of one bench config against each kernel's binding resource.

Usage: python scripts/kernel_roofline.py CONFIG TRACE_DIR FETCH_DIR WRITE_DIR VALU_DIR OUT_JSON [K [LDS_DIR]]

TRACE_DIR: `rocprofv3 --kernel-trace --stats` of `bench.py --config CONFIG` (durations: mean
of the last K dispatches per kernel, the timed steps).  FETCH_DIR / WRITE_DIR: separate
`--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes (HBM bytes; FETCH_SIZE doubled on gfx950,
MI355X_MICROARCH.md HBM section).  VALU_DIR: a `--pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
GRBM_GUI_ACTIVE` pass.  Per kernel (PMC values: mean per dispatch after the first):
  hbm_GBps  = HBM bytes / duration,          hbm_frac = hbm_GBps / 8000 (HBM3E peak)
  valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
              (quad-cycles with a VALU instruction issuing, summed over waves, over the SIMD
              cycles of the dispatch: GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles)
  lds_busy  = SQ_LDS_IDX_ACTIVE x 8 / (256 CUs x GRBM_GUI_ACTIVE) (LDS-array cycles per CU cycle),
              from an optional LDS_DIR pass `--pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT
              SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE`; with it
              lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (share of LDS cycles lost
              to bank conflicts) and lds_issue_wait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (share of
              wave cycles stalled issuing an LDS instruction)
  bound     = whichever of hbm / valu / lds is largest; frac = that fraction.
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
    ldir = sys.argv[8] if len(sys.argv) > 8 else None
    dur = durations(tdir, k)
    fetch, write, valu = counters(fdir), counters(wdir), counters(vdir)
    lds = counters(ldir) if ldir else {}
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
        L = lds.get(name, {})
        lg = L.get("GRBM_GUI_ACTIVE", 0.0)
        lbusy = L["SQ_LDS_IDX_ACTIVE"] * 8.0 / (256 * lg) if lg and "SQ_LDS_IDX_ACTIVE" in L else None
        lconf = (L.get("SQ_LDS_BANK_CONFLICT", 0.0) / L["SQ_LDS_IDX_ACTIVE"]
                 if L.get("SQ_LDS_IDX_ACTIVE") else None)
        lwait = (L.get("SQ_WAIT_INST_LDS", 0.0) / L["SQ_WAVE_CYCLES"] if L.get("SQ_WAVE_CYCLES") else None)
        fr = {"hbm": hf, "valu": busy or 0.0, "lds": lbusy or 0.0}
        bound = max(fr, key=fr.get)
        row = {"kernel": name, "ms": round(ms, 4), "hbm_bytes": round(hbm),
               "hbm_GBps": round(gbs, 1), "hbm_frac": round(hf, 3),
               "valu_busy": None if busy is None else round(busy, 3),
               "valu_insts": v.get("SQ_INSTS_VALU"),
               "bound": bound, "frac": round(fr[bound], 3)}
        if ldir:
            row.update(lds_busy=None if lbusy is None else round(lbusy, 3),
                       lds_conflict=None if lconf is None else round(lconf, 3),
                       lds_issue_wait=None if lwait is None else round(lwait, 3),
                       lds_insts=L.get("SQ_INSTS_LDS"))
        rows.append(row)
    data = {}
    if os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data[cfg] = {"kernels": rows, "method": __doc__.split("\n\n")[2].strip()}
    with open(out, "w") as fh:
        json.dump(data, fh, indent=1)
    for r in rows:
        print(f"{r['ms']:8.4f} ms  {r['bound']:4s} frac {r['frac']:.3f}  hbm {r['hbm_GBps']:7.1f} GB/s  "
              f"valu {r['valu_busy']}  lds {r.get('lds_busy')} conf {r.get('lds_conflict')} "
              f"ldswait {r.get('lds_issue_wait')}  {r['kernel']}")


if __name__ == "__main__":
    main()
