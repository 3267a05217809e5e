#!/usr/bin/env python3
"""End-to-end latency of the app-visible calls.

    python scripts/app_latency.py [--out profiles/r03/app_latency.json] [--calls 30]
                                  [--sig-calls 5] [--cpu-sig-passes 6] [--only sig]

Times the drop-in modules exactly as the Streamlit app calls them -- NumPy in, NumPy
out: H2D, every launch, D2H and the host closed forms are inside the clock:
  * src.cwt.run_cwt on sample_data/inflation.csv (n = 1333) at the module's J = 84
    (85 scales) and at C1's 64 scales (J = 63);
  * src.xwt.run_xwt on an inflation-shaped pair (n = 1333, dj = 1/8);
  * src.wct.run_wct(calculate_signficance=True) at the app's settings (n = 1333,
    dj = 1/8, 300 Monte-Carlo passes), significance cache OFF (WTMI_WCT_SIG_CACHE=0),
    plus run_wct(calculate_signficance=False);
and beside each, the CPU oracle's restatement of the same reference call (oracle/glue_spec,
oracle/pycwt_spec; fp64, one core).  The oracle's Monte Carlo is timed over
--cpu-sig-passes passes and scaled to 300 (the per-pass cost is constant; stated in the
record).  The significance call is also split into its steps (AR(1) moments, noise +
coherence launches, counter, host quantile) to name the dominant one.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd")]
os.environ["WTMI_WCT_SIG_CACHE"] = "0"
SAMPLE = os.path.join(ROOT, "tests", "golden", "sample_data")


def load_inflation():
    import pandas as pd
    df = pd.read_csv(os.path.join(SAMPLE, "inflation.csv"), sep=None, parse_dates=[0],
                     index_col=0, engine="python")
    return df.iloc[:, 0].to_numpy(dtype=float), df.index.to_numpy()


def app_pair(y):
    """Two app-shaped series: standardize_series(detrend) of inflation and of a lagged,
    noisy copy (create_xwt_dict / create_wct_dict standardise before the transform)."""
    from oracle import glue_spec as gs
    rng = np.random.default_rng(5)
    e = np.zeros(y.size)
    for t in range(1, y.size):
        e[t] = 0.7 * e[t - 1] + rng.standard_normal()
    y2 = 0.6 * np.roll(y, 6) + 0.3 * e
    return gs.standardize_series(y), gs.standardize_series(y2)


def timed(fn, calls, warm=2, sync=None):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        if sync:
            sync()
        ts.append(time.perf_counter() - t0)
    ts = np.asarray(ts) * 1e3
    return {"median_ms": float(np.median(ts)), "mean_ms": float(ts.mean()),
            "min_ms": float(ts.min()), "max_ms": float(ts.max()), "calls": calls}


def gpu_side(args, y, t, y1, y2):
    import torch

    import src.cwt as cwt
    import src.wct as wct
    import src.xwt as xwt
    from src.utils.wavelet_helpers import standardize_series
    from wtmi import transforms
    assert not transforms.SIG_CACHE
    out = {}
    ys = standardize_series(y)
    if args.only in (None, "cwt"):
        d85 = cwt.DataForCWT(t, ys, cwt.MOTHER, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
        out["run_cwt_85_scales"] = timed(lambda: cwt.run_cwt(d85, standardize=True), args.calls)
        d64 = cwt.DataForCWT(t, ys, cwt.MOTHER, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
        saved = cwt.J
        cwt.J = 63
        try:
            out["run_cwt_64_scales"] = timed(lambda: cwt.run_cwt(d64, standardize=True), args.calls)
        finally:
            cwt.J = saved
    if args.only in (None, "xwt"):
        dx = xwt.DataForXWT(y1, y2, xwt.MOTHER_DICT["morlet"], xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
        out["run_xwt"] = timed(lambda: xwt.run_xwt(dx), args.calls)
    dw = wct.DataForWCT(y1, y2, wct.MOTHER_DICT["morlet"], wct.DT, wct.DJ, wct.S0, wct.LEVELS)
    if args.only in (None, "wct"):
        out["run_wct_no_sig"] = timed(lambda: wct.run_wct(dw, calculate_signficance=False),
                                      args.calls)
    if args.only in (None, "wct", "sig"):
        # the drop-in's defaults: pycwt's masked-counter quantile step
        assert transforms.SIG_QUANTILE == "pycwt"
        out["run_wct_sig_300_passes"] = timed(lambda: wct.run_wct(dw, calculate_signficance=True),
                                              args.sig_calls, warm=1)
        # the significance call's steps, as run_wct performs them
        n0 = y1.size
        J = int(np.round(np.log2(n0 * wct.DT / wct.S0) / wct.DJ))
        steps = {}

        def st(name, fn):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            steps.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
            return r
        for _ in range(args.sig_calls):
            a1 = st("ar1 x2 (moments kernel + D2H + host quadratic)",
                    lambda: (transforms.ar1(y1)[0], transforms.ar1(y2)[0]))
            st("wct_significance (noise, coherence launches, counter, D2H, quantile)",
               lambda: transforms.wct_significance(a1[0], a1[1], wct.DT, wct.DJ, wct.S0, J,
                                                   cache=False, seed=11))
            geo = st("host geometry (noise length, COI intervals)",
                     lambda: transforms.wct_sig_geometry(wct.DT, wct.DJ, wct.S0, J))
            wlc = np.random.default_rng(0).integers(0, 50, (geo[1].size, 1000)).astype(float)
            st("host quantile rule (restatement; the call itself runs it on the device)",
               lambda: transforms.significance_from_histogram(wlc, geo[4], geo[5]))
        out["run_wct_sig_steps_median_ms"] = {k: float(np.median(v)) for k, v in steps.items()}
        N = geo[0]
        from wtmi import ops
        per_pair = max(1, ops.wct_workspace_bytes(1, N, geo[1].size))
        out["sig_geometry"] = {"noise_samples": int(N), "scales": int(geo[1].size),
                               "maxscale": int(geo[5]), "passes": 300,
                               "pairs_per_launch": int(min(300, 512, (8 << 30) // per_pair))}
    return out


def cpu_side(args, y, y1, y2):
    from oracle import glue_spec as gs
    from oracle import pycwt_spec as pc
    out = {}
    ys = gs.standardize_series(y)
    if args.only in (None, "cwt"):
        out["run_cwt_85_scales"] = timed(lambda: gs.run_cwt(ys, ys.size, standardize=True),
                                         max(3, args.calls // 10), warm=1)
        out["run_cwt_64_scales"] = timed(lambda: gs.run_cwt(ys, ys.size, standardize=True, J=63),
                                         max(3, args.calls // 10), warm=1)
    if args.only in (None, "xwt"):
        out["run_xwt"] = timed(lambda: gs.run_xwt(y1, y2, 1 / 12, 1 / 8, 2 / 12,
                                                  [0.0625, 0.125, 0.25]), 3, warm=1)
    if args.only in (None, "wct"):
        out["run_wct_no_sig"] = timed(lambda: gs.run_wct(y1, y2, 1 / 12, 1 / 8, 2 / 12), 3, warm=1)
    if args.only in (None, "wct", "sig"):
        n0 = y1.size
        J = int(np.round(np.log2(n0 * (1 / 12) / (2 / 12)) / (1 / 8)))
        a1, a2 = pc.ar1(y1)[0], pc.ar1(y2)[0]
        k = args.cpu_sig_passes
        t0 = time.perf_counter()
        pc.wct_significance(a1, a2, 1 / 12, 1 / 8, 2 / 12, J, mc_count=k,
                            rng=np.random.default_rng(1))
        per_pass = (time.perf_counter() - t0) / k
        nosig = out.get("run_wct_no_sig", {}).get("median_ms")
        out["run_wct_sig_300_passes"] = {
            "estimate_ms": per_pass * 300 * 1e3 + (nosig or 0.0),
            "per_pass_ms": per_pass * 1e3, "passes_timed": k,
            "note": f"{k} Monte-Carlo passes timed and scaled to 300 (+ the sig=False call)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "app_latency.json"))
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--sig-calls", type=int, default=5)
    ap.add_argument("--cpu-sig-passes", type=int, default=6)
    ap.add_argument("--only", default=None, choices=["cwt", "xwt", "wct", "sig"])
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    y, t = load_inflation()
    y1, y2 = app_pair(y)
    rec = {"inputs": {"series": "tests/golden/sample_data/inflation.csv", "n": int(y.size),
                      "pair": "standardize_series of inflation and of 0.6 roll(inflation, 6) + "
                              "0.3 AR(1)(0.7) noise (seed 5)"},
           "clock": "time.perf_counter around the NumPy-in / NumPy-out call (H2D, launches, D2H, "
                    "host closed forms); median of the calls after warm-up"}
    rec["gpu"] = gpu_side(args, y, t, y1, y2)
    print(json.dumps(rec["gpu"], indent=1), flush=True)
    if not args.no_cpu:
        rec["cpu_oracle"] = cpu_side(args, y, y1, y2)
        rec["cpu_oracle_kind"] = "port: oracle/ fp64 restatement of the reference call, 1 core"
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
