"""Record what the reference's own plot functions draw: tests/golden/plot_signatures.json.

Run in the BUILD container (reads /root/reference as text):

    python scripts/make_plot_golden.py

The plot functions are taken from the reference source by ``ast`` (the modules cannot be
imported here: they import pycwt, streamlit, dotenv) and executed on Agg with numpy and
matplotlib only, on the seeded synthetic inputs of ``tests/figsig.plot_inputs``.  The one
numeric dependency, ``pywt.waverec`` inside ``reconstruct_signal_component``, is served by
the oracle's PyWavelets restatement (oracle/dwt_spec.py, pinned by the PyWavelets golden
vectors).  Only the resulting figure signatures (tests/figsig.figure_signature) are
written; no reference code is stored.
"""

import json
import logging
import os
import sys
import types

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import numpy.typing as npt  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import figsig  # noqa: E402
from oracle import dwt_spec  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import refpin  # noqa: E402

REF = os.environ.get("WTMI_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "tests", "golden", "plot_signatures.json")


def extract(rel, names, ns):
    """Execute the named top-level defs / assignments of a reference file in ns -- only
    after each segment's SHA-256 matches its pin (scripts/refpin.py, scripts/refpins.json)."""
    mod = refpin.pinned_module(REF, rel, names)
    exec(compile(mod, rel, "exec"), ns)
    return ns


def base_ns():
    from typing import List, Tuple, Type
    # annotation-only names (the reference evaluates annotations at def time)
    ann = {k: object for k in ("DataForCWT", "ResultsFromCWT", "DataForXWT", "ResultsFromXWT",
                               "DataForWCT", "ResultsFromWCT")}
    return {**ann, "np": np, "npt": npt, "plt": plt, "Type": Type, "List": List, "Tuple": Tuple,
            "logger": logging.getLogger("reference"), "matplotlib": matplotlib,
            "Figure": matplotlib.figure.Figure}


def main():
    with open(os.path.join(ROOT, "tests", "golden", "pywt_filters.json")) as fh:
        db4 = json.load(fh)["filters"]["db4"]
    pywt_stub = types.SimpleNamespace(
        waverec=lambda c, w: dwt_spec.waverec(c, np.asarray(db4["rec_lo"]), np.asarray(db4["rec_hi"])))

    wh = extract("src/utils/wavelet_helpers.py",
                 ["align_series", "plot_signficance_levels", "plot_cone_of_influence"], base_ns())
    helpers = types.SimpleNamespace(**{k: wh[k] for k in ("align_series", "plot_signficance_levels",
                                                          "plot_cone_of_influence")})
    cwt = extract("src/cwt.py", ["plot_cwt"], dict(base_ns(), **vars(helpers)))
    xwt = extract("src/xwt.py", ["plot_xwt", "plot_phase_difference"],
                  dict(base_ns(), wavelet_helpers=helpers))
    wct = extract("src/wct.py", ["WCT_LEVELS", "plot_wct", "plot_phase_difference"],
                  dict(base_ns(), wavelet_helpers=helpers))
    dwt = extract("src/dwt.py", ["reconstruct_signal_component", "plot_components", "plot_smoothing"],
                  dict(base_ns(), pywt=pywt_stub, align_series=helpers.align_series))
    modwt = extract("src/modwt.py", ["plot_smoothing"], base_ns())

    inp = figsig.plot_inputs()
    P = figsig.PLOT_PROPS
    out = {}

    def axes_case(name, fn):
        fig, ax = plt.subplots(1, 1, figsize=(10, 5), dpi=72)
        fn(ax)
        out[name] = figsig.figure_signature(fig)
        plt.close(fig)

    d, r = inp["cwt"]
    axes_case("cwt.plot_cwt", lambda ax: cwt["plot_cwt"](ax, d, r, **{k: P[k] for k in list(P)[:6]}))
    axes_case("cwt.plot_cwt[no_sig]", lambda ax: cwt["plot_cwt"](ax, d, r, include_significance=False,
                                                              **{k: P[k] for k in list(P)[:6]}))
    d, r = inp["xwt"]
    axes_case("xwt.plot_xwt", lambda ax: xwt["plot_xwt"](ax, d, r, **P))
    axes_case("xwt.plot_phase_difference", lambda ax: xwt["plot_phase_difference"](
        ax, d.t_values, r.period, r.phase_diff_u, r.phase_diff_v, **P))
    d, r = inp["wct"]
    axes_case("wct.plot_wct", lambda ax: wct["plot_wct"](ax, d, r, **P))
    axes_case("wct.plot_wct[no_coi_no_arrows]", lambda ax: wct["plot_wct"](
        ax, d, r, include_cone_of_influence=False, include_phase_difference=False, **P))
    axes_case("wavelet_helpers.plot_cone_of_influence[cwt]", lambda ax: helpers.plot_cone_of_influence(
        ax, inp["cwt"][1].coi, inp["t_years"], figsig.LEVELS, inp["cwt"][1].period, 1 / 12,
        tranform_type="cwt", **P))
    axes_case("wavelet_helpers.plot_signficance_levels", lambda ax: helpers.plot_signficance_levels(
        ax, inp["cwt"][1].significance_levels, inp["t_years"], inp["cwt"][1].period, **P))

    fig = dwt["plot_components"]("series", inp["coeffs"], inp["t_years"], 5, "db4", figsize=(8, 12))
    out["dwt.plot_components"] = figsig.figure_signature(fig)
    plt.close("all")
    for asc in (False, True):
        fig = dwt["plot_smoothing"](inp["smooth"], inp["t_years"], inp["y"], ascending=asc,
                                    figsize=(8, 12), sharex=True)
        out[f"dwt.plot_smoothing[ascending={asc}]"] = figsig.figure_signature(fig)
        plt.close("all")
        fig = modwt["plot_smoothing"](inp["smooth"], inp["t_years"], inp["y"], ascending=asc,
                                      figsize=(8, 12))
        out[f"modwt.plot_smoothing[ascending={asc}]"] = figsig.figure_signature(fig)
        plt.close("all")

    with open(OUT, "w") as fh:
        json.dump({"generated_by": "scripts/make_plot_golden.py", "matplotlib": matplotlib.__version__,
                   "cases": out}, fh, indent=1)
        fh.write("\n")
    print(f"wrote {OUT}: {len(out)} cases")


if __name__ == "__main__":
    main()
