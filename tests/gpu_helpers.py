"""Shared helpers for the @gpu parity tests."""

import json
import os

import numpy as np

# CWT / XWT per (series, scale) row ||W - W_ref|| / ||W_ref|| <= 1e-5, "the same
# applies to power" (and to W12, the XWT power and the significance ratio).
ROW_TOL = 1e-5


def gate(name, err, tol=ROW_TOL):
    """Assert max(err) <= tol and print the measured maximum.  With WTMI_PARITY_LOG set, the
    (test, check, max, gate) record is appended there as one JSON line (DESIGN.md section 4's
    table of measured maxima is built from that file)."""
    worst = float(np.max(err)) if np.size(err) else 0.0
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    print(f"PARITY {test} {name}: max {worst:.3e} (gate {tol:.0e})")
    log = os.environ.get("WTMI_PARITY_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": test, "check": name, "max": worst, "gate": tol}) + "\n")
    assert worst <= tol, (name, worst, tol)
    return worst


def red_series(rng, n, a=0.7, dtype=np.float32):
    """AR(1) red noise + 3 sinusoids (the BASELINE synthetic generator)."""
    e = rng.standard_normal(n)
    x = np.empty(n)
    acc = 0.0
    for i in range(n):
        acc = a * acc + e[i]
        x[i] = acc
    t = np.arange(n)
    for _ in range(3):
        A = rng.uniform(0.5, 2)
        P = np.exp(rng.uniform(np.log(8), np.log(max(9, n / 4))))
        x += A * np.sin(2 * np.pi * t / P + rng.uniform(0, 2 * np.pi))
    return x.astype(dtype)


def row_relerr(got, ref):
    """Per-row normwise relative error ||got - ref||_2 / ||ref||_2 over the last axis."""
    num = np.linalg.norm((got - ref).reshape(-1, ref.shape[-1]), axis=-1)
    den = np.linalg.norm(ref.reshape(-1, ref.shape[-1]), axis=-1)
    return num / np.maximum(den, 1e-300)


def red_batch(seed, B, n, dtype=np.float32):
    """Vectorised red_series for full BASELINE batches (same recipe: AR(1) a = 0.7 + 3
    sinusoids with random amplitude, log-uniform period and phase)."""
    from scipy.signal import lfilter
    rng = np.random.default_rng(seed)
    x = lfilter([1.0], [1.0, -0.7], rng.standard_normal((B, n)), axis=1)
    t = np.arange(n)[None, :]
    for _ in range(3):
        A = rng.uniform(0.5, 2, (B, 1))
        P = np.exp(rng.uniform(np.log(8), np.log(max(9, n / 4)), (B, 1)))
        x += A * np.sin(2 * np.pi * t / P + rng.uniform(0, 2 * np.pi, (B, 1)))
    return x.astype(dtype)
