"""Shared helpers for the @gpu parity tests."""

import numpy as np


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
