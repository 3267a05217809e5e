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
