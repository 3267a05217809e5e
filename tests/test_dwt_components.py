"""Host logic of src.dwt.reconstruct_signal_component's component cache (CPU; the inverse DWT
itself is replaced by a stand-in that records its calls).  The reference's time-scale
regression (src/regression.py:113-114) reconstructs the levels + 1 components of two
coefficient lists alternately, one call each; here the first call per list computes all of
them in one batched launch.  The GPU values are checked in tests/test_gpu_wct_app.py."""

import threading

import numpy as np
import pytest


@pytest.fixture
def dwt_mod(monkeypatch):
    import src.dwt as dwt
    calls = []

    def fake(coeffs, wavelet, masks):
        calls.append(list(masks))
        tot = sum(float(np.sum(c)) for c in coeffs)
        # variant v: a marker of (mask, content) so cache mix-ups show
        return [np.full(8, m * 1000.0 + tot) for m in masks]

    monkeypatch.setattr(dwt.transforms, "waverec_variants", fake)
    monkeypatch.setattr(dwt, "_COMPONENTS", dwt._ComponentCache(size=4))
    return dwt, calls


def _coeffs(seed, n=4):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(5 + k) for k in range(n)]


def test_regression_pattern_is_one_launch_per_list(dwt_mod):
    dwt, calls = dwt_mod
    a, b = _coeffs(1), _coeffs(2)
    for j in range(len(a)):
        ra = dwt.reconstruct_signal_component(a, "db4", j)
        rb = dwt.reconstruct_signal_component(b, "db4", j)
        assert ra[0] == (1 << j) * 1000.0 + sum(float(np.sum(c)) for c in a)
        assert rb[0] == (1 << j) * 1000.0 + sum(float(np.sum(c)) for c in b)
    assert calls == [[1, 2, 4, 8], [1, 2, 4, 8]]


def test_results_are_copies_and_content_keyed(dwt_mod):
    dwt, calls = dwt_mod
    a = _coeffs(3)
    r = dwt.reconstruct_signal_component(a, "db4", 2)
    r[:] = -1.0  # the caller's array is its own
    assert dwt.reconstruct_signal_component(a, "db4", 2)[0] != -1.0
    a[1] = a[1] + 1.0  # new content: a new batched launch
    dwt.reconstruct_signal_component(a, "db4", 2)
    assert len(calls) == 2
    dwt.reconstruct_signal_component(a, "sym4", 2)  # another wavelet: another key
    assert len(calls) == 3


def test_out_of_range_level_is_all_zero_mask(dwt_mod):
    """The reference zeroes every entry when level matches none (src/dwt.py:113-119)."""
    dwt, calls = dwt_mod
    a = _coeffs(4)
    dwt.reconstruct_signal_component(a, "db4", len(a))
    dwt.reconstruct_signal_component(a, "db4", -1)
    assert calls == [[0], [0]]


def test_cache_is_bounded_and_thread_safe(dwt_mod):
    dwt, calls = dwt_mod
    lists = [_coeffs(10 + i) for i in range(12)]
    errs = []

    def work(k):
        try:
            for rep in range(3):
                for lst in lists[k::3]:
                    for j in range(len(lst)):
                        v = dwt.reconstruct_signal_component(lst, "db4", j)
                        if v[0] != (1 << j) * 1000.0 + sum(float(np.sum(c)) for c in lst):
                            errs.append((k, j))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    assert len(dwt._COMPONENTS._d) <= 4
