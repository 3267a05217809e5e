"""Re-entrancy of the drop-in modules (SURVEY 8(b) "Threading": Streamlit calls from
several session threads at once, /root/reference/app.py:18).

Four threads call run_cwt, run_wct (with and without the Monte-Carlo significance at a
fixed seed), modwt/imodwt and run_xwt concurrently on different series, several rounds
each, two of them on their own HIP streams; every result must be BITWISE equal to the same
call made alone on one thread.  A fifth thread overrides a launch option (thread-local,
csrc/options.hip) in a loop the whole time: the other threads must not see it.
"""

import threading

import numpy as np
import pytest
import torch

from gpu_helpers import red_series

pytestmark = pytest.mark.gpu


def _inputs():
    rng = np.random.default_rng(2024)
    ys = [red_series(rng, n).astype(np.float64) for n in (1333, 700, 2048, 4096, 1000)]
    y2 = [0.6 * np.roll(y, 3) + 0.8 * red_series(rng, y.size) for y in ys]
    return ys, y2


def _jobs(ys, y2):
    import src.cwt as cwt
    import src.modwt as modwt
    import src.wct as wct
    import src.xwt as xwt
    from wtmi import transforms

    def job_cwt(i):
        t = np.arange(ys[i].size).astype("datetime64[M]")
        d = cwt.DataForCWT(t, ys[i], cwt.MOTHER, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
        r = cwt.run_cwt(d, standardize=True)
        return [r.power, r.significance_levels, r.coi]

    def job_wct(i):
        d = wct.DataForWCT(ys[i], y2[i], wct.MOTHER_DICT["morlet"], wct.DT, wct.DJ, wct.S0,
                           wct.LEVELS)
        r = wct.run_wct(d, calculate_signficance=False)
        g1, g2 = transforms.ar1(ys[i])[0], transforms.ar1(y2[i])[0]
        J = int(np.round(np.log2(ys[i].size * wct.DT / wct.S0) / wct.DJ))
        sig = transforms.wct_significance(g1, g2, wct.DT, wct.DJ, wct.S0, J, mc_count=40,
                                          cache=False, seed=1234 + i)
        return [r.coherence, r.phase_diff_u, r.phase_diff_v, sig]

    def job_modwt(i):
        w = modwt.modwt(ys[i].astype(np.float32), "db4", 6)
        return [w, modwt.imodwt(w, "db4"), modwt.modwtmra(w, "db4")]

    def job_xwt(i):
        d = xwt.DataForXWT(ys[i], y2[i], xwt.MOTHER_DICT["morlet"], xwt.DT, xwt.DJ, xwt.S0,
                           xwt.LEVELS)
        r = xwt.run_xwt(d)
        return [r.power, r.significance_levels, r.phase_diff_u]

    return [job_cwt, job_wct, job_modwt, job_xwt]


def test_concurrent_sessions_bitwise_equal_to_sequential():
    from wtmi import _lib
    ys, y2 = _inputs()
    jobs = _jobs(ys, y2)
    n_series = len(ys)
    # sequential reference: every (job, series) alone on this thread
    ref = {(j, i): jobs[j](i) for j in range(len(jobs)) for i in range(n_series)}
    torch.cuda.synchronize()

    errors, got = [], {}
    lock = threading.Lock()
    stop = threading.Event()
    start = threading.Barrier(len(jobs) + 1)

    def worker(j):
        try:
            stream = torch.cuda.Stream() if j % 2 else None
            start.wait()
            for rnd in range(3):
                for k in range(n_series):
                    i = (k + j + rnd) % n_series  # different series on each thread at a time
                    if stream is not None:
                        with torch.cuda.stream(stream):
                            out = jobs[j](i)
                    else:
                        out = jobs[j](i)
                    with lock:
                        got.setdefault((j, i), []).append(out)
        except BaseException as e:  # noqa: BLE001  (re-raised on the main thread)
            errors.append(e)

    def option_flipper():
        start.wait()
        flips = 0
        while not stop.is_set():
            with _lib.option("cwt_prune", 0), _lib.option("wct_prune", 0):
                flips += 1
        assert flips > 0

    threads = [threading.Thread(target=worker, args=(j,)) for j in range(len(jobs))]
    flipper = threading.Thread(target=option_flipper)
    for t in threads + [flipper]:
        t.start()
    for t in threads:
        t.join(timeout=600)
    stop.set()
    flipper.join(timeout=60)
    assert not any(t.is_alive() for t in threads), "a worker thread hung"
    if errors:
        raise errors[0]
    for (j, i), runs in got.items():
        assert len(runs) == 3
        for out in runs:
            for a, b in zip(out, ref[(j, i)]):
                np.testing.assert_array_equal(a, b, err_msg=f"job {j} series {i}")
    assert len(got) == len(jobs) * n_series

