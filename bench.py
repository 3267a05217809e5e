#!/usr/bin/env python3
"""Throughput benchmark of the MI355X wavelet engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

Default workload = BASELINE config 2 (the metric's single-GPU config): batched Morlet
CWT, 1024 synthetic series x 4096 samples x 128 scales, fp32 in, complex64 W out,
inputs resident in HBM, one step = one transform of the whole batch.

Multi-GPU: series (pairs) are independent, so the units shard across ranks with
no collective on the data path; RCCL carries only the barrier and the max-over-ranks of the
timed region.  The default scaling mode follows BASELINE's wording of each config
(DEFAULT_SCALING): C4 ("512 series pairs ... sharded by pair 1->8 GPUs") and C5 ("65536 series
... sharded across 8xMI355X") are fixed totals, so ``--scaling strong`` splits the config's
batch B into contiguous per-rank blocks (wtmi.sharding.shard_range); C2 and C3 are single-GPU
configs, so at N > 1 ``--scaling weak`` gives rank r its own block [r B, (r + 1) B) of a global
batch of N B series (distinct seeded data per rank, per-GPU work fixed as N grows).  Either
mode can be forced.  The JSON carries each rank's own time for its K steps (min / max over
ranks) and the closing barrier's wait beside the max-over-ranks total.  ``--plan-only`` prints
the ranks' row ranges without touching a GPU.  ``--gpus N`` works two ways:
  * under ``torch.distributed.run --nproc-per-node N`` (RANK/WORLD_SIZE in the env):
    this process is one rank; ``--gpus`` must equal WORLD_SIZE;
  * as a plain ``python bench.py --gpus N``: this process starts N fresh rank processes
    (before it, or they, touch the GPU), waits for them and exits with their status.

Clock ramp: the first few dozen launches after an idle period run ~10 % slower (C2:
0.89 ms/step after 5 warm-up steps, 0.79 after 30 or 300, same box, same process
order).  After the W requested warm-up steps the bench keeps stepping, untimed, until
``--prewarm-s`` seconds (default 0.5) of warm-up have passed; the JSON line records it.

Rank 0 prints ONE JSON line: value = all ranks' coefficients / max-over-ranks time,
plus "roofline" (dominant kernel, HIP-event timed on its own stream) and
"cpu_baseline" (the fp64 oracle restatement of the config's reference path on a
bounded sample, host cores of this box, N = 1 only).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "wavelet-transformer_amd"))
sys.path.insert(0, ROOT)

METRIC = "CWT coefficients/sec (batch×scales×samples) at 1/2/4/8 GPUs; vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
DT = 1 / 12


def synth_batch(rng, B, n, dtype=np.float32):
    """AR(1) red noise (a = 0.7) + 3 sinusoids per series."""
    from scipy.signal import lfilter
    e = rng.standard_normal((B, n))
    x = lfilter([1.0], [1.0, -0.7], e, axis=1)
    t = np.arange(n)[None, :]
    for _ in range(3):
        A = rng.uniform(0.5, 2, (B, 1))
        P = np.exp(rng.uniform(np.log(8), np.log(n / 4), (B, 1)))
        ph = rng.uniform(0, 2 * np.pi, (B, 1))
        x += A * np.sin(2 * np.pi * t / P + ph)
    return x.astype(dtype)


# ------------------------------------------------------------------ CPU baseline
# The oracle restatements (test infrastructure, timed here as the CPU reference):
#   c2 / c5  pycwt.cwt (scipy.fftpack, fp64) per series at the config's shape
#   c3       src/modwt.py modwt + imodwt (scipy.ndimage.convolve1d on zero-stuffed
#            dilated filters -- the reference's own algorithm, bitwise pinned)
#   c4       pycwt.wct (sig=False) per pair, which also forms W12 for the XWT power
def _cpu_worker(args):
    cfg, seed, count = args
    import os as _os
    _os.environ.setdefault("OMP_NUM_THREADS", "1")
    rng = np.random.default_rng(seed)
    if cfg in ("c2", "c5"):
        from oracle import pycwt_spec as pc
        wl = CONFIGS[cfg]
        x = synth_batch(rng, count, wl.n0).astype(np.float64)
        t0 = time.perf_counter()
        for b in range(count):
            S = pc.cwt(x[b], DT, wl.dj, 2 * DT, wl.J)[0].shape[0]
        return time.perf_counter() - t0, count * S * wl.n0
    if cfg == "c3":
        from oracle import modwt_spec as ms
        from wtmi.wavelets import Wavelet
        w = Wavelet("db4")
        x = synth_batch(rng, count, C3.n)  # fp32 in -> fp32 out, as the reference
        t0 = time.perf_counter()
        for b in range(count):
            ms.imodwt(ms.modwt(x[b], w.dec_lo, w.dec_hi, C3.J), w.dec_lo, w.dec_hi)
        return time.perf_counter() - t0, count * (C3.J + 1) * C3.n
    from oracle import pycwt_spec as pc
    y1 = synth_batch(rng, count, C4.n).astype(np.float64)
    y2 = 0.6 * np.roll(y1, 3, axis=1) + 0.8 * synth_batch(rng, count, C4.n)
    t0 = time.perf_counter()
    for b in range(count):
        S = pc.wct(y1[b], y2[b], DT, dj=C4.dj, s0=2 * DT, J=-1, sig=False)[0].shape[0]
    return time.perf_counter() - t0, count * S * C4.n


CPU_SAMPLE = {"c2": "pycwt.cwt restatement (scipy.fftpack, fp64), series x 4096 samples x 128 scales",
              "c5": "pycwt.cwt restatement (scipy.fftpack, fp64), series x 8192 samples x 256 scales",
              "c3": "src/modwt.py modwt+imodwt restatement (scipy convolve1d, dilated db4, J=10), "
                    "series x 16384 samples",
              "c4": "pycwt.wct(sig=False) restatement (2 CWTs + 3 Morlet.smooth, fp64), "
                    "pairs x 8192 samples x 97 scales"}
CPU_PER_WORKER = {"c2": 96, "c5": 24, "c3": 3, "c4": 3}  # ~1-2 s of CPU per worker


def host_cpu_info():
    """Cores this process may use (affinity, capped by a cgroup CPU quota if any) and the
    CPU model, for the cpu_baseline record."""
    visible = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = min(visible, quota) if quota else visible
    return {"usable": usable, "affinity": visible, "cgroup_quota": quota, "model": model}


def cpu_baseline_child(args):
    """The CPU baseline in a child process (a fresh interpreter that never touches the GPU):
    this process then never holds a worker pool, and with --cpu-baseline-when after the host
    cores are busy only once the GPU's timed region is over."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--cpu-baseline-only",
           "--cpu-workers", str(args.cpu_workers), "--cpu-per-worker", str(args.cpu_per_worker)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError(f"CPU baseline child failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(cfg, per_worker, workers, info):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    per_worker = per_worker or CPU_PER_WORKER[cfg]
    jobs = [(cfg, 7000 + i, per_worker) for i in range(workers)]
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    busy = max(r[0] for r in res)
    units = sum(r[1] for r in res)
    return {"value": units / busy, "unit": "coeffs/s", "cores": workers, "kind": "port",
            "cpu_model": info["model"], "host_cpus_affinity": info["affinity"],
            "cgroup_cpu_quota": info["cgroup_quota"],
            "sample": f"{workers * per_worker} x {CPU_SAMPLE[cfg]}; {workers} single-threaded "
                      f"processes x {per_worker}; rate = coefficients / slowest worker's compute "
                      f"time (pool wall {wall:.1f} s)",
            "single_core_value": res[0][1] / res[0][0]}


# ------------------------------------------------------------------- workloads
GEN_BLOCK = 64  # rows per seeded generator block: a shard's rows do not depend on N


def synth_rows(seed, lo, hi, n, pairs=False):
    """Rows [lo, hi) of a config's global synthetic batch (series, or (y1, y2) pairs),
    identical whichever rank or world size asks for them."""
    b0, b1 = lo // GEN_BLOCK, -(-hi // GEN_BLOCK)
    y1, y2 = [], []
    for blk in range(b0, b1):
        rng = np.random.default_rng([seed, blk])
        a = synth_batch(rng, GEN_BLOCK, n)
        y1.append(a)
        if pairs:
            y2.append((0.6 * np.roll(a, 3, axis=1) + 0.8 * synth_batch(rng, GEN_BLOCK, n))
                      .astype(np.float32))
    cut = slice(lo - b0 * GEN_BLOCK, hi - b0 * GEN_BLOCK)
    if pairs:
        return np.concatenate(y1)[cut], np.concatenate(y2)[cut]
    return np.concatenate(y1)[cut]


class Workload:
    """One config's per-rank share: block [r B, (r + 1) B) of a global batch of N B rows
    (weak scaling) or rows [lo, hi) of the batch B split over the ranks (strong)."""
    B = 0
    seed = 0

    def __init__(self, rank, world, dev, scaling):
        import torch
        from wtmi import ops, sharding
        self.ops, self.torch, self.dev = ops, torch, dev
        self.global_batch = self.B * (world if scaling == "weak" else 1)
        if scaling == "weak":
            self.lo, self.hi = rank * self.B, (rank + 1) * self.B
        else:
            self.lo, self.hi = sharding.shard_range(self.B, rank, world)
        self.local = self.hi - self.lo
        self.setup()

    def outputs(self):
        """What this rank's step leaves in HBM for a consumer: the device tensors the host
        gather copies back, and a note saying what they are."""
        return [], "none"

    def shard_config(self, world, scaling):
        return {"global_batch": self.global_batch, "per_rank_batch": self.local,
                "rank0_rows": [self.lo, self.hi], "scaling": scaling,
                "parallelism": f"{self.axis}-sharded x{world}, contiguous blocks, "
                               "no collective on the data path"}


class C2(Workload):
    """Batched Morlet CWT: 1024 x 4096 x 128 scales, complex64 W."""
    name, axis, seed = "c2", "series", 1002
    B, n0, dj, J = 1024, 4096, 1 / 12, 127
    kernel = "cwt_morlet_kernel<12,1,0,0>"
    PER_STEP = {"wtmi::cwt_morlet_kernel<12": 1}  # kernel-name prefix -> launches per step

    def setup(self):
        torch = self.torch
        self.x = torch.tensor(synth_rows(self.seed, self.lo, self.hi, self.n0), device=self.dev)
        self.sj = 2 * DT * 2 ** (np.arange(self.J + 1) * self.dj)
        self.sjd = torch.tensor(self.sj, device=self.dev)
        self.out = torch.empty((self.local, self.sj.size, self.n0), dtype=torch.complex64,
                               device=self.dev)
        self.units = self.local * self.sj.size * self.n0
        self.bytes = self.units * 8 + self.local * self.n0 * 4  # W write + x read
        self.per_step = dict(self.PER_STEP)
        self.bytes_note = "8 B/coeff complex64 W write + 4 B/sample x read"

    def step(self):
        if self.local:
            self.ops.cwt_morlet(self.x, self.sjd, DT, 6.0, out_w=self.out)

    def _oracle_rows(self, W, x):
        from oracle import pycwt_spec as pc
        ref = pc.cwt(x.astype(np.float64), DT, self.dj, 2 * DT, self.J)[0]
        return float((np.linalg.norm(W.astype(np.complex128) - ref, axis=1)
                      / np.linalg.norm(ref, axis=1)).max())

    def outputs(self):
        return [self.out], "complex64 W [series, scales, samples]"

    def check(self):
        """First and last series of this rank's output vs the oracle (max row error)."""
        rows = sorted({0, self.local - 1})
        return max(self._oracle_rows(self.out[r].cpu().numpy(), self.x[r].cpu().numpy())
                   for r in rows)

    def config(self):
        return {"workload": "C2: batched Morlet CWT (BASELINE configs[1])", "samples": self.n0,
                "scales": int(self.sj.size), "dt": DT, "dj": self.dj, "s0": 2 * DT, "f0": 6.0,
                "output": "complex64 W"}


class C5(C2):
    """Large-batch CWT: 65536 series x 8192 x 256 scales (dj = 1/24), each rank streaming
    its series in chunks of 512 into one reused output buffer (one-box sweep, ms per 8192
    series: chunk 256 27.9-28.0, 512 27.2-27.3, 1024 27.5)."""
    name, axis, seed = "c5", "series", 1005
    B, n0, dj, J = 65536, 8192, 1 / 24, 255
    chunk = 512
    kernel = "cwt_morlet_kernel<13,1,0,0>"

    def setup(self):
        torch = self.torch
        x = np.empty((self.local, self.n0), np.float32)
        for c in range(0, self.local, 4096):  # bounded host temporaries
            x[c:c + 4096] = synth_rows(self.seed, self.lo + c, min(self.hi, self.lo + c + 4096),
                                       self.n0)
        self.x = torch.tensor(x, device=self.dev)
        del x
        self.sj = 2 * DT * 2 ** (np.arange(self.J + 1) * self.dj)
        self.sjd = torch.tensor(self.sj, device=self.dev)
        self.out = torch.empty((min(self.chunk, max(self.local, 1)), self.sj.size, self.n0),
                               dtype=torch.complex64, device=self.dev)
        self.units = self.local * self.sj.size * self.n0
        self.bytes = self.units * 8 + self.local * self.n0 * 4
        self.per_step = {"wtmi::cwt_morlet_kernel<13": -(-self.local // self.chunk)}
        self.bytes_note = "8 B/coeff complex64 W write + 4 B/sample x read"

    def step(self):
        for c in range(0, self.local, self.chunk):
            e = min(self.local, c + self.chunk)
            self.ops.cwt_morlet(self.x[c:e], self.sjd, DT, 6.0, out_w=self.out[:e - c])

    def outputs(self):
        """C5's W is never resident (1.1 PB): what a consumer takes home is a checksum per
        series of the chunk in the buffer (sum of |W|^2 over scales and samples, fp64) plus
        the sampled parity subset -- the chunk's first, middle and last series' whole W."""
        torch = self.torch
        n = min(self.chunk, self.local)
        if n == 0:
            return [], "none"
        chk = self.out[:n].abs().square().sum(dim=(1, 2), dtype=torch.float64)
        rows = sorted({0, n // 2, n - 1})
        return [chk, self.out[rows]], ("per-series checksums (f64) of the last chunk + the W rows "
                                       "of its series %s" % rows)

    def check(self):
        """The last chunk's first and last series (the buffer holds the last chunk)."""
        c0 = (self.local - 1) // self.chunk * self.chunk
        rows = sorted({0, self.local - 1 - c0})
        return max(self._oracle_rows(self.out[r].cpu().numpy(), self.x[c0 + r].cpu().numpy())
                   for r in rows)

    def config(self):
        d = super().config()
        d.update(workload="C5: large-batch streamed Morlet CWT (BASELINE configs[4])",
                 chunk_series=self.chunk)
        return d


class C3(Workload):
    """MODWT db4 J=10: 8192 x 16384, decompose + reconstruct."""
    name, axis, seed = "c3", "series", 1003
    B, n, J = 8192, 16384, 10
    kernel = "modwt_vec_kernel<8,4,1024,16>+imodwt_hyb_kernel<8,8,512,2,1024>"
    PER_STEP = {"wtmi::modwt_vec_kernel<": 1, "wtmi::imodwt_hyb_kernel<": 1}

    def setup(self):
        from wtmi.wavelets import Wavelet
        self.w = Wavelet("db4")
        x = np.empty((self.local, self.n), np.float32)
        for c in range(0, self.local, 1024):
            x[c:c + 1024] = synth_rows(self.seed, self.lo + c, min(self.hi, self.lo + c + 1024), self.n)
        self.x = self.torch.tensor(x, device=self.dev)
        self.units = self.local * (self.J + 1) * self.n
        self.bytes = self.local * self.n * 96  # 4 x + 44 W write + 44 W read + 4 x^
        self.per_step = dict(self.PER_STEP)
        self.bytes_note = "96 B per series-sample (x, W write, W read, x^)"

    def step(self):
        if self.local:
            w = self.ops.modwt(self.x, self.w.dec_lo, self.w.dec_hi, self.J)
            self.xr = self.ops.imodwt(w, self.w.dec_lo, self.w.dec_hi)
            self.coeffs = w

    def outputs(self):
        return [self.coeffs, self.xr], "f32 MODWT rows [series, J+1, samples] + reconstruction"

    def check(self):
        return float((self.xr - self.x).abs().max().item() / self.x.abs().max().item())

    def config(self):
        return {"workload": "C3: MODWT db4 J=10 decompose+reconstruct (BASELINE configs[2])",
                "samples": self.n, "levels": self.J}


class C4(Workload):
    """XWT + WCT: 512 pairs x 8192, dj = 1/8 -> 97 scales."""
    name, axis, seed = "c4", "pair", 1004
    B, n, dj = 512, 8192, 1 / 8
    kernel = ("wct_spectra_plan<13> (normalisation in the load, plan in the last workgroup) + "
              "wct_phase_a<13,full-band rows> [side stream] || wct_dec_kernel<13,8..12> + "
              "wct_phase_a<13,decimated rows> + wct_phase_b<10> [caller's stream], "
              "wct_wide_boxcar<10> + wct_phase_c<13,q windows> + wct_phase_c<13,wide windows> "
              "[side stream]; joined on the caller's stream")
    # every wtmi::wct_* kernel of the step once (r03: the normalisation runs inside
    # wct_spectra_plan; no separate moments launches)
    PER_STEP = {"wtmi::wct_": 1}

    def setup(self):
        from wtmi import transforms
        torch, dev = self.torch, self.dev
        self.T = transforms
        y1, y2 = synth_rows(self.seed, self.lo, self.hi, self.n, pairs=True)
        self.y1 = torch.tensor(y1, device=dev)
        self.y2 = torch.tensor(y2, device=dev)
        self.sj, _ = transforms.scales_for(self.n, DT, self.dj, 2 * DT, -1, transforms.as_morlet(None))
        self.sjd = torch.tensor(self.sj, device=dev)
        self.K = transforms.boxcar_rows(transforms.as_morlet(None), self.dj)
        S = self.sj.size
        self.units = self.local * S * self.n
        self.bytes = self.units * 12 + self.local * self.n * 8
        self.ws = torch.empty(self.ops.wct_workspace_bytes(max(self.local, 1), self.n, S),
                              dtype=torch.uint8, device=dev)
        self.per_step = dict(self.PER_STEP)
        self.bytes_note = "12 B/coeff (|W12|^2 + WCT + phase, f32) + 8 B/pair-sample inputs"

    def step(self):
        # one fused pass: XWT power |W1 W2*|^2, phase angle and WCT coherence
        # (transforms.wct_batch's launches: pycwt's normalisation fused into the first kernel)
        if self.local:
            self.r = self.ops.wct_morlet(self.y1, self.y2, self.sjd, DT, 6.0, boxcar=self.K,
                                         want_uv=False, want_power=True, want_phase=True,
                                         workspace=self.ws, normalize=True)

    def outputs(self):
        return [self.r["power"], self.r["coh"], self.r["phase"]], \
            "f32 |W12|^2, WCT, phase [pairs, scales, samples]"

    def check(self):
        """First and last pair's coherence vs the oracle's pycwt.wct (max abs difference)."""
        from oracle import pycwt_spec as pc
        err = 0.0
        for p in sorted({0, self.local - 1}):
            y1 = self.y1[p].cpu().numpy().astype(np.float64)
            y2 = self.y2[p].cpu().numpy().astype(np.float64)
            ref = pc.wct(y1, y2, DT, dj=self.dj, s0=2 * DT, J=-1, sig=False)[0]
            err = max(err, float(np.abs(self.r["coh"][p].cpu().numpy() - ref).max()))
        return err

    def config(self):
        return {"workload": "C4: XWT + WCT coherence (BASELINE configs[3])", "samples": self.n,
                "scales": int(self.sj.size)}


class Stub(Workload):
    """CPU-only stand-in (tests of the launcher and sharding; never a bench line)."""
    name, axis, seed = "stub", "series", 7
    B, n = 10, 256
    kernel = "stub"

    def setup(self):
        self.x = self.torch.tensor(synth_rows(self.seed, self.lo, self.hi, self.n), device=self.dev)
        self.units = self.local * self.n
        self.bytes = self.local * self.n * 8
        self.per_step = {}
        self.bytes_note = "stub"

    def step(self):
        self.y = self.torch.fft.rfft(self.x, dim=-1)

    def check(self):
        return float(self.x.sum().item())

    def config(self):
        return {"workload": "stub (CPU launcher test)", "samples": self.n}


CONFIGS = {"c2": C2, "c3": C3, "c4": C4, "c5": C5, "stub": Stub}
# Default scaling mode per config (BASELINE.json configs): C4 ("512 series pairs ...
# sharded by pair 1->8 GPUs") and C5 ("65536 series ... sharded across 8xMI355X") name a FIXED
# total batch split over the GPUs -- strong scaling; C2 and C3 are single-GPU configs, so at
# N > 1 every GPU runs the whole config on its own series -- weak scaling.
# hipGraph replay of the step (--graph 1): measured no faster for any config, C4's shards
# included (profiles/r04/shard_sizes.txt: the kernels' own tails, not the host's launches, cost
# the small-batch efficiency), so no config uses it by default
DEFAULT_GRAPH: dict = {}
DEFAULT_SCALING = {"c2": "weak", "c3": "weak", "c4": "strong", "c5": "strong", "stub": "weak"}


def shard_plan(cfg, world, scaling):
    """Every rank's rows [lo, hi) of the config under the scaling mode (no GPU touched)."""
    from wtmi import sharding
    B = CONFIGS[cfg].B
    if scaling == "weak":
        return B * world, [[r * B, (r + 1) * B] for r in range(world)]
    return B, [list(sharding.shard_range(B, r, world)) for r in range(world)]
CHECK_NAME = {"c2": "rank0_first_last_series_max_row_rel_err_vs_oracle",
              "c5": "rank0_last_chunk_first_last_series_max_row_rel_err_vs_oracle",
              "c3": "rank0_round_trip_max_err_rel_to_max_x",
              "c4": "rank0_first_last_pair_coherence_max_abs_err_vs_oracle",
              "stub": "rank0_sum"}


def kernel_roofline(cfg):
    """Per-kernel roofline of the config from the newest committed profile
    (profiles/rNN/kernel_roofline.json, scripts/kernel_roofline.py): each kernel's duration
    (rocprofv3 trace of the timed steps), HBM bytes (PMC) and VALU issue share (PMC), and the
    resource that binds it."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_roofline.json")), reverse=True):
        with open(path) as fh:
            ent = json.load(fh).get(cfg)
        if ent:
            keep = ("kernel", "ms", "bound", "frac", "hbm_GBps", "hbm_frac", "valu_busy")
            return [{k: r[k] for k in keep} for r in ent["kernels"]], os.path.relpath(path, ROOT)
    return None, None


VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 4  # 1024 SIMDs x 2.4 GHz, one wave64 VALU op per 4 cycles


def step_bound(cfg, per_step, step_ms, hbm_frac):
    """The step's binding resource from the newest committed per-kernel profile: the HBM
    fraction of the step (algorithmic bytes / step time / peak, measured live) beside its VALU
    fraction (the profile's SQ_INSTS_VALU of every kernel of the step x 4 cycles, over the
    chip's 1024 SIMDs x 2.4 GHz x the live step time); bound = the larger.  Without a profile
    holding every kernel of the step: "hbm" and no VALU fraction."""
    import glob
    out = {"bound": "hbm", "hbm": hbm_frac, "valu": None, "valu_insts_per_step": None,
           "source": None,
           "note": "valu = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz x step time): a model. "
                   "MI355X_MICROARCH's measured issue costs: v_fma_f32 2 cycles per SIMD-32 with "
                   "several waves (4 for one wave alone), transcendentals 8, so a single rate is an "
                   "approximation; the per-kernel valu_busy (SQ_ACTIVE_INST_VALU) measured beside it "
                   "agrees within ~10 % for the WCT kernels (e.g. 0.63 measured vs 0.57 modelled)"}
    if not per_step or not step_ms:
        return out
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_roofline.json")), reverse=True):
        with open(path) as fh:
            ent = json.load(fh).get(cfg)
        if not ent:
            continue
        insts, seen = 0.0, 0
        for prefix, count in per_step.items():
            hits = [k for k in ent["kernels"] if k["kernel"].startswith(prefix) and k.get("valu_insts")]
            if not hits:
                break
            insts += sum(k["valu_insts"] for k in hits) * count
            seen += 1
        if seen != len(per_step):
            continue
        valu = insts / (VALU_PEAK_WAVE_INSTS * step_ms * 1e-3)
        out.update(bound="valu" if valu > hbm_frac else "hbm", valu=valu, valu_insts_per_step=insts,
                   source=os.path.relpath(path, ROOT))
        return out
    return out


def measure_gather(wl, pageable=True):
    """Host gather of this rank's output, after and outside the timed region (SURVEY 8(d)/(e):
    "D2H into pinned buffers, timed separately"): the page-locked buffers are allocated first
    (timed on their own: a consumer keeps them), then the copy of every output tensor into
    them is timed, and the same copy into pageable memory beside it.  Bytes are the outputs'."""
    try:
        return _measure_gather(wl, pageable)
    except Exception as e:  # a host without page-locked memory to spare must not lose the line
        return {"error": f"{type(e).__name__}: {e}"}


def _measure_gather(wl, pageable):
    import torch
    from wtmi import sharding
    outs, what = wl.outputs()
    nbytes = sum(t.numel() * t.element_size() for t in outs)
    rec = {"what": what, "bytes": nbytes}
    if not outs or nbytes == 0:
        return rec
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bufs = [sharding.pinned_buffer(t.shape, t.dtype, reuse=False) for t in outs]
    rec["pinned_alloc_ms"] = (time.perf_counter() - t0) * 1e3
    # warm the copy path once on a small slice (first-call driver set-up is not transfer time)
    sharding.d2h(outs[0].reshape(-1)[:1024], out=bufs[0].reshape(-1)[:1024])
    best = None
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t, b in zip(outs, bufs):
            sharding.d2h(t, out=b)
        ms = (time.perf_counter() - t0) * 1e3
        best = ms if best is None else min(best, ms)
    rec.update(pinned_ms=best, pinned_GBps=nbytes / best / 1e6,
               note="best of 2 copies into the same page-locked buffers; value excludes it")
    if pageable:
        host = [torch.empty(t.shape, dtype=t.dtype) for t in outs]
        for h in host:  # first-touch the pages outside the clock
            h.reshape(-1).view(torch.uint8)[::4096] = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t, h in zip(outs, host):
            h.copy_(t)
        ms = (time.perf_counter() - t0) * 1e3
        rec.update(pageable_ms=ms, pageable_GBps=nbytes / ms / 1e6)
        del host
    del bufs
    return rec


def pmc_traffic(cfg, per_step):
    """HBM bytes per step of the roofline kernels from the newest committed PMC pass
    (profiles/rNN/pmc_traffic.json, written by scripts/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench), or None."""
    import glob
    if not per_step:
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        with open(path) as fh:
            ent = json.load(fh).get(cfg)
        if not ent:
            continue
        total, seen = 0.0, 0
        for prefix, count in per_step.items():  # every kernel of the prefix, `count` launches each
            hits = [v for k, v in ent["kernels"].items() if k.startswith(prefix)]
            if not hits:
                break
            total += sum(h["hbm_bytes"] for h in hits) * count
            seen += 1
        if seen == len(per_step):
            return total, os.path.relpath(path, ROOT)
    return None, None


# -------------------------------------------------------------------- launcher
def _stop_all(procs, grace=10.0):
    """SIGTERM every live rank, then SIGKILL what is still alive after `grace` seconds."""
    for q in procs:
        if q.poll() is None:
            q.terminate()
    deadline = time.monotonic() + grace
    for q in procs:
        try:
            q.wait(timeout=max(0.1, deadline - time.monotonic()))
        except Exception:  # noqa: BLE001  (subprocess.TimeoutExpired)
            q.kill()
            q.wait()


def launch_ranks(n, argv, timeout_s=0.0):
    """``python bench.py --gpus N`` without torch.distributed.run: start N fresh rank
    processes (this parent never initialises the GPU), stream their output, stop the
    others as soon as one fails, and return the worst exit status.  The ranks never
    outlive this parent: on any exit path (an exception, SIGINT / SIGTERM, or the
    optional wall-clock limit `timeout_s`, exit status 124) the survivors are terminated
    and then killed."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []

    def _on_signal(signum, _frame):
        raise SystemExit(128 + signum)

    old = {sig: signal.signal(sig, _on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    t0 = time.monotonic()
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                          env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0:
                    rc = rc or code
                    _stop_all(live)
            if timeout_s and live and time.monotonic() - t0 > timeout_s:
                print(f"bench: ranks still running after {timeout_s:.0f} s; stopping them",
                      file=sys.stderr, flush=True)
                rc = rc or 124
                _stop_all(live)
            time.sleep(0.05)
    finally:
        _stop_all(procs)
        for sig, h in old.items():
            signal.signal(sig, h)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="keep warming up (untimed) until this many seconds have passed")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="weak: every rank its own B-row block (per-GPU work fixed); strong: the "
                         "config's B rows split over the ranks.  Default: strong for c4 / c5 "
                         "(BASELINE's fixed totals sharded 1->8), weak for c2 / c3")
    ap.add_argument("--graph", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: capture one step in a hipGraph and replay it in the timed loop; "
                         "0: launch every step; -1 (default): per config (DEFAULT_GRAPH)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the ranks' row ranges for --gpus / --config / --scaling as JSON "
                         "and exit (no GPU)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = every usable host core")
    ap.add_argument("--cpu-per-worker", type=int, default=0, help="0 = per-config default")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-when", default="after", choices=["before", "after"],
                    help="run the CPU baseline (a child process) before GPU set-up or after the "
                         "timed region: run before, it slowed the timed C2 kernel 5-12 %%")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo + the stub workload only (launcher tests)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one GPU per rank: the measured mode) or gloo (smoke mode: "
                         "ranks may share a GPU, rank r on cuda:(r mod device count))")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group even at --gpus 1 (RANK 0 of WORLD_SIZE 1 on "
                         "127.0.0.1): the RCCL barrier / all-reduce / gloo side-group gather run on "
                         "one GPU")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the host-gather measurement after the timed region")
    ap.add_argument("--rank-timeout", type=float, default=0.0,
                    help="self-launched ranks: wall-clock limit in seconds (0 = none)")
    args = ap.parse_args()
    if args.device == "cpu" and args.config != "stub":
        ap.error("--device cpu runs only --config stub")
    if args.scaling is None:
        args.scaling = DEFAULT_SCALING[args.config]
    if args.plan_only:
        total, ranges = shard_plan(args.config, args.gpus, args.scaling)
        print(json.dumps({"config": args.config, "scaling": args.scaling, "global_batch": total,
                          "ranks": ranges}), flush=True)
        return 0

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:], args.rank_timeout)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wl_cls = CONFIGS[args.config]

    if args.cpu_baseline_only:  # the child of cpu_baseline_child(): no GPU, one JSON line
        info = host_cpu_info()
        workers = args.cpu_workers or info["usable"]
        print(json.dumps(cpu_baseline(args.config, args.cpu_per_worker, workers, info)), flush=True)
        return
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and args.config != "stub"
    cpu = cpu_baseline_child(args) if want_cpu and args.cpu_baseline_when == "before" else None

    import torch
    import torch.distributed as dist

    from wtmi import sharding
    rccl = args.device == "cuda" and args.dist_backend == "nccl"
    if args.device == "cuda":
        # RCCL: one GPU per rank.  gloo smoke mode: ranks may share a device.
        dev = torch.device("cuda", local if rccl else local % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        sync = torch.cuda.synchronize
    else:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    dist_on = world > 1 or args.force_dist
    if dist_on:
        if world == 1:  # --force-dist without a launcher: a one-rank group on 127.0.0.1
            import socket
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                with socket.socket() as s:
                    s.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if rccl:
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    wl = wl_cls(rank, world, dev, args.scaling)
    sync()

    def barrier():
        if dist_on:
            if rccl:
                dist.barrier(device_ids=[dev.index])
            else:
                dist.barrier()

    t_warm = time.perf_counter()
    for _ in range(args.warmup):
        wl.step()
    sync()
    extra = 0
    while time.perf_counter() - t_warm < args.prewarm_s:
        # back-to-back steps (a sync per 16): a host sync after every step left the GPU idle
        # between them, and the timed region then opened below the loaded clock
        for _ in range(16):
            wl.step()
        sync()
        extra += 16
    barrier()
    sync()

    use_graph = (DEFAULT_GRAPH.get(args.config, 0) if args.graph < 0 else args.graph) and \
        args.device == "cuda" and wl.local > 0
    if use_graph:
        # one step captured (its launches, the WCT's side-stream fork / join included) and
        # replayed: the same kernels on the same buffers, enqueued by one hipGraphLaunch
        graph = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            wl.step()
        torch.cuda.current_stream(dev).wait_stream(cs)
        sync()
        with torch.cuda.graph(graph):
            wl.step()
        for _ in range(max(3, args.warmup // 4)):
            graph.replay()
        sync()
        step = graph.replay
    else:
        step = wl.step
    barrier()
    sync()

    if args.device == "cuda":
        stream = torch.cuda.current_stream(dev)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.device == "cuda":
            evs[i][0].record(stream)
        step()
        if args.device == "cuda":
            evs[i][1].record(stream)
    sync()
    t_own = time.perf_counter() - t0  # this rank's steps, before waiting for the others
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t_barrier = elapsed - t_own
    if args.device == "cuda":
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    else:
        kern_ms = elapsed / max(args.steps, 1) * 1e3

    # max over ranks of the timed region, sum of the units (a device tensor under RCCL,
    # a host tensor under gloo: wtmi.sharding)
    tmax = sharding.max_over_ranks(elapsed)
    units_all = sharding.sum_over_ranks(float(wl.units))
    own_max, own_min = sharding.max_over_ranks(t_own), -sharding.max_over_ranks(-t_own)
    bar_max, bar_min = sharding.max_over_ranks(t_barrier), -sharding.max_over_ranks(-t_barrier)
    check = wl.check() if rank == 0 and wl.local else None
    gather_rec = None
    if args.device == "cuda" and not args.no_gather:
        # the pageable comparison only at N = 1 (N ranks' pageable copies would double the host
        # memory the gather holds)
        gather_rec = measure_gather(wl, pageable=world == 1)
        if dist_on:  # the slowest rank's copy (each rank gathers its own block)
            gather_rec["pinned_ms_max_over_ranks"] = sharding.max_over_ranks(gather_rec.get("pinned_ms", 0.0))
    gathered = None
    if dist_on:
        # the host-side gather of sharding.gather_to_rank0 (a gloo side group under RCCL):
        # every rank's first row count and units, gathered on rank 0
        mine = torch.tensor([[float(wl.lo), float(wl.units)]], dtype=torch.float64)
        g = sharding.gather_to_rank0(mine, world)
        gathered = None if g is None else g.tolist()
    if want_cpu and cpu is None:  # after the timed region (default)
        cpu = cpu_baseline_child(args)

    if rank == 0:
        achieved = wl.bytes / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(args.config, wl.per_step)
        per_kernel, ksrc = kernel_roofline(args.config)
        sb = step_bound(args.config, wl.per_step, kern_ms, achieved / HBM_PEAK_GBS)
        cfg = wl.config()
        cfg.update(wl.shard_config(world, args.scaling))
        if dist_on:
            cfg["dist_backend"] = "rccl" if rccl else "gloo"
            cfg["dist_gather"] = gathered
            if not rccl and args.device == "cuda":
                cfg["devices"] = "shared: rank r on cuda:(r mod %d) (gloo smoke mode, not a scaling "\
                                 "measurement)" % torch.cuda.device_count()
        line = {
            "metric": METRIC,
            "value": units_all * args.steps / tmax,
            "unit": "coeffs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm": {"min_seconds": args.prewarm_s, "extra_untimed_steps": extra},
            "ms_per_step": tmax / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded AR(1) red noise (a=0.7) + 3 random sinusoids per series, "
                    "resident in HBM before timing",
            "config": cfg,
            "roofline": {"bound": sb["bound"], "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "step_fractions": {"hbm": sb["hbm"], "valu": sb["valu"],
                                            "valu_insts_per_step": sb["valu_insts_per_step"],
                                            "valu_peak": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 "
                                                         "VALU instruction",
                                            "source": sb["source"],
                                            "note": "achieved / peak / frac above are the HBM "
                                                    "fraction; bound is the larger of the two"},
                         "traffic_source": tsrc, "scope": "rank 0's launches",
                         "kernel": wl.kernel, "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": wl.bytes, "bytes_model": wl.bytes_note,
                         "per_kernel": per_kernel, "per_kernel_source": ksrc},
            "cpu_baseline": cpu,
            "check": {CHECK_NAME[args.config]: check},
            "ranks": {"own_steps_ms_per_step": {"min": own_min / args.steps * 1e3,
                                                "max": own_max / args.steps * 1e3},
                      "closing_barrier_ms": {"min": bar_min * 1e3, "max": bar_max * 1e3},
                      "note": "own = a rank's K steps up to its sync, before the closing barrier; "
                              "value uses the max over ranks of own + barrier"},
            "graph": bool(use_graph),
            "gather": gather_rec,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
