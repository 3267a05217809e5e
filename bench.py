#!/usr/bin/env python3
"""Throughput benchmark of the MI355X wavelet engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

Default workload = BASELINE config 2 (the metric's single-GPU config): batched Morlet
CWT, 1024 synthetic series x 4096 samples x 128 scales, fp32 in, complex64 W out,
inputs resident in HBM, one step = one transform of the whole per-GPU batch.  With
N > 1 (launched by torch.distributed.run) every rank transforms its own 1024-series
shard (weak scaling, no collective on the data path); RCCL is used only for the
barrier and the max-over-ranks of the timed region.

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
CPU_PER_WORKER = {"c2": 32, "c5": 10, "c3": 2, "c4": 2}  # ~1 s per worker, ~16 s of CPU in all


def cpu_baseline(cfg, per_worker, workers):
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
            "sample": f"{workers * per_worker} x {CPU_SAMPLE[cfg]}; {workers} single-threaded "
                      f"processes x {per_worker}; rate = coefficients / slowest worker's compute "
                      f"time (pool wall {wall:.1f} s)",
            "single_core_value": res[0][1] / res[0][0]}


# ------------------------------------------------------------------- workloads
class C2:
    """Batched Morlet CWT: 1024 x 4096 x 128 scales, complex64 W."""
    name = "c2"
    B, n0, dj, J = 1024, 4096, 1 / 12, 127

    def __init__(self, rank, dev):
        import torch
        from wtmi import ops
        self.ops, self.torch = ops, torch
        rng = np.random.default_rng(1002 + 7919 * rank)
        self.x = torch.tensor(synth_batch(rng, self.B, self.n0), device=dev)
        self.sj = 2 * DT * 2 ** (np.arange(self.J + 1) * self.dj)
        self.sjd = torch.tensor(self.sj, device=dev)
        self.out = torch.empty((self.B, self.sj.size, self.n0), dtype=torch.complex64, device=dev)
        self.units = self.B * self.sj.size * self.n0
        self.bytes = self.units * 8 + self.B * self.n0 * 4  # W write + x read
        self.kernel = "cwt_morlet_kernel<12,1,0,0>"
        self.per_step = {"wtmi::cwt_morlet_kernel<12": 1}
        self.unit_name = "coeffs/s"
        self.bytes_note = "8 B/coeff complex64 W write + 4 B/sample x read"

    def step(self):
        self.ops.cwt_morlet(self.x, self.sjd, DT, 6.0, out_w=self.out)

    def check(self):
        """Cheap size-independent check on the timed output: row 0 vs oracle."""
        from oracle import pycwt_spec as pc
        W = self.out[0].cpu().numpy().astype(np.complex128)
        ref = pc.cwt(self.x[0].cpu().numpy().astype(np.float64), DT, self.dj, 2 * DT, self.J)[0]
        num = np.linalg.norm(W - ref, axis=1)
        den = np.linalg.norm(ref, axis=1)
        return float((num / den).max())

    def config(self, world):
        return {"workload": "C2: batched Morlet CWT (BASELINE configs[1])", "series_per_gpu": self.B,
                "global_batch": self.B * world, "samples": self.n0, "scales": int(self.sj.size),
                "dt": DT, "dj": self.dj, "s0": 2 * DT, "f0": 6.0, "output": "complex64 W",
                "parallelism": f"series-sharded x{world} (no collective on the data path)"}


class C5(C2):
    """Large-batch CWT: 8192 series/GPU x 8192 x 256 scales (dj = 1/24), streamed in
    chunks of 512 series into a reused output buffer (one-box sweep, ms per step: chunk 256
    27.9-28.0, 512 27.2-27.3, 1024 27.5)."""
    name = "c5"
    B, n0, dj, J = 8192, 8192, 1 / 24, 255
    chunk = int(os.environ.get("WTMI_C5_CHUNK", "512"))

    def __init__(self, rank, dev):
        import torch
        from wtmi import ops
        self.ops, self.torch = ops, torch
        rng = np.random.default_rng(1005 + 7919 * rank)
        self.x = torch.tensor(synth_batch(rng, self.B, self.n0), device=dev)
        self.sj = 2 * DT * 2 ** (np.arange(self.J + 1) * self.dj)
        self.sjd = torch.tensor(self.sj, device=dev)
        self.out = torch.empty((self.chunk, self.sj.size, self.n0), dtype=torch.complex64,
                               device=dev)
        self.units = self.B * self.sj.size * self.n0
        self.bytes = self.units * 8 + self.B * self.n0 * 4
        self.kernel = "cwt_morlet_kernel<13,1,0,0>"
        self.per_step = {"wtmi::cwt_morlet_kernel<13": self.B // self.chunk}
        self.unit_name = "coeffs/s"
        self.bytes_note = "8 B/coeff complex64 W write + 4 B/sample x read"

    def step(self):
        for c in range(0, self.B, self.chunk):
            self.ops.cwt_morlet(self.x[c:c + self.chunk], self.sjd, DT, 6.0, out_w=self.out)

    def check(self):
        from oracle import pycwt_spec as pc
        W = self.out[0].cpu().numpy().astype(np.complex128)  # last chunk, first series
        x0 = self.x[self.B - self.chunk].cpu().numpy().astype(np.float64)
        ref = pc.cwt(x0, DT, self.dj, 2 * DT, self.J)[0]
        return float((np.linalg.norm(W - ref, axis=1) / np.linalg.norm(ref, axis=1)).max())

    def config(self, world):
        d = super().config(world)
        d.update(workload="C5: large-batch streamed Morlet CWT (BASELINE configs[4])",
                 chunk_series=self.chunk)
        return d


class C3:
    """MODWT db4 J=10: 8192 x 16384, decompose + reconstruct."""
    name = "c3"
    B, n, J = 8192, 16384, 10

    def __init__(self, rank, dev):
        import torch
        from wtmi import ops
        from wtmi.wavelets import Wavelet
        self.ops, self.torch = ops, torch
        self.w = Wavelet("db4")
        rng = np.random.default_rng(1003 + 7919 * rank)
        self.x = torch.tensor(synth_batch(rng, self.B, self.n), device=dev)
        self.units = self.B * (self.J + 1) * self.n
        self.bytes = self.B * self.n * 96  # 4 x + 44 W write + 44 W read + 4 x^
        self.kernel = "modwt_vec_kernel<8,8,512,16>+imodwt_vec_kernel<8,8,512,3>"
        self.per_step = {"wtmi::modwt_vec_kernel<": 1, "wtmi::imodwt_vec_kernel<": 1}
        self.unit_name = "coeffs/s"
        self.bytes_note = "96 B per series-sample (x, W write, W read, x^)"

    def step(self):
        w = self.ops.modwt(self.x, self.w.dec_lo, self.w.dec_hi, self.J)
        self.xr = self.ops.imodwt(w, self.w.dec_lo, self.w.dec_hi)

    def check(self):
        return float((self.xr - self.x).abs().max().item() / self.x.abs().max().item())

    def config(self, world):
        return {"workload": "C3: MODWT db4 J=10 decompose+reconstruct (BASELINE configs[2])",
                "series_per_gpu": self.B, "global_batch": self.B * world, "samples": self.n,
                "levels": self.J, "parallelism": f"series-sharded x{world}"}


class C4:
    """XWT + WCT: 512 pairs x 8192, dj = 1/8 -> 97 scales."""
    name = "c4"
    P, n, dj = 512, 8192, 1 / 8

    def __init__(self, rank, dev):
        import torch
        from wtmi import ops, transforms
        self.ops, self.T, self.torch = ops, transforms, torch
        rng = np.random.default_rng(1004 + 7919 * rank)
        y1 = synth_batch(rng, self.P, self.n)
        y2 = (0.6 * np.roll(y1, 3, axis=1) + 0.8 * synth_batch(rng, self.P, self.n)).astype(np.float32)
        self.y1 = torch.tensor(y1, device=dev)
        self.y2 = torch.tensor(y2, device=dev)
        self.sj, _ = transforms.scales_for(self.n, DT, self.dj, 2 * DT, -1, transforms.as_morlet(None))
        S = self.sj.size
        self.units = self.P * S * self.n
        self.bytes = self.units * 12 + self.P * self.n * 8
        self.ws = torch.empty(ops.wct_workspace_bytes(self.P, self.n, S), dtype=torch.uint8,
                              device=dev)
        self.kernel = "wct_plan<13>+wct_spectra<13>+wct_phase_a<13>+wct_phase_c<13>+wct_phase_b<10>"
        self.per_step = {"wtmi::wct_plan_kernel<": 1, "wtmi::wct_spectra<": 1, "wtmi::wct_phase_a<": 1,
                         "wtmi::wct_phase_c<": 1, "wtmi::wct_phase_b<": 1}
        self.unit_name = "coeffs/s"
        self.bytes_note = "12 B/coeff (|W12|^2 + WCT + phase, f32) + 8 B/pair-sample inputs"

    def step(self):
        # one fused pass: XWT power |W1 W2*|^2, phase angle and WCT coherence
        self.r = self.T.wct_batch(self.y1, self.y2, DT, self.dj, 2 * DT, -1, workspace=self.ws,
                                  want_uv=False, want_power=True, want_phase=True)[0]

    def check(self):
        """Pair 0's coherence vs the oracle's pycwt.wct restatement (max abs difference)."""
        from oracle import pycwt_spec as pc
        y1 = self.y1[0].cpu().numpy().astype(np.float64)
        y2 = self.y2[0].cpu().numpy().astype(np.float64)
        ref = pc.wct(y1, y2, DT, dj=self.dj, s0=2 * DT, J=-1, sig=False)[0]
        return float(np.abs(self.r["coh"][0].cpu().numpy() - ref).max())

    def config(self, world):
        return {"workload": "C4: XWT + WCT coherence (BASELINE configs[3])", "pairs_per_gpu": self.P,
                "global_batch": self.P * world, "samples": self.n, "scales": int(self.sj.size),
                "parallelism": f"pair-sharded x{world}"}


CONFIGS = {"c2": C2, "c3": C3, "c4": C4, "c5": C5}
CHECK_NAME = {"c2": "max_row_rel_err_vs_oracle", "c5": "max_row_rel_err_vs_oracle",
              "c3": "round_trip_max_err_rel_to_max_x", "c4": "pair0_coherence_max_abs_err_vs_oracle"}


def pmc_traffic(cfg, per_step):
    """HBM bytes per step of the roofline kernels from the newest committed PMC pass
    (profiles/rNN/pmc_traffic.json, written by scripts/pmc_traffic.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        with open(path) as fh:
            ent = json.load(fh).get(cfg)
        if not ent:
            continue
        total, seen = 0.0, 0
        for prefix, count in per_step.items():
            hits = [v for k, v in ent["kernels"].items() if k.startswith(prefix)]
            if len(hits) != 1:
                break
            total += hits[0]["hbm_bytes"] * count
            seen += 1
        if seen == len(per_step):
            return total, os.path.relpath(path, ROOT)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--cpu-per-worker", type=int, default=0, help="0 = per-config default")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wl_cls = CONFIGS[args.config]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before any GPU initialisation (spawned workers never touch the GPU)
        workers = max(1, min(args.cpu_workers, len(os.sched_getaffinity(0))))
        cpu = cpu_baseline(args.config, args.cpu_per_worker, workers)

    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    wl = wl_cls(rank, dev)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        wl.step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tmax = float(t.item())
    check = wl.check() if rank == 0 else None

    if rank == 0:
        total_units = wl.units * args.steps * world
        achieved = wl.bytes / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(args.config, wl.per_step)
        line = {
            "metric": METRIC,
            "value": total_units / tmax,
            "unit": wl.unit_name,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": tmax / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded AR(1) red noise (a=0.7) + 3 random sinusoids per series, "
                    "resident in HBM before timing",
            "config": wl.config(world),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": tsrc,
                         "kernel": wl.kernel, "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": wl.bytes, "bytes_model": wl.bytes_note},
            "cpu_baseline": cpu,
            "check": {CHECK_NAME[args.config]: check},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
