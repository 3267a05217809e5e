"""bench.py's multi-rank launcher, weak and strong scaling, on CPU (gloo, stub workload).

`python bench.py --gpus N` must start N ranks itself when no torch.distributed.run
environment is present, give each rank its own block (weak: B rows per rank; strong: the
config's B rows split contiguously), and report n_gpus = N with value = all ranks' units /
max-over-ranks time.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "stub",
                        "--device", "cpu", "--steps", "3", "--warmup", "1", "--prewarm-s", "0",
                        *args], cwd=ROOT, env=e, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("n,per_rank", [(1, 10), (2, 5), (3, 4)])
def test_gpus_flag_launches_that_many_ranks_strong(n, per_rank):
    r, d = _run("--gpus", str(n), "--scaling", "strong")
    assert r.returncode == 0, r.stderr[-2000:]
    assert d["n_gpus"] == n and d["scaling"] == "strong"
    c = d["config"]
    assert c["global_batch"] == 10 and c["per_rank_batch"] == per_rank
    assert c["rank0_rows"] == [0, per_rank]
    # value counts every rank's units: 10 series x 256 samples per step, all ranks together
    assert d["value"] == pytest.approx(10 * 256 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=1e-6)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_weak_scaling_is_the_stub_default_one_block_per_rank(n):
    r, d = _run("--gpus", str(n))
    assert r.returncode == 0, r.stderr[-2000:]
    assert d["n_gpus"] == n and d["scaling"] == "weak"
    c = d["config"]
    assert c["global_batch"] == 10 * n and c["per_rank_batch"] == 10 and c["rank0_rows"] == [0, 10]
    assert d["value"] == pytest.approx(10 * n * 256 * 3 / (d["ms_per_step"] * 3 / 1e3), rel=1e-6)


def test_gpus_must_match_torchrun_world_size():
    r, d = _run("--gpus", "1", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and d is None and "WORLD_SIZE=2" in r.stderr


def test_shard_rows_do_not_depend_on_world_size():
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    whole = bench.synth_rows(5, 0, 200, 64)
    parts = np.concatenate([bench.synth_rows(5, lo, hi, 64) for lo, hi in ((0, 67), (67, 134), (134, 200))])
    np.testing.assert_array_equal(whole, parts)
    a1, a2 = bench.synth_rows(9, 10, 90, 32, pairs=True)
    b1, b2 = bench.synth_rows(9, 0, 100, 32, pairs=True)
    np.testing.assert_array_equal(a1, b1[10:90])
    np.testing.assert_array_equal(a2, b2[10:90])


def test_cpu_baseline_child_prints_one_record():
    """The CPU baseline runs in a child interpreter (bench.py --cpu-baseline-only), after the
    timed region: it must print one JSON record with the contract's keys and never import torch."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c3",
                        "--cpu-baseline-only", "--cpu-workers", "1", "--cpu-per-worker", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["cores"] == 1 and rec["kind"] == "port" and rec["unit"] == "coeffs/s"
    assert rec["value"] > 0 and "sample" in rec and "cpu_model" in rec


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("cfg,total", [("c4", 512), ("c5", 65536)])
def test_fixed_total_configs_default_to_strong_scaling(cfg, total, n):
    """BASELINE configs[3] (512 pairs "sharded by pair 1->8 GPUs") and configs[4] (65536
    series "sharded across 8xMI355X") are fixed totals: under the default scaling the ranks'
    blocks tile exactly [0, total) -- contiguous, disjoint, whatever N."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--gpus", str(n),
                        "--plan-only"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["scaling"] == "strong" and d["global_batch"] == total
    assert len(d["ranks"]) == n
    assert d["ranks"][0][0] == 0 and d["ranks"][-1][1] == total
    for (a, b), (c, _) in zip(d["ranks"], d["ranks"][1:]):
        assert b == c and a <= b


@pytest.mark.parametrize("cfg,per", [("c2", 1024), ("c3", 8192)])
def test_single_gpu_configs_default_to_weak_scaling(cfg, per):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--gpus", "4",
                        "--plan-only"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["scaling"] == "weak" and d["global_batch"] == 4 * per
    assert d["ranks"] == [[k * per, (k + 1) * per] for k in range(4)]


def test_per_rank_timing_fields():
    r, d = _run("--gpus", "2")
    assert r.returncode == 0, r.stderr[-2000:]
    rk = d["ranks"]
    assert 0 <= rk["own_steps_ms_per_step"]["min"] <= rk["own_steps_ms_per_step"]["max"]
    assert 0 <= rk["closing_barrier_ms"]["min"] <= rk["closing_barrier_ms"]["max"]
    assert rk["own_steps_ms_per_step"]["max"] <= d["ms_per_step"] * 1.0001
    assert d["graph"] is False


def test_force_dist_runs_a_one_rank_group_with_the_gather():
    """--force-dist at --gpus 1 initialises the process group (here gloo on CPU; on the GPU box
    RCCL, tests/test_gpu_dist.py) and runs the barrier, the max / sum over ranks and the
    host-side gather of sharding.gather_to_rank0."""
    r, d = _run("--gpus", "1", "--force-dist", "--dist-backend", "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    assert d["config"]["dist_backend"] == "gloo"
    assert d["config"]["dist_gather"] == [[0.0, 10 * 256.0]]
    r, d = _run("--gpus", "2", "--dist-backend", "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    assert d["config"]["dist_gather"] == [[0.0, 10 * 256.0], [10.0, 10 * 256.0]]


@pytest.mark.parametrize("cfg,bound", [("c2", "hbm"), ("c3", "hbm"), ("c4", "valu")])
def test_roofline_bound_follows_the_committed_profile(cfg, bound):
    """roofline.bound is the larger of the step's HBM fraction and its VALU fraction (the
    newest committed kernel_roofline.json's SQ_INSTS_VALU of the step's kernels over the
    chip's VALU issue rate): C4's kernels are VALU-bound, C2 / C3 sit on HBM.  Checked at the
    step times and HBM fractions of the committed bench lines."""
    import glob
    sys.path.insert(0, ROOT)
    import bench
    prof = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"bench_{cfg}.json")))[-1]
    with open(prof) as fh:
        line = json.load(fh)
    hbm = line["roofline"]["achieved"] / line["roofline"]["peak"]
    sb = bench.step_bound(cfg, bench.CONFIGS[cfg].PER_STEP, line["roofline"]["kernel_ms"], hbm)
    assert sb["source"] and 0 < sb["valu"] < 1 and sb["hbm"] == hbm
    # the VALU fraction is a model (every VALU instruction at 4 cycles per wave64: transcendental
    # ops issue slower, packed FP32 does two lanes' work), so the ordering is checked with a
    # margin rather than the label alone: the binding resource is ahead by at least 1.25x
    hi, lo = (sb["valu"], hbm) if bound == "valu" else (hbm, sb["valu"])
    assert hi > 1.25 * lo, sb
    assert sb["bound"] == bound, sb
    assert "note" in sb
    if "step_fractions" in line["roofline"]:  # lines written since the field exists
        assert line["roofline"]["bound"] == bound
