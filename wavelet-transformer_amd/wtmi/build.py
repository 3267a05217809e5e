"""Build libwtmi.so (all HIP kernels + the C ABI) in-tree for gfx950.

    python wavelet-transformer_amd/wtmi/build.py [--force] [-j N]

Each csrc/*.hip is compiled to an object under wtmi/_build/ (skipped when up to
date), then linked into wtmi/libwtmi.so.  Cross-compiles without a GPU.
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libwtmi.so")
ARCH = "gfx950"  # the kernels are written for CDNA4 only (fft_lds.hpp #errors elsewhere)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
         "-Wno-unused-function", "-I", CSRC]


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if _stale(obj, [src] + _headers()):
        cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    if force:
        for f in os.listdir(BUILD):
            os.remove(os.path.join(BUILD, f))
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    if force or _stale(LIB, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    print(build(a.force, a.j))
    sys.exit(0)
