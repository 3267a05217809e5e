"""SHA-256 pins of the reference source segments the fixture generators execute.

``scripts/make_plot_golden.py`` and ``tests/golden/make_golden.py`` run a few top-level
definitions of the (untrusted) reference in the build container to record golden data.
Each segment they execute must match the SHA-256 recorded in ``scripts/refpins.json`` --
pinned after reading those segments -- or nothing runs: a changed reference file cannot
slip new code into the fixtures.  ``python scripts/refpin.py --show`` prints the current
hashes of every pinned segment for review (it executes nothing).
"""

from __future__ import annotations

import ast
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PINS = os.path.join(HERE, "refpins.json")


def _name(node):
    if isinstance(node, (ast.FunctionDef, ast.ClassDef)):
        return node.name
    if isinstance(node, ast.Assign) and isinstance(node.targets[0], ast.Name):
        return node.targets[0].id
    return None


def segments(ref_root: str, rel: str, names):
    """(node, sha256 of its source text) for the named top-level defs / assignments."""
    src = open(os.path.join(ref_root, rel)).read()
    out = {}
    for node in ast.parse(src).body:
        nm = _name(node)
        if nm in names:
            seg = ast.get_source_segment(src, node)
            out[nm] = (node, hashlib.sha256(seg.encode()).hexdigest())
    missing = set(names) - set(out)
    if missing:
        raise RuntimeError(f"{rel}: segments not found: {sorted(missing)}")
    return out


def pinned_module(ref_root: str, rel: str, names) -> ast.Module:
    """The named segments as a module, after checking every one against its pin."""
    with open(PINS) as fh:
        pins = json.load(fh)
    segs = segments(ref_root, rel, names)
    bad = [nm for nm, (_, h) in segs.items() if pins.get(f"{rel}::{nm}") != h]
    if bad:
        raise RuntimeError(f"{rel}: segments {bad} differ from their SHA-256 pins in {PINS}; "
                           "review the reference change, then update the pins")
    return ast.Module(body=[segs[nm][0] for nm in names if nm in segs], type_ignores=[])


if __name__ == "__main__" and "--show" in sys.argv:
    ref = os.environ.get("WTMI_REFERENCE", "/root/reference")
    with open(PINS) as fh:
        pins = json.load(fh)
    for key, h in sorted(pins.items()):
        rel, nm = key.split("::")
        cur = segments(ref, rel, [nm])[nm][1]
        print(("ok  " if cur == h else "DIFF"), key, cur)
