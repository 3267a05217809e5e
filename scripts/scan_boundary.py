"""Scan the reference for the drop-in boundary and write tests/golden/boundary_attrs.json.

Run in the BUILD container only (it reads /root/reference as text; nothing is imported
or executed from it):

    python scripts/scan_boundary.py

Two things are recorded, both as plain data (names, parameter kinds, default-value
expressions, file:line of each use):

* ``surface``: the public top-level names of the seven modules the engine replaces --
  src/{cwt,xwt,wct,dwt,modwt}.py, src/utils/wavelet_helpers.py and
  src/utils/transform_helpers.py (the batch API) -- with the signature of
  every function, every dataclass's generated ``__init__`` and every method, and the
  value expression of every module constant.
* ``uses``: every attribute of those modules that the reference's callers touch
  (``cwt.run_cwt``, ``from src.dwt import DataForDWT``, ...), found by walking the AST
  of every other .py file in the reference (app/, src/, tests/, scripts/).

``tests/test_boundary.py`` checks the repo's modules against this file.
"""

from __future__ import annotations

import ast
import json
import os
import sys

REF = os.environ.get("WTMI_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "tests", "golden", "boundary_attrs.json")

MODULES = {
    "cwt": "src/cwt.py",
    "xwt": "src/xwt.py",
    "wct": "src/wct.py",
    "dwt": "src/dwt.py",
    "modwt": "src/modwt.py",
    "wavelet_helpers": "src/utils/wavelet_helpers.py",
    "transform_helpers": "src/utils/transform_helpers.py",
}
DOTTED = {"src." + k: k for k in ("cwt", "xwt", "wct", "dwt", "modwt")}
DOTTED["src.utils.wavelet_helpers"] = "wavelet_helpers"
DOTTED["src.utils.transform_helpers"] = "transform_helpers"

# Names that are not part of the replaced API: script entry points, loggers and the
# module-level config the reference's own __main__ blocks use.
EXCLUDED = {
    "main": "script entry point (`python -m src.<module>`), reads FRED/BLS over the network",
    "logger": "module logger (the replacement modules have their own)",
    "PROJECT_ROOT": "src/wct.py sys.path bootstrap for its __main__ block",
    "SERIES_COMPARISONS": "src/modwt.py __main__ configuration (constants.ids keys)",
}

KIND = {"posonly": "POSITIONAL_ONLY", "arg": "POSITIONAL_OR_KEYWORD",
        "vararg": "VAR_POSITIONAL", "kwonly": "KEYWORD_ONLY", "kwarg": "VAR_KEYWORD"}


def _params(args: ast.arguments):
    out = []
    pos = list(args.posonlyargs) + list(args.args)
    defaults = [None] * (len(pos) - len(args.defaults)) + list(args.defaults)
    for i, (a, d) in enumerate(zip(pos, defaults)):
        kind = KIND["posonly"] if i < len(args.posonlyargs) else KIND["arg"]
        out.append({"name": a.arg, "kind": kind, "default": None if d is None else ast.unparse(d)})
    if args.vararg:
        out.append({"name": args.vararg.arg, "kind": KIND["vararg"], "default": None})
    for a, d in zip(args.kwonlyargs, args.kw_defaults):
        out.append({"name": a.arg, "kind": KIND["kwonly"],
                    "default": None if d is None else ast.unparse(d)})
    if args.kwarg:
        out.append({"name": args.kwarg.arg, "kind": KIND["kwarg"], "default": None})
    return out


def _is_dataclass(node: ast.ClassDef):
    for d in node.decorator_list:
        name = d.func if isinstance(d, ast.Call) else d
        if isinstance(name, ast.Name) and name.id == "dataclass":
            return True
        if isinstance(name, ast.Attribute) and name.attr == "dataclass":
            return True
    return False


def _dataclass_init(node: ast.ClassDef):
    """Parameters of the generated __init__.  A method defined later in the class body
    under a field's name replaces that field's class attribute before @dataclass runs
    (src/cwt.py:59-64: ``time_range = field(init=False)`` then ``def time_range``), so
    the field becomes an ordinary parameter whose default is the function."""
    params = []
    for i, st in enumerate(node.body):
        if not isinstance(st, ast.AnnAssign) or not isinstance(st.target, ast.Name):
            continue
        shadow = [f for f in node.body[i + 1:]
                  if isinstance(f, ast.FunctionDef) and f.name == st.target.id]
        if shadow:
            params.append({"name": st.target.id, "kind": KIND["arg"],
                           "default": f"<function {node.name}.{st.target.id}>"})
            continue
        default = None
        if st.value is not None:
            v = st.value
            if isinstance(v, ast.Call) and getattr(v.func, "id", None) == "field":
                kw = {k.arg: k.value for k in v.keywords}
                if "init" in kw and isinstance(kw["init"], ast.Constant) and kw["init"].value is False:
                    continue
                if "default_factory" in kw:
                    default = "<factory>"
                elif "default" in kw:
                    default = ast.unparse(kw["default"])
            else:
                default = ast.unparse(v)
        params.append({"name": st.target.id, "kind": KIND["arg"], "default": default})
    return params


def scan_module(path):
    tree = ast.parse(open(path).read(), path)
    surface = {}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef):
            if node.name in EXCLUDED or node.name.startswith("_"):
                continue
            surface[node.name] = {"kind": "function", "line": node.lineno,
                                  "params": _params(node.args)}
        elif isinstance(node, ast.ClassDef):
            ent = {"kind": "dataclass" if _is_dataclass(node) else "class", "line": node.lineno,
                   "methods": {}}
            if ent["kind"] == "dataclass":
                ent["params"] = _dataclass_init(node)
            for st in node.body:
                if isinstance(st, ast.FunctionDef) and not st.name.startswith("__"):
                    ent["methods"][st.name] = {"line": st.lineno, "params": _params(st.args)}
            surface[node.name] = ent
        elif isinstance(node, ast.Assign) and len(node.targets) == 1 \
                and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name in EXCLUDED:
                continue
            surface[name] = {"kind": "constant", "line": node.lineno,
                             "value": ast.unparse(node.value)}
    return surface


def scan_uses(root):
    uses = []
    skip = {os.path.join(root, p) for p in MODULES.values()}
    for dirpath, dirnames, files in os.walk(root):
        dirnames[:] = [d for d in dirnames if not d.startswith(".") and d != "__pycache__"]
        for f in files:
            if not f.endswith(".py"):
                continue
            path = os.path.join(dirpath, f)
            if path in skip:
                continue
            rel = os.path.relpath(path, root)
            try:
                tree = ast.parse(open(path).read(), path)
            except SyntaxError:
                continue
            alias = {}  # local name -> module key
            for node in ast.walk(tree):
                if isinstance(node, ast.ImportFrom) and node.module:
                    for a in node.names:
                        full = f"{node.module}.{a.name}"
                        if full in DOTTED:  # from src import cwt [as c]
                            alias[a.asname or a.name] = DOTTED[full]
                        elif node.module in DOTTED:  # from src.cwt import run_cwt
                            uses.append({"module": DOTTED[node.module], "attr": a.name,
                                         "site": f"{rel}:{node.lineno}", "how": "from-import"})
                elif isinstance(node, ast.Import):
                    for a in node.names:
                        if a.name in DOTTED and a.asname:
                            alias[a.asname] = DOTTED[a.name]
            for node in ast.walk(tree):
                if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) \
                        and node.value.id in alias:
                    uses.append({"module": alias[node.value.id], "attr": node.attr,
                                 "site": f"{rel}:{node.lineno}", "how": "attribute"})
    uses.sort(key=lambda u: (u["module"], u["attr"], u["site"]))
    return uses


def main():
    if not os.path.isdir(REF):
        sys.exit(f"{REF} not found: run this in the build container")
    data = {
        "generated_by": "scripts/scan_boundary.py (AST of the reference source text; nothing executed)",
        "reference_root": REF,
        "modules": {k: {"ref_file": v, "surface": scan_module(os.path.join(REF, v))}
                    for k, v in MODULES.items()},
        "excluded": EXCLUDED,
        "uses": scan_uses(REF),
    }
    for u in data["uses"]:
        u["in_reference_module"] = u["attr"] in data["modules"][u["module"]]["surface"] \
            or u["attr"] in EXCLUDED
    with open(OUT, "w") as fh:
        json.dump(data, fh, indent=1, sort_keys=False)
        fh.write("\n")
    n_missing = sum(not u["in_reference_module"] for u in data["uses"])
    print(f"wrote {OUT}: {sum(len(m['surface']) for m in data['modules'].values())} surface names, "
          f"{len(data['uses'])} uses ({n_missing} not defined by the reference module itself)")


if __name__ == "__main__":
    main()
