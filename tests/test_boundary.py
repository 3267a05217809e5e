"""The drop-in boundary, checked against the reference's own surface (CPU only).

``tests/golden/boundary_attrs.json`` is written by ``scripts/scan_boundary.py`` from the
AST of the reference (build container): the public names and signatures of
src/{cwt,xwt,wct,dwt,modwt}.py and src/utils/wavelet_helpers.py, and every attribute of
those modules the reference's callers use (app/, src/, tests/), with file:line.  Here the
repo's modules must expose every such name with an identical parameter list (names,
kinds, defaults), constants with equal values, and the overlay must replace exactly those
seven modules inside an otherwise untouched reference-shaped ``src`` tree.
"""

import ast
import dataclasses
import inspect
import json
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import GOLDEN, PKG

with open(os.path.join(GOLDEN, "boundary_attrs.json")) as _fh:
    BOUNDARY = json.load(_fh)

MODNAMES = {"cwt": "src.cwt", "xwt": "src.xwt", "wct": "src.wct", "dwt": "src.dwt",
            "modwt": "src.modwt", "wavelet_helpers": "src.utils.wavelet_helpers",
            "transform_helpers": "src.utils.transform_helpers"}
# Constants whose reference value is a third-party object (pycwt / pywt instances): the
# name must exist; what it holds is checked by test_mother_wavelet_constants.
OBJECT_CONSTANTS = {"MOTHER", "MOTHER_DICT"}

_UNEVALUABLE = object()


def _eval(src, ns):
    """Evaluate a literal-ish expression (constants, containers, arithmetic, names of
    earlier constants); anything else is _UNEVALUABLE."""
    def ev(node):
        if isinstance(node, ast.Constant):
            return node.value
        if isinstance(node, (ast.List, ast.Tuple)):
            vals = [ev(e) for e in node.elts]
            return list(vals) if isinstance(node, ast.List) else tuple(vals)
        if isinstance(node, ast.Dict):
            return {ev(k): ev(v) for k, v in zip(node.keys, node.values)}
        if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
            return -ev(node.operand)
        if isinstance(node, ast.BinOp):
            a, b = ev(node.left), ev(node.right)
            ops = {ast.Add: lambda: a + b, ast.Sub: lambda: a - b, ast.Mult: lambda: a * b,
                   ast.Div: lambda: a / b, ast.Pow: lambda: a ** b}
            if type(node.op) in ops:
                return ops[type(node.op)]()
        if isinstance(node, ast.Name) and node.id in ns:
            return ns[node.id]
        raise ValueError(ast.dump(node))
    try:
        return ev(ast.parse(src, mode="eval").body)
    except (ValueError, SyntaxError, TypeError):
        return _UNEVALUABLE


@pytest.fixture(scope="module")
def modules():
    import importlib
    return {k: importlib.import_module(v) for k, v in MODNAMES.items()}


def _check_params(ours, ref, what):
    got = [(p.name, p.kind.name) for p in ours.parameters.values()]
    want = [(p["name"], p["kind"]) for p in ref]
    assert got == want, f"{what}: parameters {got} != reference {want}"
    for p, r in zip(ours.parameters.values(), ref):
        if r["default"] is None:
            assert p.default is inspect.Parameter.empty, f"{what}.{p.name} has a default"
        elif r["default"].startswith("<function "):  # a method shadowing a field (cwt.py:59-64)
            assert inspect.isfunction(p.default) and \
                f"<function {p.default.__qualname__}>" == r["default"], (what, p.default)
        elif r["default"] == "<factory>":
            assert repr(p.default) == "<factory>", f"{what}.{p.name}: default_factory expected"
        else:
            want_v = _eval(r["default"], {})
            assert want_v is not _UNEVALUABLE, r
            assert p.default == want_v and type(p.default) is type(want_v), \
                f"{what}.{p.name}: default {p.default!r} != reference {r['default']}"


def _surface_items():
    for mod, ent in BOUNDARY["modules"].items():
        for name, info in ent["surface"].items():
            yield pytest.param(mod, name, info, id=f"{mod}.{name}")


@pytest.mark.parametrize("mod,name,info", list(_surface_items()))
def test_surface_name_and_signature(modules, mod, name, info):
    m = modules[mod]
    where = f"{MODNAMES[mod]}.{name} (reference {BOUNDARY['modules'][mod]['ref_file']}:{info['line']})"
    assert hasattr(m, name), f"missing {where}"
    obj = getattr(m, name)
    if info["kind"] == "function":
        _check_params(inspect.signature(obj), info["params"], where)
    elif info["kind"] in ("dataclass", "class"):
        assert inspect.isclass(obj), where
        if info["kind"] == "dataclass":
            assert dataclasses.is_dataclass(obj), where
            _check_params(inspect.signature(obj), info["params"], where)
        for meth, minfo in info["methods"].items():
            assert hasattr(obj, meth), f"{where}: method {meth} missing"
            _check_params(inspect.signature(getattr(obj, meth)), minfo["params"], f"{where}.{meth}")


def test_constant_values(modules):
    for mod, ent in BOUNDARY["modules"].items():
        ns = {}
        for name, info in ent["surface"].items():
            if info["kind"] != "constant":
                continue
            want = _eval(info["value"], ns)
            got = getattr(modules[mod], name)
            if want is _UNEVALUABLE:
                assert name in OBJECT_CONSTANTS, f"{mod}.{name} = {info['value']} not checked"
                continue
            ns[name] = want
            assert got == want, f"{mod}.{name}: {got!r} != reference {info['value']}"


def test_mother_wavelet_constants(modules):
    assert modules["cwt"].MOTHER.f0 == 6
    for mod in ("xwt", "wct"):
        d = modules[mod].MOTHER_DICT
        assert list(d) == ["morlet", "paul", "DOG", "mexicanhat"]
        assert d["morlet"].f0 == 6 and d["paul"].m == 4 and d["DOG"].m == 2
    for mod in ("dwt", "modwt"):
        w = modules[mod].MOTHER
        assert w.name == "db4" and len(w.dec_lo) == 8


def test_every_caller_attribute_exists(modules):
    """Each attribute the reference's callers touch on these modules (file:line in the
    fixture).  Names the reference module itself lacks (its broken tests call
    ``dwt.smooth_signal``) are reported, not required."""
    missing = [u for u in BOUNDARY["uses"]
               if u["in_reference_module"] and not hasattr(modules[u["module"]], u["attr"])]
    assert not missing, missing
    absent_in_ref = {(u["module"], u["attr"]) for u in BOUNDARY["uses"] if not u["in_reference_module"]}
    assert absent_in_ref <= {("dwt", "smooth_signal")}, absent_in_ref


def test_mothers_resolve_and_coherence_needs_morlet():
    """Every MOTHER_DICT value is a transformable mother (CWT / XWT kernels, mother ids of
    include/wtmi.h); the coherence needs Morlet.smooth, which pycwt defines for Morlet
    only -- pycwt.wct raises AttributeError there, and so does as_morlet (also a ValueError)."""
    from wtmi.wavelets import DOG, MexicanHat, Morlet, Paul, as_morlet, as_mother, kernel_mother
    assert kernel_mother(Morlet(6)) == (0, 6.0)
    assert kernel_mother(Paul()) == (1, 4.0)
    assert kernel_mother(DOG()) == (2, 2.0) == kernel_mother(MexicanHat())
    assert kernel_mother("mexicanhat") == (2, 2.0)
    for name in ("paul", "DOG", "mexicanhat"):
        assert as_mother(name.lower()) is not None
    for w in (Paul(), DOG(), MexicanHat()):
        with pytest.raises(AttributeError, match="smooth"):
            as_morlet(w)
        with pytest.raises(ValueError):
            as_morlet(w)
    with pytest.raises(ValueError):
        as_mother("haar")


def test_run_cwt_unknown_kwarg_raises_typeerror(modules):
    """src/cwt.py:102 forwards **kwargs to standardize_series; an unknown keyword raises
    TypeError before any transform (the engine checks it before touching the GPU)."""
    from wtmi import transforms
    with pytest.raises(TypeError):
        transforms.standardize_coefs(None, detrendd=True)


def test_create_xwt_results_dict_fails_only_at_a_pair(modules):
    """The reference loops over xwt_list calling run_xwt(data, **kwargs)
    (src/utils/transform_helpers.py:126-135): no pairs -> {} whatever the keywords; the first
    pair is looked up (KeyError) before run_xwt's TypeError / NameError."""
    from src.utils import transform_helpers as th
    assert th.create_xwt_results_dict({}, [], normalize=False) == {}
    assert th.create_xwt_results_dict({}, [], bogus=1) == {}
    with pytest.raises(KeyError):
        th.create_xwt_results_dict({}, [("a", "b")], normalize=False)
    with pytest.raises(NameError):
        th.create_xwt_results_dict({("a", "b"): None}, [("a", "b")], normalize=False)
    with pytest.raises(TypeError):
        th.create_xwt_results_dict({("a", "b"): None}, [("a", "b")], bogus=1)


# ------------------------------------------------------------------------ overlay
FAKE_REF = {
    "src/__init__.py": "",
    # the reference's own transform modules import pycwt, which the app env has and this
    # one does not: if the overlay let one of them through, the import would fail loudly
    "src/cwt.py": "raise ImportError('reference src.cwt imported')\n",
    "src/xwt.py": "raise ImportError('reference src.xwt imported')\n",
    "src/wct.py": "raise ImportError('reference src.wct imported')\n",
    "src/dwt.py": "raise ImportError('reference src.dwt imported')\n",
    "src/modwt.py": "raise ImportError('reference src.modwt imported')\n",
    "src/retrieve_data.py": "WHO = 'reference'\n",
    # src/utils has no __init__.py in the reference (a namespace package)
    "src/utils/wavelet_helpers.py": "raise ImportError('reference wavelet_helpers imported')\n",
    "src/utils/transform_helpers.py": "raise ImportError('reference transform_helpers imported')\n",
    "src/utils/helpers.py": "WHO = 'reference'\n",
    "src/regression.py": textwrap.dedent("""\
        from src.utils.transform_helpers import create_dwt_dict, create_dwt_results_dict
        from src import dwt, retrieve_data
        from src.utils.wavelet_helpers import align_series
        """),
    "src/wavelet_plots.py": textwrap.dedent("""\
        from src import cwt, dwt, wct, xwt
        from src.utils.helpers import WHO
        from src.utils.transform_helpers import DataForCWT, create_cwt_results_dict
        from src.utils.wavelet_helpers import standardize_series
        """),
}

PROBE = textwrap.dedent("""\
    import json, sys
    {activate}
    import src.wavelet_plots as wp
    from src import retrieve_data, modwt
    from src.utils import helpers, wavelet_helpers
    import src.utils.transform_helpers as th
    import src.regression
    out = {{m: sys.modules[m].__file__ for m in
           ["src", "src.cwt", "src.xwt", "src.wct", "src.dwt", "src.modwt",
            "src.utils.wavelet_helpers", "src.utils.helpers", "src.retrieve_data",
            "src.wavelet_plots", "src.utils.transform_helpers", "src.regression"]}}
    out["plot_cwt"] = hasattr(wp.cwt, "plot_cwt")
    out["utils_is_namespace"] = getattr(sys.modules["src.utils"], "__file__", None) is None
    print(json.dumps(out))
    """)


def _fake_reference(root):
    for rel, text in FAKE_REF.items():
        path = os.path.join(root, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as fh:
            fh.write(text)


def _probe(ref, activate, extra_path=()):
    env = dict(os.environ)
    # the repo package dir FIRST on the path: its namespace `src` must still lose to the
    # reference's regular package
    env["PYTHONPATH"] = os.pathsep.join([PKG, *extra_path])
    r = subprocess.run([sys.executable, "-c", PROBE.format(activate=activate)], cwd=ref, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _assert_overlaid(out, ref):
    ours = os.path.realpath(os.path.join(PKG, "src"))
    for m in ("src.cwt", "src.xwt", "src.wct", "src.dwt", "src.modwt", "src.utils.wavelet_helpers",
              "src.utils.transform_helpers"):
        assert os.path.realpath(out[m]).startswith(ours + os.sep), (m, out[m])
    for m in ("src", "src.utils.helpers", "src.retrieve_data", "src.wavelet_plots", "src.regression"):
        assert os.path.realpath(out[m]).startswith(os.path.realpath(ref) + os.sep), (m, out[m])
    assert out["plot_cwt"] and out["utils_is_namespace"]


def test_repo_src_is_a_namespace_package():
    """No __init__.py: a reference checkout's regular `src` package always wins."""
    assert not os.path.exists(os.path.join(PKG, "src", "__init__.py"))
    assert not os.path.exists(os.path.join(PKG, "src", "utils", "__init__.py"))


def test_overlay_import_hook(tmp_path):
    ref = str(tmp_path / "reference")
    _fake_reference(ref)
    out = _probe(ref, "sys.path.insert(0, '.'); import wtmi.overlay as o; o.install()")
    _assert_overlaid(out, ref)


def test_overlay_without_activation_keeps_reference(tmp_path):
    """Only putting the repo on the path changes nothing: the reference's modules load
    (here they raise the marker ImportError)."""
    ref = str(tmp_path / "reference")
    _fake_reference(ref)
    env = dict(os.environ, PYTHONPATH=PKG)
    r = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, '.'); import src.cwt"],
                       cwd=ref, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "reference src.cwt imported" in r.stderr


def test_overlay_stub_files_and_restore(tmp_path):
    from wtmi import overlay
    ref = str(tmp_path / "reference")
    _fake_reference(ref)
    written = overlay.write_stubs(ref)
    assert len(written) == 7
    overlay.write_stubs(ref)  # idempotent: the originals stay in *.orig
    out = _probe(ref, "sys.path.insert(0, '.')")
    # with stubs the modules live at the reference's paths but run the engine's code
    for m in ("src.cwt", "src.utils.wavelet_helpers"):
        assert os.path.realpath(out[m]).startswith(os.path.realpath(PKG)), out[m]
    assert out["plot_cwt"] and out["utils_is_namespace"]
    overlay.restore_stubs(ref)
    with open(os.path.join(ref, "src", "cwt.py")) as fh:
        assert "reference src.cwt imported" in fh.read()
    assert not os.path.exists(os.path.join(ref, "src", "cwt.py.orig"))


def test_overlay_run_cli(tmp_path):
    """`python -m wtmi.overlay run <module> ...` runs the module with the hook active."""
    ref = str(tmp_path / "reference")
    _fake_reference(ref)
    with open(os.path.join(ref, "appmain.py"), "w") as fh:
        fh.write("import sys, src.wavelet_plots as wp\nprint('ARGS', sys.argv[1:], wp.cwt.__file__)\n")
    env = dict(os.environ, PYTHONPATH=PKG)
    r = subprocess.run([sys.executable, "-m", "wtmi.overlay", "run", "appmain", "x", "--flag"],
                       cwd=ref, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("ARGS")][0]
    assert "['x', '--flag']" in line and os.path.join(PKG, "src", "cwt.py") in line


def test_rows_gives_the_abi_a_valid_row_stride():
    """The C ABI rejects ld < n.  A one-row view may carry any batch stride in torch (NumPy's
    x[None, :] arrives with stride 0), an expanded batch has stride 0: ops._rows re-strides or
    copies both, so wtmi_modwt & co. never see an invalid ld (found by the random-shape sweep)."""
    import numpy as np
    import torch
    from wtmi import ops
    t = torch.tensor(np.arange(8, dtype=np.float32)[None, :])
    assert t.stride(0) == 0
    r = ops._rows(t)
    assert r.stride() == (8, 1) and torch.equal(r, t)
    r = ops._rows(torch.tensor(np.arange(8.0)[None, :]), torch.float32)
    assert r.stride() == (8, 1) and r.dtype == torch.float32
    r = ops._rows(torch.arange(5.0).expand(3, 5))
    assert r.stride() == (5, 1)
    r = ops._rows(torch.arange(10.0)[::2])
    assert r.stride() == (5, 1) and r.tolist() == [[0.0, 2.0, 4.0, 6.0, 8.0]]
    r1, r2 = ops._pair_rows(torch.zeros(4, 16)[:, :8], torch.zeros(4, 8))
    assert r1.stride(0) == r2.stride(0)
