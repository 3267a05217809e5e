"""Put the engine's seven drop-in modules into an unchanged reference checkout.

The reference app imports ``from src import cwt, dwt, wct, xwt`` and
``src.utils.wavelet_helpers`` (src/wavelet_plots.py:15-26, src/utils/transform_helpers.py:8-13,
src/utils/plot_helpers.py:8-10, src/regression.py:16-19), and builds its per-series
results through ``src.utils.transform_helpers`` (src/wavelet_plots.py:25, src/regression.py:16).
Everything else under the reference's ``src`` (retrieve_data, helpers, file_helpers,
wavelet_plots, ...) must keep resolving to the reference's own files.  So exactly these
module names are replaced:

    src.cwt  src.xwt  src.wct  src.dwt  src.modwt  src.utils.wavelet_helpers
    src.utils.transform_helpers   (the batch API: one launch per group of series)

The repository's own ``src`` directory has no ``__init__.py`` (a namespace package): a
reference checkout's regular ``src`` package always wins over it, whatever the order on
``sys.path``, so adding this package directory to the path never hides the app's modules.

Two ways to activate it, neither edits the app's code:

1. Import hook (nothing written into the reference tree)::

       python -m wtmi.overlay run streamlit run app.py      # from the reference root

   installs a ``sys.meta_path`` finder that serves the seven names from this repository and
   then runs the given module (``streamlit``) in the same process.  In-process users call
   ``wtmi.overlay.install()`` before the first ``import src.cwt``.

2. Stub files (for deployments that start the app themselves)::

       python -m wtmi.overlay stubs /path/to/reference      # writes 7 stubs, keeps *.orig
       python -m wtmi.overlay restore /path/to/reference    # puts the originals back

   Each stub is a three-line module that executes this repository's module of the same
   name in its own namespace, so ``src.cwt`` *is* the engine-backed module.
"""

from __future__ import annotations

import argparse
import importlib.abc
import importlib.util
import os
import runpy
import sys

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # wavelet-transformer_amd
MODULES = {
    "src.cwt": "src/cwt.py",
    "src.xwt": "src/xwt.py",
    "src.wct": "src/wct.py",
    "src.dwt": "src/dwt.py",
    "src.modwt": "src/modwt.py",
    "src.utils.wavelet_helpers": "src/utils/wavelet_helpers.py",
    "src.utils.transform_helpers": "src/utils/transform_helpers.py",
}
STUB_MARK = "# wtmi overlay stub"


def module_file(name: str) -> str:
    return os.path.join(PKG_DIR, MODULES[name])


def _ensure_engine_importable():
    """``wtmi`` must import; the package dir goes at the END of sys.path so that it can
    never take precedence over the app's own top-level packages."""
    if PKG_DIR not in sys.path:
        sys.path.append(PKG_DIR)


class OverlayFinder(importlib.abc.MetaPathFinder):
    """Serves the replaced module names from this repository; declines all others."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname not in MODULES:
            return None
        return importlib.util.spec_from_file_location(fullname, module_file(fullname))


_FINDER = OverlayFinder()


def install() -> None:
    """Activate the import hook (idempotent).  Modules already imported under the
    replaced names are dropped so that the next import resolves through the hook."""
    _ensure_engine_importable()
    if _FINDER not in sys.meta_path:
        sys.meta_path.insert(0, _FINDER)
    for name in MODULES:
        mod = sys.modules.get(name)
        if mod is not None and getattr(mod, "__file__", None) != module_file(name):
            del sys.modules[name]


def uninstall() -> None:
    if _FINDER in sys.meta_path:
        sys.meta_path.remove(_FINDER)


def exec_into(name: str, namespace: dict) -> None:
    """Run this repository's module ``name`` inside ``namespace`` (used by the stubs)."""
    _ensure_engine_importable()
    path = module_file(name)
    namespace["__file__"] = path
    with open(path) as fh:
        code = compile(fh.read(), path, "exec")
    exec(code, namespace)


def _stub_text(name: str) -> str:
    return (f"{STUB_MARK} (python -m wtmi.overlay restore <reference> puts the original back)\n"
            f"import sys as _s; _s.path.append({PKG_DIR!r})\n"
            f"from wtmi.overlay import exec_into as _e; _e({name!r}, globals())\n")


def write_stubs(reference_root: str) -> list[str]:
    """Replace the reference files by stubs; each original is kept as ``<file>.orig``."""
    written = []
    for name in MODULES:
        rel = name.replace(".", "/") + ".py"
        dst = os.path.join(reference_root, rel)
        if not os.path.isfile(dst):
            raise FileNotFoundError(f"{dst}: not a reference checkout")
        with open(dst) as fh:
            is_stub = fh.read().startswith(STUB_MARK)
        if not is_stub:
            os.replace(dst, dst + ".orig")
        with open(dst, "w") as fh:
            fh.write(_stub_text(name))
        written.append(dst)
    return written


def restore_stubs(reference_root: str) -> list[str]:
    restored = []
    for name in MODULES:
        dst = os.path.join(reference_root, name.replace(".", "/") + ".py")
        if os.path.isfile(dst + ".orig"):
            os.replace(dst + ".orig", dst)
            restored.append(dst)
    return restored


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m wtmi.overlay")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run", help="install the import hook, then run a module (e.g. streamlit)")
    r.add_argument("module")
    r.add_argument("args", nargs=argparse.REMAINDER)
    s = sub.add_parser("stubs", help="write the stub modules into a reference checkout")
    s.add_argument("reference_root")
    u = sub.add_parser("restore", help="put the reference's original modules back")
    u.add_argument("reference_root")
    a = ap.parse_args(argv)
    if a.cmd == "stubs":
        for p in write_stubs(a.reference_root):
            print("stub", p)
        return 0
    if a.cmd == "restore":
        for p in restore_stubs(a.reference_root):
            print("restored", p)
        return 0
    if os.getcwd() not in sys.path:
        sys.path.insert(0, os.getcwd())  # the app's root, as `python -m` would give it
    install()
    args = a.args[1:] if a.args[:1] == ["--"] else a.args
    sys.argv = [a.module] + args
    runpy.run_module(a.module, run_name="__main__", alter_sys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
