"""Drop-in replacements for the reference's ``src`` transform modules.

``src.cwt``, ``src.xwt``, ``src.wct``, ``src.dwt`` and ``src.modwt`` keep the
reference's dataclasses and function signatures; their numerics run
on the MI355X engine ``wtmi`` (HIP kernels behind include/wtmi.h).
"""
