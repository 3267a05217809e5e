"""CPU oracle for the wavelet-transform hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything under ``oracle/``, and only
as the checker or the timed CPU baseline.  The product path under
``wavelet-transformer_amd/`` never imports it and has no CPU fallback.

Modules:
  pycwt_spec  -- fp64 restatement of pycwt 0.4.0b0 (CWT/XWT/WCT/AR1/significance);
                 parity UNPINNED (pycwt absent), pinned by known-answer tests.
  modwt_spec  -- restatement of src/modwt.py; pinned by golden vectors produced by
                 the reference's own functions.
  dwt_spec    -- restatement of pywt wavedec/waverec (symmetric); pinned by golden
                 vectors produced by PyWavelets 1.1.1.
  glue_spec   -- the reference wrapper glue (run_cwt, run_xwt, run_wct, ...).
"""
