"""Caller-supplied operands of the device API are checked against the launch geometry
before anything reaches a kernel (CPU only: the checks run before the device check, so
CPU tensors exercise them; a well-formed CPU call then fails loudly -- no CPU fallback)."""

import numpy as np
import pytest
import torch

from wtmi import ops

B, N, S = 2, 64, 5
X = torch.zeros(B, N)
SC = np.linspace(0.2, 2.0, S)


@pytest.mark.parametrize("kw,msg", [
    (dict(out_w=torch.empty(B, S, N - 1, dtype=torch.complex64)), "out_w"),
    (dict(out_w=torch.empty(B, S, N, dtype=torch.complex128)), "out_w"),
    (dict(out_w=torch.empty(B, N, S, dtype=torch.complex64).transpose(1, 2)), "out_w"),
    (dict(affine=torch.zeros(B, 2, dtype=torch.float64)), "affine"),
    (dict(affine=torch.zeros(B + 1, 3, dtype=torch.float64)), "affine"),
    (dict(want_sig=True, sig_scale=np.ones(S - 1)), "sig_scale"),
    (dict(want_sig=True, sig_scale=np.ones((B + 1, S))), "sig_scale"),
    (dict(want_sig=True), "sig_scale"),
    (dict(want_w=False), "no output"),
])
def test_cwt_operand_checks(kw, msg):
    with pytest.raises(ValueError, match=msg):
        ops.cwt_morlet(X, SC, 0.1, **kw)


def test_cwt_scales_must_be_1d():
    with pytest.raises(ValueError, match="scales"):
        ops.cwt_morlet(X, np.ones((2, 2)), 0.1)
    with pytest.raises(ValueError, match="scales"):
        ops.cwt_morlet(X, [], 0.1)


def test_xwt_and_wct_operand_checks():
    with pytest.raises(ValueError, match="affine2"):
        ops.xwt_morlet(X, X, SC, 0.1, want_power=True, affine2=torch.zeros(B, 4))
    with pytest.raises(ValueError, match="sig_scale"):
        ops.xwt_morlet(X, X, SC, 0.1, want_sig=True, sig_scale=np.ones(S + 1))
    with pytest.raises(ValueError, match="same shape"):
        ops.xwt_morlet(X, torch.zeros(B, N + 1), SC, 0.1, want_power=True)
    with pytest.raises(ValueError, match="workspace"):
        ops.wct_morlet(X, X, SC, 0.1, boxcar=3, workspace=torch.empty(16, dtype=torch.uint8))
    with pytest.raises(ValueError, match="affine1"):
        ops.wct_morlet(X, X, SC, 0.1, boxcar=3, affine1=torch.zeros(B))


def test_well_formed_cpu_call_has_no_fallback():
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.cwt_morlet(X, SC, 0.1, want_sig=True, sig_scale=np.ones((B, S)))
