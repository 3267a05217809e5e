"""Register budgets of the hot kernels, read from the built libwtmi.so's gfx950 code-object
metadata (scripts/kernel_meta.py; no GPU).  A spill or a budget overrun is a performance
regression the parity tests cannot see: r04's first build spilled 140 bytes per lane in
phase A (C4 3.15 -> 3.47 ms) and 108 in the C5 CWT kernel before it was caught by hand."""

import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

# kernel -> VGPR budget (the occupancy its launch geometry was tuned for); spills must be 0
BUDGET = {
    "void wtmi::cwt_morlet_kernel<12, 1, 0, 0>": 168,   # C2: 3 waves / SIMD
    "void wtmi::cwt_morlet_kernel<13, 1, 0, 0>": 128,   # C5: two 512-thread workgroups / CU
    "void wtmi::wct_spectra_plan<13>": 128,
    "void wtmi::wct_phase_a<13, true, 0>": 128,          # C4 full-band rows
    "void wtmi::wct_phase_a<13, true, 2>": 128,          # C4 decimated rows
    "void wtmi::wct_phase_c<13, true, false>": 128,      # C4 q windows
    "void wtmi::wct_phase_c<13, true, true>": 128,       # C4 wide windows
    "void wtmi::wct_phase_b<10, 1, 10>": 128,            # r05 default: K rows in flight
    "void wtmi::wct_wide_boxcar<10, 10>": 128,
    "void wtmi::wct_phase_b<10, 1, 0>": 128,
    "void wtmi::wct_wide_boxcar<10, 0>": 128,
    # C3 analysis: one 1024-thread workgroup per series, two per CU (64 KiB of LDS each) = 8
    # waves per SIMD, so at most 64 VGPRs (r04: an extra code path at 68 would halve occupancy)
    "void wtmi::modwt_vec_kernel<8, 4, 1024, 16>": 64,
    "void wtmi::imodwt_hyb_kernel<8, 8, 512, 2, 1024>": 128,  # C3 synthesis: two workgroups / CU
    "void wtmi::imodwt_hyb_kernel<8, 8, 512, 2, 4>": 128,
}
BUDGET.update({f"void wtmi::wct_dec_kernel<13, {m}>": 128 for m in range(8, 13)})
BUDGET["void wtmi::wct_dec_merged<13>"] = 128  # C4 decimation classes M = 4096 .. 512, one launch


@pytest.fixture(scope="module")
def table():
    from kernel_meta import LIB, LLVM, kernel_table
    if not os.path.exists(os.path.join(LLVM, "llvm-readelf")) or not shutil.which("c++filt"):
        pytest.skip("llvm-readelf / c++filt not available")
    if not os.path.exists(LIB):
        pytest.skip("libwtmi.so not built")
    return kernel_table(LIB)


@pytest.mark.parametrize("kernel", sorted(BUDGET))
def test_hot_kernel_registers(table, kernel):
    assert kernel in table, f"{kernel} not in libwtmi.so"
    r = table[kernel]
    assert r.get("vgpr_spill", 0) == 0 and r.get("scratch", 0) == 0, (kernel, r)
    assert r["vgpr"] <= BUDGET[kernel], (kernel, r)
