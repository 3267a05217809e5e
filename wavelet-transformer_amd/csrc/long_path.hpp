// Long-row (N > 16384) CWT / XWT / WCT launchers (long.hip), shared with cwt.hip / wct.hip.
#pragma once

#include "cwt_common.hpp"

namespace wtmi {

constexpr int kLongMinLog = 15;
constexpr int kLongMaxLog = 20;  // N <= 2^20 (1,048,576 samples per row)

// Workspace of the long path for `batch` series (pair: two spectra / work planes).
long long cwt_long_workspace_bytes(long long batch, long long n0, int n_scales, bool pair);
long long wct_long_workspace_bytes(long long batch, long long n0, int n_scales);

// a: as the short path fills it (x, x2, ld, batch, n0, S, affine(s), scales, dt, f0,
// sigscale / sig_ld, outputs).  The workspace must hold cwt_long_workspace_bytes(...).
int cwt_long(const CwtArgs& a, bool pair, void* workspace, hipStream_t st);
// WCT coherence (+ power / phase / u / v through a.out_*): boxcar K rows (any K >= 1).
int wct_long(const CwtArgs& a, int K, void* workspace, float* coh, hipStream_t st);

// Phase B of wct.hip for every row (plan: plan[i] = 0 for i < S, plan[S] = S - 1).
int wct_phase_b_any(const cpx* TA, const cpx* TB, long long batch, int n0, int S, float* coh,
                    const int* plan, int K, hipStream_t st);

}  // namespace wtmi
