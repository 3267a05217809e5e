/*
 * wtmi.h -- C ABI of the MI355X wavelet-transform engine (libwtmi.so).
 *
 * Drop-in boundary for the numerics behind the reference's src.cwt / src.xwt /
 * src.wct / src.dwt / src.modwt modules.  The reference is pure Python; each entry
 * point below replaces a third-party call made from those modules (file:line into
 * the reference tree).  The Python host layer binds these with ctypes
 * (wavelet-transformer_amd/wtmi/_lib.py).
 *
 * Conventions (all entry points):
 *   - every array pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor memory)
 *     owned by the caller; row-major, series-major batches; ld = elements between
 *     consecutive series (>= n);
 *   - complex outputs are interleaved float32 pairs (re, im);
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream) and the
 *     call returns without synchronising; no allocation happens inside a call, so
 *     calls can be captured into a hipGraph;
 *   - return value: 0 success, -1 invalid argument, -2 unsupported size,
 *     > 0 a hipError_t from the kernel launch;
 *   - an empty batch (batch == 0, or no samples / scales where a size may be 0) is a
 *     no-op returning 0 once the sizes are valid, and its array pointers may then be NULL
 *     (an empty torch tensor has no storage; a rank's shard of a small batch can be empty);
 *   - calls are stateless and thread-safe.
 */
#ifndef WTMI_H
#define WTMI_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- CWT (K1+K2) --------------------------------------------------------------
 * Replaces pycwt.cwt(signal, dt, dj, s0, J, Morlet(f0)) as called from
 * src/cwt.py:110-112 (power |W|^2 at :114, significance ratio at :123-133).
 * x: [batch][ld] float32, n0 <= 2^20 samples used per series (above 16384 the long-row
 *    path runs: see wtmi_cwt_workspace_bytes).
 * affine: optional [batch][3] float64 (a0, a1, a2): x' = (x - a0 - a1*t) * a2 applied
 *         before the transform (standardize_series / pycwt normalisation), or NULL.
 * scales: [n_scales] float64 (s_j).  sig_scale: float64 1/signif_j, series b reading
 *         sig_scale[b * sig_ld + j] (sig_ld = 0: one [n_scales] row for every series,
 *         else >= n_scales: per-series AR(1) levels, one launch for a whole batch), or
 *         NULL when out_sig is NULL.
 * Outputs (any may be NULL, not all): out_w [batch][n_scales][n0] complex64,
 *         out_power / out_sig [batch][n_scales][n0] float32.                       */
int wtmi_cwt_morlet(const float* x, long long ld, long long batch, long long n0,
                    const double* affine, const double* scales, int n_scales, double dt,
                    double f0, const double* sig_scale, long long sig_ld, float* out_w,
                    float* out_power, float* out_sig, void* workspace, void* stream);

/* ---- CWT / XWT with any pycwt mother ------------------------------------------
 * The same transforms for the other mothers of the reference's MOTHER_DICT
 * (src/xwt.py:29-34, src/wct.py:36-41, constants/results_configs.py:53-58):
 * mother 0 = Morlet(f0 = param) (exactly wtmi_cwt_morlet / wtmi_xwt_morlet), 1 = Paul(m = param),
 * 2 = DOG(m = param) (pycwt MexicanHat = DOG(2)); orders 1..40.  pycwt's filter
 * sqrt(s w_1 N) conj(psi_hat(s w_k)) is evaluated in-register (full transforms: the band
 * pruning is Morlet's).  Rows up to 16384 samples for mothers 1 and 2 (-2 above).          */
int wtmi_cwt_mother(const float* x, long long ld, long long batch, long long n0,
                    const double* affine, const double* scales, int n_scales, double dt,
                    int mother, double param, const double* sig_scale, long long sig_ld,
                    float* out_w, float* out_power, float* out_sig, void* workspace, void* stream);
int wtmi_xwt_mother(const float* x1, const float* x2, long long ld, long long batch,
                    long long n0, const double* affine1, const double* affine2,
                    const double* scales, int n_scales, double dt, int mother, double param,
                    const double* sig_scale, long long sig_ld, float* out_w12, float* out_power,
                    float* out_sig, float* out_u, float* out_v, void* workspace, void* stream);

/* Device scratch a CWT (pair = 0) or XWT (pair = 1) call needs: 0 for n0 <= 16384 (one
 * workgroup holds a row; workspace may be NULL), else the four-step long-row path's
 * spectra and work rows (bounded: series and scales are processed in chunks of about
 * 1 GiB each).  Rows up to 2^20 samples; longer ones return kErrUnsupported.         */
long long wtmi_cwt_workspace_bytes(long long batch, long long n0, int n_scales, int pair);

/* ---- XWT / phase (K1+K2, pair mode) ------------------------------------------
 * Replaces the two pycwt.cwt calls and W1*conj(W2) inside pycwt.xwt
 * (src/xwt.py:93-101) and the phase angle(W12) of pycwt.wct used for the arrows
 * (src/xwt.py:122-137, src/wct.py:106-138).  Outputs: W12 complex64, |W12|^2,
 * |W12|^2 * sig_scale_j, and the arrow components u = cos(pi/2 - angle(W12)),
 * v = sin(pi/2 - angle(W12)) (calculate_phase_difference, src/xwt.py:142-154).   */
int wtmi_xwt_morlet(const float* x1, const float* x2, long long ld, long long batch,
                    long long n0, const double* affine1, const double* affine2,
                    const double* scales, int n_scales, double dt, double f0,
                    const double* sig_scale, long long sig_ld, float* out_w12, float* out_power,
                    float* out_sig, float* out_u, float* out_v, void* workspace, void* stream);

/* ---- WCT coherence + XWT power / phase (K1+K2+K7+K8) ---------------------------
 * Replaces pycwt.wct(..., sig=False) numerics (src/wct.py:106-118): two CWTs,
 * Morlet.smooth of |W1|^2/s, |W2|^2/s, W12/s (time Gaussian via FFT + scale boxcar of
 * `boxcar` rows), WCT = |S12|^2/(S1 S2), aWCT = angle(W12) and the phase arrows; the
 * same pass emits the cross-wavelet power |W1 W2*|^2 (pycwt.xwt, src/xwt.py:93).
 * workspace: device scratch of wtmi_wct_workspace_bytes(batch, n0, n_scales) bytes.
 * Outputs [batch][n_scales][n0] float32; all but out_coh may be NULL (u, v together). */
long long wtmi_wct_workspace_bytes(long long batch, long long n0, int n_scales);
int wtmi_wct_morlet(const float* x1, const float* x2, long long ld, long long batch, long long n0,
                    const double* affine1, const double* affine2, const double* scales,
                    int n_scales, double dt, double f0, int boxcar, void* workspace,
                    float* out_coh, float* out_power, float* out_phase, float* out_u,
                    float* out_v, void* stream);

/* Side-stream pool entries the full-row WCT (n0 = 2^k >= 1024) has created in this process:
 * a call takes ONE entry (two streams and five events, created together: the full-band rows'
 * chain and, when wct_pc_early selects it -- by default for batches of at most 256 pairs --
 * phase C's q windows) from a per-device pool and joins both before returning
 * (on error paths too), so the count is the most such calls that ever overlapped, not the
 * number of host threads that made one.                                             */
long long wtmi_wct_side_streams(void);

/* wtmi_wct_morlet with pycwt's own normalisation of both series, (y - mean) / std with the
 * moments in fp64 over each series (pycwt.wct / xwt normalize=True, src/wct.py:106-118), done
 * inside the transform's first kernel -- no separate moments / affine launches.  Rows of
 * 9 .. 16384 samples (-2 otherwise: normalise through wtmi_series_affine + affine1/2).    */
int wtmi_wct_morlet_norm(const float* x1, const float* x2, long long ld, long long batch,
                         long long n0, const double* scales, int n_scales, double dt, double f0,
                         int boxcar, void* workspace, float* out_coh, float* out_power,
                         float* out_phase, float* out_u, float* out_v, void* stream);

/* ---- WCT Monte-Carlo significance (K10 / K11) ---------------------------------
 * Replace the pieces of pycwt.wct_significance reached from src/wct.py:106-118 with
 * sig=True.
 * wtmi_rednoise: helpers.rednoise(n, g, 1) for `count` series into out[count][ld]:
 *   pycwt: yr = lfilter([1,0],[1,-g], randn(n + tau, 1))[tau:], tau = ceil(-2/ln|g|) (0 if
 *   g == 0), filtered along lfilter's default axis -1 -- of length 1 -- i.e. not at all:
 *   filtered = 0 (pycwt's literal behaviour) writes the white normals tau .. tau + n - 1;
 *   filtered = 1 applies the AR(1) recurrence y_i = g y_{i-1} + e_i over all n + tau normals
 *   (the MATLAB rednoise.m intent) and writes y[tau:].  |g| < 1 (-1 otherwise).
 *   Normals come from Philox4x32-10 keyed by `seed`; series c uses stream
 *   first_series + c, so batches can be drawn in pieces reproducibly; both modes draw the
 *   same normals.
 * wtmi_coherence_histogram: adds, for s < n_hist_scales, the counts of
 *   clamp(floor(coh[p][s][t] * nbins), 0, nbins-1) over all pairs p and
 *   t in [t_lo[s], t_hi[s]) (the points outside the cone of influence; t_lo/t_hi are
 *   device int arrays) into hist[n_hist_scales][nbins] (uint32, caller-zeroed).
 *   nbins <= 4096.
 * wtmi_coherence_quantile: the quantile step of wct_significance for the first n_scales
 *   rows of hist[.][nbins]: out[s] = np.interp(level, P, (bin + 1/2) / nbins) over the
 *   non-empty bins, P = (cumsum - 1/2) / total (0 for a row without counts); out is a device
 *   float64 [n_scales].                                                              */
int wtmi_rednoise(float* out, long long ld, long long count, long long n, double g, int filtered,
                  unsigned long long seed, unsigned long long first_series, void* stream);
int wtmi_coherence_histogram(const float* coh, long long batch, long long n0, int n_scales,
                             const int* t_lo, const int* t_hi, int n_hist_scales, int nbins,
                             unsigned int* hist, void* stream);
int wtmi_coherence_quantile(const unsigned int* hist, int n_scales, int nbins, double level, double* out,
                            void* stream);

/* ---- MODWT (K3 / K4) -----------------------------------------------------------
 * Replace src/modwt.py:126-144 (modwt: rows [W_1..W_J, V_J]) and :147-160 (imodwt).
 * dec_lo/dec_hi: HOST pointers to the n_taps analysis filters (pywt dec_lo/dec_hi);
 * the kernels use h~ = dec_hi/sqrt2, g~ = dec_lo/sqrt2 (n_taps <= 128).
 * w: [batch][level+1][n] float32.  keep_mask (imodwt): bit r set = row r used, others
 * treated as zero (modwtmra / smooth_signal, src/modwt.py:163-251); ~0ull = all.
 * workspace: NULL for n <= 16384 (a series lives in one workgroup's LDS); longer series
 * run one launch per level and need wtmi_modwt_workspace_bytes() of device scratch.  */
long long wtmi_modwt_workspace_bytes(long long batch, long long n, int level);
int wtmi_modwt(const float* x, long long ld, long long batch, long long n, const double* dec_lo,
               const double* dec_hi, int n_taps, int level, float* w, void* workspace,
               void* stream);
int wtmi_imodwt(const float* w, long long batch, long long n, const double* dec_lo,
                const double* dec_hi, int n_taps, int level, unsigned long long keep_mask,
                float* x, long long ld_out, void* workspace, void* stream);

/* ---- DWT (K5 / K6) -------------------------------------------------------------
 * Replace pywt.wavedec / pywt.waverec with mode "symmetric" (src/dwt.py:104,120;
 * src/utils/transform_helpers.py:96).  Coefficients of one series are stored
 * back-to-back in pywt list order [cA_J, cD_J, ..., cD_1]; wtmi_dwt_lengths() gives
 * the per-array lengths (host, lens[level+1]) and returns the total per series.
 * waverec: n_variants reconstructions per series, variant v keeps array k when bit k
 * of keep_masks[v] is set (ResultsFromDWT.smooth_signal, reconstruct_signal_component,
 * src/dwt.py:53-73,110-120); out: [batch][n_variants][out_len].
 * workspace: NULL for n <= 16384; longer series run one launch per level and need
 * wtmi_dwt_workspace_bytes(batch, n, n_taps, n_variants) (wavedec: n_variants = 1).  */
long long wtmi_dwt_lengths(long long n, int n_taps, int level, long long* lens);
long long wtmi_dwt_workspace_bytes(long long batch, long long n, int n_taps, int n_variants);
int wtmi_wavedec(const float* x, long long ld, long long batch, long long n, const double* dec_lo,
                 const double* dec_hi, int n_taps, int level, float* coeffs, void* workspace,
                 void* stream);
int wtmi_waverec(const float* coeffs, long long batch, long long n, const double* rec_lo,
                 const double* rec_hi, int n_taps, int level,
                 const unsigned long long* keep_masks, int n_variants, float* out,
                 long long out_len, void* workspace, void* stream);

/* ---- per-series moments / affine (K9) -----------------------------------------
 * Replace standardize_series (src/utils/wavelet_helpers.py:22-57) and the
 * covariances of pycwt.ar1 (src/cwt.py:106).  out: [batch][8] float64 =
 * mean, std (ddof 0), slope, intercept, c0, c1, n, 0.                              */
int wtmi_series_moments(const void* x, int x_is_f64, long long ld, long long batch, long long n,
                        double* out, void* stream);
int wtmi_affine(const void* x, int x_is_f64, long long ld_in, long long batch, long long n,
                const double* coef, void* y, int y_is_f64, long long ld_out, void* stream);
/* The affine coefficients [batch][3] (a0, a1, a2: x' = (x - a0 - a1 t) a2) in one pass over the
 * series, for the transforms' `affine` arguments: mode bits 1 detrend (polyfit deg 1), 2 remove
 * the mean, 4 divide by the std -- standardize_series(detrend, standardize, remove_mean) of
 * src/utils/wavelet_helpers.py:22-57 (1 and 2 together: -1, as its ValueError), and 6 = pycwt's
 * xwt/wct normalisation (y - mean) / std.  moments: [batch][8] as above, or NULL. */
int wtmi_series_affine(const void* x, int x_is_f64, long long ld, long long batch, long long n, int mode,
                       double* moments, double* affine, void* stream);

/* ---- launch options (no reference counterpart) ----------------------------------
 * Launch-policy knobs, read from WTMI_<NAME> environment variables once at first use
 * and settable here: cwt_prune (2 band rows + narrowed entry passes, 1 band rows, 0 full
 * transforms), cwt_target_wg, wct_prune (2 band rows + decimated spectra of full rows, 1 band
 * rows, 0 full transforms), wct_target_wg, wct_min_rows and wct_dec_rows (scale rows per WCT
 * workgroup and decimated rows per phase-A workgroup; 0 = chosen by batch size), modwt_syn
 * (n = 8192 / 16384 synthesis: 1 hybrid kernel with the low levels staged through LDS, 0
 * dilation chains only), wct_wide (0: windows touching a full-band row always take the
 * time-domain path; 1..3: from which union-band exponent on they take the spectral route),
 * wct_side_stream (1: the full-band rows' kernel on a pooled side stream beside the
 * decimated rows' chain), wct_pc_early (phase C's q windows on a third pooled stream right
 * after the decimated spectra: 1 always, 0 never, 2 for batches of at most 256 pairs),
 * wct_dec_merge (the decimation classes M = 4096 .. 512 in one launch: 1 always, 0 never, 2 for
 * batches of at most 256 pairs), modwt_ana
 * (n = 16384 analysis geometry: 0 1024 threads x 4 float4 groups, 1 512 x 8, 2 256 x 16).  The prune and kernel switches exist so that tests can
 * compare the paths; results agree to fp32 resolution either way.  The environment gives the process
 * defaults; wtmi_set_option changes the CALLING thread's value only (thread-local), so it
 * never races a launch issued by another thread, and wtmi_get_option reads it back.
 * wtmi_set_option: 0, or -1 for an unknown name / out-of-range value;
 * wtmi_get_option: the value, or -1 for an unknown name.                             */
int wtmi_set_option(const char* name, long long value);
long long wtmi_get_option(const char* name);

#ifdef __cplusplus
}
#endif

#endif /* WTMI_H */
