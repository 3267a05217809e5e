// Wavelet coherence (K7, K8, K12-K14 of DESIGN.md).
//
// Replaces the numerics of pycwt.wct(..., sig=False) as called from src/wct.py:106-118
// (SURVEY Appendix A.4):
//   W1, W2 = cwt(normalised y1, y2);  S1 = smooth(|W1|^2/s), S2 = smooth(|W2|^2/s),
//   S12 = smooth(W12/s) with W12 = W1 conj(W2);  WCT = |S12|^2 / (S1 S2);
//   aWCT = angle(W12)  -> arrows u = sin(aWCT), v = cos(aWCT)  (src/wct.py:143-158)
// where Morlet.smooth = time Gaussian F = exp(-(s/dt)^2 k^2 / 2) applied by FFT on the
// row zero-padded to N, then a [0.5, 1, .., 1, 0.5]/(K-1) boxcar over K scale rows
// (scipy convolve2d 'same': rows i - K/2 .. i + (K-1)/2, zero outside).
//
// Launch order: wct_spectra (both series' forward FFTs), wct_plan_kernel (per-row regimes,
// which rows take which route), wct_phase_a (rows not decimated), wct_dec_kernel (decimated
// spectra, one launch per M) + wct_phase_a<DEC> (decimated rows), wct_phase_c (coherence of
// band windows from band spectra), wct_phase_b (coherence of the other windows).
// Phase A (one workgroup = one pair x a chunk of scales): per scale row two inverse
// FFTs give W1, W2; |W1|^2 + i|W2|^2 and W12 are forward-transformed, multiplied by
// F/(N s) (F is real and even, so the two real fields share one complex FFT) and
// inverse-transformed: up to 6 in-LDS FFTs per row; a time-path row's smoothed fields
// T = (T1, T2, Re T12, Im T12) go to the workspace.  Decimated rows (full rows whose W1,
// W2 live in bins [0, M/2), M < N) get their forward transforms on every (N/M)-th sample
// (wct_dec_kernel) and band inverses of M bins here.
// Phase B (one thread = one time column of one pair): streams the time-path rows of T
// once, keeps the last K rows in registers and writes WCT.
#include <atomic>
#include <mutex>
#include <vector>

#include "cwt_common.hpp"
#include "long_path.hpp"

namespace wtmi {

// Cache policy of the WCT's streamed accesses, a bit mask (WTMI_WCT_NT: build knob for A/B runs):
//   1 output rows (power, phase, arrows, phase C coherence), 2 time-path rows T, 4 WB rows,
//   8 phase B's coherence stores, 16 band_load reads (DY, TA, TB), 32 phase B's reads of T,
//   64 the decimation kernels' stores (DY, SB, T, WB), 128 the wide boxcar's reads and writes of
//   WB, 256 phase C's reads of SB and WB.
// Default 191 = every class but 64 and 256, measured per class (profiles/r05/nt_policy_ab.txt):
// C4 3.09 -> 2.98 ms at 512 pairs, 0.452 -> 0.387 ms at 64 (the re-read pair spectra and plan stay
// cached); 64 and 256 cost the 64-pair shard 7-9 % (those rows are re-read while still cached).
// WTMI_WCT_AUX: the policy the buffer accesses of the set classes use (2 = nt; sc1 was slower);
// the pointer accesses (st_c / ld_c, phase B) are nt whenever their class is set.
#ifndef WTMI_WCT_NT
#define WTMI_WCT_NT 191
#endif
#ifndef WTMI_WCT_AUX
#define WTMI_WCT_AUX 2
#endif
constexpr int kWctNt = WTMI_WCT_NT;
template <int BIT> constexpr int wct_aux() { return (kWctNt & BIT) ? WTMI_WCT_AUX : 0; }
template <int BIT> __device__ __forceinline__ void st_c(cpx* p, cpx v) {
  if constexpr (wct_aux<BIT>() != 0)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
template <int BIT> __device__ __forceinline__ cpx ld_c(const cpx* p) {
  if constexpr (wct_aux<BIT>() != 0)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <int LOGN>
struct WctGeom {
  using P = FftPlan<LOGN>;
  static constexpr int ROWS = P::NT >= 256 ? 1 : 256 / P::NT;
  static constexpr int BLOCK = P::NT * ROWS;
  // as CwtGeom: LDS twiddle table from LOGN 13 on, so that phase A fits 128 VGPRs and
  // two 512-thread workgroups share a CU
  static constexpr bool TWL = LOGN >= 13;
  static constexpr int MINW = BLOCK >= 512 ? 4 : 2;
  static constexpr int MAXCHUNK = 128;
  static constexpr int TWL_F4 = TWL ? P::TWL_FLOAT4 : 0;
};

// bins this thread owns: kk = t + (m < 8 ? m : m - 16) * NT
template <int LOGN>
__device__ __forceinline__ void smooth_filter(cpx (&v)[16], float beta, float scale, int t) {
  using P = FftPlan<LOGN>;
  // kk^2 is loop-invariant in the caller's scale loop: without the barrier the
  // compiler hoists all 16 and spills them
  asm volatile("" : "+v"(t));
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float kk = static_cast<float>(t + (m < 8 ? m : m - 16) * P::NT);
    const float f = scale * __builtin_amdgcn_exp2f(beta * kk * kk);
    v[m] = cscale(v[m], f);
  }
}

// Forward spectra of both series of every pair: spec[b][which][k], natural order (with
// a.norm, of the normalised series).  Workgroup blk of wct_spectra_plan.
template <int LOGN>
__device__ __forceinline__ void spectra_body(const CwtArgs& a, cpx* __restrict__ spec, long long blk) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  __shared__ cpx lds[G::ROWS * P::PADN];
  const int tid = threadIdx.x;
  const int g = tid / P::NT;
  const int t = fft_thread<LOGN>(tid - g * P::NT);
  // row group g handles series (pair, which) = blk * ROWS + g
  const long long item = blk * G::ROWS + g;
  const bool valid = item < 2 * a.batch;
  const long long b = valid ? item >> 1 : 0;
  const int which = static_cast<int>(item & 1);
  cpx tw[P::NTW_ALLOC];
  fft_twiddles<LOGN>(tw, t);
  int par = 0;
  __shared__ float red[G::BLOCK / kWave];
  __shared__ double redd[G::BLOCK / kWave];
  cpx X[16];
  if (which == 0)
    load_series<LOGN>(X, a.x, a.norm ? nullptr : a.affine, b, a.ld, a.n0, t);
  else
    load_series<LOGN>(X, a.x2, a.norm ? nullptr : a.affine2, b, a.ld, a.n0, t);
  if (a.norm) normalize_row<LOGN>(X, a.n0, t, redd);
  const float mu = demean_row<LOGN>(X, a.n0, t, red);
  fft_row<LOGN, -1, 1>(X, lds + g * P::PADN, 0, tw, t, par);
  add_mean_spectrum<LOGN>(X, mu, a.n0, t);
  if (!valid) return;
  cpx* o = spec + (2 * b + which) * static_cast<long long>(P::N);
#pragma unroll
  for (int m = 0; m < 16; ++m) o[t + m * P::NT] = X[m];
}

// Bins m < NZ of the pair's spectrum row (the rest are not read; see row_code).  The
// spectra are loop-invariant: an opaque pointer stops the compiler from hoisting the
// 2 x 16 loads out of the scale loop (which costs 64 VGPRs and spills).
template <int LOGN, int NZ>
__device__ __forceinline__ void load_spec_nz(cpx (&X)[16], const cpx* row, int t) {
  using P = FftPlan<LOGN>;
  if constexpr (P::NT >= kWave) {
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(row);
    int voff = 8 * t;
    asm volatile("" : "+v"(voff));
#pragma unroll
    for (int m = 0; m < 16; ++m) X[m] = m < NZ ? buf_ld_c64(r, voff, 8 * m * P::NT) : mkc(0.f, 0.f);
  } else {
    asm volatile("" : "+s"(row));
#pragma unroll
    for (int m = 0; m < 16; ++m) X[m] = m < NZ ? row[t + m * P::NT] : mkc(0.f, 0.f);
  }
}

template <int LOGN>
__device__ __forceinline__ void load_spec(cpx (&X)[16], const cpx* row, int t) {
  load_spec_nz<LOGN, 16>(X, row, t);
}

// Row store of 16 positions per thread.  BUF (rows owned by whole waves): buffer stores off
// a wave-uniform row base, no per-position address registers; otherwise plain stores
// masked to pos < n0.  A padded row (n0 < N) sends the positions past
// n0 to voffset = n0 * sizeof(T), outside the descriptor's extent whether or not the
// hardware's range check counts the SGPR offset (the position's m * NT part sits there), so
// they are dropped and never reach the next row or past the buffer's end.
// FULL: the full-row kernels (n0 = N) compile only the unmasked loop, the padded-row kernels
// (launched for n0 < N) only the masked one -- a runtime choice between two copies of the
// store loop cost phase A registers (48 -> 140 spilled bytes per lane).
template <int LOGN, bool BUF, bool FULL, int AUX = 0, typename T, typename F>
__device__ __forceinline__ void put_row(T* row, int t, int n0, F&& val) {
  using P = FftPlan<LOGN>;
  if constexpr (BUF) {
    constexpr int SZ = static_cast<int>(sizeof(T));
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(row, n0 * SZ);
    if constexpr (FULL) {
#pragma unroll
      for (int m = 0; m < 16; ++m) buf_st<AUX>(val(m), r, SZ * t, SZ * m * P::NT);
    } else {
      int tt = t;  // per row, not hoisted out of the caller's row loop (16 live selects)
      asm volatile("" : "+v"(tt));
#pragma unroll
      for (int m = 0; m < 16; ++m)
        buf_st<AUX>(val(m), r, tt + m * P::NT < n0 ? SZ * t : SZ * n0, SZ * m * P::NT);
    }
  } else {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int pos = t + m * P::NT;
      if (pos < n0) row[pos] = val(m);
    }
  }
}

// Regime of the time smoother F_k = exp(-(sn k)^2 / 2) (sn = (s/dt) 2 pi / N): the largest
// Q in {1, 2} with F <= exp(-kBandT^2/2) for |k| >= K0 = N / 2^(4Q+1), else 0.  A smoothed row
// of regime Q has its spectrum in [-K0, K0): shifted by K0 it lies in [0, N/16^Q), and the
// inverse transform enters at pass Q (band_entry) with a time phasor exp(-2 pi i K0 n / N)
// undoing the shift (K0 is a multiple of 16, so the phasor depends on t only).
template <int LOGN>
__device__ __forceinline__ int smooth_regime(double sn) {
  using P = FftPlan<LOGN>;
  int q = 0;
#pragma unroll
  for (int qq = 1; qq <= 2; ++qq) {
    const int k0 = P::N >> (4 * qq + 1);
    if (qq < P::P16 && (P::NT % (1 << (4 * qq))) == 0 && k0 >= 16 && sn * k0 >= kBandT) q = qq;
  }
  return q;
}

// Band bin of a smoothed row of regime Q >= 1: thread t holds at most one bin of [-K0, K0)
// (k = t from m = 0, or k = t - NT from m = 15); returns it times F / (N s) and its slot
// k + K0 in the shifted band [0, 2 K0) (-1: none).
template <int LOGN, int Q>
__device__ __forceinline__ cpx smooth_band_bin(const cpx (&v)[16], cpx smt, int t, int& slot) {
  using P = FftPlan<LOGN>;
  constexpr int K0 = P::N >> (4 * Q + 1);
  asm volatile("" : "+v"(t));  // per-row, not hoisted (register budget)
  int k = 0;
  cpx y = mkc(0.f, 0.f);
  slot = -1;
  if (t < K0) {
    k = t;
    y = v[0];
    slot = k + K0;
  } else if (t >= P::NT - K0) {
    k = t - P::NT;
    y = v[15];
    slot = k + K0;
  }
  const float kk = static_cast<float>(k);
  return cscale(y, smt.y * __builtin_amdgcn_exp2f(smt.x * kk * kk));
}

// v[m] *= exp(-2 pi i K0 n / N) at n = t + m NT (K0 = N / 2^(4Q+1), a multiple of 16: one
// phasor per thread): undoes the K0 shift of a smoothed row's band.
template <int LOGN, int Q>
__device__ __forceinline__ void band_phasor(cpx (&v)[16], int t) {
  using P = FftPlan<LOGN>;
  constexpr int K0 = P::N >> (4 * Q + 1);
  asm volatile("" : "+v"(t));  // recompute per row: hoisted, the phasors spill (WCT VGPR budget 128)
  const cpx ph = expi_frac(-K0 * t, P::N);
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = cmul2(v[m], ph);
}

// Smoothed row from its band bin: band exchange, inverse FFT from pass Q, time phasor
// exp(-2 pi i K0 n / N) (K0 a multiple of 16: the same for the 16 positions of a thread).
template <int LOGN, int Q, bool TWL, bool PHASOR = true>
__device__ __forceinline__ void smooth_from_band(cpx (&v)[16], cpx y, int slot, cpx* my, const cpx* tw,
                                                 int t, int& par, const float4* twl) {
  using P = FftPlan<LOGN>;
  constexpr int STEP = P::NT >> (4 * Q);
  __syncthreads();
  if (slot >= 0) my[slot] = y;
  __syncthreads();
  const int base = t >> (4 * Q);
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = my[base + r * STEP];
  fft_row<LOGN, 1, 1, TWL, Q>(v, my, 0, tw, t, par, twl);
  if constexpr (PHASOR) band_phasor<LOGN, Q>(v, t);
}

// Inverse CWT row of phase A from the pair's spectrum row (global / L2), regime Q.
template <int LOGN, int Q, bool TWL, int NZ = 16>
__device__ __forceinline__ void wct_inverse_row(cpx (&v)[16], const cpx* spec_row, cpx prm, float f0,
                                                cpx* my, const cpx* tw, int t, int& par,
                                                const float4* twl) {
  if constexpr (Q >= 1) {
    asm volatile("" : "+s"(spec_row));  // keep the one load inside the scale loop
    band_entry<LOGN, Q>(v, morlet_bin0(spec_row[t], prm, f0, t), my, t);
    fft_row<LOGN, 1, 1, TWL, Q>(v, my, 0, tw, t, par, twl);
  } else {  // full band; NZ = 8: the negative-frequency half is negligible (f0 >= kBandF0)
    load_spec_nz<LOGN, NZ>(v, spec_row, t);
    if constexpr (NZ < 16)
      morlet_filter_nz<LOGN, NZ>(v, v, prm, f0, t);
    else
      morlet_filter<LOGN>(v, v, prm, f0, t);
    fft_row<LOGN, 1, 1, TWL, 0, NZ>(v, my, 0, tw, t, par, twl);
  }
}

// Row regime of phase A: the CWT band regime and the smoother's, whichever is smaller.
template <int LOGN>
__device__ __forceinline__ int wct_regime(double s, double dt, double f0, double sn) {
  const int qc = band_regime<LOGN>(s, dt, f0), qs = smooth_regime<LOGN>(sn);
  return qc < qs ? qc : qs;
}

// Per-row outputs of the XWT shape from W12 (|W12|^2, angle, arrows).
template <int LOGN, bool BUF, bool FULL>
__device__ __forceinline__ void xwt_outputs(const CwtArgs& a, const cpx (&w)[16], long long rowbase, int t) {
  const int n0 = a.n0;
  if (a.out_pow) put_row<LOGN, BUF, FULL, wct_aux<1>()>(a.out_pow + rowbase, t, n0, [&](int m) { return cabs2(w[m]); });
  if (a.out_sig) {  // phase angle, two positions per packed polynomial
    cpx ang[8];
#pragma unroll
    for (int m = 0; m < 8; ++m)
      ang[m] = fast_atan2f_x2(cpx{w[2 * m].y, w[2 * m + 1].y}, cpx{w[2 * m].x, w[2 * m + 1].x});
    put_row<LOGN, BUF, FULL, wct_aux<1>()>(a.out_sig + rowbase, t, n0, [&](int m) { return ang[m >> 1][m & 1]; });
  }
  if (a.out_u) {
    put_row<LOGN, BUF, FULL, wct_aux<1>()>(a.out_u + rowbase, t, n0, [&](int m) {
      const float r = sqrtf(cabs2(w[m]));
      return r > 0.f ? w[m].y / r : 0.f;
    });
    put_row<LOGN, BUF, FULL, wct_aux<1>()>(a.out_v + rowbase, t, n0, [&](int m) {
      const float r = sqrtf(cabs2(w[m]));
      return r > 0.f ? w[m].x / r : 1.f;
    });
  }
}

// Per-row plan (wct_plan_kernel), one int per scale row:
//   bits 0-1  q     band regime of the row's transforms (wct_regime; 0 without pruning)
//   bit 2     needT the row's time-smoothed fields go to the time-domain workspace (phase B)
//   bit 3     needS the row's smoothed band spectra go to the band workspace (phase C)
//   bit 4     spec  output row whose whole boxcar window has q >= 1: its coherence is made by
//                   phase C from band spectra (no time-domain workspace round trip)
//   bits 5-6  qw    that window's smallest regime (the union of the members' bands)
//   bit 7     needW the row's smoothed spectra go to the wide-band workspace WB (phase C's wide
//                   windows)
//   bits 8-11 e     decimation of the row (wct_dec_kernel), 0 = none: W1, W2 have their spectra in
//                   bins [0, M/2), M = N >> e, so the products |W1|^2, W1 conj(W2) have theirs in
//                   (-M/2, M/2) and the forward transforms run on every (N/M)-th sample (length M)
//   bits 12-15 ew   the row's smoothed band: both smoothed fields have their spectra in
//                   [-Mw/2, Mw/2), Mw = N >> ew (the time Gaussian's cut-off, narrowed further by
//                   the decimation's band); WB holds those Mw bins in FFT order
//   bits 16-17 eu   wide output row (spec set, qw = 0): its window's union band is Mu = N >> eu
//                   (eu in 1..3: the window holds rows of regime q = 0 but none of band ew = 0),
//                   its coherence comes from the WB spectra through one band inverse of Mu bins
//                   per field instead of the time-domain workspace
//   bits 18-21 ec   q-window output row (qw >= 1): the union of its window rows' smoothed bands
//                   is Mc = N >> ec (ec >= 4 qw: the smallest ew of the window, at least the
//                   regime's band), so phase C's band inverses enter at pass ec / 4 with
//                   16 >> (ec % 4) non-zero inputs per thread
enum : int { kPlanQ = 3, kPlanNeedT = 4, kPlanNeedS = 8, kPlanSpec = 16, kPlanQwShift = 5,
             kPlanNeedW = 128, kPlanDecShift = 8, kPlanEwShift = 12, kPlanEuShift = 16,
             kPlanEcShift = 18 };
__device__ __forceinline__ int plan_dec(int pl) { return (pl >> kPlanDecShift) & 15; }
__device__ __forceinline__ int plan_ew(int pl) { return (pl >> kPlanEwShift) & 15; }
__device__ __forceinline__ int plan_eu(int pl) { return (pl >> kPlanEuShift) & 3; }
__device__ __forceinline__ int plan_ec(int pl) { return (pl >> kPlanEcShift) & 15; }
// wide windows need M = N >> 3 >= 32 bins (one band phasor per thread): LOGN >= 8; the
// spectral boxcar keeps K rows in registers: K <= 24
constexpr int kWideMinLogn = 8;
constexpr int kWideMaxE = 3;
constexpr int kWideMaxK = 24;

// Decimated rows: M = N >> e with e in [kDecMinE(LOGN), LOGN - 5] -- M >= 32 (the band
// inverse's phasor is one per thread), M <= 4096 (256-thread decimated groups) -- for full rows
// (n0 = N; a row truncated at n0 < N is not band-limited) of LOGN >= 10.
template <int LOGN> __host__ __device__ constexpr int dec_min_e() { return LOGN - 12 > 1 ? LOGN - 12 : 1; }
constexpr int kDecMinLogn = 10;
constexpr int kDecMinLogm = 5;
constexpr int kDecMaxLogm = 12;
// the decimated transforms run at M_eng = max(M, 2^kDecEngLogm): rows of smaller M share one
// launch (their bins past M/2 are dropped on store)
constexpr int kDecEngLogm = 8;
__host__ __device__ constexpr int dec_rows_per_wg(int logm) { return logm >= 12 ? 1 : 256 >> (logm - 4); }
// schedule of wct_dec_kernel (after the plan's 3 S + 1 ints and S row-list ints):
// [4 logm + 0] first row-list index, [+1] row count, [+2] first workgroup; [64] workgroups
constexpr int kDecSched = 68;
// [kSchedWide], [kSchedWide + 1]: first and last wide output row (first > last: none)
constexpr int kSchedWide = 65;

// e of row r (0: not decimated): the smallest M = 2^m >= 32 with psi negligible from bin M/2 on
// (alpha M/2 - f0 >= kBandT, the band_regime criterion), if that M is at most N / 2.
template <int LOGN>
__device__ __forceinline__ int dec_e(double s, double dt, double f0) {
  using P = FftPlan<LOGN>;
  const double alpha = s * 2.0 * kPi / (static_cast<double>(P::N) * dt);
  int lm = kDecMinLogm;
  while (lm < LOGN && alpha * static_cast<double>(1 << (lm - 1)) - f0 < kBandT) ++lm;
  const int e = LOGN - lm;
  return (e >= dec_min_e<LOGN>() && e <= LOGN - kDecMinLogm) ? e : 0;
}

// Smoothed band exponent of a row: the largest e <= LOGN - 5 with the time Gaussian
// F_k = exp(-(sn k)^2 / 2) below exp(-kBandT^2/2) for |k| >= N >> (e + 1) (the criterion of
// smooth_regime, at every power of two).
template <int LOGN>
__device__ __forceinline__ int smooth_e(double sn) {
  using P = FftPlan<LOGN>;
  int e = 0;
  while (e < LOGN - 5 && sn * static_cast<double>(P::N >> (e + 2)) >= kBandT) ++e;
  return e;
}

template <int LOGN>
__device__ __forceinline__ int plan_q(const double* scales, int r, double dt, double f0) {
  using P = FftPlan<LOGN>;
  const double s = scales[r];
  return wct_regime<LOGN>(s, dt, f0, s / dt * 2.0 * kPi / P::N);
}

// One workgroup; plan[S] = last output row of phase B (the time path), -1 if none.
// scratch: 2 S ints (row regimes, then each output row's window regime or -1), then the
// decimated rows' list (S ints) and schedule (kDecSched ints), see wct_dec_kernel.
template <int LOGN>
__device__ __forceinline__ void wct_plan_body(const double* __restrict__ scales, int S, double dt, double f0,
                                              int K, int prune, int dec, int wide,
                                              long long batch, int* __restrict__ plan,
                                              int* __restrict__ scratch) {
  __shared__ int last;
  if (threadIdx.x == 0) last = -1;
  const int LO = K / 2, HI = (K - 1) / 2;
  int* qrow = scratch;  // regime | decimation e << 4 | smoothed band ew << 8
  int* qwin = scratch + S;  // window regime (>= 1: q window) | wide window eu << 4
  constexpr bool kWide = LOGN >= kWideMinLogn;
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    const int ed = dec ? dec_e<LOGN>(scales[r], dt, f0) : 0;
    const int es = (prune && kWide) ? smooth_e<LOGN>(scales[r] / dt * 2.0 * kPi / FftPlan<LOGN>::N) : 0;
    qrow[r] = (prune ? plan_q<LOGN>(scales, r, dt, f0) : 0) | (ed << 4) | (max(es, ed) << 8);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < S; i += blockDim.x) {  // window regime; -1: some member has q = 0
    int qw = 3, ew = 15;
    for (int r = max(0, i - LO); r <= min(S - 1, i + HI); ++r) {
      qw = min(qw, qrow[r] & 15);
      ew = min(ew, qrow[r] >> 8);
    }
    // q windows keep phase C's band route; the other windows whose rows all have a smoothed
    // band of at most N/2 take the wide route (union band N >> eu, capped at eu = 3: a wider
    // band than needed is exact), the rest the time path
    const int q_ok = (prune && qw >= 1) ? qw : -1;
    const int eu = (prune && kWide && wide >= 1 && K <= kWideMaxK && q_ok < 1 && ew >= wide)
                       ? min(ew, kWideMaxE) : 0;
    // q windows: the union band of the smoothed rows (never wider than the regime's band)
    const int ec = q_ok >= 1 ? max(4 * q_ok, min(ew, LOGN - 5)) : 0;
    qwin[i] = (q_ok >= 1 ? q_ok : 0) | (eu << 4) | (ec << 8);
  }
  __syncthreads();
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    const int q = qrow[r] & 15, e = (qrow[r] >> 4) & 15, ew = qrow[r] >> 8;
    bool needT = false, needS = false, needW = false;
    for (int i = max(0, r - HI); i <= min(S - 1, r + LO); ++i) {  // outputs whose window holds r
      const int qwi = qwin[i] & 15, eui = (qwin[i] >> 4) & 3;
      if (qwi >= 1) needS = true;
      else if (eui >= 1) needW = true;
      else needT = true;
    }
    const int qw = qwin[r] & 15, eu = (qwin[r] >> 4) & 3, ec = (qwin[r] >> 8) & 15;
    plan[r] = q | (needT ? kPlanNeedT : 0) | (needS && q >= 1 ? kPlanNeedS : 0) |
              (needW ? kPlanNeedW : 0) |
              (qw >= 1 ? kPlanSpec | (qw << kPlanQwShift) | (ec << kPlanEcShift) : 0) |
              (eu >= 1 ? kPlanSpec | (eu << kPlanEuShift) : 0) |
              (e << kPlanDecShift) | (ew << kPlanEwShift);
    if (qw < 1 && eu < 1) atomicMax(&last, r);
  }
  __syncthreads();
  // decimated rows by class (LDS counters; the order of rows within a class is immaterial)
  __shared__ int cnt[16], cur[16], wlo, whi;
  if (threadIdx.x == 0) {
    wlo = S;
    whi = -1;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < S; r += blockDim.x)
    if (plan_eu(plan[r])) {
      atomicMin(&wlo, r);
      atomicMax(&whi, r);
    }
  if (threadIdx.x < 16) cnt[threadIdx.x] = cur[threadIdx.x] = 0;
  __syncthreads();
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    const int e = plan_dec(plan[r]);
    if (e > 0) atomicAdd(&cnt[max(LOGN - e, kDecEngLogm)], 1);
  }
  __syncthreads();
  int* rows = scratch + 2 * S;
  int* sched = rows + S;
  if (threadIdx.x == 0) {
    plan[S] = last;
    int nlist = 0, wg = 0;
    for (int lm = kDecMaxLogm; lm >= kDecEngLogm; --lm) {
      sched[4 * lm + 0] = nlist;
      sched[4 * lm + 1] = cnt[lm];
      sched[4 * lm + 2] = wg;
      cur[lm] = nlist;
      nlist += cnt[lm];
      wg += static_cast<int>((batch * cnt[lm] + dec_rows_per_wg(lm) - 1) / dec_rows_per_wg(lm));
    }
    sched[64] = wg;
    sched[kSchedWide] = wlo;
    sched[kSchedWide + 1] = whi;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < S; r += blockDim.x) {
    const int e = plan_dec(plan[r]);
    if (e > 0) rows[atomicAdd(&cur[max(LOGN - e, kDecEngLogm)], 1)] = r;
  }
}

// Spectra and plan in one launch: workgroups 0 .. gridDim - 2 transform the series, the last
// one plans the rows (they are independent; one launch less on the dependent chain).
template <int LOGN>
__global__ void __launch_bounds__(WctGeom<LOGN>::BLOCK) wct_spectra_plan(CwtArgs a, cpx* __restrict__ spec,
                                                                         int K, int dec, int wide,
                                                                         int* __restrict__ plan) {
  if (blockIdx.x + 1 == gridDim.x)
    wct_plan_body<LOGN>(a.scales, a.S, a.dt, a.f0, K, a.prune, dec, wide, a.batch, plan,
                        plan + a.S + 1);
  else
    spectra_body<LOGN>(a, spec, blockIdx.x);
}

struct WctRowCtx {
  const cpx* spec1;
  const cpx* spec2;
  const cpx* prm_tab;
  const cpx* smt_tab;
  cpx* TA;
  cpx* TB;
  cpx* band;  // LDS: the band bins A1, A2 of a narrow row (2 * (N >> 8) complex)
  cpx* SB;    // smoothed band spectra [batch][S][2][NT] (index k + NT/2), see wct_plan
  const cpx* DY;  // decimated rows: W12's spectrum [batch][S][N/2] (M bins, wct_dec_kernel)
  cpx* WB;        // wide-band smoothed spectra [batch][S][2][N/2] (Mw bins, plan bits ew)
  const int* plan;
  long long b;
  int j0;
};

// WB slot of row j, field f (0: Z = FFT(|W1|^2 + i |W2|^2) F / (N s), 1: FFT(W12) F / (N s)):
// bins k in [-N/4, N/4) at index k + N/4; a row fills only its band [-Mw/2, Mw/2), Mw = N >> ew
// (plan bits 12-15), and readers mask by that band.  wct_wide_boxcar later overwrites the slot
// of a wide output row, bin by bin in place, with its window's sums (same index per bin).
template <int LOGN>
__device__ __forceinline__ cpx* wb_row(cpx* WB, long long b, int S, int j, int f) {
  return WB + ((b * S + j) * 2 + f) * static_cast<long long>(FftPlan<LOGN>::N / 2) + FftPlan<LOGN>::N / 4;
}
template <int BIT = 4>
__device__ __forceinline__ void wb_put(cpx* row, int mw, int k, cpx y) {
  if (k >= -(mw >> 1) && k < (mw >> 1)) st_c<BIT>(row + k, y);
}
// The whole smoothed spectrum of a thread (bins t + (m < 8 ? m : m - 16) NT) into a WB slot.
// Rows owned by whole waves (NT >= 64) store through a wave-uniform buffer descriptor: one
// offset VGPR, the per-m bin offsets as immediates (no 64-bit address per store).
template <int LOGN>
__device__ __forceinline__ void wb_put_full(cpx* row, int mw, const cpx (&v)[16], int t) {
  using P = FftPlan<LOGN>;
  asm volatile("" : "+v"(t));  // bin indices per row, not hoisted out of the scale loop (VGPRs)
  if constexpr (P::NT >= kWave) {
    // slot start as the descriptor base (buffer offsets are unsigned); |k| < Mw/2 <= N/4 = 4 NT
    // leaves only m = 0..3 and 12..15
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(row - P::N / 4);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (m >= 4 && m < 12) continue;
      const int off = (m < 8 ? m : m - 16) * P::NT;
      const int k = t + off;
      if (k >= -(mw >> 1) && k < (mw >> 1)) buf_st<wct_aux<4>()>(v[m], r, 8 * t, 8 * (off + P::N / 4));
    }
  } else {
#pragma unroll
    for (int m = 0; m < 16; ++m) wb_put(row, mw, t + (m < 8 ? m : m - 16) * P::NT, v[m]);
  }
}

// Full-length inverse transform of a spectrum held in bins k in [-M/2, M/2), M = N >> E, stored
// in FFT order (bin k at k mod M) in global memory: the band is shifted by H = M/2 to [0, M),
// transformed from the entry pass/width it allows (pass Q = E/4, inputs r < NZ = 16 >> E%4
// non-zero: band_entry / the narrowed first pass), and the shift undone by the time phasor
// exp(-2 pi i H n / N) (H a multiple of 16: one phasor per thread).  Split into the loads
// (band_load) and the transform (band_ifft) so that callers issue the next transform's loads
// before the current one's stores: loads and stores share one counter (vmcnt), so a load
// issued after a row of stores waits for all of them.
template <int LOGN, int E>
struct BandGeom {
  using P = FftPlan<LOGN>;
  static constexpr int M = P::N >> E;
  static constexpr int H = M / 2;
  static constexpr int Q = E / 4;
  static constexpr int NZ = 16 >> (E % 4);
  static constexpr int NLD = Q == 0 ? NZ : 1;  // loads per thread
  static_assert(M >= 32 && Q < P::P16, "band inverse");
};

template <int LOGN, int E>
__device__ __forceinline__ void band_load(cpx (&pre)[8], const cpx* __restrict__ g, int t) {
  using B = BandGeom<LOGN, E>;
  using P = FftPlan<LOGN>;
  if constexpr (B::Q == 0) {
    // shifted bin t + r NT (< M) is bin t + r NT + H (r < NZ/2) or t + r NT - H of g
    if constexpr (P::NT >= kWave) {  // rows are wave-aligned: buffer loads, offsets in SGPRs
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(g);
#pragma unroll
      for (int r = 0; r < B::NZ; ++r)
        pre[r] = buf_ld_c64<wct_aux<16>()>(rs, 8 * t, 8 * (r * P::NT + (r < B::NZ / 2 ? B::H : -B::H)));
    } else {
#pragma unroll
      for (int r = 0; r < B::NZ; ++r) pre[r] = g[t + r * P::NT + (r < B::NZ / 2 ? B::H : -B::H)];
    }
  } else {
    // per-row offsets, not hoisted: hoisted, one 64-bit address per band width and buffer
    // (DY / TA / TB) stayed live across the row loop and spilled -- 9 x 8 bytes per lane
    // written to scratch by every workgroup's prologue, 0.4 GB of C4's HBM writes
    int tt = t;
    asm volatile("" : "+v"(tt));
    if constexpr (P::NT >= kWave) {  // wave-uniform row: buffer load, lanes t >= M read 0
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(g, B::M * static_cast<int>(sizeof(cpx)));
      pre[0] = buf_ld_c64<wct_aux<16>()>(rs, tt < B::M ? 8 * ((tt + B::H) & (B::M - 1)) : 8 * B::M, 0);
    } else {
      pre[0] = tt < B::M ? g[(tt + B::H) & (B::M - 1)] : mkc(0.f, 0.f);
    }
  }
}

template <int LOGN, int E, bool TWL>
__device__ __forceinline__ void band_ifft(cpx (&v)[16], const cpx (&pre)[8], cpx* my, const cpx* tw, int t,
                                          int& par, const float4* twl) {
  using B = BandGeom<LOGN, E>;
  using P = FftPlan<LOGN>;
  if constexpr (B::Q == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = r < B::NZ ? pre[r] : mkc(0.f, 0.f);
    fft_row<LOGN, 1, 1, TWL, 0, B::NZ>(v, my, 0, tw, t, par, twl);
  } else {
    band_entry<LOGN, B::Q, B::NZ>(v, pre[0], my, t);
    fft_row<LOGN, 1, 1, TWL, B::Q, B::NZ>(v, my, 0, tw, t, par, twl);
  }
  int tt = t;
  asm volatile("" : "+v"(tt));  // per row, not hoisted (register budget)
  const cpx ph = expi_frac(-B::H * tt, P::N);
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = cmul2(v[m], ph);
}

// Phase A rows [r0, r1) of decimation e = E: the decimated spectra (wct_dec_kernel) hold W12's
// whole spectrum and, for time-path rows, the smoothed fields' spectra in the rows' TA / TB
// slots.  One band inverse gives W12 (power, phase, arrows); time-path rows add two more for
// (T1, T2) and T12, written over the spectra they were made from.
template <int LOGN, int E, bool TWL>
__device__ __forceinline__ void wct_dec_rows(const CwtArgs& a, const WctRowCtx& c, int r0, int r1, cpx* my,
                                             const cpx* tw, int g, int t, int& par, const float4* twl) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  constexpr bool BUF = P::NT >= kWave;
  const int n0 = a.n0;
  auto dy_row = [&](int r) {  // W12 spectrum of this group's row in the iteration at r
    const int jl = r + g;
    return c.DY + (c.b * a.S + c.j0 + (jl < r1 ? jl : r0)) * (P::N / 2);
  };
  cpx pre[8];
  band_load<LOGN, E>(pre, dy_row(r0), t);
  for (int r = r0; r < r1; r += G::ROWS) {
    const int jl = r + g;
    const bool valid = jl < r1;
    const long long rowbase = (c.b * a.S + c.j0 + (valid ? jl : r0)) * static_cast<long long>(n0);
    const bool more = r + G::ROWS < r1;  // uniform
    int pl_any = 0;  // workgroup-uniform (the band inverses hold barriers)
#pragma unroll
    for (int gg = 0; gg < G::ROWS; ++gg)
      if (r + gg < r1) pl_any |= c.plan[c.j0 + r + gg];
    const bool tpath = pl_any & kPlanNeedT;
    cpx v[16];
    band_ifft<LOGN, E, TWL>(v, pre, my, tw, t, par, twl);  // W12
    if (tpath)
      band_load<LOGN, E>(pre, c.TA + rowbase, t);
    else if (more)
      band_load<LOGN, E>(pre, dy_row(r + G::ROWS), t);
    if (valid) xwt_outputs<LOGN, BUF, true>(a, v, rowbase, t);
    if (tpath) {
      const bool wr = valid && (c.plan[c.j0 + (valid ? jl : r0)] & kPlanNeedT);
      band_ifft<LOGN, E, TWL>(v, pre, my, tw, t, par, twl);  // (T1, T2)
      band_load<LOGN, E>(pre, c.TB + rowbase, t);
      if (wr) put_row<LOGN, BUF, true, wct_aux<2>()>(c.TA + rowbase, t, n0, [&](int m) { return v[m]; });
      band_ifft<LOGN, E, TWL>(v, pre, my, tw, t, par, twl);  // T12
      if (more) band_load<LOGN, E>(pre, dy_row(r + G::ROWS), t);
      if (wr) put_row<LOGN, BUF, true, wct_aux<2>()>(c.TB + rowbase, t, n0, [&](int m) { return v[m]; });
    }
  }
}

// Phase A rows [r0, r1) of the workgroup's chunk, all of regime Q (one code path per loop:
// branches between transform variants inside one loop cost the register allocator dearly).
//   Q = 0: W1, W2 -> z1 = |W1|^2 + i |W2|^2, W12 -> full smoothing transforms of both.
//   Q >= 1: pruned inverse transforms, and once each forward transform is done only the one
//   band bin per thread is kept (2 VGPRs), so W12's outputs and transforms run with z1 dead.
template <int LOGN, bool FULL, int Q, bool TWL, int NZ = 16>
__device__ __forceinline__ void wct_rows(const CwtArgs& a, const WctRowCtx& c, int r0, int r1, cpx* my,
                                         const cpx* tw, int g, int t, int& par, const float4* twl) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  constexpr bool BUF = P::NT >= kWave;  // padded rows too: put_row's extent
  const float f0 = static_cast<float>(a.f0);
  const int n0 = a.n0;
  for (int r = r0; r < r1; r += G::ROWS) {
    const int jl = r + g;
    const bool valid = jl < r1;
    const cpx prm = c.prm_tab[valid ? jl : r0];
    const cpx smt = c.smt_tab[valid ? jl : r0];
    cpx w1[16], v[16];
    const long long rowbase = (c.b * a.S + c.j0 + (valid ? jl : r0)) * static_cast<long long>(n0);
    if constexpr (Q == 2 && FULL && G::ROWS == 1) {
      // Narrow rows: W1, W2 have their spectra A1, A2 in bins [0, KB) and the smoothed fields
      // theirs in [-K0, K0), 2 K0 = KB.  The forward transforms of z1 and W12 are replaced
      // by the spectral correlations they equal on a full row (n0 = N):
      //   FFT(|W1|^2)[k] = N sum_j A1[j] conj(A1[j-k]),  FFT(W1 conj W2)[k] = N sum_j A1[j] conj(A2[j-k]).
      constexpr int KB = P::N >> 8;
      constexpr int K0 = KB / 2;
      const cpx* sp = c.spec1;
      asm volatile("" : "+s"(sp));  // keep the two loads inside the scale loop
      const cpx y1 = morlet_bin0(sp[t], prm, f0, t);
      const cpx y2 = morlet_bin0(sp[P::N + t], prm, f0, t);
      __syncthreads();  // the previous row's correlation reads of c.band are done
      if (t < KB) {
        c.band[t] = y1;
        c.band[KB + t] = y2;
      }
      band_entry<LOGN, 2>(w1, y1, my, t);
      fft_row<LOGN, 1, 1, TWL, 2>(w1, my, 0, tw, t, par, twl);
      band_entry<LOGN, 2>(v, y2, my, t);
      fft_row<LOGN, 1, 1, TWL, 2>(v, my, 0, tw, t, par, twl);
#pragma unroll
      for (int m = 0; m < 16; ++m) w1[m] = cmul2_conj(w1[m], v[m]);
      if (valid) xwt_outputs<LOGN, BUF, FULL>(a, w1, rowbase, t);
      cpx zy = mkc(0.f, 0.f), wy = mkc(0.f, 0.f);
      const int k = t - P::NT / 2;  // band-workspace index t <-> bin k
      const bool holder = k >= -K0 && k < K0;
      if (holder) {  // bin k of both smoothed fields

        const int jlo = k > 0 ? k : 0, jhi = k < 0 ? KB + k : KB;
        cpx s11 = mkc(0.f, 0.f), s22 = s11, s12 = s11;
        for (int jj = jlo; jj < jhi; ++jj) {
          const cpx a1 = c.band[jj], a2 = c.band[KB + jj];
          const cpx b1 = cconj(c.band[jj - k]), b2 = cconj(c.band[KB + jj - k]);
          s11 = cfma(a1.xx, b1, s11);
          s11 = cfma(a1.yy, mkc(-b1.y, b1.x), s11);
          s22 = cfma(a2.xx, b2, s22);
          s22 = cfma(a2.yy, mkc(-b2.y, b2.x), s22);
          s12 = cfma(a1.xx, b2, s12);
          s12 = cfma(a1.yy, mkc(-b2.y, b2.x), s12);
        }
        const float kk = static_cast<float>(k);
        const float f = static_cast<float>(P::N) * smt.y * __builtin_amdgcn_exp2f(smt.x * kk * kk);
        zy = (s11 + mul_i<1>(s22)) * f;  // FFT(|W1|^2 + i |W2|^2) = S11 + i S22
        wy = s12 * f;
      }
      const int pl = c.plan[c.j0 + (valid ? jl : r0)];
      if (valid && (pl & kPlanNeedS)) {
        cpx* sb = c.SB + (c.b * a.S + c.j0 + jl) * 2ll * P::NT;
        sb[t] = zy;
        sb[P::NT + t] = wy;
      }
      if (valid && holder && (pl & kPlanNeedW)) {
        const int mw = P::N >> plan_ew(pl);
        wb_put(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 0), mw, k, zy);
        wb_put(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 1), mw, k, wy);
      }
      if (pl & kPlanNeedT) {
        const int slot = holder ? k + K0 : -1;
        smooth_from_band<LOGN, 2, TWL>(w1, wy, slot, my, tw, t, par, twl);
        if (valid) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TB + rowbase, t, n0, [&](int m) { return w1[m]; });  // smoothed W12/s
        smooth_from_band<LOGN, 2, TWL>(v, zy, slot, my, tw, t, par, twl);
        if (valid) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TA + rowbase, t, n0, [&](int m) { return v[m]; });
      }
      continue;
    }
    wct_inverse_row<LOGN, Q, TWL, NZ>(v, c.spec1, prm, f0, my, tw, t, par, twl);
#pragma unroll
    for (int m = 0; m < 16; ++m) w1[m] = v[m];
    wct_inverse_row<LOGN, Q, TWL, NZ>(v, c.spec2, prm, f0, my, tw, t, par, twl);
    // W12 = W1 conj(W2), z1 = |W1|^2 + i |W2|^2, zero past n0 (the reference smooths the
    // row zero-padded to N)
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int pos = t + m * P::NT;
      const cpx w12 = cmul2_conj(w1[m], v[m]);
      const cpx z1 = mkc(cabs2(w1[m]), cabs2(v[m]));
      const bool in = FULL || pos < n0;
      w1[m] = in ? w12 : mkc(0.f, 0.f);
      v[m] = in ? z1 : mkc(0.f, 0.f);
    }
    fft_row<LOGN, -1, 1, TWL>(v, my, 0, tw, t, par, twl);
    if constexpr (Q == 0) {
      const int pl = c.plan[c.j0 + (valid ? jl : r0)];
      int pl_any = 0;  // workgroup-uniform (the smoothing transforms hold barriers)
#pragma unroll
      for (int gg = 0; gg < G::ROWS; ++gg)
        if (r + gg < r1) pl_any |= c.plan[c.j0 + r + gg];
      const bool wb = valid && (pl & kPlanNeedW);
      const int mw = P::N >> plan_ew(pl);
      smooth_filter<LOGN>(v, smt.x, smt.y, t);
      if (wb) wb_put_full<LOGN>(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 0), mw, v, t);
      if (pl_any & kPlanNeedT) {
        fft_row<LOGN, 1, 1, TWL>(v, my, 0, tw, t, par, twl);
        // (T1, T2): smoothed |W1|^2/s, |W2|^2/s
        if (valid && (pl & kPlanNeedT)) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TA + rowbase, t, n0, [&](int m) { return v[m]; });
      }
      // the XWT-shaped outputs once z1 is dead (only W12 live: no spills around atan2)
      if (valid) xwt_outputs<LOGN, BUF, FULL>(a, w1, rowbase, t);
      fft_row<LOGN, -1, 1, TWL>(w1, my, 0, tw, t, par, twl);
      smooth_filter<LOGN>(w1, smt.x, smt.y, t);
      if (wb) wb_put_full<LOGN>(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 1), mw, w1, t);
      if (pl_any & kPlanNeedT) {
        fft_row<LOGN, 1, 1, TWL>(w1, my, 0, tw, t, par, twl);
        if (valid && (pl & kPlanNeedT)) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TB + rowbase, t, n0, [&](int m) { return w1[m]; });
      }
    } else {
      int zslot, wslot;
      const cpx zy = smooth_band_bin<LOGN, Q>(v, smt, t, zslot);
      if (valid) xwt_outputs<LOGN, BUF, FULL>(a, w1, rowbase, t);
      fft_row<LOGN, -1, 1, TWL>(w1, my, 0, tw, t, par, twl);
      const cpx wy = smooth_band_bin<LOGN, Q>(w1, smt, t, wslot);
      const int pl = c.plan[c.j0 + (valid ? jl : r0)];
      int pl_any = 0;  // workgroup-uniform (the smoothing transforms hold barriers)
#pragma unroll
      for (int gg = 0; gg < G::ROWS; ++gg)
        if (r + gg < r1) pl_any |= c.plan[c.j0 + r + gg];
      if (valid && (pl & kPlanNeedS)) {  // thread t holds bin k_t: index k_t + NT/2
        cpx* sb = c.SB + (c.b * a.S + c.j0 + jl) * 2ll * P::NT;
        const int ix = (t + P::NT / 2) & (P::NT - 1);
        sb[ix] = zy;
        sb[P::NT + ix] = wy;
      }
      if (valid && (pl & kPlanNeedW) && zslot >= 0) {  // bin k = slot - K0 (zslot == wslot)
        constexpr int K0 = P::N >> (4 * Q + 1);
        const int mw = P::N >> plan_ew(pl);
        wb_put(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 0), mw, zslot - K0, zy);
        wb_put(wb_row<LOGN>(c.WB, c.b, a.S, c.j0 + jl, 1), mw, zslot - K0, wy);
      }
      if (pl_any & kPlanNeedT) {
        smooth_from_band<LOGN, Q, TWL>(w1, wy, wslot, my, tw, t, par, twl);
        if (valid) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TB + rowbase, t, n0, [&](int m) { return w1[m]; });  // smoothed W12/s
        smooth_from_band<LOGN, Q, TWL>(v, zy, zslot, my, tw, t, par, twl);
        if (valid) put_row<LOGN, BUF, FULL, wct_aux<2>()>(c.TA + rowbase, t, n0, [&](int m) { return v[m]; });
      }
    }
  }
}

// KIND: which rows this launch runs -- 0 the full-band rows (regime 0, not decimated), 1 the
// other non-decimated rows (regimes 1, 2), 2 the decimated rows (plan e > 0).  Separate
// launches over the same chunk grid, so that each row kind gets its own kernel's register
// budget (one kernel for kinds 0 and 1 spilled 128 bytes per lane on LOGN 13, kind 0 alone 48).
template <int LOGN> __device__ __forceinline__ int phase_a_kind(int pl) {
  return plan_dec(pl) > 0 ? 2 : ((pl & kPlanQ) == 0 ? 0 : 1);
}
template <int LOGN, bool FULL, int KIND>
__global__ void __launch_bounds__((WctGeom<LOGN>::BLOCK), (WctGeom<LOGN>::MINW))
    wct_phase_a(CwtArgs a, const cpx* __restrict__ spec, cpx* __restrict__ TA, cpx* __restrict__ TB,
                cpx* __restrict__ SB, const cpx* __restrict__ DY, cpx* __restrict__ WB,
                const int* __restrict__ plan) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  constexpr int BAND_F4 = LOGN >= 12 ? (P::N >> 8) : 1;  // 2 * (N >> 8) complex
  constexpr int CSTR = P::PADN;  // row buffers: the FFT exchange
  __shared__ float4 lds4[(G::ROWS * CSTR) / 2 + G::MAXCHUNK + G::TWL_F4 + G::MAXCHUNK / 4 + BAND_F4];
  cpx* lds = reinterpret_cast<cpx*>(lds4);
  cpx* prm_tab = lds + G::ROWS * CSTR;         // (alpha, log2 c) of the Morlet filter
  cpx* smt_tab = prm_tab + G::MAXCHUNK;        // (beta, 1/(N s)) of the time smoother
  float4* twl = lds4 + (G::ROWS * CSTR) / 2 + G::MAXCHUNK;
  int* q_tab = reinterpret_cast<int*>(twl + G::TWL_F4);  // row regimes (wct_regime)
  const int tid = threadIdx.x;
  const int g = tid / P::NT;
  const int t = fft_thread<LOGN>(tid - g * P::NT);
  // the scale chunks of one pair share its two spectra: keep them on one XCD's L2
  // (chunk-major order for the decimated rows, costliest chunks first, measured neutral: r04)
  const long long blk = xcd_remap(blockIdx.x, gridDim.x);
  const long long b = blk / a.nchunks;
  const int ch = static_cast<int>(blk - b * a.nchunks);
  const int j0 = ch * a.chunk;
  const int j1 = min(a.S, j0 + a.chunk);
  cpx* my = lds + g * CSTR;
  {  // any rows of this launch's kind in the chunk?  (uniform: every thread reads the same plan)
    bool any = false;
    for (int r = j0; r < j1; ++r) any |= phase_a_kind<LOGN>(plan[r]) == KIND;
    if (!any) return;
  }

  for (int i = tid; i < j1 - j0; i += G::BLOCK) {
    const int pl = plan[j0 + i];
    // run key: the regime, 4 + e for decimated rows
    q_tab[i] = plan_dec(pl) > 0 ? 4 + plan_dec(pl) : (pl & kPlanQ);
    if (KIND == 2) continue;  // decimated rows need no filter tables
    const double s = a.scales[j0 + i];
    prm_tab[i] = morlet_params(s, a.dt, P::N);
    const double sn = s / a.dt * 2.0 * kPi / P::N;  // (s/dt) * (2 pi / N)
    smt_tab[i] = mkc(static_cast<float>(-0.5 * 1.44269504088896340736 * sn * sn),
                     static_cast<float>(1.0 / (static_cast<double>(P::N) * s)));
  }
  constexpr bool TWL = G::TWL;
  cpx tw[TWL ? P::NTW_REG : P::NTW_ALLOC];
  if constexpr (TWL) {
    fft_twiddle_table<LOGN>(twl, tid, G::BLOCK);
    fft_twiddles_tail<LOGN>(tw, t);
  } else {
    fft_twiddles<LOGN>(tw, t);
  }
  int par = 0;
  __syncthreads();

  WctRowCtx c;
  c.spec1 = spec + 2 * b * static_cast<long long>(P::N);
  c.spec2 = c.spec1 + P::N;
  c.prm_tab = prm_tab;
  c.smt_tab = smt_tab;
  c.TA = TA;
  c.TB = TB;
  c.band = reinterpret_cast<cpx*>(q_tab + G::MAXCHUNK);
  c.SB = SB;
  c.DY = DY;
  c.WB = WB;
  c.plan = plan;
  c.b = b;
  c.j0 = j0;
  // runs of equal regime (the table is shared: every thread sees the same runs)
  const int nrow = j1 - j0;
  int r0 = 0;
  while (r0 < nrow) {
    const int q = q_tab[r0];
    int r1 = r0 + 1;
    while (r1 < nrow && q_tab[r1] == q) ++r1;
    if (q >= 4) {  // decimated rows (full rows only)
      if constexpr (KIND == 2 && FULL && LOGN >= kDecMinLogn) {
        switch (q - 4) {
#define WTMI_DR(EE)                                                                     \
  case EE:                                                                              \
    if constexpr (EE >= dec_min_e<LOGN>() && EE <= LOGN - kDecMinLogm)                  \
      wct_dec_rows<LOGN, EE, TWL>(a, c, r0, r1, my, tw, g, t, par, twl);                \
    break;
          WTMI_DR(1) WTMI_DR(2) WTMI_DR(3) WTMI_DR(4) WTMI_DR(5) WTMI_DR(6) WTMI_DR(7) WTMI_DR(8) WTMI_DR(9)
#undef WTMI_DR
          default: break;
        }
      }
    } else if (KIND == 2) {
    } else if (q == 0) {
      if constexpr (KIND == 0) {
        if (a.prune && a.f0 >= kBandF0 && P::NT >= 16)  // negative frequencies dropped: half the bins
          wct_rows<LOGN, FULL, 0, TWL, 8>(a, c, r0, r1, my, tw, g, t, par, twl);
        else
          wct_rows<LOGN, FULL, 0, TWL>(a, c, r0, r1, my, tw, g, t, par, twl);
      }
    } else if constexpr (KIND == 1) {
      if constexpr (P::P16 >= 2 && (P::NT % 16) == 0 && (P::N >> 5) >= 16) {
        if constexpr (P::P16 >= 3 && (P::NT % 256) == 0 && (P::N >> 9) >= 16) {
          if (q >= 2) {
            wct_rows<LOGN, FULL, 2, TWL>(a, c, r0, r1, my, tw, g, t, par, twl);
            r0 = r1;
            continue;
          }
        }
        wct_rows<LOGN, FULL, 1, TWL>(a, c, r0, r1, my, tw, g, t, par, twl);
      }
    }
    r0 = r1;
  }
}

// Decimated spectra of the rows with plan e > 0 (full rows; M = N >> e, d = N / M):
//   W1[d n'], W2[d n'] = inverse M-point transforms of the filtered spectra's bins [0, M/2)
//     (the Morlet filter is negligible from bin M/2 on, and on the negative frequencies);
//   z = |W1|^2 + i |W2|^2 and w = W1 conj(W2) at those M samples, forward M-point transforms:
//     their spectra lie in (-M/2, M/2), so FFT_M(z[d n'])[k] = FFT_N(z)[k] / d exactly;
//   out: Y = FFT_M(w) / M (W12's spectrum, DY row) for phase A's W12 outputs, and the smoothed
//     Zs, Ys = F(k) FFT_M / (M s) (F the time Gaussian) to the band workspace SB (rows phase C
//     reads) and / or, for time-path rows, in FFT order into the row's TA / TB slots.
// Replaces, per row, two of phase A's forward N-point transforms by M-point ones, and its
// inverse transforms by band inverses of M bins.  One 256-thread workgroup = 256 / (M/16)
// (pair, row) items of one M (grid-stride over the schedule of wct_plan_kernel).  One
// 512-thread workgroup = 256 / (M/16) items; an item is two thread groups of M/16 threads:
// group f transforms W_f, the two swap through LDS, group 0 forward-transforms z and group 1 w.
template <int LOGN, int LOGM>
__device__ __forceinline__ void dec_items(const CwtArgs& a, const cpx* __restrict__ spec, cpx* __restrict__ TA,
                                          cpx* __restrict__ TB, cpx* __restrict__ SB, cpx* __restrict__ DY,
                                          cpx* __restrict__ WB,
                                          const int* __restrict__ plan, const int* __restrict__ rows,
                                          const int* __restrict__ sched, int wl, cpx* lds) {
  using P = FftPlan<LOGN>;
  using PM = FftPlan<LOGM>;
  constexpr int ITEMS = dec_rows_per_wg(LOGM);
  static_assert(2 * ITEMS * PM::NT == 512, "decimated workgroup");
  constexpr int M = PM::N;
  constexpr int NTM = PM::NT;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // per item: nothing (twiddles) hoisted out of the caller's loop
  const int g = tid / NTM;  // thread group: item g / 2, field f = g & 1
  const int f = g & 1;
  const int t = tid - g * NTM;
  const int first = sched[4 * LOGM], nr = sched[4 * LOGM + 1];
  const long long item = static_cast<long long>(wl) * ITEMS + (g >> 1);
  const bool valid = item < a.batch * nr;
  const long long b = valid ? item / nr : 0;
  const int j = rows[first + (valid ? static_cast<int>(item - b * nr) : 0)];
  const int pl = plan[j];
  cpx* my = lds + g * PM::PADN;
  cpx tw[PM::NTW_ALLOC];
  fft_twiddles<LOGM>(tw, t);
  int par = 0;
  const double s = a.scales[j];
  const float f0 = static_cast<float>(a.f0);
  cpx v[16];
  {  // W_f at every d-th sample from bins t + m NTM (m < 8) of series f's spectrum
    const cpx prm = morlet_params(s, a.dt, P::N);
    const cpx* sp = spec + (2 * b + f) * static_cast<long long>(P::N);
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = m < 8 ? sp[t + m * NTM] : mkc(0.f, 0.f);
    morlet_filter_nz<LOGM, 8>(v, v, prm, f0, t);
    fft_row<LOGM, 1, 1, false, 0, 8>(v, my, 0, tw, t, par);
  }
  // swap W1 / W2 between the item's two groups (positions t + m NTM, natural order)
  __syncthreads();  // the transform's last reads of my are done
#pragma unroll
  for (int m = 0; m < 16; ++m) my[lpad(t + m * NTM)] = v[m];
  __syncthreads();
  {
    const cpx* other = lds + (g ^ 1) * PM::PADN;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const cpx o = other[lpad(t + m * NTM)];
      const cpx w1 = f == 0 ? v[m] : o, w2 = f == 0 ? o : v[m];
      v[m] = f == 0 ? mkc(cabs2(w1), cabs2(w2)) : cmul(w1, cconj(w2));  // z / w
    }
  }
  fft_row<LOGM, -1, 1, false>(v, my, 0, tw, t, par);
  const long long row = b * a.S + j;
  const int mr = P::N >> plan_dec(pl);  // the row's own M (<= M): bins |k| < mr/2 are stored
  auto keep = [&](int m, int& ix) {     // FFT-order index of this thread's bin m in the row's M
    const int k = t + (m < 8 ? m : m - 16) * NTM;
    ix = k & (mr - 1);
    return M == mr || (k >= -mr / 2 && k < mr / 2);
  };
  if (valid && f == 1) {  // W12's spectrum / M for phase A's W12 outputs
    cpx* dy = DY + row * (P::N / 2);
    constexpr float inv_m = 1.f / M;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      int ix;
      if (keep(m, ix)) st_c<64>(dy + ix, cscale(v[m], inv_m));
    }
  }
  // smoothed band: F(k) / (M s); time-path rows -> TA / TB slot in FFT order, band rows -> SB
  const double sn = s / a.dt * 2.0 * kPi / P::N;
  const float beta = static_cast<float>(-0.5 * 1.44269504088896340736 * sn * sn);
  const float sc = static_cast<float>(1.0 / (static_cast<double>(M) * s));
  constexpr int NTN = P::NT;  // SB row: bins k in [-NTN/2, NTN/2) at k + NTN/2
  const bool needT = valid && (pl & kPlanNeedT), needS = valid && (pl & kPlanNeedS);
  const bool needW = valid && (pl & kPlanNeedW);
  cpx* trow = (f == 0 ? TA : TB) + row * static_cast<long long>(a.n0);
  cpx* sb = SB + row * 2ll * NTN + f * NTN;
  cpx* wrow = WB + (row * 2 + f) * static_cast<long long>(P::N / 2) + P::N / 4;
  const int mw = P::N >> plan_ew(pl);  // <= the row's M: ew >= its decimation e
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int k = t + (m < 8 ? m : m - 16) * NTM;
    const float kk = static_cast<float>(k);
    const cpx y = cscale(v[m], sc * __builtin_amdgcn_exp2f(beta * kk * kk));
    int ix;
    if (needT && keep(m, ix)) st_c<64>(trow + ix, y);
    if (needS && k >= -NTN / 2 && k < NTN / 2) st_c<64>(sb + k + NTN / 2, y);
    if (needW) wb_put<64>(wrow, mw, k, y);
  }
  if constexpr (M < NTN) {  // band rows' SB bins outside (-M/2, M/2): zero, by the whole workgroup
    constexpr int Z = NTN - M;
    for (int i = tid; i < ITEMS * 2 * Z; i += 2 * ITEMS * NTM) {
      const int it = i / (2 * Z), rem = i - it * 2 * Z, ff = rem / Z, e = rem - ff * Z;
      const long long item2 = static_cast<long long>(wl) * ITEMS + it;
      if (item2 >= a.batch * nr) break;
      const long long b2 = item2 / nr;
      const int j2 = rows[first + static_cast<int>(item2 - b2 * nr)];
      if (plan[j2] & kPlanNeedS)
        SB[(b2 * a.S + j2) * 2ll * NTN + ff * NTN + (e < NTN / 2 - M / 2 ? e : e + M)] = mkc(0.f, 0.f);
    }
  }
}

constexpr long long kDecGrid = 2048;  // 4 workgroups of 512 per CU on 256 CUs, twice
// grid-stride from M = 2^9 on (up to 8 rows per item); the 16-row items of M = 256 keep one item
// per workgroup (their class grid is at most batch x S / 16, and the loop spilled 60 B per lane)
constexpr int kDecStrideLogm = 9;

// One launch per decimation class (the class sizes are known on the device only).  The grid is
// capped (kDecGrid) and strides over the class's workgroup items: a grid sized for the largest
// possible class (batch x S items at M = 4096) was mostly workgroups that read the schedule
// and exit.
template <int LOGN, int LOGM>
__global__ void __launch_bounds__(512, 4) wct_dec_kernel(CwtArgs a, const cpx* __restrict__ spec,
                                                         cpx* __restrict__ TA, cpx* __restrict__ TB,
                                                         cpx* __restrict__ SB, cpx* __restrict__ DY,
                                                         cpx* __restrict__ WB, const int* __restrict__ plan) {
  __shared__ cpx lds[2 * dec_rows_per_wg(LOGM) * FftPlan<LOGM>::PADN];
  const int* rows = plan + 3 * a.S + 1;
  const int* sched = rows + a.S;
  const int w0 = sched[4 * LOGM + 2];
  const int nwg = (LOGM > kDecEngLogm ? sched[4 * (LOGM - 1) + 2] : sched[64]) - w0;
  if constexpr (LOGM >= kDecStrideLogm) {
    for (int wl = blockIdx.x; wl < nwg; wl += gridDim.x) {
      if (wl != static_cast<int>(blockIdx.x)) __syncthreads();  // the previous item's LDS reads are done
      dec_items<LOGN, LOGM>(a, spec, TA, TB, SB, DY, WB, plan, rows, sched, wl, lds);
    }
  } else if (static_cast<int>(blockIdx.x) < nwg) {
    dec_items<LOGN, LOGM>(a, spec, TA, TB, SB, DY, WB, plan, rows, sched, blockIdx.x, lds);
  }
}


// The grid-stride classes (M = 2^12 .. 2^9) in ONE launch: the schedule numbers their
// workgroup items consecutively, largest M first, so a block striding over [0, w(M = 256))
// finds its class by comparing with the classes' first items.  Four launches' ramp and drain
// fewer on the decimated chain (a strong-scaling shard's kernels are short).  Every class has
// the same workgroup shape (512 threads) and LDS size (2 x 8448 complex).
template <int LOGN>
__global__ void __launch_bounds__(512, 4) wct_dec_merged(CwtArgs a, const cpx* __restrict__ spec,
                                                         cpx* __restrict__ TA, cpx* __restrict__ TB,
                                                         cpx* __restrict__ SB, cpx* __restrict__ DY,
                                                         cpx* __restrict__ WB, const int* __restrict__ plan) {
  constexpr int kTop = LOGN - dec_min_e<LOGN>() < kDecMaxLogm ? LOGN - dec_min_e<LOGN>() : kDecMaxLogm;
  __shared__ cpx lds[2 * dec_rows_per_wg(kDecMaxLogm) * FftPlan<kDecMaxLogm>::PADN];
  static_assert(dec_rows_per_wg(kDecStrideLogm) * FftPlan<kDecStrideLogm>::PADN <=
                    dec_rows_per_wg(kDecMaxLogm) * FftPlan<kDecMaxLogm>::PADN, "LDS of the merged classes");
  const int* rows = plan + 3 * a.S + 1;
  const int* sched = rows + a.S;
  const int end = sched[4 * (kDecStrideLogm - 1) + 2];  // first item of M = 256
  for (int wl = blockIdx.x; wl < end; wl += gridDim.x) {
    if (wl != static_cast<int>(blockIdx.x)) __syncthreads();  // the previous item's LDS reads are done
#define WTMI_DM(LM)                                                                         \
  if constexpr (LM <= kTop) {                                                               \
    if (wl < (LM > kDecStrideLogm ? sched[4 * (LM - 1) + 2] : end)) {                       \
      dec_items<LOGN, LM>(a, spec, TA, TB, SB, DY, WB, plan, rows, sched, wl - sched[4 * LM + 2], lds); \
      continue;                                                                             \
    }                                                                                       \
  }
    WTMI_DM(12) WTMI_DM(11) WTMI_DM(10) WTMI_DM(9)
#undef WTMI_DM
  }
}

template <int LOGN>
static int launch_dec_merged(const CwtArgs& a, const cpx* spec, cpx* TA, cpx* TB, cpx* SB, cpx* DY,
                             cpx* WB, const int* plan, hipStream_t st) {
  long long most = 0;  // the classes' workgroup items are at most this many
  for (int lm = kDecStrideLogm; lm <= kDecMaxLogm; ++lm)
    most += (a.batch * a.S + dec_rows_per_wg(lm) - 1) / dec_rows_per_wg(lm);
  const unsigned dg = static_cast<unsigned>(most < kDecGrid ? most : kDecGrid);
  hipLaunchKernelGGL((wct_dec_merged<LOGN>), dim3(dg), dim3(512), 0, st, a, spec, TA, TB, SB, DY, WB, plan);
  return launch_status();
}

template <int LOGN, int LOGM>
static int launch_dec_class(const CwtArgs& a, const cpx* spec, cpx* TA, cpx* TB, cpx* SB, cpx* DY,
                            cpx* WB, const int* plan, hipStream_t st) {
  if constexpr (LOGM >= kDecEngLogm && LOGM <= LOGN - dec_min_e<LOGN>()) {
    // the class's workgroup items are at most this many; the grid strides over them
    const long long most = (a.batch * a.S + dec_rows_per_wg(LOGM) - 1) / dec_rows_per_wg(LOGM);
    const long long cap = LOGM >= kDecStrideLogm ? kDecGrid : most;
    const unsigned dg = static_cast<unsigned>(most < cap ? most : cap);
    hipLaunchKernelGGL((wct_dec_kernel<LOGN, LOGM>), dim3(dg), dim3(512), 0, st, a, spec, TA, TB, SB, DY, WB,
                       plan);
    return launch_status();
  }
  return kOk;
}

// Scale boxcar + coherence.  Row i uses rows i - K/2 .. i + (K-1)/2 (zero outside),
// end weights 0.5; the normalisation 1/(K-1) cancels in |S12|^2 / (S1 S2) but is kept
// so the smoothed fields match the reference.  One thread = C adjacent time columns of
// one pair (C = 2: 16-byte loads of (T1, T2) and T12 for two columns -- the pass is a
// pure stream of the workspace); the last K rows of each column stay in registers.
template <int C> struct ColVec;
template <> struct ColVec<1> { using T = float2; using E = cpx; };
template <> struct ColVec<2> { using T = float4; using E = f32x4; };
template <int C>
__device__ __forceinline__ typename ColVec<C>::T ld_col(const typename ColVec<C>::T* p) {
  using V = typename ColVec<C>::T;
  if constexpr (wct_aux<32>() != 0)
    return __builtin_bit_cast(V, __builtin_nontemporal_load(reinterpret_cast<const typename ColVec<C>::E*>(p)));
  else
    return *p;
}

template <int K, int C, int DD = 0>
__global__ void __launch_bounds__(256) wct_phase_b(const cpx* __restrict__ TA, const cpx* __restrict__ TB,
                                                   long long batch, int n0, int S, float* __restrict__ coh,
                                                   const int* __restrict__ plan) {
  using V = typename ColVec<C>::T;
  constexpr int F = 2 * C;  // floats per V
  const int ncol = n0 / C;
  const long long tiles = (ncol + 255) / 256;
  const long long b = blockIdx.x / tiles;
  const int u = static_cast<int>((blockIdx.x - b * tiles) * 256 + threadIdx.x);
  if (u >= ncol) return;
  constexpr int LO = K / 2;        // rows before i
  constexpr int HI = (K - 1) / 2;  // rows after i
  const float wn = K > 1 ? 1.f / (K - 1) : 1.f;
  const V* cola = reinterpret_cast<const V*>(TA + b * static_cast<long long>(S) * n0) + u;
  const V* colb = reinterpret_cast<const V*>(TB + b * static_cast<long long>(S) * n0) + u;
  float* out = coh + b * static_cast<long long>(S) * n0 + static_cast<long long>(u) * C;
  const long long ldv = n0 / C;  // row stride in V
  float ra[K][F], rb[K][F];
#pragma unroll
  for (int r = 0; r < K; ++r)
#pragma unroll
    for (int f = 0; f < F; ++f) ra[r][f] = rb[r][f] = 0.f;
  // row j enters the ring at slot j % K; output row i = j - HI is complete then.  Rows
  // past the last time-path output (plan[S]) are phase C's: not read, not written.
  const int last = plan[S];
  if (last < 0) return;
  const int jend = last + HI + 1;  // output rows i = j - HI <= last
  const int jlim = min(S, jend);   // rows read
  // Rows are loaded D ahead of their use (D | K, so the pending slot of row jb + r is r % D):
  // D rows of loads in flight per thread instead of one (DD: forced depth, option wct_depth).
  constexpr int D = DD ? DD : (K % 6 == 0) ? 6 : (K % 5 == 0) ? 5 : (K % 4 == 0) ? 4 : (K % 3 == 0) ? 3 : (K % 2 == 0) ? 2 : 1;
  V pa[D], pc[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (d < jlim) {
      pa[d] = ld_col<C>(cola + static_cast<long long>(d) * ldv);
      pc[d] = ld_col<C>(colb + static_cast<long long>(d) * ldv);
    }
  }
  for (int jb = 0; jb < jend; jb += K) {
    int fl[K];  // the block's output-row plan flags, loaded up front (uniform scalar loads)
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int i = jb + r - HI;
      fl[r] = (i >= 0 && i < S) ? plan[i] : kPlanSpec;
    }
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int j = jb + r;
      const int slot = r % D;
      if (j < jlim) {
        const V a = pa[slot], c = pc[slot];
        const float* pap = reinterpret_cast<const float*>(&a);
        const float* pcp = reinterpret_cast<const float*>(&c);
#pragma unroll
        for (int f = 0; f < F; ++f) {
          ra[r][f] = pap[f];
          rb[r][f] = pcp[f];
        }
        const int jn = j + D;
        if (jn < jlim) {
          pa[slot] = ld_col<C>(cola + static_cast<long long>(jn) * ldv);
          pc[slot] = ld_col<C>(colb + static_cast<long long>(jn) * ldv);
        }
      } else {
#pragma unroll
        for (int f = 0; f < F; ++f) ra[r][f] = rb[r][f] = 0.f;
      }
      const int i = j - HI;
      if (i >= 0 && i < S && !(fl[r] & kPlanSpec)) {
        float acc[2][F] = {};
#pragma unroll
        for (int q = 0; q < K; ++q) {
          // slot of row i - LO + q  (rows i-LO .. i+HI = j-K+1 .. j)
          const int slot = (r + 1 + q) % K;
          const float wq = (K > 1 && (q == 0 || q == K - 1)) ? 0.5f * wn : wn;
          if (i - LO + q >= 0) {
#pragma unroll
            for (int f = 0; f < F; ++f) {
              acc[0][f] = fmaf(wq, ra[slot][f], acc[0][f]);
              acc[1][f] = fmaf(wq, rb[slot][f], acc[1][f]);
            }
          }
        }
        float o[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const float s1 = acc[0][2 * c], s2 = acc[0][2 * c + 1];
          const float re = acc[1][2 * c], im = acc[1][2 * c + 1];
          o[c] = fast_div(re * re + im * im, s1 * s2);
        }
        float* orow = out + static_cast<long long>(i) * n0;
        if constexpr (C == 2)
          *reinterpret_cast<float2*>(orow) = make_float2(o[0], o[1]);
        else if constexpr (wct_aux<8>() != 0)
          __builtin_nontemporal_store(o[0], orow);
        else
          orow[0] = o[0];
      }
    }
  }
}

// Phase C: coherence of the output rows whose whole boxcar window consists of band rows
// (plan bit kPlanSpec).  The scale boxcar is linear, so it is applied to the stored band
// spectra of the window's rows, and the two sums go through the pruned inverse transform of
// the window's union band (regime qw):
//   S1 + i S2 = IFFT(sum_q w_q Z_q),   S12 = IFFT(sum_q w_q W_q),   WCT = |S12|^2 / (S1 S2).
// These rows skip the time-domain workspace (16 B per coefficient written by phase A and
// read back by phase B) and phase A's smoothing transforms move here.
// EC (r04, plan bits ec): the window's rows have their smoothed spectra in [-Mc/2, Mc/2), Mc =
// N >> EC, so the sums are exchanged shifted by Mc/2 (not by the regime band's half width) and
// the inverse transforms enter at pass EC / 4 with 16 >> (EC % 4) non-zero inputs per thread
// (BandGeom, as the decimated rows' band inverses); the shift's time phasor has H = Mc/2.
template <int LOGN, int EC>
__host__ __device__ constexpr bool spec_ec_ok() {
  using P = FftPlan<LOGN>;
  return EC >= 4 && EC <= LOGN - 5 && EC / 4 < P::P16 && (P::NT % (1 << (4 * (EC / 4)))) == 0 &&
         (P::N >> EC) >= 32;
}

// Smoothed row from the window sum of its band bin: band exchange of Mc = N >> EC shifted bins,
// inverse FFT from pass EC / 4 over the NZ non-zero inputs, time phasor exp(-2 pi i (Mc/2) n / N).
template <int LOGN, int EC, bool TWL, bool PHASOR = true>
__device__ __forceinline__ void smooth_from_band_ec(cpx (&v)[16], cpx y, int slot, cpx* my, const cpx* tw,
                                                    int t, int& par, const float4* twl) {
  using P = FftPlan<LOGN>;
  using BG = BandGeom<LOGN, EC>;
  constexpr int STEP = P::NT >> (4 * BG::Q);
  __syncthreads();
  if (slot >= 0) my[slot] = y;
  __syncthreads();
  const int base = t >> (4 * BG::Q);
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = r < BG::NZ ? my[base + r * STEP] : mkc(0.f, 0.f);
  fft_row<LOGN, 1, 1, TWL, BG::Q, BG::NZ>(v, my, 0, tw, t, par, twl);
  if constexpr (PHASOR) {
    int tt = t;
    asm volatile("" : "+v"(tt));  // per row, not hoisted (register budget)
    const cpx ph = expi_frac(-BG::H * tt, P::N);
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = cmul2(v[m], ph);
  }
}

template <int LOGN, int EC, bool BUF, bool TWL, bool FULL>
__device__ __forceinline__ void wct_spec_rows(const CwtArgs& a, const cpx* __restrict__ SB, int K,
                                              long long b, int j0, int r0, int r1, cpx* my, const cpx* tw,
                                              int g, int t, int& par, const float4* twl,
                                              float* __restrict__ coh) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  constexpr int K0 = BandGeom<LOGN, EC>::H;  // the window's half band: bins [-K0, K0)
  const int LO = K / 2;
  for (int r = r0; r < r1; r += G::ROWS) {
    const int jl = r + g;
    const bool valid = jl < r1;
    const int i = j0 + (valid ? jl : r0);
    int tt = t;
    asm volatile("" : "+v"(tt));  // per-row index math, not hoisted (register budget)
    const int k = tt - P::NT / 2;  // band-workspace index t <-> bin k
    const bool holder = k >= -K0 && k < K0;
    float wn = K > 1 ? 1.f / (K - 1) : 1.f;
    asm volatile("" : "+v"(wn));  // the window weights per row: hoisted, they spilled (prologue scratch)
    cpx yz = mkc(0.f, 0.f), yw = mkc(0.f, 0.f);
    if (holder) {
      // window rows in groups of U with every load of a group issued before its first
      // use (one memory latency per group, not per row); rows outside [0, S) get weight 0
      constexpr int U = 4;
      const cpx* sbb = SB + b * a.S * 2ll * P::NT + tt;
      for (int q0 = 0; q0 < K; q0 += U) {
        cpx lz[U], lw[U];
        float wq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int q = q0 + u;
          const int rr = i - LO + q;
          const bool ok = q < K && rr >= 0 && rr < a.S;
          wq[u] = ok ? ((K > 1 && (q == 0 || q == K - 1)) ? 0.5f * wn : wn) : 0.f;
          const cpx* sb = sbb + (ok ? rr : i) * 2ll * P::NT;
          lz[u] = ld_c<256>(sb);
          lw[u] = ld_c<256>(sb + P::NT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          yz = cfma(cpx{wq[u], wq[u]}, lz[u], yz);
          yw = cfma(cpx{wq[u], wq[u]}, lw[u], yw);
        }
      }
    }
    const int slot = holder ? k + K0 : -1;
    // S1 S2 first (16 floats stay live, not 16 complex); |S12|^2 needs no phasor
    cpx v[16];
    float den[16];
    smooth_from_band_ec<LOGN, EC, TWL>(v, yz, slot, my, tw, t, par, twl);
#pragma unroll
    for (int m = 0; m < 16; ++m) den[m] = v[m].x * v[m].y;
    smooth_from_band_ec<LOGN, EC, TWL, false>(v, yw, slot, my, tw, t, par, twl);
    if (valid) {
      const long long rowbase = (b * a.S + i) * static_cast<long long>(a.n0);
      put_row<LOGN, BUF, FULL, wct_aux<1>()>(coh + rowbase, t, a.n0, [&](int m) { return fast_div(cabs2(v[m]), den[m]); });
    }
  }
}

// Scale boxcar of the wide windows in the spectral domain (plan bits eu).  One thread = one bin
// k in [-N/4, N/4) of one pair; it streams the rows of the wide windows down the scale axis
// with the last K rows' (Z, W) bins in registers (a row contributes where its band [-Mw/2, Mw/2)
// covers k) and, once output row i's window is complete, writes the window sums over row i's
// own WB slot (bin k, in place: only this thread reads or writes index k, and row i's own bins
// were read before).  Rows outside [0, S) and bins past a row's band count as zero.
template <int K, int DD = 0>
__global__ void __launch_bounds__(256) wct_wide_boxcar(cpx* __restrict__ WB, long long batch, int N, int S,
                                                       const int* __restrict__ plan) {
  const int nb = N / 2;  // bins per slot
  const long long tiles = (nb + 255) / 256;
  const long long b = blockIdx.x / tiles;
  const int u = static_cast<int>((blockIdx.x - b * tiles) * 256 + threadIdx.x);
  if (u >= nb) return;
  const int k = u - N / 4;
  const int* rng = plan + 4 * S + 1 + kSchedWide;  // first / last wide output row (wct_plan_kernel)
  const int i0 = rng[0], i1 = rng[1];
  if (i0 > i1) return;
  constexpr int LO = K / 2, HI = (K - 1) / 2;
  const float wn = K > 1 ? 1.f / (K - 1) : 1.f;
  cpx* base = WB + b * S * 2ll * nb + u;  // row r field f at base + (2 r + f) nb
  const int jlo = max(0, i0 - LO), jhi = min(S - 1, i1 + HI);
  auto load = [&](int j, cpx& z, cpx& w) {  // row j's bins (zero past its band or the rows used)
    z = w = mkc(0.f, 0.f);
    if (j <= jhi) {
      const int mw = N >> plan_ew(plan[j]);
      if (k >= -(mw >> 1) && k < (mw >> 1)) {
        z = ld_c<128>(base + (2ll * j) * nb);
        w = ld_c<128>(base + (2ll * j + 1) * nb);
      }
    }
  };
  // rows are loaded D ahead of their use (D | K: the pending slot of row jb + q is q % D), so D
  // rows of loads are in flight per thread; the sums' stores follow the loads they overtake
  constexpr int D = DD ? DD : (K % 6 == 0) ? 6 : (K % 5 == 0) ? 5 : (K % 4 == 0) ? 4 : (K % 3 == 0) ? 3 : (K % 2 == 0) ? 2 : 1;
  cpx pz[D], pw[D];
#pragma unroll
  for (int d = 0; d < D; ++d) load(jlo + d, pz[d], pw[d]);
  cpx rz[K], rw[K];
#pragma unroll
  for (int q = 0; q < K; ++q) rz[q] = rw[q] = mkc(0.f, 0.f);
  // slot of row j: (j - jlo) % K; rows are taken K at a time so the slots index statically
  for (int jb = jlo; jb <= jhi + HI; jb += K) {
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const int j = jb + q;
      rz[q] = pz[q % D];
      rw[q] = pw[q % D];
      load(j + D, pz[q % D], pw[q % D]);
      const int i = j - HI;  // its window [i - LO, i + HI] = rows j - K + 1 .. j
      if (i >= i0 && i <= i1) {
        const int pl = plan[i];
        const int mu = N >> plan_eu(pl);
        if (plan_eu(pl) && k >= -(mu >> 1) && k < (mu >> 1)) {
          cpx sz = mkc(0.f, 0.f), sw = sz;
#pragma unroll
          for (int qq = 0; qq < K; ++qq) {  // row i - LO + qq sits in slot (q + 1 + qq) % K
            const int slot = (q + 1 + qq) % K;
            const float wq = (K > 1 && (qq == 0 || qq == K - 1)) ? 0.5f * wn : wn;
            if (i - LO + qq >= jlo) {
              sz = cfma(cpx{wq, wq}, rz[slot], sz);
              sw = cfma(cpx{wq, wq}, rw[slot], sw);
            }
          }
          st_c<128>(base + (2ll * i) * nb, sz);
          st_c<128>(base + (2ll * i + 1) * nb, sw);
        }
      }
    }
  }
}

// Wide output rows (plan bits eu): the window sums of wct_wide_boxcar in the row's WB slot go
// through one band inverse of Mu = N >> EU bins per field (shifted by H = Mu/2, entry pass
// narrowed to NZ = 16 >> EU inputs) -- S1 + i S2 and S12 at every sample -- and WCT is written.
// Replaces, for these rows, phase A's two inverse smoothing transforms per row, the 16-byte
// time-domain workspace write and phase B's read of it.
template <int LOGN, int EU, bool BUF, bool TWL, bool FULL>
__device__ __forceinline__ void wct_wide_rows(const CwtArgs& a, const cpx* __restrict__ WB, long long b,
                                              int j0, int r0, int r1, cpx* my, const cpx* tw, int g, int t,
                                              int& par, const float4* twl, float* __restrict__ coh) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  using BG = BandGeom<LOGN, EU>;
  static_assert(BG::Q == 0, "wide windows enter at pass 0");
  for (int r = r0; r < r1; r += G::ROWS) {
    const int jl = r + g;
    const bool valid = jl < r1;
    const int i = j0 + (valid ? jl : r0);
    const cpx* zrow = WB + ((b * a.S + i) * 2) * static_cast<long long>(P::N / 2) + (P::N / 4 - BG::H);
    cpx pre[8];
    cpx v[16];
    float den[16];
#pragma unroll
    for (int q = 0; q < BG::NZ; ++q) pre[q] = ld_c<256>(zrow + t + q * P::NT);  // shifted bin p -> k = p - H
    band_ifft<LOGN, EU, TWL>(v, pre, my, tw, t, par, twl);
#pragma unroll
    for (int m = 0; m < 16; ++m) den[m] = v[m].x * v[m].y;  // S1 S2
#pragma unroll
    for (int q = 0; q < BG::NZ; ++q) pre[q] = ld_c<256>(zrow + P::N / 2 + t + q * P::NT);
    band_ifft<LOGN, EU, TWL>(v, pre, my, tw, t, par, twl);
    if (valid) {
      const long long rowbase = (b * a.S + i) * static_cast<long long>(a.n0);
      put_row<LOGN, BUF, FULL, wct_aux<1>()>(coh + rowbase, t, a.n0, [&](int m) { return fast_div(cabs2(v[m]), den[m]); });
    }
  }
}

// WIDE: this launch runs the wide output rows only, else the q-window rows (two launches over
// the same chunk grid, so that each path gets the register budget of its own kernel: together
// they spilled 52 bytes per lane, the q rows alone 16).
template <int LOGN, bool FULL, bool WIDE>
__global__ void __launch_bounds__((WctGeom<LOGN>::BLOCK), (WctGeom<LOGN>::MINW))
    wct_phase_c(CwtArgs a, const cpx* __restrict__ SB, const cpx* __restrict__ WB, const int* __restrict__ plan,
                int K, float* __restrict__ coh) {
  using P = FftPlan<LOGN>;
  using G = WctGeom<LOGN>;
  constexpr bool BUF = P::NT >= kWave;  // padded rows too: put_row's extent
  __shared__ float4 lds4[(G::ROWS * P::PADN) / 2 + G::TWL_F4];
  cpx* lds = reinterpret_cast<cpx*>(lds4);
  float4* twl = lds4 + (G::ROWS * P::PADN) / 2;
  const int tid = threadIdx.x;
  const int g = tid / P::NT;
  const int t = fft_thread<LOGN>(tid - g * P::NT);
  const long long blk = xcd_remap(blockIdx.x, gridDim.x);
  const long long b = blk / a.nchunks;
  const int ch = static_cast<int>(blk - b * a.nchunks);
  const int j0 = ch * a.chunk;
  const int j1 = min(a.S, j0 + a.chunk);
  // any rows of this launch's kind here?  (uniform: every thread reads the same plan entries)
  bool any = false;
  for (int r = j0; r < j1; ++r) any |= (plan[r] & kPlanSpec) != 0 && (plan_eu(plan[r]) != 0) == WIDE;
  if (!any) return;
  cpx* my = lds + g * P::PADN;
  constexpr bool TWL = G::TWL;
  cpx tw[TWL ? P::NTW_REG : P::NTW_ALLOC];
  if constexpr (TWL) {
    fft_twiddle_table<LOGN>(twl, tid, G::BLOCK);
    fft_twiddles_tail<LOGN>(tw, t);
  } else {
    fft_twiddles<LOGN>(tw, t);
  }
  int par = 0;
  __syncthreads();
  const int nrow = j1 - j0;
  auto key = [&](int r) {  // 16 + ec: q windows; 4 + eu: wide windows; 0: not phase C's
    const int pl = plan[j0 + r];
    if (!(pl & kPlanSpec)) return 0;
    return plan_eu(pl) ? 4 + plan_eu(pl) : 16 + plan_ec(pl);
  };
  int r0 = 0;
  while (r0 < nrow) {
    const int q = key(r0);
    int r1 = r0 + 1;
    while (r1 < nrow && key(r1) == q) ++r1;
    if constexpr (!WIDE) {
#define WTMI_SC(EC)                                                                         \
  if constexpr (spec_ec_ok<LOGN, EC>()) {                                                   \
    if (q == 16 + EC)                                                                       \
      wct_spec_rows<LOGN, EC, BUF, TWL, FULL>(a, SB, K, b, j0, r0, r1, my, tw, g, t, par, twl, coh); \
  }
      WTMI_SC(4) WTMI_SC(5) WTMI_SC(6) WTMI_SC(7) WTMI_SC(8) WTMI_SC(9)
#undef WTMI_SC
    }
    if constexpr (WIDE && LOGN >= kWideMinLogn) {
      if (q == 5) wct_wide_rows<LOGN, 1, BUF, TWL, FULL>(a, WB, b, j0, r0, r1, my, tw, g, t, par, twl, coh);
      if (q == 6) wct_wide_rows<LOGN, 2, BUF, TWL, FULL>(a, WB, b, j0, r0, r1, my, tw, g, t, par, twl, coh);
      if (q == 7) wct_wide_rows<LOGN, 3, BUF, TWL, FULL>(a, WB, b, j0, r0, r1, my, tw, g, t, par, twl, coh);
    }
    r0 = r1;
  }
}

// Rows per workgroup when the options leave them at 0 (auto): shorter workgroups for small
// batches (one GPU's share of a strong-scaling run), so the grids still fill the CUs.  C4 rows
// at 64 / 128 / 256 / 512 pairs, one box (ms, 4+4 rows -> this rule): 0.675 -> 0.600,
// 1.075 -> 1.023, 1.914 -> 1.894, 3.54 unchanged.  r03 sweep with the decimated rows' chunks
// (wct_dec_rows; one box, two alternations, ms): 64 pairs (min 1, dec 2) 0.524-0.549 -> (1, 4)
// 0.516-0.520 or (1, 8) 0.519-0.521; 128 (1, 2) 0.959-0.962 -> (2, 8) 0.924-0.927; 256 (2, 2)
// 1.729-1.730 -> (2, 8) 1.694-1.697; 512 (4, 4) 3.227-3.236, (4, 8) 3.253-3.262, (2, 8) 3.34-3.38.
// r04 re-sweep after the merged decimation launch and phase C's third stream (one box,
// alternating in one process, ms for min rows 1 / 2 / 3 / 4): 64 pairs 0.458 / 0.450 / 0.449 /
// 0.449, 128 pairs 0.870 / 0.826 / 0.818 / 0.802, 256 pairs 1.656 / 1.635 / 1.637 / 1.562, 512
// pairs 3.235 / 3.132 / 3.106 / 3.073: four rows per workgroup from 64 pairs on.  A handful of
// pairs (the app's single-pair calls) keeps one row per workgroup: there the grid is a few
// dozen workgroups and the step is as long as one workgroup's rows.
static int wct_min_rows(long long batch) {
  const int o = options().wct_min_rows;
  return o > 0 ? o : (batch <= 32 ? 1 : 4);
}
static int wct_dec_rows_per_wg(long long batch) {
  const int o = options().wct_dec_rows;
  // 64 pairs (r04, alternating): 8 rows 0.492 ms, 6 0.487, 4 0.486, 3 0.487, 2 0.489
  return o > 0 ? o : (batch <= 64 ? 4 : batch <= 256 ? 8 : 4);
}

// Side streams for the full-band rows' kernel beside the decimated rows' chain (fork after the
// plan, join before the caller's stream proceeds).  A small batch (one GPU's shard of a
// strong-scaling run) leaves CUs idle in each kernel; two independent kernels in flight fill
// them.  One pool entry (two streams + five events) per concurrent caller, from a per-device
// pool (the second stream carries phase C's q windows for small batches): a call
// takes one (or creates one when all are in use) and hands it back after its last enqueue, so
// the pool holds as many as calls ever overlapped, however many host threads come and go (a
// thread_local stream per thread leaked one per short-lived thread: a Streamlit rerun runs on a
// fresh ScriptRunner thread).  Reuse is safe: hipStreamWaitEvent waits on the event's record
// at the time of the call, and the next owner's work follows on the same side stream.
struct SideStream {
  hipStream_t s = nullptr, s2 = nullptr;
  // fork: spectra + plan done (main); k0: full-band rows done (side); dec: decimated spectra
  // done (main); join / join2: the side streams' last kernels done
  hipEvent_t fork = nullptr, k0 = nullptr, dec = nullptr, join = nullptr, join2 = nullptr;
};
namespace {
constexpr int kMaxDev = 64;
struct SidePool {
  std::mutex mu;
  std::vector<SideStream*> idle[kMaxDev];
  std::atomic<long long> created{0};
};
// Never destroyed: the streams live as long as the process (the HIP runtime tears itself down
// at exit; destroying streams from a static destructor after that is undefined).
SidePool& side_pool() {
  static SidePool* p = new SidePool;
  return *p;
}
SideStream* side_acquire(int& dev) {
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  SidePool& pool = side_pool();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    if (!pool.idle[dev].empty()) {
      SideStream* ss = pool.idle[dev].back();
      pool.idle[dev].pop_back();
      return ss;
    }
  }
  SideStream* ss = new SideStream;
  bool ok = hipStreamCreateWithFlags(&ss->s, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&ss->s2, hipStreamNonBlocking) == hipSuccess;
  for (hipEvent_t* e : {&ss->fork, &ss->k0, &ss->dec, &ss->join, &ss->join2})
    ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    for (hipEvent_t e : {ss->fork, ss->k0, ss->dec, ss->join, ss->join2})
      if (e) (void)hipEventDestroy(e);
    if (ss->s) (void)hipStreamDestroy(ss->s);
    if (ss->s2) (void)hipStreamDestroy(ss->s2);
    delete ss;
    (void)hipGetLastError();
    return nullptr;  // the call runs single-stream
  }
  pool.created.fetch_add(1);
  return ss;
}
void side_release(SideStream* ss, int dev) {
  SidePool& pool = side_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  pool.idle[dev].push_back(ss);
}
}  // namespace

// Owns a call's side streams: on every return after a fork -- success or a failed launch /
// event call -- each forked side stream records its join event and the caller's stream waits
// on it before the entry goes back to the pool, so no side-stream kernel can still be writing
// the workspace or the outputs once the caller's stream is past the call.
struct SideJoin {
  SideStream* side = nullptr;
  hipStream_t st = nullptr;
  int dev = 0;
  bool forked = false, forked2 = false;
  SideJoin(bool want, hipStream_t caller) : st(caller) {
    if (want) side = side_acquire(dev);
  }
  ~SideJoin() {
    if (!side) return;
    if (forked) {
      (void)hipEventRecord(side->join, side->s);
      (void)hipStreamWaitEvent(st, side->join, 0);
    }
    if (forked2) {
      (void)hipEventRecord(side->join2, side->s2);
      (void)hipStreamWaitEvent(st, side->join2, 0);
    }
    side_release(side, dev);
  }
  SideJoin(const SideJoin&) = delete;
  SideJoin& operator=(const SideJoin&) = delete;
};

template <int LOGN>
static int launch_phase_a(CwtArgs& a, cpx* spec, cpx* TA, cpx* TB, cpx* SB, cpx* DY, cpx* WB, int* plan,
                          int K, float* coh, hipStream_t st, SideJoin& sj) {
  SideStream* side = sj.side;
  using G = WctGeom<LOGN>;
  const long long sgrid = (2 * a.batch + G::ROWS - 1) / G::ROWS;  // spectra workgroups
  if (sgrid + 1 > 0x7fffffffll) return kErrUnsupported;
  const int rows = G::ROWS;
  // Row costs differ a lot (full-band rows several transforms, band rows few): more,
  // shorter workgroups balance better.  C4 ms (one box, two alternations): target 2048
  // 5.10, 4096 4.53-4.58, 8192 4.11-4.23, 12800 (= 4 rows each) 4.08-4.11; 4 rows each
  // 3.95-4.09 vs 3 rows 4.01-4.09, 2 rows 4.03-4.13.  Default: 4-row workgroups.
  const long long target = options().wct_target_wg > 0 ? options().wct_target_wg : (1ll << 30);
  long long want = (target + a.batch - 1) / a.batch;
  const int min_rows = wct_min_rows(a.batch);  // rows per workgroup, at least
  const int max_chunks = (a.S + min_rows * rows - 1) / (min_rows * rows);
  int nch = static_cast<int>(want < 1 ? 1 : want);
  if (nch > max_chunks) nch = max_chunks < 1 ? 1 : max_chunks;
  int chunk = (a.S + nch - 1) / nch;
  chunk = ((chunk + rows - 1) / rows) * rows;
  if (chunk > G::MAXCHUNK) chunk = G::MAXCHUNK;
  nch = (a.S + chunk - 1) / chunk;
  a.nchunks = nch;
  a.chunk = chunk;
  a.prune = options().wct_prune;
  const long long grid = a.batch * nch;
  if (grid > 0x7fffffffll || a.batch * a.S > 0x7fffffffll - 64) return kErrUnsupported;
  // decimated rows: full rows, pruning level 2, Morlet negative frequencies negligible
  const int dec = (a.prune >= 2 && a.n0 == (1 << LOGN) && LOGN >= kDecMinLogn && a.f0 >= kBandF0) ? 1 : 0;
  hipLaunchKernelGGL(wct_spectra_plan<LOGN>, dim3(static_cast<unsigned>(sgrid + 1)), dim3(G::BLOCK), 0, st, a,
                     spec, K, dec, options().wct_wide, plan);
  int rc = launch_status();
  if (rc != kOk) return rc;
  const dim3 gd(static_cast<unsigned>(grid));
  if (a.n0 != (1 << LOGN)) {
    hipLaunchKernelGGL((wct_phase_a<LOGN, false, 0>), gd, dim3(G::BLOCK), 0, st, a, spec, TA, TB, SB, DY, WB,
                       plan);
    if ((rc = launch_status()) != kOk) return rc;
    if (a.prune) {  // band rows exist only with pruning
      hipLaunchKernelGGL((wct_phase_a<LOGN, false, 1>), gd, dim3(G::BLOCK), 0, st, a, spec, TA, TB, SB, DY, WB,
                         plan);
      rc = launch_status();
    }
    return rc;
  }
  // Full rows: the full-band rows' kernel -- on the side stream when the caller passes one (the
  // caller joins it) -- then the decimated rows' spectra and their kernel.
  hipStream_t sa = st;
  if (side) {
    if (hipEventRecord(side->fork, st) != hipSuccess) return launch_status();
    sj.forked = true;
    if (hipStreamWaitEvent(side->s, side->fork, 0) != hipSuccess) return launch_status();
    sa = side->s;
  }
  // (the full-band rows in chunks of their own, 1 or 2 rows at 64 / 128 pairs, measured slower
  // than the common 4: r04, profiles/r04/c4_shard_policy.txt)
  hipLaunchKernelGGL((wct_phase_a<LOGN, true, 0>), gd, dim3(G::BLOCK), 0, sa, a, spec, TA, TB, SB, DY, WB,
                     plan);
  if ((rc = launch_status()) != kOk) return rc;
  if (side && hipEventRecord(side->k0, side->s) != hipSuccess) return launch_status();
  // band rows that are not decimated: none when the decimation is on (a row of regime >= 1 has
  // its CWT band within N/16, hence a decimation M <= N/8), so that launch is skipped then
  if (a.prune && !dec) {
    hipLaunchKernelGGL((wct_phase_a<LOGN, true, 1>), gd, dim3(G::BLOCK), 0, st, a, spec, TA, TB, SB, DY, WB,
                       plan);
    if ((rc = launch_status()) != kOk) return rc;
  }
  if constexpr (LOGN >= kDecMinLogn) {
    if (dec) {
      // one launch for the grid-stride classes: A/B (alternating, one box, r04) 64 pairs
      // 0.492 -> 0.459 ms, 128 pairs 0.846 -> 0.821, 512 pairs 3.11 -> 3.20, so by default (2)
      // for batches of at most 256 pairs
      const int dm = options().wct_dec_merge;
      const bool merged = dm == 1 || (dm == 2 && a.batch <= 256);
      if (merged) {
        if ((rc = launch_dec_merged<LOGN>(a, spec, TA, TB, SB, DY, WB, plan, st)) != kOk) return rc;
        if ((rc = launch_dec_class<LOGN, kDecEngLogm>(a, spec, TA, TB, SB, DY, WB, plan, st)) != kOk) return rc;
      }
      for (int lm = kDecMaxLogm; lm >= kDecEngLogm && !merged; --lm) {
        switch (lm) {
#define WTMI_DC(LM) case LM: rc = launch_dec_class<LOGN, LM>(a, spec, TA, TB, SB, DY, WB, plan, st); break;
          WTMI_DC(12) WTMI_DC(11) WTMI_DC(10) WTMI_DC(9) WTMI_DC(8)
#undef WTMI_DC
          default: break;
        }
        if (rc != kOk) return rc;
      }
      if (side && hipEventRecord(side->dec, st) != hipSuccess) return launch_status();
      // decimated rows cost one to three band inverses each: chunks of their own length
      CwtArgs ad = a;
      ad.chunk = ((wct_dec_rows_per_wg(a.batch) + rows - 1) / rows) * rows;
      if (ad.chunk > G::MAXCHUNK) ad.chunk = G::MAXCHUNK;
      ad.nchunks = (a.S + ad.chunk - 1) / ad.chunk;
      hipLaunchKernelGGL((wct_phase_a<LOGN, true, 2>), dim3(static_cast<unsigned>(a.batch * ad.nchunks)),
                         dim3(G::BLOCK), 0, st, ad, spec, TA, TB, SB, DY, WB, plan);
      return launch_status();
    }
  }
  return kOk;
}

// Phase C over the chunk grid phase A used (a.nchunks / a.chunk as launch_phase_a set them).
template <int LOGN>
// which: 1 the q windows, 2 the wide windows, 3 both (in that order).
static int launch_phase_c(const CwtArgs& a, const cpx* SB, const cpx* WB, const int* plan, int K, float* coh,
                          hipStream_t st, int which = 3) {
  using G = WctGeom<LOGN>;
  const dim3 gd(static_cast<unsigned>(a.batch * a.nchunks));
  int rc = kOk;
  if (which & 1) {
    if (a.n0 == (1 << LOGN))
      hipLaunchKernelGGL((wct_phase_c<LOGN, true, false>), gd, dim3(G::BLOCK), 0, st, a, SB, WB, plan, K, coh);
    else
      hipLaunchKernelGGL((wct_phase_c<LOGN, false, false>), gd, dim3(G::BLOCK), 0, st, a, SB, WB, plan, K, coh);
    rc = launch_status();
  }
  if (!(which & 2) || rc != kOk || LOGN < kWideMinLogn || a.prune < 1 || options().wct_wide < 1 ||
      K > kWideMaxK)
    return rc;
  if (a.n0 == (1 << LOGN))
    hipLaunchKernelGGL((wct_phase_c<LOGN, true, true>), gd, dim3(G::BLOCK), 0, st, a, SB, WB, plan, K, coh);
  else
    hipLaunchKernelGGL((wct_phase_c<LOGN, false, true>), gd, dim3(G::BLOCK), 0, st, a, SB, WB, plan, K, coh);
  return launch_status();
}

template <int K>
static int launch_phase_b(const cpx* TA, const cpx* TB, long long batch, int n0, int S, float* coh,
                          const int* plan, hipStream_t st) {
  // one column per thread (16-byte column pairs measured slower: fewer loads in flight,
  // C4 4.65 vs 4.73 ms in r01)
  const long long tiles = (static_cast<long long>(n0) + 255) / 256;
  const long long grid = batch * tiles;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  if (K <= 12 && options().wct_depth == 1)
    hipLaunchKernelGGL((wct_phase_b<K, 1, (K <= 12 ? K : 0)>), dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, TA, TB,
                       batch, n0, S, coh, plan);
  else
    hipLaunchKernelGGL((wct_phase_b<K, 1>), dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, TA, TB,
                       batch, n0, S, coh, plan);
  return launch_status();
}

// Phase B for any boxcar width (K > 24, where the register ring of wct_phase_b would not
// fit): each output row sums its K window rows straight from the workspace (K loads per
// output instead of one) -- the same weights and the same rows.
__global__ void __launch_bounds__(256) wct_phase_b_generic(const cpx* __restrict__ TA,
                                                           const cpx* __restrict__ TB, long long batch,
                                                           int n0, int S, int K, float* __restrict__ coh,
                                                           const int* __restrict__ plan) {
  const long long tiles = (n0 + 255) / 256;
  const long long b = blockIdx.x / tiles;
  const int u = static_cast<int>((blockIdx.x - b * tiles) * 256 + threadIdx.x);
  if (u >= n0) return;
  const int LO = K / 2;
  const float wn = K > 1 ? 1.f / (K - 1) : 1.f;
  const long long base = b * static_cast<long long>(S) * n0 + u;
  const int last = plan[S];
  for (int i = 0; i <= last && i < S; ++i) {
    if (plan[i] & kPlanSpec) continue;
    float s1 = 0.f, s2 = 0.f, re = 0.f, im = 0.f;
    for (int q = 0; q < K; ++q) {
      const int row = i - LO + q;
      if (row < 0 || row >= S) continue;
      const float wq = (K > 1 && (q == 0 || q == K - 1)) ? 0.5f * wn : wn;
      const cpx ta = TA[base + static_cast<long long>(row) * n0];
      const cpx tb = TB[base + static_cast<long long>(row) * n0];
      s1 = fmaf(wq, ta.x, s1);
      s2 = fmaf(wq, ta.y, s2);
      re = fmaf(wq, tb.x, re);
      im = fmaf(wq, tb.y, im);
    }
    coh[base + static_cast<long long>(i) * n0] = fast_div(re * re + im * im, s1 * s2);
  }
}

int wct_phase_b_any(const cpx* TA, const cpx* TB, long long batch, int n0, int S, float* coh,
                    const int* plan, int K, hipStream_t st) {
  switch (K) {
#define WTMI_B(KK) case KK: return launch_phase_b<KK>(TA, TB, batch, n0, S, coh, plan, st);
    WTMI_B(1) WTMI_B(2) WTMI_B(3) WTMI_B(4) WTMI_B(5) WTMI_B(6) WTMI_B(7) WTMI_B(8)
    WTMI_B(9) WTMI_B(10) WTMI_B(11) WTMI_B(12) WTMI_B(13) WTMI_B(14) WTMI_B(15) WTMI_B(16)
    WTMI_B(17) WTMI_B(18) WTMI_B(19) WTMI_B(20) WTMI_B(21) WTMI_B(22) WTMI_B(23) WTMI_B(24)
#undef WTMI_B
    default: break;
  }
  if (K < 1) return kErrArg;
  const long long grid = batch * ((n0 + 255) / 256);
  if (grid > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL(wct_phase_b_generic, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, TA, TB, batch,
                     n0, S, K, coh, plan);
  return launch_status();
}

// Rows of at most 8 samples (N <= 8, below the FFT engine's 16-point minimum): the whole
// pycwt.wct of one pair in one workgroup by direct DFTs in fp64 -- two CWTs, the time
// Gaussian of |W1|^2/s, |W2|^2/s, W12/s through length-N DFTs, then the scale boxcar and
// the ratio (src/wct.py:106-118 at n0 <= 8).  Smoothed rows sit in LDS ([S][n0] x 4 floats).
constexpr size_t kWctDirectMaxLds = 150 * 1024;  // S * n0 <= 9600 smoothed points

__global__ void __launch_bounds__(256) wct_direct_kernel(CwtArgs a, int N, int K, float* __restrict__ coh) {
  extern __shared__ float4 tsm[];  // [S][n0]: (T1, T2, Re T12, Im T12)
  __shared__ double2 X[2][8];
  const long long b = blockIdx.x;
  const int n0 = a.n0, S = a.S;
  if (threadIdx.x < 2 * N) {  // spectra of the two (affine-normalised) series
    const int which = threadIdx.x / N, k = threadIdx.x % N;
    const float* row = (which ? a.x2 : a.x) + b * a.ld;
    const double* af = which ? a.affine2 : a.affine;
    double re = 0.0, im = 0.0;
    for (int n = 0; n < n0; ++n) {
      double v = row[n];
      if (af) v = static_cast<float>((v - af[3 * b] - af[3 * b + 1] * n) * af[3 * b + 2]);
      double sn, cs;
      sincospi(-2.0 * ((k * n) % N) / N, &sn, &cs);
      re += v * cs;
      im += v * sn;
    }
    X[which][k] = make_double2(re, im);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < S; j += 256) {
    const double s = a.scales[j];
    const double alpha = s * 2.0 * kPi / (N * a.dt);
    // pycwt normalises by sqrt(s * ftfreqs[1] * N) with ftfreqs = 2 pi fftfreq(N) / dt: for
    // N = 2, fftfreq(2)[1] = -1/2 and the reference's row is NaN -- kept
    const double c = N == 2 ? __builtin_nan("") : sqrt(2.0 * kPi * s / a.dt) * 0.75112554446494248286 / N;
    double2 w[2][8];
    for (int which = 0; which < 2; ++which)
      for (int t = 0; t < n0; ++t) {
        double re = 0.0, im = 0.0;
        for (int k = 0; k < N; ++k) {
          const int kk = k < N / 2 ? k : k - N;
          const double e = alpha * kk - a.f0;
          const double psi = c * exp(-0.5 * e * e);
          double sn, cs;
          sincospi(2.0 * ((k * t) % N) / N, &sn, &cs);
          const double2 x = X[which][k];
          re += psi * (x.x * cs - x.y * sn);
          im += psi * (x.x * sn + x.y * cs);
        }
        w[which][t] = make_double2(re, im);
      }
    // cross outputs and the three fields to smooth (zero past n0, as pycwt pads to N)
    double z[4][8];
    const long long rowbase = (b * S + j) * static_cast<long long>(n0);
    for (int t = 0; t < n0; ++t) {
      const double2 u = w[0][t], v = w[1][t];
      const double wr = u.x * v.x + u.y * v.y, wi = u.y * v.x - u.x * v.y;  // W1 conj(W2)
      const double pw = wr * wr + wi * wi;
      if (a.out_pow) a.out_pow[rowbase + t] = static_cast<float>(pw);
      if (a.out_sig) a.out_sig[rowbase + t] = static_cast<float>(atan2(wi, wr));  // phase plane
      if (a.out_u) {
        const double r = sqrt(pw);
        a.out_u[rowbase + t] = r > 0 ? static_cast<float>(wi / r) : 0.f;
        a.out_v[rowbase + t] = r > 0 ? static_cast<float>(wr / r) : 1.f;
      }
      z[0][t] = (u.x * u.x + u.y * u.y) / s;
      z[1][t] = (v.x * v.x + v.y * v.y) / s;
      z[2][t] = wr / s;
      z[3][t] = wi / s;
    }
    // time Gaussian F(k) = exp(-(s/dt)^2 (2 pi kk / N)^2 / 2) by length-N DFTs
    const double sg = s / a.dt * 2.0 * kPi / N;
    double T[4][8];
    for (int t = 0; t < n0; ++t) T[0][t] = T[1][t] = T[2][t] = T[3][t] = 0.0;
    for (int k = 0; k < N; ++k) {
      const int kk = k < N / 2 ? k : k - N;
      const double F = exp(-0.5 * (sg * kk) * (sg * kk)) / N;
      double Z[3][2] = {{0, 0}, {0, 0}, {0, 0}};  // spectra of z1, z2 (real) and z12
      for (int t = 0; t < n0; ++t) {
        double sn, cs;
        sincospi(-2.0 * ((k * t) % N) / N, &sn, &cs);
        Z[0][0] += z[0][t] * cs;  Z[0][1] += z[0][t] * sn;
        Z[1][0] += z[1][t] * cs;  Z[1][1] += z[1][t] * sn;
        Z[2][0] += z[2][t] * cs - z[3][t] * sn;
        Z[2][1] += z[2][t] * sn + z[3][t] * cs;
      }
      for (int t = 0; t < n0; ++t) {
        double sn, cs;
        sincospi(2.0 * ((k * t) % N) / N, &sn, &cs);
        T[0][t] += F * (Z[0][0] * cs - Z[0][1] * sn);  // real parts: the smoothed real fields
        T[1][t] += F * (Z[1][0] * cs - Z[1][1] * sn);
        T[2][t] += F * (Z[2][0] * cs - Z[2][1] * sn);
        T[3][t] += F * (Z[2][0] * sn + Z[2][1] * cs);
      }
    }
    for (int t = 0; t < n0; ++t)
      tsm[j * n0 + t] = make_float4(static_cast<float>(T[0][t]), static_cast<float>(T[1][t]),
                                    static_cast<float>(T[2][t]), static_cast<float>(T[3][t]));
  }
  __syncthreads();
  // scale boxcar (rows i - K/2 .. i + (K-1)/2, half weight at both ends) and the ratio
  const int LO = K / 2;
  const float wn = K > 1 ? 1.f / (K - 1) : 1.f;
  for (int idx = threadIdx.x; idx < S * n0; idx += 256) {
    const int i = idx / n0, t = idx - i * n0;
    float s1 = 0.f, s2 = 0.f, re = 0.f, im = 0.f;
    for (int q = 0; q < K; ++q) {
      const int row = i - LO + q;
      if (row < 0 || row >= S) continue;
      const float wq = (K > 1 && (q == 0 || q == K - 1)) ? 0.5f * wn : wn;
      const float4 v = tsm[row * n0 + t];
      s1 = fmaf(wq, v.x, s1);
      s2 = fmaf(wq, v.y, s2);
      re = fmaf(wq, v.z, re);
      im = fmaf(wq, v.w, im);
    }
    coh[(b * S + i) * static_cast<long long>(n0) + t] = (re * re + im * im) / (s1 * s2);
  }
}

static int log2_ceil_w(long long n) {
  int l = 0;
  while ((1ll << l) < n) ++l;
  return l;
}

}  // namespace wtmi

using namespace wtmi;

// workspace = [T: batch x S x n0 float4][spectra: batch x 2 x N cpx]
//             [band spectra: batch x S x 2 x N/16 cpx][decimated W12 spectra: batch x S x N/2 cpx,
//             N >= 2^kDecMinLogn][wide-band spectra: batch x S x 2 x N/2 cpx, N >= 2^kWideMinLogn]
//             [plan: S + 1 int][plan scratch: 2 S int][decimated rows: S int]
//             [decimated schedule: kDecSched int]
static long long wct_t_bytes(long long batch, long long n0, int n_scales) {
  const long long b = batch * n0 * static_cast<long long>(n_scales) * static_cast<long long>(sizeof(cpx));
  return 2 * ((b + 255) & ~255ll);
}
static long long wct_n(long long n0) { return 1ll << log2_ceil_w(n0 < 1 ? 1 : n0); }
static long long wct_spec_bytes(long long batch, long long n0) {
  return (batch * 2 * wct_n(n0) * static_cast<long long>(sizeof(cpx)) + 255) & ~255ll;
}
static long long wct_sb_bytes(long long batch, long long n0, int n_scales) {
  const long long nt = wct_n(n0) / 16 > 0 ? wct_n(n0) / 16 : 1;
  return (batch * n_scales * 2 * nt * static_cast<long long>(sizeof(cpx)) + 255) & ~255ll;
}
// wide-band smoothed spectra WB: [batch][S][2][N/2] cpx (LOGN >= kWideMinLogn)
static long long wct_wb_bytes(long long batch, long long n0, int n_scales) {
  if (wct_n(n0) < (1ll << kWideMinLogn)) return 0;
  return (batch * n_scales * wct_n(n0) * static_cast<long long>(sizeof(cpx)) + 255) & ~255ll;
}
static long long wct_dy_bytes(long long batch, long long n0, int n_scales) {
  if (wct_n(n0) < (1ll << kDecMinLogn) || wct_n(n0) != n0) return 0;  // decimated rows: full rows only
  return (batch * n_scales * (wct_n(n0) / 2) * static_cast<long long>(sizeof(cpx)) + 255) & ~255ll;
}

extern "C" long long wtmi_wct_workspace_bytes(long long batch, long long n0, int n_scales) {
  if (batch < 0 || n0 < 0 || n_scales < 0) return -1;
  if (n0 > (1 << 14)) return wct_long_workspace_bytes(batch, n0, n_scales);
  return wct_t_bytes(batch, n0, n_scales) + wct_spec_bytes(batch, n0) + wct_sb_bytes(batch, n0, n_scales) +
         wct_dy_bytes(batch, n0, n_scales) + wct_wb_bytes(batch, n0, n_scales) +
         4ll * (4 * n_scales + 1 + kDecSched);
}

static int wct_morlet_impl(const float* x1, const float* x2, long long ld, long long batch, long long n0,
                           const double* affine1, const double* affine2, int norm, const double* scales,
                           int n_scales, double dt, double f0, int boxcar, void* workspace, float* out_coh,
                           float* out_power, float* out_phase, float* out_u, float* out_v, void* stream) {
  if (n0 < 0 || batch < 0 || n_scales < 0 || ld < n0 || boxcar < 1) return kErrArg;
  if (n0 > (1ll << kLongMaxLog)) return kErrUnsupported;
  if (batch == 0 || n0 == 0 || n_scales == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x1 || !x2 || !scales || !workspace || !out_coh) return kErrArg;
  if ((out_u == nullptr) != (out_v == nullptr)) return kErrArg;
  const int logn = log2_ceil_w(n0);
  CwtArgs a{};
  a.x = x1;
  a.x2 = x2;
  a.ld = ld;
  a.batch = batch;
  a.n0 = static_cast<int>(n0);
  a.S = n_scales;
  a.affine = affine1;
  a.affine2 = affine2;
  a.scales = scales;
  a.dt = dt;
  a.f0 = f0;
  a.out_u = out_u;
  a.out_v = out_v;
  a.out_pow = out_power;
  a.out_sig = out_phase;  // phase-angle plane (atan2 of W12)
  a.norm = norm;
  if (norm && (n0 > (1 << 14) || n0 <= 8)) return kErrUnsupported;  // in-load normalisation: FFT rows
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n0 > (1 << 14)) return wct_long(a, boxcar, workspace, out_coh, st);
  if (logn < 4) {  // n0 <= 8: below the FFT engine's minimum row
    const size_t lds = static_cast<size_t>(n_scales) * n0 * sizeof(float4);
    if (lds > kWctDirectMaxLds || batch > 0x7fffffffll) return kErrUnsupported;
    if (lds > 65536)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(wct_direct_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    hipLaunchKernelGGL(wct_direct_kernel, dim3(static_cast<unsigned>(batch)), dim3(256), lds, st, a,
                       1 << logn, boxcar, out_coh);
    return launch_status();
  }
  const long long plane = wct_t_bytes(batch, n0, n_scales) / 2;
  cpx* TA = static_cast<cpx*>(workspace);
  cpx* TB = reinterpret_cast<cpx*>(static_cast<char*>(workspace) + plane);
  char* ws = static_cast<char*>(workspace) + 2 * plane;
  cpx* spec = reinterpret_cast<cpx*>(ws);
  ws += wct_spec_bytes(batch, n0);
  cpx* SB = reinterpret_cast<cpx*>(ws);
  ws += wct_sb_bytes(batch, n0, n_scales);
  cpx* DY = reinterpret_cast<cpx*>(ws);  // used only when wct_dy_bytes > 0 (launch_phase_a's dec)
  ws += wct_dy_bytes(batch, n0, n_scales);
  cpx* WB = reinterpret_cast<cpx*>(ws);  // used only when wct_wb_bytes > 0 (wide windows)
  ws += wct_wb_bytes(batch, n0, n_scales);
  int* plan = reinterpret_cast<int*>(ws);
  int rc;
  // side stream for the full-band rows beside the decimated chain (full rows with decimation:
  // LOGN >= kDecMinLogn, n0 = N, pruning 2), option wct_side_stream
  SideJoin sj(options().wct_side_stream && logn >= kDecMinLogn && n0 == (1ll << logn) &&
                  options().wct_prune >= 2 && f0 >= kBandF0,
              st);
  SideStream* side = sj.side;
  switch (logn) {
#define WTMI_A(L) case L: rc = launch_phase_a<L>(a, spec, TA, TB, SB, DY, WB, plan, boxcar, out_coh, st, sj); break;
    WTMI_A(4) WTMI_A(5) WTMI_A(6) WTMI_A(7) WTMI_A(8) WTMI_A(9) WTMI_A(10) WTMI_A(11)
    WTMI_A(12) WTMI_A(13) WTMI_A(14)
#undef WTMI_A
    default: return kErrUnsupported;
  }
  if (rc != kOk) return rc;
  const int n0i = static_cast<int>(n0);
  auto phase_c = [&](hipStream_t cs, int which) -> int {
    switch (logn) {
#define WTMI_C(L) case L: return launch_phase_c<L>(a, SB, WB, plan, boxcar, out_coh, cs, which);
      WTMI_C(4) WTMI_C(5) WTMI_C(6) WTMI_C(7) WTMI_C(8) WTMI_C(9) WTMI_C(10) WTMI_C(11)
      WTMI_C(12) WTMI_C(13) WTMI_C(14)
#undef WTMI_C
      default: return kErrUnsupported;
    }
  };
  // With the side stream (full rows, decimation on): the spectral boxcar and phase C run there
  // once the decimated spectra are done (they need the WB / SB spectra of the full-band rows,
  // which the side stream made, and of the decimated rows), while phase B runs here once the
  // full-band rows' time-domain rows are done; the caller's stream then joins the side stream.
  hipStream_t sc = st;
  // option wct_pc_early: phase C's q windows on the entry's second side stream as soon as the
  // decimated spectra are done -- every row of a q window is a decimated row, so they need
  // neither the full-band rows' kernel nor the spectral boxcar.  A/B (alternating, one box,
  // r04): 64 pairs 0.495 -> 0.482 ms, 128 pairs 0.843 -> 0.831, 512 pairs 3.039 -> 3.053, so
  // by default (2) for batches of at most 256 pairs
  const int pce = options().wct_pc_early;
  const bool third = side && (pce == 1 || (pce == 2 && batch <= 256));
  if (side) {
    if (hipStreamWaitEvent(side->s, side->dec, 0) != hipSuccess) return launch_status();
    sc = side->s;
    if (third) {
      if (hipStreamWaitEvent(side->s2, side->dec, 0) != hipSuccess) return launch_status();
      sj.forked2 = true;
      if ((rc = phase_c(side->s2, 1)) != kOk) return rc;
    }
  }
  // spectral boxcar of the wide windows (their sums over the output rows' WB slots)
  if (wct_wb_bytes(batch, n0, n_scales) > 0 && a.prune >= 1 && boxcar <= kWideMaxK) {
    const long long tiles = ((1ll << logn) / 2 + 255) / 256;
    if (batch * tiles > 0x7fffffffll) return kErrUnsupported;
    switch (boxcar) {
#define WTMI_W(KK)                                                                                         \
  case KK:                                                                                                 \
    if (KK <= 12 && options().wct_depth == 1)                                                              \
      hipLaunchKernelGGL((wct_wide_boxcar<KK, (KK <= 12 ? KK : 0)>), dim3(static_cast<unsigned>(batch * tiles)), dim3(256), 0, sc, WB, \
                         batch, 1 << logn, n_scales, plan);                                               \
    else                                                                                                   \
    hipLaunchKernelGGL(wct_wide_boxcar<KK>, dim3(static_cast<unsigned>(batch * tiles)), dim3(256), 0, sc, WB, \
                       batch, 1 << logn, n_scales, plan);                                                 \
    break;
      WTMI_W(1) WTMI_W(2) WTMI_W(3) WTMI_W(4) WTMI_W(5) WTMI_W(6) WTMI_W(7) WTMI_W(8)
      WTMI_W(9) WTMI_W(10) WTMI_W(11) WTMI_W(12) WTMI_W(13) WTMI_W(14) WTMI_W(15) WTMI_W(16)
      WTMI_W(17) WTMI_W(18) WTMI_W(19) WTMI_W(20) WTMI_W(21) WTMI_W(22) WTMI_W(23) WTMI_W(24)
#undef WTMI_W
      default: break;
    }
    if ((rc = launch_status()) != kOk) return rc;
  }
  if ((rc = phase_c(sc, third ? 2 : 3)) != kOk) return rc;
  // phase B on the caller's stream once the full-band rows are done; sj joins the side stream
  if (side && hipStreamWaitEvent(st, side->k0, 0) != hipSuccess) return launch_status();
  return wct_phase_b_any(TA, TB, batch, n0i, n_scales, out_coh, plan, boxcar, st);
}

extern "C" int wtmi_wct_morlet(const float* x1, const float* x2, long long ld, long long batch,
                               long long n0, const double* affine1, const double* affine2,
                               const double* scales, int n_scales, double dt, double f0, int boxcar,
                               void* workspace, float* out_coh, float* out_power, float* out_phase,
                               float* out_u, float* out_v, void* stream) {
  return wct_morlet_impl(x1, x2, ld, batch, n0, affine1, affine2, 0, scales, n_scales, dt, f0, boxcar, workspace,
                         out_coh, out_power, out_phase, out_u, out_v, stream);
}

extern "C" int wtmi_wct_morlet_norm(const float* x1, const float* x2, long long ld, long long batch,
                                    long long n0, const double* scales, int n_scales, double dt, double f0,
                                    int boxcar, void* workspace, float* out_coh, float* out_power,
                                    float* out_phase, float* out_u, float* out_v, void* stream) {
  return wct_morlet_impl(x1, x2, ld, batch, n0, nullptr, nullptr, 1, scales, n_scales, dt, f0, boxcar, workspace,
                         out_coh, out_power, out_phase, out_u, out_v, stream);
}

// Side-stream pool entries (two streams each) the WCT has created in this process (all
// devices): the pool's size, i.e. the most full-row WCT calls that ever ran at once, not the
// number of threads that made one.
extern "C" long long wtmi_wct_side_streams(void) { return wtmi::side_pool().created.load(); }
