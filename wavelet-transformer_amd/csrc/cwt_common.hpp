// Pieces shared by the CWT / XWT (cwt.hip) and WCT (wct.hip) kernels: argument
// block, series load with fused affine standardisation, analytic Morlet filter.
#pragma once

#include "fft_lds.hpp"

namespace wtmi {

struct CwtArgs {
  const float* x;
  const float* x2;
  long long ld;          // elements between consecutive series
  long long batch;
  int n0;                // samples per series (output length)
  int S;                 // number of scales
  const double* affine;  // [batch][3]: x' = (x - a0 - a1 * t) * a2, or null
  const double* affine2;
  const double* scales;  // [S] device
  double dt, f0;
  const double* sigscale;  // [S] multiplier for the ratio output (1 / signif), or null;
                           // series b uses sigscale + b * sig_ld (sig_ld 0: one row for all)
  long long sig_ld;
  cpx* out_w;
  float* out_pow;
  float* out_sig;
  float* out_u;
  float* out_v;
  int nchunks, chunk;
  int prune;             // 2: band-pruned rows + narrowed entry passes (row_code);
                         // 1: band-pruned rows only; 0: full FFTs
  // Non-Morlet mothers (kernels instantiated with VAR = 1, full transforms only):
  //   conj(psi_hat(f)) = (mcre + i mcim) gate(f) 2^(mA f^2 + mB f + mP log2|f| + lnorm),
  // f = s w_k; gate 0: 1, 1: f > 0 (Paul), 2: sign(f) (DOG of odd order).  See mother_consts.
  int mother;            // 0 Morlet (f0), 1 Paul (order m), 2 DOG (order m)
  float mA, mB, mP, mcre, mcim;
  int mgate;
  double mlnorm;         // log2 of the mother's normalisation (Morlet: log2 pi^-1/4)
  int norm;              // WCT: normalise each series in the load, (y - mean) / std (pycwt
                         // xwt / wct), in place of the affine pointers
};

inline namespace WTMI_FFT_NS {

// Filter constants of a mother wavelet (pycwt 0.4.0b0 mothers.py: Paul.psi_ft, DOG.psi_ft).
inline bool mother_consts(CwtArgs& a, int mother, double param) {
  a.mother = mother;
  a.mA = a.mB = a.mP = a.mcim = 0.f;
  a.mcre = 1.f;
  a.mgate = 0;
  if (mother == 0) {  // Morlet(f0): the dedicated kernels; param = f0
    a.f0 = param;
    a.mlnorm = -0.25 * 1.6514961294723187;  // log2 pi^-1/4
    return true;
  }
  const int m = static_cast<int>(param);
  if (static_cast<double>(m) != param || m < 1 || m > 40) return false;
  a.f0 = 0.0;
  a.mP = static_cast<float>(m);
  if (mother == 1) {  // Paul: 2^m / sqrt(m (2m-1)!) f^m e^-f H(f)
    double lf = 0.0;  // log2 (2m-1)!
    for (int k = 2; k < 2 * m; ++k) lf += log2(static_cast<double>(k));
    a.mlnorm = m - 0.5 * (log2(static_cast<double>(m)) + lf);
    a.mB = static_cast<float>(-1.4426950408889634);
    a.mgate = 1;
    return true;
  }
  if (mother == 2) {  // DOG: -i^m / sqrt(Gamma(m + 1/2)) f^m e^(-f^2/2); conj(-i^m)
    a.mlnorm = -0.5 * lgamma(m + 0.5) / 0.6931471805599453;
    a.mA = static_cast<float>(-0.5 * 1.4426950408889634);
    a.mgate = (m & 1) ? 2 : 0;
    static const float cre[4] = {-1.f, 0.f, 1.f, 0.f}, cim[4] = {0.f, 1.f, 0.f, -1.f};
    a.mcre = cre[m & 3];
    a.mcim = cim[m & 3];
    return true;
  }
  return false;
}

constexpr double kPi = 3.14159265358979323846;
constexpr float kLog2e = 1.44269504088896340736f;

template <int LOGN, int MODE, int VAR = 0>
struct CwtGeom {
  using P = FftPlan<LOGN>;
  static constexpr int ROWS = P::NT >= 256 ? 1 : 256 / P::NT;
  static constexpr int BLOCK = P::NT * ROWS;
  // LOGN >= 13 keeps the radix-16 twiddles in an LDS table (FftPlan::TWL_E): that is
  // what brings the single-series kernel to <= 128 VGPRs, i.e. two 512-thread
  // workgroups per CU (LDS 2 x 80 KiB) instead of one.  VAR: launch variants for A/B
  // sweeps (none at present; LDS twiddles or 4 waves/SIMD at LOGN 12 measured equal, r01).
  static constexpr bool TWL = LOGN >= 13;
  // waves per SIMD requested from the register allocator (4 -> <= 128 VGPRs,
  // 3 -> <= 168, 2 -> <= 256).  A 1024-thread block is 4 waves per SIMD by itself.
  static constexpr int MINW = BLOCK >= 1024 ? 4 : (MODE == 1 ? 2 : (BLOCK >= 512 ? 4 : 3));
  // scales per workgroup (size of the per-scale parameter table in LDS)
  static constexpr int MAXCHUNK = 128;
  static constexpr int TWL_F4 = TWL ? P::TWL_FLOAT4 : 0;
};

template <int LOGN>
__device__ __forceinline__ void load_series(cpx (&v)[16], const float* __restrict__ x,
                                            const double* __restrict__ affine, long long b,
                                            long long ld, int n0, int t) {
  using P = FftPlan<LOGN>;
  const float* row = x + b * ld;
  double a0 = 0.0, a1 = 0.0, a2 = 1.0;
  const bool aff = affine != nullptr;
  if (aff) {
    a0 = affine[3 * b + 0];
    a1 = affine[3 * b + 1];
    a2 = affine[3 * b + 2];
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int pos = t + m * P::NT;
    float val = 0.f;
    if (pos < n0) {
      val = row[pos];
      if (aff) val = static_cast<float>((static_cast<double>(val) - a0 - a1 * pos) * a2);
    }
    v[m] = mkc(val, 0.f);
  }
}

// Mean removal around the forward FFT.  pycwt.cwt transforms the raw series (no
// centring), and a large offset costs fp32 accuracy in every bin: the FFT's rounding
// error scales with ||x||, the offset's energy included.  The kernels therefore transform
// x - mu (mu = the row mean) and add mu's spectrum back exactly:
//   D[k] = sum_{n < n0} exp(-2 pi i k n / N) = exp(-i pi k (n0-1)/N) sin(pi k n0/N) / sin(pi k/N)
// (D = N delta_k0 when n0 = N).  mu is bitwise identical in every thread of the row (the
// xor-butterfly sums are commutative pairwise), so subtraction and correction agree.
// red: >= BLOCK/64 floats of LDS.  Every thread of the workgroup must call this.
template <int LOGN>
__device__ __forceinline__ float demean_row(cpx (&v)[16], int n0, int t, float* red) {
  using P = FftPlan<LOGN>;
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) s += v[m].x;  // padding entries are zero
  constexpr int W = P::NT < kWave ? P::NT : kWave;
#pragma unroll
  for (int o = 1; o < W; o <<= 1) s += __shfl_xor(s, o, W);
  if constexpr (P::NT > kWave) {
    constexpr int WPR = P::NT / kWave;  // waves per row
    const int wv = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) red[wv] = s;
    __syncthreads();
    const int w0 = wv & ~(WPR - 1);
    s = 0.f;
#pragma unroll
    for (int w = 0; w < WPR; ++w) s += red[w0 + w];
  }
  const float mu = s / static_cast<float>(n0);
#pragma unroll
  for (int m = 0; m < 16; ++m)
    if (t + m * P::NT < n0) v[m].x -= mu;
  return mu;
}

// pycwt's wct / xwt normalisation inside the load: y' = (y - mean) / std (ddof 0) with the
// moments in fp64 over the row's n0 samples (two passes over the registers: mean, then the
// centred sum of squares), applied in fp64 and rounded once to fp32 -- what the separate
// moments + affine launches (wtmi_series_affine, mode normalise) computed.  redd: >= BLOCK/64
// doubles of LDS; every thread of the workgroup must call this.
template <int LOGN>
__device__ __forceinline__ double row_sum_f64(double s, int t, double* redd) {
  using P = FftPlan<LOGN>;
  constexpr int W = P::NT < kWave ? P::NT : kWave;
#pragma unroll
  for (int o = 1; o < W; o <<= 1) s += __shfl_xor(s, o, W);
  if constexpr (P::NT > kWave) {
    constexpr int WPR = P::NT / kWave;
    const int wv = threadIdx.x / kWave;
    __syncthreads();  // redd reuse
    if ((threadIdx.x & (kWave - 1)) == 0) redd[wv] = s;
    __syncthreads();
    const int w0 = wv & ~(WPR - 1);
    s = 0.0;
#pragma unroll
    for (int w = 0; w < WPR; ++w) s += redd[w0 + w];
  }
  return s;
}

template <int LOGN>
__device__ __forceinline__ void normalize_row(cpx (&v)[16], int n0, int t, double* redd) {
  using P = FftPlan<LOGN>;
  double s = 0.0;
#pragma unroll
  for (int m = 0; m < 16; ++m) s += static_cast<double>(v[m].x);  // padding entries are zero
  const double mu = row_sum_f64<LOGN>(s, t, redd) / n0;
  double q = 0.0;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const double d = t + m * P::NT < n0 ? static_cast<double>(v[m].x) - mu : 0.0;
    q = fma(d, d, q);
  }
  const double inv = 1.0 / sqrt(row_sum_f64<LOGN>(q, t, redd) / n0);
#pragma unroll
  for (int m = 0; m < 16; ++m)
    if (t + m * P::NT < n0) v[m].x = static_cast<float>((static_cast<double>(v[m].x) - mu) * inv);
}

// X[k] += mu * D[k] for the 16 bins k = t + m*NT this thread holds (forward spectrum).
template <int LOGN>
__device__ __forceinline__ void add_mean_spectrum(cpx (&X)[16], float mu, int n0, int t) {
  using P = FftPlan<LOGN>;
  if (n0 == P::N) {
    if (t == 0) X[0].x += mu * static_cast<float>(P::N);
    return;
  }
  constexpr int N2 = 2 * P::N;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int k = t + m * P::NT;
    if (k == 0) {
      X[m].x += mu * static_cast<float>(n0);
      continue;
    }
    const int ph = static_cast<int>((static_cast<long long>(k) * (n0 - 1)) % N2);
    const int am = static_cast<int>((static_cast<long long>(k) * n0) % N2);
    float s1, c1;
    sincospif(static_cast<float>(ph) / P::N, &s1, &c1);
    const float r = mu * sinpif(static_cast<float>(am) / P::N) / sinpif(static_cast<float>(k) / P::N);
    X[m] += cpx{c1, -s1} * r;
  }
}

// Per-scale filter constants: e_k = alpha * kk - f0, psi_k = exp2(lc - log2(e)/2 * e_k^2)
// with alpha = 2 pi s / (N dt) and 2^lc = sqrt(2 pi s / dt) * pi^-1/4 / N (1/N of the IFFT).
__device__ __forceinline__ cpx morlet_params(double s, double dt, int N) {
  const double alpha = s * 2.0 * kPi / (static_cast<double>(N) * dt);
  const double c = sqrt(2.0 * kPi * s / dt) * 0.75112554446494248286 / static_cast<double>(N);
  return mkc(static_cast<float>(alpha), static_cast<float>(log2(c)));
}

// v = X * psi_bar_j / N for the 16 bins this thread owns.  Bin k = t + m*NT has the
// signed frequency index kk = t + (m < 8 ? m : m - 16) * NT (fftfreq ordering).
template <int LOGN>
__device__ __forceinline__ void morlet_filter(cpx (&v)[16], const cpx (&X)[16], cpx prm,
                                              float f0, int t) {
  using P = FftPlan<LOGN>;
  constexpr float K = -0.5f * kLog2e;
  const float eb = fmaf(prm.x, static_cast<float>(t), -f0);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float off = static_cast<float>((m < 8 ? m : m - 16) * P::NT);
    const float e = fmaf(prm.x, off, eb);
    const float psi = __builtin_amdgcn_exp2f(fmaf(e * K, e, prm.y));
    v[m] = cscale(X[m], psi);
  }
}

// Band regime of one scale for the inverse transform (see band_entry in fft_lds.hpp):
// the largest Q in {0, 1, 2} such that the filtered spectrum X * psi_bar vanishes to
// fp32 precision outside bins [0, N/16^Q).  psi_k = exp(-(alpha k - f0)^2 / 2):
//  - upper edge: bins k >= N/16^Q have alpha k - f0 >= kBandT, psi <= exp(-kBandT^2/2) = 6.8e-10;
//  - negative frequencies (k >= N/2 in fftfreq order) have psi <= exp(-f0^2/2), dropped only
//    for f0 >= kBandF0 (Morlet(6): 1.5e-8 of the peak, far below the fp32 FFT's own rounding).
// Bin 0 (the mean) is always inside the band.  A pruned row is exact up to those terms.
constexpr double kBandT = 6.5;
constexpr double kBandF0 = 5.5;

template <int LOGN>
__device__ __forceinline__ int band_regime(double s, double dt, double f0) {
  using P = FftPlan<LOGN>;
  if (f0 < kBandF0) return 0;
  const double alpha = s * 2.0 * kPi / (static_cast<double>(P::N) * dt);
  int q = 0;
#pragma unroll
  for (int qq = 1; qq <= 2; ++qq) {
    if (qq < P::P16 && (P::NT % (1 << (4 * qq))) == 0 &&
        alpha * static_cast<double>(P::N >> (4 * qq)) - f0 >= kBandT)
      q = qq;
  }
  return q;
}

// Row code (0..11) = 4 q + k: band regime q (band_regime) and width NZ = 16 >> k of the
// transform's entry pass -- its inputs r >= NZ vanish.  Entry pass q reads bins
// (t >> 4q) + r (NT >> 4q) (q >= 1) or t + r NT (q = 0), so r >= NZ means bins >= NZ * unit:
// narrowed when psi is below exp(-kBandT^2/2) there; for q = 0, r >= 8 are the negative
// frequencies (dropped for f0 >= kBandF0), so NZ <= 8 always.  A smaller code is a wider band:
// the rows of one iteration run at their smallest code.
template <int LOGN>
__device__ __forceinline__ int row_code(double s, double dt, double f0, int prune) {
  using P = FftPlan<LOGN>;
  if (!prune) return 0;
  const int q = band_regime<LOGN>(s, dt, f0);
  if (prune < 2 || f0 < kBandF0 || P::NT < 16) return 4 * q;
  const double alpha = s * 2.0 * kPi / (static_cast<double>(P::N) * dt);
  const double unit = static_cast<double>(q == 0 ? P::NT : (P::NT >> (4 * q)));
  int k = q == 0 ? 1 : 0;  // NZ = 8 / 16
  if (alpha * 4.0 * unit - f0 >= kBandT) k = 2;  // NZ = 4
  if (alpha * 2.0 * unit - f0 >= kBandT) k = 3;  // NZ = 2
  return 4 * q + k;
}

// v = X * psi_bar_j / N on the bins m < NZ (the rest zero, see row_code).
template <int LOGN, int NZ>
__device__ __forceinline__ void morlet_filter_nz(cpx (&v)[16], const cpx (&X)[16], cpx prm,
                                                 float f0, int t) {
  using P = FftPlan<LOGN>;
  constexpr float K = -0.5f * kLog2e;
  const float eb = fmaf(prm.x, static_cast<float>(t), -f0);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    if (m < NZ) {
      const float off = static_cast<float>((m < 8 ? m : m - 16) * P::NT);
      const float e = fmaf(prm.x, off, eb);
      v[m] = cscale(X[m], __builtin_amdgcn_exp2f(fmaf(e * K, e, prm.y)));
    } else {
      v[m] = mkc(0.f, 0.f);
    }
  }
}

// v = X * conj(psi_hat(s w_k)) * sqrt(2 pi s / dt) / N for a non-Morlet mother (all 16 bins;
// prm = (alpha, log2(sqrt(2 pi s / dt) / N) + lnorm), see mother_consts).
template <int LOGN>
__device__ __forceinline__ void mother_filter(cpx (&v)[16], const cpx (&X)[16], cpx prm, const CwtArgs& a,
                                              int t) {
  using P = FftPlan<LOGN>;
  const cpx cst = mkc(a.mcre, a.mcim);
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float f = prm.x * static_cast<float>(t + (m < 8 ? m : m - 16) * P::NT);
    const float e = fmaf(a.mA * f, f, fmaf(a.mB, f, fmaf(a.mP, __log2f(fabsf(f)), prm.y)));
    float psi = __builtin_amdgcn_exp2f(e);
    if (a.mgate == 1) psi = f > 0.f ? psi : 0.f;
    if (a.mgate == 2) psi = f < 0.f ? -psi : psi;
    v[m] = cmul(cscale(X[m], psi), cst);
  }
}

// fp64 conj(psi_hat(f)) * 2^lc for the direct (n0 <= 8) kernels; lc as in mother_filter.
__device__ __forceinline__ double2 mother_psi_d(double f, double lc, const CwtArgs& a) {
  if (a.mother == 0) {
    const double e = f - a.f0;
    return make_double2(exp2(lc) * exp(-0.5 * e * e), 0.0);
  }
  if (f == 0.0 || (a.mgate == 1 && f < 0.0)) return make_double2(0.0, 0.0);
  double psi = exp2(lc + a.mP * log2(fabs(f))) * exp(a.mother == 1 ? -f : -0.5 * f * f);
  if (a.mgate == 2 && f < 0.0) psi = -psi;
  return make_double2(psi * a.mcre, psi * a.mcim);
}

// Filtered bin t of a band-pruned row (thread t's m = 0 element, frequency index t >= 0).
__device__ __forceinline__ cpx morlet_bin0(cpx X0, cpx prm, float f0, int t) {
  constexpr float K = -0.5f * kLog2e;
  const float e = fmaf(prm.x, static_cast<float>(t), -f0);
  return cscale(X0, __builtin_amdgcn_exp2f(fmaf(e * K, e, prm.y)));
}

}  // inline namespace WTMI_FFT_NS
}  // namespace wtmi
