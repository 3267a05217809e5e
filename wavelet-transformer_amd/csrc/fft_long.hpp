// Long rows: N = 2^LOGN > 16384 samples through a four-step FFT in HBM (CWT / XWT / WCT
// of series longer than one workgroup's register+LDS row, SURVEY 5 "long-context").
//
// N = N1 * N2 with N2 = 2^LOG2 <= 16384 (one fft_row per row, as the short kernels) and
// N1 = 2^LOG1 >= 16 (the column transforms, LOG1 = max(4, LOGN - 14)).  A length-N row is
// viewed as the matrix M[i1][i2] = row[i2 + N2 i1] (natural order).
//
//   forward  X[k1 + N1 k2] = sum_n2 e^{-2pi i k2 n2/N2} e^{-2pi i k1 n2/N} sum_n1 x[n2 + N2 n1] e^{-2pi i k1 n1/N1}
//     column pass (over n1 per column n2, then the twiddle) -> U[k1][n2]
//     row pass    (over n2 per row k1)                      -> XT[k1][k2] = X[k1 + N1 k2]
//   inverse  w[n2 + N2 n1] = sum_k1 e^{2pi i k1 n1/N1} e^{2pi i k1 n2/N} sum_k2 Y[k1 + N1 k2] e^{2pi i k2 n2/N2}
//     row pass    (over k2 per row k1, then the twiddle)    -> Z[k1][n2]
//     column pass (over k1 per column n2)                   -> w[n2 + N2 n1] = matrix [n1][n2]
//
// The spectrum therefore lives in the transposed order XT (row k1 holds bins k1 + N1 k2),
// which is exactly what the inverse row pass reads: a filter multiply (Morlet psi_j, or
// the smoothing Gaussian) happens in that row pass's registers.  Column passes process
// ROWS = 256 / NT1 adjacent columns per workgroup with the lane index running over the
// columns, so every global access of a column pass is a run of ROWS consecutive complex
// values (2 KB for N1 = 16); a column pass writes its output in place of its input.
#pragma once

#include "long_path.hpp"

namespace wtmi {

__host__ __device__ constexpr int long_log1(int logn) { return logn - 14 > 4 ? logn - 14 : 4; }

// exp(sign * 2 pi i p / N) for 0 <= p < N <= 2^24: 2p/N is exact in float.
__device__ __forceinline__ cpx long_twiddle(long long p, int logn, float sign) {
  float s, c;
  sincospif(static_cast<float>(p) * ldexpf(2.f, -logn), &s, &c);
  return cpx{c, sign * s};
}

template <int LOG1>
struct LongCol {
  using P = FftPlan<LOG1>;
  static constexpr int NT = P::NT;              // threads per column
  static constexpr int ROWS = 256 / NT;         // columns per workgroup
  static constexpr int BLOCK = 256;
  static constexpr int LDS_CPX = P::NPASS > 1 ? ROWS * P::PADN : 1;
};

template <int LOG2>
struct LongRow {
  using P = FftPlan<LOG2>;
  static constexpr int ROWS = P::NT >= 256 ? 1 : 256 / P::NT;
  static constexpr int BLOCK = P::NT * ROWS;
  static constexpr bool TWL = LOG2 >= 13;
  static constexpr int LDS_F4 = (ROWS * P::PADN) / 2 + (TWL ? P::TWL_FLOAT4 : 0) + 1;
};

// Arguments of every long-row kernel (one struct: the launchers fill what a mode reads).
struct LongArgs {
  int logn, n0;          // transform length 2^logn, samples kept
  long long nrows;       // matrices this launch processes (series, or (series, scale) rows)
  // series input (forward column pass)
  const float* x;
  long long ld;
  const double* affine;  // [series][3] or null
  const double* mom;     // [series][8] moments (mean at [0]) of the raw series
  // spectra / scratch
  cpx* spec;             // XT rows [series][N] (forward output, inverse-row input)
  cpx* z1;               // work rows [nrows][N]
  cpx* z2;               // second work rows (pair mode) or null
  const cpx* spec2;      // second series' spectra (pair mode)
  // scales of this launch: row r = (series r / nsc, scale j0 + r % nsc)
  const double* scales;
  int j0, nsc, S;        // first scale, scales per series in this launch, scales in all
  long long b0;          // first series of this launch (output row index offset)
  double dt, f0;
  // outputs (inverse column pass)
  CwtArgs out;           // out_w / out_pow / out_sig (+ sigscale, sig_ld) / out_u / out_v
  float* out_phase;      // WCT: angle(W12)
  cpx* ta;               // WCT smoothing outputs [series][S][n0]: (T1, T2) and T12
  cpx* tb;
};

// ---------------------------------------------------------------------------- columns
enum : int {
  kColFwdSeries = 0,  // real series (affine, mean removed) -> U (forward, twiddled)
  kColFwdRows = 1,    // complex work rows in place -> U (forward, twiddled)
  kColInvCwt = 2,     // Z -> CWT outputs of row (b, j)
  kColInvPair = 3,    // Z1, Z2 -> cross outputs (+ WCT smoothing inputs written in place)
  kColInvSmooth = 4,  // smoothed Z1 = (T1, T2), Z2 = T12 -> ta / tb rows
};

template <int LOG1, int MODE, bool WCT = false>
__global__ void __launch_bounds__(256) long_col_kernel(LongArgs a) {
  using C = LongCol<LOG1>;
  using P = typename C::P;
  __shared__ cpx lds[C::LDS_CPX];
  const int tid = threadIdx.x;
  const int g = tid % C::ROWS;  // column within the tile (lanes run over columns)
  const int t = tid / C::ROWS;  // thread within the column's transform
  const int log2n2 = a.logn - LOG1;
  const int N2 = 1 << log2n2;
  const long long N = 1ll << a.logn;
  const long long tiles = N2 / C::ROWS;
  const long long r = blockIdx.x / tiles;
  const int c = static_cast<int>((blockIdx.x - r * tiles) * C::ROWS) + g;  // column n2 / k-col
  cpx tw[P::NTW_ALLOC];
  fft_twiddles<LOG1>(tw, t);
  int par = 0;
  cpx* my = P::NPASS > 1 ? lds + g * P::PADN : lds;
  constexpr int DIR = MODE <= kColFwdRows ? -1 : 1;
  cpx v[16], v2[16];
  if constexpr (MODE == kColFwdSeries) {
    const float* row = a.x + r * a.ld;
    double a0 = 0.0, a1 = 0.0, a2 = 1.0;
    if (a.affine) {
      a0 = a.affine[3 * r];
      a1 = a.affine[3 * r + 1];
      a2 = a.affine[3 * r + 2];
    }
    // mean of x' = (x - a0 - a1 t) a2 over the n0 samples, from the fp64 moments
    const float mu = static_cast<float>((a.mom[8 * r] - a0 - a1 * 0.5 * (a.n0 - 1)) * a2);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long n = c + (static_cast<long long>(t + m * P::NT) << log2n2);
      float val = 0.f;
      if (n < a.n0) {
        val = row[n];
        if (a.affine) val = static_cast<float>((static_cast<double>(val) - a0 - a1 * n) * a2);
        val -= mu;
      }
      v[m] = mkc(val, 0.f);
    }
  } else {
    const cpx* zr = a.z1 + r * N;
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = zr[c + (static_cast<long long>(t + m * P::NT) << log2n2)];
    if constexpr (MODE == kColInvPair || MODE == kColInvSmooth) {
      const cpx* zr2 = a.z2 + r * N;
#pragma unroll
      for (int m = 0; m < 16; ++m) v2[m] = zr2[c + (static_cast<long long>(t + m * P::NT) << log2n2)];
    }
  }
  fft_row<LOG1, DIR, 1>(v, my, 0, tw, t, par);
  if constexpr (MODE == kColInvPair || MODE == kColInvSmooth) fft_row<LOG1, DIR, 1>(v2, my, 0, tw, t, par);

  if constexpr (MODE == kColFwdSeries || MODE == kColFwdRows) {
    cpx* dst = (MODE == kColFwdSeries ? a.spec : a.z1) + r * N;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int k1 = t + m * P::NT;
      dst[c + (static_cast<long long>(k1) << log2n2)] =
          cmul(v[m], long_twiddle(static_cast<long long>(k1) * c, a.logn, -1.f));
    }
  } else if constexpr (MODE == kColInvCwt) {
    const long long b = a.b0 + r / a.nsc;
    const int j = a.j0 + static_cast<int>(r % a.nsc);
    const long long rowbase = (b * a.S + j) * static_cast<long long>(a.n0);
    const float sg = a.out.sigscale ? static_cast<float>(a.out.sigscale[b * a.out.sig_ld + j]) : 0.f;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long n = c + (static_cast<long long>(t + m * P::NT) << log2n2);
      if (n >= a.n0) continue;
      const long long o = rowbase + n;
      const float pw = cabs2(v[m]);
      if (a.out.out_w) a.out.out_w[o] = v[m];
      if (a.out.out_pow) a.out.out_pow[o] = pw;
      if (a.out.out_sig) a.out.out_sig[o] = pw * sg;
    }
  } else if constexpr (MODE == kColInvPair) {
    const long long b = a.b0 + r / a.nsc;
    const int j = a.j0 + static_cast<int>(r % a.nsc);
    const long long rowbase = (b * a.S + j) * static_cast<long long>(a.n0);
    const float sg = a.out.sigscale ? static_cast<float>(a.out.sigscale[b * a.out.sig_ld + j]) : 0.f;
    const float inv_s = static_cast<float>(1.0 / a.scales[j]);
    cpx* z1 = a.z1 + r * N;
    cpx* z2 = a.z2 + r * N;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long n = c + (static_cast<long long>(t + m * P::NT) << log2n2);
      const cpx w12 = cmul2_conj(v[m], v2[m]);
      if (n < a.n0) {
        const long long o = rowbase + n;
        const float pw = cabs2(w12);
        if (a.out.out_w) a.out.out_w[o] = w12;
        if (a.out.out_pow) a.out.out_pow[o] = pw;
        if (a.out.out_sig) a.out.out_sig[o] = pw * sg;
        if (a.out.out_u) {
          const float rr = sqrtf(pw);
          a.out.out_u[o] = rr > 0.f ? w12.y / rr : 0.f;
          a.out.out_v[o] = rr > 0.f ? w12.x / rr : 1.f;
        }
        if (a.out_phase) a.out_phase[o] = fast_atan2f(w12.y, w12.x);
      }
      if constexpr (WCT) {  // smoothing inputs, zero past n0 (pycwt pads W to N)
        const bool in = n < a.n0;
        z1[n] = in ? cpx{cabs2(v[m]) * inv_s, cabs2(v2[m]) * inv_s} : mkc(0.f, 0.f);
        z2[n] = in ? w12 * inv_s : mkc(0.f, 0.f);
      }
    }
  } else {  // kColInvSmooth
    const long long b = a.b0 + r / a.nsc;
    const int j = a.j0 + static_cast<int>(r % a.nsc);
    const long long rowbase = (b * a.S + j) * static_cast<long long>(a.n0);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long n = c + (static_cast<long long>(t + m * P::NT) << log2n2);
      if (n >= a.n0) continue;
      a.ta[rowbase + n] = v[m];   // (T1, T2): the two real fields of one complex transform
      a.tb[rowbase + n] = v2[m];  // T12
    }
  }
}

// ------------------------------------------------------------------------------- rows
enum : int {
  kRowFwdSpec = 0,    // U row k1 -> XT row k1 (+ the removed mean's spectrum)
  kRowInvMorlet = 1,  // XT row k1 of series b x psi_j -> Z row k1 of (b, j), twiddled
  kRowSmooth = 2,     // U row k1 of a work row -> forward, x F_j, inverse, twiddled, in place
};

template <int LOG2, int MODE>
__global__ void __launch_bounds__(LongRow<LOG2>::BLOCK) long_row_kernel(LongArgs a) {
  using R = LongRow<LOG2>;
  using P = typename R::P;
  __shared__ float4 lds4[R::LDS_F4];
  cpx* lds = reinterpret_cast<cpx*>(lds4);
  float4* twl = lds4 + (R::ROWS * P::PADN) / 2;
  const int tid = threadIdx.x;
  const int g = tid / P::NT;
  const int t = fft_thread<LOG2>(tid - g * P::NT);
  const int log1 = a.logn - LOG2;
  const int N1 = 1 << log1;
  const long long N = 1ll << a.logn;
  const long long row = static_cast<long long>(blockIdx.x) * R::ROWS + g;  // (matrix, k1)
  const long long r = row >> log1;     // matrix
  const int k1 = static_cast<int>(row & (N1 - 1));
  constexpr bool TWL = R::TWL;
  cpx tw[TWL ? P::NTW_REG : P::NTW_ALLOC];
  if constexpr (TWL) {
    fft_twiddle_table<LOG2>(twl, tid, R::BLOCK);
    fft_twiddles_tail<LOG2>(tw, t);
    __syncthreads();
  } else {
    fft_twiddles<LOG2>(tw, t);
  }
  int par = 0;
  cpx* my = lds + g * P::PADN;
  cpx v[16];
  const bool live = r < a.nrows;
  if constexpr (MODE == kRowFwdSpec) {
    cpx* src = a.spec + (live ? r : 0) * N + (static_cast<long long>(k1) << LOG2);
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = src[t + m * P::NT];
    fft_row<LOG2, -1, 1, TWL>(v, my, 0, tw, t, par, twl);
    // + mu * D[k], D[k] = sum_{n < n0} e^{-2 pi i k n / N}, for the mean the column pass removed
    const double a0 = a.affine ? a.affine[3 * r] : 0.0, a1 = a.affine ? a.affine[3 * r + 1] : 0.0;
    const double a2 = a.affine ? a.affine[3 * r + 2] : 1.0;
    const double mu = static_cast<double>(static_cast<float>(
        (a.mom[8 * (live ? r : 0)] - a0 - a1 * 0.5 * (a.n0 - 1)) * a2));
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long k = k1 + (static_cast<long long>(t + m * P::NT) << log1);
      cpx d;
      if (k == 0) {
        d = mkc(static_cast<float>(mu * a.n0), 0.f);
      } else {
        // phases reduced mod 2N in integers, then sin / cos of pi * (p / N) in fp64
        const long long twoN = 2 * N;
        const long long ph = (k * (a.n0 - 1)) % twoN;
        const long long am = (k * a.n0) % twoN;
        double s1, c1;
        sincospi(static_cast<double>(ph) / N, &s1, &c1);
        const double rr = mu * sinpi(static_cast<double>(am) / N) / sinpi(static_cast<double>(k) / N);
        d = mkc(static_cast<float>(c1 * rr), static_cast<float>(-s1 * rr));
      }
      v[m] += d;
    }
    if (live) {
#pragma unroll
      for (int m = 0; m < 16; ++m) src[t + m * P::NT] = v[m];
    }
  } else if constexpr (MODE == kRowInvMorlet) {
    const long long b = r / a.nsc;  // series within this launch's spectra
    const int j = a.j0 + static_cast<int>(r % a.nsc);
    const cpx* src = a.spec + (live ? b : 0) * N + (static_cast<long long>(k1) << LOG2);
    const cpx prm = morlet_params(a.scales[live ? j : a.j0], a.dt, 1 << a.logn);
    constexpr float K = -0.5f * kLog2e;
    const float f0 = static_cast<float>(a.f0);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const long long k = k1 + (static_cast<long long>(t + m * P::NT) << log1);
      const float kk = static_cast<float>(k < N / 2 ? k : k - N);
      const float e = fmaf(prm.x, kk, -f0);
      v[m] = cscale(src[t + m * P::NT], __builtin_amdgcn_exp2f(fmaf(e * K, e, prm.y)));
    }
    fft_row<LOG2, 1, 1, TWL>(v, my, 0, tw, t, par, twl);
    if (live) {
      cpx* dst = a.z1 + r * N + (static_cast<long long>(k1) << LOG2);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int n2 = t + m * P::NT;
        dst[n2] = cmul(v[m], long_twiddle(static_cast<long long>(k1) * n2, a.logn, 1.f));
      }
    }
  } else {  // kRowSmooth: both work planes (z1 and z2) of the row, same Gaussian
    const int j = a.j0 + static_cast<int>((live ? r : 0) % a.nsc);
    // F(k) = exp(-(s/dt)^2 w_k^2 / 2) / N, w_k = 2 pi kk / N (pycwt Morlet.smooth, 1/N of ifft)
    const float sig = static_cast<float>(a.scales[j] / a.dt * 2.0 * kPi / static_cast<double>(N));
    const float lnorm = -static_cast<float>(a.logn);
    constexpr float K = -0.5f * kLog2e;
#pragma unroll 1
    for (int plane = 0; plane < 2; ++plane) {
      cpx* src = (plane ? a.z2 : a.z1) + (live ? r : 0) * N + (static_cast<long long>(k1) << LOG2);
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = src[t + m * P::NT];
      fft_row<LOG2, -1, 1, TWL>(v, my, 0, tw, t, par, twl);
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const long long k = k1 + (static_cast<long long>(t + m * P::NT) << log1);
        const float x = sig * static_cast<float>(k < N / 2 ? k : k - N);
        v[m] = cscale(v[m], __builtin_amdgcn_exp2f(fmaf(x * K, x, lnorm)));
      }
      fft_row<LOG2, 1, 1, TWL>(v, my, 0, tw, t, par, twl);
      if (live) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const int n2 = t + m * P::NT;
          src[n2] = cmul(v[m], long_twiddle(static_cast<long long>(k1) * n2, a.logn, 1.f));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- launch
template <int LOG1, int MODE, bool WCT = false>
inline int launch_long_col(const LongArgs& a, hipStream_t st) {
  using C = LongCol<LOG1>;
  const long long tiles = (1ll << (a.logn - LOG1)) / C::ROWS;
  const long long grid = a.nrows * tiles;
  if (grid < 1) return kOk;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL((long_col_kernel<LOG1, MODE, WCT>), dim3(static_cast<unsigned>(grid)), dim3(C::BLOCK),
                     0, st, a);
  return launch_status();
}

template <int LOG2, int MODE>
inline int launch_long_row(const LongArgs& a, hipStream_t st) {
  using R = LongRow<LOG2>;
  const long long rows = a.nrows << (a.logn - LOG2);
  const long long grid = (rows + R::ROWS - 1) / R::ROWS;
  if (grid < 1) return kOk;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL((long_row_kernel<LOG2, MODE>), dim3(static_cast<unsigned>(grid)), dim3(R::BLOCK), 0,
                     st, a);
  return launch_status();
}

// Runtime dispatch on log1 / log2 of a.logn (15..20: log1 = 4..6, log2 = 11..14).
template <int MODE, bool WCT = false>
inline int long_col(const LongArgs& a, hipStream_t st) {
  switch (long_log1(a.logn)) {
    case 4: return launch_long_col<4, MODE, WCT>(a, st);
    case 5: return launch_long_col<5, MODE, WCT>(a, st);
    case 6: return launch_long_col<6, MODE, WCT>(a, st);
    default: return kErrUnsupported;
  }
}

template <int MODE>
inline int long_row(const LongArgs& a, hipStream_t st) {
  switch (a.logn - long_log1(a.logn)) {
    case 11: return launch_long_row<11, MODE>(a, st);
    case 12: return launch_long_row<12, MODE>(a, st);
    case 13: return launch_long_row<13, MODE>(a, st);
    case 14: return launch_long_row<14, MODE>(a, st);
    default: return kErrUnsupported;
  }
}

}  // namespace wtmi
