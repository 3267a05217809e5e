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
  const double* sigscale;  // [S] multiplier for the ratio output (1 / signif), or null
  cpx* out_w;
  float* out_pow;
  float* out_sig;
  float* out_u;
  float* out_v;
  int nchunks, chunk;
};

constexpr double kPi = 3.14159265358979323846;
constexpr float kLog2e = 1.44269504088896340736f;

template <int LOGN, int MODE>
struct CwtGeom {
  using P = FftPlan<LOGN>;
  static constexpr int ROWS = P::NT >= 256 ? 1 : 256 / P::NT;
  static constexpr int BLOCK = P::NT * ROWS;
  // LOGN >= 13 keeps the radix-16 twiddles in an LDS table (FftPlan::TWL_E): that is
  // what brings the single-series kernel to <= 128 VGPRs, i.e. two 512-thread
  // workgroups per CU (LDS 2 x 80 KiB) instead of one.
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

}  // namespace wtmi
