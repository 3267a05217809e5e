// Per-series moments and affine standardisation (K9 of DESIGN.md), fp64.
//
// Replaces the O(n) NumPy preprocessing around the transforms:
//   standardize_series  (src/utils/wavelet_helpers.py:22-57: std/mean of the
//                        original series, polyfit deg-1 detrend or demean, / std)
//   pycwt.ar1's lag-0/lag-1 covariances (called src/cwt.py:106)
//   pycwt xwt/wct normalisation (y - mean) / std
// One workgroup per series; two passes (mean, then centred sums) in double.
#include "common.hpp"

namespace wtmi {

constexpr int kStatThreads = 256;

template <typename T>
__device__ __forceinline__ double ld_elem(const void* p, long long i) {
  return static_cast<double>(static_cast<const T*>(p)[i]);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < kStatThreads / 64; ++i) r += sh[i];
  return r;
}

// Affine modes (wtmi_series_affine): the [B][3] coefficients (a0, a1, a2) of x' = (x - a0 - a1 t) a2
// that standardize_series / the pycwt normalisation apply, straight from the moments.
enum : int { kAffDetrend = 1, kAffRemoveMean = 2, kAffStandardize = 4 };

// out[b*8 + {0..7}] = mean, std (ddof 0), slope, intercept (least squares vs
// t = 0..n-1), c0 = sum((x-m)^2)/n, c1 = sum((x_i-m)(x_{i+1}-m))/(n-1), n, 0 (out may be null);
// aff[b*3 + {0..2}] = the affine coefficients of `mode` (aff may be null)
template <typename T>
__global__ void __launch_bounds__(kStatThreads) moments_kernel(const void* x, long long ld, int n,
                                                               double* out, int mode, double* aff) {
  __shared__ double sh[kStatThreads / 64];
  const long long b = blockIdx.x;
  const long long base = b * ld;
  // unrolled by 8: the loads of eight iterations are in flight together (the plain strided
  // loop waited on each load in turn: 24 us for 512 series of 8192 samples, latency-bound)
  double s = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < n; i += kStatThreads) s += ld_elem<T>(x, base + i);
  const double mean = block_sum(s, sh) / n;
  const double tbar = 0.5 * (n - 1);
  double sxx = 0.0, sxt = 0.0, sl1 = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < n; i += kStatThreads) {
    const double d = ld_elem<T>(x, base + i) - mean;
    sxx += d * d;
    sxt += d * (i - tbar);
    const double dn = ld_elem<T>(x, base + min(i + 1, n - 1)) - mean;  // no branch around the load
    sl1 += (i + 1 < n) ? d * dn : 0.0;
  }
  sxx = block_sum(sxx, sh);
  sxt = block_sum(sxt, sh);
  sl1 = block_sum(sl1, sh);
  if (threadIdx.x == 0) {
    const double stt = static_cast<double>(n) * (static_cast<double>(n) * n - 1.0) / 12.0;
    const double slope = stt > 0 ? sxt / stt : 0.0;
    const double sd = sqrt(sxx / n);
    if (out) {
      double* o = out + 8 * b;
      o[0] = mean;
      o[1] = sd;
      o[2] = slope;
      o[3] = mean - slope * tbar;
      o[4] = sxx / n;
      o[5] = n > 1 ? sl1 / (n - 1) : 0.0;
      o[6] = n;
      o[7] = 0.0;
    }
    if (aff) {  // as transforms.standardize_coefs / normalize_coefs (detrend wins over the mean)
      double* c = aff + 3 * b;
      c[0] = (mode & kAffDetrend) ? mean - slope * tbar : ((mode & kAffRemoveMean) ? mean : 0.0);
      c[1] = (mode & kAffDetrend) ? slope : 0.0;
      c[2] = (mode & kAffStandardize) ? 1.0 / sd : 1.0;
    }
  }
}

// y = (x - a0 - a1 * t) * a2 per series, computed in double.
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) affine_kernel(const void* x, long long ld_in, long long batch,
                                                    int n, const double* coef, void* y,
                                                    long long ld_out) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= batch * n) return;
  const long long b = idx / n;
  const int t = static_cast<int>(idx - b * n);
  const double v = ld_elem<TI>(x, b * ld_in + t);
  const double r = (v - coef[3 * b] - coef[3 * b + 1] * t) * coef[3 * b + 2];
  static_cast<TO*>(y)[b * ld_out + t] = static_cast<TO>(r);
}

}  // namespace wtmi

using namespace wtmi;

static int launch_moments(const void* x, int x_is_f64, long long ld, long long batch, long long n, double* out,
                          int mode, double* aff, void* stream) {
  if (batch == 0) return kOk;
  if (batch > 0x7fffffffll) return kErrUnsupported;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (x_is_f64)
    hipLaunchKernelGGL(moments_kernel<double>, dim3(batch), dim3(kStatThreads), 0, st, x, ld,
                       static_cast<int>(n), out, mode, aff);
  else
    hipLaunchKernelGGL(moments_kernel<float>, dim3(batch), dim3(kStatThreads), 0, st, x, ld,
                       static_cast<int>(n), out, mode, aff);
  return launch_status();
}

extern "C" int wtmi_series_moments(const void* x, int x_is_f64, long long ld, long long batch,
                                   long long n, double* out, void* stream) {
  if (batch < 0 || n < 1 || ld < n || n > 0x7fffffff) return kErrArg;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !out) return kErrArg;
  return launch_moments(x, x_is_f64, ld, batch, n, out, 0, nullptr, stream);
}

extern "C" int wtmi_series_affine(const void* x, int x_is_f64, long long ld, long long batch, long long n,
                                  int mode, double* moments, double* affine, void* stream) {
  if (batch < 0 || n < 1 || ld < n || n > 0x7fffffff || mode < 0 || mode > 7 ||
      ((mode & kAffDetrend) && (mode & kAffRemoveMean)))
    return kErrArg;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !affine) return kErrArg;
  return launch_moments(x, x_is_f64, ld, batch, n, moments, mode, affine, stream);
}

extern "C" int wtmi_affine(const void* x, int x_is_f64, long long ld_in, long long batch, long long n,
                           const double* coef, void* y, int y_is_f64, long long ld_out,
                           void* stream) {
  if (batch < 0 || n < 0 || ld_in < n || ld_out < n || n > 0x7fffffff) return kErrArg;
  const long long total = batch * n;
  if (total == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !coef || !y) return kErrArg;
  const long long blocks = (total + 255) / 256;
  if (blocks > 0x7fffffffll) return kErrUnsupported;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int ni = static_cast<int>(n);
  if (x_is_f64 && y_is_f64)
    hipLaunchKernelGGL((affine_kernel<double, double>), dim3(blocks), dim3(256), 0, st, x, ld_in, batch,
                       ni, coef, y, ld_out);
  else if (x_is_f64)
    hipLaunchKernelGGL((affine_kernel<double, float>), dim3(blocks), dim3(256), 0, st, x, ld_in, batch,
                       ni, coef, y, ld_out);
  else if (y_is_f64)
    hipLaunchKernelGGL((affine_kernel<float, double>), dim3(blocks), dim3(256), 0, st, x, ld_in, batch,
                       ni, coef, y, ld_out);
  else
    hipLaunchKernelGGL((affine_kernel<float, float>), dim3(blocks), dim3(256), 0, st, x, ld_in, batch,
                       ni, coef, y, ld_out);
  return launch_status();
}
