// Pyramid DWT analysis / synthesis, mode "symmetric" (K5 / K6 of DESIGN.md).
//
// Replaces pywt.wavedec / pywt.waverec as called from src/dwt.py:104,120 (and the
// smoothing / component reconstructions built on waverec, :53-73, :110-120):
//   analysis : c[i] = sum_{k<F} f[k] * xe[2i + 1 - k], i < (m + F - 1)/2,
//              xe = half-sample symmetric extension of the level input (length m)
//   synthesis: y[t] = sum_i cA[i] rec_lo[t + F - 2 - 2i] + cD[i] rec_hi[...],
//              t < 2*len(cD) - F + 2, cA first trimmed to len(cD) (pywt waverec)
// One workgroup per series (analysis) or per (series, variant) (synthesis); every
// level stays in LDS, only the coefficient arrays touch HBM.
#include "common.hpp"

namespace wtmi {

constexpr int kDwtMaxTaps = 128;
constexpr int kDwtMaxN = 16384;                // one workgroup, every level in LDS
constexpr long long kDwtLongMaxN = 1ll << 30;  // per-level launches
constexpr int kDwtThreads = 256;

struct DwtBank {
  float lo[kDwtMaxTaps];
  float hi[kDwtMaxTaps];
};

__device__ __forceinline__ int sym_index(int i, int m) {
  const int p = 2 * m;
  int r = i % p;
  if (r < 0) r += p;
  return r < m ? r : p - 1 - r;
}

__global__ void __launch_bounds__(kDwtThreads) wavedec_kernel(const float* __restrict__ x, long long ld,
                                                             int n, int F, int level, DwtBank fb,
                                                             float* __restrict__ coeffs, long long total) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* A = sm;
  float* B = sm + n + F;
  const long long b = blockIdx.x;
  const float* xin = x + b * ld;
  float* out = coeffs + b * total;
#pragma unroll 4  // several loads in flight per thread
  for (int i = threadIdx.x; i < n; i += kDwtThreads) A[i] = xin[i];
  __syncthreads();
  // offset of cD_j (pywt list index level - j + 1) = total - sum_{i<=j} len(cD_i)
  long long end = total;
  int m = n;
  for (int j = 1; j <= level; ++j) {
    const int M = (m + F - 1) / 2;
    float* cD = out + (end - M);
    for (int i = threadIdx.x; i < M; i += kDwtThreads) {
      float a = 0.f, d = 0.f;
      for (int k = 0; k < F; ++k) {
        const float v = A[sym_index(2 * i + 1 - k, m)];
        a = fmaf(fb.lo[k], v, a);
        d = fmaf(fb.hi[k], v, d);
      }
      B[i] = a;
      cD[i] = d;
    }
    __syncthreads();
    float* t = A; A = B; B = t;
    end -= M;
    m = M;
  }
  // cA_J at offset 0 (end == len(cA_J) here)
  for (int i = threadIdx.x; i < m; i += kDwtThreads) out[i] = A[i];
}

__global__ void __launch_bounds__(kDwtThreads) waverec_kernel(const float* __restrict__ coeffs, int n, int F,
                                                             int level, DwtBank fb,
                                                             const unsigned long long* __restrict__ masks,
                                                             int nvar, float* __restrict__ out,
                                                             long long out_len, long long total, int cap) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* A = sm;
  float* Y = sm + cap;
  const long long b = blockIdx.x / nvar;
  const int var = static_cast<int>(blockIdx.x - b * nvar);
  const unsigned long long keep = masks[var];
  const float* cin = coeffs + b * total;
  // lengths: cD_j has M_j with M_0 = n, M_j = (M_{j-1} + F - 1)/2; cA_J has M_J
  int lens[64];
  lens[0] = n;
  for (int j = 1; j <= level; ++j) lens[j] = (lens[j - 1] + F - 1) / 2;
  int alen = lens[level];
  const bool keepA = keep & 1ull;
#pragma unroll 4  // several loads in flight per thread
  for (int i = threadIdx.x; i < alen; i += kDwtThreads) A[i] = keepA ? cin[i] : 0.f;
  long long off = alen;
  for (int k = 1; k <= level; ++k) {
    const int j = level - k + 1;  // cD_j is list entry k
    const int M = lens[j];
    const bool keepD = (keep >> k) & 1ull;
    const float* cD = cin + off;
    off += M;
    if (alen == M + 1) alen = M;  // pywt trims cA to len(cD)
    const int L = 2 * M - F + 2;
    __syncthreads();
    for (int t = threadIdx.x; t < L; t += kDwtThreads) {
      // i with 0 <= t + F - 2 - 2i < F  ->  ceil((t-1)/2) <= i <= (t+F-2)/2
      int i0 = (t) / 2;  // ceil((t-1)/2) == t/2 for t >= 0
      int i1 = (t + F - 2) / 2;
      if (i1 > M - 1) i1 = M - 1;
      float acc = 0.f;
      for (int i = i0; i <= i1; ++i) {
        const int kk = t + F - 2 - 2 * i;
        acc = fmaf(A[i], fb.lo[kk], acc);
        if (keepD) acc = fmaf(cD[i], fb.hi[kk], acc);
      }
      Y[t] = acc;
    }
    __syncthreads();
    float* tmp = A; A = Y; Y = tmp;
    alen = L;
  }
  float* o = out + (b * nvar + var) * out_len;
  for (int t = threadIdx.x; t < alen && t < out_len; t += kDwtThreads) o[t] = A[t];
}

static bool make_dwt_bank(const double* lo, const double* hi, int F, DwtBank& fb) {
  if (!lo || !hi || F < 2 || F > kDwtMaxTaps) return false;
  for (int i = 0; i < kDwtMaxTaps; ++i) {
    fb.lo[i] = i < F ? static_cast<float>(lo[i]) : 0.f;
    fb.hi[i] = i < F ? static_cast<float>(hi[i]) : 0.f;
  }
  return true;
}

static long long dwt_lengths(long long n, int F, int level, long long* lens) {
  // returns total; lens (optional) in pywt order [cA_J, cD_J, ..., cD_1]
  long long m = n, total = 0;
  long long tmp[64];
  for (int j = 1; j <= level; ++j) {
    m = (m + F - 1) / 2;
    tmp[j] = m;
    total += m;
  }
  total += m;  // cA_J
  if (lens) {
    lens[0] = m;
    for (int k = 1; k <= level; ++k) lens[k] = tmp[level - k + 1];
  }
  return total;
}

// ---------------------------------------------------------------------------------
// Long series (n > 16384: the level ping-pong no longer fits one workgroup's LDS).  One
// launch per level, one thread per output coefficient; level inputs come from a scratch
// ping-pong pair (cap floats per row) or, for the first / last level, straight from the
// caller's arrays.
__global__ void __launch_bounds__(256) wavedec_level_kernel(const float* __restrict__ ain, long long ld_in,
                                                            long long batch, int m, int M, int F, DwtBank fb,
                                                            float* __restrict__ aout, long long ld_a,
                                                            float* __restrict__ dout, long long ld_d) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= batch * M) return;
  const long long b = idx / M;
  const int i = static_cast<int>(idx - b * M);
  const float* a = ain + b * ld_in;
  float sa = 0.f, sd = 0.f;
  for (int k = 0; k < F; ++k) {
    const float v = a[sym_index(2 * i + 1 - k, m)];
    sa = fmaf(fb.lo[k], v, sa);
    sd = fmaf(fb.hi[k], v, sd);
  }
  aout[b * ld_a + i] = sa;
  dout[b * ld_d + i] = sd;
}

// One synthesis level for every (series, variant) row: y[t] = sum_i A[i] lo[t+F-2-2i] +
// cD[i] hi[t+F-2-2i].  A is the level input of the row (ain + row * ld_a), or -- on the
// first level, a_shared -- cA_J of the series inside the coefficient array (all variants).
__global__ void __launch_bounds__(256) waverec_level_kernel(const float* __restrict__ ain, long long ld_a,
                                                            bool a_shared, const float* __restrict__ coeffs,
                                                            long long total, long long d_off, int M, int L,
                                                            int F, int k, DwtBank fb,
                                                            const unsigned long long* __restrict__ masks,
                                                            int nvar, long long batch,
                                                            float* __restrict__ yout, long long ld_y, int ylim) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  const int T = L < ylim ? L : ylim;
  if (idx >= batch * nvar * T) return;
  const long long row = idx / T;  // b * nvar + var
  const int t = static_cast<int>(idx - row * T);
  const long long b = row / nvar;
  const int var = static_cast<int>(row - b * nvar);
  const unsigned long long keep = masks[var];
  const float* A = a_shared ? coeffs + b * total : ain + row * ld_a;
  const float asel = (!a_shared || (keep & 1ull)) ? 1.f : 0.f;
  const float dsel = ((keep >> k) & 1ull) ? 1.f : 0.f;
  const float* cD = coeffs + b * total + d_off;
  int i0 = t / 2;
  int i1 = (t + F - 2) / 2;
  if (i1 > M - 1) i1 = M - 1;
  float acc = 0.f;
  for (int i = i0; i <= i1; ++i) {
    const int kk = t + F - 2 - 2 * i;
    acc = fmaf(asel * A[i], fb.lo[kk], acc);
    acc = fmaf(dsel * cD[i], fb.hi[kk], acc);
  }
  yout[row * ld_y + t] = acc;
}

static long long dwt_cap(long long n, int F) { return (n + F) / 2 + 2 * F + 8; }

static int wavedec_long(const float* x, long long ld, long long batch, int n, int F, int level,
                        const DwtBank& fb, float* coeffs, long long total, float* scratch, hipStream_t st) {
  const long long cap = dwt_cap(n, F);
  float* buf[2] = {scratch, scratch + batch * cap};
  const float* ain = x;
  long long ldin = ld;
  long long end = total;
  int m = n;
  if (level == 0) {  // cA_0 = x
    const hipError_t e = hipMemcpy2DAsync(coeffs, total * sizeof(float), x, ld * sizeof(float), n * sizeof(float),
                                          batch, hipMemcpyDeviceToDevice, st);
    return e == hipSuccess ? kOk : static_cast<int>(e);
  }
  for (int j = 1; j <= level; ++j) {
    const int M = (m + F - 1) / 2;
    float* aout = j == level ? coeffs : buf[j & 1];
    const long long lda = j == level ? total : cap;
    const long long grid = (batch * M + 255) / 256;
    if (grid > 0x7fffffffll) return kErrUnsupported;
    hipLaunchKernelGGL(wavedec_level_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, ain, ldin,
                       batch, m, M, F, fb, aout, lda, coeffs + (end - M), total);
    const int rc = launch_status();
    if (rc != kOk) return rc;
    ain = aout;
    ldin = lda;
    end -= M;
    m = M;
  }
  return kOk;
}

static int waverec_long(const float* coeffs, long long batch, int n, int F, int level, const DwtBank& fb,
                        const unsigned long long* masks, int nvar, float* out, long long out_len,
                        long long total, float* scratch, hipStream_t st) {
  const long long cap = dwt_cap(n, F);
  const long long rows = batch * nvar;
  float* buf[2] = {scratch, scratch + rows * cap};
  long long lens[64];
  lens[0] = n;
  for (int j = 1; j <= level; ++j) lens[j] = (lens[j - 1] + F - 1) / 2;
  if (level == 0) return kErrUnsupported;  // nothing to reconstruct (the caller copies)
  long long off = lens[level];             // cA_J first, then cD_J ... cD_1
  const float* ain = nullptr;
  long long lda = 0;
  for (int k = 1; k <= level; ++k) {
    const int j = level - k + 1;  // cD_j is list entry k
    const int M = static_cast<int>(lens[j]);
    const int L = 2 * M - F + 2;
    const bool last = k == level;
    float* yout = last ? out : buf[k & 1];
    const long long ldy = last ? out_len : cap;
    const int ylim = last ? static_cast<int>(out_len < L ? out_len : L) : L;
    const long long grid = (rows * ylim + 255) / 256;
    if (grid > 0x7fffffffll) return kErrUnsupported;
    hipLaunchKernelGGL(waverec_level_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, ain, lda,
                       k == 1, coeffs, total, off, M, L, F, k, fb, masks, nvar, batch, yout, ldy, ylim);
    const int rc = launch_status();
    if (rc != kOk) return rc;
    off += M;
    ain = yout;
    lda = ldy;
  }
  return kOk;
}

template <typename K>
static void allow_dwt_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
}

}  // namespace wtmi

using namespace wtmi;

extern "C" long long wtmi_dwt_lengths(long long n, int n_taps, int level, long long* lens) {
  if (n < 1 || n_taps < 2 || level < 0 || level > 60) return -1;
  return dwt_lengths(n, n_taps, level, lens);
}

extern "C" long long wtmi_dwt_workspace_bytes(long long batch, long long n, int n_taps, int n_variants) {
  if (batch < 0 || n < 1 || n_taps < 2 || n_variants < 1) return -1;
  if (n <= kDwtMaxN) return 0;
  // two ping-pong rows per (series, variant); wavedec uses n_variants = 1
  return 2 * batch * n_variants * dwt_cap(n, n_taps) * static_cast<long long>(sizeof(float));
}

extern "C" int wtmi_wavedec(const float* x, long long ld, long long batch, long long n,
                            const double* dec_lo, const double* dec_hi, int n_taps, int level,
                            float* coeffs, void* workspace, void* stream) {
  DwtBank fb;
  if (batch < 0 || n < 1 || ld < n || level < 0 || level > 60) return kErrArg;
  if (!make_dwt_bank(dec_lo, dec_hi, n_taps, fb)) return kErrArg;
  if (n > kDwtLongMaxN || batch > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !coeffs) return kErrArg;
  const long long total = dwt_lengths(n, n_taps, level, nullptr);
  if (n > kDwtMaxN) {
    if (!workspace) return kErrArg;
    return wavedec_long(x, ld, batch, static_cast<int>(n), n_taps, level, fb, coeffs, total,
                        static_cast<float*>(workspace), static_cast<hipStream_t>(stream));
  }
  const int ni = static_cast<int>(n);
  const size_t lds = static_cast<size_t>(2 * (ni + n_taps) + 8) * sizeof(float);
  allow_dwt_lds(wavedec_kernel, lds);
  hipLaunchKernelGGL(wavedec_kernel, dim3(batch), dim3(kDwtThreads), lds, static_cast<hipStream_t>(stream),
                     x, ld, ni, n_taps, level, fb, coeffs, total);
  return launch_status();
}

extern "C" int wtmi_waverec(const float* coeffs, long long batch, long long n, const double* rec_lo,
                            const double* rec_hi, int n_taps, int level,
                            const unsigned long long* keep_masks, int n_variants, float* out,
                            long long out_len, void* workspace, void* stream) {
  DwtBank fb;
  if (batch < 0 || n < 1 || level < 0 || level > 60 || n_variants < 1 || out_len < 1) return kErrArg;
  if (!make_dwt_bank(rec_lo, rec_hi, n_taps, fb)) return kErrArg;
  if (n > kDwtLongMaxN || batch * n_variants > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!coeffs || !out || !keep_masks) return kErrArg;
  const long long total = dwt_lengths(n, n_taps, level, nullptr);
  if (n > kDwtMaxN && level > 0) {
    if (!workspace) return kErrArg;
    return waverec_long(coeffs, batch, static_cast<int>(n), n_taps, level, fb, keep_masks, n_variants, out,
                        out_len, total, static_cast<float*>(workspace), static_cast<hipStream_t>(stream));
  }
  if (n > kDwtMaxN) return kErrUnsupported;  // level 0 of a long series: no transform to invert
  const int cap = static_cast<int>(n) + 2 * n_taps + 8;  // >= any intermediate length
  const size_t lds = static_cast<size_t>(2 * cap) * sizeof(float);
  allow_dwt_lds(waverec_kernel, lds);
  hipLaunchKernelGGL(waverec_kernel, dim3(batch * n_variants), dim3(kDwtThreads), lds,
                     static_cast<hipStream_t>(stream), coeffs, static_cast<int>(n), n_taps, level, fb,
                     keep_masks, n_variants, out, out_len, total, cap);
  return launch_status();
}
