// Monte-Carlo coherence significance pieces: pycwt's
// wct_significance, reached from src/wct.py:106-118 when run_wct is called with
// calculate_signficance=True.  Per Monte-Carlo pass pycwt draws two AR(1) red-noise
// series (helpers.rednoise), runs the coherence of the pair and counts
// floor(R2 * nbins) per scale over the points outside the cone of influence.
//
// Here the passes are batched: K10 draws all 2 x mc_count series at once, the
// coherence kernels (wct.hip) run on the batch as on any pair batch, and K11 folds
// the coherence planes into the [scale][bin] counter.  The quantile step (a few
// thousand numbers) stays on the host.
#include "common.hpp"

namespace wtmi {

// Philox4x32-10 (Salmon et al., SC'11), counter-based: stream (series, block) -> 4 words.
struct Philox {
  static constexpr unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  static constexpr unsigned W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  __device__ static uint4 gen(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const unsigned long long p0 = static_cast<unsigned long long>(M0) * c.x;
      const unsigned long long p1 = static_cast<unsigned long long>(M1) * c.z;
      const unsigned hi0 = static_cast<unsigned>(p0 >> 32), lo0 = static_cast<unsigned>(p0);
      const unsigned hi1 = static_cast<unsigned>(p1 >> 32), lo1 = static_cast<unsigned>(p1);
      c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
      k.x += W0;
      k.y += W1;
    }
    return c;
  }
};

__device__ __forceinline__ double u01(unsigned a, unsigned b) {  // (0, 1), 53 bits
  const unsigned long long v = (static_cast<unsigned long long>(a) << 21) ^ (b >> 11);
  return (static_cast<double>(v & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;
}

// K10: pycwt helpers.rednoise(N, g, a=1) (pycwt 0.4.0b0):
//   yr = lfilter([1, 0], [1, -g], np.random.randn(N + tau, 1) * a)[tau:], tau = ceil(-2 / ln|g|).
// lfilter runs along its default axis -1, which has length 1 for that (N + tau, 1) array, so
// the filter is the identity and pycwt's noise is WHITE (N normals; g only sets tau).  That
// literal reading is the default (filtered = 0: DESIGN 4, "Monte-Carlo noise").  filtered = 1
// runs the AR(1) recurrence y_i = g y_{i-1} + e_i that Grinsted's MATLAB rednoise.m (whose
// filter works along the first non-singleton dimension) intends.
// Normal i of series sid comes from Philox block (i / 2, sid) by Box-Muller (fp64); both modes
// draw the same normals.  One workgroup per series; the recurrence is split into 256 chunks of
// L consecutive samples: pass 1 runs each chunk from a zero state (its end value a_c), one
// thread chains the chunks' carries (carry_c = g^L carry_{c-1} + a_{c-1}), pass 2 reruns each
// chunk from its carry -- regenerating the same normals -- and writes y.  The sequential
// recurrence of one thread per series took milliseconds per launch (N + tau ~ 8000 steps of
// Philox + fp64 log / sincospi each); this is the same linear recurrence in a different
// summation order (fp64, rounded to fp32 on store).  With g = 0 (the white mode) every step is
// fma(0, y, e) = e exactly.
__device__ __forceinline__ void rn_normals(unsigned long long sid, uint2 key, int i0, double (&e)[2]) {
  const uint4 w = Philox::gen(make_uint4(static_cast<unsigned>(i0 >> 1), static_cast<unsigned>(sid),
                                         static_cast<unsigned>(sid >> 32), 0x5eed5u), key);
  const double r = sqrt(-2.0 * log(u01(w.x, w.y)));
  double s, co;
  sincospi(2.0 * u01(w.z, w.w), &s, &co);
  e[0] = r * co;
  e[1] = r * s;
}

constexpr int kRnThreads = 256;

__global__ void __launch_bounds__(kRnThreads) rednoise_kernel(float* __restrict__ out, long long ld,
                                                              long long count, int n, double g, int tau,
                                                              unsigned long long seed,
                                                              unsigned long long first) {
  __shared__ double carry[kRnThreads];
  const long long c = blockIdx.x;
  const unsigned long long sid = first + static_cast<unsigned long long>(c);
  const uint2 key = make_uint2(static_cast<unsigned>(seed), static_cast<unsigned>(seed >> 32));
  float* row = out + c * ld;
  const int total = n + tau;
  const int L = (((total + kRnThreads - 1) / kRnThreads) + 1) & ~1;  // even: chunks start on a block
  const int t = threadIdx.x;
  const int ib = min(total, t * L), ie = min(total, ib + L);
  double y = 0.0;
  for (int i0 = ib; i0 < ie; i0 += 2) {  // pass 1: the chunk from a zero state
    double e[2];
    rn_normals(sid, key, i0, e);
    y = fma(g, y, e[0]);
    if (i0 + 1 < ie) y = fma(g, y, e[1]);
  }
  carry[t] = y;
  __syncthreads();
  if (t == 0) {  // carry into chunk k = state after chunks 0..k-1
    const double gl = pow(g, static_cast<double>(L));
    double st = 0.0;
    for (int k = 0; k < kRnThreads; ++k) {
      const double a = carry[k];
      carry[k] = st;
      st = fma(gl, st, a);
    }
  }
  __syncthreads();
  y = carry[t];
  for (int i0 = ib; i0 < ie; i0 += 2) {  // pass 2: from the carry, writing the samples >= tau
    double e[2];
    rn_normals(sid, key, i0, e);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = i0 + q;
      if (i < ie) {
        y = fma(g, y, e[q]);
        if (i >= tau) row[i - tau] = static_cast<float>(y);
      }
    }
  }
}

// K11: per-scale coherence counter.  Block (s, part) walks the pairs
// part, part + parts, ... of scale s (s < n_hist_scales) over t in [t_lo[s], t_hi[s])
// -- the points outside the COI, an interval because the COI is a triangle -- and
// counts floor(R2 * nbins) (clamped to [0, nbins - 1]; NaN skipped) into an LDS
// histogram, then adds the non-zero bins to hist[s][:].
constexpr int kHistThreads = 256;
constexpr int kMaxBins = 4096;

__global__ void __launch_bounds__(kHistThreads) coherence_hist_kernel(
    const float* __restrict__ coh, long long batch, long long n0, int S, const int* __restrict__ t_lo,
    const int* __restrict__ t_hi, int nbins, int parts, unsigned* __restrict__ hist) {
  __shared__ unsigned h[kMaxBins];
  const int s = blockIdx.x / parts;
  const int part = blockIdx.x - s * parts;
  for (int i = threadIdx.x; i < nbins; i += kHistThreads) h[i] = 0u;
  __syncthreads();
  const long long lo = t_lo[s], hi = t_hi[s];
  const float fb = static_cast<float>(nbins);
  for (long long p = part; p < batch; p += parts) {
    const float* row = coh + (p * S + s) * n0;
#pragma unroll 4  // several loads in flight per thread
    for (long long t = lo + threadIdx.x; t < hi; t += kHistThreads) {
      const float r = row[t];
      if (!(r == r)) continue;
      int bin = static_cast<int>(floorf(r * fb));
      bin = bin < 0 ? 0 : (bin >= nbins ? nbins - 1 : bin);
      atomicAdd(&h[bin], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nbins; i += kHistThreads)
    if (h[i]) atomicAdd(&hist[static_cast<long long>(s) * nbins + i], h[i]);
}

// K15: the quantile step of pycwt's wct_significance on the device: for each scale s <
// maxscale, P = (cumsum(counts over the non-empty bins) - 1/2) / total and the level is
// np.interp(level, P, (bin + 1/2) / nbins) over those bins (clamped at both ends; a scale
// without counts keeps 0).  One workgroup per scale: an exact 64-bit integer prefix sum over
// the bins, the first non-empty bin whose P reaches the level and the non-empty bin before it
// (LDS min / max), then one thread interpolates in fp64.  Only the [maxscale] levels travel
// to the host instead of the [maxscale][nbins] counter.
constexpr int kQThreads = 256;

__global__ void __launch_bounds__(kQThreads) coherence_quantile_kernel(const unsigned* __restrict__ hist,
                                                                       int nbins, double level,
                                                                       double* __restrict__ out) {
  __shared__ unsigned long long part[kQThreads];
  __shared__ int s_hi, s_lo, s_last;
  const int s = blockIdx.x, t = threadIdx.x;
  const unsigned* h = hist + static_cast<long long>(s) * nbins;
  const int per = (nbins + kQThreads - 1) / kQThreads;
  const int b0 = min(nbins, t * per), b1 = min(nbins, b0 + per);
  unsigned long long acc = 0;
  for (int i = b0; i < b1; ++i) acc += h[i];
  part[t] = acc;
  if (t == 0) {
    s_hi = nbins;
    s_lo = -1;
    s_last = -1;
  }
  __syncthreads();
  for (int o = 1; o < kQThreads; o <<= 1) {  // inclusive scan of the per-thread sums
    const unsigned long long v = t >= o ? part[t - o] : 0ull;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const unsigned long long tot = part[kQThreads - 1];
  unsigned long long c = t > 0 ? part[t - 1] : 0ull;
  int first = nbins, last = -1;
  for (int i = b0; i < b1; ++i) {
    if (!h[i]) continue;
    c += h[i];
    last = i;
    if (first == nbins && (static_cast<double>(c) - 0.5) / static_cast<double>(tot) >= level) first = i;
  }
  if (first < nbins) atomicMin(&s_hi, first);
  if (last >= 0) atomicMax(&s_last, last);
  __syncthreads();
  const int hi = s_hi;
  for (int i = b0; i < b1 && i < hi; ++i)  // the last non-empty bin before hi
    if (h[i]) atomicMax(&s_lo, i);
  __syncthreads();
  if (t != 0) return;
  const double nb = static_cast<double>(nbins);
  if (s_last < 0) {  // no counts at all: the level stays 0
    out[s] = 0.0;
    return;
  }
  if (hi == nbins) {  // the level lies above every P: np.interp clamps to the last point
    out[s] = (s_last + 0.5) / nb;
    return;
  }
  if (s_lo < 0) {  // at or below the first point: its value
    out[s] = (hi + 0.5) / nb;
    return;
  }
  unsigned long long clo = 0, chi = 0;  // cumulative counts through lo and hi
  for (int i = 0; i <= hi; ++i) {
    chi += h[i];
    if (i == s_lo) clo = chi;
  }
  const double td = static_cast<double>(tot);
  const double p0 = (static_cast<double>(clo) - 0.5) / td, p1 = (static_cast<double>(chi) - 0.5) / td;
  const double y0 = (s_lo + 0.5) / nb, y1 = (hi + 0.5) / nb;
  out[s] = y0 + (level - p0) * (y1 - y0) / (p1 - p0);
}

}  // namespace wtmi

using namespace wtmi;

extern "C" int wtmi_rednoise(float* out, long long ld, long long count, long long n, double g, int filtered,
                             unsigned long long seed, unsigned long long first_series, void* stream) {
  if (filtered != 0 && filtered != 1) return kErrArg;
  if (count < 0 || n < 0 || ld < n || !(g > -1.0 && g < 1.0)) return kErrArg;
  if (n > (1ll << 30)) return kErrUnsupported;
  if (count == 0 || n == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!out) return kErrArg;
  int tau = 0;
  if (g != 0.0) {
    const double tt = ceil(-2.0 / log(fabs(g)));
    if (tt > (1 << 26)) return kErrUnsupported;
    tau = static_cast<int>(tt);
  }
  if (count > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL(rednoise_kernel, dim3(static_cast<unsigned>(count)), dim3(kRnThreads), 0,
                     static_cast<hipStream_t>(stream), out, ld, count, static_cast<int>(n), filtered ? g : 0.0, tau, seed,
                     first_series);
  return launch_status();
}

extern "C" int wtmi_coherence_histogram(const float* coh, long long batch, long long n0, int n_scales,
                                        const int* t_lo, const int* t_hi, int n_hist_scales, int nbins,
                                        unsigned* hist, void* stream) {
  if (batch < 0 || n0 < 0 || n_scales < 0 || n_hist_scales < 0 || n_hist_scales > n_scales || nbins < 1)
    return kErrArg;
  if (nbins > kMaxBins) return kErrUnsupported;
  if (batch == 0 || n0 == 0 || n_hist_scales == 0) return kOk;  // empty: no-op (NULL arrays allowed)
  if (!coh || !t_lo || !t_hi || !hist) return kErrArg;
  // enough blocks to fill the chip: split each scale's pairs into parts
  long long parts = (2048 + n_hist_scales - 1) / n_hist_scales;
  if (parts > batch) parts = batch;
  if (parts < 1) parts = 1;
  const long long grid = parts * n_hist_scales;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL(coherence_hist_kernel, dim3(static_cast<unsigned>(grid)), dim3(kHistThreads), 0,
                     static_cast<hipStream_t>(stream), coh, batch, n0, n_scales, t_lo, t_hi, nbins,
                     static_cast<int>(parts), hist);
  return launch_status();
}

extern "C" int wtmi_coherence_quantile(const unsigned int* hist, int n_scales, int nbins, double level,
                                       double* out, void* stream) {
  if (n_scales < 0 || nbins < 1 || !(level >= 0.0 && level <= 1.0)) return kErrArg;
  if (n_scales == 0) return kOk;  // empty: no-op (NULL arrays allowed)
  if (!hist || !out) return kErrArg;
  hipLaunchKernelGGL(coherence_quantile_kernel, dim3(static_cast<unsigned>(n_scales)), dim3(kQThreads), 0,
                     static_cast<hipStream_t>(stream), hist, nbins, level, out);
  return launch_status();
}
