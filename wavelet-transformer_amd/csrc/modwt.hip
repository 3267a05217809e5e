// MODWT analysis / synthesis cascades (K3 / K4 of DESIGN.md).
//
// Replaces src/modwt.py:126-160 (modwt / imodwt built on circular_convolve_d /
// circular_convolve_s, i.e. scipy.ndimage.convolve1d(mode="wrap") over zero-stuffed
// dilated kernels, :86-123).  Same arithmetic as the textbook a-trous form
//   W_j[t] = sum_l h~_l V_{j-1}[(t - 2^{j-1} l) mod N],  V_j likewise with g~,
//   V_{j-1}[t] = sum_l h~_l W_j[(t + 2^{j-1} l) mod N] + g~_l V_j[(t + 2^{j-1} l) mod N],
// h~ = dec_hi / sqrt2, g~ = dec_lo / sqrt2, output rows [W_1 .. W_J, V_J].
// Only the L non-zero taps are touched (the reference multiplies the stuffed zeros
// too: 8 * 2^{j-1} taps per sample at level j).
//
// One workgroup per series; the whole series stays in LDS across all J levels
// (ping-pong through registers: read taps -> barrier -> write level j).  Rows of W
// are written once with coalesced 16-byte stores; x is read once.
#include "common.hpp"

namespace wtmi {

constexpr int kMaxTaps = 128;
constexpr int kModwtMaxN = 16384;
constexpr int kModwtMaxPerThread = 16;  // scalars per thread (n <= 16 * block)

struct FilterBank {
  float h[kMaxTaps];  // applied to the detail path (dec_hi / sqrt2)
  float g[kMaxTaps];  // scaling path (dec_lo / sqrt2)
};

__device__ __forceinline__ int wrap(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

// ---------------------------------------------------------------------------------
// analysis
template <int LT>
__global__ void __launch_bounds__(1024) modwt_kernel(const float* __restrict__ x, long long ld, int n,
                                                     int level, int L, FilterBank fb,
                                                     float* __restrict__ w) {
  extern __shared__ __attribute__((aligned(16))) float V[];
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const float* xin = x + b * ld;
  float* wout = w + b * static_cast<long long>(level + 1) * n;
  const int taps = LT > 0 ? LT : L;
  const bool vec = (n & 3) == 0;
  const int ng = n >> 2;
  for (int i = tid; i < n; i += T) V[i] = xin[i];
  __syncthreads();
  for (int j = 1; j <= level; ++j) {
    const int dm = static_cast<int>((1ll << (j - 1)) % n);  // dilation mod n
    float* wrow = wout + static_cast<long long>(j - 1) * n;
    float vreg[kModwtMaxPerThread];
    if (vec) {
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread / 4; ++k) {
        const int q = tid + k * T;
        if (q < ng) {
          float4 aw = make_float4(0.f, 0.f, 0.f, 0.f), av = aw;
          for (int l = 0; l < taps; ++l) {
            const int o = (dm * l) % n;
            float4 s;
            if ((o & 3) == 0) {
              int qs = q - (o >> 2);
              if (qs < 0) qs += ng;
              s = reinterpret_cast<const float4*>(V)[qs];
            } else {
              const int p0 = 4 * q - o;
              s.x = V[wrap(p0, n)];
              s.y = V[wrap(p0 + 1, n)];
              s.z = V[wrap(p0 + 2, n)];
              s.w = V[wrap(p0 + 3, n)];
            }
            const float hl = fb.h[l], gl = fb.g[l];
            aw.x = fmaf(hl, s.x, aw.x); aw.y = fmaf(hl, s.y, aw.y);
            aw.z = fmaf(hl, s.z, aw.z); aw.w = fmaf(hl, s.w, aw.w);
            av.x = fmaf(gl, s.x, av.x); av.y = fmaf(gl, s.y, av.y);
            av.z = fmaf(gl, s.z, av.z); av.w = fmaf(gl, s.w, av.w);
          }
          reinterpret_cast<float4*>(wrow)[q] = aw;
          vreg[4 * k] = av.x; vreg[4 * k + 1] = av.y; vreg[4 * k + 2] = av.z; vreg[4 * k + 3] = av.w;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread / 4; ++k) {
        const int q = tid + k * T;
        if (q < ng)
          reinterpret_cast<float4*>(V)[q] =
              make_float4(vreg[4 * k], vreg[4 * k + 1], vreg[4 * k + 2], vreg[4 * k + 3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread; ++k) {
        const int p = tid + k * T;
        if (p < n) {
          float aw = 0.f, av = 0.f;
          for (int l = 0; l < taps; ++l) {
            const int o = (dm * l) % n;
            const float s = V[wrap(p - o, n)];
            aw = fmaf(fb.h[l], s, aw);
            av = fmaf(fb.g[l], s, av);
          }
          wrow[p] = aw;
          vreg[k] = av;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread; ++k) {
        const int p = tid + k * T;
        if (p < n) V[p] = vreg[k];
      }
    }
    __syncthreads();
  }
  float* vrow = wout + static_cast<long long>(level) * n;
  if (vec) {
    for (int q = tid; q < ng; q += T) reinterpret_cast<float4*>(vrow)[q] = reinterpret_cast<const float4*>(V)[q];
  } else {
    for (int i = tid; i < n; i += T) vrow[i] = V[i];
  }
}

// ---------------------------------------------------------------------------------
// synthesis; rows whose keep bit is clear are treated as zero (MRA / smoothing)
template <int LT>
__global__ void __launch_bounds__(1024) imodwt_kernel(const float* __restrict__ w, int n, int level,
                                                      int L, FilterBank fb, unsigned long long keep,
                                                      float* __restrict__ x, long long ld_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* V = sm;
  float* Wj = sm + ((n + 3) & ~3);
  const int T = blockDim.x;
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const float* win = w + b * static_cast<long long>(level + 1) * n;
  const int taps = LT > 0 ? LT : L;
  const bool vec = (n & 3) == 0;
  const int ng = n >> 2;
  const bool keepV = (keep >> level) & 1ull;
  for (int i = tid; i < n; i += T) V[i] = keepV ? win[static_cast<long long>(level) * n + i] : 0.f;
  for (int j = level; j >= 1; --j) {
    const bool useW = (keep >> (j - 1)) & 1ull;
    if (useW) {
      const float* wrow = win + static_cast<long long>(j - 1) * n;
      for (int i = tid; i < n; i += T) Wj[i] = wrow[i];
    }
    __syncthreads();
    const int dm = static_cast<int>((1ll << (j - 1)) % n);
    float vreg[kModwtMaxPerThread];
    if (vec) {
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread / 4; ++k) {
        const int q = tid + k * T;
        if (q < ng) {
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int l = 0; l < taps; ++l) {
            const int o = (dm * l) % n;
            float4 sv, sw = make_float4(0.f, 0.f, 0.f, 0.f);
            if ((o & 3) == 0) {
              int qs = q + (o >> 2);
              if (qs >= ng) qs -= ng;
              sv = reinterpret_cast<const float4*>(V)[qs];
              if (useW) sw = reinterpret_cast<const float4*>(Wj)[qs];
            } else {
              const int p0 = 4 * q + o;
              sv.x = V[wrap(p0, n)]; sv.y = V[wrap(p0 + 1, n)];
              sv.z = V[wrap(p0 + 2, n)]; sv.w = V[wrap(p0 + 3, n)];
              if (useW) {
                sw.x = Wj[wrap(p0, n)]; sw.y = Wj[wrap(p0 + 1, n)];
                sw.z = Wj[wrap(p0 + 2, n)]; sw.w = Wj[wrap(p0 + 3, n)];
              }
            }
            const float hl = fb.h[l], gl = fb.g[l];
            acc.x = fmaf(hl, sw.x, fmaf(gl, sv.x, acc.x));
            acc.y = fmaf(hl, sw.y, fmaf(gl, sv.y, acc.y));
            acc.z = fmaf(hl, sw.z, fmaf(gl, sv.z, acc.z));
            acc.w = fmaf(hl, sw.w, fmaf(gl, sv.w, acc.w));
          }
          vreg[4 * k] = acc.x; vreg[4 * k + 1] = acc.y; vreg[4 * k + 2] = acc.z; vreg[4 * k + 3] = acc.w;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread / 4; ++k) {
        const int q = tid + k * T;
        if (q < ng)
          reinterpret_cast<float4*>(V)[q] =
              make_float4(vreg[4 * k], vreg[4 * k + 1], vreg[4 * k + 2], vreg[4 * k + 3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread; ++k) {
        const int p = tid + k * T;
        if (p < n) {
          float acc = 0.f;
          for (int l = 0; l < taps; ++l) {
            const int src = wrap(p + (dm * l) % n, n);
            acc = fmaf(fb.g[l], V[src], acc);
            if (useW) acc = fmaf(fb.h[l], Wj[src], acc);
          }
          vreg[k] = acc;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kModwtMaxPerThread; ++k) {
        const int p = tid + k * T;
        if (p < n) V[p] = vreg[k];
      }
    }
    __syncthreads();
  }
  float* xo = x + b * ld_out;
  for (int i = tid; i < n; i += T) xo[i] = V[i];
}

static int modwt_block(int n) {
  int t = (n + kModwtMaxPerThread - 1) / kModwtMaxPerThread;
  t = ((t + 63) / 64) * 64;
  return t < 64 ? 64 : (t > 1024 ? 1024 : t);
}

static bool make_bank(const double* dec_lo, const double* dec_hi, int L, FilterBank& fb) {
  if (!dec_lo || !dec_hi || L < 1 || L > kMaxTaps) return false;
  const double r = 1.0 / sqrt(2.0);
  for (int i = 0; i < kMaxTaps; ++i) {
    fb.h[i] = i < L ? static_cast<float>(dec_hi[i] * r) : 0.f;
    fb.g[i] = i < L ? static_cast<float>(dec_lo[i] * r) : 0.f;
  }
  return true;
}

template <typename K>
static void allow_lds(K kernel, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
}

}  // namespace wtmi

using namespace wtmi;

extern "C" int wtmi_modwt(const float* x, long long ld, long long batch, long long n,
                          const double* dec_lo, const double* dec_hi, int n_taps, int level,
                          float* w, void* stream) {
  FilterBank fb;
  if (!x || !w || batch < 0 || n < 1 || ld < n || level < 1 || level > 62) return kErrArg;
  if (!make_bank(dec_lo, dec_hi, n_taps, fb)) return kErrArg;
  if (n > kModwtMaxN || batch > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;
  const int ni = static_cast<int>(n);
  const size_t lds = static_cast<size_t>((ni + 3) & ~3) * sizeof(float);
  const int block = modwt_block(ni);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n_taps == 8) {
    allow_lds(modwt_kernel<8>, lds);
    hipLaunchKernelGGL(modwt_kernel<8>, dim3(batch), dim3(block), lds, st, x, ld, ni, level, n_taps, fb, w);
  } else {
    allow_lds(modwt_kernel<0>, lds);
    hipLaunchKernelGGL(modwt_kernel<0>, dim3(batch), dim3(block), lds, st, x, ld, ni, level, n_taps, fb, w);
  }
  return launch_status();
}

extern "C" int wtmi_imodwt(const float* w, long long batch, long long n, const double* dec_lo,
                           const double* dec_hi, int n_taps, int level, unsigned long long keep_mask,
                           float* x, long long ld_out, void* stream) {
  FilterBank fb;
  if (!x || !w || batch < 0 || n < 1 || ld_out < n || level < 1 || level > 62) return kErrArg;
  if (!make_bank(dec_lo, dec_hi, n_taps, fb)) return kErrArg;
  if (n > kModwtMaxN || batch > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;
  const int ni = static_cast<int>(n);
  const size_t lds = 2 * static_cast<size_t>((ni + 3) & ~3) * sizeof(float);
  const int block = modwt_block(ni);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n_taps == 8) {
    allow_lds(imodwt_kernel<8>, lds);
    hipLaunchKernelGGL(imodwt_kernel<8>, dim3(batch), dim3(block), lds, st, w, ni, level, n_taps, fb,
                       keep_mask, x, ld_out);
  } else {
    allow_lds(imodwt_kernel<0>, lds);
    hipLaunchKernelGGL(imodwt_kernel<0>, dim3(batch), dim3(block), lds, st, w, ni, level, n_taps, fb,
                       keep_mask, x, ld_out);
  }
  return launch_status();
}
