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
#include <type_traits>

#include "common.hpp"

namespace wtmi {

constexpr int kMaxTaps = 128;
constexpr int kModwtMaxN = 16384;          // one workgroup, series in LDS
constexpr long long kModwtLongMaxN = 1ll << 30;  // per-level launches (int sample index)
constexpr int kModwtMaxPerThread = 16;  // scalars per thread (n <= 16 * block)

struct FilterBank {
  float h[kMaxTaps];  // applied to the detail path (dec_hi / sqrt2)
  float g[kMaxTaps];  // scaling path (dec_lo / sqrt2)
};

__device__ __forceinline__ int wrap(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

// 2^(j-1) mod n without a 64-bit division while 2^(j-1) < n (every level of n >= 2^J).
__device__ __forceinline__ int dilation_mod(int j, int n) {
  if (j <= 31) {
    const unsigned p = 1u << (j - 1);
    if (p < static_cast<unsigned>(n)) return static_cast<int>(p);
  }
  return static_cast<int>((1ll << (j - 1)) % n);
}

// Scalar tap offsets (dq * l) mod ng, l = 0..L-1, by repeated addition (dq < ng).
template <int L>
__device__ __forceinline__ void tap_offsets(int dq, int ng, int (&off)[L]) {
  off[0] = 0;
#pragma unroll
  for (int l = 1; l < L; ++l) {
    const int o = off[l - 1] + dq;
    off[l] = o >= ng ? o - ng : o;
  }
}

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
#pragma unroll 4  // several loads in flight per thread (a plain strided loop waits on each)
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
#pragma unroll 4
  for (int i = tid; i < n; i += T) V[i] = keepV ? win[static_cast<long long>(level) * n + i] : 0.f;
  for (int j = level; j >= 1; --j) {
    const bool useW = (keep >> (j - 1)) & 1ull;
    if (useW) {
      const float* wrow = win + static_cast<long long>(j - 1) * n;
#pragma unroll 4
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

// ---------------------------------------------------------------------------------
// Fast path: n % 4 == 0, L = 8 (db4, the reference's wavelet).  Threads own groups of
// 4 consecutive samples (float4).  Levels j >= 3 have a dilation that is a multiple
// of 4, so every tap is one aligned ds_read_b128; levels 1 and 2 read a register
// window of 3 / 5 aligned float4 blocks and form all taps from it.

// Padded LDS index of float4 group q (synthesis V: one pad group per 8).  The dilation-chain
// mapping puts lanes M = 8 groups apart for dq = 1, a 128-byte stride: an 8-way bank conflict on
// every ds_read_b128 / ds_write_b128 without the pad (63 % of LDS cycles were conflicts).
__device__ __forceinline__ int vpad(int q) { return q + (q >> 3); }

template <int L, int DM, bool FWD, bool PAD = false>
__device__ __forceinline__ void window_taps(const float4* __restrict__ V4, int q, int ng,
                                            const FilterBank& fb, float4& a, float4& b) {
  // FWD: taps at p - DM*l (analysis); else p + DM*l (synthesis).  Window of NB blocks.
  constexpr int SPAN = (L - 1) * DM;        // samples reached beyond the group
  constexpr int NB = (SPAN + 3) / 4 + 1;    // aligned float4 blocks covering it
  float f[4 * NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    int qs = FWD ? q - (NB - 1) + u : q + u;
    qs = qs < 0 ? qs + ng : (qs >= ng ? qs - ng : qs);
    const float4 v = V4[PAD ? vpad(qs) : qs];
    f[4 * u] = v.x; f[4 * u + 1] = v.y; f[4 * u + 2] = v.z; f[4 * u + 3] = v.w;
  }
  float ra[4] = {0.f, 0.f, 0.f, 0.f}, rb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float hl = fb.h[l], gl = fb.g[l];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = FWD ? 4 * (NB - 1) + i - DM * l : i + DM * l;
      ra[i] = fmaf(hl, f[idx], ra[i]);
      rb[i] = fmaf(gl, f[idx], rb[i]);
    }
  }
  a = make_float4(ra[0], ra[1], ra[2], ra[3]);
  b = make_float4(rb[0], rb[1], rb[2], rb[3]);
}

// Materialise a value here: stops the compiler from sinking the math that produced it
// past a barrier into its (conditional) consumer, which keeps every LDS operand live.
__device__ __forceinline__ void pin4(float4& v) {
  asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
}

// acc += c s as two packed v_pk_fma_f32 (the compiler left 83 % of these as scalar v_fmac_f32:
// twice the VALU issue of the synthesis' tap loops)
using f2v = float __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void fma4(float4& acc, float c, const float4& s) {
  const f2v cc = {c, c};
  const f2v lo = __builtin_elementwise_fma(cc, f2v{s.x, s.y}, f2v{acc.x, acc.y});
  const f2v hi = __builtin_elementwise_fma(cc, f2v{s.z, s.w}, f2v{acc.z, acc.w});
  acc = make_float4(lo.x, lo.y, hi.x, hi.y);
}

// Analysis: V_{j-1} in LDS (n floats), each thread owns GROUPS float4 groups (stride T).
// The level loop re-derives its addresses from an opaque copy of tid and pins each
// result before the barrier; without both, the compiler hoists per-group address math
// out of the level loop and sinks the tap FMAs past the barrier, keeping every LDS
// operand live (256 VGPRs + spills).
// CHAIN > 0: levels with a dilation of dq >= CHAIN whole groups use the dilation-chain
// mapping of syn_level_chain (taps m-L+1 .. m of the thread's chain, M+L-1 LDS reads for
// M outputs instead of L*M); W_j stores then run along the chain (coalesced for
// dq >= 64 groups, dq-group runs below: whole 128-byte lines from dq = 8).
// (the W_j stores as buffer stores at the default, nt or sc1 policy measured within noise of
// these plain stores, r05: profiles/r05/nt_policy_ab.txt)
template <int L, int GROUPS, int T, int CHAIN = 0>
__global__ void __launch_bounds__(T) modwt_vec_kernel(const float* __restrict__ x, long long ld,
                                                      int n, int level, FilterBank fb,
                                                      float* __restrict__ w) {
  extern __shared__ __attribute__((aligned(16))) float4 V4[];
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const int ng = n >> 2;
  const float4* xin = reinterpret_cast<const float4*>(x + b * ld);
  float* wout = w + b * static_cast<long long>(level + 1) * n;
  {
    float4 xv[GROUPS];  // every load in flight before the first LDS write
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) xv[k] = ld_nt4(&xin[min(tid + k * T, ng - 1)]);
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      pin4(xv[k]);  // not sunk into the guarded store (that re-serialises the loads)
      if (tid + k * T < ng) V4[tid + k * T] = xv[k];
    }
  }
  __syncthreads();
  for (int j = 1; j <= level; ++j) {
    const int dm = dilation_mod(j, n);
    float4* wrow = reinterpret_cast<float4*>(wout + static_cast<long long>(j - 1) * n);
    int tl = tid;
    asm volatile("" : "+v"(tl));
    float4 vreg[GROUPS];
    if (CHAIN > 0 && (dm & 3) == 0 && GROUPS * T == ng) {
      const int dq = dm >> 2;
      if (dq >= CHAIN && (dq & (dq - 1)) == 0 && ng % (GROUPS * dq) == 0 && (ng & (ng - 1)) == 0) {
        const int dqlog = __builtin_ctz(dq);
        const int q0 = (tl >> dqlog) * GROUPS * dq + (tl & (dq - 1));
        float4 vv[GROUPS + L - 1];  // chain elements q0 + (k - L + 1) dq
#pragma unroll
        for (int k = 0; k < GROUPS + L - 1; ++k)
          vv[k] = V4[(q0 + (k - (L - 1)) * dq + (L - 1) * ng) & (GROUPS * T - 1)];  // ng = GROUPS*T
#pragma unroll
        for (int m = 0; m < GROUPS; ++m) {
          float4 aw = make_float4(0.f, 0.f, 0.f, 0.f), av = aw;
#pragma unroll
          for (int l = 0; l < L; ++l) {
            fma4(aw, fb.h[l], vv[m + L - 1 - l]);
            fma4(av, fb.g[l], vv[m + L - 1 - l]);
          }
          wrow[q0 + m * dq] = aw;
          vreg[m] = av;
          pin4(vreg[m]);
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < GROUPS; ++m) V4[q0 + m * dq] = vreg[m];
        __syncthreads();
        continue;
      }
    }
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      const int q = min(tl + k * T, ng - 1);
      float4 aw, av;
      if (dm == 1) {
        window_taps<L, 1, true>(V4, q, ng, fb, aw, av);
      } else if (dm == 2) {
        window_taps<L, 2, true>(V4, q, ng, fb, aw, av);
      } else {
        aw = make_float4(0.f, 0.f, 0.f, 0.f);
        av = aw;
        int off[L];
        tap_offsets<L>(dm >> 2, ng, off);
#pragma unroll
        for (int l = 0; l < L; ++l) {
          int qs = q - off[l];
          if (qs < 0) qs += ng;
          const float4 s = V4[qs];
          fma4(aw, fb.h[l], s);
          fma4(av, fb.g[l], s);
        }
      }
      if (tl + k * T < ng) wrow[q] = aw;
      vreg[k] = av;
      pin4(vreg[k]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      const int q = tl + k * T;
      if (q < ng) V4[q] = vreg[k];
    }
    __syncthreads();
  }
  float4* vrow = reinterpret_cast<float4*>(wout + static_cast<long long>(level) * n);
  for (int q = tid; q < ng; q += T) vrow[q] = V4[q];
}

// Synthesis: V and W_j in LDS (128 KiB: one workgroup per CU).  GROUPS float4 groups
// per thread (GROUPS * 4 * threads >= n).  PREFETCH: the next row W_{j-1} is loaded
// into registers while level j computes (costs 4*GROUPS VGPRs); otherwise each level
// starts with a direct global -> LDS copy of W_j.
template <int L, int GROUPS, int T, bool PAD = false>
__device__ __forceinline__ void syn_level(const float4* __restrict__ V4, const float4* __restrict__ W4,
                                          int ng, int dm, float wsel, const FilterBank& fb, int tid,
                                          float4 (&vreg)[GROUPS]) {
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (dm == 1 || dm == 2) {
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      int q = min(tid + k * T, ng - 1);
      asm volatile("" : "+v"(q));  // keep tap addresses out of LICM (VGPR blow-up)
      float4 av, aw, bw, dummy;
      if (dm == 1) {
        window_taps<L, 1, false, PAD>(V4, q, ng, fb, dummy, av);
        window_taps<L, 1, false>(W4, q, ng, fb, aw, bw);
      } else {
        window_taps<L, 2, false, PAD>(V4, q, ng, fb, dummy, av);
        window_taps<L, 2, false>(W4, q, ng, fb, aw, bw);
      }
      vreg[k] = make_float4(fmaf(wsel, aw.x, av.x), fmaf(wsel, aw.y, av.y), fmaf(wsel, aw.z, av.z),
                            fmaf(wsel, aw.w, av.w));
      pin4(vreg[k]);
    }
  } else {
    int off[L];
    tap_offsets<L>(dm >> 2, ng, off);
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      int q = min(tid + k * T, ng - 1);
      asm volatile("" : "+v"(q));  // keep tap addresses out of LICM (VGPR blow-up)
      float4 acc = z4;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        int qs = q + off[l];
        if (qs >= ng) qs -= ng;
        fma4(acc, fb.g[l], V4[PAD ? vpad(qs) : qs]);
        fma4(acc, wsel * fb.h[l], W4[qs]);
      }
      vreg[k] = acc;
      pin4(vreg[k]);
    }
  }
}

// Synthesis level along dilation chains (levels with a dilation of dq >= 1 float4
// groups).  Thread (c, r) owns the M groups q = c*M*dq + m*dq + r (m = 0..M-1): output
// m needs taps m .. m+L-1 of the same chain, so the thread loads M+L-1 taps of W_j
// (global) and of V_j (LDS) once and slides over them -- (M+L-1)/M loads per output
// instead of L (the 8x re-read of W_j through L2 is what bounds the stride-T form).
// Lanes with consecutive r read consecutive groups: coalesced for dq >= 64 groups,
// dq-group contiguous runs below that.  NG = M*T groups, a power of two (the wrap is a
// mask: a per-lane '% ng' was ~30 % of the kernel's VALU instructions); NG % (M*dq) == 0.
template <int M>
__device__ __forceinline__ int chain_q0(int tid, int dqlog) {
  return (tid >> dqlog) * M * (1 << dqlog) + (tid & ((1 << dqlog) - 1));
}

template <int L, int M, int NG, int K0 = 0, int K1 = M + L - 1>
__device__ __forceinline__ void chain_load_w(const float4* __restrict__ W4, int dqlog, int tid,
                                             float4 (&wv)[M + L - 1]) {
  const int dq = 1 << dqlog;
  const int q0 = chain_q0<M>(tid, dqlog);
#pragma unroll
  for (int k = K0; k < K1; ++k) wv[k] = W4[(q0 + k * dq) & (NG - 1)];  // taps may wrap >1x
}

template <int L, int M, int NG, bool PAD>
__device__ __forceinline__ int chain_compute(const float4* __restrict__ V4, const float4 (&wv)[M + L - 1],
                                             int dqlog, const float (&hs)[L], const FilterBank& fb,
                                             int tid, float4 (&vreg)[M]) {
  const int dq = 1 << dqlog;
  const int q0 = chain_q0<M>(tid, dqlog);
  float4 vv[M + L - 1];
#pragma unroll
  for (int k = 0; k < M + L - 1; ++k) {
    const int qv = (q0 + k * dq) & (NG - 1);
    vv[k] = V4[PAD ? vpad(qv) : qv];
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      fma4(acc, fb.g[l], vv[m + l]);
      fma4(acc, hs[l], wv[m + l]);
    }
    vreg[m] = acc;
    pin4(vreg[m]);
  }
  return q0;
}

template <int L, int M, int NG, bool PAD = false>
__device__ __forceinline__ int syn_level_chain(const float4* __restrict__ V4, const float4* __restrict__ W4,
                                               int dqlog, const float (&hs)[L],
                                               const FilterBank& fb, int tid, float4 (&vreg)[M]) {
  static_assert((NG & (NG - 1)) == 0, "chain levels need a power-of-two group count");
  float4 wv[M + L - 1];
  chain_load_w<L, M, NG>(W4, dqlog, tid, wv);
  return chain_compute<L, M, NG, PAD>(V4, wv, dqlog, hs, fb, tid, vreg);
}

// MODE 0: W_j copied global -> LDS at the start of each level (rows of <= 8192 samples).
// MODE 3: W_j taps read straight from global memory (L1/L2); LDS holds V only (padded, n
//         floats), so two workgroups fit per CU and one's loads overlap the other's math;
//         levels with a whole-group dilation run along dilation chains (syn_level_chain:
//         each W_j / V_j tap loaded ~2x instead of 8x).
// (r01 also measured: W_{j-1} prefetched into registers during level j, W via LDS with
// chains, and chain taps loaded one level ahead -- all slower or spilling at the 128-VGPR
// budget of two workgroups per CU)
template <int L, int GROUPS, int T, int MODE>
__global__ void __launch_bounds__(T, 1)
    imodwt_vec_kernel(const float* __restrict__ w, int n, int level, FilterBank fb, unsigned long long keep,
                      float* __restrict__ x, long long ld_out) {
  static_assert(MODE == 0 || MODE == 3, "synthesis modes: 0 (W via LDS) or 3 (W global + chains)");
  constexpr bool PAD = MODE == 3;  // V alone in LDS: padded (vpad), see window_taps
  constexpr bool CHAINS = MODE == 3;
  constexpr int NG = GROUPS * T;
  constexpr int NGC = (NG & (NG - 1)) == 0 ? NG : 1;
  extern __shared__ __attribute__((aligned(16))) float4 sm4[];
  const int ng = n >> 2;
  float4* V4 = sm4;
  float4* W4 = sm4 + ng;
  auto vp = [](int q) { return PAD ? vpad(q) : q; };
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const float* win = w + b * static_cast<long long>(level + 1) * n;
  const bool keepV = (keep >> level) & 1ull;
  {
    // all GROUPS loads in flight before the first LDS write (a runtime-trip loop waited on
    // each load in turn: 8 serialised HBM round trips per workgroup)
    const float4* vr = reinterpret_cast<const float4*>(win + static_cast<long long>(level) * n);
    float4 vin[GROUPS];
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) vin[k] = vr[min(tid + k * T, ng - 1)];
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      const float4 v = vin[k];
      const float4 s = make_float4(keepV ? v.x : 0.f, keepV ? v.y : 0.f, keepV ? v.z : 0.f,
                                   keepV ? v.w : 0.f);
      if (tid + k * T < ng) V4[vp(tid + k * T)] = s;
    }
  }
  // chain level of dilation dm (log2 of dq in groups), or -1
  auto chain_log = [&](int dm) {
    if ((dm & 3) == 0 && NG == ng && (NG & (NG - 1)) == 0) {
      const int dq = dm >> 2;
      // chains from dq = 2 groups: at dq = 1 the chain lanes stride 128 B and every load
      // instruction touches 64 lines; the stride form's coalesced loads win there (C3 A/B on
      // one box: 2.82 -> 2.79 ms; chains from dq 4: 2.85, from 8: 2.93)
      if (dq >= 2 && (dq & (dq - 1)) == 0 && ng % (GROUPS * dq) == 0) return __builtin_ctz(dq);
    }
    return -1;
  };
  for (int j = level; j >= 1; --j) {
    const float4* wr = reinterpret_cast<const float4*>(win + static_cast<long long>(j - 1) * n);
    if (MODE == 0)
      for (int q = tid; q < ng; q += T) W4[q] = wr[q];
    __syncthreads();
    const float wsel = ((keep >> (j - 1)) & 1ull) ? 1.f : 0.f;  // masked rows count as 0
    const int dm = dilation_mod(j, n);
    int tl = tid;
    asm volatile("" : "+v"(tl));  // per-level copy: keeps address math out of LICM
    float4 vreg[GROUPS];
    const int dqlog = CHAINS ? chain_log(dm) : -1;
    if (dqlog >= 0) {
      float hs[L];
#pragma unroll
      for (int l = 0; l < L; ++l) hs[l] = wsel * fb.h[l];
      const int q0 = syn_level_chain<L, GROUPS, NGC, PAD>(V4, wr, dqlog, hs, fb, tl, vreg);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) V4[vp(q0 + (k << dqlog))] = vreg[k];
      continue;
    }
    syn_level<L, GROUPS, T, PAD>(V4, MODE == 3 ? wr : W4, ng, dm, wsel, fb, tl, vreg);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      const int q = tl + k * T;
      if (q < ng) V4[vp(q)] = vreg[k];
    }
  }
  __syncthreads();
  float4* xo = reinterpret_cast<float4*>(x + b * ld_out);
  for (int q = tid; q < ng; q += T) xo[q] = V4[vp(q)];
}

// ---------------------------------------------------------------------------------
// Synthesis, hybrid (n = 4 * GROUPS * T = 8192 or 16384; V padded in LDS, two workgroups
// per CU).  Levels with a dilation of dq >= 2 whole groups run MODE 3's dilation chains
// (V taps from LDS, W_j taps straight from L2).  The low levels (dm = 1, 2 samples and
// dq = 1 group) stage W_j through LDS instead: their global tap reads were 8 dependent
// round trips per level (one per owned group) or, along chains, 64 cache lines per load.
//   V phase: acc = sum_l g_l V_j[. + dm l]   (LDS; W_j's coalesced loads in flight)
//   barrier, W_j -> LDS over V_j, barrier, W phase: acc += sum_l h_l W_j[. + dm l]
//   barrier, acc -> LDS as V_{j-1}
// Rows whose keep bit is clear are not applied (low levels still fetch a row: a predicated
// load is a branch, and the stack arrays that came with it cost more than the bytes).
template <int L, int H, int NG, bool FIRST>
__device__ __forceinline__ void chain_pass(const float4* __restrict__ S4, int q0, int dq, int base,
                                           const float* __restrict__ c, float4* acc) {
  float4 t[H + L - 1];
#pragma unroll
  for (int k = 0; k < H + L - 1; ++k) t[k] = S4[vpad((q0 + (base + k) * dq) & (NG - 1))];
#pragma unroll
  for (int m = 0; m < H; ++m) {
    float4 a = FIRST ? make_float4(0.f, 0.f, 0.f, 0.f) : acc[m];
#pragma unroll
    for (int l = 0; l < L; ++l) fma4(a, c[l], t[m + l]);
    acc[m] = a;
  }
}

template <int L, int DM>
__device__ __forceinline__ float4 window_acc(const float4* __restrict__ S4, int q, int ngm,
                                             const float* __restrict__ c, float4 acc) {
  constexpr int NB = ((L - 1) * DM + 3) / 4 + 1;
  float f[4 * NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const float4 v = S4[vpad((q + u) & ngm)];
    f[4 * u] = v.x; f[4 * u + 1] = v.y; f[4 * u + 2] = v.z; f[4 * u + 3] = v.w;
  }
  float r[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
  for (int l = 0; l < L; ++l)
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = fmaf(c[l], f[i + DM * l], r[i]);
  return make_float4(r[0], r[1], r[2], r[3]);
}

using v4f = float __attribute__((ext_vector_type(4)));

template <int L, int GROUPS, int T, int H, int CG>
__global__ void __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(2 * T / 256)))
    imodwt_hyb_kernel(const float* __restrict__ w, int n, int level, FilterBank fb, unsigned long long keep,
                      float* __restrict__ x, long long ld_out) {
  constexpr int NG = GROUPS * T;
  static_assert((NG & (NG - 1)) == 0 && GROUPS % H == 0, "power-of-two rows, H | GROUPS");
  extern __shared__ __attribute__((aligned(16))) float4 sm4[];
  float4* S4 = sm4;
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const float* win = w + b * static_cast<long long>(level + 1) * n;
  auto row4 = [&](int r) { return reinterpret_cast<const float4*>(win + static_cast<long long>(r) * n); };
  auto kept = [&](int r) { return ((keep >> r) & 1ull) != 0; };
  {
    const float4* vr = row4(level);
    float4 vin[GROUPS];
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) vin[k] = ld_nt4(&vr[tid + k * T]);
    const bool keepV = kept(level);
#pragma unroll
    for (int k = 0; k < GROUPS; ++k) {
      const float4 v = vin[k];
      S4[vpad(tid + k * T)] = make_float4(keepV ? v.x : 0.f, keepV ? v.y : 0.f, keepV ? v.z : 0.f,
                                          keepV ? v.w : 0.f);
    }
  }
  for (int j = level; j >= 1; --j) {
    const bool useW = kept(j - 1);
    const float4* wr = row4(j - 1);
    const int dm = dilation_mod(j, n);
    int tl = tid;
    asm volatile("" : "+v"(tl));  // per-level copy: keeps address math out of LICM
    const int dq = dm >> 2;
    const bool chain = (dm & 3) == 0 && dq >= 1 && (dq & (dq - 1)) == 0 && NG % (GROUPS * dq) == 0;
    const int dqlog = chain ? __builtin_ctz(dq) : 0;
    float4 acc[GROUPS];
    __syncthreads();  // S4 = V_j
    if (chain && dq >= CG) {
      float hs[L];
      const float wsel = useW ? 1.f : 0.f;
#pragma unroll
      for (int l = 0; l < L; ++l) hs[l] = wsel * fb.h[l];
      const int q0 = syn_level_chain<L, GROUPS, NG, true>(S4, wr, dqlog, hs, fb, tl, acc);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) S4[vpad(q0 + (k << dqlog))] = acc[k];
      continue;
    }
    v4f wreg[GROUPS];  // native vectors: float4 copies of loads became stack arrays
    {
      const v4f* wv = reinterpret_cast<const v4f*>(useW ? wr : row4(level));
      // buffer loads off the wave-uniform row, streaming policy (each W_j is read once): C3
      // 2.55 -> 2.47 ms against plain global loads (2.50 as default-policy buffer loads)
      const __amdgpu_buffer_rsrc_t rw = uniform_rsrc(wv);
#pragma unroll
      for (int k = 0; k < GROUPS; ++k)
        wreg[k] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rw, 16 * tid, 16 * k * T, kNt));
    }
    const int q0 = chain ? chain_q0<GROUPS>(tl, dqlog) : 0;
    auto phase = [&](const float* c, bool first) {
      if (chain) {
#pragma unroll
        for (int h = 0; h < GROUPS; h += H) {
          if (first)
            chain_pass<L, H, NG, true>(S4, q0, dq, h, c, acc + h);
          else
            chain_pass<L, H, NG, false>(S4, q0, dq, h, c, acc + h);
        }
      } else {
#pragma unroll
        for (int k = 0; k < GROUPS; ++k) {
          int q = tl + k * T;
          asm volatile("" : "+v"(q));
          const float4 a0 = first ? make_float4(0.f, 0.f, 0.f, 0.f) : acc[k];
          if (dm == 1) {
            acc[k] = window_acc<L, 1>(S4, q, NG - 1, c, a0);
          } else if (dm == 2) {
            acc[k] = window_acc<L, 2>(S4, q, NG - 1, c, a0);
          } else {  // whole groups beyond the chain range (dq > T) or dm = 0 (2^(j-1) = 0 mod n)
            float4 a = a0;
#pragma unroll
            for (int l = 0; l < L; ++l) fma4(a, c[l], S4[vpad((q + dq * l) & (NG - 1))]);
            acc[k] = a;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) pin4(acc[k]);
    };
    phase(fb.g, true);
    if (useW) {
      __syncthreads();  // V_j reads done
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) S4[vpad(tid + k * T)] = make_float4(wreg[k].x, wreg[k].y, wreg[k].z, wreg[k].w);
      __syncthreads();  // S4 = W_j
      phase(fb.h, false);
    }
    __syncthreads();  // reads done
    if (chain) {
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) S4[vpad(q0 + (k << dqlog))] = acc[k];
    } else {
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) S4[vpad(tl + k * T)] = acc[k];
    }
  }
  __syncthreads();
  float4* xo = reinterpret_cast<float4*>(x + b * ld_out);
  float4 o[GROUPS];
#pragma unroll
  for (int k = 0; k < GROUPS; ++k) o[k] = S4[vpad(tid + k * T)];
#pragma unroll
  for (int k = 0; k < GROUPS; ++k) xo[tid + k * T] = o[k];
}

// ---------------------------------------------------------------------------------
// Long series (n > 16384: V no longer fits one workgroup's LDS).  One launch per level,
// one thread per (series, sample); the L taps of V_{j-1} come through L1/L2 (they lie
// within (L-1) 2^(j-1) samples of each other), V ping-pongs between a [batch][n] scratch
// row and the output's V_J row, arranged so that the last level lands in row J.
__global__ void __launch_bounds__(256) modwt_level_kernel(const float* __restrict__ vin, long long ld_in,
                                                          long long batch, int n, int dm, int L,
                                                          FilterBank fb, float* __restrict__ wout,
                                                          long long ld_w, float* __restrict__ vout,
                                                          long long ld_v) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= batch * n) return;
  const long long b = idx / n;
  const int t = static_cast<int>(idx - b * n);
  const float* v = vin + b * ld_in;
  float aw = 0.f, av = 0.f;
  int p = t;
  for (int l = 0; l < L; ++l) {  // taps at (t - dm l) mod n, dm < n
    const float s = v[p];
    aw = fmaf(fb.h[l], s, aw);
    av = fmaf(fb.g[l], s, av);
    p -= dm;
    if (p < 0) p += n;
  }
  wout[b * ld_w + t] = aw;
  vout[b * ld_v + t] = av;
}

__global__ void __launch_bounds__(256) imodwt_level_kernel(const float* __restrict__ w, long long ld_w,
                                                           const float* __restrict__ vin, long long ld_in,
                                                           long long batch, int n, int dm, int L, float wsel,
                                                           float vsel, FilterBank fb, float* __restrict__ vout,
                                                           long long ld_out) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  if (idx >= batch * n) return;
  const long long b = idx / n;
  const int t = static_cast<int>(idx - b * n);
  const float* wr = w + b * ld_w;
  const float* vr = vin + b * ld_in;
  float acc = 0.f;
  int p = t;
  for (int l = 0; l < L; ++l) {  // taps at (t + dm l) mod n
    acc = fmaf(vsel * fb.g[l], vr[p], acc);
    acc = fmaf(wsel * fb.h[l], wr[p], acc);
    p += dm;
    if (p >= n) p -= n;
  }
  vout[b * ld_out + t] = acc;
}

static int modwt_long(const float* x, long long ld, long long batch, int n, const FilterBank& fb, int L,
                      int level, float* w, float* scratch, hipStream_t st) {
  const long long grid = (batch * n + 255) / 256;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  const long long ldw = static_cast<long long>(level + 1) * n;
  const float* vin = x;
  long long ldin = ld;
  for (int j = 1; j <= level; ++j) {
    const int dm = static_cast<int>((1ll << (j - 1)) % n);
    // V_j into row J when (level - j) is even, else into the [batch][n] scratch
    const bool to_row = (level - j) % 2 == 0;
    float* vout = to_row ? w + static_cast<long long>(level) * n : scratch;
    const long long ldv = to_row ? ldw : static_cast<long long>(n);
    hipLaunchKernelGGL(modwt_level_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, vin, ldin,
                       batch, n, dm, L, fb, w + static_cast<long long>(j - 1) * n, ldw, vout, ldv);
    const int rc = launch_status();
    if (rc != kOk) return rc;
    vin = vout;
    ldin = ldv;
  }
  return kOk;
}

static int imodwt_long(const float* w, long long batch, int n, const FilterBank& fb, int L, int level,
                       unsigned long long keep, float* x, long long ld_out, float* scratch, hipStream_t st) {
  const long long grid = (batch * n + 255) / 256;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  const long long ldw = static_cast<long long>(level + 1) * n;
  const float* vin = w + static_cast<long long>(level) * n;
  long long ldin = ldw;
  float vsel = ((keep >> level) & 1ull) ? 1.f : 0.f;  // a dropped V_J row counts as zero
  for (int j = level; j >= 1; --j) {
    const int dm = static_cast<int>((1ll << (j - 1)) % n);
    const float wsel = ((keep >> (j - 1)) & 1ull) ? 1.f : 0.f;
    // V_{j-1} into x when (j - 1) is even, else into scratch: level 1 writes x
    float* vout = ((j - 1) % 2 == 0) ? x : scratch;
    const long long ldo = ((j - 1) % 2 == 0) ? ld_out : static_cast<long long>(n);
    hipLaunchKernelGGL(imodwt_level_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st,
                       w + static_cast<long long>(j - 1) * n, ldw, vin, ldin, batch, n, dm, L, wsel, vsel,
                       fb, vout, ldo);
    const int rc = launch_status();
    if (rc != kOk) return rc;
    vin = vout;
    ldin = ldo;
    vsel = 1.f;
  }
  return kOk;
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

extern "C" long long wtmi_modwt_workspace_bytes(long long batch, long long n, int level) {
  if (batch < 0 || n < 0 || level < 1) return -1;
  if (n <= kModwtMaxN) return 0;
  // one [batch][n] float row: the analysis's and the synthesis's V ping-pong partner
  return batch * n * static_cast<long long>(sizeof(float));
}

extern "C" int wtmi_modwt(const float* x, long long ld, long long batch, long long n,
                          const double* dec_lo, const double* dec_hi, int n_taps, int level,
                          float* w, void* workspace, void* stream) {
  FilterBank fb;
  if (batch < 0 || n < 1 || ld < n || level < 1 || level > 62) return kErrArg;
  if (!make_bank(dec_lo, dec_hi, n_taps, fb)) return kErrArg;
  if (n > kModwtLongMaxN || batch > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !w) return kErrArg;
  if (n > kModwtMaxN) {
    if (!workspace) return kErrArg;
    return modwt_long(x, ld, batch, static_cast<int>(n), fb, n_taps, level, w, static_cast<float*>(workspace),
                      static_cast<hipStream_t>(stream));
  }
  const int ni = static_cast<int>(n);
  const size_t lds = static_cast<size_t>((ni + 3) & ~3) * sizeof(float);
  const int block = modwt_block(ni);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n_taps == 8 && ni >= 64 && (ni & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(w) & 15) == 0 && ni <= 16384) {
    auto launch = [&](auto kernel, int t) {
      allow_lds(kernel, lds);
      hipLaunchKernelGGL(kernel, dim3(batch), dim3(t), lds, st, x, ld, ni, level, fb, w);
    };
    const int ng = ni / 4;
    if (ng <= 256)
      launch(modwt_vec_kernel<8, 1, 256>, 256);
    else if (ng <= 512)
      launch(modwt_vec_kernel<8, 1, 512>, 512);
    else if (ng <= 1024)
      launch(modwt_vec_kernel<8, 1, 1024>, 1024);
    else if (ng <= 2048)
      launch(modwt_vec_kernel<8, 2, 1024>, 1024);
    else  // chains from dq >= 16 groups; one-process A/B on two boxes (ms): stride form 1.248 /
          // 1.264, chains from dq 8 1.200 / 1.264, from dq 16 1.200 / 1.267 (r01)
    {
      // one 1024-thread workgroup per series (4 groups per thread): 1.256 ms against 1.280 for
      // 512 threads x 8 groups and 1.263 for 256 x 16 (C3's analysis, alternating, one box,
      // r04); option modwt_ana = 1 / 2 selects the others
      if (options().modwt_ana == 1)
        launch(modwt_vec_kernel<8, 8, 512, 16>, 512);
      else if (options().modwt_ana == 2)
        launch(modwt_vec_kernel<8, 16, 256, 16>, 256);
      else
        launch(modwt_vec_kernel<8, 4, 1024, 16>, 1024);
    }
  } else if (n_taps == 8) {
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
                           float* x, long long ld_out, void* workspace, void* stream) {
  FilterBank fb;
  if (batch < 0 || n < 1 || ld_out < n || level < 1 || level > 62) return kErrArg;
  if (!make_bank(dec_lo, dec_hi, n_taps, fb)) return kErrArg;
  if (n > kModwtLongMaxN || batch > 0x7fffffffll) return kErrUnsupported;
  if (batch == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !w) return kErrArg;
  if (n > kModwtMaxN) {
    if (!workspace) return kErrArg;
    return imodwt_long(w, batch, static_cast<int>(n), fb, n_taps, level, keep_mask, x, ld_out,
                       static_cast<float*>(workspace), static_cast<hipStream_t>(stream));
  }
  const int ni = static_cast<int>(n);
  const size_t lds = 2 * static_cast<size_t>((ni + 3) & ~3) * sizeof(float);
  const int block = modwt_block(ni);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n_taps == 8 && ni >= 64 && (ni & 3) == 0 && (ld_out & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(w) & 15) == 0 && ni <= 16384) {
    auto launch = [&](auto kernel, int t) {
      allow_lds(kernel, lds);
      hipLaunchKernelGGL(kernel, dim3(batch), dim3(t), lds, st, w, ni, level, fb, keep_mask, x, ld_out);
    };
    const size_t lds_pad = (static_cast<size_t>(ni / 4) + ni / 32) * 16;  // vpad'ed V (MODE 2/3)
    auto launch_lds = [&](auto kernel, int t, size_t bytes) {
      allow_lds(kernel, bytes);
      hipLaunchKernelGGL(kernel, dim3(batch), dim3(t), bytes, st, w, ni, level, fb, keep_mask, x, ld_out);
    };
    const int ng = ni / 4;
    if (ng <= 256)
      launch(imodwt_vec_kernel<8, 1, 256, 0>, 256);
    else if (ng <= 512)
      launch(imodwt_vec_kernel<8, 1, 512, 0>, 512);
    else if (ng <= 1024)
      launch(imodwt_vec_kernel<8, 1, 1024, 0>, 1024);
    // n = 16384 / 8192: the hybrid synthesis.  r05: every level's W_j staged through LDS
    // (CG = 1024 > any dilation; r04 kept W_j taps of the chain levels dq >= 4 groups in L2).
    // FETCH per C3 launch 6.50 -> 5.91 GB = exactly the 11 rows (the L2 taps shared by
    // neighbouring chains were partly re-fetched), 1.269-1.274 -> 1.234-1.239 ms in one
    // process, 4 alternations (profiles/r05/c3_syn_cg.txt; CG 8 / 16 / 32 / 64 in between).
    // modwt_syn 2 keeps r04's CG = 4.
    else if (ng == 4096 && options().modwt_syn == 1)
      launch_lds(imodwt_hyb_kernel<8, 8, 512, 2, 1024>, 512, lds_pad);
    else if (ng == 4096 && options().modwt_syn == 2)
      launch_lds(imodwt_hyb_kernel<8, 8, 512, 2, 4>, 512, lds_pad);
    else if (ng == 2048 && options().modwt_syn == 1)
      launch_lds(imodwt_hyb_kernel<8, 4, 512, 2, 1024>, 512, lds_pad);
    else if (ng == 2048 && options().modwt_syn == 2)
      launch_lds(imodwt_hyb_kernel<8, 4, 512, 2, 4>, 512, lds_pad);
    else if (ng <= 2048)
      launch_lds(imodwt_vec_kernel<8, 2, 1024, 3>, 1024, lds_pad);
    else
      launch_lds(imodwt_vec_kernel<8, 8, 512, 3>, 512, lds_pad);
  } else if (n_taps == 8) {
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
