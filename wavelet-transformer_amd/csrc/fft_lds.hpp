// Workgroup-cooperative power-of-two FFT held in registers + LDS (gfx950).
//
// One row of N = 2^LOGN complex64 samples is spread over NT = N/16 threads; thread
// t holds the 16 elements at positions t + m*NT (m = 0..15) in registers.  The
// transform is a Stockham autosort FFT: a radix-16 pass straight from registers,
// then radix-16 passes and at most one trailing radix-2/4/8 pass, each reading from
// and writing to LDS (one exchange per pass after the first).  On exit the thread
// again holds positions t + m*NT, so a caller can keep a spectrum resident in
// registers across many inverse transforms (the per-scale CWT loop) and stores are
// coalesced (consecutive lanes -> consecutive samples).
//
// LDS rows are padded by one complex per 32 (index i -> i + i/32).  The gather of
// every pass >= 1 reads 32 consecutive positions per 32-lane ds_read_b64 group, which
// then sit in one 32-slot block and cover the 64 banks once (a 1-per-16 pad put lane 31
// on lane 0's banks: a 2-way conflict on every read, +50 % LDS cycles).  The price is
// a 2-way conflict on pass 0's stride-16 scatter only (lanes 2k, 2k+1 of a 16-lane
// ds_write group).  DIR = -1 forward, +1 inverse; the transform is unnormalised.
#pragma once

#include "common.hpp"

// Twiddle products: cmul2 / cmul2_conj (two packed instructions each, common.hpp) unless the
// translation unit defines WTMI_PK_TWIDDLES 0 before including this header.  The asm
// products cut the WCT kernels' VALU by 5-9 % (C4 3.27 -> 3.1 ms) but cost the store-bound
// CWT kernel ~1 % (0.792 -> 0.804 ms per C2 launch, A/B on one box; the hazard recognizer
// pads each asm result's first reader with an s_nop), so cwt.hip keeps the plain products.
// Everything that depends on the choice (this header and cwt_common.hpp's kernels' pieces)
// sits in an inline namespace named after it, so the two variants are distinct entities
// (no same-named inline function with two bodies across translation units).
#ifndef WTMI_PK_TWIDDLES
#define WTMI_PK_TWIDDLES 1
#endif
#if WTMI_PK_TWIDDLES
#define WTMI_FFT_NS fft_pk
#else
#define WTMI_FFT_NS fft_plain
#endif

namespace wtmi {
inline namespace WTMI_FFT_NS {

// cos / sin of 2*pi*m/16
__host__ __device__ constexpr float cos16(int m) {
  constexpr float c1 = 0.92387953251128674f, c2 = 0.70710678118654752f, c3 = 0.38268343236508977f;
  switch (m & 15) {
    case 0: return 1.f;  case 1: return c1;   case 2: return c2;   case 3: return c3;
    case 4: return 0.f;  case 5: return -c3;  case 6: return -c2;  case 7: return -c1;
    case 8: return -1.f; case 9: return -c1;  case 10: return -c2; case 11: return -c3;
    case 12: return 0.f; case 13: return c3;  case 14: return c2;  default: return c1;
  }
}
__host__ __device__ constexpr float sin16(int m) { return cos16(m - 4); }

template <int DIR>
__device__ __forceinline__ cpx mul_i(cpx a) {  // a * (DIR * i)
  return DIR > 0 ? a.yx * cpx{-1.f, 1.f} : a.yx * cpx{1.f, -1.f};
}

template <int DIR, int M>
__device__ __forceinline__ cpx rot16(cpx a) {  // a * exp(DIR * 2 pi i M / 16)
  constexpr int m = M & 15;
  if constexpr (m == 0) {
    return a;
  } else if constexpr (m == 4) {
    return mul_i<DIR>(a);
  } else if constexpr (m == 8) {
    return mkc(-a.x, -a.y);
  } else if constexpr (m == 12) {
    return mul_i<-DIR>(a);
  } else {
    constexpr float c = cos16(m);
    constexpr float s = DIR * sin16(m);
    return cfma(a.yy, cpx{-s, c}, a.xx * cpx{c, s});
  }
}

template <int DIR>
__device__ __forceinline__ void dft2(cpx& a, cpx& b) {
  const cpx t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

template <int DIR>
__device__ __forceinline__ void dft4(cpx& x0, cpx& x1, cpx& x2, cpx& x3) {
  // X1 = t1 + DIR i d, X3 = t1 - DIR i d with d = x1 - x3: one packed fma each
  const cpx t0 = x0 + x2, t1 = x0 - x2;
  const cpx t2 = x1 + x3, d = x1 - x3;
  constexpr float sd = static_cast<float>(DIR);
  x0 = t0 + t2;
  x2 = t0 - t2;
  x1 = cfma(d.yx, cpx{-sd, sd}, t1);
  x3 = cfma(d.yx, cpx{sd, -sd}, t1);
}

// 8-point DFT on v[0..7], natural order in and out (2 x 4 Cooley-Tukey).
template <int DIR>
__device__ __forceinline__ void dft8(cpx* v) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft2<DIR>(v[n2], v[n2 + 4]);
  v[5] = rot16<DIR, 2>(v[5]);
  v[6] = rot16<DIR, 4>(v[6]);
  v[7] = rot16<DIR, 6>(v[7]);
  dft4<DIR>(v[0], v[1], v[2], v[3]);
  dft4<DIR>(v[4], v[5], v[6], v[7]);
  cpx t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = v[i];
#pragma unroll
  for (int k1 = 0; k1 < 2; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 2 * k2] = t[4 * k1 + k2];
}

// 16-point DFT on v[0..15], natural order in and out (4 x 4 Cooley-Tukey).
template <int DIR>
__device__ __forceinline__ void dft16(cpx* v) {
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft4<DIR>(v[n2], v[n2 + 4], v[n2 + 8], v[n2 + 12]);
  v[5] = rot16<DIR, 1>(v[5]);
  v[9] = rot16<DIR, 2>(v[9]);
  v[13] = rot16<DIR, 3>(v[13]);
  v[6] = rot16<DIR, 2>(v[6]);
  v[10] = rot16<DIR, 4>(v[10]);
  v[14] = rot16<DIR, 6>(v[14]);
  v[7] = rot16<DIR, 3>(v[7]);
  v[11] = rot16<DIR, 6>(v[11]);
  v[15] = rot16<DIR, 9>(v[15]);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4<DIR>(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
  cpx t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i] = v[i];
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = t[4 * k1 + k2];
}

// dft4 with x2 = x3 = 0 (the two zero inputs fold away).
template <int DIR>
__device__ __forceinline__ void dft4_2(cpx& x0, cpx& x1, cpx& x2, cpx& x3) {
  constexpr float sd = static_cast<float>(DIR);
  const cpx a = x0, b = x1;
  x0 = a + b;
  x2 = a - b;
  x1 = cfma(b.yx, cpx{-sd, sd}, a);
  x3 = cfma(b.yx, cpx{sd, -sd}, a);
}

// 16-point DFT of v[0..15] whose inputs v[m] vanish for m >= NZ (NZ = 2, 4, 8; 16 = dft16):
// the first radix-4 stage shrinks to two-input butterflies (NZ = 8) or copies (NZ <= 4), and
// for NZ = 2 half of the twiddles and of the second stage's inputs are zero as well.
template <int DIR, int NZ>
__device__ __forceinline__ void dft16_nz(cpx* v) {
  if constexpr (NZ >= 16) {
    dft16<DIR>(v);
  } else {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
      if constexpr (NZ == 8) {
        dft4_2<DIR>(v[n2], v[n2 + 4], v[n2 + 8], v[n2 + 12]);
      } else if (n2 < NZ) {
        v[n2 + 4] = v[n2];
        v[n2 + 8] = v[n2];
        v[n2 + 12] = v[n2];
      } else {
        v[n2] = v[n2 + 4] = v[n2 + 8] = v[n2 + 12] = mkc(0.f, 0.f);
      }
    }
    v[5] = rot16<DIR, 1>(v[5]);
    v[9] = rot16<DIR, 2>(v[9]);
    v[13] = rot16<DIR, 3>(v[13]);
    if constexpr (NZ > 2) {
      v[6] = rot16<DIR, 2>(v[6]);
      v[10] = rot16<DIR, 4>(v[10]);
      v[14] = rot16<DIR, 6>(v[14]);
      v[7] = rot16<DIR, 3>(v[7]);
      v[11] = rot16<DIR, 6>(v[11]);
      v[15] = rot16<DIR, 9>(v[15]);
    }
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
      if constexpr (NZ > 2)
        dft4<DIR>(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
      else
        dft4_2<DIR>(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
    }
    cpx t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = v[i];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) v[k1 + 4 * k2] = t[4 * k1 + k2];
  }
}

template <int R, int DIR>
__device__ __forceinline__ void dft_small(cpx* v) {
  if constexpr (R == 2) {
    dft2<DIR>(v[0], v[1]);
  } else if constexpr (R == 4) {
    dft4<DIR>(v[0], v[1], v[2], v[3]);
  } else if constexpr (R == 8) {
    dft8<DIR>(v);
  } else {
    dft16<DIR>(v);
  }
}

template <int LOGN>
struct FftPlan {
  static_assert(LOGN >= 4 && LOGN <= 14, "FFT length must be 16..16384");
  static constexpr int N = 1 << LOGN;
  static constexpr int NT = N / 16;              // threads per row
  static constexpr int P16 = LOGN / 4;           // radix-16 passes
  static constexpr int REM = 1 << (LOGN % 4);    // trailing radix (1 = none)
  static constexpr int NPASS = P16 + (REM > 1 ? 1 : 0);
  static constexpr int PADN = N + N / 32 + ((N / 32) & 1);  // padded row (complex, even)
  // cached base twiddles per thread: w, w^2, w^4, w^8 per radix-16 pass >= 1.  The
  // trailing radix-R pass: butterfly q (q = 0..16/R-1) of thread t has twiddle base
  // k = t + q*NT, and exp(2 pi i k/N) = exp(2 pi i t/N) * exp(2 pi i q/16): only the
  // powers w_t, w_t^2, w_t^4 (R = 2, 4, 8 -> 1, 2, 3 bases) are kept, the q-rotation is
  // a compile-time constant.
  static constexpr int NTW_REM = REM == 2 ? 1 : (REM == 4 ? 2 : (REM == 8 ? 3 : 0));
  static constexpr int NTW = (P16 - 1) * 4 + NTW_REM;
  static constexpr int NTW_ALLOC = NTW > 0 ? NTW : 1;
  // Alternative placement (TWL = true): the radix-16 bases of passes >= 1 live in a
  // per-workgroup LDS table instead of 8 registers per pass.  Pass p (ns = 16^p) has
  // ns entries k = t mod ns; the table holds (w, w^2) at [k] and (w^4, w^8) at
  // [TWL_E + k], 16-byte entries so that consecutive lanes read conflict-free.
  static constexpr int TWL_E = P16 >= 3 ? 16 + 256 : (P16 == 2 ? 16 : 0);
  static constexpr int TWL_FLOAT4 = 2 * TWL_E;
  static constexpr int NTW_REG = NTW_REM > 0 ? NTW_REM : 1;  // registers left with TWL
  // N = 8192 (NT = 512, eight waves): the trailing radix-2 pass pairs threads t and t + 256.
  // Rows of this length number their threads so that those partners are lanes p and p + 32 of
  // one wave (fft_thread); the exchange before the tail is then one v_permlane32_swap per
  // dword instead of an LDS write + read and two barriers.
  static constexpr bool XL = LOGN == 13;
};

// Logical thread index t (the element positions t + m NT it owns) of row thread rt: the
// identity, except for XL rows: wave w's lanes 0-31 are t = 32 w .. 32 w + 31 and lanes 32-63
// t + 256 (each 32-lane half still holds consecutive t: coalesced rows, conflict-free LDS).
template <int LOGN>
__device__ __forceinline__ int fft_thread(int rt) {
  if constexpr (FftPlan<LOGN>::XL)
    return 32 * (rt >> 6) + (rt & 31) + 256 * ((rt >> 5) & 1);
  else
    return rt;
}

// XL tail exchange: after the last radix-16 pass thread t holds outputs r at positions
// (t / 256) 4096 + t mod 256 + 256 r; the radix-2 tail of thread t needs positions
// t + 512 q and t + 512 q + 4096.  With X = v[2q], Y = v[2q+1], swapping the upper half of X
// with the lower half of Y leaves (X, Y) = (x[t + 512 q], x[t + 512 q + 4096]) in every lane.
// The swaps of four such pairs (q = 4h .. 4h + 3: 8 v_permlane32_swap on disjoint VGPRs, so none
// waits on another; r04, two blocks per tail instead of eight) sit in ONE asm block: the
// compiler's hazard recognizer cannot see into inline asm, so nothing it schedules may land
// between them, and the block carries its own wait states -- 5 ahead (gfx950 needs 2 after a
// VALU write of a swapped VGPR, 4 after a v_cmpx exec write) and 2 behind (a VALU read of a swap
// result).  gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "wtmi kernels are written for gfx950 (v_permlane32_swap)"
#endif
__device__ __forceinline__ void xl_swap4(cpx* v) {
  float r[8], i[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r[k] = v[k].x;
    i[k] = v[k].y;
  }
  asm volatile(
      "s_nop 4\n\t"
      "v_permlane32_swap_b32 %0, %1\n\t"
      "v_permlane32_swap_b32 %2, %3\n\t"
      "v_permlane32_swap_b32 %4, %5\n\t"
      "v_permlane32_swap_b32 %6, %7\n\t"
      "v_permlane32_swap_b32 %8, %9\n\t"
      "v_permlane32_swap_b32 %10, %11\n\t"
      "v_permlane32_swap_b32 %12, %13\n\t"
      "v_permlane32_swap_b32 %14, %15\n\t"
      "s_nop 1"
      : "+v"(r[0]), "+v"(r[1]), "+v"(i[0]), "+v"(i[1]), "+v"(r[2]), "+v"(r[3]), "+v"(i[2]), "+v"(i[3]),
        "+v"(r[4]), "+v"(r[5]), "+v"(i[4]), "+v"(i[5]), "+v"(r[6]), "+v"(r[7]), "+v"(i[6]), "+v"(i[7]));
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = mkc(r[k], i[k]);
}

// Offset of pass p's entries in the LDS twiddle table.
__host__ __device__ constexpr int twl_base(int p) { return p <= 1 ? 0 : 16; }

__device__ __forceinline__ int lpad(int i) { return i + (i >> 5); }

// exp(+2 pi i num / den) for a power-of-two den <= 2^14: 2 num / den is exact in
// float, and sincospif is accurate to ~1 ulp -- the double-precision form cost a
// measurable share of each workgroup's start-up (8-16 fp64 sincospi per thread).
// The quotient is a power-of-two scaling (ldexp): exact, and no IEEE division sequence
// where den is not a compile-time constant (the LDS twiddle-table fill).
__device__ __forceinline__ cpx expi_frac(int num, int den) {
  num &= den - 1;
  float s, c;
  sincospif(ldexpf(static_cast<float>(num), 1 - __builtin_ctz(den)), &s, &c);
  return mkc(c, s);
}

// Per-thread base twiddles (inverse sign; the forward transform conjugates them).
template <int LOGN>
__device__ __forceinline__ void fft_twiddles(cpx* tw, int t) {
  using P = FftPlan<LOGN>;
  int ns = 16;
#pragma unroll
  for (int p = 1; p < P::P16; ++p) {
    const int k = t & (ns - 1);
    const int M = ns * 16;
    tw[4 * (p - 1) + 0] = expi_frac(k, M);
    tw[4 * (p - 1) + 1] = expi_frac(2 * k, M);
    tw[4 * (p - 1) + 2] = expi_frac(4 * k, M);
    tw[4 * (p - 1) + 3] = expi_frac(8 * k, M);
    ns *= 16;
  }
  if constexpr (P::REM > 1) {
    constexpr int base = 4 * (P::P16 - 1);
#pragma unroll
    for (int e = 0; e < P::NTW_REM; ++e) tw[base + e] = expi_frac(t << e, P::N);
  }
}

// TWL variant: the trailing-pass bases only (registers), see FftPlan::TWL_E.
template <int LOGN>
__device__ __forceinline__ void fft_twiddles_tail(cpx* tw, int t) {
  using P = FftPlan<LOGN>;
  if constexpr (P::REM > 1) {
#pragma unroll
    for (int e = 0; e < P::NTW_REM; ++e) tw[e] = expi_frac(t << e, P::N);
  }
}

// Fill the LDS twiddle table (all threads of the workgroup; caller syncs before use).
template <int LOGN>
__device__ __forceinline__ void fft_twiddle_table(float4* tab, int tid, int nthreads) {
  using P = FftPlan<LOGN>;
  for (int i = tid; i < P::TWL_E; i += nthreads) {
    const int M = i < 16 ? 256 : 4096;  // pass 1: 16 * 16, pass 2: 256 * 16
    const int k = i < 16 ? i : i - 16;
    const cpx w1 = expi_frac(k, M), w2 = expi_frac(2 * k, M);
    const cpx w4 = expi_frac(4 * k, M), w8 = expi_frac(8 * k, M);
    tab[i] = make_float4(w1.x, w1.y, w2.x, w2.y);
    tab[P::TWL_E + i] = make_float4(w4.x, w4.y, w8.x, w8.y);
  }
}

template <int DIR>
__device__ __forceinline__ cpx twd(cpx w) { return DIR > 0 ? w : cconj(w); }

// Hide a value from loop-invariant code motion: keeps only the base twiddles live
// across a caller's loop instead of all 15 derived powers (+ swapped copies for
// packed math), which otherwise pushes the CWT kernel to 256 VGPRs.
__device__ __forceinline__ cpx opaque(cpx w) {
  asm volatile("" : "+v"(w.x), "+v"(w.y));
  return w;
}

constexpr bool kPkTwiddles = WTMI_PK_TWIDDLES != 0;

// (plain products) v[r] *= w^r for r = 1..NZ-1 from the bases w, w^2, w^4, w^8 (inputs r >= NZ are zero
// and stay untouched; NZ = 16: all 15).
template <int DIR, int NZ>
__device__ __forceinline__ void apply_tw16_w_nz_plain(cpx* v, cpx w1, cpx w2, cpx w4, cpx w8) {
  w1 = twd<DIR>(w1);
  if constexpr (NZ > 2) {
    w2 = twd<DIR>(w2);
    const cpx w3 = cmul(w1, w2);
    v[2] = cmul(v[2], w2);
    v[3] = cmul(v[3], w3);
    if constexpr (NZ > 4) {
      w4 = twd<DIR>(w4);
      const cpx w5 = cmul(w4, w1), w6 = cmul(w4, w2), w7 = cmul(w4, w3);
      v[4] = cmul(v[4], w4);
      v[5] = cmul(v[5], w5);
      v[6] = cmul(v[6], w6);
      v[7] = cmul(v[7], w7);
      if constexpr (NZ > 8) {
        w8 = twd<DIR>(w8);
        v[8] = cmul(v[8], w8);
        v[9] = cmul(v[9], cmul(w8, w1));
        v[10] = cmul(v[10], cmul(w8, w2));
        v[11] = cmul(v[11], cmul(w8, w3));
        v[12] = cmul(v[12], cmul(w8, w4));
        v[13] = cmul(v[13], cmul(w8, w5));
        v[14] = cmul(v[14], cmul(w8, w6));
        v[15] = cmul(v[15], cmul(w8, w7));
      }
    }
  }
  v[1] = cmul(v[1], w1);
}

// (plain products) Trailing radix-R pass, butterfly Q: v[r] *= (w_t * exp(2 pi i Q/16))^r, r = 1..R-1, from
// the bases b = (w_t, w_t^2, w_t^4) (inverse sign; DIR < 0 conjugates).
template <int R, int DIR, int Q>
__device__ __forceinline__ void apply_tw_tail_plain(cpx* v, const cpx* b) {
  if constexpr (R == 2) {
    v[1] = cmul(v[1], rot16<DIR, Q>(twd<DIR>(b[0])));
  } else if constexpr (R == 4) {
    const cpx w1 = rot16<DIR, Q>(twd<DIR>(b[0]));
    const cpx w2 = rot16<DIR, 2 * Q>(twd<DIR>(b[1]));
    v[1] = cmul(v[1], w1);
    v[2] = cmul(v[2], w2);
    v[3] = cmul(v[3], cmul(w1, w2));
  } else {
    const cpx w1 = rot16<DIR, Q>(twd<DIR>(b[0]));
    const cpx w2 = rot16<DIR, 2 * Q>(twd<DIR>(b[1]));
    const cpx w4 = rot16<DIR, 4 * Q>(twd<DIR>(b[2]));
    const cpx w3 = cmul(w1, w2);
    v[1] = cmul(v[1], w1);
    v[2] = cmul(v[2], w2);
    v[3] = cmul(v[3], w3);
    v[4] = cmul(v[4], w4);
    v[5] = cmul(v[5], cmul(w4, w1));
    v[6] = cmul(v[6], cmul(w4, w2));
    v[7] = cmul(v[7], cmul(w4, w3));
  }
}

// v[r] *= w^r for r = 1..NZ-1 from the bases w, w^2, w^4, w^8 (inputs r >= NZ are zero
// and stay untouched; NZ = 16: all 15).  The powers are derived in the inverse sign and the
// forward transform multiplies by their conjugates (cmul2_conj): no conjugation of the bases.
template <int DIR>
__device__ __forceinline__ cpx twmul(cpx v, cpx w) { return DIR > 0 ? cmul2(v, w) : cmul2_conj(v, w); }

template <int DIR, int NZ>
__device__ __forceinline__ void apply_tw16_w_nz(cpx* v, cpx w1, cpx w2, cpx w4, cpx w8) {
  if constexpr (!kPkTwiddles) {
    apply_tw16_w_nz_plain<DIR, NZ>(v, w1, w2, w4, w8);
    return;
  }
  if constexpr (NZ > 2) {
    const cpx w3 = cmul2(w1, w2);
    v[2] = twmul<DIR>(v[2], w2);
    v[3] = twmul<DIR>(v[3], w3);
    if constexpr (NZ > 4) {
      const cpx w5 = cmul2(w4, w1), w6 = cmul2(w4, w2), w7 = cmul2(w4, w3);
      v[4] = twmul<DIR>(v[4], w4);
      v[5] = twmul<DIR>(v[5], w5);
      v[6] = twmul<DIR>(v[6], w6);
      v[7] = twmul<DIR>(v[7], w7);
      if constexpr (NZ > 8) {
        v[8] = twmul<DIR>(v[8], w8);
        v[9] = twmul<DIR>(v[9], cmul2(w8, w1));
        v[10] = twmul<DIR>(v[10], cmul2(w8, w2));
        v[11] = twmul<DIR>(v[11], cmul2(w8, w3));
        v[12] = twmul<DIR>(v[12], cmul2(w8, w4));
        v[13] = twmul<DIR>(v[13], cmul2(w8, w5));
        v[14] = twmul<DIR>(v[14], cmul2(w8, w6));
        v[15] = twmul<DIR>(v[15], cmul2(w8, w7));
      }
    }
  }
  v[1] = twmul<DIR>(v[1], w1);
}

template <int DIR>
__device__ __forceinline__ void apply_tw16_w(cpx* v, cpx w1, cpx w2, cpx w4, cpx w8) {
  apply_tw16_w_nz<DIR, 16>(v, w1, w2, w4, w8);
}

template <int DIR, int NZ = 16>
__device__ __forceinline__ void apply_tw16(cpx* v, const cpx* b) {
  apply_tw16_w_nz<DIR, NZ>(v, opaque(b[0]), opaque(b[1]), opaque(b[2]), opaque(b[3]));
}

// Same from the LDS table: entry k of pass p.  The asm barrier keeps the two reads
// inside the caller's loop (their LDS region is never written, so LICM would
// otherwise hoist them and keep the 8 values live in registers).
template <int DIR, int E, int NZ = 16>
__device__ __forceinline__ void apply_tw16_lds(cpx* v, const float4* tab, int idx) {
  asm volatile("" : "+v"(idx));
  const float4 a = tab[idx], b = tab[E + idx];
  apply_tw16_w_nz<DIR, NZ>(v, mkc(a.x, a.y), mkc(a.z, a.w), mkc(b.x, b.y), mkc(b.z, b.w));
}

// Trailing radix-R pass, butterfly Q: v[r] *= (w_t * exp(2 pi i Q/16))^r, r = 1..R-1, from
// the bases b = (w_t, w_t^2, w_t^4) (inverse sign; DIR < 0 multiplies by the conjugates:
// conj(w) exp(-2 pi i Q/16) = conj(w exp(2 pi i Q/16))).
template <int R, int DIR, int Q>
__device__ __forceinline__ void apply_tw_tail(cpx* v, const cpx* b) {
  if constexpr (!kPkTwiddles) {
    apply_tw_tail_plain<R, DIR, Q>(v, b);
  } else if constexpr (R == 2) {
    v[1] = twmul<DIR>(v[1], rot16<1, Q>(b[0]));
  } else if constexpr (R == 4) {
    const cpx w1 = rot16<1, Q>(b[0]);
    const cpx w2 = rot16<1, 2 * Q>(b[1]);
    v[1] = twmul<DIR>(v[1], w1);
    v[2] = twmul<DIR>(v[2], w2);
    v[3] = twmul<DIR>(v[3], cmul2(w1, w2));
  } else {
    const cpx w1 = rot16<1, Q>(b[0]);
    const cpx w2 = rot16<1, 2 * Q>(b[1]);
    const cpx w4 = rot16<1, 4 * Q>(b[2]);
    const cpx w3 = cmul2(w1, w2);
    v[1] = twmul<DIR>(v[1], w1);
    v[2] = twmul<DIR>(v[2], w2);
    v[3] = twmul<DIR>(v[3], w3);
    v[4] = twmul<DIR>(v[4], w4);
    v[5] = twmul<DIR>(v[5], cmul2(w4, w1));
    v[6] = twmul<DIR>(v[6], cmul2(w4, w2));
    v[7] = twmul<DIR>(v[7], cmul2(w4, w3));
  }
}

template <int R, int DIR, int Q>
__device__ __forceinline__ void tail_butterflies(cpx* v, const cpx* b) {
  if constexpr (Q > 0) {
    tail_butterflies<R, DIR, Q - 1>(v, b);
    apply_tw_tail<R, DIR, Q - 1>(v + (Q - 1) * R, b);
    dft_small<R, DIR>(v + (Q - 1) * R);
  }
}

// In-place FFT of one row.  v[m] holds position t + m*NT on entry and exit.
// lds: this row's region of buffer 0; bufstride: offset (in cpx) of buffer 1
// when NBUF == 2.  par: running buffer parity (NBUF == 2), shared by all calls of
// the workgroup in the same order.  Every thread of the workgroup must call this
// the same number of times (it contains __syncthreads()).
//
// START > 0 enters at radix-16 pass START with v[r] already holding that pass's
// inputs (band-pruned inverse transforms, see band_entry below); the passes before
// it are skipped.
template <int LOGN, int DIR, int NBUF, bool TWL = false, int START = 0, int NZ = 16>
__device__ __forceinline__ void fft_row(cpx (&v)[16], cpx* __restrict__ lds, int bufstride,
                                        const cpx* tw, int t, int& par,
                                        const float4* twl = nullptr) {
  using P = FftPlan<LOGN>;
  static_assert(START == 0 || (START < P::P16 && NBUF == 1), "pruned entry: radix-16 pass, 1 buffer");
  constexpr bool kAligned = (P::NT % 32) == 0;  // strides are multiples of 32 -> pad is additive
  if constexpr (START == 0) {
    dft16_nz<DIR, NZ>(v);  // NZ < 16: inputs v[m], m >= NZ, are zero (caller's guarantee)
    if constexpr (P::NPASS == 1) return;
    cpx* buf = lds + (NBUF == 2 ? par * bufstride : 0);
    if constexpr (NBUF == 1) __syncthreads();
    cpx* w = buf + 16 * t + (t >> 1);  // lpad(16 t + r) = 16 t + t/2 + r  (r < 16)
#pragma unroll
    for (int r = 0; r < 16; ++r) w[r] = v[r];
    __syncthreads();
  }
  const int pt = lpad(t);
#pragma unroll
  for (int p = (START > 1 ? START : 1); p < P::NPASS; ++p) {
    const int ns = 1 << (4 * p);
    const bool last = (p == P::NPASS - 1);
    const cpx* rbuf = lds + (NBUF == 2 ? par * bufstride : 0);
    if (p < P::P16) {
      if (p != START) {
        if constexpr (kAligned) {
          const cpx* rb = rbuf + pt;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = rb[r * (P::NT + P::NT / 32)];
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = rbuf[lpad(t + r * P::NT)];
        }
        if constexpr (NBUF == 2) par ^= 1;
      }
      if (START > 0 && p == START) {  // entry pass of a pruned row: inputs r >= NZ are zero
        if constexpr (TWL)
          apply_tw16_lds<DIR, P::TWL_E, NZ>(v, twl, twl_base(p) + (t & (ns - 1)));
        else
          apply_tw16<DIR, NZ>(v, tw + 4 * (p - 1));
        dft16_nz<DIR, NZ>(v);
      } else {
        if constexpr (TWL)
          apply_tw16_lds<DIR, P::TWL_E>(v, twl, twl_base(p) + (t & (ns - 1)));
        else
          apply_tw16<DIR>(v, tw + 4 * (p - 1));
        dft16<DIR>(v);
      }
      if (!last && !(P::XL && NBUF == 1 && p == P::P16 - 1)) {  // (XL: the tail swaps in registers)
        cpx* wbuf = lds + (NBUF == 2 ? par * bufstride : 0);
        const int idxD = (t / ns) * ns * 16 + (t & (ns - 1));
        if constexpr (NBUF == 1) __syncthreads();
        cpx* wb = wbuf + lpad(idxD);
        if (ns >= 32) {  // r*ns is a multiple of 32: the pad is additive
#pragma unroll
          for (int r = 0; r < 16; ++r) wb[r * (ns + ns / 32)] = v[r];
        } else {  // ns = 16: idxD mod 32 < 16, so lpad(idxD + 16 r) = lpad(idxD) + 16 r + r/2
#pragma unroll
          for (int r = 0; r < 16; ++r) wb[16 * r + (r >> 1)] = v[r];
        }
        __syncthreads();
      }
    } else {
      constexpr int R = P::REM > 1 ? P::REM : 16;
      constexpr int Q = 16 / R;
      constexpr int tb = TWL ? 0 : 4 * (P::P16 - 1);
      if constexpr (P::XL && NBUF == 1) {
        static_assert(R == 2, "XL rows end with a radix-2 pass");
        static_assert(Q == 8, "XL tail: 8 radix-2 butterflies per thread");
        xl_swap4(v);
        xl_swap4(v + 8);
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if constexpr (kAligned) {
              const int off = q * P::NT + r * (P::N / R);
              v[q * R + r] = rbuf[pt + off + (off >> 5)];
            } else {
              v[q * R + r] = rbuf[lpad(t + q * P::NT + r * (P::N / R))];
            }
          }
        if constexpr (NBUF == 2) par ^= 1;
      }
      cpx tbase[P::NTW_REM > 0 ? P::NTW_REM : 1];
#pragma unroll
      for (int e = 0; e < P::NTW_REM; ++e) tbase[e] = opaque(tw[tb + e]);
      tail_butterflies<R, DIR, Q>(v, tbase);
      // register q*R + r holds position t + (q + r*Q)*NT
      cpx o[16];
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int r = 0; r < R; ++r) o[q + r * Q] = v[q * R + r];
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = o[m];
    }
  }
}

// Band-pruned entry (inverse transforms of spectra that vanish outside bins [0, N/16^Q)).
// If only bins k < N/16^Q are non-zero, passes 0..Q-1 of fft_row merely replicate
// values: pass Q's input at thread t is, for r = 0..15,
//   v[r] = x[(t >> 4Q) + r * (NT >> 4Q)]
// (pass p writes its 16 outputs to idxD = (t / 16^p) 16^(p+1) + t mod 16^p + 16^p r, all equal
// to the single non-zero input when the band is that narrow).  The caller's thread t holds
// bin t (its m = 0 element) in y; bins are exchanged through lds[0 .. N/16^Q) (one b64 write
// per thread, 16 broadcast reads), and fft_row<..., START = Q> takes it from there.
// Saves Q radix-16 passes (butterflies, twiddles, Q-1 LDS exchanges, 15/16 of one).
template <int LOGN, int Q, int NZ = 16>
__device__ __forceinline__ void band_entry(cpx (&v)[16], cpx y, cpx* __restrict__ lds, int t) {
  using P = FftPlan<LOGN>;
  static_assert(Q >= 1 && Q < P::P16 && (P::NT % (1 << (4 * Q))) == 0, "band entry");
  constexpr int KB = P::N >> (4 * Q);
  constexpr int STEP = P::NT >> (4 * Q);
  __syncthreads();  // the previous transform's readers are done with lds
  if (t < KB) lds[t] = y;
  __syncthreads();
  const int base = t >> (4 * Q);
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = r < NZ ? lds[base + r * STEP] : mkc(0.f, 0.f);
}

}  // inline namespace WTMI_FFT_NS
}  // namespace wtmi
