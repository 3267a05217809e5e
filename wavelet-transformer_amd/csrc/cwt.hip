// Fused Morlet CWT / cross-wavelet kernels (K1 + K2 of DESIGN.md).
//
// Replaces pycwt.cwt as called from src/cwt.py:110 (and the two cwt calls inside
// pycwt.xwt, src/xwt.py:93): N = 2^ceil(log2 n0); X = FFT(x zero-padded to N);
// W_j = IFFT(X * sqrt(2 pi s_j / dt) * pi^-1/4 * exp(-(s_j w_k - f0)^2 / 2))[:n0].
//
// One workgroup = one series (or pair) x a chunk of scales.  The forward FFT runs
// once per workgroup and the spectrum stays in registers (16 complex per thread);
// each scale row is an analytic-filter multiply + in-LDS inverse FFT + a fused
// epilogue writing any of {W (complex64), |W|^2, |W|^2 / signif_j} (cross mode:
// {W1 W2*, |W1 W2*|^2, ratio, phase arrows u = sin(angle), v = cos(angle)}).
// The Morlet filter is evaluated in-register: no filter bank is read from HBM.  The same
// kernels instantiated with VAR = 1 serve pycwt's other mothers (Paul, DOG / Mexican hat:
// mother_filter, full transforms -- the band pruning is Morlet's).
// plain twiddle products in this file's FFTs (fft_lds.hpp, kPkTwiddles)
#define WTMI_PK_TWIDDLES 0
#include "cwt_common.hpp"
#include "long_path.hpp"

namespace wtmi {

// cache policy of the CWT's output row stores (build knob for A/B runs): sc1 (aux 16), C2
// 0.775 -> 0.766 ms and C5 203.0 -> 201.4 ms against the default policy; nt (aux 2) was 2-3 %
// slower (profiles/r05/nt_policy_ab.txt)
#ifndef WTMI_CWT_ST_AUX
#define WTMI_CWT_ST_AUX 16
#endif
constexpr int kCwtStAux = WTMI_CWT_ST_AUX;

enum : int { kOutW = 1, kOutPow = 2, kOutSig = 4, kOutUV = 8 };

template <int LOGN, int KIND, bool FULL>
__device__ __forceinline__ void store_row(const cpx (&v)[16], const CwtArgs& a, long long rowbase,
                                          float sg, int t) {
  using P = FftPlan<LOGN>;
  cpx* pw_ = (KIND & kOutW) ? a.out_w + rowbase : nullptr;
  float* pp_ = (KIND & kOutPow) ? a.out_pow + rowbase : nullptr;
  float* ps_ = (KIND & kOutSig) ? a.out_sig + rowbase : nullptr;
  float* pu_ = (KIND & kOutUV) ? a.out_u + rowbase : nullptr;
  float* pv_ = (KIND & kOutUV) ? a.out_v + rowbase : nullptr;
  // Rows whose owner is a whole wave (NT >= 64 -> the row, hence rowbase, is wave-uniform)
  // go through buffer stores: SGPR row base + one voffset VGPR.  A padded row's positions
  // past n0 get voffset = the extent itself, so the range check drops them whether or not it
  // counts the SGPR offset (wct.hip put_row).
  constexpr bool kBuf = P::NT >= kWave;
  if constexpr (kBuf) {
    __amdgpu_buffer_rsrc_t rw, rp, rs, ru, rv;
    const int n8 = 8 * a.n0, n4 = 4 * a.n0;
    if constexpr (KIND & kOutW) rw = uniform_rsrc(pw_, n8);
    if constexpr (KIND & kOutPow) rp = uniform_rsrc(pp_, n4);
    if constexpr (KIND & kOutSig) rs = uniform_rsrc(ps_, n4);
    if constexpr (KIND & kOutUV) {
      ru = uniform_rsrc(pu_, n4);
      rv = uniform_rsrc(pv_, n4);
    }
    // (the selects depend only on t and n0: an opaque copy of t keeps the compiler from
    // hoisting all 16 out of the scale loop -- 16 live VGPRs, 108 spilled bytes at LOGN 13)
    int tt = t;
    if constexpr (!FULL) asm volatile("" : "+v"(tt));
    auto vo = [&](int m, int sz) { return (FULL || tt + m * P::NT < a.n0) ? sz * t : sz * a.n0; };
#pragma unroll
    for (int m = 0; m < 16; ++m)
      if constexpr (KIND & kOutW) buf_st<kCwtStAux>(v[m], rw, vo(m, 8), 8 * m * P::NT);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const float pw = cabs2(v[m]);
      const int o4 = vo(m, 4);
      if constexpr (KIND & kOutPow) buf_st<kCwtStAux>(pw, rp, o4, 4 * m * P::NT);
      if constexpr (KIND & kOutSig) buf_st<kCwtStAux>(pw * sg, rs, o4, 4 * m * P::NT);
      if constexpr (KIND & kOutUV) {
        const float r = sqrtf(pw);
        buf_st<kCwtStAux>(r > 0.f ? v[m].y / r : 0.f, ru, o4, 4 * m * P::NT);
        buf_st<kCwtStAux>(r > 0.f ? v[m].x / r : 1.f, rv, o4, 4 * m * P::NT);
      }
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int pos = t + m * P::NT;
    if (FULL || pos < a.n0) {
      if constexpr (KIND & kOutW) pw_[pos] = v[m];
      const float pw = cabs2(v[m]);
      if constexpr (KIND & kOutPow) pp_[pos] = pw;
      if constexpr (KIND & kOutSig) ps_[pos] = pw * sg;
      if constexpr (KIND & kOutUV) {
        const float r = sqrtf(pw);
        pu_[pos] = r > 0.f ? v[m].y / r : 0.f;
        pv_[pos] = r > 0.f ? v[m].x / r : 1.f;
      }
    }
  }
}

template <int LOGN, bool FULL>
__device__ __forceinline__ void store_any(const cpx (&v)[16], const CwtArgs& a, int kind,
                                          long long rowbase, float sg, int t) {
  switch (kind) {
#define WTMI_K(K) case K: store_row<LOGN, K, FULL>(v, a, rowbase, sg, t); break;
    WTMI_K(1) WTMI_K(2) WTMI_K(3) WTMI_K(4) WTMI_K(5) WTMI_K(6) WTMI_K(7) WTMI_K(8)
    WTMI_K(9) WTMI_K(10) WTMI_K(11) WTMI_K(12) WTMI_K(13) WTMI_K(14) WTMI_K(15)
#undef WTMI_K
    default: break;
  }
}

// W row of one scale: Morlet filter + inverse FFT, entering the FFT at pass q when the
// filtered spectrum is confined to bins [0, N/16^q) (band_regime / band_entry), with the
// entry pass narrowed to its NZ non-zero inputs (row_code).
template <int LOGN, int NBUF, bool TWL, int Q, int NZ>
__device__ __forceinline__ void inverse_row_v(cpx (&v)[16], const cpx (&X)[16], cpx prm, float f0,
                                              cpx* my, int bufstride, const cpx* tw, int t, int& par,
                                              const float4* twl) {
  if constexpr (Q == 0) {
    if constexpr (NZ < 16)
      morlet_filter_nz<LOGN, NZ>(v, X, prm, f0, t);
    else
      morlet_filter<LOGN>(v, X, prm, f0, t);
    fft_row<LOGN, 1, NBUF, TWL, 0, NZ>(v, my, bufstride, tw, t, par, twl);
  } else {
    band_entry<LOGN, Q, NZ>(v, morlet_bin0(X[0], prm, f0, t), my, t);
    fft_row<LOGN, 1, NBUF, TWL, Q, NZ>(v, my, bufstride, tw, t, par, twl);
  }
}

template <int LOGN, int NBUF, bool TWL>
__device__ __forceinline__ void inverse_row(cpx (&v)[16], const cpx (&X)[16], cpx prm, float f0,
                                            int code, cpx* my, int bufstride, const cpx* tw, int t,
                                            int& par, const float4* twl) {
  using P = FftPlan<LOGN>;
#define WTMI_ROW(Q, NZ) inverse_row_v<LOGN, NBUF, TWL, Q, NZ>(v, X, prm, f0, my, bufstride, tw, t, par, twl)
  if constexpr (NBUF == 1 && P::P16 >= 2 && (P::NT % 16) == 0) {
    switch (code) {
      case 1: WTMI_ROW(0, 8); return;
      case 2: WTMI_ROW(0, 4); return;
      case 3: WTMI_ROW(0, 2); return;
      case 4: WTMI_ROW(1, 16); return;
      case 5: WTMI_ROW(1, 8); return;
      case 6: WTMI_ROW(1, 4); return;
      case 7: WTMI_ROW(1, 2); return;
      default: break;
    }
    if constexpr (P::P16 >= 3 && (P::NT % 256) == 0) {
      switch (code) {
        case 8: WTMI_ROW(2, 16); return;
        case 9: WTMI_ROW(2, 8); return;
        case 10: WTMI_ROW(2, 4); return;
        case 11: WTMI_ROW(2, 2); return;
        default: break;
      }
    }
  }
  WTMI_ROW(0, 16);
#undef WTMI_ROW
}

template <int LOGN, int NBUF, int MODE, int VAR = 0>
__global__ void __launch_bounds__((CwtGeom<LOGN, MODE, VAR>::BLOCK), (NBUF == 2 ? 2 : CwtGeom<LOGN, MODE, VAR>::MINW)) cwt_morlet_kernel(CwtArgs a) {
  using P = FftPlan<LOGN>;
  using G = CwtGeom<LOGN, MODE, VAR>;
  // per-scale table (alpha, log2 c, 1/signif, -) in LDS: the scale loop must not issue
  // global loads -- a load's vmcnt wait would also wait for every store of the
  // previous row (loads and stores retire in order on the same counter).
  __shared__ float4 lds4[(NBUF * G::ROWS * P::PADN) / 2 + G::MAXCHUNK + G::TWL_F4];
  cpx* lds = reinterpret_cast<cpx*>(lds4);
  float4* prm_tab = lds4 + (NBUF * G::ROWS * P::PADN) / 2;
  float4* twl = prm_tab + G::MAXCHUNK;
  const int tid = threadIdx.x;
  const int g = tid / P::NT;
  const int t = fft_thread<LOGN>(tid - g * P::NT);
  const long long blk = blockIdx.x;
  const long long b = blk / a.nchunks;
  const int ch = static_cast<int>(blk - b * a.nchunks);
  const int j0 = ch * a.chunk;
  const int j1 = min(a.S, j0 + a.chunk);
  cpx* my = lds + g * P::PADN;
  constexpr int bufstride = G::ROWS * P::PADN;

  for (int i = tid; i < j1 - j0; i += G::BLOCK) {
    const double s = a.scales[j0 + i];
    cpx mp = morlet_params(s, a.dt, P::N);
    if constexpr (VAR == 1)  // log2(sqrt(2 pi s / dt) / N) + the mother's normalisation
      mp.y = static_cast<float>(log2(sqrt(2.0 * kPi * s / a.dt) / static_cast<double>(P::N)) + a.mlnorm);
    const float sg = a.sigscale ? static_cast<float>(a.sigscale[b * a.sig_ld + j0 + i]) : 0.f;
    const int code = (NBUF == 1 && VAR == 0) ? row_code<LOGN>(s, a.dt, a.f0, a.prune) : 0;
    prm_tab[i] = make_float4(mp.x, mp.y, sg, static_cast<float>(code));
  }

  constexpr bool TWL = G::TWL;
  cpx tw[TWL ? P::NTW_REG : P::NTW_ALLOC];
  if constexpr (TWL) {
    fft_twiddle_table<LOGN>(twl, tid, G::BLOCK);
    fft_twiddles_tail<LOGN>(tw, t);
    __syncthreads();
  } else {
    fft_twiddles<LOGN>(tw, t);
  }
  int par = 0;

  __shared__ float red[G::BLOCK / kWave];
  cpx X[16];
  load_series<LOGN>(X, a.x, a.affine, b, a.ld, a.n0, t);
  const float mu = demean_row<LOGN>(X, a.n0, t, red);
  fft_row<LOGN, -1, NBUF, TWL>(X, my, bufstride, tw, t, par, twl);
  add_mean_spectrum<LOGN>(X, mu, a.n0, t);
  cpx X2[MODE == 1 ? 16 : 1];
  if constexpr (MODE == 1) {
    load_series<LOGN>(X2, a.x2, a.affine2, b, a.ld, a.n0, t);
    __syncthreads();  // red reuse
    const float mu2 = demean_row<LOGN>(X2, a.n0, t, red);
    fft_row<LOGN, -1, NBUF, TWL>(X2, my, bufstride, tw, t, par, twl);
    add_mean_spectrum<LOGN>(X2, mu2, a.n0, t);
  }
  __syncthreads();  // prm_tab visible (the FFT barriers may be absent for N = 16)

  const int kind = (a.out_w ? kOutW : 0) | (a.out_pow ? kOutPow : 0) | (a.out_sig ? kOutSig : 0) |
                   (a.out_u ? kOutUV : 0);
  const bool full = a.n0 == P::N;
  const float f0 = static_cast<float>(a.f0);
  const int iters = (j1 - j0 + G::ROWS - 1) / G::ROWS;
  for (int it = 0; it < iters; ++it) {
    const int jl = it * G::ROWS + g;
    const bool valid = jl < j1 - j0;
    const float4 prm4 = prm_tab[valid ? jl : 0];
    const cpx prm = mkc(prm4.x, prm4.y);
    // the iteration's band regime: the narrowest-band common to its rows (workgroup-uniform,
    // the transforms contain barriers)
    // the iteration's row code: the widest band among its rows (workgroup-uniform, the
    // transforms contain barriers)
    int q = 12;
#pragma unroll
    for (int gg = 0; gg < G::ROWS; ++gg) {
      const int jj = it * G::ROWS + gg;
      if (jj < j1 - j0) q = min(q, static_cast<int>(prm_tab[jj].w));
    }
    cpx v[16];
    auto inverse = [&](const cpx (&Xs)[16]) {
      if constexpr (VAR == 1) {
        mother_filter<LOGN>(v, Xs, prm, a, t);
        fft_row<LOGN, 1, NBUF, TWL>(v, my, bufstride, tw, t, par, twl);
      } else {
        inverse_row<LOGN, NBUF, TWL>(v, Xs, prm, f0, q, my, bufstride, tw, t, par, twl);
      }
    };
    inverse(X);
    if constexpr (MODE == 1) {
      cpx w1[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) w1[m] = v[m];
      inverse(X2);
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = cmul2_conj(w1[m], v[m]);
    }
    if (!valid) continue;
    const int j = j0 + jl;
    const long long rowbase = (b * a.S + j) * static_cast<long long>(a.n0);
    const float sg = prm4.z;
    if (full)
      store_any<LOGN, true>(v, a, kind, rowbase, sg, t);
    else
      store_any<LOGN, false>(v, a, kind, rowbase, sg, t);
  }
}

// Direct-DFT path for N < 16 (n0 <= 8): one thread per output sample.
template <int MODE>
__global__ void __launch_bounds__(256) cwt_direct_kernel(CwtArgs a, int N) {
  const long long idx = blockIdx.x * 256ll + threadIdx.x;
  const long long total = a.batch * a.S * a.n0;
  if (idx >= total) return;
  const int tpos = static_cast<int>(idx % a.n0);
  const long long rj = idx / a.n0;
  const int j = static_cast<int>(rj % a.S);
  const long long b = rj / a.S;
  const double s = a.scales[j];
  const double alpha = s * 2.0 * kPi / (N * a.dt);
  // pycwt's sqrt(s * ftfreqs[1] * N): fftfreq(2)[1] = -1/2, so a 2-point row is NaN there too
  const double lc = N == 2 ? __builtin_nan("") : log2(sqrt(2.0 * kPi * s / a.dt) / N) + a.mlnorm;
  double2 w[2] = {make_double2(0, 0), make_double2(0, 0)};
  for (int which = 0; which < (MODE == 1 ? 2 : 1); ++which) {
    const float* row = (which ? a.x2 : a.x) + b * a.ld;
    const double* af = which ? a.affine2 : a.affine;
    double acc_re = 0, acc_im = 0;
    for (int k = 0; k < N; ++k) {
      double xr = 0, xi = 0;  // X[k]
      for (int n = 0; n < a.n0; ++n) {
        double val = row[n];
        if (af) val = static_cast<float>((val - af[3 * b] - af[3 * b + 1] * n) * af[3 * b + 2]);
        double sn, cs;
        sincospi(-2.0 * ((static_cast<long long>(k) * n) % N) / N, &sn, &cs);
        xr += val * cs;
        xi += val * sn;
      }
      const int kk = k < N / 2 ? k : k - N;
      const double2 psi = mother_psi_d(alpha * kk, lc, a);
      double sn, cs;
      sincospi(2.0 * ((static_cast<long long>(k) * tpos) % N) / N, &sn, &cs);
      const double yr = xr * cs - xi * sn, yi = xr * sn + xi * cs;  // X[k] e^{2 pi i k t / N}
      acc_re += psi.x * yr - psi.y * yi;
      acc_im += psi.x * yi + psi.y * yr;
    }
    w[which] = make_double2(acc_re, acc_im);
  }
  cpx v = mkc(static_cast<float>(w[0].x), static_cast<float>(w[0].y));
  if constexpr (MODE == 1) {
    const cpx w2 = mkc(static_cast<float>(w[1].x), static_cast<float>(w[1].y));
    v = cmul2_conj(v, w2);
  }
  const long long o = idx;
  if (a.out_w) a.out_w[o] = v;
  const float pw = cabs2(v);
  if (a.out_pow) a.out_pow[o] = pw;
  if (a.out_sig) a.out_sig[o] = pw * static_cast<float>(a.sigscale[b * a.sig_ld + j]);
  if constexpr (MODE == 1) {
    if (a.out_u) {
      const float r = sqrtf(pw);
      a.out_u[o] = r > 0.f ? v.y / r : 0.f;
      a.out_v[o] = r > 0.f ? v.x / r : 1.f;
    }
  }
}

static int log2_ceil(long long n) {
  int l = 0;
  while ((1ll << l) < n) ++l;
  return l;
}

template <int LOGN, int NBUF, int MODE, int VAR = 0>
static int launch_fft_cwt(CwtArgs& a, hipStream_t st) {
  using G = CwtGeom<LOGN, MODE, VAR>;
  // Scale chunking: enough workgroups to fill 256 CUs several times, while keeping
  // at least 4 row-iterations per workgroup to amortise the forward FFT.
  const int rows = G::ROWS;
  // Few, long workgroups: each one's start-up (twiddles, forward FFT) amortises over
  // more scales.  Measured (ms): C2 (LOGN 12, 3 WG/CU) 1024 WG 0.871, 2048 0.839,
  // 4096 0.860; C5 chunk (LOGN 13, 2 WG/CU) 512 30.9, 1024 30.86, 2048 31.2, 4096 32.9.
  // Small batches (a strong-scaling shard) get fewer, longer workgroups: 2 per series, at
  // least 512.  C2 shapes on one box (ms, target 2048 -> this rule): 128 series 0.128 -> 0.115,
  // 512 series 0.411 -> 0.402, 256 a tie, 1024 unchanged (2048 either way).
  const long long by_batch = 2 * a.batch < 512 ? 512 : 2 * a.batch;
  const int cap = LOGN >= 13 ? 1024 : 2048;
  const int target = options().cwt_target_wg > 0 ? options().cwt_target_wg
                                                 : static_cast<int>(by_batch < cap ? by_batch : cap);
  long long want = (target + a.batch - 1) / a.batch;
  const int max_chunks = (a.S + 4 * rows - 1) / (4 * rows);
  int nch = static_cast<int>(want < 1 ? 1 : want);
  if (nch > max_chunks) nch = max_chunks < 1 ? 1 : max_chunks;
  int chunk = (a.S + nch - 1) / nch;
  chunk = ((chunk + rows - 1) / rows) * rows;
  if (chunk > G::MAXCHUNK) chunk = G::MAXCHUNK;
  nch = (a.S + chunk - 1) / chunk;
  a.nchunks = nch;
  a.chunk = chunk;
  // 2: band-pruned rows and narrowed first passes; 1: band-pruned rows only; 0: full FFTs
  // (other mothers: full FFTs -- the band criteria are the Morlet filter's)
  a.prune = VAR == 1 ? 0 : options().cwt_prune;
  const long long grid = a.batch * nch;
  if (grid > 0x7fffffffll) return kErrUnsupported;
  hipLaunchKernelGGL((cwt_morlet_kernel<LOGN, NBUF, MODE, VAR>), dim3(static_cast<unsigned>(grid)),
                     dim3(G::BLOCK), 0, st, a);
  return launch_status();
}

template <int MODE>
static int dispatch(CwtArgs& a, hipStream_t st) {
  if (a.batch == 0 || a.S == 0 || a.n0 == 0) return kOk;
  const int logn = log2_ceil(a.n0);
  if (logn < 4) {
    const int N = 1 << logn;
    const long long total = a.batch * a.S * a.n0;
    const long long blocks = (total + 255) / 256;
    hipLaunchKernelGGL((cwt_direct_kernel<MODE>), dim3(static_cast<unsigned>(blocks)), dim3(256),
                       0, st, a, N);
    return launch_status();
  }
#define WTMI_CASE(L)                                                                     \
  case L:                                                                                \
    return a.mother ? launch_fft_cwt<L, 1, MODE, 1>(a, st) : launch_fft_cwt<L, 1, MODE>(a, st);
  switch (logn) {
    WTMI_CASE(4) WTMI_CASE(5) WTMI_CASE(6) WTMI_CASE(7) WTMI_CASE(8) WTMI_CASE(9)
    WTMI_CASE(10) WTMI_CASE(11) WTMI_CASE(12) WTMI_CASE(13) WTMI_CASE(14)
    default:
      return kErrUnsupported;
  }
#undef WTMI_CASE
}

}  // namespace wtmi

using namespace wtmi;

extern "C" int wtmi_cwt_mother(const float* x, long long ld, long long batch, long long n0,
                               const double* affine, const double* scales, int n_scales,
                               double dt, int mother, double param, const double* sig_scale,
                               long long sig_ld, float* out_w, float* out_power, float* out_sig,
                               void* workspace, void* stream) {
  if (n0 < 0 || batch < 0 || n_scales < 0 || ld < n0) return kErrArg;
  if (sig_ld != 0 && sig_ld < n_scales) return kErrArg;
  if (batch == 0 || n0 == 0 || n_scales == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x || !scales) return kErrArg;
  if (!out_w && !out_power && !out_sig) return kErrArg;
  if (out_sig && !sig_scale) return kErrArg;
  if (n0 > (1ll << kLongMaxLog)) return kErrUnsupported;
  if (n0 > (1 << 14) && !workspace) return kErrArg;
  CwtArgs a{};
  if (!mother_consts(a, mother, param)) return kErrArg;
  if (n0 > (1 << 14) && mother != 0) return kErrUnsupported;  // long rows: Morlet only
  a.x = x;
  a.ld = ld;
  a.batch = batch;
  a.n0 = static_cast<int>(n0);
  a.S = n_scales;
  a.affine = affine;
  a.scales = scales;
  a.dt = dt;
  a.sigscale = sig_scale;
  a.sig_ld = sig_ld;
  a.out_w = reinterpret_cast<cpx*>(out_w);
  a.out_pow = out_power;
  a.out_sig = out_sig;
  if (n0 > (1 << 14)) return batch && n_scales ? cwt_long(a, false, workspace, static_cast<hipStream_t>(stream)) : kOk;
  return dispatch<0>(a, static_cast<hipStream_t>(stream));
}

extern "C" int wtmi_cwt_morlet(const float* x, long long ld, long long batch, long long n0,
                               const double* affine, const double* scales, int n_scales,
                               double dt, double f0, const double* sig_scale, long long sig_ld,
                               float* out_w, float* out_power, float* out_sig, void* workspace,
                               void* stream) {
  return wtmi_cwt_mother(x, ld, batch, n0, affine, scales, n_scales, dt, 0, f0, sig_scale, sig_ld, out_w,
                         out_power, out_sig, workspace, stream);
}

extern "C" int wtmi_xwt_mother(const float* x1, const float* x2, long long ld, long long batch,
                               long long n0, const double* affine1, const double* affine2,
                               const double* scales, int n_scales, double dt, int mother, double param,
                               const double* sig_scale, long long sig_ld, float* out_w12,
                               float* out_power, float* out_sig, float* out_u, float* out_v,
                               void* workspace, void* stream) {
  if (n0 < 0 || batch < 0 || n_scales < 0 || ld < n0) return kErrArg;
  if (sig_ld != 0 && sig_ld < n_scales) return kErrArg;
  if (batch == 0 || n0 == 0 || n_scales == 0) return kOk;  // empty batch: no-op (NULL arrays allowed)
  if (!x1 || !x2 || !scales) return kErrArg;
  if (!out_w12 && !out_power && !out_sig && !out_u) return kErrArg;
  if ((out_u == nullptr) != (out_v == nullptr)) return kErrArg;
  if (out_sig && !sig_scale) return kErrArg;
  if (n0 > (1ll << kLongMaxLog)) return kErrUnsupported;
  if (n0 > (1 << 14) && !workspace) return kErrArg;
  CwtArgs a{};
  if (!mother_consts(a, mother, param)) return kErrArg;
  if (n0 > (1 << 14) && mother != 0) return kErrUnsupported;  // long rows: Morlet only
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
  a.sigscale = sig_scale;
  a.sig_ld = sig_ld;
  a.out_w = reinterpret_cast<cpx*>(out_w12);
  a.out_pow = out_power;
  a.out_sig = out_sig;
  a.out_u = out_u;
  a.out_v = out_v;
  if (n0 > (1 << 14)) return batch && n_scales ? cwt_long(a, true, workspace, static_cast<hipStream_t>(stream)) : kOk;
  return dispatch<1>(a, static_cast<hipStream_t>(stream));
}

extern "C" int wtmi_xwt_morlet(const float* x1, const float* x2, long long ld, long long batch,
                               long long n0, const double* affine1, const double* affine2,
                               const double* scales, int n_scales, double dt, double f0,
                               const double* sig_scale, long long sig_ld, float* out_w12,
                               float* out_power, float* out_sig, float* out_u, float* out_v,
                               void* workspace, void* stream) {
  return wtmi_xwt_mother(x1, x2, ld, batch, n0, affine1, affine2, scales, n_scales, dt, 0, f0, sig_scale,
                         sig_ld, out_w12, out_power, out_sig, out_u, out_v, workspace, stream);
}
