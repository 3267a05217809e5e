// Long-row CWT / XWT / WCT (n0 > 16384 samples, N = 2^ceil(log2 n0) up to 2^20): the
// reference path has no length limit (pycwt / scipy.fftpack), src/cwt.py:110,
// src/xwt.py:93, src/wct.py:106 -- and wct_significance draws noise of ~6 n0 samples, so
// even the app's series reach it (src/wct.py:106-118).  Four-step FFTs through HBM
// (fft_long.hpp); series are processed in sub-batches and scales in chunks so that the
// work buffers stay within fixed budgets whatever the batch.
#include "fft_long.hpp"
#include "long_path.hpp"

extern "C" int wtmi_series_moments(const void* x, int x_is_f64, long long ld, long long batch,
                                   long long n, double* out, void* stream);

namespace wtmi {

namespace {

constexpr long long kSpecBudget = 1ll << 30;  // bytes of series spectra per sub-batch
constexpr long long kWorkBudget = 1ll << 30;  // bytes of (series, scale) work rows per chunk

int log2_ceil_l(long long n) {
  int l = 0;
  while ((1ll << l) < n) ++l;
  return l;
}

long long align256(long long b) { return (b + 255) & ~255ll; }

struct LongPlan {
  int logn;
  long long N;
  int planes;         // 1 (CWT) or 2 (pair)
  long long bc;       // series per sub-batch
  long long zrows;    // (series, scale) rows per chunk
  long long mom_b, spec_b, work_b;  // bytes of each region (per plane)
};

LongPlan long_plan(long long batch, long long n0, int n_scales, int planes) {
  LongPlan p{};
  p.logn = log2_ceil_l(n0);
  p.N = 1ll << p.logn;
  p.planes = planes;
  const long long row = p.N * static_cast<long long>(sizeof(cpx));
  p.zrows = kWorkBudget / (row * planes);
  if (p.zrows < 1) p.zrows = 1;
  long long bc = kSpecBudget / (row * planes);
  if (bc < 1) bc = 1;
  if (bc > p.zrows) bc = p.zrows;  // a chunk holds at least one scale of every series
  if (bc > batch) bc = batch < 1 ? 1 : batch;
  p.bc = bc;
  long long zr = p.zrows;
  const long long need = p.bc * n_scales;  // rows if every scale fits at once
  if (zr > need) zr = need < 1 ? 1 : need;
  p.zrows = zr;
  p.mom_b = align256(p.bc * 8 * static_cast<long long>(sizeof(double)));
  p.spec_b = align256(p.bc * row);
  p.work_b = align256(p.zrows * row);
  return p;
}

long long plan_bytes(const LongPlan& p) { return p.planes * (p.mom_b + p.spec_b + p.work_b); }

struct LongBufs {
  double* mom[2];
  cpx* spec[2];
  cpx* work[2];
};

LongBufs carve(const LongPlan& p, char* ws) {
  LongBufs b{};
  for (int q = 0; q < p.planes; ++q) {
    b.mom[q] = reinterpret_cast<double*>(ws);
    ws += p.mom_b;
    b.spec[q] = reinterpret_cast<cpx*>(ws);
    ws += p.spec_b;
    b.work[q] = reinterpret_cast<cpx*>(ws);
    ws += p.work_b;
  }
  return b;
}

// Spectra (transposed order XT) of rows [bs, bs + bc) of one input plane.
int long_spectra(const CwtArgs& a, int plane, long long bs, long long bc, const LongPlan& p,
                 const LongBufs& bf, hipStream_t st) {
  const float* x = (plane ? a.x2 : a.x) + bs * a.ld;
  const double* aff = plane ? a.affine2 : a.affine;
  int rc = wtmi_series_moments(x, 0, a.ld, bc, a.n0, bf.mom[plane], st);
  if (rc != kOk) return rc;
  LongArgs la{};
  la.logn = p.logn;
  la.n0 = a.n0;
  la.nrows = bc;
  la.x = x;
  la.ld = a.ld;
  la.affine = aff ? aff + 3 * bs : nullptr;
  la.mom = bf.mom[plane];
  la.spec = bf.spec[plane];
  if ((rc = long_col<kColFwdSeries>(la, st)) != kOk) return rc;
  return long_row<kRowFwdSpec>(la, st);
}

// For every (series sub-batch, scale chunk): Z rows of both planes, then `body`.
template <typename Body>
int long_sweep(const CwtArgs& a, const LongPlan& p, const LongBufs& bf, hipStream_t st, Body body) {
  for (long long bs = 0; bs < a.batch; bs += p.bc) {
    const long long bc = a.batch - bs < p.bc ? a.batch - bs : p.bc;
    for (int q = 0; q < p.planes; ++q) {
      const int rc = long_spectra(a, q, bs, bc, p, bf, st);
      if (rc != kOk) return rc;
    }
    long long nsc = p.zrows / bc;
    if (nsc < 1) nsc = 1;
    for (int j0 = 0; j0 < a.S; j0 += static_cast<int>(nsc)) {
      const int ns = static_cast<int>(a.S - j0 < nsc ? a.S - j0 : nsc);
      LongArgs la{};
      la.logn = p.logn;
      la.n0 = a.n0;
      la.nrows = bc * ns;
      la.scales = a.scales;
      la.j0 = j0;
      la.nsc = ns;
      la.S = a.S;
      la.b0 = bs;
      la.dt = a.dt;
      la.f0 = a.f0;
      la.out = a;
      for (int q = 0; q < p.planes; ++q) {
        la.spec = bf.spec[q];
        la.z1 = bf.work[q];
        const int rc = long_row<kRowInvMorlet>(la, st);
        if (rc != kOk) return rc;
      }
      la.spec = nullptr;
      la.z1 = bf.work[0];
      la.z2 = p.planes > 1 ? bf.work[1] : nullptr;
      const int rc = body(la);
      if (rc != kOk) return rc;
    }
  }
  return kOk;
}

__global__ void long_plan_kernel(int* plan, int S) {
  for (int i = threadIdx.x; i <= S; i += blockDim.x) plan[i] = i < S ? 0 : S - 1;
}

}  // namespace

long long cwt_long_workspace_bytes(long long batch, long long n0, int n_scales, bool pair) {
  return plan_bytes(long_plan(batch, n0, n_scales, pair ? 2 : 1));
}

int cwt_long(const CwtArgs& a, bool pair, void* workspace, hipStream_t st) {
  const LongPlan p = long_plan(a.batch, a.n0, a.S, pair ? 2 : 1);
  if (p.logn > kLongMaxLog) return kErrUnsupported;
  if (!workspace) return kErrArg;
  const LongBufs bf = carve(p, static_cast<char*>(workspace));
  return long_sweep(a, p, bf, st, [&](LongArgs& la) {
    return pair ? long_col<kColInvPair>(la, st) : long_col<kColInvCwt>(la, st);
  });
}

// WCT workspace: [TA][TB] time-smoothed rows (phase B input, batch x S x n0 cpx each),
// [plan S + 1 ints], then the pair-mode long-path buffers.
long long wct_long_workspace_bytes(long long batch, long long n0, int n_scales) {
  const long long t = align256(batch * n_scales * n0 * static_cast<long long>(sizeof(cpx)));
  return 2 * t + align256(4ll * (n_scales + 1)) + cwt_long_workspace_bytes(batch, n0, n_scales, true);
}

int wct_long(const CwtArgs& a, int K, void* workspace, float* coh, hipStream_t st) {
  const LongPlan p = long_plan(a.batch, a.n0, a.S, 2);
  if (p.logn > kLongMaxLog) return kErrUnsupported;
  if (!workspace) return kErrArg;
  char* ws = static_cast<char*>(workspace);
  const long long t = align256(a.batch * a.S * static_cast<long long>(a.n0) * static_cast<long long>(sizeof(cpx)));
  cpx* TA = reinterpret_cast<cpx*>(ws);
  cpx* TB = reinterpret_cast<cpx*>(ws + t);
  int* plan = reinterpret_cast<int*>(ws + 2 * t);
  const LongBufs bf = carve(p, ws + 2 * t + align256(4ll * (a.S + 1)));
  hipLaunchKernelGGL(long_plan_kernel, dim3(1), dim3(256), 0, st, plan, a.S);
  int rc = launch_status();
  if (rc != kOk) return rc;
  rc = long_sweep(a, p, bf, st, [&](LongArgs& la) {
    la.out_phase = a.out_sig;  // the WCT entry passes the phase plane in out_sig
    la.out.out_sig = nullptr;
    la.ta = TA;
    la.tb = TB;
    int r = long_col<kColInvPair, true>(la, st);  // cross outputs + smoothing inputs in place
    if (r != kOk) return r;
    LongArgs f = la;
    if ((r = long_col<kColFwdRows>(f, st)) != kOk) return r;  // plane z1
    f.z1 = la.z2;
    if ((r = long_col<kColFwdRows>(f, st)) != kOk) return r;  // plane z2
    if ((r = long_row<kRowSmooth>(la, st)) != kOk) return r;
    return long_col<kColInvSmooth>(la, st);
  });
  if (rc != kOk) return rc;
  return wct_phase_b_any(TA, TB, a.batch, a.n0, a.S, coh, plan, K, st);
}

}  // namespace wtmi

extern "C" long long wtmi_cwt_workspace_bytes(long long batch, long long n0, int n_scales, int pair) {
  if (batch < 0 || n0 < 0 || n_scales < 0) return -1;
  if (n0 <= (1 << 14)) return 0;
  return wtmi::cwt_long_workspace_bytes(batch, n0, n_scales, pair != 0);
}
