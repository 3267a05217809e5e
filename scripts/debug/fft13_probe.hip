// fft_row<13> forward transform of x[n] = exp(2 pi i 5 n / N) + delta(n - 3): compare with the DFT.
#include <cstdio>
#include <cmath>
#include "fft_lds.hpp"
using namespace wtmi;
constexpr int LOGN = 13;
__global__ void __launch_bounds__(512) k(float2* out) {
  using P = FftPlan<LOGN>;
  __shared__ cpx lds[P::PADN];
  const int t = fft_thread<LOGN>(threadIdx.x);
  cpx tw[P::NTW_ALLOC];
  fft_twiddles<LOGN>(tw, t);
  int par = 0;
  cpx v[16];
  for (int m = 0; m < 16; ++m) {
    const int n = t + m * P::NT;
    float s, c;
    sincospif(2.f * 5.f * n / P::N, &s, &c);
    v[m] = mkc(c + (n == 3 ? 1.f : 0.f), s);
  }
  fft_row<LOGN, -1, 1>(v, lds, 0, tw, t, par);
  for (int m = 0; m < 16; ++m) out[t + m * P::NT] = make_float2(v[m].x, v[m].y);
}
int main() {
  const int N = 1 << LOGN;
  float2* d;
  float2* h = new float2[N];
  hipMalloc(&d, N * sizeof(float2));
  hipLaunchKernelGGL(k, dim3(1), dim3(512), 0, 0, d);
  hipMemcpy(h, d, N * sizeof(float2), hipMemcpyDeviceToHost);
  double err = 0;
  int worst = -1;
  for (int kk = 0; kk < N; ++kk) {
    double re = cos(-2 * M_PI * 3.0 * kk / N), im = sin(-2 * M_PI * 3.0 * kk / N);
    if (kk == 5) re += N;
    const double e = hypot(h[kk].x - re, h[kk].y - im);
    if (e > err) { err = e; worst = kk; }
  }
  printf("max abs err %g at bin %d (got %g %g)\n", err, worst, h[worst].x, h[worst].y);
  printf("bin5 %g %g  bin0 %g %g bin4096 %g %g\n", h[5].x, h[5].y, h[0].x, h[0].y, h[4096].x, h[4096].y);
  return 0;
}
