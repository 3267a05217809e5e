// Read-rate ceiling for the MODWT synthesis access pattern (diagnostic, not product code).
// 8192 series x 11 rows x 16384 floats; one workgroup per series reads its rows in turn
// (the synthesis's order) and writes one row.  Variants:
//   0: rows one after another, 8 float4 per thread (512 threads), wait per row
//   1: two rows in flight (16 float4 per thread)
//   2: 1024 threads, 4 float4 per thread per row, wait per row
//   3: rows one after another with an LDS round trip + barrier per row (the synthesis skeleton)
// hipcc --offload-arch=gfx950 -O3 read_rows.hip -o read_rows
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kB = 8192, kR = 11, kN = 16384, kNG = kN / 4;

template <int T, int ROWS_IN_FLIGHT, bool LDS>
__global__ void __launch_bounds__(T) read_rows(const float4* __restrict__ w, float4* __restrict__ x) {
  constexpr int G = kNG / T;
  __shared__ float4 s[LDS ? kNG : 1];
  const int tid = threadIdx.x;
  const float4* base = w + static_cast<long long>(blockIdx.x) * kR * kNG;
  float4 acc[G];
#pragma unroll
  for (int k = 0; k < G; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < kR; r += ROWS_IN_FLIGHT) {
    float4 v[ROWS_IN_FLIGHT][G];
#pragma unroll
    for (int i = 0; i < ROWS_IN_FLIGHT; ++i)
#pragma unroll
      for (int k = 0; k < G; ++k) v[i][k] = base[static_cast<long long>(min(r + i, kR - 1)) * kNG + tid + k * T];
#pragma unroll
    for (int i = 0; i < ROWS_IN_FLIGHT; ++i)
#pragma unroll
      for (int k = 0; k < G; ++k) {
        acc[k].x += v[i][k].x; acc[k].y += v[i][k].y; acc[k].z += v[i][k].z; acc[k].w += v[i][k].w;
      }
    if constexpr (LDS) {
      __syncthreads();
#pragma unroll
      for (int k = 0; k < G; ++k) s[tid + k * T] = acc[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < G; ++k) acc[k] = s[(tid + 37 + k * T) & (kNG - 1)];
    }
  }
#pragma unroll
  for (int k = 0; k < G; ++k) x[static_cast<long long>(blockIdx.x) * kNG + tid + k * T] = acc[k];
}

// Analysis skeleton: read one row, write 11 rows (one per "level", LDS round trip each).
template <int T>
__global__ void __launch_bounds__(T) write_rows(const float4* __restrict__ x, float4* __restrict__ w) {
  constexpr int G = kNG / T;
  __shared__ float4 s[kNG];
  const int tid = threadIdx.x;
  float4 v[G];
#pragma unroll
  for (int k = 0; k < G; ++k) v[k] = x[static_cast<long long>(blockIdx.x) * kNG + tid + k * T];
  float4* base = w + static_cast<long long>(blockIdx.x) * kR * kNG;
  for (int r = 0; r < kR; ++r) {
#pragma unroll
    for (int k = 0; k < G; ++k) base[static_cast<long long>(r) * kNG + tid + k * T] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < G; ++k) s[tid + k * T] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < G; ++k) v[k] = s[(tid + 37 + k * T) & (kNG - 1)];
  }
}

template <typename K>
static float run(K kernel, int threads, const float4* w, float4* x) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kernel, dim3(kB), dim3(threads), 0, 0, w, x);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kernel, dim3(kB), dim3(threads), 0, 0, w, x);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10.f;
}

int main() {
  float4 *w = nullptr, *x = nullptr;
  const size_t wb = static_cast<size_t>(kB) * kR * kN * 4, xb = static_cast<size_t>(kB) * kN * 4;
  if (hipMalloc(&w, wb) != hipSuccess || hipMalloc(&x, xb) != hipSuccess) return 1;
  hipMemset(w, 0, wb);
  const double gb = (wb + xb) / 1e9;
  const float t0 = run(read_rows<512, 1, false>, 512, w, x);
  const float t1 = run(read_rows<512, 2, false>, 512, w, x);
  const float t2 = run(read_rows<1024, 1, false>, 1024, w, x);
  const float t3 = run(read_rows<512, 1, true>, 512, w, x);
  const float t4 = run(read_rows<1024, 2, false>, 1024, w, x);
  const float t5 = run(write_rows<512>, 512, x, w);
  printf("analysis skeleton (1 row in, 11 out, 512 thr): %.4f ms %.2f TB/s\n", t5, gb / t5);
  printf("512 thr, 1 row in flight: %.4f ms %.2f TB/s\n", t0, gb / t0);
  printf("512 thr, 2 rows in flight: %.4f ms %.2f TB/s\n", t1, gb / t1);
  printf("1024 thr, 1 row in flight: %.4f ms %.2f TB/s\n", t2, gb / t2);
  printf("512 thr, 1 row + LDS round trip: %.4f ms %.2f TB/s\n", t3, gb / t3);
  printf("1024 thr, 2 rows in flight: %.4f ms %.2f TB/s\n", t4, gb / t4);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
