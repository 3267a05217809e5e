// Shared helpers for the wtmi HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wtmi {

constexpr int kWave = 64;  // CDNA wavefront width

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float cabs2(float2 a) { return fmaf(a.x, a.x, a.y * a.y); }

// Error codes returned by the C ABI (0 = success; >0 = hipError_t of the launch).
enum : int {
  kOk = 0,
  kErrArg = -1,        // invalid argument (null pointer, size out of range)
  kErrUnsupported = -2 // size outside what the kernels handle
};

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? kOk : static_cast<int>(e);
}

}  // namespace wtmi
