// Shared helpers for the wtmi HIP kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wtmi {

constexpr int kWave = 64;  // CDNA wavefront width

// complex64 as a native 2-lane vector: the arithmetic lowers to v_pk_{add,mul,fma}_f32
// with op_sel swizzles and folded sign constants, instead of scalar ops plus register
// shuffles (25% of the FFT loop were v_mov with a struct complex type).
typedef float cpx __attribute__((ext_vector_type(2)));
__device__ __forceinline__ cpx mkc(float re, float im) { return cpx{re, im}; }
__device__ __forceinline__ cpx cadd(cpx a, cpx b) { return a + b; }
__device__ __forceinline__ cpx csub(cpx a, cpx b) { return a - b; }
__device__ __forceinline__ cpx cfma(cpx a, cpx b, cpx c) { return __builtin_elementwise_fma(a, b, c); }
// a * b = a.x b + a.y (i b) = fma(a.yy, (-b.y, b.x), a.xx * b)
__device__ __forceinline__ cpx cmul(cpx a, cpx b) { return cfma(a.yy, b.yx * cpx{-1.f, 1.f}, a.xx * b); }
__device__ __forceinline__ cpx cconj(cpx a) { return a * cpx{1.f, -1.f}; }
__device__ __forceinline__ cpx cscale(cpx a, float s) { return a * s; }
__device__ __forceinline__ float cabs2(cpx a) { return fmaf(a.x, a.x, a.y * a.y); }

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
