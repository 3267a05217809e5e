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
// The same products in two packed instructions.  The compiler builds (-b.y, b.x) with a
// separate multiply (or xor + mov): it does not fold a one-lane sign into the VOP3P neg_lo /
// neg_hi source modifiers, which v_pk_{mul,fma}_f32 take for free.  Same roundings as cmul:
// the results are bit-identical.  Plain VALU arithmetic (no hazard-bearing instructions);
// used for the FFT twiddle products, where a third of the multiplies were sign shuffles.
//   a * b       = fma(a.yy, (-b.y, b.x), a.xx * b)
//   a * conj(b) = fma(a.yy, b.yx, (a.x b.x, -a.x b.y))
// One asm block each: with two, the hazard recognizer (blind to what an asm block holds)
// put an s_nop between them on every product.
__device__ __forceinline__ cpx cmul2(cpx a, cpx b) {
  cpx t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(r), "=&v"(t) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ cpx cmul2_conj(cpx a, cpx b) {
  cpx t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1] neg_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1]"
      : "=v"(r), "=&v"(t) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ cpx cscale(cpx a, float s) { return a * s; }
__device__ __forceinline__ float cabs2(cpx a) { return fmaf(a.x, a.x, a.y * a.y); }

// x / d by the hardware reciprocal (1 ulp) and one multiply: ~2 ulp instead of the
// ~10-instruction IEEE division sequence.  Same 0/0 = NaN and x/0 = inf; differs only for
// d below FLT_MIN (signal powers at ~1e-19 in fp32, meaningless at this precision anyway).
__device__ __forceinline__ float fast_div(float x, float d) { return x * __builtin_amdgcn_rcpf(d); }

// atan2(y, x) for finite inputs, |error| <= 4e-7 rad (the phase outputs' tolerance is 1e-4;
// r03's min/max octant form measured 3.7e-7 on the same 2e6 random points).  With
// t = (|y| - |x|) / (|y| + |x|) in [-1, 1] (hardware reciprocal), atan(|y| / |x|) =
// pi/4 + atan(t), and atan(t) = t P(t^2) is the degree-7 fit of r03 (atan is odd, so its
// [0, 1] fit serves [-1, 1]).  No min / max / swap correction: what is left per value is
// the two sums, the reciprocal, a clamp, the x < 0 reflection and the sign of y -- the
// polynomial and the reflection run packed for two values at once (fast_atan2f_x2), which
// cuts the phase output of the WCT's decimated rows from ~35 to ~25 instructions per pair.
// K = the fp32 value of P(1) (= pi/4 - 1 ulp): t = -1 (y = 0, and x = y = 0, where 0 / 0 is
// clamped to -1) then gives fma(-1, K, K) = 0 exactly.  atan2(+-0, 0) = +-0, the sign of y
// (also of a zero y) carries to the result as in atan2f; x = -0 counts as positive.
constexpr float kAtanK = 0.7853981256484985f;  // 0x3f490fda
__device__ __forceinline__ float atan_poly(float q) {
  float p = -0.004781003575772047f;
  p = fmaf(p, q, 0.02455916814506054f);
  p = fmaf(p, q, -0.059907760471105576f);
  p = fmaf(p, q, 0.0994298979640007f);
  p = fmaf(p, q, -0.1402951329946518f);
  p = fmaf(p, q, 0.19971394538879395f);
  p = fmaf(p, q, -0.3333209455013275f);
  return fmaf(p, q, 0.9999999403953552f);
}
__device__ __forceinline__ float fast_atan2f(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float t = fmaxf((ay - ax) * __builtin_amdgcn_rcpf(ay + ax), -1.f);  // 0 / 0 = NaN -> -1
  float r = fmaf(t, atan_poly(t * t), kAtanK);
  if (x < 0.f) r = 3.14159265358979324f - r;
  return copysignf(r, y);
}

// Two fast_atan2f at once (lane i of the vectors is atan2(y[i], x[i]), bitwise the scalar
// function's result): the sums, reciprocals and clamps stay scalar (no packed max / rcp on
// gfx950), the polynomial and the reflection run on v_pk_fma_f32 / v_pk_add_f32.
__device__ __forceinline__ cpx fast_atan2f_x2(cpx y, cpx x) {
  cpx t;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float ax = fabsf(x[i]), ay = fabsf(y[i]);
    t[i] = fmaxf((ay - ax) * __builtin_amdgcn_rcpf(ay + ax), -1.f);
  }
  const cpx q = t * t;
  cpx p = cpx{-0.004781003575772047f, -0.004781003575772047f};
  p = cfma(p, q, cpx{0.02455916814506054f, 0.02455916814506054f});
  p = cfma(p, q, cpx{-0.059907760471105576f, -0.059907760471105576f});
  p = cfma(p, q, cpx{0.0994298979640007f, 0.0994298979640007f});
  p = cfma(p, q, cpx{-0.1402951329946518f, -0.1402951329946518f});
  p = cfma(p, q, cpx{0.19971394538879395f, 0.19971394538879395f});
  p = cfma(p, q, cpx{-0.3333209455013275f, -0.3333209455013275f});
  p = cfma(p, q, cpx{0.9999999403953552f, 0.9999999403953552f});
  const cpx r = cfma(t, p, cpx{kAtanK, kAtanK});
  const cpx u = cpx{3.14159265358979324f, 3.14159265358979324f} - r;
  cpx o;
#pragma unroll
  for (int i = 0; i < 2; ++i) o[i] = copysignf(x[i] < 0.f ? u[i] : r[i], y[i]);
  return o;
}

// Wave-uniform buffer resource for one output/input row (T8/T20 of the CDNA guide):
// rows are addressed as SGPR descriptor + 32-bit per-lane voffset + SGPR soffset, so a
// 16-position-per-thread row store needs one offset VGPR instead of 16 64-bit address
// pairs (which the FFT kernels otherwise keep live across the scale loop).  The
// pointer must be wave-uniform; readfirstlane makes that provable to the compiler.
// bytes: the descriptor's extent; accesses past it are dropped (stores) or read 0 (loads) by
// the hardware range check.  Callers that rely on it put the out-of-range offset in voffset
// (e.g. voffset = extent), never only in soffset: whether the range check counts the SGPR
// offset is not something this code assumes (put_row, store_row, band_load).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes = 0x7fffffff) {
  const unsigned long long u = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(u));
  const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(u >> 32));
  void* q = reinterpret_cast<void*>((static_cast<unsigned long long>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
// Cache policy operand (aux) of the buffer loads / stores: 0 = default, kNt = streaming (nt).
// Measured per kernel (profiles/r05/nt_policy_ab.txt): nt on the once-read rows of the MODWT
// synthesis and on the WCT kernels' row stores pays; on the CWT's output stream it costs 2-3 %.
constexpr int kNt = 2;
typedef float f32x4 __attribute__((ext_vector_type(4)));
// a once-read float4 row element through a plain pointer, streaming policy
__device__ __forceinline__ float4 ld_nt4(const float4* p) {
  return __builtin_bit_cast(float4, __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p)));
}
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <int AUX = 0>
__device__ __forceinline__ void buf_st(float v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void buf_st(cpx v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, soff, AUX);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
template <int AUX = 0>
__device__ __forceinline__ void buf_st(float4 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, soff, AUX);
}
__device__ __forceinline__ float buf_ld_f32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
template <int AUX = 0>
__device__ __forceinline__ cpx buf_ld_c64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(cpx, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
}

// Bijective XCD-aware block remap (CDNA guide T1).  The dispatcher deals blocks
// round-robin over the 8 XCDs, so b, b+8, b+16, ... share one XCD and its L2; this
// hands each XCD a contiguous range of logical blocks, so blocks that read the same
// data (e.g. the scale chunks of one series pair) run behind the same L2.
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned nb) {
  const unsigned x = bid & 7u, slot = bid >> 3, q = nb >> 3, r = nb & 7u;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
}

// Error codes returned by the C ABI (0 = success; >0 = hipError_t of the launch).
enum : int {
  kOk = 0,
  kErrArg = -1,        // invalid argument (null pointer, size out of range)
  kErrUnsupported = -2 // size outside what the kernels handle
};

// Launch-policy knobs, read from the environment ONCE (first use) and settable through
// wtmi_set_option (options.hip); never read per launch.  prune flags exist so tests can
// compare the pruned transforms with full ones; the others are tuning defaults.
struct Options {
  int cwt_prune = 2;        // WTMI_CWT_PRUNE: 2 band rows + narrowed entry passes, 1 band rows, 0 full
  int cwt_target_wg = 0;    // WTMI_CWT_TARGET_WG: workgroups per CWT launch, 0 = by size
  int wct_prune = 2;        // WTMI_WCT_PRUNE: 2 band rows + decimated spectra, 1 band rows, 0 full
  int wct_target_wg = 0;    // WTMI_WCT_TARGET_WG: 0 = as many as wct_min_rows allows
  int wct_min_rows = 0;     // WTMI_WCT_MIN_ROWS: scale rows per WCT workgroup, at least (0 = by batch)
  int wct_dec_rows = 0;     // WTMI_WCT_DEC_ROWS: decimated scale rows per phase A workgroup (0 = by batch)
  int modwt_syn = 1;        // WTMI_MODWT_SYN: 1 hybrid synthesis, every level via LDS (r05); 2 the
                            // same with chain levels dq >= 4 groups from L2 (r04); 0 MODE 3 only
  int wct_wide = 1;         // WTMI_WCT_WIDE: windows of union band N >> e take the spectral route
                            // from e >= wct_wide (1..3); 0 = never (time path)
  int modwt_ana = 0;        // WTMI_MODWT_ANA: n = 16384 analysis with 1024 threads x 4 groups (0),
                            // 512 x 8 (1, r01-r03) or 256 x 16 (2)
  int wct_pc_early = 2;     // WTMI_WCT_PC_EARLY: phase C's q windows on a third stream right after
                            // the decimated spectra (1), after the full-band rows (0), or the
                            // former for batches of at most 256 pairs (2)
  int wct_side_stream = 1;  // WTMI_WCT_SIDE_STREAM: full-band rows on a side stream beside the
                            // decimated rows' chain (1), or all on the caller's stream (0)
  int wct_dec_merge = 2;    // WTMI_WCT_DEC_MERGE: the decimation classes M = 4096 .. 512 in one
                            // launch (1), one launch per class (0), or the former for batches of
                            // at most 256 pairs (2)
  int wct_depth = 1;        // WTMI_WCT_DEPTH: rows in flight per thread of phase B and the wide
                            // boxcar: K itself (1, K <= 12; r05) or the largest of 6..1 dividing
                            // K (0, r04).  C4 serial trace: phase B 0.2935 -> 0.2840 ms, boxcar
                            // 0.2538 -> 0.2515; 64-pair step 0.4499 -> 0.4434 (alternating)
};
const Options& options();

inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? kOk : static_cast<int>(e);
}

}  // namespace wtmi
