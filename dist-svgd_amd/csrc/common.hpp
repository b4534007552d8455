// common.hpp -- shared helpers for the gfx950 SVGD kernels (libdsvgd_hip.so).
//
// Written for CDNA4 only: 64-lane waves, fp32-input MFMA
// (v_mfma_f32_32x32x2_f32), 160 KiB LDS per CU.  No CUDA / hipify layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/dsvgd.h"

namespace dsvgd {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr float kLog2e = 1.4426950408889634f;

// ---- error plumbing (thread-local message, negative return codes) --------
void set_error(const char* fmt, ...);
int fail_arg(const char* what);
int check_launch(const char* kernel);
// resident blocks/CU x CUs of a kernel launched with `threads` threads, a multiple of 8
int persistent_blocks(const void* fn, int* blocks, int threads = 256);

inline int64_t roundup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int64_t roundup128(int64_t x) { return (x + 127) & ~(int64_t)127; }

// 32x32x2 f32 MFMA: lane l holds A[l&31][l>>5], B[l>>5][l&31]; the 16 result
// registers hold C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]  (r = register index).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int c_row(int reg, int lane) {
  return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}

// |v|'s bit pattern: unsigned order is magnitude order, finite < inf < NaN
__device__ __forceinline__ uint32_t abs_bits(float v) {
  return __float_as_uint(v) & 0x7fffffffu;
}

// FmtH2 power-of-two scale of an operand whose largest magnitude is m: s m
// in [2^14, 2^15); 1 for an all-zero or non-finite operand (NaN / inf
// propagate).  s is in [2^-113, 2^100], so pow2_inv is exact.
__device__ __forceinline__ float pow2_scale(float m) {
  if (!(m > 0.f) || !isfinite(m)) return 1.f;
  int e;
  frexpf(m, &e);                        // m in [2^(e-1), 2^e)
  return ldexpf(1.f, min(15 - e, 100));  // s m in [2^14, 2^15)
}
// 1 / s for a normal power of two s (exact; no rcp rounding)
__device__ __forceinline__ float pow2_inv(float s) {
  return __uint_as_float(0x7F000000u - __float_as_uint(s));
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace dsvgd

#define DSVGD_REQUIRE(cond, msg)          \
  do {                                    \
    if (!(cond)) return dsvgd::fail_arg(msg); \
  } while (0)
