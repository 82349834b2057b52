// Common device helpers for the distributed_learning_amd HIP kernels (gfx950 / CDNA4 only).
//
// Everything here is written for a 64-lane wavefront: reductions use 64-wide shuffles,
// block sizes are multiples of 64, and bf16 is carried as raw 16-bit storage so that
// loads/stores vectorise to 8/16-byte accesses (cdna_hip_programming.md Guideline 13).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace dla {

constexpr int kWave = 64;

using bf16_t = uint16_t;  // raw bf16 bits

typedef float float4_t __attribute__((ext_vector_type(4)));
typedef unsigned short ushort4_t __attribute__((ext_vector_type(4)));
typedef unsigned short ushort8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// Plain cast: hipcc lowers this to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN preserving).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float load(const float* p) { return *p; }
  __device__ __forceinline__ static float to_f32(float v) { return v; }
  __device__ __forceinline__ static float from_f32(float v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float to_f32(bf16_t v) { return bf16_to_f32(v); }
  __device__ __forceinline__ static bf16_t from_f32(float v) { return f32_to_bf16(v); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks that the dispatcher deals to the same XCD (b % 8 equal) get a contiguous range of
// logical tile ids, so neighbouring tiles share that XCD's L2. Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nxcd;
}

}  // namespace dla

#define DLA_HIP_CHECK(expr)                                                             \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      abort();                                                                          \
    }                                                                                   \
  } while (0)
