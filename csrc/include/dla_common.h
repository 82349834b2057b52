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

// 8 consecutive channels = one 16-byte (bf16) or two 16-byte (fp32) accesses, widened to fp32.
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
  __device__ __forceinline__ static void load(const bf16_t* p, float (&v)[8]) {
    const ushort8_t x = *reinterpret_cast<const ushort8_t*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(x[j]);
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float (&v)[8]) {
    ushort8_t x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = f32_to_bf16(v[j]);
    *reinterpret_cast<ushort8_t*>(p) = x;
  }
};
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    const float4_t a = reinterpret_cast<const float4_t*>(p)[0];
    const float4_t b = reinterpret_cast<const float4_t*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4_t*>(p)[0] = float4_t{v[0], v[1], v[2], v[3]};
    reinterpret_cast<float4_t*>(p)[1] = float4_t{v[4], v[5], v[6], v[7]};
  }
};

// 8 consecutive channels as loaded (bf16: one 16-byte register quad; fp32: two), widened on use.
// The streaming loops (bn_act.hip, pool.hip) load a whole group of rows into these before touching
// any of them, so the group's loads are in flight together (hipcc does not hoist them across the
// per-row arithmetic).
template <typename T> struct Raw8;
template <> struct Raw8<bf16_t> {
  ushort8_t v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const ushort8_t*>(p); }
  __device__ __forceinline__ void get(float (&f)[8]) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = bf16_to_f32(v[j]);
  }
};
template <> struct Raw8<float> {
  float4_t a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = reinterpret_cast<const float4_t*>(p)[0];
    b = reinterpret_cast<const float4_t*>(p)[1];
  }
  __device__ __forceinline__ void get(float (&f)[8]) const {
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
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
