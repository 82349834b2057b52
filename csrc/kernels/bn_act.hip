// Fused training-mode BatchNorm + (residual add) + (ReLU), forward and backward, NHWC.
//
// Replaces the per-block tail Conv -> BN -> (+identity) -> ReLU of ResNet / GoogLeNet, which stock
// PyTorch runs as MIOpen BN (2 passes fwd, 3 passes bwd) plus separate elementwise add / ReLU /
// threshold-backward kernels. Activations are channels_last ([M = N*H*W rows, C channels],
// C contiguous) so a lane owns 8 consecutive channels = one 16-byte bf16 vector.
//
// Forward : stats pass  — per-channel shifted sums S=Σ(x-K), Q=Σ(x-K)^2 (K = x[row 0][c], which
//                         removes the E[x^2]-E[x]^2 cancellation), per-block partials, no atomics;
//           finalize    — mean / invstd / scale / shift per channel + running-stat update;
//           apply pass  — y = relu(x*scale + shift [+ res]) in one read-modify-write.
// Backward: reduce pass — Σdy', Σdy'(x-mean) with dy' = dy * relu'(.): the ReLU branch is
//                         recomputed from x (ReLU right after BN) or read from a 1-bit mask the
//                         forward wrote (ReLU after the residual add) — never from the saved y;
//           finalize    — dgamma, dbeta and the two per-channel dx coefficients;
//           apply pass  — dx = k1*(dy' - m1 - (x-mean)*k2) [and d_residual = dy'].
// Traffic per element (bf16): fwd 2R+1W (+1R res), bwd 4R+1W (+1W dres, +1/16 R mask) vs ~7 and ~8 passes for
// the unfused chain. Partials are reduced in a fixed order -> bitwise reproducible.
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

#include <algorithm>

namespace dla {

constexpr int kBNThreads = 256;
// Row blocks of the two reduction passes (stats, backward reduce): 4 workgroups per CU stream at
// full bandwidth, and <= 1024 partial rows keep the finalize's reduction at ~2 load round trips.
constexpr int kRedBlocks = 1024;
// Rows per thread per streaming-loop iteration (loads of a group issued back to back).
constexpr int kUnroll = 4;

// Block geometry shared by the two reduction passes: the block covers CT = tpr*8 channels
// (channel tile blockIdx.x) and rows [r0, r1) (row block blockIdx.y); rpi = 256/tpr rows are in
// flight per iteration, each row segment of a wave-instruction is a contiguous 16*tpr bytes.
struct RedGeom {
  int tpr, rpi, ct;
};

__device__ __forceinline__ void block_rows(int64_t M, int nrb, int64_t& r0, int64_t& r1) {
  const int64_t per = (M + nrb - 1) / nrb;
  r0 = (int64_t)blockIdx.y * per;
  r1 = min(M, r0 + per);
}
// The same row blocks dispatched last-to-first, for a pass that reads a tensor the previous kernel finished
// writing (or reading) in row order: its first blocks then find the most recently touched rows still in the
// 256 MB Infinity Cache (MALL) instead of evicting them on the way up. Used by the forward apply (after the
// GEMM wrote x) and the backward reductions (after the data-gradient GEMM wrote dy); the backward apply then
// runs first-to-last, after the reduction's last-to-first pass. Partial rows keep their blockIdx.y slot (each
// block still writes one distinct partial; only the fixed summation order changes). DLA_BN_REV=0: off (A/B).
#ifndef DLA_BN_REV
#define DLA_BN_REV 1
#endif
__device__ __forceinline__ void block_rows_rev(int64_t M, int nrb, int64_t& r0, int64_t& r1) {
  const int64_t per = (M + nrb - 1) / nrb;
  r0 = (int64_t)(DLA_BN_REV ? nrb - 1 - (int)blockIdx.y : (int)blockIdx.y) * per;
  r1 = min(M, r0 + per);
}

// Reduce 8 channels x 2 sums across the rpi row groups of the block (LDS), then thread row-group 0
// writes the block partial. `red` holds rpi x ct x 2 floats.
__device__ __forceinline__ void block_reduce_write(float (&s)[8], float (&q)[8], int tpr, int rpi, int ct, int C,
                                                   float* __restrict__ part, int c_base, float* red) {
  const int lane_c = threadIdx.x % tpr;  // channel group within tile
  const int rg = threadIdx.x / tpr;      // row group
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[(rg * ct + lane_c * 8 + j) * 2 + 0] = s[j];
    red[(rg * ct + lane_c * 8 + j) * 2 + 1] = q[j];
  }
  __syncthreads();
  // tree over row groups, each thread handles (channel, which) pairs
  for (int idx = threadIdx.x; idx < ct * 2; idx += kBNThreads) {
    float acc = 0.f;
    for (int g = 0; g < rpi; ++g) acc += red[g * ct * 2 + idx];
    const int c = idx >> 1, w = idx & 1;
    part[((int64_t)blockIdx.y * C + c_base + c) * 2 + w] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// forward: statistics
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBNThreads) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, int nrb,
                                                              int tpr, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c_base = blockIdx.x * ct;
  const int c0 = c_base + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows(M, nrb, r0, r1);
  float K[8], s[8], q[8];
  Vec8<T>::load(x + c0, K);  // shift = row 0 (same for every block)
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for (int64_t r = r0 + rg; r < r1; r += rpi) {
    float v[8];
    Vec8<T>::load(x + r * C + c0, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - K[j];
      s[j] += d;
      q[j] = fmaf(d, d, q[j]);
    }
  }
  block_reduce_write(s, q, tpr, rpi, ct, C, part, c_base, red);
}

// Partial reduction shared by both finalize kernels: WPC waves per channel (a 256-thread block owns
// 4 / WPC channels); each lane strides over the nrb block partials with 8 independent loads in
// flight, then a 64-lane shuffle tree and (WPC > 1) a fixed-order combine through LDS. The pass is
// latency-bound (~1 us per dependent round trip): WPC = 1 for the <= 1024 partial rows of the
// reduction passes, WPC = 4 for the per-128-row-tile partials of the GEMM epilogues.
// Fixed order -> bitwise reproducible.
// NF loads in flight per lane: 8, or 4 for the lean finalize kernels (kFinalizeVgprs), which must fit
// beside a 256x256 weight-gradient block (2 x 240 of a SIMD's 512 VGPRs): the late weight gradients
// (ops/conv.py WGRAD_DEFER) then no longer hold a finalize back until their blocks retire.
template <int WPC, int NF = 8>
__device__ __forceinline__ bool reduce_partials(int bx, const float* __restrict__ part, int nrb, int C, float& S,
                                                float& Q, int& c, int ldp = 0) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  c = bx * (4 / WPC) + wave / WPC;
  float s[NF], q[NF];
#pragma unroll
  for (int u = 0; u < NF; ++u) s[u] = q[u] = 0.f;
  if (c < C) {
    const float2* p2 = reinterpret_cast<const float2*>(part);
    const int64_t ld = ldp ? ldp : C;
    constexpr int kStride = 64 * WPC;
    int b = lane + 64 * (wave % WPC);
    for (; b + (NF - 1) * kStride < nrb; b += NF * kStride) {
#pragma unroll
      for (int u = 0; u < NF; ++u) {
        const float2 v = p2[(int64_t)(b + kStride * u) * ld + c];
        s[u] += v.x;
        q[u] += v.y;
      }
    }
    for (; b < nrb; b += kStride) {
      const float2 v = p2[(int64_t)b * ld + c];
      s[0] += v.x;
      q[0] += v.y;
    }
  }
  float ss, qq;
  if constexpr (NF == 8) {
    ss = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    qq = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  } else {
    static_assert(NF == 4, "4 or 8 loads in flight");
    ss = (s[0] + s[1]) + (s[2] + s[3]);
    qq = (q[0] + q[1]) + (q[2] + q[3]);
  }
  ss = wave_sum(ss);
  qq = wave_sum(qq);
  if constexpr (WPC > 1) {
    if (lane == 0) {
      red[0][wave] = ss;
      red[1][wave] = qq;
    }
    __syncthreads();
    if (wave % WPC != 0) return false;
    ss = qq = 0.f;
#pragma unroll
    for (int w = 0; w < WPC; ++w) {
      ss += red[0][wave + w];
      qq += red[1][wave + w];
    }
  }
  if (lane != 0 || c >= C) return false;
  S = ss;
  Q = qq;
  return true;
}

// First level of the reduction of GEMM-epilogue statistics ([nrb][C][2], one row per 128-row output
// tile: 12,544 rows for a 56x56 layer at batch 512). Lanes own consecutive channels, so each wave's
// load is one 512-byte run instead of the 64 scattered lines of the lane-per-row layout of
// reduce_partials; block (cx, g) folds rows [g * kFoldRows, +kFoldRows) into out[g][C][2] with its
// 4 waves taking every 4th row and 8 loads in flight per lane. Fixed order -> bitwise reproducible.
constexpr int kFoldRows = 128;

int bn_fold_groups(int nrb) { return nrb > 1024 ? (nrb + kFoldRows - 1) / kFoldRows : 0; }

__global__ __launch_bounds__(256) void bn_partials_fold_kernel(const float* __restrict__ part, int nrb, int C,
                                                               float* __restrict__ out, int ldp = 0) {
  __shared__ float red[4][64][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * kFoldRows, r1 = min(nrb, r0 + kFoldRows);
  float s[8], q[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s[u] = q[u] = 0.f;
  if (c < C) {
    const float2* p2 = reinterpret_cast<const float2*>(part);
    const int64_t ld = ldp ? ldp : C;
    int r = r0 + wave;
    for (; r + 28 < r1; r += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float2 v = p2[(int64_t)(r + 4 * u) * ld + c];
        s[u] += v.x;
        q[u] += v.y;
      }
    }
    for (; r < r1; r += 4) {
      const float2 v = p2[(int64_t)r * ld + c];
      s[0] += v.x;
      q[0] += v.y;
    }
  }
  red[wave][lane][0] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  red[wave][lane][1] = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  __syncthreads();
  if (wave == 0 && c < C) {
    float2 o;
    o.x = (red[0][lane][0] + red[1][lane][0]) + (red[2][lane][0] + red[3][lane][0]);
    o.y = (red[0][lane][1] + red[1][lane][1]) + (red[2][lane][1] + red[3][lane][1]);
    reinterpret_cast<float2*>(out)[(int64_t)blockIdx.y * C + c] = o;
  }
}

// Partials the finalize reads: `part` itself (<= 1024 rows), or its coalesced fold written to the
// scratch rows right after it (part + nrb * C * 2; bn_partial_floats sizes for both).
static const float* bn_fold_rows(const float* part, int* nrb, int C, hipStream_t stream) {
  const int g = bn_fold_groups(*nrb);
  if (!g) return part;
  float* out = const_cast<float*>(part) + (int64_t)*nrb * C * 2;
  hipLaunchKernelGGL(bn_partials_fold_kernel, dim3((C + 63) / 64, g), dim3(256), 0, stream, part, *nrb, C, out);
  *nrb = g;
  return out;
}

int64_t bn_partial_floats(int64_t M, int C, int target_blocks) {
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, target_blocks);
  return ((int64_t)nrb + bn_fold_groups(nrb)) * C * 2;
}

// the quad stem backward reduce runs on M / 4 quads with a 4096-block target (its per-thread work
// is 4 pixels; the default 1024 blocks leave it latency-bound)
constexpr int kQuadRedBlocks = 4096;

template <int WPC>
__device__ __forceinline__ void bn_stats_finalize_body(int bx, const void* __restrict__ x0, int x_is_bf16,
                                                                const float* __restrict__ part, int nrb, int64_t M,
                                                                int C, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps,
                                                                float momentum, float* __restrict__ running_mean,
                                                                float* __restrict__ running_var,
                                                                float* __restrict__ ws, int ldp = 0) {
  float S, Q;
  int c;
  if (!reduce_partials<WPC>(bx, part, nrb, C, S, Q, c, ldp)) return;
  const float K = x0 == nullptr ? 0.f
                  : (x_is_bf16 ? bf16_to_f32(reinterpret_cast<const bf16_t*>(x0)[c]) : reinterpret_cast<const float*>(x0)[c]);
  const float inv_m = 1.f / (float)M;
  const float dm = S * inv_m;
  const float mean = K + dm;
  const float var = fmaxf(Q * inv_m - dm * dm, 0.f);
  const float invstd = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  // ws layout: [0,C) mean  [C,2C) invstd  [2C,3C) scale  [3C,4C) shift
  ws[c] = mean;
  ws[C + c] = invstd;
  ws[2 * C + c] = g * invstd;
  ws[3 * C + c] = b - mean * g * invstd;
  if (running_mean) {
    const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

template <int WPC>
__global__ __launch_bounds__(256) void bn_stats_finalize_kernel(const void* __restrict__ x0, int x_is_bf16, const float* __restrict__ part,
                                                                int nrb, int64_t M, int C, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps, float momentum,
                                                                float* __restrict__ running_mean,
                                                                float* __restrict__ running_var, float* __restrict__ ws) {
  bn_stats_finalize_body<WPC>(blockIdx.x, x0, x_is_bf16, part, nrb, M, C, gamma, beta, eps, momentum, running_mean, running_var, ws);
}

// ---------------------------------------------------------------------------------------------
// forward: apply  y = act(x*scale + shift [+ res])
// ---------------------------------------------------------------------------------------------
// kBnRes: the residual is itself a BatchNorm input (the downsample branch of a residual block):
// y = act(x*scale + shift + (res*scale2 + shift2)) with scale2/shift2 from ws2 — the downsample BN's
// output is never written and re-read.
template <typename T, bool kRes, bool kRelu, bool kBnRes = false>
__device__ __forceinline__ void bn_apply_body(int bx, const T* __restrict__ x, const T* __restrict__ res,
                                                              T* __restrict__ y, const float* __restrict__ ws,
                                                              int64_t M, int C, int nrb, int tpr,
                                                              uint8_t* __restrict__ mask,
                                                              const float* __restrict__ ws2,
                                                              int64_t ldy, int64_t ldx = 0) {
  // ldy != 0: y is a channel slice of a wider channels_last tensor (row stride ldy), e.g. one
  // Inception branch written straight into the concatenated block output
  // Same tiling as the reduction passes: a thread owns 8 fixed channels for all its rows, so the
  // per-channel coefficients live in registers (no per-element index math or table reads).
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c0 = bx * ct + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows_rev(M, nrb, r0, r1);
  float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = ws[2 * C + c0 + j];
    sh[j] = ws[3 * C + c0 + j];
    sc2[j] = kBnRes ? ws2[2 * C + c0 + j] : 1.f;
    sh2[j] = kBnRes ? ws2[3 * C + c0 + j] : 0.f;
  }
  auto row = [&](int64_t r) {
    const int64_t off = r * C + c0;
    float a[8];
    Vec8<T>::load(x + (ldx ? r * ldx + c0 : off), a);
    float rv[8];
    if (kRes) Vec8<T>::load(res + off, rv);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = fmaf(a[j], sc[j], sh[j]);
      if (kRes) o += kBnRes ? fmaf(rv[j], sc2[j], sh2[j]) : rv[j];
      if (kRelu) {
        bits |= (o > 0.f ? 1u : 0u) << j;
        o = fmaxf(o, 0.f);
      }
      a[j] = o;
    }
    Vec8<T>::store(y + (ldy ? r * ldy + c0 : off), a);
    // ReLU-after-residual: the backward cannot recompute the branch from x alone, so record it as
    // one bit per element (1/16 of the bf16 output's bytes) instead of re-reading y.
    if (kRes && kRelu && mask) mask[off >> 3] = (uint8_t)bits;
  };
  int64_t r = r0 + rg;
  for (; r + (kUnroll - 1) * rpi < r1; r += kUnroll * rpi) {
    Raw8<T> xr[kUnroll], rr[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t off = (r + u * rpi) * C + c0;
      xr[u].load(x + (ldx ? (r + u * rpi) * ldx + c0 : off));
      if (kRes) rr[u].load(res + off);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every load of the group ahead of its arithmetic
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t off = (r + u * rpi) * C + c0;
      float a[8], rv[8];
      xr[u].get(a);
      if (kRes) rr[u].get(rv);
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float o = fmaf(a[j], sc[j], sh[j]);
        if (kRes) o += kBnRes ? fmaf(rv[j], sc2[j], sh2[j]) : rv[j];
        if (kRelu) {
          bits |= (o > 0.f ? 1u : 0u) << j;
          o = fmaxf(o, 0.f);
        }
        a[j] = o;
      }
      Vec8<T>::store(y + (ldy ? (r + u * rpi) * ldy + c0 : off), a);
      if (kRes && kRelu && mask) mask[off >> 3] = (uint8_t)bits;
    }
  }
  for (; r < r1; r += rpi) row(r);
}

template <typename T, bool kRes, bool kRelu, bool kBnRes = false>
__global__ __launch_bounds__(kBNThreads) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                                                              const float* __restrict__ ws, int64_t M, int C, int nrb,
                                                              int tpr, uint8_t* __restrict__ mask,
                                                              const float* __restrict__ ws2 = nullptr, int64_t ldy = 0) {
  bn_apply_body<T, kRes, kRelu, kBnRes>(blockIdx.x, x, res, y, ws, M, C, nrb, tpr, mask, ws2, ldy);
}

// ---------------------------------------------------------------------------------------------
// backward: reduce  Σdy', Σdy'(x-mean)
// ---------------------------------------------------------------------------------------------
// ReLU branch in backward, by mask source:
//   kMaskNone   no ReLU;
//   kMaskRecomp ReLU directly after BN: recompute x*scale+shift > 0 from x, which the backward reads
//               anyway (bit-identical to the forward's decision: same fmaf on the same operands);
//   kMaskBits   ReLU after the residual add: the 1-bit mask the forward wrote;
//   kMaskY      from the saved output (generic fallback).
enum : int { kMaskNone = 0, kMaskRecomp = 1, kMaskBits = 2, kMaskY = 3 };

template <typename T, int kMask>
__device__ __forceinline__ void apply_relu_mask(float (&g)[8], const float (&xv)[8], const float (&sc)[8],
                                                const float (&sh)[8], const T* __restrict__ y,
                                                const uint8_t* __restrict__ mask, int64_t off) {
  if constexpr (kMask == kMaskRecomp) {
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = fmaf(xv[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
  } else if constexpr (kMask == kMaskBits) {
    const uint32_t bits = mask[off >> 3];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = ((bits >> j) & 1u) ? g[j] : 0.f;
  } else if constexpr (kMask == kMaskY) {
    float yv[8];
    Vec8<T>::load(y + off, yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
  }
}

// Where the backward passes read dy from: the gradient tensor itself, or (stem BN(+ReLU) fused with
// the 3x3/s2 max-pool that follows it) gathered from the pooled gradient and the forward's 1-byte
// argmax positions — the full-resolution dy is never written.
// ld != 0: dy is a channel slice of a wider channels_last tensor (row stride ld elements), e.g. one
// Inception branch's part of the concatenated output gradient — read in place, never copied out.
template <typename T>
struct DirectDy {
  static constexpr bool kRaw = true;  // plain loads: the grouped streaming loop applies
  const T* p;
  int64_t ld = 0;
  __device__ __forceinline__ const T* at(int64_t off, int64_t r, int c0) const { return p + (ld ? r * ld + c0 : off); }
  __device__ __forceinline__ void raw(int64_t off, int64_t r, int c0, Raw8<T>& v) const { v.load(at(off, r, c0)); }
  __device__ __forceinline__ void load(int64_t off, int64_t r, int c0, int /*C*/, float (&g)[8]) const {
    Vec8<T>::load(at(off, r, c0), g);
  }
};

struct PoolDy {
  static constexpr bool kRaw = false;  // a gather per element: per-row loop
  __device__ __forceinline__ void raw(int64_t, int64_t, int, Raw8<bf16_t>&) const {}
  const bf16_t* dyp;   // pooled gradient [N, OH, OW, C]
  const uint8_t* pos;  // window position of each pooled max (forward)
  int H, W, OH, OW, k, s, pad;
  mm::FastDiv fW, fH;
  __device__ __forceinline__ void load(int64_t /*off*/, int64_t r, int c0, int C, float (&g)[8]) const {
    const uint32_t q = mm::fdiv((uint32_t)r, fW);
    const int w = (int)r - (int)q * W;
    const uint32_t n = mm::fdiv(q, fH);
    const int h = (int)q - (int)n * H;
    const int hp = h + pad, wp = w + pad;
    const int oh_lo = hp < k - 1 ? 0 : (hp - k + 1 + s - 1) / s, oh_hi = min(OH - 1, hp / s);
    const int ow_lo = wp < k - 1 ? 0 : (wp - k + 1 + s - 1) / s, ow_hi = min(OW - 1, wp / s);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = 0.f;
    if (k <= 2 * s) {
      // at most 2 x 2 windows contain the pixel: issue all four (pos, dy) loads before any use so
      // they are in flight together (the data-dependent loop below serialises them)
      uint64_t pk[4];
      ushort8_t dv[4];
      uint32_t qv[4];
      bool ok[4];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int oh = oh_hi - a, ow = ow_hi - b, t = a * 2 + b;
          ok[t] = oh >= oh_lo && ow >= ow_lo;
          const int ohc = ok[t] ? oh : oh_hi, owc = ok[t] ? ow : ow_hi;
          qv[t] = (uint32_t)((hp - ohc * s) * k + (wp - owc * s));
          const int64_t o = (((int64_t)n * OH + max(ohc, 0)) * OW + max(owc, 0)) * C + c0;
          pk[t] = *reinterpret_cast<const uint64_t*>(pos + o);
          dv[t] = *reinterpret_cast<const ushort8_t*>(dyp + o);
        }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t q = ok[t] ? qv[t] : 0xffu;  // branch-free: an out-of-range window matches nothing
        const uint32_t lo32 = (uint32_t)pk[t], hi32 = (uint32_t)(pk[t] >> 32);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t byte = ((j < 4 ? lo32 : hi32) >> (8 * (j & 3))) & 0xffu;
          g[j] += byte == q ? bf16_to_f32(dv[t][j]) : 0.f;
        }
      }
      return;
    }
    for (int oh = oh_lo; oh <= oh_hi; ++oh)
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint32_t qq = (uint32_t)((hp - oh * s) * k + (wp - ow * s));
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + c0;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(pos + o);
        float d[8];
        Vec8<bf16_t>::load(dyp + o, d);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((packed >> (8 * j)) & 0xffu) == qq) g[j] += d[j];
      }
  }
};

template <typename T, int kMask, class DY = DirectDy<T>>
__device__ __forceinline__ void bn_bwd_reduce_body(int bx, DY dy, const T* __restrict__ y,
                                                                   const uint8_t* __restrict__ mask,
                                                                   const T* __restrict__ x,
                                                                   const float* __restrict__ ws, int64_t M, int C,
                                                                   int nrb, int tpr, float* __restrict__ part, int64_t ldx = 0) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c_base = bx * ct;
  const int c0 = c_base + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows_rev(M, nrb, r0, r1);
  float mean[8], sc[8], sh[8], s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = ws[c0 + j];
    sc[j] = ws[2 * C + c0 + j];
    sh[j] = ws[3 * C + c0 + j];
    s[j] = q[j] = 0.f;
  }
  // kUnroll rows per thread per iteration with no bounds test inside the group, so all their loads
  // are in flight together (the tail loop takes the < kUnroll leftover rows)
  auto row = [&](int64_t r) {
    const int64_t off = r * C + c0;
    float g[8], xv[8];
    dy.load(off, r, c0, C, g);
    Vec8<T>::load(x + (ldx ? r * ldx + c0 : off), xv);
    apply_relu_mask<T, kMask>(g, xv, sc, sh, y, mask, off);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += g[j];
      q[j] = fmaf(g[j], xv[j] - mean[j], q[j]);
    }
  };
  int64_t r = r0 + rg;
  if constexpr (DY::kRaw && kMask != kMaskY) {
    for (; r + (kUnroll - 1) * rpi < r1; r += kUnroll * rpi) {
      Raw8<T> gr[kUnroll], xr[kUnroll];
      uint32_t mb[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        dy.raw(off, r + u * rpi, c0, gr[u]);
        xr[u].load(x + (ldx ? (r + u * rpi) * ldx + c0 : off));
        mb[u] = kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu;
      }
      __builtin_amdgcn_sched_barrier(0);  // keep every load of the group ahead of its arithmetic
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        float g[8], xv[8];
        gr[u].get(g);
        xr[u].get(xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          bool keep = true;
          if constexpr (kMask == kMaskRecomp) keep = fmaf(xv[j], sc[j], sh[j]) > 0.f;
          if constexpr (kMask == kMaskBits) keep = (mb[u] >> j) & 1u;
          const float gj = keep ? g[j] : 0.f;
          s[j] += gj;
          q[j] = fmaf(gj, xv[j] - mean[j], q[j]);
        }
      }
    }
  }
  for (; r < r1; r += rpi) row(r);
  block_reduce_write(s, q, tpr, rpi, ct, C, part, c_base, red);
}

template <typename T, int kMask, class DY = DirectDy<T>>
__global__ __launch_bounds__(kBNThreads) void bn_bwd_reduce_kernel(DY dy, const T* __restrict__ y, const uint8_t* __restrict__ mask,
                                                                   const T* __restrict__ x, const float* __restrict__ ws,
                                                                   int64_t M, int C, int nrb, int tpr,
                                                                   float* __restrict__ part) {
  bn_bwd_reduce_body<T, kMask, DY>(blockIdx.x, dy, y, mask, x, ws, M, C, nrb, tpr, part);
}

template <int WPC, int NF = 8>
__device__ __forceinline__ void bn_bwd_finalize_body(int bx, const float* __restrict__ part, int nrb, int64_t M,
                                                              int C, const float* __restrict__ gamma,
                                                              float* __restrict__ ws, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, int ldp = 0) {
  float S, Q;
  int c;
  if (!reduce_partials<WPC, NF>(bx, part, nrb, C, S, Q, c, ldp)) return;
  const float invstd = ws[C + c];
  const float g = gamma ? gamma[c] : 1.f;
  if (dgamma) dgamma[c] = Q * invstd;
  if (dbeta) dbeta[c] = S;
  const float inv_m = 1.f / (float)M;
  // dx = g*invstd*(dy' - S/M - (x-mean)*invstd^2*Q/M)
  // ws layout (bwd): [4C,5C) k1 = g*invstd  [5C,6C) m1 = S/M  [6C,7C) k2 = invstd^2*Q/M
  ws[4 * C + c] = g * invstd;
  ws[5 * C + c] = S * inv_m;
  ws[6 * C + c] = invstd * invstd * Q * inv_m;
}

// build-time A/B: -D DLA_LEAN_FINALIZE=0 restores the 8-in-flight, uncapped finalize
#ifndef DLA_LEAN_FINALIZE
#define DLA_LEAN_FINALIZE 1
#endif
#if DLA_LEAN_FINALIZE
constexpr int kFinalizeVgprs = 32, kFinalizeNF = 4;
#define DLA_FINALIZE_ATTR __attribute__((amdgpu_num_vgpr(kFinalizeVgprs)))
#else
constexpr int kFinalizeNF = 8;
#define DLA_FINALIZE_ATTR
#endif

template <int WPC>
__global__ __launch_bounds__(256) DLA_FINALIZE_ATTR void bn_bwd_finalize_kernel(
    const float* __restrict__ part, int nrb, int64_t M, int C, const float* __restrict__ gamma, float* __restrict__ ws,
    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  bn_bwd_finalize_body<WPC, kFinalizeNF>(blockIdx.x, part, nrb, M, C, gamma, ws, dgamma, dbeta);
}

template <typename T, int kMask, bool kDres, class DY = DirectDy<T>>
__device__ __forceinline__ void bn_bwd_apply_body(int bx, DY dy, const T* __restrict__ y,
                                                                  const uint8_t* __restrict__ mask,
                                                                  const T* __restrict__ x,
                                                                  const float* __restrict__ ws, T* __restrict__ dx,
                                                                  T* __restrict__ dres, int64_t M, int C, int nrb, int tpr, int64_t ldx = 0, int64_t lddx = 0) {
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c0 = bx * ct + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows(M, nrb, r0, r1);
  float mean[8], sc[8], sh[8], k1[8], m1[8], k2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = ws[c0 + j];
    sc[j] = ws[2 * C + c0 + j];
    sh[j] = ws[3 * C + c0 + j];
    k1[j] = ws[4 * C + c0 + j];
    m1[j] = ws[5 * C + c0 + j];
    k2[j] = ws[6 * C + c0 + j];
  }
  auto row = [&](int64_t r) {
    const int64_t off = r * C + c0;
    float g[8], xv[8];
    dy.load(off, r, c0, C, g);
    Vec8<T>::load(x + (ldx ? r * ldx + c0 : off), xv);
    apply_relu_mask<T, kMask>(g, xv, sc, sh, y, mask, off);
    if (kDres) Vec8<T>::store(dres + off, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = k1[j] * (g[j] - m1[j] - (xv[j] - mean[j]) * k2[j]);
    Vec8<T>::store(dx + (lddx ? r * lddx + c0 : off), xv);
  };
  int64_t r = r0 + rg;
  if constexpr (DY::kRaw && kMask != kMaskY) {
    for (; r + (kUnroll - 1) * rpi < r1; r += kUnroll * rpi) {
      Raw8<T> gr[kUnroll], xr[kUnroll];
      uint32_t mb[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        dy.raw(off, r + u * rpi, c0, gr[u]);
        xr[u].load(x + (ldx ? (r + u * rpi) * ldx + c0 : off));
        mb[u] = kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu;
      }
      __builtin_amdgcn_sched_barrier(0);  // keep every load of the group ahead of its arithmetic
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t off = (r + u * rpi) * C + c0;
        float g[8], xv[8];
        gr[u].get(g);
        xr[u].get(xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          bool keep = true;
          if constexpr (kMask == kMaskRecomp) keep = fmaf(xv[j], sc[j], sh[j]) > 0.f;
          if constexpr (kMask == kMaskBits) keep = (mb[u] >> j) & 1u;
          g[j] = keep ? g[j] : 0.f;
        }
        if (kDres) Vec8<T>::store(dres + off, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = k1[j] * (g[j] - m1[j] - (xv[j] - mean[j]) * k2[j]);
        Vec8<T>::store(dx + (lddx ? (r + u * rpi) * lddx + c0 : off), xv);
      }
    }
  }
  for (; r < r1; r += rpi) row(r);
}

template <typename T, int kMask, bool kDres, class DY = DirectDy<T>>
__global__ __launch_bounds__(kBNThreads) void bn_bwd_apply_kernel(DY dy, const T* __restrict__ y, const uint8_t* __restrict__ mask,
                                                                  const T* __restrict__ x, const float* __restrict__ ws,
                                                                  T* __restrict__ dx, T* __restrict__ dres, int64_t M,
                                                                  int C, int nrb, int tpr) {
  bn_bwd_apply_body<T, kMask, kDres, DY>(blockIdx.x, dy, y, mask, x, ws, dx, dres, M, C, nrb, tpr);
}

// ---------------------------------------------------------------------------------------------
// backward of act(BN(x) + BN_d(xd)) (the dual apply above): both BNs see the same dy' = dy masked
// by the ReLU bit, so one reduce pass reads dy (+ mask) once for both, Σdy' is shared, and one apply
// pass writes dx and dxd — the residual gradient is never materialised and dy is read twice, not 4x.
// ---------------------------------------------------------------------------------------------
template <typename T, int kMask>
__global__ __launch_bounds__(kBNThreads) void bn_bwd_dual_reduce_kernel(const T* __restrict__ dy,
                                                                        const uint8_t* __restrict__ mask,
                                                                        const T* __restrict__ x,
                                                                        const T* __restrict__ xd,
                                                                        const float* __restrict__ ws,
                                                                        const float* __restrict__ wsd, int64_t M,
                                                                        int C, int nrb, int tpr,
                                                                        float* __restrict__ part,
                                                                        float* __restrict__ partd) {
  static_assert(kMask == kMaskNone || kMask == kMaskBits, "dual BN backward: no ReLU or the forward's bit mask");
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c_base = blockIdx.x * ct;
  const int c0 = c_base + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows_rev(M, nrb, r0, r1);
  float mean[8], meand[8], s[8], q[8], qd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = ws[c0 + j];
    meand[j] = wsd[c0 + j];
    s[j] = q[j] = qd[j] = 0.f;
  }
  auto accum = [&](const float (&g0)[8], uint32_t mb, const float (&xv)[8], const float (&xdv)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = (kMask == kMaskBits && !((mb >> j) & 1u)) ? 0.f : g0[j];
      s[j] += g;
      q[j] = fmaf(g, xv[j] - mean[j], q[j]);
      qd[j] = fmaf(g, xdv[j] - meand[j], qd[j]);
    }
  };
  int64_t r = r0 + rg;
  for (; r + (kUnroll - 1) * rpi < r1; r += kUnroll * rpi) {
    Raw8<T> gr[kUnroll], xr[kUnroll], dr[kUnroll];
    uint32_t mb[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t off = (r + u * rpi) * C + c0;
      gr[u].load(dy + off);
      xr[u].load(x + off);
      dr[u].load(xd + off);
      mb[u] = kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu;
    }
    __builtin_amdgcn_sched_barrier(0);  // keep every load of the group ahead of its arithmetic
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      float g[8], xv[8], xdv[8];
      gr[u].get(g);
      xr[u].get(xv);
      dr[u].get(xdv);
      accum(g, mb[u], xv, xdv);
    }
  }
  for (; r < r1; r += rpi) {
    const int64_t off = r * C + c0;
    float g[8], xv[8], xdv[8];
    Vec8<T>::load(dy + off, g);
    Vec8<T>::load(x + off, xv);
    Vec8<T>::load(xd + off, xdv);
    accum(g, kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu, xv, xdv);
  }
  float s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s2[j] = s[j];
  block_reduce_write(s, q, tpr, rpi, ct, C, part, c_base, red);
  __syncthreads();  // red is reused
  block_reduce_write(s2, qd, tpr, rpi, ct, C, partd, c_base, red);
}

template <typename T, int kMask>
__global__ __launch_bounds__(kBNThreads) void bn_bwd_dual_apply_kernel(const T* __restrict__ dy,
                                                                       const uint8_t* __restrict__ mask,
                                                                       const T* __restrict__ x,
                                                                       const T* __restrict__ xd,
                                                                       const float* __restrict__ ws,
                                                                       const float* __restrict__ wsd,
                                                                       T* __restrict__ dx, T* __restrict__ dxd,
                                                                       int64_t M, int C, int nrb, int tpr) {
  static_assert(kMask == kMaskNone || kMask == kMaskBits, "dual BN backward: no ReLU or the forward's bit mask");
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c0 = blockIdx.x * ct + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows(M, nrb, r0, r1);
  float mean[8], k1[8], m1[8], k2[8], meand[8], k1d[8], m1d[8], k2d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = ws[c0 + j];
    k1[j] = ws[4 * C + c0 + j];
    m1[j] = ws[5 * C + c0 + j];
    k2[j] = ws[6 * C + c0 + j];
    meand[j] = wsd[c0 + j];
    k1d[j] = wsd[4 * C + c0 + j];
    m1d[j] = wsd[5 * C + c0 + j];
    k2d[j] = wsd[6 * C + c0 + j];
  }
  auto emit = [&](int64_t off, const float (&g0)[8], uint32_t mb, float (&xv)[8], float (&xdv)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = (kMask == kMaskBits && !((mb >> j) & 1u)) ? 0.f : g0[j];
      xv[j] = k1[j] * (g - m1[j] - (xv[j] - mean[j]) * k2[j]);
      xdv[j] = k1d[j] * (g - m1d[j] - (xdv[j] - meand[j]) * k2d[j]);
    }
    Vec8<T>::store(dx + off, xv);
    Vec8<T>::store(dxd + off, xdv);
  };
  int64_t r = r0 + rg;
  for (; r + (kUnroll - 1) * rpi < r1; r += kUnroll * rpi) {
    Raw8<T> gr[kUnroll], xr[kUnroll], dr[kUnroll];
    uint32_t mb[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t off = (r + u * rpi) * C + c0;
      gr[u].load(dy + off);
      xr[u].load(x + off);
      dr[u].load(xd + off);
      mb[u] = kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      float g[8], xv[8], xdv[8];
      gr[u].get(g);
      xr[u].get(xv);
      dr[u].get(xdv);
      emit((r + u * rpi) * C + c0, g, mb[u], xv, xdv);
    }
  }
  for (; r < r1; r += rpi) {
    const int64_t off = r * C + c0;
    float g[8], xv[8], xdv[8];
    Vec8<T>::load(dy + off, g);
    Vec8<T>::load(x + off, xv);
    Vec8<T>::load(xd + off, xdv);
    emit(off, g, kMask == kMaskBits ? (uint32_t)mask[off >> 3] : 0xffu, xv, xdv);
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// Block target of the reduction passes (statistics / backward reduce): kRedBlocks, or
// DLA_BN_RED_BLOCKS / set_bn_red_blocks() for A/B runs and tests. Above 1024 partial rows the
// statistics and backward-reduce finalizes read them through bn_partials_fold_kernel
// (bn_fold_rows); GEMM-epilogue backward partials (ext_part) above 1024 rows use the
// wave-per-channel bn_bwd_finalize_kernel<4> instead.
static int g_red_blocks = 0;  // 0: not set (environment / default)
void set_bn_red_blocks(int blocks) { g_red_blocks = blocks > 0 ? blocks : 0; }
int bn_red_blocks() {
  if (g_red_blocks > 0) return g_red_blocks;
  static const int v = [] {
    const char* e = std::getenv("DLA_BN_RED_BLOCKS");
    const int b = e ? std::atoi(e) : 0;
    return b > 0 ? b : kRedBlocks;
  }();
  return v;
}

void bn_geometry(int64_t M, int C, int* tpr, int* nrb, int* nct, int target_blocks) {
  if (target_blocks <= 0) target_blocks = bn_red_blocks();
  int ct = C;
  if (ct > 512) ct = 512;
  while (C % ct) ct -= 8;  // C % 8 == 0 guaranteed by the caller
  *tpr = ct / 8;
  *nct = C / ct;
  const int rpi = kBNThreads / *tpr;
  int64_t want = target_blocks / *nct;
  if (want < 1) want = 1;
  int64_t maxrb = (M + rpi - 1) / rpi;
  // keep >= 4 row iterations per thread so the per-block partial write is amortised
  int64_t cap = (M + 4 * rpi - 1) / (4 * rpi);
  if (cap < 1) cap = 1;
  *nrb = (int)std::max<int64_t>(1, std::min(std::min(want, maxrb), cap));
}

void launch_bn_fwd(const void* x, const void* res, void* y, int64_t M, int C, int dtype, const float* gamma,
                   const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                   float* ws, float* part, bool relu, bool training, hipStream_t stream, const float* ext_part,
                   int ext_nrb, uint8_t* mask, int64_t ldy) {
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, 0);
  if (training && ext_part) {
    // statistics already produced by the conv GEMM epilogue (unshifted per-row-block partials)
    // many tile rows: fold them coalesced into bn_fold_groups() rows of `part` first
    if (const int g = bn_fold_groups(ext_nrb)) {
      hipLaunchKernelGGL(bn_partials_fold_kernel, dim3((C + 63) / 64, g), dim3(256), 0, stream, ext_part, ext_nrb, C,
                         part);
      hipLaunchKernelGGL(bn_stats_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, nullptr, 0, part, g, M,
                         C, gamma, beta, eps, momentum, running_mean, running_var, ws);
    } else
      hipLaunchKernelGGL(bn_stats_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, nullptr, 0, ext_part,
                         ext_nrb, M, C, gamma, beta, eps, momentum, running_mean, running_var, ws);
  } else if (training) {
    const size_t lds = (size_t)(kBNThreads / tpr) * tpr * 8 * 2 * sizeof(float);
    if (dtype == kBF16)
      hipLaunchKernelGGL(bn_stats_kernel<bf16_t>, dim3(nct, nrb), dim3(kBNThreads), lds, stream, (const bf16_t*)x, M, C,
                         nrb, tpr, part);
    else
      hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(nct, nrb), dim3(kBNThreads), lds, stream, (const float*)x, M, C,
                         nrb, tpr, part);
    const float* fp = bn_fold_rows(part, &nrb, C, stream);
    hipLaunchKernelGGL(bn_stats_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, x, dtype == kBF16, fp,
                       nrb, M, C, gamma, beta, eps, momentum, running_mean, running_var, ws);
  }
  if (!y) return;  // statistics only (the fused BN+ReLU+max-pool applies them itself)
  int atpr, anrb, anct;
  bn_geometry(M, C, &atpr, &anrb, &anct, 4096);
#define DLA_BN_APPLY(T, R, A)                                                                                      \
  hipLaunchKernelGGL((bn_apply_kernel<T, R, A>), dim3(anct, anrb), dim3(kBNThreads), 0, stream, (const T*)x,        \
                     (const T*)res, (T*)y, (const float*)ws, M, C, anrb, atpr, mask, nullptr, ldy)
  if (dtype == kBF16) {
    if (res) { if (relu) DLA_BN_APPLY(bf16_t, true, true); else DLA_BN_APPLY(bf16_t, true, false); }
    else { if (relu) DLA_BN_APPLY(bf16_t, false, true); else DLA_BN_APPLY(bf16_t, false, false); }
  } else {
    if (res) { if (relu) DLA_BN_APPLY(float, true, true); else DLA_BN_APPLY(float, true, false); }
    else { if (relu) DLA_BN_APPLY(float, false, true); else DLA_BN_APPLY(float, false, false); }
  }
#undef DLA_BN_APPLY
}

void launch_bn_dual_apply(const void* x, const void* xd, void* y, const float* ws, const float* wsd, int64_t M, int C,
                          int dtype, bool relu, uint8_t* mask, hipStream_t stream) {
  int atpr, anrb, anct;
  bn_geometry(M, C, &atpr, &anrb, &anct, 4096);
#define DLA_BN_DUAL(T, A)                                                                                         \
  hipLaunchKernelGGL((bn_apply_kernel<T, true, A, true>), dim3(anct, anrb), dim3(kBNThreads), 0, stream,          \
                     (const T*)x, (const T*)xd, (T*)y, ws, M, C, anrb, atpr, mask, wsd)
  if (dtype == kBF16) {
    if (relu) DLA_BN_DUAL(bf16_t, true); else DLA_BN_DUAL(bf16_t, false);
  } else {
    if (relu) DLA_BN_DUAL(float, true); else DLA_BN_DUAL(float, false);
  }
#undef DLA_BN_DUAL
}

void launch_bn_bwd(const void* dy, const void* y, const uint8_t* mask, const void* x, void* dx, void* dres,
                   int64_t M, int C, int dtype, const float* gamma, float* ws, float* part, float* dgamma,
                   float* dbeta, int mask_mode, hipStream_t stream, const float* ext_part, int ext_nrb,
                   int64_t ld_dy) {
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, 0);
  if (ext_part) {
    // reduction pass already fused into the producer GEMM's epilogue
    if (ext_nrb > 1024)
      hipLaunchKernelGGL(bn_bwd_finalize_kernel<4>, dim3(C), dim3(256), 0, stream, ext_part, ext_nrb, M, C, gamma, ws,
                         dgamma, dbeta);
    else
      hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, ext_part, ext_nrb, M, C,
                         gamma, ws, dgamma, dbeta);
  } else {
  const size_t lds = (size_t)(kBNThreads / tpr) * tpr * 8 * 2 * sizeof(float);
#define DLA_BN_RED(T, K)                                                                                          \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, K>), dim3(nct, nrb), dim3(kBNThreads), lds, stream, DirectDy<T>{(const T*)dy, ld_dy}, \
                     (const T*)y, mask, (const T*)x, (const float*)ws, M, C, nrb, tpr, part)
#define DLA_BN_RED_ALL(T)                                 \
  switch (mask_mode) {                                    \
    case kMaskRecomp: DLA_BN_RED(T, kMaskRecomp); break;  \
    case kMaskBits: DLA_BN_RED(T, kMaskBits); break;      \
    case kMaskY: DLA_BN_RED(T, kMaskY); break;            \
    default: DLA_BN_RED(T, kMaskNone); break;             \
  }
  if (dtype == kBF16) { DLA_BN_RED_ALL(bf16_t) } else { DLA_BN_RED_ALL(float) }
#undef DLA_BN_RED_ALL
#undef DLA_BN_RED
  const float* fp = bn_fold_rows(part, &nrb, C, stream);  // before the launch reads nrb
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, fp, nrb, M, C, gamma, ws,
                     dgamma, dbeta);
  }
  if (!dx) return;  // finalize only (the virtual-output GEMM applies the coefficients itself)
  int atpr, anrb, anct;
  bn_geometry(M, C, &atpr, &anrb, &anct, 4096);
#define DLA_BN_BAPPLY(T, K, D)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, K, D>), dim3(anct, anrb), dim3(kBNThreads), 0, stream, DirectDy<T>{(const T*)dy, ld_dy}, \
                     (const T*)y, mask, (const T*)x, (const float*)ws, (T*)dx, (T*)dres, M, C, anrb, atpr)
#define DLA_BN_BAPPLY_ALL(T, D)                                 \
  switch (mask_mode) {                                          \
    case kMaskRecomp: DLA_BN_BAPPLY(T, kMaskRecomp, D); break;  \
    case kMaskBits: DLA_BN_BAPPLY(T, kMaskBits, D); break;      \
    case kMaskY: DLA_BN_BAPPLY(T, kMaskY, D); break;            \
    default: DLA_BN_BAPPLY(T, kMaskNone, D); break;             \
  }
  if (dtype == kBF16) {
    if (dres) { DLA_BN_BAPPLY_ALL(bf16_t, true) } else { DLA_BN_BAPPLY_ALL(bf16_t, false) }
  } else {
    if (dres) { DLA_BN_BAPPLY_ALL(float, true) } else { DLA_BN_BAPPLY_ALL(float, false) }
  }
#undef DLA_BN_BAPPLY_ALL
#undef DLA_BN_BAPPLY
}

// ---------------------------------------------------------------------------------------------
// Stem BN + ReLU + max-pool (ResNet: 112x112x64 -> 56x56x64 at batch 256 = 411 MB -> 103 MB).
// Forward: the pooled output straight from the conv output, y = max over the window of
// bf16(relu(x*scale + shift)) with PyTorch's first-max tie rule on those bf16 values, plus the
// 1-byte window position; the full-resolution activation is never written or re-read.
// Backward: the BN reduce/apply passes gather dy from the pooled gradient (PoolDy) instead of a
// materialised full-resolution gradient.
// ---------------------------------------------------------------------------------------------
// K > 0: compile-time window, all taps loaded before the first comparison.
// kFast: the flat index is decoded with multiply-shift divisions (total < 2^24, host-checked).
struct PoolDivs {
  mm::FastDiv fcg, fow, foh;
};

template <int K, bool kFast>
__global__ __launch_bounds__(256) void bn_relu_maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                                  const float* __restrict__ ws, bf16_t* __restrict__ y,
                                                                  uint8_t* __restrict__ pos, int N, int H, int W, int C,
                                                                  int OH, int OW, int k, int s, int p, PoolDivs dv) {
  const int cg = C / 8;
  const int total = N * OH * OW * cg;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    int c, ow, oh, n;
    if constexpr (kFast) {
      const int q = (int)mm::fdiv((uint32_t)t, dv.fcg);
      c = (t - q * cg) * 8;
      const int q2 = (int)mm::fdiv((uint32_t)q, dv.fow);
      ow = q - q2 * OW;
      n = (int)mm::fdiv((uint32_t)q2, dv.foh);
      oh = q2 - n * OH;
    } else {
      c = (t % cg) * 8;
      int r = t / cg;
      ow = r % OW;
      r /= OW;
      oh = r % OH;
      n = r / OH;
    }
    float sc[8], sh[8], best[8];
    uint32_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = ws[2 * C + c + j];
      sh[j] = ws[3 * C + c + j];
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    const int h0 = oh * s - p, w0 = ow * s - p;
    auto take = [&](const float (&v)[8], uint32_t q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = bf16_to_f32(f32_to_bf16(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f)));
        if (a > best[j] || (a != a && best[j] == best[j])) {
          best[j] = a;
          bi[j] = q;
        }
      }
    };
    if constexpr (K > 0) {
      float v[K * K][8];
      bool ok[K * K];
#pragma unroll
      for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int h = h0 + ky, w = w0 + kx, q = ky * K + kx;
          ok[q] = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
          const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1);
          Vec8<bf16_t>::load(x + (((int64_t)n * H + hc) * W + wc) * C + c, v[q]);
        }
      // Branch-free, in the bf16 bit domain: after the ReLU every value is >= +0 or a positive NaN
      // (the fma's canonical NaN), whose bf16 patterns order as integers exactly like the floats,
      // with NaN above everything; an out-of-range tap is -1, below every valid tap. A strict '>'
      // on these keys picks the first maximum, and the first NaN, of the rounded values — what
      // max-pooling the stored bf16 BN output gives.
      int key[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) key[j] = -1;
#pragma unroll
      for (int q = 0; q < K * K; ++q) {
        const int oor = ok[q] ? 0 : -1;  // OR-ed in: no select the compiler could turn into a branch
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kq = (int)f32_to_bf16(fmaxf(fmaf(v[q][j], sc[j], sh[j]), 0.f)) | oor;
          const bool tk = kq > key[j];
          key[j] = tk ? kq : key[j];
          bi[j] = tk ? (uint32_t)q : bi[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) best[j] = bf16_to_f32((bf16_t)key[j]);
    } else {
      for (int ky = 0; ky < k; ++ky) {
        const int h = h0 + ky;
        if (h < 0 || h >= H) continue;
        for (int kx = 0; kx < k; ++kx) {
          const int w = w0 + kx;
          if (w < 0 || w >= W) continue;
          float v[8];
          Vec8<bf16_t>::load(x + (((int64_t)n * H + h) * W + w) * C + c, v);
          take(v, (uint32_t)(ky * k + kx));
        }
      }
    }
    const int64_t off = (((int64_t)n * OH + oh) * OW + ow) * C + c;
    Vec8<bf16_t>::store(y + off, best);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (uint64_t)bi[j] << (8 * j);
    *reinterpret_cast<uint64_t*>(pos + off) = packed;
  }
}

void launch_bn_relu_maxpool_fwd(const void* x, const float* ws, void* y, uint8_t* pos, int N, int H, int W, int C,
                                int OH, int OW, int k, int s, int p, hipStream_t stream) {
  const int64_t work = (int64_t)N * OH * OW * (C / 8);
  const int nb = (int)std::min<int64_t>((work + 255) / 256, 256 * 32);
  if (nb == 0) return;
  const PoolDivs dv{mm::make_fastdiv(C / 8), mm::make_fastdiv(OW), mm::make_fastdiv(OH)};
  const bool fast = work < (1 << 24);
#define DLA_BRMP(K_, F_)                                                                                          \
  hipLaunchKernelGGL((bn_relu_maxpool_fwd_kernel<K_, F_>), dim3(nb), dim3(256), 0, stream, (const bf16_t*)x, ws,   \
                     (bf16_t*)y, pos, N, H, W, C, OH, OW, k, s, p, dv)
  if (k == 3) { if (fast) DLA_BRMP(3, true); else DLA_BRMP(3, false); }
  else { if (fast) DLA_BRMP(0, true); else DLA_BRMP(0, false); }
#undef DLA_BRMP
}

// 3x3 / stride-2 max-pool over an even H x W (ResNet stem: pad 1; GoogLeNet stem / maxpool2: pad 0,
// ceil mode): the 2x2 input quad (2j..2j+1, 2i..2i+1) is covered exactly by the windows
// (j-1+P .. j+P, i-1+P .. i+P), so a thread owning a quad loads those 4 windows' (position byte, dy)
// pairs once for its 4 pixels — the per-pixel gather (PoolDy) issues 4 candidate window loads for
// every pixel. Window (oh, ow) covers input rows 2oh-P .. 2oh-P+2; the tap of pixel (h, w) in it is
// (h - 2oh + P) * 3 + (w - 2ow + P), and a (pixel, window) pair is real when both offsets are 0..2.
template <int P>
struct StemQuad {
  const bf16_t* dyp;
  const uint8_t* pos;
  int H, W, OH, OW;
  mm::FastDiv fQW, fQH;  // quads per row (W/2), quad rows (H/2)
  // dy' of the 4 pixels of quad t (channels c0..c0+7) and their element offsets
  __device__ __forceinline__ void gather(int64_t t, int c0, int C, float (&g)[4][8], int64_t (&off)[4]) const {
    const uint32_t q = mm::fdiv((uint32_t)t, fQW);
    const int i = (int)t - (int)q * (W >> 1);
    const uint32_t n = mm::fdiv(q, fQH);
    const int j = (int)q - (int)n * (H >> 1);
    uint64_t pk[4];
    float d[4][8];
    bool ok[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = j - 1 + P + a, ow = i - 1 + P + b, w = a * 2 + b;
        ok[w] = (unsigned)oh < (unsigned)OH && (unsigned)ow < (unsigned)OW;
        const int64_t o = (((int64_t)n * OH + min(max(oh, 0), OH - 1)) * OW + min(max(ow, 0), OW - 1)) * C + c0;
        pk[w] = *reinterpret_cast<const uint64_t*>(pos + o);
        Vec8<bf16_t>::load(dyp + o, d[w]);
      }
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) g[p][e] = 0.f;
    // pixel (dh, dw) of the quad in window (a, b): ky = dh - 2a + 2 - P, kx = dw - 2b + 2 - P
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int dh = 0; dh < 2; ++dh)
#pragma unroll
          for (int dw = 0; dw < 2; ++dw) {
            constexpr int lo = 0;
            const int ky = dh - 2 * a + 2 - P, kx = dw - 2 * b + 2 - P;
            if (ky < lo || ky > 2 || kx < lo || kx > 2) continue;  // compile-time after unrolling
            const int w = a * 2 + b;
            // branch-free: a window outside the output matches no tap (0xff)
            const uint32_t tap = ok[w] ? (uint32_t)(ky * 3 + kx) : 0xffu;
            const uint32_t lo32 = (uint32_t)pk[w], hi32 = (uint32_t)(pk[w] >> 32);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t byte = ((e < 4 ? lo32 : hi32) >> (8 * (e & 3))) & 0xffu;
              g[dh * 2 + dw][e] += byte == tap ? d[w][e] : 0.f;
            }
          }
    const int64_t base = ((int64_t)n * H + 2 * j) * W + 2 * i;
    off[0] = base * C + c0;
    off[1] = (base + 1) * C + c0;
    off[2] = (base + W) * C + c0;
    off[3] = (base + W + 1) * C + c0;
  }
};

template <int P>
__global__ __launch_bounds__(kBNThreads) void bn_pool_quad_reduce_kernel(StemQuad<P> sq, const bf16_t* __restrict__ x,
                                                                         const float* __restrict__ ws, int64_t Q,
                                                                         int C, int nrb, int tpr,
                                                                         float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c_base = blockIdx.x * ct;
  const int c0 = c_base + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows(Q, nrb, r0, r1);
  float mean[8], sc[8], sh[8], s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = ws[c0 + e];
    sc[e] = ws[2 * C + c0 + e];
    sh[e] = ws[3 * C + c0 + e];
    s[e] = q[e] = 0.f;
  }
  for (int64_t t = r0 + rg; t < r1; t += rpi) {
    float g[4][8], xv[4][8];
    int64_t off[4];
    sq.gather(t, c0, C, g, off);
#pragma unroll
    for (int p = 0; p < 4; ++p) Vec8<bf16_t>::load(x + off[p], xv[p]);
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gg = fmaf(xv[p][e], sc[e], sh[e]) > 0.f ? g[p][e] : 0.f;  // the forward's ReLU
        s[e] += gg;
        q[e] = fmaf(gg, xv[p][e] - mean[e], q[e]);
      }
  }
  block_reduce_write(s, q, tpr, rpi, ct, C, part, c_base, red);
}

template <int P>
__global__ __launch_bounds__(kBNThreads) void bn_pool_quad_apply_kernel(StemQuad<P> sq, const bf16_t* __restrict__ x,
                                                                        const float* __restrict__ ws,
                                                                        bf16_t* __restrict__ dx, int64_t Q, int C,
                                                                        int nrb, int tpr) {
  const int rpi = kBNThreads / tpr, ct = tpr * 8;
  const int c0 = blockIdx.x * ct + (threadIdx.x % tpr) * 8;
  const int rg = threadIdx.x / tpr;
  int64_t r0, r1;
  block_rows(Q, nrb, r0, r1);
  float mean[8], sc[8], sh[8], k1[8], m1[8], k2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mean[e] = ws[c0 + e];
    sc[e] = ws[2 * C + c0 + e];
    sh[e] = ws[3 * C + c0 + e];
    k1[e] = ws[4 * C + c0 + e];
    m1[e] = ws[5 * C + c0 + e];
    k2[e] = ws[6 * C + c0 + e];
  }
  for (int64_t t = r0 + rg; t < r1; t += rpi) {
    float g[4][8], xv[4][8];
    int64_t off[4];
    sq.gather(t, c0, C, g, off);
#pragma unroll
    for (int p = 0; p < 4; ++p) Vec8<bf16_t>::load(x + off[p], xv[p]);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gg = fmaf(xv[p][e], sc[e], sh[e]) > 0.f ? g[p][e] : 0.f;
        xv[p][e] = k1[e] * (gg - m1[e] - (xv[p][e] - mean[e]) * k2[e]);
      }
      Vec8<bf16_t>::store(dx + off[p], xv[p]);
    }
  }
}

int64_t bn_relu_maxpool_part_floats(int64_t M, int C) {
  return std::max(bn_partial_floats(M, C), bn_partial_floats(M / 4, C, kQuadRedBlocks));
}

void launch_bn_relu_maxpool_bwd(const void* dy_pool, const uint8_t* pos, const void* x, void* dx, int N, int H, int W,
                                int C, int OH, int OW, int k, int s, int p, const float* gamma, float* ws, float* part,
                                float* dgamma, float* dbeta, hipStream_t stream) {
  const int64_t M = (int64_t)N * H * W;
  // quad form: 3x3 / stride 2 over an even input whose windows all start inside it (pad 1 floor:
  // OH = H/2; pad 0 ceil: OH = H/2 as well). Same partials layout / finalize as the per-pixel passes.
  if (k == 3 && s == 2 && (p == 0 || p == 1) && H % 2 == 0 && W % 2 == 0 && OH == H / 2 && OW == W / 2) {
    const int64_t Q = M / 4;
    const mm::FastDiv fqw = mm::make_fastdiv((uint32_t)(W / 2)), fqh = mm::make_fastdiv((uint32_t)(H / 2));
    int tpr, nrb, nct;
    bn_geometry(Q, C, &tpr, &nrb, &nct, kQuadRedBlocks);  // part sized by bn_relu_maxpool_part_floats
    const size_t lds = (size_t)(kBNThreads / tpr) * tpr * 8 * 2 * sizeof(float);
    int atpr, anrb, anct;
    bn_geometry(Q, C, &atpr, &anrb, &anct, 4096);
#define DLA_QUAD(P_)                                                                                                  \
  {                                                                                                                   \
    StemQuad<P_> sq{(const bf16_t*)dy_pool, pos, H, W, OH, OW, fqw, fqh};                                             \
    hipLaunchKernelGGL(bn_pool_quad_reduce_kernel<P_>, dim3(nct, nrb), dim3(kBNThreads), lds, stream, sq,            \
                       (const bf16_t*)x, (const float*)ws, Q, C, nrb, tpr, part);                                     \
    const float* fp = bn_fold_rows(part, &nrb, C, stream);                                                            \
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, fp, nrb, M, C, gamma, ws, \
                       dgamma, dbeta);                                                                                \
    if (dx) /* dx null: reduce + finalize only; the stem weight gradient applies it (stem_wgrad_bn_kernel) */       \
      hipLaunchKernelGGL(bn_pool_quad_apply_kernel<P_>, dim3(anct, anrb), dim3(kBNThreads), 0, stream, sq,           \
                         (const bf16_t*)x, (const float*)ws, (bf16_t*)dx, Q, C, anrb, atpr);                          \
  }
    if (p == 1) DLA_QUAD(1) else DLA_QUAD(0)
#undef DLA_QUAD
    return;
  }
  PoolDy pd{(const bf16_t*)dy_pool, pos, H, W, OH, OW, k, s, p, mm::make_fastdiv((uint32_t)W),
            mm::make_fastdiv((uint32_t)H)};
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, 0);
  const size_t lds = (size_t)(kBNThreads / tpr) * tpr * 8 * 2 * sizeof(float);
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<bf16_t, kMaskRecomp, PoolDy>), dim3(nct, nrb), dim3(kBNThreads), lds, stream,
                     pd, (const bf16_t*)nullptr, (const uint8_t*)nullptr, (const bf16_t*)x, (const float*)ws, M, C, nrb,
                     tpr, part);
  const float* fp = bn_fold_rows(part, &nrb, C, stream);  // before the launch reads nrb
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, fp, nrb, M, C, gamma, ws,
                     dgamma, dbeta);
  int atpr, anrb, anct;
  bn_geometry(M, C, &atpr, &anrb, &anct, 4096);
  hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16_t, kMaskRecomp, false, PoolDy>), dim3(anct, anrb), dim3(kBNThreads), 0,
                     stream, pd, (const bf16_t*)nullptr, (const uint8_t*)nullptr, (const bf16_t*)x, (const float*)ws,
                     (bf16_t*)dx, (bf16_t*)nullptr, M, C, anrb, atpr);
}

void launch_bn_dual_bwd(const void* dy, const uint8_t* mask, const void* x, const void* xd, void* dx, void* dxd,
                        int64_t M, int C, int dtype, const float* gamma, const float* gamma_d, float* ws, float* wsd,
                        float* part, float* partd, float* dgamma, float* dbeta, float* dgamma_d, float* dbeta_d,
                        hipStream_t stream) {
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, 0);
  const size_t lds = (size_t)(kBNThreads / tpr) * tpr * 8 * 2 * sizeof(float);
  const bool bits = mask != nullptr;
#define DLA_DUAL_RED(T, K)                                                                                        \
  hipLaunchKernelGGL((bn_bwd_dual_reduce_kernel<T, K>), dim3(nct, nrb), dim3(kBNThreads), lds, stream, (const T*)dy, \
                     mask, (const T*)x, (const T*)xd, (const float*)ws, (const float*)wsd, M, C, nrb, tpr, part, partd)
  if (dtype == kBF16) {
    if (bits) DLA_DUAL_RED(bf16_t, kMaskBits); else DLA_DUAL_RED(bf16_t, kMaskNone);
  } else {
    if (bits) DLA_DUAL_RED(float, kMaskBits); else DLA_DUAL_RED(float, kMaskNone);
  }
#undef DLA_DUAL_RED
  int fr = nrb, frd = nrb;
  const float* fp = bn_fold_rows(part, &fr, C, stream);
  const float* fpd = bn_fold_rows(partd, &frd, C, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, fp, fr, M, C, gamma, ws,
                     dgamma, dbeta);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<1>, dim3((C + 3) / 4), dim3(256), 0, stream, fpd, frd, M, C, gamma_d,
                     wsd, dgamma_d, dbeta_d);
  if (!dx) return;  // finalize only: both consumers apply the coefficients themselves (gemm_dual.hip kBN)
  int atpr, anrb, anct;
  bn_geometry(M, C, &atpr, &anrb, &anct, 4096);
#define DLA_DUAL_APPLY(T, K)                                                                                      \
  hipLaunchKernelGGL((bn_bwd_dual_apply_kernel<T, K>), dim3(anct, anrb), dim3(kBNThreads), 0, stream, (const T*)dy, \
                     mask, (const T*)x, (const T*)xd, (const float*)ws, (const float*)wsd, (T*)dx, (T*)dxd, M, C, anrb, \
                     atpr)
  if (dtype == kBF16) {
    if (bits) DLA_DUAL_APPLY(bf16_t, kMaskBits); else DLA_DUAL_APPLY(bf16_t, kMaskNone);
  } else {
    if (bits) DLA_DUAL_APPLY(float, kMaskBits); else DLA_DUAL_APPLY(float, kMaskNone);
  }
#undef DLA_DUAL_APPLY
}

// ---------------------------------------------------------------------------------------------
// Grouped BatchNorm+ReLU over the branches of a channel concatenation (an Inception block's four
// branch BNs, whose outputs are channel slices of one NHWC tensor). One launch per pass for all
// branches instead of one per branch: at GoogLeNet's 14x14 / 7x7 shapes each per-branch finalize /
// apply / reduce pass is a few-microsecond launch (profiles/googlenet_bs128_graph_r3o_ksum.md).
// Block x of a grouped grid belongs to group g for begin[g] <= x < begin[g + 1] and runs the
// single-tensor body with x - begin[g] as its channel-tile index, so every group computes exactly
// what its own launch would (same tiles, same fixed-order reductions).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int bn_group_of(const BnGroups& G, int bx) {
  int g = 0;
#pragma unroll
  for (int i = 1; i < kMaxBnGroups; ++i)
    if (i < G.n && bx >= G.begin[i]) g = i;
  return g;
}

__global__ __launch_bounds__(256) void bn_group_stats_finalize_kernel(BnGroups G, int64_t M) {
  const int g = bn_group_of(G, blockIdx.x);
  bn_stats_finalize_body<1>(blockIdx.x - G.begin[g], nullptr, 0, G.part[g], G.nrb[g], M, G.C[g], G.gamma[g],
                            G.beta[g], G.eps[g], G.mom[g], G.rm[g], G.rv[g], G.ws[g], G.ldp[g]);
}

__global__ __launch_bounds__(kBNThreads) void bn_group_apply_kernel(BnGroups G, int64_t M, int nrb) {
  const int g = bn_group_of(G, blockIdx.x);
  bn_apply_body<bf16_t, false, true, false>(blockIdx.x - G.begin[g], G.x[g], nullptr, G.y[g], G.ws[g], M, G.C[g],
                                            nrb, G.tpr[g], nullptr, nullptr, G.ldy[g], G.ldx[g]);
}

__global__ __launch_bounds__(kBNThreads) void bn_group_bwd_reduce_kernel(BnGroups G, int64_t M, int nrb) {
  const int g = bn_group_of(G, blockIdx.x);
  bn_bwd_reduce_body<bf16_t, kMaskRecomp, DirectDy<bf16_t>>(blockIdx.x - G.begin[g], DirectDy<bf16_t>{G.dy[g], G.lddy[g]},
                                                            nullptr, nullptr, G.x[g], G.ws[g], M, G.C[g], nrb,
                                                            G.tpr[g], G.wpart[g], G.ldx[g]);
}

__global__ __launch_bounds__(256) void bn_group_bwd_finalize_kernel(BnGroups G, int64_t M) {
  const int g = bn_group_of(G, blockIdx.x);
  bn_bwd_finalize_body<1>(blockIdx.x - G.begin[g], G.part[g], G.nrb[g], M, G.C[g], G.gamma[g], G.ws[g], G.dgamma[g],
                          G.dbeta[g], G.ldp[g]);
}

__global__ __launch_bounds__(kBNThreads) void bn_group_bwd_apply_kernel(BnGroups G, int64_t M, int nrb) {
  const int g = bn_group_of(G, blockIdx.x);
  bn_bwd_apply_body<bf16_t, kMaskRecomp, false, DirectDy<bf16_t>>(blockIdx.x - G.begin[g],
                                                                  DirectDy<bf16_t>{G.dy[g], G.lddy[g]}, nullptr,
                                                                  nullptr, G.x[g], G.ws[g], G.dx[g], nullptr, M, G.C[g],
                                                                  nrb, G.tpr[g], G.ldx[g], G.lddx[g]);
}

// channel tiles of each group for a pass with this block target; returns the row-block count the
// groups share (bn_geometry's rule: ~target blocks in all, >= 4 row iterations per thread)
static int bn_group_tiles(BnGroups& G, int64_t M, int target_blocks) {
  int nct_tot = 0;
  int64_t cap = INT64_MAX;
  for (int g = 0; g < G.n; ++g) {
    int tpr, nrb, nct;
    bn_geometry(M, G.C[g], &tpr, &nrb, &nct, target_blocks);
    G.tpr[g] = tpr;
    G.begin[g] = nct_tot;
    nct_tot += nct;
    const int64_t rpi = kBNThreads / tpr;
    cap = std::min<int64_t>(cap, (M + 4 * rpi - 1) / (4 * rpi));
  }
  G.begin[G.n] = nct_tot;
  const int64_t want = std::max<int64_t>(1, target_blocks / std::max(1, nct_tot));
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, cap));
}

static void bn_group_finalize_blocks(BnGroups& G) {
  int b = 0;
  for (int g = 0; g < G.n; ++g) {
    G.begin[g] = b;
    b += (G.C[g] + 3) / 4;
  }
  G.begin[G.n] = b;
}

int bn_group_bwd_rows(int64_t M, const int* C, int n) {
  BnGroups G{};
  G.n = n;
  for (int g = 0; g < n; ++g) G.C[g] = C[g];
  return bn_group_tiles(G, M, bn_red_blocks() > 1024 ? 1024 : bn_red_blocks());
}

// epilogue partials of many row tiles: fold each group's rows first (into its wpart scratch)
static void bn_group_fold(BnGroups& G, hipStream_t stream) {
  for (int g = 0; g < G.n; ++g) {
    if (const int fg = bn_fold_groups(G.nrb[g])) {
      hipLaunchKernelGGL(bn_partials_fold_kernel, dim3((G.C[g] + 63) / 64, fg), dim3(256), 0, stream, G.part[g],
                         G.nrb[g], G.C[g], G.wpart[g], G.ldp[g]);
      G.part[g] = G.wpart[g];
      G.nrb[g] = fg;
      G.ldp[g] = 0;
    }
  }
}

void launch_bn_group_fwd(BnGroups G, int64_t M, hipStream_t stream) {
  bn_group_fold(G, stream);
  bn_group_finalize_blocks(G);
  hipLaunchKernelGGL(bn_group_stats_finalize_kernel, dim3(G.begin[G.n]), dim3(256), 0, stream, G, M);
  const int nrb = bn_group_tiles(G, M, 4096);
  hipLaunchKernelGGL(bn_group_apply_kernel, dim3(G.begin[G.n], nrb), dim3(kBNThreads), 0, stream, G, M, nrb);
}

void launch_bn_group_bwd(BnGroups G, bool ext, int64_t M, hipStream_t stream) {
  if (ext) {
    bn_group_fold(G, stream);  // the dgrad epilogues' partials: one row per 128-row output tile
  } else {
    const int nrb = bn_group_tiles(G, M, bn_red_blocks() > 1024 ? 1024 : bn_red_blocks());
    const size_t lds = (size_t)kBNThreads * 8 * 2 * sizeof(float);  // rpi * ct * 2 floats for any tpr
    hipLaunchKernelGGL(bn_group_bwd_reduce_kernel, dim3(G.begin[G.n], nrb), dim3(kBNThreads), lds, stream, G, M, nrb);
    for (int g = 0; g < G.n; ++g) {
      G.part[g] = G.wpart[g];
      G.nrb[g] = nrb;
      G.ldp[g] = 0;
    }
  }
  bn_group_finalize_blocks(G);
  hipLaunchKernelGGL(bn_group_bwd_finalize_kernel, dim3(G.begin[G.n]), dim3(256), 0, stream, G, M);
  const int anrb = bn_group_tiles(G, M, 4096);
  hipLaunchKernelGGL(bn_group_bwd_apply_kernel, dim3(G.begin[G.n], anrb), dim3(kBNThreads), 0, stream, G, M, anrb);
}

}  // namespace dla
