// Virtual bottleneck output, streaming form: the passes over y3 = a2 W3^T of a ResNet bottleneck's
// last (expanding, K = P -> N = 4P, stride-1 1x1) conv with y3 recomputed in registers instead of
// stored (see ops/conv.py _Conv1x1BNResVirtual for the byte accounting).
//
// A tile-per-block GEMM (gemm.hip gemm_vy_kernel) runs each pass as load-A -> MFMA -> epilogue
// loads -> stores, one latency after the other, at ~3 TB/s: slower than the plain BatchNorm passes
// it replaces. These passes are memory streams with a tiny GEMM inside (K <= 256), so here
//   * each wave keeps its 32 output channels' weights W3[32][K] in VGPRs as MFMA A-fragments for the
//     whole kernel (no LDS at all), and the per-channel BN coefficients next to them;
//   * the GEMM is computed transposed, y3^T[ch][px] = W3 a2^T (v_mfma_f32_16x16x32_bf16 with the
//     weights as A and 16 pixels' a2 rows as B), so a lane's 4 accumulators are 4 consecutive
//     channels of ONE pixel: the residual / dy / output / dx accesses are 8-byte row segments in
//     the tensors' own channels_last layout, and the ReLU bits a nibble of the mask byte;
//   * every block is persistent over a strided set of 16-pixel groups with the next group's a2, dy /
//     residual and mask loads issued before the current group's MFMAs and stores (two ping-pong
//     register buffers), so each wave keeps a group's worth of loads in flight at all times; all
//     memory ops are buffer ops whose out-of-range offsets the hardware zero-fills / drops, so there
//     is no branch around a load and the vmcnt waits stay exact;
//   * the 4 waves of a block cover 128 channels of the same pixels (a2 rows shared through L1/L2),
//     and the N/128 channel panels of one pixel stream are placed on the same XCD (shared L2).
// Statistics / backward-reduction partials are reduced in registers and across the 16 pixel lanes,
// one [N][2] row per pixel stream ([gy][N][2] in total), fixed order (run-to-run deterministic).
// Every pass recomputes y3 with the same MFMA sequence, so all passes see bit-identical y3.
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

enum : int { kVsStats = 0, kVsApply = 1, kVsBwdReduce = 2, kVsBwdApply = 3 };

struct VsArgs {
  const bf16_t* a;  // [M][K] conv input rows (channels_last), row stride lda
  int64_t lda;
  const bf16_t* w;  // [N][K] conv weights
  int64_t M;
  int N;
  int gx, gy;       // channel panels (128 channels each) x pixel streams
  const float* ws;  // BN workspace (mean | invstd | scale | shift | k1 | m1 | k2)
  const bf16_t* src;  // apply: residual; backward: dy  ([M][N])
  bf16_t* out;        // apply: activation; backward apply: dx
  uint8_t* mask;      // apply: written; backward: read (bit c of byte (px*N + c0) >> 3)
  float* part;        // stats / backward reduce: [gy][N][2]
};

constexpr int kCF = 2;  // 16-channel fragments per wave (32 channels)
constexpr int kPanel = 4 * kCF * 16;

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

template <int KF, int PF>
struct VsBuf {
  bf16x8_t a[PF][KF];
  u32x2_t d[PF][kCF];
  uint32_t m[PF][kCF];
};

template <int MODE, int KF, int PF>
__global__ __launch_bounds__(256) void vy_stream_kernel(const VsArgs v) {
  constexpr int K = KF * 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int l = blockIdx.x, xcd = l & 7, slot = l >> 3;
  const int panel = slot % v.gx, y = (slot / v.gx) * 8 + xcd;
  const int ch0 = panel * kPanel + wave * kCF * 16;
  if (ch0 >= v.N || y >= v.gy) return;
  const int N = v.N;
  const int64_t M = v.M;
  // resident weights: A-fragment f/kf = rows ch0 + 16 f + lr, k = 32 kf + 8 g .. + 7
  bf16x8_t wf[kCF][KF];
#pragma unroll
  for (int f = 0; f < kCF; ++f) {
    const int row = ch0 + f * 16 + lr;
#pragma unroll
    for (int kf = 0; kf < KF; ++kf)
      wf[f][kf] = row < N ? *reinterpret_cast<const bf16x8_t*>(v.w + (int64_t)row * K + kf * 32 + 8 * g)
                          : bf16x8_t{};
  }
  // this lane's output channels: ch0 + 16 f + 4 g + r
  float c0[kCF][4], c1[kCF][4], c2[kCF][4], c3[kCF][4];
#pragma unroll
  for (int f = 0; f < kCF; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = min(ch0 + f * 16 + 4 * g + r, N - 1);
      c0[f][r] = c1[f][r] = c2[f][r] = c3[f][r] = 0.f;
      if constexpr (MODE == kVsApply) {
        c0[f][r] = v.ws[2 * N + c];
        c1[f][r] = v.ws[3 * N + c];
      } else if constexpr (MODE != kVsStats) {
        c0[f][r] = v.ws[c];
        if constexpr (MODE == kVsBwdApply) {
          c1[f][r] = v.ws[4 * N + c];
          c2[f][r] = v.ws[5 * N + c];
          c3[f][r] = v.ws[6 * N + c];
        }
      }
    }
  float s[kCF][4], q[kCF][4];
#pragma unroll
  for (int f = 0; f < kCF; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[f][r] = q[f][r] = 0.f;

  const int64_t ngrp = (M + 16 * PF - 1) / (16 * PF);
  // Buffer resources: an out-of-range pixel's offset is past num_records, so its loads return zeros
  // and its stores are dropped by the hardware — no branches around memory ops, so the compiler's
  // vmcnt bookkeeping stays exact and the next group's loads stay in flight during this group.
  const __amdgpu_buffer_rsrc_t ra = make_srd(v.a, (uint32_t)(M * v.lda * 2));
  const __amdgpu_buffer_rsrc_t rs = make_srd(v.src, (uint32_t)(M * N * 2));
  const __amdgpu_buffer_rsrc_t ro = make_srd(v.out, (uint32_t)(M * N * 2));
  const __amdgpu_buffer_rsrc_t rm = make_srd(v.mask, (uint32_t)((M * N + 7) / 8));
  auto load = [&](int64_t grp, VsBuf<KF, PF>& b) {
#pragma unroll
    for (int pf = 0; pf < PF; ++pf) {
      const int64_t px = grp * (16 * PF) + pf * 16 + lr;
      const bool ok = px < M;
      const uint32_t ao = ok ? (uint32_t)((px * v.lda + 8 * g) * 2) : kOOB;
#pragma unroll
      for (int kf = 0; kf < KF; ++kf) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(ra, ao, kf * 64, 0);
        b.a[pf][kf] = __builtin_bit_cast(bf16x8_t, r);
      }
      if constexpr (MODE != kVsStats) {
#pragma unroll
        for (int f = 0; f < kCF; ++f) {
          const int c = ch0 + f * 16 + 4 * g;
          const bool okc = ok && c < N;
          const uint32_t e = okc ? (uint32_t)(px * N + c) : 0u;
          const auto d = __builtin_amdgcn_raw_buffer_load_b64(rs, okc ? e * 2 : kOOB, 0, 0);
          b.d[pf][f] = __builtin_bit_cast(u32x2_t, d);
          if constexpr (MODE != kVsApply)
            b.m[pf][f] = ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rm, okc ? (e >> 3) : kOOB, 0, 0) >> (c & 4)) & 0xfu;
        }
      }
    }
  };
  auto compute = [&](int64_t grp, const VsBuf<KF, PF>& b) {
#pragma unroll
    for (int pf = 0; pf < PF; ++pf) {
      const int64_t px = grp * (16 * PF) + pf * 16 + lr;
      const bool ok = px < M;
      // the kCF accumulator chains interleaved (independent MFMAs back to back)
      f32x4_t acc[kCF];
#pragma unroll
      for (int f = 0; f < kCF; ++f) acc[f] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kf = 0; kf < KF; ++kf)
#pragma unroll
        for (int f = 0; f < kCF; ++f) acc[f] = mfma16(wf[f][kf], b.a[pf][kf], acc[f]);
#pragma unroll
      for (int f = 0; f < kCF; ++f) {
        const int c = ch0 + f * 16 + 4 * g;
        const bool okc = ok && c < N;
        const uint32_t e = okc ? (uint32_t)(px * N + c) : 0u;
        float yv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) yv[r] = bf16_to_f32(f32_to_bf16(acc[f][r]));
        if constexpr (MODE == kVsStats) {
          const float z = ok ? 1.f : 0.f;  // out-of-range pixels computed zeros; keep them out anyway
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[f][r] += yv[r] * z;
            q[f][r] = fmaf(yv[r] * z, yv[r], q[f][r]);
          }
        } else {
          const float dv[4] = {bf_lo(b.d[pf][f].x), bf_hi(b.d[pf][f].x), bf_lo(b.d[pf][f].y), bf_hi(b.d[pf][f].y)};
          if constexpr (MODE == kVsApply) {
            uint32_t nib = 0;
            float ov[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float a = fmaf(yv[r], c0[f][r], c1[f][r]);
              a += dv[r];
              nib |= (a > 0.f ? 1u : 0u) << r;
              ov[r] = fmaxf(a, 0.f);
            }
            const u32x2_t o{(uint32_t)f32_to_bf16(ov[0]) | ((uint32_t)f32_to_bf16(ov[1]) << 16),
                            (uint32_t)f32_to_bf16(ov[2]) | ((uint32_t)f32_to_bf16(ov[3]) << 16)};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0)), o),
                                                  ro, okc ? e * 2 : kOOB, 0, 0);
            // channels 4g..4g+3 and those of lane g^1 form one mask byte (bit = channel % 8)
            const uint32_t other = (uint32_t)__shfl_xor((int)nib, 16, 64);
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(nib | (other << 4)), rm,
                                                 (okc && (g & 1) == 0) ? (e >> 3) : kOOB, 0, 0);
          } else {
            float gv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) gv[r] = ((b.m[pf][f] >> r) & 1u) ? dv[r] : 0.f;
            if constexpr (MODE == kVsBwdReduce) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {  // out-of-range pixels read dy = 0, mask 0: g = 0
                s[f][r] += gv[r];
                q[f][r] = fmaf(gv[r], yv[r] - c0[f][r], q[f][r]);
              }
            } else {
              float ov[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) ov[r] = c1[f][r] * (gv[r] - c2[f][r] - (yv[r] - c0[f][r]) * c3[f][r]);
              const u32x2_t o{(uint32_t)f32_to_bf16(ov[0]) | ((uint32_t)f32_to_bf16(ov[1]) << 16),
                              (uint32_t)f32_to_bf16(ov[2]) | ((uint32_t)f32_to_bf16(ov[3]) << 16)};
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0)), o),
                                                    ro, okc ? e * 2 : kOOB, 0, 0);
            }
          }
        }
      }
    }
  };
  // ping-pong over two named register buffers (no buffer copies, so the compiler's vmcnt for one
  // buffer's loads leaves the other buffer's loads outstanding): group i+1 loads during group i
  VsBuf<KF, PF> b0, b1;
  // loads are issued unconditionally (a group past the end reads zeros through the buffer bounds and
  // touches no memory), so every path reaches a compute with the same outstanding-op count and the
  // waits stay exact
  int64_t grp = y;
  load(grp, b0);
  for (;;) {
    load(grp + v.gy, b1);
    if (grp >= ngrp) break;
    compute(grp, b0);
    load(grp + 2 * v.gy, b0);
    if (grp + v.gy >= ngrp) break;
    compute(grp + v.gy, b1);
    grp += 2 * v.gy;
  }
  if constexpr (MODE == kVsStats || MODE == kVsBwdReduce) {
    // sum over the 16 pixel lanes of each channel group (lanes 16 g .. 16 g + 15), fixed order
#pragma unroll
    for (int f = 0; f < kCF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          s[f][r] += __shfl_xor(s[f][r], sh, 64);
          q[f][r] += __shfl_xor(q[f][r], sh, 64);
        }
      }
    if (lr == 0) {
#pragma unroll
      for (int f = 0; f < kCF; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = ch0 + f * 16 + 4 * g + r;
          if (c < N) {
            v.part[((int64_t)y * N + c) * 2 + 0] = s[f][r];
            v.part[((int64_t)y * N + c) * 2 + 1] = q[f][r];
          }
        }
    }
  }
}

// Resident blocks per CU of an instantiation (its VGPR count decides: 4 waves, one per SIMD), queried
// once: the persistent grid is sized to what is resident at once, so no block starts late.
template <int MODE, int KF, int PF>
int vs_blocks_per_cu() {
  static const int n = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, vy_stream_kernel<MODE, KF, PF>, 256, 0) != hipSuccess || b < 1)
      b = 2;
    return b;
  }();
  return n;
}

template <int MODE, int KF, int PF>
void launch_vs(VsArgs v, int cus, hipStream_t stream) {
  v.gy = vy_stream_streams(v.M, v.N, cus * vs_blocks_per_cu<MODE, KF, PF>());
  hipLaunchKernelGGL((vy_stream_kernel<MODE, KF, PF>), dim3(v.gx * v.gy), dim3(256), 0, stream, v);
}

template <int MODE>
int vs_rows_k(int K, int64_t M, int N, int cus) {
  switch (K) {
    case 64: return vy_stream_streams(M, N, cus * vs_blocks_per_cu<MODE, 2, 2>());
    case 128: return vy_stream_streams(M, N, cus * vs_blocks_per_cu<MODE, 4, 2>());
    default: return vy_stream_streams(M, N, cus * vs_blocks_per_cu<MODE, 8, 1>());
  }
}

int num_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    return n;
  }();
  return cus;
}

template <int MODE>
void launch_vs_k(int K, const VsArgs& v, int cus, hipStream_t stream) {
  switch (K) {
    case 64: launch_vs<MODE, 2, 2>(v, cus, stream); break;
    case 128: launch_vs<MODE, 4, 2>(v, cus, stream); break;
    default: launch_vs<MODE, 8, 1>(v, cus, stream); break;
  }
}

}  // namespace

int vy_stream_rows(int mode, int K, int64_t M, int N) {
  return mode == kVsStats ? vs_rows_k<kVsStats>(K, M, N, num_cus()) : vs_rows_k<kVsBwdReduce>(K, M, N, num_cus());
}

bool vy_stream_supported(int K, int N) { return (K == 64 || K == 128 || K == 256) && N % 32 == 0; }

// Pixel streams: as many blocks as are resident at once (target), a multiple of 8 streams (one XCD
// per stream residue); the partials have one row per stream (vy_stream_rows gives the host the count
// a pass will use).
int vy_stream_streams(int64_t M, int N, int target_blocks) {
  const int gx = (N + kPanel - 1) / kPanel;
  int gy = (target_blocks + gx - 1) / gx;
  gy = gy / 8 * 8;
  const int64_t groups = (M + 15) / 16;
  if (gy > groups) gy = (int)((groups + 7) / 8 * 8);
  return gy < 8 ? 8 : gy;
}

void launch_vy_stream(int mode, const void* A, int64_t lda, const void* W, int64_t M, int N, int K, const float* ws,
                      const void* src, void* out, uint8_t* mask, float* part, hipStream_t stream) {
  VsArgs v;
  v.a = (const bf16_t*)A;
  v.lda = lda;
  v.w = (const bf16_t*)W;
  v.M = M;
  v.N = N;
  v.gx = (N + kPanel - 1) / kPanel;
  v.gy = 0;  // per instantiation (launch_vs)
  v.ws = ws;
  v.src = (const bf16_t*)src;
  v.out = (bf16_t*)out;
  v.mask = mask;
  v.part = part;
  const int cus = num_cus();
  switch (mode) {
    case kVsStats: launch_vs_k<kVsStats>(K, v, cus, stream); break;
    case kVsApply: launch_vs_k<kVsApply>(K, v, cus, stream); break;
    case kVsBwdReduce: launch_vs_k<kVsBwdReduce>(K, v, cus, stream); break;
    default: launch_vs_k<kVsBwdApply>(K, v, cus, stream); break;
  }
}

}  // namespace dla
