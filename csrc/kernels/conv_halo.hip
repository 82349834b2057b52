// Halo-tiled 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels (ResNet stage 1: conv2 of
// every bottleneck at 56x56), forward with the fused BatchNorm-statistics epilogue; the data
// gradient is the same convolution with the flipped, transposed weights (nn_bindings.cpp).
//
// Why a separate kernel: the implicit-GEMM path (conv.hip) gathers the A operand tap by tap, so
// every input pixel crosses L2 -> LDS nine times and every 128-row block also streams the whole
// 64 x 576 weight matrix. At N = 64 that L2 -> LDS traffic (~2.8 GB per pass at batch 512, about
// the L2-served gather rate of the chip for the whole pass) and not the MFMA work bounds the layer
// (profiles/r5e/README.md). Here a block is persistent and owns a contiguous run of 128-pixel
// strips (flat NHWC order):
//   * the 73.7 KB weight matrix is DMA'd into LDS once per block (9 tap images in the swizzled
//     row-major LDS-DMA layout of dla_mfma.h, B fragments by ds_read_b128);
//   * per strip, the flat input range [p0 - W - 1, p0 + 128 + W + 1) (the strip plus one image row
//     and one pixel of halo on each side, 242 pixels at W = 56) is DMA'd into one of two 32 KB patch
//     buffers while the previous strip is multiplied: each input pixel crosses L2 -> LDS ~1.9x
//     instead of 9x;
//   * A fragments for tap (kh, kw) are the lane's own pixel shifted by kh * W + kw inside the patch
//     (XOR-swizzled 16-byte chunks: conflict-free ds_read_b128 for any shift); taps that fall
//     outside the image (or past the tensor) read a zeroed LDS slot instead;
//   * the epilogue (bf16 tile through LDS + per-strip BN-statistics partial row) is the shared
//     epilogue_bf16 / stats_flush, so the partial-row layout equals the 128x64 implicit-GEMM tile's.
// LDS: 72 KB weights + 2 x 32 KB patches + 18 KB epilogue staging + 128 B zero slot = 154 KB: one
// 4-wave block per CU, 2x2 waves of 64 x 32 (TM = 4, TN = 2), v_mfma_f32_16x16x32_bf16.
#include <algorithm>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

constexpr int kHC = 64;                         // channels in and out
constexpr int kHBM = 128;                       // pixels per strip
constexpr int kHNT = 256;                       // threads
constexpr int kHTapImg = kHC * kBK;             // elements per weight tap image (64 x 64)
constexpr int kHWBytes = 9 * kHTapImg * 2;      // 73,728
constexpr int kHPatchBytes = 32768;             // >= (128 + 2 W + 2) * 128 B for W <= 63
constexpr int kHStageBytes = kHBM * (kHC + 8) * 2;  // epilogue staging, 18,432
constexpr int kHLds = kHWBytes + 2 * kHPatchBytes + kHStageBytes + 128;
static_assert(kHLds <= 160 * 1024, "halo conv LDS budget");
static_assert(kMS == 16, "halo conv fragments assume v_mfma_f32_16x16x32_bf16");

__device__ __forceinline__ int hswz(int s) { return s & 7; }  // chunk XOR of patch pixel s

}  // namespace

// kDirect (no statistics): the product is computed transposed (weights as the MFMA A operand, dla_mfma.h mfma_t)
// so a lane holds 4 consecutive output channels of one pixel per fragment; one v_permlane16_swap per register pair
// makes them 8 channels (16 bytes), stored straight from the registers -- no LDS staging, no epilogue barrier
// (gemm_direct.hip's mapping). With one wave per SIMD nothing hides the staged epilogue (profiles/r6/g29).
template <bool kStats, bool kDirect = false>
__global__ __launch_bounds__(kHNT, 1) void conv3x3_halo_kernel(const bf16_t* __restrict__ x,
                                                               const bf16_t* __restrict__ w,
                                                               bf16_t* __restrict__ y, int H, int W, int P,
                                                               int nstrips, int per_block,
                                                               float* __restrict__ stats,
                                                               const bf16_t* __restrict__ addend, FastDiv fW,
                                                               FastDiv fH, int fast) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  using AC = Acc<kHBM, kHC, kHNT>;
  static_assert(AC::TM == 4 && AC::TN == 2 && AC::WM == 64 && AC::WN == 32, "2x2 waves of 64 x 32");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave / AC::WGN, wc = wave % AC::WGN;
  const int s_begin = blockIdx.x * per_block;
  const int s_end = min(nstrips, s_begin + per_block);
  if (s_begin >= s_end) return;

  char* wimg = smem_raw;
  char* patch0 = smem_raw + kHWBytes;
  char* stage = patch0 + 2 * kHPatchBytes;
  char* zslot = stage + kHStageBytes;
  const uint32_t lds_w = lds_addr(wimg), lds_p0 = lds_addr(patch0);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  if (tid < 8) reinterpret_cast<ushort8_t*>(zslot)[tid] = zero8();

  // weights: 9 tap images [64 co][64 ci], slot c of image t holds row c >> 3, logical k chunk
  // rm_glds_kc(c) (the swizzle rm_glds_frag reads back)
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * kHNT;
      const bf16_t* src = w + (int64_t)(c >> 3) * (9 * kHC) + t * kHC + rm_glds_kc(c);
      glds16(src, lds_w + (uint32_t)(t * kHTapImg * 2 + i * kHNT * 16) + wofs);
    }

  const int npx = kHBM + 2 * W + 2;  // patch pixels
  // patch DMA of strip s into buffer b: slot c = pixel c >> 3, physical chunk c & 7 holding logical
  // chunk (c & 7) ^ hswz(pixel); pixels outside the tensor (and slots past the patch) read zeros
  auto issue_patch = [&](int s, int b) {
    const int64_t q0 = (int64_t)s * kHBM - W - 1;
#pragma unroll
    for (int i = 0; i < kHPatchBytes / (16 * kHNT); ++i) {
      const int c = tid + i * kHNT;
      const int px = c >> 3;
      const int64_t q = q0 + px;
      const int lc = (c & 7) ^ hswz(px);
      const void* src = (px < npx && q >= 0 && q < P) ? (const void*)(x + q * kHC + lc * 8) : zero_src();
      glds16(src, lds_p0 + (uint32_t)(b * kHPatchBytes + i * kHNT * 16) + wofs);
    }
  };
  issue_patch(s_begin, 0);

  const char* zfrag = zslot + (lane >> 4) * 16;  // zero A fragment (any logical chunk)
  for (int s = s_begin; s < s_end; ++s) {
    const int b = (s - s_begin) & 1;
    if (s == s_begin) vm_wait<0>();
    else vm_wait<4>();  // this patch's DMA is older than the previous strip's 4 tile stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 1 < s_end) issue_patch(s + 1, b ^ 1);  // that buffer was last read before this barrier

    const int64_t row0 = (int64_t)s * kHBM;
    // per A fragment: the 9-bit tap validity mask of the lane's output pixel
    uint32_t vmask[AC::TM];
#pragma unroll
    for (int i = 0; i < AC::TM; ++i) {
      const int64_t p = row0 + wr * AC::WM + i * 16 + (lane & 15);
      const int pp = (int)(p < P ? p : 0);
      // (oh, ow) of the pixel: multiply-shift divisions (exact below 2^24 pixels, checked on the host) instead of
      // two 32-bit integer divisions per fragment before the strip's first MFMA (one wave per SIMD: on the
      // critical path; profiles/r6/g29 counters)
      int q, ow, oh;
      if (fast) {
        q = (int)fdiv((uint32_t)pp, fW);
        ow = pp - q * W;
        oh = q - (int)fdiv((uint32_t)q, fH) * H;
      } else {
        q = pp / W;
        ow = pp - q * W;
        oh = q % H;
      }
      uint32_t m = 0;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          if (p < P && (unsigned)(oh + kh - 1) < (unsigned)H && (unsigned)(ow + kw - 1) < (unsigned)W)
            m |= 1u << (kh * 3 + kw);
      vmask[i] = m;
    }
    const char* pbuf = patch0 + b * kHPatchBytes;
    AC acc;
    acc.zero();
    // 18 steps (tap t, k-half kk), software-pipelined: step u + 1's fragments are read before step u's
    // MFMAs issue. With one wave per SIMD nothing else covers the LDS latency, and s_setprio is a
    // scheduling barrier, so without this every step waited for its own reads (ISA: reads, wait, 8 MFMAs)
    constexpr int kSteps = 9 * (kBK / kKS);
    auto load_step = [&](int u, bf16x8_t (&af)[AC::TM], bf16x8_t (&bfr)[AC::TN]) {
      const int t = u / (kBK / kKS), kk = u % (kBK / kKS);
      const int off = (t / 3) * W + (t % 3);
      const bf16_t* wt = reinterpret_cast<const bf16_t*>(wimg + t * kHTapImg * 2);
      // fragment i reads patch pixel wr * 64 + i * 16 + (lane & 15) + off: the chunk swizzle
      // (pixel & 7) does not depend on i, so every fragment is one base address plus an immediate
      // offset of i * 2 KB; a padding tap selects a base that lands on the zero slot instead
      const int sp0 = wr * AC::WM + (lane & 15) + off;
      const char* a0 = pbuf + sp0 * 128 + (((kk * 4 + (lane >> 4)) ^ hswz(sp0)) << 4);
#pragma unroll
      for (int i = 0; i < AC::TM; ++i) {
        const char* base = ((vmask[i] >> t) & 1u) ? a0 : zfrag - i * 2048;
        af[i] = *reinterpret_cast<const bf16x8_t*>(base + i * 2048);
      }
#pragma unroll
      for (int j = 0; j < AC::TN; ++j) bfr[j] = rm_glds_frag(wt, wc * AC::WN + j * 16, kk);
    };
    bf16x8_t af[2][AC::TM], bfr[2][AC::TN];
    load_step(0, af[0], bfr[0]);
#pragma unroll
    for (int u = 0; u < kSteps; ++u) {
      const int cb = u & 1;
      if (u + 1 < kSteps) load_step(u + 1, af[cb ^ 1], bfr[cb ^ 1]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < AC::TM; ++i)
#pragma unroll
        for (int j = 0; j < AC::TN; ++j) acc.v[i][j] = mfma_t<kDirect>(af[cb][i], bfr[cb][j], acc.v[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (kDirect && kStats) {  // the forward: the generic register-direct epilogue with statistics
      epilogue_direct<kHBM, kHC, true, kHNT>(acc, y, kHC, P, kHC, row0, 0, stats + (int64_t)s * kHC * 2, stage);
    } else if constexpr (kDirect) {  // the data gradient (+ its plain addend), same epilogue
      epilogue_direct<kHBM, kHC, false, kHNT>(acc, y, kHC, P, kHC, row0, 0, nullptr, stage, addend, kHC);
    } else {
      ColStats<kHBM, kHC, kHNT> st;
      st.zero();
      epilogue_bf16<kHBM, kHC, kStats, false, kHNT>(acc, y, kHC, P, kHC, row0, 0, st, addend, kHC, stage);
      if constexpr (kStats) stats_flush<kHBM, kHC, kHNT>(st, stats + (int64_t)s * kHC * 2, kHC, 0, stage);
    }
  }
}

// Variant 2 (two blocks per CU): the 4 waves split the strip's 64 output channels (wave tile 128 x
// 16, TM = 8 fragments along M), so each wave's B fragments for all 9 taps fit in VGPRs (9 taps x
// 2 k-halves = 72 VGPRs per lane, loaded once from L2) and a block needs only one 32 KB patch buffer
// plus the 18 KB epilogue staging: two blocks share a CU and each SIMD holds two waves of different
// blocks, whose ds_read latencies and epilogues cover each other. Per strip: compute from the patch
// -> barrier -> DMA of the next strip's patch into the same buffer -> epilogue (its stores are
// younger than that DMA, so the next strip waits with a counted vmcnt). A wave owns 16 whole
// columns, so the BN statistics need no cross-wave combine.
constexpr int kH2Lds = kHPatchBytes + kHStageBytes;

// kDirect: the product computed transposed, so a lane holds 4 consecutive output channels of one pixel per
// fragment: the tile leaves as 8-byte stores straight from the registers, the statistics are an in-lane sum over
// the 8 fragments plus a 16-lane DPP row sum (a wave owns its 16 channels), no LDS staging, no epilogue barriers.
template <bool kStats, bool kDirect = false>
__global__ __launch_bounds__(kHNT, 2) void conv3x3_halo_rb_kernel(const bf16_t* __restrict__ x,
                                                                  const bf16_t* __restrict__ w,
                                                                  bf16_t* __restrict__ y, int H, int W, int P,
                                                                  int nstrips, int per_block,
                                                                  float* __restrict__ stats,
                                                                  const bf16_t* __restrict__ addend, FastDiv fW,
                                                                  FastDiv fH, int fast) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int TM = kHBM / 16;  // 8 fragments along M per wave
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int s_begin = blockIdx.x * per_block;
  const int s_end = min(nstrips, s_begin + per_block);
  if (s_begin >= s_end) return;

  char* patch = smem_raw;
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem_raw + kHPatchBytes);
  const uint32_t lds_p = lds_addr(patch);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);

  const int npx = kHBM + 2 * W + 2;
  auto issue_patch = [&](int s) {
    const int64_t q0 = (int64_t)s * kHBM - W - 1;
#pragma unroll
    for (int i = 0; i < kHPatchBytes / (16 * kHNT); ++i) {
      const int c = tid + i * kHNT;
      const int px = c >> 3;
      const int64_t q = q0 + px;
      const int lc = (c & 7) ^ hswz(px);
      const void* src = (px < npx && q >= 0 && q < P) ? (const void*)(x + q * kHC + lc * 8) : zero_src();
      glds16(src, lds_p + (uint32_t)(i * kHNT * 16) + wofs);
    }
  };
  issue_patch(s_begin);
  // B fragments (the layout rm_glds_frag returns): lane -> output channel wave * 16 + (lane & 15),
  // 8 k values at (lane >> 4) * 8 of the tap's 32-deep half kk
  bf16x8_t bw[9][2];
  {
    const bf16_t* wrow = w + (int64_t)(wave * 16 + (lane & 15)) * (9 * kHC) + (lane >> 4) * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bw[t][kk] = *reinterpret_cast<const bf16x8_t*>(wrow + t * kHC + kk * 32);
  }

  for (int s = s_begin; s < s_end; ++s) {
    if (s == s_begin) vm_wait<0>();
    else vm_wait<kDirect ? TM : 4>();  // the patch DMA is older than the previous strip's tile stores (4 staged
                                       // 16-byte / TM direct 8-byte stores per lane; addend loads are waited by use)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    const int64_t row0 = (int64_t)s * kHBM;
    uint32_t vmask[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t p = row0 + i * 16 + (lane & 15);
      const int pp = (int)(p < P ? p : 0);
      // (oh, ow) of the pixel: multiply-shift divisions (exact below 2^24 pixels, checked on the host) instead of
      // two 32-bit integer divisions per fragment before the strip's first MFMA (one wave per SIMD: on the
      // critical path; profiles/r6/g29 counters)
      int q, ow, oh;
      if (fast) {
        q = (int)fdiv((uint32_t)pp, fW);
        ow = pp - q * W;
        oh = q - (int)fdiv((uint32_t)q, fH) * H;
      } else {
        q = pp / W;
        ow = pp - q * W;
        oh = q % H;
      }
      uint32_t m = 0;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          if (p < P && (unsigned)(oh + kh - 1) < (unsigned)H && (unsigned)(ow + kw - 1) < (unsigned)W)
            m |= 1u << (kh * 3 + kw);
      vmask[i] = m;
    }
    accv_t acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[i] = accv_t{};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int off = (t / 3) * W + (t % 3);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t af[TM];
        // fragment i reads patch pixel i * 16 + (lane & 15) + off: the swizzle (pixel & 7) does not
        // depend on i, so all 8 reads share one address plus an immediate offset of i * 2 KB; taps
        // outside the image are zeroed after the read (the address stays inside the patch)
        const int sp0 = (lane & 15) + off;
        const char* a0 = patch + sp0 * 128 + (((kk * 4 + (lane >> 4)) ^ hswz(sp0)) << 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(a0 + i * 2048);
          af[i] = ((vmask[i] >> t) & 1u) ? v : bf16x8_t{};
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i] = mfma_t<kDirect>(af[i], bw[t][kk], acc[i]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // every wave's patch reads have returned before the next strip's DMA overwrites the buffer
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + 1 < s_end) issue_patch(s + 1);

    if constexpr (kDirect) {
      // acc[i][r]: channel wave * 16 + 4 g + r of pixel row0 + 16 i + p
      const int g = lane >> 4, p = lane & 15;
      const int ch = wave * 16 + 4 * g;
      typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
      typedef float f32x2_t __attribute__((ext_vector_type(2)));
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      auto pack = [](float a, float b) {
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
      };
      u32x2_t dv[TM];
      if (addend) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int64_t m = row0 + 16 * i + p;
          dv[i] = m < P ? *reinterpret_cast<const u32x2_t*>(addend + m * kHC + ch) : u32x2_t{0u, 0u};
        }
      }
      float cs[4] = {0.f, 0.f, 0.f, 0.f}, cq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int64_t m = row0 + 16 * i + p;
        u32x2_t v{pack(acc[i][0], acc[i][1]), pack(acc[i][2], acc[i][3])};
        if constexpr (kStats) {  // statistics of the stored (bf16-rounded) values; rows past P count 0
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t w2 = v[r >> 1];
            const float f = m < P ? __builtin_bit_cast(float, (r & 1) ? (w2 & 0xffff0000u) : (w2 << 16)) : 0.f;
            cs[r] += f;
            cq[r] = fmaf(f, f, cq[r]);
          }
        }
        if (addend) {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float lo = __builtin_bit_cast(float, v[e] << 16) + __builtin_bit_cast(float, dv[i][e] << 16);
            const float hi = __builtin_bit_cast(float, v[e] & 0xffff0000u) +
                             __builtin_bit_cast(float, dv[i][e] & 0xffff0000u);
            v[e] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
          }
        }
        if (m < P) *reinterpret_cast<u32x2_t*>(y + m * kHC + ch) = v;
      }
      if constexpr (kStats) {  // sum the 16 pixel lanes of each row: lane p = 0 of row g holds its 4 channels
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int x = 1; x < 16; x <<= 1) {
            cs[r] += __shfl_xor(cs[r], x, kWave);
            cq[r] += __shfl_xor(cq[r], x, kWave);
          }
        }
        if (p == 0) {
          float* dst = stats + ((int64_t)s * kHC + ch) * 2;
          *reinterpret_cast<float4_t*>(dst) = float4_t{cs[0], cq[0], cs[1], cq[1]};
          *reinterpret_cast<float4_t*>(dst + 4) = float4_t{cs[2], cq[2], cs[3], cq[3]};
        }
      }
      continue;
    }

    // epilogue: bf16 tile -> LDS (pitch 72) -> 16-byte row stores (+ addend); per-column statistics of
    // the stored values straight from the accumulators (a lane owns one column of each fragment)
    constexpr int LDC = kHC + 8;
    const int col = wave * 16 + (lane & 15);
    float cs = 0.f, cq = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < kAccN; ++r) {
        const int m = i * 16 + acc_row(lane, r);
        const bf16_t h = f32_to_bf16(acc[i][r]);
        Cs[m * LDC + col] = h;
        if constexpr (kStats) {
          const float v = (row0 + m < P) ? bf16_to_f32(h) : 0.f;
          cs += v;
          cq = fmaf(v, v, cq);
        }
      }
    if constexpr (kStats) {
      cs += __shfl_xor(cs, 16, kWave);
      cq += __shfl_xor(cq, 16, kWave);
      cs += __shfl_xor(cs, 32, kWave);
      cq += __shfl_xor(cq, 32, kWave);
      if (lane < 16) {
        stats[((int64_t)s * kHC + col) * 2 + 0] = cs;
        stats[((int64_t)s * kHC + col) * 2 + 1] = cq;
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kHBM * (kHC / 8) / kHNT; ++it) {
      const int c = tid + it * kHNT;
      const int r = c >> 3, cc = (c & 7) * 8;
      const int64_t gm = row0 + r;
      if (gm < P) {
        ushort8_t v = *reinterpret_cast<const ushort8_t*>(Cs + r * LDC + cc);
        if (addend) {
          const ushort8_t d = *reinterpret_cast<const ushort8_t*>(addend + gm * kHC + cc);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) + bf16_to_f32(d[j]));
        }
        *reinterpret_cast<ushort8_t*>(y + gm * kHC + cc) = v;
      }
    }
    __syncthreads();  // staging reads done before the next strip's epilogue writes it
  }
}

// DLA_HALO: 0 off, 1 data gradient only, 2 (default) forward and data gradient. Per-layer A/B at
// ResNet-50 bs512 (profiles/r5l, after trimming the per-fragment address VALU to one base select):
// dgrad 0.203-0.220 vs 0.228-0.255 ms, forward 0.225-0.234 vs 0.230-0.252 ms; the forward is
// bitwise equal to the implicit-GEMM kernel (same tap / k order), so the switch changes no numerics.
static int halo_mode() {
  static const int v = [] {
    const char* e = std::getenv("DLA_HALO");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

bool halo_conv_eligible(int Cin, int Cout, int W, int stride, bool fwd) {
  return halo_mode() >= (fwd ? 2 : 1) && Cin == kHC && Cout == kHC && stride == 1 && W >= 1 &&
         2 * W + 2 + kHBM <= 256;
}

void launch_conv3x3_halo(const void* x, const void* w, void* y, int N, int H, int W, float* stats,
                         hipStream_t stream, const void* addend) {
  const int64_t P64 = (int64_t)N * H * W;
  const int P = (int)P64;
  const int nstrips = (P + kHBM - 1) / kHBM;
  if (nstrips == 0) return;
  static const int cus = [] {
    int dev = 0, n = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  // DLA_HALO_V: 1 the one-block-per-CU variant with LDS-resident weights, 2 the two-blocks-per-CU variant with
  // VGPR-resident weights (forward -4 %, dgrad +5 % vs variant 1: profiles/r5j), 3 (default) 2 for the forward, 1 for
  // the data gradient
  // DLA_HALO_V=3: variant 2 for the forward (it carries the statistics epilogue), variant 1 for the data gradient
  // -- the per-direction winners of profiles/r5j (forward 0.228-0.231 vs 0.238-0.246 ms, data gradient 0.209-0.221
  // vs 0.221-0.233 ms at bs512)
  static const int ver_env = [] {
    const char* e = std::getenv("DLA_HALO_V");
    return e ? std::atoi(e) : 3;  // default 3 since profiles/r6/g32 (step 80.17 vs 80.33 ms median, interleaved x3)
  }();
  const int ver = ver_env == 3 ? (stats ? 2 : 1) : ver_env;
  const int slots = ver == 1 ? cus : 2 * cus;
  const int per_block = (nstrips + slots - 1) / slots;
  const int grid = (nstrips + per_block - 1) / per_block;
  const bf16_t* xp = (const bf16_t*)x;
  const bf16_t* wp = (const bf16_t*)w;
  const bf16_t* ap = (const bf16_t*)addend;
  bf16_t* yp = (bf16_t*)y;
  // DLA_HALO_FASTDIV=0: the integer-division form of the per-strip tap masks (A/B)
  static const int fast = [] {
    const char* e = std::getenv("DLA_HALO_FASTDIV");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  const FastDiv fW = make_fastdiv((uint32_t)W), fH = make_fastdiv((uint32_t)H);
  const int use_fast = (P < (1 << 24) && W < (1 << 16) && H < (1 << 16)) ? fast : 0;  // fdiv's exact range
  // the variant-1 data gradient stores from registers (kDirect; default since profiles/r6/g34: -0.14 ms/step,
  // interleaved x3); DLA_HALO_DIRECT=0 restores the LDS-staged epilogue
  static const bool direct = [] {
    const char* e = std::getenv("DLA_HALO_DIRECT");
    return !(e && e[0] == '0');
  }();
  // DLA_HALO_DIRECT_FWD=1: the variant-2 forward stores from registers as well (A/B)
  static const bool direct_fwd = [] {
    const char* e = std::getenv("DLA_HALO_DIRECT_FWD");
    return e && e[0] == '1';
  }();
  if (ver == 1) {
    if (stats && direct_fwd && !addend)
      hipLaunchKernelGGL((conv3x3_halo_kernel<true, true>), dim3(grid), dim3(kHNT), kHLds, stream, xp, wp, yp, H, W,
                         P, nstrips, per_block, stats, ap, fW, fH, use_fast);
    else if (stats)
      hipLaunchKernelGGL(conv3x3_halo_kernel<true>, dim3(grid), dim3(kHNT), kHLds, stream, xp, wp, yp, H, W, P,
                         nstrips, per_block, stats, ap, fW, fH, use_fast);
    else if (direct)
      hipLaunchKernelGGL((conv3x3_halo_kernel<false, true>), dim3(grid), dim3(kHNT), kHLds, stream, xp, wp, yp, H, W,
                         P, nstrips, per_block, stats, ap, fW, fH, use_fast);
    else
      hipLaunchKernelGGL(conv3x3_halo_kernel<false>, dim3(grid), dim3(kHNT), kHLds, stream, xp, wp, yp, H, W, P,
                         nstrips, per_block, stats, ap, fW, fH, use_fast);
  } else {
    if (stats && direct_fwd)
      hipLaunchKernelGGL((conv3x3_halo_rb_kernel<true, true>), dim3(grid), dim3(kHNT), kH2Lds, stream, xp, wp, yp, H,
                         W, P, nstrips, per_block, stats, ap, fW, fH, use_fast);
    else if (stats)
      hipLaunchKernelGGL(conv3x3_halo_rb_kernel<true>, dim3(grid), dim3(kHNT), kH2Lds, stream, xp, wp, yp, H, W,
                         P, nstrips, per_block, stats, ap, fW, fH, use_fast);
    else
      hipLaunchKernelGGL(conv3x3_halo_rb_kernel<false>, dim3(grid), dim3(kHNT), kH2Lds, stream, xp, wp, yp, H, W,
                         P, nstrips, per_block, stats, ap, fW, fH, use_fast);
  }
}

}  // namespace dla
