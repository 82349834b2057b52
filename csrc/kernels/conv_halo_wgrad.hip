// Halo-tiled weight gradient of the 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels
// (ResNet stage 1: conv2 of every bottleneck at 56x56):
//   dW[co][kh][kw][ci] = sum over pixels p of dy[p][co] * x[p + (kh-1, kw-1)][ci].
//
// The implicit-GEMM weight gradient (conv.hip conv3x3_wgrad_kernel) gathers the x operand tap by tap:
// every input pixel crosses L2 -> LDS nine times and its 64-row output tile (Cout = 64) leaves the
// 8-wave MFMA loop a quarter empty (profiles/r3: 0.6 ms per layer at bs1024, 18 % MFMA busy). Here:
//   * the reduction runs over a PADDED pixel space, (N, H + 2, W + 2) with zero rows / columns around
//     every image: a tap is then one constant row shift, (kh - 1)(W + 2) + kw - 1, for every pixel, and the
//     zero halo (loaded as out-of-range DMA = zeros) makes out-of-image taps vanish with no masking;
//   * a block is persistent over a contiguous run of 128-position strips. x rows arrive by LDS-DMA into
//     a 512-row ring (64 KB, k-major transposing-read image): each strip DMAs only its 128 NEW rows, so
//     every x pixel crosses L2 -> LDS once, not 9x (or the 1.9x of a per-strip halo patch); dy rows go
//     into a 3-slot ring; both two strips ahead of the MFMAs (counted vmcnt, one barrier per strip);
//   * wave w owns input channels 16w .. 16w+15 for all 64 output channels and all 9 taps
//     (36 accumulator fragments): per 32-deep k-step it reads the 4 dy fragments once and one shifted
//     x fragment per tap, 13 transposing fragment reads per 36 MFMAs;
//   * one fp32 partial [64][9][64] per block, summed by the split-K reduction kernel (fixed order).
#include <algorithm>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

constexpr int kWC = 64;                    // channels in and out
constexpr int kWS = 128;                   // positions per strip
constexpr int kWRing = 512;                // x ring rows
constexpr int kWRingBytes = kWRing * kWC * 2;  // 65,536
constexpr int kWDyBytes = kWS * kWC * 2;       // 16,384
constexpr int kWDySlots = 3;
constexpr int kWLds = kWRingBytes + kWDySlots * kWDyBytes;  // 114,688
static_assert(kMS == 16, "halo wgrad fragments assume v_mfma_f32_16x16x32_bf16");

struct HaloWgradArgs {
  const bf16_t* x;   // [P][64] channels_last input
  const bf16_t* dy;  // [P][64] output gradient
  float* part;       // [grid][64 co][9][64 ci]
  int H, W, Q;       // image size, padded positions N (H+2) (W+2)
  int nstrips, per_block;
  FastDiv fWp, fHp;  // W + 2, H + 2
};

// pixel offset (elements) of padded position q, or -1 for padding / past the end
__device__ __forceinline__ int64_t padded_pixel(const HaloWgradArgs& a, int64_t q) {
  if (q < 0 || q >= a.Q) return -1;
  const uint32_t r = fdiv((uint32_t)q, a.fWp);
  const int wp = (int)q - (int)r * (a.W + 2);
  const uint32_t n = fdiv(r, a.fHp);
  const int hp = (int)r - (int)n * (a.H + 2);
  if (hp < 1 || hp > a.H || wp < 1 || wp > a.W) return -1;
  return (((int64_t)n * a.H + hp - 1) * a.W + wp - 1) * kWC;
}

}  // namespace

__global__ __launch_bounds__(256, 1) void conv3x3_halo_wgrad_kernel(const HaloWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int s_begin = blockIdx.x * a.per_block;
  const int s_end = min(a.nstrips, s_begin + a.per_block);
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* dys = reinterpret_cast<bf16_t*>(smem_raw + kWRingBytes);
  const uint32_t lds_ring = lds_addr(ring), lds_dy = lds_addr(dys);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  const int Wp = a.W + 2;
  const int sh0 = Wp + 1;  // largest tap shift; strip s's new x rows start at s * 128 + sh0
  // ring row of position q = (q + ring_off) mod 512, ring_off = -sh0 mod 128: every strip's new rows start
  // on a 128-row boundary of the ring
  const int ring_off = ((kWS - sh0) % kWS + kWS) % kWS;

  // DMA of x rows [q_lo, q_lo + 32 * nchunks_per_thread) (q_lo + ring_off a multiple of 128) in 16-byte
  // chunks: slot c -> row c >> 3, logical 16-byte chunk from the k-major image swizzle (km_glds_col<64>)
  auto issue_x = [&](int64_t q_lo, int nchunks_per_thread) {
    for (int i = 0; i < nchunks_per_thread; ++i) {
      const int c = tid + i * 256;
      const int r = c >> 3;
      const int64_t q = q_lo + r;
      const int ring_row = (int)((q + ring_off) & (kWRing - 1));
      const int col = km_glds_col<kWC>(ring_row * 8 + (c & 7));
      const int64_t px = padded_pixel(a, q);
      const void* src = px >= 0 ? (const void*)(a.x + px + col) : zero_src();
      // the 64 lanes of a wave cover 8 consecutive ring rows (no wrap inside a 32-row group)
      const uint32_t dst = lds_ring + (uint32_t)(((int)((q_lo + ring_off + i * 32) & (kWRing - 1))) * kWC * 2) + wofs;
      glds16(src, dst);
    }
  };
  auto issue_dy = [&](int s) {
    const int64_t q0 = (int64_t)s * kWS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * 256;
      const int r = c >> 3;
      const int col = km_glds_col<kWC>(c);
      const int64_t px = padded_pixel(a, q0 + r);
      const void* src = px >= 0 ? (const void*)(a.dy + px + col) : zero_src();
      glds16(src, lds_dy + (uint32_t)((s % kWDySlots) * kWDyBytes + i * 256 * 16) + wofs);
    }
  };
  // strip s's group: its new x rows [s*128 + sh0, s*128 + sh0 + 128) and its dy rows (4 + 4 DMAs per thread)
  auto issue_strip = [&](int s) {
    const int64_t q0 = (int64_t)s * kWS;
    issue_x(q0 + sh0, 4);
    issue_dy(s);
  };

  accv_t acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[t][i] = accv_t{};

  if (s_begin < s_end) {
    // prologue: strip s_begin's halo rows [q0 - sh0, q0 + sh0) below its new rows (rounded to a whole
    // 128-row block so every wave's 8-row DMA group stays inside the ring), then groups s_begin, s_begin+1
    const int64_t q0 = (int64_t)s_begin * kWS;
    issue_x(q0 + sh0 - kWS, 4);
    issue_strip(s_begin);
    issue_strip(s_begin + 1);  // past the end: zero rows / zero dy (contributes nothing)
  }
  // LDS byte offsets (within the ring) of the two transposing reads of each (k-step, tap) step u of a strip:
  // the XOR swizzle depends on ring-row bits 1 and 3 only, so the next strip's offsets are these plus 128 rows
  // (16 KB) mod the 64 KB ring -- two VALU per offset per strip instead of the row wrap and swizzle per read
  constexpr int kSteps = kWS / 32 * 9;
  const int xg = lane >> 4, xqq = (lane & 15) >> 2, xp = lane & 3;
  const int xcn = wave * 16 + 4 * xp;
  uint32_t xo[kSteps][2];
  {
    const int rb0 = (int)(((int64_t)s_begin * kWS + 8 * xg + xqq + ring_off - (Wp + 1)) & (kWRing - 1));
#pragma unroll
    for (int u = 0; u < kSteps; ++u) {
      const int kk = u / 9, t = u % 9;
      const int o = kk * 32 + (t / 3) * Wp + (t % 3);
      const int r0 = (rb0 + o) & (kWRing - 1), r1 = (rb0 + o + 4) & (kWRing - 1);
      xo[u][0] = (uint32_t)tr_off<kWC>(r0, xcn) * 2u;
      xo[u][1] = (uint32_t)tr_off<kWC>(r1, xcn) * 2u;
    }
  }
  for (int s = s_begin; s < s_end; ++s) {
    // strip s's group is done once only strip s+1's group (8 DMAs per thread) is younger
    vm_wait<8>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // strip s+2: its new x rows overwrite ring rows last used by strip s-1, its dy slot strip s-1's
    issue_strip(s + 2);

    const int64_t q0 = (int64_t)s * kWS;
    const bf16_t* dyb = dys + (s % kWDySlots) * (kWDyBytes / 2);
    const int g = xg, qq = xqq, p = xp;
    (void)q0;
    // The 36 (k-step, tap) steps of the strip run as one unrolled sequence: step u's 4 MFMAs issue while
    // the x fragment of step u + 2 (and, in the last 4 taps of a k-step, one dy fragment of the next
    // k-step) is read. One wave per SIMD, so nothing else hides the LDS latency; and lgkmcnt is a 4-bit
    // count, so a deeper run of reads would make hipcc's waits drain to 0.
    bf16x8_t af[2][4], bx[3];
    auto load_a = [&](int kk, int b, int i) {
      const int kr = kk * 32 + 8 * g + qq;
      af[b][i] = tr_frag(dyb + tr_off<kWC>(kr, 16 * i + 4 * p), dyb + tr_off<kWC>(kr + 4, 16 * i + 4 * p));
    };
    auto load_x = [&](int u) {
      const char* rg = reinterpret_cast<const char*>(ring);
      bx[u % 3] = tr_frag(reinterpret_cast<const bf16_t*>(rg + xo[u][0]), reinterpret_cast<const bf16_t*>(rg + xo[u][1]));
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) load_a(0, 0, i);
    load_x(0);
    load_x(1);
#pragma unroll
    for (int u = 0; u < kSteps; ++u) {
      const int kk = u / 9, t = u % 9;
      if (u + 2 < kSteps) load_x(u + 2);
      const bool la = t >= 5 && kk + 1 < kWS / 32;
      if (la) load_a(kk + 1, (kk + 1) & 1, t - 5);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][i] = mfma(af[kk & 1][i], bx[u % 3], acc[t][i]);
      __builtin_amdgcn_s_setprio(0);
      if (u + 2 < kSteps) {
        if (la) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        else __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
#pragma unroll
    for (int u = 0; u < kSteps; ++u) {
      xo[u][0] = (xo[u][0] + kWS * kWC * 2u) & (uint32_t)(kWRingBytes - 1);
      xo[u][1] = (xo[u][1] + kWS * kWC * 2u) & (uint32_t)(kWRingBytes - 1);
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the block's LDS is released
  // partial slab: acc[t][i] lane value r = dW[co = 16 i + 4 g + r][t][ci = 16 wave + (lane & 15)]
  float* out = a.part + (int64_t)blockIdx.x * (kWC * 9 * kWC);
  const int ci = wave * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[((16 * i + 4 * g + r) * 9 + t) * kWC + ci] = acc[t][i][r];
}

static int g_halo_wgrad = -1;  // -1: environment (DLA_HALO_WGRAD, default on), 0 off, 1 on
void set_halo_wgrad(int mode) { g_halo_wgrad = mode < 0 ? -1 : (mode ? 1 : 0); }

bool halo_wgrad_eligible(int Cin, int Cout, int W, int stride) {
  static const bool env_on = [] {
    const char* e = std::getenv("DLA_HALO_WGRAD");
    return !(e && e[0] == '0');
  }();
  const bool on = g_halo_wgrad < 0 ? env_on : g_halo_wgrad == 1;
  // ring: the 2 (W + 2) + 2 halo rows plus three 128-row strips in flight must fit 512 rows
  return on && Cin == kWC && Cout == kWC && stride == 1 && W >= 1 && 2 * (W + 2) + 2 + 3 * kWS <= kWRing;
}

static int halo_wgrad_grid(int64_t Q) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int64_t nstrips = (Q + kWS - 1) / kWS;
  const int64_t per = (nstrips + cus - 1) / cus;
  return (int)((nstrips + per - 1) / per);
}

int halo_wgrad_splits(int N, int H, int W) { return halo_wgrad_grid((int64_t)N * (H + 2) * (W + 2)); }

void launch_conv3x3_halo_wgrad(const void* dy, const void* x, float* partial, int splits, void* dw, int out_dtype,
                               int N, int H, int W, hipStream_t stream) {
  const int64_t Q = (int64_t)N * (H + 2) * (W + 2);
  HaloWgradArgs a{};
  a.x = (const bf16_t*)x;
  a.dy = (const bf16_t*)dy;
  a.part = partial;
  a.H = H;
  a.W = W;
  a.Q = (int)Q;
  a.nstrips = (int)((Q + kWS - 1) / kWS);
  a.per_block = (a.nstrips + splits - 1) / splits;
  a.fWp = make_fastdiv((uint32_t)(W + 2));
  a.fHp = make_fastdiv((uint32_t)(H + 2));
  hipLaunchKernelGGL(conv3x3_halo_wgrad_kernel, dim3(splits), dim3(256), kWLds, stream, a);
  launch_splitk_reduce(partial, splits, (int64_t)kWC * 9 * kWC, dw, out_dtype, 1.f, false, stream);
}

}  // namespace dla
