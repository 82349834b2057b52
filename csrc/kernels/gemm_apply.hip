// 1x1-convolution forward over a deferred BatchNorm(+residual)+ReLU output ("apply on load").
//
// A bottleneck block ends in  out = relu(BN3(y) + r)  (r: the block input, or BN_d(y_d), the downsample
// shortcut's BN); `out` feeds the next block's conv1 and its identity path. Unfused, the apply pass reads y and
// r and writes out (+ its 1-bit ReLU mask), then conv1 reads out again. Here conv1's GEMM reads y and r itself:
// while staging its A operand it applies the BN(s), the add and the ReLU, writes out and the mask once (from
// the blocks of column panel 0; every element of A is in exactly one of them) and multiplies the same values.
// The block output is never re-read: one activation-sized read less per block (2.06 GB at stage 1 of ResNet-50
// at bs1280).
//
// Arithmetic is the apply kernel's (bn_act.hip bn_apply_body): o = fmaf(y, scale, shift), o += r (or
// fmaf(y_d, scale_d, shift_d)), ReLU bit, max, round to bf16 -- so out, the mask and the GEMM output are
// bit-identical to the unfused pair (tests/test_gpu_gemm_apply.py).
//
// Register-staged main loop (the PIPE 0 loop of dla_mfma.h that the 1x1 forwards use up to K = 512) split in
// two: the raw y / r chunks of k-step t+1 are loaded before k-step t's MFMAs, transformed and written to LDS
// (and to HBM) after them, so the loads stay in flight under the MFMAs. The per-channel coefficients sit in
// LDS for the whole K.
#include <algorithm>
#include <cstdlib>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

struct ApplyArgs {
  const bf16_t* y;   // BN input [M][K]
  const bf16_t* r;   // identity residual [M][K], or the shortcut BN's input (kDual)
  const float* ws;   // 7K workspace of the BN: scale at [2K, 3K), shift at [3K, 4K)
  const float* ws2;  // kDual: the shortcut BN's
  bf16_t* out;       // act(BN(y) + r) [M][K]
  uint8_t* mask;     // its ReLU bits: bit j of byte e >> 3 for element e = m * K + k
  // optional stride-2 subsample of out, [n][H/2][W/2][K] for rows m = (n H + h) W + w (the downsample conv's input
  // at a stage transition; written from the same registers instead of a second pass over out)
  bf16_t* xs;
  int H, W;
};

template <int BM, int BN, bool kStats, bool kDual>
__global__ __launch_bounds__(kThreads, blocks_per_cu(BM, BN, kThreads)) void gemm_apply_kernel(
    const ApplyArgs ap, const bf16_t* __restrict__ B, int64_t ldb, bf16_t* __restrict__ C, int64_t ldc, int M, int N,
    int K, float* __restrict__ stats, uint32_t coef_off) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  using GA = TileGeom<BM, kThreads>;
  using GB = TileGeom<BN, kThreads>;
  using LA = RowLoader<BM, kThreads>;  // the A image is the plain row-major one
  using LB = RowLoader<BN, kThreads>;
  using AC = Acc<BM, BN, kThreads>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  const int nbn = (N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  const bool writer = bn == 0;
  const int tid = threadIdx.x;

  // coefficients [scale | shift (| scale_d | shift_d)] x K
  float* coef = reinterpret_cast<float*>(smem_raw + coef_off);
  for (int i = tid; i < 2 * K; i += kThreads) {
    coef[i] = ap.ws[2 * K + i];
    if constexpr (kDual) coef[2 * K + i] = ap.ws2[2 * K + i];
  }

  bf16_t* As = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* Bs = As + GA::kRowElems;
  const LB lb{B, ldb, (int64_t)col0, N, K};
  const int wid = tid >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN;
  // chunk i of this thread: row (tid + i * NT) >> 3, the same 8 channels kc .. kc + 7 in every chunk and k-step
  const int kc = (tid & 7) * 8;
  int64_t off[GA::CH], xoff[GA::CH];
  bool ok[GA::CH];
#pragma unroll
  for (int i = 0; i < GA::CH; ++i) {
    const int64_t gr = row0 + ((tid + i * kThreads) >> 3);
    ok[i] = gr < M;
    off[i] = (ok[i] ? gr : 0) * K + kc;
    xoff[i] = -1;
    if (ap.xs && ok[i]) {  // even (h, w): its position in the subsample
      const int64_t q = gr / ap.W, w = gr - q * ap.W;
      const int64_t n = q / ap.H, h = q - n * ap.H;
      if (!((h | w) & 1)) xoff[i] = ((n * (ap.H >> 1) + (h >> 1)) * (ap.W >> 1) + (w >> 1)) * K + kc;
    }
  }
  ushort8_t ya[GA::CH], ra[GA::CH], rb[GB::CH];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < GA::CH; ++i) {
      ya[i] = *reinterpret_cast<const ushort8_t*>(ap.y + off[i] + k0);
      ra[i] = *reinterpret_cast<const ushort8_t*>(ap.r + off[i] + k0);
    }
#pragma unroll
    for (int i = 0; i < GB::CH; ++i) rb[i] = lb.load(i, k0);
  };
  auto xstore = [&](int k0) {
    float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = coef[k0 + kc + j];
      sh[j] = coef[K + k0 + kc + j];
      sc2[j] = kDual ? coef[2 * K + k0 + kc + j] : 1.f;
      sh2[j] = kDual ? coef[3 * K + k0 + kc + j] : 0.f;
    }
    ushort8_t ta[GA::CH];
#pragma unroll
    for (int i = 0; i < GA::CH; ++i) {
      uint32_t bits = 0;
      ushort8_t o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = fmaf(bf16_to_f32(ya[i][j]), sc[j], sh[j]);
        const float rv = bf16_to_f32(ra[i][j]);
        v += kDual ? fmaf(rv, sc2[j], sh2[j]) : rv;
        bits |= (v > 0.f ? 1u : 0u) << j;
        o[j] = f32_to_bf16(fmaxf(v, 0.f));
      }
      ta[i] = ok[i] ? o : zero8();
      if (writer && ok[i]) {
        *reinterpret_cast<ushort8_t*>(ap.out + off[i] + k0) = o;
        ap.mask[(off[i] + k0) >> 3] = (uint8_t)bits;
        if (xoff[i] >= 0) *reinterpret_cast<ushort8_t*>(ap.xs + xoff[i] + k0) = o;
      }
    }
    tile_store<BM, LA>(As, ta);
    tile_store<BN, LB>(Bs, rb);
  };

  AC acc;
  acc.zero();
  const int nk = K / kBK;
  fetch(0);
  __syncthreads();  // coefficient table
  xstore(0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) fetch((t + 1) * kBK);  // next k-step's raw operands in flight during this one's MFMAs
#pragma unroll
    for (int kk = 0; kk < kBK / kKS; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tile_frag<BM, LA>(As, wr * WM + i * kMS, kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tile_frag<BN, LB>(Bs, wc * WN + j * kMS, kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc.v[i][j] = mfma(af[i], bfr[j], acc.v[i][j]);
    }
    __syncthreads();
    if (t + 1 < nk) {
      xstore((t + 1) * kBK);
      __syncthreads();
    }
  }
  ColStats<BM, BN, kThreads> st;
  st.zero();
  epilogue_bf16<BM, BN, kStats, false, kThreads>(acc, C, ldc, M, N, row0, col0, st, nullptr, 0, smem_raw);
  if constexpr (kStats) stats_flush<BM, BN, kThreads>(st, stats + (int64_t)bm * N * 2, N, col0, smem_raw);
}

template <int BM, int BN, bool S, bool D>
void launch_apply(const ApplyArgs& ap, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M, int N, int K,
                  float* stats, hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t ab = mainloop_lds_bytes<BM, BN, RowLoader<BM>, RowLoader<BN>>();
  const size_t cs = epilogue_lds_bytes<BM, BN, S>();
  const size_t base = (std::max(ab, cs) + 15) / 16 * 16;
  const size_t lds = base + (size_t)(D ? 4 : 2) * K * sizeof(float);
  hipLaunchKernelGGL((gemm_apply_kernel<BM, BN, S, D>), dim3(tiles), dim3(kThreads), lds, stream, ap, B, ldb, C, ldc,
                     M, N, K, stats, (uint32_t)base);
}

}  // namespace

// Largest K served (the consumer's conv1 input channels): 512 covers stages 1-2 and the stage-2 -> 3 transition,
// where the 128-row register-staged tile is also the unfused GEMM's; above it the unfused forward runs on the
// 256x256 LDS-DMA tile. DLA_APPLY_MAX_K / set_gemm_apply_max_k (<= kGemmApplyMaxK) for A/B.
static int g_apply_max_k = [] {
  const char* e = std::getenv("DLA_APPLY_MAX_K");
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? std::min(v, kGemmApplyMaxK) : 512;
}();
void set_gemm_apply_max_k(int k) { g_apply_max_k = k > 0 ? std::min(k, kGemmApplyMaxK) : 512; }

bool gemm_apply_ok(int64_t M, int N, int K) {
  return M > 0 && K % kBK == 0 && K >= kBK && K <= g_apply_max_k && N % 64 == 0 && N > 0 &&
         M * (int64_t)K * 2 < ((int64_t)1 << 31) && M * (int64_t)N * 2 < ((int64_t)1 << 31);
}

int gemm_apply_rows(int64_t M) { return (int)((M + 127) / 128); }

void launch_gemm_apply(const void* y, const void* r, const float* ws, const float* ws2, void* out, uint8_t* mask,
                       const void* B, int64_t ldb, void* C, int M, int N, int K, float* stats, hipStream_t stream,
                       void* xs, int H, int W) {
  const ApplyArgs ap{(const bf16_t*)y, (const bf16_t*)r, ws, ws2, (bf16_t*)out, mask, (bf16_t*)xs, H, W};
  const bf16_t* b = (const bf16_t*)B;
  bf16_t* c = (bf16_t*)C;
#define DLA_APPLY(BN_)                                                                          \
  if (stats) {                                                                                  \
    if (ws2) launch_apply<128, BN_, true, true>(ap, b, ldb, c, N, M, N, K, stats, stream);      \
    else launch_apply<128, BN_, true, false>(ap, b, ldb, c, N, M, N, K, stats, stream);         \
  } else {                                                                                      \
    if (ws2) launch_apply<128, BN_, false, true>(ap, b, ldb, c, N, M, N, K, stats, stream);     \
    else launch_apply<128, BN_, false, false>(ap, b, ldb, c, N, M, N, K, stats, stream);        \
  }
  if (N <= 64) {
    DLA_APPLY(64)
  } else {
    DLA_APPLY(128)
  }
#undef DLA_APPLY
}

}  // namespace dla
