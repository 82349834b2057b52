// bf16 MFMA GEMMs for the ResNet 1x1-convolution hot path (channels_last activations).
//
// With NHWC activations a 1x1 convolution is a plain GEMM over M = N*H*W rows:
//   forward  Y[M, Cout]    = X[M, Cin]  * W[Cout, Cin]^T        -> gemm_nt (A = X,  B = W)
//   dgrad    dX[M, Cin]    = dY[M, Cout] * W[Cout, Cin]         -> gemm_nt (A = dY, B = W k-major)
//   wgrad    dW[Cout, Cin] = dY[M, Cout]^T * X[M, Cin]          -> gemm_tn, split over M
// The reference runs these as cuDNN/MIOpen convolutions. At ResNet-50 shapes the
// reduction dim is small (K = 64..2048) so most of these GEMMs sit near the HBM roofline rather than
// the MFMA roofline; the kernels are built for that regime:
//   * 256-thread workgroups, 2x2 waves, v_mfma_f32_16x16x32_bf16 (fp32 accumulate), 64-deep K
//     steps staged through LDS with a register prefetch of the next tile (global loads in flight
//     while the MFMAs of the current tile run, cdna_hip_programming.md T14), rows padded by 16 B so
//     the ds_read_b128 fragment reads are bank-conflict free;
//   * bijective XCD-aware tile remap (T1) so consecutive tiles share an XCD's L2;
//   * epilogue staged through LDS so the bf16 tile leaves in full 16-byte-per-lane row segments,
//     with an optional fused per-column (channel) sum / sum-of-squares — the BatchNorm statistics of
//     the conv output — written as per-row-block partials (no atomics, fixed-order reduction);
//   * gemm_tn reads k-major operands straight from their natural layout with the gfx950
//     ds_read_b64_tr_b16 transposing LDS read (T10) and splits the long M reduction over blocks
//     with fp32 partial slabs + a separate reduction kernel.
#include <cstdlib>
#include <type_traits>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

// ---------------------------------------------------------------------------------------------
// C[M,N] = A[M,K] * B[N,K]^T   (A K-contiguous; B K-contiguous, or k-major [K][N] when kBT),
// bf16 in/out, fp32 accumulate, optional fused addend and BN-statistics epilogue.
// ---------------------------------------------------------------------------------------------
// kD: the product computed transposed and the tile stored from the registers (dla_mfma.h epilogue_direct);
// forwards without addend / BN-backward features only
template <int BM, int BN, bool kStats, bool kBT, int PIPE, int NT, bool kD = false>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void gemm_nt_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                              const bf16_t* __restrict__ B, int64_t ldb,
                                                              bf16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                              float* __restrict__ stats, const bf16_t* __restrict__ D,
                                                              int64_t ldd, BnBwdEpi bnb) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int nbn = (N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  ColStats<BM, BN, NT> st;
  st.zero();
  Acc<BM, BN, NT> acc;
  acc.zero();
  const RowLoader<BM, NT> la{A, lda, row0, M, K};
  if constexpr (kBT) {
    const KLoader<BN, NT> lb{B, ldb, col0, N, K};
    run_mainloop<PIPE, kD>(la, lb, 0, K, acc, smem_raw);
  } else {
    const RowLoader<BN, NT> lb{B, ldb, (int64_t)col0, N, K};
    run_mainloop<PIPE, kD>(la, lb, 0, K, acc, smem_raw);
  }
  if constexpr (kD) {
    epilogue_direct<BM, BN, kStats, NT>(acc, C, ldc, M, N, row0, col0, kStats ? stats + (int64_t)bm * N * 2 : nullptr,
                                        smem_raw);
  } else {
    epilogue_bf16<BM, BN, kStats, !kStats, NT>(acc, C, ldc, M, N, row0, col0, st, D, ldd, smem_raw, &bnb, bm);
    if constexpr (kStats) stats_flush<BM, BN, NT>(st, stats + (int64_t)bm * N * 2, N, col0, smem_raw);
  }
}

// ---------------------------------------------------------------------------------------------
// P[split][Mo, No] = sum_{k in split} A[k][m] * B[k][n]   (A: [K, lda] m-contiguous, B: [K, ldb])
// fp32 partial slabs; splitk_reduce_kernel sums them.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int PIPE, int NT = kThreads>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void gemm_tn_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                              const bf16_t* __restrict__ B, int64_t ldb,
                                                                              float* __restrict__ P, int Mo, int No, int K,
                                                                              int k_per_split, int ntiles, int remap) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int nbn = (No + BN - 1) / BN;
  // 1-D grid of tiles x splits; with remap the tiles of one split (which read the same K rows of
  // both operands) are consecutive logical ids, i.e. co-scheduled on one XCD and its L2
  const int lin = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tile = lin % ntiles, split = lin / ntiles;
  const int bm = tile / nbn, bn = tile % nbn;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int m0 = bm * BM, n0 = bn * BN;
  Acc<BM, BN, NT> acc;
  acc.zero();
  const KLoader<BM, NT> la{A, lda, m0, Mo, kend};
  const KLoader<BN, NT> lb{B, ldb, n0, No, kend};
  run_mainloop<PIPE>(la, lb, kbeg, kend, acc, smem_raw);
  epilogue_f32<BM, BN, NT>(acc, P + (int64_t)split * Mo * No, Mo, No, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// Split-K gemm_nt for few output tiles and a long reduction — the fully connected heads
// (GoogLeNet aux fc1: M = batch 128, N = 1024, K = 2048 is 8 tiles of 32 k-steps each, 37 us on
// 8 of 256 CUs). P[split][M, N] = A[:, ks] * B[:, ks]^T, summed (+ the row-broadcast bias addend)
// by splitk_reduce_sg_kernel.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, bool kBT, int PIPE>
__global__ __launch_bounds__(kThreads, 2) void gemm_nt_splitk_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                     const bf16_t* __restrict__ B, int64_t ldb,
                                                                     float* __restrict__ P, int M, int N, int K,
                                                                     int k_per_split, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int nbn = (N + BN - 1) / BN;
  const int tile = blockIdx.x % ntiles, split = blockIdx.x / ntiles;
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  Acc<BM, BN> acc;
  acc.zero();
  const RowLoader<BM> la{A, lda, row0, M, kend};
  if constexpr (kBT) {
    const KLoader<BN> lb{B, ldb, col0, N, kend};
    run_mainloop<PIPE>(la, lb, kbeg, kend, acc, smem_raw);
  } else {
    const RowLoader<BN> lb{B, ldb, (int64_t)col0, N, kend};
    run_mainloop<PIPE>(la, lb, kbeg, kend, acc, smem_raw);
  }
  epilogue_f32<BM, BN>(acc, P + (int64_t)split * M * N, M, N, (int)row0, col0);
}

// Sums the split-K fp32 slabs: each thread owns 4 consecutive outputs (one 16-byte load per slab)
// and keeps 4 slabs in flight, so the loop is bandwidth- rather than latency-bound.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P, int splits, int64_t n,
                                                            T* __restrict__ out, float scale, int accumulate) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    float4_t a0{0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int k = 0;
    for (; k + 3 < splits; k += 4) {
      a0 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 0) * n)[v];
      a1 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 1) * n)[v];
      a2 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 2) * n)[v];
      a3 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 3) * n)[v];
    }
    for (; k < splits; ++k) a0 += reinterpret_cast<const float4_t*>(P + (int64_t)k * n)[v];
    const float4_t s = ((a0 + a1) + (a2 + a3)) * scale;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o = s[j];
      if (accumulate) o += Cvt<T>::to_f32(out[v * 4 + j]);
      out[v * 4 + j] = Cvt<T>::from_f32(o);
    }
  }
  if (blockIdx.x == 0) {  // tail (n % 4)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float o = 0.f;
      for (int k = 0; k < splits; ++k) o += P[(int64_t)k * n + i];
      o *= scale;
      if (accumulate) o += Cvt<T>::to_f32(out[i]);
      out[i] = Cvt<T>::from_f32(o);
    }
  }
}

// Small outputs with many splits (a 64x64 weight gradient has 1024 float4 outputs and up to 512
// slabs): one thread per output would leave a handful of blocks each walking hundreds of slabs
// one latency at a time (19-36 us per call in profiles/resnet50_bs512_r3f_ksum.md). Here SG thread
// groups of a block split the slab range (group g sums slabs g, g+SG, ...), then group 0 adds the
// SG partial sums from LDS in group order, so the result is still fixed-order and run-to-run
// deterministic.
// D (optional): bf16 addend of the [n / ncol, ncol] output with row stride ldd (0: one broadcast row,
// the bias of a split-K linear layer), added after the scale.
template <typename T, int SG>
__global__ __launch_bounds__(256) void splitk_reduce_sg_kernel(const float* __restrict__ P, int splits, int64_t n,
                                                               T* __restrict__ out, float scale, int accumulate,
                                                               const bf16_t* __restrict__ D, int64_t ldd, int ncol) {
  auto addend = [&](int64_t i) -> float {
    if (D == nullptr) return 0.f;
    const int64_t r = i / ncol;
    return bf16_to_f32(D[r * ldd + (i - r * ncol)]);
  };
  constexpr int kOpb = 256 / SG;  // float4 outputs per block
  __shared__ float4_t red[SG][kOpb];
  const int g = threadIdx.x / kOpb, o = threadIdx.x % kOpb;
  const int64_t nv = n / 4;
  const int64_t v = (int64_t)blockIdx.x * kOpb + o;
  float4_t a0{0.f, 0.f, 0.f, 0.f}, a1 = a0;
  if (v < nv) {
    int k = g;
    for (; k + SG < splits; k += 2 * SG) {
      a0 += reinterpret_cast<const float4_t*>(P + (int64_t)k * n)[v];
      a1 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + SG) * n)[v];
    }
    if (k < splits) a0 += reinterpret_cast<const float4_t*>(P + (int64_t)k * n)[v];
  }
  red[g][o] = a0 + a1;
  __syncthreads();
  if (g == 0 && v < nv) {
    float4_t s = red[0][o];
#pragma unroll
    for (int j = 1; j < SG; ++j) s += red[j][o];
    s *= scale;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float r = s[j] + addend(v * 4 + j);
      if (accumulate) r += Cvt<T>::to_f32(out[v * 4 + j]);
      out[v * 4 + j] = Cvt<T>::from_f32(r);
    }
  }
  if (blockIdx.x == 0) {  // tail (n % 4)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float r = 0.f;
      for (int k = 0; k < splits; ++k) r += P[(int64_t)k * n + i];
      r = r * scale + addend(i);
      if (accumulate) r += Cvt<T>::to_f32(out[i]);
      out[i] = Cvt<T>::from_f32(r);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
// MFMA main-loop pipeline (dla_mfma.h run_mainloop). -1 = per shape, from scripts/bench_gemm.py /
// bench_conv.py on MI355X: the 2-stage LDS-DMA loop wins once a block runs several k-steps
// (K >= 256: up to 1.45x at K = 1024-2048; every 3x3 conv, K >= 576); at K <= 128 a block has one or
// two k-steps, nothing to overlap, and the register-staged loop's third resident block wins.
// 3 stages (96 KB of LDS, 1 block/CU) never won at ResNet shapes.
static int g_pipe = -1;
void set_mfma_pipeline(int p) { g_pipe = (p == 0 || (p >= 2 && p <= 7)) ? p : -1; }
int mfma_pipeline() { return g_pipe; }
int mfma_pipeline_for(int K) { return g_pipe >= 0 ? g_pipe : (K >= 256 ? 2 : 0); }

template <int BM, int BN, bool S, bool BT, int PIPE, int NT, bool kD = false>
static void launch_nt_p(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M,
                        int N, int K, float* stats, const bf16_t* D, int64_t ldd, const BnBwdEpi& bnb,
                        hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const size_t ab = BT ? run_mainloop_lds_bytes<PIPE, BM, BN, RowLoader<BM, NT>, KLoader<BN, NT>>()
                       : run_mainloop_lds_bytes<PIPE, BM, BN, RowLoader<BM, NT>, RowLoader<BN, NT>>();
  const size_t cs = epilogue_lds_bytes<BM, BN, S, NT>();
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, S, BT, PIPE, NT, kD>), dim3(tiles), dim3(NT), std::max(ab, cs), stream, A,
                     lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb);
}

template <int BM, int BN, bool S, bool BT, int NTW = kThreads>
static void launch_nt(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M,
                      int N, int K, float* stats, const bf16_t* D, int64_t ldd, const BnBwdEpi& bnb,
                      hipStream_t stream) {
  if constexpr (NTW == 512 && BM * BN > 256 * 128) {  // 256x256: 2 stages fill 128 KB of LDS
    if (mfma_pipeline() == 2) launch_nt_p<BM, BN, S, BT, 2, 512>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
    else launch_nt_p<BM, BN, S, BT, 6, 512>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
  } else if constexpr (NTW == 512) {  // 8-wave tile: 3-stage LDS-DMA pipeline, one block per CU
    if (mfma_pipeline() == 7) launch_nt_p<BM, BN, S, BT, 7, 512>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
    else launch_nt_p<BM, BN, S, BT, 3, 512>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
  } else if constexpr (BM * BN > 128 * 128) {  // 4 large waves, one block per CU: 2 or 3 stages
    if (mfma_pipeline() == 2) launch_nt_p<BM, BN, S, BT, 2, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
    else launch_nt_p<BM, BN, S, BT, 3, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream);
  } else {
    // 1x1-conv GEMMs: register staging (36 KB LDS, 4 blocks / CU) up to K = 512, the 2-stage
    // LDS-DMA loop (64 KB, 2 blocks / CU) above — per-layer A/B at ResNet-50 bs512 shapes,
    // profiles/r2t (auto K<256 threshold: 9.58-9.71 ms fwd+dgrad; K<=512: 9.43 ms)
    const int pipe = mfma_pipeline() >= 0 ? mfma_pipeline() : (K > 512 ? 2 : 0);
    switch (pipe) {
      case 0: launch_nt_p<BM, BN, S, BT, 0, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream); break;
      case 3: launch_nt_p<BM, BN, S, BT, 3, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream); break;
      case 4: launch_nt_p<BM, BN, S, BT, 4, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream); break;
      case 6: launch_nt_p<BM, BN, S, BT, 6, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream); break;
      default: launch_nt_p<BM, BN, S, BT, 2, kThreads>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, bnb, stream); break;
    }
  }
}

// 256x256 8-wave tiles for the compute-bound shapes (per-layer A/B at ResNet-50 bs512 shapes,
// profiles/r5a: 3x3 fwd/dgrad at 14x14 and 7x7 -14..-17 %, 1x1 with K >= 1024 -10..-19 %; shorter K or
// N < 256 is HBM- or LDS-bound and loses up to 2x). At least ~3/4 of the CUs must get a tile.
// DLA_TILE256=0 restores the 128-row tiles (A/B).
bool tile256_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("DLA_TILE256");
    return !(e && e[0] == '0');
  }();
  return v;
}

// K >= 256 wins per shape in isolation (profiles/r4/g04) but not in the step (g05: +0.1 ms): 1024 stays
static int g_tile256_min_k = 1024;  // A/B setter (set_tile256_min_k)
void set_tile256_min_k(int k) { g_tile256_min_k = k > 0 ? k : 1024; }
// forwards with the BN-statistics epilogue (no addend): their 256x256 tiles win from K = 256 in isolation
// (profiles/r6/g10: stage-3 conv3 0.270 vs 0.299 ms, stage-4 conv3 0.202 vs 0.229 ms) while the data gradients
// with the identity addend lose (0.397 vs 0.354). In the step, interleaved x3 on one box (profiles/r6/g11):
// 82.30 ms (256) vs 82.40 (512) vs 82.53 (1024). set_tile256_min_k_stats / DLA_TILE256_MIN_K_STATS for A/B
static int g_tile256_min_k_stats = [] {
  const char* e = std::getenv("DLA_TILE256_MIN_K_STATS");
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? v : 256;
}();
void set_tile256_min_k_stats(int k) { g_tile256_min_k_stats = k > 0 ? k : 256; }

static int g_gemm256_direct = -1;  // -1: DLA_GEMM256_DIRECT (default off), 0 / 1
void set_gemm256_direct(int mode) { g_gemm256_direct = mode < 0 ? -1 : (mode ? 1 : 0); }
bool gemm256_direct_enabled() {
  if (g_gemm256_direct >= 0) return g_gemm256_direct == 1;
  static const bool v = [] {
    const char* e = std::getenv("DLA_GEMM256_DIRECT");
    return e && e[0] == '1';
  }();
  return v;
}

int pick_tile(int64_t M, int N, int tile, int K, bool wide_ok, bool stats) {
  if (tile != kTileAuto) return tile;
  const int min_k = stats ? std::min(g_tile256_min_k, g_tile256_min_k_stats) : g_tile256_min_k;
  if (wide_ok && tile256_enabled() && K >= min_k && N % 256 == 0 && ((M + 255) / 256) * (N / 256) >= 192)
    return kTile256x256;
  // the 128-row tiles win at every other ResNet shape, including the small-M layers, so the narrow
  // tile is used only when N itself is narrow (scripts/bench_gemm.py, bench_conv.py)
  return N <= 64 ? kTile128x64 : kTile128x128;
}

int gemm_nt_stats_rows(int M, int N, int tile, int K, bool stats_fwd) {
  const int bm = tile_bm(pick_tile(M, N, tile, K, true, stats_fwd));
  return (M + bm - 1) / bm;
}

void launch_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                    float* stats, hipStream_t stream, const void* addend, int64_t ld_addend, bool b_kmajor, int tile,
                    const BnBwdArgs* bn_bwd, const uint8_t* addend_mask, const void* addend2_s2, int H, int W) {
  BnBwdEpi bnb{};
  if (bn_bwd) {
    bnb.x = (const bf16_t*)bn_bwd->x;
    bnb.ldx = bn_bwd->ldx;
    bnb.ws = bn_bwd->ws;
    bnb.mask = bn_bwd->mask;
    bnb.mode = bn_bwd->mode;
    bnb.part = bn_bwd->part;
  }
  bnb.dmask = addend_mask;
  if (addend2_s2) {
    bnb.d2 = (const bf16_t*)addend2_s2;
    bnb.H = H;
    bnb.W = W;
    bnb.fW = make_fastdiv((uint32_t)W);
    bnb.fH = make_fastdiv((uint32_t)H);
  }
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
  bf16_t* c = (bf16_t*)C;
  const bf16_t* d = (const bf16_t*)addend;
#define DLA_NT(BM_, BN_, S_, BT_, NT_) \
  launch_nt<BM_, BN_, S_, BT_, NT_>(a, lda, b, ldb, c, ldc, M, N, K, stats, d, ld_addend, bnb, stream)
#define DLA_NT_STW(BM_, BN_, NT_)                                                              \
  if (stats) {                                                                                 \
    if (b_kmajor) DLA_NT(BM_, BN_, true, true, NT_); else DLA_NT(BM_, BN_, true, false, NT_);    \
  } else {                                                                                     \
    if (b_kmajor) DLA_NT(BM_, BN_, false, true, NT_); else DLA_NT(BM_, BN_, false, false, NT_);  \
  }
#define DLA_NT_ST(BM_, BN_) DLA_NT_STW(BM_, BN_, kThreads)
  const int cfg = pick_tile(M, N, tile, K, true, stats != nullptr && addend == nullptr);
  // the 128x128 tile without the BN-backward / stride-2 epilogue features: stored from the registers
  // (gemm_direct.hip); tile = kTile128x128 forced by a caller keeps the LDS-staged kernel (A/B)
  if (cfg == kTile128x128 && tile == kTileAuto && !bn_bwd && !addend2_s2 && !(stats && addend) &&
      gemm_direct_ok(N, ldc, addend, ld_addend)) {
    launch_gemm_direct(A, lda, B, ldb, b_kmajor, C, ldc, M, N, K, stats, addend, ld_addend, addend_mask, stream);
    return;
  }
  // the 256x256 statistics forwards stored from the registers (DLA_GEMM256_DIRECT / set_gemm256_direct, A/B)
  if (cfg == kTile256x256 && stats && !b_kmajor && !addend && !bn_bwd && !addend2_s2 && gemm256_direct_enabled()) {
    if (mfma_pipeline() == 2)
      launch_nt_p<256, 256, true, false, 2, 512, true>(a, lda, b, ldb, c, ldc, M, N, K, stats, d, ld_addend, bnb, stream);
    else
      launch_nt_p<256, 256, true, false, 6, 512, true>(a, lda, b, ldb, c, ldc, M, N, K, stats, d, ld_addend, bnb, stream);
    return;
  }
  switch (cfg) {
    case kTile256x256: DLA_NT_STW(256, 256, 512) break;
    case kTile256x128: DLA_NT_STW(256, 128, 512) break;
    case kTile256x128w4: DLA_NT_ST(256, 128) break;
    case kTile128x256w4: DLA_NT_ST(128, 256) break;
    case kTile256x64: DLA_NT_ST(256, 64) break;
    case kTile128x128: DLA_NT_ST(128, 128) break;
    case kTile128x64: DLA_NT_ST(128, 64) break;
    default: DLA_NT_ST(64, 64) break;
  }
#undef DLA_NT_ST
#undef DLA_NT_STW
#undef DLA_NT
}

// 64-wide tiles for 64-wide operands: a 128-wide tile would spend half (or three quarters, at
// 64 x 64) of its MFMAs and LDS traffic on zero columns.
static inline int tn_bm(int Mo) { return Mo <= 64 ? 64 : 128; }
static inline int tn_bn(int No) { return No <= 64 ? 64 : 128; }

// XCD-aware ordering of split-K grids (DLA_SPLITK_XCD=0 restores the split-major 2-D order, A/B)
bool splitk_xcd_remap() {
  static const bool v = [] {
    const char* e = std::getenv("DLA_SPLITK_XCD");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Workgroups a split-K weight-gradient launch aims for (tiles x splits): 512 = 2 per CU;
// DLA_SPLITK_BLOCKS overrides it for A/B runs
static int g_splitk_blocks = 0;  // set_splitk_blocks(): > 0 overrides the environment / default
void set_splitk_blocks(int blocks) { g_splitk_blocks = blocks > 0 ? blocks : 0; }
int splitk_target_blocks() {
  if (g_splitk_blocks > 0) return g_splitk_blocks;
  static const int v = [] {
    const char* e = std::getenv("DLA_SPLITK_BLOCKS");
    const int b = e ? std::atoi(e) : 0;
    return b > 0 ? b : 512;
  }();
  return v;
}

// 256x256 8-wave tiles (one block per CU) for weight gradients whose output dims are both
// multiples of 256 (the stage-3/4 1x1 convs: compute-bound, like the fwd/dgrad shapes pick_tile
// sends to kTile256x256); DLA_TILE256=0 turns them off with the other 256x256 tiles
// (DLA_TN256=0 turns off only these and the 3x3 ones, for A/B)
static int g_tn256 = -1;  // set_tn256(): -1 environment (DLA_TN256, default on), 0 off, 1 on
void set_tn256(int mode) { g_tn256 = mode < 0 ? -1 : (mode ? 1 : 0); }
bool tn256_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DLA_TN256");
    return !(e && e[0] == '0');
  }();
  return (g_tn256 < 0 ? on : g_tn256 == 1) && tile256_enabled();
}
static bool tn_wide(int Mo, int No) { return tn256_enabled() && Mo % 256 == 0 && No % 256 == 0; }

int gemm_tn_splits(int Mo, int No, int K) {
  // ~512 workgroups in flight (2 per CU; 256 one-per-CU blocks for the 8-wave tiles) and >= 16
  // K-steps per split: enough parallelism for the long M reduction while keeping the fp32 slab
  // traffic (splits * Mo * No * 4 B) small.
  const bool wide = tn_wide(Mo, No);
  const int bm = wide ? 256 : tn_bm(Mo), bn = wide ? 256 : tn_bn(No);
  const int tiles = ((Mo + bm - 1) / bm) * ((No + bn - 1) / bn);
  int splits = std::max(1, (wide ? splitk_target_blocks() / 2 : splitk_target_blocks()) / std::max(1, tiles));
  const int max_splits = std::max(1, K / (16 * kBK));
  return std::max(1, std::min(splits, max_splits));
}

void launch_gemm_tn(const void* A, int64_t lda, const void* B, int64_t ldb, float* partial, int splits, int Mo, int No,
                    int K, void* out, int out_dtype, float scale, bool accumulate, hipStream_t stream) {
  int kps = (K + splits - 1) / splits;
  kps = (kps + kBK - 1) / kBK * kBK;
  const bool wide = tn_wide(Mo, No);
  const int bm = wide ? 256 : tn_bm(Mo), bn = wide ? 256 : tn_bn(No);
  const int tiles = ((Mo + bm - 1) / bm) * ((No + bn - 1) / bn);
#define DLA_TN(BM_, BN_, P_, NT_)                                                                                 \
  hipLaunchKernelGGL((gemm_tn_kernel<BM_, BN_, P_, NT_>), dim3(tiles * splits), dim3(NT_),                        \
                     (run_mainloop_lds_bytes<P_, BM_, BN_, KLoader<BM_, NT_>, KLoader<BN_, NT_>>()), stream,        \
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, partial, Mo, No, K, kps, tiles,                 \
                     (int)splitk_xcd_remap())
#define DLA_TN_P(BM_, BN_)                            \
  switch (mfma_pipeline_for(kps)) {                   \
    case 0: DLA_TN(BM_, BN_, 0, kThreads); break;     \
    case 3: DLA_TN(BM_, BN_, 3, kThreads); break;     \
    case 4: DLA_TN(BM_, BN_, 4, kThreads); break;     \
    case 6: DLA_TN(BM_, BN_, 6, kThreads); break;     \
    default: DLA_TN(BM_, BN_, 2, kThreads); break;    \
  }
  if (wide) {
    if (mfma_pipeline() == 2) DLA_TN(256, 256, 2, 512);
    else DLA_TN(256, 256, 6, 512);
  } else if (bm == 64 && bn == 64) {
    DLA_TN_P(64, 64)
  } else if (bm == 64) {
    DLA_TN_P(64, 128)
  } else if (bn == 64) {
    DLA_TN_P(128, 64)
  } else {
    DLA_TN_P(128, 128)
  }
#undef DLA_TN_P
#undef DLA_TN
  launch_splitk_reduce(partial, splits, (int64_t)Mo * No, out, out_dtype, scale, accumulate, stream);
}

void launch_splitk_reduce(const float* partial, int splits, int64_t n, void* out, int out_dtype, float scale,
                          bool accumulate, hipStream_t stream, const void* addend, int64_t ld_addend, int ncol) {
  const int64_t nv = n / 4;
  // slab groups per block: the fewest that give >= 512 blocks, at most 64 and at most splits / 2
  // (DLA_SPLITK_SG=0: one thread per output, for A/B runs)
  static const bool sg_on = [] {
    const char* e = std::getenv("DLA_SPLITK_SG");
    return !(e && e[0] == '0');
  }();
  int sg = 1;
  while (sg_on && sg < 64 && 2 * sg <= splits / 2 && (nv * sg + 255) / 256 < 512) sg *= 2;
  const bf16_t* D = (const bf16_t*)addend;
  if (sg > 1 || D != nullptr) {
    const int grid = (int)std::max<int64_t>(1, (nv * sg + 255) / 256);
#define DLA_SKR(SG_)                                                                                              \
  case SG_:                                                                                                       \
    if (out_dtype == kF32)                                                                                        \
      hipLaunchKernelGGL((splitk_reduce_sg_kernel<float, SG_>), dim3(grid), dim3(256), 0, stream, partial, splits, \
                         n, (float*)out, scale, (int)accumulate, D, ld_addend, ncol);                             \
    else                                                                                                          \
      hipLaunchKernelGGL((splitk_reduce_sg_kernel<bf16_t, SG_>), dim3(grid), dim3(256), 0, stream, partial,       \
                         splits, n, (bf16_t*)out, scale, (int)accumulate, D, ld_addend, ncol);                    \
    break;
    switch (sg) {
      DLA_SKR(1)
      DLA_SKR(2)
      DLA_SKR(4)
      DLA_SKR(8)
      DLA_SKR(16)
      DLA_SKR(32)
      DLA_SKR(64)
    }
#undef DLA_SKR
    return;
  }
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nv + 255) / 256, 2048));
  if (out_dtype == kF32)
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(grid), dim3(256), 0, stream, partial, splits, n, (float*)out,
                       scale, (int)accumulate);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, partial, splits, n,
                       (bf16_t*)out, scale, (int)accumulate);
}

// Split-K gemm_nt (fully connected heads): few output tiles, long K. 0 / 1 = the tile kernel.
int gemm_nt_splitk_splits(int M, int N, int K) {
  const int bn = N <= 64 ? 64 : 128;
  const int tiles = ((M + 127) / 128) * ((N + bn - 1) / bn);
  if (tiles >= 128 || K < 512) return 1;
  // ~256 workgroups, >= 2 k-steps (128) per split
  return std::max(1, std::min(K / 128, 256 / tiles));
}

void launch_gemm_nt_splitk(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, float* partial,
                           int splits, void* C, int M, int N, int K, const void* addend, int64_t ld_addend,
                           hipStream_t stream) {
  int kps = (K + splits - 1) / splits;
  kps = (kps + kBK - 1) / kBK * kBK;
  splits = (K + kps - 1) / kps;
  const int bn = N <= 64 ? 64 : 128;
  const int tiles = ((M + 127) / 128) * ((N + bn - 1) / bn);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
#define DLA_NTS(BN_, BT_, P_)                                                                                       \
  hipLaunchKernelGGL((gemm_nt_splitk_kernel<128, BN_, BT_, P_>), dim3(tiles * splits), dim3(kThreads),              \
                     (run_mainloop_lds_bytes<P_, 128, BN_, RowLoader<128>,                                          \
                                             std::conditional_t<BT_, KLoader<BN_>, RowLoader<BN_>>>()),              \
                     stream, a, lda, b, ldb, partial, M, N, K, kps, tiles)
#define DLA_NTS_P(BN_, BT_)                                     \
  if (mfma_pipeline_for(kps) == 0) DLA_NTS(BN_, BT_, 0);        \
  else DLA_NTS(BN_, BT_, 2);
  if (bn == 64) {
    if (b_kmajor) { DLA_NTS_P(64, true) } else { DLA_NTS_P(64, false) }
  } else {
    if (b_kmajor) { DLA_NTS_P(128, true) } else { DLA_NTS_P(128, false) }
  }
#undef DLA_NTS_P
#undef DLA_NTS
  launch_splitk_reduce(partial, splits, (int64_t)M * N, C, kBF16, 1.f, false, stream, addend, ld_addend, N);
}


}  // namespace dla
