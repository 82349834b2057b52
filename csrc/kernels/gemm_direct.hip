// 1x1-convolution GEMMs whose 128 x 128 tiles leave straight from the accumulator registers.
//
// Why. Counter passes of the tile kernel (gemm.hip gemm_nt_kernel<128, 128, ...>) at the stage-3/4 shapes
// of ResNet-50 bs1280 (profiles/r6/g01, g02): HBM traffic is at its compulsory minimum (A read once, C
// written once) yet the kernels run at 1.4-2.3 TB/s and 18-22 % MFMA; the forward at K = 64 -- a pure
// write of its 514 MB output -- takes 0.17 ms (3.2 TB/s), and each further 64-deep k-step adds about
// 2x its MFMA time. Per wave 1,130 vector instructions accompany 128 MFMAs, and 41 % of the wave
// cycles are issue stalls: the epilogue stages every output element through LDS with a ds_write_b16
// (64 per lane), two barriers and a read-back before the 16-byte stores.
//
// Here the product is computed transposed (gemm B operand -- the weights -- as the MFMA A operand,
// dla_mfma.h mfma_t): a lane then holds, per 16 x 16 fragment, 4 consecutive output channels of ONE
// pixel. After the bf16 packing, one v_permlane16_swap per register pair exchanges fragments between
// neighbouring 16-lane rows so that every lane holds 8 consecutive channels (16 bytes) of a pixel, and
// the tile is stored with 8 global_store_dwordx4 per lane: no LDS staging, no epilogue barrier.
//   * forward: the BatchNorm statistics of the stored (bf16-rounded) values are summed in registers
//     over the lane's 4 pixel fragments, reduced over the 16 lanes of a row by a DPP butterfly, and the
//     two M-waves of the block combine through 4 KB of LDS into the same [row tile][N][2] partials the
//     tile kernel writes (bn_stats_finalize reads either);
//   * data gradient: the fused identity-gradient addend D (with its 1-bit ReLU mask) is loaded for all
//     of a lane's 8 chunks before the packing, C = bf16(bf16(acc) + (bit ? D : 0)) as in the tile kernel.
// Main loop: the tile kernel's (register-staged up to K = 512, 2-stage LDS-DMA above), same LDS images.
//
// Measured (profiles/r6/g03): bit-for-bit the staged kernel's outputs, but -1.6 ... -2.3 % at the stage-3 shapes
// and within noise elsewhere; the step is unchanged (82.89 vs 82.85 ms). The LDS staging was NOT what holds these
// tiles at 2-3 TB/s: at K = 64 the whole kernel is a 514 MB write that runs at ~3 TB/s with ~3 short-lived blocks
// per CU, i.e. per-block latency (prologue loads, store acknowledgement before the wave slot frees) with too few
// bytes in flight per CU. Kept as an opt-in (DLA_GEMM_DIRECT=1) base for a persistent multi-tile form.
#include <cstdlib>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

constexpr int kDB = 128;  // tile edge (rows = pixels, columns = channels)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}
__device__ __forceinline__ f32x2_t unpack_bf16(uint32_t u) {
  return f32x2_t{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
// sum over the 16 lanes of a DPP row (dla_mfma.h epi_row16_sum)
__device__ __forceinline__ float row16_sum(float v) { return epi_row16_sum(v); }

// bf16(x) + (bit ? d : 0) rounded to bf16, for the 2 packed values of u and d
__device__ __forceinline__ uint32_t add_pair(uint32_t u, uint32_t d, uint32_t bits) {
  const f32x2_t a = unpack_bf16(u), b = unpack_bf16(d);
  const float lo = a.x + ((bits & 1u) ? b.x : 0.f), hi = a.y + ((bits & 2u) ? b.y : 0.f);
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

// One 128 x 128 tile: main loop, then the register-stored epilogue. Ends with every LDS access done (a caller
// looping over tiles may start the next tile's main loop right away).
template <bool kStats, bool kBT, bool kAdd, int PIPE>
__device__ __forceinline__ void direct_tile(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
                                            int64_t ldb, bf16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                            float* __restrict__ stats, const bf16_t* __restrict__ D, int64_t ldd,
                                            const uint8_t* __restrict__ dmask, int tile, char* smem_raw) {
  const int nbn = (N + kDB - 1) / kDB;
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * kDB;
  const int col0 = bn * kDB;
  Acc<kDB, kDB> acc;
  acc.zero();
  const RowLoader<kDB> la{A, lda, row0, M, K};
  if constexpr (kBT) {
    const KLoader<kDB> lb{B, ldb, col0, N, K};
    run_mainloop<PIPE, true>(la, lb, 0, K, acc, smem_raw);
  } else {
    const RowLoader<kDB> lb{B, ldb, (int64_t)col0, N, K};
    run_mainloop<PIPE, true>(la, lb, 0, K, acc, smem_raw);
  }
  // acc.v[i][j][r]: pixel 16 i + p of the wave's 64-row panel, channel 16 j + 4 g + r of its 64-column panel
  constexpr int TM = Acc<kDB, kDB>::TM, TN = Acc<kDB, kDB>::TN;
  static_assert(TM == 4 && TN == 4 && kMS == 16, "64 x 64 wave tiles of 16x16 fragments");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int g = lane >> 4, p = lane & 15;
  const int64_t pix0 = row0 + wr * 64 + p;  // + 16 i
  // after the swaps: chunk (i, jp) of this lane = channels cb + 16 jp .. + 7 of pixel pix0 + 16 i
  const int cb = col0 + wc * 64 + 16 * (g & 1) + 8 * (g >> 1);
  u32x4_t dv[TM][2];
  uint32_t db[TM][2];
  if constexpr (kAdd) {  // the addends of all 8 chunks in flight before the packing
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t m = pix0 + 16 * i;
        const int n = cb + 32 * h;
        const bool ok = m < M && n < N;
        const int64_t e = ok ? m * ldd + n : 0;
        dv[i][h] = ok ? *reinterpret_cast<const u32x4_t*>(D + e) : u32x4_t{0u, 0u, 0u, 0u};
        db[i][h] = (ok && dmask) ? (uint32_t)dmask[e >> 3] : 0xffu;
      }
  }
  uint32_t u[TM][TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      u[i][j][0] = pack_bf16(acc.v[i][j][0], acc.v[i][j][1]);
      u[i][j][1] = pack_bf16(acc.v[i][j][2], acc.v[i][j][3]);
    }
  if constexpr (kStats) {
    // per channel (j, r) of this lane: sum and sum of squares over its valid pixels, bf16-rounded values
    f32x2_t ps[TN][2], pq[TN][2];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) ps[j][h] = pq[j][h] = f32x2_t{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool ok = pix0 + 16 * i < M;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x2_t v = unpack_bf16(u[i][j][h]);
          v = ok ? v : f32x2_t{0.f, 0.f};
          ps[j][h] += v;
          pq[j][h] = __builtin_elementwise_fma(v, v, pq[j][h]);
        }
    }
    // 16-lane row sums (every lane of the row ends with the totals of its row's 16 channels)
    float* red = reinterpret_cast<float*>(smem_raw);  // [2 wr][128 channels][2]
    __syncthreads();  // the main loop's last LDS reads are done before the stats reuse the bytes
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s4[4], q4[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        s4[2 * h] = row16_sum(ps[j][h].x);
        s4[2 * h + 1] = row16_sum(ps[j][h].y);
        q4[2 * h] = row16_sum(pq[j][h].x);
        q4[2 * h + 1] = row16_sum(pq[j][h].y);
      }
      if (p == 0) {  // channels wc 64 + 16 j + 4 g .. + 3: (sum, sumsq) interleaved, two 16-byte stores
        float* dst = red + (wr * kDB + wc * 64 + 16 * j + 4 * g) * 2;
        *reinterpret_cast<float4_t*>(dst) = float4_t{s4[0], q4[0], s4[1], q4[1]};
        *reinterpret_cast<float4_t*>(dst + 4) = float4_t{s4[2], q4[2], s4[3], q4[3]};
      }
    }
    __syncthreads();
    if (tid < kDB && col0 + tid < N) {
      const float a = red[tid * 2] + red[(kDB + tid) * 2];
      const float b = red[tid * 2 + 1] + red[(kDB + tid) * 2 + 1];
      *reinterpret_cast<f32x2_t*>(stats + ((int64_t)bm * N + col0 + tid) * 2) = f32x2_t{a, b};
    }
  }
  // rows g, g ^ 1 exchange fragments j / j + 1: afterwards (X = u[i][jp], Y = u[i][jp + 1]) hold channels
  // [0..3] / [4..7] of the lane's 8-channel chunk
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jp = 0; jp < TN; jp += 2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto r = __builtin_amdgcn_permlane16_swap(u[i][jp][h], u[i][jp + 1][h], false, false);
        u[i][jp][h] = r[0];
        u[i][jp + 1][h] = r[1];
      }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t m = pix0 + 16 * i;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int jp = 2 * hh;
      const int n = cb + 32 * hh;
      u32x4_t v{u[i][jp][0], u[i][jp][1], u[i][jp + 1][0], u[i][jp + 1][1]};
      if constexpr (kAdd) {
        const uint32_t bits = db[i][hh];
        v[0] = add_pair(v[0], dv[i][hh][0], bits);
        v[1] = add_pair(v[1], dv[i][hh][1], bits >> 2);
        v[2] = add_pair(v[2], dv[i][hh][2], bits >> 4);
        v[3] = add_pair(v[3], dv[i][hh][3], bits >> 6);
      }
      if (m < M && n < N) *reinterpret_cast<u32x4_t*>(C + m * ldc + n) = v;
    }
  }
}

template <bool kStats, bool kBT, bool kAdd, int PIPE>
__global__ __launch_bounds__(256, 2) void gemm_direct_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                             const bf16_t* __restrict__ B, int64_t ldb,
                                                             bf16_t* __restrict__ C, int64_t ldc, int M, int N, int K,
                                                             float* __restrict__ stats, const bf16_t* __restrict__ D,
                                                             int64_t ldd, const uint8_t* __restrict__ dmask) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  direct_tile<kStats, kBT, kAdd, PIPE>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, dmask,
                                       xcd_remap(blockIdx.x, gridDim.x), smem_raw);
}

// Persistent form: a fixed grid of blocks walks the tiles (block b takes virtual slots b, b + grid, ...; the
// XCD-aware remap of the virtual slot keeps the blocks of one XCD on consecutive tiles, i.e. on the column tiles
// of the same rows). No block launch / retirement per tile: a block's stores drain while it already loads its
// next tile. Every block runs the same number of slots; slots past the last tile do nothing, so every wave
// reaches the end.
template <bool kStats, bool kBT, bool kAdd, int PIPE>
__global__ __launch_bounds__(256, 2) void gemm_direct_persist_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, bf16_t* __restrict__ C,
    int64_t ldc, int M, int N, int K, float* __restrict__ stats, const bf16_t* __restrict__ D, int64_t ldd,
    const uint8_t* __restrict__ dmask, int tiles, int slots) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int total = slots * (int)gridDim.x;
  for (int it = 0; it < slots; ++it) {
    const int tile = xcd_remap(it * (int)gridDim.x + (int)blockIdx.x, total);
    if (tile < tiles) {
      direct_tile<kStats, kBT, kAdd, PIPE>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, dmask, tile, smem_raw);
    }
    __syncthreads();  // the statistics combine's LDS reads are done before the next tile's stores into LDS
  }
}

// 0 = one block per tile (gemm_direct_kernel); n > 0 = the persistent kernel with n blocks per CU
static int g_persist = -1;  // -1: environment (DLA_GEMM_PERSIST, default 0)
int gemm_persist_blocks() {
  if (g_persist >= 0) return g_persist;
  static const int env = [] {
    const char* e = std::getenv("DLA_GEMM_PERSIST");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return env;
}

template <bool S, bool BT, bool ADD, int PIPE>
void launch_direct_p(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M, int N,
                     int K, float* stats, const bf16_t* D, int64_t ldd, const uint8_t* dmask, hipStream_t stream) {
  const int tiles = ((M + kDB - 1) / kDB) * ((N + kDB - 1) / kDB);
  size_t lds = BT ? run_mainloop_lds_bytes<PIPE, kDB, kDB, RowLoader<kDB>, KLoader<kDB>>()
                  : run_mainloop_lds_bytes<PIPE, kDB, kDB, RowLoader<kDB>, RowLoader<kDB>>();
  if (S) lds = std::max(lds, (size_t)2 * kDB * 2 * sizeof(float));
  const int per_cu = gemm_persist_blocks();
  if (per_cu > 0 && tiles > 256 * per_cu) {
    const int grid = 256 * per_cu;  // a multiple of the 8 XCDs
    const int slots = (tiles + grid - 1) / grid;
    hipLaunchKernelGGL((gemm_direct_persist_kernel<S, BT, ADD, PIPE>), dim3(grid), dim3(256), lds, stream, A, lda, B,
                       ldb, C, ldc, M, N, K, stats, D, ldd, dmask, tiles, slots);
    return;
  }
  hipLaunchKernelGGL((gemm_direct_kernel<S, BT, ADD, PIPE>), dim3(tiles), dim3(256), lds, stream, A, lda, B, ldb, C,
                     ldc, M, N, K, stats, D, ldd, dmask);
}

template <bool S, bool BT, bool ADD>
void launch_direct(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M, int N,
                   int K, float* stats, const bf16_t* D, int64_t ldd, const uint8_t* dmask, hipStream_t stream) {
  // the tile kernel's per-K choice: register staging up to K = 512, the 2-stage LDS-DMA loop above
  const int pipe = mfma_pipeline() >= 0 ? mfma_pipeline() : (K > 512 ? 2 : 0);
  if (pipe == 0) launch_direct_p<S, BT, ADD, 0>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, dmask, stream);
  else if (pipe == 6) launch_direct_p<S, BT, ADD, 6>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, dmask, stream);
  else launch_direct_p<S, BT, ADD, 2>(A, lda, B, ldb, C, ldc, M, N, K, stats, D, ldd, dmask, stream);
}

}  // namespace

// -1: environment (DLA_GEMM_DIRECT, default OFF: same step time as the staged tile, profiles/r6/g03), 0 off, 1 on
static int g_direct = -1;
void set_gemm_direct(int mode) { g_direct = mode < 0 ? -1 : (mode ? 1 : 0); }
void set_gemm_persist(int blocks_per_cu) { g_persist = blocks_per_cu; }
bool gemm_direct_enabled() {
  static const bool env = [] {
    const char* e = std::getenv("DLA_GEMM_DIRECT");
    return e && e[0] == '1';
  }();
  return g_direct < 0 ? env : g_direct == 1;
}

bool gemm_direct_ok(int N, int64_t ldc, const void* addend, int64_t ldd) {
  return gemm_direct_enabled() && N % 8 == 0 && ldc % 8 == 0 && (!addend || ldd % 8 == 0);
}

void launch_gemm_direct(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, void* C, int64_t ldc,
                        int M, int N, int K, float* stats, const void* addend, int64_t ldd,
                        const uint8_t* addend_mask, hipStream_t stream) {
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
  bf16_t* c = (bf16_t*)C;
  const bf16_t* d = (const bf16_t*)addend;
#define DLA_DIR(S_, BT_, ADD_) \
  launch_direct<S_, BT_, ADD_>(a, lda, b, ldb, c, ldc, M, N, K, stats, d, ldd, addend_mask, stream)
  if (stats) {
    if (b_kmajor) DLA_DIR(true, true, false); else DLA_DIR(true, false, false);
  } else if (d) {
    if (b_kmajor) DLA_DIR(false, true, true); else DLA_DIR(false, false, true);
  } else {
    if (b_kmajor) DLA_DIR(false, true, false); else DLA_DIR(false, false, false);
  }
#undef DLA_DIR
}

}  // namespace dla
