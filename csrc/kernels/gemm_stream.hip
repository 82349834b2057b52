// Persistent streaming GEMM for the memory-bound 1x1 convolutions (short K, long M):
//   C[M, N] = A[M, K] * B^T,  B = W [N][K] (forward) or W [K][N] (data gradient, k-major),
//   K in {64, 128, 256}, bf16 in / out, fp32 accumulate, optional BatchNorm column statistics.
//
// Why a second 1x1 kernel. The tile-per-block gemm_nt (gemm.hip) runs each tile as
// load -> MFMA -> epilogue -> store, one latency after the other; at K <= 256 its blocks hold less than
// one tile of loads in flight per CU on average, and the per-kernel bytes table
// (profiles/r3/resnet50_bs1024_bytes_per_kernel.md) shows those kernels at 3.6-3.8 TB/s against 5.6 TB/s
// for the BatchNorm streams next to them. Here
//   * one block per CU stays resident over a strided set of 128-row tiles (grid = CUs), the weight
//     panel [BN][K] is staged into LDS ONCE per block;
//   * A moves HBM -> LDS by buffer LDS-DMA (no VGPRs) through a ring of kS 64-deep K-chunk slots, kP chunks
//     ahead of the MFMAs and ACROSS tile boundaries, so the next tile's rows are in flight while this
//     tile multiplies and stores: ~64 KB in flight per CU at all times;
//   * the product is computed transposed (weights as the MFMA A operand), with the weight rows
//     permuted in LDS so that each lane's 16 accumulators of one output row are 16 consecutive
//     channels: the tile leaves straight from registers as two 16-byte buffer stores per row and lane
//     (no LDS round trip, no barrier);
//   * every memory op is a buffer op whose out-of-range offset the hardware zero-fills / drops, so each
//     loop iteration issues the same number of them and the vmcnt waits are compile-time counts;
//   * BatchNorm statistics of the stored (bf16-rounded) outputs accumulate in registers over all of a
//     block's tiles and are reduced once at the end: one [N][2] partial row per row group, fixed order.
// Blocks of one row group (its N / BN column panels) sit on one XCD and read the same A rows from
// that XCD's L2.
#include <cstdlib>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

constexpr int kSBM = 128;  // rows per tile
constexpr int kChunkElems = kSBM * kBK;  // one ring slot [128][64]
// K-chunks in flight ahead of the MFMAs (ring slots = that + 1). The fused-addend variants run two blocks
// per CU (80 KB of LDS each) with 2 chunks in flight: their epilogue loads its addend just in time and
// waits for it, and the co-resident block's ring keeps HBM busy meanwhile. (Loading the addend a tile
// ahead into registers with hidden asm loads broke at K = 128: loop-carried registers get copied by the
// register allocator before the data lands, which no waitcnt covers.)
__host__ __device__ constexpr int stream_lookahead(int KC, bool add) { return add ? 2 : 4; }

struct StreamArgs {
  const bf16_t* a;
  int64_t lda;
  const bf16_t* b;
  int64_t ldb;
  bf16_t* c;
  int64_t ldc;
  int M, N;
  int mg;       // row groups (blocks per column panel)
  int per_xcd;  // row groups per XCD
  float* stats;  // [mg][N][2] or null
  // fused addend (data-gradient epilogue): C = bf16(bf16(acc) + (mask bit ? D : 0)), D [M][N] with row
  // stride ldd; mask: 1 bit per D element (null = all set), bit e of byte e >> 3 for element e = m * ldd + n
  const bf16_t* d;
  int64_t ldd;
  const uint8_t* dmask;
  // BatchNorm-backward partials (kBnb, data gradients): the output IS the dy of a fused BN(+ReLU) whose
  // input x [M][N] (row stride ldbx) and 7N workspace are given; per column the sums of dy' and
  // dy' (x - mean), dy' = dy masked by the BN's ReLU (mode 1: recomputed from x with the forward's
  // scale / shift, 2: its 1-bit mask laid out like the output, 0: none), accumulated over the block's
  // tiles and written like the statistics ([mg][N][2] into `stats`)
  const bf16_t* bx;
  int64_t ldbx;
  const float* bws;
  const uint8_t* bmask;
  int bmode;
  // deferred BN+ReLU of the A operand (kAp, forwards): A = y, the BN's input; the kernel multiplies
  // relu(y * scale + shift) (scale / shift at aws[2K, 3K) / [3K, 4K) of the BN's 7K workspace) and writes it to aout
  // (row stride lda) from the column panel 0 blocks
  const float* aws;
  bf16_t* aout;
  // kStem: A is the ResNet stem's implicit im2col over the space-to-depth image xs [n][BH][BW][16] (stem.hip):
  // row = output pixel (n, oh, ow), 64-deep k-step th = filter row, logical 16-byte chunk (tw, channel half) =
  // folded pixel (oh - 2 + th, ow - 2 + tw); pieces outside the image read zeros (buffer offset kOOB)
  int sBH, sBW;
  FastDiv sfW, sfH;
  uint32_t a_bytes;  // kStem: bytes of xs
};

// image row of panel-local weight row p (0..63 within a wave's 64 columns): the MFMA A-operand row
// 16 i + 4 g + r holds output column 16 g + 4 i + r, so lane group g accumulates columns 16 g .. 16 g + 15
__device__ __forceinline__ int perm64(int p) { return 16 * ((p >> 2) & 3) + 4 * (p >> 4) + (p & 3); }

// element offset of (row, logical 8-element chunk lc) in a [rows][64] LDS image (rm_glds_frag's swizzle)
__device__ __forceinline__ int img_off(int row, int lc) { return row * kBK + ((lc ^ ((row >> 1) & 7)) << 3); }

typedef int i32x4_t __attribute__((ext_vector_type(4)));


// kBM: BN-backward partials of the output's consuming BN, -1 none, else its ReLU mode (0 none, 1 recomputed
// from x, 2 bit mask): compile-time so each variant holds only the registers its mode needs
// Two blocks per CU (80 KB of LDS each, 2 chunks in flight) for the plain fused-addend variant; with the BN
// partials on top its operand registers no longer fit two blocks, so it runs one block per CU with the
// 4-chunk ring of the other variants.
__host__ __device__ constexpr bool stream_two_blocks(bool add, bool bnb) { return add && !bnb; }

// kAp: the A operand is a deferred BN+ReLU output (ops/bn_act.py PendingApply): each thread transforms the 16-byte
// pieces its own LDS-DMA brought in (after its vmcnt wait, before the barrier that publishes the chunk), writes
// them back in place and stores them to aout: the BN's apply pass and the GEMM's re-read of its output disappear.
template <int BN, int KC, bool kBT, bool kStats, bool kAdd = false, int kBM = -1, bool kAp = false,
          bool kStem = false>
__global__ __launch_bounds__(256, stream_two_blocks(kAdd, kBM >= 0) ? 2 : 1) void gemm_stream_kernel(const StreamArgs s) {
  constexpr bool kBnb = kBM >= 0;
  static_assert(!kStem || (!kBT && !kAdd && !kBnb && !kAp && KC == 4), "stem: the K = 256 forward");
  static_assert(!kAp || (!kBT && !kAdd && !kBnb), "apply-on-load: forwards only");
  static_assert(!(kStats && kBnb), "the partials buffer holds either the statistics or the BN-backward sums");
  constexpr int kSP = stream_lookahead(KC, stream_two_blocks(kAdd, kBnb));
  constexpr int kSS = kSP + 1;
  constexpr int WN = 64;                    // columns per wave
  constexpr int WGN = BN / WN;              // waves along N (2 or 1)
  constexpr int WGM = 4 / WGN;              // waves along M
  constexpr int WM = kSBM / WGM;            // rows per wave (64 or 32)
  constexpr int TJ = WM / 16;               // 16-row fragments per wave
  constexpr int Q = kSP / KC;               // tile ends inside kSP consecutive chunks
  static_assert(kSP % KC == 0, "the in-flight window must hold whole tiles");
  constexpr int D = kChunkElems / 8 / 256;  // LDS-DMA instructions per wave per chunk (4)
  constexpr int E = 2 * TJ;                 // buffer stores per wave per tile
  constexpr int F = (kAdd ? 3 * TJ : 0) + (kBnb ? (kBM == 2 ? 3 : 2) * TJ : 0);  // addend / BN x (2 x 16 B) + mask (2 B)
  // ops issued after chunk q before its wait. The epilogue's operand loads are waited for by their use
  // (which drains everything older, chunk q included), so a count clamped to the 6-bit field is only
  // stricter than necessary, never too weak
  // (kAp: each iteration also stores its chunk's D transformed pieces before issuing the next chunk)
  constexpr int kVmRaw = (kSP - 1) * (kAp ? 2 * D : D) + Q * (E + F);
  constexpr int kVmAfter = kVmRaw < 63 ? kVmRaw : 63;
  static_assert(kBnb || kVmRaw <= 63, "vmcnt is a 6-bit count");
  constexpr int kPanelElems = BN * kBK;     // one weight sub-image [BN][64]

  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* Bs = reinterpret_cast<bf16_t*>(smem_raw);  // KC sub-images [BN][64]
  bf16_t* ring = Bs + KC * kPanelElems;              // kSS slots [128][64]
  float* coef = reinterpret_cast<float*>(ring + kSS * kChunkElems);  // kAp: [scale | shift] x KC * 64

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  const int lr = lane & 15, g = lane >> 4;
  // XCD-aware block -> (column panel, row group)
  const int nbn = s.N / BN;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int bn = slot % nbn;
  const int grp = xcd * s.per_xcd + slot / nbn;
  const int col0 = bn * BN;
  const int M = s.M;
  const int mt = (M + kSBM - 1) / kSBM;
  const int ntile = grp < mt ? (mt - grp + s.mg - 1) / s.mg : 0;
  const int nchunk = ntile * KC;

  // ---- weight panel -> LDS (once): rows permuted per 64-column wave panel --------------------------
  // all of a thread's chunk loads are issued before any LDS write (one latency, not one per chunk)
  {
    constexpr int kPer = BN * KC * kBK / 8 / 256;  // 16-byte chunks per thread (2 .. 16)
    static_assert(BN * KC * kBK / 8 % 256 == 0, "whole chunks per thread");
    ushort8_t v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      if constexpr (!kBT) {
        const int n = c / (KC * 8), kc = c % (KC * 8);  // 8-element chunk kc of weight row n
        v[u] = *reinterpret_cast<const ushort8_t*>(s.b + (int64_t)(col0 + n) * s.ldb + kc * 8);
      } else {
        const int k = c / (BN / 8), nc = (c % (BN / 8)) * 8;  // 8 columns nc.. of k-row k
        v[u] = *reinterpret_cast<const ushort8_t*>(s.b + (int64_t)k * s.ldb + col0 + nc);
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      if constexpr (!kBT) {
        const int n = c / (KC * 8), kc = c % (KC * 8);
        const int row = (n & ~63) + perm64(n & 63);
        *reinterpret_cast<ushort8_t*>(Bs + (kc >> 3) * kPanelElems + img_off(row, kc & 7)) = v[u];
      } else {
        const int k = c / (BN / 8), nc = (c % (BN / 8)) * 8;
        bf16_t* sub = Bs + (k >> 6) * kPanelElems;
        const int kk = k & 63;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int n = nc + e, row = (n & ~63) + perm64(n & 63);
          sub[img_off(row, kk >> 3) + (kk & 7)] = v[u][e];
        }
      }
    }
  }

  // ---- A ring: chunk q = (tile q / KC, k-chunk q % KC) -> slot q % kSS ------------------------------
  const __amdgpu_buffer_rsrc_t ra = make_srd(s.a, kStem ? s.a_bytes : (uint32_t)((int64_t)M * s.lda * 2));
  // kStem: per row slot of the tile being issued, the folded-pixel element index at th = 0 and the bit mask of the
  // filter rows th inside the image (0: the row or its column tw is outside); this thread's (tw, half) is fixed
  int sbase[kStem ? D : 1];
  uint32_t smsk[kStem ? D : 1];
  const int stw = rm_glds_kc(tid) >> 4, shalf = rm_glds_kc(tid) & 8;
  uint32_t vo[D];
  int vr[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const int c = tid + i * 256, r = c >> 3;
    vr[i] = r;
    vo[i] = (uint32_t)(((int64_t)r * s.lda + rm_glds_kc(c)) * 2);
  }
  const uint32_t ring0 = lds_addr(ring) + (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int q) {
    const int t = q / KC, kc = q % KC;
    const int64_t row0 = (int64_t)(grp + t * s.mg) * kSBM;  // past the end for q >= nchunk: all OOB
    uint32_t o[D];
    uint32_t soff;
    if constexpr (kStem) {
      if (kc == 0) {  // a new tile: its rows' pixels (issue runs in chunk order)
#pragma unroll
        for (int i = 0; i < D; ++i) {
          const int64_t p = row0 + vr[i];
          smsk[i] = 0u;
          sbase[i] = 0;
          if (p < M) {
            const uint32_t q2 = fdiv((uint32_t)p, s.sfW);
            const int ow = (int)p - (int)q2 * s.sBW;
            const uint32_t nn = fdiv(q2, s.sfH);
            const int oh = (int)q2 - (int)nn * s.sBH;
            const int bw = ow - 2 + stw;
            if ((unsigned)bw < (unsigned)s.sBW) {
#pragma unroll
              for (int th = 0; th < 4; ++th) smsk[i] |= ((unsigned)(oh - 2 + th) < (unsigned)s.sBH) ? (1u << th) : 0u;
              sbase[i] = (((int)nn * s.sBH + oh - 2) * s.sBW + bw) * 16 + shalf;
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < D; ++i)
        o[i] = ((smsk[i] >> kc) & 1u) ? (uint32_t)(sbase[i] + kc * s.sBW * 16) * 2u : kOOB;
      soff = 0u;
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) o[i] = row0 + vr[i] < M ? vo[i] : kOOB;
      soff = row0 < M ? (uint32_t)((row0 * s.lda + kc * kBK) * 2) : 0u;
    }
    bglds<D, 256 * 16>(o, ra, (uint32_t)__builtin_amdgcn_readfirstlane(soff),
                       ring0 + (uint32_t)((q % kSS) * kChunkElems * 2));
  };

  if constexpr (kAp) {
    for (int i = tid; i < 2 * KC * kBK; i += 256) coef[i] = s.aws[2 * KC * kBK + i];
  }
  // the weight panel's (and coefficient table's) plain loads and LDS writes must be complete before the ring
  // starts counting
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // addend operands of a tile, loaded at its epilogue (all rows before the first use; the compiler's
  // wait drains this block's ring, the other block on the CU streams meanwhile): lane (lr, g) needs
  // rows wm*WM + 16 j + lr, columns wn*64 + 16 g .. + 15 (the positions it stores)
  const __amdgpu_buffer_rsrc_t rd = make_srd(kAdd ? (const void*)s.d : (const void*)s.c, kAdd ? (uint32_t)((int64_t)M * s.ldd * 2) : 0u);
  const __amdgpu_buffer_rsrc_t rmk =
      make_srd(kAdd && s.dmask ? (const void*)s.dmask : (const void*)s.c, kAdd && s.dmask ? (uint32_t)(((int64_t)M * s.ldd + 7) / 8) : 0u);
  i32x4_t dv[kAdd ? TJ : 1][2];
  uint32_t mb[kAdd ? TJ : 1];
  // BN-backward operands: x rows of the lane's 16 columns and the BN's mask bits; per-column constants
  // of the block's fixed column panel held in registers
  const __amdgpu_buffer_rsrc_t rbx = make_srd(kBnb ? (const void*)s.bx : (const void*)s.c,
                                              kBnb ? (uint32_t)((int64_t)M * s.ldbx * 2) : 0u);
  const __amdgpu_buffer_rsrc_t rbm = make_srd(kBM == 2 ? (const void*)s.bmask : (const void*)s.c,
                                              kBM == 2 ? (uint32_t)(((int64_t)M * s.ldc + 7) / 8) : 0u);
  i32x4_t xv[kBnb ? TJ : 1][2];
  uint32_t xb[kBM == 2 ? TJ : 1];
  float bmean[kBnb ? 16 : 1], bsc[kBM == 1 ? 16 : 1], bsh[kBM == 1 ? 16 : 1];
  if constexpr (kBnb) {
    const int gc = col0 + wn * WN + 16 * g;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      bmean[e] = s.bws[gc + e];
      if constexpr (kBM == 1) {
        bsc[e] = s.bws[2 * s.N + gc + e];
        bsh[e] = s.bws[3 * s.N + gc + e];
      }
    }
  }
  auto load_operands = [&](int t) {
    const int64_t row0 = (int64_t)(grp + t * s.mg) * kSBM;
    const int gc = col0 + wn * WN + 16 * g;
    if constexpr (kAdd) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int64_t gm = row0 + wm * WM + 16 * j + lr;
        const bool ok = gm < M;
        const uint32_t off = ok ? (uint32_t)((gm * s.ldd + gc) * 2) : kOOB;
        dv[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0);
        dv[j][1] = __builtin_amdgcn_raw_buffer_load_b128(rd, ok ? off + 16 : kOOB, 0, 0);
        mb[j] = __builtin_amdgcn_raw_buffer_load_b16(rmk, ok ? (uint32_t)((gm * s.ldd + gc) >> 3) : kOOB, 0, 0);
      }
    }
    if constexpr (kBnb) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int64_t gm = row0 + wm * WM + 16 * j + lr;
        const bool ok = gm < M;
        const uint32_t off = ok ? (uint32_t)((gm * s.ldbx + gc) * 2) : kOOB;
        xv[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rbx, off, 0, 0);
        xv[j][1] = __builtin_amdgcn_raw_buffer_load_b128(rbx, ok ? off + 16 : kOOB, 0, 0);
        if constexpr (kBM == 2)
          xb[j] = __builtin_amdgcn_raw_buffer_load_b16(rbm, ok ? (uint32_t)((gm * s.ldc + gc) >> 3) : kOOB, 0, 0);
      }
    }
  };
#pragma unroll
  for (int q = 0; q < kSP; ++q) issue(q);

  const __amdgpu_buffer_rsrc_t rc = make_srd(s.c, (uint32_t)((int64_t)M * s.ldc * 2));
  // kAp: the pieces of every chunk this thread DMAs share one logical 8-channel group (rm_glds_kc(tid + 256 i) does
  // not depend on i); only column panel 0 writes the transformed operand
  const __amdgpu_buffer_rsrc_t rao = make_srd(kAp ? (void*)s.aout : (void*)s.c,
                                              kAp ? (uint32_t)((int64_t)M * s.lda * 2) : 0u);
  const int alk = rm_glds_kc(tid);
  const bool awriter = bn == 0;
  float st_s[4][4], st_q[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) st_s[i][r] = st_q[i][r] = 0.f;
  accv_t acc[4][TJ];

  for (int q = 0; q < nchunk; ++q) {
    // this wave's DMAs for chunk q are done once at most the younger ones are outstanding: the chunks
    // q+1 .. q+kSP-1 (D each) and the stores (+ next-tile operand loads) of the Q tiles that ended
    // after chunk q was issued
    if (q < kSP) vm_wait<(kSP - 1) * D>();
    else vm_wait<kVmAfter>();
    if constexpr (kAp) {  // this thread's pieces of chunk q have landed: BN + ReLU in place, store the result
      const int kc = q % KC;
      const int64_t arow0 = (int64_t)(grp + (q / KC) * s.mg) * kSBM;
      bf16_t* slot = ring + (q % kSS) * kChunkElems;
      float sc[8], sh[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[j] = coef[kc * kBK + alk + j];
        sh[j] = coef[KC * kBK + kc * kBK + alk + j];
      }
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const int c = tid + i * 256;
        const int64_t gr = arow0 + vr[i];
        const ushort8_t v = *reinterpret_cast<const ushort8_t*>(slot + c * 8);
        ushort8_t o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = gr < M ? f32_to_bf16(fmaxf(fmaf(bf16_to_f32(v[j]), sc[j], sh[j]), 0.f)) : 0;
        *reinterpret_cast<ushort8_t*>(slot + c * 8) = o;
        const uint32_t off = (awriter && gr < M) ? (uint32_t)((gr * s.lda + kc * kBK + alk) * 2) : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_t, o), rao, off, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR: slot (q-1) % kSS is refilled below
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(q + kSP);  // past this block's last chunk: OOB rows, zeros into a free slot (uniform counts)
    const int kc = q % KC;
    if (kc == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = accv_t{};
    }
    const bf16_t* As = ring + (q % kSS) * kChunkElems;
    const bf16_t* Ws = Bs + kc * kPanelElems;
#pragma unroll
    for (int kk = 0; kk < kBK / 32; ++kk) {
      bf16x8_t wf[4], xf[TJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[i] = rm_glds_frag(Ws, wn * WN + 16 * i, kk);
#pragma unroll
      for (int j = 0; j < TJ; ++j) xf[j] = rm_glds_frag(As, wm * WM + 16 * j, kk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = mfma(wf[i], xf[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    if (kc == KC - 1) {
      // ---- tile epilogue: lane (lr, g) holds rows wm*WM + 16 j + lr, columns wn*64 + 16 g .. + 15 ----
      const int64_t row0 = (int64_t)(grp + (q / KC) * s.mg) * kSBM;
      const int gc = col0 + wn * WN + 16 * g;
      load_operands(q / KC);
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int64_t gm = row0 + wm * WM + 16 * j + lr;
        const bool ok = gm < M;
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bf16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = f32_to_bf16(acc[i][j][r]);
            if constexpr (kAdd) {  // column 4 i + r of the lane's 16: the unfused bf16 add, masked
              const int e = 4 * i + r;
              const uint32_t dw = (uint32_t)dv[j][e >> 3][(e >> 1) & 3];
              const float d = bf16_to_f32((bf16_t)((e & 1) ? (dw >> 16) : (dw & 0xffffu)));
              const uint32_t bits = s.dmask ? mb[j] : 0xffffu;
              h[r] = f32_to_bf16(bf16_to_f32(h[r]) + (((bits >> e) & 1u) ? d : 0.f));
            }
            if constexpr (kStats) {
              const float v = bf16_to_f32(h[r]);  // statistics of the stored values; OOB rows are 0
              st_s[i][r] += v;
              st_q[i][r] = fmaf(v, v, st_q[i][r]);
            }
            if constexpr (kBnb) {  // the BN backward's reduction of the stored dy (OOB rows: dy = x = 0)
              const int e = 4 * i + r;
              const uint32_t xw = (uint32_t)xv[j][e >> 3][(e >> 1) & 3];
              const float xf = bf16_to_f32((bf16_t)((e & 1) ? (xw >> 16) : (xw & 0xffffu)));
              float gv = bf16_to_f32(h[r]);
              if constexpr (kBM == 1) gv = fmaf(xf, bsc[e], bsh[e]) > 0.f ? gv : 0.f;  // same fmaf as the forward
              if constexpr (kBM == 2) gv = ((xb[j] >> e) & 1u) ? gv : 0.f;
              st_s[i][r] += gv;
              st_q[i][r] = fmaf(gv, xf - bmean[e], st_q[i][r]);
            }
          }
          w[2 * i] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
          w[2 * i + 1] = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
        }
        const uint32_t off = ok ? (uint32_t)((gm * s.ldc + gc) * 2) : kOOB;
        const i32x4_t lo{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
        const i32x4_t hi{(int)w[4], (int)w[5], (int)w[6], (int)w[7]};
        __builtin_amdgcn_raw_buffer_store_b128(lo, rc, ok ? off : kOOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(hi, rc, ok ? off + 16 : kOOB, 0, 0);
      }
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the block's LDS is released
  if constexpr (kStats || kBnb) {
    // columns of this lane: wn*64 + 16 g + 4 i + r; sum the 16 row lanes (lr), then the WGM waves
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int x = 1; x < 16; x <<= 1) {
          st_s[i][r] += __shfl_xor(st_s[i][r], x, 64);
          st_q[i][r] += __shfl_xor(st_q[i][r], x, 64);
        }
    __syncthreads();  // every wave is past its last ring read: reuse the LDS
    float* red = reinterpret_cast<float*>(smem_raw);  // [WGM][BN][2]
    if (lr == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = wn * WN + 16 * g + 4 * i + r;
          red[(wm * BN + n) * 2 + 0] = st_s[i][r];
          red[(wm * BN + n) * 2 + 1] = st_q[i][r];
        }
    }
    __syncthreads();
    if (tid < BN * 2 && grp < s.mg) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) v += red[w * BN * 2 + tid];
      s.stats[((int64_t)grp * s.N + col0) * 2 + tid] = v;
    }
  }
}

template <int BN, int KC, bool kTwo, bool kAp = false>
constexpr size_t stream_lds_bytes() {
  return (size_t)(KC * BN * kBK + (stream_lookahead(KC, kTwo) + 1) * kChunkElems) * sizeof(bf16_t) +
         (kAp ? (size_t)2 * KC * kBK * sizeof(float) : 0);
}

int g_stream_mode = -1;  // -1: environment (DLA_GEMM_STREAM, default on), 0 off, 1 on (every K <= 256)

bool stream_enabled() {
  if (g_stream_mode >= 0) return g_stream_mode == 1;
  static const bool v = [] {
    const char* e = std::getenv("DLA_GEMM_STREAM");
    return !(e && e[0] == '0');
  }();
  return v;
}

struct StreamPlan {
  int bn = 0, mg = 0, per_xcd = 0, grid = 0;
};

// Served shapes, from the per-layer A/B at ResNet-50 bs1024 (profiles/r3/gemm_stream_ab.md): K = 64 / 128
// win or tie everywhere (fwd K 64 x N 256 -11 %, dgrad K 128 x N 256 -45 %); at K = 256 only the data
// gradient (k-major weights) wins (-11 % at N 512); the forward K = 256 shapes lose 1-12 % (N >= 512 at
// M <= 802k: the tile kernel's 2-4 co-resident blocks beat one 4-wave block per CU there).
StreamPlan stream_geometry(int64_t M, int N, bool add, bool bnb);

StreamPlan stream_plan(int64_t M, int N, int K, int64_t lda, int64_t ldc, bool b_kmajor, bool add = false,
                       bool bnb = false) {
  StreamPlan p;
  if (add && K > 128) return p;  // 2 blocks per CU: the K = 256 weight panel does not fit 80 KB
  if (!stream_enabled() || M <= 0) return p;
  if (K != 64 && K != 128 && !(K == 256 && (b_kmajor || g_stream_mode == 1))) return p;
  if (N % 64 != 0 || lda % 8 != 0 || ldc % 8 != 0) return p;
  if (M * lda * 2 >= (int64_t)kOOB || M * ldc * 2 >= (int64_t)kOOB) return p;
  return stream_geometry(M, N, add, bnb);
}

// blocks of the persistent grid for M rows x N columns (one block per CU; N / BN panels per row group)
StreamPlan stream_geometry(int64_t M, int N, bool add, bool bnb) {
  StreamPlan p;
  p.bn = N % 128 == 0 ? 128 : 64;
  const int nbn = N / p.bn;
  const int mt = (int)((M + kSBM - 1) / kSBM);
  // one block per CU: 256 blocks = 8 XCDs x per_xcd row groups x nbn panels; at least two tiles per
  // row group, or the ring has nothing to overlap (the tile kernel serves small M)
  int per_xcd = std::max(1, (stream_two_blocks(add, bnb) ? 64 : 32) / nbn);
  while (per_xcd > 1 && mt < 2 * 8 * per_xcd) per_xcd >>= 1;
  if (mt < 2 * 8 * per_xcd) return StreamPlan{};
  p.per_xcd = per_xcd;
  p.mg = 8 * per_xcd;
  p.grid = p.mg * nbn;
  return p;
}

// The ResNet stem forward (7x7 / s2 over 3 channels, stem.hip) on this kernel: K = 256 over the space-to-depth
// image, Cout = 64 (one 64-column panel), BN statistics in registers. DLA_STEM_STREAM / set_stem_stream (default
// off: the 128x64 implicit-GEMM tile kernel)
int g_stem_stream = -1;
bool stem_stream_enabled() {
  if (g_stem_stream >= 0) return g_stem_stream == 1;
  static const bool v = [] {
    const char* e = std::getenv("DLA_STEM_STREAM");
    return e && e[0] == '1';
  }();
  return v;
}

template <int BN, int KC>
void launch_stream_kc(const StreamArgs& a, int grid, bool kmajor, bool stats, bool add, hipStream_t stream) {
  const dim3 g(grid), b(256);
  if (a.aws) {  // forward over a deferred BN+ReLU output (always with statistics: the consumer's BN)
    hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, false, true, false, -1, true>), g, b,
                       (stream_lds_bytes<BN, KC, false, true>()), stream, a);
    return;
  }
  const int bm = a.bx != nullptr ? a.bmode : -1;
#define DLA_SBN(ADD_, M_)                                                                                         \
  hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, true, false, ADD_, M_>), g, b,                                  \
                     (stream_lds_bytes<BN, KC, stream_two_blocks(ADD_, (M_) >= 0)>()), stream, a)
  if constexpr (KC <= 2) {
    if (add) {  // data gradient with the fused addend (k-major weights, no statistics)
      switch (bm) {
        case 0: DLA_SBN(true, 0); break;
        case 1: DLA_SBN(true, 1); break;
        case 2: DLA_SBN(true, 2); break;
        default: DLA_SBN(true, -1); break;
      }
      return;
    }
  }
  if (bm >= 0) {  // data gradient carrying the consuming BN's backward reduction (k-major, no statistics)
    switch (bm) {
      case 0: DLA_SBN(false, 0); break;
      case 1: DLA_SBN(false, 1); break;
      default: DLA_SBN(false, 2); break;
    }
    return;
  }
#undef DLA_SBN
  constexpr size_t lds = stream_lds_bytes<BN, KC, false>();
  if (kmajor) {
    if (stats) hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, true, true>), g, b, lds, stream, a);
    else hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, true, false>), g, b, lds, stream, a);
  } else {
    if (stats) hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, false, true>), g, b, lds, stream, a);
    else hipLaunchKernelGGL((gemm_stream_kernel<BN, KC, false, false>), g, b, lds, stream, a);
  }
}

}  // namespace

void set_gemm_stream(int mode) { g_stream_mode = mode < 0 ? -1 : (mode ? 1 : 0); }
void set_stem_stream(int mode) { g_stem_stream = mode < 0 ? -1 : (mode ? 1 : 0); }

int stem_stream_rows(int64_t P, int Cout) {
  if (!stem_stream_enabled() || Cout != 64 || P <= 0 || P >= (1 << 24)) return 0;
  return stream_geometry(P, 64, false, false).mg;
}

bool launch_stem_stream(const void* xs, const void* wpk, void* y, int N, int BH, int BW, float* stats,
                        hipStream_t stream) {
  const int64_t P = (int64_t)N * BH * BW;
  const StreamPlan p = stream_geometry(P, 64, false, false);
  if (!stats || stem_stream_rows(P, 64) != p.mg || !p.mg) return false;
  const int64_t xs_bytes = P * 16 * 2;
  if (xs_bytes >= (int64_t)kOOB || P * 64 * 2 >= (int64_t)kOOB) return false;
  StreamArgs a{};
  a.a = (const bf16_t*)xs;
  a.lda = 256;
  a.b = (const bf16_t*)wpk;
  a.ldb = 256;
  a.c = (bf16_t*)y;
  a.ldc = 64;
  a.M = (int)P;
  a.N = 64;
  a.mg = p.mg;
  a.per_xcd = p.per_xcd;
  a.stats = stats;
  a.sBH = BH;
  a.sBW = BW;
  a.sfW = make_fastdiv((uint32_t)BW);
  a.sfH = make_fastdiv((uint32_t)BH);
  a.a_bytes = (uint32_t)xs_bytes;
  hipLaunchKernelGGL((gemm_stream_kernel<64, 4, false, true, false, -1, false, true>), dim3(p.grid), dim3(256),
                     (stream_lds_bytes<64, 4, false>()), stream, a);
  return true;
}

int gemm_stream_rows(int64_t M, int N, int K, int64_t lda, int64_t ldc, bool b_kmajor, bool add, bool bnb) {
  return stream_plan(M, N, K, lda, ldc, b_kmajor, add, bnb).mg;
}

bool launch_gemm_stream(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, void* C, int64_t ldc,
                        int M, int N, int K, float* stats, hipStream_t stream, const void* addend, int64_t ldd,
                        const uint8_t* addend_mask, const BnBwdArgs* bn_bwd, const float* apply_ws,
                        void* apply_out) {
  const StreamPlan p = stream_plan(M, N, K, lda, ldc, b_kmajor, addend != nullptr, bn_bwd != nullptr);
  if (!p.mg) return false;
  if (apply_ws && (b_kmajor || !stats || addend || bn_bwd || !apply_out)) return false;
  if (addend && (stats || !b_kmajor || ldd % 8 != 0 || (int64_t)M * ldd * 2 >= (int64_t)kOOB)) return false;
  if (bn_bwd) {  // partials go where the statistics would: [mg][N][2]
    const int64_t ldbx = bn_bwd->ldx ? bn_bwd->ldx : ldc;
    if (stats || !b_kmajor || ldbx % 8 != 0 || (int64_t)M * ldbx * 2 >= (int64_t)kOOB) return false;
  }
  StreamArgs a{(const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, M, N, p.mg, p.per_xcd,
               bn_bwd ? bn_bwd->part : stats, (const bf16_t*)addend, ldd, addend_mask,
               bn_bwd ? (const bf16_t*)bn_bwd->x : nullptr, bn_bwd ? (bn_bwd->ldx ? bn_bwd->ldx : ldc) : 0,
               bn_bwd ? bn_bwd->ws : nullptr, bn_bwd ? bn_bwd->mask : nullptr, bn_bwd ? bn_bwd->mode : 0,
               apply_ws, (bf16_t*)apply_out};
  const int kc = K / kBK;
  if (p.bn == 128) {
    if (kc == 1) launch_stream_kc<128, 1>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
    else if (kc == 2) launch_stream_kc<128, 2>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
    else launch_stream_kc<128, 4>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
  } else {
    if (kc == 1) launch_stream_kc<64, 1>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
    else if (kc == 2) launch_stream_kc<64, 2>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
    else launch_stream_kc<64, 4>(a, p.grid, b_kmajor, stats != nullptr, addend != nullptr, stream);
  }
  return true;
}

}  // namespace dla
