// Both gradients of a stride-1 1x1 convolution in ONE pass over dY (ResNet-50 stages 1-2):
//   dX[M][Cin]      = dY[M][Cout] W[Cout][Cin]       data gradient, bf16
//   dW[Cout][Cin]   = dY[M][Cout]^T X[M][Cin]        weight gradient, fp32 partial per row group + split reduce
// The separate kernels (gemm_stream / gemm_nt for dX, gemm_tn for dW) each stream dY from HBM (2 GB per stage-1
// call, twice). Here every dY tile crosses HBM -> LDS once and feeds both products:
//   * persistent blocks (one per CU, XCD-aware row groups as gemm_stream.hip) walk R-row tiles; per tile the dY
//     sub-images [R rows][64 co] and the block's X slice [R rows][64 ci] arrive by buffer LDS-DMA into an
//     NS-stage ring (NS - 1 tiles in flight ahead of the MFMAs);
//   * data gradient: the transposed product of gemm_stream.hip (W^T [ci][co] as the MFMA A operand, from a
//     once-staged row-permuted LDS panel or, kWReg, per-wave registers; dY rows as B); each lane stores 4 NCF
//     consecutive channels of one row straight from registers;
//   * weight gradient: the same dY sub-images read transposed (ds_read_b64_tr_b16, K = rows) against the
//     transposed X image, accumulated in registers over all of the block's tiles; one fp32 [Cout][64] partial per
//     block at the end, summed by splitk_reduce in fixed order (deterministic).
// Wider Cin is split into 64-channel slices, one block each; the slice blocks of a row group sit on one XCD.
// Served (launch_conv1x1_dual): (Cout, Cin) = (256, 64) with 64-row tiles; (512, 128 / 256) with 32-row tiles and
// register-held weights and a 4-stage ring; (256, 64) with the consuming BN's backward apply fused (kBN, the block-final BN).
// A fork form for the block's first conv (BN apply with the ReLU recomputed + the identity gradient added in the
// epilogue) measured slower (87.2-88.1 vs 84.2-84.5 ms per step, profiles/r4/g11-g12) and was removed.
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

// Configurations: see the served list above; LDS = weight panel (unless kWReg) + NS stages of the tile images.
constexpr int kUCi = 64;  // input channels per block (slice)
// kBN: dY is the backward of the BatchNorm(+residual)+ReLU that consumed the conv's output, applied on the
// fly: the tile brings the BN's incoming gradient (into the dY slots), its input y and its 1-bit ReLU mask,
// and a pass over LDS writes dY = k1 (g - m1 - (y - mean) k2), g = masked gradient, over the gradient in
// place (bn_bwd_apply's arithmetic and rounding) -- dY is never written to HBM.
constexpr int kUMaskWave = 1024;  // bytes of mask area per wave and stage (the first R / 4 rows x CO / 8 used)
// kWReg: each wave holds its W^T fragments in registers instead of a block-wide LDS panel (Cout 512: the
// 64 KB panel would leave no room for a deeper ring or the kBN tiles).
template <int CO, int R, int NS, bool kBN = false, bool kWReg = false>
struct DualCfg {
  static constexpr int KC = CO / kBK;                 // dY sub-images per tile
  static constexpr int Sub = R * kBK;                 // elements of one [R][64] sub-image
  static constexpr int Area = 4 * kUMaskWave / 2;     // elements of a per-wave mask area set
  static constexpr int Xs = (kBN ? 2 : 1) * KC;       // sub-image index of the X slice
  static constexpr int MaskAt = (Xs + 1) * Sub;       // kBN: the mask areas
  static constexpr int Stage = MaskAt + (kBN ? Area : 0);
  static constexpr int Panel = kUCi * kBK;            // one W^T sub-image [64 ci][64 co]
  static constexpr int Slots = Sub / 8 / 256;         // LDS-DMA slots per thread per sub-image
  static constexpr int Loads = (Xs + 1) * Slots + (kBN ? 1 : 0);
  static_assert(!kBN || CO * R / 8 / 4 <= kUMaskWave, "BN mask: one DMA per wave (64 lanes x 16 B)");
  static constexpr int RF = R / 16;                   // 16-row fragments of a tile
  static constexpr int NCF = RF;                      // data gradient: 16-channel fragments per wave (4 waves)
  static constexpr int Stores = NCF / 2;              // dX stores per lane per tile (4 NCF channels)
  static constexpr int TMW = CO / 64;                 // weight gradient: 16-row co fragments per wave
  static constexpr size_t Lds = (size_t)((kWReg ? 0 : KC * Panel) + NS * Stage) * sizeof(bf16_t);
  static_assert(Lds <= 160 * 1024, "dual 1x1 LDS budget");
  static_assert(Slots >= 1 && (RF == 2 || RF == 4) && NS >= 2 && NS <= 4, "tile configuration");
};

struct DualArgs {
  const bf16_t* dy;  // [M][CO] (kBN: the BN's incoming gradient)
  const bf16_t* x;   // [M][CI]
  const bf16_t* w;   // [CO][CI]  (W[co][ci], the k-major form of the data gradient)
  bf16_t* dx;        // [M][CI]
  float* part;       // [mg][CO][CI]
  int M, CI;
  int mg, per_xcd, nsl;  // row groups, row groups per XCD, Cin slices
  const bf16_t* ybn;     // kBN: the BN input [M][CO]
  const uint8_t* mask;   // kBN: its ReLU bit mask (bit e of byte e >> 3, e = m * CO + c)
  const float* ws;       // kBN: the finalized 7 CO workspace (mean, ..., k1, m1, k2)
};

// image row of panel-local weight row p (gemm_stream.hip): MFMA A-operand row 16 i + 4 g + r holds output
// column 16 g + 4 i + r, so lane group g accumulates columns 16 g .. 16 g + 15
__device__ __forceinline__ int uperm64(int p) { return 16 * ((p >> 2) & 3) + 4 * (p >> 4) + (p & 3); }
// The tile images are read two ways: row fragments by ds_read_b128 (data gradient) and transposed fragments by
// ds_read_b64_tr_b16 (weight gradient). The LDS-DMA image's chunk XOR ((row >> 1) & 7) is conflict-free for the
// first but pairs the transposed reads' 16-byte chunks 2-way (rows 2 apart XOR to adjacent chunks; r5 g37:
// 6.4e8 conflict cycles per 5 steps in the Cout-256 kernel). The XOR below (bit 1 of the row -> chunk bit 1,
// bit 3 -> chunk bit 2; found by exhaustive search over the two instructions' lane groups) serves both.
#ifndef DLA_DUAL_SWZ
#define DLA_DUAL_SWZ 2
#endif
__device__ __forceinline__ int usw(int row) {
  if constexpr (DLA_DUAL_SWZ == 2) return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
  else return (row >> 1) & 7;
}
// element offset of (row, 8-element chunk lc) in a [rows][64] tile image
__device__ __forceinline__ int uimg(int row, int lc) { return row * kBK + ((lc ^ usw(row)) << 3); }
// logical k of LDS-DMA slot c (row c >> 3, physical chunk c & 7) of that image
__device__ __forceinline__ int uimg_kc(int c) { return ((c & 7) ^ usw(c >> 3)) << 3; }
// 16 x 32 row fragment (rm_glds_frag's operand layout) from that image
__device__ __forceinline__ bf16x8_t urm_frag(const bf16_t* s, int r0, int kk) {
  const int lane = threadIdx.x & 63;
  const int r = r0 + (lane & (kMS - 1)), lc = kk * (kKS / 8) + lane / kMS;
  return *reinterpret_cast<const bf16x8_t*>(s + uimg(r, lc));
}
// element offset of (row, col), col % 4 == 0, in the same image: 4 consecutive columns are contiguous
__device__ __forceinline__ int urm_off(int row, int col) { return uimg(row, col >> 3) + (col & 7); }

// 16 x 32 operand fragment with K along the image ROWS (the weight gradient's K = pixel rows): the
// transposed read of tile_frag's k-major path (lane 4q+p of 16-lane group g reads rows kk*32 + 8g + q and
// + 4, columns c0 + 4p .. + 3), addressed in the row-major LDS-DMA image
__device__ __forceinline__ bf16x8_t urm_tr_frag(const bf16_t* s, int c0, int kk) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int kr = kk * 32 + 8 * g + q, cn = c0 + 4 * p;
  return tr_frag(s + urm_off(kr, cn), s + urm_off(kr + 4, cn));
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));

template <int CO, int R, int NS, bool kBN = false, bool kWReg = false>
__global__ __launch_bounds__(256, 1) void conv1x1_dual_kernel(const DualArgs s) {
  using G = DualCfg<CO, R, NS, kBN, kWReg>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem_raw);  // KC sub-images [64 ci (permuted)][64 co]
  bf16_t* ring = Ws + (kWReg ? 0 : G::KC * G::Panel);  // NS stages
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  // XCD-aware: the nsl slice blocks of one row group are adjacent slots of one XCD
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int sl = slot % s.nsl;
  const int grp = xcd * s.per_xcd + slot / s.nsl;
  const int ci0 = sl * kUCi;
  const int M = s.M, CI = s.CI;
  const int mt = (M + R - 1) / R;
  const int ntile = grp < mt ? (mt - grp + s.mg - 1) / s.mg : 0;

  // data gradient of this wave: row fragment rf, channel fragments cf0 .. cf0 + NCF - 1 of the slice
  const int rf = wave % G::RF, cf0 = (wave / G::RF) * G::NCF;
  // kWReg: this wave's W^T fragments (what urm_frag would read from the panel below), loaded once
  bf16x8_t wreg[kWReg ? G::NCF : 1][kWReg ? 2 * G::KC : 1];
  if constexpr (kWReg) {
#pragma unroll
    for (int i = 0; i < G::NCF; ++i) {
      const int ci = ci0 + uperm64(16 * (cf0 + i) + lr);  // the permuted panel row's input channel
#pragma unroll
      for (int q = 0; q < 2 * G::KC; ++q) {
        const int co0 = (q >> 1) * kBK + ((q & 1) * 4 + g) * 8;
        ushort8_t v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = reinterpret_cast<const uint16_t*>(s.w)[(int64_t)(co0 + e) * CI + ci];
        wreg[i][q] = __builtin_bit_cast(bf16x8_t, v);
      }
    }
  }
  // ---- weight panel -> LDS once: W[co][ci0 .. ci0 + 63] k-major, written transposed and row-permuted ---
  if constexpr (!kWReg) {
    constexpr int kPer = CO * kUCi / 8 / 256;  // 16-byte chunks per thread
    ushort8_t v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      const int k = c / (kUCi / 8), nc = (c % (kUCi / 8)) * 8;  // columns nc .. nc + 7 of co-row k
      v[u] = *reinterpret_cast<const ushort8_t*>(s.w + (int64_t)k * CI + ci0 + nc);
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      const int k = c / (kUCi / 8), nc = (c % (kUCi / 8)) * 8;
      bf16_t* sub = Ws + (k >> 6) * G::Panel;
      const int kk = k & 63;
#pragma unroll
      for (int e = 0; e < 8; ++e) sub[uimg(uperm64(nc + e), kk >> 3) + (kk & 7)] = v[u][e];
    }
  }

  // ---- ring: tile t -> stage t % NS; slot i of a sub-image covers rows 32 i .. 32 i + 31 ----------------
  const __amdgpu_buffer_rsrc_t rdy = make_srd(s.dy, (uint32_t)((int64_t)M * CO * 2));
  const __amdgpu_buffer_rsrc_t rx = make_srd(s.x, (uint32_t)((int64_t)M * CI * 2));
  const __amdgpu_buffer_rsrc_t rybn = make_srd(kBN ? (const void*)s.ybn : (const void*)s.dy, (uint32_t)((int64_t)M * CO * 2));
  const __amdgpu_buffer_rsrc_t rmsk = make_srd(kBN ? (const void*)s.mask : (const void*)s.dy, (uint32_t)(((int64_t)M * CO + 7) / 8));
  uint32_t vdy[G::Slots], vx[G::Slots];
  int vr[G::Slots];
#pragma unroll
  for (int i = 0; i < G::Slots; ++i) {
    const int c = tid + i * 256, r = c >> 3;
    vr[i] = r;
    vdy[i] = (uint32_t)((r * CO + uimg_kc(c)) * 2);
    vx[i] = (uint32_t)((r * CI + ci0 + uimg_kc(c)) * 2);
  }
  const uint32_t ring0 = lds_addr(ring) + (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int t) {
    const int64_t row0 = (int64_t)(grp + t * s.mg) * R;  // past the end: every slot OOB (zero-filled)
    const uint32_t st = ring0 + (uint32_t)((t % NS) * G::Stage * 2);
    uint32_t o[G::Slots];
#pragma unroll
    for (int kc = 0; kc < G::KC; ++kc) {
#pragma unroll
      for (int i = 0; i < G::Slots; ++i) o[i] = row0 + vr[i] < M ? vdy[i] : kOOB;
      const uint32_t soff = row0 < M ? (uint32_t)((row0 * CO + kc * kBK) * 2) : 0u;
      bglds<G::Slots, 256 * 16>(o, rdy, (uint32_t)__builtin_amdgcn_readfirstlane(soff), st + (uint32_t)(kc * G::Sub * 2));
    }
    if constexpr (kBN) {
#pragma unroll
      for (int kc = 0; kc < G::KC; ++kc) {
#pragma unroll
        for (int i = 0; i < G::Slots; ++i) o[i] = row0 + vr[i] < M ? vdy[i] : kOOB;
        const uint32_t soff = row0 < M ? (uint32_t)((row0 * CO + kc * kBK) * 2) : 0u;
        bglds<G::Slots, 256 * 16>(o, rybn, (uint32_t)__builtin_amdgcn_readfirstlane(soff),
                                  st + (uint32_t)((G::KC + kc) * G::Sub * 2));
      }
    }
    constexpr int kXs = G::Xs;  // X slice sub-image index in the stage
#pragma unroll
    for (int i = 0; i < G::Slots; ++i) o[i] = row0 + vr[i] < M ? vx[i] : kOOB;
    const uint32_t soff = row0 < M ? (uint32_t)(row0 * CI * 2) : 0u;
    bglds<G::Slots, 256 * 16>(o, rx, (uint32_t)__builtin_amdgcn_readfirstlane(soff), st + (uint32_t)(kXs * G::Sub * 2));
    if constexpr (kBN) {
      // mask bytes of the tile: wave w fetches rows R/4 w .. (R / 4 bytes x CO / 8 per row, 16 B per lane)
      // into its own 1 KB area; the other lanes are out of range and write zeros behind them
      const uint32_t st0 = st - (uint32_t)(wave * 64 * 16);  // the stage base (st carries this wave's 1 KB offset)
      constexpr int kWaveBytes = R / 4 * CO / 8;
      const int64_t mrow = row0 + (R / 4) * wave + lane * 16 / (CO / 8);  // the row this lane's 16 bytes belong to
      uint32_t om[1] = {lane * 16 < kWaveBytes && mrow < M ? (uint32_t)(lane * 16) : kOOB};
      const uint32_t msoff = row0 < M ? (uint32_t)(row0 * CO / 8 + wave * kWaveBytes) : 0u;
      bglds<1, 0>(om, rmsk, (uint32_t)__builtin_amdgcn_readfirstlane(msoff),
                  st0 + (uint32_t)(G::MaskAt * 2) + (uint32_t)(wave * kUMaskWave));
    }
  };

  // the panel's plain loads and LDS writes complete before the ring starts counting
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue(t);

  const __amdgpu_buffer_rsrc_t rc = make_srd(s.dx, (uint32_t)((int64_t)M * CI * 2));
  // kBN: this thread's 8 channels (chunk column tid % (CO / 8)) in every row it converts
  constexpr int kCpr = CO / 8;  // 8-channel chunks per row
  float bmean[kBN ? 8 : 1], bk1[kBN ? 8 : 1], bm1[kBN ? 8 : 1], bk2[kBN ? 8 : 1];
  // kBN pass lane map (conflict-free for both its ds_read_b128 and ds_write_b128 under the usw image, found by
  // search, tests/test_lds_swizzle.py): a wave covers 2 rows x 32 chunks per step, row = lane bit 3, chunk =
  // lane bits 0-2 (chunk in sub-image) and 4-5 (sub-image); the straight map (32 lanes per row) read the 4
  // sub-images' same chunk positions from one bank slot: 2-way (r5 g41: 3.3e8 conflict cycles per 5 steps)
  static_assert(!kBN || (kCpr == 32 && R % 8 == 0), "kBN lane map: Cout 256, whole 8-row steps");
  const int bcg = (lane & 7) | (((lane >> 4) & 3) << 3), brb = (lane >> 3) & 1;
  if constexpr (kBN) {
    const int c0 = bcg * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmean[j] = s.ws[c0 + j];
      bk1[j] = s.ws[4 * CO + c0 + j];
      bm1[j] = s.ws[5 * CO + c0 + j];
      bk2[j] = s.ws[6 * CO + c0 + j];
    }
  }
  accv_t aw[G::TMW][4];  // dW rows co = (CO / 4) wave + 16 i + 4 g + r, slice columns 16 j + lr
#pragma unroll
  for (int i = 0; i < G::TMW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) aw[i][j] = accv_t{};

  for (int t = 0; t < ntile; ++t) {
    // tile t's DMAs (issued NS - 1 iterations back) are done once only the younger ones are outstanding;
    // issue order (NS = 3) L0 L1 | L2 S0 | L3 S1 | ..., (NS = 2) L0 | L1 S0 | L2 S1 | ...
    if (t >= NS - 1) vm_wait<(NS - 2) * G::Loads + (NS - 1) * G::Stores>();
    else if (t == 0) vm_wait<(NS - 2) * G::Loads>();
    else vm_wait<(NS - 2) * G::Loads + G::Stores>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR: stage (t-1) % NS is refilled below
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + NS - 1);
    bf16_t* Ds = ring + (t % NS) * G::Stage;  // dY sub-images
    const bf16_t* Xs = Ds + G::Xs * G::Sub;   // X slice
    if constexpr (kBN) {
      // dY = k1 (g - m1 - (y - mean) k2) over the gradient in place; g = the gradient where the ReLU passed
      const bf16_t* Ys = Ds + G::KC * G::Sub;
      const uint8_t* Ms = reinterpret_cast<const uint8_t*>(Ds + G::MaskAt);
      constexpr int kPer = R * kCpr / 256;  // chunks per thread
      const int cg = bcg, sub = cg >> 3, lc = cg & 7;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int r = 2 * (wave + 4 * k) + brb;
        const int o = sub * G::Sub + uimg(r, lc);
        const ushort8_t gv = *reinterpret_cast<const ushort8_t*>(Ds + o);
        const ushort8_t yv = *reinterpret_cast<const ushort8_t*>(Ys + o);
        const uint32_t bits = (uint32_t)Ms[(r / (R / 4)) * kUMaskWave + (r % (R / 4)) * kCpr + cg];
        ushort8_t out;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float y = bf16_to_f32((bf16_t)yv[j]);
          const float g = (bits >> j) & 1u ? bf16_to_f32((bf16_t)gv[j]) : 0.f;
          out[j] = f32_to_bf16(bk1[j] * (g - bm1[j] - (y - bmean[j]) * bk2[j]));
        }
        *reinterpret_cast<ushort8_t*>(Ds + o) = out;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }

    // ---- data gradient: rows 16 rf + lr, channels of fragments cf0 .. ------------------------------------
    accv_t ad[G::NCF];
#pragma unroll
    for (int i = 0; i < G::NCF; ++i) ad[i] = accv_t{};
#pragma unroll
    for (int kc = 0; kc < G::KC; ++kc) {
#pragma unroll
      for (int kk = 0; kk < kBK / 32; ++kk) {
        bf16x8_t wf[G::NCF];
#pragma unroll
        for (int i = 0; i < G::NCF; ++i) {
          if constexpr (kWReg) wf[i] = wreg[i][2 * kc + kk];
          else wf[i] = urm_frag(Ws + kc * G::Panel, 16 * (cf0 + i), kk);
        }
        const bf16x8_t yf = urm_frag(Ds + kc * G::Sub, 16 * rf, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::NCF; ++i) ad[i] = mfma(wf[i], yf, ad[i]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // ---- weight gradient: this wave's CO / 4 rows of co, the slice's 64 ci; K = the tile's R rows --------
#pragma unroll
    for (int kk = 0; kk < R / 32; ++kk) {
      bf16x8_t bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = urm_tr_frag(Xs, 16 * j, kk);
#pragma unroll
      for (int i = 0; i < G::TMW; ++i) {
        const int co = (CO / 4) * wave + 16 * i;
        const bf16x8_t af = urm_tr_frag(Ds + (co >> 6) * G::Sub, co & 63, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 4; ++j) aw[i][j] = mfma(af, bf[j], aw[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // ---- dX store: lane (lr, g) holds row 16 rf + lr, channels 16 g + 4 cf0 .. + 4 NCF - 1 ---------------
    {
      const int64_t gm = (int64_t)(grp + t * s.mg) * R + 16 * rf + lr;
      const bool ok = gm < M;
      uint32_t wv[2 * G::NCF];
#pragma unroll
        for (int i = 0; i < G::NCF; ++i) {
          wv[2 * i] = (uint32_t)f32_to_bf16(ad[i][0]) | ((uint32_t)f32_to_bf16(ad[i][1]) << 16);
          wv[2 * i + 1] = (uint32_t)f32_to_bf16(ad[i][2]) | ((uint32_t)f32_to_bf16(ad[i][3]) << 16);
        }
      const uint32_t off = ok ? (uint32_t)((gm * CI + ci0 + 16 * g + 4 * cf0) * 2) : kOOB;
#pragma unroll
      for (int h = 0; h < G::Stores; ++h) {
        const i32x4_t v{(int)wv[4 * h], (int)wv[4 * h + 1], (int)wv[4 * h + 2], (int)wv[4 * h + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rc, ok ? off + 16 * h : kOOB, 0, 0);
      }
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the block's LDS is released
  // ---- this row group's dW partial, slice columns: [co][ci0 + ..] fp32 (no tiles: zeros) -----------------
  float* P = s.part + (int64_t)grp * CO * CI + ci0;
#pragma unroll
  for (int i = 0; i < G::TMW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) P[(int64_t)((CO / 4) * wave + 16 * i + 4 * g + r) * CI + 16 * j + lr] = aw[i][j][r];
}

}  // namespace

// Served shapes (Cout, Cin): (256, 64) and (512, 128 / 256); at least 4 tiles per block.
int conv1x1_dual_blocks(int64_t M, int Cin, int Cout) {
  if (M <= 0 || Cin % kUCi) return 0;
  const int nsl = Cin / kUCi;
  int R;
  if (Cout == 256 && nsl == 1) R = 64;
  else if (Cout == 512 && (nsl == 2 || nsl == 4)) R = 32;
  else return 0;
  if (M * Cout * 2 >= (int64_t)kOOB || M * Cin * 2 >= (int64_t)kOOB) return 0;
  const int mg = 256 / nsl;
  if ((M + R - 1) / R < (int64_t)mg * 4) return 0;  // a few tiles per block, or the ring has nothing to overlap
  return 256;
}

int conv1x1_dual_groups(int64_t M, int Cin, int Cout) {
  return conv1x1_dual_blocks(M, Cin, Cout) ? 256 / (Cin / kUCi) : 0;
}

// The fused BN apply only for Cout 256: at Cout 512 (W fragments in registers, 2-stage ring, 2-4 slice blocks
// each streaming the BN's gradient AND input) it measured 1.32 ms per call against 0.50 ms for the plain kernel
// plus 0.33 ms for the separate apply pass (profiles/r4/g08).
bool conv1x1_dual_bn_ok(int64_t M, int Cin, int Cout) { return Cout == 256 && conv1x1_dual_blocks(M, Cin, Cout) > 0; }

bool launch_conv1x1_dual(const void* dy, const void* x, const void* w, void* dx, float* part, int64_t M, int Cin,
                         int Cout, hipStream_t stream, const void* ybn, const uint8_t* mask, const float* ws) {
  const int mg = conv1x1_dual_groups(M, Cin, Cout);
  if (!mg) return false;
  const int nsl = Cin / kUCi, grid = mg * nsl;
  DualArgs a{(const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)dx, part, (int)M, Cin, mg, mg / 8, nsl,
             (const bf16_t*)ybn, mask, ws};
#define DLA_DUAL(CO_, R_, NS_, BN_, WR_)                                                                       \
  hipLaunchKernelGGL((conv1x1_dual_kernel<CO_, R_, NS_, BN_, WR_>), dim3(grid), dim3(256),                      \
                     (DualCfg<CO_, R_, NS_, BN_, WR_>::Lds), stream, a)
  if (ybn) {
    if (!conv1x1_dual_bn_ok(M, Cin, Cout) || !mask || !ws) return false;
    DLA_DUAL(256, 32, 3, true, false);
    return true;
  }
  // Cout 512: weight fragments in registers + a 4-stage ring (3 tiles in flight; 3 stages: +0.19 ms/step over
  // 5 interleaved pairs, profiles/r4/g21; the LDS-panel form fits only 2 stages: slower)
  if (Cout == 256) DLA_DUAL(256, 64, 3, false, false);
  else DLA_DUAL(512, 32, 4, false, true);
#undef DLA_DUAL
  return true;
}

}  // namespace dla
