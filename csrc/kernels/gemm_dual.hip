// Both gradients of a stride-1 1x1 convolution in ONE pass over dY (ResNet-50 stage 1: conv3 and the
// downsample shortcut, Cin = 64 -> Cout = 256, 4M rows at bs1280):
//   dX[M][Cin]      = dY[M][Cout] W[Cout][Cin]       data gradient, bf16
//   dW[Cout][Cin]   = dY[M][Cout]^T X[M][Cin]        weight gradient, fp32 partial per block + split reduce
// The separate kernels (gemm_stream / gemm_nt for dX, gemm_tn for dW) each stream dY from HBM: 2 GB per
// call twice. Here every dY tile crosses HBM -> LDS once and feeds both products:
//   * persistent blocks (one per CU, XCD-aware row groups as gemm_stream.hip) walk 64-row tiles; per tile
//     4 dY sub-images [64 rows][64 co] and one X sub-image [64 rows][64 ci] arrive by buffer LDS-DMA
//     into a 3-stage ring (2 tiles in flight ahead of the MFMAs, 40 KB per stage);
//   * data gradient: the transposed product of gemm_stream.hip (W^T [ci][co] as the MFMA A operand from
//     a once-staged, row-permuted panel; dY rows as B), each lane stores 16 consecutive channels of one
//     row straight from registers;
//   * weight gradient: the same dY sub-images read transposed (ds_read_b64_tr_b16, K = rows) against the
//     transposed X image, accumulated in registers over all of the block's tiles; one fp32 [Cout][Cin]
//     partial per block at the end, summed by splitk_reduce in fixed order (deterministic).
// LDS: W panel 4 x 8 KB + 3 x 40 KB ring = 152 KB. Wave w: dX rows 16 w .. 16 w + 15 (all 64 ci), dW
// rows co 64 w .. 64 w + 63 (all 64 ci).
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using namespace mm;

namespace {

constexpr int kUR = 64;                      // rows per tile
constexpr int kUCo = 256;                    // Cout: K of the data gradient
constexpr int kUCi = 64;                     // Cin
constexpr int kUKC = kUCo / kBK;             // dY sub-images per tile (4)
constexpr int kUSub = kUR * kBK;             // elements of one [64][64] sub-image (8 KB)
constexpr int kUStage = (kUKC + 1) * kUSub;  // dY sub-images + X sub-image
constexpr int kUNS = 3;                      // ring stages: tiles t+1, t+2 in flight while t is multiplied
constexpr int kUPanel = kUCi * kBK;          // one W^T sub-image [64 ci][64 co]
constexpr int kUSlots = kUSub / 8 / 256;     // LDS-DMA slots per thread per sub-image (2)
constexpr int kULoads = (kUKC + 1) * kUSlots;  // DMA ops per wave per tile (10)
constexpr int kUStores = 2;                  // dX stores per lane per tile (16 channels = 2 x 16 B)
constexpr size_t kULds = (size_t)(kUKC * kUPanel + kUNS * kUStage) * sizeof(bf16_t);
static_assert(kULds <= 160 * 1024, "dual 1x1 LDS budget");
static_assert(kMS == 16, "fragment maps assume v_mfma_f32_16x16x32_bf16");

struct DualArgs {
  const bf16_t* dy;  // [M][256]
  const bf16_t* x;   // [M][64]
  const bf16_t* w;   // [256][64]  (W[co][ci], the k-major form of the data gradient)
  bf16_t* dx;        // [M][64]
  float* part;       // [grid][256][64]
  int M;
  int mg, per_xcd;   // row groups (= blocks), per XCD
};

// image row of panel-local weight row p (gemm_stream.hip): MFMA A-operand row 16 i + 4 g + r holds output
// column 16 g + 4 i + r, so lane group g accumulates columns 16 g .. 16 g + 15
__device__ __forceinline__ int uperm64(int p) { return 16 * ((p >> 2) & 3) + 4 * (p >> 4) + (p & 3); }
// element offset of (row, 8-element chunk lc) in a [rows][64] LDS-DMA image (rm_glds_frag's swizzle)
__device__ __forceinline__ int uimg(int row, int lc) { return row * kBK + ((lc ^ ((row >> 1) & 7)) << 3); }
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

__global__ __launch_bounds__(256, 1) void conv1x1_dual_kernel(const DualArgs s) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem_raw);  // kUKC sub-images [64 ci (permuted)][64 co]
  bf16_t* ring = Ws + kUKC * kUPanel;                 // kUNS stages of kUStage
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int grp = xcd * s.per_xcd + slot;
  const int M = s.M;
  const int mt = (M + kUR - 1) / kUR;
  const int ntile = grp < mt ? (mt - grp + s.mg - 1) / s.mg : 0;

  // ---- weight panel -> LDS once: W[co][ci] k-major, written transposed and row-permuted ---------------
  {
    constexpr int kPer = kUCo * kUCi / 8 / 256;  // 16-byte chunks per thread (8)
    ushort8_t v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      const int k = c / (kUCi / 8), nc = (c % (kUCi / 8)) * 8;  // columns nc .. nc + 7 of co-row k
      v[u] = *reinterpret_cast<const ushort8_t*>(s.w + (int64_t)k * kUCi + nc);
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = tid + u * 256;
      const int k = c / (kUCi / 8), nc = (c % (kUCi / 8)) * 8;
      bf16_t* sub = Ws + (k >> 6) * kUPanel;
      const int kk = k & 63;
#pragma unroll
      for (int e = 0; e < 8; ++e) sub[uimg(uperm64(nc + e), kk >> 3) + (kk & 7)] = v[u][e];
    }
  }

  // ---- ring: tile t -> stage t % kUNS; slot i of a sub-image covers rows 32 i .. 32 i + 31 --------------
  const __amdgpu_buffer_rsrc_t rdy = make_srd(s.dy, (uint32_t)((int64_t)M * kUCo * 2));
  const __amdgpu_buffer_rsrc_t rx = make_srd(s.x, (uint32_t)((int64_t)M * kUCi * 2));
  uint32_t vdy[kUSlots], vx[kUSlots];
  int vr[kUSlots];
#pragma unroll
  for (int i = 0; i < kUSlots; ++i) {
    const int c = tid + i * 256, r = c >> 3;
    vr[i] = r;
    vdy[i] = (uint32_t)((r * kUCo + rm_glds_kc(c)) * 2);
    vx[i] = (uint32_t)((r * kUCi + rm_glds_kc(c)) * 2);
  }
  const uint32_t ring0 = lds_addr(ring) + (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int t) {
    const int64_t row0 = (int64_t)(grp + t * s.mg) * kUR;  // past the end: every slot OOB (zero-filled)
    const uint32_t st = ring0 + (uint32_t)((t % kUNS) * kUStage * 2);
    uint32_t o[kUSlots];
#pragma unroll
    for (int kc = 0; kc < kUKC; ++kc) {
#pragma unroll
      for (int i = 0; i < kUSlots; ++i) o[i] = row0 + vr[i] < M ? vdy[i] : kOOB;
      const uint32_t soff = row0 < M ? (uint32_t)((row0 * kUCo + kc * kBK) * 2) : 0u;
      bglds<kUSlots, 256 * 16>(o, rdy, (uint32_t)__builtin_amdgcn_readfirstlane(soff), st + (uint32_t)(kc * kUSub * 2));
    }
#pragma unroll
    for (int i = 0; i < kUSlots; ++i) o[i] = row0 + vr[i] < M ? vx[i] : kOOB;
    const uint32_t soff = row0 < M ? (uint32_t)(row0 * kUCi * 2) : 0u;
    bglds<kUSlots, 256 * 16>(o, rx, (uint32_t)__builtin_amdgcn_readfirstlane(soff), st + (uint32_t)(kUKC * kUSub * 2));
  };

  // the panel's plain loads and LDS writes complete before the ring starts counting
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  issue(0);
  issue(1);

  const __amdgpu_buffer_rsrc_t rc = make_srd(s.dx, (uint32_t)((int64_t)M * kUCi * 2));
  accv_t aw[4][4];  // dW rows co = 64 wave + 16 i + 4 g + r, columns ci = 16 j + lr
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) aw[i][j] = accv_t{};

  for (int t = 0; t < ntile; ++t) {
    // tile t's DMAs (issued two iterations back) are done once only the younger ones are outstanding, in
    // issue order L0 L1 | L2 S0 | L3 S1 | ...: the stores of tiles t-2 and t-1 and the loads of tile t+1
    if (t == 0) vm_wait<kULoads>();
    else if (t == 1) vm_wait<kULoads + kUStores>();
    else vm_wait<kULoads + 2 * kUStores>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR: stage (t-1) % kUNS is refilled below
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + 2);
    const bf16_t* Ds = ring + (t % kUNS) * kUStage;  // dY sub-images
    const bf16_t* Xs = Ds + kUKC * kUSub;            // X sub-image

    // ---- data gradient: rows 16 wave + lr, all 64 input channels --------------------------------------
    accv_t ad[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ad[i] = accv_t{};
#pragma unroll
    for (int kc = 0; kc < kUKC; ++kc) {
#pragma unroll
      for (int kk = 0; kk < kBK / 32; ++kk) {
        bf16x8_t wf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) wf[i] = rm_glds_frag(Ws + kc * kUPanel, 16 * i, kk);
        const bf16x8_t yf = rm_glds_frag(Ds + kc * kUSub, 16 * wave, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i) ad[i] = mfma(wf[i], yf, ad[i]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // ---- weight gradient: co rows of this wave's dY sub-image, all 64 ci; K = the tile's 64 rows --------
#pragma unroll
    for (int kk = 0; kk < kUR / 32; ++kk) {
      bf16x8_t af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = urm_tr_frag(Ds + wave * kUSub, 16 * i, kk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = urm_tr_frag(Xs, 16 * j, kk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) aw[i][j] = mfma(af[i], bf[j], aw[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    // ---- dX store: lane (lr, g) holds row 16 wave + lr, channels 16 g .. 16 g + 15 ------------------------
    {
      const int64_t gm = (int64_t)(grp + t * s.mg) * kUR + 16 * wave + lr;
      const bool ok = gm < M;
      uint32_t wv[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wv[2 * i] = (uint32_t)f32_to_bf16(ad[i][0]) | ((uint32_t)f32_to_bf16(ad[i][1]) << 16);
        wv[2 * i + 1] = (uint32_t)f32_to_bf16(ad[i][2]) | ((uint32_t)f32_to_bf16(ad[i][3]) << 16);
      }
      const uint32_t off = ok ? (uint32_t)((gm * kUCi + 16 * g) * 2) : kOOB;
      const i32x4_t lo{(int)wv[0], (int)wv[1], (int)wv[2], (int)wv[3]};
      const i32x4_t hi{(int)wv[4], (int)wv[5], (int)wv[6], (int)wv[7]};
      __builtin_amdgcn_raw_buffer_store_b128(lo, rc, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(hi, rc, ok ? off + 16 : kOOB, 0, 0);
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the block's LDS is released
  // ---- this block's dW partial: [co][ci] fp32 (blocks without tiles write zeros) --------------------------
  float* P = s.part + (int64_t)blockIdx.x * kUCo * kUCi;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) P[(64 * wave + 16 * i + 4 * g + r) * kUCi + 16 * j + lr] = aw[i][j][r];
}

}  // namespace

int conv1x1_dual_blocks(int64_t M, int Cin, int Cout) {
  if (Cin != kUCi || Cout != kUCo || M <= 0) return 0;
  if (M * kUCo * 2 >= (int64_t)kOOB) return 0;
  const int64_t mt = (M + kUR - 1) / kUR;
  if (mt < 256 * 4) return 0;  // a few tiles per block at least, or the ring has nothing to overlap
  return 256;
}

bool launch_conv1x1_dual(const void* dy, const void* x, const void* w, void* dx, float* part, int64_t M, int Cin,
                         int Cout, hipStream_t stream) {
  const int grid = conv1x1_dual_blocks(M, Cin, Cout);
  if (!grid) return false;
  DualArgs a{(const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)dx, part, (int)M, grid, grid / 8};
  hipLaunchKernelGGL(conv1x1_dual_kernel, dim3(grid), dim3(256), kULds, stream, a);
  return true;
}

}  // namespace dla
