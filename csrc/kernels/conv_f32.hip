// fp32 convolutions on the fp32-input matrix cores (v_mfma_f32_16x16x4_f32): the reference-precision path.
//
// The reference trains GoogLeNet in fp32 (/root/reference/src/network.py:33-54, main.py:36,74-91); on MI355X an fp32
// convolution has one exact matrix-core form, v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate, the vector-fp32
// rate: 64 FLOP / clock / SIMD, MI355X_MICROARCH.md), and no reduced-precision (xf32) one. Every convolution of the
// fp32 step is an implicit GEMM on it:
//   forward   Y[m, co]           = sum_(tap, ci) X[pixel(m) + tap, ci] W[co, tap, ci]          (A = im2col X, B = W)
//   dgrad     dX = the forward of dY with the flipped, transposed weights (stride 1 only; the host transforms W)
//   wgrad     dW[co, (tap, ci)]  = sum_m dY[m, co] X[pixel(m) + tap, ci]                      (split over m)
// NHWC (channels_last) activations -- the input may be a channel slice of a wider tensor (pixel stride ldx) --, OHWI weights ([co][R][S][ci], k = tap * C + ci), C % 4 == 0 (16-byte chunks never
// cross a tap), any R x S, padding, stride (the 7x7/s2 stem after a zero channel pads its 3 input channels to 4).
//
// Kernel: 256 threads = 2 x 2 waves, BM x BN tile (128 x 128 or 64 x 64), 32-deep k-steps staged through LDS with
// the next step's global loads in flight in registers during the current step's MFMAs. The 32 k of a step are
// permuted so that the 16x16x4 MFMA slice s of lane group g (lanes 16 g .. 16 g + 15) uses physical k = 8 g + s:
// a lane's 8 k values of one fragment row are then contiguous, read as two ds_read_b128 from a row-major
// [rows][32] image (16-byte chunks XOR-swizzled by row bits 1 and 3: every ds_read_b128 lane group hits 16
// distinct bank slots), or as 8 ds_read_b32 from a k-major [32][cols] image (the weight-gradient operands, whose
// reduction runs over pixels; columns XOR 16 for k rows 8..15 and 24..31 so the two 32-lane halves of a read
// use disjoint banks). The same permutation on both operands leaves every dot product exact; only the fp32
// summation order differs from cuDNN/MIOpen's, as between any two fp32 GEMMs.
#include <algorithm>

#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

namespace dla {

using mm::FastDiv;
using mm::fdiv;
using mm::make_fastdiv;

namespace {

constexpr int kFK = 32;   // k per step
constexpr int kFT = 256;  // threads per block
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4_t zero4() { return f32x4_t{0.f, 0.f, 0.f, 0.f}; }

// row-major image [rows][32 floats]: element offset of (row, 16-byte chunk)
__device__ __forceinline__ int rm_off(int row, int chunk) {
  return row * kFK + ((chunk ^ (((row >> 1) & 1) | (((row >> 3) & 1) << 2))) << 2);
}
// k-major image [32][W floats]: element offset of (k, col)
template <int W>
__device__ __forceinline__ int km_off(int k, int col) {
  return k * W + (col ^ (((k >> 3) & 1) << 4));
}

// Stride-s implicit-GEMM geometry over an NHWC fp32 input
struct ConvGeomF {
  const float* x;
  int64_t ldp;  // elements between consecutive pixels of x (C, or the width of the tensor x is a channel slice of)
  int N, H, W, C;
  int R, S, pad, stride;
  int OH, OW;
  int K;       // R * S * C
  int64_t M;   // N * OH * OW
  FastDiv fC, fS, fOW, fOH;
};

__device__ __forceinline__ void pixel_of(const ConvGeomF& g, int64_t m, int& n, int& oh, int& ow) {
  const uint32_t q = fdiv((uint32_t)m, g.fOW);
  ow = (int)m - (int)q * g.OW;
  n = (int)fdiv(q, g.fOH);
  oh = (int)q - n * g.OH;
}

// ---- row-major operand loaders (rows = GEMM rows / columns, k contiguous) -----------------------
// A of the forward / data gradient: output pixels x (tap, ci). Thread chunk column cc = tid % 8 (the same k for
// all of its rows, so the tap decomposition is once per step), rows tid / 8 + 32 i.
template <int BM>
struct AConv {
  static constexpr bool kKMajor = false;
  static constexpr int CH = BM / 32;
  ConvGeomF g;
  int64_t base[CH];
  int ih0[CH], iw0[CH];
  __device__ void prep(int64_t row0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int64_t m = row0 + (threadIdx.x >> 3) + 32 * i;
      int n = 0, oh = 0, ow = 0;
      if (m < g.M) pixel_of(g, m, n, oh, ow);
      ih0[i] = m < g.M ? oh * g.stride - g.pad : -(1 << 28);  // out-of-range rows fail the bounds test
      iw0[i] = ow * g.stride - g.pad;
      base[i] = (((int64_t)n * g.H) * g.W) * g.ldp;
    }
  }
  __device__ void load(int k0, f32x4_t (&r)[CH]) const {
    const int k = k0 + 4 * (threadIdx.x & 7);
    if (k >= g.K) {
#pragma unroll
      for (int i = 0; i < CH; ++i) r[i] = zero4();
      return;
    }
    const int tap = (int)fdiv((uint32_t)k, g.fC), c = k - tap * g.C;
    const int rr = (int)fdiv((uint32_t)tap, g.fS), ss = tap - rr * g.S;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int ih = ih0[i] + rr, iw = iw0[i] + ss;
      const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      r[i] = ok ? *reinterpret_cast<const f32x4_t*>(g.x + base[i] + ((int64_t)ih * g.W + iw) * g.ldp + c) : zero4();
    }
  }
  __device__ void store(float* s, const f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i)
      *reinterpret_cast<f32x4_t*>(s + rm_off((threadIdx.x >> 3) + 32 * i, threadIdx.x & 7)) = r[i];
  }
};

// B of the forward / data gradient: a row-major matrix [rows][ld] (the OHWI weights)
template <int BN>
struct BRows {
  static constexpr bool kKMajor = false;
  static constexpr int CH = BN / 32;
  const float* p;
  int64_t ld;
  int rows, K;
  int64_t row0;
  __device__ void prep(int64_t r0) { row0 = r0; }
  __device__ void load(int k0, f32x4_t (&r)[CH]) const {
    const int k = k0 + 4 * (threadIdx.x & 7);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int64_t row = row0 + (threadIdx.x >> 3) + 32 * i;
      r[i] = (row < rows && k < K) ? *reinterpret_cast<const f32x4_t*>(p + row * ld + k) : zero4();
    }
  }
  __device__ void store(float* s, const f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i)
      *reinterpret_cast<f32x4_t*>(s + rm_off((threadIdx.x >> 3) + 32 * i, threadIdx.x & 7)) = r[i];
  }
};

// ---- k-major operand loaders (the weight gradient: reduction over pixels) -----------------------
// Thread layout: chunk column cc = tid % (W / 4) (4 consecutive columns), k rows tid / (W / 4) + (256 / (W / 4)) i.
// dY [M][ld] rows = pixels, columns = output channels
template <int W>
struct KRows {
  static constexpr bool kKMajor = true;
  static constexpr int CPR = W / 4, RPI = kFT / CPR, CH = kFK / RPI;
  const float* p;
  int64_t ld;
  int64_t kend;  // pixel bound (exclusive)
  int cols;
  int col;  // this thread's first column, or cols when out of range
  __device__ void prep(int col0) {
    const int c = col0 + 4 * ((int)threadIdx.x % CPR);
    col = c < cols ? c : cols;
  }
  __device__ void load(int64_t k0, f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int64_t k = k0 + (int)threadIdx.x / CPR + RPI * i;
      r[i] = (k < kend && col < cols) ? *reinterpret_cast<const f32x4_t*>(p + k * ld + col) : zero4();
    }
  }
  __device__ void store(float* s, const f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i)
      *reinterpret_cast<f32x4_t*>(s + km_off<W>((int)threadIdx.x / CPR + RPI * i, 4 * ((int)threadIdx.x % CPR))) = r[i];
  }
};

// im2col(X) seen k-major: rows = pixels m, columns = (tap, ci); a thread's 4 columns share one tap
template <int W>
struct KConv {
  static constexpr bool kKMajor = true;
  static constexpr int CPR = W / 4, RPI = kFT / CPR, CH = kFK / RPI;
  ConvGeomF g;
  int64_t kend;
  int dh, dw, c;
  bool colok;
  __device__ void prep(int col0) {
    const int k = col0 + 4 * ((int)threadIdx.x % CPR);
    colok = k < g.K;
    const int tap = colok ? (int)fdiv((uint32_t)k, g.fC) : 0;
    c = k - tap * g.C;
    const int rr = (int)fdiv((uint32_t)tap, g.fS);
    dh = rr - g.pad;
    dw = tap - rr * g.S - g.pad;
  }
  __device__ void load(int64_t k0, f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int64_t m = k0 + (int)threadIdx.x / CPR + RPI * i;
      int n = 0, oh = 0, ow = 0;
      const bool mok = colok && m < kend;
      if (mok) pixel_of(g, m, n, oh, ow);
      const int ih = oh * g.stride + dh, iw = ow * g.stride + dw;
      const bool ok = mok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      r[i] = ok ? *reinterpret_cast<const f32x4_t*>(g.x + (((int64_t)n * g.H + ih) * g.W + iw) * g.ldp + c) : zero4();
    }
  }
  __device__ void store(float* s, const f32x4_t (&r)[CH]) const {
#pragma unroll
    for (int i = 0; i < CH; ++i)
      *reinterpret_cast<f32x4_t*>(s + km_off<W>((int)threadIdx.x / CPR + RPI * i, 4 * ((int)threadIdx.x % CPR))) = r[i];
  }
};

// ---- the GEMM ------------------------------------------------------------------------------------
// 8 k values of fragment row `row` for lane group g = lane / 16 (physical k 8 g .. 8 g + 7)
template <int W, bool KM>
__device__ __forceinline__ void frag8(const float* s, int row, int g, float (&f)[8]) {
  if constexpr (KM) {
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = s[km_off<W>(8 * g + q, row)];
  } else {
    const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(s + rm_off(row, 2 * g));
    const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(s + rm_off(row, 2 * g + 1));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[q] = lo[q];
      f[4 + q] = hi[q];
    }
  }
}

// C[Mo, No] (+)= A[Mo, K] B[No, K]^T over k in this block's split; splits > 1 write fp32 slabs P[split][Mo][No].
// NB = 2: double-buffered LDS (the next step's tile is stored into the other buffer after this step's MFMAs; one
// barrier per step); NB = 1: single buffer, two barriers per step.
template <int BM, int BN, int NB, class LA, class LB>
__global__ __launch_bounds__(kFT, 2) void gemm_f32_kernel(LA la, LB lb, float* __restrict__ C, int64_t ldc, int Mo,
                                                        int No, int64_t kbeg0, int64_t K, int64_t kps, int ntiles,
                                                        int accumulate) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) float As[NB][BM * kFK];
  __shared__ __attribute__((aligned(16))) float Bs[NB][BN * kFK];
  const int nbn = (No + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % ntiles, split = lin / ntiles;
  const int bm = tile / nbn, bn = tile % nbn;
  const int row0 = bm * BM, col0 = bn * BN;
  const int64_t kbeg = kbeg0 + (int64_t)split * kps;
  const int64_t kend = std::min(K, kbeg + kps);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int g = lane >> 4, p = lane & 15;
  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  la.prep(row0);
  lb.prep(col0);
  const int nk = kend > kbeg ? (int)((kend - kbeg + kFK - 1) / kFK) : 0;
  f32x4_t ra[LA::CH], rb[LB::CH];
  if (nk > 0) {
    la.load(kbeg, ra);
    lb.load(kbeg, rb);
    la.store(As[0], ra);
    lb.store(Bs[0], rb);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = NB == 2 ? (t & 1) : 0;
    if (t + 1 < nk) {  // next step's loads in flight during this step's MFMAs
      la.load(kbeg + (int64_t)(t + 1) * kFK, ra);
      lb.load(kbeg + (int64_t)(t + 1) * kFK, rb);
    }
    float af[TM][8], bfr[TN][8];
#pragma unroll
    for (int i = 0; i < TM; ++i) frag8<BM, LA::kKMajor>(As[cur], wr * WM + 16 * i + p, g, af[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) frag8<BN, LB::kKMajor>(Bs[cur], wc * WN + 16 * j + p, g, bfr[j]);
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    if constexpr (NB == 2) {
      if (t + 1 < nk) {
        la.store(As[cur ^ 1], ra);
        lb.store(Bs[cur ^ 1], rb);
      }
      __syncthreads();
    } else {
      __syncthreads();
      if (t + 1 < nk) {
        la.store(As[0], ra);
        lb.store(Bs[0], rb);
        __syncthreads();
      }
    }
  }
  // lane holds rows 4 g + r, column p of each 16x16 fragment
  float* out = C + (int64_t)split * ((ldc == 0) ? (int64_t)Mo * No : 0);
  const int64_t ld = ldc == 0 ? No : ldc;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = col0 + wc * WN + 16 * j + p;
      if (col >= No) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wr * WM + 16 * i + 4 * g + r;
        if (row < Mo) {
          float* o = out + (int64_t)row * ld + col;
          *o = accumulate ? *o + acc[i][j][r] : acc[i][j][r];
        }
      }
    }
}

ConvGeomF make_geom(const float* x, int64_t ldp, int N, int H, int W, int C, int R, int S, int pad, int stride) {
  ConvGeomF g;
  g.x = x;
  g.ldp = ldp;
  g.N = N, g.H = H, g.W = W, g.C = C, g.R = R, g.S = S, g.pad = pad, g.stride = stride;
  g.OH = (H + 2 * pad - R) / stride + 1;
  g.OW = (W + 2 * pad - S) / stride + 1;
  g.K = R * S * C;
  g.M = (int64_t)N * g.OH * g.OW;
  g.fC = make_fastdiv((uint32_t)C);
  g.fS = make_fastdiv((uint32_t)S);
  g.fOW = make_fastdiv((uint32_t)g.OW);
  g.fOH = make_fastdiv((uint32_t)g.OH);
  return g;
}

// Tile width over a GEMM dimension of extent n: the least padded work ceil(n / b) * b over b in {128, 64, 32}, ties
// to the wider tile (more reuse per fragment); the fp32 MFMA loop is far from LDS-bound, so narrow tiles cost
// little while a 128-wide tile over 192 or 96 columns wastes a quarter of its MFMAs.
int pick_f32_width(int64_t n, int widest = 128) {
  int best = widest;
  int64_t bw = (n + widest - 1) / widest * widest;
  for (int b = widest / 2; b >= 32; b /= 2) {
    const int64_t w = (n + b - 1) / b * b;
    if (w < bw) best = b, bw = w;
  }
  return best;
}

// rows: 128 when that still gives >= 2 blocks per CU (512 tiles), else 64
int pick_f32_rows(int64_t M, int N, int bn) {
  const int64_t t128 = ((M + 127) / 128) * ((N + bn - 1) / bn);
  return t128 >= 512 ? 128 : 64;
}

static int g_f32_nb = 1;  // LDS buffers of the fp32 GEMM (set_conv_f32_buffers; profiles/r6/g06: 1 is faster)

template <int BM, int BN>
void launch_fwd_t(const ConvGeomF& g, const float* w, float* y, int Cout, int accumulate, hipStream_t st) {
  AConv<BM> la{g};
  BRows<BN> lb{w, (int64_t)g.K, Cout, g.K, 0};
  const int tiles = (int)(((g.M + BM - 1) / BM) * ((Cout + BN - 1) / BN));
  if (g_f32_nb == 2)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, 2, AConv<BM>, BRows<BN>>), dim3(tiles), dim3(kFT), 0, st, la, lb, y,
                       (int64_t)Cout, (int)g.M, Cout, (int64_t)0, (int64_t)g.K, (int64_t)g.K, tiles, accumulate);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, 1, AConv<BM>, BRows<BN>>), dim3(tiles), dim3(kFT), 0, st, la, lb, y,
                       (int64_t)Cout, (int)g.M, Cout, (int64_t)0, (int64_t)g.K, (int64_t)g.K, tiles, accumulate);
}

template <int BM, int BN>
void launch_wgrad_t(const ConvGeomF& g, const float* dy, int Cout, float* P, int splits, int64_t kps, hipStream_t st) {
  KRows<BM> la{dy, (int64_t)Cout, g.M, Cout, 0};
  KConv<BN> lb{g, g.M, 0, 0, 0, false};
  const int tiles = ((Cout + BM - 1) / BM) * ((g.K + BN - 1) / BN);
  if (g_f32_nb == 2)
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, 2, KRows<BM>, KConv<BN>>), dim3(tiles * splits), dim3(kFT), 0, st, la,
                       lb, P, (int64_t)0, Cout, g.K, (int64_t)0, g.M, kps, tiles, 0);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, 1, KRows<BM>, KConv<BN>>), dim3(tiles * splits), dim3(kFT), 0, st, la,
                       lb, P, (int64_t)0, Cout, g.K, (int64_t)0, g.M, kps, tiles, 0);
}

}  // namespace

void set_conv_f32_buffers(int nb) { g_f32_nb = nb == 2 ? 2 : 1; }

bool conv_f32_supported(int C, int Cout, int64_t M, int K) {
  return C % 4 == 0 && Cout % 4 == 0 && M > 0 && M < (int64_t(1) << 24) && K < (1 << 24);
}

void launch_conv_f32_fwd(const float* x, int64_t ldx, int N, int H, int W, int C, const float* w, int Cout, int R,
                         int S, int pad, int stride, float* y, bool accumulate, hipStream_t st) {
  const ConvGeomF g = make_geom(x, ldx, N, H, W, C, R, S, pad, stride);
  const int bn = pick_f32_width(Cout), bm = pick_f32_rows(g.M, Cout, bn);
  const int acc = accumulate ? 1 : 0;
#define DLA_F32F(BM_, BN_) \
  if (bm == BM_ && bn == BN_) return launch_fwd_t<BM_, BN_>(g, w, y, Cout, acc, st);
  DLA_F32F(128, 128) DLA_F32F(128, 64) DLA_F32F(128, 32) DLA_F32F(64, 128) DLA_F32F(64, 64) DLA_F32F(64, 32)
#undef DLA_F32F
}

static void wgrad_tile(int Cout, int K, int& bm, int& bn) {
  bm = pick_f32_width(Cout);
  bn = pick_f32_width(K);
  if (bm == 32) bm = 64;  // the k-major loaders take >= 64 columns on the A side (32 couts: 50 % of a 64 tile)
}

int conv_f32_wgrad_splits(int64_t M, int Cout, int K) {
  int bm, bn;
  wgrad_tile(Cout, K, bm, bn);
  const int tiles = ((Cout + bm - 1) / bm) * ((K + bn - 1) / bn);
  // ~512 blocks, >= 8 k-steps (256 pixels) per split
  const int64_t by_k = std::max<int64_t>(1, M / (8 * kFK));
  return (int)std::max<int64_t>(1, std::min<int64_t>(by_k, std::max(1, 512 / tiles)));
}

void launch_conv_f32_wgrad(const float* dy, const float* x, int64_t ldx, int N, int H, int W, int C, int Cout, int R,
                           int S, int pad, int stride, float* partial, int splits, float* dw, bool accumulate,
                           hipStream_t st) {
  const ConvGeomF g = make_geom(x, ldx, N, H, W, C, R, S, pad, stride);
  int64_t kps = (g.M + splits - 1) / splits;
  kps = (kps + kFK - 1) / kFK * kFK;
  splits = (int)((g.M + kps - 1) / kps);
  int bm, bn;
  wgrad_tile(Cout, g.K, bm, bn);
#define DLA_F32W(BM_, BN_) \
  if (bm == BM_ && bn == BN_) launch_wgrad_t<BM_, BN_>(g, dy, Cout, partial, splits, kps, st);
  DLA_F32W(128, 128) DLA_F32W(128, 64) DLA_F32W(128, 32) DLA_F32W(64, 128) DLA_F32W(64, 64) DLA_F32W(64, 32)
#undef DLA_F32W
  launch_splitk_reduce(partial, splits, (int64_t)Cout * g.K, dw, kF32, 1.f, accumulate, st);
}

}  // namespace dla
