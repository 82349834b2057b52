// The ResNet stem convolution (7x7, stride 2, pad 3, Cin = 3 -> Cout = 64, NHWC bf16) as MFMA
// implicit GEMMs: forward with the fused BatchNorm-statistics epilogue, and the weight gradient.
//
// Three input channels give no 16-byte (tap, channel-block) vectors, so the image is first folded
// space-to-depth: 2x2 pixel blocks become one pixel of 12 channels (ph, pw, c), padded to 16:
//   xs[n][bh][bw][(ph * 2 + pw) * 3 + c] = x[n][2 bh + ph][2 bw + pw][c]          (224^2 x 3 -> 112^2 x 16)
// and the stride-2 7x7 conv becomes a stride-1 4x4 conv over xs with offset -2: input row
// ih = 2 oh - 3 + kh = 2 (oh - 2 + th) + ph  <=>  kh = 2 th + ph - 1 (th, tw in [0, 4); kh = -1 or 7
// are zero weights). GEMM K = 16 taps x 16 channels = 256 (1.7x the true 147 MACs per output) in four
// 64-deep k-steps; k-step s is exactly filter row th = s, so every 16-byte chunk is one aligned
// half-pixel at a per-slot column offset tw and a per-step row offset: the same LDS-DMA main loop as
// the 1x1 / 3x3 kernels. Stock PyTorch runs this conv through MIOpen (an NCHW<->NHWC pass, the conv,
// and a separate BN-statistics pass over its 411 MB output).
//
//   fold     xs = space_to_depth(x)                       one streaming pass (77 MB in, 103 MB out)
//   forward  Y[p, co] = sum_k A[p, k] W'[co, k]          M = N*OH*OW, N = Cout, K = 256
//   wgrad    dW'[co, k] = sum_p dY[p, co] A[p, k]         split over p, fp32 slabs + splitk_reduce
// W'[co][(th * 4 + tw) * 16 + (ph * 2 + pw) * 3 + c] = W[co][c][2 th + ph - 1][2 tw + pw - 1]
// (ops/conv.py stem_pack_weight / stem_unpack_grad).
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

#include <algorithm>

namespace dla {

using namespace mm;

constexpr int kStemK = 256;  // GEMM K: 4 x 4 taps x 16 folded channels
constexpr int kStemC = 16;   // folded channels (12 used)

struct StemGeom {
  int N, BH, BW;  // folded image (= output image: OH = BH, OW = BW)
  FastDiv fW, fH;
};

// ---- space-to-depth fold: one thread per folded pixel, two 16-byte stores -------------------------
__global__ __launch_bounds__(256) void stem_fold_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xs,
                                                        int N, int H, int W, int BH, int BW) {
  const int64_t total = (int64_t)N * BH * BW;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int bw = (int)(t % BW);
    const int64_t q = t / BW;
    const int bh = (int)(q % BH);
    const int n = (int)(q / BH);
    ushort8_t o0 = zero8(), o1 = zero8();
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      const int ih = 2 * bh + ph;
#pragma unroll
      for (int pw = 0; pw < 2; ++pw) {
        const int iw = 2 * bw + pw;
        if (ih < H && iw < W) {
          const bf16_t* s = x + (((int64_t)n * H + ih) * W + iw) * 3;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int ch = (ph * 2 + pw) * 3 + c;
            if (ch < 8) o0[ch] = s[c];
            else o1[ch - 8] = s[c];
          }
        }
      }
    }
    ushort8_t* d = reinterpret_cast<ushort8_t*>(xs + t * kStemC);
    d[0] = o0;
    d[1] = o1;
  }
}

// A operand of the forward: row = output pixel p = (n, oh, ow), k = (th, tw, ch). Slot c of a
// k-step holds logical chunk kc: tw = kc >> 4, channel half kc & 8; the k-step index is th.
template <int W, int NT = kThreads>
struct StemRowLoader {
  static constexpr bool kKMajor = false;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* xs;
  StemGeom g;
  int n[CH], oh[CH], ow[CH];  // n = -1 past the end
  const bf16_t* sp[CH];       // source at th = 0 for the slot's (tw, half)
  uint32_t smask[CH];         // bit th: folded row oh - 2 + th and column inside the image
  __device__ void init(int64_t row0, int64_t P) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3;
      const int64_t p = row0 + r;
      if (p < P) {
        const uint32_t q = fdiv((uint32_t)p, g.fW);
        ow[i] = (int)p - (int)q * g.BW;
        const uint32_t nn = fdiv(q, g.fH);
        oh[i] = (int)q - (int)nn * g.BH;
        n[i] = (int)nn;
      } else {
        n[i] = -1;
        oh[i] = ow[i] = 0;
      }
    }
  }
  __device__ __forceinline__ uint32_t mask_of(int i, int kc) const {
    const int iw = ow[i] - 2 + (kc >> 4);
    if (n[i] < 0 || (unsigned)iw >= (unsigned)g.BW) return 0u;
    uint32_t m = 0;
#pragma unroll
    for (int th = 0; th < 4; ++th) m |= ((unsigned)(oh[i] - 2 + th) < (unsigned)g.BH) ? (1u << th) : 0u;
    return m;
  }
  __device__ __forceinline__ const bf16_t* base_of(int i, int kc) const {
    // may point before the tensor (oh - 2 < 0): only dereferenced at rows the mask admits
    const int64_t pix = ((int64_t)(n[i] < 0 ? 0 : n[i]) * g.BH + (oh[i] - 2)) * g.BW + (ow[i] - 2 + (kc >> 4));
    return xs + pix * kStemC + (kc & 8);
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = rm_glds_kc(threadIdx.x + i * NT);
      smask[i] = mask_of(i, kc);
      sp[i] = base_of(i, kc);
    }
  }
  __device__ const void* src(int i, int k0) const {
    const int th = k0 >> 6;  // uniform
    return ((smask[i] >> th) & 1u) ? (const void*)(sp[i] + (int64_t)th * g.BW * kStemC) : zero_src();
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int kc = ((threadIdx.x + i * NT) & 7) * 8, th = k0 >> 6;
    if (!((mask_of(i, kc) >> th) & 1u)) return zero8();
    return *reinterpret_cast<const ushort8_t*>(base_of(i, kc) + (int64_t)th * g.BW * kStemC);
  }
};

// B operand of the weight gradient (k-major [P][256] = the same im2col values; rows = pixels, a fixed
// column (tap, half) per slot).
template <int W, bool kGlds, int NT = kThreads>
struct StemKLoader {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* xs;
  StemGeom g;
  int kend;
  int dh[CH], dw[CH], half[CH];  // per slot: tap offsets (th - 2, tw - 2) and channel half
  __device__ void init(int col0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT;
      const int k = col0 + (kGlds ? km_glds_col<W>(c) : (c % TileGeom<W>::KPR) * 8);
      const int tap = k >> 4;
      dh[i] = (tap >> 2) - 2;
      dw[i] = (tap & 3) - 2;
      half[i] = k & 8;
    }
  }
  __device__ void prep() {}
  __device__ __forceinline__ const bf16_t* at(int i, int p) const {
    const uint32_t q = fdiv((uint32_t)p, g.fW);
    const int ow = p - (int)q * g.BW;
    const uint32_t nn = fdiv(q, g.fH);
    const int oh = (int)q - (int)nn * g.BH;
    const int ih = oh + dh[i], iw = ow + dw[i];
    if ((unsigned)ih >= (unsigned)g.BH || (unsigned)iw >= (unsigned)g.BW) return nullptr;
    return xs + (((int64_t)nn * g.BH + ih) * g.BW + iw) * kStemC + half[i];
  }
  __device__ const void* src(int i, int k0) const {
    const int p = k0 + (threadIdx.x + i * NT) / TileGeom<W>::KPR;
    const bf16_t* a = p < kend ? at(i, p) : nullptr;
    return a ? (const void*)a : zero_src();
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int p = k0 + (threadIdx.x + i * NT) / TileGeom<W>::KPR;
    const bf16_t* a = p < kend ? at(i, p) : nullptr;
    return a ? *reinterpret_cast<const ushort8_t*>(a) : zero8();
  }
};

template <int BM, int BN, bool kStats, int PIPE>
__global__ __launch_bounds__(kThreads, 2) void stem_fwd_kernel(const bf16_t* __restrict__ xs,
                                                               const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                               StemGeom g, int Cout, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int64_t P = (int64_t)g.N * g.BH * g.BW;
  const int nbn = (Cout + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  StemRowLoader<BM> la{xs, g};
  la.init(row0, P);
  const RowLoader<BN> lb{w, kStemK, (int64_t)col0, Cout, kStemK};
  ColStats<BM, BN> st;
  st.zero();
  Acc<BM, BN> acc;
  acc.zero();
  run_mainloop<PIPE>(la, lb, 0, kStemK, acc, smem_raw);
  epilogue_bf16<BM, BN, kStats>(acc, y, Cout, P, Cout, row0, col0, st, nullptr, 0, smem_raw);
  if constexpr (kStats) stats_flush<BM, BN>(st, stats + (int64_t)bm * Cout * 2, Cout, col0, smem_raw);
}

template <int BM, int BN, int PIPE>
__global__ __launch_bounds__(kThreads, 2) void stem_wgrad_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ xs, StemGeom g, int Cout,
                                                                 float* __restrict__ part, int k_per_split,
                                                                 int ntiles, int remap) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int P = g.N * g.BH * g.BW;
  const int nbn = (kStemK + BN - 1) / BN;
  const int lin = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;  // see gemm_tn_kernel
  const int tile = lin % ntiles, split = lin / ntiles;
  const int bm = tile / nbn, bn = tile % nbn;
  const int kbeg = split * k_per_split;
  const int kend = min(P, kbeg + k_per_split);
  const int m0 = bm * BM, n0 = bn * BN;
  const KLoader<BM> la{dy, Cout, m0, Cout, kend};
  StemKLoader<BN, PIPE != 0> lb{xs, g, kend};
  lb.init(n0);
  Acc<BM, BN> acc;
  acc.zero();
  run_mainloop<PIPE>(la, lb, kbeg, kend, acc, smem_raw);
  epilogue_f32<BM, BN>(acc, part + (int64_t)split * Cout * kStemK, Cout, kStemK, m0, n0);
}

static StemGeom make_stem_geom(int N, int H, int W) {
  StemGeom g;
  g.N = N;
  g.BH = (H + 1) / 2;  // = OH of the 7x7 / s2 / p3 conv
  g.BW = (W + 1) / 2;
  g.fW = make_fastdiv((uint32_t)g.BW);
  g.fH = make_fastdiv((uint32_t)g.BH);
  return g;
}

int stem_stats_rows(int64_t P) { return (int)((P + 127) / 128); }

void launch_stem_fold(const void* x, void* xs, int N, int H, int W, hipStream_t stream) {
  const StemGeom g = make_stem_geom(N, H, W);
  const int64_t total = (int64_t)N * g.BH * g.BW;
  const int nb = (int)std::min<int64_t>((total + 255) / 256, 256 * 64);
  if (nb > 0)
    hipLaunchKernelGGL(stem_fold_kernel, dim3(nb), dim3(256), 0, stream, (const bf16_t*)x, (bf16_t*)xs, N, H, W, g.BH,
                       g.BW);
}

void launch_stem_fwd(const void* xs, const void* wpk, void* y, int N, int H, int W, int Cout, float* stats,
                     hipStream_t stream) {
  const StemGeom g = make_stem_geom(N, H, W);
  const int64_t P = (int64_t)N * g.BH * g.BW;
  const int tiles = (int)((P + 127) / 128) * ((Cout + 63) / 64);
  const int pipe = mfma_pipeline() >= 0 ? mfma_pipeline() : 2;
#define DLA_STEM(S_, P_)                                                                                         \
  hipLaunchKernelGGL((stem_fwd_kernel<128, 64, S_, P_>), dim3(tiles), dim3(kThreads),                           \
                     std::max(run_mainloop_lds_bytes<P_, 128, 64, StemRowLoader<128>, RowLoader<64>>(),          \
                              epilogue_lds_bytes<128, 64, S_>()),                                                \
                     stream, (const bf16_t*)xs, (const bf16_t*)wpk, (bf16_t*)y, g, Cout, stats)
  if (pipe == 0) {
    if (stats) DLA_STEM(true, 0); else DLA_STEM(false, 0);
  } else {
    if (stats) DLA_STEM(true, 2); else DLA_STEM(false, 2);
  }
#undef DLA_STEM
}

int stem_wgrad_splits(int N, int H, int W, int Cout) {
  const StemGeom g = make_stem_geom(N, H, W);
  const int P = N * g.BH * g.BW;
  const int tiles = ((Cout + 63) / 64) * (kStemK / 128);
  const int splits = std::max(1, splitk_target_blocks() / tiles);
  return std::max(1, std::min(splits, P / (16 * kBK)));
}

void launch_stem_wgrad(const void* dy, const void* xs, float* partial, int splits, void* dwpk, int out_dtype, int N,
                       int H, int W, int Cout, hipStream_t stream) {
  const StemGeom g = make_stem_geom(N, H, W);
  const int P = N * g.BH * g.BW;
  int kps = (P + splits - 1) / splits;
  kps = (kps + kBK - 1) / kBK * kBK;
  const int tiles = ((Cout + 63) / 64) * (kStemK / 128);
  const int pipe = mfma_pipeline_for(kps);
#define DLA_STEM_WG(P_)                                                                                          \
  hipLaunchKernelGGL((stem_wgrad_kernel<64, 128, P_>), dim3(tiles * splits), dim3(kThreads),                  \
                     (run_mainloop_lds_bytes<P_, 64, 128, KLoader<64>, StemKLoader<128, P_ != 0>>()), stream,    \
                     (const bf16_t*)dy, (const bf16_t*)xs, g, Cout, partial, kps, tiles, (int)splitk_xcd_remap())
  if (pipe == 0) DLA_STEM_WG(0); else DLA_STEM_WG(2);
#undef DLA_STEM_WG
  launch_splitk_reduce(partial, splits, (int64_t)Cout * kStemK, dwpk, out_dtype, 1.f, false, stream);
}

}  // namespace dla
