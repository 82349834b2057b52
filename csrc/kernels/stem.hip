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

// ---- fused backward: BN(+ReLU)+max-pool backward apply as the weight gradient's dY operand -------------------
// The stem conv output's gradient dY is consumed by nothing but this weight gradient (the stem input is the data
// batch), so instead of the quad apply pass writing dY (2 GB at batch 1280) and this GEMM reading it back, each
// k-step computes its dY tile from what the apply would read: the conv output x, the pooled gradient and its
// argmax window positions, and the finalized BN coefficients (bn_pool_quad_apply_kernel's arithmetic and bf16
// rounding). The GEMM's K (pixels) runs in quad order -- k = 4 q + 2 dh + dw for the 2x2 quad q of conv-output
// pixels -- which the sum over pixels does not care about: a 64-pixel k-step is 16 quads, and one thread turns the
// 4 pooled windows covering its quad (for 2 channels) into the 4 pixels' dY values, as the quad apply does.
//   A (dY)  [64 px][64 co] k-major: all threads, quad tid / 32, channels (tid % 32) * 2
//   B (im2col of xs) [64 px][256 k] k-major: all threads, 4 chunks each = 64 contiguous bytes of xs
// Register-staged: the next k-step's raw loads (buffer loads; out of range reads zeros) are in flight during this
// k-step's MFMAs; the dY arithmetic runs between the MFMAs and the LDS stores. One fp32 [64][256] partial per
// split, summed by splitk_reduce. Kernel revisions and counters: profiles/r5/g11/README.md.
namespace {

constexpr int kSBCo = 64;  // stem output channels served

struct StemBnArgs {
  const bf16_t* dyp;
  const uint8_t* pos;
  const bf16_t* x;
  const float* ws;
  const bf16_t* xs;
  float* part;
  int N, H, W, OH, OW;  // conv output (= folded image) and pooled sizes
  FastDiv fQW, fQH;     // quads per row (W / 2), quad rows (H / 2)
  int64_t Q;            // quads
  int ksteps, kps;      // 16-quad k-steps in all, per split
};

struct KMajorTag {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = kThreads;
};

__device__ __forceinline__ void quad_decode(const StemBnArgs& s, int64_t q, int& n, int& j, int& i) {
  const uint32_t r = fdiv((uint32_t)q, s.fQW);
  i = (int)q - (int)r * (s.W >> 1);
  const uint32_t nn = fdiv(r, s.fQH);
  j = (int)r - (int)nn * (s.H >> 1);
  n = (int)nn;
}

}  // namespace

// 8 waves per block (2 blocks per CU: four waves per SIMD to cover the loads' latency; the 4-wave form held
// 226 VGPRs, two waves per SIMD, and waited on memory: profiles/r5/g11): wave (wr, wc) owns output channels
// 32 wr .. + 31 x GEMM columns 64 wc .. + 63 (TM = 2, TN = 4). A role: quad tid / 32, channels (tid % 32) * 2;
// B role: k-row tid / 8 (that quad's pixel (tid / 8) % 4), filter row th = (tid % 8) / 2, half-run hs = tid % 2:
// taps 2 hs, 2 hs + 1 x 2 channel halves = 64 contiguous bytes of xs.
constexpr int kSBNT = 512;
__global__ __launch_bounds__(kSBNT, 4) void stem_wgrad_bn_kernel(const StemBnArgs s) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem_raw);  // [64 px][64 co] k-major image
  bf16_t* Bs = As + kBK * kSBCo;                      // [64 px][256 k] k-major image
  constexpr int TM = 2, TN = 4, WM = 32, WN = 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 2, wc = wid & 3;
  const int split = blockIdx.x;
  const int kb = split * s.kps, ke = min(s.ksteps, kb + s.kps);
  const int C = kSBCo;

  // A role: quad qi of the k-step, channels c0, c0 + 1
  const int qi = tid >> 5, c0 = (tid & 31) * 2;
  float mean[2], sc[2], sh[2], k1[2], m1[2], k2[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    mean[e] = s.ws[c0 + e];
    sc[e] = s.ws[2 * C + c0 + e];
    sh[e] = s.ws[3 * C + c0 + e];
    k1[e] = s.ws[4 * C + c0 + e];
    m1[e] = s.ws[5 * C + c0 + e];
    k2[e] = s.ws[6 * C + c0 + e];
  }
  // B role. ds_write_b128 banks are (a / 4) mod 32 in groups of 8 lanes = one k-row: the filter rows'
  // 64-column offsets vanish mod 128 B, so register u holds chunk hs * 4 + ((u + th) & 3) -- 8 distinct
  // 16-byte slots per group
  const int br = tid >> 3, bsub = br & 3, bth = (tid & 7) >> 1, bhs = tid & 1;
  const int bdh = bth - 2 + (bsub >> 1), bdw = (bsub & 1) - 2 + 2 * bhs;

  // buffer loads: an out-of-range operand (past the batch, conv padding) reads as zeros via an offset past
  // num_records (kOOB) instead of an exec-masked branch; every tensor is < 2 GiB (stem_wgrad_bn_eligible)
  const __amdgpu_buffer_rsrc_t srx = make_srd(s.x, (uint32_t)(s.Q * 4 * C * 2));
  const __amdgpu_buffer_rsrc_t srs = make_srd(s.xs, (uint32_t)((int64_t)s.N * s.H * s.W * kStemC * 2));
  const int64_t npool = (int64_t)s.N * s.OH * s.OW * C;  // pooled elements, < 2^29
  const __amdgpu_buffer_rsrc_t srp = make_srd(s.pos, (uint32_t)npool);
  const __amdgpu_buffer_rsrc_t srd = make_srd(s.dyp, (uint32_t)(npool * 2));
  uint32_t rx[4], rd[4], rp[4];
  ushort8_t rb[4];
  bool qok = false;
  auto issue = [&](int t) {
    const int64_t q = (int64_t)t * 16 + qi;
    qok = q < s.Q;
    int n, j, i;
    quad_decode(s, qok ? q : 0, n, j, i);
    const uint32_t px = (uint32_t)(((n * s.H + 2 * j) * s.W + 2 * i) * C + c0) * 2u;  // bytes, < 2^31
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t o = px + (uint32_t)(((p >> 1) * s.W + (p & 1)) * C * 2);
      rx[p] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(srx, qok ? o : kOOB, 0, 0);
    }
    // pooled windows (j + a, i + b) cover the quad (pad 1); OH = H / 2, so only the far ones can fall outside.
    // A window outside (or past the batch) reads position 0 and gradient 0 (kOOB): it adds nothing
    const bool aok = j + 1 < s.OH, bok = i + 1 < s.OW;
    const uint32_t pw0 = (uint32_t)(((n * s.OH + j) * s.OW + i) * C + c0);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const bool in = qok && (!(w >> 1) || aok) && (!(w & 1) || bok);
      const uint32_t o = pw0 + (uint32_t)(((w >> 1) * s.OW + (w & 1)) * C);
      rp[w] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(srp, in ? o : kOOB, 0, 0);
      rd[w] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(srd, in ? 2 * o : kOOB, 0, 0);
    }
    const int ih = 2 * j + bdh, iw0 = 2 * i + bdw;
    const bool rok = qok && (unsigned)ih < (unsigned)s.H;
    const int pix0 = (n * s.H + ih) * s.W + iw0;  // may be negative: only used where the tests pass
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = (u + bth) & 3;  // chunk v of the 64-byte run: tap 2 hs + v / 2, channel half v % 2
      const bool ok = rok && (unsigned)(iw0 + (v >> 1)) < (unsigned)s.W;
      const uint32_t o = (uint32_t)(pix0 * kStemC + v * 8) * 2u;
      rb[u] = __builtin_bit_cast(ushort8_t, __builtin_amdgcn_raw_buffer_load_b128(srs, ok ? o : kOOB, 0, 0));
    }
  };
  accv_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = accv_t{};
  if (kb < ke) issue(kb);
  for (int t = kb; t < ke; ++t) {
    // dY of the quad's 4 pixels: g = sum of the pooled gradients whose argmax is the pixel, the forward's ReLU
    // recomputed from x, then bn_pool_quad_apply_kernel's k1 (g - m1 - (x - mean) k2)
    uint32_t av[4];
    {
      float g[4][2];
#pragma unroll
      for (int p = 0; p < 4; ++p) g[p][0] = g[p][1] = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int dh = 0; dh < 2; ++dh)
#pragma unroll
          for (int dw = 0; dw < 2; ++dw) {
            const int ky = dh - 2 * (w >> 1) + 1, kx = dw - 2 * (w & 1) + 1;
            if (ky < 0 || kx < 0) continue;  // compile-time after unrolling
            const uint32_t tap = (uint32_t)(ky * 3 + kx);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const uint32_t byte = (rp[w] >> (8 * e)) & 0xffu;
              g[dh * 2 + dw][e] += byte == tap ? bf16_to_f32((bf16_t)(rd[w] >> (16 * e))) : 0.f;
            }
          }
      // past the last quad: x and the window gradients read as zeros, and a zero k1 zeroes dY (branch-free)
      float kq[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) kq[e] = qok ? k1[e] : 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float xv = bf16_to_f32((bf16_t)(rx[p] >> (16 * e)));
          const float gg = fmaf(xv, sc[e], sh[e]) > 0.f ? g[p][e] : 0.f;
          packed |= (uint32_t)f32_to_bf16(kq[e] * (gg - m1[e] - (xv - mean[e]) * k2[e])) << (16 * e);
        }
        av[p] = packed;
      }
    }
    __syncthreads();  // the previous k-step's fragment reads are done
#pragma unroll
    for (int p = 0; p < 4; ++p)
      *reinterpret_cast<uint32_t*>(As + tr_off<kSBCo>(qi * 4 + p, c0 & ~3) + (c0 & 3)) = av[p];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = (u + bth) & 3;
      *reinterpret_cast<ushort8_t*>(Bs + tr_off<kStemK>(br, bth * 64 + (bhs * 4 + v) * 8)) = rb[u];
    }
    __syncthreads();
    if (t + 1 < ke) issue(t + 1);  // in flight during the MFMAs
#pragma unroll
    for (int kk = 0; kk < kBK / kKS; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tile_frag<kSBCo, KMajorTag>(As, wr * WM + i * kMS, kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tile_frag<kStemK, KMajorTag>(Bs, wc * WN + j * kMS, kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    }
  }
  // fp32 partial [64 co][256 k] of this split: lane (row acc_row, column acc_col) of each 16 x 16 fragment
  float* out = s.part + (int64_t)split * kSBCo * kStemK;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(wr * WM + i * kMS + acc_row(lane, r)) * kStemK + wc * WN + j * kMS + acc_col(lane)] = acc[i][j][r];
}

bool stem_wgrad_bn_eligible(int N, int H, int W, int Cout, int OH, int OW) {
  const int BH = (H + 1) / 2, BW = (W + 1) / 2;  // conv output = folded image
  return Cout == kSBCo && BH % 2 == 0 && BW % 2 == 0 && OH == BH / 2 && OW == BW / 2 &&
         (int64_t)N * BH * BW < (1 << 24);
}

int stem_wgrad_bn_splits(int N, int H, int W) {
  const int64_t Q = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) / 4;
  const int ks = (int)((Q + 15) / 16);
  return std::max(1, std::min(2 * 256, ks));  // two 8-wave blocks per CU
}

void launch_stem_wgrad_bn(const void* dy_pool, const uint8_t* pos, const void* x, const float* ws, const void* xs,
                          float* partial, int splits, void* dwpk, int out_dtype, int N, int H, int W, int OH, int OW,
                          hipStream_t stream) {
  StemBnArgs s{};
  s.dyp = (const bf16_t*)dy_pool;
  s.pos = pos;
  s.x = (const bf16_t*)x;
  s.ws = ws;
  s.xs = (const bf16_t*)xs;
  s.part = partial;
  s.N = N;
  s.H = (H + 1) / 2;
  s.W = (W + 1) / 2;
  s.OH = OH;
  s.OW = OW;
  s.fQW = make_fastdiv((uint32_t)(s.W / 2));
  s.fQH = make_fastdiv((uint32_t)(s.H / 2));
  s.Q = (int64_t)N * (s.H / 2) * (s.W / 2);
  s.ksteps = (int)((s.Q + 15) / 16);
  s.kps = (s.ksteps + splits - 1) / splits;
  const size_t lds = (size_t)(kBK * kSBCo + kBK * kStemK) * sizeof(bf16_t);
  hipLaunchKernelGGL(stem_wgrad_bn_kernel, dim3(splits), dim3(kSBNT), lds, stream, s);
  launch_splitk_reduce(partial, splits, (int64_t)kSBCo * kStemK, dwpk, out_dtype, 1.f, false, stream);
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

int stem_stats_rows(int64_t P, int Cout) {
  const int rows = stem_stream_rows(P, Cout);  // the persistent streaming kernel (gemm_stream.hip kStem)
  return rows > 0 ? rows : (int)((P + 127) / 128);
}

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
  if (stats && stem_stream_rows(P, Cout) > 0 && launch_stem_stream(xs, wpk, y, N, g.BH, g.BW, stats, stream)) return;
  const int tiles = (int)((P + 127) / 128) * ((Cout + 63) / 64);
  const int pipe = mfma_pipeline() >= 0 ? mfma_pipeline() : 2;
#define DLA_STEM(S_, P_)                                                                                         \
  hipLaunchKernelGGL((stem_fwd_kernel<128, 64, S_, P_>), dim3(tiles), dim3(kThreads),                           \
                     std::max(run_mainloop_lds_bytes<P_, 128, 64, StemRowLoader<128>, RowLoader<64>>(),          \
                              epilogue_lds_bytes<128, 64, S_>()),                                                \
                     stream, (const bf16_t*)xs, (const bf16_t*)wpk, (bf16_t*)y, g, Cout, stats)
  switch (pipe) {  // A/B: 0 register staging, 2 / 3 LDS-DMA stages, 4 / 5 the v2 LDS-DMA schedule
    case 0: if (stats) DLA_STEM(true, 0); else DLA_STEM(false, 0); break;
    case 3: if (stats) DLA_STEM(true, 3); else DLA_STEM(false, 3); break;
    case 4: if (stats) DLA_STEM(true, 4); else DLA_STEM(false, 4); break;
    case 5: if (stats) DLA_STEM(true, 5); else DLA_STEM(false, 5); break;
    default: if (stats) DLA_STEM(true, 2); else DLA_STEM(false, 2); break;
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
