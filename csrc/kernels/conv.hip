// Implicit-GEMM 3x3 convolutions, NHWC (channels_last) bf16, on the shared MFMA main loop.
//
// ResNet-50 spends ~45% of its FLOPs in 3x3 convolutions (the reference leaves them
// to cuDNN); stock PyTorch runs them through MIOpen, whose backward-weights path also launches
// zero-fill and cast kernels around every call. Here all three passes are GEMMs whose operand
// tiles are gathered straight from the activation tensors (no im2col buffer):
//
//   forward  Y[p, co]          = sum_{t, ci} X[src(p, t), ci] * W[co, t, ci]      M = P, N = Cout, K = 9*Cin
//   dgrad    dX[p, ci]         = sum_{t, co} dY[src'(p, t), co] * W[co, t, ci]    M = P, N = Cin,  K = 9*Cout
//   wgrad    dW[co, (t, ci)]   = sum_p dY[p, co] * X[src(p, t), ci]               split-K over P
//
// with p an output pixel (n, oh, ow), t = (kh, kw), src(p, t) = (n, oh*s - 1 + kh, ow*s - 1 + kw)
// and src'(p, t) = (n, oh + 1 - kh, ow + 1 - kw) (stride-1 transposed conv). Out-of-image taps load
// zeros (the padding). W is the channels_last weight [Cout][3][3][Cin] = [Cout][9*Cin], so forward
// reads it K-contiguous (row-major tile), dgrad reads it k-major per tap (transposed LDS reads),
// and wgrad writes exactly that layout. A 64-deep K step never straddles a tap (Cin, Cout % 64 == 0),
// so the tap of a k-step is a scalar and each thread's gather address is one add away.
// The forward epilogue can emit the BatchNorm statistics of Y (as the 1x1 GEMMs do).
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace dla {

using namespace mm;

struct ConvGeom {
  int N, H, W, Cin;  // input image (NHWC)
  int OH, OW, Cout;  // output image
  int stride;
  FastDiv fOW, fOH;  // divisors for output-pixel decode
};

// A operand of forward / dgrad: row = output pixel of this GEMM, K = (tap, channel) with the channel
// fastest. kFlip: dgrad (source = o + 1 - k), otherwise forward (source = o*s - 1 + k).
template <int W, bool kFlip, int NT = kThreads>
struct Im2colRowLoader {
  static constexpr bool kKMajor = false;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* x;
  int H, Wd, C;  // source image height, width, channels
  int stride;
  int32_t pbase[CH];  // n * H * Wd of each slot's pixel, -1 when the pixel is past the end
  int ih0[CH], iw0[CH];
  // LDS-DMA form: the slot's source address at tap (0, 0) and channel base 0, and a 9-bit mask of
  // the taps that fall inside the image (0 past the end): per k-step one wave-uniform offset
  // (tap shift + channel base) is added and the tap's bit selects it or the zero page.
  const bf16_t* sp[CH];
  uint32_t smask[CH];
  __device__ void init(const ConvGeom& g, int64_t row0, int64_t P, int oh_dim, int ow_dim, const FastDiv& fw,
                       const FastDiv& fh) {
    N_img = g.N;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3;
      const int64_t p = row0 + r;
      if (p < P) {
        const uint32_t q = fdiv((uint32_t)p, fw);
        const int ow = (int)p - (int)q * ow_dim;
        const uint32_t n = fdiv(q, fh);
        const int oh = (int)q - (int)n * oh_dim;
        pbase[i] = (int32_t)n * H * Wd;
        ih0[i] = kFlip ? oh + 1 : oh * stride - 1;
        iw0[i] = kFlip ? ow + 1 : ow * stride - 1;
      } else {
        pbase[i] = -1;
        ih0[i] = iw0[i] = 0;
      }
    }
    (void)g;
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = rm_glds_kc(threadIdx.x + i * NT);
      uint32_t m = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ih = kFlip ? ih0[i] - t / 3 : ih0[i] + t / 3;
        const int iw = kFlip ? iw0[i] - t % 3 : iw0[i] + t % 3;
        m |= ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)Wd) ? (1u << t) : 0u;
      }
      smask[i] = pbase[i] < 0 ? 0u : m;
      sp[i] = x + ((int64_t)(pbase[i] < 0 ? 0 : pbase[i]) + (int64_t)ih0[i] * Wd + iw0[i]) * C + kc;
    }
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int tap = k0 / C;  // uniform across the block
    const int ci = k0 - tap * C + (threadIdx.x & 7) * 8;
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int ih = kFlip ? ih0[i] - kh : ih0[i] + kh;
    const int iw = kFlip ? iw0[i] - kw : iw0[i] + kw;
    if (pbase[i] < 0 || tap >= 9 || (unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)Wd) return zero8();
    return *reinterpret_cast<const ushort8_t*>(x + ((int64_t)pbase[i] + ih * Wd + iw) * C + ci);
  }
  __device__ const void* src(int i, int k0) const {
    const int tap = k0 / C;  // uniform: scalar arithmetic
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int shift = kh * Wd + kw;
    const int64_t off = (int64_t)(kFlip ? -shift : shift) * C + (k0 - tap * C);
    return ((smask[i] >> tap) & 1u) ? (const void*)(sp[i] + off) : zero_src();
  }
  // v2 pipeline: the tap offset and tap bit of a k-step, once per k-step (src2 = add + select)
  int64_t koff = 0;
  uint32_t kbit = 0;
  __device__ void step(int k0) {
    const int tap = k0 / C;
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int shift = kh * Wd + kw;
    koff = (int64_t)(kFlip ? -shift : shift) * C + (k0 - tap * C);
    kbit = 1u << tap;
  }
  __device__ const void* src2(int i) const {
    const bf16_t* p = sp[i] + koff;
    return (smask[i] & kbit) ? (const void*)p : zero_src();
  }
  // buffer form (PIPE 6/7). The slot offset is taken at the tap with the smallest address (fwd:
  // tap (0,0) at (oh*s-1, ow*s-1); dgrad: tap (2,2) at (oh-1, ow-1)) so every tap adds a
  // non-negative scalar soffset; the descriptor base sits (W+1)*C elements before x so that
  // pixel (-1, -1) of image 0 still has a non-negative offset. Padding taps select kOOB.
  uint32_t bvo[CH];
  __amdgpu_buffer_rsrc_t bsrd;
  int N_img = 0;
  __device__ void bprep() {
    const int64_t bias = (int64_t)(Wd + 1) * C;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = rm_glds_kc(threadIdx.x + i * NT);
      const int ih = kFlip ? ih0[i] - 2 : ih0[i], iw = kFlip ? iw0[i] - 2 : iw0[i];
      bvo[i] = pbase[i] < 0 ? kOOB : (uint32_t)((bias + ((int64_t)pbase[i] + (int64_t)ih * Wd + iw) * C + kc) * 2);
    }
    bsrd = make_srd(x - bias, (uint32_t)((bias + (int64_t)N_img * H * Wd * C) * 2));
  }
  __device__ uint32_t bsoff(int k0) const {
    const int tap = k0 / C;
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int shift = kFlip ? (2 - kh) * Wd + (2 - kw) : kh * Wd + kw;
    return (uint32_t)(((int64_t)shift * C + (k0 - tap * C)) * 2);
  }
  __device__ bool bcheck(int) const { return true; }
  __device__ uint32_t bvoff_chk(int i, int) const { return (smask[i] & kbit) ? bvo[i] : kOOB; }
};

// B operand of dgrad: k = (tap, co) rows, n = ci columns, element W[co][tap][ci] (k-major per tap).
template <int W, int NT = kThreads>
struct WeightTapKLoader {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* w;
  int Cout, Cin, col0;
  const bf16_t* sp[CH];
  bool sok[CH];
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR, nc = (c % TileGeom<W>::KPR) * 8;
    const int tap = k0 / Cout;  // uniform
    const int co = k0 - tap * Cout + kr, ci = col0 + nc;
    if (tap >= 9 || ci >= Cin) return zero8();
    return *reinterpret_cast<const ushort8_t*>(w + ((int64_t)co * 9 + tap) * Cin + ci);
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
      const int ci = col0 + km_glds_col<W>(c);
      sok[i] = ci < Cin;
      sp[i] = w + (int64_t)kr * 9 * Cin + (sok[i] ? ci : 0);
    }
  }
  __device__ const void* src(int i, int k0) const {
    const int tap = k0 / Cout;
    const int64_t off = ((int64_t)(k0 - tap * Cout) * 9 + tap) * Cin;
    return sok[i] ? (const void*)(sp[i] + off) : zero_src();
  }
  int64_t koff = 0;
  __device__ void step(int k0) {
    const int tap = k0 / Cout;
    koff = ((int64_t)(k0 - tap * Cout) * 9 + tap) * Cin;
  }
  __device__ const void* src2(int i) const { return sok[i] ? (const void*)(sp[i] + koff) : zero_src(); }
  // buffer form (PIPE 6/7): element W[co][tap][ci] at ((co * 9 + tap) * Cin + ci) * 2 bytes
  uint32_t bvo[CH];
  __amdgpu_buffer_rsrc_t bsrd;
  __device__ void bprep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
      const int ci = col0 + km_glds_col<W>(c);
      bvo[i] = ci < Cin ? (uint32_t)(((int64_t)kr * 9 * Cin + ci) * 2) : kOOB;
    }
    bsrd = make_srd(w, (uint32_t)((int64_t)Cout * 9 * Cin * 2));
  }
  __device__ uint32_t bsoff(int k0) const {
    const int tap = k0 / Cout;
    return (uint32_t)((((int64_t)(k0 - tap * Cout) * 9 + tap) * Cin) * 2);
  }
  __device__ bool bcheck(int) const { return false; }
  __device__ uint32_t bvoff_chk(int i, int) const { return bvo[i]; }
};

// ---- any channel count (C % 8 == 0, e.g. GoogLeNet's 16/24/48/96/112/144/160-channel 3x3s) ----------
// A 64-deep k-step then spans several taps, so the tap of a 16-byte chunk (8 channels, never
// straddling a tap) is per lane: k = k0 + chunk k offset -> (tap, channel) by a FastDiv. Register
// staging (PIPE 0) and the global_load_lds pipeline (PIPE 2) use these loaders; same LDS images.
template <int W, bool kFlip, int NT = kThreads>
struct Im2colRowLoaderAnyC {
  static constexpr bool kKMajor = false;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* x;
  int H, Wd, C;
  int stride;
  int32_t pbase[CH];
  int ih0[CH], iw0[CH];
  const bf16_t* sp0[CH];  // source pixel of tap (0, 0), channel 0
  uint32_t smask[CH];
  FastDiv fC;
  __device__ void init(const ConvGeom& g, int64_t row0, int64_t P, int oh_dim, int ow_dim, const FastDiv& fw,
                       const FastDiv& fh) {
    fC = make_fastdiv((uint32_t)C);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3;
      const int64_t p = row0 + r;
      if (p < P) {
        const uint32_t q = fdiv((uint32_t)p, fw);
        const int ow = (int)p - (int)q * ow_dim;
        const uint32_t n = fdiv(q, fh);
        const int oh = (int)q - (int)n * oh_dim;
        pbase[i] = (int32_t)n * H * Wd;
        ih0[i] = kFlip ? oh + 1 : oh * stride - 1;
        iw0[i] = kFlip ? ow + 1 : ow * stride - 1;
      } else {
        pbase[i] = -1;
        ih0[i] = iw0[i] = 0;
      }
      uint32_t m = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ih = kFlip ? ih0[i] - t / 3 : ih0[i] + t / 3;
        const int iw = kFlip ? iw0[i] - t % 3 : iw0[i] + t % 3;
        m |= ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)Wd) ? (1u << t) : 0u;
      }
      smask[i] = pbase[i] < 0 ? 0u : m;
      sp0[i] = x + ((int64_t)(pbase[i] < 0 ? 0 : pbase[i]) + (int64_t)ih0[i] * Wd + iw0[i]) * C;
    }
    (void)g;
  }
  __device__ void prep() {}
  __device__ __forceinline__ const bf16_t* at(int i, int k, bool& ok) const {
    const int tap = (int)fdiv((uint32_t)k, fC);
    const int ci = k - tap * C;
    const int kh = (tap * 11) >> 5, kw = tap - 3 * kh;  // tap / 3 for tap <= 8
    const int shift = kh * Wd + kw;
    ok = tap < 9 && ((smask[i] >> tap) & 1u);
    return sp0[i] + (int64_t)(kFlip ? -shift : shift) * C + ci;
  }
  __device__ ushort8_t load(int i, int k0) const {
    bool ok;
    const bf16_t* p = at(i, k0 + (threadIdx.x & 7) * 8, ok);
    return ok ? *reinterpret_cast<const ushort8_t*>(p) : zero8();
  }
  __device__ const void* src(int i, int k0) const {
    bool ok;
    const bf16_t* p = at(i, k0 + rm_glds_kc(threadIdx.x + i * NT), ok);
    return ok ? (const void*)p : zero_src();
  }
};

// dgrad B operand for any Cout % 8: k-row (tap, co) per lane.
template <int W, int NT = kThreads>
struct WeightTapKLoaderAnyC {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* w;
  int Cout, Cin, col0;
  const bf16_t* sp[CH];  // column base (ci) of the slot
  bool sok[CH];
  FastDiv fCo;
  __device__ __forceinline__ const bf16_t* at(int k, int ci, bool& ok) const {
    const int tap = (int)fdiv((uint32_t)k, fCo);
    const int co = k - tap * Cout;
    ok = tap < 9 && ci < Cin;
    return w + ((int64_t)co * 9 + tap) * Cin + ci;
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR, nc = (c % TileGeom<W>::KPR) * 8;
    bool ok;
    const bf16_t* p = at(k0 + kr, col0 + nc, ok);
    return ok ? *reinterpret_cast<const ushort8_t*>(p) : zero8();
  }
  __device__ void prep() {
    fCo = make_fastdiv((uint32_t)Cout);
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT;
      const int ci = col0 + km_glds_col<W>(c);
      sok[i] = ci < Cin;
    }
  }
  __device__ const void* src(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
    bool ok;
    const bf16_t* p = at(k0 + kr, col0 + km_glds_col<W>(c), ok);
    return ok ? (const void*)p : zero_src();
  }
};

// ---- stride-2 data gradient ----------------------------------------------------------------------
// dX of a 3x3 / stride-2 / pad-1 conv with even H, W splits into the 4 parity classes (ph, pw) of the
// input pixel (ih, iw) = (2a + ph, 2b + pw): only taps with ih + 1 - kh even reach it, at
// oh = a + dh. Row taps: ph = 0 -> {kh 1, dh 0}; ph = 1 -> {kh 0, dh +1}, {kh 2, dh 0} (columns alike),
// so class (ph, pw) is a dense implicit GEMM over the OH x OW class image with (1 + ph)(1 + pw) taps
// (9 in total = exactly the forward's FLOPs, no zero-inserted work). Tap index t of the class:
// th = t / (1 + pw), tw = t % (1 + pw).
struct S2Class {
  int ph, pw;
  __device__ __forceinline__ int ntaps() const { return (1 + ph) * (1 + pw); }
  __device__ __forceinline__ void tap(int t, int& kh, int& kw, int& dh, int& dw) const {
    const int th = t / (1 + pw), tw = t - th * (1 + pw);
    kh = ph == 0 ? 1 : (th == 0 ? 0 : 2);
    dh = (ph == 1 && th == 0) ? 1 : 0;
    kw = pw == 0 ? 1 : (tw == 0 ? 0 : 2);
    dw = (pw == 1 && tw == 0) ? 1 : 0;
  }
};

// A operand: row = class pixel (n, a, b), k = (tap t, output channel co), element dY[n][a+dh][b+dw][co].
template <int W, int NT = kThreads>
struct S2DgradRowLoader {
  static constexpr bool kKMajor = false;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* dy;
  int OH, OW, C;  // dY image (the class image has the same size), C = Cout
  S2Class cls;
  int64_t pix[CH];  // n*OH*OW + a*OW + b of the slot's class pixel, -1 past the end
  int ra[CH], rb[CH];
  const bf16_t* sp[CH];
  uint32_t smask[CH];
  __device__ void init(int64_t row0, int64_t P, const FastDiv& fw, const FastDiv& fh) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3;
      const int64_t p = row0 + r;
      if (p < P) {
        const uint32_t q = fdiv((uint32_t)p, fw);
        rb[i] = (int)p - (int)q * OW;
        const uint32_t n = fdiv(q, fh);
        ra[i] = (int)q - (int)n * OH;
        pix[i] = p;
      } else {
        pix[i] = -1;
        ra[i] = rb[i] = 0;
      }
    }
  }
  __device__ bool tap_ok(int i, int t) const {
    int kh, kw, dh, dw;
    cls.tap(t, kh, kw, dh, dw);
    return pix[i] >= 0 && ra[i] + dh < OH && rb[i] + dw < OW;
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int kc = rm_glds_kc(threadIdx.x + i * NT);
      uint32_t m = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) m |= (t < cls.ntaps() && tap_ok(i, t)) ? (1u << t) : 0u;
      smask[i] = m;
      sp[i] = dy + (pix[i] < 0 ? 0 : pix[i]) * C + kc;
    }
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int t = k0 / C;
    if (t >= cls.ntaps() || !tap_ok(i, t)) return zero8();
    int kh, kw, dh, dw;
    cls.tap(t, kh, kw, dh, dw);
    return *reinterpret_cast<const ushort8_t*>(dy + (pix[i] + dh * OW + dw) * C + (k0 - t * C) +
                                               (threadIdx.x & 7) * 8);
  }
  __device__ const void* src(int i, int k0) const {
    const int t = k0 / C;  // uniform
    int kh, kw, dh, dw;
    cls.tap(t, kh, kw, dh, dw);
    const int64_t off = (int64_t)(dh * OW + dw) * C + (k0 - t * C);
    return ((smask[i] >> t) & 1u) ? (const void*)(sp[i] + off) : zero_src();
  }
};

// B operand: k = (tap t, co) rows, n = ci columns, element W[co][kh(t)][kw(t)][ci].
template <int W, int NT = kThreads>
struct S2WeightKLoader {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* w;
  int Cout, Cin, col0;
  S2Class cls;
  const bf16_t* sp[CH];
  bool sok[CH];
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR, nc = (c % TileGeom<W>::KPR) * 8;
    const int t = k0 / Cout;
    int kh, kw, dh, dw;
    cls.tap(t, kh, kw, dh, dw);
    const int co = k0 - t * Cout + kr, ci = col0 + nc;
    if (t >= cls.ntaps() || ci >= Cin) return zero8();
    return *reinterpret_cast<const ushort8_t*>(w + ((int64_t)co * 9 + kh * 3 + kw) * Cin + ci);
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
      const int ci = col0 + km_glds_col<W>(c);
      sok[i] = ci < Cin;
      sp[i] = w + (int64_t)kr * 9 * Cin + (sok[i] ? ci : 0);
    }
  }
  __device__ const void* src(int i, int k0) const {
    const int t = k0 / Cout;
    int kh, kw, dh, dw;
    cls.tap(t, kh, kw, dh, dw);
    const int64_t off = ((int64_t)(k0 - t * Cout) * 9 + kh * 3 + kw) * Cin;
    return sok[i] ? (const void*)(sp[i] + off) : zero_src();
  }
};

// class row (n, a, b) -> dX row (n, 2a + ph, 2b + pw)
struct S2RowMap {
  int OH, OW, ph, pw;
  FastDiv fw, fh;
  __device__ __forceinline__ int64_t operator()(int64_t p) const {
    const uint32_t q = fdiv((uint32_t)p, fw);
    const int b = (int)p - (int)q * OW;
    const uint32_t n = fdiv(q, fh);
    const int a = (int)q - (int)n * OH;
    return ((int64_t)n * (2 * OH) + 2 * a + ph) * (2 * OW) + 2 * b + pw;
  }
};

// B operand of wgrad: k = output pixel rows, n = (tap, ci) columns, element X[src(p, tap)][ci].
template <int W, bool kGlds, int NT = kThreads>
struct Im2colKLoader {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* x;
  ConvGeom g;
  int kend;
  int kh[CH], kw[CH], ci[CH];  // per slot: fixed column -> (tap, channel); kh = -100 if out of range
  __device__ void prep() {}
  __device__ void init(int col0) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT;
      const int nc = col0 + (kGlds ? km_glds_col<W>(c) : (c % TileGeom<W>::KPR) * 8);
      const int tap = nc / g.Cin;
      ci[i] = nc - tap * g.Cin;
      kh[i] = tap < 9 ? tap / 3 : -100;
      kw[i] = tap - 3 * (tap / 3);
    }
  }
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
    const int p = k0 + kr;
    if (p >= kend || kh[i] < 0) return zero8();
    const uint32_t q = fdiv((uint32_t)p, g.fOW);
    const int ow = p - (int)q * g.OW;
    const uint32_t n = fdiv(q, g.fOH);
    const int oh = (int)q - (int)n * g.OH;
    const int ih = oh * g.stride - 1 + kh[i], iw = ow * g.stride - 1 + kw[i];
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return zero8();
    return *reinterpret_cast<const ushort8_t*>(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.Cin + ci[i]);
  }
  __device__ const void* src(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
    const int p = k0 + kr;
    if (p >= kend || kh[i] < 0) return zero_src();
    const uint32_t q = fdiv((uint32_t)p, g.fOW);
    const int ow = p - (int)q * g.OW;
    const uint32_t n = fdiv(q, g.fOH);
    const int oh = (int)q - (int)n * g.OH;
    const int ih = oh * g.stride - 1 + kh[i], iw = ow * g.stride - 1 + kw[i];
    if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return zero_src();
    return x + (((int64_t)n * g.H + ih) * g.W + iw) * g.Cin + ci[i];
  }
};

// ---------------------------------------------------------------------------------------------
template <int BM, int BN, bool kStats, int PIPE, int NT>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void conv3x3_fwd_kernel(const bf16_t* __restrict__ x,
                                                                  const bf16_t* __restrict__ w,
                                                                  bf16_t* __restrict__ y, ConvGeom g,
                                                                  float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int64_t P = (int64_t)g.N * g.OH * g.OW;
  const int nbn = (g.Cout + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  const int K = 9 * g.Cin;
  // PIPE >= 100: any Cin % 8 (per-lane tap decode), main loop PIPE % 100
  constexpr bool kAny = PIPE >= 100;
  const RowLoader<BN, NT> lb{w, K, (int64_t)col0, g.Cout, K};
  std::conditional_t<kAny, Im2colRowLoaderAnyC<BM, false, NT>, Im2colRowLoader<BM, false, NT>> la{
      x, g.H, g.W, g.Cin, g.stride};
  la.init(g, row0, P, g.OH, g.OW, g.fOW, g.fOH);
  ColStats<BM, BN, NT> st;
  st.zero();
  Acc<BM, BN, NT> acc;
  acc.zero();
  run_mainloop<PIPE % 100>(la, lb, 0, K, acc, smem_raw);
  epilogue_bf16<BM, BN, kStats, false, NT>(acc, y, g.Cout, P, g.Cout, row0, col0, st, nullptr, 0, smem_raw);
  if constexpr (kStats) stats_flush<BM, BN, NT>(st, stats + (int64_t)bm * g.Cout * 2, g.Cout, col0, smem_raw);
}

// stride-1 dgrad: dX (the GEMM's M = input pixels, N = Cin), A = dY gathered with flipped taps
template <int BM, int BN, int PIPE, int NT>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void conv3x3_dgrad_kernel(const bf16_t* __restrict__ dy,
                                                                    const bf16_t* __restrict__ w,
                                                                    bf16_t* __restrict__ dx, ConvGeom g,
                                                                    const bf16_t* __restrict__ addend, BnBwdEpi bnb) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int64_t P = (int64_t)g.N * g.H * g.W;  // stride 1: OH = H, OW = W
  const int nbn = (g.Cin + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  const int K = 9 * g.Cout;
  constexpr bool kAny = PIPE >= 100;  // any Cout % 8: per-lane tap decode in both loaders
  std::conditional_t<kAny, WeightTapKLoaderAnyC<BN, NT>, WeightTapKLoader<BN, NT>> lb{w, g.Cout, g.Cin, col0};
  if constexpr (kAny) lb.prep();  // the divisor by Cout (the register main loop does not call prep)
  std::conditional_t<kAny, Im2colRowLoaderAnyC<BM, true, NT>, Im2colRowLoader<BM, true, NT>> la{dy, g.OH, g.OW,
                                                                                                 g.Cout, 1};
  la.init(g, row0, P, g.H, g.W, g.fOW, g.fOH);  // stride 1: the same divisors (OW == W, OH == H)
  ColStats<BM, BN, NT> st;
  Acc<BM, BN, NT> acc;
  acc.zero();
  run_mainloop<PIPE % 100>(la, lb, 0, K, acc, smem_raw);
  epilogue_bf16<BM, BN, false, true, NT>(acc, dx, g.Cin, P, g.Cin, row0, col0, st, addend, g.Cin, smem_raw, &bnb, bm);
}

// stride-2 dgrad: all 4 parity classes in one launch (heaviest class first: 4, 2, 2, 1 taps)
template <int BM, int BN, int PIPE, int NT = kThreads>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void conv3x3s2_dgrad_kernel(const bf16_t* __restrict__ dy,
                                                                                      const bf16_t* __restrict__ w,
                                                                                      bf16_t* __restrict__ dx,
                                                                                      ConvGeom g) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int64_t P = (int64_t)g.N * g.OH * g.OW;  // class image = dY image
  const int nbn = (g.Cin + BN - 1) / BN;
  const int per_class = (int)((P + BM - 1) / BM) * nbn;
  const int cls_slot = blockIdx.x / per_class;  // 0..3 -> class (1,1), (1,0), (0,1), (0,0)
  const S2Class cls{cls_slot < 2 ? 1 : 0, (cls_slot & 1) == 0 ? 1 : 0};
  const int tile = xcd_remap(blockIdx.x - cls_slot * per_class, per_class);
  const int bm = tile / nbn, bn = tile % nbn;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;
  const int K = cls.ntaps() * g.Cout;
  const S2WeightKLoader<BN, NT> lb{w, g.Cout, g.Cin, col0, cls};
  S2DgradRowLoader<BM, NT> la{dy, g.OH, g.OW, g.Cout, cls};
  la.init(row0, P, g.fOW, g.fOH);
  ColStats<BM, BN, NT> st;
  Acc<BM, BN, NT> acc;
  acc.zero();
  run_mainloop<PIPE>(la, lb, 0, K, acc, smem_raw);
  const S2RowMap rm{g.OH, g.OW, cls.ph, cls.pw, g.fOW, g.fOH};
  epilogue_bf16<BM, BN, false, false, NT, S2RowMap>(acc, dx, g.Cin, P, g.Cin, row0, col0, st, nullptr, 0,
                                                   smem_raw, nullptr, 0, rm);
}

// wgrad partial slabs P[split][Cout][9*Cin]
template <int BM, int BN, int PIPE, int NT = kThreads>
__global__ __launch_bounds__(NT, blocks_per_cu(BM, BN, NT)) void conv3x3_wgrad_kernel(const bf16_t* __restrict__ dy,
                                                                                    const bf16_t* __restrict__ x,
                                                                                    ConvGeom g, float* __restrict__ part,
                                                                                    int k_per_split, int ntiles,
                                                                                    int remap) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int P = g.N * g.OH * g.OW;
  const int Mo = g.Cout, No = 9 * g.Cin;
  const int nbn = (No + BN - 1) / BN;
  // tiles of one split (the 9 taps x Cin columns over the same pixels) on one XCD (gemm_tn_kernel)
  const int lin = remap ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tile = lin % ntiles, split = lin / ntiles;
  const int bm = tile / nbn, bn = tile % nbn;
  const int kbeg = split * k_per_split;
  const int kend = min(P, kbeg + k_per_split);
  const int m0 = bm * BM, n0 = bn * BN;
  const KLoader<BM, NT> la{dy, g.Cout, m0, Mo, kend};
  Im2colKLoader<BN, PIPE != 0, NT> lb{x, g, kend};
  lb.init(n0);
  Acc<BM, BN, NT> acc;
  acc.zero();
  run_mainloop<PIPE>(la, lb, kbeg, kend, acc, smem_raw);
  epilogue_f32<BM, BN, NT>(acc, part + (int64_t)split * Mo * No, Mo, No, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// Main loop of the 3x3 kernels when not forced (set_mfma_pipeline): per-layer A/B at ResNet-50
// bs512 (profiles/r2v): forward and data gradient fastest on the buffer-DMA loop (PIPE 6: 2.62 /
// 2.83 ms vs 2.69 / 2.95 on PIPE 2). The weight gradient ran on the v2 schedule (PIPE 4: 3.06 vs 3.20 then);
// after the round-5 swizzled operand images the 2-stage LDS-DMA loop is as fast or faster at every 3x3 weight
// gradient of the bs1280 step (profiles/r5/g50: stage 2 0.393 vs 0.428 ms stride 1, 0.441 vs 0.463 stride 2;
// 256x256 tiles equal or -3 %), so PIPE 2 is the weight-gradient default
static int conv_pipeline(int K, int deep) {
  const int forced = mfma_pipeline();
  if (forced >= 0) return forced;
  static const int env = [] {  // DLA_CONV_PIPE: one loop for all 3x3 passes (A/B runs)
    const char* e = std::getenv("DLA_CONV_PIPE");
    return e ? std::atoi(e) : -1;
  }();
  return K >= 256 ? (env >= 0 ? env : deep) : 0;
}

static ConvGeom make_geom(int N, int H, int W, int Cin, int Cout, int stride) {
  ConvGeom g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.Cin = Cin;
  g.Cout = Cout;
  g.stride = stride;
  g.OH = (H + 2 - 3) / stride + 1;
  g.OW = (W + 2 - 3) / stride + 1;
  g.fOW = make_fastdiv((uint32_t)g.OW);
  g.fOH = make_fastdiv((uint32_t)g.OH);
  return g;
}

template <int BM, int BN, bool S, int PIPE, int NT>
static void launch_fwd_p(const bf16_t* x, const bf16_t* w, bf16_t* y, const ConvGeom& g, float* stats,
                         hipStream_t stream) {
  const int64_t P = (int64_t)g.N * g.OH * g.OW;
  const int tiles = (int)((P + BM - 1) / BM) * ((g.Cout + BN - 1) / BN);
  const size_t lds =
      std::max(run_mainloop_lds_bytes<PIPE % 100, BM, BN, Im2colRowLoader<BM, false, NT>, RowLoader<BN, NT>>(),
               epilogue_lds_bytes<BM, BN, S, NT>());
  hipLaunchKernelGGL((conv3x3_fwd_kernel<BM, BN, S, PIPE, NT>), dim3(tiles), dim3(NT), lds, stream, x, w, y, g,
                     stats);
}
template <int BM, int BN, bool S, int NTW = kThreads>
static void launch_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, const ConvGeom& g, float* stats,
                       hipStream_t stream) {
  if constexpr (NTW == 512 && BM * BN > 256 * 128) {  // 256x256 / 512x128: 2 stages fill 128 / 160 KB of LDS
    if (mfma_pipeline() == 2) launch_fwd_p<BM, BN, S, 2, 512>(x, w, y, g, stats, stream);
    else launch_fwd_p<BM, BN, S, 6, 512>(x, w, y, g, stats, stream);
  } else if constexpr (NTW == 512) {  // 8-wave tile: 3-stage LDS-DMA pipeline, one block per CU
    if (mfma_pipeline() == 7) launch_fwd_p<BM, BN, S, 7, 512>(x, w, y, g, stats, stream);
    else launch_fwd_p<BM, BN, S, 3, 512>(x, w, y, g, stats, stream);
  } else if constexpr (BM * BN > 128 * 128) {  // 4 large waves, one block per CU
    if (mfma_pipeline() == 2) launch_fwd_p<BM, BN, S, 2, kThreads>(x, w, y, g, stats, stream);
    else launch_fwd_p<BM, BN, S, 3, kThreads>(x, w, y, g, stats, stream);
  } else if (g.Cin % 64 != 0) {  // a k-step spans taps: per-lane tap decode (register or LDS-DMA staging)
    if (mfma_pipeline_for(9 * g.Cin) == 0) launch_fwd_p<BM, BN, S, 100, kThreads>(x, w, y, g, stats, stream);
    else launch_fwd_p<BM, BN, S, 102, kThreads>(x, w, y, g, stats, stream);
  } else {
    switch (conv_pipeline(9 * g.Cin, 6)) {
      case 0: launch_fwd_p<BM, BN, S, 0, kThreads>(x, w, y, g, stats, stream); break;
      case 3: launch_fwd_p<BM, BN, S, 3, kThreads>(x, w, y, g, stats, stream); break;
      case 4: launch_fwd_p<BM, BN, S, 4, kThreads>(x, w, y, g, stats, stream); break;
      case 6: launch_fwd_p<BM, BN, S, 6, kThreads>(x, w, y, g, stats, stream); break;
      default: launch_fwd_p<BM, BN, S, 2, kThreads>(x, w, y, g, stats, stream); break;
    }
  }
}

// 512x128 tiles for the Cout = 128 passes (ResNet stage 2): 128 x 64 wave tiles read as few LDS fragment bytes
// per MFMA as the 256x256 tiles' 64 x 128 ones, which the 128x128 tile's 64 x 64 waves do not. At least 4 tiles
// per CU (one block per CU, so the last wave of tiles is a small fraction). Stage 2 at bs1280 (profiles/r5/g54):
// forward 0.359 -> 0.340 ms, data gradient 0.347 -> 0.341, stride-2 forward equal; step 82.54 -> 82.27 ms same
// box. DLA_TILE512=0: off (A/B)
static bool tile512_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("DLA_TILE512");
    return !(e && e[0] == '0');
  }();
  return v;
}

int pick_conv_tile(int64_t P, int N, int tile, int K, bool wide_ok) {
  if (tile == kTileAuto && wide_ok && tile256_enabled() && tile512_enabled() && N == 128 && K >= 1024 &&
      (P + 511) / 512 >= 1024)
    return kTile512x128;
  return pick_tile(P, N, tile, K, wide_ok);
}

int conv3x3_stats_rows(int64_t P, int Cout, int tile, int K, bool wide_ok) {
  const int bm = tile_bm(pick_conv_tile(P, Cout, tile, K, wide_ok));
  return (int)((P + bm - 1) / bm);
}

void launch_conv3x3_fwd(const void* x, const void* w, void* y, int N, int H, int W, int Cin, int Cout, int stride,
                        float* stats, hipStream_t stream, int tile) {
  if (tile == kTileAuto && halo_conv_eligible(Cin, Cout, W, stride, true)) {
    launch_conv3x3_halo(x, w, y, N, H, W, stats, stream);
    return;
  }
  const ConvGeom g = make_geom(N, H, W, Cin, Cout, stride);
  const bf16_t* xp = (const bf16_t*)x;
  const bf16_t* wp = (const bf16_t*)w;
  bf16_t* yp = (bf16_t*)y;
#define DLA_CFW(BM_, BN_, NT_)                                                  \
  if (stats) launch_fwd<BM_, BN_, true, NT_>(xp, wp, yp, g, stats, stream);   \
  else launch_fwd<BM_, BN_, false, NT_>(xp, wp, yp, g, stats, stream);
#define DLA_CF(BM_, BN_) DLA_CFW(BM_, BN_, kThreads)
  switch (pick_conv_tile((int64_t)g.N * g.OH * g.OW, Cout, tile, 9 * Cin, Cin % 64 == 0)) {
    case kTile512x128: DLA_CFW(512, 128, 512) break;
    case kTile256x256: DLA_CFW(256, 256, 512) break;
    case kTile256x128: DLA_CFW(256, 128, 512) break;
    case kTile256x128w4: DLA_CF(256, 128) break;
    case kTile128x256w4: DLA_CF(128, 256) break;
    case kTile256x64: DLA_CF(256, 64) break;
    case kTile128x128: DLA_CF(128, 128) break;
    case kTile128x64: DLA_CF(128, 64) break;
    default: DLA_CF(64, 64) break;
  }
#undef DLA_CF
#undef DLA_CFW
}

template <int BM, int BN, int PIPE, int NT>
static void launch_dgrad_p(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const ConvGeom& g, const bf16_t* addend,
                           const BnBwdEpi& bnb, hipStream_t stream) {
  const int64_t P = (int64_t)g.N * g.H * g.W;
  const int tiles = (int)((P + BM - 1) / BM) * ((g.Cin + BN - 1) / BN);
  const size_t lds =
      std::max(run_mainloop_lds_bytes<PIPE % 100, BM, BN, Im2colRowLoader<BM, true, NT>, WeightTapKLoader<BN, NT>>(),
               epilogue_lds_bytes<BM, BN, false, NT>());
  hipLaunchKernelGGL((conv3x3_dgrad_kernel<BM, BN, PIPE, NT>), dim3(tiles), dim3(NT), lds, stream, dy, w, dx, g,
                     addend, bnb);
}
template <int BM, int BN, int NTW = kThreads>
static void launch_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const ConvGeom& g, const bf16_t* addend,
                         const BnBwdEpi& bnb, hipStream_t stream) {
  if constexpr (NTW == 512 && BM * BN > 256 * 128) {
    if (mfma_pipeline() == 2) launch_dgrad_p<BM, BN, 2, 512>(dy, w, dx, g, addend, bnb, stream);
    else launch_dgrad_p<BM, BN, 6, 512>(dy, w, dx, g, addend, bnb, stream);
  } else if constexpr (NTW == 512) {
    if (mfma_pipeline() == 7) launch_dgrad_p<BM, BN, 7, 512>(dy, w, dx, g, addend, bnb, stream);
    else launch_dgrad_p<BM, BN, 3, 512>(dy, w, dx, g, addend, bnb, stream);
  } else if constexpr (BM * BN > 128 * 128) {
    if (mfma_pipeline() == 2) launch_dgrad_p<BM, BN, 2, kThreads>(dy, w, dx, g, addend, bnb, stream);
    else launch_dgrad_p<BM, BN, 3, kThreads>(dy, w, dx, g, addend, bnb, stream);
  } else if (g.Cout % 64 != 0) {
    if (mfma_pipeline_for(9 * g.Cout) == 0) launch_dgrad_p<BM, BN, 100, kThreads>(dy, w, dx, g, addend, bnb, stream);
    else launch_dgrad_p<BM, BN, 102, kThreads>(dy, w, dx, g, addend, bnb, stream);
  } else {
    switch (conv_pipeline(9 * g.Cout, 6)) {
      case 0: launch_dgrad_p<BM, BN, 0, kThreads>(dy, w, dx, g, addend, bnb, stream); break;
      case 3: launch_dgrad_p<BM, BN, 3, kThreads>(dy, w, dx, g, addend, bnb, stream); break;
      case 4: launch_dgrad_p<BM, BN, 4, kThreads>(dy, w, dx, g, addend, bnb, stream); break;
      case 6: launch_dgrad_p<BM, BN, 6, kThreads>(dy, w, dx, g, addend, bnb, stream); break;
      default: launch_dgrad_p<BM, BN, 2, kThreads>(dy, w, dx, g, addend, bnb, stream); break;
    }
  }
}

void launch_conv3x3_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                          const void* addend, hipStream_t stream, int tile, const BnBwdArgs* bn_bwd) {
  const ConvGeom g = make_geom(N, H, W, Cin, Cout, 1);
  BnBwdEpi bnb{};
  if (bn_bwd) {
    bnb.x = (const bf16_t*)bn_bwd->x;
    bnb.ldx = bn_bwd->ldx;
    bnb.ws = bn_bwd->ws;
    bnb.mask = bn_bwd->mask;
    bnb.mode = bn_bwd->mode;
    bnb.part = bn_bwd->part;
  }
  const bf16_t* d = (const bf16_t*)dy;
  const bf16_t* wp = (const bf16_t*)w;
  const bf16_t* ad = (const bf16_t*)addend;
  switch (pick_conv_tile((int64_t)N * H * W, Cin, tile, 9 * Cout, Cout % 64 == 0)) {
    case kTile512x128: launch_dgrad<512, 128, 512>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile256x256: launch_dgrad<256, 256, 512>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile256x128: launch_dgrad<256, 128, 512>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile256x128w4: launch_dgrad<256, 128>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile128x256w4: launch_dgrad<128, 256>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile256x64: launch_dgrad<256, 64>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile128x128: launch_dgrad<128, 128>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    case kTile128x64: launch_dgrad<128, 64>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
    default: launch_dgrad<64, 64>(d, wp, (bf16_t*)dx, g, ad, bnb, stream); break;
  }
}

void launch_conv3x3s2_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                            hipStream_t stream) {
  const ConvGeom g = make_geom(N, H, W, Cin, Cout, 2);  // OH = H / 2, OW = W / 2 (H, W even)
  const int64_t P = (int64_t)N * g.OH * g.OW;
  // 256x256 8-wave tiles (2-stage LDS DMA) at the compute-bound 14x14 / 7x7 shapes (Cin % 256, enough
  // tiles for the chip), as pick_tile does for the stride-1 passes; DLA_TILE256=0 turns them off
  if (tile256_enabled() && Cin % 256 == 0 && 4 * ((P + 255) / 256) * (Cin / 256) >= 192) {
    const int pc = (int)((P + 255) / 256) * (Cin / 256);
    hipLaunchKernelGGL((conv3x3s2_dgrad_kernel<256, 256, 2, 512>), dim3(4 * pc), dim3(512),
                       std::max(run_mainloop_lds_bytes<2, 256, 256, S2DgradRowLoader<256, 512>,
                                                       S2WeightKLoader<256, 512>>(),
                                epilogue_lds_bytes<256, 256, false, 512>()),
                       stream, (const bf16_t*)dy, (const bf16_t*)w, (bf16_t*)dx, g);
    return;
  }
  // 512x128 8-wave tiles for Cin = 128 (stage 2's strided conv2) with >= 1024 tiles over the 4 parity classes,
  // as pick_conv_tile does for the stride-1 passes; 2 stages fill all 160 KB of LDS. DLA_TILE512=0 turns them off
  if (tile256_enabled() && tile512_enabled() && Cin == 128 && Cout % 64 == 0 && 4 * ((P + 511) / 512) >= 1024) {
    const int pc = (int)((P + 511) / 512);
    hipLaunchKernelGGL((conv3x3s2_dgrad_kernel<512, 128, 2, 512>), dim3(4 * pc), dim3(512),
                       std::max(run_mainloop_lds_bytes<2, 512, 128, S2DgradRowLoader<512, 512>,
                                                       S2WeightKLoader<128, 512>>(),
                                epilogue_lds_bytes<512, 128, false, 512>()),
                       stream, (const bf16_t*)dy, (const bf16_t*)w, (bf16_t*)dx, g);
    return;
  }
  const int bn = Cin <= 64 ? 64 : 128;
  const int per_class = (int)((P + 127) / 128) * ((Cin + bn - 1) / bn);
#define DLA_S2(BN_, P_)                                                                                          \
  hipLaunchKernelGGL((conv3x3s2_dgrad_kernel<128, BN_, P_>), dim3(4 * per_class), dim3(kThreads),               \
                     std::max(run_mainloop_lds_bytes<P_, 128, BN_, S2DgradRowLoader<128>, S2WeightKLoader<BN_>>(), \
                              epilogue_lds_bytes<128, BN_, false>()),                                           \
                     stream, (const bf16_t*)dy, (const bf16_t*)w, (bf16_t*)dx, g)
  // the 1-tap class has K = Cout (one or two k-steps at ResNet shapes): one pipeline for all classes
  const int pipe = mfma_pipeline_for(4 * Cout);
  if (bn == 64) {
    if (pipe == 0) DLA_S2(64, 0); else DLA_S2(64, 2);
  } else {
    if (pipe == 0) DLA_S2(128, 0); else DLA_S2(128, 2);
  }
#undef DLA_S2
}

// 256x256 8-wave weight-gradient tiles (one block per CU) when both output dims are multiples of
// 256 (Cout and Cin in {256, 512, ...}: the compute-bound 14x14 / 7x7 layers), as for gemm_tn
static bool wgrad_wide(int Cin, int Cout) { return tn256_enabled() && Cout % 256 == 0 && Cin % 256 == 0; }

// 128 x 256 four-wave tiles (64 x 128 wave tiles: half the LDS fragment reads per MFMA of the 64 x 64 ones, one
// block per CU) for the Cout = 128 weight gradients (stage 2), whose 9 * Cin columns the 256x256 tiles cannot
// cover without wasting half the rows. DLA_WGRAD_W4=1 / set_wgrad_w4 (A/B; default off)
static int g_wgrad_w4 = -1;
void set_wgrad_w4(int mode) { g_wgrad_w4 = mode < 0 ? -1 : (mode ? 1 : 0); }
static bool wgrad_w4(int Cin, int Cout) {
  static const bool env = [] {
    const char* e = std::getenv("DLA_WGRAD_W4");
    return e && e[0] == '1';
  }();
  const bool on = g_wgrad_w4 < 0 ? env : g_wgrad_w4 == 1;
  return on && !wgrad_wide(Cin, Cout) && Cout == 128 && Cin % 64 == 0;
}

int conv3x3_wgrad_splits(int N, int H, int W, int Cin, int Cout, int stride) {
  const ConvGeom g = make_geom(N, H, W, Cin, Cout, stride);
  const int P = g.N * g.OH * g.OW;
  const bool wide = wgrad_wide(Cin, Cout), w4 = wgrad_w4(Cin, Cout);
  const int bm = wide ? 256 : (Cout <= 64 ? 64 : 128), bn = (wide || w4) ? 256 : 128;
  const int tiles = ((Cout + bm - 1) / bm) * ((9 * Cin + bn - 1) / bn);
  // ~2 workgroups per CU (one per CU for the 8-wave and the 128x256 tiles)
  const int splits = std::max(1, (wide || w4 ? splitk_target_blocks() / 2 : splitk_target_blocks()) / std::max(1, tiles));
  const int max_splits = std::max(1, P / (8 * kBK));          // >= 8 k-steps per split
  return std::max(1, std::min(splits, max_splits));
}

void launch_conv3x3_wgrad(const void* dy, const void* x, float* partial, int splits, void* dw, int out_dtype,
                          int N, int H, int W, int Cin, int Cout, int stride, hipStream_t stream) {
  const ConvGeom g = make_geom(N, H, W, Cin, Cout, stride);
  const int P = g.N * g.OH * g.OW;
  int kps = (P + splits - 1) / splits;
  kps = (kps + kBK - 1) / kBK * kBK;
  const int Mo = Cout, No = 9 * Cin;
#define DLA_WG(BM_, P_)                                                                                         \
  hipLaunchKernelGGL((conv3x3_wgrad_kernel<BM_, 128, P_>), dim3(((Mo + BM_ - 1) / BM_) * ((No + 127) / 128) * splits), \
                     dim3(kThreads), (run_mainloop_lds_bytes<P_, BM_, 128, KLoader<BM_>, Im2colKLoader<128, P_ != 0>>()), \
                     stream, (const bf16_t*)dy, (const bf16_t*)x, g, partial, kps,                                  \
                     ((Mo + BM_ - 1) / BM_) * ((No + 127) / 128), (int)splitk_xcd_remap())
#define DLA_WG_P(BM_)                   \
  switch (conv_pipeline(kps, 2)) {      \
    case 0: DLA_WG(BM_, 0); break;      \
    case 3: DLA_WG(BM_, 3); break;      \
    case 4: DLA_WG(BM_, 4); break;      \
    default: DLA_WG(BM_, 2); break;     \
  }
  if (wgrad_wide(Cin, Cout)) {
    const int nt = (Mo / 256) * (No / 256);
    const int pipe = conv_pipeline(kps, 2) == 4 ? 4 : 2;
#define DLA_WG8(P_)                                                                                             \
  hipLaunchKernelGGL((conv3x3_wgrad_kernel<256, 256, P_, 512>), dim3(nt * splits), dim3(512),                   \
                     (run_mainloop_lds_bytes<P_, 256, 256, KLoader<256, 512>, Im2colKLoader<256, true, 512>>()), \
                     stream, (const bf16_t*)dy, (const bf16_t*)x, g, partial, kps, nt, (int)splitk_xcd_remap())
    if (pipe == 2) DLA_WG8(2);
    else DLA_WG8(4);
#undef DLA_WG8
  } else if (wgrad_w4(Cin, Cout)) {
    const int nt = (No + 255) / 256;
    hipLaunchKernelGGL((conv3x3_wgrad_kernel<128, 256, 2>), dim3(nt * splits), dim3(kThreads),
                       (run_mainloop_lds_bytes<2, 128, 256, KLoader<128>, Im2colKLoader<256, true>>()), stream,
                       (const bf16_t*)dy, (const bf16_t*)x, g, partial, kps, nt, (int)splitk_xcd_remap());
  } else if (Cout <= 64) {
    DLA_WG_P(64)
  } else {
    DLA_WG_P(128)
  }
#undef DLA_WG_P
#undef DLA_WG
  launch_splitk_reduce(partial, splits, (int64_t)Mo * No, dw, out_dtype, 1.f, false, stream);
}

}  // namespace dla
