// Max pooling, NHWC (channels_last), forward + backward.
//
// The ResNet/GoogLeNet stems pool the largest activation of the network (ResNet-50 bs256:
// 112x112x64 bf16 = 411 MB in, 103 MB out). A lane owns 8 consecutive channels of one output
// (forward) or one input (backward) pixel: every access is a 16-byte vector and neighbouring lanes
// touch neighbouring bytes, so both passes stream at HBM rate.
//
// Forward : y = max over the k x k window (padding = -inf, NaN propagates like PyTorch), plus the
//           window position of the (first) maximum as one byte per element.
// Backward: gather form — each input element sums dy over the <= ceil(k/s)^2 windows that chose
//           it. No atomics, no zero-fill pass, deterministic; the overlap of 3x3/s2 windows is
//           resolved by reading the 1-byte positions instead of re-reading x.
#include "dla_common.h"
#include "dla_kernels.h"
#include "dla_mfma.h"

#include <algorithm>
#include <cstdlib>

namespace dla {

constexpr int kPoolThreads = 256;

struct PoolGeom {
  int N, H, W, C, OH, OW, k, s, p;
  mm::FastDiv fcg, fw, fh;  // divisors of the flat index: C/8, width, height (output or input side)
};

// Flat index t -> (n, row, col, channel) of an [N, rows, cols, C] NHWC tensor in 8-channel groups.
// kFast: multiply-shift division (t < 2^24, host-checked), else hardware integer division.
template <bool kFast>
__device__ __forceinline__ void decode(int t, const PoolGeom& g, int cols, int rows, int& n, int& row, int& col,
                                       int& c) {
  const int cg = g.C / 8;
  int q, r;
  if constexpr (kFast) {
    q = (int)mm::fdiv((uint32_t)t, g.fcg);
    c = (t - q * cg) * 8;
    r = (int)mm::fdiv((uint32_t)q, g.fw);
    col = q - r * cols;
    n = (int)mm::fdiv((uint32_t)r, g.fh);
    row = r - n * rows;
  } else {
    q = t / cg;
    c = (t - q * cg) * 8;
    r = q / cols;
    col = q - r * cols;
    n = r / rows;
    row = r - n * rows;
  }
}

// K > 0: the window size is a compile-time constant (GoogLeNet / ResNet use 3 and 2): all K*K taps
// are loaded before the first comparison (out-of-range taps read a clamped in-range pixel and are
// masked to -inf), so the loads are in flight together.
template <typename T, int K, bool kFast>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                                   uint8_t* __restrict__ pos, PoolGeom g) {
  const int total = g.N * g.OH * g.OW * (g.C / 8);  // < 2^31 (host-checked): 32-bit index math
  for (int t = blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += gridDim.x * kPoolThreads) {
    int n, oh, ow, c;
    decode<kFast>(t, g, g.OW, g.OH, n, oh, ow, c);
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
    const T* img = x + (int64_t)n * g.H * g.W * g.C + c;
    auto take = [&](const float (&v)[8], uint32_t q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // strict '>' keeps the first maximum; a NaN wins and sticks (PyTorch semantics)
        if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {
          best[j] = v[j];
          bi[j] = q;
        }
      }
    };
    if constexpr (K > 0) {
      float v[K * K][8];
      bool ok[K * K];
#pragma unroll
      for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int h = h0 + ky, w = w0 + kx, q = ky * K + kx;
          ok[q] = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
          const int hc = min(max(h, 0), g.H - 1), wc = min(max(w, 0), g.W - 1);
          Vec8<T>::load(img + ((int64_t)hc * g.W + wc) * g.C, v[q]);
        }
      // branch-free: an out-of-range tap becomes -inf, which never wins a strict '>' (as skipping it)
#pragma unroll
      for (int q = 0; q < K * K; ++q) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float vq = ok[q] ? v[q][j] : -INFINITY;
          const bool t = !(vq <= best[j]) & (best[j] == best[j]);  // vq > best, or vq NaN and best not
          best[j] = t ? vq : best[j];
          bi[j] = t ? (uint32_t)q : bi[j];
        }
      }
    } else {
      for (int ky = 0; ky < g.k; ++ky) {
        const int h = h0 + ky;
        if (h < 0 || h >= g.H) continue;
        for (int kx = 0; kx < g.k; ++kx) {
          const int w = w0 + kx;
          if (w < 0 || w >= g.W) continue;
          float v[8];
          Vec8<T>::load(img + ((int64_t)h * g.W + w) * g.C, v);
          take(v, (uint32_t)(ky * g.k + kx));
        }
      }
    }
    const int64_t off = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c;
    Vec8<T>::store(y + off, best);
    if (pos) {
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) packed |= (uint64_t)bi[j] << (8 * j);
      *reinterpret_cast<uint64_t*>(pos + off) = packed;
    }
  }
}

// 3x3 / stride-1 forward (GoogLeNet's Inception branch-4 pools), separable: a thread owns a strip
// of kStrip3 output rows at one column and 8 channels. It loads the kStrip3 + 2 input rows x 3
// columns once (27 loads for 7 outputs instead of 63), takes each input row's maximum over its 3
// columns (value + column), then each output's maximum over 3 of those row maxima. The per-tap
// compare-and-select work drops from 8 to 2 + 2 per output row shared 3 ways — the generic kernel
// is VALU-bound here (718 VALU instructions per wave, profiles/r3t).
// Same result as the row-major scan: strict '>' in both passes picks the first maximum in
// (ky, kx) order, and a NaN wins and sticks in both passes, so the first NaN in that order wins.
template <typename T, int RV, bool kFast>
__global__ __launch_bounds__(kPoolThreads) void maxpool3s1_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                                      uint8_t* __restrict__ pos, PoolGeom g,
                                                                      int nstrip) {
  const int total = g.N * nstrip * g.OW * (g.C / 8);  // < 2^31 (host-checked)
  for (int t = blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += gridDim.x * kPoolThreads) {
    int n, st, ow, c;
    decode<kFast>(t, g, g.OW, nstrip, n, st, ow, c);
    const int oh0 = st * RV;
    const T* img = x + (int64_t)n * g.H * g.W * g.C + c;
    int wc[3];
    bool okc[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int w = ow - g.p + kx;
      okc[kx] = (unsigned)w < (unsigned)g.W;
      wc[kx] = min(max(w, 0), g.W - 1);
    }
    // Branch-free: a tap outside the image reads a clamped in-range pixel and is replaced by -inf,
    // which never wins a strict '>' — the same as skipping it (a real -inf never wins either).
    // better(v, b) = v > b, or v NaN and b not: !(v <= b) && b == b.
    auto better = [](float v, float b) { return !(v <= b) & (b == b); };
    float hb[RV + 2][8];     // each input row's maximum over the window's 3 columns
    uint32_t hk[RV + 2][8];  // and its column
#pragma unroll
    for (int i = 0; i < RV + 2; ++i) {
      const int h = oh0 - g.p + i;
      const bool okr = (unsigned)h < (unsigned)g.H;
      const int hc = min(max(h, 0), g.H - 1);
      float v[3][8];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        Vec8<T>::load(img + ((int64_t)hc * g.W + wc[kx]) * g.C, v[kx]);
        const bool ok = okr && okc[kx];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[kx][j] = ok ? v[kx][j] : -INFINITY;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float b = v[0][j];  // column 0 first: the strict scan from -inf takes it unless it is -inf,
        uint32_t k = 0;     // and then position 0 is the default anyway
        const bool t1 = better(v[1][j], b);
        b = t1 ? v[1][j] : b;
        k = t1 ? 1u : k;
        const bool t2 = better(v[2][j], b);
        b = t2 ? v[2][j] : b;
        k = t2 ? 2u : k;
        hb[i][j] = b;
        hk[i][j] = k;
      }
    }
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      const int oh = oh0 + r;  // input rows r, r+1, r+2 of the strip are its window rows ky = 0, 1, 2
      float best[8];
      uint32_t bi[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float b = hb[r][j];
        uint32_t k = hk[r][j];
        const bool t1 = better(hb[r + 1][j], b);
        b = t1 ? hb[r + 1][j] : b;
        k = t1 ? 3u + hk[r + 1][j] : k;
        const bool t2 = better(hb[r + 2][j], b);
        b = t2 ? hb[r + 2][j] : b;
        k = t2 ? 6u + hk[r + 2][j] : k;
        best[j] = b;
        bi[j] = k;
      }
      if (oh < g.OH) {
        const int64_t off = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c;
        Vec8<T>::store(y + off, best);
        if (pos) {
          uint64_t packed = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) packed |= (uint64_t)bi[j] << (8 * j);
          *reinterpret_cast<uint64_t*>(pos + off) = packed;
        }
      }
    }
  }
}

// Backward, gather form: the windows covering input pixel (h, w) are oh in [oh_lo, oh_hi] (at most
// ceil(K/s) per axis). R = compile-time bound of windows per axis (0: runtime loops).
template <typename T, int R, bool kFast>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                                   const uint8_t* __restrict__ pos,
                                                                   T* __restrict__ dx, PoolGeom g) {
  const int total = g.N * g.H * g.W * (g.C / 8);
  for (int t = blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += gridDim.x * kPoolThreads) {
    int n, h, w, c;
    decode<kFast>(t, g, g.W, g.H, n, h, w, c);
    // windows covering (h, w): oh*s - p <= h <= oh*s - p + k - 1
    const int hp = h + g.p, wp = w + g.p;
    const int oh_lo = hp < g.k - 1 ? 0 : (hp - g.k + 1 + g.s - 1) / g.s;
    const int oh_hi = min(g.OH - 1, hp / g.s);
    const int ow_lo = wp < g.k - 1 ? 0 : (wp - g.k + 1 + g.s - 1) / g.s;
    const int ow_hi = min(g.OW - 1, wp / g.s);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int64_t nbase = (int64_t)n * g.OH * g.OW;
    if constexpr (R > 0) {
      uint64_t pk[R * R];
      float d[R * R][8];
      uint32_t qv[R * R];
      bool ok[R * R];
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) {
          const int oh = oh_lo + a, ow = ow_lo + b, i = a * R + b;
          ok[i] = oh <= oh_hi && ow <= ow_hi;
          const int ohc = ok[i] ? oh : oh_lo, owc = ok[i] ? ow : ow_lo;  // in range whenever any window is
          qv[i] = (uint32_t)((hp - ohc * g.s) * g.k + (wp - owc * g.s));
          const int64_t off = (nbase + (int64_t)min(ohc, g.OH - 1) * g.OW + min(owc, g.OW - 1)) * g.C + c;
          pk[i] = *reinterpret_cast<const uint64_t*>(pos + off);
          Vec8<T>::load(dy + off, d[i]);
        }
      // branch-free: a window outside the output matches no tap (0xff); the adds stay in (oh, ow) order
#pragma unroll
      for (int i = 0; i < R * R; ++i) {
        const uint32_t q = ok[i] ? qv[i] : 0xffu;
        const uint32_t lo = (uint32_t)pk[i], hi = (uint32_t)(pk[i] >> 32);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t byte = ((j < 4 ? lo : hi) >> (8 * (j & 3))) & 0xffu;
          acc[j] += byte == q ? d[i][j] : 0.f;
        }
      }
    } else {
      for (int oh = oh_lo; oh <= oh_hi; ++oh) {
        for (int ow = ow_lo; ow <= ow_hi; ++ow) {
          const uint32_t q = (uint32_t)((hp - oh * g.s) * g.k + (wp - ow * g.s));
          const int64_t off = (nbase + (int64_t)oh * g.OW + ow) * g.C + c;
          const uint64_t packed = *reinterpret_cast<const uint64_t*>(pos + off);
          float dd[8];
          Vec8<T>::load(dy + off, dd);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (((packed >> (8 * j)) & 0xffu) == q) acc[j] += dd[j];
        }
      }
    }
    Vec8<T>::store(dx + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, acc);
  }
}

static int pool_blocks(int64_t work) {
  // grid-stride: enough waves to fill 256 CUs several times over, capped to bound tail effects
  const int64_t b = (work + kPoolThreads - 1) / kPoolThreads;
  return (int)std::min<int64_t>(b, 256 * 32);
}

void launch_maxpool_fwd(const void* x, void* y, uint8_t* pos, int N, int H, int W, int C, int OH, int OW, int k,
                        int s, int p, int dtype, hipStream_t stream) {
  PoolGeom g{N, H, W, C, OH, OW, k, s, p, mm::make_fastdiv(C / 8), mm::make_fastdiv(OW), mm::make_fastdiv(OH)};
  const int64_t work = (int64_t)N * OH * OW * (C / 8);
  const int nb = pool_blocks(work);
  if (nb == 0) return;
  const bool fast = work < (1 << 24);
  // 3x3/s1: separable strips of 4 output rows (DLA_POOL3_SEP=0: generic kernel, 7: strips of 7; A/B)
  static const int sep3 = [] {
    const char* e = std::getenv("DLA_POOL3_SEP");
    return e ? std::atoi(e) : 4;
  }();
  if (k == 3 && s == 1 && (sep3 == 4 || sep3 == 7)) {
    const int nstrip = (OH + sep3 - 1) / sep3;
    PoolGeom gs{N, H, W, C, OH, OW, k, s, p, mm::make_fastdiv(C / 8), mm::make_fastdiv(OW), mm::make_fastdiv(nstrip)};
    const int64_t swork = (int64_t)N * nstrip * OW * (C / 8);
    const int snb = pool_blocks(swork);
    const bool sfast = swork < (1 << 24);
#define DLA_MPS(T, RV, F)                                                                                         \
  hipLaunchKernelGGL((maxpool3s1_fwd_kernel<T, RV, F>), dim3(snb), dim3(kPoolThreads), 0, stream, (const T*)x, (T*)y, \
                     pos, gs, nstrip)
#define DLA_MPS_RV(T, F) \
  if (sep3 == 7) DLA_MPS(T, 7, F); else DLA_MPS(T, 4, F);
    if (dtype == kBF16) { if (sfast) { DLA_MPS_RV(bf16_t, true) } else { DLA_MPS_RV(bf16_t, false) } }
    else { if (sfast) { DLA_MPS_RV(float, true) } else { DLA_MPS_RV(float, false) } }
#undef DLA_MPS_RV
#undef DLA_MPS
    return;
  }
#define DLA_MPF(T, K, F) \
  hipLaunchKernelGGL((maxpool_fwd_kernel<T, K, F>), dim3(nb), dim3(kPoolThreads), 0, stream, (const T*)x, (T*)y, pos, g)
#define DLA_MPF_K(T)                                                      \
  if (k == 3) { if (fast) DLA_MPF(T, 3, true); else DLA_MPF(T, 3, false); } \
  else if (k == 2) { if (fast) DLA_MPF(T, 2, true); else DLA_MPF(T, 2, false); } \
  else { if (fast) DLA_MPF(T, 0, true); else DLA_MPF(T, 0, false); }
  if (dtype == kBF16) { DLA_MPF_K(bf16_t) } else { DLA_MPF_K(float) }
#undef DLA_MPF_K
#undef DLA_MPF
}

void launch_maxpool_bwd(const void* dy, const uint8_t* pos, void* dx, int N, int H, int W, int C, int OH, int OW,
                        int k, int s, int p, int dtype, hipStream_t stream) {
  PoolGeom g{N, H, W, C, OH, OW, k, s, p, mm::make_fastdiv(C / 8), mm::make_fastdiv(W), mm::make_fastdiv(H)};
  const int64_t work = (int64_t)N * H * W * (C / 8);
  const int nb = pool_blocks(work);
  if (nb == 0) return;
  const bool fast = work < (1 << 24);
  const int r = (k + s - 1) / s;  // windows per axis covering one input pixel, at most
#define DLA_MPB(T, R, F)                                                                                        \
  hipLaunchKernelGGL((maxpool_bwd_kernel<T, R, F>), dim3(nb), dim3(kPoolThreads), 0, stream, (const T*)dy, pos, \
                     (T*)dx, g)
#define DLA_MPB_R(T)                                                      \
  if (r == 3) { if (fast) DLA_MPB(T, 3, true); else DLA_MPB(T, 3, false); } \
  else if (r == 2) { if (fast) DLA_MPB(T, 2, true); else DLA_MPB(T, 2, false); } \
  else if (r == 1) { if (fast) DLA_MPB(T, 1, true); else DLA_MPB(T, 1, false); } \
  else { if (fast) DLA_MPB(T, 0, true); else DLA_MPB(T, 0, false); }
  if (dtype == kBF16) { DLA_MPB_R(bf16_t) } else { DLA_MPB_R(float) }
#undef DLA_MPB_R
#undef DLA_MPB
}

// ---- global average pooling (the ResNet / GoogLeNet head) ------------------------------------------
// Forward: y[n, c] = mean over the HW pixels of x[n, :, c]. A block owns one image and 512 channels:
// lane = 8 channels (one 16-byte load per pixel, a wave reads 1 KB contiguous), the 4 waves split the
// pixels and combine through LDS in a fixed order (deterministic).
// Backward: dx[n, p, c] = dy[n, c] / HW written straight into the channels_last layout the last
// block's BN backward reads (torch's expand + copy made it a strided, non-vectorised pass).
template <typename T>
__global__ __launch_bounds__(kPoolThreads) void gap_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int HW,
                                                               int C, float inv) {
  __shared__ float part[4][64][8];
  const int n = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    const T* base = x + (int64_t)n * HW * C + c;
    for (int p = wv; p < HW; p += 4) {
      float v[8];
      Vec8<T>::load(base + (int64_t)p * C, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[wv][lane][j] = acc[j];
  __syncthreads();
  if (wv == 0 && c < C) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = ((part[0][lane][j] + part[1][lane][j]) + (part[2][lane][j] + part[3][lane][j])) * inv;
    Vec8<T>::store(y + (int64_t)n * C + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int HW,
                                                               int C, float inv, int64_t total) {
  const int cg = C / 8;
  for (int64_t t = (int64_t)blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += (int64_t)gridDim.x * kPoolThreads) {
    const int c = (int)(t % cg) * 8;
    const int64_t n = t / cg / HW;
    float v[8];
    Vec8<T>::load(dy + n * C + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= inv;
    Vec8<T>::store(dx + t * 8, v);
  }
}

// Stride-2 subsample of an NHWC bf16 activation, y[n][h][w] = x[n][2h][2w] (the input of a ResNet
// downsample 1x1 conv): 16-byte chunks, 4 chunks per thread with all loads issued before the
// stores. Replaces torch's strided elementwise copy (3.2 TB/s at the stage-2 shape).
__global__ __launch_bounds__(kPoolThreads) void subsample2_kernel(const ushort8_t* __restrict__ x,
                                                                  ushort8_t* __restrict__ y, uint32_t cg,
                                                                  uint32_t OW, uint32_t OH, int W, int H,
                                                                  uint32_t total) {
  // plain 32-bit divisions (a few dozen VALU per 32 bytes moved: free in this HBM-bound copy; the
  // 24-bit mm::fdiv would overflow at batch 1024)
  constexpr int U = 4;
  const uint32_t stride = gridDim.x * kPoolThreads;
  for (uint32_t t0 = blockIdx.x * kPoolThreads + threadIdx.x; t0 < total; t0 += U * stride) {
    ushort8_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = t0 + u * stride;
      if (t < total) {
        const uint32_t pix = t / cg, c = t - pix * cg;
        const uint32_t q = pix / OW, ow = pix - q * OW;
        const uint32_t n = q / OH, oh = q - n * OH;
        v[u] = x[(((uint64_t)n * H + 2 * oh) * W + 2 * ow) * cg + c];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = t0 + u * stride;
      if (t < total) y[t] = v[u];
    }
  }
}

void launch_subsample2(const void* x, void* y, int N, int H, int W, int C, hipStream_t stream) {
  const int OH = H / 2, OW = W / 2;
  const uint32_t total = (uint32_t)N * OH * OW * (C / 8);
  if (total == 0) return;
  const int nb = (int)std::min<int64_t>(((int64_t)total + 4 * kPoolThreads - 1) / (4 * kPoolThreads), 256 * 32);
  hipLaunchKernelGGL(subsample2_kernel, dim3(nb), dim3(kPoolThreads), 0, stream, (const ushort8_t*)x, (ushort8_t*)y,
                     (uint32_t)(C / 8), (uint32_t)OW, (uint32_t)OH, W, H, total);
}

void launch_gap_fwd(const void* x, void* y, int N, int HW, int C, int dtype, hipStream_t stream) {
  const dim3 grid((C / 8 + 63) / 64, N);
  const float inv = 1.f / (float)HW;
  if (dtype == kBF16)
    hipLaunchKernelGGL(gap_fwd_kernel<bf16_t>, grid, dim3(kPoolThreads), 0, stream, (const bf16_t*)x, (bf16_t*)y, HW,
                       C, inv);
  else
    hipLaunchKernelGGL(gap_fwd_kernel<float>, grid, dim3(kPoolThreads), 0, stream, (const float*)x, (float*)y, HW, C,
                       inv);
}

void launch_gap_bwd(const void* dy, void* dx, int N, int HW, int C, int dtype, hipStream_t stream) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  const int nb = pool_blocks(total);
  if (nb == 0) return;
  const float inv = 1.f / (float)HW;
  if (dtype == kBF16)
    hipLaunchKernelGGL(gap_bwd_kernel<bf16_t>, dim3(nb), dim3(kPoolThreads), 0, stream, (const bf16_t*)dy, (bf16_t*)dx,
                       HW, C, inv, total);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(nb), dim3(kPoolThreads), 0, stream, (const float*)dy, (float*)dx, HW,
                       C, inv, total);
}

}  // namespace dla
