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

#include <algorithm>

namespace dla {

constexpr int kPoolThreads = 256;

struct PoolGeom {
  int N, H, W, C, OH, OW, k, s, p;
};

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                                   uint8_t* __restrict__ pos, PoolGeom g) {
  const int cg = g.C / 8;
  const int total = g.N * g.OH * g.OW * cg;  // < 2^31 (host-checked): 32-bit index math
  for (int t = blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += gridDim.x * kPoolThreads) {
    const int c = (t % cg) * 8;
    int r = t / cg;
    const int ow = r % g.OW;
    r /= g.OW;
    const int oh = r % g.OH;
    const int n = r / g.OH;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
    for (int ky = 0; ky < g.k; ++ky) {
      const int h = h0 + ky;
      if (h < 0 || h >= g.H) continue;
      for (int kx = 0; kx < g.k; ++kx) {
        const int w = w0 + kx;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<T>::load(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + c, v);
        const uint32_t q = (uint32_t)(ky * g.k + kx);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // strict '>' keeps the first maximum; a NaN wins and sticks (PyTorch semantics)
          if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {
            best[j] = v[j];
            bi[j] = q;
          }
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

template <typename T>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                                   const uint8_t* __restrict__ pos,
                                                                   T* __restrict__ dx, PoolGeom g) {
  const int cg = g.C / 8;
  const int total = g.N * g.H * g.W * cg;
  for (int t = blockIdx.x * kPoolThreads + threadIdx.x; t < total; t += gridDim.x * kPoolThreads) {
    const int c = (t % cg) * 8;
    int r = t / cg;
    const int w = r % g.W;
    r /= g.W;
    const int h = r % g.H;
    const int n = r / g.H;
    // windows covering (h, w): oh*s - p <= h <= oh*s - p + k - 1
    const int hp = h + g.p, wp = w + g.p;
    const int oh_lo = hp < g.k - 1 ? 0 : (hp - g.k + 1 + g.s - 1) / g.s;
    const int oh_hi = min(g.OH - 1, hp / g.s);
    const int ow_lo = wp < g.k - 1 ? 0 : (wp - g.k + 1 + g.s - 1) / g.s;
    const int ow_hi = min(g.OW - 1, wp / g.s);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint32_t q = (uint32_t)((hp - oh * g.s) * g.k + (wp - ow * g.s));
        const int64_t off = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(pos + off);
        float d[8];
        Vec8<T>::load(dy + off, d);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((packed >> (8 * j)) & 0xffu) == q) acc[j] += d[j];
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
  PoolGeom g{N, H, W, C, OH, OW, k, s, p};
  const int nb = pool_blocks((int64_t)N * OH * OW * (C / 8));
  if (nb == 0) return;
  if (dtype == kBF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, dim3(nb), dim3(kPoolThreads), 0, stream, (const bf16_t*)x,
                       (bf16_t*)y, pos, g);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(nb), dim3(kPoolThreads), 0, stream, (const float*)x,
                       (float*)y, pos, g);
}

void launch_maxpool_bwd(const void* dy, const uint8_t* pos, void* dx, int N, int H, int W, int C, int OH, int OW,
                        int k, int s, int p, int dtype, hipStream_t stream) {
  PoolGeom g{N, H, W, C, OH, OW, k, s, p};
  const int nb = pool_blocks((int64_t)N * H * W * (C / 8));
  if (nb == 0) return;
  if (dtype == kBF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, dim3(nb), dim3(kPoolThreads), 0, stream, (const bf16_t*)dy, pos,
                       (bf16_t*)dx, g);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(nb), dim3(kPoolThreads), 0, stream, (const float*)dy, pos,
                       (float*)dx, g);
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
