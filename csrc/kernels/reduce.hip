// Elementwise reduce kernels used by the collective algorithms.
//
//   * ring step reduce   `chunks[to_recv][:] += recv_buffer`   /root/reference/src/allreduce.py:76,142
//   * central sum        `send[:] += recv_buffers[i]`           /root/reference/src/allreduce.py:32
//   * node aggregation   `agg[:len(buff)] += buff`              /root/reference/src/reducers.py:59-61
//   * average            `send /= size`                         /root/reference/src/allreduce.py:98
//
// One kernel covers all of them: dst = scale * ([dst] + src_0 + ... + src_{k-1}) with up to 8
// sources, so a k-way sum (central root, two-shot reduce-scatter, hierarchical node sum) reads
// each source once and writes once instead of k-1 read-modify-write passes. 16-byte vectors,
// grid-stride capped at 256 CUs x 8 blocks (Guideline 11). Memory-bound by construction.
#include "dla_common.h"
#include "dla_kernels.h"

namespace dla {

constexpr int kRBlock = 256;

template <typename T>
__global__ __launch_bounds__(kRBlock) void reduce_sum_kernel(T* __restrict__ dst, int accumulate, ReduceSrcs srcs,
                                                             int64_t n, float scale) {
  // vector width: 4 fp32 or 8 bf16 = 16 B
  constexpr int V = 16 / sizeof(T);
  const int64_t nvec = n / V;
  const int64_t stride = (int64_t)gridDim.x * kRBlock;
  for (int64_t v = (int64_t)blockIdx.x * kRBlock + threadIdx.x; v < nvec; v += stride) {
    float acc[V];
    if (accumulate) {
      if constexpr (V == 4) {
        float4_t x = reinterpret_cast<const float4_t*>(dst)[v];
        acc[0] = x.x; acc[1] = x.y; acc[2] = x.z; acc[3] = x.w;
      } else {
        ushort8_t x = reinterpret_cast<const ushort8_t*>(dst)[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = bf16_to_f32(x[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = 0.f;
    }
    for (int s = 0; s < srcs.count; ++s) {
      if constexpr (V == 4) {
        float4_t x = reinterpret_cast<const float4_t*>(srcs.ptr[s])[v];
        acc[0] += x.x; acc[1] += x.y; acc[2] += x.z; acc[3] += x.w;
      } else {
        ushort8_t x = reinterpret_cast<const ushort8_t*>(srcs.ptr[s])[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf16_to_f32(x[j]);
      }
    }
    if constexpr (V == 4) {
      reinterpret_cast<float4_t*>(dst)[v] = float4_t{acc[0] * scale, acc[1] * scale, acc[2] * scale, acc[3] * scale};
    } else {
      ushort8_t o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(acc[j] * scale);
      reinterpret_cast<ushort8_t*>(dst)[v] = o;
    }
  }
  // scalar tail (< V elements), handled by block 0
  if (blockIdx.x == 0) {
    for (int64_t i = nvec * V + threadIdx.x; i < n; i += kRBlock) {
      float a = accumulate ? Cvt<T>::to_f32(dst[i]) : 0.f;
      for (int s = 0; s < srcs.count; ++s) a += Cvt<T>::to_f32(reinterpret_cast<const T*>(srcs.ptr[s])[i]);
      dst[i] = Cvt<T>::from_f32(a * scale);
    }
  }
}

static int grid_for(int64_t nvec) {
  int64_t g = (nvec + kRBlock - 1) / kRBlock;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

static bool all_aligned(const void* dst, const ReduceSrcs& s) {
  uintptr_t a = reinterpret_cast<uintptr_t>(dst);
  for (int i = 0; i < s.count; ++i) a |= reinterpret_cast<uintptr_t>(s.ptr[i]);
  return (a & 15) == 0;
}

template <typename T>
__global__ __launch_bounds__(kRBlock) void reduce_sum_scalar_kernel(T* __restrict__ dst, int accumulate,
                                                                    ReduceSrcs srcs, int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * kRBlock;
  for (int64_t i = (int64_t)blockIdx.x * kRBlock + threadIdx.x; i < n; i += stride) {
    float a = accumulate ? Cvt<T>::to_f32(dst[i]) : 0.f;
    for (int s = 0; s < srcs.count; ++s) a += Cvt<T>::to_f32(reinterpret_cast<const T*>(srcs.ptr[s])[i]);
    dst[i] = Cvt<T>::from_f32(a * scale);
  }
}

void launch_reduce_sum(void* dst, bool accumulate_dst, const ReduceSrcs& srcs, int64_t n, int dtype, float scale,
                       hipStream_t stream) {
  if (n <= 0) return;
  const bool aligned = all_aligned(dst, srcs);
  if (dtype == kF32) {
    if (aligned)
      hipLaunchKernelGGL(reduce_sum_kernel<float>, dim3(grid_for(n / 4 + 1)), dim3(kRBlock), 0, stream,
                         (float*)dst, (int)accumulate_dst, srcs, n, scale);
    else
      hipLaunchKernelGGL(reduce_sum_scalar_kernel<float>, dim3(grid_for(n)), dim3(kRBlock), 0, stream,
                         (float*)dst, (int)accumulate_dst, srcs, n, scale);
  } else {
    if (aligned)
      hipLaunchKernelGGL(reduce_sum_kernel<bf16_t>, dim3(grid_for(n / 8 + 1)), dim3(kRBlock), 0, stream,
                         (bf16_t*)dst, (int)accumulate_dst, srcs, n, scale);
    else
      hipLaunchKernelGGL(reduce_sum_scalar_kernel<bf16_t>, dim3(grid_for(n)), dim3(kRBlock), 0, stream,
                         (bf16_t*)dst, (int)accumulate_dst, srcs, n, scale);
  }
}

// ---- multi-lane reduce: one launch for all single-source reductions of a ring step -----------
// Blocks are dealt to lanes in proportion to their 16-byte vector counts (blk0 prefix, <= 8 compares
// to find the lane); inside a lane a grid-stride loop over that lane's blocks. A lane whose pointers
// are not 16-byte aligned takes the scalar loop (never the case for plan slices: 64-element aligned).
template <typename T>
__global__ __launch_bounds__(kRBlock) void reduce_lanes_kernel(ReduceLanes L) {
  constexpr int V = 16 / sizeof(T);
  const int b = blockIdx.x;
  int li = 0;
  while (li + 1 < L.count && b >= L.blk0[li + 1]) ++li;
  const ReduceLane ln = L.lane[li];
  const int lb = b - L.blk0[li], nb = L.blk0[li + 1] - L.blk0[li];
  T* __restrict__ dst = static_cast<T*>(ln.dst);
  const T* __restrict__ src = static_cast<const T*>(ln.src);
  const uintptr_t al = reinterpret_cast<uintptr_t>(ln.dst) | reinterpret_cast<uintptr_t>(ln.src);
  const int64_t stride = (int64_t)nb * kRBlock;
  int64_t done = 0;
  if (ln.accumulate == 2) {  // bit copy (a virtual-rank link / plan copy): no arithmetic, -0 and NaN kept
    if ((al & 15) == 0) {
      const int64_t nvec = ln.n / V;
      for (int64_t v = (int64_t)lb * kRBlock + threadIdx.x; v < nvec; v += stride)
        reinterpret_cast<float4_t*>(dst)[v] = reinterpret_cast<const float4_t*>(src)[v];
      done = nvec * V;
    }
    for (int64_t i = done + (int64_t)lb * kRBlock + threadIdx.x; i < ln.n; i += stride) dst[i] = src[i];
    return;
  }
  if ((al & 15) == 0) {
    const int64_t nvec = ln.n / V;
    for (int64_t v = (int64_t)lb * kRBlock + threadIdx.x; v < nvec; v += stride) {
      if constexpr (V == 4) {
        float4_t x = ln.accumulate ? reinterpret_cast<const float4_t*>(dst)[v] : float4_t{0.f, 0.f, 0.f, 0.f};
        if (src) x += reinterpret_cast<const float4_t*>(src)[v];
        reinterpret_cast<float4_t*>(dst)[v] = x * ln.scale;
      } else {
        ushort8_t x = ln.accumulate ? reinterpret_cast<const ushort8_t*>(dst)[v] : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
        ushort8_t y = src ? reinterpret_cast<const ushort8_t*>(src)[v] : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
        ushort8_t o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16((bf16_to_f32(x[j]) + bf16_to_f32(y[j])) * ln.scale);
        reinterpret_cast<ushort8_t*>(dst)[v] = o;
      }
    }
    done = nvec * V;
  }
  for (int64_t i = done + (int64_t)lb * kRBlock + threadIdx.x; i < ln.n; i += stride) {
    float a = ln.accumulate ? Cvt<T>::to_f32(dst[i]) : 0.f;
    if (src) a += Cvt<T>::to_f32(src[i]);
    dst[i] = Cvt<T>::from_f32(a * ln.scale);
  }
}

void launch_reduce_lanes(ReduceLanes& L, int dtype, hipStream_t stream) {
  if (L.count <= 0) return;
  const int V = dtype == kF32 ? 4 : 8;
  int64_t total = 0;
  for (int i = 0; i < L.count; ++i) total += L.lane[i].n / V + 1;
  // ~2048 blocks over the whole step (8 per CU), at least one per lane
  const double per = total > 0 ? 2048.0 / (double)total : 0.0;
  int acc = 0;
  for (int i = 0; i < L.count; ++i) {
    L.blk0[i] = acc;
    const int64_t need = (L.lane[i].n / V + kRBlock) / kRBlock;  // blocks to cover the lane once
    int64_t nb = (int64_t)((double)(L.lane[i].n / V + 1) * per + 0.5);
    nb = nb < 1 ? 1 : (nb > need ? need : nb);
    acc += (int)nb;
  }
  L.blk0[L.count] = acc;
  if (dtype == kF32)
    hipLaunchKernelGGL(reduce_lanes_kernel<float>, dim3(acc), dim3(kRBlock), 0, stream, L);
  else
    hipLaunchKernelGGL(reduce_lanes_kernel<bf16_t>, dim3(acc), dim3(kRBlock), 0, stream, L);
}

// dst = scale * src with a dtype conversion (fp32 <-> bf16): staging of bf16 buckets in fp32 for
// full-precision accumulation across ranks (CommEngine accum_fp32).
template <typename D, typename S>
__global__ __launch_bounds__(kRBlock) void cast_kernel(D* __restrict__ dst, const S* __restrict__ src, int64_t n,
                                                       float scale) {
  const int64_t stride = (int64_t)gridDim.x * kRBlock * 4;
  for (int64_t i = ((int64_t)blockIdx.x * kRBlock + threadIdx.x) * 4; i < n; i += stride) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (i + j < n) dst[i + j] = Cvt<D>::from_f32(Cvt<S>::to_f32(src[i + j]) * scale);
  }
}

void launch_cast(void* dst, int dst_dtype, const void* src, int src_dtype, int64_t n, float scale, hipStream_t stream) {
  if (n <= 0) return;
  const dim3 g(grid_for((n + 3) / 4)), b(kRBlock);
  if (dst_dtype == kF32 && src_dtype == kBF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), g, b, 0, stream, (float*)dst, (const bf16_t*)src, n, scale);
  else if (dst_dtype == kBF16 && src_dtype == kF32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), g, b, 0, stream, (bf16_t*)dst, (const float*)src, n, scale);
  else if (dst_dtype == kF32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, stream, (float*)dst, (const float*)src, n, scale);
  else
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), g, b, 0, stream, (bf16_t*)dst, (const bf16_t*)src, n, scale);
}

void launch_scale(void* data, int64_t n, int dtype, float scale, hipStream_t stream) {
  ReduceSrcs none{};
  none.count = 0;
  launch_reduce_sum(data, true, none, n, dtype, scale, stream);
}

}  // namespace dla
