// bf16 MFMA GEMMs for the ResNet 1x1-convolution hot path (channels_last activations).
//
// With NHWC activations a 1x1 convolution is a plain GEMM over M = N*H*W rows:
//   forward  Y[M, Cout]    = X[M, Cin]  * W[Cout, Cin]^T        -> gemm_nt (A = X,  B = W)
//   dgrad    dX[M, Cin]    = dY[M, Cout] * W[Cout, Cin]         -> gemm_nt (A = dY, B = W^T)
//   wgrad    dW[Cout, Cin] = dY[M, Cout]^T * X[M, Cin]          -> gemm_tn, split over M
// The reference runs these as cuDNN/MIOpen convolutions. At ResNet-50 shapes the
// reduction dim is small (K = 64..2048) so most of these GEMMs sit near the HBM roofline rather than
// the MFMA roofline; the kernels are built for that regime:
//   * 256-thread workgroups, 2x2 waves, v_mfma_f32_16x16x32_bf16 (fp32 accumulate), 64-deep K
//     steps staged through LDS with a register prefetch of the next tile (global loads in flight
//     while the MFMAs of the current tile run, cdna_hip_programming.md T14), rows padded by 16 B so
//     the ds_read_b128 fragment reads are bank-conflict free;
//   * bijective XCD-aware tile remap (T1) so consecutive tiles share an XCD's L2;
//   * epilogue staged through LDS so the bf16 tile leaves in full 16-byte-per-lane row segments,
//     with an optional fused per-column (channel) sum / sum-of-squares — the BatchNorm statistics of
//     the conv output — written as per-row-block partials (no atomics, fixed-order reduction);
//   * gemm_tn reads k-major operands straight from their natural layout with the gfx950
//     ds_read_b64_tr_b16 transposing LDS read (T10) and splits the long M reduction over blocks
//     with fp32 partial slabs + a separate reduction kernel.
#include "dla_common.h"
#include "dla_kernels.h"

namespace dla {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

constexpr int kGemmThreads = 256;
constexpr int kBK = 64;

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// k-major tile image for ds_read_b64_tr_b16 (rows = k, W = 64 or 128 columns, unpadded rows).
// A 32-lane half of a transposed 16x16x32-operand read touches rows {r..r+3, r+8..r+11} x 4
// consecutive 8-byte chunks; with plain rows those 8 row-blocks share banks (2-way or worse for any
// constant row pitch). XOR-ing the chunk index with a row-dependent multiple of 4 gives the 8
// row-blocks disjoint 8-bank windows (conflict-free), keeps every 4-chunk (32 B) group and every
// 16-byte store contiguous, and the same function addresses stores and reads.
template <int W>
__device__ __forceinline__ int tr_off(int row, int col) {  // element offset of (row, col), col % 4 == 0
  static_assert(W == 64 || W == 128, "tr image width");
  int sw;
  if constexpr (W == 128)
    sw = 4 * ((row & 3) | (((row >> 3) & 1) << 2));  // 32 chunks/row (256 B = 64 banks)
  else
    sw = 4 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));  // 16 chunks/row; row parity adds 32 banks
  return row * W + (((col >> 2) ^ sw) << 2);
}

__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* lo_ptr, const bf16_t* hi_ptr) {
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(lo_ptr));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(hi_ptr));
  const short v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return *reinterpret_cast<const bf16x8_t*>(v);
}

// ---------------------------------------------------------------------------------------------
// C[M,N] = A[M,K] * B[N,K]^T   (all row-major; A, B K-contiguous), bf16 in/out, fp32 accumulate.
// ---------------------------------------------------------------------------------------------
// kBT: B is given k-major ([K, N], n-contiguous — e.g. the conv weight for dgrad) and its MFMA
// fragments are read with the transposing ds_read_b64_tr_b16, so no transposed copy is needed.
template <int BM, int BN, bool kStats, bool kBT>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_nt_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                  const bf16_t* __restrict__ B, int64_t ldb,
                                                                  bf16_t* __restrict__ C, int64_t ldc, int M, int N,
                                                                  int K, float* __restrict__ stats,
                                                                  const bf16_t* __restrict__ D, int64_t ldd) {
  constexpr int LDS_K = kBK + 8;  // +16 B per row: conflict-free ds_read_b128 fragment reads
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int ACH = BM * kBK / 8 / kGemmThreads;  // 16-byte chunks per thread per A tile
  constexpr int BCH = BN * kBK / 8 / kGemmThreads;
  constexpr int BPR = BN / 8;  // kBT: B tile stored [kBK][BN] in the tr_off image
  static_assert(ACH >= 1 && BCH >= 1, "tile too small for 256 threads");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* Bs = As + BM * LDS_K;

  const int nbn = (N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = tile / nbn, bn = tile % nbn;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t row0 = (int64_t)bm * BM;
  const int col0 = bn * BN;

  ushort8_t ra[ACH], rb[BCH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kGemmThreads, r = c >> 3, kc = (c & 7) * 8;
      const int64_t gm = row0 + r;
      ra[i] = (gm < M && k0 + kc < K) ? *reinterpret_cast<const ushort8_t*>(A + gm * lda + k0 + kc)
                                      : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kGemmThreads;
      if constexpr (kBT) {
        const int kr = c / BPR, nc = (c % BPR) * 8;
        const int gk = k0 + kr, gn = col0 + nc;
        rb[i] = (gk < K && gn < N) ? *reinterpret_cast<const ushort8_t*>(B + (int64_t)gk * ldb + gn)
                                   : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
      } else {
        const int r = c >> 3, kc = (c & 7) * 8;
        const int gn = col0 + r;
        rb[i] = (gn < N && k0 + kc < K) ? *reinterpret_cast<const ushort8_t*>(B + (int64_t)gn * ldb + k0 + kc)
                                        : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kGemmThreads;
      *reinterpret_cast<ushort8_t*>(As + (c >> 3) * LDS_K + (c & 7) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kGemmThreads;
      if constexpr (kBT)
        *reinterpret_cast<ushort8_t*>(Bs + tr_off<BN>(c / BPR, (c % BPR) * 8)) = rb[i];
      else
        *reinterpret_cast<ushort8_t*>(Bs + (c >> 3) * LDS_K + (c & 7) * 8) = rb[i];
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane map (kBT): lane 4q+p of 16-lane group g reads k-row 8g+q, columns 4p..4p+3
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int nk = (K + kBK - 1) / kBK;
  gload(0);
  sstore();
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) gload((t + 1) * kBK);  // next tile in flight during this tile's MFMAs
#pragma unroll
    for (int kk = 0; kk < kBK / 32; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(As + (wr * WM + i * 16 + fr) * LDS_K + kk * 32 + fk);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (kBT) {
          const int kr = kk * 32 + 8 * tg + tq, cn = wc * WN + j * 16 + 4 * tp;
          bfr[j] = tr_frag(Bs + tr_off<BN>(kr, cn), Bs + tr_off<BN>(kr + 4, cn));
        } else {
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (wc * WN + j * 16 + fr) * LDS_K + kk * 32 + fk);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    __syncthreads();
    if (t + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }

  // ---- epilogue: bf16 tile -> LDS -> coalesced 16 B stores (+ column statistics) ----
  constexpr int LDS_C = BN + 8;
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem_raw);
  // Column statistics straight from the accumulator registers: a lane owns one column of each
  // 16x16 tile and 4 of its rows, so it sums TM*4 rows per column in registers, then the 4 lane
  // groups sharing a column combine with two xor-shuffles, and the 2 M-waves through LDS.
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) cs[j] = cq[j] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wr * WM + i * 16 + (lane >> 4) * 4 + r;  // C/D map: row = 4*(lane>>4)+reg
        const int n = wc * WN + j * 16 + fr;                    //          col = lane & 15
        const bf16_t h = f32_to_bf16(acc[i][j][r]);
        Cs[m * LDS_C + n] = h;
        if constexpr (kStats) {
          const float v = (row0 + m < M) ? bf16_to_f32(h) : 0.f;  // statistics of the stored values
          cs[j] += v;
          cq[j] = fmaf(v, v, cq[j]);
        }
      }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int c = tid; c < BM * CPR; c += kGemmThreads) {
    const int r = c / CPR, cc = (c % CPR) * 8;
    const int64_t gm = row0 + r;
    const int gn = col0 + cc;
    if (gm < M && gn < N) {
      ushort8_t v = *reinterpret_cast<ushort8_t*>(Cs + r * LDS_C + cc);
      if (D) {  // fused addend (residual-gradient sum): C = bf16(bf16(A B^T) + D), as the unfused add
        const ushort8_t d = *reinterpret_cast<const ushort8_t*>(D + gm * ldd + gn);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) + bf16_to_f32(d[j]));
      }
      *reinterpret_cast<ushort8_t*>(C + gm * ldc + gn) = v;
    }
  }
  if constexpr (kStats) {
    float* red = reinterpret_cast<float*>(smem_raw + BM * LDS_C * sizeof(bf16_t));  // [2 wr][BN][2]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, kWave);
      cq[j] += __shfl_xor(cq[j], 16, kWave);
      cs[j] += __shfl_xor(cs[j], 32, kWave);
      cq[j] += __shfl_xor(cq[j], 32, kWave);
      if (lane < 16) {
        const int n = wc * WN + j * 16 + fr;
        red[(wr * BN + n) * 2 + 0] = cs[j];
        red[(wr * BN + n) * 2 + 1] = cq[j];
      }
    }
    __syncthreads();
    if (tid < BN && col0 + tid < N) {
      stats[((int64_t)bm * N + col0 + tid) * 2 + 0] = red[tid * 2 + 0] + red[(BN + tid) * 2 + 0];
      stats[((int64_t)bm * N + col0 + tid) * 2 + 1] = red[tid * 2 + 1] + red[(BN + tid) * 2 + 1];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// P[split][Mo, No] = sum_{k in split} A[k][m] * B[k][n]   (A: [K, lda] m-contiguous, B: [K, ldb])
// fp32 partial slabs; gemm_splitk_reduce sums them.
// ---------------------------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_tn_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                                  const bf16_t* __restrict__ B, int64_t ldb,
                                                                  float* __restrict__ P, int Mo, int No, int K,
                                                                  int k_per_split) {
  // both tiles k-major in the swizzled tr_off image (conflict-free transposed reads)
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int ACH = kBK * BM / 8 / kGemmThreads, BCH = kBK * BN / 8 / kGemmThreads;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem_raw);  // [BK][BM]
  bf16_t* Bs = As + kBK * BM;                        // [BK][BN]

  const int nbn = (No + BN - 1) / BN;
  const int tile = blockIdx.x;
  const int bm = tile / nbn, bn = tile % nbn;
  const int split = blockIdx.y;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int m0 = bm * BM, n0 = bn * BN;
  constexpr int APR = BM / 8, BPR = BN / 8;  // chunks per k-row

  ushort8_t ra[ACH], rb[BCH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kGemmThreads, kr = c / APR, mc = (c % APR) * 8;
      const int gk = k0 + kr;
      ra[i] = (gk < kend && m0 + mc < Mo) ? *reinterpret_cast<const ushort8_t*>(A + (int64_t)gk * lda + m0 + mc)
                                          : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kGemmThreads, kr = c / BPR, nc = (c % BPR) * 8;
      const int gk = k0 + kr;
      rb[i] = (gk < kend && n0 + nc < No) ? *reinterpret_cast<const ushort8_t*>(B + (int64_t)gk * ldb + n0 + nc)
                                          : ushort8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kGemmThreads;
      *reinterpret_cast<ushort8_t*>(As + tr_off<BM>(c / APR, (c % APR) * 8)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kGemmThreads;
      *reinterpret_cast<ushort8_t*>(Bs + tr_off<BN>(c / BPR, (c % BPR) * 8)) = rb[i];
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads: in each 16-lane group, lane 4q+p addresses row q, columns 4p..4p+3
  // of a 4 x 16 block and receives column (lane & 15) of those 4 rows (element q = k).
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk > 0) {
    gload(kbeg);
    sstore();
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) gload(kbeg + (t + 1) * kBK);
#pragma unroll
    for (int kk = 0; kk < kBK / 32; ++kk) {
      bf16x8_t af[TM], bfr[TN];
      const int kr = kk * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int cm = wr * WM + i * 16 + 4 * p;
        af[i] = tr_frag(As + tr_off<BM>(kr, cm), As + tr_off<BM>(kr + 4, cm));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int cn = wc * WN + j * 16 + 4 * p;
        bfr[j] = tr_frag(Bs + tr_off<BN>(kr, cn), Bs + tr_off<BN>(kr + 4, cn));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    __syncthreads();
    if (t + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
  float* Ps = P + (int64_t)split * Mo * No;
  const int fr = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * WM + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wc * WN + j * 16 + fr;
        if (m < Mo && n < No) Ps[(int64_t)m * No + n] = acc[i][j][r];
      }
}

// Sums the split-K fp32 slabs: each thread owns 4 consecutive outputs (one 16-byte load per slab)
// and keeps 4 slabs in flight, so the loop is bandwidth- rather than latency-bound.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ P, int splits, int64_t n,
                                                            T* __restrict__ out, float scale, int accumulate) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    float4_t a0{0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int k = 0;
    for (; k + 3 < splits; k += 4) {
      a0 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 0) * n)[v];
      a1 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 1) * n)[v];
      a2 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 2) * n)[v];
      a3 += reinterpret_cast<const float4_t*>(P + (int64_t)(k + 3) * n)[v];
    }
    for (; k < splits; ++k) a0 += reinterpret_cast<const float4_t*>(P + (int64_t)k * n)[v];
    const float4_t s = ((a0 + a1) + (a2 + a3)) * scale;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o = s[j];
      if (accumulate) o += Cvt<T>::to_f32(out[v * 4 + j]);
      out[v * 4 + j] = Cvt<T>::from_f32(o);
    }
  }
  if (blockIdx.x == 0) {  // tail (n % 4)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float o = 0.f;
      for (int k = 0; k < splits; ++k) o += P[(int64_t)k * n + i];
      o *= scale;
      if (accumulate) o += Cvt<T>::to_f32(out[i]);
      out[i] = Cvt<T>::from_f32(o);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, bool S, bool BT>
static void launch_nt(const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb, bf16_t* C, int64_t ldc, int M,
                      int N, int K, float* stats, const bf16_t* D, int64_t ldd, hipStream_t stream) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  size_t ab = ((size_t)BM * (kBK + 8) + (BT ? (size_t)kBK * BN : (size_t)BN * (kBK + 8))) * sizeof(bf16_t);
  size_t cs = (size_t)BM * (BN + 8) * sizeof(bf16_t) + (S ? (size_t)kGemmThreads / BN * BN * 2 * sizeof(float) : 0);
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, S, BT>), dim3(tiles), dim3(kGemmThreads), std::max(ab, cs), stream, A, lda, B,
                     ldb, C, ldc, M, N, K, stats, D, ldd);
}

int gemm_nt_row_block(int M, int N) {
  (void)M;
  return 128;  // BM of every shipped tile config
}

void launch_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                    float* stats, hipStream_t stream, const void* addend, int64_t ld_addend, bool b_kmajor) {
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
  bf16_t* c = (bf16_t*)C;
  const bf16_t* d = (const bf16_t*)addend;
#define DLA_NT(BN_, S_, BT_) launch_nt<128, BN_, S_, BT_>(a, lda, b, ldb, c, ldc, M, N, K, stats, d, ld_addend, stream)
#define DLA_NT_BT(BN_, S_) \
  if (b_kmajor) DLA_NT(BN_, S_, true); else DLA_NT(BN_, S_, false);
  if (N <= 64) {
    if (stats) { DLA_NT_BT(64, true) } else { DLA_NT_BT(64, false) }
  } else {
    if (stats) { DLA_NT_BT(128, true) } else { DLA_NT_BT(128, false) }
  }
#undef DLA_NT_BT
#undef DLA_NT
}

int gemm_tn_splits(int Mo, int No, int K) {
  // ~512 workgroups in flight (2 per CU) and >= 16 K-steps per split: enough parallelism for the
  // long M reduction while keeping the fp32 slab traffic (splits * Mo * No * 4 B) small.
  const int tiles = ((Mo + 127) / 128) * ((No + 127) / 128);
  int splits = std::max(1, 512 / std::max(1, tiles));
  const int max_splits = std::max(1, K / (16 * kBK));
  return std::max(1, std::min(splits, max_splits));
}

void launch_gemm_tn(const void* A, int64_t lda, const void* B, int64_t ldb, float* partial, int splits, int Mo, int No,
                    int K, void* out, int out_dtype, float scale, bool accumulate, hipStream_t stream) {
  int kps = (K + splits - 1) / splits;
  kps = (kps + kBK - 1) / kBK * kBK;
  const int tiles = ((Mo + 127) / 128) * ((No + 127) / 128);
  const size_t lds = (size_t)kBK * (128 + 128) * sizeof(bf16_t);
  hipLaunchKernelGGL((gemm_tn_kernel<128, 128>), dim3(tiles, splits), dim3(kGemmThreads), lds, stream,
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, partial, Mo, No, K, kps);
  const int64_t n = (int64_t)Mo * No;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, 2048));
  if (out_dtype == kF32)
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(grid), dim3(256), 0, stream, partial, splits, n, (float*)out,
                       scale, (int)accumulate);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<bf16_t>, dim3(grid), dim3(256), 0, stream, partial, splits, n,
                       (bf16_t*)out, scale, (int)accumulate);
}

}  // namespace dla
