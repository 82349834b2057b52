// Shared bf16 MFMA GEMM machinery (gfx950): operand loaders, LDS images, the register-staged main
// loop and the epilogues. gemm.hip (1x1 convolutions / plain GEMMs) and conv.hip (implicit-GEMM
// 3x3 convolutions) instantiate the same main loop with different global-memory loaders, so every
// conv variant inherits the tuned tile schedule instead of re-implementing it.
//
// Block = NT threads = (NT/128) x 2 waves (NT = 256: 2x2, NT = 512: 4x2); a block computes a BM x BN tile of C with
// v_mfma_f32_16x16x32_bf16 (fp32 accumulate), kBK = 64 deep K steps staged through LDS with the
// next step's global loads in flight during the current step's MFMAs (T14 register staging).
// Operand tiles live in LDS either
//   * row-major  [W][kBK] (operand is K-contiguous in memory; fragments by ds_read_b128 from
//                               XOR-swizzled 16-byte chunks -> conflict-free; DLA_RM_SWIZZLE), or
//   * k-major    [kBK][W]      (operand is K-strided; fragments by ds_read_b64_tr_b16 through the
//                               XOR-swizzled tr_off image -> conflict-free).
// C/D fragment map of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + reg.
#pragma once

#include "dla_common.h"

namespace dla {
namespace mm {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));

// n / d for n < 2^24, d < 2^16: floor(n * ceil(2^40 / d) / 2^40), 4 VALU ops.
struct FastDiv {
  uint32_t d, m_lo, m_hi;
};
__host__ __device__ inline FastDiv make_fastdiv(uint32_t d) {
  const uint64_t m = ((1ull << 40) + d - 1) / d;
  return FastDiv{d, (uint32_t)m, (uint32_t)(m >> 32)};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m_lo) + n * f.m_hi) >> 8;
}

constexpr int kThreads = 256;
// Register-staged row-major operand tiles: 1 = the XOR-swizzled 128-byte rows of the LDS-DMA image, 0 = rows
// padded by 16 B. The padding assumed 16 contiguous lanes per ds_read_b128 cycle; the instruction's lane groups
// are {0-3, 12-15, 20-27}, ..., on which the padded rows pair up 2-way (profiles/r5/g32: 3.6e8 conflict cycles
// in the 128x128 1x1 GEMM); the swizzled rows hit 16 distinct 16-byte slots.
#ifndef DLA_RM_SWIZZLE
#define DLA_RM_SWIZZLE 1
#endif
#ifndef DLA_EPI_SWZ
#define DLA_EPI_SWZ 1  // epilogue_bf16 C staging layout (1 = swizzled unpadded rows, 0 = padded rows)
#endif

constexpr int kBK = 64;

// GEMM epilogues load their addends for all of a thread's rows before the store loop (1), or per row
// inside it (0; build-time A/B: python -m distributed_learning_amd._build -D DLA_EPI_PRELOAD=0 --out ...)
#ifndef DLA_EPI_PRELOAD
#define DLA_EPI_PRELOAD 1
#endif
// transposing operand reads combined by vector concatenation (1) or element-wise (0; build-time A/B)
#ifndef DLA_TR_CONCAT
#define DLA_TR_CONCAT 1
#endif

// resident blocks per CU a kernel is compiled for: 2 for the 4-wave 128x128-or-smaller tiles
// (64 KB of 2-stage LDS each), 1 for the 8-wave tiles and the 4-wave 256x128 / 128x256 tiles
// (3-stage LDS-DMA at 144 KB)
__host__ __device__ constexpr int blocks_per_cu(int BM, int BN, int NT) {
  return (NT == kThreads && BM * BN <= 128 * 128) ? 2 : 1;
}

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// MFMA shape of every GEMM / conv main loop (build-time: -DDLA_MFMA_SHAPE=32 selects
// v_mfma_f32_32x32x16_bf16; default v_mfma_f32_16x16x32_bf16). Same wave tiles and LDS images;
// a 32x32x16 MFMA issues half as many instructions for the same work, so per k-step a wave leaves
// 3x more vector-issue slots free for address / epilogue VALU (MI355X_MICROARCH.md cycle table).
#ifndef DLA_MFMA_SHAPE
#define DLA_MFMA_SHAPE 16
#endif
constexpr int kMS = DLA_MFMA_SHAPE;       // output tile edge of one MFMA
constexpr int kKS = 512 / kMS;            // K of one MFMA (32 or 16)
constexpr int kAccN = kMS * kMS / 64;     // fp32 accumulators per lane (4 or 16)
static_assert(kMS == 16 || kMS == 32, "MFMA shape 16 or 32");
typedef float accv_t __attribute__((ext_vector_type(kAccN)));
__device__ __forceinline__ accv_t mfma(const bf16x8_t& a, const bf16x8_t& b, const accv_t& c) {
#if DLA_MFMA_SHAPE == 16
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}
// Main loops compute acc[i][j] += A-frag i x B-frag j (kT = false: output rows = A rows) or, with kT, the
// transposed product B-frag j x A-frag i (output rows = B rows, e.g. a 1x1 conv's channels, columns = A rows,
// its pixels): a lane then holds 4 consecutive channels of one pixel per fragment (gemm_direct.hip).
template <bool kT>
__device__ __forceinline__ accv_t mfma_t(const bf16x8_t& a, const bf16x8_t& b, const accv_t& c) {
  if constexpr (kT) return mfma(b, a, c);
  else return mfma(a, b, c);
}
// C/D fragment position of accumulator register `reg` of `lane` (16x16x32: col = lane & 15,
// row = 4 * (lane >> 4) + reg; 32x32x16: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5))
__device__ __forceinline__ int acc_row(int lane, int reg) {
  if constexpr (kMS == 16) return 4 * (lane >> 4) + reg;
  else return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int lane) { return lane & (kMS - 1); }

__device__ __forceinline__ ushort8_t zero8() { return ushort8_t{0, 0, 0, 0, 0, 0, 0, 0}; }

// k-major image (rows = k, W = 64 or 128 columns, unpadded rows). A 32-lane half of a transposed
// 16x16x32-operand read touches rows {r..r+3, r+8..r+11} x 4 consecutive 8-byte chunks; with plain
// rows those 8 row-blocks share banks (2-way or worse for any constant pitch). XOR-ing the chunk
// index with a row-dependent multiple of 4 gives them disjoint 8-bank windows, keeps every 32-byte
// chunk group and every 16-byte store contiguous; stores and reads share this function.
template <int W>
__device__ __forceinline__ int tr_sw(int row) {  // XOR applied to the 8-byte chunk index of a row
  static_assert(W == 64 || W == 128 || W == 256, "tr image width");
  if constexpr (kMS == 32) {
    // 32x32x16 transposed reads: a 32-lane half touches rows {r..r+3} x 8 consecutive chunks; give
    // the 4 rows disjoint 8-chunk windows (64-B rows pair up in a bank row at W = 64)
    if constexpr (W >= 128) return 8 * (row & 3);
    else return 8 * ((row >> 1) & 1);
  }
  // 256 columns (512 B rows): every row starts on bank 0 as with 128, so the same XOR pattern
  // (it stays inside each 32-chunk half) keeps the transposed reads conflict-free
  if constexpr (W >= 128)
    return 4 * ((row & 3) | (((row >> 3) & 1) << 2));  // 32 chunks/row (256 B = 64 banks)
  else
    return 4 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));  // 16 chunks/row; row parity adds 32 banks
}
template <int W>
__device__ __forceinline__ int tr_off(int row, int col) {  // element offset of (row, col), col % 4 == 0
  return row * W + (((col >> 2) ^ tr_sw<W>(row)) << 2);
}

__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* lo_ptr, const bf16_t* hi_ptr) {
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(lo_ptr));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(hi_ptr));
#if DLA_TR_CONCAT
  // a vector concatenation, not an element-wise copy: the element form made hipcc emit a v_bfi_b32 on
  // each freshly loaded register, i.e. an lgkmcnt wait right behind every read
  return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#else
  const short v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return *reinterpret_cast<const bf16x8_t*>(v);
#endif
}

template <int W, int NT = kThreads>
struct TileGeom {
  static constexpr int CH = W * kBK / 8 / NT;  // 16-byte chunks per thread per k-step
  static_assert(CH >= 1, "tile too small for the block's threads");
  static constexpr int KPR = W / 8;  // k-major: chunks per k-row
  // row-major: chunk c -> (row c >> 3, k (c & 7) * 8); k-major: chunk c -> (k c / KPR, col (c % KPR) * 8)
  static constexpr int kRowElems = W * (kBK + 8);
  static constexpr int kKElems = kBK * W;
};

// ---- LDS-DMA (global_load_lds) staging ---------------------------------------------------------
// With LDS-DMA the tile bytes go HBM/L2 -> LDS without touching VGPRs, so several k-steps can be in
// flight (the register-staged loop holds exactly one). The DMA writes each wave-instruction's 64 x
// 16 B lane-linearly (wave-uniform base + 16 * lane): chunk slot c of a tile always lands at byte
// 16 * c, and the loaders choose WHICH logical 16 B each lane fetches so that this linear image is
// the swizzled one the fragment reads expect (cdna_hip_programming.md §5 'Async global->LDS copy').
//   row-major image: row = c >> 3, physical chunk c & 7 holds logical chunk (c & 7) ^ ((row >> 1) & 7)
//                    (16 rows of a ds_read_b128 fragment hit 16 distinct 16-byte bank slots);
//   k-major image:   the tr_off image above (row = c / KPR, logical column from the inverse XOR).
// Out-of-range chunks (tile edges, conv padding) read a zero page instead of being masked.
static __device__ __attribute__((aligned(64))) uint32_t g_zero_page[16];

__device__ __forceinline__ const void* zero_src() { return g_zero_page; }

__device__ __forceinline__ int rm_glds_kc(int c) { return (((c & 7) ^ ((c >> 4) & 7)) << 3); }  // logical k
template <int W>
__device__ __forceinline__ int km_glds_col(int c) {  // logical column of chunk c in the k-major image
  const int kr = c / TileGeom<W>::KPR;
  return ((((c % TileGeom<W>::KPR) << 1) ^ tr_sw<W>(kr)) << 2);
}

// one 16-byte LDS-DMA per lane; lds_byte is the wave-uniform destination of lane 0. The asm hides
// the load from hipcc's waitcnt bookkeeping (it would drain it with vmcnt(0) before every ds_read);
// completion is tracked by the explicit vm_wait<N>() + barrier in the main loop. M0 is saved and
// restored inside the statement (§5.7).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_byte) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_byte)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- buffer LDS-DMA (buffer_load_dwordx4 ... offen lds) -----------------------------------------
// The v3 pipeline (PIPE 6 / 7) addresses operands through a buffer resource descriptor: each chunk
// slot keeps ONE 32-bit byte offset for the whole block (VGPR), the k-step advance is a scalar
// soffset, and out-of-range slots carry an offset past num_records so the hardware returns zeros.
// Per k-step a RowLoader / KLoader operand then costs no VALU at all (the global_load_lds form
// needs a 64-bit add and two selects per chunk), which is what makes the MFMA loop issue-bound
// otherwise: two 4-wave blocks per CU spend ~1 vector-issue slot of every 2 on address math.
constexpr uint32_t kOOB = 0x80000000u;  // every operand is < 2 GiB (checked on the host)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// CH slots, LDS destination of slot i = lds + i * STRIDE (wave-uniform), one statement: M0 saved
// once, written per slot (s_nop 0 before each DMA), restored; s_nop 4 lets a freshly computed
// scalar soffset settle before the first buffer op reads it. The M0 advance (s_add_u32) writes SCC,
// which the statement must declare: hipcc otherwise keeps a branch condition in SCC across it (seen
// in gemm_stream_kernel<64, 2, ...>: the q % KC == KC - 1 test read the add's carry, so every tile
// after the peeled prologue skipped its stores).
template <int CH, int STRIDE>
__device__ __forceinline__ void bglds(const uint32_t (&vo)[CH], __amdgpu_buffer_rsrc_t srd, uint32_t soff,
                                      uint32_t lds) {
  uint32_t keep;
  if constexpr (CH == 1) {
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(vo[0]), "s"(srd), "s"(lds), "s"(soff) : "memory");
  } else if constexpr (CH == 2) {
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %3, %5 offen lds\n\t"
        "s_add_u32 m0, m0, %6\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %5 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(vo[0]), "v"(vo[1]), "s"(srd), "s"(lds), "s"(soff), "i"(STRIDE) : "memory", "scc");
  } else if constexpr (CH == 4) {
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %5, %7 offen lds\n\t"
        "s_add_u32 m0, m0, %8\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %5, %7 offen lds\n\t"
        "s_add_u32 m0, m0, %8\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %5, %7 offen lds\n\t"
        "s_add_u32 m0, m0, %8\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %5, %7 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "s"(srd), "s"(lds), "s"(soff), "i"(STRIDE)
        : "memory", "scc");
  } else {
    static_assert(CH == 8, "1, 2, 4 or 8 slots");
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %10\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %5, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %6, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %7, %9, %11 offen lds\n\t"
        "s_add_u32 m0, m0, %12\n\ts_nop 0\n\tbuffer_load_dwordx4 %8, %9, %11 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "v"(vo[5]), "v"(vo[6]), "v"(vo[7]),
          "s"(srd), "s"(lds), "s"(soff), "i"(STRIDE)
        : "memory", "scc");
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// ---- loaders ------------------------------------------------------------------------------------
// A loader exposes kKMajor and  ushort8_t load(int i, int k0) const  returning the 8 elements of
// chunk slot i (chunk id c = tid + i * NT) for the k-step starting at k0, zeros out of range
// (register-staged loop), and  src(i, k0)  = the global address of that chunk or the zero page
// (LDS-DMA loop). prep() runs once per tile before the LDS-DMA loop and hoists everything that
// does not depend on k0 (row/column bounds, 64-bit row bases), so the per-k-step address of a
// chunk is one 64-bit add of a wave-uniform offset plus a select.

// Row-major matrix [rows][K] (K contiguous): A of gemm_nt, B of gemm_nt (weights [N][K]).
template <int W, int NT = kThreads>
struct RowLoader {
  static constexpr bool kKMajor = false;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* p;
  int64_t ld;
  int64_t row0, rows;
  int K;
  const bf16_t* sp[CH];
  int skc[CH];  // logical k offset of the slot, or INT_MAX / 2 when its row is out of range
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, r = c >> 3, kc = (c & 7) * 8;
    const int64_t gr = row0 + r;
    return (gr < rows && k0 + kc < K) ? *reinterpret_cast<const ushort8_t*>(p + gr * ld + k0 + kc) : zero8();
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, kc = rm_glds_kc(c);
      const int64_t gr = row0 + r;
      const bool ok = gr < rows;
      sp[i] = p + (ok ? gr * ld : 0) + kc;
      skc[i] = ok ? kc : (1 << 30);
    }
  }
  __device__ const void* src(int i, int k0) const {
    return (k0 + skc[i] < K) ? (const void*)(sp[i] + k0) : zero_src();
  }
  // buffer form (PIPE 6/7): byte offset of slot i at k0 = 0; soffset = 2 * k0
  uint32_t bvo[CH];
  __amdgpu_buffer_rsrc_t bsrd;
  __device__ void bprep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, r = c >> 3, kc = rm_glds_kc(c);
      const int64_t gr = row0 + r;
      bvo[i] = gr < rows ? (uint32_t)((gr * ld + kc) * 2) : kOOB;
    }
    bsrd = make_srd(p, (uint32_t)(rows * ld * 2));
  }
  __device__ uint32_t bsoff(int k0) const { return (uint32_t)k0 * 2u; }
  __device__ bool bcheck(int k0) const { return k0 + kBK > K; }  // K tail: per-slot k bound
  __device__ uint32_t bvoff_chk(int i, int k0) const {
    return (k0 + rm_glds_kc(threadIdx.x + i * NT) < K) ? bvo[i] : kOOB;
  }
};

// k-major matrix [K][cols] (cols contiguous): gemm_tn operands, dgrad weights as stored.
template <int W, int NT = kThreads>
struct KLoader {
  static constexpr bool kKMajor = true;
  static constexpr int kNT = NT;
  static constexpr int CH = TileGeom<W, NT>::CH;
  const bf16_t* p;
  int64_t ld;
  int col0, cols;
  int kend;
  const bf16_t* sp[CH];
  int skr[CH];  // k row of the slot, or INT_MAX / 2 when its column is out of range
  __device__ ushort8_t load(int i, int k0) const {
    const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR, nc = (c % TileGeom<W>::KPR) * 8;
    const int gk = k0 + kr, gc = col0 + nc;
    return (gk < kend && gc < cols) ? *reinterpret_cast<const ushort8_t*>(p + (int64_t)gk * ld + gc) : zero8();
  }
  __device__ void prep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
      const int gc = col0 + km_glds_col<W>(c);
      const bool ok = gc < cols;
      sp[i] = p + (int64_t)kr * ld + (ok ? gc : 0);
      skr[i] = ok ? kr : (1 << 30);
    }
  }
  __device__ const void* src(int i, int k0) const {
    return (k0 + skr[i] < kend) ? (const void*)(sp[i] + (int64_t)k0 * ld) : zero_src();
  }
  // buffer form (PIPE 6/7): byte offset of slot i at k0 = 0; soffset = 2 * k0 * ld
  uint32_t bvo[CH];
  __amdgpu_buffer_rsrc_t bsrd;
  __device__ void bprep() {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = threadIdx.x + i * NT, kr = c / TileGeom<W>::KPR;
      const int gc = col0 + km_glds_col<W>(c);
      bvo[i] = gc < cols ? (uint32_t)(((int64_t)kr * ld + gc) * 2) : kOOB;
    }
    bsrd = make_srd(p, (uint32_t)((int64_t)kend * ld * 2));
  }
  __device__ uint32_t bsoff(int k0) const { return (uint32_t)((int64_t)k0 * ld * 2); }
  __device__ bool bcheck(int k0) const { return k0 + kBK > kend; }
  __device__ uint32_t bvoff_chk(int i, int k0) const {
    return (k0 + (threadIdx.x + i * NT) / TileGeom<W>::KPR < kend) ? bvo[i] : kOOB;
  }
};

// ---- main loop -----------------------------------------------------------------------------------
// Waves along N of a block: 2 (and NT/128 along M), or 1 for the 256 x 64 tile, whose 4 waves stack
// along M so each owns a 64 x 64 wave tile like the 128 x 128 tile (a 2 x 2 layout of a 64-wide tile
// gives 64 x 32 wave tiles: a third more LDS fragment reads per MFMA).
__host__ __device__ constexpr int waves_n(int BM, int BN, int NT) { return (BN <= 64 && BM >= 256 && NT == 256) ? 1 : 2; }

template <int BM, int BN, int NT = kThreads>
struct Acc {
  static constexpr int kNT = NT, WGN = waves_n(BM, BN, NT), WGM = NT / 64 / WGN;  // waves along N / M
  static constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / kMS, TN = WN / kMS;
  static_assert(TM >= 1 && TN >= 1, "wave tile below one MFMA fragment");
  accv_t v[TM][TN];
  __device__ void zero() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) v[i][j] = accv_t{};
  }
};

template <int BM, int BN, class LA, class LB>
__host__ __device__ constexpr size_t mainloop_lds_bytes() {
  return ((LA::kKMajor ? (size_t)kBK * BM : (size_t)BM * (kBK + 8)) +
          (LB::kKMajor ? (size_t)kBK * BN : (size_t)BN * (kBK + 8))) * sizeof(bf16_t);
}

template <int W, class L>
__device__ __forceinline__ void tile_store(bf16_t* s, const ushort8_t (&r)[TileGeom<W, L::kNT>::CH]) {
#pragma unroll
  for (int i = 0; i < TileGeom<W, L::kNT>::CH; ++i) {
    const int c = threadIdx.x + i * L::kNT;
    if constexpr (L::kKMajor)
      *reinterpret_cast<ushort8_t*>(s + tr_off<W>(c / TileGeom<W>::KPR, (c % TileGeom<W>::KPR) * 8)) = r[i];
    else if constexpr (DLA_RM_SWIZZLE)  // the LDS-DMA row-major image (rm_glds_frag reads it)
      *reinterpret_cast<ushort8_t*>(s + (c >> 3) * kBK + (((c & 7) ^ ((c >> 4) & 7)) << 3)) = r[i];
    else
      *reinterpret_cast<ushort8_t*>(s + (c >> 3) * (kBK + 8) + (c & 7) * 8) = r[i];
  }
}

// kMS x kKS operand fragment for MFMA rows/cols [r0, r0 + kMS) at k offset kk * kKS.
template <int W, class L>
__device__ __forceinline__ bf16x8_t tile_frag(const bf16_t* s, int r0, int kk) {
  const int lane = threadIdx.x & 63;
  if constexpr (L::kKMajor) {
    // lane 4q+p of 16-lane group g reads k-rows (kbase + q, + 4), columns c + 4p..+3 (T10)
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    int kr, cn;
    if constexpr (kMS == 16) {
      kr = kk * 32 + 8 * g + q;
      cn = r0 + 4 * p;
    } else {
      kr = kk * 16 + 8 * (g >> 1) + q;
      cn = r0 + 16 * (g & 1) + 4 * p;
    }
    return tr_frag(s + tr_off<W>(kr, cn), s + tr_off<W>(kr + 4, cn));
  } else {
    if constexpr (DLA_RM_SWIZZLE) {
      const int r = r0 + (lane & (kMS - 1)), lc = kk * (kKS / 8) + lane / kMS;
      return *reinterpret_cast<const bf16x8_t*>(s + r * kBK + ((lc ^ ((r >> 1) & 7)) << 3));
    }
    return *reinterpret_cast<const bf16x8_t*>(s + (r0 + (lane & (kMS - 1))) * (kBK + 8) + kk * kKS +
                                              8 * (lane / kMS));
  }
}

// acc += A[BM rows, k in [kbeg, kend)] * B[BN cols, same k]^T
template <int BM, int BN, int NT, bool kT = false, class LA, class LB>
__device__ __forceinline__ void mainloop(const LA& la, const LB& lb, int kbeg, int kend, Acc<BM, BN, NT>& acc,
                                         char* smem) {
  static_assert(LA::kNT == NT && LB::kNT == NT, "loaders built for another block size");
  using GA = TileGeom<BM, NT>;
  using GB = TileGeom<BN, NT>;
  using AC = Acc<BM, BN, NT>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + (LA::kKMajor ? GA::kKElems : GA::kRowElems);
  const int wid = threadIdx.x >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN;
  ushort8_t ra[GA::CH], rb[GB::CH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < GA::CH; ++i) ra[i] = la.load(i, k0);
#pragma unroll
    for (int i = 0; i < GB::CH; ++i) rb[i] = lb.load(i, k0);
  };
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk <= 0) return;
  gload(kbeg);
  tile_store<BM, LA>(As, ra);
  tile_store<BN, LB>(Bs, rb);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) gload(kbeg + (t + 1) * kBK);  // next tile in flight during this tile's MFMAs
#pragma unroll
    for (int kk = 0; kk < kBK / kKS; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tile_frag<BM, LA>(As, wr * WM + i * kMS, kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tile_frag<BN, LB>(Bs, wc * WN + j * kMS, kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc.v[i][j] = mfma_t<kT>(af[i], bfr[j], acc.v[i][j]);
    }
    __syncthreads();
    if (t + 1 < nk) {
      tile_store<BM, LA>(As, ra);
      tile_store<BN, LB>(Bs, rb);
      __syncthreads();
    }
  }
}

// 16 x 32 row-major operand fragment from the LDS-DMA image (see the image map above)
__device__ __forceinline__ bf16x8_t rm_glds_frag(const bf16_t* s, int r0, int kk) {
  const int lane = threadIdx.x & 63;
  const int r = r0 + (lane & (kMS - 1)), lc = kk * (kKS / 8) + lane / kMS;
  return *reinterpret_cast<const bf16x8_t*>(s + r * kBK + ((lc ^ ((r >> 1) & 7)) << 3));
}

template <int W, class L>
__device__ __forceinline__ bf16x8_t glds_frag(const bf16_t* s, int r0, int kk) {
  if constexpr (L::kKMajor) return tile_frag<W, L>(s, r0, kk);  // same tr_off image
  else return rm_glds_frag(s, r0, kk);
}

template <int BM, int BN, int NS>
__host__ __device__ constexpr size_t glds_lds_bytes() {
  return (size_t)NS * (BM + BN) * kBK * sizeof(bf16_t);
}

// NS-stage LDS-DMA pipeline: tiles t+1 .. t+NS-1 are in flight while tile t is multiplied; one
// barrier per k-step. Iteration t: wait until this wave's DMAs for tile t are done (the younger
// stages may stay outstanding: counted vmcnt), barrier (everyone's tile t has landed AND everyone
// finished tile t-1, whose stage the next DMA overwrites), issue tile t+NS-1, multiply tile t.
template <int BM, int BN, int NT, int NS, bool kT = false, class LA, class LB>
__device__ __forceinline__ void mainloop_glds(const LA& la, const LB& lb, int kbeg, int kend, Acc<BM, BN, NT>& acc,
                                              char* smem) {
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  static_assert(LA::kNT == NT && LB::kNT == NT, "loaders built for another block size");
  using GA = TileGeom<BM, NT>;
  using GB = TileGeom<BN, NT>;
  using AC = Acc<BM, BN, NT>;
  constexpr int L = GA::CH + GB::CH;  // DMA instructions per wave per tile
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  constexpr int SA = BM * kBK, SB = BN * kBK;  // elements per stage
  bf16_t* base = reinterpret_cast<bf16_t*>(smem);
  const int wave = threadIdx.x >> 6, wr = wave / AC::WGN, wc = wave % AC::WGN;
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk <= 0) return;
  LA pa = la;
  LB pb = lb;
  pa.prep();
  pb.prep();
  auto issue = [&](int t) {
    const int st = t % NS;
    const int k0 = kbeg + t * kBK;
    const uint32_t a_base = lds0 + (uint32_t)(st * (SA + SB)) * 2u + wofs;
    const uint32_t b_base = a_base + (uint32_t)SA * 2u;
#pragma unroll
    for (int i = 0; i < GA::CH; ++i) glds16(pa.src(i, k0), a_base + (uint32_t)(i * NT * 16));
#pragma unroll
    for (int i = 0; i < GB::CH; ++i) glds16(pb.src(i, k0), b_base + (uint32_t)(i * NT * 16));
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) issue(p);
  for (int t = 0; t < nk; ++t) {
    if constexpr (NS == 3) {
      if (t + 1 < nk) vm_wait<L>();
      else vm_wait<0>();
    } else {
      vm_wait<0>();
    }
    // every LDS read this wave issued for tile t-1 has RETURNED before the barrier: the DMA issued
    // right after it overwrites that stage, and with an L2-hot source (the stem's folded image, the
    // weights) it can land while a read that was merely issued is still queued in the LDS pipeline
    // (measured: 2 of 30 stem launches read the new tile without this wait)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS read of tile t above the barrier
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const bf16_t* As = base + (t % NS) * (SA + SB);
    const bf16_t* Bs = As + SA;
#pragma unroll
    for (int kk = 0; kk < kBK / kKS; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = glds_frag<BM, LA>(As, wr * WM + i * kMS, kk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = glds_frag<BN, LB>(Bs, wc * WN + j * kMS, kk);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc.v[i][j] = mfma_t<kT>(af[i], bfr[j], acc.v[i][j]);
    }
  }
  __syncthreads();  // every wave done with the stages before the epilogue reuses the LDS
}

// Optional per-k-step loader hook: loaders whose chunk addresses share wave-uniform per-k-step
// terms (implicit-GEMM taps, weight-tap offsets) compute them once in step(k0), so src() is only
// an add and a select per chunk instead of re-deriving the tap under an exec-masked branch.
template <class L>
__device__ __forceinline__ auto loader_step(L& l, int k0, int) -> decltype(l.step(k0), void()) {
  l.step(k0);
}
template <class L>
__device__ __forceinline__ void loader_step(L&, int, long) {}
template <class L>
__device__ __forceinline__ auto loader_src(const L& l, int i, int, int) -> decltype(l.src2(i)) {
  return l.src2(i);
}
template <class L>
__device__ __forceinline__ const void* loader_src(const L& l, int i, int k0, long) {
  return l.src(i, k0);
}

// NS-stage LDS-DMA pipeline, v2 schedule (PIPE 4 = 2 stages, 5 = 3 stages): the next tile's DMA is
// split around the two 32-deep MFMA clusters of a k-step (A-tile pieces before the first, B-tile
// pieces between them) so the DMA issue no longer stalls the head of the k-step, per-k-step loader
// terms are hoisted (loader_step), and each MFMA cluster runs at s_setprio 1 so a co-resident
// wave's VALU/DMA issue does not preempt it (cdna_hip_programming.md T5). Same LDS images, same
// counted-vmcnt + raw-barrier protocol as mainloop_glds.
// The MFMAs of one staged k-step (kBK / kKS = 2 halves); mid() runs between the halves (the B-operand DMA of a
// later stage). (Reading both halves' fragments before the first half's MFMAs measured no faster in these
// two-waves-per-SIMD loops and was removed: profiles/r5/g18.)
template <int BM, int BN, int NT, class LA, class LB, bool kT = false, class Mid>
__device__ __forceinline__ void kstep_mfma(const bf16_t* As, const bf16_t* Bs, int wr, int wc, Acc<BM, BN, NT>& acc,
                                           Mid&& mid) {
  using AC = Acc<BM, BN, NT>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN, KK = kBK / kKS;
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    bf16x8_t af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = glds_frag<BM, LA>(As, wr * WM + i * kMS, kk);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = glds_frag<BN, LB>(Bs, wc * WN + j * kMS, kk);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc.v[i][j] = mfma_t<kT>(af[i], bfr[j], acc.v[i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (kk == 0) mid();
  }
}

template <int BM, int BN, int NT, int NS, bool kT = false, class LA, class LB>
__device__ __forceinline__ void mainloop_glds2(const LA& la, const LB& lb, int kbeg, int kend, Acc<BM, BN, NT>& acc,
                                               char* smem) {
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  static_assert(LA::kNT == NT && LB::kNT == NT, "loaders built for another block size");
  using GA = TileGeom<BM, NT>;
  using GB = TileGeom<BN, NT>;
  using AC = Acc<BM, BN, NT>;
  constexpr int L = GA::CH + GB::CH;  // DMA instructions per wave per tile
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  constexpr int SA = BM * kBK, SB = BN * kBK;  // elements per stage
  bf16_t* base = reinterpret_cast<bf16_t*>(smem);
  const int wave = threadIdx.x >> 6, wr = wave / AC::WGN, wc = wave % AC::WGN;
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk <= 0) return;
  LA pa = la;
  LB pb = lb;
  pa.prep();
  pb.prep();
  auto issue_a = [&](int t) {
    const int k0 = kbeg + t * kBK;
    loader_step(pa, k0, 0);
    const uint32_t a_base = lds0 + (uint32_t)((t % NS) * (SA + SB)) * 2u + wofs;
#pragma unroll
    for (int i = 0; i < GA::CH; ++i) glds16(loader_src(pa, i, k0, 0), a_base + (uint32_t)(i * NT * 16));
  };
  auto issue_b = [&](int t) {
    const int k0 = kbeg + t * kBK;
    loader_step(pb, k0, 0);
    const uint32_t b_base = lds0 + (uint32_t)((t % NS) * (SA + SB) + SA) * 2u + wofs;
#pragma unroll
    for (int i = 0; i < GB::CH; ++i) glds16(loader_src(pb, i, k0, 0), b_base + (uint32_t)(i * NT * 16));
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) {
      issue_a(p);
      issue_b(p);
    }
  for (int t = 0; t < nk; ++t) {
    if constexpr (NS == 3) {
      if (t + 1 < nk) vm_wait<L>();
      else vm_wait<0>();
    } else {
      vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR on the stage the next DMA overwrites
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = t + NS - 1 < nk;
    if (more) issue_a(t + NS - 1);
    const bf16_t* As = base + (t % NS) * (SA + SB);
    const bf16_t* Bs = As + SA;
    kstep_mfma<BM, BN, NT, LA, LB, kT>(As, Bs, wr, wc, acc, [&] {
      if (more) issue_b(t + NS - 1);
    });
  }
  __syncthreads();  // every wave done with the stages before the epilogue reuses the LDS
}

// v3 schedule (PIPE 6 = 2 stages, 7 = 3 stages): mainloop_glds2's structure with the buffer-form
// DMA (bglds): per k-step an operand costs one scalar soffset and, only where a slot can fall out
// of range this step (K tail, conv padding taps), one select per slot.
template <class L, int W, int NT>
__device__ __forceinline__ void bissue(const L& l, int k0, uint32_t lds) {
  constexpr int CH = TileGeom<W, NT>::CH;
  uint32_t vo[CH];
  if (l.bcheck(k0)) {
#pragma unroll
    for (int i = 0; i < CH; ++i) vo[i] = l.bvoff_chk(i, k0);
  } else {
#pragma unroll
    for (int i = 0; i < CH; ++i) vo[i] = l.bvo[i];
  }
  bglds<CH, NT * 16>(vo, l.bsrd, (uint32_t)__builtin_amdgcn_readfirstlane(l.bsoff(k0)), lds);
}

template <int BM, int BN, int NT, int NS, bool kT = false, class LA, class LB>
__device__ __forceinline__ void mainloop_bglds(const LA& la, const LB& lb, int kbeg, int kend, Acc<BM, BN, NT>& acc,
                                               char* smem) {
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  static_assert(LA::kNT == NT && LB::kNT == NT, "loaders built for another block size");
  using GA = TileGeom<BM, NT>;
  using GB = TileGeom<BN, NT>;
  using AC = Acc<BM, BN, NT>;
  constexpr int L = GA::CH + GB::CH;  // DMA instructions per wave per tile
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  constexpr int SA = BM * kBK, SB = BN * kBK;  // elements per stage
  bf16_t* base = reinterpret_cast<bf16_t*>(smem);
  const int wave = threadIdx.x >> 6, wr = wave / AC::WGN, wc = wave % AC::WGN;
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t wofs = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk <= 0) return;
  LA pa = la;
  LB pb = lb;
  pa.prep();
  pb.prep();
  pa.bprep();
  pb.bprep();
  auto issue_a = [&](int t) {
    const int k0 = kbeg + t * kBK;
    loader_step(pa, k0, 0);
    bissue<LA, BM, NT>(pa, k0, lds0 + (uint32_t)((t % NS) * (SA + SB)) * 2u + wofs);
  };
  auto issue_b = [&](int t) {
    const int k0 = kbeg + t * kBK;
    loader_step(pb, k0, 0);
    bissue<LB, BN, NT>(pb, k0, lds0 + (uint32_t)((t % NS) * (SA + SB) + SA) * 2u + wofs);
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) {
      issue_a(p);
      issue_b(p);
    }
  for (int t = 0; t < nk; ++t) {
    if constexpr (NS == 3) {
      if (t + 1 < nk) vm_wait<L>();
      else vm_wait<0>();
    } else {
      vm_wait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // WAR on the stage the next DMA overwrites
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = t + NS - 1 < nk;
    if (more) issue_a(t + NS - 1);
    const bf16_t* As = base + (t % NS) * (SA + SB);
    const bf16_t* Bs = As + SA;
    kstep_mfma<BM, BN, NT, LA, LB, kT>(As, Bs, wr, wc, acc, [&] {
      if (more) issue_b(t + NS - 1);
    });
  }
  __syncthreads();  // every wave done with the stages before the epilogue reuses the LDS
}

// Pipeline selection shared by all MFMA kernels: 0 = register staging (one k-step in flight,
// 3 blocks/CU), 2 / 3 = LDS-DMA with 2 / 3 stages, 4 / 5 = the v2 LDS-DMA schedule with 2 / 3 stages,
// 6 / 7 = the v3 buffer-DMA schedule with 2 / 3 stages (loaders with a buffer form only).
template <int PIPE, bool kT = false, int BM, int BN, int NT, class LA, class LB>
__device__ __forceinline__ void run_mainloop(const LA& la, const LB& lb, int kbeg, int kend, Acc<BM, BN, NT>& acc,
                                             char* smem) {
  if constexpr (PIPE == 0) mainloop<BM, BN, NT, kT>(la, lb, kbeg, kend, acc, smem);
  else if constexpr (PIPE >= 6) mainloop_bglds<BM, BN, NT, PIPE - 4, kT>(la, lb, kbeg, kend, acc, smem);
  else if constexpr (PIPE >= 4) mainloop_glds2<BM, BN, NT, PIPE - 2, kT>(la, lb, kbeg, kend, acc, smem);
  else mainloop_glds<BM, BN, NT, PIPE, kT>(la, lb, kbeg, kend, acc, smem);
}

template <int PIPE, int BM, int BN, class LA, class LB>
__host__ __device__ constexpr size_t run_mainloop_lds_bytes() {
  return PIPE == 0 ? mainloop_lds_bytes<BM, BN, LA, LB>()
                   : glds_lds_bytes<BM, BN, (PIPE >= 6 ? PIPE - 4 : (PIPE >= 4 ? PIPE - 2 : PIPE))>();
}

// ---- epilogues -------------------------------------------------------------------------------
template <int BM, int BN, bool kStats, int NT = kThreads>
__host__ __device__ constexpr size_t epilogue_lds_bytes() {
  // C staging tile; the BN-backward partial combine ([NT / (BN/8)][BN][2] floats = NT * 64 B) and
  // the statistics flush reuse the same bytes afterwards
  return (size_t)BM * (BN + 8) * sizeof(bf16_t) > (size_t)NT * 64 ? (size_t)BM * (BN + 8) * sizeof(bf16_t)
                                                                  : (size_t)NT * 64;
}

// Column statistics of a block's output tile(s): a lane owns one column of each 16x16 fragment, so
// each wave keeps TN (sum, sumsq) in registers until stats_flush.
template <int BM, int BN, int NT = kThreads>
struct ColStats {
  float s[Acc<BM, BN, NT>::TN], q[Acc<BM, BN, NT>::TN];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < Acc<BM, BN, NT>::TN; ++j) s[j] = q[j] = 0.f;
  }
};

// bf16 C tile -> LDS -> coalesced 16-byte row stores, optional fused addend D (C = bf16(bf16(acc) + D),
// exactly the unfused bf16 add); with kStats, the stored values' per-column (sum, sumsq) are added
// to `st` straight from the accumulator registers. Ends with a barrier (LDS free for the next tile).
// BatchNorm-backward statistics of a GEMM output that IS the gradient dy of a fused BN(+ReLU)
// (the dgrad of the conv that consumes the BN's output): per channel (column) the partial sums of
// dy' and dy' * (x - mean) over the tile's rows, dy' = dy masked by the BN's ReLU (recomputed from
// x with the forward's scale/shift, or read from its 1-bit mask) — exactly the BN backward's
// reduction pass, without re-reading dy from HBM. ws: the BN's 7C workspace (mean | invstd |
// scale | shift | ...); mode as launch_bn_bwd (0 none, 1 recompute, 2 bits).
struct BnBwdEpi {
  const bf16_t* x;  // null: no BN partials
  int64_t ldx;      // its row stride (0: ldc, the same layout as the GEMM output)
  const float* ws;
  const uint8_t* mask;
  int mode;
  float* part;  // [row tiles][N][2]
  // 1-bit mask for the fused addend (C = bf16(bf16(acc) + (bit ? D : 0))): the residual gradient
  // dy * relu'(out) of a fused BN(+residual)+ReLU taken straight from dy and the forward's mask,
  // so the BN backward never writes it out (null: plain addend)
  const uint8_t* dmask;
  // second, stride-2 addend: the gradient of the block input's stride-2 subsample (the downsample
  // 1x1 conv's input), compact [n][H/2][W/2][N]; added at the even pixels of the [n][H][W] rows of
  // C (null: none). Replaces a zero-filled full-size scatter of that gradient.
  const bf16_t* d2;
  int H, W;
  FastDiv fW, fH;
};

// Output row of GEMM row gm: the identity for every kernel except the stride-2 data gradient, whose
// GEMM rows are one parity class of the input pixels.
struct RowIdent {
  __device__ __forceinline__ int64_t operator()(int64_t gm) const { return gm; }
};

template <int BM, int BN, bool kStats, bool kEpi = false, int NT = kThreads, class RM = RowIdent>
__device__ __forceinline__ void epilogue_bf16(const Acc<BM, BN, NT>& acc, bf16_t* __restrict__ C, int64_t ldc,
                                              int64_t M, int N, int64_t row0, int col0, ColStats<BM, BN, NT>& st,
                                              const bf16_t* __restrict__ D, int64_t ldd, char* smem,
                                              const BnBwdEpi* epi = nullptr, int bm = 0, RM rowmap = RM()) {
  // kEpi compiles in the BN-backward partials and the masked addend (dgrad kernels only: they cost
  // VGPRs that would lower the forward kernels' occupancy)
  const BnBwdEpi* bnb = (kEpi && epi && epi->x) ? epi : nullptr;
  const uint8_t* __restrict__ dmask = (kEpi && epi) ? epi->dmask : nullptr;
  const bf16_t* __restrict__ d2 = (kEpi && epi) ? epi->d2 : nullptr;
  using AC = Acc<BM, BN, NT>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  // C staging: unpadded BN-wide rows, 16-byte chunk XOR ((m >> 2) & 1) << 1 (DLA_EPI_SWZ; else rows padded by
  // 8 elements). The fragment writes (ds_write_b16, rows m and m + 4 in one 32-lane half) then land in different
  // 32-byte units, and the row read-out (ds_read_b128 lane groups {0-3, 12-15, 20-27}, ...) covers 16 distinct
  // slots; the padded rows conflicted 2-way on the read-out (tests/test_lds_swizzle.py)
  static_assert(!DLA_EPI_SWZ || BN >= 32, "the staging XOR needs 4 chunks per row");
  constexpr int LDS_C = DLA_EPI_SWZ ? BN : BN + 8;
  auto cs_off = [](int m, int n) {
    if constexpr (DLA_EPI_SWZ) return m * BN + ((((n >> 3) ^ (((m >> 2) & 1) << 1))) << 3) + (n & 7);
    else return m * (BN + 8) + n;
  };
  (void)LDS_C;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN,
            fr = acc_col(lane);
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem);
  // accumulator registers in pairs (r, r + 1): one v_cvt_pk_bf16_f32 per pair, and the statistics of the
  // stored (bf16-rounded) values in packed fp32 (v_pk_add_f32 / v_pk_fma_f32); the per-row range test
  // only in a tile that crosses M. ~2.5 VALU per output element instead of ~11 (profiles/r5/g31/).
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  static_assert(kAccN % 2 == 0, "accumulator pairs");
  const bool full = row0 + BM <= M;
  f32x2_t ps[TN], pq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) ps[j] = pq[j] = f32x2_t{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < kAccN; r += 2) {
        const int m0 = wr * WM + i * kMS + acc_row(lane, r), m1 = wr * WM + i * kMS + acc_row(lane, r + 1);
        const int n = wc * WN + j * kMS + fr;
        const uint32_t u = __builtin_bit_cast(
            uint32_t, __builtin_convertvector((f32x2_t{acc.v[i][j][r], acc.v[i][j][r + 1]}), bf16x2_t));
        Cs[cs_off(m0, n)] = (bf16_t)(u & 0xffffu);
        Cs[cs_off(m1, n)] = (bf16_t)(u >> 16);
        if constexpr (kStats) {  // statistics of the stored values
          f32x2_t v{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
          if (!full) {
            v.x = row0 + m0 < M ? v.x : 0.f;
            v.y = row0 + m1 < M ? v.y : 0.f;
          }
          ps[j] += v;
          pq[j] = __builtin_elementwise_fma(v, v, pq[j]);
        }
      }
  if constexpr (kStats) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      st.s[j] += ps[j].x + ps[j].y;
      st.q[j] += pq[j].x + pq[j].y;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "a thread keeps one 8-column group in the store loop");
  // BN-backward partials: this thread's 8 columns are fixed (c % CPR) across its rows. The x (and
  // mask) chunks of all its rows are loaded up front, so those global loads overlap each other and
  // the C stores instead of each waiting a full round trip inside the loop.
  constexpr int NIT = BM * CPR / NT;
  static_assert(BM * CPR % NT == 0, "whole store-loop iterations");
  const int my_cc = (tid % CPR) * 8;
  float bs[8], bq[8], mean[8], sc[8], sh[8];
  ushort8_t xr[NIT];
  uint32_t mr[NIT];
  if (bnb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bs[j] = bq[j] = 0.f;
      const int gc = min(col0 + my_cc + j, N - 1);
      mean[j] = bnb->ws[gc];
      sc[j] = bnb->ws[2 * N + gc];
      sh[j] = bnb->ws[3 * N + gc];
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid + it * NT) / CPR;
      const int64_t gm = row0 + r;
      const int gn = col0 + my_cc;
      const bool ok = gm < M && gn < N;
      const int64_t off = ok ? gm * ldc + gn : 0;
      const int64_t xo = (ok && bnb->ldx) ? gm * bnb->ldx + gn : off;
      xr[it] = ok ? *reinterpret_cast<const ushort8_t*>(bnb->x + xo) : zero8();
      mr[it] = (ok && bnb->mode == 2) ? (uint32_t)bnb->mask[off >> 3] : 0xffu;
    }
  }
  // The addends (D, its mask bits, the stride-2 d2) of all this thread's rows are loaded up front too:
  // loaded inside the store loop, each row waited a full round trip for its addend before its store
  // (the ISA showed vmcnt(0) twice per row), so a dgrad epilogue cost ~2 NIT serial HBM latencies.
  ushort8_t dr[NIT], er[NIT];
  uint32_t dbr[NIT];
  bool eok[NIT];
  // build-time A/B switch (-DDLA_EPI_PRELOAD=0: per-row loads); dgrad instantiations (kEpi) only: the
  // preload arrays cost VGPRs that lowered the forward GEMMs' occupancy (+0.6 ms/step, g09)
  constexpr bool kPre = DLA_EPI_PRELOAD != 0 && kEpi;
  if (kPre && D) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid + it * NT) / CPR;
      const int64_t gm = row0 + r;
      const int gn = col0 + my_cc;
      const bool ok = gm < M && gn < N;
      dr[it] = ok ? *reinterpret_cast<const ushort8_t*>(D + gm * ldd + gn) : zero8();
      dbr[it] = (ok && dmask) ? (uint32_t)dmask[(gm * ldd + gn) >> 3] : 0xffu;
    }
  }
  if (kPre && d2) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = (tid + it * NT) / CPR;
      const int64_t gm = row0 + r;
      const int gn = col0 + my_cc;
      const uint32_t q = fdiv((uint32_t)gm, epi->fW);
      const int w = (int)gm - (int)q * epi->W;
      const uint32_t n = fdiv(q, epi->fH);
      const int h = (int)q - (int)n * epi->H;
      eok[it] = gm < M && gn < N && ((h | w) & 1) == 0;
      const int64_t r2 = ((int64_t)n * (epi->H >> 1) + (h >> 1)) * (epi->W >> 1) + (w >> 1);
      er[it] = eok[it] ? *reinterpret_cast<const ushort8_t*>(d2 + r2 * ldc + gn) : zero8();
    }
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = tid + it * NT;
    const int r = c / CPR, cc = (c % CPR) * 8;
    const int64_t gm = row0 + r;
    const int gn = col0 + cc;
    if (gm < M && gn < N) {
      ushort8_t v = *reinterpret_cast<ushort8_t*>(Cs + cs_off(r, cc));
      if (D) {
        const ushort8_t d = kPre ? dr[it] : *reinterpret_cast<const ushort8_t*>(D + gm * ldd + gn);
        const uint32_t db = kPre ? dbr[it] : (dmask ? (uint32_t)dmask[(gm * ldd + gn) >> 3] : 0xffu);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = f32_to_bf16(bf16_to_f32(v[j]) + (((db >> j) & 1u) ? bf16_to_f32(d[j]) : 0.f));
      }
      if (d2) {
        bool ok2;
        ushort8_t e;
        if constexpr (kPre) {
          ok2 = eok[it];
          e = er[it];
        } else {
          const uint32_t q = fdiv((uint32_t)gm, epi->fW);
          const int w = (int)gm - (int)q * epi->W;
          const uint32_t n = fdiv(q, epi->fH);
          const int h = (int)q - (int)n * epi->H;
          ok2 = ((h | w) & 1) == 0;
          e = ok2 ? *reinterpret_cast<const ushort8_t*>(
                        d2 + (((int64_t)n * (epi->H >> 1) + (h >> 1)) * (epi->W >> 1) + (w >> 1)) * ldc + gn)
                  : zero8();
        }
        if (ok2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) + bf16_to_f32(e[j]));
        }
      }
      *reinterpret_cast<ushort8_t*>(C + rowmap(gm) * ldc + gn) = v;
      if (bnb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = bf16_to_f32(xr[it][j]);
          float g = bf16_to_f32(v[j]);
          if (bnb->mode == 1) g = fmaf(xf, sc[j], sh[j]) > 0.f ? g : 0.f;  // same fmaf as the forward
          else if (bnb->mode == 2) g = ((mr[it] >> j) & 1u) ? g : 0.f;
          bs[j] += g;
          bq[j] = fmaf(g, xf - mean[j], bq[j]);
        }
      }
    }
  }
  __syncthreads();
  if (bnb) {
    // combine the NT / CPR row groups of each column through LDS (the C staging is free now)
    constexpr int RG = NT / CPR;
    float* red = reinterpret_cast<float*>(smem);  // [RG][BN][2]
    const int rg = tid / CPR;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(rg * BN + my_cc + j) * 2 + 0] = bs[j];
      red[(rg * BN + my_cc + j) * 2 + 1] = bq[j];
    }
    __syncthreads();
    for (int idx = tid; idx < BN * 2; idx += NT) {
      float a = 0.f;
      for (int g = 0; g < RG; ++g) a += red[g * BN * 2 + idx];
      const int col = idx >> 1;
      if (col0 + col < N) bnb->part[((int64_t)bm * N + col0 + col) * 2 + (idx & 1)] = a;
    }
    __syncthreads();
  }
}

// Register-direct epilogue for a main loop run with the transposed product (run_mainloop<PIPE, true>):
// acc.v[i][j][r] holds output row wr * WM + 16 i + p and column wc * WN + 16 j + 4 g + r (p = lane & 15,
// g = lane >> 4). One v_permlane16_swap per register pair of a fragment column pair gives every lane 8
// consecutive columns (16 bytes) of its rows, stored straight from the registers -- no C staging through LDS, no
// staging barriers (gemm_direct.hip, conv_halo.hip kDirect). With stats_row: the [N][2] (sum, sumsq) partial row of
// the tile's stored (bf16-rounded) values, summed in registers over the lane's rows, over the 16 lanes of a DPP
// row, and over the WGM M-waves through 2 * WGM * BN floats of LDS (the main loop's image bytes, free by then).
// D (optional, no statistics): C = bf16(bf16(acc) + D), the staged epilogue's unfused add, D [M][N] row stride ldd.
template <int CTRL>
__device__ __forceinline__ float epi_dpp_add(float v) {
  const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false);
  return v + __builtin_bit_cast(float, o);
}
__device__ __forceinline__ float epi_row16_sum(float v) {  // pairs {i, 15-i}, {i, 7-i}, xor 2, xor 1
  v = epi_dpp_add<0x140>(v);
  v = epi_dpp_add<0x141>(v);
  v = epi_dpp_add<0x4E>(v);
  return epi_dpp_add<0xB1>(v);
}

template <int BM, int BN, bool kStats, int NT = kThreads>
__device__ __forceinline__ void epilogue_direct(const Acc<BM, BN, NT>& acc, bf16_t* __restrict__ C, int64_t ldc,
                                                int64_t M, int N, int64_t row0, int col0,
                                                float* __restrict__ stats_row, char* smem,
                                                const bf16_t* __restrict__ D = nullptr, int64_t ldd = 0) {
  using AC = Acc<BM, BN, NT>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  static_assert(kMS == 16 && TN % 2 == 0, "16x16 fragments in column pairs");
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN;
  const int g = lane >> 4, p = lane & 15;
  const int64_t pix0 = row0 + wr * WM + p;  // + 16 i
  const int cb = col0 + wc * WN + 16 * (g & 1) + 8 * (g >> 1);  // + 32 hh: the lane's 16-byte chunks after the swap
  u32x4_t dv[kStats ? 1 : TM][TN / 2];
  if (!kStats && D) {  // every addend chunk in flight before the packing
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int hh = 0; hh < TN / 2; ++hh) {
        const int64_t m = pix0 + 16 * i;
        const int n = cb + 32 * hh;
        dv[kStats ? 0 : i][hh] = (m < M && n < N) ? *reinterpret_cast<const u32x4_t*>(D + m * ldd + n)
                                                   : u32x4_t{0u, 0u, 0u, 0u};
      }
  }
  uint32_t u[TM][TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        u[i][j][h] = __builtin_bit_cast(
            uint32_t, __builtin_convertvector((f32x2_t{acc.v[i][j][2 * h], acc.v[i][j][2 * h + 1]}), bf16x2_t));
  if constexpr (kStats) {
    float* red = reinterpret_cast<float*>(smem);  // [WGM][BN][2]
    __syncthreads();  // every wave's main-loop LDS reads are done before the bytes are reused
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s4[4], q4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sv = 0.f, qv = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint32_t w2 = u[i][j][r >> 1];
          const float f = pix0 + 16 * i < M ? __builtin_bit_cast(float, (r & 1) ? (w2 & 0xffff0000u) : (w2 << 16))
                                            : 0.f;
          sv += f;
          qv = fmaf(f, f, qv);
        }
        s4[r] = epi_row16_sum(sv);
        q4[r] = epi_row16_sum(qv);
      }
      if (p == 0) {
        float* dst = red + (wr * BN + wc * WN + 16 * j + 4 * g) * 2;
        *reinterpret_cast<float4_t*>(dst) = float4_t{s4[0], q4[0], s4[1], q4[1]};
        *reinterpret_cast<float4_t*>(dst + 4) = float4_t{s4[2], q4[2], s4[3], q4[3]};
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < AC::WGM; ++w) {
        a += red[(w * BN + c) * 2];
        b += red[(w * BN + c) * 2 + 1];
      }
      if (col0 + c < N) *reinterpret_cast<f32x2_t*>(stats_row + (int64_t)(col0 + c) * 2) = f32x2_t{a, b};
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jp = 0; jp < TN; jp += 2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto r = __builtin_amdgcn_permlane16_swap(u[i][jp][h], u[i][jp + 1][h], false, false);
        u[i][jp][h] = r[0];
        u[i][jp + 1][h] = r[1];
      }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t m = pix0 + 16 * i;
#pragma unroll
    for (int hh = 0; hh < TN / 2; ++hh) {
      const int n = cb + 32 * hh;
      u32x4_t v{u[i][2 * hh][0], u[i][2 * hh][1], u[i][2 * hh + 1][0], u[i][2 * hh + 1][1]};
      if (!kStats && D) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t d = dv[kStats ? 0 : i][hh][e];
          const float lo = __builtin_bit_cast(float, v[e] << 16) + __builtin_bit_cast(float, d << 16);
          const float hi = __builtin_bit_cast(float, v[e] & 0xffff0000u) + __builtin_bit_cast(float, d & 0xffff0000u);
          v[e] = (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
        }
      }
      if (m < M && n < N) *reinterpret_cast<u32x4_t*>(C + m * ldc + n) = v;
    }
  }
}

// Writes a block's accumulated column statistics as one partial row: out[N][2] at columns col0..
// (the 4 lane groups sharing a column combine by xor-shuffles, the 2 M-waves through LDS).
template <int BM, int BN, int NT = kThreads>
__device__ __forceinline__ void stats_flush(ColStats<BM, BN, NT>& st, float* __restrict__ out, int N, int col0,
                                            char* smem) {
  using AC = Acc<BM, BN, NT>;
  constexpr int WN = AC::WN, TN = AC::TN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN,
            fr = acc_col(lane);
  float* red = reinterpret_cast<float*>(smem);  // [WGM wr][BN][2]
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    float a = st.s[j], b = st.q[j];
    if constexpr (kMS == 16) {
      a += __shfl_xor(a, 16, kWave);
      b += __shfl_xor(b, 16, kWave);
    }
    a += __shfl_xor(a, 32, kWave);
    b += __shfl_xor(b, 32, kWave);
    if (lane < kMS) {
      const int n = wc * WN + j * kMS + fr;
      red[(wr * BN + n) * 2 + 0] = a;
      red[(wr * BN + n) * 2 + 1] = b;
    }
  }
  __syncthreads();
  if (tid < BN && col0 + tid < N) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int g = 0; g < AC::WGM; ++g) {
      a += red[(g * BN + tid) * 2 + 0];
      b += red[(g * BN + tid) * 2 + 1];
    }
    out[(int64_t)(col0 + tid) * 2 + 0] = a;
    out[(int64_t)(col0 + tid) * 2 + 1] = b;
  }
}

// fp32 split-K partial slab P[Mo][No] (row m = M-side index, col n = N-side index)
template <int BM, int BN, int NT = kThreads>
__device__ __forceinline__ void epilogue_f32(const Acc<BM, BN, NT>& acc, float* __restrict__ P, int Mo, int No,
                                             int m0, int n0) {
  using AC = Acc<BM, BN, NT>;
  constexpr int WM = AC::WM, WN = AC::WN, TM = AC::TM, TN = AC::TN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wr = wid / AC::WGN, wc = wid % AC::WGN,
            fr = acc_col(lane);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < kAccN; ++r) {
        const int m = m0 + wr * WM + i * kMS + acc_row(lane, r);
        const int n = n0 + wc * WN + j * kMS + fr;
        if (m < Mo && n < No) P[(int64_t)m * No + n] = acc.v[i][j][r];
      }
}

}  // namespace mm
}  // namespace dla
