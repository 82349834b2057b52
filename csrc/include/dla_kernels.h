// Host-visible launcher declarations for the distributed_learning_amd HIP kernels.
// Kernel translation units include only HIP headers; torch/ATen stays in the binding TUs so
// that kernel files compile in seconds.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dla {

enum DType : int { kF32 = 0, kBF16 = 1 };

// ---- multi-tensor (multi_tensor.hip) --------------------------------------------------------
struct SgdEntry {
  float* param;
  const void* grad;      // float* or bf16*
  float* momentum;       // may be null when momentum == 0
  uint16_t* param_bf16;  // optional bf16 shadow copy of the parameter (null = skip)
  int64_t numel;
};

struct SgdParams {
  float lr;
  float momentum;
  float dampening;
  float weight_decay;
  float grad_scale;
  int nesterov;
  int first_step;
};

struct PackEntry {
  void* tensor;    // grad tensor (pack source / unpack destination)
  int64_t numel;
  int64_t offset;  // element offset inside the flat bucket
};

// By-value tensor lists (kernel arguments, no device table): one launch covers up to kMaxList
// tensors; used when tensor addresses change between steps.
constexpr int kMaxList = 32;
struct SgdList {
  int ntensors;
  int32_t prefix[kMaxList + 1];
  SgdEntry e[kMaxList];
};
struct PackList {
  int ntensors;
  int32_t prefix[kMaxList + 1];
  PackEntry e[kMaxList];
};

int mt_chunk_elems();
void launch_sgd_list(const SgdList& list, int nblocks, int grad_dtype, bool use_momentum, const SgdParams& hp,
                     hipStream_t stream);
void launch_pack_list(const PackList& list, int nblocks, int src_dtype, int flat_dtype, void* flat, float scale,
                      hipStream_t stream);
void launch_sgd(const SgdEntry* entries, const int32_t* prefix, int ntensors, int nblocks, int grad_dtype,
                bool use_momentum, const SgdParams& hp, hipStream_t stream);
void launch_pack(const PackEntry* entries, const int32_t* prefix, int ntensors, int nblocks, int src_dtype,
                 int flat_dtype, void* flat, float scale, hipStream_t stream);
void launch_unpack(const PackEntry* entries, const int32_t* prefix, int ntensors, int nblocks, int flat_dtype,
                   int dst_dtype, const void* flat, float scale, hipStream_t stream);

// ---- elementwise reductions for the collectives (reduce.hip) --------------------------------
constexpr int kMaxReduceSrc = 8;
struct ReduceSrcs {
  const void* ptr[kMaxReduceSrc];
  int count;
};
// dst[i] = (dst_in ? dst[i] : 0) + sum_k src_k[i], times scale. All operands share dtype.
void launch_reduce_sum(void* dst, bool accumulate_dst, const ReduceSrcs& srcs, int64_t n, int dtype,
                       float scale, hipStream_t stream);
void launch_scale(void* data, int64_t n, int dtype, float scale, hipStream_t stream);
// Many independent single-source reductions in ONE launch (one ring step of C channels x N virtual
// ranks): lane i computes dst_i = scale_i * ([dst_i] + src_i) over n_i elements (src_i may be null:
// pure scale). Passed by value (no table upload), so a step costs one launch whatever C is.
constexpr int kMaxReduceLanes = 64;
struct ReduceLane {
  void* dst;
  const void* src;
  int64_t n;
  float scale;
  int accumulate;
};
struct ReduceLanes {
  ReduceLane lane[kMaxReduceLanes];
  int blk0[kMaxReduceLanes + 1];  // first block of each lane (prefix over lanes), filled by the launcher
  int count;
};
void launch_reduce_lanes(ReduceLanes& lanes, int dtype, hipStream_t stream);
// dst = scale * src with dtype conversion (fp32 / bf16 either way)
void launch_cast(void* dst, int dst_dtype, const void* src, int src_dtype, int64_t n, float scale, hipStream_t stream);

// ---- cross-process barrier over peer-mapped memory (ipc_sync.hip) ---------------------------
// One wave: publish `set` into this rank's flag (system-scope release, so everything the stream
// wrote before is visible to peers that observe it), then wait until every listed peer flag is
// >= `wait` (system-scope acquire). A peer that never arrives ends the wait after `timeout_ticks`
// of the constant 100 MHz clock with err[0] = 1 instead of spinning forever, so the grid always
// drains; the host reads err after the stream completes. The first timeout also records what it
// waited for in diag[0..2]: the awaited token, the value the peer's flag last held, and that peer's
// global rank (engine.cpp ipc_error_info), so a failure names a stuck peer or a stale mapping.
constexpr int kMaxIpcPeers = 16;
struct IpcBarrier {
  uint64_t* mine;  // null: do not publish
  uint64_t set;
  const uint64_t* peer[kMaxIpcPeers];
  int peer_rank[kMaxIpcPeers];
  int npeers;
  uint64_t wait;
  int* err;
  uint64_t* diag;  // may be null
  uint64_t timeout_ticks;
};
void launch_ipc_barrier(const IpcBarrier& b, hipStream_t stream);

// ---- synthetic data (synthetic.hip) ---------------------------------------------------------
// Philox stream position = offset [+ (*step) * per_step when `step` (device int64 counter) is set].
void launch_uniform_fill(void* out, int64_t n, int dtype, uint64_t seed, uint64_t offset, float lo, float hi,
                         hipStream_t stream, const int64_t* step = nullptr, uint64_t per_step = 0);
void launch_randint_fill(int64_t* out, int64_t n, int64_t high, uint64_t seed, uint64_t offset,
                         hipStream_t stream, const int64_t* step = nullptr, uint64_t per_step = 0);

// ---- fused log-softmax + NLL (loss.hip) -----------------------------------------------------
// logits [B, C] (dtype), target [B] int64 (< 0 = ignored). ws: 3*B floats (row lse, row loss,
// row valid). loss_out[0] = mean loss over valid rows, loss_out[1] = valid row count.
// Backward: dlogits = (softmax - onehot) * gout / count.
void launch_xent_fwd(const void* logits, const int64_t* target, float* ws, float* loss_out, int B, int C,
                     int dtype, hipStream_t stream);
void launch_xent_bwd(const void* logits, const int64_t* target, const float* ws, const float* loss_out,
                     const float* gout, void* dlogits, int B, int C, int dtype, hipStream_t stream);

// ---- fused BatchNorm + residual + ReLU, NHWC (bn_act.hip) ------------------------------------
// x/res/y/dy/dx/dres: [M, C] row-major (channels_last activations), C % 8 == 0, 16-byte aligned.
// ws: 7*C floats (mean, invstd, scale, shift | k1, m1, k2); part: bn_partial_floats(M, C) floats.
void bn_geometry(int64_t M, int C, int* tpr, int* nrb, int* nct, int target_blocks);  // <= 0: reduction passes
// fp32 scratch floats of one reduction pass's partials [rows][C][2] plus their fold rows
int64_t bn_partial_floats(int64_t M, int C, int target_blocks = 0);
int64_t bn_relu_maxpool_part_floats(int64_t M, int C);  // partials of launch_bn_relu_maxpool_bwd
// reduction-pass block target (0 = DLA_BN_RED_BLOCKS or the default 1024); tests exercise the
// > 1024-row fold path with it
void set_bn_red_blocks(int blocks);
int bn_red_blocks();
// rows of fp32 [rows][C][2] scratch launch_bn_fwd's `part` needs to fold ext_nrb epilogue partials (0: none)
int bn_fold_groups(int ext_nrb);
void launch_bn_fwd(const void* x, const void* res, void* y, int64_t M, int C, int dtype, const float* gamma,
                   const float* beta, float eps, float momentum, float* running_mean, float* running_var, float* ws,
                   float* part, bool relu, bool training, hipStream_t stream, const float* ext_part = nullptr,
                   int ext_nrb = 0, uint8_t* relu_mask = nullptr, int64_t ldy = 0);
// y = act(BN(x) + BN_d(xd)) from the two finalized workspaces (ws, wsd: launch_bn_fwd with y == nullptr);
// mask as launch_bn_fwd's ReLU-after-residual bit mask.
void launch_bn_dual_apply(const void* x, const void* xd, void* y, const float* ws, const float* wsd, int64_t M, int C,
                          int dtype, bool relu, uint8_t* mask, hipStream_t stream);
// backward of launch_bn_dual_apply: dx, dxd and both (dgamma, dbeta) from one dy (+ the forward's
// bit mask, or null without ReLU); part / partd: [bn_geometry rows][C][2] scratch each.
void launch_bn_dual_bwd(const void* dy, const uint8_t* mask, const void* x, const void* xd, void* dx, void* dxd,
                        int64_t M, int C, int dtype, const float* gamma, const float* gamma_d, float* ws, float* wsd,
                        float* part, float* partd, float* dgamma, float* dbeta, float* dgamma_d, float* dbeta_d,
                        hipStream_t stream);
// mask_mode: 0 no ReLU, 1 recompute from x (ReLU right after BN), 2 1-bit mask written by the
// forward (ReLU after the residual add), 3 from the saved output y.
// ext_part/ext_nrb: the reduction pass's partials were already produced (GEMM epilogue, BnBwdArgs).
void launch_bn_bwd(const void* dy, const void* y, const uint8_t* mask, const void* x, void* dx, void* dres,
                   int64_t M, int C, int dtype, const float* gamma, float* ws, float* part, float* dgamma,
                   float* dbeta, int mask_mode, hipStream_t stream, const float* ext_part = nullptr,
                   int ext_nrb = 0, int64_t ld_dy = 0);  // ld_dy: dy row stride when dy is a channel slice

// Grouped training BN+ReLU (bn_act.hip): one launch per pass for up to kMaxBnGroups BatchNorms of
// the same row count M — the branches of an Inception block. Group g normalises x[g] ([M, C[g]] bf16,
// row stride ldx[g]; its statistics part[g] may be a channel slice of a wider partials tensor, ldp[g])
// into y[g] (row stride ldy[g], 0 = contiguous; a channel slice of the concatenated output, or its
// own tensor). Forward: part[g] = the [nrb][C][2] conv-epilogue statistics, wpart[g] = fold scratch
// (bn_fold_groups(nrb) rows). Backward: dy[g] (row stride lddy[g]); with ext, part[g] already holds
// the dgrad epilogue's reduction partials (nrb[g] rows; wpart[g] = fold scratch), otherwise
// wpart[g] receives bn_group_bwd_rows() rows of reduce partials. ReLU mask recomputed from x.
constexpr int kMaxBnGroups = 4;
struct BnGroups {
  int n;
  int begin[kMaxBnGroups + 1];
  const uint16_t* x[kMaxBnGroups];  // bf16 bits
  uint16_t* y[kMaxBnGroups];
  const uint16_t* dy[kMaxBnGroups];
  int64_t ldy[kMaxBnGroups], lddy[kMaxBnGroups];
  int64_t ldx[kMaxBnGroups], lddx[kMaxBnGroups];  // row strides of x / dx (0: contiguous [M, C])
  int ldp[kMaxBnGroups];                          // row stride of part in channels (0: C)
  int C[kMaxBnGroups], tpr[kMaxBnGroups], nrb[kMaxBnGroups];
  const float* part[kMaxBnGroups];
  float* wpart[kMaxBnGroups];
  const float* gamma[kMaxBnGroups];
  const float* beta[kMaxBnGroups];
  float* rm[kMaxBnGroups];
  float* rv[kMaxBnGroups];
  float* ws[kMaxBnGroups];
  float eps[kMaxBnGroups], mom[kMaxBnGroups];
  uint16_t* dx[kMaxBnGroups];
  float* dgamma[kMaxBnGroups];
  float* dbeta[kMaxBnGroups];
};
int bn_group_bwd_rows(int64_t M, const int* C, int n);
void launch_bn_group_fwd(BnGroups G, int64_t M, hipStream_t stream);
void launch_bn_group_bwd(BnGroups G, bool ext, int64_t M, hipStream_t stream);

// Stem BN(+ReLU)+max-pool fused (bn_act.hip): launch_bn_fwd with y == nullptr computes ws only;
// then the pooled output + window positions come straight from the BN input x. Backward: the BN
// passes gather dy from the pooled gradient. x/dx [N,H,W,C] bf16, pooled [N,OH,OW,C].
void launch_bn_relu_maxpool_fwd(const void* x, const float* ws, void* y, uint8_t* pos, int N, int H, int W, int C,
                                int OH, int OW, int k, int s, int p, hipStream_t stream);
void launch_bn_relu_maxpool_bwd(const void* dy_pool, const uint8_t* pos, const void* x, void* dx, int N, int H, int W,
                                int C, int OH, int OW, int k, int s, int p, const float* gamma, float* ws, float* part,
                                float* dgamma, float* dbeta, hipStream_t stream);

// ---- max pooling, NHWC (pool.hip) ------------------------------------------------------------
// x [N,H,W,C], y/pos [N,OH,OW,C] (pos: window position k*ky+kx of the max, 1 byte), C % 8 == 0,
// N*H*W*C/8 < 2^31. Backward writes every dx element (no zero-fill needed).
void launch_maxpool_fwd(const void* x, void* y, uint8_t* pos, int N, int H, int W, int C, int OH, int OW, int k,
                        int s, int p, int dtype, hipStream_t stream);
void launch_maxpool_bwd(const void* dy, const uint8_t* pos, void* dx, int N, int H, int W, int C, int OH, int OW,
                        int k, int s, int p, int dtype, hipStream_t stream);
// global average pooling over the H*W pixels of NHWC x: y [N, C]; backward dx [N, H, W, C] = dy / HW
void launch_gap_fwd(const void* x, void* y, int N, int HW, int C, int dtype, hipStream_t stream);
// y [N, H/2, W/2, C] = x [N, H, W, C] at even (h, w); bf16 NHWC, C % 8 == 0
void launch_subsample2(const void* x, void* y, int N, int H, int W, int C, hipStream_t stream);
void launch_gap_bwd(const void* dy, void* dx, int N, int HW, int C, int dtype, hipStream_t stream);

// ---- bf16 MFMA GEMMs (gemm.hip) ---------------------------------------------------------------
// C[M,N] = A[M,K] B[N,K]^T [+ addend[M,N]] (b_kmajor: B given as [K,N], i.e. C = A B); optional
// per-column (sum, sumsq) partials stats[ceil(M/128)][N][2]. Requires K % 8 == 0, N % 8 == 0,
// 16-byte aligned rows.
// Tile configurations of the MFMA kernels (gemm_nt, conv3x3 fwd/dgrad). kTileAuto picks the
// largest tile that still yields >= 1024 workgroups (4 per CU), so small-M layers fill the chip.
// MFMA main-loop pipeline for every GEMM/conv kernel: 0 register staging, 2 / 3 LDS-DMA stages,
// -1 (default) per shape.
void set_mfma_pipeline(int p);  // -1 = per-shape auto
int mfma_pipeline();
int mfma_pipeline_for(int K);
// kTile256x128: 8 waves (512 threads) of 64x64, 3-stage LDS-DMA pipeline, one block per CU.
// kTile256x128w4 / kTile128x256w4: 4 waves of 128x64 / 64x128 (half the LDS fragment reads per
// MFMA of the 64x64 wave tiles), 3-stage LDS-DMA pipeline (144 KB), one block per CU.
enum TileCfg : int {
  kTileAuto = 0,
  kTile128x128 = 1,
  kTile128x64 = 2,
  kTile64x64 = 3,
  kTile256x128 = 4,
  kTile256x128w4 = 5,
  kTile128x256w4 = 6,
  kTile256x64 = 7,  // 4 waves stacked along M (64 x 64 wave tiles), 2 blocks / CU; opt-in: measured slower
                    // than 128x64 / 128x128 at every ResNet-50 shape (profiles/tiles_256x64_4x1waves_ab.jsonl)
  // 8 waves (4 x 2) of 64 x 128, 2-stage buffer-DMA pipeline (128 KB LDS), one block per CU: per MAC
  // 25 % fewer LDS fragment reads than the 64 x 64 wave tiles and half the DMA writes of two 128x128
  // blocks, for the compute-bound shapes where the 128x128 loop is LDS-bandwidth co-bound
  kTile256x256 = 8,
  // 3x3 convs only: 8 waves (4 x 2) of 128 x 64 over 512 output pixels x 128 channels, 2-stage buffer-DMA
  // pipeline (160 KB LDS, all of it), one block per CU: the per-MAC LDS fragment reads of the 256x256 tile's
  // 64 x 128 wave tiles for the Cout = 128 layers that tile cannot serve (conv.hip pick_conv_tile)
  kTile512x128 = 9
};
// K: reduction length (0 = unknown); wide_ok: the kernel family can run the 8-wave tiles (3x3 convs
// need a channel count % 64 on the loaded side)
int pick_tile(int64_t M, int N, int tile, int K = 0, bool wide_ok = true, bool stats = false);
void set_tile256_min_k_stats(int k);  // smallest K of the auto 256x256 tiles for statistics forwards (A/B)
bool tile256_enabled();  // DLA_TILE256 != 0: 256x256 tiles for the compute-bound fwd / dgrad shapes
bool tn256_enabled();    // ... and for the split-K weight gradients (also DLA_TN256 != 0)
inline int tile_bm(int cfg) {
  if (cfg == kTile512x128) return 512;
  return cfg == kTile64x64 ? 64
                           : ((cfg == kTile256x128 || cfg == kTile256x128w4 || cfg == kTile256x64 || cfg == kTile256x256)
                                  ? 256
                                  : 128);
}
inline int tile_bn(int cfg) {
  if (cfg == kTile512x128) return 128;
  return (cfg == kTile128x256w4 || cfg == kTile256x256) ? 256
                                                       : ((cfg == kTile128x128 || cfg == kTile256x128 || cfg == kTile256x128w4) ? 128 : 64);
}
// rows of BN-statistics partials ([rows][N][2]) a stats-producing launch writes (one per row tile)
// stats_fwd: the launch carries the forward statistics epilogue without an addend (its tile policy differs from
// the data gradients' whose BN-backward partials also come one row per row tile)
int gemm_nt_stats_rows(int M, int N, int tile = kTileAuto, int K = 0, bool stats_fwd = true);
void set_tile256_min_k(int k);  // smallest K of the auto 256x256 tiles (A/B runs; <= 0 restores the default)
// Persistent streaming 1x1 GEMM (gemm_stream.hip) for K in {64, 128, 256}, N % 64 == 0, long M: the
// number of BN-statistics partial rows it writes (0 = shape not served: use launch_gemm_nt), and the
// launcher (false = not served). set_gemm_stream: -1 environment (DLA_GEMM_STREAM, default on), 0 / 1.
int gemm_stream_rows(int64_t M, int N, int K, int64_t lda, int64_t ldc, bool b_kmajor, bool add = false,
                     bool bnb = false);
// addend (data gradients): C = bf16(bf16(A B^T) + (mask bit ? addend : 0)), addend [M][N] row stride ldd,
// k-major B and no statistics only (false = not served).
struct BnBwdArgs;
// bn_bwd (k-major data gradients): the output is the dy of a fused BN; its backward-reduction partials
// [gemm_stream_rows][N][2] are written to bn_bwd->part instead of statistics.
// apply_ws (forwards with statistics): A is the input of a deferred BN+ReLU (7K workspace apply_ws); the kernel
// multiplies relu(A * scale + shift) and writes it to apply_out (A's layout)
bool launch_gemm_stream(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, void* C, int64_t ldc,
                        int M, int N, int K, float* stats, hipStream_t stream, const void* addend = nullptr,
                        int64_t ldd = 0, const uint8_t* addend_mask = nullptr, const BnBwdArgs* bn_bwd = nullptr,
                        const float* apply_ws = nullptr, void* apply_out = nullptr);
void set_gemm_stream(int mode);
// 128x128 1x1 GEMM tiles stored straight from the accumulators (gemm_direct.hip): the transposed product,
// lane-exchange to 16-byte chunks, statistics by DPP row sums; same outputs / statistics layout as
// launch_gemm_nt's 128x128 tile. set_gemm_direct: -1 environment (DLA_GEMM_DIRECT, default off), 0 / 1.
bool gemm_direct_ok(int N, int64_t ldc, const void* addend, int64_t ldd);
void launch_gemm_direct(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, void* C, int64_t ldc,
                        int M, int N, int K, float* stats, const void* addend, int64_t ldd,
                        const uint8_t* addend_mask, hipStream_t stream);
void set_gemm_direct(int mode);
// 1x1-conv forward whose input is a deferred act(BN(y) + r) (gemm_apply.hip): y, r, out [M][K] bf16 contiguous,
// ws / ws2 the 7K BN workspaces (ws2 non-null: r is the shortcut BN's input), mask the ReLU bits; C [M][N]
// (row stride N), B [N][K]; statistics [gemm_apply_rows(M)][N][2] when stats is non-null. Writes out + mask
// and C in one pass.
constexpr int kGemmApplyMaxK = 2048;  // coefficient table: 4 x K fp32 of LDS (dual)
bool gemm_apply_ok(int64_t M, int N, int K);
void set_gemm_apply_max_k(int k);
// 256x256 statistics forwards stored from the registers (dla_mfma.h epilogue_direct): -1 env (DLA_GEMM256_DIRECT), 0, 1
void set_gemm256_direct(int mode);
bool gemm256_direct_enabled();
void set_wgrad_w4(int mode);  // 128x256 tiles for the Cout-128 3x3 weight gradients: -1 env (DLA_WGRAD_W4), 0, 1  // <= 0: DLA_APPLY_MAX_K / default 512
int gemm_apply_rows(int64_t M);
// xs (optional): also write out's stride-2 subsample [n][H/2][W/2][K] (rows m = (n H + h) W + w; H, W even)
void launch_gemm_apply(const void* y, const void* r, const float* ws, const float* ws2, void* out, uint8_t* mask,
                       const void* B, int64_t ldb, void* C, int M, int N, int K, float* stats, hipStream_t stream,
                       void* xs = nullptr, int H = 0, int W = 0);
// the register-stored tiles as a persistent kernel with n blocks per CU (0: one block per tile; -1: DLA_GEMM_PERSIST)
void set_gemm_persist(int blocks_per_cu);
// fp32 convolutions on v_mfma_f32_16x16x4_f32 (conv_f32.hip): x NHWC [N][H][W][C], w OHWI [Cout][R][S][C], y NHWC
// [N][OH][OW][Cout]; C % 4 == 0, Cout % 4 == 0, N * OH * OW < 2^24. accumulate: y += conv instead of y = conv.
bool conv_f32_supported(int C, int Cout, int64_t M, int K);
void set_conv_f32_buffers(int nb);  // 1 or 2 (default) LDS buffers of the fp32 GEMM main loop (A/B)
// ldx: elements between consecutive pixels of x (C, or more when x is a channel slice of a wider NHWC tensor)
void launch_conv_f32_fwd(const float* x, int64_t ldx, int N, int H, int W, int C, const float* w, int Cout, int R,
                         int S, int pad, int stride, float* y, bool accumulate, hipStream_t st);
// dw [Cout][R][S][C] (+)= sum over pixels of dy [N * OH * OW][Cout] x im2col(x); partial: splits * Cout * R * S * C floats
int conv_f32_wgrad_splits(int64_t M, int Cout, int K);
void launch_conv_f32_wgrad(const float* dy, const float* x, int64_t ldx, int N, int H, int W, int C, int Cout, int R,
                           int S, int pad, int stride, float* partial, int splits, float* dw, bool accumulate,
                           hipStream_t st);
// BatchNorm-backward reduction fused into a bf16-output GEMM epilogue (the output is the BN's dy):
// x = the BN input [M, N], ws = its 7N workspace, mask/mode as launch_bn_bwd (0, 1 or 2),
// part = [stats_rows][N][2] partial (sum dy', sum dy'(x - mean)).
struct BnBwdArgs {
  const void* x;
  const float* ws;
  const uint8_t* mask;
  int mode;
  float* part;
  int64_t ldx = 0;  // row stride of x when it is a channel slice of a wider tensor (0: the output's)
};
void launch_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                    float* stats, hipStream_t stream, const void* addend = nullptr, int64_t ld_addend = 0,
                    bool b_kmajor = false, int tile = kTileAuto, const BnBwdArgs* bn_bwd = nullptr,
                    const uint8_t* addend_mask = nullptr,  // addend element used iff its mask bit is set
                    const void* addend2_s2 = nullptr, int H = 0, int W = 0);  // compact stride-2 addend
// out[Mo,No] (= scale * A^T B [+ out]) with A [K, lda>=Mo], B [K, ldb>=No]; partial: splits*Mo*No f32.
int gemm_tn_splits(int Mo, int No, int K);
bool splitk_xcd_remap();
void set_tn256(int mode);  // 256x256 weight-gradient tiles: -1 DLA_TN256 / default on, 0 off, 1 on
void set_splitk_blocks(int blocks);  // 0: DLA_SPLITK_BLOCKS / default (512)
int splitk_target_blocks();  // split-K grids: tiles of one split co-scheduled on one XCD (DLA_SPLITK_XCD=0: off)
void launch_gemm_tn(const void* A, int64_t lda, const void* B, int64_t ldb, float* partial, int splits, int Mo, int No,
                    int K, void* out, int out_dtype, float scale, bool accumulate, hipStream_t stream);
// Both gradients of a stride-1 1x1 conv in one pass over dY (gemm_dual.hip; (Cout, Cin) = (256, 64),
// (512, 128 / 256)): dx [M][Cin] bf16 and fp32 dW partials part [groups][Cout][Cin]; 0 blocks = not served
int conv1x1_dual_blocks(int64_t M, int Cin, int Cout);
int conv1x1_dual_groups(int64_t M, int Cin, int Cout);
// ybn / mask / ws: dy is the incoming gradient of the BN(+residual)+ReLU that consumed the conv's output
// (bit-mask ReLU, finalized workspace); its backward apply runs inside the kernel (Cout 256 only)
bool conv1x1_dual_bn_ok(int64_t M, int Cin, int Cout);
bool launch_conv1x1_dual(const void* dy, const void* x, const void* w, void* dx, float* part, int64_t M, int Cin,
                         int Cout, hipStream_t stream, const void* ybn = nullptr, const uint8_t* mask = nullptr,
                         const float* ws = nullptr);
// out[n] (= scale * sum_s partial[s][n] [+ addend] [+ out]), fp32 or bf16 out; addend: bf16 rows of
// ncol with row stride ld_addend (0 = one broadcast row).
void launch_splitk_reduce(const float* partial, int splits, int64_t n, void* out, int out_dtype, float scale,
                          bool accumulate, hipStream_t stream, const void* addend = nullptr, int64_t ld_addend = 0,
                          int ncol = 1);
// Split-K C[M,N] = A B^T (+ addend) for few output tiles and a long K (fully connected heads):
// splits > 1 when it applies; partial holds splits * M * N floats.
int gemm_nt_splitk_splits(int M, int N, int K);
void launch_gemm_nt_splitk(const void* A, int64_t lda, const void* B, int64_t ldb, bool b_kmajor, float* partial,
                           int splits, void* C, int M, int N, int K, const void* addend, int64_t ld_addend,
                           hipStream_t stream);

// ---- implicit-GEMM 3x3 convolutions, pad 1, NHWC bf16 (conv.hip) -----------------------------
// x [N,H,W,Cin], w [Cout,3,3,Cin], y [N,OH,OW,Cout]; Cin % 64 == 0, Cout % 64 == 0, pixels < 2^24.
// fwd: stride 1 or 2, optional BN statistics partials stats[ceil(P/128)][Cout][2].
// dgrad: stride 1 only, dx [N,H,W,Cin] (+ optional addend). wgrad: stride 1 or 2, split-K fp32
// partials (splits * Cout * 9*Cin floats) reduced into dw [Cout][9*Cin] (fp32 or bf16).
int conv3x3_stats_rows(int64_t P, int Cout, int tile = kTileAuto, int K = 0, bool wide_ok = true);
// tile of a stride-1/2 3x3 forward or data-gradient launch (pick_tile plus the conv-only kTile512x128)
int pick_conv_tile(int64_t P, int N, int tile, int K, bool wide_ok);
// halo-tiled 64 -> 64 channel 3x3 / stride-1 conv (conv_halo.hip): persistent strips of 128 pixels,
// weights resident in LDS; stats partial rows as the 128x64 tile (ceil(P / 128)). DLA_HALO: 0 off,
// 1 data gradient only, 2 (default) also the forward.
bool halo_conv_eligible(int Cin, int Cout, int W, int stride, bool fwd);
void launch_conv3x3_halo(const void* x, const void* w, void* y, int N, int H, int W, float* stats,
                         hipStream_t stream, const void* addend = nullptr);
void launch_conv3x3_fwd(const void* x, const void* w, void* y, int N, int H, int W, int Cin, int Cout, int stride,
                        float* stats, hipStream_t stream, int tile = kTileAuto);
void launch_conv3x3_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                          const void* addend, hipStream_t stream, int tile = kTileAuto,
                          const BnBwdArgs* bn_bwd = nullptr);
// stride-2 data gradient (H, W even): dx [N,H,W,Cin] from dy [N,H/2,W/2,Cout], parity-class GEMMs.
void launch_conv3x3s2_dgrad(const void* dy, const void* w, void* dx, int N, int H, int W, int Cin, int Cout,
                            hipStream_t stream);
// ---- 7x7 / stride-2 / pad-3 stem conv, Cin = 3 (stem.hip) ------------------------------------------
// x [N,H,W,3] bf16 -> fold: xs [N,(H+1)/2,(W+1)/2,16] (space-to-depth, 4 zero channels);
// wpk = packed weight [Cout][256] (k = (th * 4 + tw) * 16 + (ph * 2 + pw) * 3 + c, see stem.hip);
// y [N,OH,OW,Cout] with optional BN-statistics partials stats[stem_stats_rows(P, Cout)][Cout][2].
int stem_stats_rows(int64_t P, int Cout = 64);
// the stem forward with statistics on the persistent streaming GEMM (gemm_stream.hip kStem): its partial rows
// (0: not used -- DLA_STEM_STREAM / set_stem_stream off, or the shape is not served)
int stem_stream_rows(int64_t P, int Cout);
bool launch_stem_stream(const void* xs, const void* wpk, void* y, int N, int BH, int BW, float* stats,
                        hipStream_t stream);
void set_stem_stream(int mode);

void launch_stem_fold(const void* x, void* xs, int N, int H, int W, hipStream_t stream);
void launch_stem_fwd(const void* xs, const void* wpk, void* y, int N, int H, int W, int Cout, float* stats,
                     hipStream_t stream);
int stem_wgrad_splits(int N, int H, int W, int Cout);
void launch_stem_wgrad(const void* dy, const void* xs, float* partial, int splits, void* dwpk, int out_dtype, int N,
                       int H, int W, int Cout, hipStream_t stream);
// The stem weight gradient with the BatchNorm(+ReLU)+max-pool (3x3 / s2 / p1) backward APPLY computed on the fly
// as its dY operand (stem.hip stem_wgrad_bn_kernel): dy_pool [N,OH,OW,64] and its argmax positions, x = the BN
// input (the conv output [N,BH,BW,64], BH = (H + 1) / 2 = 2 OH), ws = the 7 x 64 coefficients the quad reduce +
// finalize left (launch_bn_relu_maxpool_bwd with dx = nullptr). H, W: the stem INPUT image (as launch_stem_wgrad).
bool stem_wgrad_bn_eligible(int N, int H, int W, int Cout, int OH, int OW);
int stem_wgrad_bn_splits(int N, int H, int W);
void launch_stem_wgrad_bn(const void* dy_pool, const uint8_t* pos, const void* x, const float* ws, const void* xs,
                          float* partial, int splits, void* dwpk, int out_dtype, int N, int H, int W, int OH, int OW,
                          hipStream_t stream);
// Halo-tiled 64 -> 64 channel 3x3 / stride-1 weight gradient (conv_halo_wgrad.hip): persistent blocks over
// a padded pixel space, x rows through an LDS ring; splits = partial slabs of [64][9][64] fp32.
bool halo_wgrad_eligible(int Cin, int Cout, int W, int stride);
void set_halo_wgrad(int mode);  // -1 environment (DLA_HALO_WGRAD, default on), 0 off, 1 on
int halo_wgrad_splits(int N, int H, int W);
void launch_conv3x3_halo_wgrad(const void* dy, const void* x, float* partial, int splits, void* dw, int out_dtype,
                               int N, int H, int W, hipStream_t stream);
int conv3x3_wgrad_splits(int N, int H, int W, int Cin, int Cout, int stride);
void launch_conv3x3_wgrad(const void* dy, const void* x, float* partial, int splits, void* dw, int out_dtype, int N,
                          int H, int W, int Cin, int Cout, int stride, hipStream_t stream);

}  // namespace dla
