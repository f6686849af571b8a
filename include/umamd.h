/*
 * umamd -- MI355X (gfx950) kernels for the self-supervised depth+uncertainty
 * training step of Probabilistic-Surgical-Vision/uncertainty-model.
 *
 * C ABI (drop-in boundary under the Python host layer in
 * uncertainty-model_amd/umamd/).  Rules:
 *   - plain pointers, sizes and enums only; no torch types;
 *   - device pointers are caller-owned (PyTorch caching allocator); the
 *     library never allocates or frees and never synchronises the host;
 *   - every entry takes the HIP stream to launch on (torch's current stream);
 *   - returns UM_OK (0) or an error code; um_last_error() gives a
 *     thread-local message (entries are called from PyTorch's autograd thread).
 *
 * Tensor conventions: activations are NHWC with a pixel stride `ld`
 * (elements between consecutive pixels; >= channels), element type UM_F32 or
 * UM_BF16 as given by `dtype`; arithmetic is always f32.  Conv weights are
 * repacked per step from the reference's NCHW f32 parameters
 * ([K][C][R][R], reference nn.Conv2d) into [K][R][R][Cp] ("forward") and
 * [Cp][R][R][K] ("transposed", for the data gradient), Cp = C rounded up to 8.
 *
 * Each entry cites the reference operation it replaces (file:line in the
 * reference repository).
 */
#ifndef UMAMD_H
#define UMAMD_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { UM_OK = 0, UM_ERR_ARG = 1, UM_ERR_HIP = 2 };
enum { UM_F32 = 0, UM_BF16 = 1 };
/* OR'ed into the dtype of the um_bn_elu_* entries (and um_conv2d_fwd_up2's): the pre-BN conv output y is stored in the activation
 * dtype instead of f32 (the bf16 build's default, as a bf16 autocast conv
 * feeding BatchNorm2d; statistics are still taken in f32 in the conv
 * epilogue).  um_conv2d_fwd_up2: y and the low-resolution map up2. */
enum { UM_Y_ACT = 0x100 };
enum { UM_PAD_ZERO = 0, UM_PAD_REFLECT = 1 };
enum {
  UM_EPI_NONE = 0,           /* y = acc (+ bias)                               */
  UM_EPI_STATS = 1,          /* y = acc + bias, per-block BN partial sums      */
  UM_EPI_SIGMOID_SCALE = 2,  /* y(f32) = scale * sigmoid(acc + bias)           */
  UM_EPI_RESIDUAL = 3,       /* y = acc + bias + residual                      */
  UM_EPI_STAT_SLOTS = 4      /* y = acc + bias, BN sums f64-atomically added into
                                stats_partials viewed as double[UM_STAT_SLOTS][K][2]
                                (zeroed by the caller; see um_bn_elu_fwd_slots)  */
};
/* f64 slots of the atomic BN statistics (UM_EPI_STAT_SLOTS, *_slots entries) */
#define UM_STAT_SLOTS 16

const char* um_last_error(void);
int um_version(void);
/* kernel-selection knobs (tests force code paths, tuning sweeps): "halo",
 * "halo_min_tiles", "small", "small_tiles", "split_below", "split_target",
 * "split_minsteps".  Returns the previous value, -1 for an unknown key. */
int um_set_tuning(const char* key, int value);

/* ---------------------------------------------------------------- conv ---
 * Replaces nn.Conv2d forward/backward with its padding:
 *   encoder ConvELUBlock: F.pad zero + Conv2d(k, stride)
 *       reference model/layers/encoder.py:42-52
 *   decoder ConvLayer: ReflectionPad2d(1) + Conv2d(3) / 1x1 without padding
 *       reference model/layers/decoder.py:30-52
 *   attention 1x1 K/Q/V/reprojection: reference model/layers/attention.py:37-40,66-76
 * Implicit GEMM on MFMA (bf16: v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32).
 */
/* number of BN partial rows written by um_conv2d_fwd with UM_EPI_STATS for M
 * output pixels and K channels (UM_EPI_STAT_SLOTS writes UM_STAT_SLOTS f64 rows
 * instead, through the same stats_partials pointer) */
int um_conv_stats_parts(int M, int K);

/* split-K workspace (bytes) the kernels want for a shape; 0 = no split.
 * Passing a smaller (or null) workspace is allowed: the split shrinks. */
long um_conv_fwd_ws(int dtype, int N, int P, int Q, int K, int R, int C);
long um_conv_dgrad_ws(int dtype, int N, int H, int W, int C, int R, int K, int stride);
/* as um_conv_dgrad_ws, plus the padded-input buffer of the reflect data
 * gradient's padded form (knob "pad_dgrad"): a zero-pad transposed conv onto
 * the (H+2p) x (W+2p) reflect-padded input, folded back onto dx */
long um_conv_dgrad_ws_pad(int dtype, int N, int H, int W, int C, int R, int K, int stride,
                          int pad, int pad_mode);

int um_conv2d_fwd(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                  const void* wf, const float* bias, int K, int R, int stride,
                  int pad, int pad_mode, int P, int Q, int ydtype, void* y,
                  int ldy, int epilogue, float epi_scale, const void* residual,
                  int ldr, float* stats_partials, void* ws, long ws_bytes,
                  hipStream_t stream);

/* 1x1 conv forward (f32 output, zero pad, stride 1) plus the bilinear x2
 * (align_corners=True) upsample of a low-resolution f32 map added before the
 * epilogue's BN statistics: y = W x + bias + up2(z), z = [N][up2_h][up2_w]
 * [up2_ld] (channels [0, K) used).  The decoder's cat(feature_map,
 * interpolate(skip)) -> 1x1 conv (reference model/layers/decoder.py:230-238)
 * with the skip half convolved at the skip's resolution (the 1x1 conv and
 * the upsample commute): the full-resolution concat is never built. */
int um_conv2d_fwd_up2(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                      const void* wf, const float* bias, int K, int P, int Q, void* y, int ldy,
                      int epilogue, float* stats, const void* up2, int up2_h, int up2_w,
                      int up2_ld, hipStream_t stream);
/* data gradient: dx[N,H,W,C] (= or +=) conv^T(dy[N,P,Q,K], wT) incl. the
 * reflect-pad fold and the stride-2 scatter */
int um_conv2d_dgrad(int dtype, int N, int H, int W, int C, int ldx, void* dx,
                    int accumulate, const void* wT, int K, int R, int stride,
                    int pad, int pad_mode, int P, int Q, const void* dy, int ldy,
                    void* ws, long ws_bytes, hipStream_t stream);

/* weight gradient partial slabs [splits][K][R*R*C] (f32); splits from
 * um_conv_wgrad_splits (which also picks the kernel: the halo-tiled one for
 * bf16 small-channel spatial convs, the implicit-GEMM one otherwise) */
int um_conv_wgrad_splits(int dtype, int N, int H, int W, int C, int ldx, int K, int R,
                         int stride, int pad, int pad_mode, int P, int Q, int ldy);
int um_conv2d_wgrad(int dtype, int N, int H, int W, int C, int ldx, const void* x,
                    int K, int R, int stride, int pad, int pad_mode, int P, int Q,
                    const void* dy, int ldy, float* slabs, int splits,
                    hipStream_t stream);
/* sum slabs -> reference NCHW weight grad [Kreal][Creal][R][R] (f32), (+)= */
int um_conv_wgrad_reduce(const float* slabs, int splits, int K, int Kreal, int R, int C,
                         int Creal, float* dw, int accumulate, hipStream_t stream);

/* segment variants: reference input channels [src0[i], src0[i]+len[i]) are
 * placed at packed channels [dst0[i], ...) (host arrays, nseg <= 4); the rest
 * of the packed channels are zero.  Keeps concat sources 8-channel aligned. */
int um_conv_wgrad_reduce_seg(const float* slabs, int splits, int K, int Kreal, int R, int C,
                             int Creal, float* dw, int accumulate, int nseg, const int* src0,
                             const int* dst0, const int* len, hipStream_t stream);
int um_pack_weight_seg(int dtype, const float* w, int K, int Creal, int R, int C, void* wf,
                       void* wT, int ldT, int nseg, const int* src0, const int* dst0,
                       const int* len, hipStream_t stream);

/* Batched repack of many conv weights in ONE launch (the per-step weight
 * refresh of every conv in the model).  Each descriptor is one
 * um_pack_weight_seg call; a descriptor covers um_pack_tiles(K, C, R)
 * workgroups, numbered from `block0`;
 * blk2desc[b] (device int array, nblocks entries) names the descriptor of
 * workgroup b.  `table` and `blk2desc` are device memory (caller-owned). */
#define UM_PACK_MAXSEG 4
typedef struct {
  const float* w;   /* [K][Creal][R][R] f32 */
  void* wf;         /* [K][R][R][C] (nullable) */
  void* wT;         /* [C][R][R][ldT] (nullable; column offset applied) */
  int K, Creal, R, C, ldT, block0;
  int nseg, src0[UM_PACK_MAXSEG], dst0[UM_PACK_MAXSEG], len[UM_PACK_MAXSEG];
  int split;        /* bf16 only: pack 2K rows, see um_pack_weight_split (tiles: 2K) */
} um_pack_desc;
int um_pack_batch(int dtype, const um_pack_desc* table, int ndesc, const int* blk2desc,
                  int nblocks, hipStream_t stream);
int um_pack_tiles(int K, int C, int R);
/* sizeof(um_pack_desc), for bindings that build the table */
int um_pack_desc_size(void);

/* repack f32 NCHW weight [K][Creal][R][R] -> wf [K][R][R][C] (row stride ldf
 * elements) and wT [C][R][R][ldT] (column offset applied by the caller); C >= Creal, zero fill */
int um_pack_weight(int dtype, const float* w, int K, int Creal, int R, int C,
                   void* wf, void* wT, int ldT, hipStream_t stream);

/* split-bf16 pack (bf16 only): wf [2K][R][R][C] and wT [C][R][R][ldT >= 2K]
 * hold rows k < K = bf16(w[k]) and rows K + k = bf16(w[k] - bf16(w[k])), so a
 * GEMM over the 2K rows whose output pairs (k, K + k) are summed in f32 sees
 * the f32 weight to ~2^-17 relative at bf16 MFMA rates.  Used by the
 * disparity/uncertainty heads (reference model/layers/decoder.py:244-247),
 * whose 4 outputs pad to 8 GEMM columns anyway. */
int um_pack_weight_split(const float* w, int K, int Creal, int R, int C, void* wf, void* wT,
                         int ldT, hipStream_t stream);

/* per-channel column sums of y[M][C] (pixel stride ld) -> partial rows [parts][C] */
/* Several bias gradients (um_colsum + um_reduce_rows each) in two launches:
 * the weight-gradient side stream batches the bias reductions of a flush
 * (the attention's K/Q/V/reprojection and the disparity heads' conv biases,
 * reference model/layers/attention.py:24-33, decoder.py:244-247).  descs:
 * HOST array of n <= UM_CSUM_MAX entries (passed by value); out[c] =
 * sum_m y[m][c] for c < creal, parts = a [nparts][C] f32 workspace with
 * nparts = um_colsum_parts(M); one dtype for all entries. */
#define UM_CSUM_MAX 24
typedef struct {
  const void* y;
  float* parts;
  float* out;
  int M, C, ld, nparts, creal;
} um_csum_desc;
int um_colsum_batch(int dtype, const um_csum_desc* descs, int n, hipStream_t stream);
int um_colsum_parts(int M);
int um_colsum(int dtype, int M, int C, int ld, const void* y, float* partials,
              hipStream_t stream);
/* out[c] (+)= sum_p partials[p][c*1] (row stride `stride`), one launch;
 * ws: um_colred_ws(parts, C, 1) bytes (f64 slab rows of the per-workgroup sums) */
int um_reduce_rows(const float* partials, int parts, int C, int stride, float* out,
                   int accumulate, double* ws, hipStream_t stream);
/* workspace bytes of the one-launch column reductions (nv values per channel) */
long um_colred_ws(int nparts, int C, int nv);

/* ------------------------------------------------------------------ BN ---
 * Training-mode nn.BatchNorm2d + nn.ELU, reference model/layers/encoder.py:43-44,
 * model/layers/decoder.py:82-84; SyncBatchNorm semantics when the host
 * all-reduces the f64 per-channel sums between the phases
 * (reference parallel_main.py:157).
 */
/* f64 per-channel sums of [nparts][C][2] partials (the SyncBN path all-reduces them
 * before um_bn_coeffs / um_bn_bwd_coeffs); ws: um_colred_ws(nparts, C, 2) bytes */
int um_bn_stats_reduce(const float* parts, int nparts, int C, double* out, double* ws,
                       hipStream_t stream);
/* single-process BN: reduce the forward partials AND compute the coefficients
 * (+ running statistics) in one launch (um_bn_stats_reduce + um_bn_coeffs) */
int um_bn_stats_coeffs(const float* parts, int nparts, int C, double* ws, double count,
                       const float* gamma, const float* beta, float eps, float momentum,
                       float* running_mean, float* running_var, long long* num_batches_tracked,
                       float* mean, float* invstd, float* scale, float* shift,
                       hipStream_t stream);
/* single-process BN backward: reduce the bwd partials and compute k1..k3,
 * dgamma, dbeta in one launch (um_bn_stats_reduce + um_bn_bwd_coeffs).
 * dbias (optional): the gradient of the bias of the conv feeding this BN,
 * sum_m dy = k1 (sum dz - n k2 - k3 sum xhat) with sum xhat = 0 by
 * construction of the batch mean -- evaluated in closed form from the
 * reduced sums instead of a reduction of dy over the pixels */
int um_bn_bwd_stats_coeffs(const float* parts, int nparts, int C, double* ws, double count,
                           const float* gamma, const float* invstd, float* dgamma,
                           float* dbeta, float* dbias, float* k1, float* k2, float* k3,
                           hipStream_t stream);
/* count <= 0: read the element count from stats[2C] (SyncBN: the per-rank
 * counts are all-reduced with the statistics) -- also for um_bn_bwd_coeffs */
int um_bn_coeffs(const double* stats, double count, int C, const float* gamma,
                 const float* beta, float eps, float momentum, float* running_mean,
                 float* running_var, long long* num_batches_tracked, float* mean,
                 float* invstd, float* scale, float* shift, hipStream_t stream);
/* pool_parts (optional, SE squeeze of decoder.py:124-136 fused in): per-block
 * channel sums of a, [um_bn_fwd_pool_parts(M, HW)][C], HW = pixels per image */
int um_bn_fwd_pool_parts(long M, long HW);
/* the same for a C-channel layer (the forward pass may split small layers
 * into 64-channel slices with their own row blocking): the pool row count
 * um_bn_elu_fwd / um_bn_elu_fwd_slots write */
int um_bn_fwd_pool_parts_c(long M, long HW, int C);
int um_bn_elu_fwd(int dtype, long M, int C, const void* y, int ldy, const float* scale,
                  const float* shift, void* a, int lda, int apply_elu, long HW, float* pool_parts,
                  hipStream_t stream);
/* BN with the statistics in f64 slots (no reduction launch): the conv ran
 * with UM_EPI_STAT_SLOTS into `slots` ([UM_STAT_SLOTS][C][2], count = M
 * elements per channel); every workgroup sums the slots and derives
 * scale/shift itself, workgroup 0 also writes mean/invstd/scale/shift (kept
 * for the backward) and updates the running statistics -- the semantics of
 * um_bn_stats_coeffs + um_bn_elu_fwd in one launch.  The conv (and
 * um_bn_elu_bwd_reduce_slots) also store the element count after the slots
 * (slots[UM_STAT_SLOTS*C*2], so a slot buffer holds UM_STAT_SLOTS*C*2 + 1
 * doubles); SyncBN all-reduces slots + count and passes count <= 0 to read
 * the global count there. */
int um_bn_elu_fwd_slots(int dtype, long M, int C, const void* y, int ldy, const double* slots,
                        double count, const float* gamma, const float* beta, float eps,
                        float momentum, float* running_mean, float* running_var,
                        long long* num_batches_tracked, float* mean, float* invstd, float* scale,
                        float* shift, void* a, int lda, int apply_elu, long HW, float* pool_parts,
                        hipStream_t stream);
/* um_bn_elu_fwd_slots plus the NodeBlock merge of the next graph node
 * (reference model/layers/encoder.py:115-124): merged = sum_i
 * sigmoid(w[widx[i]]) * src_i over nsrc (2..8) sources [M][lda] of the
 * activation dtype, where source `self` is the a this call writes (srcs[self]
 * is ignored).  Replaces um_bn_elu_fwd_slots + um_merge_fwd when this layer
 * is the last predecessor computed before that node. */
int um_bn_elu_fwd_slots_merge(int dtype, long M, int C, const void* y, int ldy,
                              const double* slots, double count, const float* gamma,
                              const float* beta, float eps, float momentum, float* running_mean,
                              float* running_var, long long* num_batches_tracked, float* mean,
                              float* invstd, float* scale, float* shift, void* a, int lda,
                              int apply_elu, int nsrc, const void* const* srcs, const int* widx,
                              const float* w, int self, void* merged, hipStream_t stream);
/* backward sums (sum dz, sum dz*xhat) added into zeroed f64 slots
 * [UM_STAT_SLOTS][C][2] instead of partial rows */
int um_bn_elu_bwd_reduce_slots(int dtype, long M, int C, long HW, const void* da, int ldda,
                               const void* y, int ldy, const float* mean, const float* invstd,
                               const float* scale, const float* shift, const float* add_nc,
                               int apply_elu, double* slots, hipStream_t stream);
/* dy from the slot sums: every workgroup derives k1..k3 (as
 * um_bn_bwd_stats_coeffs), workgroup 0 writes dgamma, dbeta and the
 * closed-form conv-bias gradient dbias times dbias_scale (each optional).
 * SyncBN: slots are all-reduced (count <= 0 reads the count after them, as
 * um_bn_elu_fwd_slots), local_slots are this rank's slots before the
 * all-reduce (dgamma/dbeta from local sums, as torch SyncBatchNorm) and
 * dbias_scale = 1/world; single process: local_slots null, dbias_scale 1 */
int um_bn_elu_bwd_apply_slots(int dtype, long M, int C, long HW, const void* da, int ldda,
                              const void* y, int ldy, const float* mean, const float* invstd,
                              const float* scale, const float* shift, const float* add_nc,
                              int apply_elu, const double* slots, double count,
                              const double* local_slots, const float* gamma, float* dgamma,
                              float* dbeta, float* dbias, float dbias_scale, void* dy, int lddy,
                              hipStream_t stream);
int um_bn_bwd_parts(long M);
int um_bn_elu_bwd_reduce(int dtype, long M, int C, long HW, const void* da, int ldda,
                         const void* y, int ldy, const float* mean, const float* invstd,
                         const float* scale, const float* shift, const float* add_nc,
                         int apply_elu, float* parts, hipStream_t stream);
/* dbias as in um_bn_bwd_stats_coeffs from the all-reduced sums, times
 * dbias_scale (SyncBN: 1/world, so that the data-parallel gradient average
 * over ranks gives the global sum's average, as the reference's DDP does) */
int um_bn_bwd_coeffs(const double* stats, double count, int C, const float* gamma,
                     const float* invstd, const double* stats_local, float* dgamma,
                     float* dbeta, float* dbias, float dbias_scale, int accumulate, float* k1,
                     float* k2, float* k3, hipStream_t stream);
/* sum_parts (optional): per-block partial sums of dy, [um_bn_bwd_parts(M)][C]
 * (the conv-bias gradient, reduced by um_reduce_rows; only needed when no
 * coefficient kernel supplies it) */
int um_bn_elu_bwd_apply(int dtype, long M, int C, long HW, const void* da, int ldda,
                        const void* y, int ldy, const float* mean, const float* invstd,
                        const float* scale, const float* shift, const float* add_nc,
                        int apply_elu, const float* k1, const float* k2, const float* k3,
                        void* dy, int lddy, float* sum_parts, hipStream_t stream);

/* ------------------------------------------------------- encoder misc ---
 * NodeBlock merge, reference model/layers/encoder.py:115-124 (F3 index map
 * passed in widx: input i weighted by sigmoid(w[widx[i]])).
 */
/* Several um_merge_wgrad calls in ONE launch (one workgroup each): the
 * weight-gradient side stream batches the merge-weight gradients of a flush.
 * descs: HOST array of n <= UM_MWG_MAX entries, passed by value. */
#define UM_MWG_MAX 24
#define UM_MWG_SRC 8
typedef struct {
  const float* parts;  /* [nparts][nsrc] (um_merge_bwd) */
  const float* w;
  float* dw;
  int nparts, nsrc, nw, accumulate;
  int widx[UM_MWG_SRC];
} um_mwg_desc;
int um_merge_wgrad_batch(const um_mwg_desc* descs, int n, hipStream_t stream);
/* coefficient of input i: sigmoid(w[widx[i]]) if w, else coefs[i] (host array), else 1 */
int um_merge_fwd(int dtype, int nsrc, const void* const* srcs, const int* widx,
                 const float* w, const float* coefs, long count, void* dst, hipStream_t stream);
int um_merge_parts(long count);
int um_merge_bwd(int dtype, int nsrc, const void* const* srcs, void* const* dsrcs,
                 const int* accumulate, const int* widx, const float* w, const float* coefs,
                 long count, const void* dm, float* parts, hipStream_t stream);
/* um_merge_bwd that also takes the BN-ELU backward statistics of source fsrc,
 * whose gradient dsrcs[fsrc] it completes (the same sums as
 * um_bn_elu_bwd_reduce_slots over that gradient as stored, into `slots`):
 * reference model/layers/encoder.py:115-124 (merge) + 42-44 (BN+ELU).
 * dtype: activation dtype | UM_Y_ACT (the pre-BN y's type);
 * C / 8 must divide 256 */
/* partial rows of um_merge_bwd_bn's merge-weight dot products (its grid) */
int um_merge_bn_parts(long count);
int um_merge_bwd_bn(int dtype, int nsrc, const void* const* srcs, void* const* dsrcs,
                    const int* accumulate, const int* widx, const float* w, const float* coefs,
                    long count, const void* dm, float* parts, int fsrc, const void* y, int C,
                    const float* mean, const float* invstd, const float* scale,
                    const float* shift, int apply_elu, double* slots, hipStream_t stream);
int um_merge_wgrad(const float* parts, int nparts, int nsrc, const int* widx,
                   const float* w, float* dw, int nw, int accumulate, hipStream_t stream);
int um_image_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, int Cp,
                     void* out, hipStream_t stream);
int um_axpy(int dtype, long n, float alpha, const void* x, void* y, hipStream_t stream);
/* d/dlogit of scale*sigmoid(logit): disp head, reference model/layers/decoder.py:246 */
int um_sigmoid_scale_bwd(int dtype, long M, int C, const float* d, int ldd, const float* dd,
                         int lddd, float scale, void* dlogit, int ldo, hipStream_t stream);
/* split-bf16 head (um_pack_weight_split): forward finish d[m][k] = scale *
 * sigmoid(z[m][k] + z[m][K + k] + bias[k]) over the 2K-column f32 GEMM
 * output z, and the backward's dlogit written to channels k AND K + k (so the
 * data-gradient GEMM over the 2K split rows sums both halves of the weight);
 * channels [2K, ldo) zeroed. */
int um_head_split_fin(long M, int K, const float* z, int ldz, const float* bias, float scale,
                      float* d, int ldd, hipStream_t stream);
int um_sigmoid_scale_bwd_split(int dtype, long M, int C, const float* d, int ldd, const float* dd,
                               int lddd, float scale, void* dlogit, int ldo, hipStream_t stream);
/* One-pass bf16 disparity heads (csrc/disphead.hip), reference
 * model/layers/decoder.py:244-247 (ConvLayer: ReflectionPad2d(1) + Conv2d 3x3,
 * 4 outputs) + :246 (scale * sigmoid).  x NHWC bf16 [N][H][W][ldx] with C in
 * {32, 64, 128, 256} channels, W % 16 == 0 (um_disp_head_ok); wf / wT the
 * split-bf16 weights of um_pack_weight_split with K = 4 ([8][3][3][C] and
 * [C][3][3][8]).
 * fwd  : d[m][k] = scale * sigmoid(sum (w_hi + w_lo) x + bias[k]), d f32 [M][ldd]
 * dgrad: dx (+)= the reflect-pad conv adjoint of dlogit [M][ldl] bf16 (the 8
 *        channels of um_sigmoid_scale_bwd_split), dx bf16 [M][ldx] */
int um_disp_head_ok(int N, int H, int W, int C, int ldx);
int um_disp_head_fwd(int N, int H, int W, int C, const void* x, int ldx, const void* wf,
                     const float* bias, float scale, float* d, int ldd, hipStream_t stream);
int um_disp_head_dgrad(int N, int H, int W, int C, const void* dl, int ldl, const void* wT,
                       void* dx, int ldx, int accumulate, hipStream_t stream);

/* ----------------------------------------------------------- attention ---
 * EfficientAttention core, reference model/layers/attention.py:42-76.
 * qkv [N*S][ld]: K cols [0,C), Q [C,2C), V [2C,3C).
 */
long um_attn_ws_kstats(int N, int S, int C);
long um_attn_ws_ctx(int N, int S, int C, int heads);
long um_attn_ws_tiles(int N, int S, int C, int heads);
int um_attn_fwd(int dtype, int N, int S, int C, int heads, const void* qkv, int ld,
                float* kmax, float* ksum, float* ctx, float* ws, void* att, int ldo,
                hipStream_t stream);
int um_attn_bwd(int dtype, int N, int S, int C, int heads, const void* qkv, int ld,
                const float* kmax, const float* ksum, const float* ctx, const void* datt,
                int ldd, void* dqkv, int ldq, float* dks_ws, float* ws, float* dctx,
                float* r, hipStream_t stream);

/* ------------------------------------------------------------- decoder ---
 * Decoder-stage concat/upsample/pixel-shuffle/SE, reference
 * model/layers/decoder.py:90-136,210-249.
 */
enum { UM_CAT_COPY = 0, UM_CAT_UP2 = 1, UM_CAT_PSHUF = 2 };
typedef struct {
  const void* ptr;     /* source (NHWC, pixel stride ld) */
  const float* scale;  /* optional per-(n,c) gate [N][C] */
  int C, ld, op, coff, dtype, h, w; /* channels, stride, op, dst channel offset, dtype, src size */
} um_cat_src;
int um_concat_build(int dtype, int N, int H, int W, void* dst, int ld, int Ctot, int nsrc,
                    const um_cat_src* srcs, hipStream_t stream);
/* dscale (+=) needs ws: um_concat_bwd_ws(N, src.h, src.w, src.C) floats.
 * accumulate: bit 0 = dsrc (+=), bit 1 = dscale written (=) instead of (+=) */
long um_concat_bwd_ws(int N, int h, int w, int C);
int um_concat_bwd_src(int dtype, int N, int H, int W, const void* g, int ldg,
                      const um_cat_src* src, void* dsrc, int ldd, int dsrc_dtype,
                      int accumulate, float* dscale, float* ws, hipStream_t stream);
int um_channel_mean(int dtype, int N, long S, int C, const void* x, int ld, float* out,
                    hipStream_t stream);
/* pooled[n][c] = inv_hw * sum of the image's parts_per_image pool rows (written
 * for the backward), then z1 = relu(W1 pooled), s = sigmoid(W2 z1) */
int um_se_mlp_fwd(int N, int C, int R, const float* pool_parts, int parts_per_image,
                  float inv_hw, float* pooled, const float* w1, const float* w2, float* z1,
                  float* s, hipStream_t stream);
/* dw1/dw2 written (=); dz: f32 [N][R] scratch */
int um_se_mlp_bwd(int N, int C, int R, const float* ds, const float* s, const float* z1,
                  const float* pooled, const float* w1, const float* w2, float* dw1,
                  float* dw2, float* dpool_scaled, float* dz, float inv_S, hipStream_t stream);

/* ---------------------------------------------------------------- loss ---
 * Loss stack: scale_pyramid (reference train/utils.py:27-50), reconstruct
 * (train/utils.py:65-109), TukraUncertaintyLoss forward/backward
 * (train/loss.py:15-264,340-434,512-568).  Images NCHW f32 [N][6][H][W];
 * predictions NHWC f32 [N][H][W][pld] (d_L, d_R, sigma_L, sigma_R).
 * loss_type: 0 l1, 1 bayesian, 2 log_bayesian (train/loss.py:364-375).
 */
/* image pyramid, every level in ONE launch: out[l] = [NC][H>>l][W>>l], level 0
 * an exact copy (F.interpolate(bilinear, align_corners=True), utils.py:27-50) */
int um_pyramid(const float* x, int NC, int H, int W, int nlevels, float* const* out,
               hipStream_t stream);
/* reconstruct (utils.py:65-97): out = grid_sample(img, linspace grid + sign*disp) */
int um_warp(const float* img, int N, int C, int H, int W, const float* disp, long disp_sn,
            long disp_sp, float sign, float* out, hipStream_t stream);
/* its adjoint w.r.t. the disparity (the image is data): gdisp = sum_c gout_c d(warp_c)/d(disp) */
int um_warp_bwd(const float* img, int N, int C, int H, int W, const float* disp, long disp_sn,
                long disp_sp, float sign, const float* gout, float* gdisp, long g_sn, long g_sp,
                hipStream_t stream);
/* reconstruct_pyramid (utils.py:112-135), every level and both views in ONE
 * launch: out[l] = [N][6][H>>l][W>>l]; pred[l] strided [N][4][h][w] with
 * pred_strides[3l..3l+2] = (image, channel, pixel) strides in elements */
int um_recon_pyramid(int nlevels, int N, int H, int W, const float* const* img,
                     const float* const* pred, const long* pred_strides, float* const* out,
                     hipStream_t stream);
/* TukraUncertaintyLoss.forward (loss.py:512-568) over every scale in ONE launch:
 * img[s] = pyramid level s [N][6][H>>s][W>>s], pred[s] NHWC [N][H>>s][W>>s][4].
 * The recon is re-derived in the kernel (warp of the opposite view).
 * ws: um_loss_ws() bytes of f64 scratch; out[6] = disp_loss, error_loss,
 * wssim, consistency, smoothness, error term (disp_loss / error_loss,
 * optional: out[0] / out[1] again, as the two 0-d loss tensors the reference
 * returns); emap_last (optional) = the last
 * scale's error map [N][2][h][w] (WeightedSSIMLoss.previous_image_error);
 * recon_out (optional, per scale) receives the reconstruction [N][6][h][w]
 * the kernel derives (reconstruct_pyramid's result, as a side output).
 * gpart (optional, per scale NHWC [N][h][w][4] f32): the forward of a step
 * that will differentiate the loss.  The launch then also computes the
 * gradient per unit gout (channels 0/1: d disp_loss / d d_v without the
 * consistency scatter, 2/3: d error_loss / d sigma_v), one tile pass for
 * both, and um_loss_bwd completes it from gpart. */
long um_loss_ws(int nscales, int N, int H, int W);
int um_loss_fwd(int nscales, int N, int H, int W, const float* const* img,
                const float* const* pred, float alpha, int loss_type, float esw, float ecw,
                float w_wssim, float w_cons, float w_smooth, float w_err, double* ws,
                float* emap_last, float* const* recon_out, float* out, float* disp_loss,
                float* error_loss, float* const* gpart, hipStream_t stream);
/* its backward (the reference's autograd through loss.py:512-568):
 * dpred[s] NHWC [N][h][w][4] = d(gout_disp*disp_loss + gout_err*error_loss)/d pred[s]
 * (gout_disp / gout_err: device scalars, NULL = 0).  gpart NULL: two launches (the consistency scatter,
 * then every other term); gpart = um_loss_fwd's partials of the same inputs:
 * ONE launch (the scatter, which scales and completes them). */
int um_loss_bwd(int nscales, int N, int H, int W, const float* const* img,
                const float* const* pred, float alpha, int loss_type, float esw, float ecw,
                float w_wssim, float w_cons, float w_smooth, float w_err,
                const float* gout_disp, const float* gout_err, const float* const* gpart,
                float* const* dpred, hipStream_t stream);
/* WeightedSSIMLoss.image_error (loss.py:96-131) of an explicit recon: out [N][2][H][W] */
int um_image_error(const float* img, const float* rec, int N, int H, int W, float alpha,
                   float* out, hipStream_t stream);

/* ------------------------------------------------------- adversarial ---
 * RandomDiscriminator pieces around its EncoderStages (reference
 * model/discriminator.py:53-86, train/loss.py:267-337).
 */
/* adjoint of um_image_to_nhwc: NHWC [N][H][W][ld] (dtype) -> NCHW f32 [N][C][H][W] */
int um_nhwc_to_image(int dtype, const void* x, int N, int C, int H, int W, int ld, float* out,
                     hipStream_t stream);
/* prob[n] = sigmoid(b + sum w[c*HW + p] x[n][p][c]): Linear over the NCHW flatten + sigmoid */
int um_disc_head_fwd(int dtype, const void* x, int N, int HW, int C, const float* w,
                     const float* bias, float* prob, hipStream_t stream);
int um_disc_head_bwd(int dtype, const void* x, int N, int HW, int C, const float* w,
                     const float* prob, const float* dprob, void* dx, float* dw, float* db,
                     hipStream_t stream);
/* out[0] = mean |a - b| over n elements (ws: um_l1_mean_ws() bytes) and its backward */
long um_l1_mean_ws(void);
int um_l1_mean(int dtype, const void* a, const void* b, long n, double* ws, float* out,
               hipStream_t stream);
int um_l1_mean_bwd(int dtype, const void* a, const void* b, long n, const float* g, void* da,
                   void* db, hipStream_t stream);

/* ---------------------------------------------------------- evaluation ---
 * evaluate_model / sparsification (reference train/evaluate.py:66-196,
 * train/sparsification.py:8-61).  Off the training hot path.
 */
/* torchmetrics structural_similarity_index_measure (gaussian window, sigma ->
 * 11 taps, k1 0.01, k2 0.03) per image: out[n] = mean SSIM over the C x
 * (H-10) x (W-10) full windows; ws: um_ssim_ws() bytes */
long um_ssim_ws(int N, int H, int W);
int um_ssim_gauss(const float* x, const float* y, int N, int C, int H, int W, float data_range,
                  float sigma, double* ws, float* out, hipStream_t stream);
/* nn.AvgPool2d(k, stride=1): out [NC][H-k+1][W-k+1] */
int um_avgpool_valid(const float* x, int NC, int H, int W, int k, float* out, hipStream_t stream);
/* argsort(keys, descending) + gather(vals) per segment of L (nseg segments) */
long um_spars_sort_ws(int nseg, int L);
int um_spars_sort(const float* keys, const float* vals, int nseg, int L, float* keys_out,
                  float* vals_out, void* ws, long ws_bytes, hipStream_t stream);
/* curve[k] = mean_seg( mean(sorted[int(k/steps*L):]) / mean(sorted) ); ws: nseg*steps f64 */
int um_spars_curve(const float* sorted_vals, int nseg, int L, int steps, double* ws,
                   float* curve, hipStream_t stream);

/* ---------------------------------------------------------------- adam ---
 * torch.optim.Adam step, reference train/train.py:228-229.
 */
int um_adam_chunk(void);
int um_adam_step(const void* table, const void* chunks, int nchunks, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int step, hipStream_t stream);
/* graph-replayable: *dstep += 1 on the device, bias corrections from it; lr from *dlr if non-null */
int um_adam_step_dev(const void* table, const void* chunks, int nchunks, float lr,
                     const float* dlr, float beta1, float beta2, float eps, float weight_decay,
                     int* dstep, hipStream_t stream);

/* --------------------------------------------------- input pipeline ---
 * The reference's training transforms (train/transforms.py:15-129 composed
 * in main.py:78-89 / parallel_main.py:111-124: ResizeImage((256, 512)) ->
 * RandomFlip(0.5) -> ToTensor() -> RandomAugment(0.5, ...)) for a batch of
 * both views.  left/right: uint8 [N][Hs][Ws][3] (decoded RGB); the resize is
 * Pillow's 8-bit bilinear resampler (host-made coefficient tables:
 * bounds [out][2] = (first tap, taps), kk [out][ks] 22-bit fixed point),
 * horizontal pass into `tmp` (um_stereo_prep_ws bytes), then the vertical
 * pass, /255, the flip and the augment with per-sample params [N][8] =
 * (flip, augment, gamma, brightness, colour[3], 0) drawn on the host in the
 * reference's order.  out_left/out_right: f32 [N][3][Hd][Wd].
 */
long um_stereo_prep_ws(int N, int Hs, int Wd);
int um_stereo_prep(int N, int Hs, int Ws, const unsigned char* left,
                   const unsigned char* right, int Hd, int Wd, const int* bounds_h,
                   const int* kk_h, int ks_h, const int* bounds_v, const int* kk_v, int ks_v,
                   const float* params, unsigned char* tmp, float* out_left, float* out_right,
                   hipStream_t stream);

/* ------------------------------------------------ SyncBN exchange (IPC) ---
 * SyncBatchNorm statistics exchanged device-side over IPC-mapped per-rank
 * arenas instead of one RCCL all-reduce per layer and direction (reference
 * parallel_main.py:156-158: torch SyncBatchNorm's all-reduce).  Host-only:
 * um_bnx_bytes (arena size for nslots exchanges of <= max_c channels),
 * um_bnx_alloc (uncached arena, zeroed, + its 64-byte hipIpcMemHandle_t),
 * um_bnx_open / um_bnx_close (a peer's arena), um_bnx_free, um_bnx_status
 * (1 if an exchange timed out waiting for a peer).  um_bnx_allreduce: the
 * statistics slots `stats` ([UM_STAT_SLOTS][C][2] f64 + count) of this rank
 * become the rank-ordered sum over all ranks (slot 0; slots 1.. zero; the
 * global count after them) -- the in-place all-reduce of the slots.
 * table: device array of the world arena base addresses (own at [rank]). */
long um_bnx_bytes(int nslots, int max_c);
int um_bnx_alloc(long bytes, void** base, void* handle64);
int um_bnx_open(const void* handle64, void** ptr);
int um_bnx_close(void* ptr);
int um_bnx_free(void* base);
int um_bnx_status(const void* base);
int um_bnx_allreduce(double* stats, int C, const unsigned long long* table, int world, int rank,
                     int slot, int nslots, int max_c, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UMAMD_H */
