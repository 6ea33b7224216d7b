/*
 * sv_kernels.h -- C ABI of the spine-vision MI355X (gfx950) training-path kernel library.
 *
 * This is the drop-in boundary for the north-star hot path of nghiant03/spine-vision: the per-step
 * forward -> backward -> (RCCL all-reduce) -> clip -> AdamW of LocalizationTrainer /
 * ClassificationTrainer.  The reference launches every one of these computations implicitly through
 * timm modules on PyTorch/cuDNN/cuBLAS; the entry points below replace those implicit kernels one for
 * one (or fused).  Reference interfaces replaced (paths relative to the reference repo root):
 *
 *   backbone constructor   timm.create_model(...) at spine_vision/training/models/backbone.py:166-170
 *                          (timm 1.0.22 ConvNeXt / ResNet, not vendored; pinned at uv.lock:3994-3995)
 *   model forward          CoordinateRegressor.forward  spine_vision/training/models/generic.py:380-391
 *                          Classifier.forward           spine_vision/training/models/generic.py:134-145
 *   backward + DDP         accelerator.backward(loss)   spine_vision/training/trainers/base.py:590
 *   clip                   accelerator.clip_grad_norm_  spine_vision/training/trainers/base.py:592-595
 *   optimizer              torch.optim.AdamW            spine_vision/training/trainers/base.py:384-390
 *
 * ABI rules
 *   - plain C types only: raw device pointers, int / int64 sizes, an sv_dtype enum, hipStream_t.
 *   - every entry point is asynchronous on `stream` and returns SV_OK (0) or an sv_status; the message
 *     of the last failure on the calling thread is in sv_last_error_string().
 *   - the library never allocates or frees device memory and never retains a pointer after the call:
 *     activations, saved tensors, partial-sum workspaces and outputs are owned by the caller
 *     (PyTorch's caching allocator in the Python host).
 *   - activations are NHWC: a [rows = B*H*W][C] row-major matrix.  bf16 is passed as uint16 bits.
 */
#ifndef SV_KERNELS_H
#define SV_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* sv_stream_t; /* == hipStream_t */

typedef enum { SV_F32 = 0, SV_BF16 = 1 } sv_dtype;

typedef enum {
  SV_OK = 0,
  SV_ERR_INVALID_ARG = 1,
  SV_ERR_UNSUPPORTED = 2,
  SV_ERR_LAUNCH = 3
} sv_status;

/* ---- library ------------------------------------------------------------------------------- */
int sv_version(void);                        /* ABI version, bumped on any signature change      */
const char* sv_last_error_string(void);      /* thread-local message of the last failing call    */
const char* sv_build_target(void);           /* offload arch the device code was compiled for     */

/* ---- per-device context (sv_ctx_create / sv_ctx_destroy) ---------------------------------
 * The library keeps, per device, the properties its launches are sized by (CU count, LDS per workgroup) and the
 * set of kernels whose dynamic-LDS limit it has raised on that device; every entry point finds its device from the
 * stream it is given, under one mutex, so the library is reentrant across devices and threads.  sv_ctx is the
 * handle to that per-device state: sv_ctx_create(device) queries it now (instead of at the first launch) and
 * returns the device's context (the same handle for the same device, reference-counted); sv_ctx_destroy drops a
 * reference and, at zero, forgets the device's cached state (the next launch queries it again).  Entry points do
 * not take the handle: they work with or without one.                                                          */
typedef struct sv_ctx sv_ctx;
typedef struct sv_ctx_info {
  int32_t device;              /* HIP device ordinal                                                            */
  int32_t compute_units;       /* CUs the persistent grids are sized for                                        */
  int32_t lds_bytes_per_wg;    /* the device's per-workgroup LDS limit (160 KiB on gfx950)                      */
  int32_t xcds;                /* L2 domains the block order is dealt over (8 on MI355X)                         */
  int32_t lds_raised_kernels;  /* kernels whose dynamic-LDS limit the library has raised on this device so far   */
  int32_t refs;                /* live sv_ctx_create references                                                 */
  char arch[32];               /* gcnArchName                                                                   */
} sv_ctx_info;
int sv_ctx_create(int32_t device, sv_ctx** out);
int sv_ctx_destroy(sv_ctx* ctx);
int sv_ctx_get_info(const sv_ctx* ctx, sv_ctx_info* out);

/* ---- data-parallel CU reserve ---------------------------------------------------------------
 * A stream of `device` whose kernels never occupy the CUs listed in `reserved` (n_reserved CU indices in the
 * numbering of hipExtStreamCreateWithCUMask's bit vector), so RCCL's all-reduce kernels -- on streams of their
 * own -- always find free CUs while the backward runs on this one (accelerate DDP's overlap of the gradient
 * exchange with the backward, spine_vision/training/trainers/base.py:253-266).  The stream lives until the
 * process ends (the host wraps it as a torch ExternalStream).  The GEMMs launched on it should cap their
 * persistent grids (sv_gemm_policy.grid_cap) at the unmasked CU count, or their last workgroups queue.  */
int sv_stream_create_cu_reserved(int32_t device, const int32_t* reserved, int32_t n_reserved, sv_stream_t* out);

/* ---- GEMM on MFMA (bf16 in / f32 accumulate, or exact f32 in / f32 accumulate) --------------
 * C[m,n] = epilogue( sum_k A(m,k) * B(k,n) ),  m < M, n < N, k < K.
 *   A(m,k) = A[m*lda + k]  if a_kmajor  else  A[k*lda + m]
 *   B(k,n) = B[n*ldb + k]  if b_kmajor  else  B[k*ldb + n]     (b_kmajor == torch Linear weight)
 * Replaces: timm Mlp.fc1 / fc2 (+GELU, *gamma, +shortcut) and the downsample Conv2d(k2,s2) of
 * ConvNeXt (timm convnext.py ConvNeXtBlock / ConvNeXtStage) and their autograd dgrad / wgrad.     */
typedef enum {
  SV_EPI_STORE = 0,          /* C = acc (+ bias[n])                                               */
  SV_EPI_BIAS_GELU2 = 1,     /* C = acc + bias[n]  (pre-activation), C2 = GELU_erf(C)             */
  SV_EPI_BIAS_GAMMA_RES = 2, /* C = aux[m,n] + gamma[n] * (acc + bias[n])   (layer-scale residual) */
  SV_EPI_GELU_GRAD = 3,      /* C = acc * GELU_erf'(aux[m,n])                                      */
  SV_EPI_SLAB = 4,           /* split-K partial: C[s][m][n] = partial acc of K-slice s (f32, or   */
                             /* bf16 when c_dtype is SV_BF16: v9 weight-gradient shapes only);     */
                             /* if C2 != NULL also C2[s][m] = sum_{k in slice s} A(m,k) (f32), i.e.  */
                             /* the bias gradient of a wgrad GEMM (A = dY^T) without another pass.   */
  SV_EPI_BIAS_GELU_DUAL = 5, /* h = acc + bias[n]: C = GELU_erf'(h), C2 = GELU_erf(h)  (fc1 forward: */
                             /* the backward then needs no erf, only SV_EPI_MUL_AUX)                 */
  SV_EPI_MUL_AUX = 6,        /* C = acc * aux[m,n]                       (fc2 dgrad through GELU)    */
  SV_EPI_BIAS_GELU = 7,      /* C = GELU_erf(acc + bias[n])   (fc1 of the tape-free eval forward:   */
                             /* one output, no GELU' for a backward that will not run)             */
  SV_EPI_STORE_STATS = 8,    /* C = acc (+ bias[n]) and the train-mode BatchNorm statistics of C:  */
                             /* C2 (f32) [ceil(M/64)][2][N] = per 64-row group, column sum and sum */
                             /* of squares of the values as stored (rounded to c_dtype); bf16 only, */
                             /* N % 8 == 0, v3 kernels (a shape they cannot take is an error)      */
  SV_EPI_STORE_BN_BWD = 9,   /* C = acc (bf16: the gradient g0 at a BatchNorm + ReLU output, e.g. a */
                             /* data gradient) and that BatchNorm's backward statistics: C2 (f32)   */
                             /* [ceil(M/64)][2][N] = per 64-row group, sum g and sum g*xhat, g = C  */
                             /* as stored * (fmaf(gamma*rstd, y-mean, beta) > 0), xhat =            */
                             /* (y-mean)*rstd, y = aux (bf16, the BatchNorm input), the parameters */
                             /* in `bn`; bias NULL, N % 8 == 0, k-major A, m-major B, v3 kernels    */
  SV_EPI_LN_BWD = 10         /* the LayerNorm backward over C's rows, C never stored (round 6: the  */
                             /* ConvNeXt fc1 data gradient at C >= 512, ConvNeXtBlock.norm's      */
                             /* backward in the GEMM's epilogue): dy = bf16(acc) is the gradient at */
                             /* the LayerNorm output; x^ = (aux - bn->mean[m]) * bn->rstd[m] with   */
                             /* aux the saved LayerNorm input z (bf16, ld_aux); w = bn->gamma [N];  */
                             /*   C[m,n]  = bf16( rstd (dy w - mean_n(dy w) - x^ mean_n(dy w x^)) ) */
                             /*   C2 (f32) [2][ceil(M/128)][N] = per 128-row group, sum dy x^ and    */
                             /*   sum dy (the weight / bias gradient partials).                     */
                             /* The row sums span the whole row: the workgroups of a row block's    */
                             /* N / 256 column tiles exchange theirs through fold_out (f32 work-    */
                             /* space [ceil(M/256)][N/256][256][2]) and fold_counters (int32        */
                             /* [2 ceil(M/256)], zero on entry and left zero).  v9 only, bf16, k-   */
                             /* major A, N % 256 == 0, N <= 1024, one workgroup per tile resident   */
                             /* (else SV_ERR_UNSUPPORTED: the caller runs the two-pass form).       */
} sv_epilogue;

/* The BatchNorm whose backward statistics SV_EPI_STORE_BN_BWD / sv_gemm_slab_finish_bn_bwd compute
 * (device pointers, f32 [N]; the forward's batch mean / rstd and the affine parameters).             */
typedef struct {
  const float* mean;
  const float* rstd;
  const float* gamma;
  const float* beta;
} sv_bn_ref;

/* Launch policy of the GEMM kernels behind ONE call (sv_gemm, the sv_conv_* entry points).  It travels
 * with the call -- there is no process-wide GEMM state -- so launches from other streams, models, threads
 * or devices of the same process are never affected.  A zero-initialised policy is the default schedule.  */
typedef struct {
  int32_t impl;      /* 0 = the measured per-shape dispatch; 2 / 3 / 8 / 9 = force that kernel family where its
                      * contract holds (tests/test_gemm_family_gpu.py compares the families bit for bit)      */
  int32_t grid_cap;  /* > 0: the persistent v3 / v9 grids run on at most this many workgroups (the ResNet side
                      * stream's weight gradients; CUs left to RCCL under data parallelism); 0 = every CU of
                      * the stream's device.  Persistent over their tiles, so the results are bitwise unchanged */
  int32_t wg_per_cu; /* 0 = one workgroup per output tile; 1..2 = persistent grids of n workgroups per CU, so
                      * GEMMs issued on two streams at once (data + weight gradients) share every CU         */
  int32_t priority;  /* 1 = the v3 K loop's waves at raised s_setprio (critical-path GEMM beside another
                      * stream's kernels); 0 = normal.  Bitwise neutral                                    */
} sv_gemm_policy;

typedef struct {
  int32_t M, N, K;
  const void* A; int32_t a_dtype; int32_t a_kmajor; int64_t lda;
  const void* B; int32_t b_dtype; int32_t b_kmajor; int64_t ldb;
  const float* a_scale_k;    /* optional: A(m,k) *= a_scale_k[k]                                  */
  int32_t epilogue;          /* sv_epilogue                                                       */
  void* C; int32_t c_dtype; int64_t ldc;
  void* C2; int32_t c2_dtype; /* second output: SV_EPI_BIAS_GELU2 (same ldc) / SV_EPI_SLAB colsum  */
  const float* bias;         /* [N] or NULL                                                       */
  const float* gamma;        /* [N]  (SV_EPI_BIAS_GAMMA_RES)                                      */
  const void* aux; int32_t aux_dtype; int64_t ld_aux; /* residual / pre-activation input          */
  int32_t split_k;           /* SV_EPI_SLAB: number of K slices (>= 1); slab stride = M*N floats  */
  int32_t compute;           /* SV_BF16: bf16 MFMA (operands rounded to bf16); SV_F32: f32 MFMA    */
  const sv_bn_ref* bn;       /* SV_EPI_STORE_BN_BWD: the BatchNorm (NULL otherwise)                */
  sv_gemm_policy policy;     /* launch policy of THIS call (zero-initialised = the defaults)      */
  /* SV_EPI_SLAB with fold_out != NULL: the split-K fold as well, fold_out[m][n] (row stride fold_ld, f32) =  */
  /* (fold_accumulate ? fold_out : 0) + sum_s C[s][m][n], slices in order s = 0, 1, ... (bitwise the         */
  /* sv_reduce_partials fold of the slabs).  The persistent v9 kernel folds in place: when every (tile,      */
  /* slice) unit has a workgroup and the grid is at most half the CUs, each slice's workgroup waits for its  */
  /* tile's other slices and sums 1/split of the tile's rows; otherwise the last workgroup to finish a       */
  /* tile's slice sums that tile (no waiting).  fold_counters = int32 [2 * ceil(M/256) * ceil(N/256)], all   */
  /* zero on entry and left zero (one buffer per stream).  Other kernels fold with a separate pass.  C2      */
  /* (the column sums) is not folded.  ABI version 3.                                                        */
  float* fold_out; int64_t fold_ld; int32_t fold_accumulate; int32_t* fold_counters;
} sv_gemm_desc;

int sv_gemm(const sv_gemm_desc* d, sv_stream_t stream);
/* Finish of a split-K GEMM (SV_EPI_SLAB): C[m, n] = (accumulate ? C[m, n] : 0) + sum_s slab[s][m][n],
 * slices summed in order (deterministic); c_dtype f32 or bf16 (accumulate into bf16: the sum in f32, stored
 * bf16 -- the ResNet bf16 gradient stream).  stats != NULL
 * (bf16 C): also the SV_EPI_STORE_STATS partials [ceil(M/64)][2][N] of the values as stored.
 * N, ldc multiples of 4; slab, C, stats 16-byte aligned.                                          */
int sv_gemm_slab_finish(const float* slab, int32_t split, int32_t M, int32_t N, void* C, int32_t c_dtype, int64_t ldc,
                        int32_t accumulate, float* stats, sv_stream_t stream);
/* The same finish into a bf16 C (the split-K data gradient g0 at the output of a BatchNorm + ReLU) plus
 * that BatchNorm's backward statistics: part (f32) [ceil(M/64)][2][N] = per 64-row group, sum g and
 * sum g*xhat, g = g0 as stored * (fmaf(gamma*rstd, y-mean, beta) > 0), xhat = (y-mean)*rstd, y (bf16,
 * row stride N) the BatchNorm input -- the products of sv_bn_relu_bwd_stats, so bn_bwd needs no
 * statistics pass.  N % 4 == 0; slab, C, y, part and the bn vectors 16-byte aligned.                */
int sv_gemm_slab_finish_bn_bwd(const float* slab, int32_t split, int32_t M, int32_t N, void* C, const void* y,
                               const sv_bn_ref* bn, float* part, sv_stream_t stream);

/* ---- Fused ConvNeXt MLP forward (narrow stages) ------------------------------------------------
 * Replaces ConvNeXtBlock.mlp.fc1 -> GELU -> mlp.fc2 -> x gamma -> + shortcut (timm convnext.py; the two
 * sv_gemm calls SV_EPI_BIAS_GELU_DUAL / SV_EPI_BIAS_GELU then SV_EPI_BIAS_GAMMA_RES) in ONE kernel: the
 * hidden activation streams through registers in 64-unit chunks and never reaches HBM as fc2's operand.
 *   h = y . w1^T + b1;  x_out = gamma (.) (bf16(GELU(h)) . w2^T + b2) + x
 * y [M, C] bf16, w1 [4C, C] bf16 (torch Linear layout), b1 [4C] f32, w2 [C, 4C] bf16, b2 / gamma [C] f32,
 * x / x_out [M, C] f32 (must not alias).  gelu_grad / gelu_out [M, 4C] bf16, both or neither: the
 * training forward stores GELU'(h) and GELU(h) for the backward (bit for bit the dual epilogue's), the
 * eval forward passes NULL.  C in {128, 192, 256, 512} (512: the opt-in S3 kernel, measured slower than the two
 * GEMMs and not taken by default); every pointer 16-byte aligned; M * 4C * 2 < 2^31.
 * x_out is bit for bit the unfused pair's.                                                           */
int sv_mlp_fwd(const uint16_t* y, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
               const float* gamma, const float* x, float* x_out, uint16_t* gelu_grad, uint16_t* gelu_out, int64_t M,
               int32_t C, sv_stream_t stream);

/* Fused backward of the same block part at C = 128 (ConvNeXt-base S1): from d [M, C] bf16 (the bf16 copy of the
 * gradient at the block output),
 *   dh = bf16((d . w2t^T) (.) gelu_grad)        [M, 4C] bf16 (the fc1 weight gradient's operand)
 *   dy = bf16(dh . w1t^T)                        kept on chip
 *   dz = LayerNorm backward of dy over (z bf16 [M, C], mean, rstd [M], lnw [C])   [M, C] bf16
 * and the LayerNorm weight / bias partial sums ln_part [2][P][C] (sum dy x^, sum dy; P = sv_mlp_bwd_nparts(M, C),
 * fold with sv_reduce_partials_multi).  w2t = bf16(W2 gamma)^T [4C, C] and w1t = bf16(W1)^T [C, 4C]
 * (sv_transpose_scale_bf16).  Replaces the fc2 data gradient (SV_EPI_MUL_AUX), the fc1 data gradient and
 * sv_layernorm_bwd of the block: dh is bit for bit theirs, dz and the sums within f32 summation order.
 * Every pointer 16-byte aligned; M * 4C * 2 < 2^31.                                                   */
int sv_mlp_bwd_nparts(int64_t M, int32_t C);
int sv_mlp_bwd(const uint16_t* d, const uint16_t* w2t, const uint16_t* gelu_grad, const uint16_t* w1t, const uint16_t* z,
               const float* mean, const float* rstd, const float* lnw, uint16_t* dh, uint16_t* dz, float* ln_part,
               int64_t M, int32_t C, sv_stream_t stream);

/* ---- LayerNorm over the channel (last) dim -------------------------------------------------
 * Replaces timm LayerNorm / LayerNorm2d (eps 1e-6) on channels-last rows.
 * fwd: y = (x-mean)*rstd*w + b; saves mean/rstd [rows] (f32).
 * bwd: dx = rstd*(g - mean_c(g) - xhat*mean_c(g*xhat)), g = dy*w;  dx written (accumulate=0) or
 *      added (accumulate=1);  per-block partial sums of dw = sum dy*xhat, db = sum dy are written to
 *      dw_part/db_part [nparts][C]; nparts = sv_layernorm_bwd_nparts(rows, C).                       */
int sv_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                     int32_t y_dtype, float* mean, float* rstd, int64_t rows, int32_t C, float eps,
                     sv_stream_t stream);
int sv_layernorm_bwd_nparts(int64_t rows, int32_t C);
/* dy/x/dx dtype combinations: (f32,f32,f32), (f32,bf16,f32), (f32,bf16,bf16), (bf16,bf16,f32),
 * (bf16,bf16,bf16).                                                                                */
int sv_layernorm_bwd(const void* dy, int32_t dy_dtype, const void* x, int32_t x_dtype, const float* mean,
                     const float* rstd, const float* w, void* dx, int32_t dx_dtype, int32_t accumulate,
                     float* dw_part, float* db_part, int64_t rows, int32_t C, sv_stream_t stream);

/* ---- ConvNeXt block head: depthwise 7x7 (pad 3, bias) fused with the channels-last LayerNorm --
 * Replaces ConvNeXtBlock.conv_dw + permute + ConvNeXtBlock.norm (timm convnext.py).
 * x [B,H,W,C] (x_dtype), wdw [C][49] (timm weight [C,1,7,7]), bdw [C].
 * outputs: z = dwconv(x) (saved for backward, z_dtype), y = LN(z) (y_dtype), mean/rstd [B*H*W].  */
int sv_dwconv7_ln_fwd(const void* x, int32_t x_dtype, const float* wdw, const float* bdw,
                      const float* lnw, const float* lnb, float eps, void* z, int32_t z_dtype, void* y,
                      int32_t y_dtype, float* mean, float* rstd, int32_t B, int32_t H, int32_t W,
                      int32_t C, sv_stream_t stream);
/* diagnostic: per lane, the sum over its group of `lanes` (16 / 32 / 64) lanes by the cross-lane butterfly the
 * LayerNorm kernels use (xlane) and by the ds_bpermute shuffle butterfly (shuffle); the two are bitwise equal.
 * n: a multiple of 256.                                                                                       */
int sv_diag_group_sum(const float* in, float* xlane, float* shuffle, int64_t n, int32_t lanes, sv_stream_t stream);
/* 1 when sv_dwconv7_ln_fwd may be called with z == NULL for these arguments: it then runs as ONE pass (depthwise conv
 * and block LayerNorm in one workgroup per strip: C = 128 / 256 / 512, f32 x, z and y of one dtype) and writes no conv
 * output (the eval forward).  With z given it runs the two launches (SV_DW_LN_FUSED=1: the one pass there too).
 * y / mean / rstd (and z) are bitwise the same either way.                                                          */
int sv_dwconv7_ln_fused_ok(int32_t B, int32_t H, int32_t W, int32_t C, int32_t x_dtype, int32_t z_dtype,
                           int32_t y_dtype);
/* backward-data of the depthwise conv: dx[p] = (accumulate ? dx[p] : 0) + sum_tap w*dz; if dx_bf16
 * != NULL it also receives bf16(dx) -- the GEMM-operand copy of the gradient stream.  dz: f32 or bf16
 * (dz_dtype), dx: f32.                                                                             */
int sv_dwconv7_bwd_data(const void* dz, int32_t dz_dtype, const float* wdw, float* dx, uint16_t* dx_bf16,
                        int32_t accumulate, int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream);
/* backward-weight: per-workgroup partials dw_part [nparts][C*49], db_part [nparts][C].             */
int sv_dwconv7_bwd_weight_nparts(int32_t B, int32_t H, int32_t W, int32_t C);
int sv_dwconv7_bwd_weight(const void* dz, int32_t dz_dtype, const void* x, int32_t x_dtype, float* dw_part,
                          float* db_part, int32_t B, int32_t H, int32_t W, int32_t C,
                          sv_stream_t stream);

/* ---- the depthwise conv on the matrix cores (csrc/dwmfma.hip, round 6) --------------------------------
 * Per channel a banded-Toeplitz GEMM along the image row on v_mfma_f32_16x16x32_bf16.  Operands are rounded to bf16
 * (x or dz and the taps: the precision torch.autocast gives conv_dw), products exact, sums in f32.  C % 32 == 0.
 *   fwd:       z (bf16) = bf16(bdw + sum_tap bf16(w) * bf16(x)),  x f32 or bf16 [B,H,W,C] (x_dtype)
 *   bwd-data:  dx (f32) = (accumulate ? dx : 0) + sum_tap bf16(w[48 - tap]) * dz,  dz bf16; dx_bf16 (nullable)
 *              receives bf16(dx).  Same contract as sv_dwconv7_bwd_data with dz_dtype = bf16.                  */
int sv_dwconv7_fwd_mfma(const void* x, int32_t x_dtype, const float* wdw, const float* bdw, uint16_t* z, int32_t B,
                        int32_t H, int32_t W, int32_t C, sv_stream_t stream);
int sv_dwconv7_bwd_data_mfma(const uint16_t* dz, const float* wdw, float* dx, uint16_t* dx_bf16, int32_t accumulate,
                             int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream);
/* backward-weight on the matrix cores: the 7 x 7 taps of a channel are one 16 x 16 MFMA accumulator summed over the
 * tile's pixels (D[kr][j] = sum_(m,n') x[m + kr][n'] dz[m][n' - j]); dz bf16, x f32 or bf16 rounded to bf16.
 * Per-workgroup partials dw_part [nparts][C*49], db_part [nparts][C] as sv_dwconv7_bwd_weight's, nparts =
 * sv_dwconv7_bwd_weight_mfma_nparts(...).  C % 16 == 0.                                                           */
int sv_dwconv7_bwd_weight_mfma_nparts(int32_t B, int32_t H, int32_t W, int32_t C);
int sv_dwconv7_bwd_weight_mfma(const uint16_t* dz, const void* x, int32_t x_dtype, float* dw_part, float* db_part,
                               int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream);

/* ---- ConvNeXt stem: Conv2d(3, C, k=4, s=4) + LayerNorm2d, fused --------------------------------
 * img: NCHW f32 [B,3,H,W] (ImageNet-normalised, = the reference batch["image"]); w [C][3*16]
 * (timm stem.0.weight), b [C]; y: NHWC [B,H/4,W/4,C] (y_dtype); mean/rstd [B*H/4*W/4].            */
int sv_stem_patchify_ln_fwd(const float* img, const float* w, const float* b, const float* lnw,
                            const float* lnb, float eps, void* y, int32_t y_dtype, float* mean,
                            float* rstd, int32_t B, int32_t H, int32_t W, int32_t C,
                            sv_stream_t stream);
/* backward (weights only; the image needs no gradient): partials [nparts][C*48], [nparts][C] x3. */
int sv_stem_patchify_ln_bwd_nparts(int32_t B, int32_t H, int32_t W, int32_t C);
int sv_stem_patchify_ln_bwd(const float* img, const float* w, const float* b, const float* lnw,
                            const float* mean, const float* rstd, const float* dy, float* dw_part,
                            float* db_part, float* dlnw_part, float* dlnb_part, int32_t B, int32_t H,
                            int32_t W, int32_t C, sv_stream_t stream);

/* ---- ConvNeXt stem on MFMA (bf16 mode) + the batch input transform on the GPU -------------------
 * The stem conv as one sv_gemm: patches [B*(H/4)*(W/4)][64] bf16 (k = ci*16 + kh*4 + kw, the
 * flattened timm stem.0.weight [C,3,4,4]; k 48..63 zero) x wpack [C][64] bf16 (zero padded).
 * img_kind SV_IMG_F32_NCHW: the reference batch["image"] [B,3,H,W] f32 (already normalised);
 * SV_IMG_U8_GRAY: the decoded uint8 grayscale batch [B,H,W]; the reference transform
 * (training/datasets/localization.py:196-233, 254: convert("RGB") -> ToTensor -> Normalize) is
 * applied in flight as (u / 255 - mean[c]) / std[c] in f32.  norm_mean / norm_std: HOST float[3]
 * (ignored for SV_IMG_F32_NCHW, may be NULL).                                                      */
typedef enum { SV_IMG_F32_NCHW = 0, SV_IMG_U8_GRAY = 1 } sv_image_kind;
int sv_stem_patchify(const void* img, int32_t img_kind, const float* norm_mean, const float* norm_std,
                     uint16_t* patches, int32_t B, int32_t H, int32_t W, sv_stream_t stream);
int sv_stem_weight_pack(const float* w, uint16_t* wpack, int32_t C, sv_stream_t stream);
/* The same transform as a standalone op (row f1 of the scope table: the collator's ToTensor +
 * Normalize on the device): img uint8 [B,H,W] -> out f32 [B,3,H,W], bitwise equal to torchvision's
 * CPU result on the replicated RGB image.  H*W % 4 == 0; mean/std HOST float[3].                   */
int sv_normalize_u8_gray(const uint8_t* img, const float* norm_mean, const float* norm_std, float* out,
                         int32_t B, int32_t H, int32_t W, sv_stream_t stream);

/* ---- train-time augmentation of decoded uint8 images (row f1) ----------------------------------
 * Replaces the PIL/torchvision tail of the reference's train transforms after Resize
 * (training/datasets/localization.py:202-216: RandomHorizontalFlip(0.5), RandomAffine(10, (0.05,
 * 0.05), (0.95, 1.05)), ColorJitter(0.2, 0.2); classification.py:276-289: RandomAffine +
 * ColorJitter) with the SAME pixel arithmetic as Pillow's NEAREST affine and ImageEnhance blends.
 * in/out uint8 [B][H][W][C] (C = 1 grayscale plane or 3 interleaved RGB; must not alias);
 * params double [B][10] = {flip, inverse affine a0..a5, brightness, contrast, order (0 = brightness
 * first)} drawn on the host as torchvision draws them; row_sums int32 [B*H] workspace.             */
int sv_augment_u8(const uint8_t* in, uint8_t* out, int32_t B, int32_t H, int32_t W, int32_t C, const double* params,
                  int32_t* row_sums, sv_stream_t stream);

/* ---- resize of decoded uint8 images (row f1) ---------------------------------------------------
 * Replaces the reference's first transform, torchvision Resize(size) on a PIL image
 * (training/datasets/localization.py:199, classification.py:250) = PIL Image.resize((W, H),
 * BILINEAR): Pillow's two-pass fixed-point resample (libImaging/Resample.c, PRECISION_BITS 22, the
 * horizontal pass rounded to uint8), bit for bit.  Ragged batch of B source images [h][w][C] at byte
 * offsets in src; desc int64 [B][8] = {src offset, h, w, x-table offset, x taps, y-table offset, y
 * taps, 0}; coef int32 tables (per axis: bounds[out][2] = {first tap, count}, then coef[out][taps]),
 * built on the host exactly as Pillow's precompute_coeffs / normalize_coeffs_8bpc
 * (spine_vision_amd.training.datasets.resize).  dst uint8 [B][H][W][C], C = 1 or 3.              */
int sv_resize_u8(const uint8_t* src, const int64_t* desc, const int32_t* coef, int32_t B, int32_t H, int32_t W,
                 int32_t C, uint8_t* dst, sv_stream_t stream);

/* ---- ConvNeXt stage downsample: LayerNorm2d + 2x2/s2 patch gather (GEMM A operand) ------------
 * x [B,H,W,C] f32 -> patches [B*(H/2)*(W/2)][C*4] with k = c*4 + kh*2 + kw (= timm conv weight
 * [2C,C,2,2] flattened), so the Conv2d(k2,s2) is one sv_gemm with b_kmajor=1 on the weight.        */
int sv_downsample_ln_patch2_fwd(const float* x, const float* lnw, const float* lnb, float eps,
                                void* patches, int32_t p_dtype, float* mean, float* rstd, int32_t B,
                                int32_t H, int32_t W, int32_t C, sv_stream_t stream);
/* dpatches (f32, same layout) -> dx [B,H,W,C] (written), LN weight partials [nparts][C].           */
int sv_downsample_ln_patch2_bwd_nparts(int32_t B, int32_t H, int32_t W, int32_t C);
int sv_downsample_ln_patch2_bwd(const float* dpatches, const float* x, const float* mean,
                                const float* rstd, const float* lnw, float* dx, uint16_t* dx_bf16, float* dlnw_part,
                                float* dlnb_part, int32_t B, int32_t H, int32_t W, int32_t C,
                                sv_stream_t stream);

/* ---- backbone head: global average pool + LayerNorm (timm NormMlpClassifierHead, num_classes=0) -
 * x [B,HW,C] f32 -> feat [B,C] f32; saves pooled [B,C], mean/rstd [B].                             */
int sv_pool_ln_fwd(const float* x, const float* lnw, const float* lnb, float eps, float* pooled,
                   float* feat, float* mean, float* rstd, int32_t B, int32_t HW, int32_t C,
                   sv_stream_t stream);
/* dfeat [B,C] -> dx [B,HW,C] (written, + optional bf16 copy); dlnw/dlnb partials [B][C].        */
int sv_pool_ln_bwd(const float* dfeat, const float* pooled, const float* mean, const float* rstd,
                   const float* lnw, float* dx, uint16_t* dx_bf16, float* dlnw_part, float* dlnb_part, int32_t B,
                   int32_t HW, int32_t C, sv_stream_t stream);

/* ---- reductions used by backward -------------------------------------------------------------
 * Grouped partial-sum reduction (group >= P or <= 0: one group):
 *   out[g*n + i] = (accumulate ? out[g*n + i] : 0) + alpha * sum_{p in [g*group, (g+1)*group)} part[p*n + i]
 * The host reduces deep split-K slabs in two passes (groups, then the group sums).                 */
/* one-launch variant for two independent segments sharing the partial count P (a weight gradient and
 * its bias gradient): out_s[i] (+)= alpha * sum_p part_s[p*n_s + i]; n_b = 0 for a single segment.   */
/* Up to SV_MAX_RED_SEGS independent partial reductions (out_s (+)= alpha * sum_p part_s[p][:]) in ONE launch
 * -- the per-block weight-gradient folds the reference gets from autograd's accumulation (fc1 wgrad slab +
 * bias, LayerNorm and depthwise weight / bias partials), each in a fixed order (deterministic).  segs is a
 * HOST array.                                                                                         */
#define SV_MAX_RED_SEGS 8
typedef struct {
  const float* part; /* [P][n] f32 partial rows (16-B aligned when n % 4 == 0) */
  float* out;        /* [n] f32 */
  int64_t n;
  int32_t P;
  int32_t accumulate;
} sv_red_seg;
int sv_reduce_partials_multi(const sv_red_seg* segs, int32_t nseg, float alpha, sv_stream_t stream);

int sv_reduce_partials_pair(const float* part_a, int64_t n_a, float* out_a, const float* part_b, int64_t n_b,
                            float* out_b, int32_t P, float alpha, int32_t accumulate, sv_stream_t stream);
int sv_reduce_partials(const float* part, int32_t P, int32_t group, int64_t n, float* out, float alpha,
                       int32_t accumulate, sv_stream_t stream);
/* sv_reduce_partials (one group) over bf16 partial rows part[P][n] (the bf16 split-K slabs of a weight gradient,
 * sv_gemm SV_EPI_SLAB with c_dtype SV_BF16): out (+)= alpha * sum_p part[p], f32 sums in slice order.
 * n % 4 == 0: part 8-B and out 16-B aligned.  ABI version 5.                                          */
int sv_reduce_partials_bf16(const uint16_t* part, int32_t P, int64_t n, float* out, float alpha, int32_t accumulate,
                            sv_stream_t stream);
/* column sums of a [rows][C] matrix into partials [nparts][C]; nparts = sv_colsum_nparts(rows,C). */
int sv_colsum_nparts(int64_t rows, int32_t C);
int sv_colsum(const void* x, int32_t x_dtype, int64_t rows, int32_t C, float* part,
              sv_stream_t stream);
/* layer-scale fc2 weight-gradient finish.  G[C][K4] = d_out^T * GELU(h) (reduced, f32),
 * cs[C] = colsum(d_out).  Accumulates: dW2 += gamma (.) G (row scale), dgamma += rowdot(W2, G) +
 * b2 (.) cs, db2 += gamma (.) cs.                                                                   */
int sv_layerscale_wgrad_finish(const float* G, const float* cs, const float* W2, const float* gamma,
                               const float* b2, float* dW2, float* dgamma, float* db2, int32_t C,
                               int32_t K4, sv_stream_t stream);

/* fc2 weight-gradient finish fused with its split-K reduction (replaces sv_reduce_partials_pair +
 * sv_layerscale_wgrad_finish): slab[P][C][K4] and cs_part[P][C] are the SV_EPI_SLAB outputs of the
 * wgrad GEMM d_out^T * GELU(h); same accumulation semantics as sv_layerscale_wgrad_finish.  One
 * workgroup per row; ws is unused (sv_layerscale_wgrad_reduce_ws returns 0, ws may be NULL).
 * K4 % 4 == 0.                                                                                       */
int sv_layerscale_wgrad_reduce_ws(int32_t C, int32_t K4);
int sv_layerscale_wgrad_reduce(const float* slab, const float* cs_part, int32_t P, const float* W2,
                               const float* gamma, const float* b2, float* dW2, float* dgamma, float* db2,
                               float* ws, int32_t C, int32_t K4, sv_stream_t stream);
/* sv_layerscale_wgrad_reduce over bf16 slabs slab[P][C][K4] (sv_gemm SV_EPI_SLAB with c_dtype SV_BF16); the
 * column-sum partials stay f32.  slab 8-B aligned.  ABI version 5.                                    */
int sv_layerscale_wgrad_reduce_bf16(const uint16_t* slab, const float* cs_part, int32_t P, const float* W2,
                                    const float* gamma, const float* b2, float* dW2, float* dgamma, float* db2, int32_t C,
                                    int32_t K4, sv_stream_t stream);
/* The same finish over the ALREADY FOLDED G[C][K4] (the wgrad GEMM's in-kernel fold, sv_gemm_desc.fold_out) and
 * the P column-sum partials cs_part[P][C]: bitwise sv_layerscale_wgrad_reduce of the P slabs whose sum is G.  */
int sv_layerscale_wgrad_fold_finish(const float* G, const float* cs_part, int32_t P, const float* W2, const float* gamma,
                                    const float* b2, float* dW2, float* dgamma, float* db2, int32_t C, int32_t K4,
                                    sv_stream_t stream);

/* ---- optimizer step on flat buffers (all params of the model live in one f32 buffer) ----------
 * Replaces accelerator.clip_grad_norm_ (torch.nn.utils.clip_grad_norm_) + torch.optim.AdamW.step.
 * sqnorm: per-block partial sums of g^2 -> part[nparts]; clip_coef: coef = min(1, max_norm /
 * (sqrt(sum)+1e-6)) written to out[1], total norm to out[0] (device scalars; no host sync).        */
int sv_sqnorm_nparts(int64_t n);
int sv_sqnorm_partial(const float* g, int64_t n, float* part, sv_stream_t stream);
int sv_clip_coef(const float* part, int32_t nparts, float max_norm, float* out, sv_stream_t stream);
/* AdamW (decoupled weight decay, torch semantics, amsgrad=False, maximize=False):
 *   g' = g * (*grad_scale) (if grad_scale != NULL);  p *= 1 - lr*wd;
 *   m = b1*m + (1-b1) g';  v = b2*v + (1-b2) g'^2;
 *   p -= (lr / (1-b1^step)) * m / (sqrt(v)/sqrt(1-b2^step) + eps)
 * and, if p_bf16 != NULL, p_bf16 = bf16(p) (the shadow the MFMA kernels read next step).          */
int sv_adamw_flat(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n,
                  float lr, float beta1, float beta2, float eps, float weight_decay, int32_t step,
                  const float* grad_scale, sv_stream_t stream);
/* sv_adamw_flat with the per-step scalars read from DEVICE memory: hyper = f32 [lr, 1 - b1^step,
 * sqrt(1 - b2^step)] (the host values sv_adamw_flat derives from `step`, rounded to f32 the same way).
 * A captured HIP graph replays the update with the scalars the host writes into `hyper` before each
 * launch (StepEngine(cuda_graph=True)).                                                             */
int sv_adamw_flat_dev(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float beta1,
                      float beta2, float eps, float weight_decay, const float* hyper, const float* grad_scale,
                      sv_stream_t stream);
/* out[r][k] = bf16(W[r][k] * scale[r]): fc2 weight with the layer-scale gamma folded in, so the fc2
 * dgrad GEMM reads bf16 operands only.                                                              */
/* out[c][r] = bf16(W[r][c] * (scale ? scale[r] : 1)) for W [rows, cols] f32: the transposed bf16 operand images of
 * sv_mlp_bwd (scale = gamma for the fc2 weight, NULL for the fc1 weight).                             */
int sv_transpose_scale_bf16(const float* W, const float* scale, uint16_t* out, int32_t rows, int32_t cols,
                            sv_stream_t stream);
int sv_scale_rows_bf16(const float* W, const float* scale, uint16_t* out, int32_t rows, int32_t cols,
                       sv_stream_t stream);
/* y = bf16(x) over n elements (weight shadows after load_state_dict / init).                       */
int sv_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, sv_stream_t stream);

/* ---- ResNet-18/50 (ClassificationTrainer backbone) -------------------------------------------
 * Replaces timm ResNet (BasicBlock / Bottleneck, timm/models/resnet.py, not vendored) built at
 * spine_vision/training/models/backbone.py:166 for "resnet18"/"resnet50" (backbone.py:27,29) and run
 * by Classifier.forward (generic.py:134-145) / ClassificationTrainer._train_step
 * (trainers/classification.py:269-290): Conv2d (cuDNN) as implicit GEMM on MFMA, BatchNorm2d in
 * train mode (batch statistics, eps 1e-5, momentum 0.1, unbiased running_var), ReLU, MaxPool2d(3,2,1),
 * global average pool.
 *
 * Convolutions (all tensors NHWC; `dtype` is both operand and MFMA type: SV_BF16 or SV_F32):
 *   x   [B][H][W][Cs]    input, Cs = stored channels (power of two; >= the real Cin, zero padded)
 *   y   [B][OH][OW][Cout]  OH = (H + 2 pad - KH)/stride + 1
 *   wp  [Cout][KH*KW][Cs]  packed weight (sv_conv_weight_pack), dtype
 * Cout must be a multiple of 8 (bf16) / 4 (f32).  `policy` (NULL = defaults): the launch policy of the
 * convolution's GEMMs (sv_gemm_policy; the f32 register-staged kernel ignores it).                  */
typedef struct sv_conv_shape {
  int32_t B, H, W, Cs;  /* input                                      */
  int32_t Cout;         /* output channels                            */
  int32_t KH, KW, stride, pad;
  int32_t Cin;          /* real input channels (<= Cs), torch weight  */
} sv_conv_shape;
/* wp[co][t][c] = w[co][c][t] (c < Cin) else 0, cast to `dtype`; w = torch [Cout][Cin][KH][KW] f32. */
int sv_conv_weight_pack(const float* w, void* wp, int32_t dtype, const sv_conv_shape* s, sv_stream_t stream);
/* Up to SV_MAX_PACK_SEGS sv_conv_weight_pack calls in one launch: segment k packs w [Cout][Cin][T] f32 into
 * wp [Cout][T][Cs] (dtype; channels >= Cin zero), T = KH*KW.                                        */
#define SV_MAX_PACK_SEGS 32
typedef struct {
  const float* w;
  void* wp;
  int32_t Cout, Cin, T, Cs;
} sv_pack_seg;
int sv_conv_weight_pack_multi(const sv_pack_seg* segs, int32_t nseg, int32_t dtype, sv_stream_t stream);
/* y = conv(x, w).  y_dtype may differ from dtype (f32 or bf16 store).                             */
int sv_conv_fwd(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype, const sv_conv_shape* s,
                const sv_gemm_policy* policy, sv_stream_t stream);
/* dx (+)= conv_transpose(dy, w): dy [B][OH][OW][Cout] (dtype), dx [B][H][W][Cs] (dx_dtype). Stride-2
 * convolutions run as four stride-1 sub-convolutions, one per output parity class; bf16 with even H, W,
 * Cout >= 32 and Cs % 8 == 0 as ONE gathered GEMM launch whose epilogue stores each class's rows at their dx
 * pixels (no workspace, no scatter pass).  accumulate with a bf16 dx (the ResNet gradient stream, ABI v6): the
 * f32 sum of dx and the product, stored bf16.                                                        */
int sv_conv_bwd_data(const void* dy, const void* wp, void* dx, int32_t dx_dtype, int32_t accumulate,
                     int32_t dtype, const sv_conv_shape* s, const sv_gemm_policy* policy, sv_stream_t stream);
/* dw (+)= dy^T * im2col(x) into torch layout [Cout][Cin][KH][KW] f32, through split-K f32 slabs in
 * `work` (sv_conv_bwd_weight_work_floats(s) floats).                                              */
int64_t sv_conv_bwd_weight_work_floats(const sv_conv_shape* s);
int sv_conv_bwd_weight(const void* dy, const void* x, float* work, float* dw, int32_t accumulate, int32_t dtype,
                       const sv_conv_shape* s, const sv_gemm_policy* policy, sv_stream_t stream);
/* Row f1, classification side: the collated uint8 HWC crops [B][H][W][3] -- the output of the
 * reference's construct_3channel ([T2,T1,T2], or one plane replicated; spine_vision/training/
 * datasets/classification.py:40-68) before ToTensor/Normalize (:247-278) -- straight into the ResNet
 * stem's NHWC operand [B][H][W][Cs] (dtype): out[c] = (u8/255 - mean[c]) / std[c] for c < 3,
 * channels >= 3 zero.  f32 values are bitwise torchvision's CPU ToTensor+Normalize; bf16 their RNE
 * rounding.  B*H*W % 4 == 0, img 4-byte aligned, Cs in {4, 8}; mean/std HOST float[3].           */
int sv_image_u8_hwc_to_nhwc(const uint8_t* img, const float* norm_mean, const float* norm_std, void* out,
                            int32_t dtype, int32_t B, int32_t H, int32_t W, int32_t Cs, sv_stream_t stream);
/* sv_conv_fwd + the BatchNorm statistics of y from the GEMM epilogue (SV_EPI_STORE_STATS): stats =
 * f32 [ceil(M/64)][2][Cout] unshifted partials, M = B*OH*OW, folded by sv_bn_stats_finish(y = NULL).
 * Only the bf16 gathered-operand path (Cs >= 32, power of two, Cout % 8 == 0) carries it: other
 * shapes return SV_ERR_UNSUPPORTED (use sv_conv_fwd + sv_bn_stats).                                */
int sv_conv_fwd_stats(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype, const sv_conv_shape* s,
                      float* stats, const sv_gemm_policy* policy, sv_stream_t stream);
/* Split-K forms for grids smaller than the chip (the deep ResNet stages: few 256x128 output tiles,
 * long K = taps x channels): the gathered GEMM writes `split` f32 slabs [split][M][N] into `work`
 * (split * M * N floats), then sv_gemm_slab_finish sums them into y (+ the STORE_STATS partials when
 * stats != NULL) / into dx (+= when accumulate, f32 or bf16 dx).  bf16 gathered-operand shapes only (as
 * sv_conv_fwd_stats; dgrad: stride 1, Cout >= 32); others are an error.
 * Stride-2 dgrad (bf16, Cout >= 32, Cs % 8 == 0): one gathered GEMM per output parity class writes
 * compact slabs into `work` (split * B*H*W*Cs floats in all), one pass scatters them into dx (+= when
 * accumulate; dx f32 or bf16).                                                                       */
int sv_conv_fwd_split(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype, const sv_conv_shape* s,
                      float* stats, float* work, int32_t split, const sv_gemm_policy* policy, sv_stream_t stream);
int sv_conv_bwd_data_split(const void* dy, const void* wp, void* dx, int32_t dx_dtype, int32_t accumulate,
                           int32_t dtype, const sv_conv_shape* s, float* work, int32_t split,
                           const sv_gemm_policy* policy, sv_stream_t stream);
/* Stride-1 data gradient dx (bf16) of the gathered bf16 path (as sv_conv_bwd_data, no accumulate) plus
 * the backward statistics partials [ceil(B*H*W/64)][2][Cs] of the BatchNorm + ReLU that produced the
 * conv's input (y = that BatchNorm's input [B][H][W][Cs] bf16): split == 1 from the GEMM epilogue
 * (SV_EPI_STORE_BN_BWD), split >= 2 through f32 slabs in `work` (split * B*H*W*Cs floats) and
 * sv_gemm_slab_finish_bn_bwd.  Stride 2 (even H, W, more than one tap, split == 1): the one-launch
 * parity-class GEMM (sv_conv_bwd_data) with the same epilogue, partials [4][ceil(B*H*W/256)][2][Cs]
 * (class c = 2*(y&1) + (x&1) from row c * ceil(B*H*W/256)).  Other shapes are an error.              */
int sv_conv_bwd_data_bn(const void* dy, const void* wp, void* dx, int32_t dtype, const sv_conv_shape* s,
                        const void* y, const sv_bn_ref* bn, float* part, float* work, int32_t split,
                        const sv_gemm_policy* policy, sv_stream_t stream);
/* NCHW f32 image [B][C][H][W] -> NHWC [B][H][W][Cs] (dtype), channels >= C zero.                  */
int sv_image_to_nhwc(const float* img, void* out, int32_t dtype, int32_t B, int32_t C, int32_t H, int32_t W,
                     int32_t Cs, sv_stream_t stream);

/* BatchNorm2d, train mode.  stats: part [nparts][2][C] (shifted sums, shift = row 0), then
 * finish -> mean[C], rstd[C] and (running_mean, running_var) updated in place with `momentum`
 * (unbiased variance, torch semantics) when they are non-NULL.                                    */
int sv_bn_nparts(int64_t rows, int32_t C);
int sv_bn_stats(const void* y, int32_t y_dtype, int64_t rows, int32_t C, float* part, sv_stream_t stream);
/* num_batches_tracked (int64, nullable): incremented by one on the device (BatchNorm2d.num_batches_tracked).
 * y == NULL: `part` holds UNSHIFTED sums (the SV_EPI_STORE_STATS / sv_conv_fwd_stats partials).
 * The fold of nparts partials runs in chunks of 1024 (each: 128 streams, then the streams in order; chunk sums in
 * chunk order).  ctl / ws (ABI v7, nullable; SV_BN_FOLD_CTL_INTS zeroed int32 / SV_BN_FOLD_WS_FLOATS f32, one pair
 * per stream, as the fold kernels below): one workgroup per chunk and channel group instead of one per channel
 * group (the stem's 8192 partials: 43 us as one), the last to finish adding the chunk sums -- the same bits.  Same
 * for sv_bn_bwd_finish.                                                                            */
int sv_bn_stats_finish(const void* y, int32_t y_dtype, const float* part, int32_t nparts, int64_t rows, int32_t C,
                       float eps, float momentum, float* mean, float* rstd, float* running_mean,
                       float* running_var, int64_t* num_batches_tracked, int32_t* ctl, float* ws, sv_stream_t stream);
/* eval mode: mean = running_mean, rstd = 1/sqrt(running_var + eps).                               */
int sv_bn_eval_params(const float* running_mean, const float* running_var, float eps, float* mean, float* rstd,
                      int32_t C, sv_stream_t stream);
/* out = act( gamma (y - mean) rstd + beta  + res ),  act = ReLU if relu;
 * res = 0 (res == NULL) | res (res_mean == NULL) | res_gamma (res - res_mean) res_rstd + res_beta
 * (the BN'd downsample shortcut).                                                                  */
int sv_bn_act_fwd(const void* y, int32_t y_dtype, const float* mean, const float* rstd, const float* gamma,
                  const float* beta, const void* res, int32_t res_dtype, const float* res_mean,
                  const float* res_rstd, const float* res_gamma, const float* res_beta, int32_t relu, void* out,
                  int32_t out_dtype, int64_t rows, int32_t C, sv_stream_t stream);
/* backward.  g = dout * (act > 0) (act == NULL: no mask); xhat = (y - mean) rstd.
 * bn_bwd_stats: part [nparts][2][C] = (sum g, sum g xhat);  bn_bwd_finish: sums[2][C], and
 * dgamma += sum g xhat, dbeta += sum g;  bn_bwd_apply: dx = gamma rstd (g - sum g/n - xhat sum gx/n);
 * if gmask != NULL it also stores g itself there (the masked gradient, for the block shortcut).    */
int sv_bn_bwd_stats(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                    int32_t y_dtype, const float* mean, const float* rstd, int64_t rows, int32_t C, float* part,
                    sv_stream_t stream);
/* sv_bn_bwd_stats with the act mask, also overwriting dout with g = dout * (act > 0) in place, in dout's
 * dtype (the residual block's output gradient -- the gradient stream, bf16 in the bf16 model as under the
 * reference's fp16 autocast: the apply pass then runs with act == NULL and the shortcut reads dout itself,
 * no separate masked copy).  ABI v6: dout_dtype added (was f32 only).                                 */
int sv_bn_bwd_stats_mask(void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                         int32_t y_dtype, const float* mean, const float* rstd, int64_t rows, int32_t C, float* part,
                         sv_stream_t stream);
int sv_bn_bwd_finish(const float* part, int32_t nparts, int32_t C, float* sums, float* dgamma, float* dbeta,
                     int32_t* ctl, float* ws, sv_stream_t stream);
/* A residual block with a projection shortcut (timm Bottleneck's downsample): the block output's gradient
 * dout feeds the main path's last BatchNorm (y, mean, rstd) and the shortcut's (y2, mean2, rstd2) through
 * one ReLU mask.  One statistics pass writes g = dout * (act > 0) over dout and both BatchNorms' partials
 * (part: sums of g and g*xhat; part2: sums of g and g*xhat2) -- bit for bit sv_bn_bwd_stats_mask then
 * sv_bn_bwd_stats(g) of the shortcut -- reading dout once; one apply pass writes both data gradients from g
 * (bit for bit two sv_bn_bwd_apply calls).  Both BatchNorms have rows x C; dx, dx2 share dx_dtype.  ABI v6:
 * dout_dtype / g_dtype added (the gradient stream's dtype; was f32 only).                             */
int sv_bn_bwd_stats_mask_dual(void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                              int32_t y_dtype, const float* mean, const float* rstd, const void* y2, int32_t y2_dtype,
                              const float* mean2, const float* rstd2, int64_t rows, int32_t C, float* part,
                              float* part2, sv_stream_t stream);
int sv_bn_bwd_apply_dual(const void* g, int32_t g_dtype, const void* y, int32_t y_dtype, const float* mean,
                         const float* rstd, const float* gamma, const float* sums, const void* y2, int32_t y2_dtype,
                         const float* mean2, const float* rstd2, const float* gamma2, const float* sums2, void* dx,
                         void* dx2, int32_t dx_dtype, int64_t rows, int32_t C, sv_stream_t stream);
int sv_bn_bwd_apply(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                    int32_t y_dtype, const float* mean, const float* rstd, const float* gamma, const float* sums,
                    void* dx, int32_t dx_dtype, float* gmask, int64_t rows, int32_t C, sv_stream_t stream);
/* The same backward for a BN followed by its own ReLU (no residual): the mask is recomputed from y
 * exactly as sv_bn_act_fwd computes the pre-activation, fmaf(gamma rstd, y - mean, beta) > 0, so
 * the activation tensor is not read again (one 2-byte stream less per element in both passes).    */
int sv_bn_relu_bwd_stats(const void* dout, int32_t dout_dtype, const void* y, int32_t y_dtype, const float* mean,
                         const float* rstd, const float* gamma, const float* beta, int64_t rows, int32_t C,
                         float* part, sv_stream_t stream);
int sv_bn_relu_bwd_apply(const void* dout, int32_t dout_dtype, const void* y, int32_t y_dtype, const float* mean,
                         const float* rstd, const float* gamma, const float* beta, const float* sums, void* dx,
                         int32_t dx_dtype, int64_t rows, int32_t C, sv_stream_t stream);
/* The stem's BN + ReLU backward fed by the max-pool 3x3/2 (pad 1) backward: the incoming gradient of
 * input pixel p is the sum of dpool [B][OH][OW][C] (f32 or bf16, dpool_dtype: ABI v6) over the windows whose
 * argmax tap (idx, as
 * sv_maxpool3s2_fwd writes it) is p, gathered inside both passes in sv_maxpool3s2_bwd's order (bit for
 * bit sv_maxpool3s2_bwd then sv_bn_relu_bwd_*, without writing the [B][H][W][C] f32 gradient).
 * y [B*H*W][C]; dpool 16-B and idx 4-B aligned.                                                     */
int sv_bn_relu_bwd_stats_pool(const void* dpool, int32_t dpool_dtype, const uint8_t* idx, int32_t B, int32_t H,
                              int32_t W, const void* y, int32_t y_dtype, const float* mean, const float* rstd,
                              const float* gamma, const float* beta, int32_t C, float* part, sv_stream_t stream);
int sv_bn_relu_bwd_apply_pool(const void* dpool, int32_t dpool_dtype, const uint8_t* idx, int32_t B, int32_t H,
                              int32_t W, const void* y, int32_t y_dtype, const float* mean, const float* rstd,
                              const float* gamma, const float* beta, const float* sums, void* dx, int32_t dx_dtype,
                              int32_t C, sv_stream_t stream);
/* One launch per BatchNorm for small row counts (rows <= SV_BN_SMALL_MAX_ROWS and the geometry
 * sv_bn_small_ok accepts: ResNet layers 3-4 at 256 px).  One workgroup owns 8 channels over all rows, so
 * the statistics and the pass that uses them share the launch; the sums are taken in the multi-launch
 * path's order, so every output is bit for bit what that path writes:
 *   sv_bn_bwd_small  mode SV_BN_SMALL_MASK  = sv_bn_bwd_stats_mask + sv_bn_bwd_finish + sv_bn_bwd_apply (act == NULL)
 *                    mode SV_BN_SMALL_RELU  = sv_bn_relu_bwd_stats + finish + sv_bn_relu_bwd_apply; with `part`
 *                                             (nparts, e.g. from sv_conv_bwd_data_bn) the statistics pass is skipped
 *                    mode SV_BN_SMALL_DUAL  = sv_bn_bwd_stats_mask_dual + two finishes + sv_bn_bwd_apply_dual
 *                    batch_stats == 0: eval-mode apply (zero correction sums; dgamma / dbeta still accumulate)
 *   sv_bn_act_small  = sv_bn_stats_finish(y = NULL, part) + sv_bn_act_fwd, and with res_part the shortcut
 *                      BatchNorm's finish too (res = its conv output).  All pointers 16-B aligned.
 * Replaces: timm Bottleneck bn1/bn2/bn3/downsample BatchNorm2d forward + autograd backward
 * (spine_vision/training/models/backbone.py:166 -> timm resnet.py).                                  */
#define SV_BN_SMALL_MAX_ROWS 8192
#define SV_BN_SMALL_MASK 0
#define SV_BN_SMALL_RELU 1
#define SV_BN_SMALL_DUAL 2
int sv_bn_small_ok(int64_t rows, int32_t C);
int sv_bn_bwd_small(int32_t mode, void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                    int32_t y_dtype, const float* mean, const float* rstd, const float* gamma, const float* beta,
                    const void* y2, int32_t y2_dtype, const float* mean2, const float* rstd2, const float* gamma2,
                    const float* part, int32_t nparts, void* dx, void* dx2, int32_t dx_dtype, float* dgamma,
                    float* dbeta, float* dgamma2, float* dbeta2, int32_t batch_stats, int64_t rows, int32_t C,
                    sv_stream_t stream);
int sv_bn_act_small(const void* y, int32_t y_dtype, const float* part, int32_t nparts, float eps, float momentum,
                    const float* gamma, const float* beta, float* mean, float* rstd, float* running_mean,
                    float* running_var, int64_t* num_batches_tracked, const void* res, int32_t res_dtype,
                    const float* res_part, int32_t res_nparts, float res_eps, float res_momentum,
                    const float* res_gamma, const float* res_beta, float* res_mean, float* res_rstd,
                    float* res_running_mean, float* res_running_var, int64_t* res_num_batches_tracked, int32_t relu,
                    void* out, int32_t out_dtype, int64_t rows, int32_t C, sv_stream_t stream);
/* The statistics fold inside the consuming pass (ABI v7): one launch fewer per BatchNorm at any row count.
 *   sv_bn_act_fold       = sv_bn_stats_finish(y = NULL, part) [+ the shortcut's] + sv_bn_act_fwd; arguments as
 *                          sv_bn_act_small (nparts = ceil(rows / 64), the conv epilogue's; res_nparts equal).
 *   sv_bn_bwd_apply_fold = sv_bn_bwd_finish [x2] + the apply pass, after the statistics pass (or the dgrad
 *                          epilogue) wrote `part` [nparts][2][C] (and `part2`):
 *                          mode SV_BN_SMALL_MASK: sv_bn_bwd_apply(dout = the masked gradient, act = NULL)
 *                          mode SV_BN_SMALL_RELU: sv_bn_relu_bwd_apply; pool_idx != NULL: sv_bn_relu_bwd_apply_pool
 *                                                 (dout = the pooled gradient, the BN input pool_H x pool_W)
 *                          mode SV_BN_SMALL_DUAL: sv_bn_bwd_apply_dual (dout = g; part2 the shortcut's partials)
 *                          batch_stats == 0: eval-mode apply (dgamma / dbeta still accumulate)
 * Bit for bit the multi-launch results.  ctl: SV_BN_FOLD_CTL_INTS int32, zero before the first launch and left
 * zero by every launch (ctl[3] != 0 flags a poll that timed out); ws: SV_BN_FOLD_WS_FLOATS f32 scratch.  One
 * (ctl, ws) per stream: two fold launches must not run at once on one pair.  sv_bn_fold_ok: 1 when (rows, C,
 * nparts) has the fold kernels' geometry (C a power of two in 32..2048, nparts <= 16384).
 * Replaces: timm Bottleneck BatchNorm2d forward + autograd backward (backbone.py:166 -> timm resnet.py).      */
#define SV_BN_FOLD_CTL_INTS 256
#define SV_BN_FOLD_WS_FLOATS (2 * 2 * 2048 + 2 * 64 * 16 * 64)
int sv_bn_fold_ok(int64_t rows, int32_t C, int32_t nparts);
int sv_bn_act_fold(const void* y, int32_t y_dtype, const float* part, int32_t nparts, float eps, float momentum,
                   const float* gamma, const float* beta, float* mean, float* rstd, float* running_mean,
                   float* running_var, int64_t* num_batches_tracked, const void* res, int32_t res_dtype,
                   const float* res_part, int32_t res_nparts, float res_eps, float res_momentum,
                   const float* res_gamma, const float* res_beta, float* res_mean, float* res_rstd,
                   float* res_running_mean, float* res_running_var, int64_t* res_num_batches_tracked, int32_t relu,
                   void* out, int32_t out_dtype, int64_t rows, int32_t C, int32_t* ctl, float* ws, sv_stream_t stream);
int sv_bn_bwd_apply_fold(int32_t mode, const void* dout, int32_t dout_dtype, const uint8_t* pool_idx, int32_t pool_H,
                         int32_t pool_W, const void* y, int32_t y_dtype, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, const void* y2, int32_t y2_dtype, const float* mean2,
                         const float* rstd2, const float* gamma2, const float* part, const float* part2,
                         int32_t nparts, void* dx, void* dx2, int32_t dx_dtype, float* dgamma, float* dbeta,
                         float* dgamma2, float* dbeta2, int32_t batch_stats, int64_t rows, int32_t C, int32_t* ctl,
                         float* ws, sv_stream_t stream);
/* g = dout * (act > 0), f32 out (block-output ReLU of the residual join).                         */
int sv_relu_mask(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, float* g, int64_t n,
                 sv_stream_t stream);
/* MaxPool2d(3, stride 2, pad 1) NHWC; idx [B][OH][OW][C] uint8 = argmax tap (first max in (kh,kw)
 * order, torch semantics); bwd gathers dout into dx [B][H][W][C] (dx_dtype; overwrite).           */
int sv_maxpool3s2_fwd(const void* x, int32_t x_dtype, void* y, uint8_t* idx, int32_t B, int32_t H, int32_t W,
                      int32_t C, sv_stream_t stream);
int sv_maxpool3s2_bwd(const void* dout, int32_t dout_dtype, const uint8_t* idx, void* dx, int32_t dx_dtype,
                      int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream);
/* global average pool: feat[b][c] = mean_hw x; bwd: dx[b][hw][c] = dfeat[b][c] / HW, dx in dx_dtype (the
 * ResNet gradient stream's: bf16 in the bf16 model; ABI v6).                                        */
int sv_avgpool_fwd(const void* x, int32_t x_dtype, float* feat, int32_t B, int32_t HW, int32_t C,
                   sv_stream_t stream);
int sv_avgpool_bwd(const float* dfeat, void* dx, int32_t dx_dtype, int32_t B, int32_t HW, int32_t C,
                   sv_stream_t stream);

/* ---- classification loss (csrc/loss.hip, ABI v7) ------------------------------------------------
 * The multi-task loss over the fused head's logits [B][K] (f32, row-major) in one launch: loss[0] =
 * sum_k weight_k * loss_k, and dlogits [B][K] = d(loss[0]) / d(logits) (every column of a task's range
 * written; columns no task covers are left alone).  Tasks (host array, 1..8):
 *   SV_HEAD_CE : torch.nn.CrossEntropyLoss(label_smoothing) over columns [offset, offset + ncls); target
 *                int64 [B] class indices, -100 ignored; mean over the valid rows (0 if none)
 *   SV_HEAD_BCE: torch.nn.BCEWithLogitsLoss over [offset, offset + ncls); target [B][ncls] f32 / bf16
 *                (target_dtype); mean over B * ncls
 * Replaces: Classifier.get_loss (spine_vision/training/models/generic.py) with core/tasks.py's per-task losses
 * and their autograd backward.                                                                       */
#define SV_HEAD_CE 0
#define SV_HEAD_BCE 1
typedef struct {
  int32_t kind;
  int32_t offset;
  int32_t ncls;
  float weight;
  float label_smoothing;
  const void* target;
  int32_t target_dtype;
} sv_head_task;
int sv_head_loss(const float* logits, int32_t B, int32_t K, const sv_head_task* tasks, int32_t ntasks, float* loss,
                 float* dlogits, sv_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SV_KERNELS_H */
