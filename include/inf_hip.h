/*
 * inf_hip.h -- C ABI of the MI355X (gfx950) intrinsic-neural-fields hot path.
 *
 * The reference (tum-vision/intrinsic-neural-fields) has no native code: its hot path
 * is stock PyTorch ops called from Python.  This library replaces those ops; the
 * Python host layer (intrinsic-neural-fields_amd/) binds it with ctypes and keeps the
 * reference's call surface.  Each entry point names the reference interface it
 * replaces (paths relative to the reference root).
 *
 * Conventions
 *   - every function returns INF_OK (0) or a negative INF_ERR_* code and never throws;
 *     inf_last_error() returns a thread-local message for the last failure;
 *   - all pointers are device pointers owned by the caller (PyTorch's allocator);
 *     the library never allocates or synchronises on the hot path, so every call can
 *     be captured into a HIP graph;
 *   - `stream` is a hipStream_t passed as void*; all work is enqueued on it.
 */
#ifndef INF_HIP_H
#define INF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* inf_stream_t; /* hipStream_t */

enum {
  INF_OK = 0,
  INF_ERR_ARG = -1,         /* bad argument (shape, dtype, null pointer)       */
  INF_ERR_HIP = -2,         /* a HIP runtime call failed                        */
  INF_ERR_UNSUPPORTED = -3, /* configuration not supported by the kernels       */
  INF_ERR_STATE = -4        /* plan not bound / wrong call order                */
};

enum { INF_DTYPE_F32 = 0, INF_DTYPE_BF16 = 1, INF_DTYPE_I32 = 2, INF_DTYPE_I64 = 3 };
/* GEMM arithmetic: FP32 exact f32 MFMA; BF16 bf16 operands (fp32 accumulation, fp32
 * master weights); BF16X3 fp32 operands multiplied as split bf16 (hi*hi + hi*lo + lo*hi,
 * ~2^-16 relative per product) -- every buffer and kernel of the fp32 mode, only the
 * GEMMs' inner products on bf16 matrix cores */
enum { INF_MODE_FP32 = 0, INF_MODE_BF16 = 1, INF_MODE_BF16X3 = 2 };
enum { INF_LOSS_L2 = 0, INF_LOSS_L1 = 1, INF_LOSS_CAUCHY = 2 }; /* config.py:113-122   */
/* Input front-end of a batch (TextureField.input_feature_embed, model.py:33-40,98-104).
 * NONE: the table rows are the features (efuncs).  XYZ/RFF/FF: the table is the fp32
 * V x 3 vertex table (ray_dataloader.py:28-30) and the feature of a ray is its
 * barycentric hit position x (ray_dataloader.py:134-136), as is (XYZ) or encoded:
 *   RFF  [cos e | sin e | x?], e_j = sum_c (2 pi x_c) B[c][j]   (layers.py:28-39)
 *   FF   [cos e | sin e | x?], e_{c k + f} = x_c band_f        (layers.py:6-25)     */
enum { INF_ENC_NONE = 0, INF_ENC_XYZ = 1, INF_ENC_RFF = 2, INF_ENC_FF = 3,
       /* table = inf_project_table output [V][2H] bf16 (forward-only: inf_render /
        * inf_forward with save = 0 of bf16 plans) */
       INF_ENC_PROJECTED = 4 };

/* TextureField architecture (model.py:12-96, make_model model.py:199-258). */
typedef struct inf_mlp_desc {
  int32_t in_dim;     /* k (int) or len(k) (list)                          */
  int32_t hidden;     /* mlp_hidden_dim                                    */
  int32_t num_layers; /* num_layers (> 2)                                  */
  int32_t skip;       /* skip_layer_idx, 0 < skip < num_layers-1           */
  int32_t out_dim;    /* 3 (RGB_COLOR_DIM, model.py:9)                     */
  int32_t mode;       /* INF_MODE_*                                        */
  int32_t loss;       /* INF_LOSS_*                                        */
} inf_mlp_desc;

/* Sizes the caller needs to allocate for a plan (all in bytes unless noted). */
typedef struct inf_plan_info {
  int64_t num_params;     /* P: floats in the flat parameter arena            */
  int32_t num_segments;   /* parameter tensors (model.parameters() order)     */
  int32_t in_pad;         /* k padded to the GEMM tile                        */
  int32_t max_batch_pad;  /* max_batch padded to the GEMM tile                */
  int32_t dw_splits;      /* split-K factor of the weight-gradient GEMMs      */
  int64_t shadow_bytes;   /* packed GEMM-dtype weights (W and W^T, padded)    */
  int64_t workspace_bytes;/* activations, gradient slabs, loss accumulators   */
  int64_t table_ld;       /* row stride (elements) expected of a device table */
} inf_plan_info;

/* A batch of rays, in one of two forms.
 *  (a) rays:     table != NULL -> the library gathers F = sum_i bary_i * E[vid_i]
 *                (mesh.py:313-324) for rays idx[offset + b] (ray_dataloader.py:115-129);
 *  (b) features: features != NULL -> F given as fp32 [B][ld_features]
 *                (model.py:104, batch["eigenfunctions"]).                       */
typedef struct inf_batch {
  const void* table;     /* [V][table_ld], dtype table_dtype, columns >= in_dim zero */
  int32_t table_dtype;   /* INF_DTYPE_F32 / INF_DTYPE_BF16                            */
  int64_t num_vertices;  /* V                                                         */
  const void* vids;      /* [N][3] INF_DTYPE_I32 or INF_DTYPE_I64                     */
  int32_t vid_dtype;
  const float* bary;     /* [N][3]                                                    */
  const float* rgb;      /* [N][3] targets (training only)                            */
  const void* ray_idx;   /* [N] permutation (nullable: identity)                      */
  int32_t idx_dtype;     /* INF_DTYPE_I32 / INF_DTYPE_I64                             */
  int64_t idx_offset;    /* first entry of ray_idx (or of the rays) used              */
  int32_t offset_from_ctrl; /* 1: add ctrl->batch_index * batch to idx_offset         */
  const float* features; /* form (b)                                                  */
  int64_t ld_features;
  int32_t batch;         /* rays in this batch (<= max_batch)                         */
  int64_t loss_count;    /* elements of the loss mean (3 x global batch); 0 = 3*batch */
  int32_t loss;          /* INF_LOSS_* of a training call; -1 = the plan's desc.loss   */
  int64_t num_rays;      /* entries of ray_idx (rows of vids/bary/rgb when ray_idx is  */
                         /* null); rays past it read as zero features / targets.       */
                         /* 0 = unchecked.  Vertex ids >= num_vertices read as zero.   */
  int32_t encoding;      /* INF_ENC_* (form (a) only).  With vids == NULL the table    */
                         /* rows are the rays' positions x themselves (batch["xyz"]). */
  int32_t enc_k;         /* embedding size k (RFF/FF)                                  */
  const float* enc_proj; /* RFF: B [3][enc_k]; FF: freq_bands [enc_k]                  */
  int32_t enc_include_input; /* append x (embed_include_input)                        */
  int64_t num_source_rays; /* rows of vids / bary / rgb (the ray arrays ray_idx indexes);   */
                         /* a ray whose permutation entry names a row outside            */
                         /* [0, num_source_rays) reads as a zero feature row and a zero   */
                         /* target instead of being loaded.  0 = unchecked.                */
} inf_batch;

/* Device-resident step state (lets a captured HIP graph replay a whole epoch). */
typedef struct inf_ctrl {
  int32_t step;        /* Adam step count t (post-increment semantics of torch Adam) */
  int32_t batch_index; /* batch number inside the current epoch                     */
  int32_t prefetch_index; /* batch number the next inf_prefetch_batch gathers        */
  int32_t reserved;
  double lr;           /* learning rate, a double as torch's param_group["lr"]       */
  double loss_sum;     /* sum of element losses of the last step                     */
  double sse_sum;      /* sum of squared errors of the last step                     */
  double epoch_loss;   /* accumulated over the epoch (host resets)                   */
  double epoch_sse;
} inf_ctrl;

/* ---- library ----------------------------------------------------------------- */
const char* inf_last_error(void);
int inf_abi_version(void);
/* "<16 hex digits of sha256> <file> <file> ...": the hash of the concatenated bytes of the
 * listed source / header files (paths relative to csrc/) the library was linked from. */
const char* inf_build_id(void);

/* ---- gather: mesh.get_k_eigenfunc_vec_vals (mesh.py:313-324) and its chunked
 *      form get_k_eigenfunc_vec_vals_batched (mesh.py:327-339), with the loader's
 *      index-select fused in (ray_dataloader.py:122-129).
 *      out[b][j] = bary[r][0]*E[v0][j] + bary[r][1]*E[v1][j] + bary[r][2]*E[v2][j],
 *      r = idx ? idx[idx_offset+b] : idx_offset+b, j < k; columns k..ld_out-1 and rows
 *      batch..rows_out-1 are written as zero, and so are rays whose r lies outside
 *      [0, num_source_rays) (the rows of vids / bary; 0 = unchecked).                */
int inf_gather(const void* table, int table_dtype, int64_t num_vertices, int k, int64_t table_ld,
               const void* vids, int vid_dtype, const float* bary,
               const void* ray_idx, int idx_dtype, int64_t idx_offset, int batch, int64_t num_source_rays,
               void* out, int out_dtype, int64_t ld_out, int rows_out,
               void* out_t, int64_t ld_out_t, inf_stream_t stream);

/* ---- encoders: RandomFourierFeatEnc / FourierFeatEnc forward (layers.py:6-39) applied
 *      to the loader's interpolated hit positions (ray_dataloader.py:134-136).  With
 *      vids == NULL, `table` holds the positions x of the rays themselves ([rows][3]).
 *      out[b][j], j < in_dim (3, 2k(+3) or 6k(+3)); columns in_dim..ld_out-1 and rows
 *      batch..rows_out-1 are written as zero.                                        */
int inf_encode(const float* table, int64_t num_rows, const void* vids, int vid_dtype, const float* bary,
               const void* ray_idx, int idx_dtype, int64_t idx_offset, int batch, int64_t num_source_rays,
               int encoding, int enc_k, const float* enc_proj, int include_input,
               void* out, int out_dtype, int64_t ld_out, int rows_out, inf_stream_t stream);
/* in_dim of an encoding (3, 2k + 3*inc, 6k + 3*inc); -1 for a bad encoding */
int inf_encoded_dim(int encoding, int enc_k, int include_input);

/* ---- evaluation metrics (evaluation_metrics.py:5-34), images fp32 [H][W][C] ------ */
/* dssim = (1 - mean_c SSIM_c) / 2 with skimage structural_similarity(multichannel=True)
 * defaults (7 x 7 uniform window, K1 0.01, K2 0.03, sample covariance, border of 3
 * cropped); out[c] = channel c's mean SSIM (fp64, device).  data_range: 2.0 for float
 * images (skimage's dtype range of a float image), 255 for uint8-valued ones.
 * workspace: inf_ssim_workspace_bytes(H, W, C) bytes of device memory.               */
int64_t inf_ssim_workspace_bytes(int height, int width, int channels);
int inf_ssim(const float* fake, const float* real, int height, int width, int channels, double data_range,
             void* workspace, double* out, inf_stream_t stream);
/* psnr's masked mean square error (evaluation_metrics.py:5-22): out[0] = sum over the
 * pixels with mask != 0 (all when mask is NULL) of the squared channel differences,
 * out[1] = the number of those pixels (fp64, device).                                */
int64_t inf_masked_sse_workspace_bytes(void);
int inf_masked_sse(const float* fake, const float* real, const uint8_t* mask, int64_t num_pixels, int channels,
                   void* workspace, double* out, inf_stream_t stream);

/* ---- generic fp32 dense layers: the view-dependent texture field
 *      (model.py:115-191 TextureFieldWithViewDependency; no config enables it) -------- */
/* C[m][n] = act(sum_k A(m,k) B(n,k) + bias[n] + beta C[m][n]), A(m,k) = A[m sam + k sak],
 * B(n,k) = B[n sbn + k sbk]; act 0 none, 1 ReLU, 2 sigmoid (nn.Linear + activation). */
int inf_dense_gemm(int M, int N, int K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbn,
                   int64_t sbk, const float* bias, int act, float beta, float* C, int64_t ldc, inf_stream_t stream);
/* dZ = dY * act'(Y) (autograd of ReLU / Sigmoid through their outputs). */
int inf_dense_act_bwd(int64_t n, const float* Y, const float* dY, int act, float* dZ, inf_stream_t stream);
/* out[n] (+)= sum_m X[m ldx + n] (bias gradients). */
int inf_colsum(int M, int N, const float* X, int64_t ldx, float* out, int accumulate, inf_stream_t stream);
/* acos(F.cosine_similarity(-unit_dirs, face_normals[face_idxs])) (model.py:164-169). */
int inf_view_angle(int64_t n, const float* unit_dirs, const int64_t* face_idxs, const float* face_normals,
                   int64_t num_faces, float* out, inf_stream_t stream);
/* FourierFeatEnc.forward (layers.py:21-25) of [n][d] inputs: [cos e | sin e | x?],
 * e[r][c k + f] = x[r][c] bands[f]. */
int inf_ff_encode(int64_t n, int d, const float* x, const float* bands, int k, int include_input, float* out,
                  int64_t ld_out, inf_stream_t stream);
/* torch.optim.Adam (config.py:108) step `step` (1-based) of one parameter tensor that is
 * not in a plan arena: the plan update's arithmetic (adam_dev.hpp adam_elem). */
int inf_adam_dense(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int step,
                   double lr, double beta1, double beta2, double eps, inf_stream_t stream);

/* ---- plan: one TextureField (model.py:12-112) + its training step ---------------- */
typedef struct inf_plan inf_plan;

int inf_plan_create(const inf_mlp_desc* desc, int max_batch, inf_plan** plan);
void inf_plan_destroy(inf_plan* plan);
int inf_plan_get_info(const inf_plan* plan, inf_plan_info* info);
/* Offsets/numels (floats) of each parameter tensor in the flat arena, in
 * model.parameters() order: layers.{i}.0.weight/bias, layers.{s}.Lx.*, layers.{s}.Ly.* */
int inf_plan_param_layout(const inf_plan* plan, int64_t* offsets, int64_t* numels, int n);

/* Bind caller-owned buffers.  params/grads/exp_avg/exp_avg_sq: P floats each
 * (grads/exp_avg/exp_avg_sq may be NULL for inference-only plans). */
int inf_plan_bind(inf_plan* plan, float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                  void* shadow, void* workspace, inf_ctrl* ctrl);
/* Adam hyper-parameters (torch.optim.Adam defaults: 0.9, 0.999, 1e-8; config.py:108), as
 * the Python doubles torch holds them: the update derives its fp32 constants the way torch's
 * CPU kernels do (1 - beta1, beta2, 1 - beta2 and eps rounded to float from the double;
 * the bias corrections and lr / (1 - beta1^t) in double). */
int inf_plan_set_adam(inf_plan* plan, double beta1, double beta2, double eps);

/* Re-derive the packed GEMM weights from the fp32 parameters (after init,
 * load_state_dict, or any host-side parameter edit). */
int inf_sync_shadow(inf_plan* plan, inf_stream_t stream);

/* Forward (model.py:98-112): pred[B][3] fp32.  save != 0 keeps the activations for
 * inf_backward (autograd path, trainer.py:75/81). */
int inf_forward(inf_plan* plan, const inf_batch* batch, float* pred, int save, inf_stream_t stream);

/* Backward of the last saved forward given dL/dpred [B][3] (autograd, trainer.py:81).
 * Writes the reduced parameter gradient (P floats, arena layout) into `grads`; the
 * caller hands it to autograd, which accumulates into param.grad exactly as torch
 * does (zero_grad(set_to_none=True), trainer.py:80). */
int inf_backward(inf_plan* plan, const float* dpred, float* grads, inf_stream_t stream);

/* Fused training step (trainer.py:71-84 + loss config.py:113-122):
 * gather -> forward -> loss -> backward -> gradient reduction, and, with
 * INF_STEP_ADAM in `flags`, the Adam update (torch.optim.Adam, config.py:108).
 * Without it the reduced gradient is left in `grads` for a cross-GPU all-reduce
 * followed by inf_adam().  INF_STEP_ADVANCE also advances ctrl->batch_index by one
 * at the end of the step (a graph-replayed epoch; same as a following
 * inf_ctrl_advance).  pred may be NULL.  The step's loss / SSE sums are stored in
 * ctrl->loss_sum / sse_sum and added to the epoch sums. */
/* INF_STEP_PART1 / PART2 (gradient-only steps; not with ADAM / ADVANCE): the step split at
 * inf_plan_grad_split for a bucketed data-parallel all-reduce.  PART1 runs the forward,
 * loss and backward chain, the weight-gradient GEMM of the matrices in bucket 1 and the
 * reduction of bucket 1 into `grads`: the arena range [grad_split, P) -- the skip layer's
 * Ly and every tensor after it, their biases included -- plus the step's loss sums.
 * PART2 (same batch) does the GEMM and reduction of bucket 2, the arena [0, grad_split):
 * every earlier tensor, the earlier layers' biases (Lx.bias among them) included.  The
 * caller all-reduces bucket 1 while PART2 runs.  Where the step does not take the fused
 * chain, PART1 reduces the whole gradient and PART2 does nothing
 * (inf_plan_last_part1_bucketed tells which). */
/* INF_STEP_SHARD (gradient-only, after inf_plan_shard + inf_plan_bind_shard): the reduced
 * local gradient goes to the item-major gradient staging (the reduce-scatter input) instead
 * of `grads`; see inf_adam_shard.  Only where the step takes a fused chain (chain3 / chainf,
 * which read nothing but the weight images and the fp32 vectors): INF_ERR_UNSUPPORTED, with
 * nothing launched, otherwise. */
enum { INF_STEP_ADAM = 1, INF_STEP_ADVANCE = 2, INF_STEP_XSLOT0 = 4, INF_STEP_XSLOT1 = 8, INF_STEP_PART1 = 16,
       INF_STEP_PART2 = 32, INF_STEP_SHARD = 64 };
int inf_train_step(inf_plan* plan, const inf_batch* batch, float* pred, int flags,
                   inf_stream_t stream);

/* Gather of a training batch's features (mesh.py:313-324 with the loader's index select,
 * ray_dataloader.py:122-129) into pre-gather slot `slot` (0 / 1) of the plan's workspace,
 * for a later inf_train_step with INF_STEP_XSLOT0 / XSLOT1: the fused chain then reads
 * each ray's feature row instead of three table rows, so the gather can run on a side
 * stream while the previous step's dW GEMM, update and all-reduce run.  With
 * batch->offset_from_ctrl the batch offset is idx_offset + ctrl->prefetch_index * batch and
 * ctrl->prefetch_index is advanced after the gather (graph-replayed epochs).  Returns
 * INF_ERR_STATE when the batch's training step would not use the fused chain (bf16 mode,
 * a bf16 eigenfunction table, the fused shapes): the caller then steps without slots. */
int inf_prefetch_batch(inf_plan* plan, const inf_batch* batch, int slot, inf_stream_t stream);

/* Adam update from the bound `grads` arena (optim.step(), trainer.py:82).  step > 0:
 * step and lr are used as given (torch state["step"] after its increment, param_group
 * lr -- lr = 0 leaves the parameters unchanged, as torch does); step <= 0: both are read
 * from ctrl (graph-replayed steps, where the fused step has already advanced
 * ctrl->step). */
int inf_adam(inf_plan* plan, int step, double lr, inf_stream_t stream);

/* inf_adam with flags: INF_STEP_ADVANCE also advances ctrl->batch_index by one in the same
 * launch (the data-parallel step's tail: all-reduce -> Adam + advance, instead of a
 * separate inf_ctrl_advance launch).  flags = 0 is inf_adam. */
int inf_adam_ex(inf_plan* plan, int step, double lr, int flags, inf_stream_t stream);

/* Render slice (renderer.py:112-146): forward of `batch` and placement of each
 * predicted colour at image row pixel_map[hit[b]] (hit = hit_ray_idxs; pixel_map maps
 * masked-pixel index -> full-image pixel, NULL for identity).  img is [H*W][3] fp32
 * and must already hold the background. */
int inf_render(inf_plan* plan, const inf_batch* batch, const int64_t* hit, const int64_t* pixel_map,
               float* img, inf_stream_t stream);

/* Projected table for repeated forward passes over one eigenfunction table (rendering):
 * out[v][0:H] = W_0 E[v] and out[v][H:2H] = W_y E[v] (the first layer's and the skip
 * layer's input weights, no biases; model.py:43-47, layers.py:60-62), bf16, from the
 * packed bf16 table [num_vertices][k_pad] and the plan's current bf16 weight shadow.
 * Both layers are linear in the features, so a hit's pre-activations are the
 * barycentric interpolation of its vertices' rows: a batch with encoding
 * INF_ENC_PROJECTED and table = out gathers 2H instead of k_pad values per vertex and
 * skips the two k_pad-deep layers.  out has inf_projected_rows(num_vertices) rows
 * (128-row multiple); valid until the weights change.  Replaces nothing in the
 * reference: a reassociation of renderer.py:104-110's model(batch). */
int64_t inf_projected_rows(int64_t num_vertices);
int inf_project_table(inf_plan* plan, const void* table, int64_t num_vertices, void* out, inf_stream_t stream);

/* Diagnostics: re-launch one stage of the last saved training step on its saved
 * inputs (used by bench.py to time a single kernel with HIP events).  Stages:
 *   INF_STAGE_GATHER   - the gather kernel (X, X^T)
 *   INF_STAGE_FWD_GEMM - the forward GEMM of hidden layer `layer` (1..L-2)
 *   INF_STAGE_DW_GEMM  - the grouped split-K weight-gradient GEMM
 *   INF_STAGE_UPDATE   - the slab-reduction/Adam/packed-weight launch: layer 0 reduces
 *                        only (parameters are not modified), layer 1 runs it as the
 *                        training step does (Adam + weight images; parameters change)
 *   INF_STAGE_CHAIN    - the fused forward + loss + dX-chain kernel (bf16 mode; at
 *                        <= 8192 rays with the gather fused in)
 * *flops / *bytes receive the stage's algorithmic work per launch (unpadded). */
enum { INF_STAGE_GATHER = 0, INF_STAGE_FWD_GEMM = 1, INF_STAGE_DW_GEMM = 2, INF_STAGE_UPDATE = 3,
       INF_STAGE_CHAIN = 4 };
int inf_run_stage(inf_plan* plan, const inf_batch* batch, int stage, int layer, double* flops, double* bytes,
                  inf_stream_t stream);

/* Debug builds only (libinf_hip_dbg.so, -DINF_CHAIN_DEBUG): register the valid device
 * byte ranges [lo, hi) (n pairs) and a result buffer; the fused chain then checks every
 * global access against them and records violations instead of issuing them. */
int inf_debug_ranges(inf_plan* plan, const uint64_t* ranges_dev, int n, unsigned long long* out_dev);

/* Diagnostics: when `stamps_dev` is non-null, the fused chain of workgroups 0 and the last
 * records the 100 MHz wall clock (s_memrealtime) at every flat k-step once its stage has
 * landed: stamps_dev[w * (max_steps + 1) + s], w = 0 (first) / 1 (last), entry max_steps
 * = the kernel's end.  Pass null to turn it off. */
int inf_debug_timing(inf_plan* plan, unsigned long long* stamps_dev, int max_steps);

/* Diagnostics: when `stamps_dev` is non-null, every workgroup of the weight-gradient GEMM
 * (lgemm, register-streamed chain path) records the 100 MHz wall clock at entry, after its
 * operand prologue, after its main loop and at exit: stamps_dev[block * 8 + i], block in
 * launch order (before the XCD remap); with the update fused in, also [4] ticket taken,
 * [5] items decided, [6] / [7] around its update item (8 words per block).  The update
 * launch's workgroups (one work item each) record at stamps_dev[(6144 + item) * 8 + i]:
 * [0] entry, [1] item and segment loaded, [2] the item's data loaded, [3] its stores
 * issued, [4] exit after its stores completed (matrix items; the buffer must hold 8192
 * blocks).  Pass null to turn it off. */
int inf_debug_block_times(inf_plan* plan, unsigned long long* stamps_dev);

/* Diagnostics: the kernel path the last inf_train_step took -- 0 layered GEMMs, 2 the
 * LDS-ring chain (csrc/chain.hip), 3 the fused gather + register-streamed chain
 * (csrc/chain3.hip), 4 the same with the feature tile streamed in chunks (k_pad > 1024),
 * 5 the same in 64-ray tiles (batches above 8192 rays), 6 the fused fp32 chain of the
 * fp32 mode (csrc/chainf.hip), 7 the split-bf16 register chain of the bf16x3 mode
 * (csrc/chain3.hip X3), 10 the register-streamed chain after zg.hip's gather + input-layer
 * GEMM launch (the default for k_pad > 1024); -1 before any step. */
int inf_plan_last_step_path(const inf_plan* plan);

/* Weight generation: a counter of the launches issued through this plan that may have
 * changed its parameters or weight images (training-step updates, inf_adam*,
 * inf_sync_shadow), for caching what derives from the weights (the render slice's
 * projected table across frames).  -1 once such a launch was captured into a graph:
 * replays are invisible to the host, so nothing derived may then be cached. */
int64_t inf_plan_weight_generation(const inf_plan* plan);

/* First float of gradient bucket 1 in the parameter arena (the skip layer's Ly weight;
 * INF_STEP_PART1 / PART2): bucket 1 = [split, P), bucket 2 = [0, split). */
int64_t inf_plan_grad_split(const inf_plan* plan);

/* Diagnostics: a copy of a plan buffer -- which = 0: the X^T fragment images the last
 * fused step wrote; 1 + i / 101 + i: the forward / backward weight fragment image of
 * parameter segment i.  *bytes: in, the capacity of dst; out, the buffer's size (0 when it
 * does not exist).  dst NULL: the size only. */
int inf_debug_buffer(inf_plan* plan, int which, void* dst, int64_t* bytes, inf_stream_t stream);

/* 1 when the last training step ran its parameter update (or gradient reduction) inside
 * the weight-gradient GEMM launch (bf16 fused chain, lgemm's gradient-tile mode: split-K 1,
 * each block updating its own 64 x 64 tile), 0 when it launched it separately, -1 before
 * any step. */
int inf_plan_last_step_fused_update(const inf_plan* plan);

/* Whether the last INF_STEP_PART1 step really split the gradient: 1 = bucketed (PART2 still
 * to run), 0 = it reduced the whole gradient (not the fused chain3 path, or a batch not a
 * multiple of 256 x the bucket splits: PART2 is then a no-op), -1 = no PART1 step yet. */
int inf_plan_last_part1_bucketed(const inf_plan* plan);

/* ---- Sharded optimizer step (data parallel; replaces nn.DataParallel's reduce to GPU 0 +
 * GPU-0 Adam + re-broadcast, reference train.py:46-48, config.py:108, trainer.py:80-82) ----
 * One step on `world` ranks:
 *   inf_train_step(..., INF_STEP_SHARD)  the local gradient, item-major, into grad_staging
 *   reduce-scatter(sum) grad_staging [world][grad_floats] -> grad_chunk [grad_floats]
 *   inf_adam_shard                       Adam on this rank's items only, their new weights
 *                                        (GEMM dtype; fp32 vectors) into its chunk of
 *                                        weight_staging [world][weight_bytes]
 *   all-gather weight_staging (this rank's chunk in place)
 *   inf_shard_scatter                    every rank rewrites all weight images and the fp32
 *                                        vector parameters from weight_staging
 * Each parameter is updated by exactly one rank, so replicas stay bitwise equal.  The fp32
 * masters and the Adam state are then current on this rank's items only: before anything
 * reads them whole (checkpoints, evaluation, inf_adam, row-major shadows -- refused until
 * then), gather each arena: inf_shard_pack(arena -> grad_chunk), all-gather grad_chunk into
 * grad_staging, inf_shard_unpack(grad_staging -> arena). */

/* The item-major staging layout for `world` ranks (re-writes the update work list; not on
 * the hot path).  Returns the per-rank chunk sizes: grad_floats (fp32 elements) and
 * weight_bytes. */
int inf_plan_shard(inf_plan* plan, int world, int rank, int64_t* grad_floats, int64_t* weight_bytes);
/* 1 when this batch's training step can run sharded (a fused chain, see INF_STEP_SHARD), else 0. */
int inf_plan_can_shard(inf_plan* plan, const inf_batch* batch);
/* Caller-owned staging: grad_staging [world * grad_floats] f32, grad_chunk [grad_floats] f32,
 * weight_staging [world * weight_bytes] bytes (zeroed here). */
int inf_plan_bind_shard(inf_plan* plan, float* grad_staging, float* grad_chunk, void* weight_staging);
/* Adam (torch formula, ctrl's step and lr) on this rank's items from grad_chunk;
 * flags: INF_STEP_ADVANCE. */
int inf_adam_shard(inf_plan* plan, int flags, inf_stream_t stream);
int inf_shard_scatter(inf_plan* plan, inf_stream_t stream);
/* arena (P floats) -> grad_chunk (this rank's items) / grad_staging (all items) -> arena. */
int inf_shard_pack(inf_plan* plan, const float* arena, float* grad_chunk, inf_stream_t stream);
int inf_shard_unpack(inf_plan* plan, const float* grad_staging, float* arena, inf_stream_t stream);

/* Advance ctrl->batch_index by one (captured at the end of a graph-replayed step). */
int inf_ctrl_advance(inf_plan* plan, inf_stream_t stream);

/* ---- Ray casting (render path) ---------------------------------
 * Replaces trimesh/embree in mesh.get_ray_mesh_intersector (mesh.py:111-117),
 * mesh.create_ray_origins_and_directions (mesh.py:171-207) and mesh.ray_mesh_intersect
 * (mesh.py:210-251): closest hit along each ray (multiple_hits=False, two-sided, t > 0)
 * and the hit point's Cramer barycentrics w.r.t. the face's vertices in mesh order. */
typedef struct inf_bvh inf_bvh;

/* Build a BVH over a triangle mesh.  vertices: host [V][3] f32; faces: host [F][3] int64
 * (mesh.faces).  Device memory is allocated here (not on the hot path). */
int inf_bvh_create(const float* vertices, int64_t num_vertices, const int64_t* faces, int64_t num_faces,
                   inf_bvh** bvh);
void inf_bvh_destroy(inf_bvh* bvh);
int inf_bvh_info(const inf_bvh* bvh, int64_t* num_faces, int32_t* num_nodes, int32_t* depth);

/* Cast one ray per masked pixel.  cam_cv2world: host [3][4] f32 (row-major), K: host [3][3]
 * f32; pixel_idx: device [num_rays] int64 pixel indices y * W + x in increasing order (the
 * obj_mask_1d-selected pixels), or null for all H * W pixels.  Outputs (device, per ray):
 * hit_face [num_rays] int32 (-1 = miss), bary [num_rays][3] f32, unit_dirs [num_rays][3] f32
 * (or null). */
int inf_raycast(const inf_bvh* bvh, const float* cam_cv2world, const float* K, int H, int W, const int64_t* pixel_idx,
                int64_t num_rays, int32_t* hit_face, float* bary, float* unit_dirs, inf_stream_t stream);

/* Cast given rays (mesh.ray_mesh_intersect's ray_origins / ray_directions): origins, dirs
 * device [num_rays][3] f32; outputs as inf_raycast. */
int inf_raycast_rays(const inf_bvh* bvh, const float* origins, const float* dirs, int64_t num_rays, int32_t* hit_face,
                     float* bary, inf_stream_t stream);

/* The hit lists of mesh.ray_mesh_intersect, in ray order: out_vids [M][3] int64 (the hit
 * faces' vertex ids), out_bary [M][3] f32, out_ray [M] int64 (hit_ray_idxs), out_face [M]
 * int64 (face_idxs, or null); *num_hits (device int64) = M.  Outputs are sized for
 * num_rays; scratch: device int32 [ceil(num_rays / 256)]. */
int inf_compact_hits(const inf_bvh* bvh, const int32_t* hit_face, const float* bary, int64_t num_rays,
                     int32_t* scratch, int64_t* num_hits, int64_t* out_vids, float* out_bary, int64_t* out_ray,
                     int64_t* out_face, inf_stream_t stream);
/* The same compaction against an explicit face table faces [F][3] int32 (the vertex ids
 * written to out_vids; texture baking maps UV-mesh faces to eigenfunction-mesh ids). */
int inf_compact_faces(const int32_t* faces, const int32_t* hit_face, const float* bary, int64_t num_rays,
                      int32_t* scratch, int64_t* num_hits, int64_t* out_vids, float* out_bary, int64_t* out_ray,
                      int64_t* out_face, inf_stream_t stream);

/* ---- texture baking (bake_texture_field.py:96-264,334-420) ------------------------ */
/* Texel -> UV triangle search and barycentrics.  uv_px [Nv][2] f64: texel coordinates
 * ((W-1) u, (H-1)(1-v)); faces [F][3] int32 into uv_px.  A texel (x, y) takes the
 * triangle of UV area >= min_area that strictly contains it (point_in_tri_matched :66-93)
 * with the nearest centroid (get_tris_fast :134-161); texel_face [H*W] int32 (-1 none),
 * texel_bary [H*W][3] f32 by bary_matched (:196-228).  keys: device u64 [H*W] scratch. */
int inf_uv_raster(const double* uv_px, int64_t num_uv_vertices, const int32_t* faces, int64_t num_faces, int height,
                  int width, double min_area, uint64_t* keys, int32_t* texel_face, float* texel_bary,
                  inf_stream_t stream);
/* uv_fill_holes (:245-264) of an fp32 [H][W][3] texture, then (255 * CC).astype(uint8)
 * into out_u8 and/or the filled fp32 texture into out_f. */
int inf_uv_fill_holes(const float* img, int height, int width, uint8_t* out_u8, float* out_f, inf_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* INF_HIP_H */
