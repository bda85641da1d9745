// Gradient reduction / Adam / packed-weight refresh (see adam.hip).
#pragma once

#include "common.hpp"

namespace inf {

enum GradSource { GRAD_NONE = 0, GRAD_SLABS = 1, GRAD_FLAT = 2 };

struct AdamSeg {
  int64_t off;          // offset (floats) of the parameter tensor in the flat arena
  int32_t R, C;         // matrix: R = out rows, C = in cols; vector: R = 1, C = numel
  int32_t matrix;       // 1: GEMM weight (64x64 tiles, packed shadows)
  int32_t nslab;        // gradient partials to sum
  const float* slab;    // element (r, c) of partial s: slab[s * slab_stride + r * slab_ld + c]
  int64_t slab_stride;
  int64_t slab_ld;
  void* W;              // packed [R][ldw] GEMM-dtype weight
  int64_t ldw;
  void* WT;             // packed [C_pad][ldwt] transposed weight
  int64_t ldwt;
  // bf16 weight images in MFMA fragment order for the register-streamed chain (chain3.hip),
  // W_0, W_y (forward) and the hidden H x H weights (both): 1 KiB per (32-deep k block kb,
  // 16-row tile t) at (kb * (rows/16) + t) KiB, lane l's 8 elements at 16 l bytes: lane
  // l = n % 16 + 16 g holds 8 k of block kb (slot g, see wf_acc_order) of row n = 16 t + l % 16
  void* WF;             // forward: n = output row r, k = input column c
  void* WTF;            // backward (dX): n = input column c, k = output row r
  // k order inside a 32-deep block: 0 = natural (slot g, element e <-> k = 8 g + e: the input
  // layers, fed the gathered features), 1 = accumulator order (k = 16 (e / 4) + 4 g + e % 4:
  // fed activations straight from 16x16x32 accumulators, chain3.hip).  WTF: always 1.
  int32_t wf_acc_order;
  // fp32 updates (bf16x3 mode): WF / WTF hold hi / lo bf16 image pairs (lo right after hi:
  // + R ldw elements for WF, + R C for WTF) instead of fp32 images -- chain3.hip X3
  int32_t x3;
  // matrix: the index of its first work item in the update's item table (its items are
  // contiguous, row-major over the 64 x 32 tiles: item0 + (r / 64) ceil(C / 32) + c / 32)
  int32_t item0;
  int32_t pad2_;
};

// inf_debug_block_times: the update launch's stamps start at this block of the buffer
constexpr int UPDATE_STAMP_BLOCK0 = 6144;

// Matrix work item = one ADAM_TILE_R x ADAM_TILE_C tile; vector item = ADAM_VEC elements.
constexpr int ADAM_TILE_R = 64;
constexpr int ADAM_TILE_C = 32;
constexpr int ADAM_VEC = 64;
constexpr int ITEM_VEC4 = 1;  // AdamItem.pad flag: 16-byte aligned rows in the arena

struct AdamItem {
  int32_t seg;
  int32_t r0, c0;
  int32_t pad;   // flags
  // sharded update (inf_plan_shard): the item's slots in the item-major staging buffers --
  // its gradient at float goff of the gradient staging (a matrix tile as [64][32], a vector
  // chunk as [64]), its new weights at byte woff of the weight staging (the GEMM dtype for
  // matrix tiles, fp32 for vector chunks)
  int32_t goff;
  int32_t woff;
};

// AdamArgs.shard_mode
enum ShardMode {
  SHARD_NONE = 0,
  SHARD_GRAD_OUT = 1,  // write_grads into the gradient staging (gsh) instead of the arena
  SHARD_ADAM = 2,      // gradient from the staging (this rank's chunk), new weights also to wsh
  SHARD_SCATTER = 3,   // no gradient: weight images (matrix) / fp32 parameters (vector) from wsh
};

struct AdamArgs {
  const AdamSeg* segs;
  const AdamItem* items;
  int32_t num_items;
  float* params;
  float* grads;
  float* exp_avg;
  float* exp_avg_sq;
  int32_t grad_src;     // GradSource
  int32_t write_grads;
  int32_t do_adam;
  int32_t write_shadow;
  int32_t step_host;    // > 0: use this t and lr_host, else ctrl->step and ctrl->lr
  double lr_host;       // used as given (0 included) when step_host > 0
  // ... and then 1 - beta^step_host from the host's std::pow (torch forms beta ** step with
  // the platform libm's pow, as inf_adam_dense does); device-counted steps (ctrl->step) use
  // adam_dev::pow_int, a few double ulps from it before the fp32 rounding
  double bc1_host, bc2_host;
  inf_ctrl* ctrl;
  // end-of-step item (AdamItem.seg < 0): fixed-order sum of the fused chain's per-tile
  // loss / SSE partials into ctrl, and the batch-index advance of a replayed epoch
  const double* loss_part;  // [nloss][2]
  int32_t nloss;
  int32_t advance;
  double beta1_d, beta2_d;
  float one_minus_b1, beta2, one_minus_b2, eps;
  // sharded update (ShardMode): item it's gradient slot is gsh[it.goff - g_base], its weight
  // slot wsh + (it.woff - w_base) bytes (the bases: this rank's chunk of a reduce-scatter)
  int32_t shard_mode;
  float* gsh;
  int64_t g_base;
  char* wsh;
  int64_t w_base;
  // diagnostics (inf_debug_block_times): wave 0 of item workgroup i stamps the wall clock
  // (100 MHz) at entry, item + segment loaded, data loaded, update stored, exit:
  // stamps[i * 8 + 0..4] (null: off)
  unsigned long long* stamps;
};

int launch_update(const AdamArgs& a, int mode, hipStream_t stream);

// The sharded state's gather (inf_shard_pack / unpack): unpack = 0 copies `items` of the
// arena `src` into the item-major staging `dst` (item it at dst[it.goff - base]), 1 copies
// the staging `src` back into the arena `dst`.
int launch_shard_copy(const AdamSeg* segs, const AdamItem* items, int num_items, const float* src, float* dst,
                      int64_t base, int unpack, hipStream_t stream);

}  // namespace inf
