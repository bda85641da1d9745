// inf_plan: one TextureField (model.py:12-112) bound to caller-owned buffers, and the
// launch sequences of its forward, backward, fused training step (trainer.py:71-84),
// Adam update (config.py:108) and render slice (renderer.py:112-146).
//
// Launch sequence of a fused training step (L layers, skip s):
//   gather (X, X^T) -> L-1 forward GEMMs (Y_l, Y_l^T; bias+ReLU; skip layer = one GEMM
//   over two K segments [h | x]) -> head_fwd (sigmoid, loss, dz) -> head_bwd (dZ_{L-2})
//   -> L-2 dX GEMMs (ReLU mask + bias-grad partials) -> ONE grouped split-K dW GEMM over
//   all weight matrices -> ONE update launch (slab reduction + Adam + packed weights).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "adam.hpp"
#include "chain.hpp"
#include "chain3.hpp"
#include "chainf.hpp"
#include "gemm.hpp"
#include "head.hpp"
#include "fgemm.hpp"
#include "zg.hpp"
#include "lgemm.hpp"
#include "rchain.hpp"
#include "blaslt.hpp"
#include "ptab.hpp"

namespace inf {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

namespace {

__global__ void ctrl_advance_kernel(inf_ctrl* c) { c->batch_index += 1; }
__global__ void prefetch_advance_kernel(inf_ctrl* c) { c->prefetch_index += 1; }

struct ParamSeg {
  int64_t off = 0;
  int32_t R = 0, C = 0;  // weight: [R][C]; bias: R = 1
  int32_t layer = 0;
  int32_t kind = 0;      // 0 weight, 1 bias
  int32_t sub = 0;       // skip layer: 0 = Lx, 1 = Ly
  // packed shadow (GEMM weights only)
  int32_t gemm = 0;
  int32_t c_pad = 0;
  int64_t w_off = 0, wt_off = 0;  // bytes into shadow
  int64_t f_off = -1, ft_off = -1;  // MFMA-fragment images (hidden H x H weights, bf16)
};

constexpr int64_t ALIGN = 256;
// inf_plan::last_chain of a step on the fused fp32 chain (chainf.hip)
constexpr int CHAIN_F32 = 6;
constexpr int CHAIN_X3 = 7;  // the split-bf16 register chain (chain3.hip X3) of the bf16x3 mode

}  // namespace
}  // namespace inf

using namespace inf;

struct inf_plan {
  inf_mlp_desc d{};
  int max_batch = 0;
  int k_pad = 0, H = 0, L = 0, s = 0, mode = 0;
  int64_t esz = 4;
  int dw_splits = 1;
  // bucketed data-parallel steps (INF_STEP_PART1 / PART2): the dW GEMM runs as two launches
  // of half the matrices each, with bucket_splits split-K partials (2 x dw_splits: the same
  // blocks per launch as the single launch), reduced through their own seg table
  int bucket_splits = 1;
  int64_t grad_split = 0;  // bucket 1 = arena [grad_split, P) (Ly and the layers after it)
  int n_items_b1 = 0;      // update work items of bucket 1 (listed first), end-of-step item included
  int last_part1 = -1;     // the last PART1 step: 1 bucketed, 0 reduced the whole gradient
  // bf16 chain3 steps fuse the update into the dW GEMM: split-K 1, 64 x 64 tiles, each block
  // applies Adam (or writes the gradient) to its own tile from the LDS gradient tile
  // (lgemm.hip GT) -- no split-K slabs, no update launch (config D; INF_LGF=0/1 forces it)
  bool lgf = false;
  bool last_lgf = false;  // the last training step took it
  bool last_zg = false;      // ... its input layers on zg.hip ahead of chain3
  int train_unit = 128;
  int bp_max = 0;
  int grid_hb = 1;
  std::vector<ParamSeg> segs;
  int64_t P = 0;
  int64_t shadow_bytes = 0;

  // workspace layout (byte offsets)
  int64_t o_x0 = 0, o_x0t = 0, o_dz = 0, o_pred = 0, o_tables = 0, o_tables_b = 0, o_ws_end = 0;
  int64_t o_xp[2] = {-1, -1};  // pre-gather slots (bf16 [bp_max][k_pad], inf_prefetch_batch)
  int64_t o_zin = -1;          // input-layer pre-activations ahead of chain3 (zg.hip), fp32 [parts][bp_max][2H]
  int zin_parts_max = 0;       // k slices o_zin holds
  int64_t o_aux_items = 0;  // fused update in the dW GEMM (lgemm.hpp): its vector items
  // the matrix items alone (the update launch after a dW GEMM that ran the vector items)
  // sharded update (data parallel, inf_plan_shard): the item-major staging layout of
  // `shard_world` ranks, this rank's items (+ the end-of-step item) as their own table
  int shard_world = 0, shard_rank = 0;
  int64_t shard_g = 0, shard_w = 0;  // one rank's chunk: floats of the gradient staging, bytes of the weight staging
  int n_shard_items = 0;
  int64_t o_shard_items = 0;
  float* sh_gsh = nullptr;     // [world][shard_g] local gradients (reduce-scatter input)
  float* sh_gshard = nullptr;  // [shard_g] this rank's reduced chunk (reduce-scatter output)
  char* sh_wsh = nullptr;      // [world][shard_w] new weights (all-gather buffer, this rank's chunk in place)
  // bits 1 / 2 / 4: params / exp_avg / exp_avg_sq are current on this rank's items only
  // (set by inf_adam_shard, cleared by inf_shard_unpack into that arena)
  int sharded_state = 0;
  int n_aux_items = 0;
  std::vector<int64_t> o_y, o_yt, o_dZ, o_dZT, o_colsum;  // per hidden layer
  std::vector<int64_t> o_slab;                            // per param segment (weights)
  int64_t o_hw = 0, o_hb = 0;                             // head partials
  int64_t o_loss = 0;                                     // chain per-tile loss partials
  int64_t table_bytes = 0;
  int64_t o_pcat = -1;  // shadow offset of [W_0; W_y] (inf_project_table)

  // bound buffers
  float* params = nullptr;
  float* grads = nullptr;
  float* exp_avg = nullptr;
  float* exp_avg_sq = nullptr;
  char* shadow = nullptr;
  char* ws = nullptr;
  inf_ctrl* ctrl = nullptr;
  bool bound = false;

  std::vector<AdamSeg> adam_segs;
  // the bucketed steps' seg table as last uploaded: kept alive with the plan (an upload made
  // inside a stream capture is a graph node that may read its host source at replay)
  std::vector<AdamSeg> adam_segs_b;
  std::vector<AdamItem> adam_items;
  double beta1 = 0.9, beta2 = 0.999, eps = 1e-8;  // torch holds them as Python doubles

  // saved forward
  int saved_batch = 0, saved_bp = 0;
  bool saved = false;
  int last_chain = 0;  // fused chain of the last training step: 0 none, 2 LDS ring, 3 registers,
                       // CHAIN_F32 the fp32 register chain
  bool stepped = false;
  // Row-major / transposed bf16 shadows (W, W^T) are read only off the fused path (layered
  // and LDS-ring GEMMs, the table projection); the fused chain3 step's update writes the
  // fragment images alone (write_shadow = 2) and marks them stale.  rm_stale: an eager
  // lazy update ran since the last rewrite; rm_captured: a lazy update was captured into a
  // graph, whose replays the host cannot see -- consumers then rewrite them every time.
  bool rm_stale = false;
  bool rm_captured = false;
  // inf_plan_weight_generation: update launches so far; gen_captured once one was captured
  int64_t weight_gen = 0;
  bool gen_captured = false;
  const uint64_t* dbg_ranges = nullptr;
  int dbg_n = 0;
  unsigned long long* dbg_out = nullptr;
  unsigned long long* stamps = nullptr;
  int stamp_steps = 0;
  unsigned long long* lg_stamps = nullptr;  // inf_debug_block_times

  template <typename T = char>
  T* W(int64_t off) const { return reinterpret_cast<T*>(ws + off); }
  const ParamSeg* weight_seg(int layer, int sub) const {
    for (const auto& p : segs)
      if (p.layer == layer && p.kind == 0 && p.sub == sub) return &p;
    return nullptr;
  }
  const ParamSeg* bias_seg(int layer, int sub) const {
    for (const auto& p : segs)
      if (p.layer == layer && p.kind == 1 && p.sub == sub) return &p;
    return nullptr;
  }
};

namespace {

int64_t align_up(int64_t x) { return round_up(x, ALIGN); }

static bool use_zg(const inf_plan* p);

int build_layout(inf_plan* p) {
  const auto& d = p->d;
  p->H = d.hidden;
  p->L = d.num_layers;
  p->s = d.skip;
  p->mode = d.mode;
  p->esz = d.mode == INF_MODE_BF16 ? 2 : 4;
  p->k_pad = (int)round_up(d.in_dim, 128);
  const int H = p->H, L = p->L, s = p->s;

  // ---- parameter arena (model.parameters() order) ----
  int64_t off = 0;
  auto add = [&](int layer, int kind, int sub, int R, int C) {
    ParamSeg g;
    g.off = off;
    g.R = R;
    g.C = C;
    g.layer = layer;
    g.kind = kind;
    g.sub = sub;
    off += (int64_t)R * C;
    p->segs.push_back(g);
  };
  for (int i = 0; i < L; ++i) {
    if (i == s) {
      add(i, 0, 0, H, H);
      add(i, 1, 0, 1, H);
      add(i, 0, 1, H, d.in_dim);
      add(i, 1, 1, 1, H);
    } else if (i == L - 1) {
      add(i, 0, 0, d.out_dim, H);
      add(i, 1, 0, 1, d.out_dim);
    } else {
      add(i, 0, 0, H, i == 0 ? d.in_dim : H);
      add(i, 1, 0, 1, H);
    }
  }
  p->P = off;

  // ---- packed shadows for the GEMM weights ----
  int64_t sh = 0;
  int64_t gemm_tiles = 0;
  for (auto& g : p->segs) {
    if (g.kind != 0 || g.layer == L - 1) continue;
    g.gemm = 1;
    g.c_pad = g.C == H ? H : p->k_pad;
    g.w_off = sh;
    sh = align_up(sh + (int64_t)g.R * g.c_pad * p->esz);
    g.wt_off = sh;
    sh = align_up(sh + (int64_t)g.c_pad * g.R * p->esz);
    const int bt = (H % 128 == 0) ? 128 : 64;
    gemm_tiles += (g.R / bt) * (g.c_pad / bt);
  }
  // fragment images: the hidden H x H weights, forward and transposed, and W_0 / W_y
  // (forward) for the register-streamed chains -- bf16 (chain3.hip, rchain.hip) or fp32
  // (chainf.hip, the fp32 mode's fused step)
  if ((p->mode == INF_MODE_BF16 || p->mode == INF_MODE_FP32 || p->mode == INF_MODE_BF16X3) && (H == 128 || H == 256)) {
    for (auto& g : p->segs) {
      if (!g.gemm) continue;
      const bool hidden = g.layer >= 1 && g.layer <= L - 2 && g.sub == 0 && g.R == H && g.C == H;
      const bool input = (g.layer == 0 && g.sub == 0) || (g.layer == s && g.sub == 1);
      if (!hidden && !input) continue;
      g.f_off = sh;
      sh = align_up(sh + (int64_t)g.R * g.c_pad * p->esz);
      if (hidden) {
        g.ft_off = sh;
        sh = align_up(sh + (int64_t)H * H * p->esz);
      }
    }
  }
  // [W_0; W_y] row-major, the B operand of inf_project_table's single N = 2H GEMM (each
  // table tile read once; refreshed from the two shadows per call)
  if (p->mode == INF_MODE_BF16 && s >= 0 && s < L - 1) {
    p->o_pcat = sh;
    sh = align_up(sh + 2 * (int64_t)H * p->k_pad * 2);
  }
  p->shadow_bytes = sh;

  // ---- split-K factor of the weight-gradient GEMMs and batch padding ----
  int S = 1;
  const int64_t mb = round_up(std::max(p->max_batch, 1), 128);
  while (gemm_tiles * S < 512 && S < 16 && mb / (S * 2) >= 512) S *= 2;
  // bf16 steps of the register-streamed chain reduce their weight gradients with lgemm
  // (896-block grid at 4096 rays already): fewer, longer splits halve the slab traffic
  // the update launch reads (4096 rays: dW + update 30.8 -> 25.2 us at 4 splits vs 8)
  // 4096 rays: 2 splits (224 blocks of 8 k-steps, one per CU) beat 4 (448 blocks of 4 on
  // 256 CUs, the same 8-step critical path) by the halved slab bytes: step 73.0 -> 71.3 us
  // (tools/split_sweep.sh)
  // (the bf16x3 mode's dW runs on the same register GEMM over split operands: lgemm SPLIT)
  const bool reg_dw = d.mode == INF_MODE_BF16 || d.mode == INF_MODE_BF16X3;
  if (reg_dw && mb <= CHAIN3_MAX_ROWS && S > 4) S = 4;
  if (reg_dw && mb <= 4096 && S > 2) S = 2;
  // the fused gradient-tile update (lgemm.hip GT) of the bf16 chain3 step: split-K 1 over
  // 64 x 64 tiles (arena rows element-wise where they are not 16-byte aligned: config R's
  // k = 1023; tiles of the column padding c_pad > C skipped)
  // Default only for the chunked-tile tables (k_pad > C3_KC, config D: dW + update 54.8 ->
  // 47.5 us, step 145.4 -> 140.8 us).  At config B the 64 x 64 split-K-1 GEMM's longer main
  // loop (15.2 us vs the 2-split 64 x 128 GEMM's whole 15.7) plus the per-block update tail
  // (4-6 us) cost what the update launch did (stage 26.7 vs 15.7 + 8.5 us; step 69.4-70.3 vs
  // 68.1-69.3), configs A / R lose 2-3 us (profiles/r04/lgf_sweep.log).  INF_LGF=0/1 forces it.
  const char* lgf_env = std::getenv("INF_LGF");
  p->lgf = d.mode == INF_MODE_BF16 && mb <= CHAIN3_MAX_ROWS &&
           (lgf_env != nullptr ? std::atoi(lgf_env) != 0 : p->k_pad > C3_KC);
  for (const auto& g : p->segs)
    if (g.gemm && (g.c_pad % 64 != 0 || g.R % 64 != 0)) p->lgf = false;
  if (p->lgf) S = 1;
  // the 64-ray chain tiles' dW through lgemm (shapes fgemm does not tile) stream
  // K = Bp / S rays per block in 256-ray steps: 10,240 rays take 8 splits, not 16
  while (d.mode == INF_MODE_BF16 && mb > CHAIN3_MAX_ROWS && S > 1 && mb % (256 * (int64_t)S) != 0) S /= 2;
  if (const char* e = std::getenv("INF_DW_SPLITS")) {  // tuning experiments
    const int want = std::atoi(e);
    if (want >= 1 && want <= 16 && (want & (want - 1)) == 0 && mb / want >= 128) S = want;
  }
  if (S != 1) p->lgf = false;  // INF_DW_SPLITS: the slab path
  p->dw_splits = S;
  p->bucket_splits = S;
  if (d.mode == INF_MODE_BF16 && mb <= CHAIN3_MAX_ROWS && 2 * S <= 16 && (mb / (2 * S)) % 256 == 0)
    p->bucket_splits = 2 * S;
  if (const char* e = std::getenv("INF_BUCKET_SPLITS")) {  // = dw_splits: bitwise the unbucketed step
    const int want = std::atoi(e);
    if (want >= 1 && want <= 16 && (want & (want - 1)) == 0 && mb / want >= 256) p->bucket_splits = want;
  }
  p->train_unit = (int)std::max<int64_t>(128, (int64_t)S * 64);
  p->bp_max = (int)round_up(p->max_batch, p->train_unit);
  p->grid_hb = (int)std::min<int64_t>(256, p->bp_max / HEAD_BWD_RAYS);
  const int64_t Bp = p->bp_max;

  // ---- workspace ----
  int64_t w = 0;
  auto take = [&](int64_t bytes) {
    const int64_t o = w;
    w = align_up(w + bytes);
    return o;
  };
  p->o_x0 = take(Bp * p->k_pad * p->esz);
  p->o_x0t = take((int64_t)p->k_pad * Bp * p->esz);
  if (p->mode == INF_MODE_BF16 && Bp <= CHAIN3_MAX_ROWS)
    for (int i = 0; i < 2; ++i) p->o_xp[i] = take(Bp * p->k_pad * 2);
  // zg.hip's k slices (at most zg_splits of the smallest batch, 64 rays), only where the
  // step can run zg (use_zg: k_pad > C3_KC or INF_ZG=1)
  if (p->mode == INF_MODE_BF16 && Bp <= CHAIN3_MAX_ROWS && zg_supported(H, p->k_pad, Bp) && use_zg(p)) {
    p->zin_parts_max = zg_splits(p->k_pad, 64);
    p->o_zin = take((int64_t)p->zin_parts_max * Bp * 2 * H * 4);
  }
  const int64_t max_parts =
      std::max<int64_t>({chain_max_partials(Bp), std::min<int64_t>(Bp, CHAIN3_WIDE_MAX_ROWS) / 16, (int64_t)p->grid_hb});
  for (int l = 0; l < L - 1; ++l) {
    p->o_y.push_back(take(Bp * H * p->esz));
    p->o_yt.push_back(take(Bp * H * p->esz));
    p->o_dZ.push_back(take(Bp * H * p->esz));
    p->o_dZT.push_back(take(Bp * H * p->esz));
    p->o_colsum.push_back(take(max_parts * H * 4));
  }

  p->o_dz = take(Bp * 3 * 4);
  p->o_pred = take(Bp * 3 * 4);
  p->o_slab.assign(p->segs.size(), 0);
  for (size_t i = 0; i < p->segs.size(); ++i) {
    const auto& g = p->segs[i];
    if (g.gemm) p->o_slab[i] = take((int64_t)std::max(S, p->bucket_splits) * g.R * g.c_pad * 4);
  }
  p->o_hw = take(max_parts * 3 * H * 4);
  p->o_hb = take(max_parts * 3 * 4);
  p->o_loss = take(std::max<int64_t>(Bp / 16, 1) * 2 * 8);

  // update work list
  int64_t nitems = 1;  // + the end-of-step item
  for (const auto& g : p->segs) nitems += g.gemm ? ceil_div(g.R, ADAM_TILE_R) * ceil_div(g.C, ADAM_TILE_C) : ceil_div((int64_t)g.R * g.C, ADAM_VEC);
  p->table_bytes = align_up((int64_t)p->segs.size() * sizeof(AdamSeg)) + align_up(nitems * sizeof(AdamItem));
  p->o_tables = take(p->table_bytes);
  p->o_tables_b = take(align_up((int64_t)p->segs.size() * sizeof(AdamSeg)));
  p->o_aux_items = take(align_up((nitems + 8) * sizeof(AdamItem)));
  p->o_shard_items = take(align_up((nitems + 1) * sizeof(AdamItem)));
  p->o_ws_end = w;
  return INF_OK;
}

// Tile override for tuning experiments: INF_TILE_<WHAT>=128x128|128x64|64x64.
bool tile_override(const char* what, GemmTile* t) {
  char name[64];
  std::snprintf(name, sizeof(name), "INF_TILE_%s", what);
  const char* v = std::getenv(name);
  if (v == nullptr) return false;
  if (!std::strcmp(v, "128x128")) *t = TILE_128x128;
  else if (!std::strcmp(v, "128x64")) *t = TILE_128x64;
  else *t = TILE_64x64;
  return true;
}

GemmTile pick_tile(const inf_plan* p, int64_t M, int64_t N) {
  if (M % 128 || N % 128) return TILE_64x64;
  const int64_t blocks = (M / 128) * (N / 128);
  return blocks >= 256 ? TILE_128x128 : TILE_64x64;
}

GemmProblem blank_problem() {
  GemmProblem q;
  std::memset(&q, 0, sizeof(q));
  q.nseg = 1;
  q.splits = 1;
  return q;
}

int dtype_of(const inf_plan* p) { return p->mode == INF_MODE_BF16 ? INF_DTYPE_BF16 : INF_DTYPE_F32; }

// GEMM arithmetic of a layered GEMM in the split-bf16 plan mode.  3 products (hi*hi +
// hi*lo + lo*hi) put RGB within 1e-6 of the reference, but at config B a forward on them
// leaves a gradient of layers.0 8.4e-3 of its max from the reference's (pre-activations
// at rounding distance from the ReLU kink change their mask; measured with the backward on
// 6 products too), while a forward on 6 holds every gradient within 1.4e-5 of its max with
// the backward GEMMs (dX, dW) on 3 (7.9e-6 with dX on 6; 8.7e-7 with all on 6:
// tests/test_gpu_bf16x3.py, profiles/r03/bf16x3_*_tests.log).  Default: forward 6, dX 3,
// dW 3; INF_X3_{FWD,DX,DW}=3|6 override for experiments.
enum GemmRole { ROLE_FWD = 0, ROLE_DX = 1, ROLE_DW = 2 };
int gemm_mode(const inf_plan* p, GemmRole role) {
  if (p->mode != INF_MODE_BF16X3) return p->mode;
  static const char* names[3] = {"INF_X3_FWD", "INF_X3_DX", "INF_X3_DW"};
  static const int defaults[3] = {6, 3, 3};
  int terms = defaults[role];
  if (const char* e = std::getenv(names[role])) terms = std::atoi(e) == 6 ? 6 : 3;
  return terms == 6 ? GEMM_MODE_BF16X6 : INF_MODE_BF16X3;
}

// ---------------------------------------------------------------------------------
int ensure_rowmajor(inf_plan* p, hipStream_t st);

int run_input(inf_plan* p, const inf_batch* b, int Bp, bool transposed, hipStream_t st) {
  void* x0 = p->W(p->o_x0);
  void* x0t = transposed ? (void*)p->W(p->o_x0t) : nullptr;
  if (b->table != nullptr && b->encoding != INF_ENC_NONE) {
    INF_CHECK_ARG(b->table_dtype == INF_DTYPE_F32, "encoded batches read an fp32 vertex table");
    INF_CHECK_ARG(encoded_dim(b->encoding, b->enc_k, b->enc_include_input) == p->d.in_dim,
                  "encoding width does not match the model's in_dim");
    return launch_encode((const float*)b->table, b->num_vertices, b->vids, b->vid_dtype, b->bary, b->ray_idx,
                         b->idx_dtype, b->idx_offset, b->offset_from_ctrl ? &p->ctrl->batch_index : nullptr,
                         b->num_rays, b->num_source_rays, b->batch, b->encoding, b->enc_k, b->enc_proj,
                         b->enc_include_input, x0,
                         dtype_of(p), p->k_pad, Bp, x0t, Bp, st);
  }
  if (b->table != nullptr) {
    const int64_t k_table = p->k_pad;  // device tables are packed with k_pad zero-filled columns
    return launch_gather(b->table, b->table_dtype, b->num_vertices, (int)k_table, k_table, b->vids, b->vid_dtype,
                         b->bary, b->ray_idx, b->idx_dtype, b->idx_offset,
                         b->offset_from_ctrl ? &p->ctrl->batch_index : nullptr, b->num_rays, b->num_source_rays,
                         b->batch, x0, dtype_of(p),
                         p->k_pad, Bp, x0t, Bp, st);
  }
  INF_CHECK_ARG(b->features != nullptr, "batch has neither a table nor features");
  return launch_pack_features(b->features, b->ld_features, p->d.in_dim, b->batch, x0, dtype_of(p), p->k_pad, Bp,
                              x0t, Bp, st);
}

int run_forward_layer(inf_plan* p, int Bp, bool transposed, int l, hipStream_t st);

int run_forward_layers(inf_plan* p, int Bp, bool transposed, hipStream_t st) {
  if (int rc = ensure_rowmajor(p, st)) return rc;
  for (int l = 0; l < p->L - 1; ++l) {
    int rc = run_forward_layer(p, Bp, transposed, l, st);
    if (rc) return rc;
  }
  return INF_OK;
}

int run_forward_layer(inf_plan* p, int Bp, bool transposed, int l, hipStream_t st) {
  const int H = p->H;
  const GemmTile tile = pick_tile(p, Bp, H);
  {
    GemmBatch gb;
    std::memset(&gb, 0, sizeof(gb));
    gb.nprob = 1;
    GemmProblem& q = gb.p[0];
    q = blank_problem();
    const ParamSeg* w = p->weight_seg(l, 0);
    const ParamSeg* bs = p->bias_seg(l, 0);
    q.A[0] = l == 0 ? (const void*)p->W(p->o_x0) : (const void*)p->W(p->o_y[l - 1]);
    q.lda[0] = l == 0 ? p->k_pad : H;
    q.B[0] = p->shadow + w->w_off;
    q.ldb[0] = w->c_pad;
    q.K[0] = l == 0 ? p->k_pad : H;
    q.bias0 = p->params + bs->off;
    if (l == p->s) {
      const ParamSeg* wy = p->weight_seg(l, 1);
      q.nseg = 2;
      q.A[1] = p->W(p->o_x0);
      q.lda[1] = p->k_pad;
      q.B[1] = p->shadow + wy->w_off;
      q.ldb[1] = wy->c_pad;
      q.K[1] = p->k_pad;
      q.bias1 = p->params + p->bias_seg(l, 1)->off;
    }
    q.M = Bp;
    q.N = H;
    q.relu = 1;
    q.C = p->W(p->o_y[l]);
    q.ldc = H;
    if (transposed) {
      q.CT = p->W(p->o_yt[l]);
      q.ldct = Bp;
    }
    int rc = launch_gemm(gb, gemm_mode(p, ROLE_FWD), tile, st);
    if (rc) return rc;
  }
  return INF_OK;
}

bool use_fgemm(const inf_plan* p, int Bp, int splits);
bool use_split_lgemm(const inf_plan* p, int Bp);
int run_weight_grads(inf_plan* p, int Bp, hipStream_t st, int chain = 0, const AdamArgs* fuse = nullptr,
                     int bucket = 0);

// Backward from dZ_{L-2} (already produced by head_bwd) to the reduced gradients.
int run_backward_layers(inf_plan* p, int Bp, hipStream_t st) {
  if (int rc = ensure_rowmajor(p, st)) return rc;
  const int H = p->H, L = p->L;
  const GemmTile tile = pick_tile(p, Bp, H);
  for (int l = L - 2; l >= 1; --l) {
    GemmBatch gb;
    std::memset(&gb, 0, sizeof(gb));
    gb.nprob = 1;
    GemmProblem& q = gb.p[0];
    q = blank_problem();
    const ParamSeg* w = p->weight_seg(l, 0);  // Lx at the skip layer
    q.A[0] = p->W(p->o_dZ[l]);
    q.lda[0] = H;
    q.B[0] = p->shadow + w->wt_off;
    q.ldb[0] = w->R;
    q.K[0] = H;
    q.M = Bp;
    q.N = H;
    q.mask = p->W(p->o_y[l - 1]);
    q.ldmask = H;
    if (l - 1 >= 1) {
      q.C = p->W(p->o_dZ[l - 1]);
      q.ldc = H;
    }
    q.CT = p->W(p->o_dZT[l - 1]);
    q.ldct = Bp;
    q.colsum = p->W<float>(p->o_colsum[l - 1]);
    int rc = launch_gemm(gb, gemm_mode(p, ROLE_DX), tile, st);
    if (rc) return rc;
  }
  return run_weight_grads(p, Bp, st);
}

// chain (2, 3): Y^T / dZ^T were written by the fused chain in its 16-ray blocked layout;
// with the register-streamed chain (3) Y_0^T comes plain from the input GEMM
// bf16x3 mode behind the fused fp32 chain: the chain writes X^T / Y^T / dZ^T as hi / lo bf16
// fragment images and the dW runs on the register GEMM with three MFMAs per k block
// (lgemm.hip SPLIT) instead of gemm.hip's split-bf16 over 16-ray blocked fp32 operands.
// INF_NO_SPLIT_LGEMM=1: the blocked operands and gemm.hip.
bool use_split_lgemm(const inf_plan* p, int Bp) {
  if (p->mode != INF_MODE_BF16X3 || std::getenv("INF_NO_SPLIT_LGEMM") != nullptr) return false;
  if (Bp % p->dw_splits != 0 || (Bp / p->dw_splits) % (64 * 4) != 0) return false;
  for (const ParamSeg& g : p->segs)
    if (g.gemm && (g.c_pad % 64 != 0 || g.R % LG_BN != 0)) return false;
  return true;
}

int run_weight_grads(inf_plan* p, int Bp, hipStream_t st, int chain, const AdamArgs* fuse, int bucket) {
  const int H = p->H, s = p->s;
  if ((chain == CHAIN_F32 || chain == CHAIN_X3) && use_split_lgemm(p, Bp)) {
    INF_CHECK_ARG(fuse == nullptr, "split-operand dW: no fused update");
    const int splits = bucket ? p->bucket_splits : p->dw_splits;
    LgemmBatch lb;
    std::memset(&lb, 0, sizeof(lb));
    lb.split = 1;
    for (size_t i = 0; i < p->segs.size(); ++i) {
      const ParamSeg& g = p->segs[i];
      if (!g.gemm) continue;
      if ((bucket == 1 && g.off < p->grad_split) || (bucket == 2 && g.off >= p->grad_split)) continue;
      INF_CHECK_ARG(lb.nprob < LGEMM_MAX_PROBLEMS, "lgemm: too many weight matrices");
      LgemmProblem& q = lb.p[lb.nprob++];
      const int l = g.layer;
      const bool from_input = (l == 0) || (l == s && g.sub == 1);
      const int R = from_input ? p->k_pad : H;
      bf16* a_img = from_input ? p->W<bf16>(p->o_x0t) : p->W<bf16>(p->o_yt[l - 1]);
      bf16* b_img = p->W<bf16>(p->o_dZT[l]);
      q.Af = a_img;
      q.Af_lo = a_img + (int64_t)R * Bp;
      q.a_tiles = R / 16;
      q.Bf = b_img;
      q.Bf_lo = b_img + (int64_t)H * Bp;
      q.b_tiles = H / 16;
      q.M = g.c_pad;
      q.N = g.R;
      q.K = Bp;
      q.splits = splits;
      q.slab = p->W<float>(p->o_slab[i]);
      q.slab_ld = g.c_pad;
      q.slab_stride = (int64_t)g.R * g.c_pad;
    }
    // rows per block: 64 (INF_SPLIT_LGEMM_BM=32: twice the blocks, half the A tile each)
    const char* e = std::getenv("INF_SPLIT_LGEMM_BM");
    return launch_lgemm(lb, e != nullptr && std::atoi(e) == 32 ? 32 : 64, st);
  }
  if (chain == 3) {
    // bucket 1 / 2: only the matrices of arena [grad_split, P) / [0, grad_split), with
    // bucket_splits partials each (the data-parallel bucketed step)
    const int splits = bucket ? p->bucket_splits : p->dw_splits;
    // large batches (the 64-ray chain tiles): 256 x 256 output tiles over the same images
    // (fgemm.hip), when every matrix is a whole number of them
    if (fuse == nullptr && use_fgemm(p, Bp, splits)) {
      FgemmBatch fb;
      std::memset(&fb, 0, sizeof(fb));
      fb.K = Bp;
      fb.splits = splits;
      for (size_t i = 0; i < p->segs.size(); ++i) {
        const ParamSeg& g = p->segs[i];
        if (!g.gemm) continue;
        if ((bucket == 1 && g.off < p->grad_split) || (bucket == 2 && g.off >= p->grad_split)) continue;
        INF_CHECK_ARG(fb.nprob < FGEMM_MAX_PROBLEMS, "fgemm: too many weight matrices");
        FgemmProblem& q = fb.p[fb.nprob++];
        const int l = g.layer;
        const bool from_input = (l == 0) || (l == s && g.sub == 1);
        q.Af = from_input ? p->W<bf16>(p->o_x0t) : p->W<bf16>(p->o_yt[l - 1]);
        q.a_tiles = (from_input ? p->k_pad : H) / 16;
        q.Bf = p->W<bf16>(p->o_dZT[l]);
        q.b_tiles = H / 16;
        q.M = g.c_pad;
        q.N = g.R;
        q.slab = p->W<float>(p->o_slab[i]);
        q.slab_ld = g.c_pad;
        q.slab_stride = (int64_t)g.R * g.c_pad;
      }
      return launch_fgemm(fb, st);
    }
    // register-streamed chain: X^T, Y_l^T and dZ_l^T are fragment images (chain3.hip); one
    // lgemm launch computes every dW^T tile into the split-K slabs the update launch reduces
    // (GT: split-K 1, each block updates its own tile from LDS -- the fused default)
    const bool gt = fuse != nullptr && p->lgf && splits == 1 && bucket == 0;
    LgemmBatch lb;
    std::memset(&lb, 0, sizeof(lb));
    for (size_t i = 0; i < p->segs.size(); ++i) {
      const ParamSeg& g = p->segs[i];
      if (!g.gemm) continue;
      if ((bucket == 1 && g.off < p->grad_split) || (bucket == 2 && g.off >= p->grad_split)) continue;
      INF_CHECK_ARG(lb.nprob < LGEMM_MAX_PROBLEMS, "lgemm: too many weight matrices");
      LgemmProblem& q = lb.p[lb.nprob++];
      q.adam_seg = (int32_t)i;
      q.adam_vec4 = (g.C % 4 == 0 && g.off % 4 == 0) ? ITEM_VEC4 : 0;
      const int l = g.layer;
      const bool from_input = (l == 0) || (l == s && g.sub == 1);
      // layer inputs as the chain wrote them: X^T / Y_{l-1}^T fragment images
      q.Af = from_input ? p->W<bf16>(p->o_x0t) : p->W<bf16>(p->o_yt[l - 1]);
      q.a_tiles = (from_input ? p->k_pad : H) / 16;
      q.a_row0 = 0;
      q.Bf = p->W<bf16>(p->o_dZT[l]);
      q.b_tiles = H / 16;
      q.M = g.c_pad;
      q.N = g.R;
      q.K = Bp;
      q.splits = splits;
      q.slab = gt ? nullptr : p->W<float>(p->o_slab[i]);
      q.slab_ld = g.c_pad;
      q.slab_stride = (int64_t)g.R * g.c_pad;
    }
    lb.stamps = p->lg_stamps;
    if (fuse != nullptr) {
      INF_CHECK_ARG(gt, "lgemm: the update fuses into split-K-1 gradient tiles only");
      lb.fused = 2;
      lb.adam = *fuse;
      lb.n_aux_items = p->n_aux_items;
      lb.n_aux = (int)round_up(p->n_aux_items, 8);
      lb.aux_items = reinterpret_cast<const AdamItem*>(p->ws + p->o_aux_items);
    }
    // (128 x 128 tiles measured slower at 2 and 4 splits: step 75.3 / 71.6 vs 68.1-69.9 us,
    // profiles/r04/lgemm_tile_split_sweep.log; so were 4 splits of 64 x 128: 70.5-70.9)
    return launch_lgemm(lb, 64, st);
  }
  // weight gradients: one grouped split-K launch (chunks of GEMM_MAX_PROBLEMS)
  std::vector<GemmProblem> probs;
  for (size_t i = 0; i < p->segs.size(); ++i) {
    const ParamSeg& g = p->segs[i];
    if (!g.gemm) continue;
    GemmProblem q = blank_problem();
    const int l = g.layer;
    q.A[0] = p->W(p->o_dZT[l]);
    q.lda[0] = chain ? (int64_t)H * 16 : Bp;
    q.a_kblk = chain ? 1 : 0;
    const bool from_input = (l == 0) || (l == s && g.sub == 1);
    // chainf (CHAIN_F32) writes every operand 16-ray blocked, X^T included
    const bool b_blocked = chain && (chain == CHAIN_F32 || (!from_input && !(chain == 3 && l == 1)));
    q.B[0] = from_input ? (const void*)p->W(p->o_x0t) : (const void*)p->W(p->o_yt[l - 1]);
    q.ldb[0] = b_blocked ? (int64_t)(from_input ? p->k_pad : H) * 16 : Bp;
    q.b_kblk = b_blocked ? 1 : 0;
    q.K[0] = Bp;
    q.M = g.R;
    q.N = g.c_pad;
    q.splits = p->dw_splits;
    q.slab = p->W<float>(p->o_slab[i]);
    q.slab_ld = g.c_pad;
    q.slab_stride = (int64_t)g.R * g.c_pad;
    probs.push_back(q);
  }
  GemmTile wtile = (H % 128 == 0) ? TILE_128x128 : TILE_64x64;
  tile_override("DW", &wtile);
  for (size_t i0 = 0; i0 < probs.size(); i0 += GEMM_MAX_PROBLEMS) {
    GemmBatch gb;
    std::memset(&gb, 0, sizeof(gb));
    gb.nprob = (int)std::min<size_t>(GEMM_MAX_PROBLEMS, probs.size() - i0);
    for (int j = 0; j < gb.nprob; ++j) gb.p[j] = probs[i0 + j];
    int rc = launch_gemm(gb, gemm_mode(p, ROLE_DW), wtile, st);
    if (rc) return rc;
  }
  return INF_OK;
}

AdamArgs update_args(inf_plan* p, int Bp) {
  AdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.segs = p->W<AdamSeg>(p->o_tables);
  a.items = reinterpret_cast<const AdamItem*>(p->ws + p->o_tables + align_up(p->segs.size() * sizeof(AdamSeg)));
  a.num_items = (int)p->adam_items.size();
  a.params = p->params;
  a.grads = p->grads;
  a.exp_avg = p->exp_avg;
  a.exp_avg_sq = p->exp_avg_sq;
  a.ctrl = p->ctrl;
  a.beta1_d = p->beta1;
  a.beta2_d = p->beta2;
  // the fp32 constants torch's CPU kernels use: the double expressions rounded once
  // (lerp_ weight 1 - beta1, mul_ beta2, addcmul_ value 1 - beta2, add_ eps)
  a.one_minus_b1 = (float)(1.0 - p->beta1);
  a.beta2 = (float)p->beta2;
  a.one_minus_b2 = (float)(1.0 - p->beta2);
  a.eps = (float)p->eps;
  // diagnostics (inf_debug_block_times): the update's item stamps after the dW GEMM's blocks
  a.stamps = p->lg_stamps != nullptr ? p->lg_stamps + (int64_t)UPDATE_STAMP_BLOCK0 * 8 : nullptr;
  (void)Bp;
  return a;
}

bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// An update launch that leaves W / W^T behind (write_shadow = 2) or rewrites them (1).
void note_shadow_write(inf_plan* p, const AdamArgs& a, hipStream_t st) {
  const bool capturing = stream_capturing(st);
  if (a.write_shadow != 0 || a.do_adam) {
    ++p->weight_gen;
    if (capturing) p->gen_captured = true;
  }
  if (a.write_shadow == 2) {
    p->rm_stale = true;
    if (capturing) p->rm_captured = true;
  } else if (a.write_shadow == 1 && !capturing) {
    p->rm_stale = false;
  }
}

// A launch that reads the fp32 masters or the Adam state of every parameter: refused while
// a sharded update left them current on this rank's items only (inf_shard_unpack first).
int check_unsharded(const inf_plan* p, const char* what) {
  if (p->sharded_state == 0) return INF_OK;
  set_error(std::string(what) + ": the optimizer state is sharded (inf_adam_shard); gather it with inf_shard_pack / "
            "all-gather / inf_shard_unpack of params, exp_avg and exp_avg_sq first");
  return INF_ERR_STATE;
}

// Before any launch that reads W / W^T: rewrite every shadow from the fp32 masters if a
// lazy update may have run since they were last written (always, once one was captured).
int ensure_rowmajor(inf_plan* p, hipStream_t st) {
  if (!p->rm_stale && !p->rm_captured) return INF_OK;
  if (int rc = check_unsharded(p, "row-major weight refresh")) return rc;
  AdamArgs a = update_args(p, p->bp_max);
  a.grad_src = GRAD_NONE;
  a.write_shadow = 1;
  const int rc = launch_update(a, p->mode, st);
  if (rc == INF_OK && !stream_capturing(st)) p->rm_stale = false;
  return rc;
}

// fused chain3 steps in bf16 leave the row-major shadows to ensure_rowmajor
// (INF_EAGER_SHADOWS=1: every update rewrites all shadows)
int step_shadow_mode(const inf_plan* p, int chain) {
  return ((chain == 3 && p->mode == INF_MODE_BF16) || ((chain == CHAIN_F32 || chain == CHAIN_X3) && p->mode != INF_MODE_BF16)) &&
                 std::getenv("INF_EAGER_SHADOWS") == nullptr
             ? 2
             : 1;
}

// The seg table of the bucketed steps: the matrices' gradients summed over bucket_splits
// split-K partials.
std::vector<AdamSeg> bucket_segs(const inf_plan* p) {
  std::vector<AdamSeg> t = p->adam_segs;
  for (auto& a : t)
    if (a.matrix) a.nslab = p->bucket_splits;
  return t;
}

// The bias partial counts depend on the padded batch: refresh the seg table for it.
int refresh_tables(inf_plan* p, int Bp, hipStream_t st, int chain = 0) {
  const int parts = chain == 3 ? Bp / chain3_bm(Bp)
                    : (chain == CHAIN_F32 || chain == CHAIN_X3) ? Bp / 16
                    : chain ? Bp / chain_partial_rows(chain_bm(Bp))
                            : Bp / 64;
  bool changed = false;
  for (size_t i = 0; i < p->segs.size(); ++i) {
    const ParamSeg& g = p->segs[i];
    AdamSeg& a = p->adam_segs[i];
    if (g.gemm) continue;
    // hidden biases: one partial per 64 rays; the last hidden layer's and the output
    // layer's come from head_bwd (grid_hb partials) on the layered path
    const bool from_head = g.layer == p->L - 1 || (g.kind == 1 && g.layer == p->L - 2);
    const int want = (from_head && !chain) ? p->grid_hb : parts;
    if (a.nslab != want) {
      a.nslab = want;
      changed = true;
    }
  }
  if (!changed) return INF_OK;
  // Outside a capture, pageable-source async copies are staged by the runtime before
  // returning; inside one (a plan whose first step is captured) the copy is a graph node, and
  // a replay measured as if it re-read its source, so the sources are
  // the plan's own vectors, updated in place (same storage).
  INF_HIP_TRY(hipMemcpyAsync(p->ws + p->o_tables, p->adam_segs.data(), p->adam_segs.size() * sizeof(AdamSeg),
                             hipMemcpyHostToDevice, st));
  {
    const std::vector<AdamSeg> tb = bucket_segs(p);
    if (p->adam_segs_b.size() != tb.size()) p->adam_segs_b.resize(tb.size());
    std::copy(tb.begin(), tb.end(), p->adam_segs_b.begin());
  }
  INF_HIP_TRY(hipMemcpyAsync(p->ws + p->o_tables_b, p->adam_segs_b.data(), p->adam_segs_b.size() * sizeof(AdamSeg),
                             hipMemcpyHostToDevice, st));
  return INF_OK;
}

int pad_batch(inf_plan* p, int B, bool train, int* Bp) {
  INF_CHECK_ARG(B >= 1 && B <= p->max_batch, "batch size out of range for this plan");
  *Bp = (int)round_up(B, train ? p->train_unit : 128);
  INF_CHECK_ARG(*Bp <= p->bp_max, "padded batch exceeds the plan");
  return INF_OK;
}

int head_forward(inf_plan* p, const inf_batch* b, int Bp, float* pred, bool loss, const int64_t* hit,
                 const int64_t* pixel_map, float* img, hipStream_t st) {
  HeadFwdArgs a;
  std::memset(&a, 0, sizeof(a));
  const ParamSeg* w = p->weight_seg(p->L - 1, 0);
  a.h = p->W(p->o_y[p->L - 2]);
  a.ldh = p->H;
  a.H = p->H;
  a.W = p->params + w->off;
  a.bias = p->params + p->bias_seg(p->L - 1, 0)->off;
  a.batch = b->batch;
  a.rows = Bp;
  a.pred = pred;
  if (loss) {
    INF_CHECK_ARG(b->rgb != nullptr, "training batch without target colours");
    a.rgb = b->rgb;
    a.ray_idx = b->ray_idx;
    a.idx_dtype = b->idx_dtype;
    a.idx_offset = b->idx_offset;
    a.num_rays = b->num_rays;
    a.num_src = b->num_source_rays;
    a.offset_from_ctrl = b->offset_from_ctrl;
    a.loss = b->loss >= 0 ? b->loss : p->d.loss;
    INF_CHECK_ARG(a.loss >= INF_LOSS_L2 && a.loss <= INF_LOSS_CAUCHY, "loss type");
    const int64_t cnt = b->loss_count > 0 ? b->loss_count : (int64_t)3 * b->batch;
    a.inv_count = (float)(1.0 / (double)cnt);
    a.dz = p->W<float>(p->o_dz);
  }
  a.ctrl = p->ctrl;
  a.hit = hit;
  a.pixel_map = pixel_map;
  a.img = img;
  return launch_head_fwd(a, p->mode, st);
}

int head_backward(inf_plan* p, int Bp, const float* dpred, bool count_step, hipStream_t st) {
  HeadBwdArgs a;
  std::memset(&a, 0, sizeof(a));
  const int L = p->L;
  a.dz = dpred == nullptr ? p->W<float>(p->o_dz) : nullptr;
  a.dpred = dpred;
  a.pred = p->W<float>(p->o_pred);
  a.h = p->W(p->o_y[L - 2]);
  a.ldh = p->H;
  a.H = p->H;
  a.W = p->params + p->weight_seg(L - 1, 0)->off;
  a.batch = p->saved_batch;
  a.rows = Bp;
  a.dZ = (L - 2 >= 1) ? p->W(p->o_dZ[L - 2]) : nullptr;
  a.ldz = p->H;
  a.dZT = p->W(p->o_dZT[L - 2]);
  a.ldzt = Bp;
  a.colsum = p->W<float>(p->o_colsum[L - 2]);
  a.dW_part = p->W<float>(p->o_hw);
  a.db_part = p->W<float>(p->o_hb);
  a.step_ctrl = count_step ? p->ctrl : nullptr;
  a.grid = p->grid_hb;
  return launch_head_bwd(a, p->mode, st);
}

bool use_chain(const inf_plan* p) {
  return p->mode == INF_MODE_BF16 && chain_supported(p->H) && p->L - 1 <= CHAIN_MAX_HIDDEN &&
         std::getenv("INF_NO_CHAIN") == nullptr;
}

// Forward (train = 0) or fused forward + loss + backward chain (train = 1) of a padded
// batch whose features are already in X0 (csrc/chain.hip).
int run_chain(inf_plan* p, const inf_batch* b, int Bp, bool train, float* pred, const int64_t* hit,
              const int64_t* pixel_map, float* img, hipStream_t st) {
  if (int rc = ensure_rowmajor(p, st)) return rc;
  const int H = p->H, L = p->L, s = p->s;
  const int bm = chain_bm(Bp);
  const int BK = chain_bk(bm);
  ChainArgs a;
  std::memset(&a, 0, sizeof(a));
  a.L = L;
  a.s = s;
  a.H = H;
  a.k_pad = p->k_pad;
  a.rows = Bp;
  a.batch = b->batch;
  a.X = p->W<bf16>(p->o_x0);
  int np = 0, steps = 0;
  auto add = [&](const void* B, int ldb, int K, int a_src, int layer, int kind, int epi) {
    ChainPhase& ph = a.ph[np++];
    ph.B = reinterpret_cast<const bf16*>(B);
    ph.ldb = ldb;
    ph.ktiles = K / BK;
    ph.a_src = a_src;
    ph.layer = layer;
    ph.kind = kind;
    ph.epilogue = epi;
    ph.step0 = steps;
    steps += ph.ktiles;
  };
  for (int l = 0; l <= L - 2; ++l) {
    const ParamSeg* w = p->weight_seg(l, 0);
    if (l == 0) {
      add(p->shadow + w->w_off, w->c_pad, p->k_pad, 1, l, 0, 1);
    } else if (l == s) {
      const ParamSeg* wy = p->weight_seg(l, 1);
      add(p->shadow + w->w_off, w->c_pad, H, 0, l, 0, 0);
      add(p->shadow + wy->w_off, wy->c_pad, p->k_pad, 1, l, 0, 1);
    } else {
      add(p->shadow + w->w_off, w->c_pad, H, 0, l, 0, 1);
    }
    a.bias[l] = p->params + p->bias_seg(l, 0)->off;
    a.YT[l] = p->W<bf16>(p->o_yt[l]);
    a.dZT[l] = p->W<bf16>(p->o_dZT[l]);
    a.colsum[l] = p->W<float>(p->o_colsum[l]);
  }
  a.bias_y = p->params + p->bias_seg(s, 1)->off;
  if (train) {
    for (int l = L - 2; l >= 1; --l) {
      const ParamSeg* w = p->weight_seg(l, 0);  // Lx at the skip layer
      add(p->shadow + w->wt_off, w->R, H, 0, l, 1, 1);
    }
  }
  a.nphase = np;
  a.nsteps = steps;
  a.W7 = p->params + p->weight_seg(L - 1, 0)->off;
  a.b7 = p->params + p->bias_seg(L - 1, 0)->off;
  a.hw_part = p->W<float>(p->o_hw);
  a.hb_part = p->W<float>(p->o_hb);
  a.ldt = Bp;
  a.pred = pred;
  a.ctrl = p->ctrl;
  a.loss_part = train ? p->W<double>(p->o_loss) : nullptr;
  a.hit = hit;
  a.pixel_map = pixel_map;
  a.img = img;
  a.dbg_ranges = p->dbg_ranges;
  a.dbg_nranges = p->dbg_n;
  a.dbg_out = p->dbg_out;
  a.stamps = p->stamps;
  a.stamp_steps = p->stamp_steps;
  a.train = train ? 1 : 0;
  a.save = train ? 1 : 0;
  a.count_step = train ? 1 : 0;
  if (train) {
    INF_CHECK_ARG(b->rgb != nullptr, "training batch without target colours");
    a.rgb = b->rgb;
    a.ray_idx = b->ray_idx;
    a.idx_dtype = b->idx_dtype;
    a.idx_offset = b->idx_offset;
    a.num_rays = b->num_rays;
    a.num_src = b->num_source_rays;
    a.offset_from_ctrl = b->offset_from_ctrl;
    a.loss = b->loss >= 0 ? b->loss : p->d.loss;
    INF_CHECK_ARG(a.loss >= INF_LOSS_L2 && a.loss <= INF_LOSS_CAUCHY, "loss type");
    const int64_t cnt = b->loss_count > 0 ? b->loss_count : (int64_t)3 * b->batch;
    a.inv_count = (float)(1.0 / (double)cnt);
  }
  return launch_chain(a, bm, st);
}

// The large-batch dW GEMM (fgemm.hip) for this padded batch: 64-ray chain tiles and every
// weight matrix a whole number of 256 x 256 tiles
bool use_fgemm(const inf_plan* p, int Bp, int splits) {
  // (the 16-ray chain's 4096-ray step on fgemm measured slower at every split count: 4 / 8 /
  // 16 splits -> step 86.3 / 80.1 / 81.5 vs 68.7 us on lgemm, profiles/r04/fgemm_narrow_sweep.log)
  if (!chain3_wide(Bp) || std::getenv("INF_NO_FGEMM") != nullptr) return false;
  for (const ParamSeg& g : p->segs)
    if (g.gemm && !fgemm_shape_ok(g.c_pad, g.R, Bp, splits)) return false;
  return true;
}

bool use_chain3(const inf_plan* p, const inf_batch* b, int Bp) {
  const ParamSeg* w1 = p->weight_seg(1, 0);
  const ParamSeg* w0 = p->weight_seg(0, 0);
  // the fused gather reads a device-resident bf16 table; the dW lgemm streams
  // K = Bp / dw_splits rays per block in 256-ray steps
  // (the gather addresses table rows with 64-bit offsets: any table size; the extrinsic
  // front-ends keep their encoded tile whole in LDS, in_dim <= C3_KC)
  return use_chain(p) && chain3_supported(p->H, p->L, p->k_pad, Bp) && w1 != nullptr && w1->f_off >= 0 &&
         w0->f_off >= 0 && b->table != nullptr &&
         (b->encoding == INF_ENC_NONE ? b->table_dtype == INF_DTYPE_BF16
                                      : (b->table_dtype == INF_DTYPE_F32 && b->vids != nullptr && p->k_pad <= C3_KC)) &&
         // the dW GEMM's split-K: lgemm streams K = Bp / dw_splits rays per block in 256-ray
         // steps, fgemm any multiple of 64 rays per split
         (use_fgemm(p, Bp, p->dw_splits) ||
          ((Bp / p->dw_splits) % 256 == 0 && Bp % p->dw_splits == 0)) &&
         std::getenv("INF_NO_CHAIN3") == nullptr;
}

// Fused gather + forward + loss + dX chain of a bf16 training batch (csrc/chain3.hip).
// Weight stream: layer 0 over X (k_pad / 32 k-blocks of W_0), the hidden layers (the skip
// layer as Lx over the activation tile then Ly over X), then the dX layers L-2..1.
// k_pad > C3_KC (config D): X is streamed in C3_KC-column chunks and phase 0 runs W_y then
// W_0 over each chunk (W_y x kept in the second accumulator set until the skip layer).

// The input layers on zg.hip ahead of the chain: the default for the chunked-tile tables
// (k_pad > C3_KC, config D: gather + input GEMM 26.5 us + the hidden-layer chain 31.9 us
// against the chunked chain's 83 us, whose 16-ray workgroups each stream 4 MB of W_0 / W_y;
// profiles/r05/zg/).  At config B it loses (16.1 + 31.1 us against 40 us: its 1 MB stream is
// cheaper than the Z slices' 32 MB round trip).  INF_ZG=0/1 forces it.
static bool use_zg(const inf_plan* p) {
  const char* e = std::getenv("INF_ZG");
  if (e != nullptr) return e[0] == '1';
  return p->k_pad > C3_KC;
}

int run_chain3(inf_plan* p, const inf_batch* b, int Bp, float* pred, hipStream_t st, const bf16* xpre = nullptr,
               bool x3 = false) {
  const int H = p->H, L = p->L, s = p->s;
  const int upl = H / 32;
  const int nx = p->k_pad / (32 * upl);  // stream blocks of X
  Chain3Args a;
  std::memset(&a, 0, sizeof(a));
  a.L = L;
  a.s = s;
  a.H = H;
  a.k_pad = p->k_pad;
  a.rows = Bp;
  a.batch = b->batch;
  if (b->encoding != INF_ENC_NONE) {
    INF_CHECK_ARG(b->table != nullptr && b->table_dtype == INF_DTYPE_F32 && b->vids != nullptr,
                  "chain3: encoded batches need the fp32 vertex table and vertex ids");
    a.encoding = b->encoding;
    a.enc_k = b->enc_k;
    a.enc_ne = b->encoding == INF_ENC_XYZ ? 0 : (b->encoding == INF_ENC_RFF ? b->enc_k : 3 * b->enc_k);
    a.enc_in_dim = encoded_dim(b->encoding, b->enc_k, b->enc_include_input);
    INF_CHECK_ARG(a.enc_in_dim == p->d.in_dim, "encoding width does not match the model's in_dim");
    a.enc_proj = b->enc_proj;
    a.pos = reinterpret_cast<const float*>(b->table);
  } else if (x3) {
    INF_CHECK_ARG(b->table != nullptr && b->table_dtype == INF_DTYPE_F32, "chain3 (split-bf16): fp32 table batch required");
    a.x3 = 1;
    a.table_f32 = reinterpret_cast<const float*>(b->table);
  } else {
    INF_CHECK_ARG(b->table != nullptr && b->table_dtype == INF_DTYPE_BF16, "chain3: bf16 table batch required");
    a.table = reinterpret_cast<const bf16*>(b->table);
  }
  a.num_vertices = b->num_vertices;
  a.vids = b->vids;
  a.vid_dtype = b->vid_dtype;
  a.bary = b->bary;
  INF_CHECK_ARG(b->rgb != nullptr, "training batch without target colours");
  a.rgb = b->rgb;
  a.ray_idx = b->ray_idx;
  a.idx_dtype = b->idx_dtype;
  a.idx_offset = b->idx_offset;
  a.num_rays = b->num_rays;
  a.num_src = b->num_source_rays;
  a.offset_from_ctrl = b->offset_from_ctrl;
  auto img = [&](const ParamSeg* w, bool fwd) -> const bf16* {
    const int64_t off = fwd ? w->f_off : w->ft_off;
    return off >= 0 ? reinterpret_cast<const bf16*>(p->shadow + off) : nullptr;
  };
  auto add = [&](const bf16* im, int kb0, int a_x, int ak0, int phase, int last) -> int {
    INF_CHECK_ARG(im != nullptr, "chain3: fragment image missing");
    INF_CHECK_ARG(a.nblk < C3_MAX_BLOCKS, "chain3: too many weight-stream blocks");
    C3Block& blk = a.blk[a.nblk++];
    blk.img = im;
    blk.kb0 = kb0;
    blk.a_x = a_x;
    blk.ak0 = ak0;
    blk.phase = phase;
    blk.last = last;
    return INF_OK;
  };
  int rc;
  const int kc = chain3_kc(p->k_pad, Bp);
  const bool xc = p->k_pad > kc;
  a.kc = kc;
  a.nchunk = (int)ceil_div(p->k_pad, a.kc);
  // zg.hip (use_zg: the default for k_pad > C3_KC, INF_ZG=1 forces it): the input layers
  // ahead of the chain, gather and GEMM in one launch (64 rays x all 2H features x a k slice
  // per workgroup, the slices added by the chain); the chain's stream keeps the hidden layers
  // only.  (Round 3 measured the same schedule as a separate gather + GEMM, igemm.hip, at
  // config B: the chain dropped 42.3 -> 29.4 us but gather 9.2 + GEMM 10.6 us cost more than
  // the 1 MB per-CU stream they replaced; removed in round 6)
  const int zg_s = zg_splits(p->k_pad, Bp);
  const bool zgp = p->o_zin >= 0 && b->encoding == INF_ENC_NONE && xpre == nullptr && chain3_bm(Bp) == 16 &&
                   zg_supported(H, p->k_pad, Bp) && zg_s <= p->zin_parts_max && use_zg(p);
  a.zin_parts = 1;
  p->last_zg = zgp;
  if (zgp) {
    ZgArgs g;
    std::memset(&g, 0, sizeof(g));
    g.table = a.table;
    g.num_vertices = b->num_vertices;
    g.k_pad = p->k_pad;
    g.H = H;
    g.vids = b->vids;
    g.vid_dtype = b->vid_dtype;
    g.bary = b->bary;
    g.ray_idx = b->ray_idx;
    g.idx_dtype = b->idx_dtype;
    g.idx_offset = b->idx_offset;
    g.num_rays = b->num_rays;
    g.num_src = b->num_source_rays;
    g.ctrl = p->ctrl;
    g.offset_from_ctrl = b->offset_from_ctrl;
    g.batch = b->batch;
    g.rows = Bp;
    g.splits = zg_s;
    g.gather_nt = (size_t)b->num_vertices * (size_t)p->k_pad * 2 > C3_NT_TABLE_BYTES;
    g.W0 = img(p->weight_seg(0, 0), true);
    g.Wy = img(p->weight_seg(s, 1), true);
    g.Z = p->W<float>(p->o_zin);
    g.z_stride = (int64_t)Bp * 2 * H;
    g.XT = p->W<bf16>(p->o_x0t);
    if ((rc = launch_zg(g, st))) return rc;
    a.zin = g.Z;
    a.zin_parts = zg_s;
    a.zin_stride = g.z_stride;
  } else if (!xc) {
    for (int i = 0; i < nx; ++i)
      if ((rc = add(img(p->weight_seg(0, 0), true), i * upl, 1, i * upl, 0, i == nx - 1))) return rc;
  } else {
    INF_CHECK_ARG(b->encoding == INF_ENC_NONE, "chain3: chunked feature tiles are eigenfunction tables only");
    for (int c = 0; c < a.nchunk; ++c) {
      const int nb = std::min(kc, p->k_pad - c * kc) / (32 * upl);  // stream blocks of the chunk
      const int kb = c * (kc / 32);
      for (int i = 0; i < nb; ++i) {
        if ((rc = add(img(p->weight_seg(s, 1), true), kb + i * upl, 1, i * upl, 0, 0))) return rc;
        if (i == 0) a.blk[a.nblk - 1].flags = C3F_SWAP | (c > 0 ? C3F_GATHER | (c << C3F_CHUNK_SHIFT) : 0);
      }
      for (int i = 0; i < nb; ++i) {
        if ((rc = add(img(p->weight_seg(0, 0), true), kb + i * upl, 1, i * upl, 0,
                      c == a.nchunk - 1 && i == nb - 1)))
          return rc;
        if (i == 0) a.blk[a.nblk - 1].flags = C3F_SWAP;
      }
    }
  }
  for (int l = 1; l <= L - 2; ++l) {
    if ((rc = add(img(p->weight_seg(l, 0), true), 0, 0, 0, l, xc || zgp || l != s))) return rc;
    if (l == s && !xc && !zgp)
      for (int i = 0; i < nx; ++i)
        if ((rc = add(img(p->weight_seg(s, 1), true), i * upl, 1, i * upl, l, i == nx - 1))) return rc;
  }
  for (int l = L - 2; l >= 1; --l)
    if ((rc = add(img(p->weight_seg(l, 0), false), 0, 0, 0, (L - 1) + (L - 2 - l), 1))) return rc;
  a.nphase = 2 * L - 3;
  for (int l = 0; l <= L - 2; ++l) {
    a.bias[l] = p->params + p->bias_seg(l, 0)->off;
    a.YT[l] = p->W<bf16>(p->o_yt[l]);
    a.dZT[l] = p->W<bf16>(p->o_dZT[l]);
    a.colsum[l] = p->W<float>(p->o_colsum[l]);
  }
  a.bias_y = p->params + p->bias_seg(s, 1)->off;
  a.W7 = p->params + p->weight_seg(L - 1, 0)->off;
  a.b7 = p->params + p->bias_seg(L - 1, 0)->off;
  a.XT = p->W<bf16>(p->o_x0t);
  a.hw_part = p->W<float>(p->o_hw);
  a.hb_part = p->W<float>(p->o_hb);
  a.loss_part = p->W<double>(p->o_loss);
  a.pred = pred;
  a.loss = b->loss >= 0 ? b->loss : p->d.loss;
  INF_CHECK_ARG(a.loss >= INF_LOSS_L2 && a.loss <= INF_LOSS_CAUCHY, "loss type");
  const int64_t cnt = b->loss_count > 0 ? b->loss_count : (int64_t)3 * b->batch;
  a.inv_count = (float)(1.0 / (double)cnt);
  a.ctrl = p->ctrl;
  a.count_step = 1;
  a.stamps = p->stamps;
  a.xpre = b->encoding == INF_ENC_NONE ? xpre : nullptr;
  return launch_chain3(a, chain3_bm(Bp), st);
}

// The fused step of the bf16x3 parity mode (chain3.hip X3): chain3's
// register-streamed schedule on bf16 matrix cores with every product split -- hi / lo bf16
// weight images (the update writes the pair), hi / lo feature and activation tiles, three
// MFMAs per k block -- from the fp32 table; the dW on lgemm SPLIT over the hi / lo X^T /
// Y^T / dZ^T images it writes.  16-ray tiles, k_pad <= 1024, batches lgemm's split-K tiles
// (Bp / dw_splits a multiple of 256); smaller batches take the layered split-bf16 kernels.
// INF_NO_CHAIN3X3=1: the layered kernels.
bool use_chain3x3(const inf_plan* p, const inf_batch* b, int Bp) {
  if (p->mode != INF_MODE_BF16X3 || p->k_pad > C3_KC || chain3_wide(Bp) ||
      !chain3_supported(p->H, p->L, p->k_pad, Bp) || !chain3_x3_lds_fits(p->H, p->L, p->k_pad))
    return false;
  if (b->table == nullptr || b->encoding != INF_ENC_NONE || b->table_dtype != INF_DTYPE_F32 || b->vids == nullptr ||
      b->rgb == nullptr || !use_split_lgemm(p, Bp))
    return false;
  for (int l = 0; l <= p->L - 2; ++l) {
    const ParamSeg* w = p->weight_seg(l, 0);
    if (w == nullptr || w->f_off < 0 || (l >= 1 && w->ft_off < 0)) return false;
  }
  const ParamSeg* wy = p->weight_seg(p->s, 1);
  return wy != nullptr && wy->f_off >= 0 && std::getenv("INF_NO_CHAIN3X3") == nullptr;
}

// The fused step of the fp32 parity mode (chainf.hip): eigenfunction tables up to k_pad =
// 1024, fp32 fragment images, a dW GEMM over 16-ray blocked operands (K = Bp split
// dw_splits ways in 32-ray k-tiles), exact-f32 throughout.  (The bf16x3 mode's images are hi /
// lo bf16 pairs since round 4: chain3 X3, above.)  INF_NO_CHAINF=1: the layered kernels.
bool use_chainf(const inf_plan* p, const inf_batch* b, int Bp) {
  if (p->mode != INF_MODE_FP32 || !chainf_supported(p->H, p->L, p->k_pad)) return false;
  if (b->table == nullptr || b->encoding != INF_ENC_NONE || b->table_dtype != INF_DTYPE_F32 || b->vids == nullptr ||
      b->rgb == nullptr)
    return false;
  if (b->num_vertices >= ((int64_t)1 << 31) || Bp % 16 != 0 || (Bp / 32) % p->dw_splits != 0) return false;
  for (int l = 0; l <= p->L - 2; ++l) {
    const ParamSeg* w = p->weight_seg(l, 0);
    if (w == nullptr || w->f_off < 0 || (l >= 1 && w->ft_off < 0)) return false;
  }
  const ParamSeg* wy = p->weight_seg(p->s, 1);
  return wy != nullptr && wy->f_off >= 0 && std::getenv("INF_NO_CHAINF") == nullptr;
}

// Fused gather + forward + loss + dX chain of an fp32 training batch (csrc/chainf.hip).
// Weight stream as chain3's unchunked schedule: W_0 over X, the hidden layers (the skip
// layer as Lx over the activation tile then Ly over X), then the dX layers L-2..1.
int run_chainf(inf_plan* p, const inf_batch* b, int Bp, float* pred, hipStream_t st) {
  const int H = p->H, L = p->L, s = p->s;
  const int upl = H / 32;
  const int nx = p->k_pad / (32 * upl);
  ChainFArgs a;
  std::memset(&a, 0, sizeof(a));
  a.L = L;
  a.s = s;
  a.H = H;
  a.k_pad = p->k_pad;
  a.rows = Bp;
  a.batch = b->batch;
  a.table = reinterpret_cast<const float*>(b->table);
  a.num_vertices = b->num_vertices;
  a.vids = b->vids;
  a.vid_dtype = b->vid_dtype;
  a.bary = b->bary;
  a.rgb = b->rgb;
  a.ray_idx = b->ray_idx;
  a.idx_dtype = b->idx_dtype;
  a.idx_offset = b->idx_offset;
  a.num_rays = b->num_rays;
  a.num_src = b->num_source_rays;
  a.offset_from_ctrl = b->offset_from_ctrl;
  auto img = [&](const ParamSeg* w, bool fwd) -> const float* {
    const int64_t off = fwd ? w->f_off : w->ft_off;
    return off >= 0 ? reinterpret_cast<const float*>(p->shadow + off) : nullptr;
  };
  auto add = [&](const float* im, int kb0, int a_x, int ak0, int phase, int last) -> int {
    INF_CHECK_ARG(im != nullptr, "chainf: fragment image missing");
    INF_CHECK_ARG(a.nblk < C3_MAX_BLOCKS, "chainf: too many weight-stream blocks");
    CFBlock& blk = a.blk[a.nblk++];
    blk.img = im;
    blk.kb0 = kb0;
    blk.a_x = a_x;
    blk.ak0 = ak0;
    blk.phase = phase;
    blk.last = last;
    return INF_OK;
  };
  int rc;
  for (int i = 0; i < nx; ++i)
    if ((rc = add(img(p->weight_seg(0, 0), true), i * upl, 1, i * upl, 0, i == nx - 1))) return rc;
  for (int l = 1; l <= L - 2; ++l) {
    if ((rc = add(img(p->weight_seg(l, 0), true), 0, 0, 0, l, l != s))) return rc;
    if (l == s)
      for (int i = 0; i < nx; ++i)
        if ((rc = add(img(p->weight_seg(s, 1), true), i * upl, 1, i * upl, l, i == nx - 1))) return rc;
  }
  for (int l = L - 2; l >= 1; --l)
    if ((rc = add(img(p->weight_seg(l, 0), false), 0, 0, 0, (L - 1) + (L - 2 - l), 1))) return rc;
  a.nphase = 2 * L - 3;
  for (int l = 0; l <= L - 2; ++l) {
    a.bias[l] = p->params + p->bias_seg(l, 0)->off;
    a.YT[l] = p->W<float>(p->o_yt[l]);
    a.dZT[l] = p->W<float>(p->o_dZT[l]);
    a.colsum[l] = p->W<float>(p->o_colsum[l]);
  }
  a.bias_y = p->params + p->bias_seg(s, 1)->off;
  a.W7 = p->params + p->weight_seg(L - 1, 0)->off;
  a.b7 = p->params + p->bias_seg(L - 1, 0)->off;
  a.XT = p->W<float>(p->o_x0t);
  a.hw_part = p->W<float>(p->o_hw);
  a.hb_part = p->W<float>(p->o_hb);
  a.loss_part = p->W<double>(p->o_loss);
  a.pred = pred;
  a.loss = b->loss >= 0 ? b->loss : p->d.loss;
  INF_CHECK_ARG(a.loss >= INF_LOSS_L2 && a.loss <= INF_LOSS_CAUCHY, "loss type");
  const int64_t cnt = b->loss_count > 0 ? b->loss_count : (int64_t)3 * b->batch;
  a.inv_count = (float)(1.0 / (double)cnt);
  a.ctrl = p->ctrl;
  a.count_step = 1;
  a.split_images = use_split_lgemm(p, Bp) ? 1 : 0;
  return launch_chainf(a, st);
}

bool use_rchain(const inf_plan* p, const inf_batch* b) {
  const ParamSeg* w0 = p->weight_seg(0, 0);
  const ParamSeg* wy = p->weight_seg(p->s, 1);
  if (!use_chain(p) || !rchain_supported(p->H, p->L, p->k_pad) || w0->f_off < 0 || wy->f_off < 0) return false;
  for (int l = 1; l <= p->L - 2; ++l)
    if (p->weight_seg(l, 0)->f_off < 0) return false;
  if (b->encoding == INF_ENC_PROJECTED) return b->table != nullptr && b->table_dtype == INF_DTYPE_BF16 && b->vids != nullptr;
  return b->table != nullptr && b->encoding == INF_ENC_NONE && b->table_dtype == INF_DTYPE_BF16 &&
         b->vids != nullptr && !b->offset_from_ctrl && std::getenv("INF_NO_RCHAIN") == nullptr;
}

// Forward-only register-streamed chain (csrc/rchain.hip): gather + every layer + head +
// placement in one launch.  Weight stream: per RC_KC-column feature chunk the W_y then
// the W_0 k-blocks (W_y x in the second accumulator set), then one block per hidden layer.
int run_rchain(inf_plan* p, const inf_batch* b, float* pred, const int64_t* hit, const int64_t* pixel_map,
               float* img, hipStream_t st) {
  const int H = p->H, L = p->L, s = p->s;
  const int upl = H / 32;
  RchainArgs a;
  std::memset(&a, 0, sizeof(a));
  a.L = L;
  a.s = s;
  a.H = H;
  a.k_pad = p->k_pad;
  a.batch = b->batch;
  a.table = reinterpret_cast<const bf16*>(b->table);
  a.num_vertices = b->num_vertices;
  a.vids = b->vids;
  a.vid_dtype = b->vid_dtype;
  a.bary = b->bary;
  a.ray_idx = b->ray_idx;
  a.idx_dtype = b->idx_dtype;
  a.idx_offset = b->idx_offset;
  a.num_rays = b->num_rays;
  a.num_src = b->num_source_rays;
  a.nchunk = (int)ceil_div(p->k_pad, RC_KC);
  auto add = [&](const ParamSeg* w, int kb0, int a_x, int ak0, int phase, int last, int flags) -> int {
    INF_CHECK_ARG(w != nullptr && w->f_off >= 0, "rchain: fragment image missing");
    INF_CHECK_ARG(a.nblk < RC_MAX_BLOCKS, "rchain: too many weight-stream blocks");
    C3Block& blk = a.blk[a.nblk++];
    blk.img = reinterpret_cast<const bf16*>(p->shadow + w->f_off);
    blk.kb0 = kb0;
    blk.a_x = a_x;
    blk.ak0 = ak0;
    blk.phase = phase;
    blk.last = last;
    blk.flags = flags;
    return INF_OK;
  };
  int rc;
  if (b->encoding == INF_ENC_PROJECTED) {
    // projected table (inf_project_table, rproj.hip): no feature chunks, the hidden layers
    a.projected = 1;
    a.nchunk = 0;
  }
  for (int c = 0; c < a.nchunk; ++c) {
    const int nb = std::min(RC_KC, p->k_pad - c * RC_KC) / (32 * upl);
    const int kb = c * (RC_KC / 32);
    for (int i = 0; i < nb; ++i)
      if ((rc = add(p->weight_seg(s, 1), kb + i * upl, 1, i * upl, 0, 0,
                    i == 0 ? C3F_SWAP | (c > 0 ? C3F_GATHER | (c << C3F_CHUNK_SHIFT) : 0) : 0)))
        return rc;
    for (int i = 0; i < nb; ++i)
      if ((rc = add(p->weight_seg(0, 0), kb + i * upl, 1, i * upl, 0, c == a.nchunk - 1 && i == nb - 1,
                    i == 0 ? C3F_SWAP : 0)))
        return rc;
  }
  for (int l = 1; l <= L - 2; ++l)
    if ((rc = add(p->weight_seg(l, 0), 0, 0, 0, l, 1, 0))) return rc;
  a.nphase = L - 1;
  for (int l = 0; l <= L - 2; ++l) a.bias[l] = p->params + p->bias_seg(l, 0)->off;
  a.bias_y = p->params + p->bias_seg(s, 1)->off;
  a.W7 = p->params + p->weight_seg(L - 1, 0)->off;
  a.b7 = p->params + p->bias_seg(L - 1, 0)->off;
  a.pred = pred;
  a.hit = hit;
  a.pixel_map = pixel_map;
  a.img = img;
  a.stamps = p->stamps;
  return launch_rchain(a, st);
}

int forward_impl(inf_plan* p, const inf_batch* b, float* pred, bool save, bool loss, const int64_t* hit,
                 const int64_t* pixel_map, float* img, hipStream_t st) {
  INF_CHECK_ARG(b != nullptr, "null batch");
  int rc;
  if (b->encoding == INF_ENC_PROJECTED) {
    // no workspace: any number of rays per call (a whole frame in one persistent launch)
    INF_CHECK_ARG(b->batch >= 1, "empty batch");
    INF_CHECK_ARG(b->offset_from_ctrl == 0, "projected batches take an explicit offset");
    if (save || loss || !use_rchain(p, b)) {
      set_error("projected tables feed the forward-only register chain (bf16 plan, inference) only");
      return INF_ERR_UNSUPPORTED;
    }
    if ((rc = run_rchain(p, b, pred, hit, pixel_map, img, st))) return rc;
    p->saved = false;
    return INF_OK;
  }
  int Bp = 0;
  if ((rc = pad_batch(p, b->batch, save, &Bp))) return rc;
  if (!save && !loss && use_rchain(p, b)) {
    if ((rc = run_rchain(p, b, pred, hit, pixel_map, img, st))) return rc;
    p->saved = false;
    return INF_OK;
  }
  if ((rc = run_input(p, b, Bp, save, st))) return rc;
  if (!save && use_chain(p)) {
    if ((rc = run_chain(p, b, Bp, false, pred, hit, pixel_map, img, st))) return rc;
    p->saved = false;
    return INF_OK;
  }
  if ((rc = run_forward_layers(p, Bp, save, st))) return rc;
  float* pred_ws = p->W<float>(p->o_pred);
  if ((rc = head_forward(p, b, Bp, save ? pred_ws : pred, loss, hit, pixel_map, img, st))) return rc;
  if (save && pred != nullptr && pred != pred_ws)
    INF_HIP_TRY(hipMemcpyAsync(pred, pred_ws, (size_t)b->batch * 3 * 4, hipMemcpyDeviceToDevice, st));
  p->saved = save;
  p->saved_batch = b->batch;
  p->saved_bp = Bp;
  return INF_OK;
}

}  // namespace

// =================================================================================
extern "C" {

const char* inf_last_error(void) { return g_last_error.c_str(); }
int inf_abi_version(void) { return 3; }  // 3: double lr / Adam constants, inf_ctrl 56 bytes

int inf_gather(const void* table, int table_dtype, int64_t num_vertices, int k, int64_t table_ld, const void* vids,
               int vid_dtype, const float* bary, const void* ray_idx, int idx_dtype, int64_t idx_offset, int batch,
               int64_t num_source_rays, void* out, int out_dtype, int64_t ld_out, int rows_out, void* out_t,
               int64_t ld_out_t, inf_stream_t stream) {
  return launch_gather(table, table_dtype, num_vertices, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype,
                       idx_offset, nullptr, 0, num_source_rays, batch, out, out_dtype, ld_out, rows_out, out_t, ld_out_t,
                       (hipStream_t)stream);
}

int inf_encode(const float* table, int64_t num_rows, const void* vids, int vid_dtype, const float* bary,
               const void* ray_idx, int idx_dtype, int64_t idx_offset, int batch, int64_t num_source_rays,
               int encoding, int enc_k, const float* enc_proj, int include_input, void* out, int out_dtype,
               int64_t ld_out, int rows_out, inf_stream_t stream) {
  return launch_encode(table, num_rows, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset, nullptr, 0,
                       num_source_rays, batch,
                       encoding, enc_k, enc_proj, include_input, out, out_dtype, ld_out, rows_out, nullptr, 0,
                       (hipStream_t)stream);
}

int inf_encoded_dim(int encoding, int enc_k, int include_input) {
  return encoded_dim(encoding, enc_k, include_input);
}

int inf_plan_create(const inf_mlp_desc* desc, int max_batch, inf_plan** plan) {
  INF_CHECK_ARG(desc != nullptr && plan != nullptr, "null argument");
  const inf_mlp_desc& d = *desc;
  INF_CHECK_ARG(d.num_layers > 2 && d.skip > 0 && d.skip < d.num_layers - 1,
                "need num_layers > 2 and 0 < skip_layer_idx < num_layers-1 (model.py:27)");
  INF_CHECK_ARG(d.in_dim >= 1, "in_dim must be positive");
  INF_CHECK_ARG(d.hidden >= 64 && d.hidden % 64 == 0 && d.hidden <= 512,
                "mlp_hidden_dim must be a multiple of 64 in [64, 512]");
  INF_CHECK_ARG(d.out_dim == 3, "out_dim must be 3 (RGB head)");
  INF_CHECK_ARG(d.mode == INF_MODE_FP32 || d.mode == INF_MODE_BF16 || d.mode == INF_MODE_BF16X3, "mode");
  INF_CHECK_ARG(d.loss >= INF_LOSS_L2 && d.loss <= INF_LOSS_CAUCHY, "loss type");
  INF_CHECK_ARG(max_batch >= 1, "max_batch");
  inf_plan* p = new inf_plan();
  p->d = d;
  p->max_batch = max_batch;
  int rc = build_layout(p);
  if (rc) {
    delete p;
    return rc;
  }
  *plan = p;
  return INF_OK;
}

void inf_plan_destroy(inf_plan* plan) { delete plan; }

int inf_plan_get_info(const inf_plan* p, inf_plan_info* info) {
  INF_CHECK_ARG(p != nullptr && info != nullptr, "null argument");
  info->num_params = p->P;
  info->num_segments = (int32_t)p->segs.size();
  info->in_pad = p->k_pad;
  info->max_batch_pad = p->bp_max;
  info->dw_splits = p->dw_splits;
  info->shadow_bytes = p->shadow_bytes;
  info->workspace_bytes = p->o_ws_end;
  info->table_ld = p->k_pad;
  return INF_OK;
}

int inf_plan_param_layout(const inf_plan* p, int64_t* offsets, int64_t* numels, int n) {
  INF_CHECK_ARG(p != nullptr && offsets != nullptr && numels != nullptr, "null argument");
  INF_CHECK_ARG(n == (int)p->segs.size(), "segment count mismatch");
  for (int i = 0; i < n; ++i) {
    offsets[i] = p->segs[i].off;
    numels[i] = (int64_t)p->segs[i].R * p->segs[i].C;
  }
  return INF_OK;
}

// The item subset the fused dW + update reads (lgemm.hip): the vector and end-of-step
// items its leading blocks run.  A copy of p->adam_items: re-uploaded
// whenever those change (bind, and inf_plan_shard's staging offsets goff / woff, which the
// fused update's SHARD_GRAD_OUT items write through).
static int upload_item_subsets(inf_plan* p) {
  std::vector<AdamItem> aux;
  for (const auto& it : p->adam_items)
    if (it.seg < 0 || !p->adam_segs[it.seg].matrix) aux.push_back(it);
  p->n_aux_items = (int)aux.size();
  INF_HIP_TRY(hipMemcpy(p->ws + p->o_aux_items, aux.data(), aux.size() * sizeof(AdamItem), hipMemcpyHostToDevice));
  return INF_OK;
}

int inf_plan_bind(inf_plan* p, float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* shadow,
                  void* workspace, inf_ctrl* ctrl) {
  INF_CHECK_ARG(p != nullptr && params != nullptr && shadow != nullptr && workspace != nullptr && ctrl != nullptr,
                "bind: params, shadow, workspace and ctrl are required");
  INF_CHECK_ARG(((uintptr_t)shadow % 256) == 0 && ((uintptr_t)workspace % 256) == 0,
                "bind: shadow/workspace must be 256-byte aligned");
  p->params = params;
  p->grads = grads;
  p->exp_avg = exp_avg;
  p->exp_avg_sq = exp_avg_sq;
  p->shadow = (char*)shadow;
  p->ws = (char*)workspace;
  p->ctrl = ctrl;

  // update work list (a shard layout of an earlier bind is gone with it)
  INF_CHECK_ARG(p->sharded_state == 0, "bind: the optimizer state is sharded (gather it first)");
  p->shard_world = 0;
  p->sh_gsh = p->sh_gshard = nullptr;
  p->sh_wsh = nullptr;
  p->adam_segs.clear();
  p->adam_items.clear();
  const int L = p->L;
  for (size_t i = 0; i < p->segs.size(); ++i) {
    const ParamSeg& g = p->segs[i];
    AdamSeg a;
    std::memset(&a, 0, sizeof(a));
    a.off = g.off;
    if (g.gemm) {
      a.R = g.R;
      a.C = g.C;
      a.matrix = 1;
      a.nslab = p->dw_splits;
      a.slab = p->W<float>(p->o_slab[i]);
      a.slab_stride = (int64_t)g.R * g.c_pad;
      a.slab_ld = g.c_pad;
      a.W = p->shadow + g.w_off;
      a.ldw = g.c_pad;
      a.WT = p->shadow + g.wt_off;
      a.ldwt = g.R;
      a.WF = g.f_off >= 0 ? p->shadow + g.f_off : nullptr;
      a.WTF = g.ft_off >= 0 ? p->shadow + g.ft_off : nullptr;
      a.wf_acc_order = g.ft_off >= 0 ? 1 : 0;  // hidden layers: fed by the activation tile
      a.x3 = p->mode == INF_MODE_BF16X3 ? 1 : 0;  // images as hi / lo bf16 pairs (chain3 X3)
      const int flags = (g.C % 4 == 0 && g.off % 4 == 0) ? ITEM_VEC4 : 0;
      for (int r = 0; r < g.R; r += ADAM_TILE_R)
        for (int c = 0; c < g.C; c += ADAM_TILE_C) p->adam_items.push_back(AdamItem{(int32_t)i, r, c, flags});
    } else {
      a.R = 1;
      a.C = g.R * g.C;
      a.matrix = 0;
      if (g.layer == L - 1) {  // output layer: partials from head_bwd
        a.nslab = p->grid_hb;
        a.slab = g.kind == 0 ? p->W<float>(p->o_hw) : p->W<float>(p->o_hb);
        a.slab_stride = (int64_t)g.R * g.C;
      } else {  // hidden bias: column-sum partials of dZ_layer
        a.nslab = g.layer == L - 2 ? p->grid_hb : p->bp_max / 64;
        a.slab = p->W<float>(p->o_colsum[g.layer]);
        a.slab_stride = p->H;
      }
      for (int e = 0; e < a.C; e += ADAM_VEC) p->adam_items.push_back(AdamItem{(int32_t)i, 0, e, 0});
    }
    p->adam_segs.push_back(a);
  }
  p->adam_items.push_back(AdamItem{-1, 0, 0, 0});  // end-of-step: loss sums, batch advance
  // gradient buckets of the data-parallel step: bucket 1 = the arena from the skip layer's
  // Ly weight on (its items listed first, with the end-of-step item), bucket 2 = the rest
  const ParamSeg* ly = p->weight_seg(p->s, 1);
  p->grad_split = ly != nullptr ? ly->off : 0;
  std::stable_partition(p->adam_items.begin(), p->adam_items.end(), [&](const AdamItem& it) {
    return it.seg < 0 || p->segs[it.seg].off >= p->grad_split;
  });
  p->n_items_b1 = 0;
  for (const auto& it : p->adam_items)
    if (it.seg < 0 || p->segs[it.seg].off >= p->grad_split) ++p->n_items_b1;
  // each matrix's first item (stable_partition kept a segment's items contiguous and in order)
  for (int i = (int)p->adam_items.size() - 1; i >= 0; --i)
    if (p->adam_items[i].seg >= 0) p->adam_segs[p->adam_items[i].seg].item0 = i;
  const int64_t seg_bytes = align_up(p->adam_segs.size() * sizeof(AdamSeg));
  INF_CHECK_ARG(seg_bytes + (int64_t)(p->adam_items.size() * sizeof(AdamItem)) <= p->table_bytes, "table size");
  INF_HIP_TRY(hipMemcpy(p->ws + p->o_tables, p->adam_segs.data(), p->adam_segs.size() * sizeof(AdamSeg),
                        hipMemcpyHostToDevice));
  INF_HIP_TRY(hipMemcpy(p->ws + p->o_tables + seg_bytes, p->adam_items.data(),
                        p->adam_items.size() * sizeof(AdamItem), hipMemcpyHostToDevice));
  {
    const std::vector<AdamSeg> tb = bucket_segs(p);
    INF_HIP_TRY(hipMemcpy(p->ws + p->o_tables_b, tb.data(), tb.size() * sizeof(AdamSeg), hipMemcpyHostToDevice));
  }
  if (int rc = upload_item_subsets(p)) return rc;
  // padded shadow columns/rows must read as zero
  INF_HIP_TRY(hipMemset(p->shadow, 0, p->shadow_bytes));
  p->bound = true;
  p->saved = false;
  return INF_OK;
}

int inf_plan_set_adam(inf_plan* p, double beta1, double beta2, double eps) {
  INF_CHECK_ARG(p != nullptr, "null plan");
  INF_CHECK_ARG(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0, "Adam hyper-parameters");
  p->beta1 = beta1;
  p->beta2 = beta2;
  p->eps = eps;
  return INF_OK;
}

int inf_sync_shadow(inf_plan* p, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->bound, "plan not bound");
  if (int rc = check_unsharded(p, "sync_shadow")) return rc;
  AdamArgs a = update_args(p, p->bp_max);
  a.grad_src = GRAD_NONE;
  a.write_shadow = 1;
  const int rc = launch_update(a, p->mode, (hipStream_t)stream);
  if (rc == INF_OK) note_shadow_write(p, a, (hipStream_t)stream);
  return rc;
}

int inf_forward(inf_plan* p, const inf_batch* batch, float* pred, int save, inf_stream_t stream) {
  if (p == nullptr || !p->bound) {
    set_error("plan not bound");
    return INF_ERR_STATE;
  }
  INF_CHECK_ARG(pred != nullptr, "forward: pred output required");
  return forward_impl(p, batch, pred, save != 0, false, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

int inf_backward(inf_plan* p, const float* dpred, float* grads, inf_stream_t stream) {
  if (p == nullptr || !p->bound || !p->saved) {
    set_error("backward without a saved forward");
    return INF_ERR_STATE;
  }
  INF_CHECK_ARG(dpred != nullptr && grads != nullptr, "backward: dpred and grads required");
  hipStream_t st = (hipStream_t)stream;
  const int Bp = p->saved_bp;
  int rc;
  if ((rc = head_backward(p, Bp, dpred, false, st))) return rc;
  if ((rc = run_backward_layers(p, Bp, st))) return rc;
  if ((rc = refresh_tables(p, Bp, st))) return rc;
  AdamArgs a = update_args(p, Bp);
  a.grads = grads;
  a.grad_src = GRAD_SLABS;
  a.write_grads = 1;
  return launch_update(a, p->mode, st);
}

int inf_train_step(inf_plan* p, const inf_batch* batch, float* pred, int flags, inf_stream_t stream) {
  if (p == nullptr || !p->bound) {
    set_error("plan not bound");
    return INF_ERR_STATE;
  }
  const bool apply_adam = (flags & INF_STEP_ADAM) != 0;
  INF_CHECK_ARG((flags & ~(INF_STEP_ADAM | INF_STEP_ADVANCE | INF_STEP_XSLOT0 | INF_STEP_XSLOT1 | INF_STEP_PART1 |
                           INF_STEP_PART2 | INF_STEP_SHARD)) == 0,
                "train_step: unknown flags");
  const bool shard = (flags & INF_STEP_SHARD) != 0;
  INF_CHECK_ARG(!shard || ((flags & (INF_STEP_ADAM | INF_STEP_PART1 | INF_STEP_PART2)) == 0 && p->sh_gsh != nullptr),
                "train_step: INF_STEP_SHARD is a gradient-only step of a plan with bound shard buffers "
                "(not with ADAM / PART1 / PART2)");
  if (flags & INF_STEP_ADAM) {
    if (int rc = check_unsharded(p, "train_step with Adam")) return rc;
  }
  const int part = (flags & INF_STEP_PART1) ? 1 : (flags & INF_STEP_PART2) ? 2 : 0;
  INF_CHECK_ARG(part == 0 || (!apply_adam && (flags & INF_STEP_ADVANCE) == 0 && !((flags & INF_STEP_PART1) &&
                                                                                  (flags & INF_STEP_PART2))),
                "train_step: PART1 / PART2 are gradient-only halves of one step");
  const int xslot = (flags & INF_STEP_XSLOT0) ? 0 : (flags & INF_STEP_XSLOT1) ? 1 : -1;
  INF_CHECK_ARG(batch != nullptr && batch->rgb != nullptr, "train_step: batch with target colours required");
  if (batch->encoding == INF_ENC_PROJECTED) {
    set_error("train_step: projected tables are forward-only");
    return INF_ERR_UNSUPPORTED;
  }
  INF_CHECK_ARG(p->grads != nullptr || apply_adam, "train_step: grads not bound");
  INF_CHECK_ARG(!apply_adam || (p->exp_avg != nullptr && p->exp_avg_sq != nullptr), "train_step: Adam state");
  hipStream_t st = (hipStream_t)stream;
  int rc;
  const bool chain = use_chain(p);
  int nloss = 0;
  int ck = 0;
  int Bp3 = 0;
  if ((rc = pad_batch(p, batch->batch, true, &Bp3))) return rc;
  // bucketed halves of a gradient-only step (fused chain3 path): PART1 = the fused chain,
  // the dW GEMM of bucket 1's matrices and the reduction of bucket 1 -- the arena range
  // [grad_split, P): the matrices and biases from the skip layer's Ly on, plus the step's
  // loss sums -- into `grads`; PART2 = the same for bucket 2, the arena [0, grad_split)
  // (the earlier layers' biases included).  The caller all-reduces bucket 1 while PART2 runs.
  const bool bucketed = part != 0 && use_chain3(p, batch, Bp3) && Bp3 % (256 * p->bucket_splits) == 0;
  if (part == 1) p->last_part1 = bucketed ? 1 : 0;
  if (shard && !use_chain3(p, batch, Bp3) && !use_chainf(p, batch, Bp3) && !use_chain3x3(p, batch, Bp3)) {
    // the other paths read the row-major shadows, rewritten from the fp32 masters, which a
    // sharded update leaves current on this rank's items only
    set_error("train_step: INF_STEP_SHARD needs the fused chain (chain3 / chainf) for this batch");
    return INF_ERR_UNSUPPORTED;
  }
  if (part == 2 && !bucketed) return INF_OK;  // PART1 reduced the whole gradient
  if (part == 2) {
    INF_CHECK_ARG(p->stepped && p->last_chain == 3 && p->saved_bp == Bp3, "train_step: PART2 without its PART1");
    if ((rc = run_weight_grads(p, Bp3, st, 3, nullptr, 2))) return rc;
    AdamArgs a = update_args(p, Bp3);
    a.segs = p->W<AdamSeg>(p->o_tables_b);
    a.items += p->n_items_b1;
    a.num_items -= p->n_items_b1;
    a.grad_src = GRAD_SLABS;
    a.write_grads = 1;
    return launch_update(a, p->mode, st);
  }
  // the update launch's arguments for a step whose gradient partials are complete
  auto step_update = [&](int Bp_, int nloss_) {
    AdamArgs a = update_args(p, Bp_);
    a.grad_src = GRAD_SLABS;
    if (apply_adam) {
      a.do_adam = 1;
      a.write_shadow = step_shadow_mode(p, ck);
    } else {
      a.write_grads = 1;
      if (shard) {  // the reduced local gradient into the item-major staging (reduce-scatter input)
        a.shard_mode = SHARD_GRAD_OUT;
        a.gsh = p->sh_gsh;
        a.g_base = 0;
      }
    }
    a.loss_part = p->W<double>(p->o_loss);
    a.nloss = nloss_;
    a.advance = (flags & INF_STEP_ADVANCE) ? 1 : 0;
    return a;
  };
  if (use_chain3(p, batch, Bp3)) {
    // fused gather + chain -> dW GEMM (-> update below, or inside the dW launch: lgf)
    const int Bp = Bp3;
    const bf16* xpre = nullptr;
    if (xslot >= 0) {
      INF_CHECK_ARG(p->o_xp[xslot] >= 0 && batch->encoding == INF_ENC_NONE, "train_step: no pre-gather slot");
      xpre = p->W<bf16>(p->o_xp[xslot]);
    }
    if ((rc = run_chain3(p, batch, Bp, pred, st, xpre))) return rc;
    p->saved = false;
    p->saved_batch = batch->batch;
    p->saved_bp = Bp;
    ck = 3;
    nloss = Bp / chain3_bm(Bp);
    p->stepped = true;
    p->last_lgf = false;
    if (!bucketed && p->lgf) {
      // the update inside the dW launch (split-K 1: each block its own tile from LDS)
      p->last_chain = 3;
      p->last_lgf = p->lgf;
      if ((rc = refresh_tables(p, Bp, st, 3))) return rc;
      const AdamArgs a = step_update(Bp, nloss);
      if ((rc = run_weight_grads(p, Bp, st, 3, &a))) return rc;
      note_shadow_write(p, a, st);
      return INF_OK;
    }
    if (bucketed) {  // PART1
      p->last_chain = 3;
      if ((rc = run_weight_grads(p, Bp, st, 3, nullptr, 1))) return rc;
      if ((rc = refresh_tables(p, Bp, st, 3))) return rc;
      AdamArgs a = step_update(Bp, nloss);
      a.segs = p->W<AdamSeg>(p->o_tables_b);
      a.num_items = p->n_items_b1;
      return launch_update(a, p->mode, st);
    }
    if ((rc = run_weight_grads(p, Bp, st, 3))) return rc;
  } else if (use_chain3x3(p, batch, Bp3)) {
    // bf16x3 mode: fused gather + split-bf16 chain -> split-operand dW (-> update below)
    const int Bp = Bp3;
    if ((rc = run_chain3(p, batch, Bp, pred, st, nullptr, true))) return rc;
    if ((rc = run_weight_grads(p, Bp, st, CHAIN_X3))) return rc;
    p->saved = false;
    p->saved_batch = batch->batch;
    p->saved_bp = Bp;
    ck = CHAIN_X3;
    nloss = Bp / 16;
  } else if (use_chainf(p, batch, Bp3)) {
    // fp32 mode: fused gather + chain (exact f32 MFMA) -> dW GEMM over its blocked
    // operands (-> update below); the chain leaves per-workgroup loss partials
    const int Bp = Bp3;
    if ((rc = run_chainf(p, batch, Bp, pred, st))) return rc;
    if ((rc = run_weight_grads(p, Bp, st, CHAIN_F32))) return rc;
    p->saved = false;
    p->saved_batch = batch->batch;
    p->saved_bp = Bp;
    ck = CHAIN_F32;
    nloss = Bp / 16;
  } else if (chain) {
    // the chain leaves per-tile loss partials; the update launch stores their sum
    int Bp = 0;
    if ((rc = pad_batch(p, batch->batch, true, &Bp))) return rc;
    if ((rc = run_input(p, batch, Bp, true, st))) return rc;
    if ((rc = run_chain(p, batch, Bp, true, pred, nullptr, nullptr, nullptr, st))) return rc;
    if ((rc = run_weight_grads(p, Bp, st, true))) return rc;
    p->saved = false;
    p->saved_batch = batch->batch;
    p->saved_bp = Bp;
    ck = 2;
    nloss = Bp / chain_bm(Bp);
  } else {
    // the layered head accumulates the step's sums with atomics: clear them first
    INF_HIP_TRY(hipMemsetAsync(&p->ctrl->loss_sum, 0, 2 * sizeof(double), st));
    if ((rc = forward_impl(p, batch, pred, true, true, nullptr, nullptr, nullptr, st))) return rc;
    const int Bp0 = p->saved_bp;
    if ((rc = head_backward(p, Bp0, nullptr, true, st))) return rc;
    if ((rc = run_backward_layers(p, Bp0, st))) return rc;
  }
  p->last_chain = ck;
  p->stepped = true;
  const int Bp = p->saved_bp;
  if ((rc = refresh_tables(p, Bp, st, ck))) return rc;
  const AdamArgs ua = step_update(Bp, nloss);
  if ((rc = launch_update(ua, p->mode, st))) return rc;
  note_shadow_write(p, ua, st);
  return INF_OK;
}

int inf_adam(inf_plan* p, int step, double lr, inf_stream_t stream) { return inf_adam_ex(p, step, lr, 0, stream); }

int inf_adam_ex(inf_plan* p, int step, double lr, int flags, inf_stream_t stream) {
  INF_CHECK_ARG((flags & ~INF_STEP_ADVANCE) == 0, "adam: unknown flags");
  if (p == nullptr || !p->bound || p->grads == nullptr || p->exp_avg == nullptr || p->exp_avg_sq == nullptr) {
    set_error("adam: plan not bound with grads and Adam state");
    return INF_ERR_STATE;
  }
  if (int rc = check_unsharded(p, "adam")) return rc;
  AdamArgs a = update_args(p, p->bp_max);
  a.grad_src = GRAD_FLAT;
  a.do_adam = 1;
  a.write_shadow = 1;
  a.step_host = step;
  a.lr_host = lr;
  if (step > 0) {  // torch's 1 - beta ** step (Python double pow), as inf_adam_dense
    a.bc1_host = 1.0 - std::pow(p->beta1, (double)step);
    a.bc2_host = 1.0 - std::pow(p->beta2, (double)step);
  }
  a.advance = (flags & INF_STEP_ADVANCE) ? 1 : 0;
  // after a fused chain3 step (the data-parallel tail) only the fragment images
  a.write_shadow = step_shadow_mode(p, p->last_chain);
  const int rc = launch_update(a, p->mode, (hipStream_t)stream);
  if (rc == INF_OK) note_shadow_write(p, a, (hipStream_t)stream);
  return rc;
}

// ---- sharded update (data parallel): reduce-scatter -> Adam on 1/world of the items ->
// all-gather of the new weights in the GEMM dtype -> every rank rewrites the images ----

int inf_plan_shard(inf_plan* p, int world, int rank, int64_t* grad_floats, int64_t* weight_bytes) {
  INF_CHECK_ARG(p != nullptr && p->bound, "shard: plan not bound");
  INF_CHECK_ARG(world >= 1 && rank >= 0 && rank < world && grad_floats != nullptr && weight_bytes != nullptr,
                "shard: world >= 1, 0 <= rank < world");
  if (int rc = check_unsharded(p, "shard")) return rc;
  const int64_t wsz = p->mode == INF_MODE_BF16 ? 2 : 4;  // the update's image dtype (launch_update)
  auto pay_g = [&](const AdamItem& it) -> int64_t {
    if (it.seg < 0) return 0;
    return p->adam_segs[it.seg].matrix ? ADAM_TILE_R * ADAM_TILE_C : ADAM_VEC;
  };
  auto pay_w = [&](const AdamItem& it) -> int64_t {
    if (it.seg < 0) return 0;
    return p->adam_segs[it.seg].matrix ? ADAM_TILE_R * ADAM_TILE_C * wsz : ADAM_VEC * 4;
  };
  int64_t total = 0;
  for (const auto& it : p->adam_items) total += pay_g(it);
  // contiguous groups of the item list, cut where the running gradient size passes r / world
  // of the total; each rank's chunk is the largest group rounded up (256-byte aligned)
  std::vector<int> group(p->adam_items.size());
  std::vector<int64_t> gsz(world, 0), wszr(world, 0);
  int64_t run = 0;
  int r = 0;
  for (size_t i = 0; i < p->adam_items.size(); ++i) {
    const AdamItem& it = p->adam_items[i];
    while (r + 1 < world && run >= (total * (r + 1) + world - 1) / world) ++r;
    group[i] = it.seg < 0 ? -1 : r;
    if (it.seg >= 0) {
      gsz[r] += pay_g(it);
      wszr[r] += pay_w(it);
      run += pay_g(it);
    }
  }
  int64_t Sg = 0, Sw = 0;
  for (int q = 0; q < world; ++q) {
    Sg = std::max(Sg, gsz[q]);
    Sw = std::max(Sw, wszr[q]);
  }
  Sg = round_up(std::max<int64_t>(Sg, 64), 64);
  Sw = round_up(std::max<int64_t>(Sw, 256), 256);
  INF_CHECK_ARG(Sg * world < (1ll << 31) && Sw * world < (1ll << 31), "shard: staging offsets exceed 32 bits");
  std::vector<int64_t> lg(world, 0), lw(world, 0);
  std::vector<AdamItem> own;
  AdamItem end_item{-1, 0, 0, 0, 0, 0};
  for (size_t i = 0; i < p->adam_items.size(); ++i) {
    AdamItem& it = p->adam_items[i];
    if (group[i] < 0) {
      it.goff = it.woff = 0;
      end_item = it;
      continue;
    }
    const int q = group[i];
    it.goff = (int32_t)(q * Sg + lg[q]);
    it.woff = (int32_t)(q * Sw + lw[q]);
    lg[q] += pay_g(it);
    lw[q] += pay_w(it);
    if (q == rank) own.push_back(it);
  }
  own.push_back(end_item);  // the end-of-step item: the batch advance of a replayed epoch
  const int64_t seg_bytes = align_up(p->adam_segs.size() * sizeof(AdamSeg));
  INF_HIP_TRY(hipMemcpy(p->ws + p->o_tables + seg_bytes, p->adam_items.data(),
                        p->adam_items.size() * sizeof(AdamItem), hipMemcpyHostToDevice));
  if (int rc = upload_item_subsets(p)) return rc;  // the fused dW + update's copies carry goff too
  INF_HIP_TRY(hipMemcpy(p->ws + p->o_shard_items, own.data(), own.size() * sizeof(AdamItem), hipMemcpyHostToDevice));
  p->n_shard_items = (int)own.size();
  p->shard_world = world;
  p->shard_rank = rank;
  p->shard_g = Sg;
  p->shard_w = Sw;
  p->sh_gsh = p->sh_gshard = nullptr;
  p->sh_wsh = nullptr;
  *grad_floats = Sg;
  *weight_bytes = Sw;
  return INF_OK;
}

int inf_plan_can_shard(inf_plan* p, const inf_batch* batch) {
  if (p == nullptr || !p->bound || batch == nullptr || batch->rgb == nullptr || batch->encoding == INF_ENC_PROJECTED)
    return 0;
  int Bp3 = 0;
  if (pad_batch(p, batch->batch, true, &Bp3) != INF_OK) return 0;
  return use_chain3(p, batch, Bp3) || use_chainf(p, batch, Bp3) || use_chain3x3(p, batch, Bp3) ? 1 : 0;
}

int inf_plan_bind_shard(inf_plan* p, float* grad_staging, float* grad_chunk, void* weight_staging) {
  INF_CHECK_ARG(p != nullptr && p->shard_world > 0, "bind_shard: inf_plan_shard first");
  INF_CHECK_ARG(grad_staging != nullptr && grad_chunk != nullptr && weight_staging != nullptr,
                "bind_shard: three staging buffers required");
  INF_CHECK_ARG(((uintptr_t)grad_staging % 16) == 0 && ((uintptr_t)grad_chunk % 16) == 0 &&
                    ((uintptr_t)weight_staging % 16) == 0,
                "bind_shard: staging buffers must be 16-byte aligned");
  p->sh_gsh = grad_staging;
  p->sh_gshard = grad_chunk;
  p->sh_wsh = (char*)weight_staging;
  // slots past an item's elements are never written: they must read as zero
  INF_HIP_TRY(hipMemset(grad_staging, 0, (size_t)(p->shard_g * p->shard_world * 4)));
  INF_HIP_TRY(hipMemset(grad_chunk, 0, (size_t)(p->shard_g * 4)));
  INF_HIP_TRY(hipMemset(weight_staging, 0, (size_t)(p->shard_w * p->shard_world)));
  return INF_OK;
}

int inf_adam_shard(inf_plan* p, int flags, inf_stream_t stream) {
  INF_CHECK_ARG((flags & ~INF_STEP_ADVANCE) == 0, "adam_shard: unknown flags");
  INF_CHECK_ARG(p != nullptr && p->bound && p->sh_gsh != nullptr && p->exp_avg != nullptr && p->exp_avg_sq != nullptr,
                "adam_shard: plan with Adam state and bound shard buffers required");
  AdamArgs a = update_args(p, p->bp_max);
  a.items = p->W<AdamItem>(p->o_shard_items);
  a.num_items = p->n_shard_items;
  a.grad_src = GRAD_FLAT;
  a.shard_mode = SHARD_ADAM;
  a.gsh = p->sh_gshard;
  a.g_base = (int64_t)p->shard_rank * p->shard_g;
  a.wsh = p->sh_wsh;
  a.w_base = 0;
  a.do_adam = 1;
  a.write_shadow = 2;  // this rank's images now; the row-major shadows wait for the gathered masters
  a.advance = (flags & INF_STEP_ADVANCE) ? 1 : 0;
  const int rc = launch_update(a, p->mode, (hipStream_t)stream);
  if (rc == INF_OK) {
    note_shadow_write(p, a, (hipStream_t)stream);
    p->sharded_state = 7;
  }
  return rc;
}

int inf_shard_scatter(inf_plan* p, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->bound && p->sh_wsh != nullptr, "shard_scatter: bound shard buffers required");
  AdamArgs a = update_args(p, p->bp_max);
  a.grad_src = GRAD_NONE;
  a.shard_mode = SHARD_SCATTER;
  a.wsh = p->sh_wsh;
  a.w_base = 0;
  a.write_shadow = 2;
  const int rc = launch_update(a, p->mode, (hipStream_t)stream);
  if (rc == INF_OK) note_shadow_write(p, a, (hipStream_t)stream);
  return rc;
}

int inf_shard_pack(inf_plan* p, const float* arena, float* chunk, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->bound && p->shard_world > 0 && arena != nullptr && chunk != nullptr,
                "shard_pack: plan with a shard layout, arena and chunk required");
  return launch_shard_copy(p->W<AdamSeg>(p->o_tables), p->W<AdamItem>(p->o_shard_items), p->n_shard_items, arena,
                           chunk, (int64_t)p->shard_rank * p->shard_g, 0, (hipStream_t)stream);
}

int inf_shard_unpack(inf_plan* p, const float* staging, float* arena, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->bound && p->shard_world > 0 && arena != nullptr && staging != nullptr,
                "shard_unpack: plan with a shard layout, staging and arena required");
  const int64_t seg_bytes = align_up(p->adam_segs.size() * sizeof(AdamSeg));
  const int rc = launch_shard_copy(p->W<AdamSeg>(p->o_tables), reinterpret_cast<const AdamItem*>(p->ws + p->o_tables + seg_bytes),
                                   (int)p->adam_items.size(), staging, arena, 0, 1, (hipStream_t)stream);
  if (rc == INF_OK) {
    if (arena == p->params) p->sharded_state &= ~1;
    if (arena == p->exp_avg) p->sharded_state &= ~2;
    if (arena == p->exp_avg_sq) p->sharded_state &= ~4;
  }
  return rc;
}

int inf_render(inf_plan* p, const inf_batch* batch, const int64_t* hit, const int64_t* pixel_map, float* img,
               inf_stream_t stream) {
  if (p == nullptr || !p->bound) {
    set_error("plan not bound");
    return INF_ERR_STATE;
  }
  INF_CHECK_ARG(hit != nullptr && img != nullptr, "render: hit indices and image required");
  return forward_impl(p, batch, nullptr, false, false, hit, pixel_map, img, (hipStream_t)stream);
}

int64_t inf_projected_rows(int64_t num_vertices) { return num_vertices <= 0 ? 0 : round_up(num_vertices, 128); }

// out[v] = (W_0 E[v], W_y E[v]) in bf16: one plain NT GEMM over the packed table (A = E
// [V][k_pad], B = [W_0; W_y] [2H][k_pad] bf16, C = out [.][2H]) by the hand-written
// 256 x 256-tile GEMM of ptab.hip (2H a multiple of 256); INF_PROJECT_GEMM=blaslt takes
// hipBLASLt instead (and so does a 2H ptab.hip cannot tile), INF_PROJECT_GEMM=own the
// plan's grouped GEMM in 2^24-row slices, the last partial 128-row tile staged through X0
// (the GEMM reads whole tiles; out has inf_projected_rows(V) rows, so its stores stay in
// bounds).
int inf_project_table(inf_plan* p, const void* table, int64_t num_vertices, void* out, inf_stream_t stream) {
  if (p == nullptr || !p->bound) {
    set_error("plan not bound");
    return INF_ERR_STATE;
  }
  INF_CHECK_ARG(table != nullptr && out != nullptr && num_vertices >= 1, "project_table: table and output required");
  if (p->mode != INF_MODE_BF16 || p->weight_seg(p->s, 1) == nullptr) {
    set_error("project_table: bf16 plans with the input skip layer only");
    return INF_ERR_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  const int H = p->H, k_pad = p->k_pad;
  const ParamSeg* w[2] = {p->weight_seg(0, 0), p->weight_seg(p->s, 1)};
  INF_CHECK_ARG(p->o_pcat >= 0 && w[0]->c_pad == k_pad && w[1]->c_pad == k_pad, "project_table: weight layout");
  if (int rc = ensure_rowmajor(p, st)) return rc;  // W_0 / W_y rows below
  char* pcat = p->shadow + p->o_pcat;
  const size_t wbytes = (size_t)H * k_pad * 2;
  for (int h = 0; h < 2; ++h)
    INF_HIP_TRY(hipMemcpyAsync(pcat + h * wbytes, p->shadow + w[h]->w_off, wbytes, hipMemcpyDeviceToDevice, st));
  const char* gsel = std::getenv("INF_PROJECT_GEMM");
  const std::string sel = gsel != nullptr ? gsel : "";
  if (sel.empty() && (2 * H) % 256 == 0)  // ptab.hip: any row count, rows past V untouched
    return launch_proj_gemm(reinterpret_cast<const bf16*>(table), num_vertices, k_pad,
                            reinterpret_cast<const bf16*>(pcat), 2 * H, k_pad, reinterpret_cast<bf16*>(out), 2 * H, st);
  const bool own = sel == "own";
  if (!own)  // hipBLASLt: any row count, rows past V untouched
    return blaslt_gemm_nt_bf16(table, k_pad, pcat, k_pad, out, 2 * H, num_vertices, 2 * H, k_pad, st);
  const int64_t full = num_vertices / 128 * 128, tail = num_vertices - full;
  const size_t row_bytes = (size_t)k_pad * 2;
  if (tail > 0) {
    INF_CHECK_ARG(p->bp_max >= 128, "project_table: staging tile");
    char* x0 = p->W(p->o_x0);
    INF_HIP_TRY(hipMemsetAsync(x0 + tail * row_bytes, 0, (size_t)(128 - tail) * row_bytes, st));
    INF_HIP_TRY(hipMemcpyAsync(x0, (const char*)table + full * row_bytes, (size_t)tail * row_bytes,
                               hipMemcpyDeviceToDevice, st));
  }
  // the GEMM's M is a 32-bit row count: the full tiles in slices of 2^24 rows
  constexpr int64_t SLICE = (int64_t)1 << 24;
  GemmBatch gb;
  std::memset(&gb, 0, sizeof(gb));
  auto flush = [&]() -> int {
    if (gb.nprob == 0) return INF_OK;
    const int rc = launch_gemm(gb, p->mode, TILE_128x128, st);
    std::memset(&gb, 0, sizeof(gb));
    return rc;
  };
  auto add = [&](const void* A, int64_t rows, int64_t r0) -> int {
    if (gb.nprob + 1 > GEMM_MAX_PROBLEMS)
      if (int rc = flush()) return rc;
    GemmProblem& q = gb.p[gb.nprob++];
    q = blank_problem();
    q.A[0] = A;
    q.lda[0] = k_pad;
    q.B[0] = pcat;
    q.ldb[0] = k_pad;
    q.K[0] = k_pad;
    q.M = (int32_t)rows;
    q.N = 2 * H;
    q.C = reinterpret_cast<char*>(out) + r0 * 2 * H * 2;
    q.ldc = 2 * H;
    return INF_OK;
  };
  int rc;
  for (int64_t m0 = 0; m0 < full; m0 += SLICE)
    if ((rc = add((const char*)table + m0 * row_bytes, std::min(SLICE, full - m0), m0))) return rc;
  if (tail > 0 && (rc = add(p->W(p->o_x0), 128, full))) return rc;
  if ((rc = flush())) return rc;
  p->saved = false;  // X0 held the staged tail
  return INF_OK;
}

int inf_run_stage(inf_plan* p, const inf_batch* b, int stage, int layer, double* flops, double* bytes,
                  inf_stream_t stream) {
  if (p == nullptr || !p->bound || !(p->saved || p->last_chain)) {
    set_error("run_stage needs a saved training step");
    return INF_ERR_STATE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int Bp = p->saved_bp;
  const double B = p->saved_batch, H = p->H, k = p->d.in_dim;
  const double e = (double)p->esz;
  double f = 0, by = 0;
  int rc = INF_OK;
  switch (stage) {
    case INF_STAGE_GATHER:
      INF_CHECK_ARG(b != nullptr && b->table != nullptr, "gather stage needs the ray batch");
      rc = run_input(p, b, Bp, true, st);
      f = 6.0 * B * k;
      // three table rows per ray + ids/bary; outputs X and X^T
      by = B * (3.0 * k * (b->table_dtype == INF_DTYPE_BF16 ? 2 : 4) + 24.0) + 2.0 * B * p->k_pad * e;
      break;
    case INF_STAGE_FWD_GEMM: {
      INF_CHECK_ARG(layer >= 1 && layer <= p->L - 2, "forward stage layer must be a hidden layer");
      if ((rc = ensure_rowmajor(p, st))) return rc;
      rc = run_forward_layer(p, Bp, true, layer, st);
      const double K = (layer == p->s) ? H + k : H;
      f = 2.0 * B * H * K;
      by = B * (K + 2.0 * H) * e;
      break;
    }
    case INF_STAGE_DW_GEMM: {
      if (p->last_lgf) {  // the step's fused dW + update launch (Adam, lr from ctrl: parameters change)
        if ((rc = refresh_tables(p, Bp, st, 3))) return rc;
        AdamArgs a = update_args(p, Bp);
        a.grad_src = GRAD_SLABS;
        a.do_adam = 1;
        a.write_shadow = step_shadow_mode(p, 3);
        rc = run_weight_grads(p, Bp, st, 3, &a);
        if (rc == INF_OK) note_shadow_write(p, a, st);
        for (const auto& g : p->segs)
          if (g.gemm) {
            f += 2.0 * g.R * g.C * B;
            by += (double)B * (g.R + g.C) * e;
          }
        break;
      }
      rc = run_weight_grads(p, Bp, st, p->last_chain);
      for (const auto& g : p->segs)
        if (g.gemm) {
          f += 2.0 * g.R * g.C * B;
          by += (double)B * (g.R + g.C) * e + 4.0 * g.R * g.C * p->dw_splits;
        }
      break;
    }
    case INF_STAGE_CHAIN: {
      INF_CHECK_ARG(b != nullptr && b->rgb != nullptr &&
                        (use_chain(p) || p->last_chain == CHAIN_F32 || p->last_chain == CHAIN_X3),
                    "chain stage needs a fused training batch");
      // replay on the saved inputs; the step counter it advances is restored by the caller
      const double Lh = p->L;
      if (p->last_chain == CHAIN_F32) {
        rc = run_chainf(p, b, Bp, nullptr, st);
        f = 2.0 * B * (2.0 * k * H + (Lh - 2) * H * H + 3 * H) + 2.0 * B * ((Lh - 2) * H * H + 3 * H);
        // fp32 weight images streamed per workgroup (L2 -> CU); rows in; blocked operands out
        by = (double)(Bp / 16) * (2.0 * p->k_pad * H + 2.0 * (Lh - 2) * H * H) * 4.0 +
             B * (3.0 * p->k_pad * 4.0 + 24.0) + B * (p->k_pad + (2.0 * Lh - 3) * H) * 4.0;
      } else if (p->last_chain == CHAIN_X3) {
        rc = run_chain3(p, b, Bp, nullptr, st, nullptr, true);
        // algorithmic FLOPs (the MFMAs issued are three times these: bench.py prices the
        // mode against a third of the bf16 peak)
        f = 2.0 * B * (2.0 * k * H + (Lh - 2) * H * H + 3 * H) + 2.0 * B * ((Lh - 2) * H * H + 3 * H);
        // hi / lo bf16 weight images streamed per workgroup; fp32 rows in; hi / lo images out
        by = (double)(Bp / 16) * (2.0 * p->k_pad * H + 2.0 * (Lh - 2) * H * H) * 4.0 +
             B * (3.0 * p->k_pad * 4.0 + 24.0) + B * (p->k_pad + (2.0 * Lh - 3) * H) * 4.0;
      } else if (p->last_chain == 3) {
        rc = run_chain3(p, b, Bp, nullptr, st);
        f = 2.0 * B * (2.0 * k * H + (Lh - 2) * H * H + 3 * H) + 2.0 * B * ((Lh - 2) * H * H + 3 * H);
        // every workgroup streams W_0, W_y and the hidden weights twice over (L2 -> CU);
        // three table rows per ray in; X^T, Y^T, dZ^T out
        by = (double)(Bp / chain3_bm(Bp)) * (2.0 * p->k_pad * H + 2.0 * (Lh - 2) * H * H) * e +
             B * (3.0 * p->k_pad * e + 24.0) + B * (p->k_pad + (2.0 * Lh - 3) * H) * e;
      } else {
        rc = run_chain(p, b, Bp, true, nullptr, nullptr, nullptr, nullptr, st);
        f = 2.0 * B * (2.0 * k * H + (Lh - 2) * H * H + 3 * H) + 2.0 * B * ((Lh - 2) * H * H + 3 * H);
        by = B * (2.0 * p->k_pad * e + 2.0 * (Lh - 1) * H * e) + 2.0 * 4 * p->P;
      }
      break;
    }
    case INF_STAGE_UPDATE: {
      if ((rc = refresh_tables(p, Bp, st, p->last_chain))) return rc;
      AdamArgs a = update_args(p, Bp);
      a.grad_src = GRAD_SLABS;
      if (layer == 1) {
        // the step's update as launched by inf_train_step: Adam and the weight images
        // (parameters change; lr from ctrl)
        a.do_adam = 1;
        a.write_shadow = step_shadow_mode(p, p->last_chain);
      } else {
        INF_CHECK_ARG(p->grads != nullptr, "update stage needs a bound grads arena");
        a.write_grads = 1;  // reduce only into the grads arena: parameters unchanged
      }
      rc = launch_update(a, p->mode, st);
      if (rc == INF_OK) note_shadow_write(p, a, st);
      const int nimg_rm = a.write_shadow == 2 ? 0 : 2;  // W, W^T
      for (const auto& g : p->segs) {
        const double n = (double)g.R * g.C;
        by += 4.0 * n * (g.gemm ? p->dw_splits : 1) + 4.0 * n;  // partials in, gradient out
        if (layer == 1) by += 20.0 * n + (g.gemm ? 2.0 * n * ((g.ft_off >= 0 ? 2 : 1) + nimg_rm) : 0.0);
      }
      break;
    }
    default:
      INF_CHECK_ARG(false, "unknown stage");
  }
  if (flops) *flops = f;
  if (bytes) *bytes = by;
  return rc;
}

int inf_debug_ranges(inf_plan* p, const uint64_t* ranges, int n, unsigned long long* out) {
  INF_CHECK_ARG(p != nullptr && n >= 0, "debug ranges");
  p->dbg_ranges = ranges;
  p->dbg_n = n;
  p->dbg_out = out;
  return INF_OK;
}

int inf_debug_block_times(inf_plan* p, unsigned long long* stamps) {
  INF_CHECK_ARG(p != nullptr, "debug block times");
  p->lg_stamps = stamps;
  return INF_OK;
}

int inf_debug_timing(inf_plan* p, unsigned long long* stamps, int max_steps) {
  INF_CHECK_ARG(p != nullptr && max_steps >= 0, "debug timing");
  p->stamps = stamps;
  p->stamp_steps = max_steps;
  return INF_OK;
}

int inf_prefetch_batch(inf_plan* p, const inf_batch* b, int slot, inf_stream_t stream) {
  if (p == nullptr || !p->bound) {
    set_error("plan not bound");
    return INF_ERR_STATE;
  }
  INF_CHECK_ARG(b != nullptr && (slot == 0 || slot == 1), "prefetch: batch and slot 0 / 1 required");
  int Bp = 0;
  int rc = pad_batch(p, b->batch, true, &Bp);
  if (rc) return rc;
  if (p->o_xp[slot] < 0 || b->encoding != INF_ENC_NONE || !use_chain3(p, b, Bp)) {
    set_error("prefetch: this batch's step does not run the fused chain");
    return INF_ERR_STATE;
  }
  hipStream_t st = (hipStream_t)stream;
  if ((rc = launch_gather(b->table, b->table_dtype, b->num_vertices, p->k_pad, p->k_pad, b->vids, b->vid_dtype,
                          b->bary, b->ray_idx, b->idx_dtype, b->idx_offset,
                          b->offset_from_ctrl ? &p->ctrl->prefetch_index : nullptr, b->num_rays,
                          b->num_source_rays, b->batch,
                          p->W(p->o_xp[slot]), INF_DTYPE_BF16, p->k_pad, Bp, nullptr, 0, st)))
    return rc;
  if (b->offset_from_ctrl) {
    prefetch_advance_kernel<<<1, 1, 0, st>>>(p->ctrl);
    INF_LAUNCH_CHECK();
  }
  return INF_OK;
}

int64_t inf_plan_grad_split(const inf_plan* p) { return p == nullptr ? -1 : p->grad_split; }

int inf_plan_last_part1_bucketed(const inf_plan* p) { return p == nullptr ? -1 : p->last_part1; }

int inf_plan_last_step_fused_update(const inf_plan* p) { return p == nullptr || !p->stepped ? -1 : (p->last_lgf ? 1 : 0); }

int inf_debug_buffer(inf_plan* p, int which, void* dst, int64_t* bytes, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->bound && bytes != nullptr, "debug_buffer: bound plan");
  const char* src = nullptr;
  int64_t n = 0;
  if (which == 0) {
    src = p->ws + p->o_x0t;
    n = (int64_t)p->k_pad * p->bp_max * p->esz;
  } else {
    const int i = which >= 100 ? which - 101 : which - 1;
    INF_CHECK_ARG(i >= 0 && i < (int)p->segs.size(), "debug_buffer: segment index");
    const ParamSeg& g = p->segs[i];
    const int64_t off = which >= 100 ? g.ft_off : g.f_off;
    if (off >= 0) {
      src = p->shadow + off;
      n = which >= 100 ? (int64_t)p->H * p->H * p->esz : (int64_t)g.R * g.c_pad * p->esz;
    }
  }
  if (dst != nullptr && n > 0) {
    INF_CHECK_ARG(*bytes >= n, "debug_buffer: destination too small");
    INF_HIP_TRY(hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  }
  *bytes = n;
  return INF_OK;
}

int inf_plan_last_step_path(const inf_plan* p) {
  if (p == nullptr || !p->stepped) return -1;
  if (p->last_chain == 3 && p->last_zg) return 10;
  if (p->last_chain == 3 && chain3_wide(p->saved_bp)) return 5;
  return p->last_chain == 3 && p->k_pad > C3_KC ? 4 : p->last_chain;
}

int64_t inf_plan_weight_generation(const inf_plan* p) {
  if (p == nullptr) return -1;
  return p->gen_captured ? -1 : p->weight_gen;
}

int inf_ctrl_advance(inf_plan* p, inf_stream_t stream) {
  INF_CHECK_ARG(p != nullptr && p->ctrl != nullptr, "plan not bound");
  ctrl_advance_kernel<<<1, 1, 0, (hipStream_t)stream>>>(p->ctrl);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // extern "C"
