// Fused per-ray-tile MLP chain (bf16 perf mode), see chain.hip.
#pragma once

#include <cstdlib>

#include "common.hpp"

namespace inf {

constexpr int CHAIN_MAX_HIDDEN = 12;  // hidden layers (num_layers - 1)
constexpr int CHAIN_MAX_PHASES = 2 * CHAIN_MAX_HIDDEN + 2;

// One phase = one K segment of one layer: C += A * B^T with A = the LDS activation tile
// (a_src 0) or the streamed feature tile X (a_src 1), B = streamed packed weights.
struct ChainPhase {
  const bf16* B;     // [H rows][ldb] bf16, K-contiguous
  int32_t ldb;
  int32_t ktiles;    // K / BK
  int32_t a_src;     // 0: activation tile in LDS, 1: X rows from global
  int32_t layer;     // layer index (forward) / layer whose dX this is (backward)
  int32_t kind;      // 0: forward segment, 1: backward (dX) segment
  int32_t epilogue;  // 1: last segment of the layer -> run its epilogue
  int32_t step0;     // first flat step index of the phase
};

struct ChainArgs {
  int32_t L, s, H, k_pad;
  int32_t rows, batch;
  const bf16* X;                  // [rows][k_pad] gathered features
  ChainPhase ph[CHAIN_MAX_PHASES];
  int32_t nphase, nsteps;
  const float* bias[CHAIN_MAX_HIDDEN];
  const float* bias_y;            // skip layer: Ly.bias (added after Lx.bias)
  const float* W7;                // [3][H] fp32 output layer
  const float* b7;
  bf16* YT[CHAIN_MAX_HIDDEN];     // [H][ldt] forward activations, transposed
  bf16* dZT[CHAIN_MAX_HIDDEN];    // [H][ldt] pre-activation grads, transposed
  float* colsum[CHAIN_MAX_HIDDEN];// [rows/64][H] bias-grad partials
  float* hw_part;                 // [rows/64][3][H]
  float* hb_part;                 // [rows/64][3]
  int64_t ldt;
  // head / loss / placement
  float* pred;
  const float* rgb;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;  // bound on idx_offset + b (0 = unchecked), inf_batch::num_rays
  int64_t num_src;   // rows of vids / bary / rgb (inf_batch::num_source_rays; 0 = unchecked)
  int32_t offset_from_ctrl;
  int32_t loss;
  float inv_count;
  inf_ctrl* ctrl;
  double* loss_part;              // [rows/BM][2] per-tile loss / SSE sums (train)
  const int64_t* hit;
  const int64_t* pixel_map;
  float* img;
  int32_t train;       // loss + backward chain
  int32_t save;        // write YT
  int32_t count_step;  // ctrl->step += 1
  // debug builds (-DINF_CHAIN_DEBUG): every global access is checked against these
  // [lo, hi) byte ranges; violations are counted and recorded in dbg_out, never issued
  const uint64_t* dbg_ranges;
  int32_t dbg_nranges;
  unsigned long long* dbg_out;  // [0] count, then (site, address) pairs
  // diagnostics (any build): per-step wall-clock stamps of the first and last workgroup
  unsigned long long* stamps;
  int32_t stamp_steps;
};

// Supported hidden widths of the fused chain (others use the layered path).
inline bool chain_supported(int H) { return H == 128 || H == 256; }
// Ray-tile height for a padded batch: about one workgroup per CU while the batch is
// small (every workgroup streams all weights, so more tiles = more CUs streaming), then
// taller tiles that do more MFMA work per streamed weight byte.
inline int chain_bm(int64_t rows) {
  if (const char* e = std::getenv("INF_CHAIN_BM")) {  // tuning: 64 or 128 (partials stay per 64 rays)
    const int v = std::atoi(e);
    if ((v == 64 || v == 128) && rows % v == 0 && rows > 16384) return v;
  }
  if (rows <= 4096) return 16;
  if (rows <= 8192) return 32;
  if (rows <= 16384) return 64;
  return 128;
}
inline int chain_bk(int bm) { return bm >= 64 ? 32 : 64; }
// Rays per bias-gradient / output-layer partial written by the chain.
inline int chain_partial_rows(int bm) { return bm >= 64 ? 64 : bm; }
// Upper bound on the chain's partial count for padded batches up to bp_max.
inline int64_t chain_max_partials(int64_t bp_max) { return bp_max / 64 > 256 ? bp_max / 64 : 256; }

int launch_chain(const ChainArgs& a, int bm, hipStream_t stream);

}  // namespace inf
