// Register-streamed fused training chain for small bf16 batches, see chain3.hip.
#pragma once

#include "chain.hpp"

#include <cstdlib>

namespace inf {

constexpr int C3_MAX_PHASES = 2 * CHAIN_MAX_HIDDEN;
constexpr int C3_MAX_BLOCKS = 64;

// One block of the weight stream = UPL k-blocks of 32 (one hidden layer's K).  The A
// operand of a block is the activation tile (a_x = 0) or the gathered feature tile X
// (a_x = 1) from its 32-k block ak0 on; B is a fragment image (adam.hip WF / WTF) from
// its k-block kb0 on.  `last`: the block ends phase `phase` (run its epilogue).
// `flags` (chunked feature tile only, Chain3Args::kc < k_pad): C3F_SWAP exchanges the
// layer-0 and Ly accumulators before the block; C3F_GATHER gathers feature chunk
// flags >> C3F_CHUNK_SHIFT into the LDS tile first (both input layers stream over each
// chunk once, so the table rows are read once per step).
constexpr int C3F_SWAP = 1, C3F_GATHER = 2, C3F_CHUNK_SHIFT = 8;
struct C3Block {
  const bf16* img;
  int32_t kb0;
  int32_t a_x;
  int32_t ak0;
  int32_t phase;
  int32_t last;
  int32_t flags;
};

struct Chain3Args {
  int32_t L, s, H, k_pad;
  int32_t rows, batch;
  // rays: the barycentric gather (mesh.py:313-324) with the loader's index select
  // (ray_dataloader.py:122-129), fused: feature rows never leave the CU
  const bf16* table;  // [V][k_pad] bf16, zero columns past k
  int64_t num_vertices;
  const void* vids;
  int32_t vid_dtype;
  const float* bary;
  const float* rgb;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;  // bound on idx_offset + b (0 = unchecked)
  int64_t num_src;   // rows of vids / bary / rgb (inf_batch::num_source_rays; 0 = unchecked)
  int32_t offset_from_ctrl;
  // extrinsic front-end (INF_ENC_*, model.py:33-40): the feature tile is the encoding of
  // the rays' interpolated positions pos[V][3] (gather.hip encode_kernel's numerics)
  int32_t encoding, enc_k, enc_ne, enc_in_dim;
  const float* enc_proj;
  const float* pos;
  // feature columns held in LDS at a time (chain3_kc): k_pad (whole tile) or C3_KC (chunked,
  // k_pad > C3_KC: config D's k = 4096 tile is 128 KiB for 16 rays, above the LDS budget);
  // C3_KC_WIDE for the 64-ray tiles
  int32_t kc, nchunk;
  int32_t table_big;  // table of 4 GiB or more: 64-bit row addresses (set by launch_chain3)
  int32_t gather_nt;  // table rows read non-temporally: tables above the MALL (set by launch_chain3)
  // pre-gathered features (inf_prefetch_batch): row b of xpre [rows][k_pad] bf16 is ray b's
  // feature row, read instead of gathering three table rows (null: gather)
  const bf16* xpre;
  // split-bf16 parity mode (INF_MODE_BF16X3): every weight image is a hi /
  // lo pair of bf16 images (lo right after hi: k block kb of lo = k block kb + kblocks of
  // the image), the feature and activation tiles hold hi / lo pairs, and each k block runs
  // three MFMAs (lo.hi + hi.lo + hi.hi); the table is fp32 (table_f32) and the X^T / Y^T /
  // dZ^T outputs are hi / lo image pairs for lgemm's SPLIT dW (lo image at + features x rows)
  int32_t x3;
  const float* table_f32;
  // precomputed input layers (zg.hip): Z = [W_0; W_y] X^T without biases, fp32, in the
  // accumulator layout ([rows / 16][2H / 16] KiB); X^T already written (null: the kernel
  // gathers and streams W_0 / W_y itself)
  const float* zin;
  // ... as zin_parts slices at zin + s zin_stride (zg.hip's k slices), added in order s = 0, 1, ..
  int32_t zin_parts;
  int64_t zin_stride;
  // weight stream: phases 0..L-2 forward layer p, L-1.. dX of layer (L-2) - (p - (L-1))
  C3Block blk[C3_MAX_BLOCKS];
  int32_t nblk, nphase;
  const float* bias[CHAIN_MAX_HIDDEN];  // layer l bias (Lx.bias at the skip layer)
  const float* bias_y;                   // Ly.bias
  const float* W7;                       // [3][H] fp32 output layer
  const float* b7;
  // outputs for the weight-gradient GEMM (lgemm.hip) and the update launch
  // fragment images (lgemm.hpp: rows = features, k = rays; 1 KiB per 16 features x 32 rays)
  bf16* XT;                        // X^T, k_pad rows
  bf16* YT[CHAIN_MAX_HIDDEN];      // Y_l^T, H rows, l = 0..L-3 (lgemm operand A)
  bf16* dZT[CHAIN_MAX_HIDDEN];     // dZ_l^T, H rows, l = 0..L-2 (lgemm operand B)
  float* colsum[CHAIN_MAX_HIDDEN]; // [rows/16][H] bias-gradient partials
  float* hw_part;                  // [rows/16][3][H]
  float* hb_part;                  // [rows/16][3]
  double* loss_part;               // [rows/16][2]
  float* pred;                     // [batch][3] or null
  int32_t loss;
  float inv_count;
  inf_ctrl* ctrl;
  int32_t count_step;
  // diagnostics: wall-clock stamps (100 MHz) of wave 0 of the first and the last
  // workgroup: [2][nphase * 5 + 6] = entry, {phase start, MFMAs done, epilogue done} ...,
  // end, weight prologue issued, feature tile written, barrier 0 passed, {after B1} ...,
  // {before B2} ...
  unsigned long long* stamps;
};

// Rays per workgroup: one 16-row MFMA tile up to CHAIN3_MAX_ROWS.  Every workgroup streams
// the whole weight set per step either way, so the smallest tile puts the most CUs on the
// stream (4096 rays -> 256 workgroups).  Larger batches fill the chip with 16-ray tiles many
// times over and pay the stream once per 16 rays: there a workgroup takes C3_NR_WIDE tiles
// (64 rays; 65,536 rays -> 1024 workgroups), each weight fragment feeding C3_NR_WIDE MFMAs.
// tables above this size are read with non-temporal row loads (chain3.hip, zg.hip)
constexpr size_t C3_NT_TABLE_BYTES = (size_t)256 << 20;
constexpr int64_t CHAIN3_MAX_ROWS = 8192;
#ifndef C3_NR_WIDE_DEF  // experiments (variant libraries only)
#define C3_NR_WIDE_DEF 4
#endif
constexpr int C3_NR_WIDE = C3_NR_WIDE_DEF;
constexpr int64_t CHAIN3_WIDE_MAX_ROWS = (int64_t)1 << 24;
// INF_CHAIN3_WIDE=1: wide tiles at any batch that is a multiple of 64 rays (tests compare
// the two widths on one batch)
inline bool chain3_force_wide() { return std::getenv("INF_CHAIN3_WIDE") != nullptr; }
inline bool chain3_wide(int64_t rows) {
  return rows > CHAIN3_MAX_ROWS || (chain3_force_wide() && rows % (16 * C3_NR_WIDE) == 0);
}
inline int chain3_bm(int64_t rows) { return chain3_wide(rows) ? 16 * C3_NR_WIDE : 16; }
// Feature columns per LDS chunk when the whole 16 x k_pad tile does not fit (k_pad > C3_KC).
#ifndef C3_KC_DEF  // experiments (variant libraries only)
#define C3_KC_DEF 1024
#endif
constexpr int C3_KC = C3_KC_DEF;
// ... and for the wide tiles, which always stream the feature tile in chunks
// (512: two chunk gathers per 1024-column tile instead of four, 64 KB of X beside the 64 KB
// of activation tiles: 65,536 rays 569 -> 559 us, profiles/r04/large_b10_*.log)
#ifndef C3_KC_WIDE_DEF
#define C3_KC_WIDE_DEF 512
#endif
constexpr int C3_KC_WIDE = C3_KC_WIDE_DEF;
// Weight-stream blocks of a training step: the input layers' k_pad / (32 upl) blocks each,
// one per hidden layer forward and backward.
inline int chain3_blocks(int H, int L, int k_pad) { return 2 * (k_pad / H) + 2 * (L - 2); }
// The kernel's LDS footprint for this shape fits the CU (chain3.hip)
bool chain3_lds_fits(int H, int L, int k_pad, int64_t rows);
// ... and that of the split-bf16 variant (Chain3Args::x3: 16-ray tiles, k_pad <= C3_KC)
bool chain3_x3_lds_fits(int H, int L, int k_pad);
inline int chain3_kc(int k_pad, int64_t rows);
inline bool chain3_supported(int H, int L, int k_pad, int64_t rows) {
  const int upl = H / 32;
  const bool wide = chain3_wide(rows);
  return (H == 128 || H == 256) && L >= 3 && L - 1 <= CHAIN_MAX_HIDDEN && rows <= CHAIN3_WIDE_MAX_ROWS &&
         (!wide || (rows % (16 * C3_NR_WIDE) == 0 && C3_KC_WIDE % (32 * upl) == 0 &&
                    (k_pad <= C3_KC_WIDE || H == 256))) &&
         k_pad % (32 * upl) == 0 && (k_pad <= C3_KC || C3_KC % (32 * upl) == 0) &&
         chain3_blocks(H, L, k_pad) <= C3_MAX_BLOCKS && chain3_lds_fits(H, L, k_pad, rows);
}
// Feature columns held in LDS at a time for a batch of `rows`
inline int chain3_kc(int k_pad, int64_t rows) {
  if (chain3_wide(rows)) return k_pad < C3_KC_WIDE ? k_pad : C3_KC_WIDE;
  return k_pad > C3_KC ? C3_KC : k_pad;
}

int launch_chain3(const Chain3Args& a, int bm, hipStream_t stream);


}  // namespace inf
