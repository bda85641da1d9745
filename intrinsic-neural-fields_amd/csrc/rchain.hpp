// Register-streamed forward-only chain (render / inference), see rchain.hip.
#pragma once

#include "chain3.hpp"

namespace inf {

constexpr int RC_RT = 4;            // 16-ray MFMA tiles per workgroup
constexpr int RC_BM = 16 * RC_RT;   // rays per workgroup
constexpr int RC_KC = 512;          // feature columns per LDS chunk
constexpr int RC_MAX_BLOCKS = 64;

struct RchainArgs {
  int32_t L, s, H, k_pad;
  int32_t batch;  // rays of this launch
  // rays: ray b reads row r = ray_idx ? ray_idx[idx_offset + b] : idx_offset + b of vids / bary
  const bf16* table;  // [V][k_pad] bf16, or the projected table [V][2H] (projected = 1)
  int32_t projected;  // table rows are (W_0 E[v], W_y E[v]) (inf_project_table)
  int64_t num_vertices;
  int32_t table_big;  // 4 GiB or more: 64-bit row addresses
  const void* vids;
  int32_t vid_dtype;
  const float* bary;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;  // bound on idx_offset + b (0 = unchecked)
  int64_t num_src;   // rows of vids / bary / rgb (inf_batch::num_source_rays; 0 = unchecked)
  // weight stream (C3Block; flags C3F_SWAP / C3F_GATHER as in the chunked chain3 schedule)
  C3Block blk[RC_MAX_BLOCKS];
  int32_t nblk, nphase, nchunk;
  const float* bias[CHAIN_MAX_HIDDEN];
  const float* bias_y;
  const float* W7;  // [3][H] fp32
  const float* b7;
  // outputs: pred [batch][3] and/or the image placement img[pixel_map ? pixel_map[hit[b]] : hit[b]]
  float* pred;
  const int64_t* hit;
  const int64_t* pixel_map;
  float* img;
  // diagnostics (inf_debug_timing): wall-clock stamps of wave 0 of workgroups 0 and
  // gridDim / 2: [2][RC_STAMPS] = entry, records in LDS, chunk 0 in LDS, each block's
  // start, end
  unsigned long long* stamps;
};
constexpr int RC_STAMPS = 4 + RC_MAX_BLOCKS;

inline int rchain_blocks(int H, int L, int k_pad) { return 2 * (k_pad / H) + (L - 2); }
inline bool rchain_supported(int H, int L, int k_pad) {
  return (H == 128 || H == 256) && L >= 3 && L - 1 <= CHAIN_MAX_HIDDEN && k_pad % H == 0 &&
         RC_KC % H == 0 && rchain_blocks(H, L, k_pad) <= RC_MAX_BLOCKS;
}

// projected = 0: rchain.hip; 1: the persistent projected-table chain (rproj.hip; blk =
// the hidden layers 1 .. L - 2, nchunk = 0)
int launch_rchain(const RchainArgs& a, hipStream_t stream);
int launch_rproj(const RchainArgs& a, hipStream_t stream);
// rprojw.hip: the projected-table chain on 128-ray tiles (the 8 x 256 field, skip 4; the
// default there, INF_RPROJ_WIDE=0 keeps rproj.hip's 64-ray tiles)
bool rprojw_supported(const RchainArgs& a);
int launch_rprojw(const RchainArgs& a, hipStream_t stream);

}  // namespace inf
