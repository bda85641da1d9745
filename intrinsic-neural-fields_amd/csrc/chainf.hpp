// Fused fp32 training chain (the parity mode's step), see chainf.hip.
#pragma once

#include "chain3.hpp"

namespace inf {

// One block of the weight stream: UPL k-blocks of 32 of an fp32 fragment image (below),
// the B operand the gathered feature tile (a_x = 1, from its k-block ak0 on) or the
// activation tile (a_x = 0); `last` ends phase `phase` (its epilogue runs).
struct CFBlock {
  const float* img;
  int32_t kb0;
  int32_t a_x;
  int32_t ak0;
  int32_t phase;
  int32_t last;
};

// fp32 MFMA fragment image of a matrix A [R][K] (the A operand of v_mfma_f32_16x16x4_f32:
// lane l supplies A[l % 16][l / 16]): 2 KiB per (32-deep k block kb, 16-row tile t) at
// (kb * R / 16 + t) * 2 KiB; half h (1 KiB) holds, at 16 l, lane l's four values
// A[16 t + l % 16][32 kb + 8 (l / 16) + 4 h + e], e = 0..3.  MFMA i (0..7) of the k block
// takes element i % 4 of half i / 4: every MFMA sums k = 8 g + i over the lane groups g,
// and the B operand (a [ray][k] LDS tile) is read the same way -- 8 consecutive k of one
// ray per lane.  Written by the update launch (adam_dev.hpp, fp32 plans).
inline int64_t cf_image_floats(int R, int K) { return (int64_t)R * K; }

struct ChainFArgs {
  int32_t L, s, H, k_pad;
  int32_t rows, batch;
  // rays: the barycentric gather (mesh.py:313-324) with the loader's index select
  // (ray_dataloader.py:122-129) over an fp32 table [V][k_pad] (zero columns past k)
  const float* table;
  int64_t num_vertices;
  const void* vids;
  int32_t vid_dtype;
  const float* bary;
  const float* rgb;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;
  int64_t num_src;
  int32_t offset_from_ctrl;
  CFBlock blk[C3_MAX_BLOCKS];
  int32_t nblk, nphase;
  const float* bias[CHAIN_MAX_HIDDEN];  // layer l bias (Lx.bias at the skip layer)
  const float* bias_y;                   // Ly.bias
  const float* W7;                       // [3][H] output layer
  const float* b7;
  // outputs for the weight-gradient GEMM (gemm.hip, 16-ray blocked operands: block
  // b / 16 holds [features][16 rays]) and the update launch
  float* XT;                        // [rows / 16][k_pad][16]
  float* YT[CHAIN_MAX_HIDDEN];      // [rows / 16][H][16], l = 0..L-3
  float* dZT[CHAIN_MAX_HIDDEN];     // [rows / 16][H][16], l = 0..L-2
  float* colsum[CHAIN_MAX_HIDDEN];  // [rows / 16][H] bias-gradient partials
  float* hw_part;                   // [rows / 16][3][H]
  float* hb_part;                   // [rows / 16][3]
  double* loss_part;                // [rows / 16][2]
  float* pred;                      // [batch][3] or null
  int32_t loss;
  float inv_count;
  inf_ctrl* ctrl;
  int32_t count_step;
  // bf16x3 mode's dW on the split-bf16 register GEMM (lgemm.hip SPLIT): X^T, Y^T and dZ^T
  // are written instead as pairs of bf16 fragment images (lgemm.hpp: rows = features,
  // k = rays), hi = bf16(x) at the buffer's start and lo = bf16(x - hi) right after the R x
  // rows hi image
  int32_t split_images;
};

constexpr int CHAINF_MAX_KPAD = 1024;  // the 16 x k_pad fp32 feature tile stays in LDS

bool chainf_supported(int H, int L, int k_pad);
int launch_chainf(const ChainFArgs& a, hipStream_t stream);

}  // namespace inf
