// Large-batch bf16 training step as layer GEMMs with fused epilogues, see layer.hip.
#pragma once

#include "common.hpp"

namespace inf {

constexpr int LY_RAYS = 128;  // rays per workgroup (eight 16-ray MFMA tiles)
constexpr int LY_KC = 256;    // K columns staged in LDS per chunk
constexpr int LY_MODE_FWD = 0, LY_MODE_BWD = 1, LY_MODE_HEAD = 2;

// One layer over `rows` rays, H = 256 output features, 128-ray workgroups.
// Activations live in "B-operand images": per 16-ray tile n and 32-feature k block kb one
// KiB at (n * (K / 32) + kb) * 1024, lane l's 16 bytes = ray l % 16 of the tile and that
// lane's 8 features of the block -- xgather's X image (natural column order) or a layer
// output (accumulator order: tiles 2 kb, 2 kb + 1 x 4 rows of the lane group, the order the
// hidden layers' fragment images are stored in, adam.hip WF / WTF with wf_acc_order).
//   FWD:  out = relu(sum_s W_s in_s + bias0 (+ bias1)) -> out image + out^T fragment image
//   BWD:  out = (W^T in) * (mask_in > 0) -> out image + out^T + bias-gradient partials
//   HEAD: the last hidden layer's FWD, then the head (model.py:89-94), the loss
//         (config.py:113-122), dL/dz and the head backward in the same workgroup:
//         dZ_{L-2} -> out image + out^T + its bias partials, the output layer's weight /
//         bias partials and the loss partials (chain3's layouts: one partial per workgroup)
struct LayerArgs {
  int32_t rows, H, mode, nsrc;
  const bf16* in[2];  // B-operand images
  int32_t kin[2];     // K of each source (multiple of LY_KC)
  const bf16* w[2];   // A operand: fragment images, H rows (k order = the source's column order)
  const float* bias0;
  const float* bias1;
  const bf16* mask_in;  // BWD: the image whose > 0 entries pass the gradient (Y_{l-1})
  bf16* out;            // B-operand image of the output (FWD, BWD, HEAD: dZ_{L-2})
  bf16* outT;           // fragment image of the output (lgemm.hpp: rows = features, k = rays)
  float* colsum;        // BWD / HEAD: [rows / LY_RAYS][H] bias-gradient partials
  // HEAD
  const float* W7;  // [3][H]
  const float* b7;
  float* hw_part;     // [rows / LY_RAYS][3][H]
  float* hb_part;     // [rows / LY_RAYS][3]
  double* loss_part;  // [rows / LY_RAYS][2]
  float* pred;        // [batch][3] or null
  const float* rgb;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset, num_rays, num_src;
  int32_t offset_from_ctrl, batch, loss;
  float inv_count;
  inf_ctrl* ctrl;
  int32_t count_step;
};

inline bool layer_supported(int H, int64_t rows) { return H == 256 && rows % LY_RAYS == 0 && rows > 0; }

int launch_layer(const LayerArgs& a, hipStream_t stream);

}  // namespace inf
