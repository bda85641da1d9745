// The input layers of the bf16 training step as a gather + GEMM ahead of the register
// chain (chain3.hip's ZP schedule), see igemm.hip.
#pragma once

#include "common.hpp"

namespace inf {

// Barycentric gather of a training batch (mesh.py:313-324 with the loader's index select,
// ray_dataloader.py:122-129) into the row-major feature matrix X and its fragment image X^T
// (lgemm.hpp: rows = features, k = rays) -- chain3's gather numerics, bit for bit.  X is
// stored as the input-layer GEMM's B-operand image: [rows / 16][k_pad / 32] KiB pieces,
// lane l's 16 bytes = ray l % 16 of the tile, columns 8 (l / 16) .. + 7 of the k block.
struct XGatherArgs {
  const bf16* table;  // [V][k_pad] bf16
  int64_t num_vertices;
  int32_t k_pad;
  const void* vids;
  int32_t vid_dtype;
  const float* bary;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays, num_src;
  const inf_ctrl* ctrl;
  int32_t offset_from_ctrl;
  int32_t batch, rows;  // rays of the batch; padded rows (zero features past the batch)
  int32_t gather_nt;    // table rows read non-temporally (tables above the MALL)
  bf16* X;              // B-operand image (above)
  bf16* XT;             // fragment image, k_pad rows, `rows` k
};

// Pre-activations of layer 0 and of the skip layer's Ly (model.py:98-104, layers.py:60-62)
// without their biases: Z = [W_0; W_y] X^T over the batch, fp32, stored in the register
// chain's accumulator layout -- per 16-ray tile w and 16-feature tile t (t < H / 16: W_0's
// rows, then W_y's) one KiB at ((w (2H / 16) + t) 64 + lane) 16 holding lane l's f32x4
// (ray l % 16, features 16 t + 4 (l / 16) + r).
struct IGemmArgs {
  const bf16* X;   // xgather's B-operand image
  int32_t rows, k_pad, H;
  const bf16* W0;  // forward fragment images (H rows, natural k order: adam.hip WF)
  const bf16* Wy;
  float* Z;
};

// rows % 32 == 0 (gather) / % 64 (GEMM); k_pad % 256 == 0 and <= 1024
inline bool igemm_supported(int H, int k_pad, int64_t rows) {
  return (H == 128 || H == 256) && k_pad % 256 == 0 && k_pad <= 1024 && k_pad >= 2 * H && rows % 64 == 0 &&
         rows > 0;
}

int launch_xgather(const XGatherArgs& a, hipStream_t stream);
int launch_igemm(const IGemmArgs& a, hipStream_t stream);

}  // namespace inf
