// Gather + input-layer GEMM ahead of the register chain (chain3.hip's ZP schedule), see zg.hip.
#pragma once

#include "common.hpp"

namespace inf {

// Z_s = [W_0; W_y] X_s^T over the k slice s of the features (fp32, no biases), stored in the
// register chain's accumulator layout: per 16-ray tile w and 16-feature tile t (t < H / 16:
// W_0's rows, then W_y's) one KiB at ((w (2H / 16) + t) 64 + lane) 16 of slice s (at
// Z + s z_stride), lane l's f32x4 = (ray l % 16, features 16 t + 4 (l / 16) + r).  The chain
// adds the slices in order s = 0, 1, ...  X^T (the dW GEMM's fragment image) is written too.
struct ZgArgs {
  const bf16* table;  // [V][k_pad] bf16
  int64_t num_vertices;
  int32_t k_pad, H;
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
  int32_t splits;       // k slices (zg_splits)
  int32_t gather_nt;    // table rows read non-temporally (tables above the MALL)
  const bf16* W0;       // forward fragment images (H rows, natural k order: adam.hip WF)
  const bf16* Wy;
  float* Z;             // [splits][rows / 16][2H / 16] KiB
  int64_t z_stride;     // floats per slice
  bf16* XT;             // X^T fragment image, k_pad rows, `rows` k
};

bool zg_supported(int H, int k_pad, int64_t rows);
int zg_splits(int k_pad, int64_t rows);
int launch_zg(const ZgArgs& a, hipStream_t stream);

}  // namespace inf
