// Output layer + loss kernels (see head.hip).
#pragma once

#include "common.hpp"

namespace inf {

constexpr int HEAD_RAYS_PER_BLOCK = 64;  // head_fwd: 4 waves x 16 rays
constexpr int HEAD_BWD_RAYS = 32;        // head_bwd: rays per chunk

struct HeadFwdArgs {
  const void* h;        // [rows][ldh] GEMM dtype: last hidden activation
  int64_t ldh;
  int32_t H;
  const float* W;       // [3][H] fp32 (layers.{L-1}.0.weight)
  const float* bias;    // [3]
  int32_t batch;        // valid rays
  int32_t rows;         // padded rays (>= batch)
  float* pred;          // [batch][3] or null
  // training (rgb != null): loss, dz
  const float* rgb;     // [N][3] target colours, row = ray_idx[offset + b]
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;     // bound on idx_offset + b (0 = unchecked)
  int64_t num_src;   // rows of vids / bary / rgb (inf_batch::num_source_rays; 0 = unchecked)
  int32_t offset_from_ctrl;
  int32_t loss;
  float inv_count;      // 1 / (elements of the loss mean)
  float* dz;            // [rows][3]
  inf_ctrl* ctrl;       // loss sums (atomics), batch index
  // render placement (img != null)
  const int64_t* hit;
  const int64_t* pixel_map;
  float* img;
};

struct HeadBwdArgs {
  const float* dz;      // [rows][3] (fused path) or null
  const float* dpred;   // [batch][3] dL/dpred (autograd path)
  const float* pred;    // [batch][3]
  const void* h;        // [rows][ldh] last hidden activation (GEMM dtype)
  int64_t ldh;
  int32_t H;
  const float* W;       // [3][H]
  int32_t batch, rows;
  void* dZ;             // [rows][ldz] GEMM dtype or null
  int64_t ldz;
  void* dZT;            // [H][ldzt] GEMM dtype or null
  int64_t ldzt;
  float* colsum;        // [grid][H]  partial bias grad of the last hidden layer
  float* dW_part;       // [grid][3][H]
  float* db_part;       // [grid][3]
  inf_ctrl* step_ctrl;  // if non-null: ctrl->step += 1 (one optimizer step per backward)
  int32_t grid;
};

int launch_head_fwd(const HeadFwdArgs& a, int mode, hipStream_t stream);
int launch_head_bwd(const HeadBwdArgs& a, int mode, hipStream_t stream);

}  // namespace inf
