// Register-streamed fused MLP chain for small bf16 training batches, see chain3.hip.
#pragma once

#include "chain.hpp"

namespace inf {

constexpr int C3_MAX_PHASES = 2 * CHAIN_MAX_HIDDEN;

struct Chain3Args {
  int32_t L, s, H;
  int32_t rows, batch;
  // the input GEMM's outputs (plan.hip run_input_gemm): Y_0 = relu(X W_0^T + b_0) and
  // the skip layer's data term Z_y = X W_y^T + b_y
  const bf16* Y0;   // [rows][H] bf16 row-major
  const float* Zy;  // [rows][H] f32 row-major
  // phase p < L-2: forward of hidden layer p+1; p >= L-2: dX of layer (L-2) - (p-(L-2))
  const bf16* img[C3_MAX_PHASES];  // weight image in MFMA fragment order (adam.hip)
  int32_t nphase;
  const float* bias[CHAIN_MAX_HIDDEN];  // Lx.bias at the skip layer (Ly.bias is in Z_y)
  const float* W7;                       // [3][H] fp32 output layer
  const float* b7;
  bf16* YT[CHAIN_MAX_HIDDEN];      // 16-ray blocked Y_l^T, l = 1..L-3
  bf16* dZT[CHAIN_MAX_HIDDEN];     // dZ_l^T as fragment images (H/16 tiles x rows/32 k-blocks,
                                   // lgemm.hpp operand B), l = 0..L-2
  float* colsum[CHAIN_MAX_HIDDEN]; // [rows/BM][H] bias-gradient partials
  float* hw_part;                  // [rows/BM][3][H]
  float* hb_part;                  // [rows/BM][3]
  double* loss_part;               // [rows/BM][2]
  float* pred;                     // [batch][3] or null
  const float* rgb;
  const void* ray_idx;
  int32_t idx_dtype;
  int64_t idx_offset;
  int64_t num_rays;
  int32_t offset_from_ctrl;
  int32_t loss;
  float inv_count;
  inf_ctrl* ctrl;
  int32_t count_step;
  // diagnostics: per-phase wall-clock stamps (100 MHz) of wave 0 of the first and the last
  // workgroup: [2][nphase * 3 + 6] = entry, {phase start, MFMAs done, epilogue done} ..., end,
  // loads issued, Y_0 tile written, barrier 0 passed
  unsigned long long* stamps;
};

// Rays per workgroup.  One 16-row MFMA tile: every CU streams the whole weight set per
// step either way, so the smallest tile puts the most CUs on the stream (4096 rays ->
// 256 workgroups); TM = 2 would need more than the 256 VGPRs a 5-wave workgroup allows.
inline int chain3_bm(int64_t) { return 16; }
// Largest padded batch routed to it (above, the LDS-ring chain's taller tiles win).
constexpr int64_t CHAIN3_MAX_ROWS = 8192;
inline bool chain3_supported(int H, int L, int64_t rows) {
  return (H == 128 || H == 256) && L >= 3 && L - 1 <= CHAIN_MAX_HIDDEN && rows <= CHAIN3_MAX_ROWS;
}

int launch_chain3(const Chain3Args& a, int bm, hipStream_t stream);

}  // namespace inf
