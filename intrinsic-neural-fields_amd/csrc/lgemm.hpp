// Grouped bf16 GEMM with one operand shared through LDS and the other streamed from an
// MFMA-fragment-order image straight into registers (see lgemm.hip).
//
//   C[m][n] = epilogue( sum_k A[m][k] * B[n][k] )
//
//   dW GEMM      A = In^T [n_in][rays]        (X^T / Y_l^T fragment images, chain3.hip)
//                B = dZ_l^T [n_out][rays]     (fragment image, chain3.hip)
//                C = dW^T, stored transposed into the split-K slab [n_out][n_in]
//
// Fragment image of an R x K matrix: 1 KiB per (32-deep k block kb, 16-row tile t) at
// (kb * R/16 + t) KiB, lane l's 16 bytes at 16 l = row 16 t + l % 16, k = 32 kb + 8 (l / 16) + e.
#pragma once

#include "adam.hpp"
#include "common.hpp"

namespace inf {

constexpr int LGEMM_MAX_PROBLEMS = 12;
constexpr int LG_BN = 128;  // columns per block: 4 waves x 32

struct LgemmProblem {
  // A: fragment image with a_tiles row tiles; rows [a_row0, a_row0 + M) are this problem's rows
  const bf16* Af;
  int32_t a_tiles;
  int32_t a_row0;
  // B: fragment image with b_tiles row tiles; rows [b_row0, b_row0 + N) are its columns
  const bf16* Bf;
  int32_t b_tiles;  // R / 16
  int32_t b_row0;
  // LgemmBatch::split: the lo parts of both operands (same layout; Af / Bf are the hi parts)
  const bf16* Af_lo;
  const bf16* Bf_lo;
  int32_t M, N, K;  // M % BM == 0, N % 128 == 0, (K / splits) % 256 == 0
  int32_t splits;
  // epilogue (non-split): + bias[n], ReLU, row-major C and/or plain transposed CT
  const float* bias;
  int32_t relu;
  void* C;
  int64_t ldc;
  int32_t c_f32;
  bf16* CT;  // [N][ldct]
  int64_t ldct;
  // epilogue (split-K): C^T of split s at slab + s * slab_stride + n * slab_ld + m (f32)
  float* slab;
  int64_t slab_ld, slab_stride;
  int32_t tiles_m, tiles_n, block_begin;
  // fused update (LgemmBatch::fused): the weight's AdamSeg index and its ITEM_VEC4 flag
  int32_t adam_seg, adam_vec4;
};

struct LgemmBatch {
  LgemmProblem p[LGEMM_MAX_PROBLEMS];
  int32_t nprob;
  int32_t total_blocks;
  unsigned long long* stamps;  // diagnostics (inf_debug_block_times) or null
  // Fused parameter update (adam.hip work items, same code), fused == 2 ("gradient tile";
  // 0 = none): split-K 1 with 64 x 64 tiles, each block runs its own tile's items on the
  // gradient in LDS (no slab, no update launch); the first n_aux blocks of the grid (a
  // multiple of 8; n_aux_items of them busy) run the vector and end-of-step items.
  int32_t fused;
  int32_t n_aux, n_aux_items;
  const AdamItem* aux_items;
  AdamArgs adam;
  // split-bf16 operands (hi + lo images, three MFMAs per k block: the bf16x3 mode's dW)
  int32_t split;
};

// Rows per block for an M: 64 (the shapes of config B) or 32.
int launch_lgemm(LgemmBatch& b, int bm, hipStream_t stream);

}  // namespace inf
