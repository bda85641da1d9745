// Grouped "NT" GEMM engine for the TextureField layers (model.py:43-96, layers.py:60-62)
// and their autograd backward (trainer.py:81).
//
//   C[m][n] = epilogue( sum_seg sum_k A_seg[m][k] * B_seg[n][k] )
//
// Every operand is K-contiguous ("NT"), so a lane's MFMA fragment is one 16-byte LDS
// read.  The callers arrange that by keeping transposed copies where needed:
//   forward        A = X[b][k]       B = W[n][k]       (nn.Linear weight layout)
//   backward dX    A = dZ[b][n]      B = W^T[k][n]     (packed transposed weights)
//   backward dW    A = dZ^T[n][b]    B = X^T[k][b]     (transposed activations)
#pragma once

#include "common.hpp"

namespace inf {

constexpr int GEMM_MAX_PROBLEMS = 12;

struct GemmProblem {
  const void* A[2];
  const void* B[2];
  int64_t lda[2];
  int64_t ldb[2];
  // K-blocked operand (segment 0 only): element (row, k) at (k/16) * ld + row * 16 + k % 16,
  // i.e. ld = rows * 16 -- the layout the fused chain writes Y^T / dZ^T in (whole 128-byte
  // lines per 16-ray tile).  0: plain row-major row * ld + k.
  int32_t a_kblk, b_kblk;
  int32_t K[2];  // per segment, multiple of the k-tile
  int32_t nseg;
  int32_t M, N;  // multiples of the block tile
  int32_t splits;         // split-K over segment 0 (nseg must be 1 when > 1)
  int32_t relu;           // epilogue ReLU (model.py:47,75)
  const float* bias0;     // [N] or null
  const float* bias1;     // [N] or null (skip layer: Lx.bias + Ly.bias, layers.py:61)
  const void* mask;       // [M][ldmask] GEMM dtype: multiply by (mask > 0) (ReLU backward)
  int64_t ldmask;
  void* C;                // [M][ldc] GEMM dtype (or f32 if c_f32) row-major output
  int64_t ldc;
  int32_t c_f32;
  void* CT;               // [N][ldct] GEMM dtype transposed output
  int64_t ldct;
  float* colsum;          // [M/64][N] column sums of the final values per 64 rows (bias grads)
  float* slab;            // split-K fp32 output: slab + split*slab_stride + m*slab_ld + n
  int64_t slab_ld;
  int64_t slab_stride;
  int32_t tiles_m, tiles_n;
  int32_t block_begin;
};

struct GemmBatch {
  GemmProblem p[GEMM_MAX_PROBLEMS];
  int32_t nprob;
  int32_t total_blocks;
  int32_t xcd_remap;  // 1: XCD-aware block -> tile order (set by launch_gemm)
};

// Tile configuration selector.
enum GemmTile { TILE_128x128 = 0, TILE_64x64 = 1, TILE_128x64 = 2 };
inline int tile_bm(GemmTile t) { return t == TILE_64x64 ? 64 : 128; }
inline int tile_bn(GemmTile t) { return t == TILE_128x128 ? 128 : 64; }

// GEMM arithmetic beyond the plan modes: fp32 operands as three bf16 parts, six products
// (fp32-class; the split-bf16 plan mode's GEMMs that need it, plan.hip split_gemm_mode)
constexpr int GEMM_MODE_BF16X6 = 16;

// Fills tiles_m/tiles_n/block_begin/total_blocks and launches.  mode = INF_MODE_* or
// GEMM_MODE_BF16X6.
int launch_gemm(GemmBatch& batch, int mode, GemmTile tile, hipStream_t stream);

}  // namespace inf
