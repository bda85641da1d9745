// Split-K weight-gradient GEMM over fragment images for large batches, see fgemm.hip.
#pragma once

#include "common.hpp"

namespace inf {

constexpr int FGEMM_MAX_PROBLEMS = 12;
constexpr int FG_TILE = 256;  // output rows and columns per block
constexpr int FG_BK = 64;     // rays per k-step (two 32-ray fragment-image k blocks)

// One dW^T problem: C[m][n] = sum_k A[m][k] B[n][k] over K rays, A / B fragment images
// (lgemm.hpp: 1 KiB per 32-deep k block kb and 16-row tile t at (kb * tiles + t) KiB).
// Split s of `splits` writes its partial C^T to slab + s * slab_stride + n * slab_ld + m
// (f32), the layout the update launch reduces.
struct FgemmProblem {
  const bf16* Af;
  int32_t a_tiles;  // row tiles of the A image (rows / 16)
  const bf16* Bf;
  int32_t b_tiles;
  int32_t M, N;  // multiples of FG_TILE
  float* slab;
  int64_t slab_ld, slab_stride;
  int32_t block_begin;  // first tile of this problem within a split (set by launch_fgemm)
};

struct FgemmBatch {
  FgemmProblem p[FGEMM_MAX_PROBLEMS];
  int32_t nprob;
  int32_t K;       // rays (multiple of FG_BK)
  int32_t splits;  // split-K factor shared by every problem
  int32_t total_blocks;
  int32_t tiles_per_split;  // blocks of one split: every problem's tiles (set by launch_fgemm)
};

// True when every matrix of the step is a whole number of 256 x 256 tiles.
inline bool fgemm_shape_ok(int M, int N, int K, int splits) {
  return M % FG_TILE == 0 && N % FG_TILE == 0 && K % FG_BK == 0 && splits >= 1 && K / FG_BK >= splits;
}

int launch_fgemm(FgemmBatch& b, hipStream_t stream);

}  // namespace inf
