// Vertex-projection GEMM of the render slice (ptab.hip).
#pragma once

#include "common.hpp"

namespace inf {

// Row-major C[M][N] = A[M][K] B[N][K]^T, bf16 in and out, fp32 accumulation; N a multiple
// of 256, K of 32, 16-byte aligned rows; rows of C past M untouched.
int launch_proj_gemm(const bf16* A, int64_t M, int64_t lda, const bf16* B, int N, int K, bf16* C, int64_t ldc,
                     hipStream_t stream);

}  // namespace inf
