// hipBLASLt wrapper for plain library GEMMs (blaslt.hip).
#pragma once

#include "common.hpp"

namespace inf {

// Row-major C[M][N] = A[M][K] B[N][K]^T in bf16 (fp32 accumulation), on `stream`.
int blaslt_gemm_nt_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
                        int64_t N, int64_t K, hipStream_t stream);

}  // namespace inf
