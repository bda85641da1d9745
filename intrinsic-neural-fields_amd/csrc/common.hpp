// Shared helpers for the gfx950 kernels of the intrinsic-neural-fields hot path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "inf_hip.h"

namespace inf {

using bf16 = __bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- error channel ---------------------------------------------------------------
void set_error(const std::string& msg);

#define INF_CHECK_ARG(cond, msg)                                  \
  do {                                                            \
    if (!(cond)) {                                                \
      ::inf::set_error(std::string("invalid argument: ") + (msg)); \
      return INF_ERR_ARG;                                         \
    }                                                             \
  } while (0)

#define INF_HIP_TRY(expr)                                                               \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::inf::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));              \
      return INF_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

#define INF_LAUNCH_CHECK()                                                              \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess) {                                                             \
      ::inf::set_error(std::string("kernel launch: ") + hipGetErrorString(e_));         \
      return INF_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

// ---- element conversion ----------------------------------------------------------
template <typename T>
__device__ __forceinline__ float to_f32(T x) { return (float)x; }

template <typename T>
__device__ __forceinline__ T from_f32(float x) { return (T)x; }

__host__ __device__ constexpr inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ constexpr inline int64_t ceil_div(int64_t x, int64_t m) { return (x + m - 1) / m; }

// Index of ray b of a batch: ray_idx[offset + b] (int32/int64) or offset + b.
// Ray b of a batch starting at entry `offset` exists (num_rays 0 = unchecked).
__device__ __forceinline__ bool ray_in_range(int64_t offset, int b, int64_t num_rays) {
  return num_rays <= 0 || (offset + b >= 0 && offset + b < num_rays);
}

__device__ __forceinline__ int64_t ray_row(const void* ray_idx, int idx_dtype, int64_t offset, int b) {
  if (ray_idx == nullptr) return offset + b;
  if (idx_dtype == INF_DTYPE_I64) return reinterpret_cast<const int64_t*>(ray_idx)[offset + b];
  return reinterpret_cast<const int32_t*>(ray_idx)[offset + b];
}

// Source row of ray b of a batch that starts at entry `offset` of ray_idx (or of the rays
// themselves when ray_idx is null), or -1 when the position offset + b is past num_rays or
// the row it names lies outside [0, num_src) (inf_batch::num_source_rays; 0 = unchecked).
// Such a ray reads as a zero feature row and a zero target: a bad permutation entry is
// never turned into a load outside vids / bary / rgb.
__device__ __forceinline__ int64_t source_row(const void* ray_idx, int idx_dtype, int64_t offset, int b,
                                              int64_t num_rays, int64_t num_src) {
  if (!ray_in_range(offset, b, num_rays)) return -1;
  const int64_t r = ray_row(ray_idx, idx_dtype, offset, b);
  if (num_src > 0 && (uint64_t)r >= (uint64_t)num_src) return -1;
  return r;
}

__device__ __forceinline__ int64_t vid_at(const void* vids, int vid_dtype, int64_t i) {
  if (vid_dtype == INF_DTYPE_I64) return reinterpret_cast<const int64_t*>(vids)[i];
  return reinterpret_cast<const int32_t*>(vids)[i];
}

// ---- encoders (gather.hip, chain3.hip) --------------------------------------------
__device__ __forceinline__ float pick3(const float (&x)[3], int i) { return i == 0 ? x[0] : (i == 1 ? x[1] : x[2]); }

// sin and cos of e: three-constant Cody-Waite reduction by pi/2, minimax polynomials on
// [-pi/4, pi/4] (<= 1e-7 abs for |e| < 2^15); larger arguments take ocml's sincosf.
__device__ __forceinline__ void fast_sincos(float e, float* s, float* c) {
  if (!(fabsf(e) < 32768.f)) {
    sincosf(e, s, c);
    return;
  }
  const float n = rintf(e * 0.636619772367581343f);
  float r = fmaf(-n, 1.5703125f, e);  // pi/2 split: 1.5703125 + 4.837512969970703125e-4 + ...
  r = fmaf(-n, 4.837512969970703125e-4f, r);
  r = fmaf(-n, 7.54978995489188216e-8f, r);
  const float r2 = r * r;
  const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f), r2 * r, r);
  const float cp = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2,
                                   4.166664568298827e-2f), r2, -0.5f), r2, 1.0f);
  const int q = (int)n & 3;
  const float ss = (q & 1) ? cp : sp;
  const float cc = (q & 1) ? sp : cp;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}

// ---- kernel launch wrappers (defined in the .hip files) --------------------------
int encoded_dim(int enc, int k, int inc);
int launch_encode(const float* table, int64_t V, const void* vids, int vid_dtype, const float* bary,
                  const void* ray_idx, int idx_dtype, int64_t idx_offset, const int32_t* ctrl_batch_index,
                  int64_t num_rays, int64_t num_src, int batch, int enc, int enc_k, const float* proj, int inc,
                  void* out, int out_dtype, int64_t ld_out, int rows_out, void* out_t, int64_t ld_out_t,
                  hipStream_t stream);
int launch_gather(const void* table, int table_dtype, int64_t V, int k, int64_t table_ld, const void* vids,
                  int vid_dtype, const float* bary, const void* ray_idx, int idx_dtype, int64_t idx_offset,
                  const int32_t* ctrl_batch_index, int64_t num_rays, int64_t num_src, int batch, void* out,
                  int out_dtype,
                  int64_t ld_out, int rows_out, void* out_t, int64_t ld_out_t, hipStream_t stream);

// Pack fp32 features [B][ld_in] into the GEMM dtype [rows_out][ld_out] (+ transposed copy).
int launch_pack_features(const float* in, int64_t ld_in, int k, int batch, void* out, int out_dtype,
                         int64_t ld_out, int rows_out, void* out_t, int64_t ld_out_t, hipStream_t stream);

}  // namespace inf
