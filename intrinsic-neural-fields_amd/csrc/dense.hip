// Generic fp32 dense layers for the view-dependent texture field (reference
// model.py:115-191 TextureFieldWithViewDependency): its spatial MLP ends in a ReLU
// bottleneck instead of the sigmoid RGB head the fused plan is built around, and its
// directional MLP is two small layers.  No configuration in configs/ enables view
// dependence, so these layers favour generality (arbitrary shapes and strides, exact
// fp32 FMA accumulation in k order) over speed; the hot path stays in the plan.
//
//   inf_dense_gemm:    C[m][n] = act(sum_k A(m,k) B(n,k) + bias[n] + beta C[m][n])
//                      A(m,k) = A[m sam + k sak], B(n,k) = B[n sbn + k sbk]
//   inf_dense_act_bwd: dZ = dY * act'(Y)            (ReLU: Y > 0; sigmoid: Y (1 - Y))
//   inf_colsum:        out[n] (+)= sum_m X[m ldx + n]            (bias gradients)
//   inf_view_angle:    acos(cos_sim(-d, normals[face]))          (model.py:164-169, 179-185)
//   inf_ff_encode:     FourierFeatEnc of 1- or 3-wide inputs     (layers.py:6-25)
#include <cmath>

#include "common.hpp"

namespace inf {
namespace {

constexpr int DG_T = 64;  // output tile
constexpr int DG_K = 16;  // k tile

__global__ __launch_bounds__(256) void dense_gemm_kernel(int M, int N, int K, const float* __restrict__ A,
                                                         int64_t sam, int64_t sak, const float* __restrict__ B,
                                                         int64_t sbn, int64_t sbk, const float* __restrict__ bias,
                                                         int act, float beta, float* __restrict__ C, int64_t ldc) {
  __shared__ float As[DG_K][DG_T + 1];
  __shared__ float Bs[DG_K][DG_T + 1];
  const int t = threadIdx.x;
  const int tm = (t / 16) * 4, tn = (t % 16) * 4;
  const int m0 = blockIdx.y * DG_T, n0 = blockIdx.x * DG_T;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += DG_K) {
    for (int i = t; i < DG_K * DG_T; i += 256) {
      const int kk = i / DG_T, r = i % DG_T;
      const int m = m0 + r, n = n0 + r, k = k0 + kk;
      As[kk][r] = (m < M && k < K) ? A[(int64_t)m * sam + (int64_t)k * sak] : 0.f;
      Bs[kk][r] = (n < N && k < K) ? B[(int64_t)n * sbn + (int64_t)k * sbk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < DG_K; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = As[kk][tm + i];
        b[i] = Bs[kk][tn + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tn + j;
      if (n >= N) continue;
      float v = acc[i][j];
      if (bias != nullptr) v += bias[n];
      float* c = C + (int64_t)m * ldc + n;
      if (beta != 0.f) v += beta * *c;
      if (act == 1) v = fmaxf(v, 0.f);
      if (act == 2) v = 1.f / (1.f + expf(-v));
      *c = v;
    }
  }
}

__global__ void act_bwd_kernel(int64_t n, const float* __restrict__ Y, const float* __restrict__ dY, int act,
                               float* __restrict__ dZ) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float y = Y[i], g = dY[i];
    dZ[i] = act == 1 ? (y > 0.f ? g : 0.f) : (act == 2 ? g * (y * (1.f - y)) : g);
  }
}

__global__ __launch_bounds__(256) void colsum_kernel(int M, int N, const float* __restrict__ X, int64_t ldx,
                                                     float* __restrict__ out, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += X[(int64_t)m * ldx + n];
  out[n] = accumulate ? out[n] + s : s;
}

__global__ void view_angle_kernel(int64_t n, const float* __restrict__ dirs, const int64_t* __restrict__ face,
                                  const float* __restrict__ normals, int64_t num_faces, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = face[i];
    float ang = 0.f;
    if ((uint64_t)f < (uint64_t)num_faces) {
      const float ax = -dirs[3 * i], ay = -dirs[3 * i + 1], az = -dirs[3 * i + 2];
      const float bx = normals[3 * f], by = normals[3 * f + 1], bz = normals[3 * f + 2];
      // F.cosine_similarity: x.y / sqrt(max(|x|^2 |y|^2, eps^2)), eps = 1e-8
      const float w12 = ax * bx + ay * by + az * bz;
      const float w1 = ax * ax + ay * ay + az * az, w2 = bx * bx + by * by + bz * bz;
      const float c = w12 / sqrtf(fmaxf(w1 * w2, 1e-16f));
      ang = acosf(c);
    }
    out[i] = ang;
  }
}

__global__ void ff_encode_kernel(int64_t n, int d, const float* __restrict__ x, const float* __restrict__ bands,
                                 int k, int inc, float* __restrict__ out, int64_t ldo) {
  const int w = 2 * d * k + (inc ? d : 0);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / w;
    const int c = (int)(i % w);
    float v;
    if (c < 2 * d * k) {
      const int j = c < d * k ? c : c - d * k;
      const float e = x[r * d + j / k] * bands[j % k];
      v = c < d * k ? cosf(e) : sinf(e);
    } else {
      v = x[r * d + (c - 2 * d * k)];
    }
    out[r * ldo + c] = v;
  }
}

int blocks_for(int64_t n) { return (int)std::min<int64_t>(4096, std::max<int64_t>(1, (n + 255) / 256)); }

}  // namespace
}  // namespace inf

using namespace inf;

extern "C" {

int inf_dense_gemm(int M, int N, int K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbn,
                   int64_t sbk, const float* bias, int act, float beta, float* C, int64_t ldc, inf_stream_t stream) {
  INF_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && ldc >= N, "dense_gemm: bad shape");
  INF_CHECK_ARG(act >= 0 && act <= 2, "dense_gemm: act must be 0 (none), 1 (ReLU) or 2 (sigmoid)");
  if (M == 0 || N == 0) return INF_OK;
  INF_CHECK_ARG(C != nullptr && (K == 0 || (A != nullptr && B != nullptr)), "dense_gemm: null operand");
  dim3 grid((unsigned)ceil_div(N, DG_T), (unsigned)ceil_div(M, DG_T));
  dense_gemm_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(M, N, K, A, sam, sak, B, sbn, sbk, bias, act, beta, C,
                                                           ldc);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_dense_act_bwd(int64_t n, const float* Y, const float* dY, int act, float* dZ, inf_stream_t stream) {
  INF_CHECK_ARG(n >= 0 && act >= 0 && act <= 2, "act_bwd: bad arguments");
  if (n == 0) return INF_OK;
  INF_CHECK_ARG(Y != nullptr && dY != nullptr && dZ != nullptr, "act_bwd: null argument");
  act_bwd_kernel<<<blocks_for(n), 256, 0, (hipStream_t)stream>>>(n, Y, dY, act, dZ);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_colsum(int M, int N, const float* X, int64_t ldx, float* out, int accumulate, inf_stream_t stream) {
  INF_CHECK_ARG(M >= 0 && N >= 0 && ldx >= N && out != nullptr, "colsum: bad arguments");
  if (N == 0) return INF_OK;
  colsum_kernel<<<(unsigned)ceil_div(N, 256), 256, 0, (hipStream_t)stream>>>(M, N, X, ldx, out, accumulate);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_view_angle(int64_t n, const float* unit_dirs, const int64_t* face_idxs, const float* face_normals,
                   int64_t num_faces, float* out, inf_stream_t stream) {
  INF_CHECK_ARG(n >= 0, "view_angle: bad size");
  if (n == 0) return INF_OK;
  INF_CHECK_ARG(unit_dirs != nullptr && face_idxs != nullptr && face_normals != nullptr && out != nullptr,
                "view_angle: null argument");
  view_angle_kernel<<<blocks_for(n), 256, 0, (hipStream_t)stream>>>(n, unit_dirs, face_idxs, face_normals,
                                                                     num_faces, out);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_ff_encode(int64_t n, int d, const float* x, const float* bands, int k, int include_input, float* out,
                  int64_t ld_out, inf_stream_t stream) {
  INF_CHECK_ARG(n >= 0 && d >= 1 && k >= 1 && ld_out >= 2 * d * k + (include_input ? d : 0), "ff_encode: shape");
  if (n == 0) return INF_OK;
  INF_CHECK_ARG(x != nullptr && bands != nullptr && out != nullptr, "ff_encode: null argument");
  const int64_t total = n * (2 * d * k + (include_input ? d : 0));
  ff_encode_kernel<<<blocks_for(total), 256, 0, (hipStream_t)stream>>>(n, d, x, bands, k, include_input, out, ld_out);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // extern "C"

namespace {
__global__ void adam_dense_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                  float* __restrict__ m, float* __restrict__ v, float one_minus_b1, float beta2,
                                  float one_minus_b2, float eps, float step_neg, float bc2_sqrt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma clang fp contract(off)
    const float gi = g[i];
    float mi = m[i], vi = v[i];
    // the plan's update arithmetic (adam_dev.hpp adam_elem): torch's single-tensor Adam,
    // roundings pinned (no contraction)
    mi = __builtin_fmaf(one_minus_b1, gi - mi, mi);
    const float vb = vi * beta2;
    vi = __builtin_fmaf(one_minus_b2 * gi, gi, vb);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (step_neg * mi) / denom;
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace

extern "C" int inf_adam_dense(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              int step, double lr, double beta1, double beta2, double eps, inf_stream_t stream) {
  INF_CHECK_ARG(n >= 0 && step >= 1, "adam_dense: bad arguments");
  if (n == 0) return INF_OK;
  INF_CHECK_ARG(param != nullptr && grad != nullptr && exp_avg != nullptr && exp_avg_sq != nullptr,
                "adam_dense: null argument");
  // torch's scalars (Python doubles: beta ** step, lr / bc1, sqrt(bc2)), each rounded to
  // float where its CPU kernel takes it
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  adam_dense_kernel<<<blocks_for(n), 256, 0, (hipStream_t)stream>>>(
      n, param, grad, exp_avg, exp_avg_sq, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
      (float)(-(lr / bc1)), (float)std::sqrt(bc2));
  INF_LAUNCH_CHECK();
  return INF_OK;
}
