// Output layer (Linear(H,3) + Sigmoid, model.py:89-94), the training losses
// (config.py:113-122) and the first backward stage, on the vector ALUs.
//
// head_fwd:  one wave per ray; lanes split the H-wide dot products, wave-reduced.
//            pred = sigmoid(h . W^T + b); with targets also the loss (mean over
//            loss_count elements), dL/dpred and dz = dL/dpred * p * (1 - p); with a
//            pixel map the colour is placed into the image (renderer.py:124-146).
// head_bwd:  one thread per hidden column, a contiguous chunk of rays per block:
//            dZ[b][k] = (sum_n dz[b][n] W[n][k]) * (h[b][k] > 0)  (ReLU backward,
//            threshold on the layer output as torch does), its transposed copy, the
//            per-block partial sums of dZ (bias grad of the last hidden layer),
//            dW_head = dz^T h and db_head = sum dz.
#include "head.hpp"

namespace inf {
namespace {

constexpr float CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

template <typename T>
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int H = a.H;
  const int epl = H >> 6;  // elements per lane (H multiple of 64, <= 512)
  float w0[8], w1[8], w2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int kk = lane * epl + e;
    const bool ok = e < epl;
    w0[e] = ok ? a.W[kk] : 0.f;
    w1[e] = ok ? a.W[H + kk] : 0.f;
    w2[e] = ok ? a.W[2 * H + kk] : 0.f;
  }
  const float b0 = a.bias[0], b1 = a.bias[1], b2 = a.bias[2];

  int64_t offset = a.idx_offset;
  if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;

  float loss_acc = 0.f, sse_acc = 0.f;
  const int ray0 = blockIdx.x * HEAD_RAYS_PER_BLOCK + wave * (HEAD_RAYS_PER_BLOCK / 4);
#pragma unroll 1
  for (int rr = 0; rr < HEAD_RAYS_PER_BLOCK / 4; ++rr) {
    const int b = ray0 + rr;
    if (b >= a.rows) break;
    float z0 = 0.f, z1 = 0.f, z2 = 0.f;
    const T* hrow = reinterpret_cast<const T*>(a.h) + (int64_t)b * a.ldh + lane * epl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (e < epl) {
        const float hv = (float)hrow[e];
        z0 = fmaf(hv, w0[e], z0);
        z1 = fmaf(hv, w1[e], z1);
        z2 = fmaf(hv, w2[e], z2);
      }
    }
    z0 = wave_sum(z0) + b0;
    z1 = wave_sum(z1) + b1;
    z2 = wave_sum(z2) + b2;
    const float p[3] = {1.f / (1.f + expf(-z0)), 1.f / (1.f + expf(-z1)), 1.f / (1.f + expf(-z2))};
    const bool valid = b < a.batch;
    if (lane < 3) {
      const float pv = p[lane];
      if (valid && a.pred != nullptr) a.pred[(int64_t)b * 3 + lane] = pv;
      if (valid && a.img != nullptr) {
        int64_t pix = a.hit[b];
        if (a.pixel_map != nullptr) pix = a.pixel_map[pix];
        a.img[pix * 3 + lane] = pv;
      }
      if (a.rgb != nullptr) {
        float dz = 0.f;
        if (valid) {
          const int64_t row = ray_row(a.ray_idx, a.idx_dtype, offset, b);
          const float d = pv - a.rgb[row * 3 + lane];
          float l, g;
          if (a.loss == INF_LOSS_L2) {
            l = d * d;
            g = 2.f * d;
          } else if (a.loss == INF_LOSS_L1) {
            l = fabsf(d);
            g = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
          } else {
            const float q = d * d / CAUCHY_C2;
            l = CAUCHY_C2 * logf(1.f + q);
            g = 2.f * d / (1.f + q);
          }
          g *= a.inv_count;
          dz = g * (1.f - pv) * pv;  // sigmoid backward (torch: grad * (1 - y) * y)
          loss_acc += l;
          sse_acc += d * d;
        }
        a.dz[(int64_t)b * 3 + lane] = dz;
      }
    }
  }
  if (a.rgb != nullptr && a.ctrl != nullptr) {
    __shared__ float red[2][4];
    // lanes 0..2 hold partial sums; fold them into lane 0
    float ls = loss_acc + __shfl_down(loss_acc, 1, 64) + __shfl_down(loss_acc, 2, 64);
    float ss = sse_acc + __shfl_down(sse_acc, 1, 64) + __shfl_down(sse_acc, 2, 64);
    if (lane == 0) {
      red[0][wave] = ls;
      red[1][wave] = ss;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double L = (double)red[0][0] + red[0][1] + red[0][2] + red[0][3];
      const double S = (double)red[1][0] + red[1][1] + red[1][2] + red[1][3];
      atomicAdd(&a.ctrl->loss_sum, L);
      atomicAdd(&a.ctrl->sse_sum, S);
      atomicAdd(&a.ctrl->epoch_loss, L);
      atomicAdd(&a.ctrl->epoch_sse, S);
    }
  }
}

template <typename T>
__global__ void head_bwd_kernel(HeadBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [HEAD_BWD_RAYS][H + 4]
  const int k = threadIdx.x;  // hidden column, blockDim.x == H
  const int H = a.H;
  const int LD = H + 4;
  const float w0 = a.W[k], w1 = a.W[H + k], w2 = a.W[2 * H + k];
  float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f, db = 0.f;
  const T* h = reinterpret_cast<const T*>(a.h);
  T* dZ = reinterpret_cast<T*>(a.dZ);
  T* dZT = reinterpret_cast<T*>(a.dZT);

  if (blockIdx.x == 0 && threadIdx.x == 0 && a.step_ctrl != nullptr) a.step_ctrl->step += 1;

#pragma unroll 1
  for (int chunk = blockIdx.x; chunk * HEAD_BWD_RAYS < a.rows; chunk += gridDim.x) {
    const int b0 = chunk * HEAD_BWD_RAYS;
#pragma unroll 4
    for (int r = 0; r < HEAD_BWD_RAYS; ++r) {
      const int b = b0 + r;
      float d0, d1, d2;
      if (a.dz != nullptr) {
        d0 = a.dz[(int64_t)b * 3 + 0];
        d1 = a.dz[(int64_t)b * 3 + 1];
        d2 = a.dz[(int64_t)b * 3 + 2];
      } else if (b < a.batch) {  // autograd: dL/dpred given, apply sigmoid backward here
        const float p0 = a.pred[(int64_t)b * 3 + 0], p1 = a.pred[(int64_t)b * 3 + 1], p2 = a.pred[(int64_t)b * 3 + 2];
        d0 = a.dpred[(int64_t)b * 3 + 0] * (1.f - p0) * p0;
        d1 = a.dpred[(int64_t)b * 3 + 1] * (1.f - p1) * p1;
        d2 = a.dpred[(int64_t)b * 3 + 2] * (1.f - p2) * p2;
      } else {
        d0 = d1 = d2 = 0.f;
      }
      const float hv = (float)h[(int64_t)b * a.ldh + k];
      float g = fmaf(d2, w2, fmaf(d1, w1, d0 * w0));
      g = hv > 0.f ? g : 0.f;
      const T gq = (T)g;
      if (dZ != nullptr) dZ[(int64_t)b * a.ldz + k] = gq;
      tile[r * LD + k] = (float)gq;
      cs += g;
      g0 = fmaf(d0, hv, g0);
      g1 = fmaf(d1, hv, g1);
      g2 = fmaf(d2, hv, g2);
      if (k == 0) db += d0;
      if (k == 1) db += d1;
      if (k == 2) db += d2;
    }
    if (dZT != nullptr) {
      __syncthreads();
      // transposed store: row k of dZ^T, 4 consecutive rays per thread-chunk
      constexpr int Q = HEAD_BWD_RAYS / 4;
      for (int c = threadIdx.x; c < H * Q; c += blockDim.x) {
        const int kk = c / Q, q = c - kk * Q;
        const float x0 = tile[(4 * q + 0) * LD + kk], x1 = tile[(4 * q + 1) * LD + kk];
        const float x2 = tile[(4 * q + 2) * LD + kk], x3 = tile[(4 * q + 3) * LD + kk];
        T* dst = dZT + (int64_t)kk * a.ldzt + b0 + 4 * q;
        dst[0] = (T)x0;
        dst[1] = (T)x1;
        dst[2] = (T)x2;
        dst[3] = (T)x3;
      }
      __syncthreads();
    }
  }
  const int64_t slab = blockIdx.x;
  a.colsum[slab * H + k] = cs;
  a.dW_part[slab * 3 * H + k] = g0;
  a.dW_part[slab * 3 * H + H + k] = g1;
  a.dW_part[slab * 3 * H + 2 * H + k] = g2;
  if (k < 3) a.db_part[slab * 3 + k] = db;
}

}  // namespace

int launch_head_fwd(const HeadFwdArgs& a, int mode, hipStream_t stream) {
  INF_CHECK_ARG(a.H % 64 == 0 && a.H <= 512, "head: hidden width must be a multiple of 64 and <= 512");
  INF_CHECK_ARG(a.rows >= a.batch, "head: rows < batch");
  if (a.rows == 0) return INF_OK;
  const unsigned grid = (unsigned)ceil_div(a.rows, HEAD_RAYS_PER_BLOCK);
  if (mode == INF_MODE_BF16)
    head_fwd_kernel<bf16><<<grid, 256, 0, stream>>>(a);
  else
    head_fwd_kernel<float><<<grid, 256, 0, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int launch_head_bwd(const HeadBwdArgs& a, int mode, hipStream_t stream) {
  INF_CHECK_ARG(a.H % 64 == 0 && a.H <= 1024, "head_bwd: hidden width");
  INF_CHECK_ARG(a.rows % HEAD_BWD_RAYS == 0, "head_bwd: rows must be a multiple of HEAD_BWD_RAYS");
  INF_CHECK_ARG(a.grid >= 1, "head_bwd: grid");
  const size_t lds = (size_t)HEAD_BWD_RAYS * (a.H + 4) * sizeof(float);
  if (mode == INF_MODE_BF16)
    head_bwd_kernel<bf16><<<a.grid, a.H, lds, stream>>>(a);
  else
    head_bwd_kernel<float><<<a.grid, a.H, lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
