// Output layer (Linear(H,3) + Sigmoid, model.py:89-94), the training losses
// (config.py:113-122) and the first backward stage, on the vector ALUs.
//
// head_fwd:  16 lanes per ray; lanes split the H-wide dot products, shuffle-reduced.
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

// 16 lanes per ray (EPL = H/16 hidden units each, contiguous), 16 rays per 256-thread
// block, one ray per lane group: every load of a ray (index, colour, activation row) is
// issued up front, the three dot products finish with 4 xor-shuffles.
template <typename T, int EPL>
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadFwdArgs a) {
  __shared__ float red[2][16];
  const int lane16 = threadIdx.x & 15;
  const int grp = threadIdx.x >> 4;
  const int b = blockIdx.x * 16 + grp;
  const int H = a.H;
  const bool in_rows = b < a.rows;
  const bool valid = b < a.batch;

  int64_t offset = a.idx_offset;
  if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
  float tgt = 0.f;
  if (a.rgb != nullptr && valid && lane16 < 3) {
    const int64_t row = source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src);
    if (row >= 0) tgt = a.rgb[row * 3 + lane16];
  }
  float hv[EPL];
  const T* hrow = reinterpret_cast<const T*>(a.h) + (int64_t)(in_rows ? b : 0) * a.ldh + lane16 * EPL;
#pragma unroll
  for (int e = 0; e < EPL; ++e) hv[e] = (float)hrow[e];
  float z0 = 0.f, z1 = 0.f, z2 = 0.f;
  const float* W = a.W + lane16 * EPL;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    z0 = fmaf(hv[e], W[e], z0);
    z1 = fmaf(hv[e], W[H + e], z1);
    z2 = fmaf(hv[e], W[2 * H + e], z2);
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) {
    z0 += __shfl_xor(z0, o, 16);
    z1 += __shfl_xor(z1, o, 16);
    z2 += __shfl_xor(z2, o, 16);
  }
  float lsum = 0.f, ssum = 0.f;
  if (lane16 < 3 && in_rows) {
    const float z = (lane16 == 0 ? z0 : (lane16 == 1 ? z1 : z2)) + a.bias[lane16];
    const float pv = 1.f / (1.f + expf(-z));
    if (valid && a.pred != nullptr) a.pred[(int64_t)b * 3 + lane16] = pv;
    if (valid && a.img != nullptr) {
      int64_t pix = a.hit[b];
      if (a.pixel_map != nullptr) pix = a.pixel_map[pix];
      a.img[pix * 3 + lane16] = pv;
    }
    if (a.rgb != nullptr) {
      float dz = 0.f;
      if (valid) {
        const float d = pv - tgt;
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
        lsum = l;
        ssum = d * d;
      }
      a.dz[(int64_t)b * 3 + lane16] = dz;
    }
  }
  if (a.rgb != nullptr && a.ctrl != nullptr) {
    // lanes 0..2 of each group hold the ray's three element losses
    lsum += __shfl_down(lsum, 1, 16) + __shfl_down(lsum, 2, 16);
    ssum += __shfl_down(ssum, 1, 16) + __shfl_down(ssum, 2, 16);
    if (lane16 == 0) {
      red[0][grp] = lsum;
      red[1][grp] = ssum;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      const int which = threadIdx.x >> 4, i = threadIdx.x & 15;
      float v = red[which][i];
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 16);
      if (i == 0) {
        atomicAdd(which == 0 ? &a.ctrl->loss_sum : &a.ctrl->sse_sum, (double)v);
        atomicAdd(which == 0 ? &a.ctrl->epoch_loss : &a.ctrl->epoch_sse, (double)v);
      }
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
  const unsigned grid = (unsigned)ceil_div(a.rows, 16);
#define HEAD_FWD_CASE(EPL)                                                    \
  case EPL:                                                                   \
    if (mode == INF_MODE_BF16)                                                \
      head_fwd_kernel<bf16, EPL><<<grid, 256, 0, stream>>>(a);                \
    else                                                                      \
      head_fwd_kernel<float, EPL><<<grid, 256, 0, stream>>>(a);               \
    break;
  switch (a.H / 16) {
    HEAD_FWD_CASE(4)
    HEAD_FWD_CASE(8)
    HEAD_FWD_CASE(12)
    HEAD_FWD_CASE(16)
    HEAD_FWD_CASE(20)
    HEAD_FWD_CASE(24)
    HEAD_FWD_CASE(28)
    HEAD_FWD_CASE(32)
    default:
      INF_CHECK_ARG(false, "head: unsupported hidden width");
  }
#undef HEAD_FWD_CASE
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
