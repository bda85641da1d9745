// Parameter update stage: gradient-slab reduction, Adam (torch.optim.Adam defaults as
// created at config.py:108 and stepped at trainer.py:82) and the refresh of the packed
// GEMM weights, as ONE launch over a work list built at plan creation.
//
// Work items
//   matrix tile (GEMM weight, 64 x 64): the gradient is the fixed-order sum of the split-K
//       slabs of the weight-gradient GEMM; the new weight is stored to the packed
//       row-major shadow and, through a padded LDS tile, to the packed transposed shadow
//       that the dX GEMMs read, both with coalesced stores;
//   vector chunk (bias, output-layer weight, 8 elements): the gradient is a sum over many
//       per-block partials, so 32 lanes share one element and reduce with shuffles.
// Both sums run in a fixed order: results are bitwise reproducible run to run.
//
// Adam, per element, exactly the single-tensor formula of torch 2.x:
//   m = m + (1 - b1) * (g - m)            (lerp_, weight < 0.5 branch)
//   v = v * b2 + (1 - b2) * g * g         (mul_ + addcmul_)
//   p = p + (-lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
#include "adam.hpp"

namespace inf {
namespace {

struct Scalars {
  float step_neg;  // -lr / (1 - b1^t)
  float bc2_sqrt;  // sqrt(1 - b2^t)
};

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamArgs& a, const Scalars& s) {
  m = m + a.one_minus_b1 * (g - m);
  v = v * a.beta2 + (a.one_minus_b2 * g) * g;
  const float denom = sqrtf(v) / s.bc2_sqrt + a.eps;
  p = p + s.step_neg * (m / denom);
}

template <typename T>
__global__ __launch_bounds__(256) void update_kernel(AdamArgs a) {
  __shared__ float tile[64][65];
  __shared__ Scalars sc;
  const AdamItem item = a.items[blockIdx.x];
  const AdamSeg seg = a.segs[item.seg];
  const int tid = threadIdx.x;

  if (a.do_adam && tid == 0) {
    int t = a.step_host;
    float lr = a.lr_host;
    if (t <= 0) t = a.ctrl->step;
    if (!(lr > 0.f)) lr = a.ctrl->lr;
    const double bc1 = 1.0 - pow((double)a.beta1_d, (double)t);
    const double bc2 = 1.0 - pow((double)a.beta2_d, (double)t);
    sc.step_neg = (float)(-((double)lr / bc1));
    sc.bc2_sqrt = (float)sqrt(bc2);
  }
  if (a.do_adam) __syncthreads();

  if (seg.matrix) {
    const int r0 = item.r0, c0 = item.c0;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx >> 6, c = idx & 63;
      const int gr = r0 + r, gc = c0 + c;
      float w = 0.f;
      if (gr < seg.R && gc < seg.C) {
        const int64_t e = seg.off + (int64_t)gr * seg.C + gc;
        w = a.params[e];
        if (a.grad_src != GRAD_NONE) {
          float g;
          if (a.grad_src == GRAD_FLAT) {
            g = a.grads[e];
          } else {
            const float* s = seg.slab + (int64_t)gr * seg.slab_ld + gc;
            g = s[0];
            for (int k = 1; k < seg.nslab; ++k) g += s[k * seg.slab_stride];
          }
          if (a.write_grads) a.grads[e] = g;
          if (a.do_adam) {
            float m = a.exp_avg[e], v = a.exp_avg_sq[e];
            adam_elem(w, m, v, g, a, sc);
            a.params[e] = w;
            a.exp_avg[e] = m;
            a.exp_avg_sq[e] = v;
          }
        }
        if (a.write_shadow) reinterpret_cast<T*>(seg.W)[(int64_t)gr * seg.ldw + gc] = (T)w;
      }
      tile[c][r] = w;
    }
    if (!a.write_shadow) return;
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int idx = tid + 256 * i;
      const int c = idx >> 6, r = idx & 63;
      const int gr = r0 + r, gc = c0 + c;
      if (gr < seg.R && gc < seg.C) reinterpret_cast<T*>(seg.WT)[(int64_t)gc * seg.ldwt + gr] = (T)tile[c][r];
    }
  } else {
    // vector chunk: 8 elements x 32 lanes
    const int el = tid >> 5, j = tid & 31;
    const int gi = item.c0 + el;
    const bool ok = gi < seg.C;
    float g = 0.f;
    if (a.grad_src == GRAD_SLABS && ok) {
      for (int s = j; s < seg.nslab; s += 32) g += seg.slab[(int64_t)s * seg.slab_stride + gi];
    }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) g += __shfl_xor(g, o, 32);
    if (j == 0 && ok) {
      const int64_t e = seg.off + gi;
      if (a.grad_src == GRAD_FLAT) g = a.grads[e];
      if (a.grad_src != GRAD_NONE) {
        if (a.write_grads) a.grads[e] = g;
        if (a.do_adam) {
          float w = a.params[e], m = a.exp_avg[e], v = a.exp_avg_sq[e];
          adam_elem(w, m, v, g, a, sc);
          a.params[e] = w;
          a.exp_avg[e] = m;
          a.exp_avg_sq[e] = v;
        }
      }
    }
  }
}

}  // namespace

int launch_update(const AdamArgs& a, int mode, hipStream_t stream) {
  INF_CHECK_ARG(a.num_items > 0 && a.items != nullptr && a.segs != nullptr, "update: empty work list");
  INF_CHECK_ARG(!a.do_adam || (a.exp_avg != nullptr && a.exp_avg_sq != nullptr), "update: Adam state not bound");
  INF_CHECK_ARG(!(a.write_grads || a.grad_src == GRAD_FLAT) || a.grads != nullptr, "update: grads not bound");
  INF_CHECK_ARG(!a.do_adam || a.step_host > 0 || a.ctrl != nullptr, "update: no step source");
  if (mode == INF_MODE_BF16)
    update_kernel<bf16><<<a.num_items, 256, 0, stream>>>(a);
  else
    update_kernel<float><<<a.num_items, 256, 0, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
