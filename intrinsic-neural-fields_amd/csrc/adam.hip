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
    // 16 elements per thread; every load of a phase is issued before its first use so
    // one thread keeps 16 (slab sum) or 48 (Adam state) loads in flight
    const int r0 = item.r0, c0 = item.c0;
    const int c = tid & 63;
    const int rb = tid >> 6;  // rows rb, rb+4, ..., rb+60
    const int gc = c0 + c;
    bool ok[16];
    int64_t e[16];
    float w[16], g[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int gr = r0 + rb + 4 * i;
      ok[i] = gr < seg.R && gc < seg.C;
      e[i] = seg.off + (int64_t)(ok[i] ? gr : 0) * seg.C + (ok[i] ? gc : 0);
      w[i] = ok[i] ? a.params[e[i]] : 0.f;
    }
    if (a.grad_src == GRAD_FLAT) {
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = ok[i] ? a.grads[e[i]] : 0.f;
    } else if (a.grad_src == GRAD_SLABS) {
      const float* base = seg.slab + gc;
#pragma unroll
      for (int i = 0; i < 16; ++i) g[i] = ok[i] ? base[(int64_t)(r0 + rb + 4 * i) * seg.slab_ld] : 0.f;
#pragma unroll 1
      for (int k = 1; k < seg.nslab; ++k) {
        const float* sk = base + (int64_t)k * seg.slab_stride;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (ok[i]) g[i] += sk[(int64_t)(r0 + rb + 4 * i) * seg.slab_ld];
      }
    }
    if (a.grad_src != GRAD_NONE) {
      if (a.write_grads) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (ok[i]) a.grads[e[i]] = g[i];
      }
      if (a.do_adam) {
        float m[16], v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          m[i] = ok[i] ? a.exp_avg[e[i]] : 0.f;
          v[i] = ok[i] ? a.exp_avg_sq[e[i]] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if (ok[i]) {
            adam_elem(w[i], m[i], v[i], g[i], a, sc);
            a.params[e[i]] = w[i];
            a.exp_avg[e[i]] = m[i];
            a.exp_avg_sq[e[i]] = v[i];
          }
        }
      }
    }
    if (!a.write_shadow) return;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = rb + 4 * i;
      if (ok[i]) reinterpret_cast<T*>(seg.W)[(int64_t)(r0 + r) * seg.ldw + gc] = (T)w[i];
      tile[c][r] = w[i];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int idx = tid + 256 * i;
      const int cc = idx >> 6, r = idx & 63;
      const int gr = r0 + r, gcc = c0 + cc;
      if (gr < seg.R && gcc < seg.C) reinterpret_cast<T*>(seg.WT)[(int64_t)gcc * seg.ldwt + gr] = (T)tile[cc][r];
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
