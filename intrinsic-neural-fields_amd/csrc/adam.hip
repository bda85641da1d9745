// Parameter update stage: gradient-slab reduction, Adam (torch.optim.Adam defaults as
// created at config.py:108 and stepped at trainer.py:82) and the refresh of the packed
// GEMM weights, as ONE launch over a work list built at plan creation.
//
// Work items
//   matrix tile (GEMM weight, 64 x 64): the gradient is the fixed-order sum of the split-K
//       slabs of the weight-gradient GEMM; the new weight is stored to the packed
//       row-major shadow and, through a padded LDS tile, to the packed transposed shadow
//       that the dX GEMMs read, both with coalesced stores;
//   vector chunk (bias, output-layer weight, 64 elements): the gradient is a sum over many
//       per-tile partials: four waves split them, one coalesced row per partial.
// Both sums run in a fixed order: results are bitwise reproducible run to run.
//
// Adam, per element, exactly the single-tensor formula of torch 2.x:
//   m = m + (1 - b1) * (g - m)            (lerp_, weight < 0.5 branch)
//   v = v * b2 + (1 - b2) * g * g         (mul_ + addcmul_)
//   p = p + (-lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
#include "adam_dev.hpp"

namespace inf {
namespace {

// ST: the diagnostics build of the launch (AdamArgs::stamps set), per-item wall-clock stamps
template <typename T, bool ST>
__global__ __launch_bounds__(256) void update_kernel(AdamArgs a) {
  __shared__ float tile[ADAM_TILE_C][ADAM_TILE_R + 1];
  __shared__ adam_dev::Scalars sc;
  unsigned long long* st = ST ? a.stamps + (int64_t)blockIdx.x * 8 : nullptr;
  if constexpr (ST) adam_dev::stamp(st, 0);
  // (every thread forming the step's scalars itself instead of thread 0 + an LDS barrier,
  // update_item LOCAL_SC, measured 8.5 vs 8.1 us per launch: the barrier is not on the
  // critical path -- the stamps (tools/update_items.py) put it in the data: ~1.5 us of loads
  // at ~12 TB/s from the MALL, then ~2 us of stores, profiles/r06/update/)
  adam_dev::update_item<T, 64, 8, false, false, ST>(a, a.items[blockIdx.x], tile, sc, st);
  if constexpr (ST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    adam_dev::stamp(st, 4);
  }
}

// one item per workgroup: a 64 x 32 matrix tile (row-major [64][32] in the staging, zero
// beyond the tensor) or a 64-element vector chunk
__global__ __launch_bounds__(256) void shard_copy_kernel(const AdamSeg* segs, const AdamItem* items, const float* src,
                                                         float* dst, int64_t base, int unpack) {
  const AdamItem it = items[blockIdx.x];
  if (it.seg < 0) return;
  const AdamSeg seg = segs[it.seg];
  const int64_t s0 = it.goff - base;
  if (seg.matrix) {
    for (int q = threadIdx.x; q < ADAM_TILE_R * ADAM_TILE_C; q += 256) {
      const int gr = it.r0 + q / ADAM_TILE_C, gc = it.c0 + q % ADAM_TILE_C;
      const bool ok = gr < seg.R && gc < seg.C;
      const int64_t e = seg.off + (int64_t)gr * seg.C + gc;
      if (unpack) {
        if (ok) dst[e] = src[s0 + q];
      } else {
        dst[s0 + q] = ok ? src[e] : 0.f;
      }
    }
  } else if (threadIdx.x < ADAM_VEC) {
    const int gi = it.c0 + threadIdx.x;
    const bool ok = gi < seg.C;
    if (unpack) {
      if (ok) dst[seg.off + gi] = src[s0 + threadIdx.x];
    } else {
      dst[s0 + threadIdx.x] = ok ? src[seg.off + gi] : 0.f;
    }
  }
}

}  // namespace

int launch_shard_copy(const AdamSeg* segs, const AdamItem* items, int num_items, const float* src, float* dst,
                      int64_t base, int unpack, hipStream_t stream) {
  INF_CHECK_ARG(num_items > 0 && items != nullptr && segs != nullptr && src != nullptr && dst != nullptr,
                "shard_copy: empty work list");
  shard_copy_kernel<<<num_items, 256, 0, stream>>>(segs, items, src, dst, base, unpack);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int launch_update(const AdamArgs& a, int mode, hipStream_t stream) {
  INF_CHECK_ARG(a.num_items > 0 && a.items != nullptr && a.segs != nullptr, "update: empty work list");
  INF_CHECK_ARG(!a.do_adam || (a.exp_avg != nullptr && a.exp_avg_sq != nullptr), "update: Adam state not bound");
  INF_CHECK_ARG(!(a.write_grads || a.grad_src == GRAD_FLAT) || a.grads != nullptr, "update: grads not bound");
  INF_CHECK_ARG(!a.do_adam || a.step_host > 0 || a.ctrl != nullptr, "update: no step source");
  const bool st = a.stamps != nullptr;
  if (mode == INF_MODE_BF16) {
    if (st)
      update_kernel<bf16, true><<<a.num_items, 256, 0, stream>>>(a);
    else
      update_kernel<bf16, false><<<a.num_items, 256, 0, stream>>>(a);
  } else {
    if (st)
      update_kernel<float, true><<<a.num_items, 256, 0, stream>>>(a);
    else
      update_kernel<float, false><<<a.num_items, 256, 0, stream>>>(a);
  }
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
