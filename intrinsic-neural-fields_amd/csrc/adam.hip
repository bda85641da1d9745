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

template <typename T>
__global__ __launch_bounds__(256) void update_kernel(AdamArgs a) {
  __shared__ float tile[ADAM_TILE_C][ADAM_TILE_R + 1];
  __shared__ adam_dev::Scalars sc;
  adam_dev::update_item<T>(a, a.items[blockIdx.x], tile, sc);
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
