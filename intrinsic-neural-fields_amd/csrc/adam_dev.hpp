// Device side of the parameter update (adam.hip), shared with the weight-gradient GEMM
// (lgemm.hip GT), which runs the same work items on each gradient tile it has just summed:
// one definition of the arithmetic either way.
#pragma once

#include <cmath>

#include "adam.hpp"

namespace inf {
namespace adam_dev {

// beta^t for the step count t >= 1 by binary exponentiation in double (libm's double pow
// is a long software sequence on one lane that every other thread of the block waits for;
// this differs from it by a few double ulps, far below the fp32 rounding of the result)
__device__ __forceinline__ double pow_int(double b, int t) {
  double r = 1.0;
  while (t > 0) {
    if (t & 1) r *= b;
    b *= b;
    t >>= 1;
  }
  return r;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also drains vmcnt: every
// store and every prefetched load of the thread would be waited for at each item.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Scalars {
  float step_neg;  // -lr / (1 - b1^t)
  float bc2_sqrt;  // sqrt(1 - b2^t)
};

// The step's bias-correction scalars, by every thread that needs them (uniform: the same
// double arithmetic on every lane, so bitwise the value one thread would publish in LDS)
__device__ __forceinline__ Scalars step_scalars(const AdamArgs& a) {
  // host-driven step (step_host > 0): t, lr and the bias corrections as given, lr = 0
  // included (a frozen group); otherwise t and lr from ctrl (graph-replayed steps)
  double lr = a.lr_host, bc1 = a.bc1_host, bc2 = a.bc2_host;
  if (a.step_host <= 0) {
    const int t = a.ctrl->step;
    lr = a.ctrl->lr;
    bc1 = 1.0 - pow_int(a.beta1_d, t);
    bc2 = 1.0 - pow_int(a.beta2_d, t);
  }
  Scalars s;
  s.step_neg = (float)(-(lr / bc1));
  s.bc2_sqrt = (float)sqrt(bc2);
  return s;
}

// Four consecutive floats at a dword-aligned (not necessarily 16-byte-aligned) address as one
// 16-byte access: the rows of an arena tensor whose column count is not a multiple of 4
// (config R's k = 1023) start at every dword offset.  Bitwise the element-wise accesses.
__device__ __forceinline__ void load4_unaligned(const float* p, float (&dst)[4]) {
  __builtin_memcpy(dst, p, 16);
}
__device__ __forceinline__ void store4_unaligned(float* p, const float (&src)[4]) { __builtin_memcpy(p, src, 16); }

__device__ __forceinline__ void stamp(unsigned long long* st, int i) {
  if (st != nullptr && threadIdx.x == 0) st[i] = wall_clock64();
}

// torch's single-tensor Adam op by op (torch/optim/adam.py, CPU kernels), with the
// roundings pinned so no code path's FMA contraction can move a bit (the compiler contracted
// differently in different inlined copies, which made two update paths disagree in the last
// bit): measured against torch 2.10 CPU on 2^20 random elements (tools/adam_bits.py), m and v
// match bitwise, p in 99.99 % of elements (torch's vectorised sqrt is not correctly rounded
// in 0.6 % of them; ours is).
//   exp_avg.lerp_(grad, 1 - b1)              m = fma(1 - b1, g - m, m)
//   exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2) v = fma((1 - b2) g, g, v b2)
//   denom = sqrt(v) / sqrt(bc2) + eps
//   param.addcdiv_(exp_avg, denom, -step)    p = p + (-step m) / denom
// The pinned target is torch's CPU single-tensor kernel (the goldens are made on the CPU).
// The reference trains on a GPU, where torch's default foreach Adam computes
// p + step (m / denom) -- a different rounding of the last op, up to 1 ulp of p apart; no
// fixture made here can tell which one the reference's own GPU runs took, so this is NOT
// claimed as the reference's GPU op order.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamArgs& a, const Scalars& s) {
#pragma clang fp contract(off)
  m = __builtin_fmaf(a.one_minus_b1, g - m, m);
  const float vb = v * a.beta2;
  v = __builtin_fmaf(a.one_minus_b2 * g, g, vb);
  const float denom = sqrtf(v) / s.bc2_sqrt + a.eps;
  p = p + (s.step_neg * m) / denom;
}

// The part of a matrix item after its gradient is summed: Adam (or the gradient store),
// the fp32 master write-back and the packed shadows / fragment images.  `tile`: LDS.
template <typename T, bool VEC4>
__device__ __forceinline__ void mt_apply(const AdamArgs& a, const AdamSeg& seg, const AdamItem& item,
                                         const Scalars& sc, float (*tile)[ADAM_TILE_R + 1],
                                         const bool (&ok)[ADAM_TILE_R / 32], const int64_t (&e)[ADAM_TILE_R / 32],
                                         float (&w)[ADAM_TILE_R / 32][4], float (&m)[ADAM_TILE_R / 32][4],
                                         float (&v)[ADAM_TILE_R / 32][4], const float (&g)[ADAM_TILE_R / 32][4]) {
  const int tid = threadIdx.x;
  const int c4 = tid & 7, rb = tid >> 3;
  const int cl = 4 * c4;
  const int gc = item.c0 + cl;
  constexpr int NR = ADAM_TILE_R / 32;
  const bool adam = a.do_adam && a.grad_src != GRAD_NONE;
  auto st4 = [&](float* base, int i, const float (&src)[4]) {
    if (!ok[i]) return;
    if (VEC4) {
      *reinterpret_cast<float4*>(base + e[i]) = make_float4(src[0], src[1], src[2], src[3]);
    } else if (gc + 3 < seg.C) {
      // a whole 4-column group of a row that is not 16-byte aligned in the arena (config R's
      // k = 1023): one dword-aligned 16-byte store (global dwordx4 needs dword alignment only)
      store4_unaligned(base + e[i], src);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (gc + j < seg.C) base[e[i] + j] = src[j];
    }
  };
  if (a.grad_src != GRAD_NONE) {
    if (a.write_grads && a.shard_mode == SHARD_GRAD_OUT) {
      // the item's tile in the gradient staging, [64][32] (out-of-range elements are 0)
      float* gs = a.gsh + (item.goff - a.g_base) + cl;
#pragma unroll
      for (int i = 0; i < NR; ++i)
        *reinterpret_cast<float4*>(gs + (rb + 32 * i) * ADAM_TILE_C) = make_float4(g[i][0], g[i][1], g[i][2], g[i][3]);
    } else if (a.write_grads) {
#pragma unroll
      for (int i = 0; i < NR; ++i) st4(a.grads, i, g[i]);
    }
    if (adam) {
#pragma unroll
      for (int i = 0; i < NR; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) adam_elem(w[i][j], m[i][j], v[i][j], g[i][j], a, sc);
        st4(a.params, i, w[i]);
        st4(a.exp_avg, i, m[i]);
        st4(a.exp_avg_sq, i, v[i]);
      }
      if (a.shard_mode == SHARD_ADAM) {
        // the new weights in the GEMM dtype, [64][32], for the all-gather of the images
        T* ws = reinterpret_cast<T*>(a.wsh + (item.woff - a.w_base)) + cl;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          T* d = ws + (rb + 32 * i) * ADAM_TILE_C;
          if constexpr (sizeof(T) == 2) {
            const bf16x4 pk = {(bf16)w[i][0], (bf16)w[i][1], (bf16)w[i][2], (bf16)w[i][3]};
            *reinterpret_cast<bf16x4*>(d) = pk;
          } else {
            *reinterpret_cast<float4*>(d) = make_float4(w[i][0], w[i][1], w[i][2], w[i][3]);
          }
        }
      }
    }
  }
  if (!a.write_shadow) return;
  const bool rowmajor = a.write_shadow != 2;
  // packed row-major shadow: 4 consecutive columns per store (padded columns stay zero)
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = rb + 32 * i;
    if (ok[i] && rowmajor) {
      T* dst = reinterpret_cast<T*>(seg.W) + (int64_t)(item.r0 + r) * seg.ldw + gc;
      if (VEC4) {
        if constexpr (sizeof(T) == 2) {
          const bf16x4 pk = {(bf16)w[i][0], (bf16)w[i][1], (bf16)w[i][2], (bf16)w[i][3]};
          *reinterpret_cast<bf16x4*>(dst) = pk;
        } else {
          *reinterpret_cast<float4*>(dst) = make_float4(w[i][0], w[i][1], w[i][2], w[i][3]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (gc + j < seg.C) dst[j] = (T)w[i][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) tile[cl + j][r] = w[i][j];
    if constexpr (sizeof(T) == 2) {
      if (seg.WF != nullptr && ok[i]) {
        // forward fragment image: 4 consecutive k of one lane's 8 (gc % 4 == 0), in natural
        // or accumulator k order (adam.hpp wf_acc_order)
        const int gr = item.r0 + r;
        const int kk = gc & 31;
        const int slot = seg.wf_acc_order ? (kk & 15) >> 2 : kk >> 3;
        const int e0 = seg.wf_acc_order ? (kk >> 4) << 2 : kk & 7;
        const int64_t e = ((int64_t)((gc >> 5) * (seg.R >> 4) + (gr >> 4)) * 64 + (gr & 15) + 16 * slot) * 8 + e0;
        const bf16x4 pk = {(bf16)w[i][0], (bf16)w[i][1], (bf16)w[i][2], (bf16)w[i][3]};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(seg.WF) + e) = pk;
      }
    } else {
      if (seg.WF != nullptr && ok[i] && seg.x3) {
        // hi / lo bf16 fragment images (the bf16 layout above; lo = bf16(w - hi), R ldw
        // elements after hi)
        const int gr = item.r0 + r;
        const int kk = gc & 31;
        const int slot = seg.wf_acc_order ? (kk & 15) >> 2 : kk >> 3;
        const int e0 = seg.wf_acc_order ? (kk >> 4) << 2 : kk & 7;
        const int64_t e = ((int64_t)((gc >> 5) * (seg.R >> 4) + (gr >> 4)) * 64 + (gr & 15) + 16 * slot) * 8 + e0;
        bf16x4 hi, lo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hi[j] = (bf16)w[i][j];
          lo[j] = (bf16)(w[i][j] - (float)hi[j]);
        }
        bf16* base = reinterpret_cast<bf16*>(seg.WF);
        *reinterpret_cast<bf16x4*>(base + e) = hi;
        *reinterpret_cast<bf16x4*>(base + (int64_t)seg.R * seg.ldw + e) = lo;
      } else if (seg.WF != nullptr && ok[i]) {
        // fp32 fragment image (chainf.hpp): 2 KiB per (k block, 16-row tile), half
        // (gc / 4) % 2 of lane (gr % 16) + 16 ((gc % 32) / 8)
        const int gr = item.r0 + r;
        const int kk = gc & 31;
        const int64_t e = (((int64_t)((gc >> 5) * (seg.R >> 4) + (gr >> 4)) * 2 + ((kk >> 2) & 1)) * 64 + (gr & 15) +
                           16 * (kk >> 3)) * 4;
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(seg.WF) + e) = make_float4(w[i][0], w[i][1], w[i][2], w[i][3]);
      }
    }
  }
  lds_barrier();
  if constexpr (sizeof(T) == 2) {
    if (seg.WTF != nullptr) {
      // backward fragment image, accumulator k order: thread (column c, 32-row block kbl,
      // row group g) stores one lane's 16 bytes = rows 4 g .. 4 g + 3 and 16 + 4 g .. 16 + 4 g + 3
      const int cc = tid >> 3, kbl = (tid >> 2) & 1, g = tid & 3;
      const int gcc = item.c0 + cc, gr = item.r0 + kbl * 32;
      if (gcc < seg.C && gr + 31 < seg.R) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)tile[cc][kbl * 32 + 16 * (e >> 2) + 4 * g + (e & 3)];
        const int64_t off = ((int64_t)((gr >> 5) * (seg.C >> 4) + (gcc >> 4)) * 64 + (gcc & 15) + 16 * g) * 8;
        *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(seg.WTF) + off) = v;
      }
    }
  } else if (seg.x3) {
    if (seg.WTF != nullptr) {
      // hi / lo bf16 backward images (the bf16 layout above; lo R C elements after hi)
      const int cc = tid >> 3, kbl = (tid >> 2) & 1, g = tid & 3;
      const int gcc = item.c0 + cc, gr = item.r0 + kbl * 32;
      if (gcc < seg.C && gr + 31 < seg.R) {
        bf16x8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = tile[cc][kbl * 32 + 16 * (e >> 2) + 4 * g + (e & 3)];
          hi[e] = (bf16)x;
          lo[e] = (bf16)(x - (float)hi[e]);
        }
        const int64_t off = ((int64_t)((gr >> 5) * (seg.C >> 4) + (gcc >> 4)) * 64 + (gcc & 15) + 16 * g) * 8;
        bf16* base = reinterpret_cast<bf16*>(seg.WTF);
        *reinterpret_cast<bf16x8*>(base + off) = hi;
        *reinterpret_cast<bf16x8*>(base + (int64_t)seg.R * seg.C + off) = lo;
      }
    }
  } else {
    if (seg.WTF != nullptr) {
      // fp32 backward fragment image (A = W^T: rows = input features, k = output
      // features): per (column cc, 32-row block kbl, lane group g, half h) four consecutive
      // rows 32 kb + 8 g + 4 h .. + 3 of one column
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int idx = tid + 256 * s2;
        const int cc = idx >> 4, kbl = (idx >> 3) & 1, g = (idx >> 1) & 3, h = idx & 1;
        const int gcc = item.c0 + cc, gr = item.r0 + kbl * 32;
        if (gcc < seg.C && gr + 31 < seg.R) {
          const int rr = kbl * 32 + 8 * g + 4 * h;
          const int64_t off = (((int64_t)((gr >> 5) * (seg.C >> 4) + (gcc >> 4)) * 2 + h) * 64 + (gcc & 15) + 16 * g) * 4;
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(seg.WTF) + off) =
              make_float4(tile[cc][rr], tile[cc][rr + 1], tile[cc][rr + 2], tile[cc][rr + 3]);
        }
      }
    }
  }
  // packed transposed shadow: 64 consecutive rows of one column per wave
  if (!rowmajor) return;  // write_shadow = 2: fragment images only (plan.hip ensure_rowmajor)
#pragma unroll
  for (int i = 0; i < ADAM_TILE_R * ADAM_TILE_C / 256; ++i) {
    const int idx = tid + 256 * i;
    const int cc = idx / ADAM_TILE_R, r = idx % ADAM_TILE_R;
    const int gr = item.r0 + r, gcc = item.c0 + cc;
    if (gr < seg.R && gcc < seg.C) reinterpret_cast<T*>(seg.WT)[(int64_t)gcc * seg.ldwt + gr] = (T)tile[cc][r];
  }
}

// Matrix tile: ADAM_TILE_R (64) rows x ADAM_TILE_C (32) columns, 256 threads; thread
// (rb, c4) owns rows rb and rb + 32 at columns 4*c4 .. 4*c4+3.  Every load of a phase is
// issued before its first use (parameters + Adam state, then the split-K slabs eight at a
// time) so each thread keeps 16-24 16-byte loads in flight.  VEC4: the tensor's rows are
// 16-byte aligned in the flat arena (C % 4 == 0, offset % 4 == 0); otherwise the arena
// side is accessed element-wise (slabs are always padded and aligned).
// PB: split-K partials loaded per batch
// ST: diagnostics stamps at st (compiled in only for the stamped launch: the asm wait would
// otherwise constrain the schedule of the product kernel)
template <typename T, bool VEC4, int PB, bool ST = false>
__device__ __forceinline__ void matrix_tile(const AdamArgs& a, const AdamSeg& seg, const AdamItem& item,
                                            const Scalars& sc, float (*tile)[ADAM_TILE_R + 1],
                                            unsigned long long* st = nullptr) {
  const int tid = threadIdx.x;
  const int c4 = tid & 7, rb = tid >> 3;
  const int cl = 4 * c4;
  const int gc = item.c0 + cl;
  constexpr int NR = ADAM_TILE_R / 32;
  bool ok[NR];
  int64_t e[NR];
  float w[NR][4], g[NR][4], m[NR][4], v[NR][4];
  auto ld4 = [&](const float* base, int i, float (&dst)[4]) {
    if (VEC4) {
      const float4 t = ok[i] ? *reinterpret_cast<const float4*>(base + e[i]) : make_float4(0.f, 0.f, 0.f, 0.f);
      dst[0] = t.x, dst[1] = t.y, dst[2] = t.z, dst[3] = t.w;
    } else if (ok[i] && gc + 3 < seg.C) {
      load4_unaligned(base + e[i], dst);  // (see st4 in mt_apply)
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = (ok[i] && gc + j < seg.C) ? base[e[i] + j] : 0.f;
    }
  };
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int gr = item.r0 + rb + 32 * i;
    ok[i] = gr < seg.R && gc < seg.C;
    e[i] = seg.off + (int64_t)(ok[i] ? gr : 0) * seg.C + (ok[i] ? gc : 0);
    if (a.shard_mode == SHARD_SCATTER) {
      // another rank's (or this rank's) new weights from the gathered staging: the images only
      const T* ws = reinterpret_cast<const T*>(a.wsh + (item.woff - a.w_base)) + cl + (rb + 32 * i) * ADAM_TILE_C;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[i][j] = (float)ws[j];
    } else {
      ld4(a.params, i, w[i]);
    }
  }
  const bool adam = a.do_adam && a.grad_src != GRAD_NONE;
  if (adam) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      ld4(a.exp_avg, i, m[i]);
      ld4(a.exp_avg_sq, i, v[i]);
    }
  }
  if (a.grad_src == GRAD_FLAT && a.shard_mode == SHARD_ADAM) {
    // this rank's chunk of the reduce-scattered gradient staging
    const float* gs = a.gsh + (item.goff - a.g_base) + cl;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const float4 t = *reinterpret_cast<const float4*>(gs + (rb + 32 * i) * ADAM_TILE_C);
      g[i][0] = t.x, g[i][1] = t.y, g[i][2] = t.z, g[i][3] = t.w;
    }
  } else if (a.grad_src == GRAD_FLAT) {
#pragma unroll
    for (int i = 0; i < NR; ++i) ld4(a.grads, i, g[i]);
  } else if (a.grad_src == GRAD_SLABS) {
#pragma unroll
    for (int i = 0; i < NR; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) g[i][j] = 0.f;
    const float* base = seg.slab + gc;
    const int ns = seg.nslab;
#pragma unroll 1
    for (int k0 = 0; k0 < ns; k0 += PB) {
      float4 t[PB][NR];
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const float* sk = base + (int64_t)(k0 + q) * seg.slab_stride;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const int64_t eo = (int64_t)(item.r0 + rb + 32 * i) * seg.slab_ld;
          t[q][i] = (ok[i] && k0 + q < ns) ? *reinterpret_cast<const float4*>(sk + eo) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      // fixed order: partial 0, 1, ..., ns-1
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        if (k0 + q < ns) {
#pragma unroll
          for (int i = 0; i < NR; ++i) {
            g[i][0] += t[q][i].x;
            g[i][1] += t[q][i].y;
            g[i][2] += t[q][i].z;
            g[i][3] += t[q][i].w;
          }
        }
      }
    }
  }
  if constexpr (ST) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(st, 2);
  }
  mt_apply<T, VEC4>(a, seg, item, sc, tile, ok, e, w, m, v, g);
  if constexpr (ST) stamp(st, 3);
}

// NI matrix items whose reduced gradient is an LDS tile (lgemm.hip GT: the dW^T tile of a
// split-K-1 block -- row m - m0 = input feature, column n - n0 = output feature, the column
// XOR-swizzled by (row / 4) % 16); item it + 1's parameters and moments load while item it
// is applied.  The arithmetic of matrix_tile (mt_apply): bitwise the update launch on the
// same gradient.  An item with seg < 0 (the GEMM's column padding) is skipped.  VEC4:
// 16-byte aligned arena rows (else element-wise, config R's k = 1023).  (Loading every
// item's state ahead of the GEMM's main loop instead was measured slower: the dependent
// item-table loads stall the block's operand prologue, +3 us, for -1.6 us at the tail.)
template <typename T, int NI, bool VEC4>
__device__ __forceinline__ void matrix_items_lds(const AdamArgs& a, const AdamSeg& seg, const AdamItem (&items)[NI],
                                                 Scalars& sc, float (*tile)[ADAM_TILE_R + 1], const float* cs,
                                                 int cld, int m0, int n0) {
  constexpr int NR = ADAM_TILE_R / 32;
  const int tid = threadIdx.x;
  const int c4 = tid & 7, rb = tid >> 3;
  const bool adam = a.do_adam && a.grad_src != GRAD_NONE;
  if (a.do_adam && tid == 0) sc = step_scalars(a);
  struct Regs {
    bool ok[NR];
    int64_t e[NR];
    float w[NR][4], m[NR][4], v[NR][4];
  } R[2];
  auto load = [&](const AdamItem& item, Regs& r) {
    const int gc = item.c0 + 4 * c4;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int gr = item.r0 + rb + 32 * i;
      r.ok[i] = item.seg >= 0 && gr < seg.R && gc < seg.C;
      r.e[i] = seg.off + (int64_t)(r.ok[i] ? gr : 0) * seg.C + (r.ok[i] ? gc : 0);
      auto ld = [&](const float* base, float (&dst)[4]) {
        if constexpr (VEC4) {
          const float4 x = r.ok[i] ? *reinterpret_cast<const float4*>(base + r.e[i]) : make_float4(0.f, 0.f, 0.f, 0.f);
          dst[0] = x.x, dst[1] = x.y, dst[2] = x.z, dst[3] = x.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[j] = (r.ok[i] && gc + j < seg.C) ? base[r.e[i] + j] : 0.f;
        }
      };
      ld(a.params, r.w[i]);
      if (adam) {
        ld(a.exp_avg, r.m[i]);
        ld(a.exp_avg_sq, r.v[i]);
      }
    }
  };
  load(items[0], R[0]);
  if (a.do_adam) lds_barrier();  // sc
#pragma unroll
  for (int it = 0; it < NI; ++it) {
    Regs& r = R[it & 1];
    if (it + 1 < NI) load(items[it + 1], R[(it + 1) & 1]);
    if (items[it].seg < 0) continue;  // column padding of the GEMM (block-uniform)
    float g[NR][4];
    const int row0 = items[it].c0 + 4 * c4 - m0;  // input features row0 .. row0 + 3 of the tile
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int col = items[it].r0 + rb + 32 * i - n0;  // output feature
#pragma unroll
      for (int j = 0; j < 4; ++j) g[i][j] = cs[(row0 + j) * cld + (col ^ ((row0 >> 2) & 15))];
    }
    lds_barrier();  // the previous item's transposed-image tile reads are done
    mt_apply<T, VEC4>(a, seg, items[it], sc, tile, r.ok, r.e, r.w, r.m, r.v, g);
  }
}

// End-of-step item: loss / SSE partials (one per chain tile) summed in a fixed order, so
// the epoch loss is bitwise reproducible (unlike per-tile atomics), then the step's sums
// are stored and added to the epoch sums; optionally the replayed batch index advances.
__device__ inline void finish_step(const AdamArgs& a) {
  __shared__ double rl[256], rs[256];
  const int tid = threadIdx.x;
  double l = 0.0, s = 0.0;
  for (int i = tid; i < a.nloss; i += 256) {
    l += a.loss_part[2 * i];
    s += a.loss_part[2 * i + 1];
  }
  rl[tid] = l;
  rs[tid] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (tid < w) {
      rl[tid] += rl[tid + w];
      rs[tid] += rs[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (a.nloss > 0) {
      a.ctrl->loss_sum = rl[0];
      a.ctrl->sse_sum = rs[0];
      a.ctrl->epoch_loss += rl[0];
      a.ctrl->epoch_sse += rs[0];
    }
    if (a.advance) a.ctrl->batch_index += 1;
  }
}

// One work item (adam.hpp AdamItem) on 256 threads: a matrix tile, a vector chunk or the
// end-of-step item.  `tile` and `sc` are the caller's LDS.
// VT: vector-partial loads in flight per thread; PB: matrix_tile; VEC_ONLY: the caller
// runs vector / end-of-step items only: the matrix path is not compiled into it
// LOCAL_SC: one item per workgroup (the update launch): every thread forms the step's
// scalars itself, so no LDS hand-off and no barrier stand between the item's table loads and
// its data loads (callers that run several items per workgroup keep the barrier, which also
// separates one item's LDS tile from the next).  `st`: diagnostics stamps (AdamArgs::stamps).
template <typename T, int VT = 64, int PB = 8, bool VEC_ONLY = false, bool LOCAL_SC = false, bool ST = false>
__device__ __forceinline__ void update_item(const AdamArgs& a, const AdamItem& item, float (*tile)[ADAM_TILE_R + 1],
                                            Scalars& sc_lds, unsigned long long* st = nullptr) {
  if (item.seg < 0) {
    if ((a.nloss > 0 || a.advance) && a.ctrl != nullptr) finish_step(a);
    return;
  }
  const AdamSeg seg = a.segs[item.seg];
  const int tid = threadIdx.x;

  Scalars sc_loc{0.f, 1.f};
  if constexpr (LOCAL_SC) {
    if (a.do_adam) sc_loc = step_scalars(a);
  } else {
    if (a.do_adam && tid == 0) sc_lds = step_scalars(a);
    if (a.do_adam) lds_barrier();
  }
  const Scalars& sc = LOCAL_SC ? sc_loc : sc_lds;

  if (seg.matrix) {
    if constexpr (!VEC_ONLY) {
      if constexpr (ST) stamp(st, 1);
      if (item.pad & ITEM_VEC4)
        matrix_tile<T, true, PB, ST>(a, seg, item, sc, tile, st);
      else
        matrix_tile<T, false, PB, ST>(a, seg, item, sc, tile, st);
    }
  } else {
    // vector chunk: ADAM_VEC (64) consecutive elements; wave w sums the partials w, w + 4,
    // ... (one coalesced 256-byte load per partial, up to 64 in flight: one round trip for
    // the 256 partials of a 4096-ray step), then the four wave sums are added in a fixed order
    const int el = tid & 63, w = tid >> 6;
    const int gi = item.c0 + el;
    const bool ok = gi < seg.C;
    const int64_t e = seg.off + gi;
    // wave 0's parameter and Adam state load with the partials (one round trip, not two)
    const bool pre = w == 0 && ok && a.do_adam && a.grad_src != GRAD_NONE;
    float pw = 0.f, pm = 0.f, pv = 0.f;
    if (pre) {
      pw = a.params[e];
      pm = a.exp_avg[e];
      pv = a.exp_avg_sq[e];
    }
    float g = 0.f;
    if (a.grad_src == GRAD_SLABS) {
      const float* base = seg.slab + (ok ? gi : 0);
      const int ns = seg.nslab;
#pragma unroll 1
      for (int s0 = w; s0 < ns; s0 += 4 * VT) {
        float t[VT];
#pragma unroll
        for (int q = 0; q < VT; ++q) {
          const int sl = s0 + 4 * q;
          t[q] = (ok && sl < ns) ? base[(int64_t)sl * seg.slab_stride] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < VT; ++q) g += t[q];
      }
    }
    float* vs = &tile[0][0];  // [4][64]
    vs[w * 64 + el] = g;
    lds_barrier();
    if (w == 0 && ok) {
      g = ((vs[el] + vs[64 + el]) + vs[128 + el]) + vs[192 + el];
      if (a.grad_src == GRAD_FLAT) g = a.shard_mode == SHARD_ADAM ? a.gsh[item.goff - a.g_base + el] : a.grads[e];
      if (a.grad_src != GRAD_NONE) {
        if (a.write_grads) {
          if (a.shard_mode == SHARD_GRAD_OUT)
            a.gsh[item.goff - a.g_base + el] = g;
          else
            a.grads[e] = g;
        }
        if (a.do_adam) {
          float m = pm, v = pv;
          adam_elem(pw, m, v, g, a, sc);
          a.params[e] = pw;
          a.exp_avg[e] = m;
          a.exp_avg_sq[e] = v;
          if (a.shard_mode == SHARD_ADAM) reinterpret_cast<float*>(a.wsh + (item.woff - a.w_base))[el] = pw;
        }
      } else if (a.shard_mode == SHARD_SCATTER) {
        a.params[e] = reinterpret_cast<const float*>(a.wsh + (item.woff - a.w_base))[el];
      }
    }
  }
}

}  // namespace adam_dev
}  // namespace inf
