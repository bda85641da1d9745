// Fused per-ray-tile MLP chain for the bf16 perf mode.
//
// One workgroup owns BM rays and runs, in ONE launch:
//   forward   layers 0..L-2  (TextureField.forward, model.py:98-112; the skip layer
//             layers.py:60-62 as two K segments [h | x] into one accumulator),
//   head      Linear(H,3) + sigmoid (model.py:89-94), loss (config.py:113-122),
//             dL/dz = dL/dp * p (1 - p),
//   backward  dZ_{L-2} = (dz W_head) * (h > 0), then dZ_{l-1} = (dZ_l W_l) * (Y_{l-1} > 0)
//             for l = L-2..1 (autograd of trainer.py:81).
// The activation / gradient tile (BM x H bf16) stays in LDS across all layers and is
// overwritten in place (the layer's accumulators are in registers until every wave has
// finished reading it).  Only what the weight-gradient GEMM needs leaves the CU: Y_l^T
// and dZ_l^T (bf16, transposed, 8-byte stores), per-64-row bias-gradient partials and the
// output layer's partial gradients.  Packed weights (W, W^T) and the gathered feature
// rows X stream through a double-buffered LDS stage: the loads of flat step t+1 -- which
// may belong to the next layer -- are in flight while the MFMAs of step t run.
//
// Wave layout: (BM/64) x 4 waves; a wave owns 64 rows x H/4 columns as 4 x (H/64)
// v_mfma_f32_16x16x32_bf16 tiles with fp32 accumulators.
// LDS swizzles (16-byte chunk c of row r):
//   activation rows (>= 256 B): c ^ (r & 15)            -> 16 rows of a ds_read_b128 lane
//   stage rows of 128 B:        c ^ ((r >> 1) & 7)         group hit 16 distinct bank
//   stage rows of  64 B:        c ^ ((r >> 2) & 3)         slots (conflict-free)
#include "chain.hpp"

namespace inf {
namespace {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr float CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);

template <int H, int BM, int BK>
struct CT {
  static constexpr int THREADS = 4 * BM;
  static constexpr int WN = H / 4;
  static constexpr int TM = 4, TN = WN / 16;
  static constexpr int ACT_ROW = H * 2;
  static constexpr int STAGE_ROW = BK * 2;
  static constexpr int CH_ROW = BK / 8;
  static constexpr int W_CHUNKS = H * CH_ROW / THREADS;
  static constexpr int X_CHUNKS = BM * CH_ROW / THREADS;
  static constexpr int OFF_ACT = 0;
  static constexpr int OFF_W = BM * ACT_ROW;
  static constexpr int OFF_X = OFF_W + 2 * H * STAGE_ROW;
  static constexpr int OFF_DZ = OFF_X + 2 * BM * STAGE_ROW;
  static constexpr int OFF_RED = OFF_DZ + BM * 3 * 4;
  static constexpr int LDS = OFF_RED + 2 * 16 * 4;
  static_assert(W_CHUNKS >= 1 && X_CHUNKS >= 1, "tile too small for the block");
  static_assert(H * (BM / 64) <= THREADS, "column walk needs one thread per column and 64-row group");
};

template <int BK>
__device__ __forceinline__ int stage_off(int row, int c) {
  if constexpr (BK == 64) return row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
}

template <int H>
__device__ __forceinline__ int act_off(int row, int col) {  // byte offset of element (row, col)
  return row * (H * 2) + (((col >> 3) ^ (row & 15)) << 4) + ((col & 7) << 1);
}

__device__ __forceinline__ unsigned short bf_bits(float x) {
  bf16 h = (bf16)x;
  return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float bf_val(unsigned short u) { return (float)__builtin_bit_cast(bf16, u); }

#ifdef INF_CHAIN_DEBUG
__device__ bool dbg_ok(const ChainArgs& a, const void* ptr, int bytes, int site) {
  const uint64_t x = (uint64_t)ptr;
  for (int i = 0; i < a.dbg_nranges; ++i)
    if (x >= a.dbg_ranges[2 * i] && x + bytes <= a.dbg_ranges[2 * i + 1]) return true;
  const unsigned long long n = atomicAdd(&a.dbg_out[0], 1ull);
  if (n < 32) {
    a.dbg_out[1 + 2 * n] = site;
    a.dbg_out[2 + 2 * n] = x;
  }
  return false;
}
#define GOK(ptr, bytes, site) dbg_ok(a, (const void*)(ptr), bytes, site)
#else
#define GOK(ptr, bytes, site) true
#endif

template <int H, int BM, int BK>
__global__ __launch_bounds__(4 * BM) void chain_kernel(const ChainArgs a) {
  using C = CT<H, BM, BK>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act = smem + C::OFF_ACT;
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* red = reinterpret_cast<float*>(smem + C::OFF_RED);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int L = a.L;

  if (a.count_step && blockIdx.x == 0 && tid == 0 && GOK(&a.ctrl->step, 4, 1)) a.ctrl->step += 1;

  i32x4 rw[C::W_CHUNKS], rx[C::X_CHUNKS];
  auto prefetch = [&](int step, int p) {
    const ChainPhase& P = a.ph[p];
    const int k0 = (step - P.step0) * BK;
#pragma unroll
    for (int i = 0; i < C::W_CHUNKS; ++i) {
      const int c = tid + C::THREADS * i;
      const int row = c / C::CH_ROW, ch = c % C::CH_ROW;
      const bf16* src = P.B + (int64_t)row * P.ldb + k0 + ch * 8;
      rw[i] = GOK(src, 16, 2) ? *reinterpret_cast<const i32x4*>(src) : i32x4{0, 0, 0, 0};
    }
    if (P.a_src) {
#pragma unroll
      for (int i = 0; i < C::X_CHUNKS; ++i) {
        const int c = tid + C::THREADS * i;
        const int row = c / C::CH_ROW, ch = c % C::CH_ROW;
        const bf16* src = a.X + (int64_t)(b0 + row) * a.k_pad + k0 + ch * 8;
        rx[i] = GOK(src, 16, 3) ? *reinterpret_cast<const i32x4*>(src) : i32x4{0, 0, 0, 0};
      }
    }
  };
  auto stage_store = [&](int buf, int p) {
    char* ws = smem + C::OFF_W + buf * H * C::STAGE_ROW;
#pragma unroll
    for (int i = 0; i < C::W_CHUNKS; ++i) {
      const int c = tid + C::THREADS * i;
      *reinterpret_cast<i32x4*>(ws + stage_off<BK>(c / C::CH_ROW, c % C::CH_ROW)) = rw[i];
    }
    if (a.ph[p].a_src) {
      char* xs = smem + C::OFF_X + buf * BM * C::STAGE_ROW;
#pragma unroll
      for (int i = 0; i < C::X_CHUNKS; ++i) {
        const int c = tid + C::THREADS * i;
        *reinterpret_cast<i32x4*>(xs + stage_off<BK>(c / C::CH_ROW, c % C::CH_ROW)) = rx[i];
      }
    }
  };

  f32x4 acc[C::TM][C::TN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto compute = [&](int buf, int p, int kt) {
    const char* ws = smem + C::OFF_W + buf * H * C::STAGE_ROW;
    const char* xs = smem + C::OFF_X + buf * BM * C::STAGE_ROW;
    const bool from_x = a.ph[p].a_src != 0;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 av[C::TM], bv[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * 64 + i * 16 + r16;
        const char* src = from_x ? xs + stage_off<BK>(row, kk * 4 + g4)
                                 : act + row * C::ACT_ROW + ((((kt * BK + kk * 32) >> 3) + g4) ^ (row & 15)) * 16;
        av[i] = *reinterpret_cast<const bf16x8*>(src);
      }
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int row = wc * C::WN + j * 16 + r16;
        bv[j] = *reinterpret_cast<const bf16x8*>(ws + stage_off<BK>(row, kk * 4 + g4));
      }
#pragma unroll
      for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };

  // forward epilogue of layer l: bias + ReLU -> activation tile (in place) and Y_l^T
  auto fwd_epilogue = [&](int l) {
    const float* bias = a.bias[l];
    const float* bias_y = (l == a.s) ? a.bias_y : nullptr;
    bf16* yt = a.save ? a.YT[l] : nullptr;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = wc * C::WN + j * 16 + r16;
      const float bv = GOK(bias + col, 4, 4) ? bias[col] : 0.f;
      const float by = (bias_y != nullptr && GOK(bias_y + col, 4, 5)) ? bias_y[col] : 0.f;
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * 64 + i * 16 + g4 * 4;
        u16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bv;
          if (bias_y != nullptr) v += by;
          v = fmaxf(v, 0.f);
          q[r] = bf_bits(v);
          *reinterpret_cast<unsigned short*>(act + act_off<H>(row + r, col)) = q[r];
        }
        if (yt != nullptr && GOK(yt + (int64_t)col * a.ldt + b0 + row, 8, 6))
          *reinterpret_cast<u16x4*>(yt + (int64_t)col * a.ldt + b0 + row) = q;
      }
    }
  };

  // backward epilogue of layer l: mask by Y_{l-1} > 0 -> dZ_{l-1} (tile, ^T, bias partials)
  auto bwd_epilogue = [&](int l) {
    const bf16* yt = a.YT[l - 1];
    bf16* dzt = a.dZT[l - 1];
    const bool keep = (l - 1) >= 1;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = wc * C::WN + j * 16 + r16;
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * 64 + i * 16 + g4 * 4;
        const u16x4 m = GOK(yt + (int64_t)col * a.ldt + b0 + row, 8, 7)
                            ? *reinterpret_cast<const u16x4*>(yt + (int64_t)col * a.ldt + b0 + row)
                            : u16x4{0, 0, 0, 0};
        u16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = bf_val(m[r]) > 0.f ? acc[i][j][r] : 0.f;
          cs += v;
          q[r] = bf_bits(v);
          if (keep) *reinterpret_cast<unsigned short*>(act + act_off<H>(row + r, col)) = q[r];
        }
        if (GOK(dzt + (int64_t)col * a.ldt + b0 + row, 8, 8))
          *reinterpret_cast<u16x4*>(dzt + (int64_t)col * a.ldt + b0 + row) = q;
      }
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (g4 == 0 && GOK(&a.colsum[l - 1][(int64_t)(b0 / 64 + wr) * H + col], 4, 9))
        a.colsum[l - 1][(int64_t)(b0 / 64 + wr) * H + col] = cs;
    }
  };

  // output layer + loss on the activation tile of layer L-2
  auto head = [&]() {
    const int ray = tid >> 2, part = tid & 3;
    const int b = b0 + ray;
    const bool valid = b < a.batch;
    float tgt = 0.f;
    int64_t offset = a.idx_offset;
    if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
    if (a.rgb != nullptr && valid && part < 3) {
      const void* ip = a.idx_dtype == INF_DTYPE_I64 ? (const void*)((const int64_t*)a.ray_idx + offset + b)
                                                    : (const void*)((const int32_t*)a.ray_idx + offset + b);
      (void)ip;
      if (a.ray_idx == nullptr || GOK(ip, 4, 10)) {
        const int64_t rr = ray_row(a.ray_idx, a.idx_dtype, offset, b);
        if (GOK(a.rgb + rr * 3 + part, 4, 11)) tgt = a.rgb[rr * 3 + part];
      }
    }
    float z0 = 0.f, z1 = 0.f, z2 = 0.f;
    constexpr int CPP = H / 32;  // 16-byte chunks per thread
#pragma unroll
    for (int q = 0; q < CPP; ++q) {
      const int c = part * CPP + q;
      const u16x8 v = *reinterpret_cast<const u16x8*>(act + ray * C::ACT_ROW + ((c ^ (ray & 15)) << 4));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = c * 8 + e;
        const float h = bf_val(v[e]);
        if (!GOK(a.W7 + 2 * H + k, 4, 12)) continue;
        z0 = fmaf(h, a.W7[k], z0);
        z1 = fmaf(h, a.W7[H + k], z1);
        z2 = fmaf(h, a.W7[2 * H + k], z2);
      }
    }
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
      z0 += __shfl_xor(z0, o, 4);
      z1 += __shfl_xor(z1, o, 4);
      z2 += __shfl_xor(z2, o, 4);
    }
    float lsum = 0.f, ssum = 0.f;
    if (part < 3) {
      const float z = (part == 0 ? z0 : (part == 1 ? z1 : z2)) + (GOK(a.b7 + part, 4, 13) ? a.b7[part] : 0.f);
      const float pv = 1.f / (1.f + expf(-z));
      if (valid && a.pred != nullptr) a.pred[(int64_t)b * 3 + part] = pv;
      if (valid && a.img != nullptr) {
        int64_t pix = a.hit[b];
        if (a.pixel_map != nullptr) pix = a.pixel_map[pix];
        a.img[pix * 3 + part] = pv;
      }
      if (a.train) {
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
          dz = (g * a.inv_count) * (1.f - pv) * pv;
          lsum = l;
          ssum = d * d;
        }
        dzs[ray * 3 + part] = dz;
      }
    }
    if (a.train && a.ctrl != nullptr) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        lsum += __shfl_xor(lsum, o, 64);
        ssum += __shfl_xor(ssum, o, 64);
      }
      if (lane == 0) {
        red[wave] = lsum;
        red[16 + wave] = ssum;
      }
    }
  };

  // dZ_{L-2}, output-layer partial gradients, bias partials, then dZ_{L-2}^T
  auto head_bwd = [&]() {
    if (a.ctrl != nullptr && tid == 0) {
      double L_ = 0, S_ = 0;
      for (int w = 0; w < C::THREADS / 64; ++w) {
        L_ += red[w];
        S_ += red[16 + w];
      }
      if (GOK(&a.ctrl->epoch_sse, 8, 14)) atomicAdd(&a.ctrl->loss_sum, L_);
      atomicAdd(&a.ctrl->sse_sum, S_);
      atomicAdd(&a.ctrl->epoch_loss, L_);
      atomicAdd(&a.ctrl->epoch_sse, S_);
    }
    if (tid < H * (BM / 64)) {
      const int k = tid % H, rg = tid / H;
      const float w0 = a.W7[k], w1 = a.W7[H + k], w2 = a.W7[2 * H + k];
      float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f, db = 0.f;
#pragma unroll 4
      for (int r = rg * 64; r < rg * 64 + 64; ++r) {
        unsigned short* p = reinterpret_cast<unsigned short*>(act + act_off<H>(r, k));
        const float h = bf_val(*p);
        const float d0 = dzs[r * 3 + 0], d1 = dzs[r * 3 + 1], d2 = dzs[r * 3 + 2];
        float g = fmaf(d2, w2, fmaf(d1, w1, d0 * w0));
        g = h > 0.f ? g : 0.f;
        *p = bf_bits(g);
        cs += g;
        g0 = fmaf(d0, h, g0);
        g1 = fmaf(d1, h, g1);
        g2 = fmaf(d2, h, g2);
        if (k < 3) db += dzs[r * 3 + k];
      }
      const int64_t part = b0 / 64 + rg;
      if (GOK(&a.colsum[L - 2][part * H + k], 4, 15)) a.colsum[L - 2][part * H + k] = cs;
      if (!GOK(&a.hw_part[(part * 3 + 2) * H + k], 4, 16)) return;
      a.hw_part[(part * 3 + 0) * H + k] = g0;
      a.hw_part[(part * 3 + 1) * H + k] = g1;
      a.hw_part[(part * 3 + 2) * H + k] = g2;
      if (k < 3 && GOK(&a.hb_part[part * 3 + k], 4, 17)) a.hb_part[part * 3 + k] = db;
    }
  };

  auto write_dzt_head = [&]() {
    bf16* dzt = a.dZT[L - 2];
    constexpr int Q = BM / 8;
    for (int idx = tid; idx < H * Q; idx += C::THREADS) {
      const int k = idx / Q, q = idx - k * Q;
      u16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = *reinterpret_cast<const unsigned short*>(act + act_off<H>(q * 8 + e, k));
      if (GOK(dzt + (int64_t)k * a.ldt + b0 + q * 8, 16, 18)) *reinterpret_cast<u16x8*>(dzt + (int64_t)k * a.ldt + b0 + q * 8) = v;
    }
  };

  // ---- main loop over flat k-steps -----------------------------------------------
  zero_acc();
  prefetch(0, 0);
  stage_store(0, 0);
  __syncthreads();
  int p = 0;
#pragma unroll 1
  for (int step = 0; step < a.nsteps; ++step) {
    const int buf = step & 1;
    const bool more = step + 1 < a.nsteps;
    // the last step of phase p (the last phase ends at nsteps)
    const int phase_stop = (p + 1 < a.nphase) ? a.ph[p + 1].step0 : a.nsteps;
    const bool phase_end = step + 1 == phase_stop;
    const int pn = (more && phase_end) ? p + 1 : p;
    if (more) prefetch(step + 1, pn);
    compute(buf, p, step - a.ph[p].step0);
    if (more) stage_store(buf ^ 1, pn);
    __syncthreads();
    if (phase_end) {
      const ChainPhase& P = a.ph[p];
      if (P.epilogue) {
        if (P.kind == 0) fwd_epilogue(P.layer);
        else bwd_epilogue(P.layer);
        zero_acc();
        __syncthreads();
        if (P.kind == 0 && P.layer == L - 2) {
          head();
          if (a.train) {
            __syncthreads();
            head_bwd();
            __syncthreads();
            write_dzt_head();
            __syncthreads();
          }
        }
      }
      p = pn;
    }
  }
}

template <int H, int BM>
int launch_typed(const ChainArgs& a, hipStream_t stream) {
  constexpr int BK = BM == 128 ? 32 : 64;
  using C = CT<H, BM, BK>;
  static bool attr_set = false;
  if (!attr_set) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain_kernel<H, BM, BK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    C::LDS));
    attr_set = true;
  }
  chain_kernel<H, BM, BK><<<dim3((unsigned)(a.rows / BM)), dim3(C::THREADS), C::LDS, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_chain(const ChainArgs& a, int bm, hipStream_t stream) {
  INF_CHECK_ARG(chain_supported(a.H), "chain: unsupported hidden width");
  INF_CHECK_ARG(bm == 64 || bm == 128, "chain: tile height");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase >= 1 && a.nphase <= CHAIN_MAX_PHASES && a.nsteps >= 1, "chain: phases");
  INF_CHECK_ARG(a.L - 1 <= CHAIN_MAX_HIDDEN, "chain: too many layers");
  INF_CHECK_ARG(a.ldt % 8 == 0 && a.k_pad % 64 == 0, "chain: strides");
  if (a.H == 256) return bm == 128 ? launch_typed<256, 128>(a, stream) : launch_typed<256, 64>(a, stream);
  return bm == 128 ? launch_typed<128, 128>(a, stream) : launch_typed<128, 64>(a, stream);
}

}  // namespace inf
