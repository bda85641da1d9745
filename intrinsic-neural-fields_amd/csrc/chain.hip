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
// overwritten in place (a layer's accumulators stay in registers until every wave has
// finished reading the tile).  Only what the weight-gradient GEMM needs leaves the CU:
// Y_l^T and dZ_l^T (bf16, transposed), bias-gradient partials (one per PR rays) and the
// output layer's partial gradients.
//
// Weight stream.  Every workgroup reads every packed weight once per step (forward W,
// backward W^T), ~2.8 MB at config B, from L2 / the Infinity Cache: at small tiles the
// kernel is bound by how many of those bytes each CU keeps in flight, not by the MFMAs.
// The stream is a ring of NS stages filled by direct-to-LDS loads (global_load_lds,
// 1 KiB per wave instruction) NS-1 flat k-steps ahead -- across layer boundaries: the
// weights do not depend on the activations -- with one counted `s_waitcnt vmcnt` +
// barrier per step.  Nothing else the kernel reads from global memory is loaded while
// the ring runs: biases, the head weights, the targets (loaded before the ring starts)
// and the ReLU masks of the forward activations (wave ballots) live in LDS, so no
// epilogue load drains the ring.
//
// The tile height follows the batch (chain_bm): enough workgroups to cover the 256 CUs
// at the reference's 4096-ray batch (BM 16), taller tiles (more MFMA work per streamed
// byte) once the batch fills the chip several times over.
//
// Wave layout: WR x 4 waves (WR = max(1, BM/64)); a wave owns WROWS = min(BM, 64) rows x
// H/4 columns as (WROWS/16) x (H/64) v_mfma_f32_16x16x32_bf16 tiles, fp32 accumulators.
// LDS swizzles (16-byte chunk c of row r):
//   activation rows (>= 256 B): c ^ (r & 15)
//   stage rows of 128 B:        c ^ ((r >> 1) & 7)
//   stage rows of  64 B:        c ^ (3 * ((r >> 3) & 1))
// The stage image is lane-linear (lane l of a direct-to-LDS load writes bytes
// 16l..16l+15 of the instruction's 1 KiB), so the swizzle goes on the source address.
#include "chain.hpp"

#ifndef CHAIN_X_CPOL
#define CHAIN_X_CPOL 0  // cache policy of the feature-tile loads (2: non-temporal)
#endif

namespace inf {
namespace {

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr float CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
constexpr int LDS_CAP = 160 * 1024;

template <int H, int BM, int BK, int NS>
struct CT {
  static constexpr int WR = BM >= 64 ? BM / 64 : 1;
  static constexpr int WROWS = BM >= 64 ? 64 : BM;
  static constexpr int NW = 4 * WR;
  static constexpr int THREADS = 64 * NW;
  static constexpr int WN = H / 4;
  static constexpr int TM = WROWS / 16, TN = WN / 16;
  static constexpr int PR = WROWS;  // rays per bias / head partial
  static constexpr int ACT_ROW = H * 2;
  static constexpr int ROWB = BK * 2;
  static constexpr int CPR = BK / 8;    // 16-byte chunks per stage row
  static constexpr int RPI = 64 / CPR;  // stage rows per 1 KiB wave instruction
  static constexpr int W_BYTES = H * ROWB;
  static constexpr int X_BYTES = BM * ROWB;
  static constexpr int W_INS = W_BYTES / 1024 / NW;  // per wave per stage
  static constexpr int X_INS_ALL = X_BYTES / 1024;   // feature instructions per stage, all waves
  static constexpr int STAGE = W_BYTES + X_BYTES;
  static constexpr int MAXWAIT = (NS - 2) * (W_INS + (X_INS_ALL + NW - 1) / NW);
  // fixed LDS regions; the per-layer vectors and masks follow (sized from L at launch)
  static constexpr int OFF_ACT = 0;
  static constexpr int OFF_RING = BM * ACT_ROW;
  static constexpr int OFF_DZ = OFF_RING + NS * STAGE;  // [BM][3] f32 head gradient
  static constexpr int OFF_TGT = OFF_DZ + BM * 12;      // [BM][3] f32 targets
  static constexpr int OFF_RED = OFF_TGT + BM * 12;     // [2][16] f32
  static constexpr int OFF_W7 = OFF_RED + 128;          // [3][H] f32, then b7[3] (+pad)
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;
  static constexpr int MASK_BYTES = BM * H / 8;  // one layer of ReLU bits
  // the ReLU masks exist only for the backward chain: a forward-only (render) launch
  // leaves their LDS to a deeper weight ring
  static int lds_bytes(int L, bool train) {
    return OFF_VEC + L * H * 4 + (train && L > 2 ? (L - 2) : 0) * MASK_BYTES;
  }
  static_assert(W_BYTES % (1024 * NW) == 0, "weight stage must split into whole wave instructions");
  static_assert(X_BYTES % 1024 == 0, "feature stage must be whole wave instructions");
  static_assert(NS >= 2 && MAXWAIT <= 40, "ring depth");
};

template <int BK>
__device__ __forceinline__ int stage_swz(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  // 64-B rows: a ds_read_b128 lane group {0-3,12-15,20-27} reads rows 0-3 and 12-15 at
  // chunk c and rows 4-11 at chunk c+1 (4 rows per 256-B bank row); XOR 0 for row blocks
  // 0-1 and 3 for blocks 2-3 puts those 16 reads on 16 distinct slots (the old (r>>2)&3
  // left two per slot: SQ_LDS_BANK_CONFLICT was 43 % of the render chain's LDS cycles)
  else return ((row >> 3) & 1) * 3;
}

template <int BK>
__device__ __forceinline__ int stage_off(int row, int c) {
  return row * (BK * 2) + ((c ^ stage_swz<BK>(row)) << 4);
}

// Y^T / dZ^T as the chain writes them: 16-ray blocks, element (col, ray b) at
// (b / 16) * (H * 16) + col * 16 + b % 16 -- one 16-ray tile fills whole 128-byte lines
// (the dW GEMM reads this layout through GemmProblem::a_kblk / b_kblk).
template <int H>
__device__ __forceinline__ int64_t tofs(int col, int b) {
  return (int64_t)(b >> 4) * (H * 16) + col * 16 + (b & 15);
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

// s_waitcnt vmcnt(n) + s_barrier for a wave-uniform n in [0, N] (vmcnt takes an immediate)
template <int N>
__device__ __forceinline__ void wait_vm_barrier(int n) {
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    if (n >= N)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
    else
      wait_vm_barrier<N - 1>(n);
  }
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also fences global memory,
// which compiles to `s_waitcnt vmcnt(0)` and would drain the weight ring.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

template <int H, int BM, int BK, int NS>
__global__ __launch_bounds__((BM >= 64 ? BM / 64 : 1) * 256) void chain_kernel(const ChainArgs a) {
  using C = CT<H, BM, BK, NS>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act = smem + C::OFF_ACT;
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* red = reinterpret_cast<float*>(smem + C::OFF_RED);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);  // [3][H], then b7
  const int L = a.L;
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);  // biases [L-1][H], bias_y [H]
  unsigned long long* masks = reinterpret_cast<unsigned long long*>(smem + C::OFF_VEC + L * H * 4);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int wr = wave >> 2, wc = wave & 3;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;

  if (a.count_step && blockIdx.x == 0 && tid == 0 && GOK(&a.ctrl->step, 4, 1)) a.ctrl->step += 1;

  // ---- per-launch vectors into LDS, before the weight stream starts ---------------------
  for (int i = tid; i < (L - 1) * H; i += C::THREADS) {
    const float* src = a.bias[i / H] + (i % H);
    vecs[i] = GOK(src, 4, 4) ? *src : 0.f;
  }
  for (int i = tid; i < H; i += C::THREADS) vecs[(L - 1) * H + i] = GOK(a.bias_y + i, 4, 5) ? a.bias_y[i] : 0.f;
  for (int i = tid; i < 3 * H + 3; i += C::THREADS) {
    const float* src = i < 3 * H ? a.W7 + i : a.b7 + (i - 3 * H);
    w7s[i] = GOK(src, 4, 12) ? *src : 0.f;
  }
  if (a.train) {
    int64_t offset = a.idx_offset;
    if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
    for (int i = tid; i < BM * 3; i += C::THREADS) {
      const int b = b0 + i / 3;
      float t = 0.f;
      if (b < a.batch && a.rgb != nullptr && ray_in_range(offset, b, a.num_rays)) {
        const void* ip = a.idx_dtype == INF_DTYPE_I64 ? (const void*)((const int64_t*)a.ray_idx + offset + b)
                                                      : (const void*)((const int32_t*)a.ray_idx + offset + b);
        (void)ip;
        if (a.ray_idx == nullptr || GOK(ip, 4, 10)) {
          const int64_t rr = source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src);
          if (rr >= 0 && GOK(a.rgb + rr * 3 + i % 3, 4, 11)) t = a.rgb[rr * 3 + i % 3];
        }
      }
      tgs[i] = t;
    }
  }
  __syncthreads();

  // ---- the weight / feature ring ---------------------------------------------------------
  // wave wv fills weight rows [(wv*W_INS + i) * RPI, +RPI) and, in feature phases, feature
  // instructions q = wv + NW*i of the X tile (xw of them; waves past X_INS_ALL issue none)
  const int xw = C::X_INS_ALL / C::NW + (wv < C::X_INS_ALL % C::NW ? 1 : 0);
  const int lrow = lane / C::CPR, lslot = lane % C::CPR;
  int p_issue = 0;
  unsigned xbits = 0;  // bit s: ring slot s holds a feature stage
  auto issue = [&](int step) {
    while (p_issue + 1 < a.nphase && step >= a.ph[p_issue + 1].step0) ++p_issue;
    const ChainPhase& P = a.ph[p_issue];
    const int k0 = (step - P.step0) * BK;
    const int slot = step % NS;
    char* ws = smem + C::OFF_RING + slot * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::W_INS; ++i) {
      const int r0 = (wv * C::W_INS + i) * C::RPI;
      const int row = r0 + lrow;
      const bf16* src = P.B + (int64_t)row * P.ldb + k0 + ((lslot ^ stage_swz<BK>(row)) << 3);
      if (GOK(src, 16, 2)) __builtin_amdgcn_global_load_lds(src, (lds_void*)(ws + r0 * C::ROWB), 16, 0, 0);
    }
    if (P.a_src) {
      xbits |= 1u << slot;
      char* xs = ws + C::W_BYTES;
      for (int i = 0; i < xw; ++i) {
        const int r0 = (wv + C::NW * i) * C::RPI;
        const int row = r0 + lrow;
        const bf16* src = a.X + (int64_t)(b0 + row) * a.k_pad + k0 + ((lslot ^ stage_swz<BK>(row)) << 3);
        if (GOK(src, 16, 3)) __builtin_amdgcn_global_load_lds(src, (lds_void*)(xs + r0 * C::ROWB), 16, 0, CHAIN_X_CPOL);
      }
    } else {
      xbits &= ~(1u << slot);
    }
  };

  f32x4 acc[C::TM][C::TN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto compute = [&](int slot, bool from_x, int kt) {
    const char* ws = smem + C::OFF_RING + slot * C::STAGE;
    const char* xs = ws + C::W_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 av[C::TM], bv[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * C::WROWS + i * 16 + r16;
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

  // ReLU-mask word of accumulator register (i, j, r) of this wave: one ballot covers the
  // 4 rows x 16 columns of that register across the wave; bit = lane
  auto mask_word = [&](int layer, int i, int j, int r) -> unsigned long long* {
    return masks + layer * (C::MASK_BYTES / 8) + ((wave * C::TM + i) * C::TN + j) * 4 + r;
  };

  // forward epilogue of layer l: bias + ReLU -> activation tile (in place), Y_l^T, mask
  auto fwd_epilogue = [&](int l) {
    const float* bias = vecs + l * H;
    const bool skip = l == a.s;
    bf16* yt = a.save ? a.YT[l] : nullptr;
    const bool keep_mask = a.train && l <= L - 3;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = wc * C::WN + j * 16 + r16;
      const float bv = bias[col];
      const float by = skip ? vecs[(L - 1) * H + col] : 0.f;
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * C::WROWS + i * 16 + g4 * 4;
        u16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bv;
          if (skip) v += by;
          v = fmaxf(v, 0.f);
          q[r] = bf_bits(v);
          *reinterpret_cast<unsigned short*>(act + act_off<H>(row + r, col)) = q[r];
          if (keep_mask) {
            const unsigned long long bits = __ballot(bf_val(q[r]) > 0.f);
            if (lane == 0) *mask_word(l, i, j, r) = bits;
          }
        }
        if (yt != nullptr && GOK(yt + tofs<H>(col, b0 + row), 8, 6))
          *reinterpret_cast<u16x4*>(yt + tofs<H>(col, b0 + row)) = q;
      }
    }
  };

  // backward epilogue of layer l: mask by Y_{l-1} > 0 -> dZ_{l-1} (tile, ^T, bias partials)
  auto bwd_epilogue = [&](int l) {
    bf16* dzt = a.dZT[l - 1];
    const bool keep = (l - 1) >= 1;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int col = wc * C::WN + j * 16 + r16;
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const int row = wr * C::WROWS + i * 16 + g4 * 4;
        u16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool on = (*mask_word(l - 1, i, j, r) >> lane) & 1ull;
          const float v = on ? acc[i][j][r] : 0.f;
          cs += v;
          q[r] = bf_bits(v);
          if (keep) *reinterpret_cast<unsigned short*>(act + act_off<H>(row + r, col)) = q[r];
        }
        if (GOK(dzt + tofs<H>(col, b0 + row), 8, 8)) *reinterpret_cast<u16x4*>(dzt + tofs<H>(col, b0 + row)) = q;
      }
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      const int64_t part = b0 / C::PR + wr;
      if (g4 == 0 && GOK(&a.colsum[l - 1][part * H + col], 4, 9)) a.colsum[l - 1][part * H + col] = cs;
    }
  };

  // output layer + loss on the activation tile of layer L-2 (4 threads per ray)
  auto head = [&]() {
    const int ray = tid >> 2, part = tid & 3;
    const int b = b0 + ray;
    const bool in_tile = ray < BM;
    const bool valid = in_tile && b < a.batch;
    float z0 = 0.f, z1 = 0.f, z2 = 0.f;
    constexpr int CPP = H / 32;  // 16-byte chunks per thread
    if (in_tile) {
#pragma unroll
      for (int q = 0; q < CPP; ++q) {
        const int c = part * CPP + q;
        const u16x8 v = *reinterpret_cast<const u16x8*>(act + ray * C::ACT_ROW + ((c ^ (ray & 15)) << 4));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = c * 8 + e;
          const float h = bf_val(v[e]);
          z0 = fmaf(h, w7s[k], z0);
          z1 = fmaf(h, w7s[H + k], z1);
          z2 = fmaf(h, w7s[2 * H + k], z2);
        }
      }
    }
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
      z0 += __shfl_xor(z0, o, 4);
      z1 += __shfl_xor(z1, o, 4);
      z2 += __shfl_xor(z2, o, 4);
    }
    float lsum = 0.f, ssum = 0.f;
    if (in_tile && part < 3) {
      const float z = (part == 0 ? z0 : (part == 1 ? z1 : z2)) + w7s[3 * H + part];
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
          const float d = pv - tgs[ray * 3 + part];
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
    if (a.train && a.loss_part != nullptr) {
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

  // dZ_{L-2}, output-layer partial gradients, bias partials: one thread per column and
  // PR-row group
  auto head_bwd = [&]() {
    // per-tile partials (summed in a fixed order by the update launch's end-of-step item:
    // no same-address atomics from every workgroup, which the in-order vmcnt would wait on)
    if (a.loss_part != nullptr && tid == 0) {
      double L_ = 0, S_ = 0;
      for (int w = 0; w < C::NW; ++w) {
        L_ += red[w];
        S_ += red[16 + w];
      }
      if (GOK(a.loss_part + 2 * blockIdx.x + 1, 8, 14)) {
        a.loss_part[2 * blockIdx.x] = L_;
        a.loss_part[2 * blockIdx.x + 1] = S_;
      }
    }
    if (tid < H * C::WR) {
      const int k = tid % H, rg = tid / H;
      const float w0 = w7s[k], w1 = w7s[H + k], w2 = w7s[2 * H + k];
      float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f, db = 0.f;
#pragma unroll 4
      for (int r = rg * C::PR; r < rg * C::PR + C::PR; ++r) {
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
      const int64_t part = b0 / C::PR + rg;
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
      if (GOK(dzt + tofs<H>(k, b0 + q * 8), 16, 18)) *reinterpret_cast<u16x8*>(dzt + tofs<H>(k, b0 + q * 8)) = v;
    }
  };

  // ---- main loop over flat k-steps -------------------------------------------------------
  unsigned long long* stamp = nullptr;
  if (a.stamps != nullptr && tid == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    stamp = a.stamps + (blockIdx.x == 0 ? 0 : a.stamp_steps + 1);
  zero_acc();
  const int nsteps = a.nsteps;
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < nsteps) issue(q);
  int p = 0;
#pragma unroll 1
  for (int step = 0; step < nsteps; ++step) {
    // this wave's instructions of the stages after `step` that may stay in flight; other
    // memory operations issued since (epilogue stores) only make the wait stricter
    const int ahead = min(NS - 2, nsteps - 1 - step);
    int n = 0;
    for (int d = 1; d <= ahead; ++d) n += C::W_INS + (((xbits >> ((step + d) % NS)) & 1u) ? xw : 0);
    wait_vm_barrier<C::MAXWAIT>(n);
    if (stamp != nullptr && step < a.stamp_steps) stamp[step] = wall_clock64();
    if (step + NS - 1 < nsteps) issue(step + NS - 1);
    const ChainPhase& P = a.ph[p];
    compute(step % NS, P.a_src != 0, step - P.step0);
    const int phase_stop = (p + 1 < a.nphase) ? a.ph[p + 1].step0 : nsteps;
    if (step + 1 == phase_stop) {
      if (P.epilogue) {
        lds_barrier();  // every wave is done reading the activation tile
        if (P.kind == 0) fwd_epilogue(P.layer);
        else bwd_epilogue(P.layer);
        zero_acc();
        lds_barrier();
        if (P.kind == 0 && P.layer == L - 2) {
          head();
          if (a.train) {
            lds_barrier();
            head_bwd();
            lds_barrier();
            write_dzt_head();
            lds_barrier();
          }
        }
      }
      ++p;
    }
  }
  if (stamp != nullptr) stamp[a.stamp_steps] = wall_clock64();
}

template <int H, int BM, int BK, int NS>
int launch_typed(const ChainArgs& a, hipStream_t stream) {
  using C = CT<H, BM, BK, NS>;
  const int lds = C::lds_bytes(a.L, a.train != 0);
  INF_CHECK_ARG(lds <= LDS_CAP, "chain: LDS budget exceeded for this depth");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain_kernel<H, BM, BK, NS>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  chain_kernel<H, BM, BK, NS><<<dim3((unsigned)(a.rows / BM)), dim3(C::THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

// deepest ring that fits the LDS for this depth
template <int H, int BM, int BK, int NS_HI, int NS_LO>
int launch_fit(const ChainArgs& a, hipStream_t stream) {
  if (CT<H, BM, BK, NS_HI>::lds_bytes(a.L, a.train != 0) <= LDS_CAP) return launch_typed<H, BM, BK, NS_HI>(a, stream);
  return launch_typed<H, BM, BK, NS_LO>(a, stream);
}

template <int H>
int launch_h(const ChainArgs& a, int bm, hipStream_t stream) {
  switch (bm) {
    case 16: return launch_fit<H, 16, 64, 4, 3>(a, stream);
    case 32: return launch_fit<H, 32, 64, 3, 2>(a, stream);
    case 64: return launch_fit<H, 64, 32, 4, 2>(a, stream);
    default: return launch_fit<H, 128, 32, 3, 2>(a, stream);
  }
}

}  // namespace

int launch_chain(const ChainArgs& a, int bm, hipStream_t stream) {
  INF_CHECK_ARG(chain_supported(a.H), "chain: unsupported hidden width");
  INF_CHECK_ARG(bm == 16 || bm == 32 || bm == 64 || bm == 128, "chain: tile height");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase >= 1 && a.nphase <= CHAIN_MAX_PHASES && a.nsteps >= 1, "chain: phases");
  INF_CHECK_ARG(a.L - 1 <= CHAIN_MAX_HIDDEN, "chain: too many layers");
  INF_CHECK_ARG(a.ldt % 8 == 0 && a.k_pad % 64 == 0, "chain: strides");
  if (a.H == 256) return launch_h<256>(a, bm, stream);
  return launch_h<128>(a, bm, stream);
}

}  // namespace inf
