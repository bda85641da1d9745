// Register-streamed fused MLP chain: the bf16 training step of small batches (the
// reference's 4096-ray batch, intrinsic_cat.yaml:32) after the input GEMM.
//
// One workgroup owns BM = 16*TM rays and runs, in ONE launch:
//   forward   hidden layers 1..L-2 (model.py:98-112); layer 0 and the skip layer's data
//             term Ly(x) + Ly.bias come precomputed from the input GEMM (Y_0, Z_y), so
//             the skip layer here is relu(Lx(h) + Lx.bias + Z_y) (layers.py:60-62),
//   head      Linear(H,3) + sigmoid (model.py:89-94), loss (config.py:113-122),
//             dL/dz = dL/dp * p (1 - p),
//   backward  dZ_{L-2} = (dz W_head) * (h > 0), then dZ_{l-1} = (dZ_l W_l) * (Y_{l-1} > 0)
//             for l = L-2..1 (autograd of trainer.py:81).
//
// Why registers, not an LDS ring.  At 16 rays per workgroup every weight element feeds
// exactly one wave (the 4 waves split the output columns), so staging weights through
// LDS buys no reuse; what bounds the kernel is how many weight bytes each CU keeps in
// flight.  The packed weights are stored in MFMA fragment order (adam.hip: 1 KiB per
// 16 columns x 32 k, lane l's 16 bytes at 16 l), so a wave's B operand for one 32-deep k
// block is TN coalesced 1 KiB loads straight into VGPRs.  Each wave holds one whole
// phase of fragments (UPL x TN x 16 B per lane = 128 VGPRs at H = 256) and refills slot
// kb with the NEXT phase's block kb right after its MFMAs consumed it: the next layer's
// weights (128 KiB per CU) stream in while this one computes, across the epilogue, with
// no per-k-step barrier.  The only vector-memory instructions of the compute waves are
// these loads, so the compiler's vmcnt waits are exact (each waits for one block).
//
// Stores.  Every global output (Y^T, dZ^T, bias / output-layer partials, loss, pred) is
// written into an LDS box by the compute waves and copied out by a fifth "store" wave
// that mirrors the compute waves' barriers.  Stores in the compute waves would join the
// in-order vmcnt queue and make the next fragment wait for their completion.
#include "chain3.hpp"

namespace inf {
namespace {

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr float C3_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
constexpr int C3_THREADS = 320;  // 4 compute waves + 1 store wave
constexpr int C3_LDS_CAP = 160 * 1024;

template <int H, int TM>
struct L3 {
  static constexpr int BM = 16 * TM;
  static constexpr int TN = H / 64;   // 16-column tiles per wave (a wave owns H/4 columns)
  static constexpr int WN = H / 4;
  static constexpr int UPL = H / 32;  // 32-deep k blocks per phase
  static constexpr int NT = H / 16;   // 16-column tiles per k block of a weight image
  static constexpr int ACT_ROW = H * 2;
  static constexpr int ZY_LD = H + 4;  // floats; 4 row groups of a wave land on distinct banks
  static constexpr int TILE_BYTES = BM * H * 2;
  static constexpr int BOX_BYTES = TILE_BYTES + H * 4;  // Y^T / dZ^T tile + bias partial
  static constexpr int OFF_ACT = 0;
  static constexpr int OFF_ZY = OFF_ACT + BM * ACT_ROW;
  static constexpr int OFF_BOX = OFF_ZY + BM * ZY_LD * 4;
  static constexpr int OFF_HW = OFF_BOX + 2 * BOX_BYTES;  // [3][H] output-layer weight grad
  static constexpr int OFF_HB = OFF_HW + 3 * H * 4;       // [4]
  static constexpr int OFF_LS = OFF_HB + 16;              // [2] f64 loss / SSE
  static constexpr int OFF_PRED = OFF_LS + 16;            // [BM][3]
  static constexpr int OFF_DZ = OFF_PRED + BM * 12;       // [BM][3] head gradient
  static constexpr int OFF_TGT = OFF_DZ + BM * 12;        // [BM][3] targets
  static constexpr int OFF_RED = OFF_TGT + BM * 12;       // [16] per-wave loss / SSE
  static constexpr int OFF_W7 = OFF_RED + 64;             // [3][H] then b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16; // biases [L-1][H]
  static constexpr int MASK_BYTES = BM * H / 8;           // ReLU bits of one layer
  static int lds_bytes(int L) { return OFF_VEC + (L - 1) * H * 4 + (L - 2) * MASK_BYTES; }
  // initial tile loads per compute thread
  static constexpr int YPT = BM * H / 8 / 256;   // 16-byte chunks of Y_0
  static constexpr int ZPT = BM * H / 4 / 256;   // 16-byte chunks of Z_y
  static_assert(BM * H / 8 % 256 == 0 && BM * H / 4 % 256 == 0, "tile loads");
};

template <int H>
__device__ __forceinline__ int act_off3(int row, int col) {
  return row * (H * 2) + (((col >> 3) ^ (row & 15)) << 4) + ((col & 7) << 1);
}

// element (col, ray r) of a box tile: the 16-ray blocked layout of the dW GEMM operands
// (gemm.hpp a_kblk / b_kblk), whole tile contiguous in global memory
template <int H>
__device__ __forceinline__ int box_off(int col, int r) {
  return (((r >> 4) * H + col) * 16 + (r & 15)) * 2;
}

__device__ __forceinline__ unsigned short bf_bits3(float x) {
  bf16 h = (bf16)x;
  return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float bf_val3(unsigned short u) { return (float)__builtin_bit_cast(bf16, u); }

// LDS hand-off barrier that does not drain the vector-memory queue (__syncthreads()
// would add `s_waitcnt vmcnt(0)` and stall on the weight fragments in flight)
__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int H, int TM>
__global__ __launch_bounds__(C3_THREADS) void chain3_kernel(const Chain3Args a) {
  using C = L3<H, TM>;
  constexpr int BM = C::BM, TN = C::TN, UPL = C::UPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act = smem + C::OFF_ACT;
  float* zy = reinterpret_cast<float*>(smem + C::OFF_ZY);
  float* hws = reinterpret_cast<float*>(smem + C::OFF_HW);
  float* hbs = reinterpret_cast<float*>(smem + C::OFF_HB);
  double* lss = reinterpret_cast<double*>(smem + C::OFF_LS);
  float* preds = reinterpret_cast<float*>(smem + C::OFF_PRED);
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* red = reinterpret_cast<float*>(smem + C::OFF_RED);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  const int L = a.L;
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  unsigned long long* masks = reinterpret_cast<unsigned long long*>(smem + C::OFF_VEC + (L - 1) * H * 4);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int nphase = a.nphase;
  const int nfwd = L - 2;

  // ---- per-launch vectors and targets (all waves) ---------------------------------------
  if (a.count_step && blockIdx.x == 0 && tid == 0) a.ctrl->step += 1;
  for (int i = tid; i < (L - 1) * H; i += C3_THREADS) vecs[i] = a.bias[i / H][i % H];
  for (int i = tid; i < 3 * H + 3; i += C3_THREADS) w7s[i] = i < 3 * H ? a.W7[i] : a.b7[i - 3 * H];
  {
    int64_t offset = a.idx_offset;
    if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
    for (int i = tid; i < BM * 3; i += C3_THREADS) {
      const int b = b0 + i / 3;
      float t = 0.f;
      if (b < a.batch && ray_in_range(offset, b, a.num_rays)) {
        const int64_t rr = ray_row(a.ray_idx, a.idx_dtype, offset, b);
        t = a.rgb[rr * 3 + i % 3];
      }
      tgs[i] = t;
    }
  }

  if (wave < 4) {
    // =========================== compute waves ============================================
    const int wc = wave;
    // Y_0 / Z_y tiles into registers first, then the first phase's fragments: the
    // compiler's wait for the tile loads then leaves the fragments in flight
    u16x8 yv[C::YPT];
    f32x4 zv[C::ZPT];
#pragma unroll
    for (int q = 0; q < C::YPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 8), ch = c % (H / 8);
      yv[q] = *reinterpret_cast<const u16x8*>(a.Y0 + (int64_t)(b0 + row) * H + ch * 8);
    }
#pragma unroll
    for (int q = 0; q < C::ZPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 4), ch = c % (H / 4);
      zv[q] = *reinterpret_cast<const f32x4*>(a.Zy + (int64_t)(b0 + row) * H + ch * 4);
    }
    bf16x8 fr[UPL][TN];
    const int64_t lane_off = ((int64_t)wc * TN * 64 + lane) * 8;
    {
      const bf16* base = a.img[0] + lane_off;
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j) fr[kb][j] = *reinterpret_cast<const bf16x8*>(base + (kb * C::NT + j) * 512);
        // keep block order: the loop's waits assume block kb was issued before kb + 1
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int q = 0; q < C::YPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 8), ch = c % (H / 8);
      *reinterpret_cast<u16x8*>(act + row * C::ACT_ROW + ((ch ^ (row & 15)) << 4)) = yv[q];
    }
#pragma unroll
    for (int q = 0; q < C::ZPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 4), ch = c % (H / 4);
      *reinterpret_cast<f32x4*>(zy + row * C::ZY_LD + ch * 4) = zv[q];
    }
    lbar();  // tiles and vectors in LDS

    auto mask_word = [&](int layer, int i, int j, int r) -> unsigned long long* {
      return masks + layer * (C::MASK_BYTES / 8) + ((wc * TM + i) * TN + j) * 4 + r;
    };
    // ReLU bits of Y_0 (the last backward phase masks dZ_0 with them)
    if (nfwd >= 1) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wc * C::WN + j * 16 + r16;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = i * 16 + g4 * 4 + r;
            const float h = bf_val3(*reinterpret_cast<const unsigned short*>(act + act_off3<H>(row, col)));
            const unsigned long long bits = __ballot(h > 0.f);
            if (lane == 0) *mask_word(0, i, j, r) = bits;
          }
      }
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      // ---- MFMAs of phase p; slot kb refilled with phase p+1 (the last phase reloads
      // itself: a few harmless extra loads keep every wait exact)
      const bf16* nbase = a.img[p + 1 < nphase ? p + 1 : p] + lane_off;
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
        bf16x8 av[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = i * 16 + r16;
          av[i] = *reinterpret_cast<const bf16x8*>(act + row * C::ACT_ROW + (((kb * 4 + g4) ^ (row & 15)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], fr[kb][j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j) fr[kb][j] = *reinterpret_cast<const bf16x8*>(nbase + (kb * C::NT + j) * 512);
        __builtin_amdgcn_sched_barrier(0);
      }

      // ---- epilogue ----------------------------------------------------------------
      lbar();  // B1: every wave is done reading the activation tile
      char* box = smem + C::OFF_BOX + (p & 1) * C::BOX_BYTES;
      float* csb = reinterpret_cast<float*>(box + C::TILE_BYTES);
      if (p < nfwd) {
        // forward of layer l: bias (+ Z_y at the skip layer) + ReLU -> tile, Y^T, mask
        const int l = p + 1;
        const float* bias = vecs + l * H;
        const bool skip = l == a.s;
        const bool keep = l <= L - 3;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * C::WN + j * 16 + r16;
          const float bv = bias[col];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int row0 = i * 16 + g4 * 4;
            u16x4 q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[i][j][r] + bv;
              if (skip) v += zy[(row0 + r) * C::ZY_LD + col];
              v = fmaxf(v, 0.f);
              q[r] = bf_bits3(v);
              *reinterpret_cast<unsigned short*>(act + act_off3<H>(row0 + r, col)) = q[r];
              if (keep) {
                const unsigned long long bits = __ballot(bf_val3(q[r]) > 0.f);
                if (lane == 0) *mask_word(l, i, j, r) = bits;
              }
            }
            if (keep) *reinterpret_cast<u16x4*>(box + box_off<H>(col, row0)) = q;
          }
        }
        if (l == L - 2) {
          lbar();  // Bh1: last hidden activation complete
          // head + loss, 4 threads per ray (model.py:89-94, config.py:113-122)
          {
            const int ray = tid >> 2, part = tid & 3;
            const int b = b0 + ray;
            const bool in_tile = ray < BM;
            const bool valid = in_tile && b < a.batch;
            float z0 = 0.f, z1 = 0.f, z2 = 0.f;
            constexpr int CPP = H / 32;
            if (in_tile) {
#pragma unroll
              for (int q = 0; q < CPP; ++q) {
                const int c = part * CPP + q;
                const u16x8 v = *reinterpret_cast<const u16x8*>(act + ray * C::ACT_ROW + ((c ^ (ray & 15)) << 4));
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                  const int k = c * 8 + e;
                  const float h = bf_val3(v[e]);
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
              preds[ray * 3 + part] = pv;
              float dz = 0.f;
              if (valid) {
                const float d = pv - tgs[ray * 3 + part];
                float lv, g;
                if (a.loss == INF_LOSS_L2) {
                  lv = d * d;
                  g = 2.f * d;
                } else if (a.loss == INF_LOSS_L1) {
                  lv = fabsf(d);
                  g = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                } else {
                  const float qq = d * d / C3_CAUCHY_C2;
                  lv = C3_CAUCHY_C2 * logf(1.f + qq);
                  g = 2.f * d / (1.f + qq);
                }
                dz = (g * a.inv_count) * (1.f - pv) * pv;
                lsum = lv;
                ssum = d * d;
              }
              dzs[ray * 3 + part] = dz;
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
              lsum += __shfl_xor(lsum, o, 64);
              ssum += __shfl_xor(ssum, o, 64);
            }
            if (lane == 0) {
              red[wc] = lsum;
              red[8 + wc] = ssum;
            }
          }
          lbar();  // Bh2: dz, per-wave loss sums
          // head backward: dZ_{L-2} (in place), its bias partial, output-layer partials
          if (tid == 0) {
            double L_ = 0, S_ = 0;
            for (int w = 0; w < 4; ++w) {
              L_ += red[w];
              S_ += red[8 + w];
            }
            lss[0] = L_;
            lss[1] = S_;
          }
          if (tid < H) {
            const int k = tid;
            const float w0 = w7s[k], w1 = w7s[H + k], w2 = w7s[2 * H + k];
            float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f, db = 0.f;
#pragma unroll 4
            for (int r = 0; r < BM; ++r) {
              unsigned short* hp = reinterpret_cast<unsigned short*>(act + act_off3<H>(r, k));
              const float h = bf_val3(*hp);
              const float d0 = dzs[r * 3 + 0], d1 = dzs[r * 3 + 1], d2 = dzs[r * 3 + 2];
              float g = fmaf(d2, w2, fmaf(d1, w1, d0 * w0));
              g = h > 0.f ? g : 0.f;
              const unsigned short gb = bf_bits3(g);
              *hp = gb;
              *reinterpret_cast<unsigned short*>(box + box_off<H>(k, r)) = gb;
              cs += g;
              g0 = fmaf(d0, h, g0);
              g1 = fmaf(d1, h, g1);
              g2 = fmaf(d2, h, g2);
              if (k < 3) db += dzs[r * 3 + k];
            }
            csb[k] = cs;
            hws[k] = g0;
            hws[H + k] = g1;
            hws[2 * H + k] = g2;
            if (k < 3) hbs[k] = db;
          }
        }
      } else {
        // dX of layer l masked by Y_{l-1} > 0 -> dZ_{l-1} (tile, dZ^T, bias partial)
        const int l = (L - 2) - (p - nfwd);
        const bool keep_act = l - 1 >= 1;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * C::WN + j * 16 + r16;
          float cs = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int row0 = i * 16 + g4 * 4;
            u16x4 q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const bool on = (*mask_word(l - 1, i, j, r) >> lane) & 1ull;
              const float v = on ? acc[i][j][r] : 0.f;
              cs += v;
              q[r] = bf_bits3(v);
              if (keep_act) *reinterpret_cast<unsigned short*>(act + act_off3<H>(row0 + r, col)) = q[r];
            }
            *reinterpret_cast<u16x4*>(box + box_off<H>(col, row0)) = q;
          }
          cs += __shfl_xor(cs, 16, 64);
          cs += __shfl_xor(cs, 32, 64);
          if (g4 == 0) csb[col] = cs;
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      lbar();  // B2: tile of the next phase and this phase's box complete
    }
  } else {
    // =========================== store wave ===============================================
    lbar();
    const int64_t tile_elems = (int64_t)(b0 / 16) * H * 16;
    auto copy_out = [&](const char* src, void* dst, int bytes) {
      char* d = reinterpret_cast<char*>(dst);
      for (int c = lane * 16; c < bytes; c += 64 * 16)
        *reinterpret_cast<u16x8*>(d + c) = *reinterpret_cast<const u16x8*>(src + c);
    };
#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      lbar();  // B1
      const bool head_phase = p == nfwd - 1;
      if (head_phase) {
        lbar();  // Bh1
        lbar();  // Bh2
      }
      lbar();  // B2
      const char* box = smem + C::OFF_BOX + (p & 1) * C::BOX_BYTES;
      const char* csb = box + C::TILE_BYTES;
      if (p < nfwd) {
        const int l = p + 1;
        if (l <= L - 3) copy_out(box, a.YT[l] + tile_elems, C::TILE_BYTES);
        if (head_phase) {
          copy_out(box, a.dZT[L - 2] + tile_elems, C::TILE_BYTES);
          copy_out(csb, a.colsum[L - 2] + (int64_t)blockIdx.x * H, H * 4);
          copy_out(reinterpret_cast<const char*>(hws), a.hw_part + (int64_t)blockIdx.x * 3 * H, 3 * H * 4);
          if (lane < 3) a.hb_part[(int64_t)blockIdx.x * 3 + lane] = hbs[lane];
          if (lane < 2 && a.loss_part != nullptr) a.loss_part[2 * (int64_t)blockIdx.x + lane] = lss[lane];
          if (a.pred != nullptr)
            for (int c = lane; c < BM * 3; c += 64)
              if (b0 + c / 3 < a.batch) a.pred[(int64_t)b0 * 3 + c] = preds[c];
        }
      } else {
        const int l = (L - 2) - (p - nfwd);
        copy_out(box, a.dZT[l - 1] + tile_elems, C::TILE_BYTES);
        copy_out(csb, a.colsum[l - 1] + (int64_t)blockIdx.x * H, H * 4);
      }
    }
  }
}

template <int H, int TM>
int launch3_typed(const Chain3Args& a, hipStream_t stream) {
  using C = L3<H, TM>;
  const int lds = C::lds_bytes(a.L);
  INF_CHECK_ARG(lds <= C3_LDS_CAP, "chain3: LDS budget exceeded for this depth");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain3_kernel<H, TM>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    lds));
    attr_set = lds;
  }
  chain3_kernel<H, TM><<<dim3((unsigned)(a.rows / C::BM)), dim3(C3_THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_chain3(const Chain3Args& a, int bm, hipStream_t stream) {
  INF_CHECK_ARG(chain3_supported(a.H, a.L, a.rows), "chain3: unsupported shape");
  INF_CHECK_ARG(bm == 16, "chain3: tile height");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain3: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase == 2 * (a.L - 2), "chain3: phases");
  INF_CHECK_ARG(a.rgb != nullptr && a.Y0 != nullptr && a.Zy != nullptr, "chain3: inputs");
  for (int p = 0; p < a.nphase; ++p) INF_CHECK_ARG(a.img[p] != nullptr, "chain3: weight image missing");
  if (a.H == 256) return launch3_typed<256, 1>(a, stream);
  return launch3_typed<128, 1>(a, stream);
}

}  // namespace inf
