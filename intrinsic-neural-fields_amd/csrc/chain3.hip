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
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr float C3_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
constexpr int C3_THREADS = 320;  // 4 compute waves + 1 store wave
constexpr int C3_LDS_CAP = 160 * 1024;
#ifndef C3_DEPTH
#define C3_DEPTH 4
#endif

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
  static constexpr int OFF_DZ = OFF_PRED + BM * 12;       // [4 waves][BM][3] head gradient
  static constexpr int OFF_TGT = OFF_DZ + 4 * BM * 12;    // [BM][3] targets
  static constexpr int OFF_ZP = OFF_TGT + BM * 12;        // [4 waves][BM][3] head partial sums
  static constexpr int OFF_W7 = OFF_ZP + 4 * BM * 12;     // [3][H] then b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16; // biases [L-1][H]
  // ReLU bits: per layer one 32-bit word per compute lane, bit (i*TN + j)*4 + r for
  // accumulator element (i, j, r) of that lane
  static constexpr int MASK_BYTES = 256 * 4;
  __host__ __device__ static int off_mask(int L) { return OFF_VEC + (L - 1) * H * 4; }
  __host__ __device__ static int off_stamp(int L) { return off_mask(L) + (L - 2) * MASK_BYTES; }
  static int lds_bytes(int L) { return off_stamp(L) + (3 * 2 * CHAIN_MAX_HIDDEN + 8) * 8; }
  static constexpr int YPT = BM * H / 8 / 256;   // 16-byte chunks of Y_0 per compute thread
  static_assert(BM * H / 8 % 256 == 0 && BM * H / 4 % 256 == 0, "tile loads");
  static_assert(TM * TN * 4 <= 32, "ReLU bits of a lane must fit one word");
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

// element (col, ray r < 16) of a workgroup's dZ^T box: the fragment image the dW GEMM
// streams (lgemm.hip operand B: rows = columns of dZ, k = rays): per 16-column tile one
// 512-byte piece = the workgroup's half (16 of 32 rays) of that tile's 1 KiB k-block
__device__ __forceinline__ int frag_box_off(int col, int r) {
  return (col >> 4) * 512 + ((col & 15) + 16 * (r >> 3)) * 16 + (r & 7) * 2;
}

__device__ __forceinline__ unsigned short bf_bits3(float x) {
  bf16 h = (bf16)x;
  return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float bf_val3(unsigned short u) { return (float)__builtin_bit_cast(bf16, u); }

// Sum over the 16 lanes of a row (lanes 16 q .. 16 q + 15) with DPP adds.
__device__ __forceinline__ float row_sum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// Sum over lanes l, l ^ 16, l ^ 32, l ^ 48 (the four row groups of an accumulator column)
// with the gfx950 permlane swaps.  v_permlane16_swap x, y exchanges the odd 16-lane rows
// of x with the even rows of y: on two copies of v, x becomes v with odd rows <- even rows
// and y v with even rows <- odd rows, so x + y is the partner sum in every lane (32: the
// same with halves).  Inline asm: the ROCm 7.2 builtin returned the first register twice.
__device__ __forceinline__ float col_sum4(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  v = x + y;
  x = v;
  y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  return x + y;
}

// LDS hand-off barrier that does not drain the vector-memory queue (__syncthreads()
// would add `s_waitcnt vmcnt(0)` and stall on the weight fragments in flight)
__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int H, int TM, int LOSS>
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
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  const int L = a.L;
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  unsigned* maskw = reinterpret_cast<unsigned*>(smem + C::off_mask(L));

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int nphase = a.nphase;
  const int nfwd = L - 2;

  unsigned long long* stl = nullptr;  // diagnostics only
  if (a.stamps != nullptr && wave == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    stl = reinterpret_cast<unsigned long long*>(smem + C::off_stamp(L));
  const unsigned long long t_entry = stl != nullptr ? wall_clock64() : 0ull;
  auto stamp = [&](int i) {
    if (stl != nullptr) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = wall_clock64();
      if (lane == 0) stl[i] = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };


  if (wave < 4) {
    // =========================== compute waves ============================================
    const int wc = wave;
    // Y_0 / Z_y tiles into registers first, then the first phase's fragments: the
    // compiler's wait for the tile loads then leaves the fragments in flight
    u16x8 yv[C::YPT];
#pragma unroll
    for (int q = 0; q < C::YPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 8), ch = c % (H / 8);
      yv[q] = *reinterpret_cast<const u16x8*>(a.Y0 + (int64_t)(b0 + row) * H + ch * 8);
    }
    // fragment ring: D k-blocks (D * TN KiB per wave) in flight; 16 KiB per wave kept the
    // L2 -> CU stream at its best rate in tools/microbench/l2ring (32 KiB: -35 %)
    constexpr int D = C3_DEPTH < UPL ? C3_DEPTH : UPL;
    bf16x8 fr[D][TN];
    // byte offset of this lane's 16 bytes in a wave's TN KiB of one k block; the block
    // base stays uniform (SGPR) so every load is saddr + lane offset + immediate
    // buffer loads: descriptor per image in SGPRs, k-block offset in soffset, tile offset
    // as the immediate, one VGPR of lane offset -- no 64-bit address registers
    const unsigned lane_off = (unsigned)(wc * TN * 64 + lane) * 16u;
    auto rsrc_of = [&](const bf16* img) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, H * H * 2, 0x00020000);
    };
    auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j) -> bf16x8 {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024, kb * C::NT * 1024, 0);
      return __builtin_bit_cast(bf16x8, v);
    };
    {
      const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(a.img[0]);
#pragma unroll
      for (int kb = 0; kb < D; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j) fr[kb][j] = frag(rs0, kb, j);
        // keep block order: the loop's waits assume block kb was issued before kb + 1
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stamp(3 * nphase + 3);
#pragma unroll
    for (int q = 0; q < C::YPT; ++q) {
      const int c = tid + 256 * q, row = c / (H / 8), ch = c % (H / 8);
      *reinterpret_cast<u16x8*>(act + row * C::ACT_ROW + ((ch ^ (row & 15)) << 4)) = yv[q];
    }
    stamp(3 * nphase + 4);
    lbar();  // barrier 0: Y_0 tile in LDS
    stamp(3 * nphase + 5);

    unsigned* my_mask = maskw + tid;  // + layer * 256
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      stamp(1 + 3 * p);
      // ---- MFMAs of phase p; slot kb % D refilled with k-block kb + D of this phase or
      // of phase p+1 (the last phase reloads itself: harmless extra loads keep every wait
      // exact)
      const __amdgpu_buffer_rsrc_t crs = rsrc_of(a.img[p]);
      const __amdgpu_buffer_rsrc_t nrs = rsrc_of(a.img[p + 1 < nphase ? p + 1 : p]);
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
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], fr[kb % D][j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fr[kb % D][j] = kb + D < UPL ? frag(crs, kb + D, j) : frag(nrs, kb + D - UPL, j);
        __builtin_amdgcn_sched_barrier(0);
      }

      // ---- epilogue: LDS reads first, then arithmetic, then LDS writes ----------------
      stamp(2 + 3 * p);
      lbar();  // B1: every wave is done reading the activation tile
      char* box = smem + C::OFF_BOX + (p & 1) * C::BOX_BYTES;
      float* csb = reinterpret_cast<float*>(box + C::TILE_BYTES);
      if (p < nfwd) {
        // forward of layer l: bias (+ Z_y at the skip layer) + ReLU -> tile, Y^T, ReLU bits
        const int l = p + 1;
        const bool skip = l == a.s;
        const bool last = l == L - 2;
        float bv[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = vecs[l * H + wc * C::WN + j * 16 + r16];
        float hq[TM][TN][4];  // bf16-rounded activations as f32
        if (skip) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                hq[i][j][r] = zy[(i * 16 + g4 * 4 + r) * C::ZY_LD + wc * C::WN + j * 16 + r16];
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r) hq[i][j][r] = 0.f;
        }
        unsigned bits = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[i][j][r] + bv[j];
              if (skip) v += hq[i][j][r];
              v = fmaxf(v, 0.f);
              hq[i][j][r] = bf_val3(bf_bits3(v));
              bits |= (hq[i][j][r] > 0.f ? 1u : 0u) << ((i * TN + j) * 4 + r);
            }
        if (!last) {
          my_mask[l * 256] = bits;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = wc * C::WN + j * 16 + r16;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const int row0 = i * 16 + g4 * 4;
              u16x4 q;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                q[r] = bf_bits3(hq[i][j][r]);
                *reinterpret_cast<unsigned short*>(act + act_off3<H>(row0 + r, col)) = q[r];
              }
              if (l <= L - 3) *reinterpret_cast<u16x4*>(box + box_off<H>(col, row0)) = q;
            }
          }
        } else {
          // ---- head on the registers of the last hidden layer (model.py:89-94) ----------
          // (W7 is read from LDS twice rather than held across the loss code: registers)
          float w7r[3][TN];
          auto load_w7 = [&]() {
#pragma unroll
            for (int o = 0; o < 3; ++o)
#pragma unroll
              for (int j = 0; j < TN; ++j) w7r[o][j] = w7s[o * H + wc * C::WN + j * 16 + r16];
          };
          load_w7();
          // z partials over this lane's columns, reduced over the 16 lanes of a row group
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int o = 0; o < 3; ++o) {
                float z = 0.f;
#pragma unroll
                for (int j = 0; j < TN; ++j) z = fmaf(hq[i][j][r], w7r[o][j], z);
                z = row_sum16(z);
                if (r16 == 0) zps[(wc * BM + i * 16 + g4 * 4 + r) * 3 + o] = z;
              }
          lbar();  // Bh1: per-wave head partial sums complete
          // sigmoid, loss and dL/dz (model.py:89-94, config.py:113-122, trainer.py:76):
          // every compute wave computes all BM x 3 of them (one lane each) into its own
          // copy of dz, so only same-wave LDS ordering is needed, no second barrier
          {
            float* dzw = dzs + wc * BM * 3;
            float lsum = 0.f, ssum = 0.f;
            if (lane < BM * 3) {
              const int b = b0 + lane / 3, o = lane % 3;
              float z = w7s[3 * H + o];
#pragma unroll
              for (int w = 0; w < 4; ++w) z += zps[w * BM * 3 + lane];
              const float pv = 1.f / (1.f + expf(-z));
              float dz = 0.f;
              if (b < a.batch) {
                const float d = pv - tgs[lane];
                float lv, g;
                if constexpr (LOSS == INF_LOSS_L2) {
                  lv = d * d;
                  g = 2.f * d;
                } else if constexpr (LOSS == INF_LOSS_L1) {
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
              dzw[lane] = dz;
              if (wc == 0) preds[lane] = pv;
            }
            static_assert(BM * 3 <= 64, "one lane per (ray, output)");
            if (wc == 0) {  // all 64 lanes active for the cross-lane sums
              lsum = col_sum4(row_sum16(lsum));
              ssum = col_sum4(row_sum16(ssum));
              if (lane == 0) {
                lss[0] = lsum;
                lss[1] = ssum;
              }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's dz writes
          }
          // head backward in registers: dZ_{L-2} = (dz W7) * (h > 0), its column sums, and
          // the output layer's weight-gradient partials sum_rays dz_o * h
          load_w7();
          float dzr[TM][4][3];
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int o = 0; o < 3; ++o) dzr[i][r][o] = dzs[wc * BM * 3 + (i * 16 + g4 * 4 + r) * 3 + o];
          if (tid < 3) {
            float db = 0.f;
            for (int r = 0; r < BM; ++r) db += dzs[r * 3 + tid];
            hbs[tid] = db;
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = wc * C::WN + j * 16 + r16;
            float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const int row0 = i * 16 + g4 * 4;
              u16x4 q;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float h = hq[i][j][r];
                const float d0 = dzr[i][r][0], d1 = dzr[i][r][1], d2 = dzr[i][r][2];
                float g = fmaf(d2, w7r[2][j], fmaf(d1, w7r[1][j], d0 * w7r[0][j]));
                g = h > 0.f ? g : 0.f;
                q[r] = bf_bits3(g);
                *reinterpret_cast<unsigned short*>(act + act_off3<H>(row0 + r, col)) = q[r];
                cs += g;
                g0 = fmaf(d0, h, g0);
                g1 = fmaf(d1, h, g1);
                g2 = fmaf(d2, h, g2);
              }
              *reinterpret_cast<u16x4*>(box + frag_box_off(col, row0)) = q;
            }
            cs = col_sum4(cs);
            g0 = col_sum4(g0);
            g1 = col_sum4(g1);
            g2 = col_sum4(g2);
            if (g4 == 0) {
              csb[col] = cs;
              hws[col] = g0;
              hws[H + col] = g1;
              hws[2 * H + col] = g2;
            }
          }
        }
      } else {
        // dX of layer l masked by Y_{l-1} > 0 -> dZ_{l-1} (tile, dZ^T, bias partial)
        const int l = (L - 2) - (p - nfwd);
        const bool keep_act = l - 1 >= 1;
        const unsigned bits = my_mask[(l - 1) * 256];
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
              const bool on = (bits >> ((i * TN + j) * 4 + r)) & 1u;
              const float v = on ? acc[i][j][r] : 0.f;
              cs += v;
              q[r] = bf_bits3(v);
              if (keep_act) *reinterpret_cast<unsigned short*>(act + act_off3<H>(row0 + r, col)) = q[r];
            }
            *reinterpret_cast<u16x4*>(box + frag_box_off(col, row0)) = q;
          }
          cs = col_sum4(cs);
          if (g4 == 0) csb[col] = cs;
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      lbar();  // B2: tile of the next phase and this phase's box complete
      stamp(3 + 3 * p);
    }
    stamp(2 + 3 * nphase);
    if (stl != nullptr) {
      if (lane == 0) stl[0] = t_entry;
      if (lane < 3 * nphase + 6) a.stamps[(blockIdx.x == 0 ? 0 : 3 * nphase + 6) + lane] = stl[lane];
    }
  } else {
    // =========================== store wave ===============================================
    // per-launch vectors, targets and the Z_y tile, loaded while the compute waves start:
    // the store wave joins barrier 0 at once and writes these into LDS before phase 0's
    // B1 (the first reader is phase 0's epilogue); every load is issued before any write
    {
      // one 16-byte (H = 256) / 8-byte (H = 128) load per lane per row of H
      constexpr int CPL = H / 64;
      typedef float rowv __attribute__((ext_vector_type(CPL)));
      rowv tv[CHAIN_MAX_HIDDEN], tw[3];
      float tb = 0.f, tt = 0.f;
      f32x4 zv[BM * H / 4 / 64];
#pragma unroll
      for (int q = 0; q < BM * H / 4 / 64; ++q) {
        const int c = lane + 64 * q, row = c / (H / 4), ch = c % (H / 4);
        zv[q] = *reinterpret_cast<const f32x4*>(a.Zy + (int64_t)(b0 + row) * H + ch * 4);
      }
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) tv[l] = *reinterpret_cast<const rowv*>(a.bias[l] + lane * CPL);
#pragma unroll
      for (int o = 0; o < 3; ++o) tw[o] = *reinterpret_cast<const rowv*>(a.W7 + o * H + lane * CPL);
      if (lane < 3) tb = a.b7[lane];
      lbar();  // barrier 0 (the compute waves' Y_0 tile)
      if (a.count_step && blockIdx.x == 0 && lane == 0) a.ctrl->step += 1;
      // targets: the replayed batch index, then the ray index, then the colour -- three
      // dependent loads, kept behind barrier 0 (the head is phases away)
      {
        int64_t offset = a.idx_offset;
        if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
        const int bt = b0 + lane / 3;
        if (lane < BM * 3 && bt < a.batch && ray_in_range(offset, bt, a.num_rays))
          tt = a.rgb[ray_row(a.ray_idx, a.idx_dtype, offset, bt) * 3 + lane % 3];
      }
      // ReLU bits of Y_0 for every compute lane (the last backward phase masks dZ_0 with
      // them), read from the Y_0 tile before phase 0's B1 lets the epilogue overwrite it
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = lane * 4 + u;  // compute thread
        const int twc = t >> 6, tg4 = (t & 63) >> 4, tr16 = t & 15;
        unsigned short hv[TM][TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              hv[i][j][r] = *reinterpret_cast<const unsigned short*>(
                  act + act_off3<H>(i * 16 + tg4 * 4 + r, twc * C::WN + j * 16 + tr16));
        unsigned bits = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) bits |= (bf_val3(hv[i][j][r]) > 0.f ? 1u : 0u) << ((i * TN + j) * 4 + r);
        maskw[t] = bits;
      }
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) *reinterpret_cast<rowv*>(vecs + l * H + lane * CPL) = tv[l];
#pragma unroll
      for (int o = 0; o < 3; ++o) *reinterpret_cast<rowv*>(w7s + o * H + lane * CPL) = tw[o];
      if (lane < 3) w7s[3 * H + lane] = tb;
      if (lane < BM * 3) tgs[lane] = tt;
#pragma unroll
      for (int q = 0; q < BM * H / 4 / 64; ++q) {
        const int c = lane + 64 * q, row = c / (H / 4), ch = c % (H / 4);
        *reinterpret_cast<f32x4*>(zy + row * C::ZY_LD + ch * 4) = zv[q];
      }
    }
    const int64_t tile_elems = (int64_t)(b0 / 16) * H * 16;
    auto copy_out = [&](const char* src, void* dst, int bytes) {
      char* d = reinterpret_cast<char*>(dst);
      for (int c = lane * 16; c < bytes; c += 64 * 16)
        *reinterpret_cast<u16x8*>(d + c) = *reinterpret_cast<const u16x8*>(src + c);
    };
    // dZ^T box -> fragment image: piece t (512 B) to k-block b0 / 32, tile t, half
    // (b0 / 16) % 2 of its 1 KiB
    const int64_t frag_base = (int64_t)(b0 >> 5) * (H / 16) * 1024 + ((b0 >> 4) & 1) * 512;
    auto copy_frag = [&](const char* src, bf16* dst) {
      char* d = reinterpret_cast<char*>(dst) + frag_base;
      for (int c = lane; c < C::TILE_BYTES / 16; c += 64)
        *reinterpret_cast<u16x8*>(d + (c >> 5) * 1024 + (c & 31) * 16) = *reinterpret_cast<const u16x8*>(src + c * 16);
    };
#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      lbar();  // B1
      const bool head_phase = p == nfwd - 1;
      if (head_phase) lbar();  // Bh1
      lbar();  // B2
      const char* box = smem + C::OFF_BOX + (p & 1) * C::BOX_BYTES;
      const char* csb = box + C::TILE_BYTES;
      if (p < nfwd) {
        const int l = p + 1;
        if (l <= L - 3) copy_out(box, a.YT[l] + tile_elems, C::TILE_BYTES);
        if (head_phase) {
          copy_frag(box, a.dZT[L - 2]);
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
        copy_frag(box, a.dZT[l - 1]);
        copy_out(csb, a.colsum[l - 1] + (int64_t)blockIdx.x * H, H * 4);
      }
    }
  }
}

template <int H, int TM, int LOSS>
int launch3_loss(const Chain3Args& a, hipStream_t stream) {
  using C = L3<H, TM>;
  const int lds = C::lds_bytes(a.L);
  INF_CHECK_ARG(lds <= C3_LDS_CAP, "chain3: LDS budget exceeded for this depth");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain3_kernel<H, TM, LOSS>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  chain3_kernel<H, TM, LOSS><<<dim3((unsigned)(a.rows / C::BM)), dim3(C3_THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

// the loss is a template parameter: one branch-free head per loss type keeps the compute
// waves under the 256 VGPRs of a 5-wave workgroup (a spill would drain the weight queue)
template <int H, int TM>
int launch3_typed(const Chain3Args& a, hipStream_t stream) {
  if (a.loss == INF_LOSS_L2) return launch3_loss<H, TM, INF_LOSS_L2>(a, stream);
  if (a.loss == INF_LOSS_L1) return launch3_loss<H, TM, INF_LOSS_L1>(a, stream);
  return launch3_loss<H, TM, INF_LOSS_CAUCHY>(a, stream);
}

}  // namespace

int launch_chain3(const Chain3Args& a, int bm, hipStream_t stream) {
  INF_CHECK_ARG(chain3_supported(a.H, a.L, a.rows), "chain3: unsupported shape");
  INF_CHECK_ARG(bm == 16, "chain3: tile height");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain3: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase == 2 * (a.L - 2), "chain3: phases");
  INF_CHECK_ARG(a.rgb != nullptr && a.Y0 != nullptr && a.Zy != nullptr, "chain3: inputs");
  for (int p = 0; p < a.nphase; ++p) INF_CHECK_ARG(a.img[p] != nullptr, "chain3: weight image missing");
  // bias / output-layer rows are read as H/64-float vectors per lane
  for (int l = 0; l < a.L - 1; ++l) INF_CHECK_ARG((uintptr_t)a.bias[l] % 16 == 0, "chain3: bias alignment");
  INF_CHECK_ARG((uintptr_t)a.W7 % 16 == 0, "chain3: output-layer weight alignment");
  if (a.H == 256) return launch3_typed<256, 1>(a, stream);
  return launch3_typed<128, 1>(a, stream);
}

}  // namespace inf
