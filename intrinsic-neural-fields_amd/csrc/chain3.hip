// Register-streamed fused training chain: the bf16 training step of small batches (the
// reference's 4096-ray batch, intrinsic_cat.yaml:32) up to the weight gradients.
//
// One workgroup owns BM = 16 rays and runs, in ONE launch:
//   gather    X[b] = sum_i bary[r][i] * E[vids[r][i]] for its rays r = ray_idx[offset + b]
//             (mesh.py:313-324 with ray_dataloader.py:122-129), into LDS,
//   forward   layers 0..L-2 (model.py:98-112); the skip layer (layers.py:60-62) as two
//             K segments [h | x] into one accumulator,
//   head      Linear(H,3) + sigmoid (model.py:89-94), loss (config.py:113-122),
//             dL/dz = dL/dp * p (1 - p),
//   backward  dZ_{L-2} = (dz W_head) * (h > 0), then dZ_{l-1} = (dZ_l W_l) * (Y_{l-1} > 0)
//             for l = L-2..1 (autograd of trainer.py:81),
// and leaves what the weight-gradient GEMM needs: X^T, Y_l^T, dZ_l^T, bias partials.
//
// Why registers, not an LDS ring.  At 16 rays per workgroup every weight element feeds
// exactly one wave (the 4 waves split the output columns), so staging weights through
// LDS buys no reuse; what bounds the kernel is the L2 -> CU weight stream.  The packed
// weights are stored in MFMA fragment order (adam.hip: 1 KiB per 16 columns x 32 k,
// lane l's 16 bytes at 16 l), so a wave's B operand for one 32-deep k block is TN
// coalesced 1 KiB loads straight into VGPRs.  The weight stream is a list of blocks
// (C3Block: UPL k-blocks each, one hidden layer's K); each wave keeps a ring of D k-blocks
// of fragments in flight and refills a slot right after its MFMAs consumed it -- across
// block, phase and epilogue boundaries, with no per-k-step barrier.  After the gather the
// only vector-memory instructions of the compute waves are these loads, so the
// compiler's vmcnt waits are exact (each waits for one k-block).
//
// Stores.  Every global output (X^T, Y^T, dZ^T, bias / output-layer partials, loss, pred)
// is written into LDS by the compute waves and copied out by a fifth "store" wave that
// mirrors the compute waves' barriers.  Stores in the compute waves would join the
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
constexpr int C3BM = 16;  // rays per workgroup

template <int H>
struct L3 {
  static constexpr int BM = C3BM;
  static constexpr int TN = H / 64;   // 16-column tiles per wave (a wave owns H/4 columns)
  static constexpr int WN = H / 4;
  static constexpr int UPL = H / 32;  // 32-deep k blocks per hidden layer (= per stream block)
  static constexpr int NT = H / 16;   // 16-row tiles per k block of a weight image
  static constexpr int ACT_ROW = H * 2;
  static constexpr int TILE_BYTES = BM * H * 2;
  static constexpr int BOX_BYTES = TILE_BYTES + H * 4;  // Y^T / dZ^T tile + bias partial
  static constexpr int OFF_ACT = 0;
  static constexpr int OFF_BOX = OFF_ACT + BM * ACT_ROW;
  static constexpr int OFF_HW = OFF_BOX + 2 * BOX_BYTES;  // [3][H] output-layer weight grad
  static constexpr int OFF_HB = OFF_HW + 3 * H * 4;       // [4]
  static constexpr int OFF_LS = OFF_HB + 16;              // [2] f64 loss / SSE
  static constexpr int OFF_PRED = OFF_LS + 16;            // [BM][3]
  static constexpr int OFF_DZ = OFF_PRED + BM * 12;       // [4 waves][BM][3] head gradient
  static constexpr int OFF_TGT = OFF_DZ + 4 * BM * 12;    // [BM][3] targets
  static constexpr int OFF_ZP = OFF_TGT + BM * 12;        // [4 waves][BM][3] head partial sums
  static constexpr int OFF_RAY = OFF_ZP + 4 * BM * 12;    // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RBARY = OFF_RAY + BM * 16 + BM * 12 + 16;  // [BM][3] barycentrics
  static constexpr int OFF_W7 = OFF_RBARY + BM * 12 + 16;  // [3][H] then b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;  // biases [L-1][H], then Ly.bias [H]
  // ReLU bits: per layer one 32-bit word per compute lane, bit j*4 + r for accumulator
  // element (j, r) of that lane
  static constexpr int MASK_BYTES = 256 * 4;
  __host__ __device__ static int off_mask(int L) { return OFF_VEC + L * H * 4; }
  __host__ __device__ static int off_x(int L) { return off_mask(L) + (L - 2) * MASK_BYTES; }
  __host__ __device__ static int off_stamp(int L, int k_pad) { return off_x(L) + BM * k_pad * 2; }
  static int lds_bytes(int L, int k_pad) { return off_stamp(L, k_pad) + (5 * C3_MAX_PHASES + 8) * 8; }
  static_assert(TN * 4 <= 32, "ReLU bits of a lane must fit one word");
};

// byte offset of element (row, col) of a bf16 LDS tile with `rowb`-byte rows: 16-byte
// chunk c of row r stored at chunk c ^ (r & 15) (a ds_read_b128 lane group of 16 rows
// at one chunk is conflict-free)
__device__ __forceinline__ int tile_off(int rowb, int row, int col) {
  return row * rowb + (((col >> 3) ^ (row & 15)) << 4) + ((col & 7) << 1);
}

// element (col, ray r) of a Y^T box: the 16-ray blocked layout of the dW GEMM's A operand
// (lgemm a_kblk), the whole tile contiguous in global memory
__device__ __forceinline__ int box_off(int col, int r) { return (col * 16 + r) * 2; }

// element (col, ray r < 16) of a dZ^T box: the fragment image the dW GEMM streams
// (lgemm operand B: rows = columns of dZ, k = rays): per 16-column tile one 512-byte
// piece = the workgroup's half (16 of 32 rays) of that tile's 1 KiB k-block
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

template <int H, int LOSS>
__global__ __launch_bounds__(C3_THREADS) void chain3_kernel(const Chain3Args a) {
  using C = L3<H>;
  constexpr int BM = C::BM, TN = C::TN, UPL = C::UPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L;
  const int k_pad = a.k_pad;
  char* act = smem + C::OFF_ACT;
  float* hws = reinterpret_cast<float*>(smem + C::OFF_HW);
  float* hbs = reinterpret_cast<float*>(smem + C::OFF_HB);
  double* lss = reinterpret_cast<double*>(smem + C::OFF_LS);
  float* preds = reinterpret_cast<float*>(smem + C::OFF_PRED);
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);                 // [BM][4]
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RBARY);         // [BM][3]
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  unsigned* maskw = reinterpret_cast<unsigned*>(smem + C::off_mask(L));
  char* xs = smem + C::off_x(L);  // gathered features [BM][k_pad] bf16 (tile_off layout)
  const int xrow = k_pad * 2;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int nphase = a.nphase;
  const int nfwd = L - 1;  // forward phases 0..L-2

  unsigned long long* stl = nullptr;  // diagnostics only
  if (a.stamps != nullptr && wave == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    stl = reinterpret_cast<unsigned long long*>(smem + C::off_stamp(L, k_pad));
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
    // fragment ring: D k-blocks (D * TN KiB per wave) in flight; 16 KiB per wave kept the
    // L2 -> CU stream at its best rate in tools/microbench/l2ring (32 KiB: -35 %)
    constexpr int D = C3_DEPTH < UPL ? C3_DEPTH : UPL;
    bf16x8 fr[D][TN];
    // buffer loads: descriptor per image in SGPRs, k-block offset in soffset, tile offset
    // as the immediate, one VGPR of lane offset -- no 64-bit address registers
    const unsigned lane_off = (unsigned)(wc * TN * 64 + lane) * 16u;
    auto rsrc_of = [&](const bf16* img) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
    };
    auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j) -> bf16x8 {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024, kb * C::NT * 1024, 0);
      return __builtin_bit_cast(bf16x8, v);
    };
    // ---- gather: ray records of the 16 rays (index, vertex ids, barycentrics), one
    // thread per (ray, corner) ------------------------------------------------------------
    if (tid < BM * 3) {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int rl = tid / 3, i = tid % 3;
      const int b = b0 + rl;
      int v = 0, ok = 0;
      float w = 0.f;
      if (b < a.batch && ray_in_range(offset, b, a.num_rays)) {
        const int64_t rr = ray_row(a.ray_idx, a.idx_dtype, offset, b);
        const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
        // an out-of-range vertex id reads as a zero feature row (gather.hip)
        ok = (uint64_t)e < (uint64_t)a.num_vertices;
        v = ok ? (int)e : 0;
        w = a.bary[3 * rr + i];
      }
      rvid[rl * 4 + i] = v;
      rbary[rl * 3 + i] = w;
      // the ray's flag: all three corners in range (bit i per corner, summed by the gather)
      rvid[BM * 4 + tid] = ok;
    }
    // the first block's fragments, in k order (the loop's waits assume that order); issued
    // after the dependent ray-record loads so those are not queued behind 64 KiB per CU
    {
      const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(a.blk[0].img);
#pragma unroll
      for (int kb = 0; kb < D; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j) fr[kb][j] = frag(rs0, a.blk[0].kb0 + kb, j);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stamp(3 * nphase + 3);
    lbar();  // barrier R: ray records in LDS

    // ---- gather: the feature tile, 16-byte chunks (8 columns) per thread ---------------
    // fp32 FMA in the reference order b0 e0 + b1 e1 + b2 e2, rounded to bf16 once (the
    // gather kernel's numerics); every load of a round is issued before any use
    {
      const int cpr = k_pad >> 3;          // chunks per row
      const int nch = BM * cpr;            // chunks of the tile
      constexpr int GR = 8;                // chunks per thread per round (k_pad 1024: one round)
      const __amdgpu_buffer_rsrc_t rt =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.table), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll 1
      for (int q0 = tid; q0 < nch; q0 += 256 * GR) {
        u16x8 ev[GR][3];
        float wv[GR][3];
        int okv[GR];
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + 256 * g;
          const int r = (q < nch ? q : 0) / cpr, ch = (q < nch ? q : 0) % cpr;
          okv[g] = q < nch ? (rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2]) : 0;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            wv[g][i] = rbary[r * 3 + i];
            const unsigned off = ((unsigned)rvid[r * 4 + i] * (unsigned)k_pad + ch * 8) * 2u;
            ev[g][i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rt, off, 0, 0));
          }
        }
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + 256 * g;
          if (q < nch) {
            const int r = q / cpr, ch = q % cpr;
            u16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = fmaf(wv[g][2], bf_val3(ev[g][2][e]), fmaf(wv[g][1], bf_val3(ev[g][1][e]),
                                                                       wv[g][0] * bf_val3(ev[g][0][e])));
              o[e] = bf_bits3(okv[g] ? x : 0.f);
            }
            *reinterpret_cast<u16x8*>(xs + r * xrow + ((ch ^ (r & 15)) << 4)) = o;
          }
        }
      }
    }
    stamp(3 * nphase + 4);
    lbar();  // barrier 0: feature tile in LDS
    stamp(3 * nphase + 5);

    unsigned* my_mask = maskw + tid;  // + layer * 256
    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
    for (int i = 0; i < a.nblk; ++i) {
      const C3Block& B = a.blk[i];
      const C3Block& Bn = a.blk[i + 1 < a.nblk ? i + 1 : i];
      if (i == 0 || a.blk[i - 1].last) stamp(1 + 3 * B.phase);
      // ---- MFMAs of block i; slot kb % D refilled with k-block kb + D of this block or
      // of block i+1 (the last block reloads itself: harmless loads keep waits exact)
      const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
      const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
      const char* abase = B.a_x ? xs : act;
      const int arow = B.a_x ? xrow : C::ACT_ROW;
      const int ak0 = B.ak0, ckb = B.kb0, nkb = Bn.kb0;
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
        const bf16x8 av =
            *reinterpret_cast<const bf16x8*>(abase + r16 * arow + ((((ak0 + kb) * 4 + g4) ^ r16) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, fr[kb % D][j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fr[kb % D][j] = kb + D < UPL ? frag(crs, ckb + kb + D, j) : frag(nrs, nkb + kb + D - UPL, j);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (!B.last) continue;

      // ---- epilogue of phase p: LDS reads first, then arithmetic, then LDS writes -------
      const int p = B.phase;
      stamp(2 + 3 * p);
      lbar();  // B1: every wave is done reading the activation tile
      stamp(3 * nphase + 6 + p);
      char* box = smem + C::OFF_BOX + (p & 1) * C::BOX_BYTES;
      float* csb = reinterpret_cast<float*>(box + C::TILE_BYTES);
      if (p < nfwd) {
        // forward of layer l: bias (+ Ly.bias at the skip layer) + ReLU -> tile, Y^T, bits
        const int l = p;
        const bool skip = l == a.s;
        const bool last = l == L - 2;
        float bv[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * C::WN + j * 16 + r16;
          bv[j] = vecs[l * H + col];
        }
        float by[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) by[j] = skip ? vecs[(L - 1) * H + wc * C::WN + j * 16 + r16] : 0.f;
        float hq[TN][4];  // bf16-rounded activations as f32
        unsigned bits = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[j][r] + bv[j];
            if (skip) v += by[j];
            v = fmaxf(v, 0.f);
            hq[j][r] = bf_val3(bf_bits3(v));
            bits |= (hq[j][r] > 0.f ? 1u : 0u) << (j * 4 + r);
          }
        if (!last) {
          my_mask[l * 256] = bits;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = wc * C::WN + j * 16 + r16;
            const int row0 = g4 * 4;
            u16x4 q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              q[r] = bf_bits3(hq[j][r]);
              *reinterpret_cast<unsigned short*>(act + tile_off(C::ACT_ROW, row0 + r, col)) = q[r];
            }
            *reinterpret_cast<u16x4*>(box + box_off(col, row0)) = q;
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
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int o = 0; o < 3; ++o) {
              float z = 0.f;
#pragma unroll
              for (int j = 0; j < TN; ++j) z = fmaf(hq[j][r], w7r[o][j], z);
              z = row_sum16(z);
              if (r16 == 0) zps[(wc * BM + g4 * 4 + r) * 3 + o] = z;
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
            static_assert(C3BM * 3 <= 64, "one lane per (ray, output)");
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
          float dzr[4][3];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int o = 0; o < 3; ++o) dzr[r][o] = dzs[wc * BM * 3 + (g4 * 4 + r) * 3 + o];
          if (tid < 3) {
            float db = 0.f;
            for (int r = 0; r < BM; ++r) db += dzs[r * 3 + tid];
            hbs[tid] = db;
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = wc * C::WN + j * 16 + r16;
            const int row0 = g4 * 4;
            float cs = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
            u16x4 q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float h = hq[j][r];
              const float d0 = dzr[r][0], d1 = dzr[r][1], d2 = dzr[r][2];
              float g = fmaf(d2, w7r[2][j], fmaf(d1, w7r[1][j], d0 * w7r[0][j]));
              g = h > 0.f ? g : 0.f;
              q[r] = bf_bits3(g);
              *reinterpret_cast<unsigned short*>(act + tile_off(C::ACT_ROW, row0 + r, col)) = q[r];
              cs += g;
              g0 = fmaf(d0, h, g0);
              g1 = fmaf(d1, h, g1);
              g2 = fmaf(d2, h, g2);
            }
            *reinterpret_cast<u16x4*>(box + frag_box_off(col, row0)) = q;
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
          const int row0 = g4 * 4;
          float cs = 0.f;
          u16x4 q;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool on = (bits >> (j * 4 + r)) & 1u;
            const float v = on ? acc[j][r] : 0.f;
            cs += v;
            q[r] = bf_bits3(v);
            if (keep_act) *reinterpret_cast<unsigned short*>(act + tile_off(C::ACT_ROW, row0 + r, col)) = q[r];
          }
          *reinterpret_cast<u16x4*>(box + frag_box_off(col, row0)) = q;
          cs = col_sum4(cs);
          if (g4 == 0) csb[col] = cs;
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      stamp(4 * nphase + 6 + p);
      lbar();  // B2: tile of the next phase and this phase's box complete
      stamp(3 + 3 * p);
    }
    stamp(2 + 3 * nphase);
    if (stl != nullptr) {
      if (lane == 0) stl[0] = t_entry;
      for (int i = lane; i < 5 * nphase + 6; i += 64) a.stamps[(blockIdx.x == 0 ? 0 : 5 * nphase + 6) + i] = stl[i];
    }
  } else {
    // =========================== store wave ===============================================
    // per-launch vectors (biases, Ly.bias, W7, b7), loaded while the compute waves gather;
    // written into LDS between barriers R and 0 (the first reader is phase 0's epilogue)
    constexpr int CPL = H / 64;  // one 16-byte (H = 256) / 8-byte (H = 128) load per lane per row
    typedef float rowv __attribute__((ext_vector_type(CPL)));
    {
      rowv tv[CHAIN_MAX_HIDDEN], tyb, tw[3];
      float tb = 0.f;
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) tv[l] = *reinterpret_cast<const rowv*>(a.bias[l] + lane * CPL);
      tyb = *reinterpret_cast<const rowv*>(a.bias_y + lane * CPL);
#pragma unroll
      for (int o = 0; o < 3; ++o) tw[o] = *reinterpret_cast<const rowv*>(a.W7 + o * H + lane * CPL);
      if (lane < 3) tb = a.b7[lane];
      lbar();  // barrier R
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) *reinterpret_cast<rowv*>(vecs + l * H + lane * CPL) = tv[l];
      *reinterpret_cast<rowv*>(vecs + (L - 1) * H + lane * CPL) = tyb;
#pragma unroll
      for (int o = 0; o < 3; ++o) *reinterpret_cast<rowv*>(w7s + o * H + lane * CPL) = tw[o];
      if (lane < 3) w7s[3 * H + lane] = tb;
    }
    lbar();  // barrier 0: feature tile in LDS
    if (a.count_step && blockIdx.x == 0 && lane == 0) a.ctrl->step += 1;
    // targets: the replayed batch index, the ray index, the colour -- dependent loads,
    // kept behind barrier 0 (the head is phases away)
    {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int bt = b0 + lane / 3;
      float tt = 0.f;
      if (lane < BM * 3 && bt < a.batch && ray_in_range(offset, bt, a.num_rays))
        tt = a.rgb[ray_row(a.ray_idx, a.idx_dtype, offset, bt) * 3 + lane % 3];
      if (lane < BM * 3) tgs[lane] = tt;
    }
    // X^T for the dW GEMM (layer 0 and Ly): 16-ray blocked tile [k_pad][16], one 8-column
    // group per lane: 16 row reads, 8 x 32-byte column stores
    {
      bf16* xt = a.XT + (int64_t)(b0 / 16) * k_pad * 16;
#pragma unroll 1
      for (int cg = lane; cg < (k_pad >> 3); cg += 64) {
        u16x8 rv[BM];
#pragma unroll
        for (int r = 0; r < BM; ++r) rv[r] = *reinterpret_cast<const u16x8*>(xs + r * xrow + ((cg ^ (r & 15)) << 4));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          u16x8 lo, hi;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            lo[r] = rv[r][e];
            hi[r] = rv[8 + r][e];
          }
          u16x8* dst = reinterpret_cast<u16x8*>(xt + (int64_t)(cg * 8 + e) * 16);
          dst[0] = lo;
          dst[1] = hi;
        }
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
        const int l = p;
        if (!head_phase) copy_out(box, a.YT[l] + tile_elems, C::TILE_BYTES);
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

template <int H, int LOSS>
int launch3_loss(const Chain3Args& a, hipStream_t stream) {
  using C = L3<H>;
  const int lds = C::lds_bytes(a.L, a.k_pad);
  INF_CHECK_ARG(lds <= C3_LDS_CAP, "chain3: LDS budget exceeded for this depth / feature width");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain3_kernel<H, LOSS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    lds));
    attr_set = lds;
  }
  chain3_kernel<H, LOSS><<<dim3((unsigned)(a.rows / C3BM)), dim3(C3_THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

// the loss is a template parameter: one branch-free head per loss type keeps the compute
// waves under the 256 VGPRs of a 5-wave workgroup (a spill would drain the weight queue)
template <int H>
int launch3_typed(const Chain3Args& a, hipStream_t stream) {
  if (a.loss == INF_LOSS_L2) return launch3_loss<H, INF_LOSS_L2>(a, stream);
  if (a.loss == INF_LOSS_L1) return launch3_loss<H, INF_LOSS_L1>(a, stream);
  return launch3_loss<H, INF_LOSS_CAUCHY>(a, stream);
}

}  // namespace

int launch_chain3(const Chain3Args& a, int bm, hipStream_t stream) {
  INF_CHECK_ARG(chain3_supported(a.H, a.L, a.k_pad, a.rows), "chain3: unsupported shape");
  INF_CHECK_ARG(bm == C3BM, "chain3: tile height");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain3: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase == 2 * a.L - 3, "chain3: phases");
  INF_CHECK_ARG(a.nblk >= 1 && a.nblk <= C3_MAX_BLOCKS, "chain3: weight-stream blocks");
  INF_CHECK_ARG(a.rgb != nullptr && a.table != nullptr && a.vids != nullptr && a.bary != nullptr && a.XT != nullptr,
                "chain3: inputs");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "chain3: vertex id dtype");
  INF_CHECK_ARG(a.num_vertices * (int64_t)a.k_pad * 2 < (int64_t)1 << 31, "chain3: table exceeds 2 GiB");
  for (int i = 0; i < a.nblk; ++i) INF_CHECK_ARG(a.blk[i].img != nullptr, "chain3: weight image missing");
  // bias / output-layer rows are read as H/64-float vectors per lane
  for (int l = 0; l < a.L - 1; ++l) INF_CHECK_ARG((uintptr_t)a.bias[l] % 16 == 0, "chain3: bias alignment");
  INF_CHECK_ARG((uintptr_t)a.bias_y % 16 == 0 && (uintptr_t)a.W7 % 16 == 0, "chain3: vector alignment");
  if (a.H == 256) return launch3_typed<256>(a, stream);
  return launch3_typed<128>(a, stream);
}

}  // namespace inf
