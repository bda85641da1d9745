// Grouped NT GEMM on gfx950 matrix cores.  See gemm.hpp for the operand contract.
//
// Block = 256 threads = 4 waves in a 2x2 arrangement; each wave owns a (BM/2)x(BN/2)
// sub-tile built from 16x16 MFMA tiles.
//   bf16 mode: v_mfma_f32_16x16x32_bf16, k-tile BK = 64 (128-byte LDS rows)
//   fp32 mode: v_mfma_f32_16x16x4_f32 (exact f32 FMA chain), k-tile BK = 32 (128-byte
//              rows); a lane's 16-byte fragment read holds 4 consecutive k that feed 4
//              consecutive MFMAs, so every operand read is one ds_read_b128 in both modes.
//   split-bf16 modes (SPLIT 3 / 6): fp32 operands in memory and LDS exactly as the fp32
//              mode; each lane splits its 8 k of a 32-k tile into bf16 parts and sums the
//              significant cross products on v_mfma_f32_16x16x32_bf16 (fp32 accumulation,
//              smallest terms first):
//                3: x = hi + lo (+ 2^-16 |x|), hi*hi + hi*lo + lo*hi       -- ~2^-16 per product
//                6: x = hi + mid + lo (+ 2^-24 |x|), the six terms down to
//                   2^-16: hi*lo + lo*hi + mid*mid + hi*mid + mid*hi + hi*hi -- fp32-class
//              at 3 / 6 bf16 MFMAs per 32 k instead of 8 fp32 ones of twice the cycles each
//              (SURVEY.md §0.3's split-bf16 parity mode).
// Operand tiles are staged global -> registers -> LDS with a double buffer: the loads
// for k-tile t+1 are issued before the MFMAs of tile t and written to the other LDS
// buffer afterwards (one barrier per k-tile).  LDS rows are 8 x 16-byte chunks stored
// at chunk ^ (row & 7), which spreads the 16 rows a ds_read_b128 lane group touches
// over all bank slots of a 256-byte bank row pair (2-way at worst).
// Epilogue: accumulators -> padded fp32 LDS tile -> bias / ReLU / ReLU-mask ->
// coalesced row-major store, transposed store and per-tile column sums.
#include <algorithm>
#include <cstdlib>

#include "gemm.hpp"

namespace inf {
namespace {

template <typename T>
struct ModeTraits;

template <>
struct ModeTraits<bf16> {
  static constexpr int BK = 64;  // elements per k-tile (128 B rows)

};
template <>
struct ModeTraits<float> {
  static constexpr int BK = 32;

};

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// 16-byte chunk `chunk` of 128-byte LDS row `row`.  The 16 lanes of a ds_read_b128 group
// read 16 consecutive rows at one chunk: (row & 1, row >> 1) select distinct slots of the
// 256-byte bank row pair, so the group is conflict-free.
__device__ __forceinline__ int swz_slot(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + (swz_slot(row, chunk) << 4); }

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  // wait until at most N of this wave's vector-memory ops (direct-to-LDS loads) are in
  // flight, then a workgroup barrier; one asm statement so no LDS access moves across
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// wait until at most n * PER direct-to-LDS loads of this wave are in flight (n <= N,
// wave-uniform; vmcnt takes an immediate), then the workgroup barrier
template <int N, int PER>
__device__ __forceinline__ void wait_ahead_barrier(int n) {
  if constexpr (N <= 0) {
    wait_vm_barrier<0>();
  } else {
    if (n >= N) wait_vm_barrier<N * PER>();
    else wait_ahead_barrier<N - 1, PER>(n);
  }
}

template <typename T, int BM, int BN>
struct Tile {
  static constexpr int BK = ModeTraits<T>::BK;

  static constexpr int A_CHUNKS = BM * 8 / 256;  // 16-byte chunks per thread per k-tile
  static constexpr int B_CHUNKS = BN * 8 / 256;
#ifndef INF_GEMM128_STAGES
#define INF_GEMM128_STAGES 2
#endif
#ifndef INF_GEMM64_STAGES
#define INF_GEMM64_STAGES 4
#endif
  // 128x128: 2 stages (64 KiB, under the 67.6 KiB C staging tile) keep two workgroups per
  // CU; the 64x64 tile affords 4 stages (64 KiB) at the same occupancy
  static constexpr int STAGES =
      (BM == 128 && BN == 128) ? INF_GEMM128_STAGES : ((BM == 64 && BN == 64) ? INF_GEMM64_STAGES : 4);
  static constexpr int STAGE_BYTES = (BM + BN) * 128;
  static constexpr int OPER_BYTES = STAGES * STAGE_BYTES;
  static constexpr int CLD = BN + 4;  // fp32 C staging row stride
  static constexpr int C_BYTES = BM * CLD * 4;
  static constexpr int LDS_BYTES = OPER_BYTES > C_BYTES ? OPER_BYTES : C_BYTES;
  static constexpr int WM = BM / 2, WN = BN / 2;
  static constexpr int TM = WM / 16, TN = WN / 16;
};

// x = hi + lo + O(2^-16 |x|) (SPLIT 3) or hi + mid + lo + O(2^-24 |x|) (SPLIT 6); every
// part rounds to nearest (bf16 conversions)
template <int SPLIT>
__device__ __forceinline__ void split_bf16(const f32x4& x0, const f32x4& x1, bf16x8 (&part)[SPLIT == 6 ? 3 : 2]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = e < 4 ? x0[e] : x1[e - 4];
    const bf16 h = (bf16)x;
    const float r = x - (float)h;
    const bf16 m = (bf16)r;
    part[0][e] = h;
    part[1][e] = m;
    if constexpr (SPLIT == 6) part[2][e] = (bf16)(r - (float)m);
  }
}

template <typename T, int BM, int BN, int SPLIT = 0>
__device__ __forceinline__ void compute_tile(const char* __restrict__ As, const char* __restrict__ Bs, int wm0,
                                             int wn0, int lane, f32x4 (&acc)[Tile<T, BM, BN>::TM][Tile<T, BM, BN>::TN]) {
  using TL = Tile<T, BM, BN>;
  constexpr int TM = TL::TM, TN = TL::TN;
  const int r16 = lane & 15;
  const int g = lane >> 4;
  if constexpr (SPLIT != 0) {
    // lane (r16, g) holds k = 8 g .. 8 g + 7 of the 32-k tile (chunks 2 g, 2 g + 1) for A
    // and B alike -- one 16x16x32 MFMA per term covers the whole fp32 k-tile
    static_assert(sizeof(T) == 4 && (SPLIT == 3 || SPLIT == 6), "split-bf16 of fp32 operands");
    constexpr int NP = SPLIT == 6 ? 3 : 2;
    bf16x8 ap[TM][NP], bp[TN][NP];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm0 + i * 16 + r16;
      split_bf16<SPLIT>(*reinterpret_cast<const f32x4*>(As + swz(row, 2 * g)),
                        *reinterpret_cast<const f32x4*>(As + swz(row, 2 * g + 1)), ap[i]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn0 + j * 16 + r16;
      split_bf16<SPLIT>(*reinterpret_cast<const f32x4*>(Bs + swz(row, 2 * g)),
                        *reinterpret_cast<const f32x4*>(Bs + swz(row, 2 * g + 1)), bp[j]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[i][j];
        if constexpr (SPLIT == 6) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][0], bp[j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][2], bp[j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][1], bp[j][1], c, 0, 0, 0);
        }
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][1], bp[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][0], bp[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[i][0], bp[j][0], c, 0, 0, 0);
      }
  } else if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm0 + i * 16 + r16;
        a[i] = *reinterpret_cast<const bf16x8*>(As + swz(row, kk * 4 + g));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn0 + j * 16 + r16;
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + swz(row, kk * 4 + g));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      f32x4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm0 + i * 16 + r16;
        a[i] = *reinterpret_cast<const f32x4*>(As + swz(row, kk * 4 + g));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn0 + j * 16 + r16;
        b[j] = *reinterpret_cast<const f32x4*>(Bs + swz(row, kk * 4 + g));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
  }
}

template <typename T>
__device__ __forceinline__ float ld_elem(const void* p, int64_t i) {
  return (float)reinterpret_cast<const T*>(p)[i];
}

template <typename T, int BM, int BN, int SPLIT = 0>
__global__ __launch_bounds__(256, 1) void gemm_nt_kernel(const GemmBatch batch) {
  using TL = Tile<T, BM, BN>;
  constexpr int BK = TL::BK;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // ---- locate problem / tile -----------------------------------------------------
  // XCD-aware order (batch.xcd_remap): blocks b, b + 8, b + 16, ... are dealt to one
  // XCD, so they take consecutive tiles (same row panel, n fastest) and share its L2
  int bid = (int)blockIdx.x;
  if (batch.xcd_remap && batch.total_blocks % 8 == 0) bid = (bid & 7) * (batch.total_blocks >> 3) + (bid >> 3);
  int pi = 0;
#pragma unroll 1
  for (int i = 1; i < batch.nprob; ++i)
    if (bid >= batch.p[i].block_begin) pi = i;
  const GemmProblem& P = batch.p[pi];
  int local = bid - P.block_begin;
  const int tiles = P.tiles_m * P.tiles_n;
  const int split = local / tiles;
  local -= split * tiles;
  const int tm = local / P.tiles_n;
  const int tn = local - tm * P.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave >> 1) * TL::WM;
  const int wn0 = (wave & 1) * TL::WN;

  // ---- k-tile schedule ------------------------------------------------------------
  const int kt0 = P.K[0] / BK;
  const int kt1 = P.nseg > 1 ? P.K[1] / BK : 0;
  int t_begin = 0, t_end = kt0 + kt1;
  if (P.splits > 1) {
    const int per = kt0 / P.splits;
    t_begin = split * per;
    t_end = t_begin + per;
  }

  // ---- S-stage direct-to-LDS pipeline ------------------------------------------------
  // Each 1 KiB wave-instruction fills 8 consecutive 128-byte rows of a stage image; lane
  // L writes row L/8, slot L%8, so the source address carries the swizzle (the image is
  // lane-linear).  Wave w fills A rows [w*BM/4, (w+1)*BM/4) and B rows likewise.
  constexpr int STAGES = TL::STAGES;
  constexpr int A_INS = BM / 32, B_INS = BN / 32;  // glds per wave per stage
  constexpr int PER = A_INS + B_INS;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int lrow = lane >> 3, lslot = lane & 7;
  auto issue = [&](int t) {
    const int buf = (t - t_begin) % STAGES;
    const int seg = t < kt0 ? 0 : 1;
    const int k0 = (seg == 0 ? t : t - kt0) * BK;
    char* As = smem + buf * TL::STAGE_BYTES;
    char* Bs = As + BM * 128;
    // byte offset of 16-byte chunk c (element k0 + c*EPC) of operand row r
    constexpr int EPC = 16 / sizeof(T);
    auto chunk_off = [&](int64_t ld, bool kblk, int64_t r, int c) -> int64_t {
      const int64_t k = k0 + c * EPC;
      return (kblk ? (k >> 4) * ld + r * 16 + (k & 15) : r * ld + k) * (int64_t)sizeof(T);
    };
    const bool akb = seg == 0 && P.a_kblk, bkb = seg == 0 && P.b_kblk;
    const char* A = reinterpret_cast<const char*>(P.A[seg]);
    const char* Bm = reinterpret_cast<const char*>(P.B[seg]);
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int r0 = wv * (BM / 4) + i * 8;
      const int row = r0 + lrow;
      const char* src = A + chunk_off(P.lda[seg], akb, m0 + row, swz_slot(row, lslot));
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(As + r0 * 128), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int r0 = wv * (BN / 4) + i * 8;
      const int row = r0 + lrow;
      const char* src = Bm + chunk_off(P.ldb[seg], bkb, n0 + row, swz_slot(row, lslot));
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(Bs + r0 * 128), 16, 0, 0);
    }
  };

  f32x4 acc[TL::TM][TL::TN];
#pragma unroll
  for (int i = 0; i < TL::TM; ++i)
#pragma unroll
    for (int j = 0; j < TL::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t_begin < t_end) {
#pragma unroll
    for (int q = 0; q < STAGES - 1; ++q)
      if (t_begin + q < t_end) issue(t_begin + q);
#pragma unroll 1
    for (int t = t_begin; t < t_end; ++t) {
      // stages issued after t that may stay in flight
      const int ahead = min(STAGES - 2, t_end - 1 - t);
      wait_ahead_barrier<STAGES - 2, PER>(ahead);
      if (t + STAGES - 1 < t_end) issue(t + STAGES - 1);
      const char* As = smem + ((t - t_begin) % STAGES) * TL::STAGE_BYTES;
      compute_tile<T, BM, BN, SPLIT>(As, As + BM * 128, wm0, wn0, lane, acc);
    }
  }
  __syncthreads();

  // ---- epilogue ------------------------------------------------------------------
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int CLD = TL::CLD;
  {
    const int cr = (lane >> 4) * 4;
    const int cc = lane & 15;
#pragma unroll
    for (int i = 0; i < TL::TM; ++i)
#pragma unroll
      for (int j = 0; j < TL::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) Cs[(wm0 + i * 16 + cr + r) * CLD + wn0 + j * 16 + cc] = acc[i][j][r];
  }
  __syncthreads();

  constexpr int NQ = BN / 4;  // float4 chunks per row
  if (P.slab != nullptr) {
    float* dst = P.slab + (int64_t)split * P.slab_stride;
#pragma unroll 4
    for (int c = tid; c < BM * NQ; c += 256) {
      const int row = c / NQ, q = c - row * NQ;
      const f32x4 v = *reinterpret_cast<const f32x4*>(Cs + row * CLD + q * 4);
      *reinterpret_cast<f32x4*>(dst + (int64_t)(m0 + row) * P.slab_ld + n0 + q * 4) = v;
    }
    return;
  }

  const bool need_back = P.CT != nullptr || P.colsum != nullptr;
#pragma unroll 4
  for (int c = tid; c < BM * NQ; c += 256) {
    const int row = c / NQ, q = c - row * NQ;
    const int m = m0 + row, n = n0 + q * 4;
    f32x4 v = *reinterpret_cast<const f32x4*>(Cs + row * CLD + q * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (P.bias0 != nullptr) x += P.bias0[n + e];
      if (P.bias1 != nullptr) x += P.bias1[n + e];
      if (P.relu) x = fmaxf(x, 0.f);
      if (P.mask != nullptr && !(ld_elem<T>(P.mask, (int64_t)m * P.ldmask + n + e) > 0.f)) x = 0.f;
      v[e] = x;
    }
    if (need_back) *reinterpret_cast<f32x4*>(Cs + row * CLD + q * 4) = v;
    if (P.C != nullptr) {
      if (P.c_f32 || sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.C) + (int64_t)m * P.ldc + n) = v;
      } else {
        bf16x4 h = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(P.C) + (int64_t)m * P.ldc + n) = h;
      }
    }
  }
  if (!need_back) return;
  __syncthreads();

  if (P.CT != nullptr) {
    constexpr int MQ = BM / 4;
#pragma unroll 4
    for (int c = tid; c < BN * MQ; c += 256) {
      const int col = c / MQ, q = c - col * MQ;
      const float x0 = Cs[(q * 4 + 0) * CLD + col];
      const float x1 = Cs[(q * 4 + 1) * CLD + col];
      const float x2 = Cs[(q * 4 + 2) * CLD + col];
      const float x3 = Cs[(q * 4 + 3) * CLD + col];
      const int64_t off = (int64_t)(n0 + col) * P.ldct + m0 + q * 4;
      if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.CT) + off) = f32x4{x0, x1, x2, x3};
      } else {
        bf16x4 h = {(bf16)x0, (bf16)x1, (bf16)x2, (bf16)x3};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(P.CT) + off) = h;
      }
    }
  }
  if (P.colsum != nullptr) {
    // one partial per 64 rows, independent of the tile height: the number of partials
    // of a bias gradient is then a function of the batch only
    constexpr int PARTS = BM / 64;
    for (int c = tid; c < BN * PARTS; c += 256) {
      const int col = c % BN, part = c / BN;
      float s = 0.f;
#pragma unroll 8
      for (int row = part * 64; row < part * 64 + 64; ++row) s += Cs[row * CLD + col];
      P.colsum[(int64_t)(m0 / 64 + part) * P.N + n0 + col] = s;
    }
  }
}

template <typename T, int BM, int BN, int SPLIT = 0>
int launch_typed(const GemmBatch& b, hipStream_t stream) {
  int lds = Tile<T, BM, BN>::LDS_BYTES;
  // INF_GEMM_LDS (experiments): reserve at least this much LDS per workgroup, e.g. > 80 KiB
  // for one workgroup per CU
  if (const char* e = std::getenv("INF_GEMM_LDS")) lds = std::max(lds, std::min(std::atoi(e), 160 * 1024));
  static int attr = 0;
  if (attr < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)gemm_nt_kernel<T, BM, BN, SPLIT>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = lds;
  }
  gemm_nt_kernel<T, BM, BN, SPLIT><<<dim3((unsigned)b.total_blocks), dim3(256), lds, stream>>>(b);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_gemm(GemmBatch& b, int mode, GemmTile tile, hipStream_t stream) {
  const int BM = tile_bm(tile), BN = tile_bn(tile);
  const int BK = mode == INF_MODE_BF16 ? 64 : 32;  // split modes stage fp32 tiles
  INF_CHECK_ARG(b.nprob >= 1 && b.nprob <= GEMM_MAX_PROBLEMS, "gemm: problem count");
  int blocks = 0;
  for (int i = 0; i < b.nprob; ++i) {
    GemmProblem& p = b.p[i];
    INF_CHECK_ARG(p.M > 0 && p.N > 0 && p.M % BM == 0 && p.N % BN == 0, "gemm: M/N not tile multiples");
    INF_CHECK_ARG(p.nseg == 1 || p.nseg == 2, "gemm: nseg");
    for (int s = 0; s < p.nseg; ++s) {
      INF_CHECK_ARG(p.K[s] > 0 && p.K[s] % BK == 0, "gemm: K not a k-tile multiple");
      INF_CHECK_ARG(p.A[s] != nullptr && p.B[s] != nullptr, "gemm: null operand");
      INF_CHECK_ARG(p.lda[s] % 8 == 0 && p.ldb[s] % 8 == 0, "gemm: operand rows must be 16-byte aligned");
    }
    if (p.splits < 1) p.splits = 1;
    INF_CHECK_ARG(p.splits == 1 || (p.nseg == 1 && (p.K[0] / BK) % p.splits == 0 && p.slab != nullptr),
                  "gemm: split-K needs one segment, divisible k-tiles and a slab");
    INF_CHECK_ARG(p.slab != nullptr || p.C != nullptr || p.CT != nullptr || p.colsum != nullptr, "gemm: no output");
    p.tiles_m = p.M / BM;
    p.tiles_n = p.N / BN;
    p.block_begin = blocks;
    blocks += p.tiles_m * p.tiles_n * p.splits;
  }
  b.total_blocks = blocks;
  b.xcd_remap = std::getenv("INF_NO_XCD_REMAP") == nullptr ? 1 : 0;
  if (mode == INF_MODE_BF16) {
    if (tile == TILE_128x128) return launch_typed<bf16, 128, 128>(b, stream);
    if (tile == TILE_128x64) return launch_typed<bf16, 128, 64>(b, stream);
    return launch_typed<bf16, 64, 64>(b, stream);
  }
  if (mode == INF_MODE_BF16X3) {
    if (tile == TILE_128x128) return launch_typed<float, 128, 128, 3>(b, stream);
    if (tile == TILE_128x64) return launch_typed<float, 128, 64, 3>(b, stream);
    return launch_typed<float, 64, 64, 3>(b, stream);
  }
  if (mode == GEMM_MODE_BF16X6) {
    if (tile == TILE_128x128) return launch_typed<float, 128, 128, 6>(b, stream);
    if (tile == TILE_128x64) return launch_typed<float, 128, 64, 6>(b, stream);
    return launch_typed<float, 64, 64, 6>(b, stream);
  }
  if (tile == TILE_128x128) return launch_typed<float, 128, 128>(b, stream);
  if (tile == TILE_128x64) return launch_typed<float, 128, 64>(b, stream);
  return launch_typed<float, 64, 64>(b, stream);
}

}  // namespace inf
