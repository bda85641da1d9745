// The render slice's vertex projection (inf_project_table): C[V][2H] = E[V][k_pad] W^T with
// W = [W_0; W_y] [2H][k_pad], bf16 in and out, fp32 accumulation -- one large, plain NT
// GEMM per frame (400k x 512 x 1024 at config E: 419 GFLOP).
//
// Tile.  256 vertex rows x 256 output columns per workgroup, 8 waves as 2 (rows) x 4
// (columns), each wave 128 rows x 64 columns: 8 x 4 v_mfma_f32_16x16x32_bf16 tiles, 128
// fp32 accumulators per lane.  The weight rows are the MFMA's A operand and the table rows
// its B operand, so a lane's accumulator holds 4 consecutive OUTPUT COLUMNS of one vertex
// row -- one 8-byte bf16 write per tile in the epilogue.  Per 32-deep k-step the workgroup
// moves 32 KB (256 rows of each operand x 64 B) for 2 x 256 x 256 x 32 FLOP: 128 FLOP/B,
// the MFMA-bound side of a CU's L2 -> LDS rate.
//
// Pipeline.  A ring of 4 LDS stages (4 x 32 KB) filled by direct-to-LDS loads
// (global_load_lds_dwordx4, 4 per thread per stage) three k-steps ahead; one counted
// `s_waitcnt vmcnt` + raw s_barrier per k-step retires the oldest stage (never vmcnt(0)
// in the loop: the next stages stay in flight across the barrier; all LDS in one
// __shared__ array, MI355X guide §5 'Pipelining across barriers').  The stage a k-step
// refills was last read in the previous k-step, before the barrier every wave has passed.
// Stage rows are 64 B; 16-byte chunk c of row r lives at chunk c ^ (3 ((r >> 3) & 1)),
// the conflict-free swizzle of chain.hip's 64-B stage rows, applied on the SOURCE address
// (the DMA writes lane-linear).
//
// Epilogue.  The accumulators are rounded to bf16 into a [256][256] LDS image (512-B rows,
// chunk c of row r at c ^ (r & 31): the 16 rows of a tile's 8-byte writes hit 16 distinct
// chunks) and written out with 16-byte coalesced stores, rows past V skipped.
// XCD-aware order: the 2 column tiles of a row panel are consecutive on one XCD (the
// panel's table rows are read once from HBM and once from that XCD's L2).
#include <cstdlib>

#include "ptab.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::pack_bf16x2;
using c3::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

template <int BM_, int BN_, int BK_, int STAGES_, int WAVES_M_>
struct PT {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, STAGES = STAGES_;
  static constexpr int THREADS = 512;                    // 8 waves
  static constexpr int WAVES_M = WAVES_M_, WAVES_N = 8 / WAVES_M_;
  static constexpr int WROWS = BM / WAVES_M, WCOLS = BN / WAVES_N;  // per wave: vertex rows, output columns
  static constexpr int TI = WROWS / 16, TJ = WCOLS / 16;            // MFMA tiles per wave
  static constexpr int ROWB = BK * 2;                    // stage row bytes (64 / 128)
  static constexpr int CPR = ROWB / 16;                  // 16-byte chunks per stage row
  static constexpr int STAGE_BYTES = (BM + BN) * ROWB;
  static constexpr int LDS = STAGES * STAGE_BYTES > BM * BN * 2 ? STAGES * STAGE_BYTES : BM * BN * 2;
  static constexpr int GLDS = STAGE_BYTES / (THREADS * 16);  // direct-to-LDS loads per thread per stage
  static_assert(STAGE_BYTES % (THREADS * 16) == 0 && LDS <= 160 * 1024 && TI >= 1 && TJ >= 1, "tile");
  static_assert(BN % 8 == 0 && (BN / 8) <= 64, "epilogue image rows of at most 64 chunks");
  // chunk swizzle of a stage row: 64-B rows c ^ 3 ((r >> 3) & 1) (chain.hip), 128-B rows
  // c ^ ((r >> 1) & 7) (gemm.hip): conflict-free 16-row ds_read_b128 groups either way
  __device__ static int swz(int row) { return BK == 32 ? ((row >> 3) & 1) * 3 : (row >> 1) & 7; }
};

// wait until at most N of this wave's direct-to-LDS loads are in flight, then the
// workgroup barrier (one asm statement: no LDS access moves across it)
template <int N>
__device__ __forceinline__ void pt_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// at most `ahead` stages (each G loads) in flight after the oldest, ahead <= A
template <int A, int G>
__device__ __forceinline__ void pt_wait_ahead(int ahead) {
  if constexpr (A <= 0) {
    pt_wait_barrier<0>();
  } else {
    if (ahead >= A) pt_wait_barrier<A * G>();
    else pt_wait_ahead<A - 1, G>(ahead);
  }
}

// (a kernel template over an internal-linkage type gets no host stub from hipcc: the tile
// parameters are template ints and the traits struct is named inside)
template <int BM_, int BN_, int BK_, int STAGES_, int WAVES_M_>
__global__ __launch_bounds__(512, 1) void proj_gemm_kernel(const bf16* __restrict__ A, int64_t M, int64_t lda,
                                                           const bf16* __restrict__ B, int N, int K,
                                                           bf16* __restrict__ C, int64_t ldc, int tiles_n,
                                                           int nblocks) {
  using P = PT<BM_, BN_, BK_, STAGES_, WAVES_M_>;
  constexpr int BM = P::BM, BN = P::BN, BK = P::BK, ROWB = P::ROWB, CPR = P::CPR, TI = P::TI, TJ = P::TJ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // bijective XCD remap: the blocks one XCD receives (orig % 8 equal) take consecutive tiles
  const int orig = (int)blockIdx.x;
  const int q = nblocks / 8, rr = nblocks % 8, xcd = orig % 8;
  const int bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / P::WAVES_N, wc = wave % P::WAVES_N;
  const int r16 = lane & 15, g4 = lane >> 4;

  // ---- stage fill: thread t loads 16-byte pieces p = t + 512 i of the stage image: rows
  // 0..BN-1 = W rows n0.., BN.. = table rows m0..; piece p is row p / CPR, LDS chunk
  // p % CPR holding source chunk (p % CPR) ^ swz(row).  Table rows past M are clamped (their
  // outputs are never stored).
  const int KT = K / BK;
  const char* srcp[P::GLDS];
#pragma unroll
  for (int i = 0; i < P::GLDS; ++i) {
    const int p = tid + P::THREADS * i;
    const int row = p / CPR;
    if (row < BN) {
      srcp[i] = reinterpret_cast<const char*>(B + (int64_t)(n0 + row) * K) + (((p % CPR) ^ P::swz(row)) << 4);
    } else {
      const int lr = row - BN;
      int64_t m = m0 + lr;
      if (m >= M) m = M - 1;
      srcp[i] = reinterpret_cast<const char*>(A + m * lda) + (((p % CPR) ^ P::swz(lr)) << 4);
    }
  }
  auto issue = [&](int t) {
    char* st = smem + (t % P::STAGES) * P::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < P::GLDS; ++i)
    {
      // (the source as its own variable: with the pointer arithmetic inside the builtin's
      // argument list hipcc's host pass drops this kernel template's stub -- an undefined
      // symbol at load time)
      const char* src = srcp[i] + (int64_t)t * ROWB;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(st + (wave + 8 * i) * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[TJ][TI];  // [output-column tile j][vertex-row tile i]
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < P::STAGES - 1; ++t)
    if (t < KT) issue(t);

  const int aw0 = wc * P::WCOLS, bt0 = BN + wr * P::WROWS;
#pragma unroll 1
  for (int t = 0; t < KT; ++t) {
    // stage t landed (each wave's own loads, then the barrier); at most STAGES - 2 newer ones
    // stay in flight across it
    pt_wait_ahead<P::STAGES - 2, P::GLDS>(KT - 1 - t);
    if (t + P::STAGES - 1 < KT) issue(t + P::STAGES - 1);
    const char* st = smem + (t % P::STAGES) * P::STAGE_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 wf[TJ], ef[TI];
      const int c = kk * 4 + g4;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = aw0 + 16 * j + r16;
        wf[j] = *reinterpret_cast<const bf16x8*>(st + row * ROWB + ((c ^ P::swz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int lr = wr * P::WROWS + 16 * i + r16;
        ef[i] = *reinterpret_cast<const bf16x8*>(st + (BN + lr) * ROWB + ((c ^ P::swz(lr)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int i = 0; i < TI; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], ef[i], acc[j][i], 0, 0, 0);
    }
  }
  (void)bt0;
  __syncthreads();  // every wave's last fragment reads done before the image overwrites the ring

  // ---- epilogue: lane holds output columns aw0 + 16 j + 4 g4 + (0..3) of tile row
  // wr WROWS + 16 i + r16; bf16 image [BM][BN], chunk c of row r at c ^ (r & (BN/8 - 1))
  constexpr int RB = BN * 2, RC = BN / 8;
  auto img_off = [&](int row, int col) { return row * RB + ((((col >> 3) ^ (row & (RC - 1)))) << 4) + ((col & 7) << 1); };
#pragma unroll
  for (int j = 0; j < TJ; ++j)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = wr * P::WROWS + 16 * i + r16, col = aw0 + 16 * j + 4 * g4;
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      u32x2 w;
      w[0] = pack_bf16x2(acc[j][i][0], acc[j][i][1]);
      w[1] = pack_bf16x2(acc[j][i][2], acc[j][i][3]);
      *reinterpret_cast<u32x2*>(smem + img_off(row, col)) = w;
    }
  __syncthreads();
#pragma unroll 4
  for (int p = tid; p < BM * RC; p += P::THREADS) {
    const int row = p / RC, c = p % RC;
    if (m0 + row < M) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(smem + row * RB + ((c ^ (row & (RC - 1))) << 4));
      *reinterpret_cast<u32x4*>(C + (m0 + row) * ldc + n0 + c * 8) = v;
    }
  }
}

template <class P>
int launch_pt(const bf16* A, int64_t M, int64_t lda, const bf16* B, int N, int K, bf16* C, int64_t ldc,
              hipStream_t stream) {
  INF_CHECK_ARG(N % P::BN == 0 && K % P::BK == 0 && K >= P::BK, "proj_gemm: N / K not tile multiples");
  const int64_t tiles_m = ceil_div(M, P::BM);
  const int tiles_n = N / P::BN;
  INF_CHECK_ARG(tiles_m * tiles_n < (int64_t)1 << 31, "proj_gemm: too many tiles");
  const int nblocks = (int)(tiles_m * tiles_n);
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)proj_gemm_kernel<P::BM, P::BN, P::BK, P::STAGES, P::WAVES_M>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, P::LDS));
    attr = true;
  }
  proj_gemm_kernel<P::BM, P::BN, P::BK, P::STAGES, P::WAVES_M>
      <<<dim3((unsigned)nblocks), dim3(P::THREADS), P::LDS, stream>>>(A, M, lda, B, N, K, C, ldc, tiles_n, nblocks);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_proj_gemm(const bf16* A, int64_t M, int64_t lda, const bf16* B, int N, int K, bf16* C, int64_t ldc,
                     hipStream_t stream) {
  INF_CHECK_ARG(A != nullptr && B != nullptr && C != nullptr && M >= 1, "proj_gemm: operands");
  INF_CHECK_ARG(lda % 8 == 0 && ldc % 8 == 0 && lda >= K && ldc >= N, "proj_gemm: 16-byte aligned rows");
  INF_CHECK_ARG(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 == 0, "proj_gemm: 16-byte aligned operands");
  // tile variants (INF_PTAB_TILE, tools/ptab_sweep.py; 400k x 512 x 1024 on one MI355X,
  // profiles/r03/ptab_sweep.log): 1 = 256 x 256 x 64, 2 stages (default: 0.442 ms, hipBLASLt
  // 0.430), 0 = 256 x 256 x 32, 4 stages (0.489), 2 = 256 x 128 x 64, 3 stages (0.512),
  // 3 = 128 x 256 x 64, 3 stages (0.496), 4 = 256 x 128 x 32, 4 stages (0.612)
  int v = 1;
  if (const char* e = std::getenv("INF_PTAB_TILE")) v = std::atoi(e);
  if (v == 5 && N % 256 == 0 && K % 64 == 0) return launch_pt<PT<256, 256, 64, 2, 4>>(A, M, lda, B, N, K, C, ldc, stream);
  if (v == 1 && N % 256 == 0 && K % 64 == 0) return launch_pt<PT<256, 256, 64, 2, 2>>(A, M, lda, B, N, K, C, ldc, stream);
  if (v == 2 && N % 128 == 0 && K % 64 == 0) return launch_pt<PT<256, 128, 64, 3, 4>>(A, M, lda, B, N, K, C, ldc, stream);
  if (v == 3 && N % 256 == 0 && K % 64 == 0) return launch_pt<PT<128, 256, 64, 3, 2>>(A, M, lda, B, N, K, C, ldc, stream);
  if (v == 4 && N % 128 == 0 && K % 32 == 0) return launch_pt<PT<256, 128, 32, 4, 4>>(A, M, lda, B, N, K, C, ldc, stream);
  if (v == 0 && N % 256 == 0) return launch_pt<PT<256, 256, 32, 4, 2>>(A, M, lda, B, N, K, C, ldc, stream);
  INF_CHECK_ARG(N % 256 == 0 && K % 64 == 0, "proj_gemm: N must be a multiple of 256, K of 64");
  return launch_pt<PT<256, 256, 64, 2, 2>>(A, M, lda, B, N, K, C, ldc, stream);
}

}  // namespace inf
