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
#include "ptab.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::pack_bf16x2;
using c3::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int PT_BM = 256, PT_BN = 256, PT_BK = 32;
constexpr int PT_THREADS = 512;
constexpr int PT_STAGES = 4;
constexpr int PT_STAGE_BYTES = (PT_BM + PT_BN) * PT_BK * 2;  // 32 KB
constexpr int PT_LDS = PT_STAGES * PT_STAGE_BYTES;             // 128 KB (epilogue image: 128 KB)
constexpr int PT_GLDS = PT_STAGE_BYTES / (PT_THREADS * 16);    // 4 per thread per stage
static_assert(PT_BM * PT_BN * 2 <= PT_LDS, "epilogue image");

__device__ __forceinline__ int pt_swz(int row) { return ((row >> 3) & 1) * 3; }

// wait until at most N of this wave's direct-to-LDS loads are in flight, then the
// workgroup barrier (one asm statement: no LDS access moves across it)
template <int N>
__device__ __forceinline__ void pt_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(PT_THREADS, 1) void proj_gemm_kernel(const bf16* __restrict__ A, int64_t M, int64_t lda,
                                                                  const bf16* __restrict__ B, int N, int K,
                                                                  bf16* __restrict__ C, int64_t ldc, int tiles_n,
                                                                  int nblocks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // bijective XCD remap: the blocks one XCD receives (orig % 8 equal) take consecutive tiles
  const int orig = (int)blockIdx.x;
  const int q = nblocks / 8, rr = nblocks % 8, xcd = orig % 8;
  const int bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * PT_BM;
  const int n0 = tn * PT_BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // rows 128 wr .., columns 64 wc ..
  const int r16 = lane & 15, g4 = lane >> 4;

  // ---- stage fill: thread t loads 16-byte pieces p = t + 512 i (i < 4) of the stage image:
  // rows 0..255 = W rows n0.., 256..511 = table rows m0..; piece p is row p / 4, LDS chunk
  // p % 4 holding source chunk (p % 4) ^ swz(row).  Table rows past M are clamped (their
  // outputs are never stored).
  const int KT = K / PT_BK;
  const char* srcp[PT_GLDS];
#pragma unroll
  for (int i = 0; i < PT_GLDS; ++i) {
    const int p = tid + PT_THREADS * i;
    const int row = p >> 2, ch = (p & 3) ^ pt_swz(row & 255);
    if (row < PT_BN) {
      srcp[i] = reinterpret_cast<const char*>(B + (int64_t)(n0 + row) * K) + ch * 16;
    } else {
      int64_t m = m0 + (row - PT_BN);
      if (m >= M) m = M - 1;
      srcp[i] = reinterpret_cast<const char*>(A + m * lda) + ch * 16;
    }
  }
  auto issue = [&](int t) {
    char* st = smem + (t % PT_STAGES) * PT_STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < PT_GLDS; ++i)
      __builtin_amdgcn_global_load_lds(srcp[i] + (int64_t)t * PT_BK * 2, (lds_void*)(st + (wave + 8 * i) * 1024),
                                       16, 0, 0);
  };

  f32x4 acc[4][8];  // [column tile j][row tile i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < PT_STAGES - 1; ++t)
    if (t < KT) issue(t);

  // a lane's operand: 16-byte chunk g4 of row (tile row + r16)
  const int aw0 = wc * 64, bt0 = PT_BN + wr * 128;
#pragma unroll 1
  for (int t = 0; t < KT; ++t) {
    const int ahead = KT - 1 - t;  // stages issued after t (at most 2 in flight here)
    if (ahead >= 2) pt_wait_barrier<2 * PT_GLDS>();
    else if (ahead == 1) pt_wait_barrier<PT_GLDS>();
    else pt_wait_barrier<0>();
    if (t + PT_STAGES - 1 < KT) issue(t + PT_STAGES - 1);
    const char* st = smem + (t % PT_STAGES) * PT_STAGE_BYTES;
    bf16x8 wf[4], ef[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = aw0 + 16 * j + r16;
      wf[j] = *reinterpret_cast<const bf16x8*>(st + row * 64 + ((g4 ^ pt_swz(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = bt0 + 16 * i + r16;
      ef[i] = *reinterpret_cast<const bf16x8*>(st + row * 64 + ((g4 ^ pt_swz(row & 255)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], ef[i], acc[j][i], 0, 0, 0);
  }
  __syncthreads();  // every wave's last fragment reads done before the image overwrites the ring

  // ---- epilogue: lane holds output columns 64 wc + 16 j + 4 g4 + (0..3) of table row
  // 128 wr + 16 i + r16; bf16 image [256][256], chunk c of row r at c ^ (r & 31)
  auto img_off = [](int row, int col) { return row * 512 + ((((col >> 3) ^ (row & 31))) << 4) + ((col & 7) << 1); };
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + 16 * i + r16, col = wc * 64 + 16 * j + 4 * g4;
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      u32x2 w;
      w[0] = pack_bf16x2(acc[j][i][0], acc[j][i][1]);
      w[1] = pack_bf16x2(acc[j][i][2], acc[j][i][3]);
      *reinterpret_cast<u32x2*>(smem + img_off(row, col)) = w;
    }
  __syncthreads();
#pragma unroll 4
  for (int p = tid; p < PT_BM * (PT_BN / 8); p += PT_THREADS) {
    const int row = p >> 5, c = p & 31;
    if (m0 + row < M) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(smem + row * 512 + ((c ^ (row & 31)) << 4));
      *reinterpret_cast<u32x4*>(C + (m0 + row) * ldc + n0 + c * 8) = v;
    }
  }
}

}  // namespace

int launch_proj_gemm(const bf16* A, int64_t M, int64_t lda, const bf16* B, int N, int K, bf16* C, int64_t ldc,
                     hipStream_t stream) {
  INF_CHECK_ARG(A != nullptr && B != nullptr && C != nullptr && M >= 1, "proj_gemm: operands");
  INF_CHECK_ARG(N % PT_BN == 0 && K % PT_BK == 0 && K >= PT_BK, "proj_gemm: N must be a multiple of 256, K of 32");
  INF_CHECK_ARG(lda % 8 == 0 && ldc % 8 == 0 && lda >= K && ldc >= N, "proj_gemm: 16-byte aligned rows");
  INF_CHECK_ARG(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 == 0, "proj_gemm: 16-byte aligned operands");
  const int64_t tiles_m = ceil_div(M, PT_BM);
  const int tiles_n = N / PT_BN;
  INF_CHECK_ARG(tiles_m * tiles_n < (int64_t)1 << 31, "proj_gemm: too many tiles");
  const int nblocks = (int)(tiles_m * tiles_n);
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)proj_gemm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, PT_LDS));
    attr = true;
  }
  proj_gemm_kernel<<<dim3((unsigned)nblocks), dim3(PT_THREADS), PT_LDS, stream>>>(A, M, lda, B, N, K, C, ldc, tiles_n,
                                                                                  nblocks);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
