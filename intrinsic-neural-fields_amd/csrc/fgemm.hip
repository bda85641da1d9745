// Weight gradients of a large training batch: dW^T = In^T dZ over K rays, split-K, with
// both operands the fragment images the fused chain writes (chain3.hip: X^T, Y_l^T, dZ_l^T;
// lgemm.hpp layout), for batches where the per-block tiles of lgemm.hip are too small.
//
// Tile.  256 x 256 outputs per workgroup (the whole hidden-layer dW, a quarter of an
// input layer's at k = 1024), 8 waves as 2 (rows) x 4 (columns), each wave 128 x 64: 8 x 4
// v_mfma_f32_16x16x32_bf16 tiles, 128 fp32 accumulators per lane.  Per 32-ray k-step the
// workgroup moves 32 KB for 2 x 256 x 256 x 32 FLOP (128 FLOP/B: ptab.hip's ratio).
//
// Operands need no layout work: a fragment image's k block holds each 16-row tile's MFMA
// operand as one contiguous KiB (lane l's 16 bytes at 16 l), so a stage is 64 whole-KiB
// pieces (2 k blocks x 16 tiles of A, the same of B) copied by direct-to-LDS loads
// (global_load_lds_dwordx4, lane-linear: the KiB lands in fragment order) and every
// fragment read is one lane-contiguous ds_read_b128 (conflict-free, no swizzle).
//
// Pipeline: FG_NSTAGE LDS stages of one 32-ray k block each (32 KB: 16 KiB pieces of A and
// of B); up to FG_NSTAGE - 1 stages in flight per workgroup (128 KB at 5 stages), so the
// HBM latency of the streamed images is covered; one counted `s_waitcnt vmcnt` + raw
// s_barrier per k-step.  (Two 64 KB stages of 64 rays -- one stage in flight behind a
// vmcnt(0) wait -- ran at 0.29 of the MFMA peak: profiles/r03.)
// Output.  Split s writes its partial dW (f32, the update launch's slab layout): a lane's
// 4 accumulators of a tile are 4 consecutive input features of one output feature -- one
// 16-byte store.  Blocks are ordered [split][problem][row tile][column tile] and remapped
// so consecutive ones share an XCD: every tile of one split reads the same rays' panels, so
// a panel two problems share (X^T for W_0 and W_y, dZ_s^T for the skip layer's two halves,
// dZ_l^T for the column tiles of one matrix) comes from HBM once and then from that XCD's
// L2 -- problem-major order had put W_0's and W_y's tiles of a split on different XCDs.
#include "fgemm.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int FG_THREADS = 512;
#ifndef FG_NSTAGE
#define FG_NSTAGE 5
#endif
constexpr int FG_STAGES = FG_NSTAGE;
constexpr int FG_KS = 32;                                     // rays per k-step (one k block)
constexpr int FG_PIECES = 2 * (FG_KS / 32) * (FG_TILE / 16);  // KiB pieces per stage (A then B)
constexpr int FG_STAGE_BYTES = FG_PIECES * 1024;
constexpr int FG_GLDS = FG_PIECES / 8;  // direct-to-LDS loads per wave per stage
constexpr int FG_LDS = FG_STAGES * FG_STAGE_BYTES;
constexpr int FG_TI = 8, FG_TJ = 4;  // MFMA tiles per wave: A (rows) x B (columns)
static_assert(FG_LDS <= 160 * 1024, "fgemm LDS");

template <int N>
__device__ __forceinline__ void fg_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// wait until at most `ahead` stages (wave-uniform, <= N) of this wave's direct-to-LDS loads
// are in flight, then the workgroup barrier (vmcnt takes an immediate)
template <int N>
__device__ __forceinline__ void fg_wait_ahead(int ahead) {
  if constexpr (N <= 0) {
    fg_wait_barrier<0>();
  } else {
    if (ahead >= N) fg_wait_barrier<N * FG_GLDS>();
    else fg_wait_ahead<N - 1>(ahead);
  }
}

__global__ __launch_bounds__(FG_THREADS, 1) void fgemm_kernel(const FgemmBatch b) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // bijective XCD remap: the blocks one XCD receives (orig % 8 equal) take consecutive ids
  const int nblocks = b.total_blocks;
  const int orig = (int)blockIdx.x;
  const int q8 = nblocks / 8, r8 = nblocks % 8, xcd = orig % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
  const int split = bid / b.tiles_per_split;
  int r = bid - split * b.tiles_per_split;
  int pi = 0;
#pragma unroll 1
  while (pi + 1 < b.nprob && r >= b.p[pi + 1].block_begin) ++pi;
  const FgemmProblem& P = b.p[pi];
  const int tiles_n = P.N / FG_TILE;
  r -= P.block_begin;
  const int tm = r / tiles_n, tn = r - tm * tiles_n;
  // the split's 32-ray k-steps
  const int KT = b.K / FG_KS;
  const int kt0 = (int)((int64_t)split * KT / b.splits), kt1 = (int)((int64_t)(split + 1) * KT / b.splits);
  const int nk = kt1 - kt0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  // piece p = wave + 8 i of a stage: A pieces (k block p / 16, tile p % 16), then B
  const char* srcp[FG_GLDS];
  int64_t kb_stride[FG_GLDS];
#pragma unroll
  for (int i = 0; i < FG_GLDS; ++i) {
    const int p = wave + 8 * i;
    const bool isa = p < FG_PIECES / 2;
    const int pp = isa ? p : p - FG_PIECES / 2;
    const int kbl = pp / 16, t = pp % 16;
    const bf16* img = isa ? P.Af : P.Bf;
    const int tiles = isa ? P.a_tiles : P.b_tiles;
    const int t0 = (isa ? tm : tn) * (FG_TILE / 16);
    srcp[i] = reinterpret_cast<const char*>(img) +
              ((int64_t)((FG_KS / 32) * kt0 + kbl) * tiles + t0 + t) * 1024 + lane * 16;
    kb_stride[i] = (int64_t)(FG_KS / 32) * tiles * 1024;  // bytes per k-step
  }
  auto issue = [&](int t) {
    char* st = smem + (t % FG_STAGES) * FG_STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < FG_GLDS; ++i) {
      // (the source as its own variable: ptab.hip's hipcc host-stub note)
      const char* src = srcp[i] + (int64_t)t * kb_stride[i];
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(st + (wave + 8 * i) * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[FG_TJ][FG_TI];
#pragma unroll
  for (int j = 0; j < FG_TJ; ++j)
#pragma unroll
    for (int i = 0; i < FG_TI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int q = 0; q < FG_STAGES - 1; ++q)
    if (q < nk) issue(q);
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    // stage t landed (every wave's loads; later stages may stay in flight) and stage t - 1
    // is read out, so its buffer takes stage t + FG_STAGES - 1
    fg_wait_ahead<FG_STAGES - 2>(min(FG_STAGES - 2, nk - 1 - t));
    if (t + FG_STAGES - 1 < nk) issue(t + FG_STAGES - 1);
    const char* st = smem + (t % FG_STAGES) * FG_STAGE_BYTES + lane * 16;
#pragma unroll
    for (int kbl = 0; kbl < FG_KS / 32; ++kbl) {
      bf16x8 af[FG_TI], bfr[FG_TJ];
#pragma unroll
      for (int i = 0; i < FG_TI; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(st + (kbl * 16 + wr * FG_TI + i) * 1024);
#pragma unroll
      for (int j = 0; j < FG_TJ; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(st + (FG_PIECES / 2 + kbl * 16 + wc * FG_TJ + j) * 1024);
#pragma unroll
      for (int j = 0; j < FG_TJ; ++j)
#pragma unroll
        for (int i = 0; i < FG_TI; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[j][i], 0, 0, 0);
    }
  }

  // ---- partial dW of this split: output feature n = column, input features m .. m + 3
  float* slab = P.slab + (int64_t)split * P.slab_stride;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, 0x7FFFFFFF, 0x00020000);
  const int mb = tm * FG_TILE + wr * 128 + 4 * (lane >> 4);
  const int nb = tn * FG_TILE + wc * 64 + (lane & 15);
#pragma unroll
  for (int j = 0; j < FG_TJ; ++j)
#pragma unroll
    for (int i = 0; i < FG_TI; ++i) {
      const int64_t off = (int64_t)(nb + 16 * j) * P.slab_ld + mb + 16 * i;
      // write-through (sc1), as lgemm's slab stores: the update launch reads them next
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j][i]), rs, (unsigned)(off * 4), 0, 16);
    }
}

}  // namespace

int launch_fgemm(FgemmBatch& b, hipStream_t stream) {
  INF_CHECK_ARG(b.nprob >= 1 && b.nprob <= FGEMM_MAX_PROBLEMS, "fgemm: problem count");
  int64_t blocks = 0;
  for (int i = 0; i < b.nprob; ++i) {
    FgemmProblem& q = b.p[i];
    INF_CHECK_ARG(q.Af != nullptr && q.Bf != nullptr && q.slab != nullptr, "fgemm: operands");
    INF_CHECK_ARG(fgemm_shape_ok(q.M, q.N, b.K, b.splits), "fgemm: shape");
    INF_CHECK_ARG(q.a_tiles * 16 >= q.M && q.b_tiles * 16 >= q.N && q.slab_ld >= q.M &&
                      q.slab_stride >= (int64_t)q.N * q.slab_ld && q.slab_ld % 4 == 0,
                  "fgemm: image / slab extents");
    // 32-bit buffer offsets into each split's slab
    INF_CHECK_ARG((int64_t)q.N * q.slab_ld * 4 < ((int64_t)1 << 31), "fgemm: slab too large");
    q.block_begin = (int32_t)blocks;  // first tile of this problem inside a split
    blocks += (int64_t)(q.M / FG_TILE) * (q.N / FG_TILE);
  }
  INF_CHECK_ARG(blocks >= 1 && blocks * b.splits < ((int64_t)1 << 31), "fgemm: block count");
  b.tiles_per_split = (int32_t)blocks;
  b.total_blocks = (int32_t)(blocks * b.splits);
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)fgemm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, FG_LDS));
    attr = true;
  }
  fgemm_kernel<<<dim3((unsigned)b.total_blocks), dim3(FG_THREADS), FG_LDS, stream>>>(b);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
