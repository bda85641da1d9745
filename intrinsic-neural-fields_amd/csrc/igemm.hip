// Input layers of the bf16 training step ahead of the register chain (chain3.hip, ZP).
//
// Why.  Inside the fused chain every 16-ray workgroup streams the whole of W_0 and W_y
// (2 x H x k_pad bf16: 1 MB at config B, 40 % of its 2.6 MB weight stream) from L2 into
// its registers, because a workgroup needs every output feature of a layer before the next
// one.  The input layers have no such dependency on each other or on the hidden layers
// (W_y x does not depend on h), so they are a plain GEMM Z = [W_0; W_y] X^T that can be
// tiled over output features: a 128-feature x 64-ray tile moves 384 KB per CU for 16.8
// MFLOP, against 1 MB per 16 rays inside the chain.  The chain then starts from Z (its
// phase 0 is the layer-0 epilogue) and adds W_y x in the skip layer's epilogue.
//
// xgather_kernel  the barycentric gather (mesh.py:313-324; the loader's index select,
//                 ray_dataloader.py:122-129) of a 32-ray x 128-column tile: fp32 FMA in the
//                 reference order b0 e0 + b1 e1 + b2 e2 rounded to bf16 once (chain3's
//                 gather, bit for bit); writes X as this GEMM's B-operand image (whole
//                 KiB pieces, see below) and the X^T fragment image of the dW GEMM (what
//                 chain3's store wave wrote).
// igemm_kernel    Z^T tile = W rows (A: the forward fragment images, streamed into a
//                 registers per wave) x X rows (B: the tile's 64 rays staged once in LDS
//                 by direct-to-LDS loads of whole pieces -- one 1 KiB piece per 32
//                 features x 16 rays, lane l's 16 bytes = ray l % 16, features 8 (l / 16)..);
//                 each A fragment feeds four MFMAs (the four 16-ray tiles), and the
//                 accumulators are stored as they are: the chain's accumulator layout.
#include "igemm.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::u16x8;
using c3::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int XG_R = 32, XG_C = 128, XG_T = 256;
constexpr int XG_ROWB = XG_C * 2 + 16;  // padded LDS row: the column reads of X^T hit 2 banks per group

__global__ __launch_bounds__(XG_T) void xgather_kernel(const XGatherArgs a) {
  __shared__ __attribute__((aligned(16))) char tile[XG_R * XG_ROWB];
  __shared__ int rvid[XG_R][3];  // vertex ids
  __shared__ int rok[XG_R][3];   // vertex id in range
  __shared__ float rbary[XG_R][3];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * XG_R;
  const int c0 = blockIdx.y * XG_C;
  const int k_pad = a.k_pad;
  if (tid < XG_R * 3) {
    int64_t offset = a.idx_offset;
    if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
    const int rl = tid / 3, i = tid % 3;
    const int b = r0 + rl;
    int v = 0, ok = 0;
    float w = 0.f;
    const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src) : -1;
    if (rr >= 0) {
      const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
      ok = (uint64_t)e < (uint64_t)a.num_vertices;  // out of range: a zero feature row
      v = ok ? (int)e : 0;
      w = a.bary[3 * rr + i];
    }
    rvid[rl][i] = v;
    rbary[rl][i] = w;
    rok[rl][i] = ok;
  }
  __syncthreads();
  // 32 rays x 16 chunks of 8 columns: two chunks per thread, all six row loads first
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.table), (short)0, (int)0xFFFFFFFFu, 0x00020000);
  u16x8 ev[2][3];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int q = tid + XG_T * g;
    const int r = q >> 4, ch = q & 15;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const unsigned off = ((unsigned)rvid[r][i] * (unsigned)k_pad + c0 + ch * 8) * 2u;
      ev[g][i] = __builtin_bit_cast(u16x8, a.gather_nt ? __builtin_amdgcn_raw_buffer_load_b128(rt, off, 0, 2)
                                                        : __builtin_amdgcn_raw_buffer_load_b128(rt, off, 0, 0));
    }
  }
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int q = tid + XG_T * g;
    const int r = q >> 4, ch = q & 15;
    const bool ok = (rok[r][0] & rok[r][1] & rok[r][2]) != 0;  // any corner out of range: a zero row
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = fmaf(rbary[r][2], c3::bf_val3(ev[g][2][e]),
                           fmaf(rbary[r][1], c3::bf_val3(ev[g][1][e]), rbary[r][0] * c3::bf_val3(ev[g][0][e])));
      o[e] = c3::bf_bits3(ok ? x : 0.f);
    }
    *reinterpret_cast<u16x8*>(tile + r * XG_ROWB + ch * 16) = o;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  // X as the GEMM's B-operand image: per 16-ray tile n and 32-column k block kb one KiB,
  // lane l's 16 bytes = ray 16 n + l % 16, columns 32 kb + 8 (l / 16) .. + 7 (so the GEMM's
  // direct-to-LDS loads read whole KiB pieces); 2 ray tiles x 4 k blocks, two per wave
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int piece = wave * 2 + pp;
    const int n = piece >> 2, kbl = piece & 3;
    const u16x8 v = *reinterpret_cast<const u16x8*>(tile + (16 * n + (lane & 15)) * XG_ROWB + (kbl * 4 + (lane >> 4)) * 16);
    char* dst = reinterpret_cast<char*>(a.X) + (((int64_t)(r0 / 16 + n) * (k_pad / 32) + c0 / 32 + kbl) * 64 + lane) * 16;
    *reinterpret_cast<u16x8*>(dst) = v;
  }
  // X^T: eight 1 KiB blocks of 16 features x 32 rays; lane i + 16 g holds feature i's rays
  // 8 g .. 8 g + 7 (natural k order); wave w writes blocks 2 w and 2 w + 1
  const int fi = lane & 15, fg = lane >> 4;
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const int fb = wave * 2 + bb;
    const unsigned short* col = reinterpret_cast<const unsigned short*>(tile + (fb * 16 + fi) * 2);
    u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = col[(8 * fg + e) * (XG_ROWB / 2)];
    char* dst = reinterpret_cast<char*>(a.XT) + ((int64_t)(r0 / 32) * (k_pad / 16) + c0 / 16 + fb) * 1024 + lane * 16;
    *reinterpret_cast<u16x8*>(dst) = v;
  }
}

constexpr int IG_T = 512;    // 8 waves, one 16-feature tile each
constexpr int IG_RAYS = 64;  // four 16-ray tiles per workgroup

// NKB = k_pad / 32 k blocks.  Every load is issued up front, in two halves (each: the
// wave's A fragments of the half's k blocks, then its share of the B pieces), so a CU has
// its whole 384 KB in flight -- a ring refilled one k block at a time was latency-bound
// (11.8 us at config B); the first half's MFMAs run while the second half lands.
template <int NKB>
__global__ __launch_bounds__(IG_T) void igemm_kernel(const IGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [NKB][4] KiB pieces
  static_assert(NKB % 4 == 0, "halves of whole piece rounds");
  constexpr int HALF = NKB / 2;
  constexpr int PPW = HALF * 4 / 8;  // B pieces per wave per half
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = blockIdx.x * IG_RAYS;
  const int NT = a.H / 16;               // row tiles of a weight image
  const int ft = blockIdx.y * 8 + wave;  // feature tile of [W_0; W_y]
  const bf16* img = ft < NT ? a.W0 : a.Wy;
  const int t = ft < NT ? ft : ft - NT;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
  const unsigned aoff = (unsigned)t * 1024u + (unsigned)lane * 16u;
  // B piece p = kb 4 + n (k block kb, ray tile n) <- the contiguous KiB of X's image (ray
  // tile row0 / 16 + n, k block kb), one direct-to-LDS load per piece
  const char* xim = reinterpret_cast<const char*>(a.X) + ((int64_t)(row0 / 16) * NKB * 64 + lane) * 16;
  bf16x8 fr[NKB];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int u = 0; u < HALF; ++u)
      fr[h * HALF + u] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff, (h * HALF + u) * NT * 1024, 0));
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = h * HALF * 4 + wave + 8 * i;
      const char* src = xim + ((int64_t)(p & 3) * NKB + (p >> 2)) * 1024;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(smem + p * 1024), 16, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* bl = smem + lane * 16;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // this half's loads landed (every wave's: the barrier)
    if (h == 0) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HALF + PPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int u = 0; u < HALF; ++u) {
      const int kb = h * HALF + u;
      bf16x8 bv[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) bv[n] = *reinterpret_cast<const bf16x8*>(bl + (kb * 4 + n) * 1024);
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb], bv[n], acc[n], 0, 0, 0);
    }
  }
  const int NFT = 2 * NT;
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(a.Z, (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const unsigned off = ((unsigned)((row0 / 16 + n) * NFT + ft) * 64u + (unsigned)lane) * 16u;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[n]), rz, off, 0, 0);
  }
}

template <int NKB>
int launch_igemm_k(const IGemmArgs& a, hipStream_t stream) {
  const int lds = NKB * 4 * 1024;
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)igemm_kernel<NKB>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = true;
  }
  igemm_kernel<NKB><<<dim3((unsigned)(a.rows / IG_RAYS), (unsigned)(2 * a.H / 128)), dim3(IG_T), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_xgather(const XGatherArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr && a.X != nullptr && a.XT != nullptr,
                "xgather: inputs");
  INF_CHECK_ARG(a.k_pad % XG_C == 0 && a.rows % XG_R == 0 && a.rows > 0 && a.batch <= a.rows, "xgather: shape");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "xgather: vertex id dtype");
  // 32-bit buffer offsets of table rows
  INF_CHECK_ARG(a.num_vertices * (int64_t)a.k_pad * 2 < ((int64_t)1 << 32), "xgather: table above 4 GiB");
  xgather_kernel<<<dim3((unsigned)(a.rows / XG_R), (unsigned)(a.k_pad / XG_C)), dim3(XG_T), 0, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int launch_igemm(const IGemmArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(a.X != nullptr && a.W0 != nullptr && a.Wy != nullptr && a.Z != nullptr, "igemm: operands");
  INF_CHECK_ARG(igemm_supported(a.H, a.k_pad, a.rows), "igemm: shape");
  // 32-bit buffer offsets into Z
  INF_CHECK_ARG((int64_t)a.rows * 2 * a.H * 4 < ((int64_t)1 << 31), "igemm: Z too large");
  switch (a.k_pad / 32) {
    case 8: return launch_igemm_k<8>(a, stream);
    case 16: return launch_igemm_k<16>(a, stream);
    case 24: return launch_igemm_k<24>(a, stream);
    default: return launch_igemm_k<32>(a, stream);
  }
}

}  // namespace inf
