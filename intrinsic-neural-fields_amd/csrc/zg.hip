// Input layers of the bf16 training step ahead of the register chain (chain3.hip's ZP
// schedule), gather and GEMM in one launch.
//
// Why.  Inside the fused chain every 16-ray workgroup streams the whole of W_0 and W_y
// (2 H k_pad bf16: 1 MB at config B, 4 MB at config D's k = 4096) from L2 into its
// registers -- at config D 36 of the chain's 81 us, at the per-CU L2 rate.  The input
// layers depend on nothing but the gathered features, so here they are a GEMM
// Z = [W_0; W_y] X^T tiled so that each workgroup owns 64 rays x ALL 2H output features x a
// k_pad / S slice of the features: the three table rows of a ray are read once per step
// (no feature tiling, which would re-gather them), each fragment of [W_0; W_y] feeds four
// MFMAs (the four 16-ray tiles), and the gather's HBM reads run under the MFMAs of the
// previous chunk.  The S partial sums Z_s (fp32, the chain's accumulator layout) are added
// by the chain in a fixed order (s = 0, 1, ..); X^T's fragment image for the dW GEMM is
// written from the same LDS tiles (each (ray, feature) element by exactly one workgroup).
//
// Workgroup: 512 threads, 8 waves; wave w owns output features [64 w, 64 w + 64) of the 2H
// (W_0's rows for w < 4, W_y's after), for the four ray tiles: 16 accumulators.  The feature
// slice is consumed in 256-column chunks: the gather of chunk c + 1 (12 row loads of 16 B per
// thread into registers) is in flight while the MFMAs run on chunk c from LDS; then it is
// interpolated (fp32 FMA in the reference order b0 e0 + b1 e1 + b2 e2, one bf16 rounding:
// chain3's gather numerics, mesh.py:313-324) into the other LDS chunk buffer.
#include "zg.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::u16x8;
using c3::u32x4;
using c3::s16x4x8;

constexpr int ZG_T = 512;      // 8 waves
constexpr int ZG_RAYS = 64;    // four 16-ray tiles per workgroup
constexpr int ZG_KC = 256;     // feature columns per chunk
constexpr int ZG_XROW = ZG_KC * 2;  // bytes per ray row of a chunk buffer (512)
constexpr int ZG_CHUNK = ZG_RAYS * ZG_XROW;  // 32 KB
constexpr int ZG_ITEMS = ZG_RAYS * (ZG_KC / 8) / ZG_T;  // 16-byte gather items per thread per chunk (4)
constexpr int ZG_D = 4;        // k blocks of [W_0; W_y] fragments in flight per wave

template <int H>
__global__ __launch_bounds__(ZG_T) __attribute__((amdgpu_waves_per_eu(2, 2))) void zg_kernel(const ZgArgs a) {
  static_assert(H == 256, "2H = 512 output features over 8 waves of 64");
  constexpr int TJ = 4;                 // 16-feature tiles per wave
  constexpr int NTI = 4;                // 16-ray tiles per workgroup
  constexpr int NT = H / 16;            // row tiles of one input layer's image
  __shared__ __attribute__((aligned(16))) char xs[2 * ZG_CHUNK];
  __shared__ int rvid[ZG_RAYS][3];
  __shared__ int rok[ZG_RAYS][3];
  __shared__ float rbary[ZG_RAYS][3];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int row0 = blockIdx.x * ZG_RAYS;
  const int split = blockIdx.y;
  const int k_pad = a.k_pad;
  const int kper = k_pad / a.splits;
  const int k0 = split * kper;
  const int nch = kper / ZG_KC;

  // ---- ray records (ray_dataloader.py:122-129: the loader's index select) ----------------
  if (tid < ZG_RAYS * 3) {
    int64_t offset = a.idx_offset;
    if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
    const int rl = tid / 3, i = tid % 3;
    const int b = row0 + rl;
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

  // ---- the gather: item q = tid + ZG_T g of a chunk is ray q / 32, 16-byte piece q % 32 ----
  u32x4 ev[ZG_ITEMS][3];
  auto gather = [&](int c) {
    const int col0 = k0 + c * ZG_KC;
#pragma unroll
    for (int g = 0; g < ZG_ITEMS; ++g) {
      const int q = tid + ZG_T * g;
      const int r = q >> 5, pc = q & 31;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const u32x4* src = reinterpret_cast<const u32x4*>(a.table + (int64_t)rvid[r][i] * k_pad + col0 + pc * 8);
        ev[g][i] = a.gather_nt ? __builtin_nontemporal_load(src) : *src;
      }
    }
  };
  // chunk buffer b: ray row r (512 B), 16-byte chunk p at p ^ (r & 15)
  auto interpolate = [&](int b) {
    char* xb = xs + b * ZG_CHUNK;
#pragma unroll
    for (int g = 0; g < ZG_ITEMS; ++g) {
      const int q = tid + ZG_T * g;
      const int r = q >> 5, pc = q & 31;
      const u16x8 e0 = __builtin_bit_cast(u16x8, ev[g][0]), e1 = __builtin_bit_cast(u16x8, ev[g][1]),
                  e2 = __builtin_bit_cast(u16x8, ev[g][2]);
      const float w0 = rbary[r][0], w1 = rbary[r][1], w2 = rbary[r][2];
      const bool ok = (rok[r][0] & rok[r][1] & rok[r][2]) != 0;  // any corner out of range: a zero row
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = fmaf(w2, c3::bf_val3(e2[e]), fmaf(w1, c3::bf_val3(e1[e]), w0 * c3::bf_val3(e0[e])));
        o[e] = c3::bf_bits3(ok ? x : 0.f);
      }
      *reinterpret_cast<u16x8*>(xb + r * ZG_XROW + ((pc ^ (r & 15)) << 4)) = o;
    }
  };

  // ---- [W_0; W_y] fragments: k block kb (absolute), this wave's 4 tiles --------------------
  const bf16* img = wave < 4 ? a.W0 : a.Wy;
  const int t0 = (wave & 3) * TJ;  // first row tile of this wave in its layer's image
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
  const int kb_begin = k0 / 32, nkb = kper / 32;
  auto frag = [&](int i, bf16x8 (&dst)[TJ]) {  // i: this workgroup's k block number
    i = i < nkb ? i : nkb - 1;                  // past the end: harmless reloads
#pragma unroll
    for (int j = 0; j < TJ; ++j)
      dst[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                              rw, (unsigned)((t0 + j) * 64 + lane) * 16u, (kb_begin + i) * NT * 1024, 0));
  };

  f32x4 acc[NTI][TJ];
#pragma unroll
  for (int n = 0; n < NTI; ++n)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: chunk 0's rows, the first D k blocks of fragments
  gather(0);
  bf16x8 fr[ZG_D][TJ];
#pragma unroll
  for (int d = 0; d < ZG_D; ++d) {
    frag(d, fr[d]);
    __builtin_amdgcn_sched_barrier(0);
  }
  interpolate(0);
  __syncthreads();

  // ---- X^T of a chunk (the dW GEMM's fragment image: 1 KiB per 16 features x 32 rays, lane
  // l = feature l % 16, rays 8 (l / 16) ..): units (ray tile n, feature-tile pair u), 32 per
  // chunk, four per wave; a 16-lane group reads 4 rays x 16 features with ds_read_b64_tr_b16
  const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3, trh = tg & 1;
  const int64_t img_lane = (int64_t)(ti + 16 * trh) * 16;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const __amdgpu_buffer_rsrc_t rxt = __builtin_amdgcn_make_buffer_rsrc(a.XT, (short)0, 0x7FFFFFFF, 0x00020000);
  auto copy_xt = [&](int c) {
    const char* xb = xs + (c & 1) * ZG_CHUNK;
    constexpr int NU = NTI * (ZG_KC / 32);  // 32 units
    constexpr int PER = NU / 8;             // 4 per wave
    auto addr = [&](int t, int n, int r, int q) -> const char* {  // features 16 t + 4 q .. of ray 16 n + r
      const int R = 16 * n + r;
      return xb + R * ZG_XROW + (((2 * t + (q >> 1)) ^ r) << 4) + 8 * (q & 1);
    };
#pragma unroll
    for (int h = 0; h < PER; h += 2) {  // two units at a time (registers)
      s16x4 lo[2], hi[2];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int qu = wave + 8 * (h + v);
        const int n = qu / (ZG_KC / 32), u = qu % (ZG_KC / 32);
        const int t = 2 * u + (tg >> 1);
        lo[v] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(addr(t, n, 8 * trh + tq, tp)));
        hi[v] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(addr(t, n, 8 * trh + 4 + tq, tp)));
      }
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int qu = wave + 8 * (h + v);
        const int n = qu / (ZG_KC / 32), u = qu % (ZG_KC / 32);
        const int t = (k0 + c * ZG_KC) / 16 + 2 * u + (tg >> 1);  // absolute feature tile
        const int b0n = row0 + 16 * n;
        const int64_t off = (int64_t)(b0n >> 5) * (k_pad / 16) * 1024 + ((b0n >> 4) & 1) * 512 + img_lane + (int64_t)t * 1024;
        const s16x4x8 o = {lo[v][0], lo[v][1], lo[v][2], lo[v][3], hi[v][0], hi[v][1], hi[v][2], hi[v][3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rxt, (unsigned)off, 0, 0);
      }
    }
  };

  // chunk c's MFMAs (8 k blocks; the ring slot of k block kb is (8 c + kb) % D = kb % D) and
  // its X^T pieces
  auto body = [&](int c) {
    const char* xb = xs + (c & 1) * ZG_CHUNK;
#pragma unroll
    for (int kb = 0; kb < ZG_KC / 32; ++kb) {
      const int slot = kb % ZG_D;
      bf16x8 bq[NTI];
#pragma unroll
      for (int n = 0; n < NTI; ++n)
        bq[n] = *reinterpret_cast<const bf16x8*>(xb + (16 * n + r16) * ZG_XROW + (((kb * 4 + g4) ^ r16) << 4));
#pragma unroll
      for (int n = 0; n < NTI; ++n)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[n][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[slot][j], bq[n], acc[n][j], 0, 0, 0);
      frag(c * (ZG_KC / 32) + kb + ZG_D, fr[slot]);
      __builtin_amdgcn_sched_barrier(0);
    }
    copy_xt(c);
  };
  // (the next chunk's rows are requested unconditionally inside the loop and the last chunk
  // runs after it: a conditional request would leave the compiler's waits for the ring at
  // the no-request path's count, i.e. waiting for the rows too)
#pragma unroll 1
  for (int c = 0; c + 1 < nch; ++c) {
    gather(c + 1);
    __builtin_amdgcn_sched_barrier(0);
    body(c);
    interpolate((c + 1) & 1);
    __syncthreads();
  }
  body(nch - 1);

  // ---- Z_s: the accumulators as they are (the chain's layout) -----------------------------
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
      a.Z + (int64_t)split * a.z_stride, (short)0, 0x7FFFFFFF, 0x00020000);
  constexpr int NFT = 2 * H / 16;
#pragma unroll
  for (int n = 0; n < NTI; ++n)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int ft = wave * TJ + j;  // feature tile of [W_0; W_y]
      const unsigned off = ((unsigned)((row0 / 16 + n) * NFT + ft) * 64u + (unsigned)lane) * 16u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[n][j]), rz, off, 0, 0);
    }
}

}  // namespace

int zg_splits(int k_pad, int64_t rows) {
  // S k slices so that rows / 64 x S fills the 256 CUs (at least one 256-column chunk each);
  // at most 4: the chain stages S slices of W_y x (16 KB each) in LDS beside its tiles
  int s = 1;
  while (s < 4 && (rows / ZG_RAYS) * s < 256 && k_pad % (ZG_KC * 2 * s) == 0) s *= 2;
  return s;
}

bool zg_supported(int H, int k_pad, int64_t rows) {
  return H == 256 && k_pad % ZG_KC == 0 && rows % ZG_RAYS == 0 && rows > 0 && rows <= ((int64_t)1 << 20);
}

int launch_zg(const ZgArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr && a.Z != nullptr && a.XT != nullptr &&
                    a.W0 != nullptr && a.Wy != nullptr,
                "zg: operands");
  INF_CHECK_ARG(zg_supported(a.H, a.k_pad, a.rows) && a.batch <= a.rows, "zg: shape");
  INF_CHECK_ARG(a.splits >= 1 && a.k_pad % (ZG_KC * a.splits) == 0, "zg: k slices of whole chunks");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "zg: vertex id dtype");
  INF_CHECK_ARG(a.num_vertices >= 1 && a.num_vertices <= ((int64_t)1 << 31), "zg: vertex count");
  // 32-bit buffer offsets into a Z slice and into X^T
  INF_CHECK_ARG((int64_t)a.rows * 2 * a.H * 4 < ((int64_t)1 << 31) && a.z_stride >= (int64_t)a.rows * 2 * a.H,
                "zg: Z layout");
  INF_CHECK_ARG((int64_t)a.rows * a.k_pad * 2 < ((int64_t)1 << 31), "zg: X^T too large");
  zg_kernel<256><<<dim3((unsigned)(a.rows / ZG_RAYS), (unsigned)a.splits), dim3(ZG_T), 0, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
