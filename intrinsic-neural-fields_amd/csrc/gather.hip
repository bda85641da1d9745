// Barycentric eigenfunction gather (reference: mesh.py:313-324 get_k_eigenfunc_vec_vals,
// with the loader's per-batch index-select ray_dataloader.py:122-129 fused in).
//
//   F[b][j] = bary[r][0] * E[v0][j] + bary[r][1] * E[v1][j] + bary[r][2] * E[v2][j]
//   r = ray_idx[offset + b], (v0, v1, v2) = vids[r]
//
// One 256-thread workgroup produces a 64-ray x 64-column tile.  Four consecutive lanes
// cover one 64-column segment of a vertex row (256 B fp32 / 128 B bf16), so every
// table read is a full, aligned run of cache lines; the three vertex rows of a ray are
// read by the same lanes so their FMAs stay in registers.  The row-major tile is stored
// straight from registers; the transposed copy (used by the weight-gradient GEMMs) goes
// through a padded LDS tile so both stores are coalesced.
#include <cstdlib>

#include "common.hpp"

namespace inf {

namespace {

constexpr int GT_ROWS = 64;  // rays per tile
constexpr int GT_COLS = 64;  // columns per tile
constexpr int GT_THREADS = 256;

template <typename TabT>
__device__ __forceinline__ void load16(const TabT* __restrict__ p, float (&v)[16]);

template <>
__device__ __forceinline__ void load16<float>(const float* __restrict__ p, float (&v)[16]) {
  const f32x4* q = reinterpret_cast<const f32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x4 t = q[i];
    v[4 * i + 0] = t[0];
    v[4 * i + 1] = t[1];
    v[4 * i + 2] = t[2];
    v[4 * i + 3] = t[3];
  }
}

template <>
__device__ __forceinline__ void load16<bf16>(const bf16* __restrict__ p, float (&v)[16]) {
  const bf16x8* q = reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    bf16x8 t = q[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[8 * i + j] = (float)t[j];
  }
}

template <typename OutT>
__device__ __forceinline__ void store16(OutT* __restrict__ p, const float (&v)[16]);

template <>
__device__ __forceinline__ void store16<float>(float* __restrict__ p, const float (&v)[16]) {
  f32x4* q = reinterpret_cast<f32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
}

template <>
__device__ __forceinline__ void store16<bf16>(bf16* __restrict__ p, const float (&v)[16]) {
  bf16x8* q = reinterpret_cast<bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    bf16x8 t;
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = (bf16)v[8 * i + j];
    q[i] = t;
  }
}

// Stores a 64-ray x 64-column tile held as 16 columns per lane (lane t: ray t/4, columns
// 16(t%4)..+15): the row-major copy straight from registers, the transposed copy (used by
// the weight-gradient GEMMs) through a padded LDS tile so both stores are coalesced.
template <typename OutT, bool VEC>
__device__ __forceinline__ void store_tile(const float (&acc)[16], float (&tile)[GT_COLS][GT_ROWS + 1],
                                           OutT* __restrict__ out, int64_t ld_out, int rows_out,
                                           OutT* __restrict__ out_t, int64_t ld_out_t) {
  const int t = threadIdx.x;
  const int r = t >> 2;
  const int cq = (t & 3) * 16;
  const int b = blockIdx.x * GT_ROWS + r;
  const int64_t c0 = (int64_t)blockIdx.y * GT_COLS + cq;
  if (out != nullptr && b < rows_out) {
    OutT* dst = out + (int64_t)b * ld_out + c0;
    if (VEC) {
      if (c0 < ld_out) store16<OutT>(dst, acc);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (c0 + i < ld_out) dst[i] = (OutT)acc[i];
    }
  }
  if (out_t != nullptr) {
#pragma unroll
    for (int i = 0; i < 16; ++i) tile[cq + i][r] = acc[i];
    __syncthreads();
    const int c = t >> 2;
    const int rq = (t & 3) * 16;
    const int64_t gc = (int64_t)blockIdx.y * GT_COLS + c;
    const int gb = blockIdx.x * GT_ROWS + rq;
    if (gc < ld_out) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = tile[c][rq + i];
      OutT* dst = out_t + gc * ld_out_t + gb;
      if (VEC && gb + 16 <= rows_out) {
        store16<OutT>(dst, v);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (gb + i < rows_out) dst[i] = (OutT)v[i];
      }
    }
  }
}

// VEC: table rows / output rows are 16-byte aligned and ld multiple of 16 elements, so a
// lane moves its 16 columns with vector loads/stores.  Otherwise a masked scalar path.
template <typename TabT, typename OutT, bool VEC>
__global__ __launch_bounds__(GT_THREADS) void gather_kernel(
    const TabT* __restrict__ table, int64_t V, int k, int64_t table_ld, const void* __restrict__ vids,
    int vid_dtype, const float* __restrict__ bary, const void* __restrict__ ray_idx, int idx_dtype,
    int64_t idx_offset, const int32_t* __restrict__ ctrl_batch_index, int64_t num_rays, int64_t num_src, int batch,
    OutT* __restrict__ out,
    int64_t ld_out, int rows_out, OutT* __restrict__ out_t, int64_t ld_out_t) {
  __shared__ float tile[GT_COLS][GT_ROWS + 1];

  const int t = threadIdx.x;
  const int r = t >> 2;        // ray within tile
  const int cq = (t & 3) * 16; // first column within tile
  const int b = blockIdx.x * GT_ROWS + r;
  const int64_t c0 = (int64_t)blockIdx.y * GT_COLS + cq;

  int64_t offset = idx_offset;
  if (ctrl_batch_index != nullptr) offset += (int64_t)(*ctrl_batch_index) * batch;

  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  const int64_t row = b < batch ? source_row(ray_idx, idx_dtype, offset, b, num_rays, num_src) : -1;
  if (row >= 0) {
    const float w0 = bary[3 * row + 0];
    const float w1 = bary[3 * row + 1];
    const float w2 = bary[3 * row + 2];
    const int64_t v0 = vid_at(vids, vid_dtype, 3 * row + 0);
    const int64_t v1 = vid_at(vids, vid_dtype, 3 * row + 1);
    const int64_t v2 = vid_at(vids, vid_dtype, 3 * row + 2);
    const bool vok = (uint64_t)v0 < (uint64_t)V && (uint64_t)v1 < (uint64_t)V && (uint64_t)v2 < (uint64_t)V;
    if (!vok) {
      // an out-of-range vertex id reads as a zero feature row (never outside the table)
    } else if (VEC) {
      if (c0 < k) {  // k is a multiple of 16 on this path
        float e0[16], e1[16], e2[16];
        load16<TabT>(table + v0 * table_ld + c0, e0);
        load16<TabT>(table + v1 * table_ld + c0, e1);
        load16<TabT>(table + v2 * table_ld + c0, e2);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = fmaf(w2, e2[i], fmaf(w1, e1[i], w0 * e0[i]));
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t c = c0 + i;
        if (c < k) {
          const float e0 = (float)table[v0 * table_ld + c];
          const float e1 = (float)table[v1 * table_ld + c];
          const float e2 = (float)table[v2 * table_ld + c];
          acc[i] = fmaf(w2, e2, fmaf(w1, e1, w0 * e0));
        }
      }
    }
  }

  store_tile<OutT, VEC>(acc, tile, out, ld_out, rows_out, out_t, ld_out_t);
}

// Row-major output only (no transposed copy): the reference's own product, the B x k
// feature matrix (mesh.py:313-324; inf_gather, the render's feature-gather path, the
// pre-gather slots).  A work item is (ray b, 16-byte chunk c of the table row); consecutive
// threads take consecutive chunks of one ray, so a wave reads whole 1 KiB runs of each of
// the three vertex rows and its ray records are wave-uniform (broadcast) loads.  Each thread
// takes G items (their records first, then all 3 G row chunks) and writes each output chunk
// whole.  Same arithmetic as gather_kernel: b0 e0, + b1 e1, + b2 e2 (fma).  Measured at
// config D (4096 rays x 3 rows of a 4.1 GB bf16 table, k = 4096, bf16 output;
// profiles/r05/gather_variants.txt): G = 1 22.2 us (4.5 TB/s of rows, 6.1 TB/s with the
// output), G = 2 22.9, G = 4 26.1, G = 8 33.1; non-temporal row loads +4 us; the 64 x 64
// tile kernel 25.2 us -- more, smaller workgroups keep the HBM queues fuller than deep
// per-thread batches.
constexpr int GR_ROWS_ITEMS = 1;
typedef unsigned int g_u32x4 __attribute__((ext_vector_type(4)));

template <typename TabT, typename OutT, int G, bool NT>
__global__ __launch_bounds__(GT_THREADS) void gather_rows_kernel(
    const TabT* __restrict__ table, int64_t V, int k, int64_t table_ld, const void* __restrict__ vids, int vid_dtype,
    const float* __restrict__ bary, const void* __restrict__ ray_idx, int idx_dtype, int64_t idx_offset,
    const int32_t* __restrict__ ctrl_batch_index, int64_t num_rays, int64_t num_src, int batch,
    OutT* __restrict__ out, int64_t ld_out, unsigned nchunk, unsigned total) {
  constexpr int EPC = 16 / sizeof(TabT);  // table elements per 16-byte chunk
  int64_t offset = idx_offset;
  if (ctrl_batch_index != nullptr) offset += (int64_t)(*ctrl_batch_index) * batch;
  const unsigned stride = gridDim.x * GT_THREADS;
  const unsigned i0 = blockIdx.x * GT_THREADS * G + threadIdx.x;
  unsigned bi[G], ci[G];
  bool live[G];
  int64_t v0[G], v1[G], v2[G];
  float w0[G], w1[G], w2[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const unsigned i = i0 + g * GT_THREADS;
    bi[g] = i / nchunk;
    ci[g] = i - bi[g] * nchunk;
    live[g] = false;
    v0[g] = v1[g] = v2[g] = 0;
    w0[g] = w1[g] = w2[g] = 0.f;
    if (i < total && (int)bi[g] < batch && (int)(ci[g] * EPC) < k) {
      const int64_t row = source_row(ray_idx, idx_dtype, offset, (int)bi[g], num_rays, num_src);
      if (row >= 0) {
        v0[g] = vid_at(vids, vid_dtype, 3 * row + 0);
        v1[g] = vid_at(vids, vid_dtype, 3 * row + 1);
        v2[g] = vid_at(vids, vid_dtype, 3 * row + 2);
        w0[g] = bary[3 * row + 0];
        w1[g] = bary[3 * row + 1];
        w2[g] = bary[3 * row + 2];
        // an out-of-range vertex id reads as a zero feature row (never outside the table)
        live[g] = (uint64_t)v0[g] < (uint64_t)V && (uint64_t)v1[g] < (uint64_t)V && (uint64_t)v2[g] < (uint64_t)V;
      }
    }
  }
  g_u32x4 e[G][3];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t c = (int64_t)ci[g] * EPC;
#pragma unroll
    for (int j = 0; j < 3; ++j) e[g][j] = g_u32x4{0u, 0u, 0u, 0u};
    if (live[g]) {
      const g_u32x4* p0 = reinterpret_cast<const g_u32x4*>(table + v0[g] * table_ld + c);
      const g_u32x4* p1 = reinterpret_cast<const g_u32x4*>(table + v1[g] * table_ld + c);
      const g_u32x4* p2 = reinterpret_cast<const g_u32x4*>(table + v2[g] * table_ld + c);
      if constexpr (NT) {  // rows read once: keep them out of the caches
        e[g][0] = __builtin_nontemporal_load(p0);
        e[g][1] = __builtin_nontemporal_load(p1);
        e[g][2] = __builtin_nontemporal_load(p2);
      } else {
        e[g][0] = *p0;
        e[g][1] = *p1;
        e[g][2] = *p2;
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const unsigned i = i0 + g * GT_THREADS;
    if (i >= total) continue;
    float x[EPC];
    if constexpr (sizeof(TabT) == 4) {
      // whole vectors bit-cast (a bit_cast of one subscripted element compiles to a load of
      // element 0 -- DESIGN.md section 7, round 4)
      const f32x4 a = __builtin_bit_cast(f32x4, e[g][0]), b = __builtin_bit_cast(f32x4, e[g][1]),
                  d = __builtin_bit_cast(f32x4, e[g][2]);
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = fmaf(w2[g], d[q], fmaf(w1[g], b[q], w0[g] * a[q]));
    } else {
      const bf16x8 a = __builtin_bit_cast(bf16x8, e[g][0]), b = __builtin_bit_cast(bf16x8, e[g][1]),
                   d = __builtin_bit_cast(bf16x8, e[g][2]);
#pragma unroll
      for (int q = 0; q < 8; ++q) x[q] = fmaf(w2[g], (float)d[q], fmaf(w1[g], (float)b[q], w0[g] * (float)a[q]));
    }
    if (!live[g]) {
#pragma unroll
      for (int q = 0; q < EPC; ++q) x[q] = 0.f;
    }
    OutT* dst = out + (int64_t)bi[g] * ld_out + (int64_t)ci[g] * EPC;
    if constexpr (sizeof(OutT) == 4) {
#pragma unroll
      for (int q = 0; q < EPC; q += 4) *reinterpret_cast<f32x4*>(dst + q) = f32x4{x[q], x[q + 1], x[q + 2], x[q + 3]};
    } else if constexpr (EPC == 8) {
      bf16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (bf16)x[q];
      *reinterpret_cast<bf16x8*>(dst) = o;
    } else {
      bf16x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)x[q];
      *reinterpret_cast<bf16x4*>(dst) = o;
    }
  }
  (void)stride;
}

template <typename TabT, typename OutT>
int launch_typed(const void* table, int64_t V, int k, int64_t table_ld, const void* vids, int vid_dtype,
                 const float* bary, const void* ray_idx, int idx_dtype, int64_t idx_offset, const int32_t* ctrl_bi,
                 int64_t num_rays, int64_t num_src, int batch, void* out, int64_t ld_out, int rows_out, void* out_t,
                 int64_t ld_out_t, hipStream_t stream) {
  dim3 grid((unsigned)ceil_div(rows_out, GT_ROWS), (unsigned)ceil_div(ld_out, GT_COLS));
  const bool vec = (k % 16 == 0) && (table_ld % 16 == 0) && (ld_out % 16 == 0) &&
                   (out_t == nullptr || ld_out_t % 16 == 0) && ((uintptr_t)table % 16 == 0) &&
                   ((uintptr_t)out % 16 == 0) && ((uintptr_t)out_t % 16 == 0);
  constexpr int EPC = 16 / sizeof(TabT);
  const int64_t nchunk = ld_out / EPC, total = (int64_t)rows_out * nchunk;
  if (vec && out_t == nullptr && total < ((int64_t)1 << 31) && std::getenv("INF_GATHER_TILES") == nullptr) {
    // row-major only: whole-row chunks (gather_rows_kernel); INF_GATHER_TILES=1 keeps the
    // 64 x 64 tile kernel (A/B)
    static const int gsel = [] {
      const char* e = std::getenv("INF_GATHER_G");
      return e != nullptr ? std::atoi(e) : GR_ROWS_ITEMS;
    }();
    // INF_GATHER_NT=1: non-temporal row loads (measured slower, even for tables above the MALL)
    const char* ent = std::getenv("INF_GATHER_NT");
    const bool nt = ent != nullptr && std::atoi(ent) != 0;
#define INF_GR_LAUNCH(G_, NT_)                                                                                   \
  gather_rows_kernel<TabT, OutT, G_, NT_><<<dim3((unsigned)ceil_div(total, (int64_t)GT_THREADS * G_)), GT_THREADS, 0, \
                                            stream>>>((const TabT*)table, V, k, table_ld, vids, vid_dtype, bary,        \
                                                      ray_idx, idx_dtype, idx_offset, ctrl_bi, num_rays, num_src, batch, \
                                                      (OutT*)out, ld_out, (unsigned)nchunk, (unsigned)total)
    if (gsel == 1) {
      if (nt) INF_GR_LAUNCH(1, true); else INF_GR_LAUNCH(1, false);
    } else if (gsel == 8) {
      if (nt) INF_GR_LAUNCH(8, true); else INF_GR_LAUNCH(8, false);
    } else if (gsel == 2) {
      if (nt) INF_GR_LAUNCH(2, true); else INF_GR_LAUNCH(2, false);
    } else {
      if (nt) INF_GR_LAUNCH(4, true); else INF_GR_LAUNCH(4, false);
    }
#undef INF_GR_LAUNCH
  } else if (vec) {
    gather_kernel<TabT, OutT, true><<<grid, GT_THREADS, 0, stream>>>(
        (const TabT*)table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset, ctrl_bi, num_rays,
        num_src, batch, (OutT*)out, ld_out, rows_out, (OutT*)out_t, ld_out_t);
  } else {
    gather_kernel<TabT, OutT, false><<<grid, GT_THREADS, 0, stream>>>(
        (const TabT*)table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset, ctrl_bi, num_rays,
        num_src, batch, (OutT*)out, ld_out, rows_out, (OutT*)out_t, ld_out_t);
  }
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_gather(const void* table, int table_dtype, int64_t V, int k, int64_t table_ld, const void* vids,
                  int vid_dtype, const float* bary, const void* ray_idx, int idx_dtype, int64_t idx_offset,
                  const int32_t* ctrl_batch_index, int64_t num_rays, int64_t num_src, int batch, void* out,
                  int out_dtype, int64_t ld_out, int rows_out, void* out_t, int64_t ld_out_t, hipStream_t stream) {
  INF_CHECK_ARG(table != nullptr && vids != nullptr && bary != nullptr, "gather: null input");
  INF_CHECK_ARG(k > 0 && table_ld >= k && V > 0, "gather: bad table shape");
  INF_CHECK_ARG(batch >= 0 && rows_out >= batch && ld_out >= k, "gather: bad output shape");
  INF_CHECK_ARG(out != nullptr || out_t != nullptr, "gather: no output");
  INF_CHECK_ARG(out_t == nullptr || ld_out_t >= rows_out, "gather: bad transposed output stride");
  INF_CHECK_ARG(vid_dtype == INF_DTYPE_I32 || vid_dtype == INF_DTYPE_I64, "gather: vids must be int32/int64");
  INF_CHECK_ARG(ray_idx == nullptr || idx_dtype == INF_DTYPE_I32 || idx_dtype == INF_DTYPE_I64,
                "gather: ray_idx must be int32/int64");
  if (rows_out == 0) return INF_OK;
  const bool tf = table_dtype == INF_DTYPE_F32, of = out_dtype == INF_DTYPE_F32;
  INF_CHECK_ARG(tf || table_dtype == INF_DTYPE_BF16, "gather: table dtype must be f32/bf16");
  INF_CHECK_ARG(of || out_dtype == INF_DTYPE_BF16, "gather: out dtype must be f32/bf16");
  if (tf && of)
    return launch_typed<float, float>(table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset,
                                      ctrl_batch_index, num_rays, num_src, batch, out, ld_out, rows_out, out_t, ld_out_t,
                                      stream);
  if (tf && !of)
    return launch_typed<float, bf16>(table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset,
                                     ctrl_batch_index, num_rays, num_src, batch, out, ld_out, rows_out, out_t, ld_out_t,
                                      stream);
  if (!tf && of)
    return launch_typed<bf16, float>(table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset,
                                     ctrl_batch_index, num_rays, num_src, batch, out, ld_out, rows_out, out_t, ld_out_t,
                                      stream);
  return launch_typed<bf16, bf16>(table, V, k, table_ld, vids, vid_dtype, bary, ray_idx, idx_dtype, idx_offset,
                                  ctrl_batch_index, num_rays, num_src, batch, out, ld_out, rows_out, out_t, ld_out_t,
                                      stream);
}

// Extrinsic front-ends (model.py:33-40,98-104): the barycentric hit position
// x = sum_i bary_i * P[vid_i] over the V x 3 vertex table (ray_dataloader.py:134-136),
// then RandomFourierFeatEnc / FourierFeatEnc (layers.py:6-39), written straight into the
// plan's X / X^T tiles (or an fp32 feature matrix): the B x in_dim encoding never exists
// as a separate tensor.
//
// Tiles and stores as in gather_kernel (64 rays x 64 columns, whole-line vector stores
// of X and, through LDS, X^T -- scattered 2-byte stores made this kernel 8x slower).
// Each lane recomputes its ray's x (3 x 12 B of L2-resident vertex rows); sincos uses a
// three-constant Cody-Waite reduction by pi/2 and minimax polynomials on [-pi/4, pi/4]
// (<= 1e-7 abs for |e| < 2^15; larger arguments take ocml's sincosf).
namespace {
template <typename OutT, bool VEC>
__global__ __launch_bounds__(GT_THREADS) void encode_kernel(
    const float* __restrict__ table, int64_t V, const void* __restrict__ vids, int vid_dtype,
    const float* __restrict__ bary, const void* __restrict__ ray_idx, int idx_dtype, int64_t idx_offset,
    const int32_t* __restrict__ ctrl_batch_index, int64_t num_rays, int64_t num_src, int batch, int enc, int ek,
    const float* __restrict__ proj, int in_dim, int ne, OutT* __restrict__ out, int64_t ld_out, int rows_out,
    OutT* __restrict__ out_t, int64_t ld_out_t) {
  __shared__ float tile[GT_COLS][GT_ROWS + 1];
  const int t = threadIdx.x;
  const int r = t >> 2;
  const int cq = (t & 3) * 16;
  const int b = blockIdx.x * GT_ROWS + r;
  const int c0 = (int)blockIdx.y * GT_COLS + cq;
  int64_t offset = idx_offset;
  if (ctrl_batch_index != nullptr) offset += (int64_t)(*ctrl_batch_index) * batch;

  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const int64_t row = b < batch && c0 < in_dim ? source_row(ray_idx, idx_dtype, offset, b, num_rays, num_src) : -1;
  if (row >= 0) {
    float x[3] = {0.f, 0.f, 0.f};
    if (vids == nullptr) {
      if ((uint64_t)row < (uint64_t)V) {
        x[0] = table[3 * row + 0];
        x[1] = table[3 * row + 1];
        x[2] = table[3 * row + 2];
      }
    } else {
      const float w0 = bary[3 * row + 0], w1 = bary[3 * row + 1], w2 = bary[3 * row + 2];
      const int64_t v0 = vid_at(vids, vid_dtype, 3 * row + 0);
      const int64_t v1 = vid_at(vids, vid_dtype, 3 * row + 1);
      const int64_t v2 = vid_at(vids, vid_dtype, 3 * row + 2);
      if ((uint64_t)v0 < (uint64_t)V && (uint64_t)v1 < (uint64_t)V && (uint64_t)v2 < (uint64_t)V) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          x[c] = fmaf(w2, table[3 * v2 + c], fmaf(w1, table[3 * v1 + c], w0 * table[3 * v0 + c]));
      }
    }
    // RFF: (2 * torch.pi * x) is an fp32 product with the fp32-rounded 2 pi
    const float tp = 6.283185307179586f;
    const float px[3] = {tp * x[0], tp * x[1], tp * x[2]};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = c0 + i;
      float v = 0.f;
      if (c < 2 * ne) {
        const int j = c < ne ? c : c - ne;
        float e;
        if (enc == INF_ENC_RFF)
          e = fmaf(px[2], proj[2 * ek + j], fmaf(px[1], proj[ek + j], px[0] * proj[j]));
        else
          e = pick3(x, j / ek) * proj[j % ek];
        float sn, cs;
        fast_sincos(e, &sn, &cs);
        v = c < ne ? cs : sn;
      } else if (c < in_dim) {
        v = pick3(x, c - 2 * ne);  // the include_input tail (or the xyz strategy itself)
      }
      acc[i] = v;
    }
  }
  store_tile<OutT, VEC>(acc, tile, out, ld_out, rows_out, out_t, ld_out_t);
}
}  // namespace

int encoded_dim(int enc, int k, int inc) {
  if (enc == INF_ENC_XYZ) return 3;
  if (k < 1 || (inc != 0 && inc != 1)) return -1;
  if (enc == INF_ENC_RFF) return 2 * k + 3 * inc;
  if (enc == INF_ENC_FF) return 6 * k + 3 * inc;
  return -1;
}

int launch_encode(const float* table, int64_t V, const void* vids, int vid_dtype, const float* bary,
                  const void* ray_idx, int idx_dtype, int64_t idx_offset, const int32_t* ctrl_batch_index,
                  int64_t num_rays, int64_t num_src, int batch, int enc, int enc_k, const float* proj, int inc,
                  void* out, int out_dtype, int64_t ld_out, int rows_out, void* out_t, int64_t ld_out_t,
                  hipStream_t stream) {
  const int in_dim = encoded_dim(enc, enc_k, inc);
  INF_CHECK_ARG(in_dim > 0, "encode: bad encoding / k / include_input");
  INF_CHECK_ARG(table != nullptr && V > 0, "encode: null or empty vertex table");
  INF_CHECK_ARG(vids == nullptr || (bary != nullptr && (vid_dtype == INF_DTYPE_I32 || vid_dtype == INF_DTYPE_I64)),
                "encode: vids must be int32/int64 with barycentrics");
  INF_CHECK_ARG(enc == INF_ENC_XYZ || proj != nullptr, "encode: missing projection / frequency bands");
  INF_CHECK_ARG(batch >= 0 && rows_out >= batch && ld_out >= in_dim, "encode: bad output shape");
  INF_CHECK_ARG(out != nullptr || out_t != nullptr, "encode: no output");
  INF_CHECK_ARG(out_t == nullptr || ld_out_t >= rows_out, "encode: bad transposed output stride");
  INF_CHECK_ARG(ray_idx == nullptr || idx_dtype == INF_DTYPE_I32 || idx_dtype == INF_DTYPE_I64,
                "encode: ray_idx must be int32/int64");
  INF_CHECK_ARG(out_dtype == INF_DTYPE_F32 || out_dtype == INF_DTYPE_BF16, "encode: out dtype must be f32/bf16");
  if (rows_out == 0) return INF_OK;
  const int ne = enc == INF_ENC_XYZ ? 0 : (enc == INF_ENC_RFF ? enc_k : 3 * enc_k);  // arguments per ray
  dim3 grid((unsigned)ceil_div(rows_out, GT_ROWS), (unsigned)ceil_div(ld_out, GT_COLS));
  const bool vec = (ld_out % 16 == 0) && (out_t == nullptr || ld_out_t % 16 == 0) && ((uintptr_t)out % 16 == 0) &&
                   ((uintptr_t)out_t % 16 == 0);
#define INF_ENC_LAUNCH(T, V)                                                                                      \
  encode_kernel<T, V><<<grid, GT_THREADS, 0, stream>>>(table, V_rows, vids, vid_dtype, bary, ray_idx, idx_dtype,   \
                                                       idx_offset, ctrl_batch_index, num_rays, num_src, batch, enc, enc_k, \
                                                       proj, in_dim, ne, (T*)out, ld_out, rows_out, (T*)out_t,    \
                                                       ld_out_t)
  const int64_t V_rows = V;
  if (out_dtype == INF_DTYPE_F32) {
    if (vec) INF_ENC_LAUNCH(float, true); else INF_ENC_LAUNCH(float, false);
  } else {
    if (vec) INF_ENC_LAUNCH(bf16, true); else INF_ENC_LAUNCH(bf16, false);
  }
#undef INF_ENC_LAUNCH
  INF_LAUNCH_CHECK();
  return INF_OK;
}

// Features given by the caller (model(batch) with batch["eigenfunctions"], model.py:104):
// the same tile machinery with an identity "gather" (one vertex, weight 1).
namespace {
template <typename OutT>
__global__ __launch_bounds__(GT_THREADS) void pack_kernel(const float* __restrict__ in, int64_t ld_in, int k, int batch,
                                                          OutT* __restrict__ out, int64_t ld_out, int rows_out,
                                                          OutT* __restrict__ out_t, int64_t ld_out_t) {
  __shared__ float tile[GT_COLS][GT_ROWS + 1];
  const int t = threadIdx.x;
  const int r = t >> 2;
  const int cq = (t & 3) * 16;
  const int b = blockIdx.x * GT_ROWS + r;
  const int64_t c0 = (int64_t)blockIdx.y * GT_COLS + cq;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t c = c0 + i;
    v[i] = (b < batch && c < k) ? in[(int64_t)b * ld_in + c] : 0.f;
  }
  if (out != nullptr && b < rows_out) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (c0 + i < ld_out) out[(int64_t)b * ld_out + c0 + i] = (OutT)v[i];
  }
  if (out_t != nullptr) {
#pragma unroll
    for (int i = 0; i < 16; ++i) tile[cq + i][r] = v[i];
    __syncthreads();
    const int c = t >> 2;
    const int rq = (t & 3) * 16;
    const int64_t gc = (int64_t)blockIdx.y * GT_COLS + c;
    const int gb = blockIdx.x * GT_ROWS + rq;
    if (gc < ld_out) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (gb + i < rows_out) out_t[gc * ld_out_t + gb + i] = (OutT)tile[c][rq + i];
    }
  }
}
}  // namespace

int launch_pack_features(const float* in, int64_t ld_in, int k, int batch, void* out, int out_dtype, int64_t ld_out,
                         int rows_out, void* out_t, int64_t ld_out_t, hipStream_t stream) {
  INF_CHECK_ARG(in != nullptr && ld_in >= k && ld_out >= k && rows_out >= batch, "pack_features: bad shape");
  if (rows_out == 0) return INF_OK;
  dim3 grid((unsigned)ceil_div(rows_out, GT_ROWS), (unsigned)ceil_div(ld_out, GT_COLS));
  if (out_dtype == INF_DTYPE_F32)
    pack_kernel<float><<<grid, GT_THREADS, 0, stream>>>(in, ld_in, k, batch, (float*)out, ld_out, rows_out,
                                                         (float*)out_t, ld_out_t);
  else
    pack_kernel<bf16><<<grid, GT_THREADS, 0, stream>>>(in, ld_in, k, batch, (bf16*)out, ld_out, rows_out,
                                                        (bf16*)out_t, ld_out_t);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace inf
