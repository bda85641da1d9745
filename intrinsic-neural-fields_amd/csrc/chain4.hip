// Large-batch fused training chain (chain3.hip's step, re-tiled for batches above
// CHAIN3_MAX_ROWS): gather -> forward -> head + loss -> dX chain for 128 rays per workgroup,
// leaving the X^T / Y^T / dZ^T fragment images and the bias / head / loss partials the dW
// GEMM (fgemm.hip) and the update launch read -- the same outputs as chain3's wide tiles.
//
// Why a second kernel.  chain3's wide tiles (64 rays per workgroup) re-stream the whole
// weight set (2.6 MB of fragment images) once per 64 rays; at 128 rays every fragment
// fetched from L2 feeds 8 MFMAs and the per-CU stream halves per ray.  A workgroup is EIGHT
// waves, two per SIMD (256 registers each): wave w owns output features [32 w, 32 w + 32)
// (TN = 2 tiles of 16) for all RT = 8 ray tiles, with a D = 8 k-block fragment ring in the
// hidden layers (one whole layer in flight: 8 waves x 8 x 2 KB = 128 KB per CU) and D0 = 4
// (one chunk's k blocks) in phase 0, where W_y x holds a second accumulator set.  Both input layers'
// accumulator sets (W_0 x and W_y x) stay in registers from phase 0 to the skip layer, so
// the feature tile is gathered once per step, in 64-column chunks.
//
// The gather.  Table rows move by direct-to-LDS loads (global_load_lds_dwordx4, no
// registers): chunk c's raw rows (128 rays x 3 vertices x 128 B) land in one of two LDS
// buffers, two chunks ahead of the MFMAs -- the activation region (unused until the first
// epilogue) and a second 48 KB buffer that the head's scratch reuses later.  The vector-
// memory counter retires in order, so a chunk issues its ring refills (the next chunk's
// fragments) BEFORE the loads of chunk c + 2, and the wait for chunk c is a fixed count of
// this wave's later memory operations (c4_wait below); every wave issues the same sequence.
// Each chunk is then interpolated (fp32 FMA in the reference order b0 e0 + b1 e1 + b2 e2,
// one bf16 rounding: chain3's gather numerics) into the 16 KB feature chunk X.
//
// One activation buffer (64 KiB for 128 rays x 256 features): an epilogue writes the next
// layer's input into the tile the layer just read, behind a barrier that ends the reads
// (B1), and a second barrier publishes it (B2).  The X^T / Y^T / dZ^T images are copied by
// all eight waves out of the LDS tiles (ds_read_b64_tr_b16 transposes, whole-line write-
// through stores) right after B2, while the next phase's fragments are in flight.
//
// Numerics are chain3's chunked wide schedule's: the same MFMA k order for W_0 x and W_y x
// (two fp32 sums, added in the skip epilogue with the biases last), bf16-rounded ReLU
// outputs, the head, loss and dL/dz in fp32.  Only the fp32 summation orders of the head's
// dot products and of the per-workgroup partials differ (128 rays, 8 waves).
#include <cstdlib>
#include <utility>

#include "c3common.hpp"
#include "chain3.hpp"

namespace inf {
namespace {

using namespace c3;
typedef __attribute__((address_space(3))) void lds_void;

constexpr float C4_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);

// 1 if x != 0 else 0, as one v_min_u32 (a compare would put its lane mask in an SGPR pair)
__device__ __forceinline__ unsigned nz1_4(unsigned x) {
  unsigned r;
  asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(x));
  return r;
}

// wait until at most n of this wave's vector-memory operations are in flight, then the
// workgroup barrier (n: one of the counts the phase-0 schedule produces; else a full drain)
__device__ __forceinline__ void c4_wait(int n) {
  switch (n) {
    case 14: asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
  }
}

template <int NL>
struct L4 {
  static constexpr int H = 256, CW = 8, THREADS = CW * 64;
  static constexpr int RT = C4_BM / 16;           // 16-ray MFMA tiles per workgroup (8)
  static constexpr int BM = C4_BM;
  static constexpr int TN = H / (16 * CW);        // 16-feature tiles per wave (2)
  static constexpr int UPL = H / 32;              // k blocks per hidden layer (8)
  static constexpr int NT = H / 16;               // 16-row tiles per k block of a hidden image
  static constexpr int KC = C4_KC;                // feature columns per gathered chunk (64)
  static constexpr int KBC = KC / 32;             // k blocks per chunk (2)
  static constexpr int TILE_BYTES = 16 * H * 2;   // one 16-ray activation tile (act_off layout)
  static constexpr int ACT_BYTES = RT * TILE_BYTES;
  static constexpr int XROW = KC * 2;             // bytes per ray row of a chunk (128)
  static constexpr int RAW_BYTES = BM * 3 * XROW; // raw rows of a chunk: [ray][vertex][KC] bf16
  static constexpr int DMA = RAW_BYTES / (CW * 1024);  // direct-to-LDS loads per wave per chunk (6)
  static constexpr int XT_STORES = RT * (KC / 32) / CW;  // X^T image stores per wave per chunk (2)
  static constexpr int OFF_ACT = 0;                                   // raw buffer 0 in phase 0
  static constexpr int OFF_RAW1 = OFF_ACT + ACT_BYTES;                // raw buffer 1 in phase 0
  static constexpr int OFF_YPARK = OFF_RAW1;                          // after phase 0: W_y x of ray tiles RT/2.., fp32
  static constexpr int OFF_ZP = OFF_RAW1;                             // [CW][BM][3] head partial dots
  static constexpr int OFF_DZ = OFF_ZP + CW * BM * 12;                // [CW][BM][3] dL/dz (a copy per wave)
  static constexpr int OFF_X = OFF_RAW1 + RAW_BYTES;                  // [BM][KC] bf16, 16-B chunks swizzled
  static constexpr int OFF_VEC = OFF_X + BM * XROW;                   // biases [NL-1][H], Ly.bias [H]
  static constexpr int OFF_W7 = OFF_VEC + NL * H * 4;                 // [3][H], b7[3]
  static constexpr int OFF_TGT = OFF_W7 + 3 * H * 4 + 16;             // [BM][3] targets
  static constexpr int OFF_PRED = OFF_TGT + BM * 12;                  // [BM][3]
  static constexpr int OFF_RAY = OFF_PRED + BM * 12;                  // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RBARY = OFF_RAY + BM * 16 + BM * 12;       // [BM][3] barycentrics
  static constexpr int OFF_LS = OFF_RBARY + BM * 12;                  // [2] f64 loss / SSE
  static constexpr int LDS = OFF_LS + 16;
  static_assert(RAW_BYTES % (CW * 1024) == 0 && (RT * (KC / 32)) % CW == 0, "uniform per-wave memory ops");
  static_assert(OFF_DZ + CW * BM * 12 <= OFF_X, "head scratch inside raw buffer 1");
  static_assert(OFF_YPARK + (RT / 2) * TN * THREADS * 16 <= OFF_VEC, "W_y x park inside raw buffer 1 + X");
  static_assert(OFF_VEC % 16 == 0 && OFF_W7 % 16 == 0 && OFF_LS % 8 == 0, "LDS alignment");
  static_assert(LDS <= 160 * 1024, "chain4: LDS budget");
};

// NL = num_layers (one instantiation: the 8-layer field of configs B / C / D / E)
template <int NL, int LOSS>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void chain4_kernel(const Chain3Args a) {
  using C = L4<NL>;
  constexpr int H = C::H, RT = C::RT, BM = C::BM, TN = C::TN, UPL = C::UPL, KBC = C::KBC, CW = C::CW;
  constexpr int NV = TN * 4;          // accumulator values per lane and ray tile (8)
  constexpr int PW = 32 / NV;         // ray tiles per mask word (4)
  constexpr int MW = RT / PW;         // mask words per layer (2)
  constexpr int D = 8;                // fragment ring depth (k blocks in flight), hidden layers
  constexpr int D0 = 2 * KBC;         // ... phase 0: one chunk's k blocks (4)
  constexpr int MST = NL - 2;         // ReLU masks kept: Y_0 .. Y_{NL-3}
  static_assert(UPL % D == 0 && D % D0 == 0, "ring slots are static per k block");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int s = a.s, k_pad = a.k_pad;
  char* act = smem + C::OFF_ACT;
  char* xs = smem + C::OFF_X;
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* preds = reinterpret_cast<float*>(smem + C::OFF_PRED);
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RBARY);
  double* lss = reinterpret_cast<double*>(smem + C::OFF_LS);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int64_t part0 = blockIdx.x;  // one partial per workgroup
  const int t0 = wc * TN;           // the wave's first 16-feature tile
  // diagnostics (tools/chain4_timing.py): wave 0 of the first and the last workgroup stamps
  // the wall clock (100 MHz) at every step of its schedule, C4_STAMPS slots each
  unsigned long long* stl = nullptr;
  if (a.stamps != nullptr && wc == 0 && lane == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    stl = a.stamps + (blockIdx.x == 0 ? 0 : C4_STAMPS);
  int nst = 0;
  auto stamp = [&]() {
    if (stl != nullptr) {
      __builtin_amdgcn_sched_barrier(0);
      if (nst < C4_STAMPS) stl[nst] = wall_clock64();
      ++nst;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp();  // entry

  // ---- ray records, targets, vectors ----------------------------------------------------
  int64_t offset = a.idx_offset;
  if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
  for (int x = tid; x < BM * 3; x += C::THREADS) {
    const int rl = x / 3, i = x % 3;
    const int b = b0 + rl;
    int v = 0, ok = 0;
    float w = 0.f, tt = 0.f;
    const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src) : -1;
    if (rr >= 0) {
      const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
      ok = (uint64_t)e < (uint64_t)a.num_vertices;  // an out-of-range id reads as a zero row
      v = ok ? (int)e : 0;
      w = a.bary[3 * rr + i];
      tt = a.rgb[3 * rr + i];
    }
    rvid[rl * 4 + i] = v;
    rbary[rl * 3 + i] = w;
    rvid[BM * 4 + x] = ok;
    tgs[x] = tt;
  }
  for (int i = tid; i < (NL - 1) * H; i += C::THREADS) vecs[i] = a.bias[i / H][i % H];
  for (int i = tid; i < H; i += C::THREADS) vecs[(NL - 1) * H + i] = a.bias_y[i];
  for (int i = tid; i < 3 * H + 3; i += C::THREADS) w7s[i] = i < 3 * H ? a.W7[i] : a.b7[i - 3 * H];
  if (a.count_step && blockIdx.x == 0 && tid == 0) a.ctrl->step += 1;
  lbar();  // records, targets, vectors in LDS
  stamp();

  // ---- the gather's direct-to-LDS loads: raw rows of chunk c into buffer c & 1 -----------
  // piece p = (ray 3 + vertex) 8 + q (16 bytes, columns c KC + 8 q ..); wave wc's load j
  // writes the KiB of pieces (wc + CW j) 64 .. + 63 (lane-linear)
  const int nchunk = k_pad / C::KC;
  auto dma = [&](int c) {
    char* rb = smem + ((c & 1) ? C::OFF_RAW1 : C::OFF_ACT);
#pragma unroll
    for (int j = 0; j < C::DMA; ++j) {
      const int p = (wc + CW * j) * 64 + lane;
      const int r = p / 24, i = (p >> 3) % 3, q = p & 7;
#ifdef C4_DIAG_ROW0  // diagnostic: every ray reads vertex 0's row (cache hits)
      const bf16* src = a.table + (int64_t)(0 * rvid[r * 4 + i]) * k_pad + c * C::KC + q * 8;
#else
      const bf16* src = a.table + (int64_t)rvid[r * 4 + i] * k_pad + c * C::KC + q * 8;
#endif
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(rb + (wc + CW * j) * 1024), 16, 0, 0);
    }
  };
  dma(0);
  if (nchunk > 1) dma(1);

  // ---- the weight stream: k block i of the step's sequence --------------------------------
  //   phase 0, chunk c: W_0 k blocks KBC c .. + KBC - 1, then W_y the same (i < P0 = 2 k_pad / 32)
  //   forward layers l = 1 .. NL-2: W_l k blocks 0..7 (the skip layer: Lx)
  //   backward l = NL-2 .. 1: W_l^T k blocks 0..7
  const int nkx = k_pad / 32, P0 = 2 * nkx;
  const int nseq = P0 + 2 * (NL - 2) * UPL;
  const unsigned lane_off = (unsigned)(t0 * 64 + lane) * 16u;
  auto frag_src = [&](int i, const bf16*& img, int& kb) {
    i = i < nseq ? i : nseq - 1;  // past the end: harmless reloads keep the waits exact
    if (i < P0) {
      const int c = i / (2 * KBC), j = i % (2 * KBC);
      img = j < KBC ? a.w0_img : a.wy_img;
      kb = c * KBC + (j % KBC);
    } else if (i < P0 + (NL - 2) * UPL) {
      const int q = i - P0;
      img = a.wf[1 + q / UPL];
      kb = q % UPL;
    } else {
      const int q = i - P0 - (NL - 2) * UPL;
      img = a.wb[(NL - 2) - q / UPL];
      kb = q % UPL;
    }
  };
  // k block kb of image img (the refills take img / kb from the caller, computed once per
  // layer or chunk: an image pointer looked up per k block is a scalar load whose
  // lgkmcnt(0) wait also drained the B-operand reads in flight)
  auto frag_at = [&](const bf16* img, int kb, bf16x8 (&dst)[TN]) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      dst[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024,
                                                                                  kb * C::NT * 1024, 0));
  };
  auto frag_i = [&](int i, bf16x8 (&dst)[TN]) {
    const bf16* img;
    int kb;
    frag_src(i, img, kb);
    frag_at(img, kb, dst);
  };
  // Phase 0 loads its fragments by inline asm, and waits for them with explicit counts: the
  // compiler treats the direct-to-LDS loads in flight as a second kind of vector-memory
  // event, assumes out-of-order completion and would drain the whole queue (vmcnt(0)) before
  // every k block -- the gather's two chunks in flight with it.
  auto frag_asm_at = [&](const bf16* img, int kb, bf16x8 (&dst)[TN]) {
    const unsigned vo = lane_off + (unsigned)kb * C::NT * 1024u;
    static_assert(TN == 2, "two fragment loads per k block");
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst[0]) : "v"(vo), "s"(img) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:1024" : "=v"(dst[1]) : "v"(vo), "s"(img) : "memory");
  };
  auto frag_asm = [&](int i, bf16x8 (&dst)[TN]) {
    const bf16* img;
    int kb;
    frag_src(i, img, kb);
    frag_asm_at(img, kb, dst);
  };
  bf16x8 fr[D][TN];
  sfor<D0>([&](auto KB) { frag_asm(decltype(KB)::value, fr[decltype(KB)::value]); });

  // ---- LDS tile helpers ------------------------------------------------------------------
  int aoffs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) aoffs[q] = act_off(q, r16, g4) - q * 1024;
  auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
  // feat(j) from an opaque copy of the lane id: recomputed where it is used (two VALU ops)
  // instead of kept live across the layers -- the compiler had spilled it, and reloading a
  // spill is a vector-memory wait that drains the fragment ring at every epilogue
  auto feat_now = [&](int j) {
    int x = lane;
    asm volatile("" : "+v"(x));
    return 16 * (t0 + j) + 4 * (x >> 4);
  };
  auto put_act = [&](const float (&v)[TN][4], char* tile) {
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      u32x4 w;
      w[0] = pack_bf16x2(v[j][0], v[j][1]);
      w[1] = pack_bf16x2(v[j][2], v[j][3]);
      w[2] = pack_bf16x2(v[j + 1][0], v[j + 1][1]);
      w[3] = pack_bf16x2(v[j + 1][2], v[j + 1][3]);
      *reinterpret_cast<u32x4*>(tile + act_off((t0 + j) >> 1, r16, g4)) = w;
    }
  };
  auto get_act = [&](float (&v)[TN][4], const char* tile) {
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(tile + act_off((t0 + j) >> 1, r16, g4));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[j + q / 2][2 * (q % 2)] = __builtin_bit_cast(float, w[q] << 16);
        v[j + q / 2][2 * (q % 2) + 1] = __builtin_bit_cast(float, w[q] & 0xFFFF0000u);
      }
    }
  };
  // sums over the 16 rays (lanes of a row) of per-lane values -> the owner lane of feature
  // feat(idx / 4) + idx % 4 returns it (lanes r16 < NV)
  auto ray_sums = [&](const float (&v)[TN][4], int& fo) -> float {
    float t[NV];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) t[j * 4 + r] = v[j][r];
    const float sm = ray_sum<NV>(t, lane);
    const int idx = r16 % NV;
    fo = feat(idx >> 2) + (idx & 3);
    return sm;
  };

  // ---- fragment images for the dW GEMM out of an LDS tile (chain3's store wave's copy) ----
  // a 16-lane group reads 4 rays x 16 features with ds_read_b64_tr_b16 (lane 4 q + p: ray
  // q's features 4 p .. 4 p + 3; lane i receives feature i of the 4 rays); one store
  // instruction writes the 512-byte pieces of 16-feature tiles 2 u and 2 u + 1 of a 16-ray
  // tile (whole lines, write-through: the next launch reads them)
  const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3, trh = tg & 1;
  const int64_t img_lane = (int64_t)(ti + 16 * trh) * 16;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  // (inline asm: the compiler would order the builtin's LDS read behind every direct-to-LDS
  // load in flight -- a vmcnt(0) in each phase-0 chunk; the count is waited for below)
  auto tr_read = [&](const char* p8) -> s16x4 {
    s16x4 r;
    const unsigned la = (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p8);
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(la) : "memory");
    return r;
  };
  // units (n, u): ray tile n, tile pair u of R / 32 pairs in [u_begin, u_end); wave wc takes
  // every CW-th unit.  addr(t, n, ray, quad): LDS address of features 16 t + 4 quad .. of
  // `ray` of ray tile n.
  // reps > 1 stores the same pieces again (identical bytes): phase 0's tail chunks keep the
  // per-chunk count of memory operations that its waits assume
  auto copy_image = [&](auto NBc, auto addr, int R, bf16* img, int u_begin, int u_end, int reps = 1) {
    const int nu = u_end - u_begin;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(img, (short)0, 0x7FFFFFFF, 0x00020000);
    constexpr int NB = decltype(NBc)::value;
#pragma unroll 1
    for (int q0 = wc; q0 < RT * nu; q0 += CW * NB) {
      s16x4 lo[NB], hi[NB];
#pragma unroll
      for (int v = 0; v < NB; ++v) {
        const int q = min(q0 + v * CW, RT * nu - 1);
        const int n = q / nu, t = 2 * (u_begin + q % nu) + (tg >> 1);
        lo[v] = tr_read(addr(t, n, 8 * trh + tq, tp));
        hi[v] = tr_read(addr(t, n, 8 * trh + 4 + tq, tp));
      }
      static_assert(NB == 2 || NB == 4, "tied registers below");
      if constexpr (NB == 2)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1])::"memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]), "+v"(lo[2]), "+v"(hi[2]), "+v"(lo[3]), "+v"(hi[3])::"memory");
#pragma unroll 1
      for (int rp = 0; rp < reps; ++rp)
#pragma unroll
      for (int v = 0; v < NB; ++v) {
        const int q = q0 + v * CW;
        if (q < RT * nu) {
          const int n = q / nu, t = 2 * (u_begin + q % nu) + (tg >> 1);
          const int b0n = b0 + 16 * n;
          const int64_t off = (int64_t)(b0n >> 5) * (R / 16) * 1024 + ((b0n >> 4) & 1) * 512 + img_lane + (int64_t)t * 1024;
          const s16x4x8 o = {lo[v][0], lo[v][1], lo[v][2], lo[v][3], hi[v][0], hi[v][1], hi[v][2], hi[v][3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rd, (unsigned)off, 0, 16);
        }
      }
    }
  };
  auto act_addr = [&](int t, int n, int r, int q) -> const char* {
    return act + n * C::TILE_BYTES + act_off(t >> 1, r, q) + 8 * (t & 1);
  };
  // one float to base[idx] through a buffer resource (a scalar base and a 32-bit lane
  // offset: per-lane 64-bit addresses of the partials' stores had been spilled in the head)
  auto st_f32 = [&](float* base, int idx, float v) {
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rb, (unsigned)idx * 4u, 0, 0);
  };
  // the feature chunk X: row = ray (128 B), 16-byte chunk q of row R at q ^ ((R >> 1) & 7)
  // (16 rows at one chunk hit 16 distinct 16-byte bank slots)
  auto x_addr = [&](int t, int n, int r, int q) -> const char* {  // t: feature tile within the chunk
    const int R = 16 * n + r;
    return xs + R * C::XROW + (((2 * t + (q >> 1)) ^ ((R >> 1) & 7)) << 4) + 8 * (q & 1);
  };
  // raw rows of chunk c -> X: 16-byte pieces (8 columns) per item, two items per thread
  auto interpolate = [&](int c) {
    const char* rb = smem + ((c & 1) ? C::OFF_RAW1 : C::OFF_ACT);
#pragma unroll 1
    for (int it = 0; it < BM * 8 / C::THREADS; ++it) {
      const int q = tid + C::THREADS * it;
      const int r = q >> 3, pc = q & 7;
      const char* src = rb + (r * 24 + pc) * 16;
      const u16x8 e0 = *reinterpret_cast<const u16x8*>(src);
      const u16x8 e1 = *reinterpret_cast<const u16x8*>(src + 128);
      const u16x8 e2 = *reinterpret_cast<const u16x8*>(src + 256);
      const float w0 = rbary[r * 3], w1 = rbary[r * 3 + 1], w2 = rbary[r * 3 + 2];
      const int ok = rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2];
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = fmaf(w2, bf_val3(e2[e]), fmaf(w1, bf_val3(e1[e]), w0 * bf_val3(e0[e])));
        o[e] = bf_bits3(ok ? x : 0.f);
      }
      *reinterpret_cast<u16x8*>(xs + r * C::XROW + ((pc ^ ((r >> 1) & 7)) << 4)) = o;
    }
  };

  // ---- accumulators, ReLU masks ------------------------------------------------------------
  f32x4 acc[RT][TN], accy[RT][TN];
#pragma unroll
  for (int n = 0; n < RT; ++n)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      accy[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // W_y x of ray tiles RT/2 .. RT-1 leaves the registers after phase 0 for the LDS the gather
  // no longer needs (fp32, element (idx, thread) at (idx THREADS + tid) 16: conflict-free),
  // so layers 1 .. s hold one accumulator set and a half; the skip epilogue reads it back
  f32x4* ypark = reinterpret_cast<f32x4*>(smem + C::OFF_YPARK);
  // masks of Y_0 .. Y_{NL-3}: bit ((n % PW) NV + j 4 + r) of word n / PW ... kept as a stack
  // (the forward pushes in layer order, the backward pops in reverse: static register indices)
  unsigned mst[MST][MW];
#pragma unroll
  for (int i = 0; i < MST; ++i)
#pragma unroll
    for (int w = 0; w < MW; ++w) mst[i][w] = 0u;

  // one k block of the stream: global index i (its fragments in ring slot SLOT), B operand
  // from the feature chunk (from_x; kbl: its k block inside the chunk) or the activation
  // tile (kbl: k block of the tile); the slot is refilled with k block i + DEP
  // (ASM: phase 0 -- the slot's loads are retired by an explicit count of this wave's later
  // vector-memory operations, `first` chunk 6 else 14, and the refill goes through frag_asm;
  // else the compiler's waits)
  // (rimg / rkb: the refill's image and k block, i.e. k block i + DEP of the sequence)
  auto kblock = [&](f32x4 (&tgt)[RT][TN], auto SLOTc, const bf16* rimg, const int rkb, const bool from_x, const int kbl,
                    auto ASMc, const bool first = false) {
    constexpr int slot = decltype(SLOTc)::value;
    constexpr bool use_asm = decltype(ASMc)::value;
    if constexpr (use_asm) {
      static_assert(2 * (2 * KBC - 1) == 6 && 2 * (2 * KBC - 1) + C::XT_STORES + C::DMA == 14, "phase-0 counts");
      if (first)
        asm volatile("s_waitcnt vmcnt(6)" : "+v"(fr[slot][0]), "+v"(fr[slot][1]) :: "memory");
      else
        asm volatile("s_waitcnt vmcnt(14)" : "+v"(fr[slot][0]), "+v"(fr[slot][1]) :: "memory");
    }
    auto bread = [&](int n) -> bf16x8 {
      if (from_x)
        return *reinterpret_cast<const bf16x8*>(xs + (16 * n + r16) * C::XROW + (((kbl * 4 + g4) ^ ((r16 >> 1) & 7)) << 4));
      return *reinterpret_cast<const bf16x8*>(act + n * C::TILE_BYTES + kbl * 1024 + aoffs[kbl & 3]);
    };
    // B operands RA ray tiles ahead: a read's LDS latency (~120 cycles) under RA MFMAs
#ifndef C4_RA
#define C4_RA 4
#endif
    constexpr int RA = C4_RA;
    bf16x8 bq[RA];
#pragma unroll
    for (int n = 0; n < RA; ++n) bq[n] = bread(n);
#pragma unroll
    for (int n = 0; n < RT; ++n) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        tgt[n][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[slot][j], bq[n % RA], tgt[n][j], 0, 0, 0);
      if (n + RA < RT) bq[n % RA] = bread(n + RA);
    }
    if constexpr (use_asm)
      frag_asm_at(rimg, rkb, fr[slot]);
    else
      frag_at(rimg, rkb, fr[slot]);
    __builtin_amdgcn_sched_barrier(0);
  };
  using NOW = std::false_type;

  // ================= phase 0: both input layers over the gathered feature chunks ==========
  // This wave's vector-memory operations, in issue order: the prologue's DMA(0), DMA(1) and
  // D0 TN = 8 ring loads; per chunk c the 8 ring refills (chunk c + 1's fragments), its
  // XT_STORES = 2 X^T stores, then the DMA of chunk c + 2 -- or, in the last two chunks, the
  // X^T stores three more times -- 6 operations either way.  So a k block's fragments are
  // retired with 14 operations after them (chunk 0: 6), and chunk c's rows with
  // ops_after(c) = 14 (c = 0), 24 (c = 1), 16.
  auto ops_after = [&](int c) -> int { return c == 0 ? C::DMA + D0 * TN : c == 1 ? 2 * D0 * TN + C::XT_STORES + C::DMA : D0 * TN + C::XT_STORES + C::DMA; };
  static_assert(C::DMA == 3 * C::XT_STORES, "tail chunks repeat the X^T stores in place of a DMA");
  using ASM = std::true_type;
#pragma unroll 1
  for (int c = 0; c < nchunk; ++c) {
    c4_wait(ops_after(c));  // raw chunk c landed (every wave's share); chunk c - 1's readers of X done
    interpolate(c);
    lbar();                 // X holds chunk c; raw buffer c & 1 free
    stamp();
    const bool first = c == 0;
    // the refills: chunk c + 1's k blocks (W_0, then W_y), after the last chunk the first
    // hidden layer's k blocks 0 .. D0 - 1
    const bool lastc = c + 1 == nchunk;
    const bf16* r0img = lastc ? a.wf[1] : a.w0_img;
    const bf16* ryimg = lastc ? a.wf[1] : a.wy_img;
    const int r0kb = lastc ? 0 : (c + 1) * KBC, rykb = lastc ? KBC : (c + 1) * KBC;
    sfor<KBC>([&](auto KB) {
      kblock(acc, std::integral_constant<int, decltype(KB)::value>{}, r0img, r0kb + KB, true, KB, ASM{}, first);
    });
    sfor<KBC>([&](auto KB) {
      kblock(accy, std::integral_constant<int, KBC + decltype(KB)::value>{}, ryimg, rykb + KB, true, KB, ASM{}, first);
    });
    const bool tail = c + 2 >= nchunk;
    {  // X^T of the chunk for the dW of W_0 and W_y (feature tiles c KC / 16 ..)
      auto xa = [&](int t, int n, int r, int q) -> const char* { return x_addr(t - c * (C::KC / 16), n, r, q); };
      copy_image(std::integral_constant<int, 2>{}, xa, k_pad, a.XT, c * (C::KC / 32), (c + 1) * (C::KC / 32),
                 tail ? 4 : 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!tail) dma(c + 2);
    __builtin_amdgcn_sched_barrier(0);
    stamp();
  }
  // Drain the queue once, with a wait the compiler sees: its model still holds the direct-
  // to-LDS loads of phase 0 as pending, and the hidden-layer loop's waits (merged with that
  // state at the loop header) would otherwise stay vmcnt(0) in every layer.  (Slots 0 .. D0 -
  // 1, the first hidden layer's k blocks, are in flight from the last chunk's refills.)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  // the ring deepens to D for the hidden layers: k blocks P0 + D0 .. P0 + D - 1
  sfor<D - D0>([&](auto KB) {
    frag_i(P0 + D0 + decltype(KB)::value, fr[D0 + decltype(KB)::value]);
    __builtin_amdgcn_sched_barrier(0);
  });
  // ... the asm-loaded slots 0 .. D0 - 1 have landed (the drain above; the tie keeps their
  // first uses below it)
  static_assert(D0 == 4, "four slots tied below");
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(fr[0][0]), "+v"(fr[0][1]), "+v"(fr[1][0]), "+v"(fr[1][1]), "+v"(fr[2][0]), "+v"(fr[2][1]),
                 "+v"(fr[3][0]), "+v"(fr[3][1])
               : "n"((D - D0) * TN)
               : "memory");

  // ---- forward epilogue of layer l: bias (+ W_y x and Ly.bias at the skip layer) + ReLU ---
  // -> the activation tile (B1 before: every wave's reads of the tile are done), the masks
  auto fwd_epilogue = [&](int l) {
    const bool skip = l == s;
    unsigned bits[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) bits[w] = 0u;
    lbar();  // B1
    stamp();
    if (l == 0) {  // every wave is past phase 0's reads of X: park W_y x of the upper ray tiles
#pragma unroll
      for (int n = RT / 2; n < RT; ++n)
#pragma unroll
        for (int j = 0; j < TN; ++j) ypark[((n - RT / 2) * TN + j) * C::THREADS + tid] = accy[n][j];
    }
#pragma unroll
    for (int n = 0; n < RT; ++n) {
      unsigned wd[TN][2];  // the packed bf16 pairs, as put_act lays them out
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(vecs + l * H + feat_now(j));
        f32x4 z = acc[n][j];
        if (skip) {
          const f32x4 yv = *reinterpret_cast<const f32x4*>(vecs + (NL - 1) * H + feat_now(j));
          const f32x4 ay = n < RT / 2 ? accy[n][j] : ypark[((n - RT / 2) * TN + j) * C::THREADS + tid];
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] = ((z[r] + ay[r]) + bv[r]) + yv[r];
        } else {
          z += bv;
        }
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const unsigned w = pack_bf16x2(relu1(z[r]), relu1(z[r + 1]));
          wd[j][r / 2] = w;
          // h > 0 <=> the bf16 bits without the sign are nonzero
          bits[n / PW] |= nz1_4(w & 0x7FFFu) << ((n % PW) * NV + j * 4 + r);
          bits[n / PW] |= nz1_4(w & 0x7FFF0000u) << ((n % PW) * NV + j * 4 + r + 1);
        }
        acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        const u32x4 w = {wd[j][0], wd[j][1], wd[j + 1][0], wd[j + 1][1]};
        *reinterpret_cast<u32x4*>(act + n * C::TILE_BYTES + act_off((t0 + j) >> 1, r16, g4)) = w;
      }
    }
#pragma unroll
    for (int i = MST - 1; i > 0; --i)
#pragma unroll
      for (int w = 0; w < MW; ++w) mst[i][w] = mst[i - 1][w];
#pragma unroll
    for (int w = 0; w < MW; ++w) mst[0][w] = bits[w];
    lbar();  // B2: the next layer's input complete
    stamp();
    if (l <= NL - 3) copy_image(std::integral_constant<int, 4>{}, act_addr, H, a.YT[l], 0, H / 32);  // Y_l^T
    stamp();
  };

  fwd_epilogue(0);
#pragma unroll 1
  for (int l = 1; l <= NL - 3; ++l) {
    const bf16* nimg = a.wf[l + 1];  // the refills: the next layer's k blocks (D = UPL)
    sfor<UPL>([&](auto KB) { kblock(acc, std::integral_constant<int, decltype(KB)::value % D>{}, nimg, KB, false, KB, NOW{}); });
    stamp();
    fwd_epilogue(l);
  }

  // ================= the last hidden layer, the head, the loss, the head backward =========
  {
    const bf16* nimg = a.wb[NL - 2];  // the refills: the first backward layer
    sfor<UPL>([&](auto KB) { kblock(acc, std::integral_constant<int, decltype(KB)::value % D>{}, nimg, KB, false, KB, NOW{}); });
  }
  stamp();
  {
    const int l = NL - 2;
    const bool skip = l == s;
    lbar();  // B1: the tile's reads are done (it takes this layer's activations next)
    // ReLU activations of the last hidden layer (bf16) into the tile, the head's partial
    // dot products over this wave's features into zps
#pragma unroll
    for (int n = 0; n < RT; ++n) {
      float hq[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(vecs + l * H + feat_now(j));
        f32x4 z = acc[n][j];
        if (skip) {  // (s == NL - 2: not taken, chain4_supported requires s < NL - 2)
          const f32x4 yv = *reinterpret_cast<const f32x4*>(vecs + (NL - 1) * H + feat_now(j));
          const f32x4 ay = n < RT / 2 ? accy[n][j] : ypark[((n - RT / 2) * TN + j) * C::THREADS + tid];
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] = ((z[r] + ay[r]) + bv[r]) + yv[r];
        } else {
          z += bv;
        }
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const unsigned w = pack_bf16x2(relu1(z[r]), relu1(z[r + 1]));
          hq[j][r] = __builtin_bit_cast(float, w << 16);
          hq[j][r + 1] = __builtin_bit_cast(float, w & 0xFFFF0000u);
        }
      }
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        float z = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(w7s + o * H + feat_now(j));
#pragma unroll
          for (int r = 0; r < 4; ++r) z = fmaf(hq[j][r], w[r], z);
        }
        z = col_sum4(z);
        if (g4 == 0) zps[(wc * BM + 16 * n + r16) * 3 + o] = z;
      }
      put_act(hq, act + n * C::TILE_BYTES);
    }
    lbar();  // Bh: every wave's head partial sums complete
    stamp();
    // sigmoid, loss and dL/dz (model.py:89-94, config.py:113-122, trainer.py:76): every wave
    // computes all BM x 3 of them into its own copy of dz (same-wave LDS order only)
    {
      float* dzw = dzs + wc * BM * 3;
      float lsum = 0.f, ssum = 0.f;
#pragma unroll 1
      for (int e0 = 0; e0 < BM * 3; e0 += 64) {
        const int e = e0 + lane;
        const int b = b0 + e / 3, o = e % 3;
        float z = w7s[3 * H + o];
#pragma unroll
        for (int w = 0; w < CW; ++w) z += zps[w * BM * 3 + e];
        const float pv = 1.f / (1.f + expf(-z));
        float dz = 0.f;
        if (b < a.batch) {
          const float d = pv - tgs[e];
          float lv, g;
          if constexpr (LOSS == INF_LOSS_L2) {
            lv = d * d;
            g = 2.f * d;
          } else if constexpr (LOSS == INF_LOSS_L1) {
            lv = fabsf(d);
            g = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
          } else {
            const float qq = d * d / C4_CAUCHY_C2;
            lv = C4_CAUCHY_C2 * logf(1.f + qq);
            g = 2.f * d / (1.f + qq);
          }
          dz = (g * a.inv_count) * (1.f - pv) * pv;
          lsum += lv;
          ssum += d * d;
        }
        dzw[e] = dz;
        if (wc == 0) preds[e] = pv;
      }
      if (wc == 0) {
        lsum = col_sum4(row_sum16(lsum));
        ssum = col_sum4(row_sum16(ssum));
        if (lane == 0) {
          lss[0] = lsum;
          lss[1] = ssum;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's dz writes
    }
    // head backward: dZ_{L-2} = (dz W7) * (h > 0) into the tile (each lane its own slots),
    // its ray sums (the bias partial), the output layer's weight-gradient partials
    float cst[TN][4], hst[3][TN][4], dbs[3];
    // (one ray tile at a time: unrolled, the compiler hoisted every tile's activation reads
    // and spilled them)
#pragma unroll 1
    for (int n = 0; n < RT; ++n) {
      float dzr[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) dzr[o] = dzs[wc * BM * 3 + (16 * n + r16) * 3 + o];
#pragma unroll
      for (int o = 0; o < 3; ++o) dbs[o] = n == 0 ? dzr[o] : dbs[o] + dzr[o];
      float hq[TN][4];
      get_act(hq, act + n * C::TILE_BYTES);
      float gv[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(w7s + 0 * H + feat_now(j));
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(w7s + 1 * H + feat_now(j));
        const f32x4 w2 = *reinterpret_cast<const f32x4*>(w7s + 2 * H + feat_now(j));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float g = fmaf(dzr[2], w2[r], fmaf(dzr[1], w1[r], dzr[0] * w0[r]));
          gv[j][r] = hq[j][r] > 0.f ? g : 0.f;
        }
      }
      put_act(gv, act + n * C::TILE_BYTES);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          cst[j][r] = n == 0 ? gv[j][r] : cst[j][r] + gv[j][r];
#pragma unroll
          for (int o = 0; o < 3; ++o) hst[o][j][r] = n == 0 ? dzr[o] * hq[j][r] : fmaf(dzr[o], hq[j][r], hst[o][j][r]);
        }
    }
    if (wc == 0) {
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        const float db = row_sum16(dbs[o]);
        if (lane == 0) st_f32(a.hb_part, (int)part0 * 3 + o, db);
      }
    }
    {
      int fo;
      const float sm = ray_sums(cst, fo);
      if (r16 < NV) st_f32(a.colsum[NL - 2], (int)part0 * H + fo, sm);
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        const float sh = ray_sums(hst[o], fo);
        if (r16 < NV) st_f32(a.hw_part, ((int)part0 * 3 + o) * H + fo, sh);
      }
    }
    lbar();  // B2: dZ_{L-2} complete
    stamp();
    if (tid < 2 && a.loss_part != nullptr) a.loss_part[2 * part0 + tid] = lss[tid];
    if (a.pred != nullptr)
      for (int e = tid; e < BM * 3; e += C::THREADS)
        if (b0 + e / 3 < a.batch) a.pred[(int64_t)b0 * 3 + e] = preds[e];
    copy_image(std::integral_constant<int, 4>{}, act_addr, H, a.dZT[NL - 2], 0, H / 32);
    stamp();
  }
  // (the accumulators restart here, not in the head: their registers serve the head meanwhile)
#pragma unroll
  for (int n = 0; n < RT; ++n)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ================= backward: dX of layers NL-2 .. 1 ======================================
#pragma unroll 1
  for (int l = NL - 2; l >= 1; --l) {
    // the refills: the next backward layer (past the last: harmless reloads of its last k block)
    const bf16* nimg = a.wb[l > 1 ? l - 1 : 1];
    const int nkb0 = l > 1 ? 0 : UPL - 1, nstep = l > 1 ? 1 : 0;
    sfor<UPL>([&](auto KB) {
      kblock(acc, std::integral_constant<int, decltype(KB)::value % D>{}, nimg, nkb0 + nstep * KB, false, KB, NOW{});
    });
    stamp();
    // dZ_{l-1} = acc * (Y_{l-1} > 0): the mask stack's top
    unsigned bits[MW];
#pragma unroll
    for (int w = 0; w < MW; ++w) bits[w] = mst[0][w];
#pragma unroll
    for (int i = 0; i + 1 < MST; ++i)
#pragma unroll
      for (int w = 0; w < MW; ++w) mst[i][w] = mst[i + 1][w];
    float cst[TN][4];
    lbar();  // B1
    stamp();
#pragma unroll
    for (int n = 0; n < RT; ++n) {
      float v[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[j][r] = ((bits[n / PW] >> ((n % PW) * NV + j * 4 + r)) & 1u) ? acc[n][j][r] : 0.f;
          cst[j][r] = n == 0 ? v[j][r] : cst[j][r] + v[j][r];
        }
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      put_act(v, act + n * C::TILE_BYTES);
    }
    {
      int fo;
      const float sm = ray_sums(cst, fo);
      if (r16 < NV) st_f32(a.colsum[l - 1], (int)part0 * H + fo, sm);
    }
    lbar();  // B2
    stamp();
    copy_image(std::integral_constant<int, 4>{}, act_addr, H, a.dZT[l - 1], 0, H / 32);
    stamp();
  }
  stamp();  // end
}

template <int NL, int LOSS>
int launch_typed(const Chain3Args& a, hipStream_t stream) {
  using C = L4<NL>;
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain4_kernel<NL, LOSS>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
    attr = true;
  }
  chain4_kernel<NL, LOSS><<<dim3((unsigned)(a.rows / C::BM)), dim3(C::THREADS), C::LDS, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_chain4(const Chain3Args& a_in, hipStream_t stream) {
  Chain3Args a = a_in;
  a.table_big = a.num_vertices * (int64_t)a.k_pad * 2 >= ((int64_t)1 << 32);
  INF_CHECK_ARG(chain4_supported(a.H, a.L, a.k_pad, a.rows), "chain4: unsupported shape");
  INF_CHECK_ARG(a.s >= 1 && a.s <= a.L - 3, "chain4: skip layer inside the hidden stack (its W_y x park)");
  INF_CHECK_ARG(a.encoding == INF_ENC_NONE && a.xpre == nullptr && !a.x3 && a.zin == nullptr,
                "chain4: eigenfunction-table batches only");
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr && a.rgb != nullptr && a.XT != nullptr,
                "chain4: inputs");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "chain4: vertex id dtype");
  INF_CHECK_ARG(a.num_vertices >= 1, "chain4: empty table");
  INF_CHECK_ARG(a.w0_img != nullptr && a.wy_img != nullptr, "chain4: input-layer images");
  for (int l = 1; l <= a.L - 2; ++l) INF_CHECK_ARG(a.wf[l] != nullptr && a.wb[l] != nullptr, "chain4: hidden images");
  for (int l = 0; l <= a.L - 2; ++l)
    INF_CHECK_ARG(a.colsum[l] != nullptr && a.dZT[l] != nullptr && (l > a.L - 3 || a.YT[l] != nullptr), "chain4: outputs");
  if (a.loss == INF_LOSS_L2) return launch_typed<8, INF_LOSS_L2>(a, stream);
  if (a.loss == INF_LOSS_L1) return launch_typed<8, INF_LOSS_L1>(a, stream);
  return launch_typed<8, INF_LOSS_CAUCHY>(a, stream);
}

}  // namespace inf
