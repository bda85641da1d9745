// Persistent forward-only chain over a projected table: the render slice
// (renderer.py:112-146) when the frame's hits are interpolated from the vertices' first-
// layer projections (inf_project_table: rows (W_0 E[v], W_y E[v]), bf16 [V][2H]).
//
// Layer 0 and the skip layer's Ly are linear in the features, so a hit's pre-activations
// are sum_i b_i (W E[v_i]) (mesh.py:313-324 then model.py:43-47 / layers.py:60-62,
// reassociated): per hit three 2H-wide rows instead of three k-wide rows, and only the
// hidden layers and the head left to stream.  Per 64-ray tile that is ~18 us of weight
// streaming (rchain.hip's loop: 8 compute waves, 4 ray tiles, 1 fragment -> 4 MFMAs) and
// a 192 KB row interpolation whose HBM latency a one-tile workgroup cannot hide (13 us
// exposed per tile), nor can the compute waves issue it beside their weight stream: the
// vector-memory counter retires in order, so the first fragment load behind a row load
// waits for it (measured: +2 us per hidden layer).  So each workgroup owns a contiguous
// range of tiles and runs 4 LOADER waves beside the 8 compute waves: while the hidden
// layers of tile i stream, the loader waves fetch tile i+1's records and rows and fold
// them into the LDS staging tile Z.  The loader waves take part in every barrier of
// the compute waves (a fixed per-tile barrier schedule, below); only the first tile of
// a workgroup waits for its rows.
//
//   Z [64 rays][2H] bf16 (sum_i b_i P[v_i] | sum_i b_i Q[v_i]), fp32 FMAs in the
//   gather's order, one bf16 rounding.  Compute waves read their accumulator elements of
//   z0 out of Z for layer 0's epilogue and those of zy in the skip layer's epilogue, so
//   the next tile's W_0 half may land once layer 0 has started and its W_y half once the
//   skip layer's epilogue is done.
//
// Barriers of one tile, compute side: [read z0] B_a [epilogue 0] B_0 [layer 1] B_1 ...
// [layer L-2 + head partials] B_{L-2} (+ extra barriers when the loader schedule needs
// more intervals), then the sigmoid + placement.  Loader side, in the intervals ending
// at those barriers: I0 record loads of tile + 1, I1 record stores, then the rows in
// four groups -- loads in one interval, interpolation into Z in the next: W_0 half
// I2 -> I3, I3 -> I4, W_y half I4 -> I_jy, I_jy -> I_jy+1 (jy >= s + 2: after B_s).
#include <cstdlib>

#include "c3common.hpp"
#include "rchain.hpp"

namespace inf {
namespace {

using namespace c3;

#ifndef RP_DEPTH
#define RP_DEPTH 4
#endif
#ifndef RP_BQ
#define RP_BQ 2
#endif
// diagnostics (tools/rchain_timing.py; results wrong): RP_DIAG bit 0 = no fragment refills,
// bit 1 = no LDS B-operand reads, bit 2 = no epilogue work
#ifndef RP_DIAG
#define RP_DIAG 0
#endif
// diagnostics (tools/rchain_timing.py): 1 = loader waves only take part in the barriers,
// 2 = they load the rows but neither interpolate nor store, 3 = interpolate and store
// constants without loading
#ifndef RP_LOADER_IDLE
#define RP_LOADER_IDLE 0
#endif

template <int H, int CW_>
struct LP {
  static constexpr int CW = CW_, LW = 4, RT = 4, BM = 64;  // compute waves, loader waves
  static constexpr int THREADS = (CW + LW) * 64, LT = LW * 64;
  static constexpr int TN = H / (16 * CW);
  static constexpr int UPL = H / 32, NT = H / 16;
  static constexpr int ACT_T = 16 * H * 2, ACT_BYTES = RT * ACT_T;
  static constexpr int ZROW = 4 * H;             // bytes of one ray's (z0, zy) bf16 row
  static constexpr int CPR = ZROW / 16;          // 16-byte chunks per row
  static constexpr int HC = CPR / 2;             // chunks per half row
  static constexpr int NH = BM * HC / LT;        // row chunks per loader thread per half
  static constexpr int OFF_ACT = 0;                         // [2][RT] activation tiles
  static constexpr int OFF_Z = 2 * ACT_BYTES;               // [BM][2H] staging tile
  static constexpr int OFF_RAY = OFF_Z + BM * ZROW;         // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RB = OFF_RAY + BM * 16 + BM * 12;  // [BM][3] barycentrics
  static constexpr int OFF_ZP = OFF_RB + BM * 12;           // [CW][BM][3] head partials
  static constexpr int OFF_W7 = OFF_ZP + CW * BM * 12;      // [3][H], b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;   // biases [L-1][H], Ly.bias [H]
  static int lds_bytes(int L) { return OFF_VEC + L * H * 4; }
  static_assert((BM * HC) % (2 * LT) == 0 && LT % HC == 0 && 3 * BM <= LT, "row items, records");
  static_assert(OFF_RAY % 16 == 0 && OFF_W7 % 16 == 0 && OFF_VEC % 16 == 0, "LDS alignment");
};

template <int H, int CW_>
__global__ __launch_bounds__((LP<H, CW_>::THREADS)) void rproj_kernel(const RchainArgs a) {
  using C = LP<H, CW_>;
  constexpr int RT = C::RT, BM = C::BM, TN = C::TN, UPL = C::UPL, CW = C::CW, NH = C::NH, HC = C::HC,
                THREADS = C::THREADS, LT = C::LT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L, nh = a.nblk;  // hidden layers 1 .. L - 2, one stream block each
  char* act = smem + C::OFF_ACT;
  char* zs = smem + C::OFF_Z;
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RB);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  // a contiguous range of tiles per workgroup; workgroup i runs on XCD i % 8, so
  // neighbouring ranges (hits in pixel order share vertices) go to one XCD's L2
  const int ntile = (int)ceil_div(a.batch, BM);
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xq = nb / 8, xr = nb % 8, xcd = bid % 8;
  const int wg = xcd * xq + min(xcd, xr) + bid / 8;
  const int tb = (int)((int64_t)ntile * wg / nb), te = (int)((int64_t)ntile * (wg + 1) / nb);
  if (tb >= te) return;
  unsigned long long* stl = nullptr;
  if (a.stamps != nullptr && tid == 0 && (bid == 0 || bid == nb / 2)) stl = a.stamps + (bid == 0 ? 0 : RC_STAMPS);
  auto stamp = [&](int i) {
    if (stl != nullptr && i < RC_STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      stl[i] = wall_clock64();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);

  for (int i = tid; i < (L - 1) * H; i += THREADS) vecs[i] = a.bias[i / H][i % H];
  for (int i = tid; i < H; i += THREADS) vecs[(L - 1) * H + i] = a.bias_y[i];
  for (int i = tid; i < 3 * H + 3; i += THREADS) w7s[i] = i < 3 * H ? a.W7[i] : a.b7[i - 3 * H];

  // ---- weight fragments of the hidden layers (rchain.hip's ring) --------------------------
  const int t0 = wc * TN;
  constexpr int D = RP_DEPTH < UPL ? RP_DEPTH : UPL;
  bf16x8 fr[D][TN];
  const unsigned lane_off = (unsigned)(t0 * 64 + lane) * 16u;
  auto rsrc_of = [&](const bf16* img) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
  };
  auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j) -> bf16x8 {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024, kb * C::NT * 1024, 0);
    return __builtin_bit_cast(bf16x8, v);
  };
  if (wc < CW) {
    const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(a.blk[0].img);
#pragma unroll
    for (int kb = 0; kb < D; ++kb) {
#pragma unroll
      for (int j = 0; j < TN; ++j) fr[kb][j] = frag(rs0, kb, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---- ray records of a tile: thread (ray, vertex) for tid < 3 BM ------------------------
  struct Rec {
    int v, ok;
    float w;
  };
  auto rec_load = [&](int tile, int x) -> Rec {
    Rec r{0, 0, 0.f};
    if (x < BM * 3) {
      const int b = tile * BM + x / 3, i = x % 3;
      const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, a.idx_offset, b, a.num_rays, a.num_src) : -1;
      if (rr >= 0) {
        const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
        r.ok = (uint64_t)e < (uint64_t)a.num_vertices;  // out-of-range ids read as zero rows (gather.hip)
        r.v = r.ok ? (int)e : 0;
        r.w = a.bary[3 * rr + i];
      }
    }
    return r;
  };
  auto rec_store = [&](const Rec& r, int x) {
    if (x < BM * 3) {
      const int rl = x / 3, i = x % 3;
      rvid[rl * 4 + i] = r.v;
      rbary[rl * 3 + i] = r.w;
      rvid[BM * 4 + x] = r.ok;
    }
  };

  // ---- 16-byte chunk c (< HC) of half h (0: W_0 E, 1: W_y E) of ray r's row: the three
  // vertex rows' chunks (32 consecutive threads read one vertex's 512-byte half row;
  // non-temporal loads measured no faster)
  auto rows_load = [&](int h, int r, int c, u16x8 (&ev)[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      ev[i] = __builtin_bit_cast(
          u16x8, *reinterpret_cast<const u32x4*>(a.table + (int64_t)rvid[r * 4 + i] * (2 * H) + (h * HC + c) * 8));
  };
  auto rows_store = [&](int h, int r, int c, const u16x8 (&ev)[3]) {
    const int ok = rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2];
    const float w0 = rbary[r * 3], w1 = rbary[r * 3 + 1], w2 = rbary[r * 3 + 2];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = fmaf(w2, bf_val3(ev[2][e]), fmaf(w1, bf_val3(ev[1][e]), w0 * bf_val3(ev[0][e])));
      o[e] = bf_bits3(ok ? x : 0.f);
    }
    *reinterpret_cast<u16x8*>(zs + r * C::ZROW + (((h * HC + c) ^ (r & 15)) << 4)) = o;
  };

  // ---- prologue: the first tile's records and rows, every wave -------------------------
  rec_store(rec_load(tb, tid), tid);
  lbar();  // records, vectors in LDS
  stamp(1);
#pragma unroll 1
  for (int q0 = tid; q0 < 2 * BM * HC; q0 += 4 * THREADS) {
    u16x8 ev[4][3];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int q = q0 + n * THREADS;
      if (q < 2 * BM * HC) rows_load(q / (BM * HC), q % (BM * HC) / HC, q % HC, ev[n]);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int q = q0 + n * THREADS;
      if (q < 2 * BM * HC) rows_store(q / (BM * HC), q % (BM * HC) / HC, q % HC, ev[n]);
    }
  }
  lbar();  // Z holds the first tile
  stamp(2);

  // barriers per tile (see the top): B_a, B_0 .. B_{L-2}, plus extras so that the loader's
  // last interval (jy + 1; jy after B_s = barrier 1 + s) ends before the last one
  const int nbar_c = 2 + nh;
  const int jy = max(5, a.s + 2);
  const int nbar = max(nbar_c, jy + 2);

  if (wc >= CW) {
    // ---- loader waves: tile + 1's records, then its rows in four groups (W_0 half g0,
    // g1, W_y half g0, g1), each loaded in one interval and folded into Z in the next ----
    // loader thread x: chunk x % HC of rays x / HC + RPI m (per-item LDS addresses are
    // the thread's base plus immediates)
    constexpr int G = NH / 2, RPI = LT / HC;
    const int x = tid - CW * 64;
    const int lc = x % HC, lr = x / HC;
    auto load_group = [&](int h, int g, u16x8 (&ev)[G][3]) {
      if constexpr (RP_LOADER_IDLE == 3) {  // diagnostics: interpolation + stores of constants, no loads
#pragma unroll
        for (int m = 0; m < G; ++m)
#pragma unroll
          for (int i = 0; i < 3; ++i) ev[m][i] = u16x8{(unsigned short)(x + m), 1, 2, 3, 4, 5, 6, (unsigned short)i};
        return;
      }
#pragma unroll
      for (int m = 0; m < G; ++m) rows_load(h, lr + RPI * (g * G + m), lc, ev[m]);
    };
    auto store_group = [&](int h, int g, u16x8 (&ev)[G][3]) {
      // pin the raw loaded registers here: otherwise the bf16 -> fp32 unpacking is hoisted
      // next to the loads and the group's live registers double across the barrier
#pragma unroll
      for (int m = 0; m < G; ++m)
#pragma unroll
        for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(ev[m][i]));
      if constexpr (RP_LOADER_IDLE == 2) {  // diagnostics: the loads, no interpolation / stores
        if (ev[0][0][0] == 0x1234 && ev[G - 1][2][7] == 0x4321) zs[x] = 1;
        return;
      }
#pragma unroll
      for (int m = 0; m < G; ++m) rows_store(h, lr + RPI * (g * G + m), lc, ev[m]);
    };
#pragma unroll 1
    for (int tile = tb; tile < te; ++tile) {
      const bool has_next = tile + 1 < te;
      Rec rec{0, 0, 0.f};
      u16x8 ev[G][3];
#pragma unroll 1
      for (int j = 0; j < nbar; ++j) {
        if (has_next && RP_LOADER_IDLE != 1) {
          if (j == 0) rec = rec_load(tile + 1, x);
          if (j == 1) rec_store(rec, x);
          // stores first: the group registers are reloaded in the same interval
          if (j == 3) store_group(0, 0, ev);
          if (j == 4) store_group(0, 1, ev);
          if (j == jy) store_group(1, 0, ev);
          if (j == jy + 1) store_group(1, 1, ev);
          if (j == 2) load_group(0, 0, ev);
          if (j == 3) load_group(0, 1, ev);
          if (j == 4) load_group(1, 0, ev);
          if (j == jy) load_group(1, 1, ev);
        }
        lbar();
      }
    }
    return;
  }

  int aoffs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) aoffs[q] = act_off(q, r16, g4) - q * 1024;
  auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
  f32x4 acc[RT][TN];

  // epilogue of layer l: bias (+ W_y x and Ly.bias at the skip layer) + ReLU into the next
  // activation tile, or the head partials at l = L - 2 (rchain.hip's)
  // layer l's bias (+ Ly.bias and the tile's W_y x at the skip layer) as the start value of
  // the accumulators, so the epilogue is ReLU + bf16 packing only
  auto init_acc = [&](int l) {
    const bool skip = l == a.s;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 bb = *reinterpret_cast<const f32x4*>(vecs + l * H + feat(j));
      if (skip) bb += *reinterpret_cast<const f32x4*>(vecs + (L - 1) * H + feat(j));
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        acc[t][j] = bb;
        if (skip) {
          const u16x4 zy = *reinterpret_cast<const u16x4*>(zs + tile_off(C::ZROW, t * 16 + r16, H + feat(j)));
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][j][r] += bf_val3(zy[r]);
        }
      }
    }
  };

  // epilogue of layer l < L - 2: ReLU -> bf16 -> the next layer's activation tile
  auto epilogue_act = [&](int l) {
    char* act_out = act + ((l + 1) & 1) * C::ACT_BYTES;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      char* dst = act_out + t * C::ACT_T;
      if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int j = 0; j < TN; j += 2) {
          u32x4 w;
          w[0] = pack_bf16x2(relu1(acc[t][j][0]), relu1(acc[t][j][1]));
          w[1] = pack_bf16x2(relu1(acc[t][j][2]), relu1(acc[t][j][3]));
          w[2] = pack_bf16x2(relu1(acc[t][j + 1][0]), relu1(acc[t][j + 1][1]));
          w[3] = pack_bf16x2(relu1(acc[t][j + 1][2]), relu1(acc[t][j + 1][3]));
          *reinterpret_cast<u32x4*>(dst + act_off((t0 + j) >> 1, r16, g4)) = w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          u32x2 w;
          w[0] = pack_bf16x2(relu1(acc[t][j][0]), relu1(acc[t][j][1]));
          w[1] = pack_bf16x2(relu1(acc[t][j][2]), relu1(acc[t][j][3]));
          const int tt = t0 + j;
          *reinterpret_cast<u32x2*>(dst + act_off(tt >> 1, r16, g4) + 8 * (tt & 1)) = w;
        }
      }
    }
    lbar();  // the next layer's tile complete; after the skip layer, Z's W_y half is free
  };

  // epilogue of layer L - 2: ReLU, bf16 rounding and the head's partial dot products
  // (model.py:89-94) over this lane's features, summed over the row groups
  auto epilogue_head = [&]() {
    float zp[RT][3];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float hq[TN][4];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const unsigned w = pack_bf16x2(relu1(acc[t][j][r]), relu1(acc[t][j][r + 1]));
          hq[j][r] = __builtin_bit_cast(float, w << 16);
          hq[j][r + 1] = __builtin_bit_cast(float, w & 0xFFFF0000u);
        }
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        float z = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(w7s + o * H + feat(j));
#pragma unroll
          for (int r = 0; r < 4; ++r) z = fmaf(hq[j][r], w[r], z);
        }
        zp[t][o] = col_sum4(z);
      }
    }
    if (g4 == 0)
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int o = 0; o < 3; ++o) zps[(wc * BM + t * 16 + r16) * 3 + o] = zp[t][o];
    lbar();  // the head partials complete (and Z's W_y half free when s = L - 2)
  };
  auto epilogue = [&](int l) {
    if constexpr ((RP_DIAG & 4) != 0) {  // diagnostics (4): a minimal epilogue (keeps the MFMAs live)
      float sm = 0.f;
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j) sm += acc[t][j][0] + acc[t][j][1] + acc[t][j][2] + acc[t][j][3];
      if (sm == 1234.5f) zps[tid] = sm;
      lbar();
      return;
    }
    if (l == L - 2) epilogue_head();
    else epilogue_act(l);
  };

  // one hidden layer: UPL k-blocks of the activation tile (rchain.hip's run_block)
  auto run_block = [&](int hb) {
    const C3Block& B = a.blk[hb];
    const C3Block& Bn = a.blk[hb + 1 < nh ? hb + 1 : 0];
    const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
    const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
    const char* act_in = act + (B.phase & 1) * C::ACT_BYTES;
    auto read_b = [&](int kb, bf16x8 (&bv)[RT]) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        if constexpr ((RP_DIAG & 2) != 0) {  // diagnostics: no LDS operand reads
          bv[t] = __builtin_bit_cast(bf16x8, u32x4{(unsigned)kb, (unsigned)t, 0u, 0u});
        } else {
          bv[t] = *reinterpret_cast<const bf16x8*>(act_in + t * C::ACT_T + kb * 1024 + aoffs[kb & 3]);
        }
      }
    };
    constexpr int NB = RP_BQ;  // B-operand buffers: 2 = next k-block's read ahead of the MFMAs
    bf16x8 bq[NB][RT];
    read_b(0, bq[0]);
#pragma unroll
    for (int kb = 0; kb < UPL; ++kb) {
      if (NB == 2 && kb + 1 < UPL) read_b(kb + 1, bq[(kb + 1) % NB]);
      if (NB == 1 && kb > 0) read_b(kb, bq[0]);
      // issue them ahead of this k-block's MFMAs (the scheduler otherwise sinks the reads to
      // just before their first use, one MFMA ahead, exposing the LDS latency every k-block)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < RT; ++t)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bq[kb % NB][t], acc[t][j], 0, 0, 0);
      if constexpr ((RP_DIAG & 1) == 0) {  // diagnostics (1): no fragment refills
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fr[kb % D][j] = kb + D < UPL ? frag(crs, kb + D, j) : frag(nrs, kb + D - UPL, j);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

#pragma unroll 1
  for (int tile = tb; tile < te; ++tile) {
    const int sbase = 3 + (tile - tb) * (nh + 2);
    if (tile - tb < 2) stamp(sbase);
    // this tile's layer-0 pre-activations out of Z (tile_off's swizzle), then Z's W_0
    // half is free (the W_y half is read by the skip layer's epilogue)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(vecs + feat(j));
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const u16x4 p = *reinterpret_cast<const u16x4*>(zs + tile_off(C::ZROW, t * 16 + r16, feat(j)));
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][j][r] = bf_val3(p[r]) + b0[r];
      }
    }
    lbar();  // every wave holds its pre-activations
    epilogue(0);

#pragma unroll 1
    for (int hb = 0; hb < nh; ++hb) {
      if (tile - tb < 2) stamp(sbase + 1 + hb);
      init_acc(hb + 1);
      run_block(hb);
      epilogue(hb + 1);
    }
#pragma unroll 1
    for (int j = nbar_c; j < nbar; ++j) lbar();  // the loader's remaining intervals
    if (tile - tb < 2) stamp(sbase + nh + 1);

    // ---- sigmoid head and placement (renderer.py:132-141) ---------------------------------
    if (tid < BM * 3) {
      const int ray = tid / 3, o = tid % 3;
      const int b = tile * BM + ray;
      if (b < a.batch) {
        float z = w7s[3 * H + o];
#pragma unroll
        for (int w = 0; w < CW; ++w) z += zps[(w * BM + ray) * 3 + o];
        const float pv = 1.f / (1.f + expf(-z));
        if (a.pred != nullptr) a.pred[(int64_t)b * 3 + o] = pv;
        if (a.img != nullptr) {
          int64_t pix = a.hit[b];
          if (a.pixel_map != nullptr) pix = a.pixel_map[pix];
          a.img[pix * 3 + o] = pv;
        }
      }
    }
  }
}

template <int H, int CW_>
int launch_typed(const RchainArgs& a, hipStream_t stream) {
  using C = LP<H, CW_>;
  const int lds = C::lds_bytes(a.L);
  INF_CHECK_ARG(lds <= 160 * 1024, "rproj: LDS budget exceeded");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)rproj_kernel<H, CW_>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    INF_HIP_TRY(hipGetDevice(&dev));
    INF_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int64_t ntile = ceil_div(a.batch, C::BM);
  const int grid = (int)std::min<int64_t>(ntile, ncu);
  rproj_kernel<H, CW_><<<dim3((unsigned)grid), dim3(C::THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_rproj(const RchainArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(a.projected && (a.H == 128 || a.H == 256) && a.L >= 3 && a.nblk == a.L - 2 && a.nchunk == 0,
                "rproj: unsupported shape");
  INF_CHECK_ARG(a.batch >= 1, "rproj: empty batch");
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr, "rproj: inputs");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "rproj: vertex id dtype");
  INF_CHECK_ARG(a.pred != nullptr || (a.img != nullptr && a.hit != nullptr), "rproj: no output");
  for (int i = 0; i < a.nblk; ++i)
    INF_CHECK_ARG(a.blk[i].img != nullptr && a.blk[i].phase == i + 1 && a.blk[i].kb0 == 0, "rproj: weight stream");
  if (rprojw_supported(a)) return launch_rprojw(a, stream);
  // compute waves: 8 (32 output features each; default) or INF_RPROJ_WAVES=4 (64 each: half
  // the LDS operand reads, one compute wave per SIMD)
  static const int waves = [] {
    const char* e = std::getenv("INF_RPROJ_WAVES");
    return e != nullptr && std::atoi(e) == 4 ? 4 : 8;
  }();
  if (a.H == 256) return waves == 4 ? launch_typed<256, 4>(a, stream) : launch_typed<256, 8>(a, stream);
  return waves == 4 ? launch_typed<128, 4>(a, stream) : launch_typed<128, 8>(a, stream);
}

}  // namespace inf
