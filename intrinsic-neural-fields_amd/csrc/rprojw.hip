// Persistent forward-only chain over a projected table on 128-ray tiles: the render slice
// (renderer.py:112-146) of the 8-layer H = 256 field (configs B-E: skip 4), rproj.hip's
// arithmetic up to the head, with twice its rays per weight pass.
//
// rproj.hip streams the hidden layers' 768 KB of weight fragments once per 64-ray tile:
// per layer 128 KB against 64 rays' MFMAs, about as long as the per-CU L2 -> CU stream
// (≈1.1 µs at 120 GB/s) and the MFMAs (≈1.3 µs measured) each, which the tile's waits do
// not fully overlap (2.5 µs per layer).  Here a tile is 128 rays (8 MFMA ray tiles):
// every weight fragment feeds 8 MFMAs per wave, the stream per ray halves and the MFMAs
// set a layer's time.  To fit 160 KB of LDS:
//   * one activation buffer: a layer's epilogue writes it in place, between B1 (every
//     wave's MFMAs have read it) and B2 (the next layer's input is complete);
//   * one half of the staging tile Z (128 rays x 256 bf16): the loader waves fold tile
//     i's W_y half (zy, read by the skip layer's accumulator start) into Z once layer 0
//     has taken z0 out of it, and tile i + 1's W_0 half (z0) once the skip layer has
//     taken zy.
// The head runs on MFMAs too: the last hidden layer's epilogue writes h = bf16(ReLU(.))
// into the activation tile like any other, and wave w multiplies ray tile w by W7 split
// into bf16 hi + lo fragments (16 MFMAs; W7 = hi + lo to 2^-17 of |W7|, fp32 sums): the
// 3 x 256 dot products per ray of rproj.hip's VALU head (2.4 µs per tile here) cost
// ≈0.3 µs.  The sums run in another order than rproj.hip's (RGB within 1e-5 of it).
//
// Barriers of one tile (NBAR = 2 + 2 (L - 2) = 14), compute side: [z0 + bias 0 -> ReLU ->
// act] 0, per hidden layer l = 1 .. 6: [accumulator start (bias; + Ly.bias + zy at
// l = s), MFMAs] 2l - 1 [ReLU -> act] 2l, then [head MFMAs, sigmoid, placement] 13.
// Interval j ends at barrier j; the odd ones (1 .. 11) are the MFMA phases.  Loader side,
// in groups of 12 row loads per thread (two register sets, A and B), every fold into Z in
// an MFMA phase so that the epilogue intervals stay short:
//   1: fold zy(i) g0; load zy(i) g2 -> A
//   3: fold zy(i) g1; load zy(i) g3 -> B
//   5: fold zy(i) g2, g3 (zy complete before layer s's start: 2s - 1); load z0(i + 1) g0 -> A, g1 -> B
//   7: load records(i + 2), pixels(i + 1)
//   9: fold z0(i + 1) g0, g1 (Z free after barrier 2s - 1); load g2 -> A, g3 -> B
//  11: fold z0(i + 1) g2, g3; load zy(i + 1) g0 -> A, g1 -> B
//  12: store records(i + 2) (set (tile - first) & 1); 0 (of i + 1): store pixels(i + 1)
// (zy of the first tile: loaded ahead of the loop.)  The schedule is unrolled, so the
// compiler's vmcnt waits count each group's loads exactly.
#include <cstdlib>

#include "c3common.hpp"
#include "rchain.hpp"

namespace inf {
namespace {

using namespace c3;

#ifndef RW_DEPTH
#define RW_DEPTH 4
#endif
#ifndef RW_RA
#define RW_RA 2  // (4: 4 spills, 2.05 vs 1.96 ms per 2M hits; depth 5 / 6 no better)
#endif
// loader schedule: 2 = the default (below), 0 = the zy folds in intervals 1 and 3 (8 items
// each) and the records in 11, 1 = as 0 with the group loads in the epilogue intervals.
// The loader waves are the stragglers of every interval with 8 folds and 24 loads (their
// barrier arrivals, RW_LSTAMP: 3.7-4.1 us against the compute waves' 2.7-3.3), so 2 spreads
// the zy folds over 1 / 3 / 5 and moves the records to 7: 1913-1930 vs 1944-1946 us
#ifndef RW_SCHED
#define RW_SCHED 2
#endif
// the loader's row loads paced: s_sleep RW_PACE (x 64 cycles) after each item's 3 loads
#ifndef RW_PACE
#define RW_PACE 0
#endif
// diagnostics (tools/rchain_timing.py; results wrong): the loader waves' row work, 1 = none
// (barriers only), 2 = loads without folds, 3 = folds of constants without loads
// diagnostics (results wrong): RW_ROWS_L2 = 1 reads every row from the first 1024 vertices
// (an L2-resident 1 MB): the row loads' cost without their HBM latency
#ifndef RW_LSTAMP
#define RW_LSTAMP 0
#endif
#ifndef RW_ROWS_L2
#define RW_ROWS_L2 0
#endif
#ifndef RW_LOADER_IDLE
#define RW_LOADER_IDLE 0
#endif

template <int L_, int S_>
struct WP {
  static constexpr int L = L_, S = S_, NH = L - 2, NBAR = 2 + 2 * NH;
  static constexpr int H = 256, CW = 8, LW = 4, RT = 8, BM = 16 * RT;
  static constexpr int THREADS = (CW + LW) * 64, LT = LW * 64;
  static constexpr int TN = H / (16 * CW);
  static constexpr int UPL = H / 32, NT = H / 16;
  static constexpr int ACT_T = 16 * H * 2, ACT_BYTES = RT * ACT_T;
  static constexpr int ZROW = 2 * H;         // bytes of one ray's half row (z0 or zy)
  static constexpr int HC = ZROW / 16;       // 16-byte chunks per half row
  static constexpr int NI = BM * HC / LT;    // (ray, chunk) items per loader thread and half
  static constexpr int NG = 4, G = NI / NG;  // groups per half, items per group
  static constexpr int RPI = LT / HC;        // rays between one thread's items
  static constexpr int NREC = 3 * BM;        // (ray, vertex) records per tile
  static constexpr int OFF_ACT = 0;                         // [RT] activation tiles
  static constexpr int OFF_Z = ACT_BYTES;                   // [BM][H] bf16: z0 or zy
  static constexpr int OFF_REC = OFF_Z + BM * ZROW;         // [2][NREC] vertex ids (-1: zero row)
  static constexpr int OFF_RB = OFF_REC + 2 * NREC * 4;     // [2][NREC] barycentrics
  static constexpr int OFF_W7F = OFF_RB + 2 * NREC * 4;     // [UPL][hi, lo][64 lanes] W7 A fragments
  static constexpr int OFF_PIX = OFF_W7F + UPL * 2 * 64 * 16;  // [BM] image pixel of each ray
  static constexpr int OFF_B7 = OFF_PIX + BM * 8;           // b7[3]
  static constexpr int OFF_VEC = OFF_B7 + 16;               // biases [L-1][H], Ly.bias [H]
  static constexpr int LDS = OFF_VEC + L * H * 4;
  static_assert(NG == 4 && NI % NG == 0 && LT % HC == 0 && NREC <= 2 * LT && BM <= LT, "loader items");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(CW == RT, "the head: one ray tile per compute wave");
  // the loader schedule (top of the file): zy folded by interval 3 <= 2s - 2, z0 from
  // interval 9 >= 2s + 1 on
  static_assert(S == 4 && NH == 6, "loader schedule");
};

// SIMPLE: rays in batch order with 32-bit vertex ids (no permutation)
template <int L_, int S_, bool SIMPLE>
__global__ __launch_bounds__((WP<L_, S_>::THREADS)) void rprojw_kernel(const RchainArgs a) {
  using C = WP<L_, S_>;
  constexpr int RT = C::RT, BM = C::BM, TN = C::TN, UPL = C::UPL, CW = C::CW, G = C::G, HC = C::HC,
                THREADS = C::THREADS, LT = C::LT, L = C::L, S = C::S, NH = C::NH, NBAR = C::NBAR, H = C::H;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* act = smem + C::OFF_ACT;
  char* zs = smem + C::OFF_Z;
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_REC);
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RB);
  char* w7f = smem + C::OFF_W7F;
  int64_t* rpix = reinterpret_cast<int64_t*>(smem + C::OFF_PIX);
  float* b7s = reinterpret_cast<float*>(smem + C::OFF_B7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  // a contiguous range of tiles per workgroup, neighbouring ranges on one XCD (rproj.hip)
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
  if (tid < 3) b7s[tid] = a.b7[tid];
  // W7 as MFMA A fragments, bf16 hi and lo parts: lane (o = row, g) of k block kb holds
  // W7[o][32 kb + 16 (e / 4) + 4 g + e % 4] for e = 0 .. 7 (the activation tile's k order),
  // rows o >= 3 zero
  for (int i = tid; i < UPL * 64; i += THREADS) {
    const int kb = i / 64, l = i % 64, o = l & 15, g = l >> 4;
    u16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float w = o < 3 ? a.W7[o * H + 32 * kb + 16 * (e >> 2) + 4 * g + (e & 3)] : 0.f;
      hi[e] = bf_bits3(w);
      lo[e] = bf_bits3(w - bf_val3(hi[e]));
    }
    *reinterpret_cast<u16x8*>(w7f + ((kb * 2 + 0) * 64 + l) * 16) = hi;
    *reinterpret_cast<u16x8*>(w7f + ((kb * 2 + 1) * 64 + l) * 16) = lo;
  }

  // ---- weight fragments of the hidden layers (rproj.hip's ring) ---------------------------
  const int t0 = wc * TN;
  constexpr int D = RW_DEPTH < UPL ? RW_DEPTH : UPL;
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

  // ---- ray records: (ray, vertex) item x of a tile -> record set `set` -------------------
  struct Rec {
    int v;  // vertex id, -1: the ray's row reads as zero (out-of-range id or ray index)
    float w;
  };
  auto rec_load = [&](int tile, int x) -> Rec {
    Rec r{-1, 0.f};
    if (x < C::NREC) {
      const int b = tile * BM + x / 3, i = x % 3;
      const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, a.idx_offset, b, a.num_rays, a.num_src) : -1;
      if (rr >= 0) {
        const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
        r.v = (uint64_t)e < (uint64_t)a.num_vertices ? (int)e : -1;  // out-of-range ids: zero rows (gather.hip)
        r.w = a.bary[3 * rr + i];
      }
    }
    return r;
  };
  auto rec_store = [&](const Rec& r, int set, int x) {
    if (x < C::NREC) {
      rvid[set * C::NREC + x] = r.v;
      rbary[set * C::NREC + x] = r.w;
    }
  };
  // The loader's records and pixel indices, issued one interval set ahead of their stores
  // with no use in between (branch-free addresses), so that no wait of theirs lands in a
  // short interval: a record's raw vertex id and weight, and whether the ray has a row
  struct RecRaw {
    int e;  // vertex id (-1: out of range in the general path; range-checked at the store)
    float w;
    int ok;  // the ray has a source row
  };
  auto rec_issue = [&](int tile, int x) -> RecRaw {
    const int b = tile * BM + x / 3, i = x % 3;
    if constexpr (SIMPLE) {
      // rays in order, 32-bit ids (the render's batches): two independent loads, no waits
      const int64_t rr = x < C::NREC && b < a.batch ? source_row(nullptr, 0, a.idx_offset, b, a.num_rays, a.num_src) : -1;
      const int64_t q = rr >= 0 ? 3 * rr + i : 0;
      return RecRaw{reinterpret_cast<const int32_t*>(a.vids)[q], a.bary[q], rr >= 0};
    }
    else {  // (a permutation or 64-bit ids: the loads' waits land in interval 11)
      const int64_t rr =
          x < C::NREC && b < a.batch ? source_row(a.ray_idx, a.idx_dtype, a.idx_offset, b, a.num_rays, a.num_src) : -1;
      const int64_t q = rr >= 0 ? 3 * rr + i : 0;
      const int64_t e = vid_at(a.vids, a.vid_dtype, q);
      return RecRaw{(uint64_t)e < (uint64_t)a.num_vertices ? (int)e : -1, a.bary[q], rr >= 0};
    }
  };
  auto rec_put = [&](const RecRaw& r, int set, int x) {  // out-of-range ids: zero rows (gather.hip)
    rec_store(Rec{r.ok && (uint32_t)r.e < (uint64_t)a.num_vertices ? r.e : -1, r.w}, set, x);
  };
  // the image pixel of ray x of a tile (renderer.py:139-141's placement index): hit[b]
  // issued, the pixel map applied at the store
  auto pix_issue = [&](int tile, int x) -> int64_t {
    const int b = tile * BM + x;
    return a.img != nullptr ? a.hit[x < BM && b < a.batch ? b : 0] : -1;
  };
  auto pix_put = [&](int64_t p, int tile, int x) {
    const int b = tile * BM + x;
    if (x < BM) rpix[x] = a.img != nullptr && b < a.batch ? (a.pixel_map != nullptr ? a.pixel_map[p] : p) : -1;
  };

  // ---- 16-byte chunk c of half h (0: W_0 E, 1: W_y E) of ray r's projected row: the three
  // vertex rows' chunks, and their fold into Z (rproj.hip's arithmetic: fp32 FMAs in the
  // gather's order, one bf16 rounding; a ray with any zero-row vertex reads as zero)
  auto rows_load = [&](int h, int set, int r, int c, u16x8 (&ev)[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int v = max(rvid[set * C::NREC + r * 3 + i], 0) & (RW_ROWS_L2 ? 1023 : -1);
      ev[i] = __builtin_bit_cast(u16x8,
                                 *reinterpret_cast<const u32x4*>(a.table + (int64_t)v * (2 * H) + (h * HC + c) * 8));
    }
  };
  auto rows_store = [&](int set, int r, int c, const u16x8 (&ev)[3]) {
    const int* rv = rvid + set * C::NREC + r * 3;
    const float* rw = rbary + set * C::NREC + r * 3;
    // a zero-row ray: zero weights (its rows are row 0's, finite), so the fold is a signed
    // zero instead of rproj.hip's +0 (the same sums downstream) at 3 selects, not 8
    const bool ok = (rv[0] | rv[1] | rv[2]) >= 0;
    const float w0 = ok ? rw[0] : 0.f, w1 = ok ? rw[1] : 0.f, w2 = ok ? rw[2] : 0.f;
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      o[e] = bf_bits3(fmaf(w2, bf_val3(ev[2][e]), fmaf(w1, bf_val3(ev[1][e]), w0 * bf_val3(ev[0][e]))));
    *reinterpret_cast<u16x8*>(zs + r * C::ZROW + ((c ^ (r & 15)) << 4)) = o;
  };

  // ---- prologue: the first tile's records and z0, every wave ------------------------------
  for (int x = tid; x < C::NREC; x += THREADS) rec_store(rec_load(tb, x), 0, x);
  lbar();  // records, vectors, W7 fragments in LDS
  stamp(1);
#pragma unroll 1
  for (int q0 = tid; q0 < BM * HC; q0 += 2 * THREADS) {
    u16x8 ev[2][3];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int q = q0 + n * THREADS;
      if (q < BM * HC) rows_load(0, 0, q / HC, q % HC, ev[n]);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int q = q0 + n * THREADS;
      if (q < BM * HC) rows_store(0, q / HC, q % HC, ev[n]);
    }
  }
  lbar();  // Z holds the first tile's z0
  stamp(2);

  if (wc >= CW) {
    // ---- loader waves.  Thread x: chunk x % HC of rays x / HC + RPI m (m = g G .. g G +
    // G - 1 in group g)
    const int x = tid - CW * 64;
    const int lc = x % HC, lr = x / HC;
    u16x8 eA[G][3], eB[G][3];
    // diagnostics (RW_LSTAMP): the first loader thread of workgroup 0 stamps its arrival at
    // each barrier of the second tile (stamps 34 + j)
    unsigned long long* lst = nullptr;
    if (RW_LSTAMP && a.stamps != nullptr && x == 0 && bid == 0) lst = a.stamps + 34;
    auto load_group = [&](int h, int set, int g, u16x8 (&e)[G][3]) {
      if constexpr (RW_LOADER_IDLE == 1 || RW_LOADER_IDLE == 3) {  // diagnostics: no loads
#pragma unroll
        for (int m = 0; m < G; ++m)
#pragma unroll
          for (int i = 0; i < 3; ++i) e[m][i] = u16x8{(unsigned short)(x + m), 1, 2, 3, 4, 5, 6, (unsigned short)i};
        return;
      }
#pragma unroll
      for (int m = 0; m < G; ++m) {
        rows_load(h, set, lr + C::RPI * (g * G + m), lc, e[m]);
        if constexpr (RW_PACE > 0) __builtin_amdgcn_s_sleep(RW_PACE);
      }
    };
    auto store_group = [&](int set, int g, u16x8 (&e)[G][3]) {
      // pin the raw loaded registers here (rproj.hip: the unpacking is otherwise hoisted to
      // the loads and the live registers double across the barriers)
#pragma unroll
      for (int m = 0; m < G; ++m)
#pragma unroll
        for (int i = 0; i < 3; ++i) asm volatile("" : "+v"(e[m][i]));
      if constexpr (RW_LOADER_IDLE == 1 || RW_LOADER_IDLE == 2) {  // diagnostics: no folds
        if (e[0][0][0] == 0x1234 && e[G - 1][2][7] == 0x4321) zs[x] = 1;
        return;
      }
#pragma unroll
      for (int m = 0; m < G; ++m) rows_store(set, lr + C::RPI * (g * G + m), lc, e[m]);
    };
    // ahead of the loop: the second tile's records (set 1), the first tile's pixels, zy of
    // the first tile (groups 0 and 1)
    if (tb + 1 < te) {
      rec_put(rec_issue(tb + 1, x), 1, x);
      rec_put(rec_issue(tb + 1, x + LT), 1, x + LT);
    }
    int64_t px = pix_issue(tb, x);
    load_group(1, 0, 0, eA);
    load_group(1, 0, 1, eB);
#pragma unroll 1
    for (int tile = tb; tile < te; ++tile) {
      const int cur = (tile - tb) & 1, nxt = cur ^ 1;
      const bool has_next = tile + 1 < te;
      RecRaw r0{-1, 0.f, 0}, r1{-1, 0.f, 0};
      sfor<NBAR>([&](auto J) {
        constexpr int j = decltype(J)::value;
        constexpr bool E = RW_SCHED == 1;
        if constexpr (j == 0) pix_put(px, tile, x);  // (the previous tile's head has read rpix)
        if constexpr (RW_SCHED == 2) {
          // balanced: the zy folds over intervals 1, 3, 5 (4, 4, 8 items), the records and
          // pixels issued in interval 7 (no other loader work there)
          if constexpr (j == 1) {
            store_group(cur, 0, eA);
            load_group(1, cur, 2, eA);
          }
          if constexpr (j == 3) {
            store_group(cur, 1, eB);
            load_group(1, cur, 3, eB);
          }
          if constexpr (j == 5) {
            store_group(cur, 2, eA);
            store_group(cur, 3, eB);
            if (has_next) {
              load_group(0, nxt, 0, eA);
              load_group(0, nxt, 1, eB);
            }
          }
          if constexpr (j == 7) {
            if (tile + 2 < te) {
              r0 = rec_issue(tile + 2, x);
              r1 = rec_issue(tile + 2, x + LT);
            }
            if (has_next) px = pix_issue(tile + 1, x);
          }
          if constexpr (j == 9) {
            if (has_next) {
              store_group(nxt, 0, eA);
              store_group(nxt, 1, eB);
              load_group(0, nxt, 2, eA);
              load_group(0, nxt, 3, eB);
            }
          }
          if constexpr (j == 11) {
            if (has_next) {
              store_group(nxt, 2, eA);
              store_group(nxt, 3, eB);
              load_group(1, nxt, 0, eA);
              load_group(1, nxt, 1, eB);
            }
          }
          if constexpr (j == 12) {
            if (tile + 2 < te) {
              rec_put(r0, cur, x);
              rec_put(r1, cur, x + LT);
            }
          }
        } else {
        if constexpr (j == 1) {
          store_group(cur, 0, eA);
          store_group(cur, 1, eB);
        }
        if constexpr (j == (E ? 2 : 1)) {
          load_group(1, cur, 2, eA);
          load_group(1, cur, 3, eB);
        }
        if constexpr (j == 3) {
          store_group(cur, 2, eA);
          store_group(cur, 3, eB);
        }
        if constexpr (j == (E ? 6 : 5)) {
          if (has_next) {
            load_group(0, nxt, 0, eA);
            load_group(0, nxt, 1, eB);
          }
        }
        if constexpr (j == 9) {
          if (has_next) {
            store_group(nxt, 0, eA);
            store_group(nxt, 1, eB);
          }
        }
        if constexpr (j == (E ? 10 : 9)) {
          if (has_next) {
            load_group(0, nxt, 2, eA);
            load_group(0, nxt, 3, eB);
          }
        }
        if constexpr (j == 11) {
          if (has_next) {
            store_group(nxt, 2, eA);
            store_group(nxt, 3, eB);
          }
          // records of tile + 2 (stored in interval 12, into this tile's set: its last
          // reader, zy's fold, was interval 3) and pixels of tile + 1 (stored in its interval 0)
          if (tile + 2 < te) {
            r0 = rec_issue(tile + 2, x);
            r1 = rec_issue(tile + 2, x + LT);
          }
          if (has_next) px = pix_issue(tile + 1, x);
        }
        if constexpr (j == 12) {
          if (tile + 2 < te) {
            rec_put(r0, cur, x);
            rec_put(r1, cur, x + LT);
          }
        }
        if constexpr (j == (E ? 12 : 11)) {
          if (has_next) {
            load_group(1, nxt, 0, eA);
            load_group(1, nxt, 1, eB);
          }
        }
        }
        if constexpr (RW_LSTAMP) {
          if (lst != nullptr && tile == tb + 1) {
            __builtin_amdgcn_sched_barrier(0);
            lst[j] = wall_clock64();
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        lbar();
      });
    }
    return;
  }

  int aoffs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) aoffs[q] = act_off(q, r16, g4) - q * 1024;
  auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
  auto bread = [&](int kb, int t) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(act + t * C::ACT_T + kb * 1024 + aoffs[kb & 3]);
  };
  f32x4 acc[RT][TN];

  // layer l's bias (+ Ly.bias and the tile's W_y x at the skip layer) as the accumulators'
  // start (rproj.hip's order)
  auto init_acc = [&](int l) {
    const bool skip = l == S;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 bb = *reinterpret_cast<const f32x4*>(vecs + l * H + feat(j));
      if (skip) bb += *reinterpret_cast<const f32x4*>(vecs + (L - 1) * H + feat(j));
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        acc[t][j] = bb;
        if (skip) {
          const u16x4 zy = *reinterpret_cast<const u16x4*>(zs + tile_off(C::ZROW, t * 16 + r16, feat(j)));
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][j][r] += bf_val3(zy[r]);
        }
      }
    }
  };

  // ReLU -> bf16 -> the activation tile (in place: after B1)
  auto epilogue_act = [&]() {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      char* dst = act + t * C::ACT_T;
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        u32x4 w;
        w[0] = pack_bf16x2(relu1(acc[t][j][0]), relu1(acc[t][j][1]));
        w[1] = pack_bf16x2(relu1(acc[t][j][2]), relu1(acc[t][j][3]));
        w[2] = pack_bf16x2(relu1(acc[t][j + 1][0]), relu1(acc[t][j + 1][1]));
        w[3] = pack_bf16x2(relu1(acc[t][j + 1][2]), relu1(acc[t][j + 1][3]));
        *reinterpret_cast<u32x4*>(dst + act_off((t0 + j) >> 1, r16, g4)) = w;
      }
    }
  };

  // one hidden layer: UPL k blocks of the activation tile; the B operands RA reads ahead
  // over the (k block, ray tile) sequence
  auto run_block = [&](int hb) {
    const C3Block& B = a.blk[hb];
    const C3Block& Bn = a.blk[hb + 1 < NH ? hb + 1 : 0];
    const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
    const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
    constexpr int RA = RW_RA, NSEQ = UPL * RT;
    bf16x8 bq[RA];
#pragma unroll
    for (int i = 0; i < RA; ++i) bq[i] = bread(i / RT, i % RT);
#pragma unroll
    for (int kb = 0; kb < UPL; ++kb) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int i = kb * RT + t;
        const bf16x8 b = bq[i % RA];
        if (i + RA < NSEQ) bq[i % RA] = bread((i + RA) / RT, (i + RA) % RT);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], b, acc[t][j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fr[kb % D][j] = kb + D < UPL ? frag(crs, kb + D, j) : frag(nrs, kb + D - UPL, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

#pragma unroll 1
  for (int tile = tb; tile < te; ++tile) {
    const bool st = tile - tb < 2;
    const int sbase = 3 + (tile - tb) * NBAR;
    // this tile's layer-0 pre-activations out of Z (+ bias 0), ReLU into the activation tile
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
    epilogue_act();
    lbar();  // 0: layer 1's input complete, Z free for zy
    if (st) stamp(sbase);

#pragma unroll 1
    for (int hb = 0; hb < NH; ++hb) {
      init_acc(hb + 1);
      run_block(hb);
      lbar();  // 2l - 1: every wave's MFMAs have read the activation tile
      if (st) stamp(sbase + 1 + 2 * hb);
      epilogue_act();
      lbar();  // 2l: the next layer's input (after layer L - 2: h) complete
      if (st) stamp(sbase + 2 + 2 * hb);
    }

    // ---- the head (model.py:89-94) on ray tile wc: z = W7 h + b7 (hi and lo W7 fragments),
    // sigmoid and placement (renderer.py:132-141) ---------------------------------------------
    {
      // (the lane's addresses from the lane id recomputed here by volatile asm: kept live
      // across the tile they had been spilled, and a spill reload waits for the whole
      // vector-memory queue -- the next tile's fragments in flight)
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      f32x4 hz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
        const bf16x8 b = bread(kb, wc);
        const bf16x8 whi = *reinterpret_cast<const bf16x8*>(w7f + ((kb * 2 + 0) * 64 + ln) * 16);
        const bf16x8 wlo = *reinterpret_cast<const bf16x8*>(w7f + ((kb * 2 + 1) * 64 + ln) * 16);
        hz = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi, b, hz, 0, 0, 0);
        hz = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo, b, hz, 0, 0, 0);
      }
      // lanes 0 .. 15 hold rows 0 .. 3 (the outputs) of ray wc 16 + lane
      const int ray = wc * 16 + (ln & 15);
      const int b = tile * BM + ray;
      if (ln < 16 && b < a.batch) {
        const int64_t pix = a.img != nullptr ? rpix[ray] : -1;
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          const float z = hz[o] + b7s[o];
          const float pv = 1.f / (1.f + expf(-z));
          if (a.pred != nullptr) a.pred[(int64_t)b * 3 + o] = pv;
          if (a.img != nullptr) a.img[pix * 3 + o] = pv;
        }
      }
    }
    lbar();  // 13: the activation tile free for the next tile (the loader: its intervals)
    if (st) stamp(sbase + 13);
  }
}

template <int L, int S, bool SIMPLE>
int launch_typed(const RchainArgs& a, hipStream_t stream) {
  using C = WP<L, S>;
  static bool attr_set = false;
  if (!attr_set) {
    INF_HIP_TRY(
        hipFuncSetAttribute((const void*)rprojw_kernel<L, S, SIMPLE>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
    attr_set = true;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    INF_HIP_TRY(hipGetDevice(&dev));
    INF_HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int64_t ntile = ceil_div(a.batch, C::BM);
  const int grid = (int)std::min<int64_t>(ntile, ncu);
  rprojw_kernel<L, S, SIMPLE><<<dim3((unsigned)grid), dim3(C::THREADS), C::LDS, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

bool rprojw_supported(const RchainArgs& a) {
  const char* e = std::getenv("INF_RPROJ_WIDE");  // "0": rproj.hip's 64-ray tiles
  return (e == nullptr || e[0] != '0') && a.H == 256 && a.L == 8 && a.s == 4;
}

// (launch_rproj has checked the arguments)
int launch_rprojw(const RchainArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(rprojw_supported(a), "rprojw: unsupported shape");
  if (a.ray_idx == nullptr && a.vid_dtype == INF_DTYPE_I32) return launch_typed<8, 4, true>(a, stream);
  return launch_typed<8, 4, false>(a, stream);
}

}  // namespace inf
