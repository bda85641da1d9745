// Register-streamed fused training chain: the bf16 training step of small batches (the
// reference's 4096-ray batch, intrinsic_cat.yaml:32) up to the weight gradients.
//
// One workgroup owns BM = 16 rays and runs, in ONE launch:
//   gather    X[b] = sum_i bary[r][i] * E[vids[r][i]] for its rays r = ray_idx[offset + b]
//             (mesh.py:313-324 with ray_dataloader.py:122-129), into LDS,
//   forward   layers 0..L-2 (model.py:98-112); the skip layer (layers.py:60-62) as two
//             K segments [h | x] into one accumulator,
//   head      Linear(H,3) + sigmoid (model.py:89-94), loss (config.py:113-122),
//             dL/dz = dL/dp * p (1 - p),
//   backward  dZ_{L-2} = (dz W_head) * (h > 0), then dZ_{l-1} = (dZ_l W_l) * (Y_{l-1} > 0)
//             for l = L-2..1 (autograd of trainer.py:81),
// and leaves what the weight-gradient GEMM needs: X^T, Y_l^T, dZ_l^T, bias partials.
//
// Why registers, not an LDS ring.  At 16 rays per workgroup every weight element feeds
// exactly one wave (the 8 compute waves split the output features), so staging weights
// through LDS buys no reuse; what bounds the kernel is the L2 -> CU weight stream.  The
// packed weights are stored in MFMA fragment order (adam.hip: 1 KiB per 16 rows x 32 k,
// lane l's 16 bytes at 16 l), so a wave's operand for one 32-deep k block is TN coalesced
// 1 KiB loads straight into VGPRs.  The weight stream is a list of blocks (C3Block: UPL
// k-blocks each, one hidden layer's K); each wave keeps a ring of D k-blocks of fragments
// in flight and refills a slot right after its MFMAs consumed it -- across block, phase
// and epilogue boundaries, with no per-k-step barrier.  After the gather the only
// vector-memory instructions of the compute waves are these loads, so the compiler's
// vmcnt waits are exact (each waits for one k-block).  Eight compute waves (two per SIMD)
// keep twice the loads of four in flight: the L2 -> CU stream rate grows with them
// (tools/microbench/l2ring.hip).
//
// Orientation.  The weights are the A operand and the 16 rays the B operand, so a wave's
// accumulators hold Z^T: lane l has ray l % 16 and features 16 t + 4 (l / 16) + r.  Eight
// such values of a tile pair (2q, 2q + 1) are exactly the lane's B operand of k block q of
// the next layer, with the k order inside the block permuted (slot (g, e) = feature
// 16 (e / 4) + 4 g + e % 4); the weight images of the layers fed by activations are written
// in that order (adam.hip, wf_acc_order).  An epilogue therefore stores each lane's
// activations to the LDS tile with one 16-byte write per k block, and nothing has to be
// transposed on the compute waves' critical path.
//
// Stores.  Every global output (X^T, Y^T, dZ^T, bias / output-layer partials, loss, pred)
// is copied to HBM by a ninth "store" wave that mirrors the compute waves' barriers and
// does the ray-major -> feature-major transposes from the LDS tile.  Stores in the compute
// waves would join the in-order vmcnt queue and make the next fragment wait for them.
#include "chain3.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using namespace c3;

constexpr float C3_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
constexpr int C3_CW = 8;                      // compute waves
constexpr int C3_CT = C3_CW * 64;             // compute threads
constexpr int C3_THREADS = C3_CT + 64;        // + the store wave
constexpr int C3_LDS_CAP = 160 * 1024;
#ifndef C3_DEPTH
#define C3_DEPTH 8
#endif
constexpr int C3BM = 16;  // rays per 16-row MFMA tile (= per workgroup at NR = 1)
// Wide tiles (NR = C3_NR_WIDE ray tiles per workgroup, batches above CHAIN3_MAX_ROWS):
// each fetched weight fragment feeds NR MFMAs instead of one, so the L2 -> CU weight
// stream per ray drops NR-fold; the feature tile is streamed in C3_KC_WIDE-column chunks
// (64 x 1024 bf16 would not fit beside the activation tiles) and the fragment ring is
// shallower (each k block now carries NR times the MFMA work)
#ifndef C3_DEPTH_WIDE
#define C3_DEPTH_WIDE 4
#endif
// Cache policy of the table-row loads: non-temporal for tables larger than the MALL (rows
// read once per step would evict the weight stream's L2 lines; config D's 4.1 GB table),
// the default policy below it -- a MALL-resident table (config B's 102 MB) measured 0.8-1.0
// us per step faster that way (profiles/r02/sweeps/gather_policy.log); config D with it 2.5
// us slower
constexpr int C3_CPOL_NT = 2;

// 1 if x != 0 else 0, as one v_min_u32 (asm: the compiler turns min(x, 1) back into a
// compare whose lane mask lives in an SGPR pair)
__device__ __forceinline__ unsigned nz1(unsigned x) {
  unsigned r;
  asm("v_min_u32 %0, 1, %1" : "=v"(r) : "v"(x));
  return r;
}

template <int H, int NR, bool X3 = false>
struct L3 {
  static constexpr int BM = C3BM * NR;          // rays per workgroup
  static constexpr int TN = H / (16 * C3_CW);  // 16-feature tiles per wave (2: H = 256, 1: H = 128)
  static constexpr int WN = H / C3_CW;          // features per wave
  static constexpr int UPL = H / 32;            // 32-deep k blocks per hidden layer (= per stream block)
  static constexpr int NT = H / 16;             // 16-row tiles per k block of a weight image
  static constexpr int TILE_BYTES = C3BM * H * 2;  // one 16-ray activation tile
  static constexpr int ACT_BYTES = NR * TILE_BYTES;
  static constexpr int KC = NR == 1 ? C3_KC : C3_KC_WIDE;  // feature columns per chunk (XC)
  // activation / dZ tiles (act_off layout per 16-ray tile), double-buffered: epilogue p
  // writes tile (p + 1) & 1, phase p reads tile p & 1, so one barrier per phase suffices
  // per-workgroup partials (sums over all BM rays) of the bias / output-layer gradients
  // and the loss
  // X3 (split-bf16 mode): the lo halves of the two activation buffers follow the hi ones
  // (buffer b: hi at b ACT_BYTES, lo at (2 + b) ACT_BYTES), the lo feature tile the hi one
  static constexpr int OFF_ACT = 0;
  static constexpr int ACT_LO = 2 * ACT_BYTES;  // lo tile of a buffer, from its hi tile
  static constexpr int OFF_CS = OFF_ACT + (X3 ? 4 : 2) * ACT_BYTES;  // [2][H] bias-gradient partials (epilogue p: p & 1)
  static constexpr int OFF_HW = OFF_CS + 2 * H * 4;       // [3][H] output-layer weight grad
  static constexpr int OFF_HB = OFF_HW + 3 * H * 4;       // [4]
  static constexpr int OFF_LS = OFF_HB + 16;              // [2] f64 loss / SSE
  static constexpr int OFF_PRED = OFF_LS + 16;            // [BM][3]
  // [waves][BM][3] head gradient; wide tiles: in the head phase's input activation tile,
  // idle from barrier Bh1 on (all MFMAs of the phase and its Y^T copy are done)
  static constexpr int OFF_DZ = OFF_PRED + BM * 12;
  static constexpr int DZ_BYTES = NR == 1 ? C3_CW * BM * 12 : 0;
  static constexpr int OFF_TGT = OFF_DZ + DZ_BYTES;       // [BM][3] targets
  static constexpr int OFF_ZP = OFF_TGT + BM * 12;        // [waves][BM][3] head partial sums
  static constexpr int OFF_RAY = OFF_ZP + C3_CW * BM * 12;  // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RBARY = OFF_RAY + BM * 16 + BM * 12 + 16;  // [BM][3] barycentrics
  static constexpr int OFF_W7 = OFF_RBARY + BM * 12 + 16;  // [3][H] then b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;  // biases [L-1][H], then Ly.bias [H]
  // the feature tile holds kx columns: k_pad, or KC when it is streamed in chunks.  Wide
  // chunked tiles park the W_y x accumulators of phase 0 in the same region from barrier
  // B2(0) on ([wave][NR TN][lane] 16-byte slots), when the last chunk is done with
  static constexpr int ACCY_BYTES = C3_CW * 64 * NR * TN * 16;
  __host__ __device__ static int off_x(int L) { return OFF_VEC + L * H * 4; }
  __host__ __device__ static int x_region(int kx, bool xc) {
    return (NR > 1 && xc && ACCY_BYTES > BM * kx * 2) ? ACCY_BYTES : (X3 ? 2 : 1) * BM * kx * 2;
  }
  __host__ __device__ static int off_stamp(int L, int kx, bool xc) { return off_x(L) + x_region(kx, xc); }
  static int lds_bytes(int L, int kx, bool xc) { return off_stamp(L, kx, xc) + (7 * C3_MAX_PHASES + 8) * 8; }
  static_assert(TN >= 1 && TN * 4 <= 8, "ReLU bits of a lane: at most 8 per layer");
  static_assert(TN * 4 * NR <= 32, "ReLU bits of a lane: one 32-bit word per layer (wide tiles)");
  static_assert(OFF_LS % 8 == 0 && OFF_W7 % 16 == 0 && OFF_VEC % 16 == 0, "LDS alignment");
};

// ENC: the extrinsic front-end (Chain3Args::encoding != INF_ENC_NONE) -- a separate
// instantiation so the eigenfunction gather's code and registers stay as they were.
// XC: the feature tile is streamed in C3_KC-column chunks (k_pad > C3_KC, config D's
// k = 4096).  Phase 0 then runs BOTH input layers over each chunk -- Ly's product
// W_y x is independent of h, so it is accumulated in a second register set (accy) while
// the chunk is resident and added in the skip layer's epilogue; each chunk is gathered
// once, at its first block (two barriers: everyone is done with the previous chunk /
// the new one is in LDS), and the store wave copies its X^T between them.
// NR: 16-ray tiles per workgroup (1, or C3_NR_WIDE for large batches; not with ENC).
// ZP: the input layers were computed ahead of the chain (zg.hip: Z = [W_0; W_y] X^T in
// the accumulator layout, X^T written by its gather): no gather here, phase 0 is the
// layer-0 epilogue on Z, the skip layer adds W_y x from LDS (staged by the store wave with
// direct-to-LDS loads) in its epilogue, and the weight stream holds the hidden layers only.
// X3: the split-bf16 parity mode (Chain3Args::x3): hi / lo weight images, hi / lo
// feature and activation tiles, three MFMAs per k block, fp32 gather / epilogues / head.
template <int H, int LOSS, bool ENC, bool XC, int NR, bool ZP, bool X3>
__global__ __launch_bounds__(C3_THREADS) void chain3_kernel(const Chain3Args a) {
  using C = L3<H, NR, X3>;
  constexpr int BM = C::BM, TN = C::TN, UPL = C::UPL;
  constexpr int NV = TN * 4;  // accumulator values per lane and ray tile
  static_assert(NR == 1 || !ENC, "wide tiles: eigenfunction tables only");
  static_assert(!ZP || (NR == 1 && !ENC && !XC), "precomputed input layers: narrow whole-tile schedule only");
  static_assert(!X3 || (NR == 1 && !ENC && !XC && !ZP), "split-bf16 chain: narrow whole-tile schedule only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L;
  const int k_pad = a.k_pad;
  char* act = smem + C::OFF_ACT;
  float* csb = reinterpret_cast<float*>(smem + C::OFF_CS);
  float* hws = reinterpret_cast<float*>(smem + C::OFF_HW);
  float* hbs = reinterpret_cast<float*>(smem + C::OFF_HB);
  double* lss = reinterpret_cast<double*>(smem + C::OFF_LS);
  float* preds = reinterpret_cast<float*>(smem + C::OFF_PRED);
  float* dzs = reinterpret_cast<float*>(NR == 1 ? smem + C::OFF_DZ : smem + C::OFF_ACT + ((L - 2) & 1) * C::ACT_BYTES);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);          // [BM][4]
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RBARY);  // [BM][3]
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  char* xs = smem + C::off_x(L);  // gathered features [BM][kx] bf16 (tile_off layout)
  // columns resident in LDS (ZP: the region holds W_y x, zin_parts slices of 16 rays x H fp32)
  const int kx = ZP ? a.zin_parts * 2 * H : (XC ? C::KC : k_pad);
  const int xrow = kx * 2;
  const int x_lo = BM * xrow;  // X3: the lo feature tile, from the hi one

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int nphase = a.nphase;
  const int nfwd = L - 1;  // forward phases 0..L-2

  unsigned long long* stl = nullptr;  // diagnostics only
  // wave 0 records everything; the last compute wave and the store wave their B1 arrivals
  const bool stamp_wg = a.stamps != nullptr && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1);
  if (stamp_wg && (wave == 0 || wave == C3_CW - 1 || wave == C3_CW))
    stl = reinterpret_cast<unsigned long long*>(smem + C::off_stamp(L, kx, XC));
  const unsigned long long t_entry = stl != nullptr ? wall_clock64() : 0ull;
  auto stamp = [&](int i) {
    if (stl != nullptr) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = wall_clock64();
      if (lane == 0 && (wave == 0 || i >= 5 * nphase + 6)) stl[i] = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (wave < C3_CW) {
    // =========================== compute waves ============================================
    const int wc = wave;
    const int t0 = wc * TN;  // the wave's first 16-feature tile
    // fragment ring: D k-blocks (D * TN KiB per wave) in flight
    // X3: hi and lo fragments per k block, half the depth (the same bytes in flight)
#ifndef C3_X3_DEPTH
#define C3_X3_DEPTH (C3_DEPTH / 2)
#endif
    constexpr int D0 = NR == 1 ? (X3 ? C3_X3_DEPTH : C3_DEPTH) : C3_DEPTH_WIDE;
    constexpr int D = D0 < UPL ? D0 : UPL;
    // every block starts at ring slot 0 (slot = k block % D)
    static_assert(UPL % D == 0, "the fragment ring depth must divide a block's k blocks");
    bf16x8 fr[D][TN];
    bf16x8 frl[X3 ? D : 1][TN];  // X3: the lo image's fragments
    // X3: the lo image of a block's weight follows its hi image -- k block kb of lo is k
    // block kb + (k blocks of the image): k_pad / 32 for the input layers (fed X), H / 32
    // for the hidden ones (forward and transposed)
    auto lo_kb = [&](const C3Block& B) { return B.a_x ? k_pad / 32 : UPL; };
    // buffer loads: descriptor per image in SGPRs, k-block offset in soffset, tile offset
    // as the immediate, one VGPR of lane offset -- no 64-bit address registers
    const unsigned lane_off = (unsigned)(t0 * 64 + lane) * 16u;
    auto rsrc_of = [&](const bf16* img) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
    };
    auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j) -> bf16x8 {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024, kb * C::NT * 1024, 0);
      return __builtin_bit_cast(bf16x8, v);
    };
    // ---- gather: ray records of the 16 rays (index, vertex ids, barycentrics), one
    // thread per (ray, corner) ------------------------------------------------------------
    if (!ZP && tid < BM * 3 && a.xpre == nullptr) {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int rl = tid / 3, i = tid % 3;
      const int b = b0 + rl;
      int v = 0, ok = 0;
      float w = 0.f;
      const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src) : -1;
      if (rr >= 0) {
        const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
        // an out-of-range vertex id reads as a zero feature row (gather.hip)
        ok = (uint64_t)e < (uint64_t)a.num_vertices;
        v = ok ? (int)e : 0;
        w = a.bary[3 * rr + i];
      }
      rvid[rl * 4 + i] = v;
      rbary[rl * 3 + i] = w;
      rvid[BM * 4 + tid] = ok;
    }
    // extrinsic front-end: thread (ray, coordinate c) forms x_c of its ray (the gather's
    // fma order) into activation buffer 0, unused until phase 1; [BM][4] = x, live
    if (ENC && tid < BM * 3) {
      float* rx = reinterpret_cast<float*>(act);
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int rl = tid / 3, c = tid % 3;
      const int b = b0 + rl;
      float x = 0.f;
      const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src) : -1;
      const bool live = rr >= 0;
      if (live) {
        const int64_t v0 = vid_at(a.vids, a.vid_dtype, 3 * rr), v1 = vid_at(a.vids, a.vid_dtype, 3 * rr + 1),
                      v2 = vid_at(a.vids, a.vid_dtype, 3 * rr + 2);
        const float w0 = a.bary[3 * rr], w1 = a.bary[3 * rr + 1], w2 = a.bary[3 * rr + 2];
        const uint64_t nv = (uint64_t)a.num_vertices;
        if ((uint64_t)v0 < nv && (uint64_t)v1 < nv && (uint64_t)v2 < nv)
          x = fmaf(w2, a.pos[3 * v2 + c], fmaf(w1, a.pos[3 * v1 + c], w0 * a.pos[3 * v0 + c]));
      }
      rx[rl * 4 + c] = x;
      if (c == 0) rx[rl * 4 + 3] = live ? 1.f : 0.f;
    }
    // gather of table columns [col0, col0 + ncols) of the 16 rays into the LDS feature tile,
    // 16-byte chunks (8 columns) per thread: fp32 FMA in the reference order
    // b0 e0 + b1 e1 + b2 e2, rounded to bf16 once (the gather kernel's numerics); every
    // load of a round is issued before any use.  Tables below 4 GiB are read through one
    // buffer descriptor (32-bit unsigned byte offsets); larger ones with 64-bit row
    // addresses (BIGc, a uniform choice per launch).
    // GRc: chunks per thread per round (4: 1024 columns in one round; 2 inside the weight
    // stream of the chunked schedule, where the fragment ring and both accumulator sets
    // are live)
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.table), (short)0, (int)0xFFFFFFFFu, 0x00020000);
    // pre-gathered rows (inf_prefetch_batch): the workgroup's 16 feature rows are one
    // contiguous block of xpre, copied 16 bytes per thread, all loads of a round first
    const __amdgpu_buffer_rsrc_t rxp = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(a.xpre != nullptr ? a.xpre + (int64_t)b0 * k_pad : a.table), (short)0, 0x7FFFFFFF, 0x00020000);
    auto copy_cols = [&](int col0, int ncols) {
      const int cpr = ncols >> 3;
      const int nch = BM * cpr;
      constexpr int GR = 4;
#pragma unroll 1
      for (int q0 = tid; q0 < nch; q0 += C3_CT * GR) {
        u32x4 v[GR];
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          const int r = (q < nch ? q : 0) / cpr, ch = (q < nch ? q : 0) % cpr;
          v[g] = __builtin_amdgcn_raw_buffer_load_b128(rxp, (unsigned)(r * k_pad + col0 + ch * 8) * 2u, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          if (q < nch) {
            const int r = q / cpr, ch = q % cpr;
            *reinterpret_cast<u32x4*>(xs + r * xrow + ((ch ^ (r & 15)) << 4)) = v[g];
          }
        }
      }
    };
    auto gather_cols = [&](auto GRc, auto BIGc, auto NTc, int col0, int ncols) {
      constexpr int GR = decltype(GRc)::value;
      constexpr bool BIG = decltype(BIGc)::value;
      constexpr int CPOL = decltype(NTc)::value ? C3_CPOL_NT : 0;
      if (a.xpre != nullptr) {
        copy_cols(col0, ncols);
        return;
      }
      const int cpr = ncols >> 3;          // chunks per row
      const int nch = BM * cpr;            // chunks of the tile
#pragma unroll 1
      for (int q0 = tid; q0 < nch; q0 += C3_CT * GR) {
        u16x8 ev[GR][3];
        float wv[GR][3];
        int okv[GR];
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          const int r = (q < nch ? q : 0) / cpr, ch = (q < nch ? q : 0) % cpr;
          okv[g] = q < nch ? (rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2]) : 0;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            wv[g][i] = rbary[r * 3 + i];
            if constexpr (BIG) {
              const bf16* src = a.table + (int64_t)rvid[r * 4 + i] * k_pad + col0 + ch * 8;
              ev[g][i] = __builtin_bit_cast(u16x8, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src)));
            } else {
              const unsigned off = ((unsigned)rvid[r * 4 + i] * (unsigned)k_pad + col0 + ch * 8) * 2u;
              ev[g][i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rt, off, 0, CPOL));
            }
          }
        }
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          if (q < nch) {
            const int r = q / cpr, ch = q % cpr;
            u16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = fmaf(wv[g][2], bf_val3(ev[g][2][e]), fmaf(wv[g][1], bf_val3(ev[g][1][e]),
                                                                       wv[g][0] * bf_val3(ev[g][0][e])));
              o[e] = bf_bits3(okv[g] ? x : 0.f);
            }
            *reinterpret_cast<u16x8*>(xs + r * xrow + ((ch ^ (r & 15)) << 4)) = o;
          }
        }
      }
    };
    // X3: the gather from the fp32 table (the split-bf16 mode keeps fp32 eigenfunctions): a
    // thread's 8 columns are two 16-byte loads per corner, x in fp32 in the reference order
    // (b0 e0 + b1 e1 + b2 e2), then hi = bf16(x) into the feature tile and lo = bf16(x - hi)
    // into the lo tile (chainf.hip's split of the same fp32 values)
    const __amdgpu_buffer_rsrc_t rtf = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(X3 ? a.table_f32 : reinterpret_cast<const float*>(a.table)), (short)0, (int)0xFFFFFFFFu,
        0x00020000);
    auto gather_x3 = [&](auto BIGc, int col0, int ncols) {
      constexpr bool BIG = decltype(BIGc)::value;
      constexpr int GR = 2;
      const int cpr = ncols >> 3;
      const int nch = BM * cpr;
#pragma unroll 1
      for (int q0 = tid; q0 < nch; q0 += C3_CT * GR) {
        // (whole vectors bit-cast at the load: a __builtin_bit_cast of one element of a
        // vector with a non-constant subscript reads element 0 -- it takes the operand's
        // address, and a vector element has none)
        f32x4 ev[GR][3][2];
        float wv[GR][3];
        int okv[GR];
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          const int r = (q < nch ? q : 0) / cpr, ch = (q < nch ? q : 0) % cpr;
          okv[g] = q < nch ? (rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2]) : 0;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            wv[g][i] = rbary[r * 3 + i];
            if constexpr (BIG) {
              const float* src = a.table_f32 + (int64_t)rvid[r * 4 + i] * k_pad + col0 + ch * 8;
              ev[g][i][0] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src)));
              ev[g][i][1] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 4)));
            } else {
              const unsigned off = ((unsigned)rvid[r * 4 + i] * (unsigned)k_pad + col0 + ch * 8) * 4u;
              ev[g][i][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtf, off, 0, 0));
              ev[g][i][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtf, off + 16u, 0, 0));
            }
          }
        }
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + C3_CT * g;
          if (q < nch) {
            const int r = q / cpr, ch = q % cpr;
            u32x4 oh, ol;
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              float x[2];
#pragma unroll
              for (int u = 0; u < 2; ++u) {
                const int ee = e + u;
                const float e0 = ev[g][0][ee >> 2][ee & 3];
                const float e1 = ev[g][1][ee >> 2][ee & 3];
                const float e2 = ev[g][2][ee >> 2][ee & 3];
                const float v = fmaf(wv[g][2], e2, fmaf(wv[g][1], e1, wv[g][0] * e0));
                x[u] = okv[g] ? v : 0.f;
              }
              const unsigned w = pack_bf16x2(x[0], x[1]);
              oh[e >> 1] = w;
              ol[e >> 1] = pack_bf16x2(x[0] - __builtin_bit_cast(float, w << 16), x[1] - __builtin_bit_cast(float, w & 0xFFFF0000u));
            }
            char* d = xs + r * xrow + ((ch ^ (r & 15)) << 4);
            *reinterpret_cast<u32x4*>(d) = oh;
            *reinterpret_cast<u32x4*>(d + x_lo) = ol;
          }
        }
      }
    };
    // ZP: the lane's layer-0 pre-activations (its accumulators of phase 0), ahead of the
    // fragment prologue in the in-order vmcnt queue
    f32x4 z0[ZP ? TN : 1];
    if constexpr (ZP) {
      const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.zin), (short)0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        z0[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rz, ((unsigned)(blockIdx.x * (2 * H / 16) + t0 + j) * 64u + lane) * 16u, 0, 0));
      // further k slices (zg.hip), added in order
#pragma unroll 1
      for (int sl = 1; sl < a.zin_parts; ++sl)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          z0[j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rz, ((unsigned)(blockIdx.x * (2 * H / 16) + t0 + j) * 64u + lane) * 16u,
                                                 (int)(sl * a.zin_stride * 4), 0));
    }
    // the first block's fragments, in k order (the loop's waits assume that order); issued
    // after the dependent ray-record loads so those are not queued behind them
    {
      const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(a.blk[0].img);
#pragma unroll
      for (int kb = 0; kb < D; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j) fr[kb][j] = frag(rs0, a.blk[0].kb0 + kb, j);
        if constexpr (X3) {
#pragma unroll
          for (int j = 0; j < TN; ++j) frl[kb][j] = frag(rs0, a.blk[0].kb0 + lo_kb(a.blk[0]) + kb, j);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stamp(3 * nphase + 3);
    lbar();  // barrier R: ray records in LDS

    // ---- gather: the feature tile, 16-byte chunks (8 columns) per thread ---------------
    // fp32 FMA in the reference order b0 e0 + b1 e1 + b2 e2, rounded to bf16 once (the
    // gather kernel's numerics); every load of a round is issued before any use
    if constexpr (ENC) {
      // extrinsic front-end: RFF / FF / xyz columns of the rays' positions x (LDS, above),
      // bitwise gather.hip encode_kernel's values, rounded to bf16.  A thread keeps one
      // 8-column chunk (ch = tid % cpr when cpr divides the thread count) across its rays,
      // so its projection coefficients are loaded once.
      const float* rx = reinterpret_cast<const float*>(act);
      const int cpr = k_pad >> 3;
      const int nch = BM * cpr;
      const int ne = a.enc_ne, ek = a.enc_k;
      const bool rff = a.encoding == INF_ENC_RFF;
      const int ch0 = tid % cpr;
      float pc[8][3];
      auto coef = [&](int ch, float (&pcv)[8][3]) {
#pragma unroll
        for (int e8 = 0; e8 < 8; ++e8) {
          const int c = ch * 8 + e8;
          const int j = c < ne ? c : c - ne;
          const bool t = c < 2 * ne;
          pcv[e8][0] = t ? (rff ? a.enc_proj[j] : a.enc_proj[j % ek]) : 0.f;
          pcv[e8][1] = t && rff ? a.enc_proj[ek + j] : 0.f;
          pcv[e8][2] = t && rff ? a.enc_proj[2 * ek + j] : 0.f;
        }
      };
      coef(ch0, pc);
#pragma unroll 1
      for (int q = tid; q < nch; q += C3_CT) {
        const int r = q / cpr, ch = q % cpr;
        float pq[8][3];
        if (ch != ch0) coef(ch, pq);
        const float x[3] = {rx[r * 4], rx[r * 4 + 1], rx[r * 4 + 2]};
        const bool live = rx[r * 4 + 3] != 0.f;
        const float tp = 6.283185307179586f;
        const float px[3] = {tp * x[0], tp * x[1], tp * x[2]};
        u16x8 o;
#pragma unroll
        for (int e8 = 0; e8 < 8; ++e8) {
          const int c = ch * 8 + e8;
          const float p0 = ch == ch0 ? pc[e8][0] : pq[e8][0];
          const float p1 = ch == ch0 ? pc[e8][1] : pq[e8][1];
          const float p2 = ch == ch0 ? pc[e8][2] : pq[e8][2];
          float v = 0.f;
          if (c < 2 * ne) {
            const int j = c < ne ? c : c - ne;
            const float e = rff ? fmaf(px[2], p2, fmaf(px[1], p1, px[0] * p0)) : pick3(x, j / ek) * p0;
            float sn, cs;
            fast_sincos(e, &sn, &cs);
            v = c < ne ? cs : sn;
          } else if (c < a.enc_in_dim) {
            v = pick3(x, c - 2 * ne);
          }
          o[e8] = bf_bits3(live ? v : 0.f);
        }
        *reinterpret_cast<u16x8*>(xs + r * xrow + ((ch ^ (r & 15)) << 4)) = o;
      }
    } else if constexpr (X3) {
      if (a.table_big) gather_x3(std::true_type{}, 0, k_pad);
      else gather_x3(std::false_type{}, 0, k_pad);
    } else if constexpr (!ZP) {
      const int n0 = XC ? min(C::KC, k_pad) : k_pad;
      if (a.table_big) gather_cols(std::integral_constant<int, 4>{}, std::true_type{}, std::true_type{}, 0, n0);
      else if (a.gather_nt || (XC && NR == 1)) gather_cols(std::integral_constant<int, 4>{}, std::false_type{}, std::true_type{}, 0, n0);
      else gather_cols(std::integral_constant<int, 4>{}, std::false_type{}, std::false_type{}, 0, n0);
    }
    // every load issued so far has landed (the gather's data is in LDS and the fragment
    // prologue was issued before it; vmcnt is in order): an explicit wait here costs
    // nothing and clears the compiler's scoreboard of the gather registers, which it
    // otherwise drains the whole fragment ring for (vmcnt(0)) at every stream block
    // (ZP: no gather; the compiler's counted waits cover Z's loads, the prologue stays in flight)
    if constexpr (!ZP) __builtin_amdgcn_s_waitcnt(0);
    stamp(3 * nphase + 4);
    lbar();  // barrier 0: feature tile in LDS
    stamp(3 * nphase + 5);

    // ReLU bits of the lane's NV accumulator elements for layers 0..L-3 (bit j 4 + r), in
    // registers: 64 / NV layers per word.  Wide tiles (NR > 1): NR NV <= 32 bits per layer
    // (tile n at bit n NV), kept as a stack -- the forward pushes layers 0..L-3 in order
    // and the backward pops them in reverse (dX of layer l masks by Y_{l-1}), so every
    // access is a static register index
    constexpr int MPW = 64 / NV;
    static_assert(2 * MPW >= CHAIN_MAX_HIDDEN - 1, "ReLU bit words");
    unsigned long long mbits[2] = {0ull, 0ull};
    constexpr int MST = NR == 1 ? 1 : CHAIN_MAX_HIDDEN - 1;
    unsigned mst[MST];
#pragma unroll
    for (int i = 0; i < MST; ++i) mst[i] = 0u;
    // B-operand slot offsets of this lane inside a k block of the activation tile (the
    // swizzle repeats every 4 k blocks)
    int aoffs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) aoffs[q] = act_off(q, r16, g4) - q * 1024;
    const char* xlane = xs + r16 * xrow;
    // the lane's accumulator element (j, r) is ray r16 (of each ray tile), feature feat(j) + r
    auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
    // activations / dZ -> the LDS tile: one 16-byte write per k block (tile pair), 8 bytes
    // for a lone tile (H = 128: a wave owns half a k block)
    // (pairs of values through one v_cvt_pk_bf16_f32: the same RNE bits as one at a time)
    auto put_act = [&](const float (&v)[TN][4], char* act) {
      if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int j = 0; j < TN; j += 2) {
          u32x4 w;
          w[0] = pack_bf16x2(v[j][0], v[j][1]);
          w[1] = pack_bf16x2(v[j][2], v[j][3]);
          w[2] = pack_bf16x2(v[j + 1][0], v[j + 1][1]);
          w[3] = pack_bf16x2(v[j + 1][2], v[j + 1][3]);
          *reinterpret_cast<u32x4*>(act + act_off((t0 + j) >> 1, r16, g4)) = w;
        }
      } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          u32x2 w;
          w[0] = pack_bf16x2(v[j][0], v[j][1]);
          w[1] = pack_bf16x2(v[j][2], v[j][3]);
          const int t = t0 + j;
          *reinterpret_cast<u32x2*>(act + act_off(t >> 1, r16, g4) + 8 * (t & 1)) = w;
        }
      }
    };
    // X3: the hi tile as put_act, then lo = v - bf16(v) into the buffer's lo tile
    auto put_act2 = [&](const float (&v)[TN][4], char* act) {
      put_act(v, act);
      if constexpr (X3) {
        float lo[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) lo[j][r] = v[j][r] - __builtin_bit_cast(float, (unsigned)bf_bits3(v[j][r]) << 16);
        put_act(lo, act + C::ACT_LO);
      }
    };
    // the inverse of put_act for this lane's own slots
    auto get_act = [&](float (&v)[TN][4], const char* act) {
      auto unpack = [](unsigned w, float& lo, float& hi) {
        lo = __builtin_bit_cast(float, w << 16);
        hi = __builtin_bit_cast(float, w & 0xFFFF0000u);
      };
      if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int j = 0; j < TN; j += 2) {
          const u32x4 w = *reinterpret_cast<const u32x4*>(act + act_off((t0 + j) >> 1, r16, g4));
          unpack(w[0], v[j][0], v[j][1]);
          unpack(w[1], v[j][2], v[j][3]);
          unpack(w[2], v[j + 1][0], v[j + 1][1]);
          unpack(w[3], v[j + 1][2], v[j + 1][3]);
        }
      } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int t = t0 + j;
          const u32x2 w = *reinterpret_cast<const u32x2*>(act + act_off(t >> 1, r16, g4) + 8 * (t & 1));
          unpack(w[0], v[j][0], v[j][1]);
          unpack(w[1], v[j][2], v[j][3]);
        }
      }
    };
    // sums over the 16 rays of per-lane values v[j][r] -> dst[feature] (lane r16 < NV
    // holds value r16 after the reduce-scatter)
    auto ray_sums_to = [&](const float (&v)[TN][4], float* dst) {
      float t[NV];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[j * 4 + r] = v[j][r];
      const float s = ray_sum<NV>(t, lane);
      const int idx = r16 % NV;
      int fo = feat(idx >> 2) + (idx & 3);
      if constexpr (NR > 1) asm volatile("" : "+v"(fo));  // computed here, not hoisted (and spilled)
      if (r16 < NV) dst[fo] = s;
    };

    // The chunked schedule's second accumulator set (W_y x, phase 0 .. the skip layer):
    // ACCY -- in registers (accy, NR = 1); PARK -- wide tiles, whose NR-fold sets leave no
    // registers for it: during phase 0 the set not being accumulated waits in the lane's
    // own slots of the two activation tiles (unused until phase 0's epilogue; slot (j, n)
    // = tile j, ray tile n, the wave's k block -- exactly the slots the wave's own
    // epilogue writes later), exchanged at every C3F_SWAP block; at the end of phase 0
    // W_y x moves to the feature-tile region (free once every wave and the store wave are
    // past the last chunk: barrier BX) until the skip layer's epilogue reads it back
    constexpr bool ACCY = XC && NR == 1;
    constexpr bool PARK = XC && NR > 1;
    static_assert(!PARK || TN == 2, "wide chunked tiles: one 16-byte slot per ray tile and tile pair");
    auto park_slot = [&](int n, int j) -> char* { return act + j * C::ACT_BYTES + n * C::TILE_BYTES + wc * 1024 + lane * 16; };
    auto wy_slot = [&](int n, int j) -> char* { return xs + ((wc * NR * TN + n * TN + j) * 64 + lane) * 16; };
    f32x4 acc[NR][TN], accy[ACCY ? NR : 1][TN];
#pragma unroll
    for (int n = 0; n < NR; ++n)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < TN; ++j) accy[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PARK) {
#pragma unroll
      for (int n = 0; n < NR; ++n)
#pragma unroll
        for (int j = 0; j < TN; ++j) *reinterpret_cast<f32x4*>(park_slot(n, j)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // epilogue of phase p (after the phase's last stream block)
    auto epilogue = [&](const int p) {
      // ---- epilogue of phase p ---------------------------------------------------------
      stamp(2 + 3 * p);
      // no barrier before the writes: this epilogue's tiles (act (p + 1) & 1, colsum p & 1)
      // were last read in phase p - 1 / copied by the store wave before B2(p - 1)
      char* act_out = act + ((p + 1) & 1) * C::ACT_BYTES;
      float* cs_out = csb + (p & 1) * H;
      if constexpr (PARK) {
        if (p == 0) {
          lbar();  // BX: every wave and the store wave are done with the last feature chunk
#pragma unroll
          for (int n = 0; n < NR; ++n)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              *reinterpret_cast<f32x4*>(wy_slot(n, j)) = *reinterpret_cast<const f32x4*>(park_slot(n, j));
        }
      }
      if (p < nfwd) {
        // forward of layer l: bias (+ Ly.bias at the skip layer) + ReLU -> tile, bits; one
        // ray tile at a time (wide tiles: keeps one tile's activations live, not NR)
        const int l = p;
        const bool skip = l == a.s;
        const bool last = l == L - 2;
        unsigned bits = 0;
        float hq1[TN][4];  // NR = 1: the head's activations stay in registers
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          // + bias (+ the chunked schedule's W_y x and Ly.bias at the skip layer), in the
          // layered GEMM epilogue's order (the bias last: the fp32 sums match it).  Wide
          // chunked tiles read W_y x back from this lane's own LDS slots
          float hq[TN][4];  // bf16-rounded activations as f32
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(vecs + l * H + feat(j));
            f32x4 z = acc[n][j];
            if (skip) {
              const f32x4 yv = *reinterpret_cast<const f32x4*>(vecs + (L - 1) * H + feat(j));
              f32x4 wy = f32x4{0.f, 0.f, 0.f, 0.f};
              if constexpr (ACCY) wy = accy[n][j];
              else if constexpr (PARK) wy = *reinterpret_cast<const f32x4*>(wy_slot(n, j));
              else if constexpr (ZP) {
                wy = *reinterpret_cast<const f32x4*>(xs + ((t0 + j) * 64 + lane) * 16);
                for (int sl = 1; sl < a.zin_parts; ++sl)  // the k slices in order
                  wy += *reinterpret_cast<const f32x4*>(xs + ((sl * (H / 16) + t0 + j) * 64 + lane) * 16);
              }
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float v = z[r];
                if constexpr (XC || ZP) v += wy[r];
                z[r] = (v + bv[r]) + yv[r];
              }
            } else {
              z += bv;
            }
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              if constexpr (X3) {  // fp32 activations: the head reads them, put_act2 splits them
                hq[j][r] = relu1(z[r]);
                hq[j][r + 1] = relu1(z[r + 1]);
                bits |= (hq[j][r] > 0.f ? 1u : 0u) << (n * NV + j * 4 + r);
                bits |= (hq[j][r + 1] > 0.f ? 1u : 0u) << (n * NV + j * 4 + r + 1);
                continue;
              }
              const unsigned w = pack_bf16x2(relu1(z[r]), relu1(z[r + 1]));
              hq[j][r] = __builtin_bit_cast(float, w << 16);
              hq[j][r + 1] = __builtin_bit_cast(float, w & 0xFFFF0000u);
              // h > 0 <=> the bf16 bits without the sign are nonzero (ReLU left no negatives
              // but possibly a -0)
              if constexpr (NR == 1) {
                bits |= ((w & 0x7FFFu) != 0u ? 1u : 0u) << (n * NV + j * 4 + r);
                bits |= ((w & 0x7FFF0000u) != 0u ? 1u : 0u) << (n * NV + j * 4 + r + 1);
              } else {  // v_min_u32 x, 1: the flag in a VGPR (NR TN 8 compares would each
                        // take an SGPR pair, and spill)
                bits |= nz1(w & 0x7FFFu) << (n * NV + j * 4 + r);
                bits |= nz1(w & 0x7FFF0000u) << (n * NV + j * 4 + r + 1);
              }
            }
          }
          if (!last) {
            put_act2(hq, act_out + n * C::TILE_BYTES);
          } else {
            // ---- head on the registers of the last hidden layer (model.py:89-94) --------
            // z partials over this lane's features, then over the 4 row groups (a wave's WN
            // features), then over the waves through LDS
#pragma unroll
            for (int o = 0; o < 3; ++o) {
              float z = 0.f;
#pragma unroll
              for (int j = 0; j < TN; ++j) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(w7s + o * H + feat(j));
#pragma unroll
                for (int r = 0; r < 4; ++r) z = fmaf(hq[j][r], w[r], z);
              }
              z = col_sum4(z);
              if (g4 == 0) zps[(wc * BM + 16 * n + r16) * 3 + o] = z;
            }
            // wide tiles: the activations wait in this lane's own slots of the output tile
            // (bf16, exact: they are bf16-rounded) until the head backward overwrites them
            if constexpr (NR == 1) {
#pragma unroll
              for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) hq1[j][r] = hq[j][r];
            } else {
              put_act(hq, act_out + n * C::TILE_BYTES);
            }
          }
        }
        if (!last) {
          if constexpr (NR == 1) {
            if (l < MPW) mbits[0] |= (unsigned long long)bits << (NV * l);
            else mbits[1] |= (unsigned long long)bits << (NV * (l - MPW));
          } else {
#pragma unroll
            for (int i = MST - 1; i > 0; --i) mst[i] = mst[i - 1];
            mst[0] = bits;
          }
        } else {
          lbar();  // Bh1: per-wave head partial sums complete
          // sigmoid, loss and dL/dz (model.py:89-94, config.py:113-122, trainer.py:76):
          // every compute wave computes all BM x 3 of them (one lane each per 64) into its
          // own copy of dz, so only same-wave LDS ordering is needed, no second barrier
          {
            float* dzw = dzs + wc * BM * 3;
            float lsum = 0.f, ssum = 0.f;
            // (not unrolled: the unrolled copies' LDS addresses were hoisted to the kernel
            // entry and spilled -- a scratch reload drains the fragment queue)
#pragma unroll 1
            for (int e0 = 0; e0 < BM * 3; e0 += 64) {
              const int e = e0 + lane;
              if (e < BM * 3) {
                const int b = b0 + e / 3, o = e % 3;
                float z = w7s[3 * H + o];
#pragma unroll
                for (int w = 0; w < C3_CW; ++w) z += zps[w * BM * 3 + e];
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
                    const float qq = d * d / C3_CAUCHY_C2;
                    lv = C3_CAUCHY_C2 * logf(1.f + qq);
                    g = 2.f * d / (1.f + qq);
                  }
                  dz = (g * a.inv_count) * (1.f - pv) * pv;
                  lsum += lv;
                  ssum += d * d;
                }
                dzw[e] = dz;
                if (wc == 0) preds[e] = pv;
              }
            }
            if (wc == 0) {  // all 64 lanes active for the cross-lane sums
              lsum = col_sum4(row_sum16(lsum));
              ssum = col_sum4(row_sum16(ssum));
              if (lane == 0) {
                lss[0] = lsum;
                lss[1] = ssum;
              }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's dz writes
          }
          // head backward in registers: dZ_{L-2} = (dz W7) * (h > 0), its ray sums, and the
          // output layer's weight-gradient partials sum_rays dz_o * h (the ray tiles summed
          // in registers first: one partial per workgroup)
          float cst[TN][4], hst[3][TN][4], dbs[3];
#pragma unroll
          for (int n = 0; n < NR; ++n) {
            float dzr[3];
#pragma unroll
            for (int o = 0; o < 3; ++o) dzr[o] = dzs[wc * BM * 3 + (16 * n + r16) * 3 + o];
#pragma unroll
            for (int o = 0; o < 3; ++o) dbs[o] = n == 0 ? dzr[o] : dbs[o] + dzr[o];
            float hq[TN][4];
            if constexpr (NR == 1) {
#pragma unroll
              for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) hq[j][r] = hq1[j][r];
            } else {
              get_act(hq, act_out + n * C::TILE_BYTES);
            }
            float gv[TN][4];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const f32x4 w0 = *reinterpret_cast<const f32x4*>(w7s + 0 * H + feat(j));
              const f32x4 w1 = *reinterpret_cast<const f32x4*>(w7s + 1 * H + feat(j));
              const f32x4 w2 = *reinterpret_cast<const f32x4*>(w7s + 2 * H + feat(j));
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float g = fmaf(dzr[2], w2[r], fmaf(dzr[1], w1[r], dzr[0] * w0[r]));
                gv[j][r] = hq[j][r] > 0.f ? g : 0.f;
              }
            }
            put_act2(gv, act_out + n * C::TILE_BYTES);
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                cst[j][r] = n == 0 ? gv[j][r] : cst[j][r] + gv[j][r];
#pragma unroll
                for (int o = 0; o < 3; ++o)
                  hst[o][j][r] = n == 0 ? dzr[o] * hq[j][r] : fmaf(dzr[o], hq[j][r], hst[o][j][r]);
              }
          }
          // the output bias partials (sum over the rays of dz_o): a DPP row sum in wave 0
          // (lane r16 holds ray r16's dz) instead of a 16-deep dependent LDS loop
          if (wc == 0) {
#pragma unroll
            for (int o = 0; o < 3; ++o) {
              const float db = row_sum16(dbs[o]);
              if (lane == 0) hbs[o] = db;
            }
          }
          ray_sums_to(cst, cs_out);
#pragma unroll
          for (int o = 0; o < 3; ++o) ray_sums_to(hst[o], hws + o * H);
        }
      } else {
        // dX of layer l masked by Y_{l-1} > 0 -> dZ_{l-1} (tile, bias partial)
        const int l = (L - 2) - (p - nfwd);
        unsigned bits;
        if constexpr (NR == 1) {
          bits = (unsigned)((l - 1 < MPW ? mbits[0] >> (NV * (l - 1)) : mbits[1] >> (NV * (l - 1 - MPW))) &
                            ((1u << NV) - 1));
        } else {
          bits = mst[0];
#pragma unroll
          for (int i = 0; i + 1 < MST; ++i) mst[i] = mst[i + 1];
        }
        float cst[TN][4];
#pragma unroll
        for (int n = 0; n < NR; ++n) {
          float v[TN][4];
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[j][r] = ((bits >> (n * NV + j * 4 + r)) & 1u) ? acc[n][j][r] : 0.f;
              cst[j][r] = n == 0 ? v[j][r] : cst[j][r] + v[j][r];
            }
          put_act2(v, act_out + n * C::TILE_BYTES);
        }
        ray_sums_to(cst, cs_out);
      }
#pragma unroll
      for (int n = 0; n < NR; ++n)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[n][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      stamp(wave == 0 ? 4 * nphase + 6 + p : 6 * nphase + 6 + p);
      lbar();  // B2: tile of the next phase and this phase's partials complete
      stamp(3 + 3 * p);
    };

    // one block of the weight stream (and the epilogue of the phase it ends)
    auto run_block = [&](int i) {
      const C3Block& B = a.blk[i];
      const C3Block& Bn = a.blk[i + 1 < a.nblk ? i + 1 : i];
      if (i == 0 || a.blk[i - 1].last) stamp(1 + 3 * B.phase);
      // ---- MFMAs of block i; slot kb % D refilled with k-block kb + D of this block or
      // of block i+1 (the last block reloads itself: harmless loads keep waits exact)
      if constexpr (XC) {
        if (B.flags & C3F_GATHER) {
          const int c = B.flags >> C3F_CHUNK_SHIFT;
          lbar();  // G1: every wave is done with the previous chunk (and the store wave with its X^T)
          const int nc = min(C::KC, k_pad - c * C::KC);
          // chunked tiles (k_pad > C3_KC) are the large tables: non-temporal rows (wide
          // tiles: the MALL policy decides, as for the whole-tile gather); one load set
          // per thread in the wide variant (four accumulator sets are live)
#ifndef C3_GRX_WIDE
#define C3_GRX_WIDE 1
#endif
          constexpr int GRX = NR == 1 ? 2 : C3_GRX_WIDE;
#ifdef EXP_NOGATHER
          if (NR > 1) {} else
#endif
          if (a.table_big)
            gather_cols(std::integral_constant<int, GRX>{}, std::true_type{}, std::true_type{}, c * C::KC, nc);
          else if (NR == 1 || a.gather_nt)
            gather_cols(std::integral_constant<int, GRX>{}, std::false_type{}, std::true_type{}, c * C::KC, nc);
          else
            gather_cols(std::integral_constant<int, GRX>{}, std::false_type{}, std::false_type{}, c * C::KC, nc);
          lbar();  // G2: chunk c in LDS
        }
        if (B.flags & C3F_SWAP) {
#pragma unroll
          for (int n = 0; n < NR; ++n)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              if constexpr (PARK) {
                f32x4* q = reinterpret_cast<f32x4*>(park_slot(n, j));
                const f32x4 t = *q;
                *q = acc[n][j];
                acc[n][j] = t;
              } else {
                const f32x4 t = acc[n][j];
                acc[n][j] = accy[n][j];
                accy[n][j] = t;
              }
            }
        }
      }
      const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
      const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
      const bool from_x = B.a_x != 0;
      const char* act_in = act + (B.phase & 1) * C::ACT_BYTES;
      const int ak0 = B.ak0, ckb = B.kb0, nkb = Bn.kb0;
      // B operand: the feature tile (natural k order) or the activation tile.  One base per
      // block and a branch-free per-k-block offset (a select on the uniform source flag):
      // a pointer ternary inside the unrolled loop had compiled to scalar branches between
      // the MFMAs.  X: chunk (m 4 + g4) ^ r16 of row r16 with m = ak0 + kb, and ak0 a
      // multiple of UPL keeps the xor inside the k-block's 32-chunk (UPL = 8) / 16-chunk
      // (UPL = 4) span: xlane + 64 ak0 + ((kb 4 + g4) ^ r16) 16.  Ray tile n: 16 rows of X
      // / one activation tile further
      const int fx = from_x ? 1 : 0;
      const char* bbase = from_x ? xlane + ak0 * 64 : act_in;
      const int nstride = from_x ? 16 * xrow : C::TILE_BYTES;
      auto bread = [&](int kb, int n) -> bf16x8 {
        const int xo = ((kb * 4 + g4) ^ r16) << 4;
        const int ao = kb * 1024 + aoffs[kb & 3];
        return *reinterpret_cast<const bf16x8*>(bbase + n * nstride + ao + fx * (xo - ao));
      };
      if constexpr (X3) {
        // split-bf16: per k block the lo operands too, three MFMAs per tile in gemm.hip's
        // order (lo.hi, hi.lo, hi.hi: the small terms first); both operands read one k block
        // ahead, hi and lo fragments refilled together
        const int lod = from_x ? x_lo : C::ACT_LO;
        const int clo = lo_kb(B), nlo = lo_kb(Bn);
        auto bread_lo = [&](int kb) -> bf16x8 {
          const int xo = ((kb * 4 + g4) ^ r16) << 4;
          const int ao = kb * 1024 + aoffs[kb & 3];
          return *reinterpret_cast<const bf16x8*>(bbase + lod + ao + fx * (xo - ao));
        };
        bf16x8 bq[2], bl[2];
        bq[0] = bread(0, 0);
        bl[0] = bread_lo(0);
#pragma unroll
        for (int kb = 0; kb < UPL; ++kb) {
          if (kb + 1 < UPL) {
            bq[(kb + 1) & 1] = bread(kb + 1, 0);
            bl[(kb + 1) & 1] = bread_lo(kb + 1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
#ifndef X3_DBG_NOLO  // diagnostics: the hi.hi product alone
            acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frl[kb % D][j], bq[kb & 1], acc[0][j], 0, 0, 0);
            acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bl[kb & 1], acc[0][j], 0, 0, 0);
#endif
            acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bq[kb & 1], acc[0][j], 0, 0, 0);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            fr[kb % D][j] = kb + D < UPL ? frag(crs, ckb + kb + D, j) : frag(nrs, nkb + kb + D - UPL, j);
            frl[kb % D][j] = kb + D < UPL ? frag(crs, ckb + clo + kb + D, j) : frag(nrs, nkb + nlo + kb + D - UPL, j);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr (NR == 1) {
        // the B operand of k-block kb + 1 is read ahead of kb's MFMAs (a scheduling barrier
        // keeps the read there: left alone, the scheduler sinks it to its use and the LDS
        // latency is exposed at every k-block, behind only TN MFMAs)
        // (not in the chunked variant: its second accumulator set leaves no room -- it spills)
        constexpr bool BPF = !XC;
        bf16x8 bq[2];
        if constexpr (BPF) bq[0] = bread(0, 0);
#pragma unroll
        for (int kb = 0; kb < UPL; ++kb) {
          if constexpr (BPF) {
            if (kb + 1 < UPL) bq[(kb + 1) & 1] = bread(kb + 1, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
          const bf16x8 bv = BPF ? bq[kb & 1] : bread(kb, 0);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bv, acc[0][j], 0, 0, 0);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            fr[kb % D][j] = kb + D < UPL ? frag(crs, ckb + kb + D, j) : frag(nrs, nkb + kb + D - UPL, j);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        // wide tiles: NR TN MFMAs per k block; ray tile n's operand for k block kb + 1 is
        // read right after its MFMAs of kb (one operand register set, rolling)
#ifdef C3_WIDE_NOBQ
        constexpr bool RB = false;
#else
        constexpr bool RB = true;
#endif
        auto mfma_block = [&](f32x4 (&tgt)[NR][TN]) {
          bf16x8 bq[NR];
          if constexpr (RB) {
#pragma unroll
            for (int n = 0; n < NR; ++n) bq[n] = bread(0, n);
          }
#pragma unroll
          for (int kb = 0; kb < UPL; ++kb) {
#pragma unroll
            for (int n = 0; n < NR; ++n) {
              const bf16x8 bv = RB ? bq[n] : bread(kb, n);
#pragma unroll
              for (int j = 0; j < TN; ++j)
                tgt[n][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bv, tgt[n][j], 0, 0, 0);
              if (RB && kb + 1 < UPL) bq[n] = bread(kb + 1, n);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j)
              fr[kb % D][j] = kb + D < UPL ? frag(crs, ckb + kb + D, j) : frag(nrs, nkb + kb + D - UPL, j);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        mfma_block(acc);
      }
#ifdef C3_STREAM_ONLY  // diagnostics: the weight stream and MFMAs alone (wrong results);
                      // with C3_STREAM_BARRIERS also the two barriers per phase
      if (B.last) {
        stamp(2 + 3 * B.phase);
#ifdef C3_STREAM_BARRIERS
        lbar();
        lbar();
#endif
      }
      return;
#endif
      if (!B.last) return;
      epilogue(B.phase);
    };
    if constexpr (ZP) {
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[0][j] = z0[j];
      stamp(1);
      epilogue(0);
    }
#pragma unroll 1
    for (int i = 0; i < a.nblk; ++i) run_block(i);
#ifdef C3_STREAM_ONLY
    if (acc[0][0][0] == 1234.5f) act[lane] = 1;  // keep the MFMAs (and their loads) alive
#endif
    stamp(2 + 3 * nphase);
    if (stl != nullptr && wave == 0) {
      if (lane == 0) stl[0] = t_entry;
      for (int i = lane; i < 7 * nphase + 6; i += 64) a.stamps[(blockIdx.x == 0 ? 0 : 7 * nphase + 6) + i] = stl[i];
    }
  } else {
    // =========================== store wave ===============================================
#ifdef C3_STORE_PRIO
    __builtin_amdgcn_s_setprio(C3_STORE_PRIO);
#endif
    // per-launch vectors (biases, Ly.bias, W7, b7), loaded while the compute waves gather;
    // written into LDS between barriers R and 0 (the first reader is phase 0's epilogue)
    constexpr int CPL = H / 64;  // one 16-byte (H = 256) / 8-byte (H = 128) load per lane per row
    typedef float rowv __attribute__((ext_vector_type(CPL)));
    {
      rowv tv[CHAIN_MAX_HIDDEN], tyb, tw[3];
      float tb = 0.f;
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) tv[l] = *reinterpret_cast<const rowv*>(a.bias[l] + lane * CPL);
      tyb = *reinterpret_cast<const rowv*>(a.bias_y + lane * CPL);
#pragma unroll
      for (int o = 0; o < 3; ++o) tw[o] = *reinterpret_cast<const rowv*>(a.W7 + o * H + lane * CPL);
      if (lane < 3) tb = a.b7[lane];
      lbar();  // barrier R
#pragma unroll
      for (int l = 0; l < CHAIN_MAX_HIDDEN; ++l)
        if (l < L - 1) *reinterpret_cast<rowv*>(vecs + l * H + lane * CPL) = tv[l];
      *reinterpret_cast<rowv*>(vecs + (L - 1) * H + lane * CPL) = tyb;
#pragma unroll
      for (int o = 0; o < 3; ++o) *reinterpret_cast<rowv*>(w7s + o * H + lane * CPL) = tw[o];
      if (lane < 3) w7s[3 * H + lane] = tb;
    }
    // ZP: the workgroup's W_y x tiles (H / 16 KiB) into the idle feature-tile region, lane-
    // linear (1 KiB per 16-feature tile: the compute lanes' accumulator slots); landed before
    // B2(0), read in the skip layer's epilogue (phase s >= 1)
    if constexpr (ZP) {
      const char* zy = reinterpret_cast<const char*>(a.zin) + ((int64_t)blockIdx.x * (2 * H / 16) + H / 16) * 1024 + lane * 16;
#pragma unroll 1
      for (int sl = 0; sl < a.zin_parts; ++sl)  // slice sl at H / 16 KiB steps
#pragma unroll
        for (int t = 0; t < H / 16; ++t)
          __builtin_amdgcn_global_load_lds(zy + (int64_t)sl * a.zin_stride * 4 + t * 1024,
                                           (__attribute__((address_space(3))) void*)(xs + (sl * (H / 16) + t) * 1024), 16, 0, 0);
    }
    lbar();  // barrier 0: feature tile in LDS
    if (a.count_step && blockIdx.x == 0 && lane == 0) a.ctrl->step += 1;
    // targets: the replayed batch index, the ray index, the colour -- dependent loads,
    // kept behind barrier 0 (the head is phases away)
    {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
#pragma unroll
      for (int e0 = 0; e0 < BM * 3; e0 += 64) {
        const int e = e0 + lane;
        const int bt = b0 + e / 3;
        float tt = 0.f;
        const int64_t trow =
            e < BM * 3 && bt < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, bt, a.num_rays, a.num_src) : -1;
        if (trow >= 0) tt = a.rgb[trow * 3 + e % 3];
        if (e < BM * 3) tgs[e] = tt;
      }
    }
    // ---- fragment images for the dW GEMM (lgemm.hpp: rows = features, k = rays) ----------
    // A 16-ray tile at b0n = b0 + 16 n is half (b0n / 16) % 2 of k block b0n / 32: per 16-feature
    // tile t one 512-byte piece, lane slot i + 16 rh = feature 16 t + i, rays 8 rh .. 8 rh + 7.
    // One store instruction writes the pieces of tiles 2 s and 2 s + 1 (2 x 512 contiguous
    // bytes, whole lines); the feature-major transpose comes from ds_read_b64_tr_b16: a
    // 16-lane group reads 4 rays x 16 features, lane 4 q + p giving ray q's features
    // 4 p .. 4 p + 3, and lane i receives feature i of the 4 rays.
    const int tg = lane >> 4;                 // 16-lane group: (tile 2 s + tg / 2, rays 8 (tg % 2) ..)
    const int ti = lane & 15;                 // slot in the piece = feature within the tile
    const int tq = ti >> 2, tp = ti & 3;      // this lane's address: ray row tq, feature quad tp
    const int trh = tg & 1;
    const int64_t lane_off = (int64_t)(ti + 16 * trh) * 16;
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    auto tr_read = [&](const char* p8) -> s16x4 {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p8));
    };
    // tiles: R / 16 of an image with R rows; addr(t, n, ray, quad) -> the 8-byte LDS address
    // of features 16 t + 4 quad .. + 3 of `ray` of ray tile n
    auto copy_image = [&](auto addr, int R, bf16* img, int s_begin, int s_end, int n) {
      const int b0n = b0 + 16 * n;
      char* d = reinterpret_cast<char*>(img) + (int64_t)(b0n >> 5) * (R / 16) * 1024 + ((b0n >> 4) & 1) * 512 + lane_off;
      // batches of 4 instructions: all 8 transposing reads issued before the first store
      // waits on them (counted lgkmcnt), so LDS latency is paid once per batch
      constexpr int NB = 4;
#pragma unroll 1
      for (int s0 = s_begin; s0 < s_end; s0 += NB) {
        s16x4 lo[NB], hi[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int t = 2 * min(s0 + u, s_end - 1) + (tg >> 1);
          lo[u] = tr_read(addr(t, n, 8 * trh + tq, tp));
          hi[u] = tr_read(addr(t, n, 8 * trh + 4 + tq, tp));
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (s0 + u < s_end) {
            const int t = 2 * (s0 + u) + (tg >> 1);
            const s16x4x8 o = {lo[u][0], lo[u][1], lo[u][2], lo[u][3], hi[u][0], hi[u][1], hi[u][2], hi[u][3]};
            // write-through (sc1): the dW GEMM reads these images in the next launch, and
            // lines left dirty in the XCD L2s are written back at the kernel boundary
            // (measured -0.8 us per step against plain stores; profiles/r02/sweeps/chain_images_sc1.log)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4, o), __builtin_amdgcn_make_buffer_rsrc(img, (short)0, 0x7FFFFFFF, 0x00020000),
                (unsigned)(d - reinterpret_cast<char*>(img) + (int64_t)t * 1024), 0, 16);
          }
        }
      }
    };
    int x_tile0 = 0;  // first 16-feature tile held in LDS (chunked tile)
    auto x_addr = [&](int t, int n, int r, int q) -> const char* {
      return xs + (16 * n + r) * xrow + (((2 * (t - x_tile0) + (q >> 1)) ^ (r & 15)) << 4) + 8 * (q & 1);
    };
    // every ray tile's piece of an image
    auto copy_tiles = [&](auto addr, int R, bf16* img, int s_begin, int s_end) {
#pragma unroll 1
      for (int n = 0; n < NR; ++n) copy_image(addr, R, img, s_begin, s_end, n);
    };
    // X3: the lo tile (lo_delta bytes from the hi one) into the lo image, R x rows after
    // the hi one (lgemm SPLIT's operand pair)
    auto copy_tiles2 = [&](auto addr, int lo_delta, int R, bf16* img, int s_begin, int s_end) {
      copy_tiles(addr, R, img, s_begin, s_end);
      if constexpr (X3) {
        auto lo_addr = [&](int t, int n, int r, int q) -> const char* { return addr(t, n, r, q) + lo_delta; };
        copy_tiles(lo_addr, R, img + (int64_t)R * a.rows, s_begin, s_end);
      }
    };
    // X^T for the dW GEMMs of layer 0 and Ly, copied while the compute waves stream the
    // long input-layer phases (W_0: phase 0, W_y: the skip phase s), half in each
    const int xs_total = k_pad / 32;
    const int xs_mid = XC ? xs_total : (a.s >= 1 ? xs_total / 2 : xs_total);
    if constexpr (XC) {
      // chunked tile: X^T of chunk c between barriers G2(c) and G1(c + 1) (x_tile0 shifts
      // the image's tile index to the chunk's LDS columns)
      for (int c = 0; c < a.nchunk; ++c) {
        if (c > 0) {
          lbar();  // G1(c)
          lbar();  // G2(c)
        }
        x_tile0 = c * (C::KC / 16);
        copy_tiles(x_addr, k_pad, a.XT, c * (C::KC / 32), min((c + 1) * C::KC, k_pad) / 32);
      }
      if (NR > 1) lbar();  // BX: the feature-tile region takes the parked W_y x
    } else if constexpr (!ZP) {
      copy_tiles2(x_addr, x_lo, k_pad, a.XT, 0, xs_mid);
    }
    if constexpr (ZP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // W_y x landed before B2(0)
    auto copy_out = [&](const char* src, void* dst, int bytes) {
      char* d = reinterpret_cast<char*>(dst);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, 0x7FFFFFFF, 0x00020000);
      for (int c = lane * 16; c < bytes; c += 64 * 16)
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(src + c), rd, (unsigned)c, 0, 16);
    };
#ifdef C3_STREAM_ONLY
#ifdef C3_STREAM_BARRIERS
    for (int p = 0; p < nphase; ++p) {
      lbar();
      lbar();
    }
#endif
    return;
#endif
#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      stamp(5 * nphase + 6 + p);
      const bool head_phase = p == nfwd - 1;
      if (head_phase) lbar();  // Bh1
      lbar();  // B2
      // phase p's outputs: act tile (p + 1) & 1, colsum p & 1 -- to be copied before B2(p + 1)
      const char* act_p = act + ((p + 1) & 1) * C::ACT_BYTES;
      auto act_addr = [&](int t, int n, int r, int q) -> const char* {
        return act_p + n * C::TILE_BYTES + act_off(t >> 1, r, q) + 8 * (t & 1);
      };
      const char* cs = reinterpret_cast<const char*>(csb + (p & 1) * H);
      // one partial per workgroup (Bp / BM of them: refresh_tables)
      const int64_t part0 = blockIdx.x;
      if (p < nfwd) {
        const int l = p;
        if (!head_phase) copy_tiles2(act_addr, C::ACT_LO, H, a.YT[l], 0, H / 32);
        if (!XC && !ZP && p == a.s - 1) copy_tiles2(x_addr, x_lo, k_pad, a.XT, xs_mid, xs_total);
        if (head_phase) {
          copy_tiles2(act_addr, C::ACT_LO, H, a.dZT[L - 2], 0, H / 32);
          copy_out(cs, a.colsum[L - 2] + part0 * H, H * 4);
          copy_out(reinterpret_cast<const char*>(hws), a.hw_part + part0 * 3 * H, 3 * H * 4);
          if (lane < 3) a.hb_part[part0 * 3 + lane] = hbs[lane];
          if (lane < 2 && a.loss_part != nullptr) a.loss_part[2 * part0 + lane] = lss[lane];
          if (a.pred != nullptr)
            for (int c = lane; c < BM * 3; c += 64)
              if (b0 + c / 3 < a.batch) a.pred[(int64_t)b0 * 3 + c] = preds[c];
        }
      } else {
        const int l = (L - 2) - (p - nfwd);
        copy_tiles2(act_addr, C::ACT_LO, H, a.dZT[l - 1], 0, H / 32);
        copy_out(cs, a.colsum[l - 1] + part0 * H, H * 4);
      }
    }
  }
}

template <int H, int LOSS, bool ENC, bool XC, int NR, bool ZP = false, bool X3 = false>
int launch3_enc(const Chain3Args& a, hipStream_t stream) {
  using C = L3<H, NR, X3>;
  const int lds = C::lds_bytes(a.L, ZP ? a.zin_parts * 2 * H : a.kc, XC);
  INF_CHECK_ARG(lds <= C3_LDS_CAP, "chain3: LDS budget exceeded for this depth / feature width");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chain3_kernel<H, LOSS, ENC, XC, NR, ZP, X3>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  chain3_kernel<H, LOSS, ENC, XC, NR, ZP, X3><<<dim3((unsigned)(a.rows / C::BM)), dim3(C3_THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

template <int H, int LOSS>
int launch3_loss(const Chain3Args& a, int bm, hipStream_t stream) {
  if (bm != C3BM) {
    if constexpr (H == 256) {  // chain3_supported: chunked wide tiles need H = 256
      if (a.kc < a.k_pad) return launch3_enc<H, LOSS, false, true, C3_NR_WIDE>(a, stream);
    }
    INF_CHECK_ARG(a.kc == a.k_pad, "chain3: chunked wide tiles need H = 256");
    return launch3_enc<H, LOSS, false, false, C3_NR_WIDE>(a, stream);
  }
  if (a.x3) {
    INF_CHECK_ARG(a.kc == a.k_pad && a.encoding == INF_ENC_NONE && a.zin == nullptr && a.xpre == nullptr,
                  "chain3: the split-bf16 chain is the whole-tile eigenfunction schedule");
    return launch3_enc<H, LOSS, false, false, 1, false, true>(a, stream);
  }
  if (a.zin != nullptr) return launch3_enc<H, LOSS, false, false, 1, true>(a, stream);
  if (a.encoding != INF_ENC_NONE) return launch3_enc<H, LOSS, true, false, 1>(a, stream);
  if (a.kc < a.k_pad) return launch3_enc<H, LOSS, false, true, 1>(a, stream);
  return launch3_enc<H, LOSS, false, false, 1>(a, stream);
}

// the loss is a template parameter: one branch-free head per loss type keeps the compute
// waves inside their VGPR budget (a spill would drain the weight queue)
template <int H>
int launch3_typed(const Chain3Args& a, int bm, hipStream_t stream) {
  if (a.loss == INF_LOSS_L2) return launch3_loss<H, INF_LOSS_L2>(a, bm, stream);
  if (a.loss == INF_LOSS_L1) return launch3_loss<H, INF_LOSS_L1>(a, bm, stream);
  return launch3_loss<H, INF_LOSS_CAUCHY>(a, bm, stream);
}

}  // namespace

bool chain3_x3_lds_fits(int H, int L, int k_pad) {
  if ((H != 128 && H != 256) || k_pad > C3_KC) return false;
  const int lds = H == 256 ? L3<256, 1, true>::lds_bytes(L, k_pad, false) : L3<128, 1, true>::lds_bytes(L, k_pad, false);
  return lds <= C3_LDS_CAP;
}

bool chain3_lds_fits(int H, int L, int k_pad, int64_t rows) {
  if (H != 128 && H != 256) return false;
  const int kc = chain3_kc(k_pad, rows);
  const bool xc = kc < k_pad;
  int lds;
  if (chain3_bm(rows) == C3BM) lds = H == 256 ? L3<256, 1>::lds_bytes(L, kc, xc) : L3<128, 1>::lds_bytes(L, kc, xc);
  else lds = H == 256 ? L3<256, C3_NR_WIDE>::lds_bytes(L, kc, xc) : L3<128, C3_NR_WIDE>::lds_bytes(L, kc, xc);
  return lds <= C3_LDS_CAP;
}

int launch_chain3(const Chain3Args& a_in, int bm, hipStream_t stream) {
  Chain3Args a = a_in;
  a.table_big = a.encoding == INF_ENC_NONE && a.num_vertices * (int64_t)a.k_pad * (a.x3 ? 4 : 2) >= ((int64_t)1 << 32);
  a.gather_nt = a.encoding == INF_ENC_NONE && (size_t)a.num_vertices * (size_t)a.k_pad * 2 > C3_NT_TABLE_BYTES;
  INF_CHECK_ARG(chain3_supported(a.H, a.L, a.k_pad, a.rows), "chain3: unsupported shape");
  INF_CHECK_ARG(bm == chain3_bm(a.rows), "chain3: tile height");
  INF_CHECK_ARG(bm == C3BM || (a.encoding == INF_ENC_NONE && a.xpre == nullptr), "chain3: wide tiles gather tables only");
  INF_CHECK_ARG(a.rows % bm == 0 && a.rows >= bm, "chain3: rows must be a multiple of the tile height");
  INF_CHECK_ARG(a.nphase == 2 * a.L - 3, "chain3: phases");
  // precomputed input layers: the narrow schedule, W_y x (zin_parts k slices) staged in
  // the feature-tile region
  INF_CHECK_ARG(a.zin == nullptr || (bm == C3BM && a.encoding == INF_ENC_NONE && a.xpre == nullptr &&
                                     a.zin_parts >= 1 && a.zin_parts <= 8 && a.k_pad >= 2 * a.H),
                "chain3: precomputed input layers need the narrow schedule");
  INF_CHECK_ARG(a.nblk >= 1 && a.nblk <= C3_MAX_BLOCKS, "chain3: weight-stream blocks");
  INF_CHECK_ARG(!a.x3 || (bm == C3BM && a.table_f32 != nullptr && chain3_x3_lds_fits(a.H, a.L, a.k_pad)),
                "chain3: split-bf16 chain: 16-ray tiles over an fp32 table");
  INF_CHECK_ARG(a.rgb != nullptr && (a.encoding != INF_ENC_NONE ? a.pos != nullptr : (a.table != nullptr || a.x3)) &&
                    a.vids != nullptr && a.bary != nullptr && a.XT != nullptr,
                "chain3: inputs");
  INF_CHECK_ARG(a.encoding == INF_ENC_NONE || a.encoding == INF_ENC_XYZ || a.enc_proj != nullptr,
                "chain3: encoding projection missing");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "chain3: vertex id dtype");
  INF_CHECK_ARG(a.kc == chain3_kc(a.k_pad, a.rows) && a.nchunk == ceil_div(a.k_pad, a.kc) &&
                    (a.kc == a.k_pad || a.encoding == INF_ENC_NONE),
                "chain3: feature chunking");
  for (int i = 0; i < a.nblk; ++i) INF_CHECK_ARG(a.blk[i].img != nullptr, "chain3: weight image missing");
  // bias / output-layer rows are read as H/64-float vectors per lane
  for (int l = 0; l < a.L - 1; ++l) INF_CHECK_ARG((uintptr_t)a.bias[l] % 16 == 0, "chain3: bias alignment");
  INF_CHECK_ARG((uintptr_t)a.bias_y % 16 == 0 && (uintptr_t)a.W7 % 16 == 0, "chain3: vector alignment");
  if (a.H == 256) return launch3_typed<256>(a, bm, stream);
  return launch3_typed<128>(a, bm, stream);
}

}  // namespace inf
