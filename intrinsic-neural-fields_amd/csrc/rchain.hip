// Register-streamed forward-only chain: the render slice (renderer.py:112-146) and the
// no-grad forward (model.py:98-112) of bf16 batches.
//
// One workgroup of 8 waves owns RC_BM = 64 rays (four 16-ray MFMA tiles) and runs, in ONE
// launch: the barycentric gather of its rays' table rows (mesh.py:313-324) into LDS, every
// forward layer (the skip layer's Ly over the features, layers.py:60-62), the sigmoid head
// (model.py:89-94) and the placement of each colour into the image (renderer.py:132-141:
// img[hit_ray_idxs] = pred, un-masked through the object mask's pixel list) or pred.
//
// Why this shape.  A forward pass streams the whole forward weight set (W_0, the hidden
// layers, W_y: 1.8 MB bf16 at k = 1024, 8 x 256) from L2 into every workgroup; the bytes
// each workgroup moves are fixed, so the rays per workgroup set the L2 -> CU traffic of a
// frame.  Weights are the MFMA A operand, loaded in fragment order (adam.hip fragment
// images, the training chain's own) straight into a D-deep register ring, and each
// fragment feeds RC_RT = 4 MFMAs (one per ray tile): 4x the reuse of the 16-ray training
// chain at the same ring depth.  The 64 x k feature tile does not fit next to two
// activation tiles, so it is gathered in RC_KC-column chunks and BOTH input layers stream
// over each chunk while it is resident -- W_y x is independent of h, so it accumulates in
// a second register set (accy) and joins the skip layer's epilogue (chain3.hip's chunked
// schedule).  Consecutive ray tiles go to one XCD (render hits are in pixel order, so
// their table rows repeat across neighbouring tiles and stay in that XCD's L2).
#include <cstdlib>

#include "c3common.hpp"
#include "rchain.hpp"

namespace inf {
namespace {

using namespace c3;

// fragment ring depth: the block time does not move between 4 and 8 (tools/rchain_timing.py:
// the loop is bound by its MFMA + LDS issue, not by loads in flight), and 4 leaves the
// registers for the next k-block's B operands
#ifndef RC_DEPTH
#define RC_DEPTH 4
#endif

// CW waves per workgroup, RT 16-ray tiles: <8, 4> one 147 KB workgroup per CU (4 MFMAs
// per fragment); <4, 2> two 72 KB workgroups per CU, so one gathers while the other streams
template <int H, int CW, int RT_>
struct LR {
  static constexpr int RT = RT_, BM = 16 * RT_, THREADS = CW * 64;
  static constexpr int TN = H / (16 * CW);  // 16-feature tiles per wave
  static constexpr int UPL = H / 32;           // 32-deep k blocks per stream block
  static constexpr int NT = H / 16;            // 16-row tiles per k block of a weight image
  static constexpr int ACT_T = 16 * H * 2;     // one ray tile of activations
  static constexpr int ACT_BYTES = RT * ACT_T;
  static constexpr int OFF_ACT = 0;                            // [2][RT] activation tiles
  static constexpr int OFF_X = 2 * ACT_BYTES;                  // [BM][RC_KC] bf16 feature chunk
  static constexpr int OFF_RAY = OFF_X + BM * RC_KC * 2;       // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RB = OFF_RAY + BM * 16 + BM * 12;   // [BM][3] barycentrics
  static constexpr int OFF_ZP = OFF_RB + BM * 12;              // [waves][BM][3] head partial sums
  static constexpr int OFF_W7 = OFF_ZP + CW * BM * 12;         // [3][H], b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;      // biases [L-1][H], Ly.bias [H]
  static int lds_bytes(int L) { return OFF_VEC + L * H * 4; }
  static_assert(OFF_RAY % 16 == 0 && OFF_W7 % 16 == 0 && OFF_VEC % 16 == 0, "LDS alignment");
};

template <int H, int CW, int RT_>
__global__ __launch_bounds__(CW * 64) void rchain_kernel(const RchainArgs a) {
  using C = LR<H, CW, RT_>;
  constexpr int RC_THREADS = C::THREADS;
  constexpr int RT = C::RT, BM = C::BM, TN = C::TN, UPL = C::UPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L, k_pad = a.k_pad;
  char* act = smem + C::OFF_ACT;
  char* xs = smem + C::OFF_X;
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RB);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  constexpr int xrow = RC_KC * 2;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  // XCD-aware tile order: the dispatcher deals workgroups round-robin to the 8 XCDs, so
  // workgroup i runs on XCD i % 8; give XCD x a contiguous run of ray tiles
  const int nb = gridDim.x, bid = blockIdx.x;
  const int xq = nb / 8, xr = nb % 8, xcd = bid % 8;
  const int tile = xcd * xq + min(xcd, xr) + bid / 8;
  const int b0 = tile * BM;
  unsigned long long* stl = nullptr;
  if (a.stamps != nullptr && tid == 0 && (bid == 0 || bid == nb / 2)) stl = a.stamps + (bid == 0 ? 0 : RC_STAMPS);
  auto stamp = [&](int i) {
    if (stl != nullptr) {
      __builtin_amdgcn_sched_barrier(0);
      stl[i] = wall_clock64();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  stamp(0);

  // ---- ray records and the per-launch vectors --------------------------------------------
  if (tid < BM * 3) {
    const int rl = tid / 3, i = tid % 3;
    const int b = b0 + rl;
    int v = 0, ok = 0;
    float w = 0.f;
    const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, a.idx_offset, b, a.num_rays, a.num_src) : -1;
    if (rr >= 0) {
      const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
      ok = (uint64_t)e < (uint64_t)a.num_vertices;  // out-of-range ids read as zero rows (gather.hip)
      v = ok ? (int)e : 0;
      w = a.bary[3 * rr + i];
    }
    rvid[rl * 4 + i] = v;
    rbary[rl * 3 + i] = w;
    rvid[BM * 4 + tid] = ok;
  }
  for (int i = tid; i < (L - 1) * H; i += RC_THREADS) vecs[i] = a.bias[i / H][i % H];
  for (int i = tid; i < H; i += RC_THREADS) vecs[(L - 1) * H + i] = a.bias_y[i];
  for (int i = tid; i < 3 * H + 3; i += RC_THREADS) w7s[i] = i < 3 * H ? a.W7[i] : a.b7[i - 3 * H];

  // ---- weight fragments: buffer descriptor per image, k-block offset in soffset --------
  const int t0 = wc * TN;  // the wave's first 16-feature tile
  constexpr int D = RC_DEPTH < UPL ? RC_DEPTH : UPL;
  bf16x8 fr[D][TN];
  const unsigned lane_off = (unsigned)(t0 * 64 + lane) * 16u;
  auto rsrc_of = [&](const bf16* img) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
  };
  auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j) -> bf16x8 {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 1024, kb * C::NT * 1024, 0);
    return __builtin_bit_cast(bf16x8, v);
  };
  {
    const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(a.blk[0].img);
#pragma unroll
    for (int kb = 0; kb < D; ++kb) {
#pragma unroll
      for (int j = 0; j < TN; ++j) fr[kb][j] = frag(rs0, a.blk[0].kb0 + kb, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  lbar();  // ray records, vectors in LDS
  stamp(1);

  // ---- gather of columns [col0, col0 + ncols) of the BM rays into the feature chunk ----
  // (fp32 FMA in the reference order, one bf16 rounding: chain3.hip / gather.hip numerics)
  const __amdgpu_buffer_rsrc_t rt_tab =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.table), (short)0, (int)0xFFFFFFFFu, 0x00020000);
  auto gather_cols = [&](auto BIGc, int col0, int ncols) {
    constexpr bool BIG = decltype(BIGc)::value;
    constexpr int GR = 4;
    const int cpr = ncols >> 3;
    const int nch = BM * cpr;
#pragma unroll 1
    for (int q0 = tid; q0 < nch; q0 += RC_THREADS * GR) {
      u16x8 ev[GR][3];
      float wv[GR][3];
      int okv[GR];
#pragma unroll
      for (int g = 0; g < GR; ++g) {
        const int q = q0 + RC_THREADS * g;
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
            ev[g][i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rt_tab, off, 0, 0));
          }
        }
      }
#pragma unroll
      for (int g = 0; g < GR; ++g) {
        const int q = q0 + RC_THREADS * g;
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
  auto gather_chunk = [&](int c) {
    const int n = min(RC_KC, k_pad - c * RC_KC);
    if (a.table_big) gather_cols(std::true_type{}, c * RC_KC, n);
    else gather_cols(std::false_type{}, c * RC_KC, n);
  };
  gather_chunk(0);
  lbar();  // chunk 0 in LDS
  stamp(2);

  int aoffs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) aoffs[q] = act_off(q, r16, g4) - q * 1024;
  auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
  f32x4 acc[RT][TN], accy[RT][TN];
  // start value of layer l's accumulators: its bias (+ Ly.bias at the skip layer), so the
  // epilogue is ReLU + packing (accy, W_y x of the input phase, starts at zero)
  auto init_acc = [&](int l) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 bb = *reinterpret_cast<const f32x4*>(vecs + l * H + feat(j));
      if (l == a.s) bb += *reinterpret_cast<const f32x4*>(vecs + (L - 1) * H + feat(j));
#pragma unroll
      for (int t = 0; t < RT; ++t) acc[t][j] = bb;
    }
  };
  init_acc(0);
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int j = 0; j < TN; ++j) accy[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};


#pragma unroll 1
  for (int i = 0; i < a.nblk; ++i) {
    const C3Block& B = a.blk[i];
    const C3Block& Bn = a.blk[i + 1 < a.nblk ? i + 1 : i];
    stamp(3 + i);
    if (B.flags & C3F_GATHER) {
      lbar();  // every wave is done with the previous chunk
      gather_chunk(B.flags >> C3F_CHUNK_SHIFT);
      lbar();  // the chunk is in LDS
    }
    if (B.flags & C3F_SWAP) {
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const f32x4 tmp = acc[t][j];
          acc[t][j] = accy[t][j];
          accy[t][j] = tmp;
        }
    }
    const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
    const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
    const bool from_x = B.a_x != 0;
    const char* act_in = act + (B.phase & 1) * C::ACT_BYTES;
    const int ak0 = B.ak0, ckb = B.kb0, nkb = Bn.kb0;
    // the k-blocks of this stream block, B operands from the feature chunk (X) or the
    // activation tile: two straight-line copies of the unrolled loop (a uniform branch
    // outside it), the B operands of k-block kb + 1 read before the MFMAs of kb so their
    // LDS latency hides under them
    auto run_block = [&](auto FROMXc) {
      constexpr bool FROMX = decltype(FROMXc)::value;
      auto read_b = [&](int kb, bf16x8 (&bv)[RT]) {
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          const char* bp;
          if constexpr (FROMX) bp = xs + (t * 16 + r16) * xrow + ((((ak0 + kb) * 4 + g4) ^ r16) << 4);
          else bp = act_in + t * C::ACT_T + kb * 1024 + aoffs[kb & 3];
          bv[t] = *reinterpret_cast<const bf16x8*>(bp);
        }
      };
      bf16x8 bq[2][RT];
      read_b(0, bq[0]);
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
        if (kb + 1 < UPL) read_b(kb + 1, bq[(kb + 1) & 1]);
        // issue them ahead of this k-block's MFMAs (the scheduler otherwise sinks the reads to
        // just before their first use, one MFMA ahead, exposing the LDS latency every k-block)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int t = 0; t < RT; ++t)
            acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kb % D][j], bq[kb & 1][t], acc[t][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fr[kb % D][j] = kb + D < UPL ? frag(crs, ckb + kb + D, j) : frag(nrs, nkb + kb + D - UPL, j);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (from_x) run_block(std::true_type{});
    else run_block(std::false_type{});
    if (!B.last) continue;

    // ---- epilogue of layer l = phase (its accumulators started from the biases; W_y x
    // joins at the skip layer): ReLU -> bf16 -> the next activation tile, or the head
    const int l = B.phase;
    if (l == a.s)
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[t][j] += accy[t][j];
    if (l < L - 2) {
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
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            u32x2 w;
            w[0] = pack_bf16x2(relu1(acc[t][j][0]), relu1(acc[t][j][1]));
            w[1] = pack_bf16x2(relu1(acc[t][j][2]), relu1(acc[t][j][3]));
            const int tt = t0 + j;
            *reinterpret_cast<u32x2*>(dst + act_off(tt >> 1, r16, g4) + 8 * (tt & 1)) = w;
          }
        }
      }
      init_acc(l + 1);
    } else {
      // head partials over this lane's features (model.py:89-94), then the row groups
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
    }
    lbar();  // the next layer's tile (or the head partials) complete
  }

  stamp(3 + a.nblk);
  // ---- sigmoid head and placement (renderer.py:132-141) -----------------------------------
  if (tid < BM * 3) {
    const int ray = tid / 3, o = tid % 3;
    const int b = b0 + ray;
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

template <int H, int CW, int RT_>
int launch_typed(const RchainArgs& a_in, hipStream_t stream) {
  using C = LR<H, CW, RT_>;
  RchainArgs a = a_in;
  a.table_big = a.num_vertices * (int64_t)a.k_pad * 2 >= ((int64_t)1 << 32);
  const int lds = C::lds_bytes(a.L);
  INF_CHECK_ARG(lds <= 160 * 1024, "rchain: LDS budget exceeded");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)rchain_kernel<H, CW, RT_>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  const int64_t grid = ceil_div(a.batch, C::BM);
  rchain_kernel<H, CW, RT_><<<dim3((unsigned)grid), dim3(C::THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_rchain(const RchainArgs& a, hipStream_t stream) {
  if (a.projected) return launch_rproj(a, stream);
  INF_CHECK_ARG(rchain_supported(a.H, a.L, a.k_pad), "rchain: unsupported shape");
  INF_CHECK_ARG(a.batch >= 1, "rchain: empty batch");
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr, "rchain: inputs");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "rchain: vertex id dtype");
  INF_CHECK_ARG(a.nblk >= 1 && a.nblk <= RC_MAX_BLOCKS && a.nphase == a.L - 1, "rchain: weight stream");
  INF_CHECK_ARG(a.nchunk == ceil_div(a.k_pad, RC_KC), "rchain: feature chunking");
  INF_CHECK_ARG(a.pred != nullptr || (a.img != nullptr && a.hit != nullptr), "rchain: no output");
  for (int i = 0; i < a.nblk; ++i) INF_CHECK_ARG(a.blk[i].img != nullptr, "rchain: weight image missing");
  // INF_RCHAIN_CFG=84 / 42: <8 waves, 4 ray tiles> / <4 waves, 2 ray tiles>
  static const int cfg = [] {
    const char* e = std::getenv("INF_RCHAIN_CFG");
    return e != nullptr ? std::atoi(e) : 84;
  }();
  if (a.H == 256) return cfg == 42 ? launch_typed<256, 4, 2>(a, stream) : launch_typed<256, 8, 4>(a, stream);
  return cfg == 42 ? launch_typed<128, 4, 2>(a, stream) : launch_typed<128, 8, 4>(a, stream);
}

}  // namespace inf
