// Fused fp32 training chain: the parity mode's (INF_MODE_FP32) training step up to the
// weight gradients, in ONE launch per batch -- chain3.hip's structure with exact-f32
// arithmetic (v_mfma_f32_16x16x4_f32, fp32 activations and features; no bf16 rounding
// anywhere), replacing the layered path's gather + 7 forward GEMMs + head + 6 dX GEMMs.
//
// One workgroup owns 16 rays and runs
//   gather    X[b] = b0 E[v0] + b1 E[v1] + b2 E[v2] (fp32 FMA in gather.hip's order) for
//             its rays r = ray_idx[offset + b] (mesh.py:313-324, ray_dataloader.py:122-129),
//   forward   layers 0..L-2 (model.py:98-112), the skip layer (layers.py:60-62) as two K
//             segments [h | x] into one accumulator, bias added last (the layered GEMM's
//             epilogue order),
//   head      Linear(H,3) + sigmoid, loss (config.py:113-122), dL/dz,
//   backward  dZ_{L-2} = (dz W_head) * (h > 0), dZ_{l-1} = (dZ_l W_l) * (Y_{l-1} > 0),
// and writes X^T, Y_l^T and dZ_l^T as 16-ray blocked fp32 operands for the dW GEMM
// (gemm.hip a_kblk / b_kblk: block b/16 = [features][16 rays]) plus the per-workgroup bias,
// output-layer and loss partials the update launch sums (chain3's layout).
//
// Weights are the A operand and stream from fp32 fragment images (chainf.hpp) into a
// register ring of D k-blocks that runs across block and epilogue boundaries; the 16 rays
// are the B operand, read from LDS tiles stored [ray][feature] with 16-byte chunks
// swizzled by the ray (conflict-free: a 16-lane group reads one chunk column of 16 rays).
// The accumulator of 16x16x4 holds (feature 16 t + 4 g + r, ray l % 16): a lane writes its
// 4 features of a tile as one 16-byte chunk, and reads its 8 k of the next layer as two.
// Eight compute waves split the output features (32 per wave at H = 256); a ninth store
// wave mirrors the barriers and does every global store (transposing the LDS tiles), so
// the compute waves' vmcnt queue holds weight loads only.
//
// At 4096 rays the f32 MFMAs (64 FLOP/clk/SIMD, 1/16 of bf16) bound the kernel: 10.7 GFLOP
// of forward + dX per step = 68 us at 157 TFLOP/s; the fp32 weight stream (5.2 MB per
// workgroup, twice chain3's) is below that at the per-CU L2 -> register rate.
#include "chainf.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using namespace c3;

constexpr float CF_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
constexpr int CF_CW = 8;                // compute waves
constexpr int CF_CT = CF_CW * 64;       // compute threads
constexpr int CF_THREADS = CF_CT + 64;  // + the store wave
constexpr int CF_LDS_CAP = 160 * 1024;
#ifndef CF_DEPTH
#define CF_DEPTH 4
#endif
// 16-byte feature chunks per thread per gather round (4: two rounds at k_pad = 1024 with the
// fragment prologue in flight; 8: one round, the prologue after it)
#ifndef CF_GR
#define CF_GR 4
#endif

template <int H>
struct LF {
  static constexpr int BM = 16;
  static constexpr int TN = H / (16 * CF_CW);  // 16-feature tiles per wave
  static constexpr int UPL = H / 32;           // k-blocks per hidden layer (= per stream block)
  static constexpr int NT = H / 16;            // 16-row tiles of a hidden-layer image
  static constexpr int NV = TN * 4;            // accumulator values per lane
  static constexpr int ROWB = H * 4;           // bytes per ray row of an activation tile
  static constexpr int TILE_BYTES = BM * ROWB;
  static constexpr int OFF_ACT = 0;                        // [2] activation / dZ tiles
  static constexpr int OFF_CS = OFF_ACT + 2 * TILE_BYTES;  // [2][H] bias-gradient partials
  static constexpr int OFF_HW = OFF_CS + 2 * H * 4;        // [3][H] output-layer weight grad
  static constexpr int OFF_HB = OFF_HW + 3 * H * 4;        // [4]
  static constexpr int OFF_LS = OFF_HB + 16;               // [2] f64 loss / SSE
  static constexpr int OFF_PRED = OFF_LS + 16;             // [BM][3]
  static constexpr int OFF_DZ = OFF_PRED + BM * 12;        // [waves][BM][3] head gradient
  static constexpr int OFF_TGT = OFF_DZ + CF_CW * BM * 12; // [BM][3] targets
  static constexpr int OFF_ZP = OFF_TGT + BM * 12;         // [waves][BM][3] head partial sums
  static constexpr int OFF_RAY = OFF_ZP + CF_CW * BM * 12; // [BM][4] vertex ids, [BM][3] ok
  static constexpr int OFF_RBARY = OFF_RAY + BM * 16 + BM * 12 + 16;  // [BM][3]
  static constexpr int OFF_W7 = OFF_RBARY + BM * 12 + 16;             // [3][H] then b7[3]
  static constexpr int OFF_VEC = OFF_W7 + 3 * H * 4 + 16;             // biases [L-1][H], Ly.bias
  __host__ __device__ static int off_x(int L) { return OFF_VEC + L * H * 4; }
  static int lds_bytes(int L, int k_pad) { return off_x(L) + BM * k_pad * 4; }
  static_assert(TN >= 1 && NV <= 8, "ReLU bits of a lane: at most 8 per layer");
  static_assert(OFF_LS % 8 == 0 && OFF_W7 % 16 == 0 && OFF_VEC % 16 == 0, "LDS alignment");
};

// byte offset of 16-byte chunk c (features 4 c .. 4 c + 3) of ray row r of a [16][cols]
// fp32 tile with `rowb`-byte rows
__device__ __forceinline__ int cf_off(int rowb, int r, int c) { return r * rowb + ((c ^ r) << 4); }

template <int H, int LOSS>
__global__ __launch_bounds__(CF_THREADS) void chainf_kernel(const ChainFArgs a) {
  using C = LF<H>;
  constexpr int BM = C::BM, TN = C::TN, UPL = C::UPL, NT = C::NT, NV = C::NV;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L;
  const int k_pad = a.k_pad;
  const int xrow = k_pad * 4;
  char* act = smem + C::OFF_ACT;
  float* csb = reinterpret_cast<float*>(smem + C::OFF_CS);
  float* hws = reinterpret_cast<float*>(smem + C::OFF_HW);
  float* hbs = reinterpret_cast<float*>(smem + C::OFF_HB);
  double* lss = reinterpret_cast<double*>(smem + C::OFF_LS);
  float* preds = reinterpret_cast<float*>(smem + C::OFF_PRED);
  float* dzs = reinterpret_cast<float*>(smem + C::OFF_DZ);
  float* tgs = reinterpret_cast<float*>(smem + C::OFF_TGT);
  float* zps = reinterpret_cast<float*>(smem + C::OFF_ZP);
  int* rvid = reinterpret_cast<int*>(smem + C::OFF_RAY);
  float* rbary = reinterpret_cast<float*>(smem + C::OFF_RBARY);
  float* w7s = reinterpret_cast<float*>(smem + C::OFF_W7);
  float* vecs = reinterpret_cast<float*>(smem + C::OFF_VEC);
  char* xs = smem + C::off_x(L);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int b0 = blockIdx.x * BM;
  const int nphase = a.nphase;
  const int nfwd = L - 1;

  if (wave < CF_CW) {
    // =========================== compute waves ============================================
    const int wc = wave;
    const int t0 = wc * TN;
    constexpr int D0 = CF_DEPTH;
    constexpr int D = D0 < UPL ? D0 : UPL;
    static_assert(UPL % D == 0, "the fragment ring depth must divide a block's k blocks");
    f32x4 fr[D][TN][2];
    const unsigned lane_off = (unsigned)t0 * 2048u + (unsigned)lane * 16u;
    auto rsrc_of = [&](const float* img) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, 0x7FFFFFFF, 0x00020000);
    };
    // fragment (k block kb, the wave's tile j, half h)
    // (every streamed image has H rows: W_0, W_y and the hidden W forward, the hidden W^T
    // of the dX phases)
    auto frag = [&](__amdgpu_buffer_rsrc_t rs, int kb, int j, int h) -> f32x4 {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane_off + j * 2048 + h * 1024, kb * NT * 2048, 0);
      return __builtin_bit_cast(f32x4, v);
    };
    // ---- ray records of the 16 rays: one thread per (ray, corner) ------------------------
    if (tid < BM * 3) {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int rl = tid / 3, i = tid % 3;
      const int b = b0 + rl;
      int v = 0, ok = 0;
      float w = 0.f;
      const int64_t rr = b < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src) : -1;
      if (rr >= 0) {
        const int64_t e = vid_at(a.vids, a.vid_dtype, 3 * rr + i);
        ok = (uint64_t)e < (uint64_t)a.num_vertices;  // out of range: a zero feature row
        v = ok ? (int)e : 0;
        w = a.bary[3 * rr + i];
      }
      rvid[rl * 4 + i] = v;
      rbary[rl * 3 + i] = w;
      rvid[BM * 4 + tid] = ok;
    }
#if CF_GR <= 4
    // the first block's fragments (k order: the loop's waits assume it)
    {
      const CFBlock& B0 = a.blk[0];
      const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(B0.img);
#pragma unroll
      for (int kb = 0; kb < D; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) fr[kb][j][h] = frag(rs0, B0.kb0 + kb, j, h);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#endif
    lbar();  // barrier R: ray records in LDS

    // ---- gather: the fp32 feature tile, 16-byte chunks (4 columns) per thread -----------
#ifndef CF_NO_GATHER  // diagnostics: no feature gather (garbage X)
    {
      const int cpr = k_pad >> 2;
      const int nch = BM * cpr;
      constexpr int GR = CF_GR;
#pragma unroll 1
      for (int q0 = tid; q0 < nch; q0 += CF_CT * GR) {
        f32x4 ev[GR][3];
        float wv[GR][3];
        int okv[GR];
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + CF_CT * g;
          const int r = (q < nch ? q : 0) / cpr, ch = (q < nch ? q : 0) % cpr;
          okv[g] = q < nch ? (rvid[BM * 4 + r * 3] & rvid[BM * 4 + r * 3 + 1] & rvid[BM * 4 + r * 3 + 2]) : 0;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            wv[g][i] = rbary[r * 3 + i];
            ev[g][i] = *reinterpret_cast<const f32x4*>(a.table + (int64_t)rvid[r * 4 + i] * k_pad + ch * 4);
          }
        }
#pragma unroll
        for (int g = 0; g < GR; ++g) {
          const int q = q0 + CF_CT * g;
          if (q < nch) {
            const int r = q / cpr, ch = q % cpr;
            f32x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = fmaf(wv[g][2], ev[g][2][e], fmaf(wv[g][1], ev[g][1][e], wv[g][0] * ev[g][0][e]));
              o[e] = okv[g] ? x : 0.f;
            }
            *reinterpret_cast<f32x4*>(xs + cf_off(xrow, r, ch)) = o;
          }
        }
      }
    }
#endif
#if CF_GR > 4
    // one gather round (CF_GR = 8): the fragment prologue after it, outside the gather's
    // register peak
    {
      const CFBlock& B0 = a.blk[0];
      const __amdgpu_buffer_rsrc_t rs0 = rsrc_of(B0.img);
#pragma unroll
      for (int kb = 0; kb < D; ++kb) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h) fr[kb][j][h] = frag(rs0, B0.kb0 + kb, j, h);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#endif
    // every load so far has landed (the fragment prologue was issued before the gather;
    // vmcnt is in order): clears the compiler's scoreboard of the gather registers
    __builtin_amdgcn_s_waitcnt(0);
    lbar();  // barrier 0: feature tile in LDS

    // ReLU bits of the lane's NV accumulator values for layers 0..L-3, 64 / NV per word
    constexpr int MPW = 64 / NV;
    static_assert(2 * MPW >= CHAIN_MAX_HIDDEN - 1, "ReLU bit words");
    unsigned long long mbits[2] = {0ull, 0ull};
    auto feat = [&](int j) { return 16 * (t0 + j) + 4 * g4; };
    // the lane's 4 values of tile j -> chunk feat(j) / 4 of its ray row
    auto put_act = [&](const float (&v)[TN][4], char* tile) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<f32x4*>(tile + cf_off(C::ROWB, r16, 4 * (t0 + j) + g4)) = f32x4{v[j][0], v[j][1], v[j][2], v[j][3]};
    };
    auto ray_sums_to = [&](const float (&v)[TN][4], float* dst) {
      float t[NV];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[j * 4 + r] = v[j][r];
      const float s = ray_sum<NV>(t, lane);
      const int idx = r16 % NV;
      const int fo = feat(idx >> 2) + (idx & 3);
      if (r16 < NV) dst[fo] = s;
    };

    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto run_block = [&](int i) {
      const CFBlock& B = a.blk[i];
      const CFBlock& Bn = a.blk[i + 1 < a.nblk ? i + 1 : i];
      const __amdgpu_buffer_rsrc_t crs = rsrc_of(B.img);
      const __amdgpu_buffer_rsrc_t nrs = rsrc_of(Bn.img);
      const bool from_x = B.a_x != 0;
      const char* bbase = from_x ? xs : act + (B.phase & 1) * C::TILE_BYTES;
      const int rowb = from_x ? xrow : C::ROWB;
      const int c0 = (from_x ? B.ak0 * 8 : 0) + 2 * g4;  // the lane's first chunk of k block 0
      const char* brow = bbase + r16 * rowb;
      auto bread = [&](int kb, f32x4 (&bv)[2]) {
        bv[0] = *reinterpret_cast<const f32x4*>(brow + (((c0 + 8 * kb) ^ r16) << 4));
        bv[1] = *reinterpret_cast<const f32x4*>(brow + (((c0 + 8 * kb + 1) ^ r16) << 4));
      };
      const int ckb = B.kb0, nkb = Bn.kb0;
      f32x4 bq[2][2];
      bread(0, bq[0]);
#pragma unroll
      for (int kb = 0; kb < UPL; ++kb) {
        if (kb + 1 < UPL) bread(kb + 1, bq[(kb + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const f32x4(&bv)[2] = bq[kb & 1];
        // (tiles interleaved: consecutive MFMAs update different accumulators)
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fr[kb % D][j][q >> 2][q & 3], bv[q >> 2][q & 3], acc[j], 0, 0, 0);
#ifndef CF_NO_LOADS  // diagnostics: the MFMAs on the prologue's fragments (wrong results)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            fr[kb % D][j][h] = kb + D < UPL ? frag(crs, ckb + kb + D, j, h) : frag(nrs, nkb + kb + D - UPL, j, h);
#endif
        __builtin_amdgcn_sched_barrier(0);
      }
      if (!B.last) return;
#ifdef CF_NO_EPI  // diagnostics: the weight stream and MFMAs with the barriers alone
      if (B.phase == nfwd - 1) lbar();
      {  // keep every MFMA (and its loads) alive
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) t += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
        if (t == 1234.5f) act[lane] = 1;
      }
      lbar();
      return;
#endif

      // ---- epilogue of phase p ---------------------------------------------------------
      const int p = B.phase;
      char* act_out = act + ((p + 1) & 1) * C::TILE_BYTES;
      float* cs_out = csb + (p & 1) * H;
      if (p < nfwd) {
        const int l = p;
        const bool skip = l == a.s;
        const bool last = l == L - 2;
        unsigned bits = 0;
        float hq[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(vecs + l * H + feat(j));
          f32x4 z = acc[j];
          if (skip) {
            const f32x4 yv = *reinterpret_cast<const f32x4*>(vecs + (L - 1) * H + feat(j));
#pragma unroll
            for (int r = 0; r < 4; ++r) z[r] = (z[r] + bv[r]) + yv[r];
          } else {
            z += bv;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            hq[j][r] = relu1(z[r]);
            bits |= (hq[j][r] > 0.f ? 1u : 0u) << (j * 4 + r);
          }
        }
        if (!last) {
          put_act(hq, act_out);
          if (l < MPW) mbits[0] |= (unsigned long long)bits << (NV * l);
          else mbits[1] |= (unsigned long long)bits << (NV * (l - MPW));
        } else {
          // ---- head on the registers of the last hidden layer (model.py:89-94) ----------
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
            if (g4 == 0) zps[(wc * BM + r16) * 3 + o] = z;
          }
          lbar();  // Bh1: per-wave head partial sums complete
          // sigmoid, loss and dL/dz (config.py:113-122, trainer.py:76): every compute wave
          // computes all 48 into its own copy of dz (same-wave LDS ordering only)
          {
            float* dzw = dzs + wc * BM * 3;
            float lsum = 0.f, ssum = 0.f;
            const int e = lane;
            if (e < BM * 3) {
              const int b = b0 + e / 3, o = e % 3;
              float z = w7s[3 * H + o];
#pragma unroll
              for (int w = 0; w < CF_CW; ++w) z += zps[w * BM * 3 + e];
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
                  const float qq = d * d / CF_CAUCHY_C2;
                  lv = CF_CAUCHY_C2 * logf(1.f + qq);
                  g = 2.f * d / (1.f + qq);
                }
                dz = (g * a.inv_count) * (1.f - pv) * pv;
                lsum = lv;
                ssum = d * d;
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
          // head backward: dZ_{L-2} = (dz W7) * (h > 0), its ray sums, and the output
          // layer's weight-gradient partials sum_rays dz_o * h
          float dzr[3];
#pragma unroll
          for (int o = 0; o < 3; ++o) dzr[o] = dzs[wc * BM * 3 + r16 * 3 + o];
          float gv[TN][4], hst[3][TN][4];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(w7s + 0 * H + feat(j));
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(w7s + 1 * H + feat(j));
            const f32x4 w2 = *reinterpret_cast<const f32x4*>(w7s + 2 * H + feat(j));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float g = fmaf(dzr[2], w2[r], fmaf(dzr[1], w1[r], dzr[0] * w0[r]));
              gv[j][r] = hq[j][r] > 0.f ? g : 0.f;
#pragma unroll
              for (int o = 0; o < 3; ++o) hst[o][j][r] = dzr[o] * hq[j][r];
            }
          }
          put_act(gv, act_out);
          if (wc == 0) {
#pragma unroll
            for (int o = 0; o < 3; ++o) {
              const float db = row_sum16(dzr[o]);
              if (lane == 0) hbs[o] = db;
            }
          }
          ray_sums_to(gv, cs_out);
#pragma unroll
          for (int o = 0; o < 3; ++o) ray_sums_to(hst[o], hws + o * H);
        }
      } else {
        // dX of layer l masked by Y_{l-1} > 0 -> dZ_{l-1} (tile, bias partial)
        const int l = (L - 2) - (p - nfwd);
        const unsigned bits = (unsigned)((l - 1 < MPW ? mbits[0] >> (NV * (l - 1)) : mbits[1] >> (NV * (l - 1 - MPW))) &
                                         ((1u << NV) - 1));
        float v[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = ((bits >> (j * 4 + r)) & 1u) ? acc[j][r] : 0.f;
        put_act(v, act_out);
        ray_sums_to(v, cs_out);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      lbar();  // B2: tile of the next phase and this phase's partials complete
    };
#pragma unroll 1
    for (int i = 0; i < a.nblk; ++i) run_block(i);
  } else {
    // =========================== store wave ===============================================
    constexpr int CPL = H / 64;
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
    lbar();  // barrier 0: feature tile in LDS
    if (a.count_step && blockIdx.x == 0 && lane == 0) a.ctrl->step += 1;
    {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int e = lane;
      const int bt = b0 + e / 3;
      float tt = 0.f;
      const int64_t trow =
          e < BM * 3 && bt < a.batch ? source_row(a.ray_idx, a.idx_dtype, offset, bt, a.num_rays, a.num_src) : -1;
      if (trow >= 0) tt = a.rgb[trow * 3 + e % 3];
      if (e < BM * 3) tgs[e] = tt;
    }
    // [16 rays][nf features] LDS tile -> the workgroup's [nf][16] block of a blocked
    // operand: per 16 features, lane (f = lane / 4, rays 4 q .. 4 q + 3 with q = lane % 4)
    // gathers 4 rays of one feature (conflict-free: the 64 lanes hit 16 chunk slots x 4
    // words) and the wave writes 1 KiB contiguous; 4 groups of reads issued per batch
    const int tf = lane >> 2, tq = lane & 3;
    auto copy_block = [&](const char* tile, int rowb, int nf, float* dst) {
#ifdef CF_NO_STORE  // diagnostics: the store wave mirrors the barriers only
      return;
#endif
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFFF, 0x00020000);
      constexpr int NB = 4;
#pragma unroll 1
      for (int f0 = 0; f0 < nf; f0 += 16 * NB) {
        f32x4 v[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int f = min(f0 + 16 * u, nf - 16) + tf;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * tq + i;
            v[u][i] = *reinterpret_cast<const float*>(tile + cf_off(rowb, r, f >> 2) + 4 * (f & 3));
          }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (f0 + 16 * u < nf) {
            const int f = f0 + 16 * u + tf;
            // write-through (sc1): the dW GEMM reads these blocks in the next launch
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), rd,
                                                   (unsigned)((f * 16 + 4 * tq) * 4), 0, 16);
          }
        }
      }
    };
    // split_images: [16 rays][nf] fp32 tile -> the hi / lo bf16 fragment images of the
    // [nf features][rows] operand.  The workgroup's 16 rays are half h of 32-ray k block
    // b0 / 32: per 16-feature tile one 512-byte piece, lane slot i + 16 rh = feature i, rays
    // 8 rh .. 8 rh + 7 (natural k order).  Lane (i, rh, tt) builds the slot of tile
    // 2 s + tt from 8 fp32 reads, so one store writes the pieces of two tiles (2 x 512
    // contiguous bytes) per image
    auto copy_split = [&](const char* tile, int rowb, int nf, void* img) {
#ifdef CF_NO_STORE
      return;
#endif
      char* hi = reinterpret_cast<char*>(img);
      const int64_t part = (int64_t)nf * a.rows * 2;  // bytes of one image
      const __amdgpu_buffer_rsrc_t rh_ = __builtin_amdgcn_make_buffer_rsrc(hi, (short)0, 0x7FFFFFFF, 0x00020000);
      const __amdgpu_buffer_rsrc_t rl_ = __builtin_amdgcn_make_buffer_rsrc(hi + part, (short)0, 0x7FFFFFFF, 0x00020000);
      const int fi = lane & 15, rh = (lane >> 4) & 1, tt = lane >> 5;
      const unsigned base = (unsigned)((b0 >> 5) * (nf / 16) * 1024 + ((b0 >> 4) & 1) * 512 + (lane & 31) * 16);
      // NB passes per batch: all their LDS reads issued before the first conversion
      constexpr int NB = 4;
#pragma unroll 1
      for (int s0 = 0; s0 < nf / 32; s0 += NB) {
        float x[NB][8];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int f = 16 * (2 * min(s0 + u, nf / 32 - 1) + tt) + fi;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            x[u][e] = *reinterpret_cast<const float*>(tile + cf_off(rowb, 8 * rh + e, f >> 2) + 4 * (f & 3));
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          if (s0 + u >= nf / 32) break;
          // pairs through v_cvt_pk_bf16_f32 (RNE, the bits of a scalar conversion): hi, then
          // lo = bf16(x - hi) with hi unpacked exactly (the store wave's VALU time is what
          // the split images add to the chain)
          u32x4 vh, vl;
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const unsigned w = pack_bf16x2(x[u][e], x[u][e + 1]);
            vh[e >> 1] = w;
            vl[e >> 1] = pack_bf16x2(x[u][e] - __builtin_bit_cast(float, w << 16),
                                     x[u][e + 1] - __builtin_bit_cast(float, w & 0xFFFF0000u));
          }
          // write-through (sc1), as the blocked operands: the dW GEMM reads them next launch
          const unsigned o = base + (unsigned)(2 * (s0 + u) + tt) * 1024u;
          __builtin_amdgcn_raw_buffer_store_b128(vh, rh_, o, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(vl, rl_, o, 0, 16);
        }
      }
    };
    auto copy_out = [&](const char* src, void* dst, int bytes) {
      char* d = reinterpret_cast<char*>(dst);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d, (short)0, 0x7FFFFFFF, 0x00020000);
      for (int c = lane * 16; c < bytes; c += 64 * 16)
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(src + c), rd, (unsigned)c, 0, 16);
    };
    // X^T while the compute waves stream W_0 (phase 0: the longest)
    if (a.split_images) copy_split(xs, xrow, k_pad, a.XT);
    else copy_block(xs, xrow, k_pad, a.XT + (int64_t)blockIdx.x * k_pad * 16);
#pragma unroll 1
    for (int p = 0; p < nphase; ++p) {
      const bool head_phase = p == nfwd - 1;
      if (head_phase) lbar();  // Bh1
      lbar();                  // B2
      const char* act_p = act + ((p + 1) & 1) * C::TILE_BYTES;
      const char* cs = reinterpret_cast<const char*>(csb + (p & 1) * H);
      const int64_t part0 = blockIdx.x;
      if (p < nfwd) {
        const int l = p;
        if (!head_phase) {
          if (a.split_images) copy_split(act_p, C::ROWB, H, a.YT[l]);
          else copy_block(act_p, C::ROWB, H, a.YT[l] + part0 * H * 16);
        }
        if (head_phase) {
          if (a.split_images) copy_split(act_p, C::ROWB, H, a.dZT[L - 2]);
          else copy_block(act_p, C::ROWB, H, a.dZT[L - 2] + part0 * H * 16);
          copy_out(cs, a.colsum[L - 2] + part0 * H, H * 4);
          copy_out(reinterpret_cast<const char*>(hws), a.hw_part + part0 * 3 * H, 3 * H * 4);
          if (lane < 3) a.hb_part[part0 * 3 + lane] = hbs[lane];
          if (lane < 2 && a.loss_part != nullptr) a.loss_part[2 * part0 + lane] = lss[lane];
          if (a.pred != nullptr && lane < BM * 3 && b0 + lane / 3 < a.batch) a.pred[(int64_t)b0 * 3 + lane] = preds[lane];
        }
      } else {
        const int l = (L - 2) - (p - nfwd);
        if (a.split_images) copy_split(act_p, C::ROWB, H, a.dZT[l - 1]);
        else copy_block(act_p, C::ROWB, H, a.dZT[l - 1] + part0 * H * 16);
        copy_out(cs, a.colsum[l - 1] + part0 * H, H * 4);
      }
    }
  }
}

template <int H, int LOSS>
int launchf_loss(const ChainFArgs& a, hipStream_t stream) {
  const int lds = LF<H>::lds_bytes(a.L, a.k_pad);
  INF_CHECK_ARG(lds <= CF_LDS_CAP, "chainf: LDS budget exceeded for this depth / feature width");
  static int attr_set = 0;
  if (attr_set < lds) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)chainf_kernel<H, LOSS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = lds;
  }
  chainf_kernel<H, LOSS><<<dim3((unsigned)(a.rows / LF<H>::BM)), dim3(CF_THREADS), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

template <int H>
int launchf_typed(const ChainFArgs& a, hipStream_t stream) {
  if (a.loss == INF_LOSS_L2) return launchf_loss<H, INF_LOSS_L2>(a, stream);
  if (a.loss == INF_LOSS_L1) return launchf_loss<H, INF_LOSS_L1>(a, stream);
  return launchf_loss<H, INF_LOSS_CAUCHY>(a, stream);
}

}  // namespace

bool chainf_supported(int H, int L, int k_pad) {
  if (H != 128 && H != 256) return false;
  if (L < 3 || L - 1 > CHAIN_MAX_HIDDEN || k_pad > CHAINF_MAX_KPAD || k_pad % H != 0) return false;
  if (2 * (k_pad / H) + 2 * (L - 2) > C3_MAX_BLOCKS) return false;
  const int lds = H == 256 ? LF<256>::lds_bytes(L, k_pad) : LF<128>::lds_bytes(L, k_pad);
  return lds <= CF_LDS_CAP;
}

int launch_chainf(const ChainFArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(chainf_supported(a.H, a.L, a.k_pad), "chainf: unsupported shape");
  INF_CHECK_ARG(a.rows % 16 == 0 && a.rows >= 16, "chainf: rows must be a multiple of 16");
  INF_CHECK_ARG(a.nphase == 2 * a.L - 3, "chainf: phases");
  INF_CHECK_ARG(a.nblk >= 1 && a.nblk <= C3_MAX_BLOCKS, "chainf: weight-stream blocks");
  INF_CHECK_ARG(a.table != nullptr && a.vids != nullptr && a.bary != nullptr && a.rgb != nullptr && a.XT != nullptr,
                "chainf: inputs");
  INF_CHECK_ARG(a.vid_dtype == INF_DTYPE_I32 || a.vid_dtype == INF_DTYPE_I64, "chainf: vertex id dtype");
  INF_CHECK_ARG(a.num_vertices < ((int64_t)1 << 31), "chainf: vertex ids must fit 32 bits");
  for (int i = 0; i < a.nblk; ++i) INF_CHECK_ARG(a.blk[i].img != nullptr, "chainf: weight image missing");
  for (int l = 0; l < a.L - 1; ++l) INF_CHECK_ARG((uintptr_t)a.bias[l] % 16 == 0, "chainf: bias alignment");
  INF_CHECK_ARG((uintptr_t)a.bias_y % 16 == 0 && (uintptr_t)a.W7 % 16 == 0, "chainf: vector alignment");
  if (a.H == 256) return launchf_typed<256>(a, stream);
  return launchf_typed<128>(a, stream);
}

}  // namespace inf
