// Large-batch bf16 training step, layer at a time (opt-in: INF_BIG_LAYERED=1, plan.hip).
//
// Why.  The fused chain (chain3.hip) keeps a ray tile's activations on chip across the
// whole network, but a workgroup runs its phases back to back: every hidden phase is the
// weight stream + MFMAs (≈1.4 µs per 64 rays) and then an epilogue + barrier (≈1.5 µs) in
// which the CU's matrix cores idle, and phase 0 waits on its chunk gathers.  At 65,536 rays
// there are enough rays for each layer to be one GEMM whose epilogue overlaps other waves'
// work: 128 rays per workgroup (each weight fragment feeds eight MFMAs), all of a chunk's
// activations in LDS, the bias / ReLU / mask / head fused into the epilogue, and the
// outputs written once in the two layouts the next kernels read (the next layer's B
// operand and the dW GEMM's fragment image).  The dW (fgemm.hip) and the update are the
// fused chain's.
//
// layer_kernel  8 waves x 32 output features (two 16-feature MFMA tiles), 8 x 16 rays.
//               Per 256-column chunk of a source: the workgroup's 64 B-operand pieces
//               (1 KiB each) land in LDS by direct-to-LDS loads while each wave loads its
//               16 weight fragments into registers, then 128 v_mfma_f32_16x16x32_bf16 per
//               wave.  Epilogues: see layer.hpp.
#include "layer.hpp"
#include "c3common.hpp"

namespace inf {
namespace {

using c3::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int LY_T = 512;
constexpr int LY_W = 8;                        // waves
constexpr int LY_NR = LY_RAYS / 16;            // ray tiles per workgroup
constexpr int LY_KBC = LY_KC / 32;             // k blocks per chunk
constexpr int LY_CHUNK = LY_KBC * LY_NR * 1024;  // bytes of B pieces per chunk (64 KiB)
constexpr int LY_STAGE = 2 * 16 * LY_RAYS * 2;   // per wave: the transposed output tile pair (8 KiB)
constexpr int LY_HEAD_OFF = LY_CHUNK;            // head scratch after the chunk buffer
constexpr int LY_HEAD_BYTES = LY_W * LY_RAYS * 3 * 4 + LY_RAYS * 3 * 4 + 2 * LY_W * 4 + 64;
constexpr float LY_CAUCHY_C2 = (20.f / 255.f) * (20.f / 255.f);
static_assert(LY_W * LY_STAGE <= LY_CHUNK, "the transposition stage reuses the chunk buffer");

template <int MODE, int LOSS>
__global__ __launch_bounds__(LY_T) void layer_kernel(const LayerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int H = 256;
  const int rt0 = blockIdx.x * LY_NR;  // first 16-ray tile of the workgroup
  const int b0 = blockIdx.x * LY_RAYS;

  f32x4 acc[LY_NR][2];
#pragma unroll
  for (int n = 0; n < LY_NR; ++n) acc[n][0] = acc[n][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- K loop: sources, then 256-column chunks -------------------------------------------
#pragma unroll 1
  for (int s = 0; s < a.nsrc; ++s) {
    const int kb_src = a.kin[s] / 32;
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.w[s]), (short)0, 0x7FFFFFFF, 0x00020000);
    const unsigned aoff = (unsigned)((2 * w) * 64 + lane) * 16u;  // the wave's row tiles 2 w, 2 w + 1
    const char* img = reinterpret_cast<const char*>(a.in[s]);
#pragma unroll 1
    for (int c = 0; c < kb_src / LY_KBC; ++c) {
      __syncthreads();  // every wave is done with the previous chunk's pieces
      // B: piece (kb, n) of the chunk at LDS (kb * 8 + n) KiB; wave w loads ray tile n = w
#pragma unroll
      for (int i = 0; i < LY_KBC; ++i) {
        const char* src = img + ((int64_t)(rt0 + w) * kb_src + c * LY_KBC + i) * 1024 + lane * 16;
        __builtin_amdgcn_global_load_lds(src, (lds_void*)(smem + (i * LY_NR + w) * 1024), 16, 0, 0);
      }
      // A: the wave's 2 x 8 fragments of the chunk
      bf16x8 fr[LY_KBC][2];
#pragma unroll
      for (int i = 0; i < LY_KBC; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fr[i][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                    ra, aoff + j * 1024, (c * LY_KBC + i) * (H / 16) * 1024, 0));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every wave's pieces landed
      const char* bl = smem + lane * 16;
#pragma unroll
      for (int i = 0; i < LY_KBC; ++i) {
#pragma unroll
        for (int n = 0; n < LY_NR; ++n) {
          const bf16x8 bv = *reinterpret_cast<const bf16x8*>(bl + (i * LY_NR + n) * 1024);
          acc[n][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i][0], bv, acc[n][0], 0, 0, 0);
          acc[n][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i][1], bv, acc[n][1], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();  // the chunk buffer becomes the transposition stage

  // this lane's accumulator element (n, j, r): ray 16 n + r16, feature 32 w + 16 j + 4 g4 + r
  auto feat = [&](int j, int r) { return 32 * w + 16 * j + 4 * g4 + r; };
  char* stage = smem + w * LY_STAGE;  // [j][feature i][ray] bf16
  const int64_t npiece_out = H / 32;

  // the output: B-operand piece (n, kb = w) and, through the stage, the fragment image
  auto write_out = [&](const float (&v)[LY_NR][2][4]) {
    unsigned short* st = reinterpret_cast<unsigned short*>(stage);
#pragma unroll
    for (int n = 0; n < LY_NR; ++n) {
      u32x4 o;
      o[0] = c3::pack_bf16x2(v[n][0][0], v[n][0][1]);
      o[1] = c3::pack_bf16x2(v[n][0][2], v[n][0][3]);
      o[2] = c3::pack_bf16x2(v[n][1][0], v[n][1][1]);
      o[3] = c3::pack_bf16x2(v[n][1][2], v[n][1][3]);
      *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(a.out) + (((int64_t)(rt0 + n) * npiece_out + w) * 64 + lane) * 16) = o;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned word = o[2 * j + (r >> 1)];
          st[(j * 16 + 4 * g4 + r) * LY_RAYS + 16 * n + r16] = (unsigned short)((r & 1) ? (word >> 16) : (word & 0xFFFFu));
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's stage writes (read back by its own lanes)
    // fragment image: per 32-ray block kb and feature tile t = 2 w + j one KiB, lane i + 16 g:
    // feature i of the tile, rays 8 g .. 8 g + 7 of the block
    const int fi = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int kb = 0; kb < LY_RAYS / 32; ++kb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const u32x4 t = *reinterpret_cast<const u32x4*>(stage + ((j * 16 + fi) * LY_RAYS + 32 * kb + 8 * fg) * 2);
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(a.outT) +
                                   (((int64_t)(b0 / 32 + kb) * (H / 16) + 2 * w + j) * 64 + lane) * 16) = t;
      }
  };
  // bias-gradient partial of this workgroup: sum over its 128 rays of v (fp32), one row
  auto col_partials = [&](const float (&v)[LY_NR][2][4], float* dst) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sum = v[0][j][r];
#pragma unroll
        for (int n = 1; n < LY_NR; ++n) sum += v[n][j][r];
        sum = c3::row_sum16(sum);
        if (r16 == 0) dst[feat(j, r)] = sum;
      }
  };

  if constexpr (MODE == LY_MODE_BWD) {
    // dX masked by the previous layer's activations (the same piece layout as the output)
    float v[LY_NR][2][4];
#pragma unroll
    for (int n = 0; n < LY_NR; ++n) {
      const u32x4 m = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(a.mask_in) +
                                                      (((int64_t)(rt0 + n) * npiece_out + w) * 64 + lane) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned word = m[2 * j + (r >> 1)];
          const unsigned h = (r & 1) ? (word >> 16) : (word & 0xFFFFu);
          v[n][j][r] = (h & 0x7FFFu) != 0u ? acc[n][j][r] : 0.f;
        }
    }
    write_out(v);
    col_partials(v, a.colsum + (int64_t)blockIdx.x * H);
    return;
  }

  // forward epilogue: + bias (+ Ly.bias at the skip layer, the layered GEMM's order), ReLU,
  // bf16 -- hq holds the bf16-rounded activations as floats
  float hq[LY_NR][2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 bv = *reinterpret_cast<const f32x4*>(a.bias0 + feat(j, 0));
    f32x4 yv = f32x4{0.f, 0.f, 0.f, 0.f};
    if (a.bias1 != nullptr) yv = *reinterpret_cast<const f32x4*>(a.bias1 + feat(j, 0));
#pragma unroll
    for (int n = 0; n < LY_NR; ++n)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        float z0 = acc[n][j][r] + bv[r], z1 = acc[n][j][r + 1] + bv[r + 1];
        if (a.bias1 != nullptr) {
          z0 += yv[r];
          z1 += yv[r + 1];
        }
        const unsigned wd = c3::pack_bf16x2(c3::relu1(z0), c3::relu1(z1));
        hq[n][j][r] = __builtin_bit_cast(float, wd << 16);
        hq[n][j][r + 1] = __builtin_bit_cast(float, wd & 0xFFFF0000u);
      }
  }
  if constexpr (MODE == LY_MODE_FWD) {
    write_out(hq);
    return;
  }

  // ---- HEAD: z = W7 h + b7 over the 256 features (8 waves), sigmoid, loss, dL/dz ----------
  float* zps = reinterpret_cast<float*>(smem + LY_HEAD_OFF);  // [wave][ray][3]
  float* dzs = zps + LY_W * LY_RAYS * 3;                      // [ray][3]
  float* red = dzs + LY_RAYS * 3;                             // [2][wave] loss / SSE
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int n = 0; n < LY_NR; ++n) {
      float z = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 wv = *reinterpret_cast<const f32x4*>(a.W7 + o * H + feat(j, 0));
#pragma unroll
        for (int r = 0; r < 4; ++r) z = fmaf(hq[n][j][r], wv[r], z);
      }
      z = c3::col_sum4(z);
      if (g4 == 0) zps[(w * LY_RAYS + 16 * n + r16) * 3 + o] = z;
    }
  __syncthreads();
  if (a.count_step && blockIdx.x == 0 && tid == 0) a.ctrl->step += 1;
  float lsum = 0.f, ssum = 0.f;
  if (tid < LY_RAYS * 3) {
    const int e = tid, ray = e / 3, o = e % 3;
    const int b = b0 + ray;
    float z = a.b7[o];
#pragma unroll
    for (int ww = 0; ww < LY_W; ++ww) z += zps[(ww * LY_RAYS + ray) * 3 + o];
    const float pv = 1.f / (1.f + expf(-z));
    float dz = 0.f;
    if (b < a.batch) {
      int64_t offset = a.idx_offset;
      if (a.ctrl != nullptr && a.offset_from_ctrl) offset += (int64_t)a.ctrl->batch_index * a.batch;
      const int64_t row = source_row(a.ray_idx, a.idx_dtype, offset, b, a.num_rays, a.num_src);
      const float tgt = row >= 0 ? a.rgb[row * 3 + o] : 0.f;
      const float d = pv - tgt;
      float lv, g;
      if constexpr (LOSS == INF_LOSS_L2) {
        lv = d * d;
        g = 2.f * d;
      } else if constexpr (LOSS == INF_LOSS_L1) {
        lv = fabsf(d);
        g = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      } else {
        const float qq = d * d / LY_CAUCHY_C2;
        lv = LY_CAUCHY_C2 * logf(1.f + qq);
        g = 2.f * d / (1.f + qq);
      }
      dz = (g * a.inv_count) * (1.f - pv) * pv;
      lsum = lv;
      ssum = d * d;
      if (a.pred != nullptr) a.pred[(int64_t)b * 3 + o] = pv;
    }
    dzs[e] = dz;
  }
  // loss partials: 64-lane sums, then the waves in order
  lsum = c3::col_sum4(c3::row_sum16(lsum));
  ssum = c3::col_sum4(c3::row_sum16(ssum));
  if (lane == 0) {
    red[w] = lsum;
    red[LY_W + w] = ssum;
  }
  __syncthreads();
  if (tid < 2) {
    float t = 0.f;
#pragma unroll
    for (int ww = 0; ww < LY_W; ++ww) t += red[tid * LY_W + ww];
    if (a.loss_part != nullptr) a.loss_part[2 * (int64_t)blockIdx.x + tid] = (double)t;
  }
  // head backward: dZ_{L-2} = (dz W7) * (h > 0), its bias partials, the output layer's
  // weight / bias partials (sums over the workgroup's rays)
  float v[LY_NR][2][4], hst[3][2][4];
  float dbs[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < LY_NR; ++n) {
    float dzr[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) dzr[o] = dzs[(16 * n + r16) * 3 + o];
#pragma unroll
    for (int o = 0; o < 3; ++o) dbs[o] += dzr[o];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(a.W7 + 0 * H + feat(j, 0));
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(a.W7 + 1 * H + feat(j, 0));
      const f32x4 w2 = *reinterpret_cast<const f32x4*>(a.W7 + 2 * H + feat(j, 0));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float g = fmaf(dzr[2], w2[r], fmaf(dzr[1], w1[r], dzr[0] * w0[r]));
        v[n][j][r] = hq[n][j][r] > 0.f ? g : 0.f;
#pragma unroll
        for (int o = 0; o < 3; ++o) hst[o][j][r] = n == 0 ? dzr[o] * hq[n][j][r] : fmaf(dzr[o], hq[n][j][r], hst[o][j][r]);
      }
    }
  }
  __syncthreads();  // the head scratch and the stage are read; the stage is written next
  write_out(v);
  col_partials(v, a.colsum + (int64_t)blockIdx.x * H);
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sum = c3::row_sum16(hst[o][j][r]);
        if (r16 == 0) a.hw_part[((int64_t)blockIdx.x * 3 + o) * H + feat(j, r)] = sum;
      }
  if (w == 0) {
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const float db = c3::row_sum16(dbs[o]);
      if (lane == 0) a.hb_part[(int64_t)blockIdx.x * 3 + o] = db;
    }
  }
}

template <int MODE, int LOSS>
int launch_mode(const LayerArgs& a, hipStream_t stream) {
  const int lds = MODE == LY_MODE_HEAD ? LY_HEAD_OFF + LY_HEAD_BYTES : LY_CHUNK;
  static bool attr = false;
  if (!attr) {
    INF_HIP_TRY(hipFuncSetAttribute((const void*)layer_kernel<MODE, LOSS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr = true;
  }
  layer_kernel<MODE, LOSS><<<dim3((unsigned)(a.rows / LY_RAYS)), dim3(LY_T), lds, stream>>>(a);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // namespace

int launch_layer(const LayerArgs& a, hipStream_t stream) {
  INF_CHECK_ARG(layer_supported(a.H, a.rows), "layer: H = 256, rows a multiple of 128");
  INF_CHECK_ARG(a.nsrc >= 1 && a.nsrc <= 2 && a.out != nullptr && a.outT != nullptr, "layer: operands");
  for (int s = 0; s < a.nsrc; ++s)
    INF_CHECK_ARG(a.in[s] != nullptr && a.w[s] != nullptr && a.kin[s] > 0 && a.kin[s] % LY_KC == 0, "layer: source");
  INF_CHECK_ARG(a.mode != LY_MODE_BWD || (a.mask_in != nullptr && a.colsum != nullptr && a.nsrc == 1), "layer: dX inputs");
  INF_CHECK_ARG(a.mode == LY_MODE_BWD || a.bias0 != nullptr, "layer: bias");
  if (a.mode == LY_MODE_HEAD) {
    INF_CHECK_ARG(a.W7 != nullptr && a.b7 != nullptr && a.hw_part != nullptr && a.hb_part != nullptr &&
                      a.colsum != nullptr && a.rgb != nullptr && a.ctrl != nullptr,
                  "layer: head inputs");
    switch (a.loss) {
      case INF_LOSS_L2: return launch_mode<LY_MODE_HEAD, INF_LOSS_L2>(a, stream);
      case INF_LOSS_L1: return launch_mode<LY_MODE_HEAD, INF_LOSS_L1>(a, stream);
      default: return launch_mode<LY_MODE_HEAD, INF_LOSS_CAUCHY>(a, stream);
    }
  }
  if (a.mode == LY_MODE_BWD) return launch_mode<LY_MODE_BWD, 0>(a, stream);
  return launch_mode<LY_MODE_FWD, 0>(a, stream);
}

}  // namespace inf
