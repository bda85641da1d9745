// Image metrics of the evaluation path (reference evaluation_metrics.py:29-34 dssim, via
// scikit-image's structural_similarity(multichannel=True) with its defaults: 7 x 7
// uniform window, K1 = 0.01, K2 = 0.03, sample covariance (N / (N - 1)), data_range of
// the input dtype, the mean of S over the image cropped by (7 - 1) / 2 on every side,
// averaged over channels).
//
// Only windows that lie entirely inside the image survive the crop, so the filter's
// boundary mode never matters.  One 256-thread workgroup owns a 16 x 16 block of
// output pixels: it stages the 22 x 22 x C input patch of both images in LDS, each lane
// forms the five window sums of its pixel in fp64 (skimage works in float64), and the
// block's S sum is reduced in a fixed order (lanes, then waves) into a per-block
// partial.  A second one-workgroup pass adds the partials in block order, so the result
// is deterministic.
#include <algorithm>

#include "common.hpp"

namespace inf {

namespace {

constexpr int SS_T = 16;             // output pixels per block side
constexpr int SS_WIN = 7;
constexpr int SS_P = SS_T + SS_WIN - 1;  // 22
constexpr int SS_MAXC = 4;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void ssim_block_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         int H, int W, int C, double c1, double c2,
                                                         double* __restrict__ partials) {
  __shared__ float pa[SS_MAXC][SS_P][SS_P + 1];
  __shared__ float pb[SS_MAXC][SS_P][SS_P + 1];
  __shared__ double red[4][SS_MAXC];
  const int t = threadIdx.x;
  const int y0 = blockIdx.y * SS_T, x0 = blockIdx.x * SS_T;  // first window's top-left corner
  for (int i = t; i < SS_P * SS_P; i += 256) {
    const int py = i / SS_P, px = i % SS_P;
    const int gy = y0 + py, gx = x0 + px;
    const bool in = gy < H && gx < W;
    const int64_t base = ((int64_t)gy * W + gx) * C;
    for (int c = 0; c < C; ++c) {
      pa[c][py][px] = in ? a[base + c] : 0.f;
      pb[c][py][px] = in ? b[base + c] : 0.f;
    }
  }
  __syncthreads();
  const int ty = t / SS_T, tx = t % SS_T;
  // window covering rows y0+ty .. +6: its centre pixel is interior iff the window fits
  const bool valid = (y0 + ty + SS_WIN <= H) && (x0 + tx + SS_WIN <= W);
  const double np = SS_WIN * SS_WIN;
  const double cov_norm = np / (np - 1.0);
  double s[SS_MAXC];
  for (int c = 0; c < SS_MAXC; ++c) s[c] = 0.0;
  if (valid) {
    for (int c = 0; c < C; ++c) {
      double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
#pragma unroll
      for (int dy = 0; dy < SS_WIN; ++dy) {
#pragma unroll
        for (int dx = 0; dx < SS_WIN; ++dx) {
          const double x = pa[c][ty + dy][tx + dx];
          const double y = pb[c][ty + dy][tx + dx];
          sx += x;
          sy += y;
          sxx = fma(x, x, sxx);
          syy = fma(y, y, syy);
          sxy = fma(x, y, sxy);
        }
      }
      const double ux = sx / np, uy = sy / np;
      const double vx = cov_norm * (sxx / np - ux * ux);
      const double vy = cov_norm * (syy / np - uy * uy);
      const double vxy = cov_norm * (sxy / np - ux * uy);
      const double A1 = 2.0 * ux * uy + c1, A2 = 2.0 * vxy + c2;
      const double B1 = ux * ux + uy * uy + c1, B2 = vx + vy + c2;
      s[c] = (A1 * A2) / (B1 * B2);
    }
  }
  const int wv = t >> 6, ln = t & 63;
  for (int c = 0; c < C; ++c) {
    const double w = wave_sum(s[c]);
    if (ln == 0) red[wv][c] = w;
  }
  __syncthreads();
  if (t < C) {
    const double v = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    partials[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * C + t] = v;
  }
}

__global__ __launch_bounds__(256) void ssim_final_kernel(const double* __restrict__ partials, int64_t nblocks, int C,
                                                         double inv_count, double* __restrict__ out) {
  __shared__ double red[4];
  const int t = threadIdx.x;
  for (int c = 0; c < C; ++c) {
    double v = 0.0;
    for (int64_t i = t; i < nblocks; i += 256) v += partials[i * C + c];
    v = wave_sum(v);
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    if (t == 0) out[c] = (((red[0] + red[1]) + red[2]) + red[3]) * inv_count;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void masked_sse_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         const uint8_t* __restrict__ mask, int64_t n_pix, int C,
                                                         double* __restrict__ partials) {
  __shared__ double red[4][2];
  double sse = 0.0, cnt = 0.0;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n_pix; p += (int64_t)gridDim.x * 256) {
    if (mask != nullptr && mask[p] == 0) continue;
    for (int c = 0; c < C; ++c) {
      const double d = (double)a[p * C + c] - (double)b[p * C + c];
      sse = fma(d, d, sse);
    }
    cnt += 1.0;
  }
  sse = wave_sum(sse);
  cnt = wave_sum(cnt);
  const int t = threadIdx.x;
  if ((t & 63) == 0) {
    red[t >> 6][0] = sse;
    red[t >> 6][1] = cnt;
  }
  __syncthreads();
  if (t < 2) partials[blockIdx.x * 2 + t] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
}

__global__ __launch_bounds__(64) void sse_final_kernel(const double* __restrict__ partials, int nblocks,
                                                       double* __restrict__ out) {
  const int t = threadIdx.x;
  double s = 0.0, n = 0.0;
  for (int i = t; i < nblocks; i += 64) {
    s += partials[2 * i];
    n += partials[2 * i + 1];
  }
  s = wave_sum(s);
  n = wave_sum(n);
  if (t == 0) {
    out[0] = s;
    out[1] = n;
  }
}

constexpr int SSE_BLOCKS = 1024;

int64_t ssim_blocks(int H, int W) {
  const int oh = H - SS_WIN + 1, ow = W - SS_WIN + 1;
  return (int64_t)ceil_div(oh, SS_T) * ceil_div(ow, SS_T);
}

}  // namespace

}  // namespace inf

using namespace inf;

extern "C" {

int64_t inf_ssim_workspace_bytes(int height, int width, int channels) {
  if (height < SS_WIN || width < SS_WIN || channels < 1 || channels > SS_MAXC) return -1;
  return ssim_blocks(height, width) * channels * (int64_t)sizeof(double);
}

int inf_ssim(const float* fake, const float* real, int height, int width, int channels, double data_range,
             void* workspace, double* out, inf_stream_t stream) {
  INF_CHECK_ARG(fake != nullptr && real != nullptr && workspace != nullptr && out != nullptr, "ssim: null argument");
  INF_CHECK_ARG(height >= SS_WIN && width >= SS_WIN,
                "ssim: images must be at least 7 x 7 (structural_similarity's win_size)");
  INF_CHECK_ARG(channels >= 1 && channels <= SS_MAXC, "ssim: 1..4 channels");
  INF_CHECK_ARG(data_range > 0, "ssim: data_range must be positive");
  hipStream_t st = (hipStream_t)stream;
  const int oh = height - SS_WIN + 1, ow = width - SS_WIN + 1;
  dim3 grid((unsigned)ceil_div(ow, SS_T), (unsigned)ceil_div(oh, SS_T));
  const double c1 = (0.01 * data_range) * (0.01 * data_range);
  const double c2 = (0.03 * data_range) * (0.03 * data_range);
  ssim_block_kernel<<<grid, 256, 0, st>>>(fake, real, height, width, channels, c1, c2, (double*)workspace);
  INF_LAUNCH_CHECK();
  ssim_final_kernel<<<1, 256, 0, st>>>((const double*)workspace, (int64_t)grid.x * grid.y, channels,
                                       1.0 / ((double)oh * (double)ow), out);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int64_t inf_masked_sse_workspace_bytes(void) { return (int64_t)SSE_BLOCKS * 2 * sizeof(double); }

int inf_masked_sse(const float* fake, const float* real, const uint8_t* mask, int64_t num_pixels, int channels,
                   void* workspace, double* out, inf_stream_t stream) {
  INF_CHECK_ARG(fake != nullptr && real != nullptr && workspace != nullptr && out != nullptr, "sse: null argument");
  INF_CHECK_ARG(num_pixels >= 0 && channels >= 1, "sse: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)std::min<int64_t>(SSE_BLOCKS, std::max<int64_t>(1, ceil_div(num_pixels, (int64_t)256)));
  masked_sse_kernel<<<nb, 256, 0, st>>>(fake, real, mask, num_pixels, channels, (double*)workspace);
  INF_LAUNCH_CHECK();
  sse_final_kernel<<<1, 64, 0, st>>>((const double*)workspace, nb, out);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // extern "C"
