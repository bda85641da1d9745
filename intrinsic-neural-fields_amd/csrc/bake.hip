// Texture baking on the device (reference bake_texture_field.py:96-245,334-420).
//
// The reference finds, for every texel p = (x, y) of the H x W texture, a UV triangle
// that strictly contains it (point_in_tri_matched :66-93 -- a texel on an edge matches
// no triangle, because a zero sign counts as both signs), searching the 10 triangles
// with the nearest centroids (get_tris_fast :134-161, cKDTree) among those of UV area
// >= 1e-4 (clean_tris :96-112), then its barycentrics by Cramer's rule on the 2-D Gram
// system (bary_matched :196-228).  After the MLP colours the texels, uv_fill_holes
// (:245-264) fills each empty texel that has a non-empty 5 x 5 neighbour with the
// binomial-weighted mean of its non-empty neighbours.
//
// Here the search is a scatter: one lane per triangle walks the texels of its bounding
// box and keeps, per texel, the containing triangle with the nearest centroid through a
// 64-bit atomicMin on (fp32 bits of the squared distance << 32 | triangle) -- the
// nearest-centroid order the kd-tree query returns, with no 10-candidate horizon.  A
// per-texel pass then resolves the winner and its barycentrics in fp64 (the reference
// uses numpy longdouble).  The MLP runs through the plan's render path over the
// compacted texels; the hole filling and the 8-bit quantisation are one more pass.
#include "common.hpp"

namespace inf {

namespace {

constexpr int BK_THREADS = 256;
constexpr unsigned long long BK_EMPTY = ~0ull;

__device__ __forceinline__ double orient(double p1x, double p1y, double p2x, double p2y, double p3x, double p3y) {
  return (p1x - p3x) * (p2y - p3y) - (p2x - p3x) * (p1y - p3y);
}

__global__ __launch_bounds__(BK_THREADS) void uv_raster_kernel(const double* __restrict__ uv, int64_t nv,
                                                               const int32_t* __restrict__ faces, int64_t T, int H,
                                                               int W, double min_area,
                                                               unsigned long long* __restrict__ keys) {
  const int64_t f = (int64_t)blockIdx.x * BK_THREADS + threadIdx.x;
  if (f >= T) return;
  const int32_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
  if ((uint64_t)i0 >= (uint64_t)nv || (uint64_t)i1 >= (uint64_t)nv || (uint64_t)i2 >= (uint64_t)nv) return;
  const double ax = uv[2 * i0], ay = uv[2 * i0 + 1];
  const double bx = uv[2 * i1], by = uv[2 * i1 + 1];
  const double cx = uv[2 * i2], cy = uv[2 * i2 + 1];
  const double area = 0.5 * ((ax - cx) * (by - cy) - (ay - cy) * (bx - cx));
  if (!(fabs(area) >= min_area)) return;  // clean_tris (also drops NaN corners)
  const double gx = (ax + bx + cx) / 3.0, gy = (ay + by + cy) / 3.0;
  const int x0 = (int)fmax(0.0, ceil(fmin(ax, fmin(bx, cx))));
  const int x1 = (int)fmin((double)(W - 1), floor(fmax(ax, fmax(bx, cx))));
  const int y0 = (int)fmax(0.0, ceil(fmin(ay, fmin(by, cy))));
  const int y1 = (int)fmin((double)(H - 1), floor(fmax(ay, fmax(by, cy))));
  for (int y = y0; y <= y1; ++y) {
    for (int x = x0; x <= x1; ++x) {
      const double px = x, py = y;
      const double d1 = orient(px, py, ax, ay, bx, by);
      const double d2 = orient(px, py, bx, by, cx, cy);
      const double d3 = orient(px, py, cx, cy, ax, ay);
      const bool neg = d1 <= 0 || d2 <= 0 || d3 <= 0;
      const bool pos = d1 >= 0 || d2 >= 0 || d3 >= 0;
      if (neg && pos) continue;
      const float dist2 = (float)((px - gx) * (px - gx) + (py - gy) * (py - gy));
      const unsigned long long key =
          ((unsigned long long)__float_as_uint(dist2) << 32) | (unsigned long long)(uint32_t)f;
      atomicMin(keys + (int64_t)y * W + x, key);
    }
  }
}

__global__ __launch_bounds__(BK_THREADS) void uv_resolve_kernel(const double* __restrict__ uv,
                                                                const int32_t* __restrict__ faces, int H, int W,
                                                                const unsigned long long* __restrict__ keys,
                                                                int32_t* __restrict__ texel_face,
                                                                float* __restrict__ texel_bary) {
  const int64_t t = (int64_t)blockIdx.x * BK_THREADS + threadIdx.x;
  if (t >= (int64_t)H * W) return;
  const unsigned long long key = keys[t];
  float u = 0.f, v = 0.f, w = 0.f;
  int32_t f = -1;
  if (key != BK_EMPTY) {
    f = (int32_t)(uint32_t)(key & 0xffffffffull);
    const int32_t i0 = faces[3 * (int64_t)f], i1 = faces[3 * (int64_t)f + 1], i2 = faces[3 * (int64_t)f + 2];
    const double ax = uv[2 * i0], ay = uv[2 * i0 + 1];
    const double px = (double)(t % W), py = (double)(t / W);
    const double v0x = uv[2 * i1] - ax, v0y = uv[2 * i1 + 1] - ay;
    const double v1x = uv[2 * i2] - ax, v1y = uv[2 * i2 + 1] - ay;
    const double v2x = px - ax, v2y = py - ay;
    const double d00 = v0x * v0x + v0y * v0y, d01 = v0x * v1x + v0y * v1y, d11 = v1x * v1x + v1y * v1y;
    const double d20 = v2x * v0x + v2y * v0y, d21 = v2x * v1x + v2y * v1y;
    const double den = fmax(d00 * d11 - d01 * d01, 0.0);
    const double bv = (d11 * d20 - d01 * d21) / den;
    const double bw = (d00 * d21 - d01 * d20) / den;
    u = (float)(1.0 - bv - bw);
    v = (float)bv;
    w = (float)bw;
  }
  texel_face[t] = f;
  texel_bary[3 * t] = u;
  texel_bary[3 * t + 1] = v;
  texel_bary[3 * t + 2] = w;
}

// uv_fill_holes + (255 * CC).astype(uint8): 16 x 16 texels per block, the 20 x 20 x 3
// neighbourhood staged in LDS (zero outside the texture, convolve2d's fill boundary).
constexpr int FH_T = 16;
constexpr int FH_P = FH_T + 4;

__global__ __launch_bounds__(BK_THREADS) void fill_holes_kernel(const float* __restrict__ img, int H, int W,
                                                                uint8_t* __restrict__ out_u8,
                                                                float* __restrict__ out_f) {
  __shared__ float tile[3][FH_P][FH_P + 1];
  const int t = threadIdx.x;
  const int by = blockIdx.y * FH_T - 2, bx = blockIdx.x * FH_T - 2;
  for (int i = t; i < FH_P * FH_P; i += BK_THREADS) {
    const int py = i / FH_P, px = i % FH_P;
    const int gy = by + py, gx = bx + px;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    for (int c = 0; c < 3; ++c) tile[c][py][px] = in ? img[((int64_t)gy * W + gx) * 3 + c] : 0.f;
  }
  __syncthreads();
  const int ty = t / FH_T, tx = t % FH_T;
  const int y = blockIdx.y * FH_T + ty, x = blockIdx.x * FH_T + tx;
  if (y >= H || x >= W) return;
  const double k1[5] = {1.0, 4.0, 6.0, 4.0, 1.0};
  double rgb[3] = {tile[0][ty + 2][tx + 2], tile[1][ty + 2][tx + 2], tile[2][ty + 2][tx + 2]};
  const bool filled = rgb[0] != 0.0 || rgb[1] != 0.0 || rgb[2] != 0.0;
  if (!filled) {
    double wf = 0.0, acc[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int dy = 0; dy < 5; ++dy) {
#pragma unroll
      for (int dx = 0; dx < 5; ++dx) {
        const double k = k1[dy] * k1[dx] / 256.0;
        const float r = tile[0][ty + dy][tx + dx], g = tile[1][ty + dy][tx + dx], b = tile[2][ty + dy][tx + dx];
        acc[0] += k * r;
        acc[1] += k * g;
        acc[2] += k * b;
        if (r != 0.f || g != 0.f || b != 0.f) wf += k;
      }
    }
    if (wf > 0.0)
      for (int c = 0; c < 3; ++c) rgb[c] = acc[c] / wf;
  }
  const int64_t o = ((int64_t)y * W + x) * 3;
  for (int c = 0; c < 3; ++c) {
    if (out_f != nullptr) out_f[o + c] = (float)rgb[c];
    if (out_u8 != nullptr) out_u8[o + c] = (uint8_t)(255.0 * rgb[c]);
  }
}

}  // namespace

}  // namespace inf

using namespace inf;

extern "C" {

int inf_uv_raster(const double* uv_px, int64_t num_uv_vertices, const int32_t* faces, int64_t num_faces, int height,
                  int width, double min_area, uint64_t* keys, int32_t* texel_face, float* texel_bary,
                  inf_stream_t stream) {
  INF_CHECK_ARG(height > 0 && width > 0 && num_faces >= 0 && num_uv_vertices >= 0, "uv_raster: bad sizes");
  INF_CHECK_ARG(num_faces < (1ll << 31), "uv_raster: too many faces");
  INF_CHECK_ARG(keys != nullptr && texel_face != nullptr && texel_bary != nullptr, "uv_raster: null output");
  INF_CHECK_ARG(num_faces == 0 || (uv_px != nullptr && faces != nullptr), "uv_raster: null input");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)height * width;
  INF_HIP_TRY(hipMemsetAsync(keys, 0xff, n * sizeof(uint64_t), st));
  if (num_faces > 0) {
    uv_raster_kernel<<<dim3((unsigned)ceil_div(num_faces, BK_THREADS)), BK_THREADS, 0, st>>>(
        uv_px, num_uv_vertices, faces, num_faces, height, width, min_area, (unsigned long long*)keys);
    INF_LAUNCH_CHECK();
  }
  uv_resolve_kernel<<<dim3((unsigned)ceil_div(n, BK_THREADS)), BK_THREADS, 0, st>>>(
      uv_px, faces, height, width, (const unsigned long long*)keys, texel_face, texel_bary);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_uv_fill_holes(const float* img, int height, int width, uint8_t* out_u8, float* out_f, inf_stream_t stream) {
  INF_CHECK_ARG(img != nullptr && height > 0 && width > 0, "fill_holes: bad input");
  INF_CHECK_ARG(out_u8 != nullptr || out_f != nullptr, "fill_holes: no output");
  dim3 grid((unsigned)ceil_div(width, FH_T), (unsigned)ceil_div(height, FH_T));
  fill_holes_kernel<<<grid, BK_THREADS, 0, (hipStream_t)stream>>>(img, height, width, out_u8, out_f);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // extern "C"
