// GPU ray casting for the render path: the reference's
// create_ray_origins_and_directions (mesh.py:171-207) + closest-hit ray-mesh intersection
// with Cramer barycentrics (mesh.py:210-251, trimesh/embree `intersects_location(...,
// multiple_hits=False)` + `points_to_barycentric(method='cramer')`), and the compaction
// into the hit lists mesh.ray_mesh_intersect returns.
//
// Host: a binned-SAH BVH over the triangles (8 bins per axis, leaves of <= 4 triangles),
// flattened depth-first (left child follows its parent), triangles re-ordered into leaf
// order and pre-transformed to (v0, e1, e2, face id) float4 triples.
// Device: one thread per masked pixel generates its ray (R K^-1 [x y 1], normalised, from
// the camera centre), walks the BVH with a per-thread stack in LDS (nearer child first),
// and intersects two-sided with Moller-Trumbore in fp32 (t > 0, closest hit).  For a point
// on the triangle Moller-Trumbore's (u, v) are the Cramer barycentrics of that point: the
// ray's barycentrics are (1 - u - v, u, v) w.r.t. the face's vertices in mesh order.
// Compaction keeps hits in ray order (per-block counts -> one-block scan -> scatter), so
// the lists are deterministic.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"

struct inf_bvh {
  int64_t num_vertices = 0, num_faces = 0;
  int32_t num_nodes = 0, depth = 0;
  float4* nodes = nullptr;   // [num_nodes][2]: {bmin, left_or_first (bits)}, {bmax, count (bits)}
  float4* tris = nullptr;    // [num_faces][3]: {v0, face id (bits)}, {e1, 0}, {e2, 0}
  int32_t* faces = nullptr;  // [num_faces][3] vertex ids (mesh order), for the hit lists
};

namespace inf {
namespace {

constexpr int RC_THREADS = 128;
constexpr int RC_STACK = 64;  // BVH depth bound (checked at build)

struct Aabb {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float* p) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  void grow(const Aabb& b) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  float area() const {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return (dx < 0 || dy < 0 || dz < 0) ? 0.f : 2.f * (dx * dy + dy * dz + dz * dx);
  }
};

struct HostNode {
  Aabb box;
  int32_t left_or_first = 0, count = 0;
};

struct Builder {
  const std::vector<Aabb>& tb;
  const std::vector<float>& cen;  // [F][3]
  std::vector<int32_t>& order;
  std::vector<HostNode>& nodes;
  int max_depth = 0;

  // node `ni` covers order[first, first + n)
  void build(int ni, int first, int n, int depth) {
    max_depth = std::max(max_depth, depth);
    Aabb box, cb;
    for (int i = first; i < first + n; ++i) {
      box.grow(tb[order[i]]);
      cb.grow(&cen[3 * order[i]]);
    }
    nodes[ni].box = box;
    if (n <= 4) {
      nodes[ni].left_or_first = first;
      nodes[ni].count = n;
      return;
    }
    // binned SAH over the centroid bounds
    constexpr int NB = 8;
    float best = INFINITY;
    int best_axis = -1, best_bin = 0;
    for (int a = 0; a < 3; ++a) {
      const float ext = cb.hi[a] - cb.lo[a];
      if (!(ext > 0.f)) continue;
      Aabb bb[NB];
      int bc[NB] = {0};
      for (int i = first; i < first + n; ++i) {
        int b = (int)((cen[3 * order[i] + a] - cb.lo[a]) / ext * NB);
        b = std::min(std::max(b, 0), NB - 1);
        bb[b].grow(tb[order[i]]);
        ++bc[b];
      }
      float la[NB], ra[NB];
      int lc[NB], rc[NB];
      Aabb acc;
      int c = 0;
      for (int b = 0; b < NB; ++b) {
        acc.grow(bb[b]);
        c += bc[b];
        la[b] = acc.area();
        lc[b] = c;
      }
      acc = Aabb();
      c = 0;
      for (int b = NB - 1; b >= 0; --b) {
        acc.grow(bb[b]);
        c += bc[b];
        ra[b] = acc.area();
        rc[b] = c;
      }
      for (int b = 0; b < NB - 1; ++b) {
        if (lc[b] == 0 || rc[b + 1] == 0) continue;
        const float cost = la[b] * lc[b] + ra[b + 1] * rc[b + 1];
        if (cost < best) {
          best = cost;
          best_axis = a;
          best_bin = b;
        }
      }
    }
    int mid;
    if (best_axis < 0) {
      mid = first + n / 2;  // all centroids coincide: split by count
    } else {
      const int a = best_axis;
      const float ext = cb.hi[a] - cb.lo[a];
      auto goes_left = [&](int32_t t) {
        int b = (int)((cen[3 * t + a] - cb.lo[a]) / ext * NB);
        b = std::min(std::max(b, 0), NB - 1);
        return b <= best_bin;
      };
      mid = (int)(std::stable_partition(order.begin() + first, order.begin() + first + n, goes_left) - order.begin());
      if (mid == first || mid == first + n) mid = first + n / 2;
    }
    const int left = (int)nodes.size();
    nodes.emplace_back();
    nodes.emplace_back();
    nodes[ni].left_or_first = left;
    nodes[ni].count = 0;
    build(left, first, mid - first, depth + 1);
    build(left + 1, mid, first + n - mid, depth + 1);
  }
};

__device__ __forceinline__ float3 f3(const float4& v) { return make_float3(v.x, v.y, v.z); }
__device__ __forceinline__ float3 sub3(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ float dot3(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float3 cross3(float3 a, float3 b) {
  return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

struct RayCam {
  float R[9];     // camCv2world[:3, :3], row-major
  float c[3];     // camCv2world[:, 3]
  float Kinv[9];  // K[:3, :3]^-1, row-major
};

// slab test: entry distance of [lo, hi] along the ray, or +inf if missed / beyond tmax
__device__ __forceinline__ float box_entry(const float4& lo, const float4& hi, float3 o, float3 inv, float tmax) {
  const float tx0 = (lo.x - o.x) * inv.x, tx1 = (hi.x - o.x) * inv.x;
  const float ty0 = (lo.y - o.y) * inv.y, ty1 = (hi.y - o.y) * inv.y;
  const float tz0 = (lo.z - o.z) * inv.z, tz1 = (hi.z - o.z) * inv.z;
  const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
  const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
  return tn <= tf ? tn : INFINITY;
}

// Closest hit of one ray (two-sided Moller-Trumbore, t > 0): face id (-1 = miss) and the
// hit point's barycentrics (1 - u - v, u, v).  `st`: this thread's LDS stack column.
__device__ __forceinline__ int trace(const float4* __restrict__ nodes, const float4* __restrict__ tris, float3 o,
                                     float3 d, int32_t* st, float& bu, float& bv) {
  const float3 inv = make_float3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  float best_t = INFINITY;
  int best_face = -1;
  bu = bv = 0.f;
  int sp = 0;
  int ni = box_entry(nodes[0], nodes[1], o, inv, best_t) == INFINITY ? -1 : 0;
  while (ni >= 0) {
    const float4 lo = nodes[2 * ni], hi = nodes[2 * ni + 1];
    const int count = __float_as_int(hi.w);
    if (count > 0) {
      const int first = __float_as_int(lo.w);
      for (int i = first; i < first + count; ++i) {
        const float4 a = tris[3 * i], b = tris[3 * i + 1], c = tris[3 * i + 2];
        const float3 e1 = f3(b), e2 = f3(c);
        const float3 pv = cross3(d, e2);
        const float det = dot3(e1, pv);
        if (fabsf(det) < 1e-20f) continue;
        const float id = 1.f / det;
        const float3 s = sub3(o, f3(a));
        const float u = dot3(s, pv) * id;
        if (u < 0.f || u > 1.f) continue;
        const float3 q = cross3(s, e1);
        const float v = dot3(d, q) * id;
        if (v < 0.f || u + v > 1.f) continue;
        const float t = dot3(e2, q) * id;
        if (t > 0.f && t < best_t) {
          best_t = t;
          bu = u;
          bv = v;
          best_face = __float_as_int(a.w);
        }
      }
      ni = sp > 0 ? st[--sp * RC_THREADS] : -1;
      continue;
    }
    // internal: visit the nearer child first, push the other
    const int l = __float_as_int(lo.w);
    const float tl = box_entry(nodes[2 * l], nodes[2 * l + 1], o, inv, best_t);
    const float tr = box_entry(nodes[2 * l + 2], nodes[2 * l + 3], o, inv, best_t);
    if (tl == INFINITY && tr == INFINITY) {
      ni = sp > 0 ? st[--sp * RC_THREADS] : -1;
    } else if (tl == INFINITY || tr == INFINITY) {
      ni = tl != INFINITY ? l : l + 1;
    } else {
      const int nearc = tl <= tr ? l : l + 1;
      st[sp++ * RC_THREADS] = nearc == l ? l + 1 : l;
      ni = nearc;
    }
  }
  return best_face;
}

// One ray per thread: generated for masked pixel r (mesh.py:171-207: R K^-1 [x y 1],
// normalised, from the camera centre) when `origins` is null, else the given ray.
__global__ __launch_bounds__(RC_THREADS) void raycast_kernel(const float4* __restrict__ nodes,
                                                            const float4* __restrict__ tris, RayCam cam, int H,
                                                            int W, const int64_t* __restrict__ pixel_idx,
                                                            const float* __restrict__ origins,
                                                            const float* __restrict__ dirs_in, int64_t L,
                                                            int32_t* __restrict__ hit_face, float* __restrict__ bary,
                                                            float* __restrict__ dirs_out) {
  __shared__ int32_t stack[RC_STACK * RC_THREADS];
  const int64_t r = (int64_t)blockIdx.x * RC_THREADS + threadIdx.x;
  if (r >= L) return;
  float3 o, d;
  if (origins != nullptr) {
    o = make_float3(origins[3 * r], origins[3 * r + 1], origins[3 * r + 2]);
    d = make_float3(dirs_in[3 * r], dirs_in[3 * r + 1], dirs_in[3 * r + 2]);
  } else {
    const int64_t p = pixel_idx != nullptr ? pixel_idx[r] : r;
    const float px = (float)(p % W), py = (float)(p / W);
    // K^-1 [x y 1], then R (..) -- the reference's fp32 matmul order
    const float kx = cam.Kinv[0] * px + cam.Kinv[1] * py + cam.Kinv[2];
    const float ky = cam.Kinv[3] * px + cam.Kinv[4] * py + cam.Kinv[5];
    const float kz = cam.Kinv[6] * px + cam.Kinv[7] * py + cam.Kinv[8];
    d = make_float3(cam.R[0] * kx + cam.R[1] * ky + cam.R[2] * kz, cam.R[3] * kx + cam.R[4] * ky + cam.R[5] * kz,
                    cam.R[6] * kx + cam.R[7] * ky + cam.R[8] * kz);
    const float inv_n = 1.f / sqrtf(dot3(d, d));
    d = make_float3(d.x * inv_n, d.y * inv_n, d.z * inv_n);
    o = make_float3(cam.c[0], cam.c[1], cam.c[2]);
    if (dirs_out != nullptr) {
      dirs_out[3 * r] = d.x;
      dirs_out[3 * r + 1] = d.y;
      dirs_out[3 * r + 2] = d.z;
    }
  }
  float bu, bv;
  const int f = trace(nodes, tris, o, d, stack + threadIdx.x, bu, bv);
  hit_face[r] = f;
  bary[3 * r] = 1.f - bu - bv;
  bary[3 * r + 1] = bu;
  bary[3 * r + 2] = bv;
}

// ---- compaction in ray order ------------------------------------------------------------
constexpr int CP_THREADS = 256;

__global__ __launch_bounds__(CP_THREADS) void hit_count_kernel(const int32_t* __restrict__ hit_face, int64_t L,
                                                               int32_t* __restrict__ block_counts) {
  __shared__ int32_t s[CP_THREADS / 64];
  const int64_t r = (int64_t)blockIdx.x * CP_THREADS + threadIdx.x;
  const int h = r < L && hit_face[r] >= 0;
  const unsigned long long m = __ballot(h);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < CP_THREADS / 64; ++w) t += s[w];
    block_counts[blockIdx.x] = t;
  }
}

// exclusive scan of the block counts (one block, serial over chunks of 1024); total -> *num_hits
__global__ __launch_bounds__(1024) void hit_scan_kernel(int32_t* __restrict__ block_counts, int nblocks,
                                                        int64_t* __restrict__ num_hits) {
  __shared__ int32_t s[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < nblocks; base += 1024) {
    const int i = base + threadIdx.x;
    const int32_t v = i < nblocks ? block_counts[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int32_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += x;
      __syncthreads();
    }
    if (i < nblocks) block_counts[i] = carry + s[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *num_hits = carry;
}

__global__ __launch_bounds__(CP_THREADS) void hit_scatter_kernel(
    const int32_t* __restrict__ hit_face, const float* __restrict__ bary, int64_t L,
    const int32_t* __restrict__ block_offsets, const int32_t* __restrict__ faces, int64_t* __restrict__ out_vids,
    float* __restrict__ out_bary, int64_t* __restrict__ out_ray, int64_t* __restrict__ out_face) {
  __shared__ int32_t s[CP_THREADS / 64];
  const int64_t r = (int64_t)blockIdx.x * CP_THREADS + threadIdx.x;
  const int f = r < L ? hit_face[r] : -1;
  const int h = f >= 0;
  const unsigned long long m = __ballot(h);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s[w] = __popcll(m);
  __syncthreads();
  int off = block_offsets[blockIdx.x];
  for (int i = 0; i < w; ++i) off += s[i];
  off += __popcll(m & ((1ull << lane) - 1));
  if (!h) return;
  for (int c = 0; c < 3; ++c) {
    out_vids[3 * (int64_t)off + c] = faces[3 * (int64_t)f + c];
    out_bary[3 * (int64_t)off + c] = bary[3 * r + c];
  }
  out_ray[off] = r;
  if (out_face != nullptr) out_face[off] = f;
}

}  // namespace
}  // namespace inf

using namespace inf;

extern "C" {

int inf_bvh_create(const float* vertices, int64_t num_vertices, const int64_t* faces, int64_t num_faces,
                   inf_bvh** out) {
  INF_CHECK_ARG(out != nullptr && vertices != nullptr && faces != nullptr, "bvh: null argument");
  INF_CHECK_ARG(num_vertices > 0 && num_faces > 0 && num_faces < (1ll << 31), "bvh: mesh size");
  *out = nullptr;
  const int F = (int)num_faces;
  std::vector<Aabb> tb(F);
  std::vector<float> cen(3 * (size_t)F);
  for (int f = 0; f < F; ++f) {
    for (int c = 0; c < 3; ++c) {
      const int64_t v = faces[3 * (int64_t)f + c];
      INF_CHECK_ARG(v >= 0 && v < num_vertices, "bvh: face vertex id out of range");
      tb[f].grow(vertices + 3 * v);
    }
    for (int a = 0; a < 3; ++a) cen[3 * (size_t)f + a] = 0.5f * (tb[f].lo[a] + tb[f].hi[a]);
  }
  std::vector<int32_t> order(F);
  for (int f = 0; f < F; ++f) order[f] = f;
  std::vector<HostNode> nodes;
  nodes.reserve(2 * (size_t)F);
  nodes.emplace_back();
  Builder b{tb, cen, order, nodes};
  b.build(0, 0, F, 0);
  INF_CHECK_ARG(b.max_depth < RC_STACK, "bvh: tree deeper than the traversal stack");
  std::vector<float4> hn(2 * nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) {
    const HostNode& n = nodes[i];
    int32_t lf = n.left_or_first, cnt = n.count;
    float lfv, cv;
    std::memcpy(&lfv, &lf, 4);
    std::memcpy(&cv, &cnt, 4);
    hn[2 * i] = make_float4(n.box.lo[0], n.box.lo[1], n.box.lo[2], lfv);
    hn[2 * i + 1] = make_float4(n.box.hi[0], n.box.hi[1], n.box.hi[2], cv);
  }
  std::vector<float4> ht(3 * (size_t)F);
  std::vector<int32_t> hf(3 * (size_t)F);
  for (int i = 0; i < F; ++i) {
    const int f = order[i];
    const float* v0 = vertices + 3 * faces[3 * (int64_t)f];
    const float* v1 = vertices + 3 * faces[3 * (int64_t)f + 1];
    const float* v2 = vertices + 3 * faces[3 * (int64_t)f + 2];
    float fv;
    std::memcpy(&fv, &f, 4);
    ht[3 * (size_t)i] = make_float4(v0[0], v0[1], v0[2], fv);
    ht[3 * (size_t)i + 1] = make_float4(v1[0] - v0[0], v1[1] - v0[1], v1[2] - v0[2], 0.f);
    ht[3 * (size_t)i + 2] = make_float4(v2[0] - v0[0], v2[1] - v0[1], v2[2] - v0[2], 0.f);
  }
  for (int64_t i = 0; i < 3 * (int64_t)F; ++i) hf[i] = (int32_t)faces[i];
  inf_bvh* h = new inf_bvh();
  h->num_vertices = num_vertices;
  h->num_faces = num_faces;
  h->num_nodes = (int32_t)nodes.size();
  h->depth = b.max_depth;
  auto fail = [&](hipError_t e) {
    set_error(std::string("bvh: ") + hipGetErrorString(e));
    (void)hipFree(h->nodes);
    (void)hipFree(h->tris);
    (void)hipFree(h->faces);
    delete h;
    return INF_ERR_HIP;
  };
  hipError_t e;
  if ((e = hipMalloc(&h->nodes, hn.size() * sizeof(float4))) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->tris, ht.size() * sizeof(float4))) != hipSuccess) return fail(e);
  if ((e = hipMalloc(&h->faces, hf.size() * sizeof(int32_t))) != hipSuccess) return fail(e);
  if ((e = hipMemcpy(h->nodes, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e);
  if ((e = hipMemcpy(h->tris, ht.data(), ht.size() * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e);
  if ((e = hipMemcpy(h->faces, hf.data(), hf.size() * sizeof(int32_t), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e);
  *out = h;
  return INF_OK;
}

void inf_bvh_destroy(inf_bvh* bvh) {
  if (bvh == nullptr) return;
  (void)hipFree(bvh->nodes);
  (void)hipFree(bvh->tris);
  (void)hipFree(bvh->faces);
  delete bvh;
}

int inf_bvh_info(const inf_bvh* bvh, int64_t* num_faces, int32_t* num_nodes, int32_t* depth) {
  INF_CHECK_ARG(bvh != nullptr, "bvh: null");
  if (num_faces) *num_faces = bvh->num_faces;
  if (num_nodes) *num_nodes = bvh->num_nodes;
  if (depth) *depth = bvh->depth;
  return INF_OK;
}

int inf_raycast(const inf_bvh* bvh, const float* cam_cv2world, const float* K, int H, int W, const int64_t* pixel_idx,
                int64_t num_rays, int32_t* hit_face, float* bary, float* unit_dirs, inf_stream_t stream) {
  INF_CHECK_ARG(bvh != nullptr && cam_cv2world != nullptr && K != nullptr, "raycast: null argument");
  INF_CHECK_ARG(H > 0 && W > 0 && num_rays >= 0, "raycast: arguments");
  INF_CHECK_ARG(num_rays == 0 || (hit_face != nullptr && bary != nullptr), "raycast: null output");
  INF_CHECK_ARG(pixel_idx != nullptr || num_rays == (int64_t)H * W, "raycast: without a pixel list every pixel is a ray");
  RayCam cam;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) cam.R[3 * i + j] = cam_cv2world[4 * i + j];
    cam.c[i] = cam_cv2world[4 * i + 3];
  }
  // K^-1 in double, then fp32
  const double a = K[0], b = K[1], c = K[2], d = K[3], e = K[4], f = K[5], g = K[6], h = K[7], k = K[8];
  const double det = a * (e * k - f * h) - b * (d * k - f * g) + c * (d * h - e * g);
  INF_CHECK_ARG(std::fabs(det) > 0.0, "raycast: singular intrinsics");
  const double inv[9] = {(e * k - f * h) / det, (c * h - b * k) / det, (b * f - c * e) / det,
                         (f * g - d * k) / det, (a * k - c * g) / det, (c * d - a * f) / det,
                         (d * h - e * g) / det, (b * g - a * h) / det, (a * e - b * d) / det};
  for (int i = 0; i < 9; ++i) cam.Kinv[i] = (float)inv[i];
  if (num_rays == 0) return INF_OK;
  const int64_t grid = ceil_div(num_rays, RC_THREADS);
  INF_CHECK_ARG(grid < (1ll << 31), "raycast: too many rays");
  raycast_kernel<<<dim3((unsigned)grid), dim3(RC_THREADS), 0, (hipStream_t)stream>>>(
      bvh->nodes, bvh->tris, cam, H, W, pixel_idx, nullptr, nullptr, num_rays, hit_face, bary, unit_dirs);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_raycast_rays(const inf_bvh* bvh, const float* origins, const float* dirs, int64_t num_rays, int32_t* hit_face,
                     float* bary, inf_stream_t stream) {
  INF_CHECK_ARG(bvh != nullptr && num_rays >= 0, "raycast_rays: arguments");
  if (num_rays == 0) return INF_OK;
  INF_CHECK_ARG(origins != nullptr && dirs != nullptr && hit_face != nullptr && bary != nullptr,
                "raycast_rays: null argument");
  const int64_t grid = ceil_div(num_rays, RC_THREADS);
  INF_CHECK_ARG(grid < (1ll << 31), "raycast_rays: too many rays");
  RayCam cam{};
  raycast_kernel<<<dim3((unsigned)grid), dim3(RC_THREADS), 0, (hipStream_t)stream>>>(
      bvh->nodes, bvh->tris, cam, 1, 1, nullptr, origins, dirs, num_rays, hit_face, bary, nullptr);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

int inf_compact_hits(const inf_bvh* bvh, const int32_t* hit_face, const float* bary, int64_t num_rays,
                     int32_t* scratch, int64_t* num_hits, int64_t* out_vids, float* out_bary, int64_t* out_ray,
                     int64_t* out_face, inf_stream_t stream) {
  INF_CHECK_ARG(bvh != nullptr, "compact_hits: null bvh");
  return inf_compact_faces(bvh->faces, hit_face, bary, num_rays, scratch, num_hits, out_vids, out_bary, out_ray,
                           out_face, stream);
}

int inf_compact_faces(const int32_t* faces, const int32_t* hit_face, const float* bary, int64_t num_rays,
                      int32_t* scratch, int64_t* num_hits, int64_t* out_vids, float* out_bary, int64_t* out_ray,
                      int64_t* out_face, inf_stream_t stream) {
  INF_CHECK_ARG(faces != nullptr && num_hits != nullptr && num_rays >= 0, "compact_hits: arguments");
  hipStream_t st = (hipStream_t)stream;
  if (num_rays == 0) {
    INF_HIP_TRY(hipMemsetAsync(num_hits, 0, sizeof(int64_t), st));
    return INF_OK;
  }
  INF_CHECK_ARG(hit_face != nullptr && bary != nullptr && scratch != nullptr, "compact_hits: null argument");
  INF_CHECK_ARG(out_vids != nullptr && out_bary != nullptr && out_ray != nullptr, "compact_hits: outputs");
  const int64_t nb = ceil_div(num_rays, CP_THREADS);
  INF_CHECK_ARG(nb < (1ll << 31), "compact_hits: too many rays");
  hit_count_kernel<<<dim3((unsigned)nb), dim3(CP_THREADS), 0, st>>>(hit_face, num_rays, scratch);
  INF_LAUNCH_CHECK();
  hit_scan_kernel<<<1, 1024, 0, st>>>(scratch, (int)nb, num_hits);
  INF_LAUNCH_CHECK();
  hit_scatter_kernel<<<dim3((unsigned)nb), dim3(CP_THREADS), 0, st>>>(hit_face, bary, num_rays, scratch, faces,
                                                                       out_vids, out_bary, out_ray, out_face);
  INF_LAUNCH_CHECK();
  return INF_OK;
}

}  // extern "C"
