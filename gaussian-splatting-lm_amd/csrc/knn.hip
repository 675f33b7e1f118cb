// knn.hip -- distCUDA2: per point, the mean squared distance to its 3 nearest other points
// (called by GaussianModel.create_from_pcd, scene/gaussian_model.py:249, to initialise
// the scales).  The reference's simple-knn submodule (absent here) sorts by Morton code and prunes
// 1024-point boxes against the 3rd-best distance of the point's Morton neighbours; its result is the
// exact 3-NN mean.  This is the same result from a uniform grid:
//   1. bounding box (block partials + one final block), copied to the host once to size the grid:
//      cubic cells of side h chosen so the grid has about as many cells as points (capped per axis);
//   2. cell keys, the in-tree LSD radix sort (cell, point) and per-cell [start, end) ranges; the
//      points are gathered in cell order (float4) so a cell's points are one coalesced read;
//   3. one thread per point (in cell order): scan the cells at Chebyshev cell distance 0..r, keeping the
//      three smallest squared distances, until the third is <= (r h)^2 -- every unvisited point is at
//      least r h away -- or the whole grid has been covered.  Exact, like the reference's.
// Per-point arithmetic as the reference's updateKBest: d = q - p, dist = d.x d.x + d.y d.y + d.z d.z,
// result (b0 + b1 + b2) / 3 (fewer than 3 other points: the missing ones are FLT_MAX, as there).
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "gslm_internal.hpp"

namespace gslm {

constexpr int KNN_THREADS = 256;
constexpr int KNN_BBOX_BLOCKS = 512;

__global__ __launch_bounds__(KNN_THREADS) void k_bbox_partial(int64_t n, const float* __restrict__ xyz,
                                                              float* __restrict__ part) {
  __shared__ float s[6][KNN_THREADS];
  float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * KNN_THREADS)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float v = xyz[3 * i + a];
      lo[a] = fminf(lo[a], v);
      hi[a] = fmaxf(hi[a], v);
    }
#pragma unroll
  for (int a = 0; a < 3; ++a) { s[a][threadIdx.x] = lo[a]; s[3 + a][threadIdx.x] = hi[a]; }
  __syncthreads();
  for (int o = KNN_THREADS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        s[a][threadIdx.x] = fminf(s[a][threadIdx.x], s[a][threadIdx.x + o]);
        s[3 + a][threadIdx.x] = fmaxf(s[3 + a][threadIdx.x], s[3 + a][threadIdx.x + o]);
      }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

__global__ void k_bbox_final(int np, const float* __restrict__ part, float* __restrict__ bbox) {
  if (threadIdx.x >= 6) return;
  const int a = threadIdx.x;
  float v = a < 3 ? FLT_MAX : -FLT_MAX;
  for (int b = 0; b < np; ++b) v = a < 3 ? fminf(v, part[6 * b + a]) : fmaxf(v, part[6 * b + a]);
  bbox[a] = v;
}

struct Grid {
  float ox, oy, oz, inv_h, h;
  int nx, ny, nz;
};

__device__ __forceinline__ int cell_coord(float v, float o, float inv_h, int n) {
  return min(n - 1, max(0, (int)((v - o) * inv_h)));
}

__global__ __launch_bounds__(KNN_THREADS) void k_cell_keys(int64_t n, const float* __restrict__ xyz, Grid g,
                                                           uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
  if (i >= n) return;
  const int cx = cell_coord(xyz[3 * i + 0], g.ox, g.inv_h, g.nx);
  const int cy = cell_coord(xyz[3 * i + 1], g.oy, g.inv_h, g.ny);
  const int cz = cell_coord(xyz[3 * i + 2], g.oz, g.inv_h, g.nz);
  keys[i] = (uint32_t)((cz * g.ny + cy) * g.nx + cx);
  vals[i] = (uint32_t)i;
}

__global__ __launch_bounds__(KNN_THREADS) void k_cell_ranges(int64_t n, const uint32_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ vals,
                                                             const float* __restrict__ xyz, uint2* __restrict__ range,
                                                             float4* __restrict__ sorted) {
  const int64_t k = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
  if (k >= n) return;
  const uint32_t c = keys[k];
  if (k == 0 || keys[k - 1] != c) range[c].x = (uint32_t)k;
  if (k == n - 1 || keys[k + 1] != c) range[c].y = (uint32_t)(k + 1);
  const uint32_t i = vals[k];
  sorted[k] = make_float4(xyz[3 * i + 0], xyz[3 * i + 1], xyz[3 * i + 2], __uint_as_float(i));
}

__device__ __forceinline__ void update_k3(float dist, float best[3]) {
#pragma unroll
  for (int j = 0; j < 3; ++j)
    if (best[j] > dist) {
      const float t = best[j];
      best[j] = dist;
      dist = t;
    }
}

__global__ __launch_bounds__(KNN_THREADS) void k_knn3(int64_t n, Grid g, const uint2* __restrict__ range,
                                                      const float4* __restrict__ sorted, float* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * KNN_THREADS + threadIdx.x;
  if (k >= n) return;
  const float4 p = sorted[k];
  const int cx = cell_coord(p.x, g.ox, g.inv_h, g.nx);
  const int cy = cell_coord(p.y, g.oy, g.inv_h, g.ny);
  const int cz = cell_coord(p.z, g.oz, g.inv_h, g.nz);
  float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
  const int rmax = max(g.nx, max(g.ny, g.nz));
  for (int r = 0; r <= rmax; ++r) {
    for (int dz = -r; dz <= r; ++dz) {
      const int z = cz + dz;
      if (z < 0 || z >= g.nz) continue;
      for (int dy = -r; dy <= r; ++dy) {
        const int y = cy + dy;
        if (y < 0 || y >= g.ny) continue;
        const bool face = (dz == -r || dz == r || dy == -r || dy == r);
        for (int dx = -r; dx <= r; dx += (face ? 1 : 2 * max(r, 1))) {  // only the shell at distance r
          const int x = cx + dx;
          if (x < 0 || x >= g.nx) continue;
          const uint2 rg = range[(z * g.ny + y) * g.nx + x];
          for (uint32_t j = rg.x; j < rg.y; ++j) {
            if ((int64_t)j == k) continue;
            const float4 q = sorted[j];
            const float ddx = q.x - p.x, ddy = q.y - p.y, ddz = q.z - p.z;
            update_k3((ddx * ddx + ddy * ddy) + ddz * ddz, best);
          }
          if (r == 0) break;
        }
      }
    }
    // unvisited points lie in cells at Chebyshev distance > r: at least r h away
    const float reach = (float)r * g.h * 0.999f;  // margin for the float cell assignment
    if (best[2] <= reach * reach) break;
  }
  out[__float_as_uint(p.w)] = ((best[0] + best[1]) + best[2]) / 3.0f;
}

struct KnnBufs {
  float* part;
  float* bbox;
  uint32_t *k0, *v0, *k1, *v1, *hist;
  float4* sorted;
  uint2* range;
};

static size_t knn_layout(int64_t n, int64_t cells, void* base, KnnBufs* o) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    void* p = base ? (char*)base + off : nullptr;
    off = align_up(off + bytes);
    return p;
  };
  KnnBufs b;
  b.part = (float*)take((size_t)6 * KNN_BBOX_BLOCKS * sizeof(float));
  b.bbox = (float*)take(8 * sizeof(float));
  b.k0 = (uint32_t*)take((size_t)n * 4);
  b.v0 = (uint32_t*)take((size_t)n * 4);
  b.k1 = (uint32_t*)take((size_t)n * 4);
  b.v1 = (uint32_t*)take((size_t)n * 4);
  b.hist = (uint32_t*)take(sort_hist_bytes(n));
  b.sorted = (float4*)take((size_t)n * sizeof(float4));
  b.range = (uint2*)take((size_t)cells * sizeof(uint2));
  if (o) *o = b;
  return off;
}

// cubic cells, about one per point, at most 2048 per axis and 4n + 64 in total
static Grid make_grid(const float bbox[6], int64_t n) {
  Grid g;
  double ext[3], vol = 1.0, emax = 0.0;
  for (int a = 0; a < 3; ++a) emax = std::max(emax, (double)bbox[3 + a] - (double)bbox[a]);
  if (!(emax > 0.0)) emax = 1.0;
  for (int a = 0; a < 3; ++a) {
    ext[a] = std::max((double)bbox[3 + a] - (double)bbox[a], emax * 1e-6);
    vol *= ext[a];
  }
  double h = std::max(std::cbrt(vol / (double)std::max<int64_t>(n, 1)), emax / 2048.0);
  int d[3];
  for (;;) {
    double total = 1.0;
    for (int a = 0; a < 3; ++a) {
      d[a] = std::max(1, (int)std::ceil(ext[a] / h));
      total *= d[a];
    }
    if (total <= 4.0 * (double)n + 64.0) break;
    h *= 1.26;
  }
  g.ox = bbox[0]; g.oy = bbox[1]; g.oz = bbox[2];
  g.h = (float)h;
  g.inv_h = (float)(1.0 / h);
  g.nx = d[0]; g.ny = d[1]; g.nz = d[2];
  return g;
}

}  // namespace gslm

using namespace gslm;

extern "C" {

size_t gslm_knn_scratch_bytes(int64_t n) { return knn_layout(n, 4 * n + 64, nullptr, nullptr) + 4096; }

int gslm_knn3_mean_dist(int64_t n, const float* xyz, float* out, void* scratch, size_t scratch_bytes, void* stream) {
  if (n < 0 || (n > 0 && (!xyz || !out))) { set_error("knn: NULL points / output"); return GSLM_ERR_INVALID; }
  if (n == 0) return GSLM_OK;
  if (n > (int64_t)UINT32_MAX / 4) { set_error("knn: too many points"); return GSLM_ERR_INVALID; }
  if (!scratch || scratch_bytes < gslm_knn_scratch_bytes(n)) { set_error("knn: scratch too small"); return GSLM_ERR_CAPACITY; }
  hipStream_t s = (hipStream_t)stream;
  KnnBufs b;
  knn_layout(n, 4 * n + 64, scratch, &b);
  const int nbb = (int)std::min<int64_t>(KNN_BBOX_BLOCKS, (n + KNN_THREADS - 1) / KNN_THREADS);
  hipLaunchKernelGGL(k_bbox_partial, dim3(nbb), dim3(KNN_THREADS), 0, s, n, xyz, b.part);
  hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(64), 0, s, nbb, b.part, b.bbox);
  GSLM_LAUNCH_CHECK();
  float bbox[6];
  GSLM_HIP_CHECK(hipMemcpyAsync(bbox, b.bbox, sizeof(bbox), hipMemcpyDeviceToHost, s));
  GSLM_HIP_CHECK(hipStreamSynchronize(s));
  for (int a = 0; a < 6; ++a)
    if (!std::isfinite(bbox[a])) { set_error("knn: non-finite point coordinates"); return GSLM_ERR_INVALID; }
  const Grid g = make_grid(bbox, n);
  const int64_t cells = (int64_t)g.nx * g.ny * g.nz;
  int end_bit = 1;
  while ((1ll << end_bit) < cells) ++end_bit;
  const unsigned nb = (unsigned)((n + KNN_THREADS - 1) / KNN_THREADS);
  hipLaunchKernelGGL(k_cell_keys, dim3(nb), dim3(KNN_THREADS), 0, s, n, xyz, g, b.k0, b.v0);
  GSLM_LAUNCH_CHECK();
  bool alt = false;
  int st = radix_sort_pairs(b.k0, b.v0, b.k1, b.v1, n, end_bit, b.hist, &alt, s);
  if (st) return st;
  const uint32_t* keys = alt ? b.k1 : b.k0;
  const uint32_t* vals = alt ? b.v1 : b.v0;
  GSLM_HIP_CHECK(hipMemsetAsync(b.range, 0, (size_t)cells * sizeof(uint2), s));
  hipLaunchKernelGGL(k_cell_ranges, dim3(nb), dim3(KNN_THREADS), 0, s, n, keys, vals, xyz, b.range, b.sorted);
  hipLaunchKernelGGL(k_knn3, dim3(nb), dim3(KNN_THREADS), 0, s, n, g, b.range, b.sorted, out);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // extern "C"
