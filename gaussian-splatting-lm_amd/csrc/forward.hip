// forward.hip -- rasterizer forward for gfx950.
//
//   k_preprocess   one thread per Gaussian: cull, project, cov3D, EWA cov2D, conic, radius,
//                  rect, SH->RGB; writes a 48-B render record (64-B stride) + depth key + tile count.
//   (depth sort of P keys + scan of tile counts in depth order: sort.hip)
//   k_duplicate    emits (tile id, Gaussian id) pairs in depth order: the later *stable* sort on
//                  the tile id alone then yields upstream's (tile, depth, index) order with
//                  2 radix passes over N_dup instead of 6 (SURVEY §7 "Sort"); the sorted values
//                  ARE the point list.
//   k_ranges       per-tile [start, end) from key changes (identifyTileRanges).
//   (k_render_fwd, the per-tile blend: render_fwd.hip)
#include "gslm_internal.hpp"
#include "gslm_kernels.hpp"

namespace gslm {

// STAGE: the block's SH-rest rows (3(M-1) floats per Gaussian, contiguous: the GaussianModel leaf) are
// staged through LDS with coalesced float4 loads first -- per-thread reads at a 180-B stride made every
// load instruction touch 64 cache lines (k_preprocess ran at ~2.2 TB/s).
template <bool RAW, bool STAGE>
__global__ __launch_bounds__(256) void k_preprocess(ViewK v, GaussK g, float4* __restrict__ rec,
                                                     uint32_t* __restrict__ depth_key,
                                                     uint32_t* __restrict__ tiles, uint2* __restrict__ rect,
                                                     uint32_t* __restrict__ clampw, int* __restrict__ radii_out,
                                                     int lead) {
  extern __shared__ __attribute__((aligned(16))) float s_sh[];  // STAGE: [256 * rest_stride]
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (STAGE) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
    const int64_t nv = min((int64_t)blockDim.x, g.P - i0);
    const int64_t total = nv * g.rest_stride;  // floats; i0 * rest_stride * 4 B is 16-B aligned (i0 % 256 == 0)
    const float* rows = g.rest - lead + i0 * g.rest_stride;  // stage_lead
    const float4* src4 = reinterpret_cast<const float4*>(rows);
    float4* dst4 = reinterpret_cast<float4*>(s_sh);
    for (int64_t e = threadIdx.x; e < total / 4; e += blockDim.x) dst4[e] = src4[e];
    for (int64_t e = (total / 4) * 4 + threadIdx.x; e < total; e += blockDim.x) s_sh[e] = rows[e];
    __syncthreads();
    g.rest = s_sh + lead;
    g.rest_base = i0;
  }
  if (i >= g.P) return;
  tiles[i] = 0u;
  depth_key[i] = 0xFFFFFFFFu;
  if (radii_out) radii_out[i] = 0;
  PreOut o;
  o.depth = 0.f;
  const bool vis = preprocess_one<RAW>(v, g, i, o);
  // Every Gaussian in front of the near plane gets its depth key, culled by its footprint or not: the depth order
  // then depends on means3D and the view alone, so one view's order is reusable while xyz is unchanged (the LM
  // step freezes xyz, train_jvp.py:221-227: gslm_preprocess_ordered).  The point list is the same either way
  // (Gaussians culled later emit no tile).
  if (o.depth > 0.2f) depth_key[i] = __float_as_uint(o.depth);
  if (!vis) return;

  const float4 r0 = make_float4(o.x, o.y, o.conic[0], o.conic[1]);
  const float4 r1 = make_float4(o.conic[2], o.opac, o.rgb[0], o.rgb[1]);
  const float4 r2 = make_float4(o.rgb[2], 1.0f / o.depth, __uint_as_float(o.clamped), o.tq);
  rec[RECS * i + 0] = r0;
  rec[RECS * i + 1] = r1;
  rec[RECS * i + 2] = r2;
  tiles[i] = (uint32_t)((o.rmax_x - o.rmin_x) * (o.rmax_y - o.rmin_y));
  const uint2 rc = make_uint2((uint32_t)o.rmin_x | ((uint32_t)o.rmin_y << 16), (uint32_t)o.rmax_x | ((uint32_t)o.rmax_y << 16));
  rect[i] = rc;
  // the rect again in the record's padding slot: k_duplicate's random per-Gaussian read is then one 64-B record
  // (one cache line) instead of the record and a rect line
  rec[RECS * i + 3] = make_float4(__uint_as_float(rc.x), __uint_as_float(rc.y), 0.f, 0.f);
  clampw[i] = o.clamped;  // read only where tiles[i] != 0
  if (radii_out) radii_out[i] = o.radius;
}

// k_preprocess with the block's SH-rest rows staged by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction,
// no VGPR round trip) and the staging overlapped with the geometry: every thread loads its Gaussian's geometry
// inputs first (and waits for them), the waves then issue the block's DMA chunks, run the geometry arithmetic
// (cull, EWA, conic, radius, rect) while the rows land, and meet at one barrier before the colour.  The register
// path (k_preprocess<_, true>) keeps one 16-B load per thread in flight per round trip of its staging loop.
// Same arithmetic in the same order: bitwise the same records.
__device__ __forceinline__ void glds16(const float4* src, float4* lds_dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <bool RAW>
__global__ __launch_bounds__(256) void k_preprocess_dma(ViewK v, GaussK g, float4* __restrict__ rec,
                                                         uint32_t* __restrict__ depth_key,
                                                         uint32_t* __restrict__ tiles, uint2* __restrict__ rect,
                                                         uint32_t* __restrict__ clampw, int* __restrict__ radii_out,
                                                         int lead) {
  extern __shared__ __attribute__((aligned(16))) float s_sh[];  // [256 * rest_stride]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const bool live = i < g.P;
  // 1. this Gaussian's geometry inputs, waited for before any DMA is in flight (hipcc waits vmcnt(0) at the first
  //    use of an ordinary load issued while an LDS-DMA is outstanding)
  PreIn in{};
  if (live) load_pre_in<RAW>(g, i, in);
  asm volatile("" : : "v"(in.x), "v"(in.y), "v"(in.z), "v"(in.c[0]), "v"(in.c[1]), "v"(in.c[2]), "v"(in.c[3]),
               "v"(in.c[4]), "v"(in.c[5]), "v"(in.qw), "v"(in.op));
  // 2. the block's SH-rest rows, [nv][rest_stride] floats, contiguous in the leaf: 64-float4 chunks per wave
  const int64_t nv = min((int64_t)blockDim.x, g.P - i0);
  const int64_t total = nv * g.rest_stride;  // i0 * rest_stride * 4 B is 16-B aligned (i0 % 256 == 0)
  const int64_t n4 = total / 4;
  const float* rows = g.rest - lead + i0 * g.rest_stride;  // stage_lead
  const float4* src4 = reinterpret_cast<const float4*>(rows);
  float4* dst4 = reinterpret_cast<float4*>(s_sh);
  for (int64_t c = w; c * 64 < n4; c += 4) {
    const int64_t e = min(c * 64 + lane, n4 - 1);  // past the rows: re-read the last float4 (its slot is unused)
    glds16(src4 + e, dst4 + c * 64);
  }
  // 3. the geometry while the rows land
  PreOut o;
  o.depth = 0.f;
  const bool vis = live && preprocess_core<RAW, false>(v, g, i, in, o);
  // 4. the DMA landed (the barrier's vmcnt(0)); a row tail that is not a whole float4 (last block only) by plain loads
  __syncthreads();
  if (n4 * 4 < total) {
    for (int64_t e = n4 * 4 + tid; e < total; e += blockDim.x) s_sh[e] = rows[e];
    __syncthreads();
  }
  if (!live) return;
  tiles[i] = 0u;
  depth_key[i] = 0xFFFFFFFFu;
  if (radii_out) radii_out[i] = 0;
  if (o.depth > 0.2f) depth_key[i] = __float_as_uint(o.depth);  // as k_preprocess: every Gaussian before the near plane
  if (!vis) return;
  g.rest = s_sh + lead;
  g.rest_base = i0;
  preprocess_color(v, g, i, in, o);
  const float4 r0 = make_float4(o.x, o.y, o.conic[0], o.conic[1]);
  const float4 r1 = make_float4(o.conic[2], o.opac, o.rgb[0], o.rgb[1]);
  const float4 r2 = make_float4(o.rgb[2], 1.0f / o.depth, __uint_as_float(o.clamped), o.tq);
  rec[RECS * i + 0] = r0;
  rec[RECS * i + 1] = r1;
  rec[RECS * i + 2] = r2;
  tiles[i] = (uint32_t)((o.rmax_x - o.rmin_x) * (o.rmax_y - o.rmin_y));
  const uint2 rc = make_uint2((uint32_t)o.rmin_x | ((uint32_t)o.rmin_y << 16), (uint32_t)o.rmax_x | ((uint32_t)o.rmax_y << 16));
  rect[i] = rc;
  // the rect again in the record's padding slot: k_duplicate's random per-Gaussian read is then one 64-B record
  // (one cache line) instead of the record and a rect line
  rec[RECS * i + 3] = make_float4(__uint_as_float(rc.x), __uint_as_float(rc.y), 0.f, 0.f);
  clampw[i] = o.clamped;
  if (radii_out) radii_out[i] = o.radius;
}

// k_preprocess_dma for up to MAX_PRE_VIEWS views in one pass over the Gaussians (gslm_preprocess_views: the line
// search's parameter sets over a batch of validation views).  A view's inputs cost 236 B per Gaussian at SH 3 against
// 84 B of its outputs; the block loads its Gaussians' inputs and stages their SH rows once, then writes every view's
// records, depth keys, tile counts and rects from them.  Per view the same functions in the same order as
// k_preprocess_dma: bitwise the same geometry.
// STAGE: the block's SH-rest rows are staged in LDS by LDS-DMA (views_pass_ok); otherwise (SH degree 0, colours or
// cov3D given, an odd layout) every view reads its inputs from global memory -- the same outputs, depth space included.
template <bool RAW, bool STAGE>
__global__ __launch_bounds__(256) void k_preprocess_views(PreViewsK pv, GaussK g) {
  extern __shared__ __attribute__((aligned(16))) float s_sh[];  // [256 * rest_stride] (STAGE)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const bool live = i < g.P;
  PreIn in{};
  if (live) load_pre_in<RAW>(g, i, in);
  asm volatile("" : : "v"(in.x), "v"(in.y), "v"(in.z), "v"(in.c[0]), "v"(in.c[1]), "v"(in.c[2]), "v"(in.c[3]),
               "v"(in.c[4]), "v"(in.c[5]), "v"(in.qw), "v"(in.op));
  int64_t total = 0, n4 = 0;
  if constexpr (STAGE) {
    const int64_t nv = min((int64_t)blockDim.x, g.P - i0);
    total = nv * g.rest_stride;
    n4 = total / 4;
    const float4* src4 = reinterpret_cast<const float4*>(g.rest + i0 * g.rest_stride);
    float4* dst4 = reinterpret_cast<float4*>(s_sh);
    for (int64_t c = w; c * 64 < n4; c += 4) {
      const int64_t e = min(c * 64 + lane, n4 - 1);
      glds16(src4 + e, dst4 + c * 64);
    }
  }
  // view 0's geometry while the rows land (as k_preprocess_dma)
  PreOut o0;
  o0.depth = 0.f;
  const bool vis0 = live && preprocess_core<RAW, false>(pv.v[0], g, i, in, o0);
  if constexpr (STAGE) {
    __syncthreads();
    if (n4 * 4 < total) {
      for (int64_t e = n4 * 4 + tid; e < total; e += blockDim.x) s_sh[e] = g.rest[i0 * g.rest_stride + e];
      __syncthreads();
    }
  }
  if (!live) return;
  if constexpr (STAGE) {
    g.rest = s_sh;
    g.rest_base = i0;
  }
#pragma unroll 1
  for (int b = 0; b < pv.n; ++b) {
    const ViewK& v = pv.v[b];
    const PreOutBufs& ob = pv.out[b];
    PreOut o;
    bool vis;
    if (b == 0) {
      o = o0;
      vis = vis0;
    } else {
      o.depth = 0.f;
      vis = preprocess_core<RAW, false>(v, g, i, in, o);
    }
    if (ob.pos) {
      // depth space (the line search's union lists): the render record alone, at the Gaussian's depth position, its
      // rect slot zero when culled -- one 64-B record per Gaussian, read in depth order by the union binning
      float4* rec = ob.rec + RECS * (size_t)ob.pos[i];
      if (vis) {
        preprocess_color(v, g, i, in, o);
        rec[0] = make_float4(o.x, o.y, o.conic[0], o.conic[1]);
        rec[1] = make_float4(o.conic[2], o.opac, o.rgb[0], o.rgb[1]);
        rec[2] = make_float4(o.rgb[2], 1.0f / o.depth, __uint_as_float(o.clamped), o.tq);
        rec[3] = make_float4(__uint_as_float((uint32_t)o.rmin_x | ((uint32_t)o.rmin_y << 16)),
                             __uint_as_float((uint32_t)o.rmax_x | ((uint32_t)o.rmax_y << 16)), 0.f, 0.f);
      } else {
        rec[3] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      continue;
    }
    ob.tiles[i] = 0u;
    ob.depth_key[i] = o.depth > 0.2f ? __float_as_uint(o.depth) : 0xFFFFFFFFu;
    if (!vis) continue;
    preprocess_color(v, g, i, in, o);
    float4* rec = ob.rec + RECS * i;
    rec[0] = make_float4(o.x, o.y, o.conic[0], o.conic[1]);
    rec[1] = make_float4(o.conic[2], o.opac, o.rgb[0], o.rgb[1]);
    rec[2] = make_float4(o.rgb[2], 1.0f / o.depth, __uint_as_float(o.clamped), o.tq);
    ob.tiles[i] = (uint32_t)((o.rmax_x - o.rmin_x) * (o.rmax_y - o.rmin_y));
    const uint2 rc = make_uint2((uint32_t)o.rmin_x | ((uint32_t)o.rmin_y << 16), (uint32_t)o.rmax_x | ((uint32_t)o.rmax_y << 16));
    ob.rect[i] = rc;
    rec[3] = make_float4(__uint_as_float(rc.x), __uint_as_float(rc.y), 0.f, 0.f);
    ob.clampw[i] = o.clamped;
  }
}

// whether k_preprocess_views can stage the SH rows: raw GaussianModel leaves with the SH rest as its contiguous 16-B
// aligned leaf (otherwise the unstaged instantiation runs; until round 5 a per-view launch_preprocess did, which
// ignored the depth positions of the line search's union workspaces: ADVICE r04)
static bool views_pass_ok(const GaussK& g) {
  return g.raw && !g.colors && !g.cov3D && g.rest && g.M > 1 && g.rest_stride == 3 * (g.M - 1) &&
         ((uintptr_t)g.rest & 15u) == 0;
}

int launch_preprocess_views(const PreViewsK& pv, const GaussK& g, const GeomBufs* gbs, hipStream_t s) {
  (void)gbs;
  if (g.P == 0 || pv.n == 0) return GSLM_OK;
  const dim3 grid((unsigned)((g.P + 255) / 256));
  if (views_pass_ok(g)) {
    const size_t lds = (size_t)256 * g.rest_stride * sizeof(float);
    hipLaunchKernelGGL((k_preprocess_views<true, true>), grid, dim3(256), lds, s, pv, g);
  } else if (g.raw) {  // every layout and both output spaces (depth positions included): no per-view fallback
    hipLaunchKernelGGL((k_preprocess_views<true, false>), grid, dim3(256), 0, s, pv, g);
  } else {
    hipLaunchKernelGGL((k_preprocess_views<false, false>), grid, dim3(256), 0, s, pv, g);
  }
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// One block per 256 consecutive Gaussians of the depth order: their (tile, id) pairs are one contiguous
// output range, written by the whole block in element order (coalesced, and a large Gaussian's tiles are
// spread over the block instead of one thread's loop).  Element e belongs to the last Gaussian whose
// local offset is <= e (binary search in LDS); inside a Gaussian the rect is walked row-major.
// n_dev (or NULL): N is the list capacity and *n_dev the pair count (the depth-order scan's total, not read back
// by the host: gslm_rasterize_dev); pairs past the capacity are not written (the host sees the count and renders
// that view again with a larger list)
// zero_ranges (ntiles of them): the tile ranges the binning's k_ranges fills afterwards, zeroed here by a grid-stride
// store (every range left [0, 0) stays an empty tile) -- one memset launch less per binning
__device__ __forceinline__ void zero_tile_ranges(uint2* __restrict__ ranges, int ntiles) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x)
    ranges[t] = make_uint2(0u, 0u);
}

__global__ __launch_bounds__(256) void k_duplicate(int64_t P, int gx, const uint32_t* __restrict__ sorted_idx,
                                                    const uint32_t* __restrict__ offsets, uint32_t N,
                                                    const uint32_t* __restrict__ n_dev,
                                                    const uint2* __restrict__ rect, const float4* __restrict__ rec,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    uint2* __restrict__ zero_ranges, int ntiles) {
  __shared__ QuadCull s_q[256];
  __shared__ uint32_t s_off[257];
  __shared__ uint32_t s_g[256];
  __shared__ uint32_t s_rc[256][3];  // x0, y0, width
  zero_tile_ranges(zero_ranges, ntiles);
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * 256, s = s0 + tid;
  const int64_t slast = min(s0 + 255, P - 1);
  const uint32_t base = offsets[s0];
  const uint32_t Ntot = n_dev ? *n_dev : N;
  uint32_t n = 0;
  if (s < P) {
    const uint32_t g = sorted_idx[s];
    // the tile count from the depth-order scan (coalesced) instead of tiles[g] (a random line per Gaussian);
    // culled Gaussians (n = 0) then touch nothing else
    const uint32_t o = offsets[s];
    n = (s + 1 < P ? offsets[s + 1] : Ntot) - o;
    s_off[tid] = o - base;
    if (n) {
      const float4 r3 = rec[RECS * (int64_t)g + 3];  // the rect (k_preprocess' copy in the record's padding)
      const uint2 rc = make_uint2(__float_as_uint(r3.x), __float_as_uint(r3.y));
      const int x0 = rc.x & 0xFFFF, y0 = rc.x >> 16, x1 = rc.y & 0xFFFF;
      s_rc[tid][0] = (uint32_t)x0;
      s_rc[tid][1] = (uint32_t)y0;
      s_rc[tid][2] = (uint32_t)(x1 - x0);
      s_g[tid] = g;
      const float4 r0 = rec[RECS * (int64_t)g + 0];
      s_q[tid] = quad_cull_prep(r0.x, r0.y, r0.z, r0.w, rec[RECS * (int64_t)g + 1].x, rec[RECS * (int64_t)g + 2].w);
    }
  } else {
    s_off[tid] = 0xFFFFFFFFu;  // past the block's last Gaussian: never an owner
  }
  if (s == slast) s_off[256] = offsets[s] - base + n;
  __syncthreads();
  // the block's pairs [base, base + total), clipped to the capacity (a no-op when N is the count)
  const uint32_t total = base < N ? min(s_off[256], N - base) : 0u;
  for (uint32_t e = tid; e < total; e += 256) {
    // last t with s_off[t] <= e (s_off[0] = 0; non-decreasing, 0xFFFFFFFF past the block's last Gaussian): 8 fixed
    // steps, no divergent loop (its per-lane exit made every step a few scalar exec-mask instructions)
    int lo = 0;
#pragma unroll
    for (int step = 128; step > 0; step >>= 1) lo = s_off[lo + step] <= e ? lo + step : lo;
    const uint32_t li = e - s_off[lo];
    const uint32_t w = s_rc[lo][2];
    const uint32_t dy = li / w;
    const int tx = (int)(s_rc[lo][0] + (li - dy * w)), ty = (int)(s_rc[lo][1] + dy);
    keys[base + e] = (uint32_t)(ty * gx + tx);
    vals[base + e] = s_g[lo] | (quad_mask(s_q[lo], tx, ty) << ID_BITS);
  }
}

// Launch order of the tile passes: tiles by descending list length (a longest-first schedule, so the
// costliest tiles do not start last and set the kernel's tail).  One block; buckets of the length
// (exact below 768 entries, 32-wide above), order inside a bucket arbitrary.  Only scheduling
// changes: every tile's results are independent of when it runs.
// cost (or NULL): a per-tile cost key instead of the list length (k_tile_cost: the LM product's modelled wave-visits).
__global__ __launch_bounds__(1024) void k_tile_order(int ntiles, const uint2* __restrict__ ranges,
                                                      uint32_t* __restrict__ order, const uint32_t* __restrict__ cost) {
  __shared__ uint32_t s_cnt[1024];
  const int tid = threadIdx.x;
  s_cnt[tid] = 0u;
  __syncthreads();
  auto bucket = [&](int t) {
    const uint32_t n = cost ? cost[t] : ranges[t].y - ranges[t].x;
    return 1023u - (n < 768u ? n : min(1023u, 768u + ((n - 768u) >> 5)));  // heaviest first
  };
  for (int t = tid; t < ntiles; t += 1024) atomicAdd(&s_cnt[bucket(t)], 1u);
  __syncthreads();
  // exclusive scan of the 1024 bucket counts: each wave's 64 by shuffles, then the 16 wave totals (two barriers;
  // a block-wide Hillis-Steele scan took 20)
  __shared__ uint32_t s_wsum[16];
  const int lane = tid & 63, w = tid >> 6;
  const uint32_t v = s_cnt[tid];
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_wsum[w] = inc;
  __syncthreads();
  uint32_t wbase = 0u;
  for (int k = 0; k < w; ++k) wbase += s_wsum[k];
  s_cnt[tid] = wbase + inc - v;  // exclusive
  __syncthreads();
  for (int t = tid; t < ntiles; t += 1024) order[atomicAdd(&s_cnt[bucket(t)], 1u)] = (uint32_t)t;
}

// XCD-aware form of the launch order (the LM product's).  Blocks are dealt round-robin over the 8
// XCDs, so blocks b and b + 8 share one XCD's L2 (MI355X_MICROARCH.md §Workgroup dispatch: observed, a speed choice,
// never correctness).  The tiles are cut, in row-major order, into XG contiguous bands of equal total weight (the
// cost key, or the list length, + 1), band g longest-first as k_tile_order orders the whole frame, and band g's k-th
// tile launched as block 8 k + g while every band still has tiles (the bands' leftover, cheapest tiles close the
// order).  Each XCD then gathers the records of about an eighth of the frame's Gaussians instead of all of them.
constexpr int XG = 8;
__global__ __launch_bounds__(1024) void k_tile_order_xcd(int ntiles, const uint2* __restrict__ ranges,
                                                          uint32_t* __restrict__ order,
                                                          const uint32_t* __restrict__ cost) {
  __shared__ uint32_t s_cnt[XG][1024];
  __shared__ unsigned long long s_w64[16];
  __shared__ uint32_t s_w32[16];
  __shared__ uint32_t s_n[XG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto len = [&](int t) { return cost ? cost[t] : ranges[t].y - ranges[t].x; };
  auto bucket = [&](uint32_t n) { return 1023u - (n < 768u ? n : min(1023u, 768u + ((n - 768u) >> 5))); };
  // 1. each thread a contiguous run of tiles: its weight, the block-wide exclusive prefix of the runs' weights
  const int seg = (ntiles + 1023) / 1024, t0 = min(ntiles, tid * seg), t1 = min(ntiles, t0 + seg);
  unsigned long long mine = 0ull;
  for (int t = t0; t < t1; ++t) mine += (unsigned long long)len(t) + 1ull;
  unsigned long long inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_w64[w] = inc;
#pragma unroll
  for (int g = 0; g < XG; ++g) s_cnt[g][tid] = 0u;
  __syncthreads();
  unsigned long long before = 0ull, total = 0ull;
  for (int k = 0; k < 16; ++k) {
    if (k < w) before += s_w64[k];
    total += s_w64[k];
  }
  before += inc - mine;
  // band of a tile: where the middle of its weight falls in the frame's total
  auto band = [&](unsigned long long pre, uint32_t wt) {
    return (int)min((unsigned long long)(XG - 1), ((2ull * pre + wt) * XG) / (2ull * total));
  };
  // 2. histogram of (band, length bucket)
  {
    unsigned long long pre = before;
    for (int t = t0; t < t1; ++t) {
      const uint32_t n = len(t);
      atomicAdd(&s_cnt[band(pre, n + 1u)][bucket(n)], 1u);
      pre += n + 1u;
    }
  }
  __syncthreads();
  // 3. per band, the exclusive scan of its 1024 bucket counts (the existing k_tile_order scan, once per band)
  for (int g = 0; g < XG; ++g) {
    const uint32_t v = s_cnt[g][tid];
    uint32_t inc32 = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc32, o, 64);
      if (lane >= o) inc32 += y;
    }
    if (lane == 63) s_w32[w] = inc32;
    __syncthreads();
    uint32_t wbase = 0u, tot = 0u;
    for (int k = 0; k < 16; ++k) {
      if (k < w) wbase += s_w32[k];
      tot += s_w32[k];
    }
    s_cnt[g][tid] = wbase + inc32 - v;
    if (tid == 0) s_n[g] = tot;
    __syncthreads();
  }
  // 4. each tile's rank in its band -> its block
  uint32_t m = s_n[0];
#pragma unroll
  for (int g = 1; g < XG; ++g) m = min(m, s_n[g]);
  unsigned long long pre = before;
  for (int t = t0; t < t1; ++t) {
    const uint32_t n = len(t);
    const int g = band(pre, n + 1u);
    pre += n + 1u;
    const uint32_t r = atomicAdd(&s_cnt[g][bucket(n)], 1u);
    uint32_t b;
    if (r < m) {
      b = r * XG + (uint32_t)g;
    } else {
      b = m * XG + (r - m);
      for (int h = 0; h < g; ++h) b += s_n[h] - m;
    }
    order[b] = (uint32_t)t;
  }
}

// the launch order of a tile pass: by the LM product's modelled cost (cost != NULL) k_tile_order_xcd, unless
// GSLM_TILE_ORDER=flat (A/B); by list length (the forward, the loss blends) the frame-wide k_tile_order -- banded by
// length the blends ran 11-15% slower (profiles/r05/ab/tile_order_xcd_lm_kept/): a list's length does not price a
// blend that stops at T < 1e-4, so equal-length bands are unequal work for their XCDs, while the modelled cost does
static bool tile_order_xcd() {
  static const bool on = [] {
    const char* e = getenv("GSLM_TILE_ORDER");
    return !(e && std::string(e) == "flat");
  }();
  return on;
}
int launch_tile_order(int ntiles, const uint2* ranges, uint32_t* order, const uint32_t* cost, hipStream_t s) {
  if (cost && tile_order_xcd())
    hipLaunchKernelGGL(k_tile_order_xcd, dim3(1), dim3(1024), 0, s, ntiles, ranges, order, cost);
  else
    hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, s, ntiles, ranges, order, cost);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// Gaussian ids of the sorted list (mask bits stripped), for gslm_inspect.
__global__ __launch_bounds__(256) void k_point_ids(int64_t N, const uint32_t* __restrict__ pl, uint32_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < N) out[k] = pl_id(pl[k]);
}

// n_dev (or NULL): as k_duplicate (N the capacity, *n_dev the count); n_out (or NULL) receives the count.
// RANGES_KEYS consecutive keys per thread from one 16-B load (the list's key buffers are 256-B aligned), the keys just
// before and after the group from memory (the neighbouring threads' loads: cache hits): a quarter of the threads of a
// key per thread, each with one vector load instead of three scalar ones.
constexpr int RANGES_KEYS = 4;
__global__ __launch_bounds__(256) void k_ranges(int64_t N, const uint32_t* __restrict__ keys,
                                                 uint2* __restrict__ ranges, const uint32_t* __restrict__ n_dev,
                                                 uint32_t* __restrict__ n_out) {
  const int64_t k0 = RANGES_KEYS * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (n_dev) {
    const uint32_t c = *n_dev;
    if (n_out && k0 == 0) *n_out = c;
    N = min(N, (int64_t)c);
  }
  if (k0 >= N) return;
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // never a tile id: a list edge
  uint32_t t[RANGES_KEYS];
  if (k0 + RANGES_KEYS <= N) {
    const uint4 v = *reinterpret_cast<const uint4*>(keys + k0);
    t[0] = v.x, t[1] = v.y, t[2] = v.z, t[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < RANGES_KEYS; ++j) t[j] = k0 + j < N ? keys[k0 + j] : NONE;
  }
  const uint32_t before = k0 > 0 ? keys[k0 - 1] : NONE;
  const uint32_t after = k0 + RANGES_KEYS < N ? keys[k0 + RANGES_KEYS] : NONE;
#pragma unroll
  for (int j = 0; j < RANGES_KEYS; ++j) {
    if (t[j] == NONE) break;  // past the list's end
    const uint32_t p = j ? t[j - 1] : before, q = j + 1 < RANGES_KEYS ? t[j + 1] : after;
    if (p != t[j]) ranges[t[j]].x = (uint32_t)(k0 + j);
    if (q != t[j]) ranges[t[j]].y = (uint32_t)(k0 + j + 1);
  }
}

// ---- the LM row map (ScratchBufs::hscan), once per geometry ----
// Computed by the first LM product on a geometry (GSLM_MV_TAIL_CLEAN protocol), not by the forward: the
// goff / rect gathers are random over 12 B per Gaussian and the drop-in backward does not need the map.
// largest n_contrib over each tile quadrant's pixels (wave q's 8x8 block, tile_pixel): list positions at or past it
// are blended by no pixel of that quadrant
__global__ __launch_bounds__(256) void k_tile_neff(ViewK v, const uint32_t* __restrict__ n_contrib,
                                                    uint32_t* __restrict__ neff) {
  const int tile = blockIdx.x, tile_x = tile % v.gx, tile_y = tile / v.gx;
  int px, py;
  tile_pixel(tile_x, tile_y, threadIdx.x, px, py);
  int wm = (px < v.W && py < v.H) ? (int)n_contrib[(int64_t)py * v.W + px] : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) wm = max(wm, __shfl_xor(wm, o));
  if ((threadIdx.x & 63) == 0) neff[4 * tile + (threadIdx.x >> 6)] = (uint32_t)wm;
}

// The LM product's cost of a tile, in wave-visits (k_render_matvec's schedule model): the J v pass runs one
// independent wave per quadrant, so its busiest wave -- the largest count over quadrants q of the list positions
// below the quadrant's bound neff[q] whose mask holds q -- sets its time; the VJP pass runs 128-entry batches from
// max_q neff down with a block barrier around each, so every batch costs its busiest wave's count.  Cost = the two
// summed.  Tiles ordered by it (k_tile_order) schedule the product's blocks longest-first by what they actually do:
// the list length, the forward's key, ranks them by entries no LM pass visits (tools/exp/tile_sched.py: modelled
// idle tail 11.8% of the launch by length, 5.3% by this cost).  One block per tile; threads 0..127 take batch b,
// 128..255 batch b + 1 (two waves per batch).
__global__ __launch_bounds__(256) void k_tile_cost(const uint2* __restrict__ ranges,
                                                    const uint32_t* __restrict__ point_list,
                                                    const uint32_t* __restrict__ neff, uint32_t* __restrict__ cost) {
  __shared__ uint32_t s_c[4][4];  // [wave][quadrant] counts of the current pair of batches
  const int tile = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
  const uint2 r = ranges[tile];
  const uint32_t len = r.y - r.x;
  uint32_t wm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) wm[q] = min(neff[4 * tile + q], len);
  const int n_eff = (int)max(max(wm[0], wm[1]), max(wm[2], wm[3]));
  uint32_t tot[4] = {0u, 0u, 0u, 0u}, vjp = 0u;
  for (int base = 0; base < n_eff; base += 256) {
    // batch b = base / 128 + (tid >> 7): list position n_eff - 1 - (base + tid)
    const int pos = n_eff - 1 - (base + tid);
    uint32_t m = 0u;
    if (pos >= 0) {
      const uint32_t e = point_list[r.x + pos];
      m = pl_mask(e) & (((uint32_t)pos < wm[0] ? 1u : 0u) | ((uint32_t)pos < wm[1] ? 2u : 0u) |
                        ((uint32_t)pos < wm[2] ? 4u : 0u) | ((uint32_t)pos < wm[3] ? 8u : 0u));
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t c = (uint32_t)__popcll(__ballot((m >> q) & 1u));
      if ((tid & 63) == 0) s_c[w][q] = c;
    }
    __syncthreads();
    uint32_t b0 = 0u, b1 = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t c0 = s_c[0][q] + s_c[1][q], c1 = s_c[2][q] + s_c[3][q];
      tot[q] += c0 + c1;
      b0 = max(b0, c0);
      b1 = max(b1, c1);
    }
    vjp += b0 + b1;
    __syncthreads();
  }
  if (tid == 0) cost[tile] = max(max(tot[0], tot[1]), max(tot[2], tot[3])) + vjp;
}

// The quadrants whose pixels still blend at list position pos (vjp_tile's per-wave bounds) and the entry's
// effective mask: its quadrant mask restricted to them.  A head entry is one with a non-empty effective mask.
__device__ __forceinline__ uint32_t eff_mask(uint32_t e, uint32_t pos, const uint32_t* wm4) {
  const uint32_t wb = (pos < wm4[0] ? 1u : 0u) | (pos < wm4[1] ? 2u : 0u) | (pos < wm4[2] ? 4u : 0u) |
                      (pos < wm4[3] ? 8u : 0u);
  return pl_mask(e) & wb;
}

// head flag of every sorted entry at its goff-order slot, and the goff slot itself in slots[k]
__global__ __launch_bounds__(256) void k_row_flags(int64_t N, int gx, const uint32_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ point_list,
                                                    const uint2* __restrict__ ranges, const uint32_t* __restrict__ neff,
                                                    const uint32_t* __restrict__ goff, const uint2* __restrict__ rect,
                                                    uint32_t* __restrict__ slots, uint32_t* __restrict__ flags) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  const uint32_t t = keys[k];
  const uint32_t e = point_list[k];
  const uint32_t g = pl_id(e);
  const uint32_t o = row_slot(goff[g], rect[g], (int)(t % (uint32_t)gx), (int)(t / (uint32_t)gx));
  slots[k] = o;
  flags[o] = eff_mask(e, (uint32_t)k - ranges[t].x, neff + 4 * (size_t)t) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_row_final(int64_t N, const uint32_t* __restrict__ hscan,
                                                    uint32_t* __restrict__ slots) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < N) slots[k] = hscan[slots[k]];  // non-heads get the next head's slot; they are never written
}

int launch_lm_rowmap(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb,
                     int64_t N, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (N <= 0 || ntiles == 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(sb.hscan, 0, sizeof(uint32_t), s));
    return GSLM_OK;
  }
  const unsigned nb = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_tile_neff, dim3(ntiles), dim3(TILE_PIX), 0, s, v, ib.n_contrib, bb.tile_neff);
  if (N + 1 >= ntiles) {
    // the LM tile passes' launch order by their modelled cost (hscan holds the costs until k_row_flags rewrites it;
    // only the schedule changes, every tile's results are independent of when it runs)
    hipLaunchKernelGGL(k_tile_cost, dim3(ntiles), dim3(256), 0, s, bb.ranges, bb.point_list, bb.tile_neff, sb.hscan);
    if (int st = launch_tile_order(ntiles, bb.ranges, bb.tile_order, sb.hscan, s)) return st;
  }
  hipLaunchKernelGGL(k_row_flags, dim3(nb), dim3(256), 0, s, N, v.gx, bb.keys_sorted, bb.point_list, bb.ranges,
                     bb.tile_neff, gb.goff, gb.rect, bb.slots, sb.hscan);
  GSLM_LAUNCH_CHECK();
  // in place (exclusive_scan_u32 picks k_scan_apply_inplace: no __restrict__ aliasing of in and out)
  const int st = exclusive_scan_u32(sb.hscan, nullptr, sb.hscan, N, sb.scan_tmp, sb.hscan + N, s);
  if (st) return st;
  hipLaunchKernelGGL(k_row_final, dim3(nb), dim3(256), 0, s, N, sb.hscan, bb.slots);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// ---- the line search's shared binning (gslm_union_*) ----
// The seven line-search points of train_jvp.py:262-280 differ only in the groups the LM step moves (xyz is masked,
// :221-227), so one view's Gaussians keep their screen centre and depth order at every point and only their
// footprints change.  Each point's exact point list -- the (tile, Gaussian) pairs of its rects in (tile, depth,
// index) order -- is then the subsequence of ONE list binned over the union of the points' rects: the entries whose
// tile lies in that point's rect.  k_duplicate_union gives every entry 4 bits per point: that point's quadrant mask
// (quad_mask of its own record, the bits its exact k_duplicate would write) where the tile is in its rect, 0
// elsewhere; the tile sort carries them with the pairs.  A blend that visits by those bits visits the exact list's
// entries, in its order, with the same records: the same image and loss, bitwise (gslm_rasterize_loss_slot).

// The union list is built in DEPTH SPACE: the sets' records sit at their Gaussians' depth positions s (gslm_preprocess_
// views with depth positions), so every pass below reads them coalesced in s and the point list's values are depth
// positions.  The blend indexes the set's records by them (the same records, the same (tile, depth, index) order).

// k_depth_positions: pos[order[s]] = s (the depth order's inverse)
__global__ __launch_bounds__(256) void k_depth_positions(int64_t P, const uint32_t* __restrict__ order,
                                                          uint32_t* __restrict__ pos) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < P) pos[order[s]] = (uint32_t)s;
}

// per depth position: the union of the sets' rects (a culled set's rect slot is zero), as the union geometry's tile
// count and rect
__global__ __launch_bounds__(256) void k_union_rect(int64_t P, UnionSets u, uint32_t* __restrict__ utiles,
                                                     uint2* __restrict__ urect) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  uint32_t x0 = 0xFFFFu, y0 = 0xFFFFu, x1 = 0u, y1 = 0u;
  for (int a = 0; a < u.n; ++a) {
    const float4 r3 = u.rec[a][RECS * i + 3];
    const uint32_t lo = __float_as_uint(r3.x), hi = __float_as_uint(r3.y);
    if (hi == 0u) continue;  // culled in set a
    x0 = min(x0, lo & 0xFFFFu);
    y0 = min(y0, lo >> 16);
    x1 = max(x1, hi & 0xFFFFu);
    y1 = max(y1, hi >> 16);
  }
  const bool any = x1 > x0 && y1 > y0;
  utiles[i] = any ? (x1 - x0) * (y1 - y0) : 0u;
  urect[i] = any ? make_uint2(x0 | (y0 << 16), x1 | (y1 << 16)) : make_uint2(0u, 0u);
}

// k_duplicate over the union rects in depth space (the same emission as k_duplicate: one block per DUPU_G depth
// positions, elements in order, a Gaussian's rect row-major), the value the depth position with quadrant bits 0xF,
// and amask[e] = bits 4a..4a+3 the quadrant mask of set a.  Each (Gaussian, set) quadrant test is prepared once
// (quad_cull_prep on the set's record, read coalesced in depth space) into LDS -- [ia b det ta] [ydom yr sqm mode]
// and the set's rect -- and every element evaluates quad_mask on it: the bits k_duplicate writes for that set's own
// list.  (Preparing per element was 6 square roots and 4 divisions per set and entry: 252 us per 1080p view at 1M,
// 5x the plain k_duplicate.)  The centre is the same in every set that keeps the Gaussian (the points share xyz and
// the view), so its copy in s_gxy is written by each such set with the same bits.  Quarter-size blocks keep the
// staging at NS * 2.5 KB of LDS (dynamic: NS * 2 * DUPU_G float4); DUPU_SPLIT threads share a Gaussian's sets.
#ifndef GSLM_DUPU_G
#define GSLM_DUPU_G 64  // 64: 15 KB of staging at six sets, 8 blocks per CU (union binning 0.290 -> 0.272 ms against 128)
#endif
constexpr int DUPU_G = GSLM_DUPU_G;
constexpr int DUPU_SPLIT = 256 / DUPU_G;  // threads per Gaussian in the staging
template <int NS>
__global__ __launch_bounds__(256) void k_duplicate_union(int64_t P, int gx, const uint32_t* __restrict__ offsets,
                                                          uint32_t N, const uint2* __restrict__ urect, UnionSets u,
                                                          uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                          uint32_t* __restrict__ amask, uint2* __restrict__ zero_ranges,
                                                          int ntiles) {
  extern __shared__ float4 s_set[];  // [NS][2][DUPU_G]
  zero_tile_ranges(zero_ranges, ntiles);
  __shared__ uint2 s_srect[NS][DUPU_G];
  __shared__ float2 s_gxy[DUPU_G];
  __shared__ uint32_t s_off[DUPU_G + 1];
  __shared__ uint32_t s_rc[DUPU_G][3];  // x0, y0, width of the union rect
  const int tid = threadIdx.x, gi = tid & (DUPU_G - 1), half = tid / DUPU_G;
  const int64_t s0 = (int64_t)blockIdx.x * DUPU_G, s = s0 + gi;
  const int64_t slast = min(s0 + DUPU_G - 1, P - 1);
  const uint32_t base = offsets[s0];
  uint32_t n = 0;
  if (s < P) {
    const uint32_t o = offsets[s];
    n = (s + 1 < P ? offsets[s + 1] : N) - o;
    if (half == 0) {
      s_off[gi] = o - base;
      if (n) {
        const uint2 rc = urect[s];
        const int x0 = rc.x & 0xFFFF, y0 = rc.x >> 16, x1 = rc.y & 0xFFFF;
        s_rc[gi][0] = (uint32_t)x0;
        s_rc[gi][1] = (uint32_t)y0;
        s_rc[gi][2] = (uint32_t)(x1 - x0);
      }
    }
    if (n) {
#pragma unroll
      for (int k = 0; k < (NS + DUPU_SPLIT - 1) / DUPU_SPLIT; ++k) {
        const int a = DUPU_SPLIT * k + half;
        if (a >= NS) break;
        const float4* r = u.rec[a] + RECS * (size_t)s;
        const float4 r0 = r[0], r3 = r[3];
        const float r1x = r[1].x, r2w = r[2].w;
        const uint2 rc = make_uint2(__float_as_uint(r3.x), __float_as_uint(r3.y));
        s_srect[a][gi] = rc;  // zero when set a culls the Gaussian (its other record fields are stale: unused)
        if (rc.y != 0u) {
          const QuadCull q = quad_cull_prep(r0.x, r0.y, r0.z, r0.w, r1x, r2w);
          s_set[(2 * a) * DUPU_G + gi] = make_float4(q.ia, q.b, q.det, q.ta);
          s_set[(2 * a + 1) * DUPU_G + gi] = make_float4(q.ydom, q.yr, q.sqm, __int_as_float(q.mode));
          s_gxy[gi] = make_float2(r0.x, r0.y);
        }
      }
    }
  } else if (half == 0) {
    s_off[gi] = 0xFFFFFFFFu;  // past the block's last Gaussian: never an owner
  }
  if (s == slast && half == 0) s_off[DUPU_G] = offsets[s] - base + n;
  __syncthreads();
  const uint32_t total = base < N ? min(s_off[DUPU_G], N - base) : 0u;
  for (uint32_t e = tid; e < total; e += 256) {
    int lo = 0;
#pragma unroll
    for (int step = DUPU_G / 2; step > 0; step >>= 1) lo = s_off[lo + step] <= e ? lo + step : lo;
    const uint32_t li = e - s_off[lo];
    const uint32_t w = s_rc[lo][2];
    const uint32_t dy = li / w;
    const int tx = (int)(s_rc[lo][0] + (li - dy * w)), ty = (int)(s_rc[lo][1] + dy);
    const float2 gxy = s_gxy[lo];
    uint32_t m = 0u;
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      const uint2 rc = s_srect[a][lo];
      if (tx < (int)(rc.x & 0xFFFFu) || ty < (int)(rc.x >> 16) || tx >= (int)(rc.y & 0xFFFFu) || ty >= (int)(rc.y >> 16))
        continue;  // outside set a's rect (an empty rect when set a culls the Gaussian)
      const float4 qa = s_set[(2 * a) * DUPU_G + lo], qb = s_set[(2 * a + 1) * DUPU_G + lo];
      QuadCull q;
      q.gx = gxy.x;
      q.gy = gxy.y;
      q.ia = qa.x;
      q.b = qa.y;
      q.det = qa.z;
      q.ta = qa.w;
      q.ydom = qb.x;
      q.yr = qb.y;
      q.sqm = qb.z;
      q.mode = __float_as_int(qb.w);
      m |= quad_mask(q, tx, ty) << (4 * a);
    }
    keys[base + e] = (uint32_t)(ty * gx + tx);
    vals[base + e] = (uint32_t)(s0 + lo) | (0xFu << ID_BITS);
    amask[base + e] = m;
  }
}

int launch_depth_positions(int64_t P, const uint32_t* order, uint32_t* pos, hipStream_t s) {
  if (P <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_depth_positions, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, order, pos);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_union_rect(int64_t P, const UnionSets& u, const GeomBufs& ug, hipStream_t s) {
  if (P <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_union_rect, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, u, ug.tiles, ug.rect);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_union_binning(const ViewK& v, int64_t P, const GeomBufs& ug, const BinBufs& bb, const UnionMasks& um,
                         int64_t N, const UnionSets& u, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (P == 0 || N == 0) GSLM_HIP_CHECK(hipMemsetAsync(bb.ranges, 0, (size_t)ntiles * sizeof(uint2), s));
  if (P > 0 && N > 0) {  // (k_duplicate_union also zeroes the tile ranges)
    const size_t lds = (size_t)u.n * 2 * DUPU_G * sizeof(float4);
    const dim3 grid((unsigned)((P + DUPU_G - 1) / DUPU_G));
    switch (u.n) {
#define GSLM_DUP_UNION(NS)                                                                                         \
  case NS:                                                                                                         \
    hipLaunchKernelGGL(k_duplicate_union<NS>, grid, dim3(256), lds, s, P, v.gx, ug.offsets, (uint32_t)N, ug.rect, u, \
                       bb.keys0, bb.vals0, um.m0, bb.ranges, ntiles);                                                \
    break;
      GSLM_DUP_UNION(1) GSLM_DUP_UNION(2) GSLM_DUP_UNION(3) GSLM_DUP_UNION(4)
      GSLM_DUP_UNION(5) GSLM_DUP_UNION(6) GSLM_DUP_UNION(7) GSLM_DUP_UNION(8)
#undef GSLM_DUP_UNION
      default:
        set_error("union binning: 1..8 parameter sets");
        return GSLM_ERR_INVALID;
    }
    GSLM_LAUNCH_CHECK();
    bool alt = false;
    int st = radix_sort_pairs(bb.keys0, bb.vals0, bb.keys1, bb.vals1, N, bb.end_bit, um.hist, &alt, s, false, nullptr,
                              nullptr, um.m0, um.m1);
    if (st != GSLM_OK) return st;
    if ((alt ? bb.vals1 : bb.vals0) != bb.point_list || (alt ? um.m1 : um.m0) != um.sorted) {
      set_error("internal: radix pass count disagrees with the union binning layout");
      return GSLM_ERR_INVALID;
    }
    const unsigned nbN = (unsigned)((N + 256 * RANGES_KEYS - 1) / (256 * RANGES_KEYS));
    hipLaunchKernelGGL(k_ranges, dim3(nbN), dim3(256), 0, s, N, bb.keys_sorted, bb.ranges, (const uint32_t*)nullptr,
                       (uint32_t*)nullptr);
    GSLM_LAUNCH_CHECK();
  }
  if (int st = launch_tile_order(ntiles, bb.ranges, bb.tile_order, nullptr, s)) return st;
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// ------------------------------------------------------------------ launchers

// k_preprocess_dma (default) or the register-staged k_preprocess: GSLM_PREPROCESS_STAGING=reg selects the latter
// (an A/B switch; both write the bitwise same records)
static const bool g_preprocess_dma = [] {
  const char* e = getenv("GSLM_PREPROCESS_STAGING");
  return !(e && e[0] == 'r');
}();

int launch_preprocess(const ViewK& v, const GaussK& g, const GeomBufs& gb, int* radii_out, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  const int nb = (int)((g.P + 255) / 256);
  // stage the SH rows through LDS: the contiguous [P, M-1, 3] rest leaf (raw GaussianModel tensors, or the dc / rest
  // pair of render(separate_sh=True)), or the rest inside upstream's [P, M, 3] features tensor (render()'s
  // get_features: each rest row 3 floats past its dc at one 3M stride) -- whole rows staged from the dc slot
  const int lead = stage_lead(g);
  const bool stage = lead >= 0;
  const size_t lds = stage ? (size_t)256 * g.rest_stride * sizeof(float) : 0;
  if (g.raw && stage && g_preprocess_dma)
    hipLaunchKernelGGL((k_preprocess_dma<true>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  else if (stage && g_preprocess_dma)
    hipLaunchKernelGGL((k_preprocess_dma<false>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  else if (g.raw && stage)
    hipLaunchKernelGGL((k_preprocess<true, true>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  else if (g.raw)
    hipLaunchKernelGGL((k_preprocess<true, false>), dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  else if (stage)
    hipLaunchKernelGGL((k_preprocess<false, true>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  else
    hipLaunchKernelGGL((k_preprocess<false, false>), dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.depth_key, gb.tiles,
                       gb.rect, gb.clampw, radii_out, lead);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_binning(const ViewK& v, int64_t P, const GeomBufs& gb, const BinBufs& bb, int64_t N, hipStream_t s,
                   bool device_count, uint32_t* n_out) {
  const int ntiles = v.gx * v.gy;
  // device_count: N is the list capacity, the pair count stays on the device (gb.counters[0])
  const uint32_t* n_dev = device_count ? gb.counters : nullptr;
  if (P > 0)  // (k_duplicate also zeroes the tile ranges)
    hipLaunchKernelGGL(k_duplicate, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, v.gx, gb.sorted_idx,
                       gb.offsets, (uint32_t)N, n_dev, gb.rect, gb.rec, bb.keys0, bb.vals0, bb.ranges, ntiles);
  else
    GSLM_HIP_CHECK(hipMemsetAsync(bb.ranges, 0, (size_t)ntiles * sizeof(uint2), s));
  GSLM_LAUNCH_CHECK();
  if (N == 0) {  // every range stays [0, 0); the tile passes still read a launch order
    if (n_out) {
      if (P > 0) GSLM_HIP_CHECK(hipMemcpyAsync(n_out, gb.counters, 4, hipMemcpyDeviceToDevice, s));
      else GSLM_HIP_CHECK(hipMemsetAsync(n_out, 0, 4, s));
    }
    if (int st = launch_tile_order(ntiles, bb.ranges, bb.tile_order, nullptr, s)) return st;
    GSLM_LAUNCH_CHECK();
    return GSLM_OK;
  }
  bool alt = false;
  int st = radix_sort_pairs(bb.keys0, bb.vals0, bb.keys1, bb.vals1, N, bb.end_bit, bb.hist, &alt, s, false, nullptr,
                            n_dev);
  if (st != GSLM_OK) return st;
  if ((alt ? bb.vals1 : bb.vals0) != bb.point_list) {
    set_error("internal: radix pass count disagrees with the binning layout");
    return GSLM_ERR_INVALID;
  }
  const unsigned nbN = (unsigned)((N + 256 * RANGES_KEYS - 1) / (256 * RANGES_KEYS));
  hipLaunchKernelGGL(k_ranges, dim3(nbN), dim3(256), 0, s, N, bb.keys_sorted, bb.ranges, n_dev, n_out);
  GSLM_LAUNCH_CHECK();
  if (int st = launch_tile_order(ntiles, bb.ranges, bb.tile_order, nullptr, s)) return st;
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_point_ids(const uint32_t* point_list, int64_t N, uint32_t* out, hipStream_t s) {
  if (N <= 0) return GSLM_OK;
  hipLaunchKernelGGL(k_point_ids, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, N, point_list, out);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
