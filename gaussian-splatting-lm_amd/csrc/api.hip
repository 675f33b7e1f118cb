// api.hip -- extern "C" entry points of libgslm.so (declared in include/gslm.h).
#include <cstring>
#include <string>
#include "gslm_kernels.hpp"

namespace gslm {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

thread_local DebugSync g_debug;

int launch_failed(hipError_t e, const char* file, int line) {
  const char* base = std::strrchr(file, '/');
  set_error(std::string(g_debug.on ? "kernel failed (debug mode: stream synchronised after the launch at " : "kernel launch (") +
            (base ? base + 1 : file) + ":" + std::to_string(line) + "): " + hipGetErrorString(e));
  return GSLM_ERR_HIP;
}

namespace {

struct Carver {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t count) {
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off = align_up(off + count * sizeof(T));
    return p;
  }
};

}  // namespace

size_t geom_layout(int64_t P, void* base, GeomBufs* o) {
  Carver c{(char*)base};
  GeomBufs g;
  g.rec = c.take<float4>((size_t)P * RECS);
  g.depth_key = c.take<uint32_t>(P);
  g.tiles = c.take<uint32_t>(P);
  g.rect = c.take<uint2>(P);
  g.vals_init = c.take<uint32_t>(P);
  g.sorted_idx = g.vals_init;
  g.keys_alt = c.take<uint32_t>(P);
  g.vals_alt = c.take<uint32_t>(P);
  g.offsets = c.take<uint32_t>(P);
  g.goff = c.take<uint32_t>(P);
  g.hist = c.take<uint32_t>(sort_hist_bytes(P) / 4);
  g.scan_tmp = c.take<uint32_t>(scan_tmp_bytes(P) / 4);
  g.counters = c.take<uint32_t>(16);
  g.clampw = c.take<uint32_t>(P);
  if (o) *o = g;
  return c.off;
}

size_t bin_layout(int64_t N, int ntiles, void* base, BinBufs* o) {
  Carver c{(char*)base};
  BinBufs b;
  b.keys0 = c.take<uint32_t>(N);
  b.keys1 = c.take<uint32_t>(N);
  b.vals0 = c.take<uint32_t>(N);
  b.vals1 = c.take<uint32_t>(N);
  b.hist = c.take<uint32_t>(sort_hist_bytes(N) / 4);
  b.ranges = c.take<uint2>(ntiles);
  b.tile_order = c.take<uint32_t>(ntiles);
  b.tile_neff = c.take<uint32_t>((size_t)4 * ntiles);
  b.end_bit = 1;
  while ((1ll << b.end_bit) < (long long)ntiles) ++b.end_bit;
  b.passes = (b.end_bit + 7) / 8;
  b.point_list = (b.passes & 1) ? b.vals1 : b.vals0;
  b.keys_sorted = (b.passes & 1) ? b.keys1 : b.keys0;
  b.slots = (b.passes & 1) ? b.keys0 : b.keys1;
  if (o) *o = b;
  return c.off;
}

size_t img_layout(int H, int W, void* base, ImgBufs* o) {
  Carver c{(char*)base};
  ImgBufs b;
  b.final_T = c.take<float>((size_t)H * W);
  b.n_contrib = c.take<uint32_t>((size_t)H * W);
  if (o) *o = b;
  return c.off;
}

size_t scratch_layout(int64_t P, int64_t N, void* base, ScratchBufs* o) {
  Carver c{(char*)base};
  ScratchBufs b;
  b.trec = c.take<float4>((size_t)P * REC_F4);
  b.contrib = c.take<float4>((size_t)N * REC_F4);
  b.hscan = c.take<uint32_t>((size_t)N + 1);
  b.scan_tmp = c.take<uint32_t>(scan_tmp_bytes(N) / 4);
  if (o) *o = b;
  return c.off;
}

static int make_view(const gslm_view* in, int M, ViewK* v) {
  if (!in) { set_error("view is NULL"); return GSLM_ERR_INVALID; }
  if (in->image_height <= 0 || in->image_width <= 0) { set_error("image size must be positive"); return GSLM_ERR_INVALID; }
  if (in->image_height > 65535 * 16 || in->image_width > 65535 * 16) { set_error("image too large"); return GSLM_ERR_INVALID; }
  if (in->sh_degree < 0 || in->sh_degree > 3) { set_error("sh_degree must be in [0,3]"); return GSLM_ERR_INVALID; }
  if (!(in->tanfovx > 0.0) || !(in->tanfovy > 0.0)) { set_error("tanfov must be positive"); return GSLM_ERR_INVALID; }
  v->H = in->image_height;
  v->W = in->image_width;
  v->gx = (v->W + TILE_X - 1) / TILE_X;
  v->gy = (v->H + TILE_Y - 1) / TILE_Y;
  v->focal_x = (float)((double)v->W / (2.0 * in->tanfovx));
  v->focal_y = (float)((double)v->H / (2.0 * in->tanfovy));
  v->limx = (float)(1.3 * in->tanfovx);
  v->limy = (float)(1.3 * in->tanfovy);
  std::memcpy(v->view, in->viewmatrix, sizeof(v->view));
  std::memcpy(v->proj, in->projmatrix, sizeof(v->proj));
  for (int k = 0; k < 3; ++k) { v->campos[k] = in->campos[k]; v->bg[k] = in->bg[k]; }
  v->scale_mod = (float)in->scale_modifier;
  v->D = in->sh_degree;
  v->M = M;
  v->antialiasing = in->antialiasing ? 1 : 0;
  v->exhaustive = in->debug ? 1 : 0;
  return GSLM_OK;
}

static int make_gauss(const gslm_gaussians* in, const ViewK* v, GaussK* g, bool tangent) {
  if (!in) { set_error("gaussians is NULL"); return GSLM_ERR_INVALID; }
  if (in->P < 0 || in->P > MAX_P) { set_error("P out of range [0, 2^28 - 1]"); return GSLM_ERR_INVALID; }
  g->P = in->P;
  g->raw = in->raw ? 1 : 0;
  g->M = in->max_coeffs;
  g->means3D = in->means3D;
  g->opac = in->opacities;
  g->scales = in->scales;
  g->rot = in->rotations;
  g->cov3D = in->cov3D_precomp;
  g->dc = in->sh_dc;
  g->dc_stride = in->sh_dc_stride;
  g->rest = in->sh_rest;
  g->rest_stride = in->sh_rest_stride;
  g->colors = in->colors_precomp;
  if (tangent || in->P == 0) return GSLM_OK;
  if (!g->means3D || !g->opac) { set_error("means3D and opacities are required"); return GSLM_ERR_INVALID; }
  if (!g->cov3D && !(g->scales && g->rot)) { set_error("need scales+rotations or cov3D_precomp"); return GSLM_ERR_INVALID; }
  if (!g->colors) {
    if (!g->dc) { set_error("need shs or colors_precomp"); return GSLM_ERR_INVALID; }
    if ((v->D + 1) * (v->D + 1) > g->M) { set_error("sh_degree exceeds stored coefficients"); return GSLM_ERR_INVALID; }
    if (g->M > 1 && !g->rest) { set_error("sh_rest is NULL"); return GSLM_ERR_INVALID; }
  }
  return GSLM_OK;
}

// order_mode (gslm_preprocess_ordered): 0 sort, 1 sort and copy the order out to depth_order, 2 take the order from
// depth_order instead of sorting
int do_preprocess(const ViewK& v, const GaussK& g, const GeomBufs& gb, int32_t* radii, hipStream_t s,
                  uint32_t* depth_order = nullptr, int order_mode = 0) {
  int st = launch_preprocess(v, g, gb, radii, s);
  if (st) return st;
  const int64_t P = g.P;
  if (P == 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(gb.counters, 0, 4, s));
    return GSLM_OK;
  }
  const uint32_t* tiles_sorted = nullptr;  // the tile counts in depth order, when the sort gathered them
  if (order_mode == 2) {
    GSLM_HIP_CHECK(hipMemcpyAsync(gb.sorted_idx, depth_order, (size_t)P * 4, hipMemcpyDeviceToDevice, s));
  } else {
    // depth sort of (key, index) pairs: the first scatter generates the indices (no iota pass), the last writes
    // tiles[index] where the sorted keys would go.  key_range: the passes sort the bytes of key - min and those past
    // the frame's span run as copies (the 32-bit order exactly; sort.hip KeyRange): 3 working passes at the bench
    // scene's depths, -7 us per forward (profiles/r06/ab_depth_key_range/; routing the working passes through a third
    // buffer pair instead of copying measured the same).  (Round 6 also measured 3 passes of 11-bit digits against 4 of
    // 8 bits: 90.9 against 90.8 us per 1M keys -- the 2048-digit scatter and scan cost what the fourth pass did --
    // profiles/r06/ab_depth_sort_d11_neutral/.)
    bool alt = false;
    st = radix_sort_pairs(gb.depth_key, gb.vals_init, gb.keys_alt, gb.vals_alt, P, 32, gb.hist, &alt, s, true, gb.tiles,
                          nullptr, nullptr, nullptr, true);
    if (st) return st;
    if (alt) GSLM_HIP_CHECK(hipMemcpyAsync(gb.sorted_idx, gb.vals_alt, (size_t)P * 4, hipMemcpyDeviceToDevice, s));
    tiles_sorted = alt ? gb.keys_alt : gb.depth_key;
    if (order_mode == 1)
      GSLM_HIP_CHECK(hipMemcpyAsync(depth_order, gb.sorted_idx, (size_t)P * 4, hipMemcpyDeviceToDevice, s));
  }
  // tile-count scans in index order (gradient-row offsets goff) and in depth order (duplicate offsets)
  return exclusive_scan_u32_dual(gb.tiles, gb.sorted_idx, gb.goff, gb.offsets, P, gb.scan_tmp, gb.counters + 1,
                                 gb.counters, s, tiles_sorted);
}

// the line search's shared binning: the n parameter sets' geometries, and the union list's per-set masks
// the depth-space render records of gslm_preprocess_views(depth_pos): [P][RECS] float4 at the start of a workspace
size_t depth_records_bytes(int64_t P) { return align_up((size_t)(P > 0 ? P : 0) * RECS * sizeof(float4)); }

// the n per-set depth-space workspaces (each set_bytes long): only their render records are read
int union_sets(const void* const* geoms, int32_t n, int64_t P, size_t set_bytes, UnionSets* u) {
  if (n < 1 || n > MAX_UNION_SETS) {
    set_error("union: 1 <= n <= 8 parameter sets");
    return GSLM_ERR_INVALID;
  }
  if (!geoms) { set_error("union: NULL geoms"); return GSLM_ERR_INVALID; }
  if (set_bytes < depth_records_bytes(P)) { set_error("union: a set's workspace is below gslm_depth_records_bytes(P)"); return GSLM_ERR_CAPACITY; }
  *u = UnionSets{};
  u->n = n;
  for (int a = 0; a < n; ++a) {
    if (!geoms[a] && P) { set_error("union: NULL geometry"); return GSLM_ERR_INVALID; }
    u->rec[a] = reinterpret_cast<const float4*>(geoms[a]);  // geom_layout's first region (rec at offset 0)
    u->tiles[a] = nullptr;
    u->rect[a] = nullptr;
  }
  return GSLM_OK;
}

size_t union_masks_layout(int64_t N, int ntiles, void* binning, UnionMasks* o) {
  BinBufs bb;
  const size_t off = bin_layout(N, ntiles, nullptr, &bb);
  Carver c{(char*)binning};
  c.off = off;
  UnionMasks m;
  m.m0 = c.take<uint32_t>(N);
  m.m1 = c.take<uint32_t>(N);
  m.hist = c.take<uint32_t>(sort_hist_bytes(N, true) / 4);
  m.nsets = c.take<uint32_t>(4);
  m.sorted = (bb.passes & 1) ? m.m1 : m.m0;
  if (o) *o = m;
  return c.off;
}

}  // namespace gslm

using namespace gslm;

extern "C" {

const char* gslm_last_error(void) { return g_last_error.c_str(); }
int gslm_abi_version(void) { return GSLM_ABI_VERSION; }

size_t gslm_geom_bytes(int64_t P) { return geom_layout(P, nullptr, nullptr); }
size_t gslm_image_bytes(int32_t H, int32_t W) { return img_layout(H, W, nullptr, nullptr); }
size_t gslm_binning_bytes(int64_t N, int32_t H, int32_t W) {
  const int ntiles = ((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y);
  return bin_layout(N, ntiles, nullptr, nullptr);
}
size_t gslm_scratch_bytes(int64_t P, int64_t N) { return scratch_layout(P, N, nullptr, nullptr); }

int gslm_preprocess(const gslm_view* view, const gslm_gaussians* gi, void* geom, size_t geom_bytes, int32_t* out_radii,
                    void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  ViewK v;
  GaussK g;
  int st = make_view(view, gi ? gi->max_coeffs : 0, &v);
  if (st) return st;
  if ((st = make_gauss(gi, &v, &g, false))) return st;
  if (geom_bytes < gslm_geom_bytes(g.P) || (!geom && g.P)) { set_error("geometry workspace too small"); return GSLM_ERR_CAPACITY; }
  GeomBufs gb;
  geom_layout(g.P, geom, &gb);
  return do_preprocess(v, g, gb, out_radii, (hipStream_t)stream);
}

int gslm_preprocess_ordered(const gslm_view* view, const gslm_gaussians* gi, void* geom, size_t geom_bytes,
                            int32_t* out_radii, uint32_t* depth_order, int32_t order_mode, void* stream) {
  if (order_mode < 0 || order_mode > 2) { set_error("preprocess_ordered: order_mode must be 0, 1 or 2"); return GSLM_ERR_INVALID; }
  if (order_mode && gi && gi->P > 0 && !depth_order) { set_error("preprocess_ordered: NULL depth_order"); return GSLM_ERR_INVALID; }
  ViewK v;
  GaussK g;
  int st = make_view(view, gi ? gi->max_coeffs : 0, &v);
  if (st) return st;
  if ((st = make_gauss(gi, &v, &g, false))) return st;
  if (geom_bytes < gslm_geom_bytes(g.P) || (!geom && g.P)) { set_error("geometry workspace too small"); return GSLM_ERR_CAPACITY; }
  GeomBufs gb;
  geom_layout(g.P, geom, &gb);
  return do_preprocess(v, g, gb, out_radii, (hipStream_t)stream, depth_order, order_mode);
}

int gslm_preprocess_views(const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, void* const* geoms,
                          size_t geom_bytes, const uint32_t* const* depth_pos, void* stream) {
  if (!views || !gi || !geoms || nviews < 1 || nviews > MAX_PRE_VIEWS) {
    set_error("preprocess_views: NULL argument or nviews outside 1..8");
    return GSLM_ERR_INVALID;
  }
  PreViewsK pv;
  GeomBufs gbs[MAX_PRE_VIEWS];
  GaussK g;
  int st;
  for (int b = 0; b < nviews; ++b) {
    if ((st = make_view(&views[b], gi->max_coeffs, &pv.v[b]))) return st;
    if ((st = make_gauss(gi, &pv.v[b], &g, false))) return st;  // each view's SH degree against the stored coefficients
    const size_t need = depth_pos ? depth_records_bytes(g.P) : gslm_geom_bytes(g.P);
    if (geom_bytes < need || (!geoms[b] && g.P)) { set_error("geometry workspace too small"); return GSLM_ERR_CAPACITY; }
    geom_layout(g.P, geoms[b], &gbs[b]);  // depth space writes the records (offset 0) only
    const uint32_t* pos = depth_pos ? depth_pos[b] : nullptr;
    if (depth_pos && !pos && g.P) { set_error("preprocess_views: NULL depth positions"); return GSLM_ERR_INVALID; }
    pv.out[b] = PreOutBufs{gbs[b].rec, gbs[b].depth_key, gbs[b].tiles, gbs[b].rect, gbs[b].clampw, pos};
  }
  pv.n = nviews;
  return launch_preprocess_views(pv, g, gbs, (hipStream_t)stream);
}

int gslm_depth_positions(const uint32_t* depth_order, int64_t P, uint32_t* depth_pos, void* stream) {
  if (P < 0 || P > MAX_P || (P && (!depth_order || !depth_pos))) {
    set_error("depth_positions: NULL order / positions or P out of range");
    return GSLM_ERR_INVALID;
  }
  return launch_depth_positions(P, depth_order, depth_pos, (hipStream_t)stream);
}

int gslm_num_rendered(const void* geom, int64_t P, int64_t* out, void* stream) {
  GeomBufs gb;
  geom_layout(P, const_cast<void*>(geom), &gb);
  // a pinned word per host thread: the read-back is one DMA + stream sync instead of a staged pageable copy
  thread_local uint32_t* pinned = nullptr;
  if (!pinned) GSLM_HIP_CHECK(hipHostMalloc((void**)&pinned, sizeof(uint32_t), hipHostMallocDefault));
  GSLM_HIP_CHECK(hipMemcpyAsync(pinned, gb.counters, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  GSLM_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  *out = (int64_t)*pinned;
  return GSLM_OK;
}

}  // extern "C"

namespace gslm {
constexpr int READ_COUNTS_MAX = 32;
struct CountPtrs {
  const uint32_t* p[READ_COUNTS_MAX];
};
// the pair counts of up to 32 geometries into pinned host memory in ONE launch (thread k: count k), where one
// 4-byte device-to-host copy per geometry is a blit launch each, in series on the stream
__global__ void k_read_counts(CountPtrs c, int n, uint32_t* __restrict__ out) {
  const int k = threadIdx.x;
  if (k < n) out[k] = *c.p[k];
}
}  // namespace gslm

extern "C" {

int gslm_num_rendered_many(const void* const* geoms, const int64_t* Ps, int32_t n, int64_t* out, void* stream) {
  if (n < 0 || (n > 0 && (!geoms || !Ps || !out))) { set_error("num_rendered_many: NULL argument"); return GSLM_ERR_INVALID; }
  if (n == 0) return GSLM_OK;
  // one pinned array per host thread, grown on demand: one gather launch per 32 geometries writing into it, then
  // ONE stream sync
  thread_local uint32_t* pinned = nullptr;
  thread_local uint32_t* pinned_dev = nullptr;
  thread_local int32_t cap = 0;
  if (cap < n) {
    if (pinned) GSLM_HIP_CHECK(hipHostFree(pinned));
    pinned = pinned_dev = nullptr;
    cap = 0;
    GSLM_HIP_CHECK(hipHostMalloc((void**)&pinned, sizeof(uint32_t) * (size_t)n, hipHostMallocDefault));
    GSLM_HIP_CHECK(hipHostGetDevicePointer((void**)&pinned_dev, pinned, 0));
    cap = n;
  }
  for (int32_t k0 = 0; k0 < n; k0 += READ_COUNTS_MAX) {
    CountPtrs c{};
    const int m = n - k0 < READ_COUNTS_MAX ? n - k0 : READ_COUNTS_MAX;
    for (int k = 0; k < m; ++k) {
      GeomBufs gb;
      geom_layout(Ps[k0 + k], const_cast<void*>(geoms[k0 + k]), &gb);
      c.p[k] = gb.counters;
    }
    hipLaunchKernelGGL(k_read_counts, dim3(1), dim3(64), 0, (hipStream_t)stream, c, m, pinned_dev + k0);
    GSLM_LAUNCH_CHECK();
  }
  GSLM_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  for (int32_t k = 0; k < n; ++k) out[k] = (int64_t)pinned[k];
  return GSLM_OK;
}

int gslm_rasterize(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                   int64_t N, void* image, size_t image_bytes, float* out_color, float* out_invdepth,
                   void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (binning_bytes < gslm_binning_bytes(N, v.H, v.W)) { set_error("binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (image_bytes < gslm_image_bytes(v.H, v.W)) { set_error("image workspace too small"); return GSLM_ERR_CAPACITY; }
  if (!out_color) { set_error("out_color is NULL"); return GSLM_ERR_INVALID; }
  GeomBufs gb;
  BinBufs bb;
  ImgBufs ib;
  geom_layout(P, geom, &gb);
  bin_layout(N, v.gx * v.gy, binning, &bb);
  img_layout(v.H, v.W, image, &ib);
  hipStream_t s = (hipStream_t)stream;
  if ((st = launch_binning(v, P, gb, bb, N, s))) return st;
  return launch_render_fwd(v, gb, bb, ib, out_color, out_invdepth, s);
}

size_t gslm_loss_scratch_bytes(int32_t H, int32_t W) {
  const int64_t ntiles = (int64_t)((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y);
  return (size_t)(ntiles > 0 ? ntiles : 1) * sizeof(double);
}

int gslm_rasterize_loss(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes, int64_t N,
                        const float* gt, const float* alpha_mask, void* scratch, size_t scratch_bytes, double* loss_dev,
                        int32_t accumulate, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (binning_bytes < gslm_binning_bytes(N, v.H, v.W)) { set_error("binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (scratch_bytes < gslm_loss_scratch_bytes(v.H, v.W)) { set_error("loss scratch too small"); return GSLM_ERR_CAPACITY; }
  if (!gt || !loss_dev || !scratch) { set_error("rasterize_loss: NULL gt / loss / scratch"); return GSLM_ERR_INVALID; }
  GeomBufs gb;
  BinBufs bb;
  geom_layout(P, geom, &gb);
  bin_layout(N, v.gx * v.gy, binning, &bb);
  hipStream_t s = (hipStream_t)stream;
  if ((st = launch_binning(v, P, gb, bb, N, s))) return st;
  return launch_render_loss(v, gb, bb, gt, alpha_mask, (double*)scratch, loss_dev, accumulate ? 1 : 0, s);
}

// ---- device-count forms: the pair count stays on the device (no read-back between preprocess and binning) ----
int64_t gslm_binning_capacity(size_t binning_bytes, int32_t H, int32_t W) {
  if (H <= 0 || W <= 0 || binning_bytes < gslm_binning_bytes(0, H, W)) return 0;
  // gslm_binning_bytes is non-decreasing in N: the largest N that fits, by bisection
  int64_t lo = 0, hi = (int64_t)1 << 40;
  while (hi - lo > 1) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (gslm_binning_bytes(mid, H, W) <= binning_bytes) lo = mid;
    else hi = mid;
  }
  return lo > (int64_t)0xFFFFFFFFu ? (int64_t)0xFFFFFFFFu : lo;
}

int gslm_rasterize_dev(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes, void* image,
                       size_t image_bytes, float* out_color, float* out_invdepth, uint32_t* n_out, void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (image_bytes < gslm_image_bytes(v.H, v.W)) { set_error("image workspace too small"); return GSLM_ERR_CAPACITY; }
  if (!out_color) { set_error("out_color is NULL"); return GSLM_ERR_INVALID; }
  const int64_t cap = gslm_binning_capacity(binning_bytes, v.H, v.W);
  if (binning_bytes < gslm_binning_bytes(0, v.H, v.W)) { set_error("binning workspace too small"); return GSLM_ERR_CAPACITY; }
  GeomBufs gb;
  BinBufs bb;
  ImgBufs ib;
  geom_layout(P, geom, &gb);
  bin_layout(cap, v.gx * v.gy, binning, &bb);
  img_layout(v.H, v.W, image, &ib);
  hipStream_t s = (hipStream_t)stream;
  if ((st = launch_binning(v, P, gb, bb, cap, s, true, n_out))) return st;
  return launch_render_fwd(v, gb, bb, ib, out_color, out_invdepth, s);
}

int gslm_rasterize_loss_dev(const gslm_view* view, int64_t P, void* geom, void* binning, size_t binning_bytes,
                            const float* gt, const float* alpha_mask, void* scratch, size_t scratch_bytes, double* loss_dev,
                            int32_t accumulate, uint32_t* n_out, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (binning_bytes < gslm_binning_bytes(0, v.H, v.W)) { set_error("binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (scratch_bytes < gslm_loss_scratch_bytes(v.H, v.W)) { set_error("loss scratch too small"); return GSLM_ERR_CAPACITY; }
  if (!gt || !loss_dev || !scratch) { set_error("rasterize_loss: NULL gt / loss / scratch"); return GSLM_ERR_INVALID; }
  const int64_t cap = gslm_binning_capacity(binning_bytes, v.H, v.W);
  GeomBufs gb;
  BinBufs bb;
  geom_layout(P, geom, &gb);
  bin_layout(cap, v.gx * v.gy, binning, &bb);
  hipStream_t s = (hipStream_t)stream;
  if ((st = launch_binning(v, P, gb, bb, cap, s, true, n_out))) return st;
  return launch_render_loss(v, gb, bb, gt, alpha_mask, (double*)scratch, loss_dev, accumulate ? 1 : 0, s);
}

// ---- the line search's shared binning (ABI 8; forward.hip k_union_rect / k_duplicate_union) ----
size_t gslm_union_binning_bytes(int64_t N, int32_t H, int32_t W) {
  const int ntiles = ((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y);
  return union_masks_layout(N, ntiles, nullptr, nullptr);
}

size_t gslm_depth_records_bytes(int64_t P) { return depth_records_bytes(P); }

int gslm_union_geometry(const gslm_view* view, int64_t P, const void* const* geoms, int32_t n, size_t set_bytes,
                        void* union_geom, size_t union_geom_bytes, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (P < 0 || P > MAX_P) { set_error("P out of range [0, 2^28 - 1]"); return GSLM_ERR_INVALID; }
  if (union_geom_bytes < gslm_geom_bytes(P) || (!union_geom && P)) { set_error("union geometry workspace too small"); return GSLM_ERR_CAPACITY; }
  UnionSets u;
  if ((st = union_sets(geoms, n, P, set_bytes, &u))) return st;
  GeomBufs ug;
  geom_layout(P, union_geom, &ug);
  hipStream_t s = (hipStream_t)stream;
  if (P == 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(ug.counters, 0, 4, s));
    return GSLM_OK;
  }
  if ((st = launch_union_rect(P, u, ug, s))) return st;
  // the union tile counts, already in depth order: k_duplicate_union's offsets, and the pair count in counters[0]
  return exclusive_scan_u32(ug.tiles, nullptr, ug.offsets, P, ug.scan_tmp, ug.counters, s);
}

int gslm_union_binning(const gslm_view* view, int64_t P, const void* union_geom, void* binning, size_t binning_bytes,
                       int64_t N, const void* const* geoms, int32_t n, size_t set_bytes, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (P < 0 || P > MAX_P || N < 0 || N > 0xFFFFFFFFll) { set_error("union_binning: P or N out of range"); return GSLM_ERR_INVALID; }
  if (binning_bytes < gslm_union_binning_bytes(N, v.H, v.W) || !binning) { set_error("union binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (P && !union_geom) { set_error("union_binning: NULL union geometry"); return GSLM_ERR_INVALID; }
  UnionSets u;
  if ((st = union_sets(geoms, n, P, set_bytes, &u))) return st;
  GeomBufs ug;
  BinBufs bb;
  UnionMasks um;
  geom_layout(P, const_cast<void*>(union_geom), &ug);
  bin_layout(N, v.gx * v.gy, binning, &bb);
  union_masks_layout(N, v.gx * v.gy, binning, &um);
  // the set count the masks are built for (gslm_rasterize_loss_slot renders a NaN loss for a slot past it)
  GSLM_HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(um.nsets), (int)n, 1, (hipStream_t)stream));
  return launch_union_binning(v, P, ug, bb, um, N, u, (hipStream_t)stream);
}

int gslm_rasterize_loss_slot(const gslm_view* view, int64_t P, const void* geom, size_t set_bytes, const void* binning,
                             size_t binning_bytes, int64_t N, int32_t slot, int32_t n_sets, const float* gt,
                             const float* alpha_mask, void* scratch, size_t scratch_bytes, double* loss_dev,
                             int32_t accumulate, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (n_sets < 1 || n_sets > MAX_UNION_SETS || slot < 0 || slot >= n_sets) {
    set_error("rasterize_loss_slot: need 0 <= slot < n_sets <= 8");
    return GSLM_ERR_INVALID;
  }
  if (set_bytes < depth_records_bytes(P)) { set_error("rasterize_loss_slot: set workspace below gslm_depth_records_bytes(P)"); return GSLM_ERR_CAPACITY; }
  if (N < 0 || N > 0xFFFFFFFFll) { set_error("rasterize_loss_slot: N out of range"); return GSLM_ERR_INVALID; }
  if (binning_bytes < gslm_union_binning_bytes(N, v.H, v.W) || !binning) { set_error("union binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (scratch_bytes < gslm_loss_scratch_bytes(v.H, v.W)) { set_error("loss scratch too small"); return GSLM_ERR_CAPACITY; }
  if (!gt || !loss_dev || !scratch) { set_error("rasterize_loss_slot: NULL gt / loss / scratch"); return GSLM_ERR_INVALID; }
  if (P && !geom) { set_error("rasterize_loss_slot: NULL geometry"); return GSLM_ERR_INVALID; }
  GeomBufs gb;
  BinBufs bb;
  UnionMasks um;
  geom_layout(P, const_cast<void*>(geom), &gb);
  bin_layout(N, v.gx * v.gy, const_cast<void*>(binning), &bb);
  union_masks_layout(N, v.gx * v.gy, const_cast<void*>(binning), &um);
  return launch_render_loss(v, gb, bb, gt, alpha_mask, (double*)scratch, loss_dev, accumulate ? 1 : 0,
                            (hipStream_t)stream, N > 0 ? um.sorted : nullptr, 4 * slot, um.nsets);
}

size_t gslm_loss_sets_scratch_bytes(int32_t n, int32_t H, int32_t W) {
  return (size_t)(n > 0 ? n : 1) * gslm_loss_scratch_bytes(H, W);
}

int gslm_rasterize_loss_sets(const gslm_view* view, int64_t P, const void* const* geoms, int32_t n, int32_t first_set,
                             size_t set_bytes, const void* binning, size_t binning_bytes, int64_t N, const float* gt,
                             const float* alpha_mask, void* scratch, size_t scratch_bytes, double* const* loss_dev,
                             int32_t accumulate, void* stream) {
  ViewK v;
  int st = make_view(view, 1, &v);
  if (st) return st;
  if (n < 1 || first_set < 0 || first_set + n > MAX_UNION_SETS) {
    set_error("rasterize_loss_sets: 1 <= n parameter sets, slots first_set .. first_set + n - 1 within [0, 8)");
    return GSLM_ERR_INVALID;
  }
  if (N < 0 || N > 0xFFFFFFFFll) { set_error("rasterize_loss_sets: N out of range"); return GSLM_ERR_INVALID; }
  if (binning_bytes < gslm_union_binning_bytes(N, v.H, v.W) || !binning) { set_error("union binning workspace too small"); return GSLM_ERR_CAPACITY; }
  if (scratch_bytes < gslm_loss_sets_scratch_bytes(n, v.H, v.W)) { set_error("loss scratch too small"); return GSLM_ERR_CAPACITY; }
  if (!gt || !loss_dev || !scratch || !geoms) { set_error("rasterize_loss_sets: NULL gt / loss / scratch / geoms"); return GSLM_ERR_INVALID; }
  if (set_bytes < depth_records_bytes(P)) { set_error("rasterize_loss_sets: set workspace below gslm_depth_records_bytes(P)"); return GSLM_ERR_CAPACITY; }
  SetRecsK sr{};
  LossPtrsK lp{};
  for (int a = 0; a < n; ++a) {
    if ((P && !geoms[a]) || !loss_dev[a]) { set_error("rasterize_loss_sets: NULL geometry / loss"); return GSLM_ERR_INVALID; }
    GeomBufs gb;
    geom_layout(P, const_cast<void*>(geoms[a]), &gb);
    sr.rec[a] = gb.rec;
    lp.loss[a] = loss_dev[a];
  }
  BinBufs bb;
  UnionMasks um;
  bin_layout(N, v.gx * v.gy, const_cast<void*>(binning), &bb);
  union_masks_layout(N, v.gx * v.gy, const_cast<void*>(binning), &um);
  // um.nsets: slots at or past the set count gslm_union_binning recorded render a NaN loss (as the slot form)
  return launch_render_loss_sets(v, sr, n, bb, um.sorted, gt, alpha_mask, (double*)scratch, lp, accumulate ? 1 : 0,
                                 (hipStream_t)stream, first_set, um.nsets);
}

int gslm_num_rendered_copy(const void* geom, int64_t P, uint32_t* dst, void* stream) {
  if (!dst || (P > 0 && !geom)) { set_error("num_rendered_copy: NULL geom / dst"); return GSLM_ERR_INVALID; }
  if (P == 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(dst, 0, 4, (hipStream_t)stream));
    return GSLM_OK;
  }
  GeomBufs gb;
  geom_layout(P, const_cast<void*>(geom), &gb);
  GSLM_HIP_CHECK(hipMemcpyAsync(dst, gb.counters, 4, hipMemcpyDefault, (hipStream_t)stream));
  return GSLM_OK;
}

int gslm_forward(const gslm_view* view, const gslm_gaussians* gi, void* geom, size_t geom_bytes, void* binning,
                 size_t binning_bytes, void* image, size_t image_bytes, float* out_color, float* out_invdepth,
                 int32_t* out_radii, int64_t* out_num_rendered, void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  int st = gslm_preprocess(view, gi, geom, geom_bytes, out_radii, stream);
  if (st) return st;
  int64_t N = 0;
  if ((st = gslm_num_rendered(geom, gi->P, &N, stream))) return st;
  if (out_num_rendered) *out_num_rendered = N;
  if (binning_bytes < gslm_binning_bytes(N, view->image_height, view->image_width)) {
    set_error("binning workspace too small for num_rendered");
    return GSLM_ERR_CAPACITY;
  }
  return gslm_rasterize(view, gi->P, geom, binning, binning_bytes, N, image, image_bytes, out_color, out_invdepth,
                        stream);
}


static GradK make_gradk(const gslm_grads* o) {
  GradK k;
  k.means2D = o->means2D;
  k.means3D = o->means3D;
  k.opac = o->opacities;
  k.scales = o->scales;
  k.rot = o->rotations;
  k.cov3D = o->cov3D;
  k.dc = o->sh_dc;
  k.dc_stride = o->sh_dc_stride;
  k.rest = o->sh_rest;
  k.rest_stride = o->sh_rest_stride;
  k.colors = o->colors;
  k.accumulate = o->accumulate;
  return k;
}

static GaussK tangent_from_grads(const gslm_grads* t, const GaussK& g, bool mask_xyz) {
  GaussK k;
  k.P = g.P;
  k.raw = g.raw;
  k.M = g.M;
  k.means3D = mask_xyz ? nullptr : t->means3D;
  k.opac = t->opacities;
  k.scales = t->scales;
  k.rot = t->rotations;
  k.cov3D = t->cov3D;
  k.dc = t->sh_dc;
  k.dc_stride = t->sh_dc_stride;
  k.rest = t->sh_rest;
  k.rest_stride = t->sh_rest_stride;
  k.colors = t->colors;
  return k;
}

struct Bound {
  ViewK v;
  GaussK g;
  GeomBufs gb;
  BinBufs bb;
  ImgBufs ib;
  ScratchBufs sb;
};

static int bind_all(const gslm_view* view, const gslm_gaussians* gi, const void* geom, const void* binning,
                    int64_t N, const void* image, void* scratch, size_t scratch_bytes, Bound* b) {
  int st = make_view(view, gi ? gi->max_coeffs : 0, &b->v);
  if (st) return st;
  if ((st = make_gauss(gi, &b->v, &b->g, false))) return st;
  if (scratch_bytes < gslm_scratch_bytes(b->g.P, N)) {
    set_error("scratch workspace too small");
    return GSLM_ERR_CAPACITY;
  }
  geom_layout(b->g.P, const_cast<void*>(geom), &b->gb);
  bin_layout(N, b->v.gx * b->v.gy, const_cast<void*>(binning), &b->bb);
  img_layout(b->v.H, b->v.W, const_cast<void*>(image), &b->ib);
  scratch_layout(b->g.P, N, scratch, &b->sb);
  return GSLM_OK;
}

int gslm_backward(const gslm_view* view, const gslm_gaussians* gi, const void* geom, const void* binning, int64_t N,
                  const void* image, const float* dL_dcolor, const float* dL_dinvdepth, void* scratch,
                  size_t scratch_bytes, const gslm_grads* out, void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  Bound b;
  int st = bind_all(view, gi, geom, binning, N, image, scratch, scratch_bytes, &b);
  if (st) return st;
  if (!out || !dL_dcolor) { set_error("backward: NULL dL_dcolor or outputs"); return GSLM_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  if ((st = launch_render_bwd(b.v, b.gb, b.bb, b.ib, N, dL_dcolor, dL_dinvdepth, b.sb, s))) return st;
  return launch_preprocess_bwd(b.v, b.g, b.gb, b.bb, b.sb, make_gradk(out), true, s);
}

int gslm_jvp(const gslm_view* view, const gslm_gaussians* gi, const gslm_gaussians* tangent,
             const float* means2D_tangent, const void* geom, const void* binning, int64_t N, const void* image,
             void* scratch, size_t scratch_bytes, float* out_color_t, float* out_invdepth_t, void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  Bound b;
  int st = bind_all(view, gi, geom, binning, N, image, scratch, scratch_bytes, &b);
  if (st) return st;
  if (!out_color_t) { set_error("jvp: NULL out_color_t"); return GSLM_ERR_INVALID; }
  GaussK t;
  if ((st = make_gauss(tangent, &b.v, &t, true))) return st;
  t.P = b.g.P;
  t.raw = b.g.raw;
  t.M = b.g.M;
  return launch_jvp(b.v, b.g, t, means2D_tangent, b.gb, b.bb, b.ib, b.sb, out_color_t, out_invdepth_t,
                    (hipStream_t)stream);
}

// The fused CG direction update of gslm_matvec_opts (xpby_s .. xpby_x_offset) as a kernel argument; R is
// the SH-rest width of v and s (3(M-1), or 3 projected).
static int build_xpby(const gslm_matvec_opts* opts, const gslm_grads* vin, int R, bool mask_xyz, XpbyK* out) {
  const gslm_grads* sv = opts->xpby_s;
  if (!opts->beta_num || !opts->beta_den) {
    set_error("matvec: xpby needs the TANGENT stage and beta_num / beta_den");
    return GSLM_ERR_INVALID;
  }
  if (vin->sh_dc_stride != 3 || sv->sh_dc_stride != 3 || (R > 0 && (vin->sh_rest_stride != R || sv->sh_rest_stride != R))) {
    set_error("matvec: xpby needs contiguous SH groups (dc stride 3, rest stride 3(M-1), or 3 projected)");
    return GSLM_ERR_INVALID;
  }
  XpbyK xp{};
  float* pp[6] = {vin->means3D, vin->sh_dc, vin->sh_rest, vin->scales, vin->rotations, vin->opacities};
  const float* ss[6] = {sv->means3D, sv->sh_dc, sv->sh_rest, sv->scales, sv->rotations, sv->opacities};
  const int ww[6] = {3, 3, R, 3, 4, 1};
  for (int k = 0; k < 6; ++k) {
    if ((pp[k] == nullptr) != (ss[k] == nullptr) || (ww[k] == 0 && pp[k])) {
      set_error("matvec: xpby groups of v and s must match");
      return GSLM_ERR_INVALID;
    }
    // with mask_xyz the xyz group is left untouched: it is zero in every LM iterate (s and p alike)
    xp.p[k] = (ww[k] && !(k == 0 && mask_xyz)) ? pp[k] : nullptr;
    xp.s[k] = ss[k];
    xp.w[k] = ww[k];
  }
  xp.num = opts->beta_num;
  xp.den = opts->beta_den;
  xp.tail_p = opts->xpby_tail_n > 0 ? opts->xpby_tail_v : nullptr;
  xp.tail_s = opts->xpby_tail_s;
  xp.tail_n = opts->xpby_tail_n;
  if (xp.tail_p && !xp.tail_s) { set_error("matvec: xpby tail without s"); return GSLM_ERR_INVALID; }
  xp.anum = opts->alpha_num;
  xp.aden = opts->alpha_den;
  xp.xoff = opts->xpby_x_offset / (int64_t)sizeof(float);
  if (xp.anum && (!xp.aden || opts->xpby_x_offset % (int64_t)sizeof(float) != 0)) {
    set_error("matvec: deferred x update needs alpha_den and a float-aligned xpby_x_offset");
    return GSLM_ERR_INVALID;
  }
  *out = xp;
  return GSLM_OK;
}

int gslm_matvec_view_ex(const gslm_view* view, const gslm_gaussians* gi, const gslm_grads* vin,
                        const float* pixel_weight, int32_t mask_xyz, const void* geom, const void* binning,
                        int64_t N, const void* image, void* scratch, size_t scratch_bytes, const gslm_grads* y,
                        const gslm_matvec_opts* opts, void* stream) {
  DebugScope dbg_scope(view != nullptr && view->debug != 0, stream);
  Bound b;
  int st = bind_all(view, gi, geom, binning, N, image, scratch, scratch_bytes, &b);
  if (st) return st;
  if (!vin || !y || !pixel_weight) { set_error("matvec: NULL argument"); return GSLM_ERR_INVALID; }
  const int32_t stages = (opts && opts->stages) ? opts->stages : GSLM_STAGE_ALL;
  const double* damp7 = opts ? opts->damp7 : nullptr;
  double* dot_out = opts ? opts->dot_vy : nullptr;
  if (dot_out && (!opts->dot_scratch || opts->dot_scratch_bytes < gslm_dot_scratch_bytes(b.g.P))) {
    set_error("matvec: dot scratch too small");
    return GSLM_ERR_CAPACITY;
  }
  if (!b.g.raw) { set_error("matvec: gaussians must be the raw GaussianModel leaves (raw = 1)"); return GSLM_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  b.v.stop = opts ? opts->cg_ctl : nullptr;
  if (opts && opts->rest_basis) {
    set_error("matvec: rest_basis is an option of gslm_tangent_views / gslm_gather_screen");
    return GSLM_ERR_INVALID;
  }
  const bool proj = opts && (opts->flags & GSLM_MV_SH_REST_PROJECTED) && b.g.M > 1;
  GaussK t = tangent_from_grads(vin, b.g, mask_xyz != 0);
  if (proj) {
    if (vin->sh_rest && vin->sh_rest_stride != 3) {
      set_error("matvec: a projected SH-rest group has 3 floats per Gaussian (sh_rest_stride 3)");
      return GSLM_ERR_INVALID;
    }
    if (stages & GSLM_STAGE_SCREEN) {
      set_error("matvec: GSLM_MV_SH_REST_PROJECTED is a single-view mode (no SCREEN stage)");
      return GSLM_ERR_INVALID;
    }
    t.rest_proj = 1;
  }
  XpbyK xp{};
  const bool fused_xpby = opts && opts->xpby_s;
  if (fused_xpby) {
    if (!(stages & GSLM_STAGE_TANGENT)) {
      set_error("matvec: xpby needs the TANGENT stage and beta_num / beta_den");
      return GSLM_ERR_INVALID;
    }
    if ((st = build_xpby(opts, vin, proj ? 3 : 3 * (b.g.M - 1), mask_xyz != 0, &xp))) return st;
  }
  if (opts && opts->trec_in) {
    if (stages & GSLM_STAGE_TANGENT) {
      set_error("matvec: trec_in replaces the TANGENT stage");
      return GSLM_ERR_INVALID;
    }
    b.sb.trec = reinterpret_cast<float4*>(const_cast<float*>(opts->trec_in));
  }
  const float* seed = opts ? opts->pixel_seed : nullptr;
  if (seed && (!mask_xyz || fused_xpby || (stages & (GSLM_STAGE_TANGENT | GSLM_STAGE_SCREEN)))) {
    set_error("matvec: pixel_seed (J^T seed) needs mask_xyz and excludes TANGENT / SCREEN / xpby");
    return GSLM_ERR_INVALID;
  }
  if ((stages & GSLM_STAGE_TANGENT) &&
      (st = launch_tangent_pre(b.v, b.g, t, nullptr, b.gb, b.sb, fused_xpby ? &xp : nullptr, s, mask_xyz != 0)))
    return st;
  float* jv_out = opts ? opts->jv_out : nullptr;
  if (jv_out) {
    if (seed || (stages & (GSLM_STAGE_GATHER | GSLM_STAGE_SCREEN))) {
      set_error("matvec: jv_out excludes pixel_seed, GATHER and SCREEN");
      return GSLM_ERR_INVALID;
    }
    if (stages & GSLM_STAGE_RENDER) {
      if (N == 0) {
        GSLM_HIP_CHECK(hipMemsetAsync(jv_out, 0, (size_t)3 * b.v.H * b.v.W * sizeof(float), s));
      } else if ((st = launch_render_jv(b.v, t, b.gb, b.bb, b.ib, b.sb, mask_xyz != 0, jv_out, s))) {
        return st;
      }
    }
    return GSLM_OK;
  }
  if (seed) {
    if ((stages & GSLM_STAGE_RENDER) &&
        (st = launch_render_vjp_lm(b.v, b.gb, b.bb, b.ib, N, seed, b.sb, opts->flags & GSLM_MV_TAIL_CLEAN, s)))
      return st;
  } else if ((stages & GSLM_STAGE_RENDER) && N > 0 &&
      (st = launch_matvec_render(b.v, t, b.gb, b.bb, b.ib, b.sb, N, pixel_weight, mask_xyz != 0,
                                 opts && (opts->flags & GSLM_MV_TAIL_CLEAN), s)))
    return st;
  if (stages & GSLM_STAGE_SCREEN) {
    if (!mask_xyz || !opts->screen_out) {
      set_error("matvec: GSLM_STAGE_SCREEN needs mask_xyz and opts->screen_out");
      return GSLM_ERR_INVALID;
    }
    return launch_rowsum_screen(b.g, b.gb, b.sb, opts->screen_out, s);
  }
  if (!(stages & GSLM_STAGE_GATHER)) return GSLM_OK;
  double* part = dot_out ? (double*)opts->dot_scratch : nullptr;
  if ((st = launch_gather_lm(b.v, b.g, b.gb, b.sb, make_gradk(y), make_gradk(vin), damp7,
                             (stages & GSLM_STAGE_OVERWRITE) != 0, mask_xyz != 0, part, s, proj)))
    return st;
  if (dot_out) return gslm_dot_finalize(part, (int32_t)((b.g.P + 255) / 256), dot_out, stream);
  return GSLM_OK;
}

int gslm_sh_rest_project(const gslm_view* view, const gslm_gaussians* gi, int32_t mode, const float* in,
                         int64_t in_stride, float* out, int64_t out_stride, void* stream) {
  ViewK v;
  GaussK g;
  int st;
  if (!view || !gi) { set_error("sh_rest_project: NULL view / gaussians"); return GSLM_ERR_INVALID; }
  if ((st = make_view(view, gi->max_coeffs, &v))) return st;
  if ((st = make_gauss(gi, &v, &g, false))) return st;
  if (mode != 0 && mode != 1) { set_error("sh_rest_project: mode must be 0 (expand) or 1 (project)"); return GSLM_ERR_INVALID; }
  if (g.P > 0 && g.M > 1 && (!in || !out || !g.means3D)) { set_error("sh_rest_project: NULL buffer"); return GSLM_ERR_INVALID; }
  const int64_t full = 3 * (int64_t)(g.M - 1);
  if ((mode == 0 && (in_stride < 3 || out_stride < full)) || (mode == 1 && (in_stride < full || out_stride < 3))) {
    set_error("sh_rest_project: strides too small for [P,3] / [P,M-1,3] rows");
    return GSLM_ERR_INVALID;
  }
  return launch_sh_rest_project(v, g, mode, in, in_stride, out, out_stride, (hipStream_t)stream);
}

// the views of one SH-rest coordinate system: 1..GSLM_MAX_REST_VIEWS, one SH degree
static int rest_views(const char* who, const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, ViewK* vk,
                      GaussK* g) {
  if (!views || !gi || nviews < 1 || nviews > GSLM_MAX_REST_VIEWS) {
    set_error(std::string(who) + ": NULL views / gaussians or nviews outside 1..GSLM_MAX_REST_VIEWS");
    return GSLM_ERR_INVALID;
  }
  int st;
  for (int b = 0; b < nviews; ++b) {
    if ((st = make_view(&views[b], gi->max_coeffs, &vk[b]))) return st;
    if (vk[b].D != vk[0].D) {
      set_error(std::string(who) + ": the views must share one SH degree");
      return GSLM_ERR_INVALID;
    }
  }
  if ((st = make_gauss(gi, &vk[0], g, false))) return st;
  if (g->P > 0 && !g->means3D) {
    set_error(std::string(who) + ": NULL means3D");
    return GSLM_ERR_INVALID;
  }
  return GSLM_OK;
}

int gslm_rest_basis(const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, float* R_out, void* stream) {
  ViewK vk[GSLM_MAX_REST_VIEWS];
  GaussK g;
  int st;
  if ((st = rest_views("rest_basis", views, nviews, gi, vk, &g))) return st;
  if (g.P > 0 && !R_out) { set_error("rest_basis: NULL R_out"); return GSLM_ERR_INVALID; }
  return launch_rest_basis(vk, nviews, g, R_out, (hipStream_t)stream);
}

int gslm_rest_coords(const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, const float* R, int32_t mode,
                     const float* in, int64_t in_stride, float* out, int64_t out_stride, void* stream) {
  ViewK vk[GSLM_MAX_REST_VIEWS];
  GaussK g;
  int st;
  if ((st = rest_views("rest_coords", views, nviews, gi, vk, &g))) return st;
  if (mode != 0 && mode != 1) { set_error("rest_coords: mode must be 0 (expand) or 1 (project)"); return GSLM_ERR_INVALID; }
  if (g.M < 2) return GSLM_OK;
  if (g.P > 0 && (!R || !in || !out)) { set_error("rest_coords: NULL buffer"); return GSLM_ERR_INVALID; }
  const int64_t full = 3 * (int64_t)(g.M - 1), coords = 3 * (int64_t)nviews;
  if ((mode == 0 && (in_stride < coords || out_stride < full)) || (mode == 1 && (in_stride < full || out_stride < coords))) {
    set_error("rest_coords: strides too small for [P,V,3] / [P,M-1,3] rows");
    return GSLM_ERR_INVALID;
  }
  return launch_rest_coords(vk, nviews, g, R, mode, in, in_stride, out, out_stride, (hipStream_t)stream);
}

// opts->rest_basis of gslm_tangent_views / gslm_gather_screen: the coordinate system and this call's columns
static int rest_opts(const char* who, const gslm_matvec_opts* opts, int32_t nviews, RestK* rc) {
  *rc = RestK{};
  if (!opts || !opts->rest_basis) return GSLM_OK;
  if (opts->rest_views < 1 || opts->rest_views > GSLM_MAX_REST_VIEWS || opts->view_base < 0 ||
      opts->view_base + nviews > opts->rest_views) {
    set_error(std::string(who) + ": rest_views outside 1..GSLM_MAX_REST_VIEWS or views past its last column");
    return GSLM_ERR_INVALID;
  }
  rc->R = opts->rest_basis;
  rc->V = opts->rest_views;
  rc->view_base = opts->view_base;
  return GSLM_OK;
}

int gslm_gather_screen(const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, const float* screen,
                       const gslm_grads* vin, const gslm_grads* y, const gslm_matvec_opts* opts, void* stream) {
  if (!views || nviews < 1 || nviews > 16 || !gi || !screen || !vin || !y) {
    set_error("gather_screen: NULL argument or nviews outside 1..16");
    return GSLM_ERR_INVALID;
  }
  ViewK vk[16];
  GaussK g;
  int st;
  for (int b = 0; b < nviews; ++b) {
    if ((st = make_view(&views[b], gi->max_coeffs, &vk[b]))) return st;
    vk[b].stop = opts ? opts->cg_ctl : nullptr;  // a stopped solve's gather returns at once
  }
  if ((st = make_gauss(gi, &vk[0], &g, false))) return st;
  if (!g.raw) { set_error("gather_screen: gaussians must be the raw GaussianModel leaves (raw = 1)"); return GSLM_ERR_INVALID; }
  const int32_t stages = (opts && opts->stages) ? opts->stages : GSLM_STAGE_ALL;
  const double* damp7 = opts ? opts->damp7 : nullptr;
  double* dot_out = opts ? opts->dot_vy : nullptr;
  if (dot_out && (!opts->dot_scratch || opts->dot_scratch_bytes < gslm_dot_scratch_bytes(g.P))) {
    set_error("gather_screen: dot scratch too small");
    return GSLM_ERR_CAPACITY;
  }
  double* part = dot_out ? (double*)opts->dot_scratch : nullptr;
  const int64_t sstride = (opts && opts->screen_stride) ? opts->screen_stride : g.P;
  if (sstride < g.P) { set_error("gather_screen: screen_stride below P"); return GSLM_ERR_INVALID; }
  RestK rc;
  if ((st = rest_opts("gather_screen", opts, nviews, &rc))) return st;
  if ((st = launch_gather_screen(vk, nviews, g, screen, sstride, make_gradk(y), make_gradk(vin), damp7,
                                 (stages & GSLM_STAGE_OVERWRITE) != 0, part, (hipStream_t)stream, rc)))
    return st;
  if (dot_out) return gslm_dot_finalize(part, (int32_t)((g.P + 255) / 256), dot_out, stream);
  return GSLM_OK;
}

int gslm_view_flags(const void* geom, int64_t P, uint32_t* out, void* stream) {
  if (P < 0 || (P > 0 && (!geom || !out))) { set_error("view_flags: NULL geom / out"); return GSLM_ERR_INVALID; }
  GeomBufs gb;
  geom_layout(P, const_cast<void*>(geom), &gb);
  return launch_view_flags(P, gb, out, (hipStream_t)stream);
}

int gslm_tangent_views(const gslm_view* views, int32_t nviews, const gslm_gaussians* gi, const gslm_grads* vin,
                       int32_t mask_xyz, const uint32_t* vflags, int64_t flags_stride, float* trec_out,
                       int64_t trec_stride, const gslm_matvec_opts* opts, void* stream) {
  if (!views || nviews < 1 || nviews > MAX_SCREEN_VIEWS || !gi || !vin) {
    set_error("tangent_views: NULL argument or nviews outside 1..16");
    return GSLM_ERR_INVALID;
  }
  ViewK vk[MAX_SCREEN_VIEWS];
  GaussK g;
  int st;
  for (int b = 0; b < nviews; ++b) {
    if ((st = make_view(&views[b], gi->max_coeffs, &vk[b]))) return st;
    vk[b].stop = opts ? opts->cg_ctl : nullptr;  // a stopped solve's tangent records (and direction update) are skipped
  }
  if ((st = make_gauss(gi, &vk[0], &g, false))) return st;
  if (!g.raw || g.cov3D || g.colors) {
    set_error("tangent_views: gaussians must be the raw GaussianModel leaves (raw = 1)");
    return GSLM_ERR_INVALID;
  }
  if (g.P > 0 && (!vflags || !trec_out || flags_stride < g.P || trec_stride < g.P)) {
    set_error("tangent_views: NULL vflags / trec_out or a stride below P");
    return GSLM_ERR_INVALID;
  }
  GaussK t = tangent_from_grads(vin, g, mask_xyz != 0);
  RestK rc;
  if ((st = rest_opts("tangent_views", opts, nviews, &rc))) return st;
  const int R = rc.R ? 3 * rc.V : 3 * (g.M - 1);
  if (t.rest && t.rest_stride != R) {
    set_error(rc.R ? "tangent_views: SH-rest coordinates need stride 3 rest_views"
                   : "tangent_views: the SH-rest tangent needs stride 3(M-1)");
    return GSLM_ERR_INVALID;
  }
  if (rc.R && g.M > 1) {
    t.rest_R = rc.R;
    t.rest_V = rc.V;
  }
  XpbyK xp{};
  const bool fused = opts && opts->xpby_s;
  if (fused && (st = build_xpby(opts, vin, R, mask_xyz != 0, &xp))) return st;
  return launch_tangent_views(vk, nviews, g, t, vflags, flags_stride, trec_out, trec_stride, fused ? &xp : nullptr,
                              (hipStream_t)stream, mask_xyz != 0, rc.view_base);
}

int gslm_matvec_view(const gslm_view* view, const gslm_gaussians* gi, const gslm_grads* vin,
                     const float* pixel_weight, int32_t mask_xyz, const void* geom, const void* binning, int64_t N,
                     const void* image, void* scratch, size_t scratch_bytes, const gslm_grads* y, void* stream) {
  return gslm_matvec_view_ex(view, gi, vin, pixel_weight, mask_xyz, geom, binning, N, image, scratch, scratch_bytes,
                             y, nullptr, stream);
}

int gslm_inspect(const void* geom, int64_t P, const void* binning, int64_t N, int32_t H, int32_t W,
                 const void* image, uint32_t* point_list, uint32_t* ranges, uint32_t* tiles_touched, float* final_T,
                 uint32_t* n_contrib, float* records, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  GeomBufs gb;
  BinBufs bb;
  ImgBufs ib;
  const int ntiles = ((W + TILE_X - 1) / TILE_X) * ((H + TILE_Y - 1) / TILE_Y);
  geom_layout(P, const_cast<void*>(geom), &gb);
  bin_layout(N, ntiles, const_cast<void*>(binning), &bb);
  img_layout(H, W, const_cast<void*>(image), &ib);
  const auto D2D = hipMemcpyDeviceToDevice;
  if (point_list && N) {
    const int st = launch_point_ids(bb.point_list, N, point_list, s);
    if (st) return st;
  }
  if (ranges && binning) GSLM_HIP_CHECK(hipMemcpyAsync(ranges, bb.ranges, (size_t)ntiles * 8, D2D, s));
  if (tiles_touched && P) GSLM_HIP_CHECK(hipMemcpyAsync(tiles_touched, gb.tiles, (size_t)P * 4, D2D, s));
  if (final_T && image) GSLM_HIP_CHECK(hipMemcpyAsync(final_T, ib.final_T, (size_t)H * W * 4, D2D, s));
  if (n_contrib && image) GSLM_HIP_CHECK(hipMemcpyAsync(n_contrib, ib.n_contrib, (size_t)H * W * 4, D2D, s));
  if (records && P)  // 12 floats per Gaussian out of the 64-B record stride
    GSLM_HIP_CHECK(hipMemcpy2DAsync(records, 48, gb.rec, RECS * sizeof(float4), 48, (size_t)P, D2D, s));
  return GSLM_OK;
}

}  // extern "C"
