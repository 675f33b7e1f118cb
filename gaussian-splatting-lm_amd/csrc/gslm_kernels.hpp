// gslm_kernels.hpp -- device structs, per-Gaussian preprocess routine, workspace views, launchers.
#pragma once
#include "gslm_internal.hpp"

namespace gslm {

// Device view of gslm_gaussians (also used for tangents: NULL pointer = zero tangent).
struct GaussK {
  int64_t P;
  int raw;
  int M;
  const float* means3D;
  const float* opac;
  const float* scales;
  const float* rot;
  const float* cov3D;
  const float* dc;
  int64_t dc_stride;
  const float* rest;
  int64_t rest_stride;
  const float* colors;
  __device__ __forceinline__ float sh(int64_t i, int k, int c) const {
    return k == 0 ? dc[i * dc_stride + c] : rest[i * rest_stride + 3 * (k - 1) + c];
  }
};

// Device view of gslm_grads.
struct GradK {
  float* means2D;
  float* means3D;
  float* opac;
  float* scales;
  float* rot;
  float* cov3D;
  float* dc;
  int64_t dc_stride;
  float* rest;
  int64_t rest_stride;
  float* colors;
  int accumulate;
};

struct PreOut {
  float x, y;
  float conic[3];
  float opac;
  float rgb[3];
  float depth;
  uint32_t clamped;
  uint32_t ext;  // packed half-extents (1/8 px units) of the alpha >= 1/255 ellipse's bounding box
  int radius;
  int rmin_x, rmin_y, rmax_x, rmax_y;
};

// Conservative bounding box of the pixels that can pass the alpha >= 1/255 test, packed as two u16
// half-extents in 1/8 px (0xFFFF = unbounded).  Used by the tile passes to skip a Gaussian for a whole
// wave when no pixel of the wave's 16x4 strip can blend it: the skipped lanes would all fail the
// alpha test, so results are bit-identical with and without the cull.
//
// Exact math: alpha >= 1/255  <=>  Q(d) = A dx^2 + C dy^2 + 2 B dx dy <= t = 2 ln(255 o).  The float
// evaluation of Q in the tile passes has absolute error <= e |d|^2 with e = 32 eps (A + C) (each
// term carries a few roundings and |2 B dx dy| <= max(A, C) |d|^2), so every accepted pixel lies in
// {d : d^T (Q - e I) d <= t}, whose half-extents are sqrt(t (Q - e I)^-1_ii) -- computed in double
// from the *stored* conic.  A 2 % margin on t covers exp/log error; +0.1 px covers the box test.
// Needle-like splats for which Q - e I is not positive definite get an unbounded box.
__device__ __forceinline__ uint32_t alpha_extent(float op_eff, float A, float B, float C) {
  if (!(op_eff * 255.0f > 1.0f)) return 0u;  // alpha = o G <= o < 1/255 everywhere: never blended
  const double t = 2.0 * log(255.0 * (double)op_eff) * 1.02 + 1e-6;
  const double e = 32.0 * 5.9604644775390625e-8 * ((double)A + (double)C);
  const double a = (double)A - e, c = (double)C - e;
  const double det = a * c - (double)B * (double)B;
  if (!(a > 0.0 && c > 0.0 && det > 0.0)) return 0xFFFFFFFFu;
  const double ex = sqrt(t * c / det) + 0.1, ey = sqrt(t * a / det) + 0.1;
  const uint32_t qx = (uint32_t)fmin(65535.0, ceil(ex * 8.0));
  const uint32_t qy = (uint32_t)fmin(65535.0, ceil(ey * 8.0));
  return qx | (qy << 16);
}

// Strip mask of a Gaussian in tile (tile_x, tile_y): bit s set when its alpha box can reach strip s =
// tile rows 4s..4s+3 (all 16 columns) -- the pixels of wave s in the 256-thread tile passes.
__device__ __forceinline__ uint32_t strip_mask4(float gx, float gy, uint32_t ext, int tile_x, int tile_y) {
#ifdef GSLM_NO_STRIP_CULL
  return 0xFu;
#endif
  const uint32_t qx = ext & 0xFFFFu, qy = ext >> 16;
  const float ex = qx == 0xFFFFu ? INFINITY : (float)qx * 0.125f;
  const float ey = qy == 0xFFFFu ? INFINITY : (float)qy * 0.125f;
  const float x0 = (float)(tile_x * TILE_X), y0 = (float)(tile_y * TILE_Y);
  if (!(fabsf(gx - fminf(fmaxf(gx, x0), x0 + (TILE_X - 1))) <= ex)) return 0u;
  uint32_t m = 0u;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float ys = y0 + 4.0f * s;
    if (fabsf(gy - fminf(fmaxf(gy, ys), ys + 3.0f)) <= ey) m |= 1u << s;
  }
  return m;
}

// Called by all 256 threads after thread tid has fetched batch element tid (`valid`: tid < cnt).
// Publishes, per strip s, the 256-bit set of batch elements that can touch it: s_bits[4 s + c] holds
// elements 64c..64c+63.  Wave s then visits only those elements (wave_bits / s_ff1), skipping the
// rest for the whole wave: every skipped lane would have failed the alpha test, so the pass's
// results are bit-identical to visiting every element.  Returns this element's own mask.
__device__ __forceinline__ uint32_t publish_strip_masks(bool valid, float gx, float gy, uint32_t ext, int tile_x,
                                                        int tile_y, uint64_t* s_bits) {
  const uint32_t m = valid ? strip_mask4(gx, gy, ext, tile_x, tile_y) : 0u;
  const int c = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint64_t b = __ballot((m >> s) & 1u);
    if ((threadIdx.x & 63) == 0) s_bits[4 * s + c] = b;
  }
  return m;
}

// The 64-element hit set c of strip (wave) s as a wave-uniform (SGPR) value.
__device__ __forceinline__ uint64_t wave_bits(const uint64_t* s_bits, int s, int c) {
  const uint64_t b = s_bits[4 * s + c];
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Activated scale / rotation of Gaussian i (fusing exp / normalize when RAW).
template <bool RAW>
__device__ __forceinline__ void load_scale_rot(const GaussK& g, int64_t i, float s[3], float q[4]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = RAW ? expf(g.scales[3 * i + k]) : g.scales[3 * i + k];
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = g.rot[4 * i + k];
  if (RAW) {
    const float nrm = fmaxf(sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]), 1e-12f);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = q[k] / nrm;
  }
}

// SURVEY Appendix A steps 1-9 for one Gaussian; returns false when culled.
template <bool RAW>
__device__ __forceinline__ bool preprocess_one(const ViewK& v, const GaussK& g, int64_t i, PreOut& o) {
  const float x = g.means3D[3 * i + 0], y = g.means3D[3 * i + 1], z = g.means3D[3 * i + 2];
  const float tz = tp_row(v.view, x, y, z, 2);
  if (!(tz > 0.2f)) return false;
  const float tx = tp_row(v.view, x, y, z, 0), ty = tp_row(v.view, x, y, z, 1);
  const float hx = tp_row(v.proj, x, y, z, 0), hy = tp_row(v.proj, x, y, z, 1), hw = tp_row(v.proj, x, y, z, 3);
  const float p_w = 1.0f / (hw + 0.0000001f);
  const float pxn = hx * p_w, pyn = hy * p_w;

  float c[6];
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = g.cov3D[6 * i + k];
  } else {
    float s[3], q[4], R[9];
    load_scale_rot<RAW>(g, i, s, q);
    quat_rot(q[0], q[1], q[2], q[3], R);
    cov3d_from(v.scale_mod * s[0], v.scale_mod * s[1], v.scale_mod * s[2], R, c);
  }
  Proj2 pj;
  ewa_jacobian(v, tx, ty, tz, pj);
  float c00 = quad_form(pj.A0, c, pj.A0);
  const float c01 = quad_form(pj.A0, c, pj.A1);
  float c11 = quad_form(pj.A1, c, pj.A1);
  const float det0 = c00 * c11 - c01 * c01;
  c00 = c00 + 0.3f;
  c11 = c11 + 0.3f;
  const float det = c00 * c11 - c01 * c01;
  float h = 1.0f;
  if (v.antialiasing) h = sqrtf(fmaxf(0.000025f, det0 / det));
  if (det == 0.0f) return false;
  const float det_inv = 1.0f / det;
  o.conic[0] = c11 * det_inv;
  o.conic[1] = -c01 * det_inv;
  o.conic[2] = c00 * det_inv;
  const float mid = 0.5f * (c00 + c11);
  const float lam1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
  const float radius = ceilf(3.0f * sqrtf(lam1));
  o.x = ndc2pix(pxn, v.W);
  o.y = ndc2pix(pyn, v.H);
  o.rmin_x = min(v.gx, max(0, trunc_i((o.x - radius) / 16.0f)));
  o.rmin_y = min(v.gy, max(0, trunc_i((o.y - radius) / 16.0f)));
  o.rmax_x = min(v.gx, max(0, trunc_i((((o.x + radius) + 16.0f) - 1.0f) / 16.0f)));
  o.rmax_y = min(v.gy, max(0, trunc_i((((o.y + radius) + 16.0f) - 1.0f) / 16.0f)));
  if ((o.rmax_x - o.rmin_x) * (o.rmax_y - o.rmin_y) == 0) return false;

  o.clamped = 0u;
  if (g.colors) {
#pragma unroll
    for (int k = 0; k < 3; ++k) o.rgb[k] = g.colors[3 * i + k];
  } else {
    float dx = x - v.campos[0], dy = y - v.campos[1], dz = z - v.campos[2];
    const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    auto shf = [&](int k, int ch) { return g.sh(i, k, ch); };
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float r = sh_color(v.D, dx, dy, dz, shf, ch);
      if (r < 0.0f) o.clamped |= (1u << ch);
      o.rgb[ch] = fmaxf(r, 0.0f);
    }
  }
  const float op = RAW ? sigmoidf_(g.opac[i]) : g.opac[i];
  o.opac = op * h;
  o.depth = tz;
  o.radius = (int)radius;
  o.ext = alpha_extent(o.opac, o.conic[0], o.conic[1], o.conic[2]);
  return true;
}

// ---------------- workspace views ----------------
struct GeomBufs {
  float4* rec;            // [P*3]
  uint32_t* depth_key;    // [P]
  uint32_t* tiles;        // [P]
  uint2* rect;            // [P]
  uint32_t* sorted_idx;   // [P] Gaussian ids in depth order (after sort)
  uint32_t* keys_alt;     // [P]
  uint32_t* vals_alt;     // [P]
  uint32_t* vals_init;    // [P] identity
  uint32_t* offsets;      // [P] exclusive scan of tiles in depth order (duplicate emission)
  uint32_t* goff;         // [P] exclusive scan of tiles in Gaussian-index order (gradient-row slots)
  uint32_t* hist;         // radix histogram
  uint32_t* scan_tmp;     // scan block sums
  uint32_t* counters;     // [0] = num_rendered, [1] = sum of tiles (== [0])
};
// Binning: (tile id, Gaussian id) pairs emitted in depth order, stably sorted by tile id.
// The number of radix passes (hence which ping-pong buffer holds the result) depends only on the
// tile count, so every consumer derives the same point_list / keys_sorted pointers.
struct BinBufs {
  uint32_t* keys0;
  uint32_t* keys1;
  uint32_t* vals0;
  uint32_t* vals1;
  uint32_t* point_list;   // sorted Gaussian ids (aliases vals0 or vals1)
  uint32_t* keys_sorted;  // sorted tile ids (aliases keys0 or keys1)
  uint32_t* hist;
  uint2* ranges;
  int passes;
  int end_bit;
};
// Gradient rows: one row per (Gaussian, touched tile), at slot goff[g] + (ty - ymin) * nx + (tx - xmin),
// i.e. grouped by Gaussian index so the per-Gaussian sum reads contiguous memory.
__device__ __forceinline__ uint32_t row_slot(uint32_t goff_g, uint2 rc, int tx, int ty) {
  const int x0 = rc.x & 0xFFFF, y0 = rc.x >> 16, x1 = rc.y & 0xFFFF;
  return goff_g + (uint32_t)((ty - y0) * (x1 - x0) + (tx - x0));
}
struct ImgBufs {
  float* final_T;
  uint32_t* n_contrib;
};
struct ScratchBufs {
  float4* trec;   // [P*3] tangent render records
  float4* contrib; // [N*3] per (tile, Gaussian) reduced gradient rows
};

size_t geom_layout(int64_t P, void* base, GeomBufs* out);
size_t bin_layout(int64_t N, int ntiles, void* base, BinBufs* out);
size_t img_layout(int H, int W, void* base, ImgBufs* out);
size_t scratch_layout(int64_t P, int64_t N, void* base, ScratchBufs* out);

int launch_preprocess(const ViewK& v, const GaussK& g, const GeomBufs& gb, int* radii_out, hipStream_t s);
int launch_binning(const ViewK& v, int64_t P, const GeomBufs& gb, const BinBufs& bb, int64_t N, hipStream_t s);
int launch_render_fwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, float* out_color,
                      float* out_invdepth, hipStream_t s);

}  // namespace gslm

namespace gslm {
int launch_render_bwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                      const float* dL_dcolor, const float* dL_dinv, const ScratchBufs& sb, hipStream_t s);
int launch_preprocess_bwd(const ViewK& v, const GaussK& g, const GeomBufs& gb, const BinBufs& bb,
                          const ScratchBufs& sb, const GradK& out, bool want_means, hipStream_t s);
int launch_tangent_pre(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
                       const ScratchBufs& sb, hipStream_t s);
int launch_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
               const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb, float* out_color_t, float* out_inv_t,
               hipStream_t s);
int launch_matvec_render(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                         const ScratchBufs& sb, const float* weight, bool mask_xyz, hipStream_t s);
int launch_gather_lm(const ViewK& v, const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, const GradK& y,
                     const GradK& vin, const double* damp7, bool overwrite, bool mask_xyz, double* dot_part,
                     hipStream_t s);
}  // namespace gslm
