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
  int64_t rest_base = 0;  // rest holds Gaussians rest_base.. (an LDS-staged block slice) when nonzero
  // tangents only (GSLM_MV_SH_REST_PROJECTED): rest holds 3 floats per Gaussian, the coordinates of the
  // SH-rest tangent along the unit basis direction B_rest(dir) / |B_rest(dir)| of this view
  int rest_proj = 0;
  // tangents only, the Gaussian-sharded exchange's SH-rest coordinates (gslm_rest_basis): rest holds 3 rest_V
  // floats per Gaussian, rest_R the Gaussians' packed factors R (rest_V (rest_V + 1) / 2 floats each) and
  // rest_col this view's column of R
  const float* rest_R = nullptr;
  int rest_V = 0;
  int rest_col = 0;
  __device__ __forceinline__ float sh(int64_t i, int k, int c) const {
    return k == 0 ? dc[i * dc_stride + c] : rest[(i - rest_base) * rest_stride + 3 * (k - 1) + c];
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
  float tq;  // alpha threshold of the quadrant cull (alpha_threshold), stored in the record's r2.w
  int radius;
  int rmin_x, rmin_y, rmax_x, rmax_y;
};

// ---------------- quadrant culling (an exact-results skip, not an approximation) ----------------
// A 16x16 tile pass runs one wave per 8x8 quadrant (tile_pixel).  For every batch element the block
// computes which quadrants its alpha >= 1/255 region can reach, and each wave visits only those
// elements.  A skipped lane would have failed the alpha test, so results are bit-identical to
// visiting every element; only wasted iterations go.
//
// Exact math: alpha >= 1/255  <=>  Q(d) = A dx^2 + C dy^2 + 2 B dx dy <= t = 2 ln(255 o), with
// (A, B, C) the stored conic.  The float evaluation of Q in the tile passes (-ffp-contract=off, a
// handful of roundings per term, |2 B dx dy| <= max(A, C) |d|^2) errs by at most 14 eps (A + C) |d|^2,
// so every pixel a pass can accept satisfies d^T (Q - e I) d <= tq with e = 32 eps (A + C) and
// tq = t * 1.02 + 1e-4 (exp / log / 1/255-constant rounding), rounded up to float.  The quadrant test keeps a
// quadrant whenever that ellipse can reach it (quad_mask below), evaluated in float with widened bounds.

// tq for effective opacity o; negative when o <= 1/255 (no pixel can ever pass).
__device__ __forceinline__ float alpha_threshold(float op_eff) {
  if (!(op_eff * 255.0f > 1.0f)) return -1.0f;
  const double t = 2.0 * log(255.0 * (double)op_eff) * 1.02 + 1e-4;
  float f = (float)t;  // t > 0: the next float up is the next bit pattern
  if ((double)f < t) f = __uint_as_float(__float_as_uint(f) + 1u);
  return f;
}

// How the preprocess kernels may stage the block's SH rows in LDS: -1 not at all (colours given, degree 0, an odd
// layout); else the floats between a staged row's start and its rest -- 0 for the contiguous rest leaf, 3 for the rest
// inside a [P, M, 3] features tensor (rows staged from the dc slot).  The staged span must start 16-B aligned.
inline int stage_lead(const GaussK& g) {
  if (g.colors || !g.rest || g.M <= 1) return -1;
  int lead = -1;
  if (g.rest_stride == 3 * (g.M - 1)) lead = 0;
  else if (g.dc && g.rest == g.dc + 3 && g.dc_stride == g.rest_stride && g.rest_stride == 3 * g.M) lead = 3;
  if (lead < 0 || ((uintptr_t)(g.rest - lead) & 15u) != 0) return -1;
  return lead;
}

// Copies the block's [nv][rest_stride] SH rows (from `lead` floats before g.rest, stage_lead) to LDS with coalesced
// 16-B loads and points g.rest at the copy.  Block-uniform; ends with a barrier.
__device__ __forceinline__ void stage_sh_rows(GaussK& g, int lead, float* s_rows) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t nv = min((int64_t)blockDim.x, g.P - i0);
  const int64_t total = nv > 0 ? nv * g.rest_stride : 0;  // i0 * rest_stride * 4 B is 16-B aligned (i0 % 256 == 0)
  const float* rows = g.rest - lead + i0 * g.rest_stride;
  const float4* src4 = reinterpret_cast<const float4*>(rows);
  float4* dst4 = reinterpret_cast<float4*>(s_rows);
  for (int64_t e = threadIdx.x; e < total / 4; e += blockDim.x) dst4[e] = src4[e];
  for (int64_t e = (total / 4) * 4 + threadIdx.x; e < total; e += blockDim.x) s_rows[e] = rows[e];
  __syncthreads();
  g.rest = s_rows + lead;
  g.rest_base = i0;
}

// Per-Gaussian part of the quadrant test (k_duplicate prepares it once and tests every tile of the
// rect).  mode: 0 = reaches no pixel, 1 = treat every quadrant as reachable, 2 = test.
//
// The test works on E' = {d : a x^2 + 2 b x y + c y^2 <= t} with (a, b, c) = the conic minus e I (e above) and t = tq:
// every pixel a tile pass can accept lies in E'.  For a band of pixel rows y in [ya, yb] (offsets from the centre)
// E' spans x in [xmin(band), xmax(band)]: x_hi(y) = (-b y + sqrt(t a - det y^2)) / a is concave, so its maximum over
// the band is at the band point nearest y_r = -b x_r / c (the ellipse's rightmost point, x_r = sqrt(t c / det)),
// and by symmetry the minimum of x_lo(y) is at the point nearest -y_r.  A quadrant is kept when its columns meet
// that interval -- two square roots per band of 8 rows, for both quadrants of the band (the round-2 test bounded
// min over each quadrant of the form from its facing edges: four rectangles per entry, ~4x the VALU).  The
// interval is widened by 1e-4 of its terms' magnitude + 0.01 px, far above the few float roundings of its
// evaluation: looser only ever keeps a quadrant, so the cull stays exact.
struct QuadCull {
  float gx, gy, ia, b, det, ta, ydom, yr, sqm;
  int mode;
};

// NaN-safe: any NaN input yields mode 1 ("reachable").
__device__ __forceinline__ QuadCull quad_cull_prep(float gx, float gy, float A, float B, float C, float tq) {
  QuadCull q;
  q.mode = 2;
#ifdef GSLM_NO_STRIP_CULL
  q.mode = 1;
  return q;
#endif
  if (tq < 0.0f) {
    q.mode = 0;
    return q;
  }
  const float e = 32.0f * 5.9604644775390625e-8f * (A + C);
  const float a = A - e, c = C - e;
  const float det = a * c - B * B;
  // unbounded, nearly degenerate (ill-conditioned), an infinite threshold (the exhaustive traversal) or NaN:
  // every quadrant
  if (!(a > 0.0f && c > 0.0f && det > 1e-6f * (a * c) && tq < INFINITY)) {
    q.mode = 1;
    return q;
  }
  q.gx = gx;
  q.gy = gy;
  q.ia = 1.0f / a;
  q.b = B;
  q.det = det;
  q.ta = tq * a;
  q.ydom = sqrtf(q.ta / det) * 1.0001f + 0.01f;  // |y| over E'
  q.yr = -B * sqrtf(tq * c / det) / c;          // y of E''s rightmost point
  // sqrt(t a - det y^2) near the band ends of E' loses up to sqrt(eps t a) to the cancellation: widen by
  // sqrt(1e-6 t a) / a (16x that), besides the relative 1e-4 and the 0.01 px of band_x_extent
  q.sqm = sqrtf(1e-6f * q.ta) * q.ia;
  return q;
}

// [lo, hi] = the x extent of E' over the row band [ya, yb] (offsets), widened; false when the band misses E'.
__device__ __forceinline__ bool band_x_extent(const QuadCull& q, float ya, float yb, float& lo, float& hi) {
  const float y0 = fmaxf(ya, -q.ydom), y1 = fminf(yb, q.ydom);
  if (!(y0 <= y1)) return false;
  const float yh = fminf(fmaxf(q.yr, y0), y1), yl = fminf(fmaxf(-q.yr, y0), y1);
  // the hardware square root (v_sqrt_f32, within 1 ulp; sqrtf's correctly rounded expansion is ~4x the
  // instructions, and this runs per (tile, Gaussian) pair): its error is far inside the 1e-4 widening below
  const float sh = __builtin_amdgcn_sqrtf(fmaxf(q.ta - q.det * yh * yh, 0.0f));
  const float sl = __builtin_amdgcn_sqrtf(fmaxf(q.ta - q.det * yl * yl, 0.0f));
  const float bh = q.b * yh, bl = q.b * yl;
  hi = (sh - bh) * q.ia;
  lo = -(sl + bl) * q.ia;
  hi += 1e-4f * (fabsf(bh) + sh) * q.ia + q.sqm + 0.01f;
  lo -= 1e-4f * (fabsf(bl) + sl) * q.ia + q.sqm + 0.01f;
  return true;
}

// Quadrant mask of a Gaussian in tile (tile_x, tile_y): bit s set when its alpha region can reach
// quadrant s = pixels [8 (s & 1), +7] x [8 (s >> 1), +7] of the tile (wave s).
__device__ __forceinline__ uint32_t quad_mask(const QuadCull& q, int tile_x, int tile_y) {
  if (q.mode != 2) return q.mode ? 0xFu : 0u;
  const float bx = (float)(tile_x * TILE_X) - q.gx, by = (float)(tile_y * TILE_Y) - q.gy;
  uint32_t m = 0u;
#pragma unroll
  for (int band = 0; band < 2; ++band) {
    float lo, hi;
    const float ya = by + 8.0f * (float)band;
    if (!band_x_extent(q, ya, ya + 7.0f, lo, hi)) continue;
#pragma unroll
    for (int col = 0; col < 2; ++col) {
      const float xa = bx + 8.0f * (float)col;
      if (xa <= hi && xa + 7.0f >= lo) m |= 1u << (2 * band + col);
    }
  }
  return m;
}

// Upstream's Gaussian exponent -0.5 (a dx^2 + c dy^2) - b dx dy (renderCUDA's `power`), rounded exactly as its
// separate float operations: the products and the sum are formed as written (-ffp-contract=off), and since
// halving is exact, folding it and the final subtraction into one FMA gives the same rounded result as the
// separate multiply and subtract -- one instruction less per (entry, pixel) visit in every tile pass.
__device__ __forceinline__ float gpower(float a, float b, float c, float dx, float dy) {
  const float s = a * dx * dx + c * dy * dy;
  return __builtin_fmaf(-0.5f, s, -(b * dx * dy));
}

// point_list entries carry the Gaussian id in the low 28 bits and its quadrant mask (quad_mask,
// computed once per (tile, Gaussian) pair by k_duplicate) in the top 4 bits.
constexpr int ID_BITS = 28;
constexpr uint32_t ID_MASK = (1u << ID_BITS) - 1u;
constexpr int64_t MAX_P = (int64_t)ID_MASK;  // 268M Gaussians per view and GPU
__device__ __forceinline__ uint32_t pl_id(uint32_t e) { return e & ID_MASK; }
__device__ __forceinline__ uint32_t pl_mask(uint32_t e) { return e >> ID_BITS; }

// Pixel of thread tid in a 16x16 tile: wave w = tid >> 6 holds the 8x8 quadrant (w & 1, w >> 1).
__device__ __forceinline__ void tile_pixel(int tile_x, int tile_y, int tid, int& px, int& py) {
  const int w = tid >> 6, l = tid & 63;
  px = tile_x * TILE_X + 8 * (w & 1) + (l & 7);
  py = tile_y * TILE_Y + 8 * (w >> 1) + (l >> 3);
}

// Called by all 256 threads after thread tid has fetched batch element tid with quadrant mask m (0
// when tid is past the batch).  Publishes, per quadrant s, the 256-bit set of batch elements that
// can touch it: s_bits[4 s + c] holds elements 64c..64c+63.  Wave s then visits only those
// elements, in list order (wave_bits / s_ff1).
__device__ __forceinline__ void publish_quad_masks(uint32_t m, uint64_t* s_bits) {
  const int c = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint64_t b = __ballot((m >> s) & 1u);
    if ((threadIdx.x & 63) == 0) s_bits[4 * s + c] = b;
  }
}

// The 64-element hit set c of quadrant (wave) s as a wave-uniform (SGPR) value.
__device__ __forceinline__ uint64_t wave_bits(const uint64_t* s_bits, int s, int c) {
  const uint64_t b = s_bits[4 * s + c];
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Mask m with bit j cleared, one scalar ALU instruction: the hit loops' `hb &= hb - 1` for j = ctz(hb) was three
// (s_add_u32 + s_addc_u32 + s_and_b64), and those loops issue about as many SALU as VALU instructions per visit.
// Register-only (no memory access).
__device__ __forceinline__ uint64_t clear_bit(uint64_t m, int j) {
  asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(j));
  return m;
}

// Wave-uniform iterator over wave s's hit set of the current batch, in list order.
struct HitIter {
  const uint64_t* s_bits;
  uint64_t cur;
  int s, c;
  __device__ __forceinline__ HitIter(const uint64_t* sb, int s_) : s_bits(sb), s(s_), c(0) { cur = wave_bits(sb, s_, 0); }
  // next batch index, or -1 once the set is exhausted
  __device__ __forceinline__ int next() {
    while (cur == 0ull) {
      if (c == 3) return -1;
      cur = wave_bits(s_bits, s, ++c);
    }
    const int b = (int)__builtin_ctzll(cur);
    cur = clear_bit(cur, b);
    return 64 * c + b;
  }
};

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

// The per-Gaussian inputs of the preprocess, loaded apart from its arithmetic (k_preprocess_dma loads them before
// it issues the SH-rest LDS-DMA, so the arithmetic runs while that lands).
struct PreIn {
  float x, y, z;
  float c[6];  // cov3D_precomp, or (s0 s1 s2 | q0 q1 q2 q3 in c[3..5] and qw) -- see load_pre_in
  float qw;
  float op;
};

template <bool RAW>
__device__ __forceinline__ void load_pre_in(const GaussK& g, int64_t i, PreIn& in) {
  in.x = g.means3D[3 * i + 0];
  in.y = g.means3D[3 * i + 1];
  in.z = g.means3D[3 * i + 2];
  // one load per element from a selected address (no branch): with two branches the compiler sank their stores
  // into one store at a run-time index, which put in.c in scratch memory
  const bool cv = g.cov3D != nullptr;
#pragma unroll
  for (int k = 0; k < 3; ++k) in.c[k] = *(cv ? g.cov3D + 6 * i + k : g.scales + 3 * i + k);
#pragma unroll
  for (int k = 0; k < 3; ++k) in.c[3 + k] = *(cv ? g.cov3D + 6 * i + 3 + k : g.rot + 4 * i + k);
  in.qw = cv ? 0.f : g.rot[4 * i + 3];
  in.op = g.opac[i];
}

// Step 8 (colour) of one Gaussian: colors_precomp, or SH (utils/sh_utils.py:57-112) -> max(result + 0.5, 0) with
// the clamp mask (gaussian_renderer/__init__.py:79-80).
__device__ __forceinline__ void preprocess_color(const ViewK& v, const GaussK& g, int64_t i, const PreIn& in, PreOut& o) {
  o.clamped = 0u;
  if (g.colors) {
#pragma unroll
    for (int k = 0; k < 3; ++k) o.rgb[k] = g.colors[3 * i + k];
  } else {
    float dx = in.x - v.campos[0], dy = in.y - v.campos[1], dz = in.z - v.campos[2];
    const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    auto shf = [&](int k, int ch) { return g.sh(i, k, ch); };
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float r = sh_color(v.D, dx, dy, dz, shf, ch);
      if (r < 0.0f) o.clamped |= (1u << ch);
      o.rgb[ch] = r < 0.0f ? 0.0f : r;  // upstream's glm::max(result, 0): a NaN coefficient stays a NaN colour
    }
  }
}

// SURVEY Appendix A steps 1-9 for one Gaussian from its loaded inputs; returns false when culled.  COLOR = false
// leaves o.rgb / o.clamped to preprocess_color (the SH-rest rows not yet staged).
template <bool RAW, bool COLOR>
__device__ __forceinline__ bool preprocess_core(const ViewK& v, const GaussK& g, int64_t i, const PreIn& in, PreOut& o) {
  const float x = in.x, y = in.y, z = in.z;
  const float tz = tp_row(v.view, x, y, z, 2);
  o.depth = tz;  // set before any cull: the depth order of every Gaussian in front of the near plane
  if (!(tz > 0.2f)) return false;
  const float tx = tp_row(v.view, x, y, z, 0), ty = tp_row(v.view, x, y, z, 1);
  const float hx = tp_row(v.proj, x, y, z, 0), hy = tp_row(v.proj, x, y, z, 1), hw = tp_row(v.proj, x, y, z, 3);
  const float p_w = 1.0f / (hw + 0.0000001f);
  const float pxn = hx * p_w, pyn = hy * p_w;

  float c[6];
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = in.c[k];
  } else {
    float s[3], q[4], R[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] = RAW ? expf(in.c[k]) : in.c[k];
    q[0] = in.c[3];
    q[1] = in.c[4];
    q[2] = in.c[5];
    q[3] = in.qw;
    if (RAW) {  // load_scale_rot's normalisation (gaussian_model.py:198)
      const float nrm = fmaxf(sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]), 1e-12f);
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = q[k] / nrm;
    }
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

  if (COLOR) preprocess_color(v, g, i, in, o);
  const float op = RAW ? sigmoidf_(in.op) : in.op;
  o.opac = op * h;
  o.depth = tz;
  o.radius = (int)radius;
  o.tq = v.exhaustive ? INFINITY : alpha_threshold(o.opac);  // INFINITY: every quadrant visited
  return true;
}

template <bool RAW>
__device__ __forceinline__ bool preprocess_one(const ViewK& v, const GaussK& g, int64_t i, PreOut& o) {
  PreIn in;
  load_pre_in<RAW>(g, i, in);
  return preprocess_core<RAW, true>(v, g, i, in, o);
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
  uint32_t* clampw;       // [P] SH clamp bits of each visible Gaussian's colour (rec r2.z), read coalesced by the
                          //     per-Gaussian passes instead of a 64-B record line each
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
  uint32_t* tile_order;   // tiles by descending list length: the launch order of the tile passes
  uint32_t* slots;        // [N] gradient-row slot of each sorted entry, in the sort's free ping-pong key
                          // buffer: the LM row map (launch_lm_rowmap) once an LM product computed it for the
                          // current binning
  uint32_t* tile_neff;    // [4 ntiles] largest n_contrib of each tile quadrant's pixels (the LM row map's head bounds)
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
  // The LM row map: the rows of the LM tile passes exist only for HEAD entries (their quadrant mask holds a
  // quadrant whose largest n_contrib lies past their list position -- every other entry's row would be zero: no
  // pixel still blending at that position can reach it).  hscan[o] = number of head
  // entries among the goff-order slots [0, o), o <= N, so Gaussian g's rows are [hscan[goff[g]],
  // hscan[goff[g] + tiles[g]]), contiguous; each sorted head entry's row slot is hscan of its goff slot.
  uint32_t* hscan;    // [N + 1]
  uint32_t* scan_tmp; // block sums of the scan over N
};

size_t geom_layout(int64_t P, void* base, GeomBufs* out);
size_t bin_layout(int64_t N, int ntiles, void* base, BinBufs* out);
size_t img_layout(int H, int W, void* base, ImgBufs* out);
size_t scratch_layout(int64_t P, int64_t N, void* base, ScratchBufs* out);

int launch_preprocess(const ViewK& v, const GaussK& g, const GeomBufs& gb, int* radii_out, hipStream_t s);
// several views in one pass over the Gaussians (gslm_preprocess_views): each view's records, depth keys, tile counts,
// rects and clamp words, no sort and no scan
constexpr int MAX_PRE_VIEWS = 8;
struct PreOutBufs {
  float4* rec;
  uint32_t* depth_key;
  uint32_t* tiles;
  uint2* rect;
  uint32_t* clampw;
  const uint32_t* pos;  // or NULL: depth space (the render records alone, at pos[i]; rect slot zero when culled)
};
struct PreViewsK {
  ViewK v[MAX_PRE_VIEWS];
  PreOutBufs out[MAX_PRE_VIEWS];
  int n;
};
int launch_preprocess_views(const PreViewsK& pv, const GaussK& g, const GeomBufs* gbs, hipStream_t s);
// device_count: N is the list capacity and the count stays on the device (gslm_rasterize_dev); n_out (device, or
// NULL) receives the count
int launch_binning(const ViewK& v, int64_t P, const GeomBufs& gb, const BinBufs& bb, int64_t N, hipStream_t s,
                   bool device_count = false, uint32_t* n_out = nullptr);
int launch_lm_rowmap(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb,
                     int64_t N, hipStream_t s);
int launch_point_ids(const uint32_t* point_list, int64_t N, uint32_t* out, hipStream_t s);
// amask (or NULL): the blend visits by the union list's per-set masks (bits `shift` .. shift + 3 of amask[k],
// k_duplicate_union) with the records of gb (that set's geometry) instead of the point list's own quadrant bits
int launch_render_loss(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const float* gt, const float* mask,
                       double* part, double* loss, int accumulate, hipStream_t s, const uint32_t* amask = nullptr,
                       int shift = 0, const uint32_t* nsets = nullptr);
// ---- the line search's shared binning (forward.hip, gslm_union_*) ----
constexpr int MAX_UNION_SETS = 8;  // 4 mask bits per set in one uint32 per list entry
struct UnionSets {
  const float4* rec[MAX_UNION_SETS];
  const uint32_t* tiles[MAX_UNION_SETS];
  const uint2* rect[MAX_UNION_SETS];
  int n;
};
// the union list's per-entry set masks: the tile sort's ping-pong pair after the binning layout; `sorted` is the one
// holding the result (the same pass parity as the point list)
struct UnionMasks {
  uint32_t* m0;
  uint32_t* m1;
  uint32_t* sorted;
  uint32_t* hist;  // the payload sort's histograms (sort_hist_bytes(N, true): more, smaller blocks than the pair sort)
  uint32_t* nsets; // [4]: the set count gslm_union_binning built the masks for (a slot past it renders a NaN loss)
};
size_t union_masks_layout(int64_t N, int ntiles, void* binning, UnionMasks* out);
// all sets' blends + losses over a union list in one pass (render_fwd.hip, gslm_rasterize_loss_sets)
struct SetRecsK {
  const float4* rec[MAX_UNION_SETS];
};
struct LossPtrsK {
  double* loss[MAX_UNION_SETS];
};
int launch_render_loss_sets(const ViewK& v, const SetRecsK& sr, int nsets, const BinBufs& bb, const uint32_t* amask,
                            const float* gt, const float* mask, double* part, const LossPtrsK& lp, int accumulate,
                            hipStream_t s, int first_set = 0, const uint32_t* nsets_dev = nullptr);
int launch_union_rect(int64_t P, const UnionSets& u, const GeomBufs& ug, hipStream_t s);
int launch_depth_positions(int64_t P, const uint32_t* order, uint32_t* pos, hipStream_t s);
int launch_union_binning(const ViewK& v, int64_t P, const GeomBufs& ug, const BinBufs& bb, const UnionMasks& um,
                         int64_t N, const UnionSets& u, hipStream_t s);
int launch_render_fwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, float* out_color,
                      float* out_invdepth, hipStream_t s);

}  // namespace gslm

namespace gslm {
int launch_render_bwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                      const float* dL_dcolor, const float* dL_dinv, const ScratchBufs& sb, hipStream_t s);
int launch_render_vjp_lm(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                         const float* dL_dcolor, const ScratchBufs& sb, bool tail_clean, hipStream_t s);
int launch_preprocess_bwd(const ViewK& v, const GaussK& g, const GeomBufs& gb, const BinBufs& bb,
                          const ScratchBufs& sb, const GradK& out, bool want_means, hipStream_t s);
// Fused CG direction update run by the tangent kernel before it reads the direction: every
// per-Gaussian group k (xyz, dc, rest, scaling, rotation, opacity) of p becomes s + beta p over its
// contiguous slice of width w[k] floats per Gaussian, plus a flat tail (the exposure group).
struct XpbyK {
  float* p[6];
  const float* s[6];
  int w[6];
  const double* num;
  const double* den;
  float* tail_p;
  const float* tail_s;
  int64_t tail_n;
  // deferred x update of the previous CG step, applied to the old p first: x += (anum / aden) p, with x at
  // p + xoff floats for every group and for the tail (anum == NULL: off)
  const double* anum;
  const double* aden;
  int64_t xoff;
};
// compact: the LM rows' 8-float tangent records (store_trec, tangent.hip) instead of 12 floats
int launch_tangent_pre(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
                       const ScratchBufs& sb, const XpbyK* xp, hipStream_t s, bool compact);
int launch_rowsum_screen(const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, float* out, hipStream_t s);
constexpr int MAX_SCREEN_VIEWS = 16;
constexpr int MAX_REST_VIEWS = GSLM_MAX_REST_VIEWS;
// packed upper-triangular factor R of gslm_rest_basis: column b starts at b (b + 1) / 2
__host__ __device__ constexpr int rest_basis_floats(int V) { return V * (V + 1) / 2; }
// SH-rest coordinates for launch_gather_screen (nullptr R: the full [M-1][3] layout)
struct RestK {
  const float* R = nullptr;
  int V = 0;
  int view_base = 0;
};
struct ViewsK {
  ViewK v[MAX_SCREEN_VIEWS];
  int n;
};
int launch_gather_screen(const ViewK* views, int nviews, const GaussK& g, const float* screen, int64_t sstride,
                         const GradK& y, const GradK& vin, const double* damp7, bool overwrite, double* dot_part,
                         hipStream_t s, const RestK& rc = RestK{});
int launch_rest_basis(const ViewK* views, int nviews, const GaussK& g, float* R, hipStream_t s);
int launch_rest_coords(const ViewK* views, int nviews, const GaussK& g, const float* R, int mode, const float* in,
                       int64_t in_stride, float* out, int64_t out_stride, hipStream_t s);
int launch_view_flags(int64_t P, const GeomBufs& gb, uint32_t* out, hipStream_t s);
int launch_tangent_views(const ViewK* views, int nviews, const GaussK& g, const GaussK& t, const uint32_t* vflags,
                         int64_t fstride, float* out, int64_t ostride, const XpbyK* xp, hipStream_t s, bool compact,
                         int view_base = 0);
int launch_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
               const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb, float* out_color_t, float* out_inv_t,
               hipStream_t s);
int launch_render_jv(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                     const ScratchBufs& sb, bool mask_xyz, float* jv_out, hipStream_t s);
int launch_matvec_render(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                         const ScratchBufs& sb, int64_t N, const float* weight, bool mask_xyz, bool tail_clean,
                         hipStream_t s);
int launch_gather_lm(const ViewK& v, const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, const GradK& y,
                     const GradK& vin, const double* damp7, bool overwrite, bool mask_xyz, double* dot_part,
                     hipStream_t s, bool rest_proj = false);
int launch_sh_rest_project(const ViewK& v, const GaussK& g, int mode, const float* in, int64_t in_stride, float* out,
                           int64_t out_stride, hipStream_t s);
}  // namespace gslm
