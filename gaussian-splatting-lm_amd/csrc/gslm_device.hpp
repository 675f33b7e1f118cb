// gslm_device.hpp -- device-side math shared by the forward / JVP / VJP kernels (gfx950, wave64).
//
// Semantics: SURVEY Appendix A (upstream graphdeco rasterizer, restated in oracle/torch_raster.py).
// Operation order deliberately mirrors the oracle so that primal decisions (cull, radius, rect,
// alpha skip, T stop) agree bit-for-bit with the CPU restatement; the library is built with
// -ffp-contract=off for the same reason.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gslm.h"

// The product library has no experiment branches: a build that skips or stubs out part of a product kernel
// (the round-1/2 timing experiments) computes wrong results, so such flags are refused outright.
#if defined(GSLM_EXPERIMENT_COUNT) || defined(GSLM_EXPERIMENT_TIMELINE) || defined(GSLM_EXPERIMENT_SKIP_JVP) || \
    defined(GSLM_EXPERIMENT_SKIP_VJP) || defined(GSLM_EXPERIMENT_NOSYNC)
#error "GSLM_EXPERIMENT_* flags are not part of the product build (libgslm.so)"
#endif

namespace gslm {

constexpr int TILE_X = 16;
constexpr int TILE_Y = 16;
constexpr int TILE_PIX = TILE_X * TILE_Y;  // 256 threads = 4 wave64 per tile
constexpr int REC_F4 = 3;                  // 3 float4 (48 B): drop-in tangent records and gradient rows
// Render records [x y a b | c o r g | b 1/z clampbits z] (48 B) at a 64-B stride: a record never straddles a
// 128-B line, so each gather of one by the tile passes pulls a single line.
constexpr int RECS = 4;

// utils/sh_utils.py:26-55
__constant__ static const float SH_C0 = 0.28209479177387814f;
__constant__ static const float SH_C1 = 0.4886025119029199f;

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk3(float x, float y, float z) { return {x, y, z}; }

// Per-view constants handed to every kernel by value (kernarg -> SGPRs).
struct ViewK {
  int H, W, gx, gy;
  float focal_x, focal_y, limx, limy;   // W/(2 tanfovx), H/(2 tanfovy), 1.3 tanfov (rounded from double on host)
  float view[16];                        // column-major world->view (world_view_transform storage)
  float proj[16];                        // column-major full projection
  float campos[3];
  float bg[3];
  float scale_mod;
  int D;                                 // active SH degree
  int M;                                 // SH coefficients stored per Gaussian
  int antialiasing;
  int exhaustive;                        // gslm_view.debug: disable the quadrant cull (reference traversal)
  // gslm_matvec_opts.cg_ctl: the device CG control block; a product kernel of a stopped solve (stop[0] != 0)
  // returns at once (cgls_fused's device-side stopping tests; NULL outside the CG loop)
  const double* stop = nullptr;
};

// torch.clamp(x, 0, 1) (the reference's rendered_image.clamp(0, 1), batch_render.py:118): a NaN stays a NaN, as in
// torch -- fminf / fmaxf would turn it into 0 or 1 and hide it from the reference's NaN asserts (solver_functions.py:
// 125-130).  Identical to fminf(fmaxf(x, 0), 1) for every other input.
// Thread-strided in-order sum ((x[t] + x[t + T]) + x[t + 2T]) + ... (T = blockDim.x) with the loads issued 8 at a
// time: one memory latency per 8 partials, where the one-at-a-time loop waited on every load.  The additions keep
// that loop's order (a skipped slot adds nothing), so the sum is bitwise the same -- the deterministic reductions'
// contract.
template <typename F>
__device__ __forceinline__ F strided_sum_in_order(const F* __restrict__ x, int64_t n) {
  F acc = F(0);
  const int64_t T = blockDim.x;
  for (int64_t i = threadIdx.x; i < n; i += 8 * T) {
    F v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i + k * T < n ? x[i + k * T] : F(0);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i + k * T < n) acc += v[k];
  }
  return acc;
}

__device__ __forceinline__ float clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

// block-uniform early exit of a product kernel once the device-side CG stopping tests fired
__device__ __forceinline__ bool cg_stopped(const ViewK& v) { return v.stop != nullptr && *v.stop != 0.0; }

// transformPoint4x3 / 4x4, one row at a time (same association as the oracle)
__device__ __forceinline__ float tp_row(const float* m, float x, float y, float z, int r) {
  return ((x * m[r] + y * m[4 + r]) + z * m[8 + r]) + m[12 + r];
}

// quaternion (r,x,y,z) -> rotation matrix, utils/general_utils.py:91-99 (no renormalisation)
__device__ __forceinline__ void quat_rot(float r, float x, float y, float z, float R[9]) {
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - r * z); R[2] = 2.f * (x * z + r * y);
  R[3] = 2.f * (x * y + r * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - r * x);
  R[6] = 2.f * (x * z - r * y); R[7] = 2.f * (y * z + r * x); R[8] = 1.f - 2.f * (x * x + y * y);
}

// cov3D = R diag(s)^2 R^T upper triangle (scene/gaussian_model.py:36-40)
__device__ __forceinline__ void cov3d_from(float sx, float sy, float sz, const float R[9], float c[6]) {
  const float s[3] = {sx, sy, sz};
  float L[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) L[i * 3 + j] = R[i * 3 + j] * s[j];
  auto dotrow = [&](int a, int b) { return (L[a * 3 + 0] * L[b * 3 + 0] + L[a * 3 + 1] * L[b * 3 + 1]) + L[a * 3 + 2] * L[b * 3 + 2]; };
  c[0] = dotrow(0, 0); c[1] = dotrow(0, 1); c[2] = dotrow(0, 2);
  c[3] = dotrow(1, 1); c[4] = dotrow(1, 2); c[5] = dotrow(2, 2);
}

// EWA projection pieces: A = J * W2C (2x3).  W2C[j][k] = view[4k + j].
struct Proj2 {
  float A0[3], A1[3];
  float J00, J02, J11, J12;
  float tz, tcx, tcy;
  bool inx, iny;
};

__device__ __forceinline__ void ewa_jacobian(const ViewK& v, float tx, float ty, float tz, Proj2& p) {
  const float txtz = tx / tz, tytz = ty / tz;
  p.inx = (txtz >= -v.limx) && (txtz <= v.limx);
  p.iny = (tytz >= -v.limy) && (tytz <= v.limy);
  p.tcx = fminf(v.limx, fmaxf(-v.limx, txtz)) * tz;
  p.tcy = fminf(v.limy, fmaxf(-v.limy, tytz)) * tz;
  p.tz = tz;
  p.J00 = v.focal_x / tz;
  p.J02 = -(v.focal_x * p.tcx) / (tz * tz);
  p.J11 = v.focal_y / tz;
  p.J12 = -(v.focal_y * p.tcy) / (tz * tz);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    p.A0[k] = p.J00 * v.view[4 * k + 0] + p.J02 * v.view[4 * k + 2];
    p.A1[k] = p.J11 * v.view[4 * k + 1] + p.J12 * v.view[4 * k + 2];
  }
}

// a^T Sigma b with Sigma from the 6-vector, summation order of the oracle's quad()
__device__ __forceinline__ float quad_form(const float a[3], const float c[6], const float b[3]) {
  const float S0[3] = {c[0], c[1], c[2]}, S1[3] = {c[1], c[3], c[4]}, S2[3] = {c[2], c[4], c[5]};
  const float r0 = (S0[0] * b[0] + S0[1] * b[1]) + S0[2] * b[2];
  const float r1 = (S1[0] * b[0] + S1[1] * b[1]) + S1[2] * b[2];
  const float r2 = (S2[0] * b[0] + S2[1] * b[1]) + S2[2] * b[2];
  return (a[0] * r0 + a[1] * r1) + a[2] * r2;
}

// SH basis values B_k(dir) with the reference's signs folded in, so rgb = sum_k B_k * sh_k.
// Order of evaluation of the colour itself is done in sh_color() to mirror eval_sh.
__device__ __forceinline__ void sh_basis(int D, float x, float y, float z, float B[16]) {
  B[0] = SH_C0;
  if (D > 0) { B[1] = -SH_C1 * y; B[2] = SH_C1 * z; B[3] = -SH_C1 * x; }
  if (D > 1) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    B[4] = 1.0925484305920792f * xy;
    B[5] = -1.0925484305920792f * yz;
    B[6] = 0.31539156525252005f * (2.0f * zz - xx - yy);
    B[7] = -1.0925484305920792f * xz;
    B[8] = 0.5462742152960396f * (xx - yy);
    if (D > 2) {
      B[9] = -0.5900435899266435f * y * (3.0f * xx - yy);
      B[10] = 2.890611442640554f * xy * z;
      B[11] = -0.4570457994644658f * y * (4.0f * zz - xx - yy);
      B[12] = 0.3731763325901154f * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
      B[13] = -0.4570457994644658f * x * (4.0f * zz - xx - yy);
      B[14] = 1.445305721320277f * z * (xx - yy);
      B[15] = -0.5900435899266435f * x * (xx - 3.0f * yy);
    }
  }
}

// d B_k / d dir (3 components per k), used by the xyz tangent / gradient through the view direction.
__device__ __forceinline__ void sh_basis_grad(int D, float x, float y, float z, float dB[16][3]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) dB[k][0] = dB[k][1] = dB[k][2] = 0.f;
  if (D > 0) { dB[1][1] = -SH_C1; dB[2][2] = SH_C1; dB[3][0] = -SH_C1; }
  if (D > 1) {
    const float C20 = 1.0925484305920792f, C21 = -1.0925484305920792f, C22 = 0.31539156525252005f,
                C23 = -1.0925484305920792f, C24 = 0.5462742152960396f;
    dB[4][0] = C20 * y; dB[4][1] = C20 * x;
    dB[5][1] = C21 * z; dB[5][2] = C21 * y;
    dB[6][0] = C22 * (-2.f * x); dB[6][1] = C22 * (-2.f * y); dB[6][2] = C22 * (4.f * z);
    dB[7][0] = C23 * z; dB[7][2] = C23 * x;
    dB[8][0] = C24 * (2.f * x); dB[8][1] = C24 * (-2.f * y);
    if (D > 2) {
      const float xx = x * x, yy = y * y, zz = z * z;
      const float C30 = -0.5900435899266435f, C31 = 2.890611442640554f, C32 = -0.4570457994644658f,
                  C33 = 0.3731763325901154f, C34 = -0.4570457994644658f, C35 = 1.445305721320277f,
                  C36 = -0.5900435899266435f;
      // B9 = C30 y (3xx - yy)
      dB[9][0] = C30 * y * 6.f * x; dB[9][1] = C30 * (3.f * xx - 3.f * yy);
      // B10 = C31 x y z
      dB[10][0] = C31 * y * z; dB[10][1] = C31 * x * z; dB[10][2] = C31 * x * y;
      // B11 = C32 y (4zz - xx - yy)
      dB[11][0] = C32 * y * (-2.f * x); dB[11][1] = C32 * (4.f * zz - xx - 3.f * yy); dB[11][2] = C32 * y * 8.f * z;
      // B12 = C33 z (2zz - 3xx - 3yy)
      dB[12][0] = C33 * z * (-6.f * x); dB[12][1] = C33 * z * (-6.f * y); dB[12][2] = C33 * (6.f * zz - 3.f * xx - 3.f * yy);
      // B13 = C34 x (4zz - xx - yy)
      dB[13][0] = C34 * (4.f * zz - 3.f * xx - yy); dB[13][1] = C34 * x * (-2.f * y); dB[13][2] = C34 * x * 8.f * z;
      // B14 = C35 z (xx - yy)
      dB[14][0] = C35 * z * 2.f * x; dB[14][1] = C35 * z * (-2.f * y); dB[14][2] = C35 * (xx - yy);
      // B15 = C36 x (xx - 3yy)
      dB[15][0] = C36 * (3.f * xx - 3.f * yy); dB[15][1] = C36 * x * (-6.f * y);
    }
  }
}

// Colour from SH, mirroring eval_sh's association (utils/sh_utils.py:57-112) channel by channel.
// sh(k, c) accessor; returns result + 0.5 (before the clamp).
template <typename SH>
__device__ __forceinline__ float sh_color(int D, float x, float y, float z, const SH& sh, int c) {
  float result = SH_C0 * sh(0, c);
  if (D > 0) {
    result = ((result - SH_C1 * y * sh(1, c)) + SH_C1 * z * sh(2, c)) - SH_C1 * x * sh(3, c);
    if (D > 1) {
      const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
      result = ((((result + 1.0925484305920792f * xy * sh(4, c)) + -1.0925484305920792f * yz * sh(5, c))
                 + 0.31539156525252005f * (2.0f * zz - xx - yy) * sh(6, c))
                + -1.0925484305920792f * xz * sh(7, c)) + 0.5462742152960396f * (xx - yy) * sh(8, c);
      if (D > 2) {
        result = ((((((result + -0.5900435899266435f * y * (3.0f * xx - yy) * sh(9, c))
                      + 2.890611442640554f * xy * z * sh(10, c))
                     + -0.4570457994644658f * y * (4.0f * zz - xx - yy) * sh(11, c))
                    + 0.3731763325901154f * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh(12, c))
                   + -0.4570457994644658f * x * (4.0f * zz - xx - yy) * sh(13, c))
                  + 1.445305721320277f * z * (xx - yy) * sh(14, c))
                 + -0.5900435899266435f * x * (xx - 3.0f * yy) * sh(15, c);
      }
    }
  }
  return result + 0.5f;
}

__device__ __forceinline__ int trunc_i(float v) {
  v = fminf(fmaxf(v, -1073741824.f), 1073741824.f);
  return (int)v;
}

__device__ __forceinline__ float ndc2pix(float v, int S) {
  // upstream evaluates ((v + 1.0) * S - 1.0) * 0.5 in double
  return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

// exp of the Gaussian falloff in the tile passes.  Every GPU tile pass (forward, JVP, VJP, fused
// matvec) uses this same function, so their skip / stop decisions agree bit for bit with each
// other.  Default: the hardware exp2 path (v_exp_f32, ~2 ulp); -DGSLM_PRECISE_EXP selects the
// correctly-rounded-ish libm expf (closer to the CPU oracle's decisions, ~10 more instructions).
__device__ __forceinline__ float gexp(float x) {
#ifdef GSLM_PRECISE_EXP
  return expf(x);
#else
  return __expf(x);
#endif
}
// 1/x via v_rcp_f32 (1 ulp); used where upstream divides T by (1 - alpha)
__device__ __forceinline__ float rcp_f(float x) { return __builtin_amdgcn_rcpf(x); }

// numerically stable sigmoid matching torch.sigmoid for float
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

}  // namespace gslm
