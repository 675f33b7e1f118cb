// gslm_chain.hpp -- per-Gaussian derivative chains between the screen-space render record
// (xy, conic, opacity, rgb, invdepth) and the inputs (means3D, scales, rotations, opacities, SH or
// the precomputed cov3D / colours), in reverse mode (chain_vjp) and forward mode (chain_jvp).
//
// Upstream references (absent submodule, SURVEY §2 kernel table): BACKWARD::preprocess,
// computeCov2DCUDA, computeCov3D, computeColorFromSH.  Linearisation quirks kept:
//   * tan-FoV clamp: dt.x / dt.y masked outside +-1.3 tanfov, t.x / t.y treated as independent of
//     t.z inside J (upstream dL_dtz formula);
//   * SH clamp mask; alpha clamp pass-through (in the tile passes).
// chain_jvp is the exact transpose of chain_vjp (checked by the adjoint test).
#pragma once
#include "gslm_kernels.hpp"

namespace gslm {

struct Geo {
  float x, y, z;
  float tx, ty, tz;
  float hx, hy, p_w;
  float c[6];       // cov3D upper triangle
  float s[3], sp[3];// activated scale, scale * modifier
  float q[4];       // activated (normalised) quaternion
  float qnorm;      // |q_raw| (RAW)
  float R[9];
  Proj2 pj;
  float a, b, cc;   // cov2D + low-pass: (c00+0.3, c01, c11+0.3)
  float det, det0, h;
  float op;         // activated opacity (before AA)
  float dir[3], dirlen;
  uint32_t clamped;
};

template <bool RAW>
__device__ __forceinline__ void compute_geo(const ViewK& v, const GaussK& g, int64_t i, uint32_t clamped, Geo& e) {
  e.x = g.means3D[3 * i + 0];
  e.y = g.means3D[3 * i + 1];
  e.z = g.means3D[3 * i + 2];
  e.tx = tp_row(v.view, e.x, e.y, e.z, 0);
  e.ty = tp_row(v.view, e.x, e.y, e.z, 1);
  e.tz = tp_row(v.view, e.x, e.y, e.z, 2);
  e.hx = tp_row(v.proj, e.x, e.y, e.z, 0);
  e.hy = tp_row(v.proj, e.x, e.y, e.z, 1);
  const float hw = tp_row(v.proj, e.x, e.y, e.z, 3);
  e.p_w = 1.0f / (hw + 0.0000001f);
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; ++k) e.c[k] = g.cov3D[6 * i + k];
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k) e.s[k] = RAW ? expf(g.scales[3 * i + k]) : g.scales[3 * i + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) e.q[k] = g.rot[4 * i + k];
    e.qnorm = 1.f;
    if (RAW) {
      e.qnorm = fmaxf(sqrtf(((e.q[0] * e.q[0] + e.q[1] * e.q[1]) + e.q[2] * e.q[2]) + e.q[3] * e.q[3]), 1e-12f);
#pragma unroll
      for (int k = 0; k < 4; ++k) e.q[k] = e.q[k] / e.qnorm;
    }
    quat_rot(e.q[0], e.q[1], e.q[2], e.q[3], e.R);
#pragma unroll
    for (int k = 0; k < 3; ++k) e.sp[k] = v.scale_mod * e.s[k];
    cov3d_from(e.sp[0], e.sp[1], e.sp[2], e.R, e.c);
  }
  ewa_jacobian(v, e.tx, e.ty, e.tz, e.pj);
  const float c00 = quad_form(e.pj.A0, e.c, e.pj.A0);
  const float c01 = quad_form(e.pj.A0, e.c, e.pj.A1);
  const float c11 = quad_form(e.pj.A1, e.c, e.pj.A1);
  e.det0 = c00 * c11 - c01 * c01;
  e.a = c00 + 0.3f;
  e.b = c01;
  e.cc = c11 + 0.3f;
  e.det = e.a * e.cc - e.b * e.b;
  e.h = v.antialiasing ? sqrtf(fmaxf(0.000025f, e.det0 / e.det)) : 1.0f;
  e.op = RAW ? sigmoidf_(g.opac[i]) : g.opac[i];
  float dx = e.x - v.campos[0], dy = e.y - v.campos[1], dz = e.z - v.campos[2];
  e.dirlen = sqrtf((dx * dx + dy * dy) + dz * dz);
  e.dir[0] = dx / e.dirlen;
  e.dir[1] = dy / e.dirlen;
  e.dir[2] = dz / e.dirlen;
  e.clamped = clamped;
}

// derivative of h = sqrt(max(2.5e-5, det0/det)) w.r.t. (a, b, c); zero when the max clamps
__device__ __forceinline__ void aa_grad(const Geo& e, float& ha, float& hb, float& hc) {
  ha = hb = hc = 0.f;
  const float ratio = e.det0 / e.det;
  if (ratio > 0.000025f) {
    const float k = 0.5f / e.h / (e.det * e.det);
    ha = k * ((e.cc - 0.3f) * e.det - e.det0 * e.cc);
    hb = k * (-2.f * e.b * e.det + 2.f * e.b * e.det0);
    hc = k * ((e.a - 0.3f) * e.det - e.det0 * e.a);
  }
}

// |B_rest(dir)|: the norm of the SH basis values of coefficients 1..nc-1 (for real orthonormal SH it is
// sqrt(sum_{l=1..D} (2l+1) / 4 pi) at every direction; computed from the values themselves so the tangent
// and the gather of a projected SH-rest group use the same number)
__device__ __forceinline__ float sh_rest_norm(const float B[16], int nc) {
  float acc = 0.f;
#pragma unroll
  for (int k = 1; k < 16; ++k)
    if (k < nc) acc += B[k] * B[k];
  return sqrtf(acc);
}

struct ChainOut {
  float dm2[2];
  float dmean[3];
  float dop;
  float dscale[3];
  float drot[4];
  float dcov[6];
  float dsh[16][3];
  float dcol[3];
  // the SH gradient in factored form, dsh[k][ch] = shB[k] * dres[ch] (k < active coefficients): the
  // per-Gaussian epilogues stage these 19 floats instead of the 3M products
  float shB[16];
  float dres[3];
  // DEFER_DIR: the view direction (unit) and its length, for the SH colour's view-direction term of dmean that the
  // caller adds itself (add_dir_term)
  float dir[3];
  float dirlen;
};

// Reverse mode: G2 = reduced screen-space gradient [x_pix, y_pix, conic a, b, c, opacity_eff, r, g, b, invdepth].
// DEFER_DIR: dmean leaves out the SH colour's view-direction term, sum_k dB_k/ddir <dres, sh_k> (the only use of the
// primal SH coefficients), and co.dir / co.dirlen are set for the caller's add_dir_term.
template <bool RAW, bool DEFER_DIR = false>
__device__ __forceinline__ void chain_vjp(const ViewK& v, const GaussK& g, int64_t i, bool visible,
                                          uint32_t clamped, const float G2[10], bool want_means, ChainOut& co) {
  co.dm2[0] = co.dm2[1] = 0.f;
  co.dop = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) { co.dmean[k] = 0.f; co.dscale[k] = 0.f; co.dcol[k] = 0.f; }
#pragma unroll
  for (int k = 0; k < 4; ++k) co.drot[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) co.dcov[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    co.dsh[k][0] = co.dsh[k][1] = co.dsh[k][2] = 0.f;
    co.shB[k] = 0.f;
  }
  // the factored SH epilogues stage shB x dres for every Gaussian, culled ones included (0 x garbage
  // would be NaN when the register happens to hold one)
  co.dres[0] = co.dres[1] = co.dres[2] = 0.f;
  if (!visible) return;
  Geo e;
  compute_geo<RAW>(v, g, i, clamped, e);

  // screen position (NDC means2D gradient, upstream ddelx_dx = 0.5 W)
  const float gpx = G2[0] * (0.5f * (float)v.W), gpy = G2[1] * (0.5f * (float)v.H);
  co.dm2[0] = gpx;
  co.dm2[1] = gpy;

  // opacity (with AA factor)
  const float dop_act = G2[5] * e.h;
  const float gh = G2[5] * e.op;

  // conic -> 2D covariance (a = c00 + 0.3, b = c01, c = c11 + 0.3)
  const float ga = G2[2], gb = G2[3], gc = G2[4];
  const float id2 = 1.f / (e.det * e.det);
  float dA = (-e.cc * e.cc * ga + e.b * e.cc * gb - e.b * e.b * gc) * id2;
  float dB = (2.f * e.b * e.cc * ga - (e.det + 2.f * e.b * e.b) * gb + 2.f * e.a * e.b * gc) * id2;
  float dC = (-e.b * e.b * ga + e.a * e.b * gb - e.a * e.a * gc) * id2;
  if (v.antialiasing) {
    float ha, hb, hc;
    aa_grad(e, ha, hb, hc);
    dA += gh * ha;
    dB += gh * hb;
    dC += gh * hc;
  }

  // 2D covariance -> 3D covariance (6-vector; off-diagonals appear twice in Sigma)
  const float* A0 = e.pj.A0;
  const float* A1 = e.pj.A1;
  co.dcov[0] = dA * A0[0] * A0[0] + dB * A0[0] * A1[0] + dC * A1[0] * A1[0];
  co.dcov[3] = dA * A0[1] * A0[1] + dB * A0[1] * A1[1] + dC * A1[1] * A1[1];
  co.dcov[5] = dA * A0[2] * A0[2] + dB * A0[2] * A1[2] + dC * A1[2] * A1[2];
  co.dcov[1] = 2.f * dA * A0[0] * A0[1] + dB * (A0[0] * A1[1] + A0[1] * A1[0]) + 2.f * dC * A1[0] * A1[1];
  co.dcov[2] = 2.f * dA * A0[0] * A0[2] + dB * (A0[0] * A1[2] + A0[2] * A1[0]) + 2.f * dC * A1[0] * A1[2];
  co.dcov[4] = 2.f * dA * A0[1] * A0[2] + dB * (A0[1] * A1[2] + A0[2] * A1[1]) + 2.f * dC * A1[1] * A1[2];

  if (!g.cov3D) {
    // Sigma = R diag(sp)^2 R^T ; Gs = symmetric dL/dSigma
    const float Gs[9] = {co.dcov[0], 0.5f * co.dcov[1], 0.5f * co.dcov[2],
                         0.5f * co.dcov[1], co.dcov[3], 0.5f * co.dcov[4],
                         0.5f * co.dcov[2], 0.5f * co.dcov[4], co.dcov[5]};
    const float* R = e.R;
    float GR[9];  // Gs * R
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) GR[r * 3 + k] = Gs[r * 3 + 0] * R[0 * 3 + k] + Gs[r * 3 + 1] * R[1 * 3 + k] + Gs[r * 3 + 2] * R[2 * 3 + k];
    float dR[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) dR[r * 3 + k] = 2.f * GR[r * 3 + k] * e.sp[k] * e.sp[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float rgr = R[0 * 3 + k] * GR[0 * 3 + k] + R[1 * 3 + k] * GR[1 * 3 + k] + R[2 * 3 + k] * GR[2 * 3 + k];
      const float dsp = 2.f * e.sp[k] * rgr;
      const float ds = v.scale_mod * dsp;
      co.dscale[k] = RAW ? ds * e.s[k] : ds;
    }
    const float qr = e.q[0], qx = e.q[1], qy = e.q[2], qz = e.q[3];
    float dq[4];
    dq[0] = 2.f * (-qz * dR[1] + qy * dR[2] + qz * dR[3] - qx * dR[5] - qy * dR[6] + qx * dR[7]);
    dq[1] = 2.f * (qy * dR[1] + qz * dR[2] + qy * dR[3] - 2.f * qx * dR[4] - qr * dR[5] + qz * dR[6] + qr * dR[7] -
                   2.f * qx * dR[8]);
    dq[2] = 2.f * (-2.f * qy * dR[0] + qx * dR[1] + qr * dR[2] + qx * dR[3] + qz * dR[5] - qr * dR[6] + qz * dR[7] -
                   2.f * qy * dR[8]);
    dq[3] = 2.f * (-2.f * qz * dR[0] - qr * dR[1] + qx * dR[2] + qr * dR[3] - 2.f * qz * dR[4] + qy * dR[5] +
                   qx * dR[6] + qy * dR[7]);
    if (RAW) {
      const float qd = ((e.q[0] * dq[0] + e.q[1] * dq[1]) + e.q[2] * dq[2]) + e.q[3] * dq[3];
#pragma unroll
      for (int k = 0; k < 4; ++k) co.drot[k] = (dq[k] - e.q[k] * qd) / e.qnorm;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) co.drot[k] = dq[k];
    }
  }

  // colour
  float dres[3] = {0.f, 0.f, 0.f};
  if (g.colors) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) co.dcol[ch] = G2[6 + ch];
  } else {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) dres[ch] = (e.clamped >> ch) & 1u ? 0.f : G2[6 + ch];
    float B[16];
    sh_basis(v.D, e.dir[0], e.dir[1], e.dir[2], B);
    const int nc = (v.D + 1) * (v.D + 1);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      co.shB[k] = k < nc ? B[k] : 0.f;
      if (k < nc) {
        co.dsh[k][0] = B[k] * dres[0];
        co.dsh[k][1] = B[k] * dres[1];
        co.dsh[k][2] = B[k] * dres[2];
      }
    }
  }
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) co.dres[ch] = dres[ch];

  if (want_means) {
    // J (EWA) dependence on the view-space mean
    float SA0[3], SA1[3];
    const float* c = e.c;
    SA0[0] = c[0] * A0[0] + c[1] * A0[1] + c[2] * A0[2];
    SA0[1] = c[1] * A0[0] + c[3] * A0[1] + c[4] * A0[2];
    SA0[2] = c[2] * A0[0] + c[4] * A0[1] + c[5] * A0[2];
    SA1[0] = c[0] * A1[0] + c[1] * A1[1] + c[2] * A1[2];
    SA1[1] = c[1] * A1[0] + c[3] * A1[1] + c[4] * A1[2];
    SA1[2] = c[2] * A1[0] + c[4] * A1[1] + c[5] * A1[2];
    float dJ00 = 0.f, dJ02 = 0.f, dJ11 = 0.f, dJ12 = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float dA0 = 2.f * dA * SA0[k] + dB * SA1[k];
      const float dA1 = dB * SA0[k] + 2.f * dC * SA1[k];
      dJ00 += dA0 * v.view[4 * k + 0];
      dJ02 += dA0 * v.view[4 * k + 2];
      dJ11 += dA1 * v.view[4 * k + 1];
      dJ12 += dA1 * v.view[4 * k + 2];
    }
    const float tz = e.tz, tz2 = 1.f / (tz * tz), tz3 = tz2 / tz;
    const float dtx = e.pj.inx ? -v.focal_x * tz2 * dJ02 : 0.f;
    const float dty = e.pj.iny ? -v.focal_y * tz2 * dJ12 : 0.f;
    float dtz = -v.focal_x * tz2 * dJ00 - v.focal_y * tz2 * dJ11 + 2.f * v.focal_x * e.pj.tcx * tz3 * dJ02 +
                2.f * v.focal_y * e.pj.tcy * tz3 * dJ12;
    dtz += -G2[9] * tz2;  // invdepth = 1 / t.z
    co.dmean[0] = v.view[0] * dtx + v.view[1] * dty + v.view[2] * dtz;
    co.dmean[1] = v.view[4] * dtx + v.view[5] * dty + v.view[6] * dtz;
    co.dmean[2] = v.view[8] * dtx + v.view[9] * dty + v.view[10] * dtz;
    // projection to NDC
    const float* pm = v.proj;
    const float mul1 = e.hx * e.p_w * e.p_w, mul2 = e.hy * e.p_w * e.p_w;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      co.dmean[j] += (pm[4 * j + 0] * e.p_w - pm[4 * j + 3] * mul1) * gpx + (pm[4 * j + 1] * e.p_w - pm[4 * j + 3] * mul2) * gpy;
    // view direction of the SH colour
    if (DEFER_DIR) {
#pragma unroll
      for (int j = 0; j < 3; ++j) co.dir[j] = e.dir[j];
      co.dirlen = e.dirlen;
    } else if (!g.colors && v.D > 0) {
      float dB[16][3];
      sh_basis_grad(v.D, e.dir[0], e.dir[1], e.dir[2], dB);
      float ddir[3] = {0.f, 0.f, 0.f};
      const int nc = (v.D + 1) * (v.D + 1);
      // compile-time k (unrolled, guarded): dB stays in registers instead of a scratch array indexed at run time
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < nc) {
          const float s0 = g.sh(i, k, 0), s1 = g.sh(i, k, 1), s2 = g.sh(i, k, 2);
          const float w = dres[0] * s0 + dres[1] * s1 + dres[2] * s2;
#pragma unroll
          for (int j = 0; j < 3; ++j) ddir[j] += dB[k][j] * w;
        }
      const float dd = e.dir[0] * ddir[0] + e.dir[1] * ddir[1] + e.dir[2] * ddir[2];
#pragma unroll
      for (int j = 0; j < 3; ++j) co.dmean[j] += (ddir[j] - e.dir[j] * dd) / e.dirlen;
    }
  }
  co.dop = RAW ? dop_act * e.op * (1.f - e.op) : dop_act;
}

// chain_vjp's view-direction term of dmean from w[k] = <dres, sh_k> (k = 1 .. nc - 1): the same operations in the
// same order, so the same dmean bitwise.
__device__ __forceinline__ void add_dir_term(int D, const float dir[3], float dirlen, const float* w, float dmean[3]) {
  float dB[16][3];
  sh_basis_grad(D, dir[0], dir[1], dir[2], dB);
  float ddir[3] = {0.f, 0.f, 0.f};
  const int nc = (D + 1) * (D + 1);
#pragma unroll
  for (int k = 1; k < 16; ++k)
    if (k < nc) {
      const float wk = w[k];
#pragma unroll
      for (int j = 0; j < 3; ++j) ddir[j] += dB[k][j] * wk;
    }
  const float dd = dir[0] * ddir[0] + dir[1] * ddir[1] + dir[2] * ddir[2];
#pragma unroll
  for (int j = 0; j < 3; ++j) dmean[j] += (ddir[j] - dir[j] * dd) / dirlen;
}

__device__ __forceinline__ void put(float* p, float v, int acc) {
  if (acc) *p += v;
  else *p = v;
}

// Store a ChainOut into the requested outputs (NULL pointers skipped).
__device__ __forceinline__ void write_grads(const GaussK& g, const GradK& o, int64_t i, const ChainOut& co, int M,
                                            int nc, bool want_means, bool skip_sh = false) {
  const int acc = o.accumulate;
  if (o.means2D) {
    put(&o.means2D[3 * i + 0], co.dm2[0], acc);
    put(&o.means2D[3 * i + 1], co.dm2[1], acc);
    if (!acc) o.means2D[3 * i + 2] = 0.f;
  }
  if (o.means3D && want_means)
#pragma unroll
    for (int k = 0; k < 3; ++k) put(&o.means3D[3 * i + k], co.dmean[k], acc);
  if (o.opac) put(&o.opac[i], co.dop, acc);
  if (g.cov3D) {
    if (o.cov3D)
#pragma unroll
      for (int k = 0; k < 6; ++k) put(&o.cov3D[6 * i + k], co.dcov[k], acc);
  } else {
    if (o.scales)
#pragma unroll
      for (int k = 0; k < 3; ++k) put(&o.scales[3 * i + k], co.dscale[k], acc);
    if (o.rot)
#pragma unroll
      for (int k = 0; k < 4; ++k) put(&o.rot[4 * i + k], co.drot[k], acc);
  }
  if (g.colors) {
    if (o.colors)
#pragma unroll
      for (int k = 0; k < 3; ++k) put(&o.colors[3 * i + k], co.dcol[k], acc);
  } else if (!skip_sh) {
    if (o.dc)
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) put(&o.dc[i * o.dc_stride + ch], co.dsh[0][ch], acc);
    if (o.rest) {
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < M) {
          const float* d = co.dsh[k];
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) put(&o.rest[i * o.rest_stride + 3 * (k - 1) + ch], k < nc ? d[ch] : 0.f, acc);
        }
    }
  }
}

// Forward mode: tangent of the render record from input tangents t (NULL = 0).
// out: [dx_pix, dy_pix, dconic a, b, c, dopacity_eff, dr, dg, db, dinvdepth]
template <bool RAW>
__device__ __forceinline__ void chain_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t,
                                          int64_t i, uint32_t clamped, float T2[10]) {
  Geo e;
  compute_geo<RAW>(v, g, i, clamped, e);
  float dm[3] = {0.f, 0.f, 0.f};
  if (t.means3D)
#pragma unroll
    for (int k = 0; k < 3; ++k) dm[k] = t.means3D[3 * i + k];
  const float dtx = (v.view[0] * dm[0] + v.view[4] * dm[1]) + v.view[8] * dm[2];
  const float dty = (v.view[1] * dm[0] + v.view[5] * dm[1]) + v.view[9] * dm[2];
  const float dtz = (v.view[2] * dm[0] + v.view[6] * dm[1]) + v.view[10] * dm[2];

  // screen position
  const float* pm = v.proj;
  const float mul1 = e.hx * e.p_w * e.p_w, mul2 = e.hy * e.p_w * e.p_w;
  float dpx = 0.f, dpy = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    dpx += (pm[4 * j + 0] * e.p_w - pm[4 * j + 3] * mul1) * dm[j];
    dpy += (pm[4 * j + 1] * e.p_w - pm[4 * j + 3] * mul2) * dm[j];
  }
  if (m2t) {
    dpx += m2t[3 * i + 0];
    dpy += m2t[3 * i + 1];
  }
  T2[0] = dpx * (0.5f * (float)v.W);
  T2[1] = dpy * (0.5f * (float)v.H);

  // d Sigma
  float dS[6];
  if (g.cov3D) {
#pragma unroll
    for (int k = 0; k < 6; ++k) dS[k] = t.cov3D ? t.cov3D[6 * i + k] : 0.f;
  } else {
    float ds[3] = {0.f, 0.f, 0.f}, dq[4] = {0.f, 0.f, 0.f, 0.f};
    if (t.scales)
#pragma unroll
      for (int k = 0; k < 3; ++k) ds[k] = RAW ? e.s[k] * t.scales[3 * i + k] : t.scales[3 * i + k];
    if (t.rot) {
#pragma unroll
      for (int k = 0; k < 4; ++k) dq[k] = t.rot[4 * i + k];
      if (RAW) {
        const float qd = ((e.q[0] * dq[0] + e.q[1] * dq[1]) + e.q[2] * dq[2]) + e.q[3] * dq[3];
#pragma unroll
        for (int k = 0; k < 4; ++k) dq[k] = (dq[k] - e.q[k] * qd) / e.qnorm;
      }
    }
    const float r = e.q[0], x = e.q[1], y = e.q[2], z = e.q[3];
    const float dr_ = dq[0], dx_ = dq[1], dy_ = dq[2], dz_ = dq[3];
    float dR[9];
    dR[0] = -4.f * (y * dy_ + z * dz_);
    dR[1] = 2.f * (dx_ * y + x * dy_ - dr_ * z - r * dz_);
    dR[2] = 2.f * (dx_ * z + x * dz_ + dr_ * y + r * dy_);
    dR[3] = 2.f * (dx_ * y + x * dy_ + dr_ * z + r * dz_);
    dR[4] = -4.f * (x * dx_ + z * dz_);
    dR[5] = 2.f * (dy_ * z + y * dz_ - dr_ * x - r * dx_);
    dR[6] = 2.f * (dx_ * z + x * dz_ - dr_ * y - r * dy_);
    dR[7] = 2.f * (dy_ * z + y * dz_ + dr_ * x + r * dx_);
    dR[8] = -4.f * (x * dx_ + y * dy_);
    float dsp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) dsp[k] = v.scale_mod * ds[k];
    const float* R = e.R;
    auto dsig = [&](int i0, int j0) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float s2 = e.sp[k] * e.sp[k];
        acc += dR[i0 * 3 + k] * s2 * R[j0 * 3 + k] + R[i0 * 3 + k] * s2 * dR[j0 * 3 + k] +
               2.f * R[i0 * 3 + k] * e.sp[k] * dsp[k] * R[j0 * 3 + k];
      }
      return acc;
    };
    dS[0] = dsig(0, 0); dS[1] = dsig(0, 1); dS[2] = dsig(0, 2);
    dS[3] = dsig(1, 1); dS[4] = dsig(1, 2); dS[5] = dsig(2, 2);
  }

  // d J (quirk: t.x, t.y independent of t.z; masked outside the clamp)
  const float tz = e.tz, tz2 = 1.f / (tz * tz), tz3 = tz2 / tz;
  const float dtxq = e.pj.inx ? dtx : 0.f, dtyq = e.pj.iny ? dty : 0.f;
  const float dJ00 = -v.focal_x * tz2 * dtz;
  const float dJ02 = -v.focal_x * tz2 * dtxq + 2.f * v.focal_x * e.pj.tcx * tz3 * dtz;
  const float dJ11 = -v.focal_y * tz2 * dtz;
  const float dJ12 = -v.focal_y * tz2 * dtyq + 2.f * v.focal_y * e.pj.tcy * tz3 * dtz;
  float dA0[3], dA1[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    dA0[k] = dJ00 * v.view[4 * k + 0] + dJ02 * v.view[4 * k + 2];
    dA1[k] = dJ11 * v.view[4 * k + 1] + dJ12 * v.view[4 * k + 2];
  }
  const float* A0 = e.pj.A0;
  const float* A1 = e.pj.A1;
  const float dc00 = 2.f * quad_form(dA0, e.c, A0) + quad_form(A0, dS, A0);
  const float dc01 = quad_form(dA0, e.c, A1) + quad_form(A0, e.c, dA1) + quad_form(A0, dS, A1);
  const float dc11 = 2.f * quad_form(dA1, e.c, A1) + quad_form(A1, dS, A1);

  const float id2 = 1.f / (e.det * e.det);
  T2[2] = (-e.cc * e.cc * dc00 + 2.f * e.b * e.cc * dc01 - e.b * e.b * dc11) * id2;
  T2[3] = (e.b * e.cc * dc00 - (e.det + 2.f * e.b * e.b) * dc01 + e.a * e.b * dc11) * id2;
  T2[4] = (-e.b * e.b * dc00 + 2.f * e.a * e.b * dc01 - e.a * e.a * dc11) * id2;

  float dh = 0.f;
  if (v.antialiasing) {
    float ha, hb, hc;
    aa_grad(e, ha, hb, hc);
    dh = ha * dc00 + hb * dc01 + hc * dc11;
  }
  float dop = t.opac ? t.opac[i] : 0.f;
  if (RAW) dop = e.op * (1.f - e.op) * dop;
  T2[5] = dop * e.h + e.op * dh;

  // colour
  if (g.colors) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) T2[6 + ch] = t.colors ? t.colors[3 * i + ch] : 0.f;
  } else {
    float dres[3] = {0.f, 0.f, 0.f};
    const int nc = (v.D + 1) * (v.D + 1);
    if (t.dc) {
      float B[16];
      sh_basis(v.D, e.dir[0], e.dir[1], e.dir[2], B);
      if (t.rest_R) {
        // SH-rest coordinates c_j in the orthonormal basis Q of span{B_rest(dir_b)}: B_rest(dir)^T Q c = sum_j R[j][col] c_j
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) dres[ch] += B[0] * t.sh(i, 0, ch);
        if (t.rest && nc > 1) {
          const float* Rc = t.rest_R + i * rest_basis_floats(t.rest_V) + rest_basis_floats(t.rest_col);
          const float* c = t.rest + (i - t.rest_base) * t.rest_stride;
#pragma unroll
          for (int j = 0; j < MAX_REST_VIEWS; ++j)
            if (j <= t.rest_col) {
              const float r = Rc[j];
#pragma unroll
              for (int ch = 0; ch < 3; ++ch) dres[ch] += r * c[3 * j + ch];
            }
        }
      } else if (t.rest_proj) {
        // projected SH-rest tangent: sum_k B_k v_k = |B_rest| c for v = (B_rest / |B_rest|) (x) c
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) dres[ch] += B[0] * t.sh(i, 0, ch);
        if (t.rest && nc > 1) {
          const float nb = sh_rest_norm(B, nc);
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) dres[ch] += nb * t.rest[(i - t.rest_base) * t.rest_stride + ch];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < nc && (k == 0 || t.rest)) {
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) dres[ch] += B[k] * t.sh(i, k, ch);
          }
      }
    }
    if (t.means3D && v.D > 0) {
      const float dd = e.dir[0] * dm[0] + e.dir[1] * dm[1] + e.dir[2] * dm[2];
      float ddir[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) ddir[j] = (dm[j] - e.dir[j] * dd) / e.dirlen;
      float dB[16][3];
      sh_basis_grad(v.D, e.dir[0], e.dir[1], e.dir[2], dB);
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < nc) {
          const float w = dB[k][0] * ddir[0] + dB[k][1] * ddir[1] + dB[k][2] * ddir[2];
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) dres[ch] += w * g.sh(i, k, ch);
        }
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) T2[6 + ch] = (e.clamped >> ch) & 1u ? 0.f : dres[ch];
  }
  T2[9] = -dtz * tz2;
}

}  // namespace gslm
