# variant: k_preprocess_jvp<.., XPBY> loads the Gaussian's primal parameters (xyz, scale, rotation, opacity, clamp bits)
# into registers before the fused direction update, and forms the geometry from them after it (the loads' latency under
# the update's; the full geometry before the update took 159 VGPRs)
p = "gslm_chain.hpp"
s = open(p).read()
old = """template <bool RAW>
__device__ __forceinline__ void compute_geo(const ViewK& v, const GaussK& g, int64_t i, uint32_t clamped, Geo& e) {
  e.x = g.means3D[3 * i + 0];
  e.y = g.means3D[3 * i + 1];
  e.z = g.means3D[3 * i + 2];"""
new = """struct GeoIn {
  float x, y, z, s[3], q[4], op;
};
template <bool RAW>
__device__ __forceinline__ void load_geo_in(const GaussK& g, int64_t i, GeoIn& in) {
  in.x = g.means3D[3 * i + 0];
  in.y = g.means3D[3 * i + 1];
  in.z = g.means3D[3 * i + 2];
#pragma unroll
  for (int k = 0; k < 3; ++k) in.s[k] = g.scales[3 * i + k];
#pragma unroll
  for (int k = 0; k < 4; ++k) in.q[k] = g.rot[4 * i + k];
  in.op = g.opac[i];
}
// compute_geo from preloaded inputs (no cov3D_precomp: the LM path's raw leaves)
template <bool RAW>
__device__ __forceinline__ void compute_geo_in(const ViewK& v, const GeoIn& in, uint32_t clamped, Geo& e) {
  e.x = in.x;
  e.y = in.y;
  e.z = in.z;
  e.tx = tp_row(v.view, e.x, e.y, e.z, 0);
  e.ty = tp_row(v.view, e.x, e.y, e.z, 1);
  e.tz = tp_row(v.view, e.x, e.y, e.z, 2);
  e.hx = tp_row(v.proj, e.x, e.y, e.z, 0);
  e.hy = tp_row(v.proj, e.x, e.y, e.z, 1);
  const float hw = tp_row(v.proj, e.x, e.y, e.z, 3);
  e.p_w = 1.0f / (hw + 0.0000001f);
#pragma unroll
  for (int k = 0; k < 3; ++k) e.s[k] = RAW ? expf(in.s[k]) : in.s[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) e.q[k] = in.q[k];
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
  e.op = RAW ? sigmoidf_(in.op) : in.op;
  float dx = e.x - v.campos[0], dy = e.y - v.campos[1], dz = e.z - v.campos[2];
  e.dirlen = sqrtf((dx * dx + dy * dy) + dz * dz);
  e.dir[0] = dx / e.dirlen;
  e.dir[1] = dy / e.dirlen;
  e.dir[2] = dz / e.dirlen;
  e.clamped = clamped;
}

template <bool RAW>
__device__ __forceinline__ void compute_geo(const ViewK& v, const GaussK& g, int64_t i, uint32_t clamped, Geo& e) {
  e.x = g.means3D[3 * i + 0];
  e.y = g.means3D[3 * i + 1];
  e.z = g.means3D[3 * i + 2];"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
p = "tangent.hip"
s = open(p).read()
old = """    if (act) compute_geo<RAW>(v, g, i, clampw[i], e);"""
new = """    GeoIn gin;
    uint32_t cw = 0;
    if (act) {
      load_geo_in<RAW>(g, i, gin);
      cw = clampw[i];
    }"""
assert old in s
s = s.replace(old, new)
old = """    __syncthreads();
    if (t.rest) {
      t.rest = s_rest;
      t.rest_base = (int64_t)blockIdx.x * blockDim.x;
    }
  }
  if (!act) return;"""
new = """    __syncthreads();
    if (t.rest) {
      t.rest = s_rest;
      t.rest_base = (int64_t)blockIdx.x * blockDim.x;
    }
    if (act && !g.cov3D) compute_geo_in<RAW>(v, gin, cw, e);
    else if (act) compute_geo<RAW>(v, g, i, cw, e);
  }
  if (!act) return;"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
