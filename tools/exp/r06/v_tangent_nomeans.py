# variant (round 6): the LM tangent kernel's chain (the fused-update instantiation, XPBY: xyz frozen, no means2D
# tangent -- api.hip builds the LM tangent with means3D = NULL under mask_xyz) specialised at compile time, so the
# view-space / screen-position / EWA-Jacobian tangent terms fold away instead of running on zeros
s = open("gslm_chain.hpp").read()
a = """template <bool RAW>
__device__ __forceinline__ void chain_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t,
                                          int64_t i, uint32_t clamped, float T2[10]) {
  Geo e;
  compute_geo<RAW>(v, g, i, clamped, e);
  float dm[3] = {0.f, 0.f, 0.f};
  if (t.means3D)"""
assert a in s
s = s.replace(a, """template <bool RAW, bool TMEANS = true>
__device__ __forceinline__ void chain_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t,
                                          int64_t i, uint32_t clamped, float T2[10]) {
  Geo e;
  compute_geo<RAW>(v, g, i, clamped, e);
  float dm[3] = {0.f, 0.f, 0.f};
  if (!TMEANS) m2t = nullptr;
  if (TMEANS && t.means3D)""")
a = "    if (t.means3D && v.D > 0) {"
assert a in s
s = s.replace(a, "    if (TMEANS && t.means3D && v.D > 0) {")
open("gslm_chain.hpp", "w").write(s)
s = open("tangent.hip").read()
a = "  chain_jvp<RAW>(v, g, t, m2t, i, clampw[i], T2);\n"
assert a in s
s = s.replace(a, "  if constexpr (XPBY) chain_jvp<RAW, false>(v, g, t, m2t, i, clampw[i], T2);\n"
                 "  else chain_jvp<RAW>(v, g, t, m2t, i, clampw[i], T2);\n")  # timing: assumes the fused update is the LM (mask_xyz) path
open("tangent.hip", "w").write(s)
