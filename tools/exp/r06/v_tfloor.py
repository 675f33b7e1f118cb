# timing-only variant (round 6): the LM tangent kernel's per-Gaussian chain replaced by a 24-float linear map read
# coalesced from a [24][P] array (emulated with the primal SH rest, 45 P floats) -- the floor of a precomputed
# frozen-geometry linearisation.  Wrong records.
s = open("tangent.hip").read()
a = "  chain_jvp<RAW>(v, g, t, m2t, i, clampw[i], T2);\n"
assert a in s
s = s.replace(a, """  if (XPBY) {
    float m[24];
#pragma unroll
    for (int k = 0; k < 24; ++k) m[k] = g.rest[(int64_t)k * g.P + i];
    float u[14];
#pragma unroll
    for (int k = 0; k < 3; ++k) u[k] = t.dc[i * t.dc_stride + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) u[3 + k] = t.rest[(i - t.rest_base) * t.rest_stride + k];
#pragma unroll
    for (int k = 0; k < 3; ++k) u[6 + k] = t.scales[3 * i + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[9 + k] = t.rot[4 * i + k];
    u[13] = t.opac[i];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 7; ++k) acc += m[7 * r + k] * u[6 + k];
      T2[2 + r] = acc;
    }
    T2[5] = m[21] * u[13];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) T2[6 + ch] = ((clampw[i] >> ch) & 1u) ? 0.f : m[22] * u[ch] + m[23] * u[3 + ch];
    T2[0] = T2[1] = T2[9] = 0.f;
  } else {
    chain_jvp<RAW>(v, g, t, m2t, i, clampw[i], T2);
  }
""")
open("tangent.hip", "w").write(s)
