# timing-only variant (round 6): the LM gather's per-Gaussian chain (chain_vjp) replaced by the transpose of a
# 24-float linear map read coalesced from a [24][P] array (emulated with the primal SH rest) -- the floor of a
# precomputed frozen-geometry linearisation on the gather side.  Wrong products.
s = open("gather.hip").read()
a = "  if (i < g.P) chain_vjp<true>(v, g, i, n != 0, n ? clampw[i] : 0u, G2, WANT_MEANS, co);\n"
assert a in s
s = s.replace(a, """  if (WANT_MEANS) {
    if (i < g.P) chain_vjp<true>(v, g, i, n != 0, n ? clampw[i] : 0u, G2, WANT_MEANS, co);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) { co.shB[k] = 0.f; co.dsh[k][0] = co.dsh[k][1] = co.dsh[k][2] = 0.f; }
#pragma unroll
    for (int k = 0; k < 3; ++k) { co.dres[k] = 0.f; co.dscale[k] = 0.f; co.dmean[k] = 0.f; }
#pragma unroll
    for (int k = 0; k < 4; ++k) co.drot[k] = 0.f;
    co.dop = 0.f;
    if (i < g.P && n) {
      float m[24];
#pragma unroll
      for (int k = 0; k < 24; ++k) m[k] = g.rest[(int64_t)k * g.P + i];
      float d[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) d[k] = (m[k] * G2[2] + m[7 + k] * G2[3]) + m[14 + k] * G2[4];
#pragma unroll
      for (int k = 0; k < 3; ++k) co.dscale[k] = d[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) co.drot[k] = d[3 + k];
      co.dop = m[21] * G2[5];
      const uint32_t cw = clampw[i];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        co.dres[ch] = ((cw >> ch) & 1u) ? 0.f : G2[6 + ch];
        co.dsh[0][ch] = m[22] * co.dres[ch];
      }
      co.shB[0] = m[22];
      co.shB[1] = m[23];
    }
  }
""")
open("gather.hip", "w").write(s)
