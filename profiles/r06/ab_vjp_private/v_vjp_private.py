# variant (round 6, VERDICT r05 item 1's exact suggestion): the LM VJP pass without block barriers, each wave staging
# the records of ITS OWN hits (wave-private, as the J v pass does), the four waves' partials combined per entry by the
# last of the four to arrive at a window (LDS ticket), in fixed quadrant order -- the same rows bitwise.  AW entries per
# window (GSLM_VJP_AW, default 64), a two-slot ring for the partials.  Every wait bounded.
import os
AW = int(os.environ.get("GSLM_VJP_AW", "64"))
s = open("gslm_tile.hpp").read()
fn = r'''
// ---- vjp_tile_lm_private (round-6 experiment) ----
template <int AW>
struct VPriv {
  static constexpr int NU = 7;
  static constexpr int PRIV_F = 5 * AW * 2;    // per wave: five float2 record planes
  static constexpr int PART_F = 4 * NU * AW;   // per slot: [wave][value][entry] partials
  static constexpr int SLOT_F = PART_F + AW;   // + the entries' opacities
  static constexpr int NSLOT = 2;
  static constexpr int CTL = 16;               // win[2], arrive[2] (at 6, 7), wm[4] (at 8)
  __host__ __device__ static constexpr int floats() { return 4 * PRIV_F + NSLOT * SLOT_F + CTL; }
};
#ifndef GSLM_PRIV_SPIN_MAX
#define GSLM_PRIV_SPIN_MAX (1 << 22)
#endif
__device__ __forceinline__ uint32_t vp_load_acq(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void vp_store_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool vp_wait_eq(uint32_t* p, uint32_t v) {
  for (int it = 0; it < GSLM_PRIV_SPIN_MAX; ++it) {
    const uint32_t x = __builtin_amdgcn_readfirstlane(vp_load_acq(p));
    if (x == v) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
__device__ __forceinline__ uint32_t vp_ticket(uint32_t* p) {
  uint32_t t = 0;
  if ((threadIdx.x & 63) == 0) t = __hip_atomic_fetch_add(p, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(t);
}

template <int AW>
__device__ __forceinline__ void vjp_tile_lm_private(VjpPix& st, float pxf, float pyf, uint2 range,
                                                    const uint32_t* __restrict__ point_list,
                                                    const float4* __restrict__ rec, const uint32_t* __restrict__ slots,
                                                    float* lds, float4* __restrict__ rows) {
  using C = VPriv<AW>;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
  float2* priv = reinterpret_cast<float2*>(lds + q * C::PRIV_F);
  float* ring = lds + 4 * C::PRIV_F;
  uint32_t* ctl = reinterpret_cast<uint32_t*>(ring + C::NSLOT * C::SLOT_F);
  __syncthreads();  // the J v pass's LDS is aliased
  const int wmax = wave_max_u((int)st.last);
  if (lane == 0) ctl[8 + q] = (uint32_t)wmax;
  if (tid == 0) {
    ctl[0] = 0u;
    ctl[1] = 1u;
    ctl[6] = ctl[7] = 0u;
  }
  __syncthreads();
  const int wm0 = (int)ctl[8], wm1 = (int)ctl[9], wm2 = (int)ctl[10], wm3 = (int)ctl[11];
  const int n_eff = max(max(wm0, wm1), max(wm2, wm3));
  const int nwin = (n_eff + AW - 1) / AW;
  for (int r = 0; r < nwin; ++r) {
    const int sl = r & 1;
    float* part = ring + sl * C::SLOT_F;
    float* s_op = part + C::PART_F;
    const int top = n_eff - 1 - AW * r;
    const int pos = top - lane;
    uint32_t m = 0u;
    float op = 0.f;
    bool mine = false;
    if (lane < AW && pos >= 0) {
      const uint32_t e = point_list[range.x + pos];
      m = pl_mask(e) & ((pos < wm0 ? 1u : 0u) | (pos < wm1 ? 2u : 0u) | (pos < wm2 ? 4u : 0u) | (pos < wm3 ? 8u : 0u));
      mine = ((m >> q) & 1u) != 0u;
      if (mine) {
        const uint32_t g = pl_id(e);
        const float4 r0 = rec[RECS * (int64_t)g + 0], r1 = rec[RECS * (int64_t)g + 1], r2 = rec[RECS * (int64_t)g + 2];
        priv[lane] = make_float2(r0.x, r0.y);
        priv[AW + lane] = make_float2(r0.z, r0.w);
        priv[2 * AW + lane] = make_float2(r1.x, r1.y);
        priv[3 * AW + lane] = make_float2(r1.z, r1.w);
        priv[4 * AW + lane] = make_float2(r2.x, r2.y);
        op = r1.y;
      }
    }
    // the slot is free once window r - 2 is combined; every wave waits (its arrival counts on the slot's counter)
    if (!vp_wait_eq(ctl + sl, (uint32_t)r)) return;
    if (mine) s_op[lane] = op;
    wave_lds_sync();
    uint64_t hits = __ballot(mine);
    while (hits) {
      const int j = (int)__builtin_ctzll(hits);
      hits = clear_bit(hits, j);
      const float2 p0 = priv[j], p1 = priv[AW + j], p2 = priv[2 * AW + j], p3 = priv[3 * AW + j];
      const float2 c = priv[4 * AW + j];
      const float4 a = make_float4(p0.x, p0.y, p1.x, p1.y), b = make_float4(p2.x, p2.y, p3.x, p3.y);
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(c.x));
      const uint32_t contributor = (uint32_t)(top - j);
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      const bool c_last = contributor < st.last, c_pow = !(power > 0.0f), c_alpha = alpha >= 1.0f / 255.0f;
      const bool valid = c_last && c_pow && c_alpha;
      float cd;
      {
#pragma clang fp contract(fast)
        cd = (b.z * st.dpix[0] + b.w * st.dpix[1]) + c.x * st.dpix[2];
      }
      const bool any = (__builtin_amdgcn_ballot_w64(c_last) & __builtin_amdgcn_ballot_w64(c_pow) &
                        __builtin_amdgcn_ballot_w64(c_alpha)) != 0ull;
      float rr = 0.f;
      if (any) {
        float gv[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) gv[k] = 0.f;
        const float a_e = valid ? alpha : 0.f;
        const float G_e = valid ? G : 0.f;
        {
#pragma clang fp contract(fast)
          const float inv1ma = rcp_f(1.f - a_e);
          st.T = st.T * inv1ma;
          const float dchannel = a_e * st.T;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) gv[6 + ch] = dchannel * st.dpix[ch];
          const float cd_acc = cd - st.accd;
          const float dL_dalpha = cd_acc * st.T + st.tb * inv1ma;
          st.accd = st.accd + a_e * cd_acc;
          gv[5] = G_e * dL_dalpha;
          const float hdx = gv[5] * dx, hdy = gv[5] * dy;
          gv[2] = hdx * dx;
          gv[3] = hdx * dy;
          gv[4] = hdy * dy;
        }
        float pv[8];
#pragma unroll
        for (int k = 0; k < C::NU; ++k) pv[k] = gv[2 + k];
        pv[7] = dy;
        rr = wave_reduce8_t(pv, lane);
      }
      const int k = lane >> 3;
      if ((lane & 7) == 0 && k < C::NU) part[(q * C::NU + k) * AW + (j ^ ((k << 3) & (AW - 1)))] = rr;
    }
    if (vp_ticket(ctl + 6 + sl) == 3u) {
      // the fourth arrival combines window r (lane j = entry j), in fixed quadrant order
      uint32_t slot = 0;
      if (m) slot = slots[range.x + pos];
      float t[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) t[k] = 0.f;
      if (lane < AW) {
#pragma unroll
        for (int k = 0; k < C::NU; ++k) {
          const int sw = lane ^ ((k << 3) & (AW - 1));
          const float a0 = part[(0 * C::NU + k) * AW + sw], a1 = part[(1 * C::NU + k) * AW + sw];
          const float a2 = part[(2 * C::NU + k) * AW + sw], a3 = part[(3 * C::NU + k) * AW + sw];
          const float q0 = (m & 1u) ? a0 : 0.f;
          const float q1 = (m & 2u) ? a1 : 0.f;
          const float q2 = (m & 4u) ? a2 : 0.f;
          const float q3 = (m & 8u) ? a3 : 0.f;
          t[2 + k] = ((q0 + q1) + q2) + q3;
        }
      }
      const float opj = (lane < AW && m) ? s_op[lane] : 0.f;
      if (lane == 0) ctl[6 + sl] = 0u;
      wave_lds_sync();
      if (lane == 0) vp_store_rel(ctl + sl, (uint32_t)(r + 2));
      if (m) {
        t[2] *= -0.5f * opj;
        t[3] *= -opj;
        t[4] *= -0.5f * opj;
        store_row<2>(rows, slot, t);
      }
    }
  }
}
'''
marker = "}  // namespace gslm"
idx = s.rfind(marker)
assert idx > 0
s = s[:idx] + fn + "\n" + s[idx:]
open("gslm_tile.hpp", "w").write(s)

j = open("jvp.hip").read()
a = "  constexpr int kVjp = kAcc + B + B + B / 2;  // + s_r0, s_r1, s_r2 (vjp_tile: 5 float2 planes)\n"
assert a in j
j = j.replace(a, "  constexpr int kVjpBatch = kAcc + B + B + B / 2;\n"
                 "  constexpr int kVjpPriv = (VPriv<%d>::floats() + 3) / 4;\n"
                 "  constexpr int kVjp = WITH_XY ? kVjpBatch : kVjpPriv;\n" % AW)
a = """  vjp_tile<WITH_XY, false, WITH_XY ? 3 : 2, B>(st, inside, (float)px, (float)py, tile_x, tile_y, range, point_list, rec,
                                            slots, rect, goff, reinterpret_cast<float2*>(s_r0), s_bits, s_acc, s_misc, contrib,
                                            write_tail != 0);
}"""
assert a in j
j = j.replace(a, """  if constexpr (!WITH_XY) {
    (void)write_tail;
    vjp_tile_lm_private<%d>(st, (float)px, (float)py, range, point_list, rec, slots, reinterpret_cast<float*>(s_lds),
                            contrib);
  } else {
    vjp_tile<WITH_XY, false, WITH_XY ? 3 : 2, B>(st, inside, (float)px, (float)py, tile_x, tile_y, range, point_list,
                                              rec, slots, rect, goff, reinterpret_cast<float2*>(s_r0), s_bits, s_acc,
                                              s_misc, contrib, write_tail != 0);
  }
}""" % AW)
open("jvp.hip", "w").write(j)
