// tangent.hip -- per-Gaussian side of the forward-mode tangent.
//
//   k_preprocess_jvp   one thread per visible Gaussian: tangent render record (48 B) from the
//                      input tangents (chain_jvp, exact transpose of chain_vjp); optionally first
//                      the deferred CG direction update p = s + beta p of its block (block_xpby).
// Compiled apart from the tile passes: these per-Gaussian kernels keep clang's SLP vectoriser,
// which the tile passes turn off (Makefile).
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

// p = s + beta p over this block's 256 Gaussians' slices of every group, and the flat tail by block 0.
// Same arithmetic as k_xpby_dev (bitwise).  The narrow groups (xyz, dc, scaling, rotation, opacity, and the
// SH rest when projected: <= 4 floats per Gaussian, so <= 4 elements per thread each) are loaded in one pass --
// every s / p / x load of the block in flight before the first store -- instead of one latency per group; a
// full-layout SH rest (3(M-1) floats per Gaussian) streams in its own loop.
__device__ __forceinline__ void block_xpby(const XpbyK& xp, int64_t P, float* s_rest) {
  const float b = (float)((*xp.num) / (*xp.den));
  const bool with_x = xp.anum != nullptr;
  const float a = with_x ? (float)((*xp.anum) / (*xp.aden)) : 0.f;  // gslm_cg_update's alpha, bitwise
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t nv = min((int64_t)blockDim.x, P - i0);
  const int tid = threadIdx.x;
  constexpr int MAXW[6] = {3, 3, 3, 3, 4, 1};  // per-Gaussian widths the one-pass path covers
  const bool rest_narrow = xp.w[2] <= 3;
  float sv[17], pv[17], xv[17];
  int n = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
#pragma unroll
    for (int j = 0; j < MAXW[k]; ++j, ++n) {
      const int64_t e = (int64_t)j * blockDim.x + tid;
      const bool on = xp.p[k] && (k != 2 || rest_narrow) && e < nv * xp.w[k];
      const int64_t gi = i0 * xp.w[k] + e;
      sv[n] = on ? xp.s[k][gi] : 0.f;
      pv[n] = on ? xp.p[k][gi] : 0.f;
      xv[n] = (on && with_x) ? xp.p[k][xp.xoff + gi] : 0.f;
    }
  }
  n = 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
#pragma unroll
    for (int j = 0; j < MAXW[k]; ++j, ++n) {
      const int64_t e = (int64_t)j * blockDim.x + tid;
      const bool on = xp.p[k] && (k != 2 || rest_narrow) && e < nv * xp.w[k];
      if (on) {
        const int64_t gi = i0 * xp.w[k] + e;
        if (with_x) xp.p[k][xp.xoff + gi] = xv[n] + a * pv[n];
        const float r = sv[n] + b * pv[n];
        xp.p[k][gi] = r;
        if (k == 2) s_rest[e] = r;  // the SH-rest slice stays in LDS for the tangent below
      }
    }
  }
  if (xp.p[2] && !rest_narrow) {
    float* p = xp.p[2] + i0 * xp.w[2];
    const float* s = xp.s[2] + i0 * xp.w[2];
    const int64_t len = nv * xp.w[2];
    constexpr int U = 8;
    for (int64_t e0 = 0; e0 < len; e0 += (int64_t)U * blockDim.x) {
      float su[U], pu[U], xu[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + (int64_t)u * blockDim.x + tid;
        su[u] = e < len ? s[e] : 0.f;
        pu[u] = e < len ? p[e] : 0.f;
        xu[u] = (e < len && with_x) ? p[xp.xoff + e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + (int64_t)u * blockDim.x + tid;
        if (e < len) {
          if (with_x) p[xp.xoff + e] = xu[u] + a * pu[u];
          const float r = su[u] + b * pu[u];
          p[e] = r;
          s_rest[e] = r;
        }
      }
    }
  }
  if (blockIdx.x == 0 && xp.tail_p)
    for (int64_t e = threadIdx.x; e < xp.tail_n; e += blockDim.x) {
      const float pvt = xp.tail_p[e];
      if (with_x) xp.tail_p[xp.xoff + e] = xp.tail_p[xp.xoff + e] + a * pvt;
      xp.tail_p[e] = xp.tail_s[e] + b * pvt;
    }
}

// Tangent render record of Gaussian i: 12 floats [dx dy da db | dc dop dr dg | db dinv 0 0] (3 float4), or for
// the LM rows (xyz frozen, no inverse-depth term; `compact`) 8 floats [da db dc dop | dr dg db 0] (2 float4).
__device__ __forceinline__ void store_trec(float4* __restrict__ out, int64_t i, const float T2[10], bool compact) {
  if (compact) {
    out[2 * i + 0] = make_float4(T2[2], T2[3], T2[4], T2[5]);
    out[2 * i + 1] = make_float4(T2[6], T2[7], T2[8], 0.f);
  } else {
    out[3 * i + 0] = make_float4(T2[0], T2[1], T2[2], T2[3]);
    out[3 * i + 1] = make_float4(T2[4], T2[5], T2[6], T2[7]);
    out[3 * i + 2] = make_float4(T2[8], T2[9], 0.f, 0.f);
  }
}

template <bool RAW, bool XPBY>
__global__ __launch_bounds__(256) void k_preprocess_jvp(ViewK v, GaussK g, GaussK t, const float* __restrict__ m2t,
                                                         const uint32_t* __restrict__ clampw,
                                                         const uint32_t* __restrict__ tiles,
                                                         float4* __restrict__ trec, XpbyK xp, int compact,
                                                         int lead) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // XPBY: [256 * 3(M-1)]; lead >= 0: [256 * rest_stride]
  if (cg_stopped(v)) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!XPBY && lead >= 0) {
    // the drop-in JVP: the block's primal SH rows through LDS (per-thread reads at a 3M-float stride touch a line
    // per lane per load; stage_lead)
    stage_sh_rows(g, lead, s_rest);
  }
  if (XPBY) {
    // the direction this kernel reads is the updated one: each thread reads back only its own
    // Gaussian's elements, all written by this block before the barrier; its SH-rest tangent (the
    // bulk of them, 3(M-1) floats at a 180-B stride) from the LDS copy instead of memory
    block_xpby(xp, g.P, s_rest);
    __syncthreads();
    if (t.rest) {
      t.rest = s_rest;
      t.rest_base = (int64_t)blockIdx.x * blockDim.x;
    }
  }
  if (i >= g.P) return;
  if (tiles[i] == 0) return;  // never gathered by the render passes
  float T2[10];
  chain_jvp<RAW>(v, g, t, m2t, i, clampw[i], T2);
  store_trec(trec, i, T2, compact != 0);
}

// ------------------------------------------------------------------ launcher
int launch_tangent_pre(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
                       const ScratchBufs& sb, const XpbyK* xp, hipStream_t s, bool compact) {
  // P = 0 with a fused direction update: one block still applies the flat tail's update (block_xpby)
  if (g.P == 0 && !(xp && xp->tail_p)) return GSLM_OK;
  const unsigned nb = (unsigned)((g.P + 255) / 256) + (g.P == 0 ? 1u : 0u);
  XpbyK none{};
  const XpbyK& x = xp ? *xp : none;
  if (xp) {
    if (t.rest && (t.rest != xp->p[2] || t.rest_stride != xp->w[2])) {
      set_error("internal: fused xpby expects the tangent's SH-rest group to be p's");
      return GSLM_ERR_INVALID;
    }
    const size_t lds = (size_t)256 * xp->w[2] * sizeof(float);
    if (g.raw)
      hipLaunchKernelGGL((k_preprocess_jvp<true, true>), dim3(nb), dim3(256), lds, s, v, g, t, m2t, gb.clampw, gb.tiles,
                         sb.trec, x, compact ? 1 : 0, -1);
    else
      hipLaunchKernelGGL((k_preprocess_jvp<false, true>), dim3(nb), dim3(256), lds, s, v, g, t, m2t, gb.clampw, gb.tiles,
                         sb.trec, x, compact ? 1 : 0, -1);
  } else {
    const int lead = g.P > 0 ? stage_lead(g) : -1;
    const size_t lds = lead >= 0 ? (size_t)256 * g.rest_stride * sizeof(float) : 0;
    if (g.raw)
      hipLaunchKernelGGL((k_preprocess_jvp<true, false>), dim3(nb), dim3(256), lds, s, v, g, t, m2t, gb.clampw, gb.tiles,
                         sb.trec, x, compact ? 1 : 0, lead);
    else
      hipLaunchKernelGGL((k_preprocess_jvp<false, false>), dim3(nb), dim3(256), lds, s, v, g, t, m2t, gb.clampw, gb.tiles,
                         sb.trec, x, compact ? 1 : 0, lead);
  }
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// Gaussian-sharded exchange: the tangent render records of a Gaussian range for several views (the
// TANGENT stage of k_preprocess_jvp, looped over views), after the optional fused direction update.
// The block's SH-rest tangent slice is staged in LDS once and read by every view's chain.
template <bool XPBY>
__global__ __launch_bounds__(256) void k_tangent_views(ViewsK vs, GaussK g, GaussK t, const uint32_t* __restrict__ vflags,
                                                        int64_t fstride, float4* __restrict__ out, int64_t ostride,
                                                        XpbyK xp, int compact, int view_base) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // [256 * 3(M-1)]
  if (cg_stopped(vs.v[0])) return;  // a stopped solve (gslm_matvec_opts.cg_ctl): block-uniform, before any barrier
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + threadIdx.x;
  if (XPBY) {
    block_xpby(xp, g.P, s_rest);
  } else if (t.rest) {
    const int64_t len = min((int64_t)blockDim.x, g.P - i0) * t.rest_stride;
    const float* src = t.rest + i0 * t.rest_stride;
    for (int64_t e = threadIdx.x; e < len; e += blockDim.x) s_rest[e] = src[e];
  }
  __syncthreads();
  if (t.rest) {
    t.rest = s_rest;
    t.rest_base = i0;
  }
  if (i >= g.P) return;
#pragma unroll 1
  for (int b = 0; b < vs.n; ++b) {
    const uint32_t f = vflags[(int64_t)b * fstride + i];
    if (!(f >> 31)) continue;
    t.rest_col = view_base + b;  // SH-rest coordinates: this view's column of R
    float T2[10];
    chain_jvp<true>(vs.v[b], g, t, nullptr, i, f & 7u, T2);
    store_trec(out, (int64_t)b * ostride + i, T2, compact != 0);
  }
}

int launch_tangent_views(const ViewK* views, int nviews, const GaussK& g, const GaussK& t, const uint32_t* vflags,
                         int64_t fstride, float* out, int64_t ostride, const XpbyK* xp, hipStream_t s, bool compact,
                         int view_base) {
  if (nviews < 1 || nviews > MAX_SCREEN_VIEWS) {
    set_error("tangent_views: 1..16 views per call");
    return GSLM_ERR_INVALID;
  }
  if (g.P == 0 && !(xp && xp->tail_p)) return GSLM_OK;  // an empty shard with a tail: one block updates it
  if (xp && t.rest && (t.rest != xp->p[2] || t.rest_stride != xp->w[2])) {
    set_error("internal: fused xpby expects the tangent's SH-rest group to be p's");
    return GSLM_ERR_INVALID;
  }
  ViewsK vs;
  for (int b = 0; b < nviews; ++b) vs.v[b] = views[b];
  vs.n = nviews;
  const unsigned nb = (unsigned)((g.P + 255) / 256) + (g.P == 0 ? 1u : 0u);
  const size_t lds = t.rest ? (size_t)256 * t.rest_stride * sizeof(float) : 0;
  XpbyK none{};
  float4* o = reinterpret_cast<float4*>(out);
  if (xp)
    hipLaunchKernelGGL(k_tangent_views<true>, dim3(nb), dim3(256), lds, s, vs, g, t, vflags, fstride, o, ostride, *xp,
                       compact ? 1 : 0, view_base);
  else
    hipLaunchKernelGGL(k_tangent_views<false>, dim3(nb), dim3(256), lds, s, vs, g, t, vflags, fstride, o, ostride, none,
                       compact ? 1 : 0, view_base);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
