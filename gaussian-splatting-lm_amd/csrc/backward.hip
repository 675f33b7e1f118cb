// backward.hip -- VJP of the rasterizer (upstream BACKWARD::render + BACKWARD::preprocess semantics).
//
//   k_render_bwd       one 16x16 tile per block, back-to-front replay from final_T / n_contrib,
//                      wave-DPP + LDS reduction per Gaussian, one plain-stored row per list slot.
//   k_preprocess_bwd   one thread per Gaussian: gathers its rows (through inv[]) and chains the
//                      screen-space gradient to means3D / scales / rotations / SH / opacity (or to
//                      cov3D_precomp / colors_precomp), fusing the activation derivatives when the
//                      inputs are raw GaussianModel leaves.
// Linearisation = SURVEY Appendix B: alpha clamp pass-through, tan-FoV clamp zero derivative with
// no t.z cross term, SH clamp mask.  gslm_jvp (jvp.hip) is its exact transpose.
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

template <bool WITH_XY, bool WITH_INV>
__global__ __launch_bounds__(256) void k_render_bwd(ViewK v, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ point_list,
                                                     const float4* __restrict__ rec, const float* __restrict__ final_T,
                                                     const uint32_t* __restrict__ n_contrib,
                                                     const float* __restrict__ dL_dcolor,
                                                     const float* __restrict__ dL_dinv, float4* __restrict__ contrib) {
  __shared__ float4 s_r0[TILE_PIX], s_r1[TILE_PIX], s_r2[TILE_PIX];
  __shared__ float s_acc[4 * NV * TILE_PIX];
  __shared__ int s_misc[4];
  const int tile = blockIdx.x;
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  const int px = tile_x * TILE_X + (tid & 15), py = tile_y * TILE_Y + (tid >> 4);
  const bool inside = px < v.W && py < v.H;
  const int64_t pid = (int64_t)py * v.W + px;
  const int64_t HW = (int64_t)v.H * v.W;
  float d0 = 0.f, d1 = 0.f, d2 = 0.f, di = 0.f, Tf = 0.f;
  uint32_t last = 0;
  if (inside) {
    d0 = dL_dcolor[pid];
    d1 = dL_dcolor[HW + pid];
    d2 = dL_dcolor[2 * HW + pid];
    if (WITH_INV) di = dL_dinv[pid];
    Tf = final_T[pid];
    last = n_contrib[pid];
  }
  VjpPix st;
  vjp_init(st, v, inside, Tf, last, d0, d1, d2, di);
  vjp_tile<WITH_XY, WITH_INV>(st, inside, (float)px, (float)py, ranges[tile], point_list, rec, s_r0, s_r1, s_r2,
                              s_acc, s_misc, contrib);
}

template <bool RAW>
__global__ __launch_bounds__(256) void k_preprocess_bwd(ViewK v, GaussK g, const float4* __restrict__ rec,
                                                         const uint32_t* __restrict__ tiles,
                                                         const uint32_t* __restrict__ offset_by_g,
                                                         const uint32_t* __restrict__ inv,
                                                         const float4* __restrict__ contrib, GradK out,
                                                         int want_means) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P) return;
  const uint32_t n = tiles[i];
  float G2[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) G2[q] = 0.f;
  if (n) {
    const uint32_t off = offset_by_g[i];
    for (uint32_t t = 0; t < n; ++t) {
      const int64_t k = inv[off + t];
      const float4 a = contrib[3 * k + 0], b = contrib[3 * k + 1], c = contrib[3 * k + 2];
      G2[0] += a.x; G2[1] += a.y; G2[2] += a.z; G2[3] += a.w;
      G2[4] += b.x; G2[5] += b.y; G2[6] += b.z; G2[7] += b.w;
      G2[8] += c.x; G2[9] += c.y;
    }
  }
  ChainOut co;
  chain_vjp<RAW>(v, g, i, n != 0, rec, G2, want_means != 0, co);
  write_grads(g, out, i, co, v.M, (v.D + 1) * (v.D + 1), want_means != 0);
}

int launch_render_bwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                      const float* dL_dcolor, const float* dL_dinv, const ScratchBufs& sb, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (N == 0) return GSLM_OK;
  if (dL_dinv)
    hipLaunchKernelGGL((k_render_bwd<true, true>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv, sb.contrib);
  else
    hipLaunchKernelGGL((k_render_bwd<true, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv, sb.contrib);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_preprocess_bwd(const ViewK& v, const GaussK& g, const GeomBufs& gb, const BinBufs& bb,
                          const ScratchBufs& sb, const GradK& out, bool want_means, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  if (g.raw)
    hipLaunchKernelGGL(k_preprocess_bwd<true>, dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.tiles, gb.offset_by_g,
                       bb.inv, sb.contrib, out, want_means ? 1 : 0);
  else
    hipLaunchKernelGGL(k_preprocess_bwd<false>, dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.tiles, gb.offset_by_g,
                       bb.inv, sb.contrib, out, want_means ? 1 : 0);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
