// backward.hip -- tile side of the VJP of the rasterizer (upstream BACKWARD::render semantics);
// the per-Gaussian side (k_preprocess_bwd, k_gather_lm) is in gather.hip.
//
//   k_render_bwd       one 16x16 tile per block, back-to-front replay from final_T / n_contrib,
//                      wave-DPP + LDS reduction per Gaussian, one plain-stored row per
//                      (tile, Gaussian) pair, rows grouped by Gaussian index.
// Linearisation = SURVEY Appendix B: alpha clamp pass-through, tan-FoV clamp zero derivative with
// no t.z cross term, SH clamp mask.  gslm_jvp (jvp.hip) is its exact transpose.
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"
#include "gslm_gather.hpp"

#ifndef GSLM_BWD_FILL
#define GSLM_BWD_FILL 1
#endif

namespace gslm {

// ROWF4 = 3: drop-in rows (screen position and inverse depth too); ROWF4 = 2: the LM rows of
// k_render_matvec (xyz frozen, no depth term), which k_gather_lm consumes -- the J^T b of an LM step.
template <bool WITH_XY, bool WITH_INV, int ROWF4>
__global__ __launch_bounds__(256, 8) void k_render_bwd(ViewK v, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ tile_order,
                                                     const uint32_t* __restrict__ point_list,
                                                     const float4* __restrict__ rec,
                                                     const uint32_t* __restrict__ slots,
                                                     const uint2* __restrict__ rect, const uint32_t* __restrict__ goff,
                                                     const float* __restrict__ final_T,
                                                     const uint32_t* __restrict__ n_contrib,
                                                     const float* __restrict__ dL_dcolor,
                                                     const float* __restrict__ dL_dinv, float4* __restrict__ rows,
                                                     int write_tail) {
  // 128-entry batches for the LM rows (as k_render_matvec: 19.7 KB of LDS); 96 for the drop-in's 9-10 values per row,
  // whose partials at 128 entries took 24-26 KB of LDS per block -> 6 blocks per CU, at 96 entries 17.9-19.5 KB -> 8
  // blocks per CU, and under __launch_bounds__(256, 8) 44-45 VGPRs (74-76 without the hint): 8 waves per SIMD
  constexpr int B = WITH_XY ? 96 : 128;
  __shared__ float2 s_rp[5 * B];  // vjp_tile's record planes
  __shared__ uint64_t s_bits[16];
  __shared__ float s_acc[vjp_acc_floats<WITH_XY, WITH_INV, B>()];
  __shared__ int s_misc[4];
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
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
  vjp_tile<WITH_XY, WITH_INV, ROWF4, B>(st, inside, (float)px, (float)py, tile_x, tile_y, ranges[tile], point_list,
                                     rec, slots, rect, goff, s_rp, s_bits, s_acc, s_misc, rows,
                                     write_tail != 0);
}

// ---------------------------------------------------------------- launchers
int launch_render_bwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                      const float* dL_dcolor, const float* dL_dinv, const ScratchBufs& sb, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (N == 0) return GSLM_OK;
  // every (tile, Gaussian) row zero first -- a streaming fill -- and the tile pass writes only the rows of entries some
  // wave visits (until round 5 it wrote every row, the never-blended ones as zeros through the rectangle's row slot:
  // three dependent random loads and a scattered 48-B store per entry, for about half of the list)
#if GSLM_BWD_FILL
  GSLM_HIP_CHECK(hipMemsetAsync(sb.contrib, 0, (size_t)N * 3 * sizeof(float4), s));
  constexpr int write_tail = 0;
#else
  constexpr int write_tail = 1;
#endif
  if (dL_dinv)
    hipLaunchKernelGGL((k_render_bwd<true, true, 3>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, nullptr, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv,
                       sb.contrib, write_tail);
  else
    hipLaunchKernelGGL((k_render_bwd<true, false, 3>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, nullptr, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv,
                       sb.contrib, write_tail);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_render_vjp_lm(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                         const float* dL_dcolor, const ScratchBufs& sb, bool tail_clean, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (N == 0) return GSLM_OK;
  if (!tail_clean) {  // the LM row map: once per geometry, shared with k_render_matvec
    const int st = launch_lm_rowmap(v, gb, bb, ib, sb, N, s);
    if (st) return st;
  }
  hipLaunchKernelGGL((k_render_bwd<false, false, 2>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                     bb.point_list, gb.rec, bb.slots, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, nullptr,
                     sb.contrib, 0);  // head rows only (launch_lm_rowmap)
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
