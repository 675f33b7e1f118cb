// exchange.hip -- the view-sharded multi-GPU LM product without a param-space reduction.
//
// Each rank renders only its views.  The reference-order reduction of the partial products
// sum_b J_b^T W_b J_b v over ranks would move F = 59 floats per Gaussian (SH 3) through an all-reduce
// (2 (n-1)/n * 236 MB per rank at 1M Gaussians).  Every per-view product factors as
// J_b^T = C_b^T S_b^T: S_b^T (the tile passes) reduces to 7 screen-space floats per Gaussian
// (conic 3, opacity 1, rgb 3), and C_b^T (the per-Gaussian chain) needs only the view's camera, the
// replicated parameters and 3 clamp bits.  So ranks all-gather 8 floats per (view, Gaussian) and each
// applies every view's chain itself:
//   k_rowsum_screen   this view's rows -> [P x 8] screen block (block-cooperative, coalesced)
//   k_gather_screen   sum over views of chain_vjp(screen_b) -> flat y [+ D v], <v, y> partials
// Same arithmetic on every rank, views in index order: the ranks' y (and the CG scalars) agree
// bitwise without a broadcast.
#include "gslm_gather.hpp"

namespace gslm {

__global__ __launch_bounds__(256) void k_rowsum_screen(int64_t P, const uint32_t* __restrict__ clampw,
                                                        const uint32_t* __restrict__ tiles,
                                                        const uint32_t* __restrict__ goff,
                                                        const uint32_t* __restrict__ hscan,
                                                        const float4* __restrict__ rows, float4* __restrict__ out) {
  __shared__ float4 s_buf[GATHER_CHUNK * 2];
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + threadIdx.x;
  const int64_t nvalid = min((int64_t)blockDim.x, P - i0);
  const uint32_t n = i < P ? tiles[i] : 0u;
  float G2[NV];
  // the Gaussian's head rows of the LM row map (k_gather_lm)
  const int64_t il = i0 + nvalid - 1;
  const uint32_t R0 = hscan[goff[i0]], R1 = hscan[goff[il] + tiles[il]];
  const uint32_t h0 = i < P ? hscan[goff[i]] : R1, h1 = i < P ? hscan[goff[i] + n] : R1;
  block_sum_rows<2>(rows, R0, R1, h0, h1 - h0, s_buf, G2);
  if (i >= P) return;
  const uint32_t flags = n ? (0x80000000u | (clampw[i] & 7u)) : 0u;
  out[2 * i + 0] = make_float4(G2[2], G2[3], G2[4], G2[5]);
  out[2 * i + 1] = make_float4(G2[6], G2[7], G2[8], __uint_as_float(flags));
}

__global__ __launch_bounds__(256) void k_gather_screen(ViewsK vs, GaussK g, const float4* __restrict__ screen,
                                                        int64_t sstride, FlatK o) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // [256 * 3(M-1)]
  __shared__ double s_dot[4];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  ChainOut acc;
  acc.dop = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) { acc.dscale[k] = 0.f; acc.dmean[k] = 0.f; }
#pragma unroll
  for (int k = 0; k < 4; ++k) acc.drot[k] = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc.dsh[k][0] = acc.dsh[k][1] = acc.dsh[k][2] = 0.f;
  if (i < g.P) {
#pragma unroll 1
    for (int b = 0; b < vs.n; ++b) {
      const float4 a = screen[2 * ((int64_t)b * sstride + i) + 0];
      const float4 c = screen[2 * ((int64_t)b * sstride + i) + 1];
      const uint32_t flags = __float_as_uint(c.w);
      if (!(flags >> 31)) continue;
      const float G2[NV] = {0.f, 0.f, a.x, a.y, a.z, a.w, c.x, c.y, c.z, 0.f};
      ChainOut co;
      chain_vjp<true>(vs.v[b], g, i, true, flags & 7u, G2, false, co);
      acc.dop += co.dop;
#pragma unroll
      for (int k = 0; k < 3; ++k) acc.dscale[k] += co.dscale[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc.drot[k] += co.drot[k];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        acc.dsh[k][0] += co.dsh[k][0];
        acc.dsh[k][1] += co.dsh[k][1];
        acc.dsh[k][2] += co.dsh[k][2];
      }
    }
  }
  lm_epilogue<false>(g.M, g, acc, o, s_rest, s_dot);
}

int launch_rowsum_screen(const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, float* out, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  hipLaunchKernelGGL(k_rowsum_screen, dim3((unsigned)((g.P + 255) / 256)), dim3(256), 0, s, g.P, gb.clampw, gb.tiles,
                     gb.goff, sb.hscan, sb.contrib, reinterpret_cast<float4*>(out));
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_gather_screen(const ViewK* views, int nviews, const GaussK& g, const float* screen, int64_t sstride,
                         const GradK& y, const GradK& vin, const double* damp7, bool overwrite, double* dot_part,
                         hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  FlatK o;
  const int st = make_flatk(g, y, vin, damp7, overwrite, dot_part, &o);
  if (st) return st;
  if (nviews < 1 || nviews > MAX_SCREEN_VIEWS) {
    set_error("gather_screen: 1..16 views per call");
    return GSLM_ERR_INVALID;
  }
  ViewsK vs;
  for (int b = 0; b < nviews; ++b) vs.v[b] = views[b];
  vs.n = nviews;
  const size_t lds = sh_stage_floats<false>(g.M) * sizeof(float) + 16;
  hipLaunchKernelGGL(k_gather_screen, dim3((unsigned)((g.P + 255) / 256)), dim3(256), lds, s, vs, g,
                     reinterpret_cast<const float4*>(screen), sstride, o);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// Visibility / SH-clamp word of every Gaussian of a preprocessed view (the SCREEN rows' flags), for
// the Gaussian-sharded exchange's once-per-geometry all-to-all.
__global__ __launch_bounds__(256) void k_view_flags(int64_t P, const uint32_t* __restrict__ clampw,
                                                     const uint32_t* __restrict__ tiles, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  out[i] = tiles[i] ? (0x80000000u | (clampw[i] & 7u)) : 0u;
}

int launch_view_flags(int64_t P, const GeomBufs& gb, uint32_t* out, hipStream_t s) {
  if (P == 0) return GSLM_OK;
  hipLaunchKernelGGL(k_view_flags, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, gb.clampw, gb.tiles, out);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
