// backward.hip -- VJP of the rasterizer (upstream BACKWARD::render + BACKWARD::preprocess semantics).
//
//   k_render_bwd       one 16x16 tile per block, back-to-front replay from final_T / n_contrib,
//                      wave-DPP + LDS reduction per Gaussian, one plain-stored row per
//                      (tile, Gaussian) pair, rows grouped by Gaussian index.
//   k_preprocess_bwd   one thread per Gaussian: sums its contiguous rows and chains the
//                      screen-space gradient to means3D / scales / rotations / SH / opacity (or to
//                      cov3D_precomp / colors_precomp), fusing the activation derivatives when the
//                      inputs are raw GaussianModel leaves (drop-in backward, every input variant).
//   k_gather_lm        the LM specialisation of k_preprocess_bwd (raw leaves, SH colours): writes
//                      the flat param-space vector directly, overwrite or accumulate, with the
//                      damping term D v fused in, SH-rest stores staged through LDS so every
//                      store instruction is a contiguous 256-B wave segment.
// Linearisation = SURVEY Appendix B: alpha clamp pass-through, tan-FoV clamp zero derivative with
// no t.z cross term, SH clamp mask.  gslm_jvp (jvp.hip) is its exact transpose.
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

template <bool WITH_XY, bool WITH_INV>
__global__ __launch_bounds__(256) void k_render_bwd(ViewK v, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ point_list,
                                                     const float4* __restrict__ rec, const uint2* __restrict__ rect,
                                                     const uint32_t* __restrict__ goff,
                                                     const float* __restrict__ final_T,
                                                     const uint32_t* __restrict__ n_contrib,
                                                     const float* __restrict__ dL_dcolor,
                                                     const float* __restrict__ dL_dinv, float4* __restrict__ rows) {
  __shared__ float4 s_r0[TILE_PIX], s_r1[TILE_PIX];
  __shared__ float2 s_r2[TILE_PIX];
  __shared__ uint64_t s_bits[16];
  __shared__ float s_acc[vjp_acc_floats<WITH_XY, WITH_INV, TILE_PIX>()];
  __shared__ int s_misc[4];
  const int tile = blockIdx.x;
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
  vjp_tile<WITH_XY, WITH_INV, 3, TILE_PIX>(st, inside, (float)px, (float)py, tile_x, tile_y, ranges[tile], point_list, rec,
                                 rect, goff, s_r0, s_r1, s_r2, s_bits, s_acc, s_misc, rows);
}

template <int ROWF4>
__device__ __forceinline__ void sum_rows(const float4* __restrict__ rows, uint32_t off, uint32_t n, float G2[NV]) {
#pragma unroll
  for (int q = 0; q < NV; ++q) G2[q] = 0.f;
  for (uint32_t t = 0; t < n; ++t) {
    float r[NV];
    load_row<ROWF4>(rows, (size_t)off + t, r);
#pragma unroll
    for (int q = 0; q < NV; ++q) G2[q] += r[q];
  }
}

template <bool RAW>
__global__ __launch_bounds__(256) void k_preprocess_bwd(ViewK v, GaussK g, const float4* __restrict__ rec,
                                                         const uint32_t* __restrict__ tiles,
                                                         const uint32_t* __restrict__ goff,
                                                         const float4* __restrict__ rows, GradK out, int want_means) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P) return;
  const uint32_t n = tiles[i];
  float G2[NV];
  sum_rows<3>(rows, n ? goff[i] : 0u, n, G2);
  ChainOut co;
  chain_vjp<RAW>(v, g, i, n != 0, rec, G2, want_means != 0, co);
  write_grads(g, out, i, co, v.M, (v.D + 1) * (v.D + 1), want_means != 0);
}

// ---------------------------------------------------------------- LM gather (flat param space)
struct FlatK {
  float* y[6];        // xyz, dc, rest, scaling, rotation, opacity groups of the output vector
  const float* v[6];  // same groups of the input vector (damping term)
  float damp[6];
  int use_damp;
  int overwrite;
  double* dot_part;   // per-block partials of <v, y> over the written elements (NULL = off)
};

// y[idx] (op)= val (+ d v[idx]); returns v[idx] * y_new for the fused <v, y> (0 when dot is off)
__device__ __forceinline__ double emit(float* y, const float* v, float d, int use_damp, int overwrite, bool dot,
                                       int64_t idx, float val) {
  const float vv = (use_damp || dot) ? v[idx] : 0.f;
  if (use_damp) val += d * vv;
  float out = val;
  if (overwrite) y[idx] = val;
  else {
    out = y[idx] + val;
    y[idx] = out;
  }
  return dot ? (double)vv * (double)out : 0.0;
}

template <bool WANT_MEANS, int ROWF4>
__global__ __launch_bounds__(256) void k_gather_lm(ViewK v, GaussK g, const float4* __restrict__ rec,
                                                    const uint32_t* __restrict__ tiles,
                                                    const uint32_t* __restrict__ goff,
                                                    const float4* __restrict__ rows, FlatK o) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // [256 * 3(K-1)]
  __shared__ double s_dot[4];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const int R = 3 * (g.M - 1);
  const int nc = (v.D + 1) * (v.D + 1);
  const bool dot = o.dot_part != nullptr;
  double dacc = 0.0;
  if (i < g.P) {
    const uint32_t n = tiles[i];
    float G2[NV];
    sum_rows<ROWF4>(rows, n ? goff[i] : 0u, n, G2);
    ChainOut co;
    chain_vjp<true>(v, g, i, n != 0, rec, G2, WANT_MEANS, co);
    const int u = o.use_damp, ow = o.overwrite;
    if (WANT_MEANS) {
#pragma unroll
      for (int k = 0; k < 3; ++k) dacc += emit(o.y[0], o.v[0], o.damp[0], u, ow, dot, 3 * i + k, co.dmean[k]);
    } else if (ow) {
#pragma unroll
      for (int k = 0; k < 3; ++k) dacc += emit(o.y[0], o.v[0], o.damp[0], u, 1, dot && u, 3 * i + k, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) dacc += emit(o.y[1], o.v[1], o.damp[1], u, ow, dot, 3 * i + k, co.dsh[0][k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) dacc += emit(o.y[3], o.v[3], o.damp[3], u, ow, dot, 3 * i + k, co.dscale[k]);
#pragma unroll
    for (int k = 0; k < 4; ++k) dacc += emit(o.y[4], o.v[4], o.damp[4], u, ow, dot, 4 * i + k, co.drot[k]);
    dacc += emit(o.y[5], o.v[5], o.damp[5], u, ow, dot, i, co.dop);
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < g.M) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) s_rest[tid * R + 3 * (k - 1) + ch] = k < nc ? co.dsh[k][ch] : 0.f;
      }
  }
  __syncthreads();
  // coalesced store of the block's contiguous [nvalid * R] slice of the SH-rest group
  const int64_t nvalid = min((int64_t)blockDim.x, g.P - i0);
  const int64_t base = i0 * R;
  for (int64_t e = tid; e < nvalid * R; e += blockDim.x)
    dacc += emit(o.y[2], o.v[2], o.damp[2], o.use_damp, o.overwrite, dot, base + e, s_rest[e]);
  if (dot) {
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dacc += __shfl_down(dacc, off, 64);
    if (lane == 0) s_dot[w] = dacc;
    __syncthreads();
    if (tid == 0) o.dot_part[blockIdx.x] = ((s_dot[0] + s_dot[1]) + s_dot[2]) + s_dot[3];
  }
}

// ---------------------------------------------------------------- launchers
int launch_render_bwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, int64_t N,
                      const float* dL_dcolor, const float* dL_dinv, const ScratchBufs& sb, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (N == 0) return GSLM_OK;
  if (dL_dinv)
    hipLaunchKernelGGL((k_render_bwd<true, true>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv, sb.contrib);
  else
    hipLaunchKernelGGL((k_render_bwd<true, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv, sb.contrib);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_preprocess_bwd(const ViewK& v, const GaussK& g, const GeomBufs& gb, const BinBufs& bb,
                          const ScratchBufs& sb, const GradK& out, bool want_means, hipStream_t s) {
  (void)bb;
  if (g.P == 0) return GSLM_OK;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  if (g.raw)
    hipLaunchKernelGGL(k_preprocess_bwd<true>, dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.tiles, gb.goff,
                       sb.contrib, out, want_means ? 1 : 0);
  else
    hipLaunchKernelGGL(k_preprocess_bwd<false>, dim3(nb), dim3(256), 0, s, v, g, gb.rec, gb.tiles, gb.goff,
                       sb.contrib, out, want_means ? 1 : 0);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_gather_lm(const ViewK& v, const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, const GradK& y,
                     const GradK& vin, const double* damp7, bool overwrite, bool mask_xyz, double* dot_part,
                     hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  if (g.cov3D || g.colors || !g.raw || y.rest_stride != 3 * (g.M - 1) || y.dc_stride != 3) {
    set_error("LM gather expects raw leaves with SH colours and a flat param-space output");
    return GSLM_ERR_INVALID;
  }
  FlatK o;
  o.y[0] = y.means3D; o.y[1] = y.dc; o.y[2] = y.rest; o.y[3] = y.scales; o.y[4] = y.rot; o.y[5] = y.opac;
  o.v[0] = vin.means3D; o.v[1] = vin.dc; o.v[2] = vin.rest; o.v[3] = vin.scales; o.v[4] = vin.rot; o.v[5] = vin.opac;
  // damp7 = xyz, dc, rest, scaling, rotation, opacity, exposure (GaussianModelDampMatrix order)
  for (int k = 0; k < 6; ++k) o.damp[k] = damp7 ? (float)damp7[k] : 0.f;
  o.use_damp = damp7 ? 1 : 0;
  o.overwrite = overwrite ? 1 : 0;
  o.dot_part = dot_part;
  if (o.use_damp || dot_part)
    for (int k = 0; k < 6; ++k)
      if (!o.v[k] && !(k == 2 && g.M == 1)) { set_error("damping needs every group of v"); return GSLM_ERR_INVALID; }
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  const size_t lds = (size_t)256 * 3 * (g.M - 1) * sizeof(float) + 16;
  if (mask_xyz)
    hipLaunchKernelGGL((k_gather_lm<false, 2>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.tiles, gb.goff,
                       sb.contrib, o);
  else
    hipLaunchKernelGGL((k_gather_lm<true, 3>), dim3(nb), dim3(256), lds, s, v, g, gb.rec, gb.tiles, gb.goff,
                       sb.contrib, o);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
