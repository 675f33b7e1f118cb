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
                                                     const uint32_t* __restrict__ tile_order,
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

// Block-cooperative version of sum_rows for the 256 consecutive Gaussians of a block: their rows are
// one contiguous range (row_slot groups rows by Gaussian index), streamed through LDS in chunks of
// GATHER_CHUNK rows with coalesced float4 loads; each thread then adds its own rows from LDS, in the
// same order as sum_rows (bitwise-identical sums).  Must be called by all 256 threads.
constexpr int GATHER_CHUNK = 512;
template <int ROWF4>
__device__ __forceinline__ void block_sum_rows(const float4* __restrict__ rows, uint32_t R0, uint32_t R1,
                                               uint32_t my_off, uint32_t my_n, float4* s_buf, float G2[NV]) {
#pragma unroll
  for (int q = 0; q < NV; ++q) G2[q] = 0.f;
  const uint32_t my_end = my_off + my_n;
  for (uint32_t c0 = R0; c0 < R1; c0 += GATHER_CHUNK) {
    const uint32_t cn = min((uint32_t)GATHER_CHUNK, R1 - c0);
    __syncthreads();  // the previous chunk has been consumed
    for (uint32_t e = threadIdx.x; e < cn * ROWF4; e += blockDim.x) s_buf[e] = rows[(size_t)c0 * ROWF4 + e];
    __syncthreads();
    const uint32_t lo = max(my_off, c0), hi = min(my_end, c0 + cn);
    for (uint32_t r = lo; r < hi; ++r) {
      float t[NV];
      load_row<ROWF4>(s_buf, r - c0, t);
#pragma unroll
      for (int q = 0; q < NV; ++q) G2[q] += t[q];
    }
  }
  __syncthreads();  // s_buf may be reused by the caller
}

template <int K>
__device__ __forceinline__ void load_group(const float* v, const float* y, int64_t base, bool need_v, bool need_y,
                                           float vin[K], float yold[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    vin[k] = need_v ? v[base + k] : 0.f;
    yold[k] = need_y ? y[base + k] : 0.f;
  }
}

// y = (overwrite ? 0 : y_old) + val + d v; returns sum of v * y_new (0 when dot is off)
template <int K>
__device__ __forceinline__ double store_group(float* y, float d, int use_damp, int64_t base, int overwrite, bool dot,
                                              const float val[K], const float vin[K], const float yold[K]) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float x = val[k];
    if (use_damp) x += d * vin[k];
    const float out = overwrite ? x : yold[k] + x;
    y[base + k] = out;
    if (dot) acc += (double)vin[k] * (double)out;
  }
  return acc;
}

template <bool WANT_MEANS, int ROWF4>
__global__ __launch_bounds__(256) void k_gather_lm(ViewK v, GaussK g, const float4* __restrict__ rec,
                                                    const uint32_t* __restrict__ tiles,
                                                    const uint32_t* __restrict__ goff,
                                                    const float4* __restrict__ rows, FlatK o) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // [256 * 3(K-1)], first the row chunks
  __shared__ double s_dot[4];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const int R = 3 * (g.M - 1);
  const int nc = (v.D + 1) * (v.D + 1);
  const bool dot = o.dot_part != nullptr;
  double dacc = 0.0;
  const int64_t nvalid = min((int64_t)blockDim.x, g.P - i0);
  const uint32_t n = i < g.P ? tiles[i] : 0u;
  float G2[NV];
  {
    const int64_t il = i0 + nvalid - 1;
    const uint32_t R0 = goff[i0], R1 = goff[il] + tiles[il];
    block_sum_rows<ROWF4>(rows, R0, R1, i < g.P ? goff[i] : R1, n, reinterpret_cast<float4*>(s_rest), G2);
  }
  const int u = o.use_damp, ow = o.overwrite;
  const bool need_v = u || dot;
  if (i < g.P) {
    ChainOut co;
    chain_vjp<true>(v, g, i, n != 0, rec, G2, WANT_MEANS, co);
    // Load phase first, store phase second: y may alias nothing, but the compiler cannot know, so
    // interleaved load/store pairs would serialise on memory latency.
    const bool xyz_on = WANT_MEANS || ow;
    float vx[3], yx[3], vdc[3], ydc[3], vs[3], ys[3], vr[4], yr[4], vo[1], yo[1];
    load_group<3>(o.v[0], o.y[0], 3 * i, xyz_on && need_v, xyz_on && !ow, vx, yx);
    load_group<3>(o.v[1], o.y[1], 3 * i, need_v, !ow, vdc, ydc);
    load_group<3>(o.v[3], o.y[3], 3 * i, need_v, !ow, vs, ys);
    load_group<4>(o.v[4], o.y[4], 4 * i, need_v, !ow, vr, yr);
    load_group<1>(o.v[5], o.y[5], i, need_v, !ow, vo, yo);
    if (WANT_MEANS) {
      dacc += store_group<3>(o.y[0], o.damp[0], u, 3 * i, ow, dot, co.dmean, vx, yx);
    } else if (ow) {
      const float z[3] = {0.f, 0.f, 0.f};
      dacc += store_group<3>(o.y[0], o.damp[0], u, 3 * i, 1, dot && u, z, vx, yx);
    }
    dacc += store_group<3>(o.y[1], o.damp[1], u, 3 * i, ow, dot, co.dsh[0], vdc, ydc);
    dacc += store_group<3>(o.y[3], o.damp[3], u, 3 * i, ow, dot, co.dscale, vs, ys);
    dacc += store_group<4>(o.y[4], o.damp[4], u, 4 * i, ow, dot, co.drot, vr, yr);
    const float dop[1] = {co.dop};
    dacc += store_group<1>(o.y[5], o.damp[5], u, i, ow, dot, dop, vo, yo);
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < g.M) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) s_rest[tid * R + 3 * (k - 1) + ch] = k < nc ? co.dsh[k][ch] : 0.f;
      }
  }
  __syncthreads();
  // coalesced store of the block's contiguous [nvalid * R] slice of the SH-rest group, 8 elements per
  // thread per step with all loads issued before any store
  const int64_t base = i0 * R, total = nvalid * R;
  constexpr int U = 8;
  for (int64_t e0 = 0; e0 < total; e0 += (int64_t)U * blockDim.x) {
    float vin[U], yold[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t e = e0 + (int64_t)k * blockDim.x + tid;
      const bool in = e < total;
      vin[k] = (in && need_v) ? o.v[2][base + e] : 0.f;
      yold[k] = (in && !ow) ? o.y[2][base + e] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t e = e0 + (int64_t)k * blockDim.x + tid;
      if (e < total) {
        float val = s_rest[e];
        if (u) val += o.damp[2] * vin[k];
        const float out = ow ? val : yold[k] + val;
        o.y[2][base + e] = out;
        if (dot) dacc += (double)vin[k] * (double)out;
      }
    }
  }
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
    hipLaunchKernelGGL((k_render_bwd<true, true>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list,
                       gb.rec, gb.rect, gb.goff, ib.final_T, ib.n_contrib, dL_dcolor, dL_dinv, sb.contrib);
  else
    hipLaunchKernelGGL((k_render_bwd<true, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list,
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
  const size_t rest_lds = (size_t)256 * 3 * (g.M - 1) * sizeof(float);
  const size_t chunk_lds = (size_t)GATHER_CHUNK * (mask_xyz ? 2 : 3) * sizeof(float4);
  const size_t lds = (rest_lds > chunk_lds ? rest_lds : chunk_lds) + 16;
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
