// gslm_gather.hpp -- the per-Gaussian side of the LM product (J^T W J v + D v): block-cooperative
// row sums and the flat param-space epilogue shared by k_gather_lm (one view, rows of this GPU) and
// k_gather_screen (the view-sharded exchange, exchange.hip).
#pragma once
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

struct FlatK {
  float* y[6];        // xyz, dc, rest, scaling, rotation, opacity groups of the output vector
  const float* v[6];  // same groups of the input vector (damping term)
  float damp[6];
  int use_damp;
  int overwrite;
  int rest_proj;      // GSLM_MV_SH_REST_PROJECTED: the rest group is 3 floats per Gaussian (see chain_jvp)
  int rest_V;         // SH-rest coordinates (gslm_rest_basis): the rest group is 3 rest_V floats, staged from dsh[1..V]
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

// y = (overwrite ? 0 : y_old) + val + d v; returns sum of v * y_new (0 when dot is off).  y is stored nontemporal:
// the gather's output is not re-read before the next kernel boundary writes the L2s back; measured -7 us on the
// gather and -2.7 us per CG iteration (4 of 4 alternations; nontemporal gradient rows, which the gather reads at
// once, cost +20 us: profiles/r06/ab_nontemporal_stores/)
template <int K>
__device__ __forceinline__ double store_group(float* y, float d, int use_damp, int64_t base, int overwrite, bool dot,
                                              const float val[K], const float vin[K], const float yold[K]) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float x = val[k];
    if (use_damp) x += d * vin[k];
    const float out = overwrite ? x : yold[k] + x;
    __builtin_nontemporal_store(out, &y[base + k]);  // streamed (profiles/r06/ab_nontemporal_stores/)
    if (dot) acc += (double)vin[k] * (double)out;
  }
  return acc;
}

// FlatK over a flat param-space output y and input v (GradK views of the 7-group vectors).
inline int make_flatk(const GaussK& g, const GradK& y, const GradK& vin, const double* damp7, bool overwrite,
                      double* dot_part, FlatK* out, bool rest_proj = false, int rest_V = 0) {
  const int64_t R = rest_V ? 3 * rest_V : rest_proj ? 3 : 3 * (g.M - 1);
  if (g.cov3D || g.colors || !g.raw || (g.M > 1 && y.rest_stride != R) || y.dc_stride != 3) {
    set_error("LM gather expects raw leaves with SH colours and a flat param-space output");
    return GSLM_ERR_INVALID;
  }
  if (rest_proj && g.M > 1 && vin.rest && vin.rest_stride != 3) {
    set_error("LM gather: a projected SH-rest group has 3 floats per Gaussian in v and y");
    return GSLM_ERR_INVALID;
  }
  if (rest_V && g.M > 1 && vin.rest && vin.rest_stride != R) {
    set_error("LM gather: SH-rest coordinates need 3 rest_views floats per Gaussian in v and y");
    return GSLM_ERR_INVALID;
  }
  FlatK o;
  o.y[0] = y.means3D; o.y[1] = y.dc; o.y[2] = y.rest; o.y[3] = y.scales; o.y[4] = y.rot; o.y[5] = y.opac;
  o.v[0] = vin.means3D; o.v[1] = vin.dc; o.v[2] = vin.rest; o.v[3] = vin.scales; o.v[4] = vin.rot; o.v[5] = vin.opac;
  // damp7 = xyz, dc, rest, scaling, rotation, opacity, exposure (GaussianModelDampMatrix order)
  for (int k = 0; k < 6; ++k) o.damp[k] = damp7 ? (float)damp7[k] : 0.f;
  o.use_damp = damp7 ? 1 : 0;
  o.overwrite = overwrite ? 1 : 0;
  o.rest_proj = (rest_proj && g.M > 1) ? 1 : 0;
  o.rest_V = g.M > 1 ? rest_V : 0;
  o.dot_part = dot_part;
  if (o.use_damp || dot_part)
    for (int k = 0; k < 6; ++k)
      if (!o.v[k] && !(k == 2 && g.M == 1)) {
        set_error("damping needs every group of v");
        return GSLM_ERR_INVALID;
      }
  *out = o;
  return GSLM_OK;
}

// LDS staging of a block's SH gradients.  FACTORED (one view's chain): dsh[k][ch] = shB[k] dres[ch],
// so 16 + 4 floats per Gaussian are staged (rows padded to 17 floats: conflict-free stores) and the
// products are formed in the coalesced store loop -- 21 KB of LDS for 256 Gaussians instead of 46 KB,
// which is the difference between 7 and 3 resident blocks per CU.  Otherwise (sums over views) the
// 3(M-1) products themselves are staged.
constexpr int SHB_STRIDE = 17;
template <bool FACTORED>
__host__ __device__ constexpr size_t sh_stage_floats(int M) {
  return FACTORED ? (size_t)256 * (SHB_STRIDE + 4) : (size_t)256 * 3 * (M > 1 ? M - 1 : 0);
}

// Writes one block's 256 Gaussians' share of y (groups xyz, dc, rest, scaling, rotation, opacity)
// from their ChainOut: y = (overwrite ? 0 : y) + J^T... + d v, and the block's partial of <v, y>.
// Called by all 256 threads; co is ignored for threads past P.  s_rest: sh_stage_floats<FACTORED>(M).
template <bool WANT_MEANS, bool FACTORED = false>
__device__ __forceinline__ void lm_epilogue(int nc, const GaussK& g, const ChainOut& co, const FlatK& o, float* s_rest,
                                            double* s_dot) {
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const int64_t nvalid = min((int64_t)blockDim.x, g.P - i0);
  // a projected SH-rest group is a 3-wide group of its own below; the LDS-staged stream covers none
  const int R = o.rest_proj ? 0 : o.rest_V ? 3 * o.rest_V : 3 * (g.M - 1);
  const bool dot = o.dot_part != nullptr;
  const int u = o.use_damp, ow = o.overwrite;
  const bool need_v = u || dot;
  double dacc = 0.0;
  __syncthreads();  // s_rest may still hold the caller's row chunks
  if (i < g.P) {
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
    if (o.rest_proj) {
      // B_rest (x) dres in the coordinate along B_rest / |B_rest|: |B_rest| dres
      float vp[3], yp[3], val[3];
      load_group<3>(o.v[2], o.y[2], 3 * i, need_v, !ow, vp, yp);
      const float nb = sh_rest_norm(co.shB, nc);
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) val[ch] = nb * co.dres[ch];
      dacc += store_group<3>(o.y[2], o.damp[2], u, 3 * i, ow, dot, val, vp, yp);
    } else if (o.rest_V) {
      // SH-rest coordinates: dsh[1 + j] holds coordinate j's gradient (k_gather_screen<true>)
#pragma unroll
      for (int j = 0; j < MAX_REST_VIEWS; ++j)
        if (j < o.rest_V) {
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) s_rest[tid * R + 3 * j + ch] = co.dsh[1 + j][ch];
        }
    } else if (FACTORED) {
#pragma unroll
      for (int k = 0; k < 16; ++k) s_rest[tid * SHB_STRIDE + k] = co.shB[k];
      float* s_d = s_rest + 256 * SHB_STRIDE;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) s_d[tid * 4 + ch] = co.dres[ch];
    } else {
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < g.M) {
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) s_rest[tid * R + 3 * (k - 1) + ch] = k < nc ? co.dsh[k][ch] : 0.f;
        }
    }
  }
  __syncthreads();
  // coalesced store of the block's contiguous [nvalid * R] slice of the SH-rest group, 8 elements per
  // thread per step with all loads issued before any store
  const int64_t base = i0 * R, total = nvalid * R;
  const float invR = R ? 1.0f / (float)R : 0.f;
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
        float val;
        if (FACTORED) {
          // e -> (Gaussian ii, coefficient k >= 1, channel ch); float quotient is exact here:
          // e < 256 R, so (e + 0.5) / R stays >= 0.5 / R away from every integer
          const int ii = (int)(((float)e + 0.5f) * invR);
          const int r = (int)e - ii * R;
          const int k = 1 + r / 3, ch = r - 3 * (k - 1);
          val = k < nc ? s_rest[ii * SHB_STRIDE + k] * s_rest[256 * SHB_STRIDE + ii * 4 + ch] : 0.f;
        } else {
          val = s_rest[e];
        }
        if (u) val += o.damp[2] * vin[k];
        const float out = ow ? val : yold[k] + val;
        __builtin_nontemporal_store(out, &o.y[2][base + e]);
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

}  // namespace gslm
