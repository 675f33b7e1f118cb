// gather.hip -- per-Gaussian side of the VJP: row sums and the chain rule to the parameters.
//
//   k_preprocess_bwd   one block per 256 consecutive Gaussians: sums their contiguous rows and
//                      chains the screen-space gradient to means3D / scales / rotations / SH /
//                      opacity (or to cov3D_precomp / colors_precomp), fusing the activation
//                      derivatives when the inputs are raw GaussianModel leaves (drop-in backward).
//   k_gather_lm        the LM specialisation (raw leaves, SH colours): writes the flat param-space
//                      vector directly, overwrite or accumulate, with the damping term D v fused in,
//                      SH-rest stores staged through LDS so every store instruction is a contiguous
//                      256-B wave segment.
// Compiled apart from the tile passes: these keep clang's SLP vectoriser (Makefile).
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"
#include "gslm_gather.hpp"

namespace gslm {

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

// Drop-in backward, one block per 256 consecutive Gaussians: block-cooperative row sums (their rows
// are one contiguous range), the chain rule per thread, and the SH gradient -- 3M floats per Gaussian,
// the bulk of the output -- staged through LDS and stored as contiguous wave segments (per-thread
// stores at a 3M-float stride would touch a cache line per lane per store).
template <bool RAW>
__global__ __launch_bounds__(256) void k_preprocess_bwd(ViewK v, GaussK g, const uint32_t* __restrict__ clampw,
                                                         const uint32_t* __restrict__ tiles,
                                                         const uint32_t* __restrict__ goff,
                                                         const float4* __restrict__ rows, GradK out, int want_means) {
  extern __shared__ __attribute__((aligned(16))) float s_buf[];  // row chunks, then the factored SH stage
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const int64_t nvalid = min((int64_t)blockDim.x, g.P - i0);
  const uint32_t n = i < g.P ? tiles[i] : 0u;
  float G2[NV];
  {
    const int64_t il = i0 + nvalid - 1;
    const uint32_t R0 = goff[i0], R1 = goff[il] + tiles[il];
    block_sum_rows<3>(rows, R0, R1, i < g.P ? goff[i] : R1, n, reinterpret_cast<float4*>(s_buf), G2);
  }
  const int nc = (v.D + 1) * (v.D + 1);
  const bool sh_out = !g.colors && (out.dc || out.rest);
  // the SH colour's view-direction term of the means gradient needs <dres, sh_k> for every coefficient: per thread at a
  // 3M-float stride each of those 3(nc - 1) loads touches a line per lane, so it is formed block-cooperatively below
  // from coalesced reads of the block's SH rows (DEFER_DIR; block-uniform)
  const bool dir_term = want_means && out.means3D && !g.colors && v.D > 0;
  ChainOut co;
  if (i < g.P) {
    chain_vjp<RAW, true>(v, g, i, n != 0, n ? clampw[i] : 0u, G2, want_means != 0, co);
    write_grads(g, out, i, co, v.M, nc, want_means != 0 && !dir_term, /*skip_sh=*/true);
  }
  if (!sh_out && !dir_term) return;  // block-uniform
  // factored staging (gslm_gather.hpp): dsh[k][ch] = shB[k] dres[ch]
  float* s_d = s_buf + 256 * SHB_STRIDE;
  float* s_w = s_d + 256 * 4;  // [256][SHB_STRIDE]: <dres, sh_k> of the block's Gaussians
  if (i < g.P) {
#pragma unroll
    for (int k = 0; k < 16; ++k) s_buf[tid * SHB_STRIDE + k] = co.shB[k];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) s_d[tid * 4 + ch] = co.dres[ch];
  }
  __syncthreads();
  if (dir_term) {
    // element e = (Gaussian ii, coefficient k): 64 lanes read 4 Gaussians' consecutive 48-float rows
    for (int e = tid; e < (int)nvalid * 16; e += blockDim.x) {
      const int ii = e >> 4, k = e & 15;
      float w = 0.f;
      if (k >= 1 && k < nc) {
        const int64_t gi = i0 + ii;
        const float s0 = g.sh(gi, k, 0), s1 = g.sh(gi, k, 1), s2 = g.sh(gi, k, 2);
        w = s_d[ii * 4 + 0] * s0 + s_d[ii * 4 + 1] * s1 + s_d[ii * 4 + 2] * s2;  // chain_vjp's w, bitwise
      }
      s_w[ii * SHB_STRIDE + k] = w;
    }
    __syncthreads();
    if (i < g.P && n != 0) {
      float dm[3] = {co.dmean[0], co.dmean[1], co.dmean[2]};
      add_dir_term(v.D, co.dir, co.dirlen, s_w + tid * SHB_STRIDE, dm);
#pragma unroll
      for (int k = 0; k < 3; ++k) put(&out.means3D[3 * i + k], dm[k], out.accumulate);
    } else if (i < g.P) {
#pragma unroll
      for (int k = 0; k < 3; ++k) put(&out.means3D[3 * i + k], co.dmean[k], out.accumulate);
    }
  }
  if (!sh_out) return;
  const int acc = out.accumulate;
  const int R = 3 * v.M;
  const float invR = 1.0f / (float)R;
  for (int e = tid; e < (int)nvalid * R; e += blockDim.x) {
    const int ii = (int)(((float)e + 0.5f) * invR);  // exact: e < 256 R (see lm_epilogue)
    const int r = e - ii * R, k = r / 3, ch = r - 3 * k;
    const float val = k < nc ? s_buf[ii * SHB_STRIDE + k] * s_d[ii * 4 + ch] : 0.f;
    const int64_t gi = i0 + ii;
    if (k == 0) {
      if (out.dc) put(&out.dc[gi * out.dc_stride + ch], val, acc);
    } else if (out.rest) {
      put(&out.rest[gi * out.rest_stride + 3 * (k - 1) + ch], val, acc);
    }
  }
}

// PROJ: the projected SH-rest layout (FlatK::rest_proj) as a compile-time fact, which drops the full layout's
// SH-rest epilogue from the code: at 5 waves per SIMD (96 VGPRs) over the 4 the unconstrained register count
// allows it runs 76 -> 71 us at 1M (the kernel is latency-bound: row sums, then the parameters, then the
// vector groups).  The full-layout variant keeps the compiler's register count: forced to 96 VGPRs its SH-rest
// epilogue spills and takes 0.18 -> 0.31 ms.
template <bool WANT_MEANS, int ROWF4, bool PROJ>
__global__ __launch_bounds__(256, PROJ ? 5 : 1) void k_gather_lm(ViewK v, GaussK g, const uint32_t* __restrict__ clampw,
                                                    const uint32_t* __restrict__ tiles,
                                                    const uint32_t* __restrict__ goff,
                                                    const uint32_t* __restrict__ hscan,
                                                    const float4* __restrict__ rows, FlatK o) {
  o.rest_proj = PROJ ? 1 : 0;  // the launcher picked the variant from it
  if (cg_stopped(v)) return;
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // row chunks, then the factored SH stage
  __shared__ double s_dot[4];
  const int tid = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t i = i0 + tid;
  const int64_t nvalid = min((int64_t)blockDim.x, g.P - i0);
  const uint32_t n = i < g.P ? tiles[i] : 0u;
  float G2[NV];
  {
    // this Gaussian's head rows (the LM row map): [hscan[goff], hscan[goff + tiles])
    const int64_t il = i0 + nvalid - 1;
    const uint32_t R0 = hscan[goff[i0]], R1 = hscan[goff[il] + tiles[il]];
    const uint32_t h0 = i < g.P ? hscan[goff[i]] : R1, h1 = i < g.P ? hscan[goff[i] + n] : R1;
    block_sum_rows<ROWF4>(rows, R0, R1, h0, h1 - h0, reinterpret_cast<float4*>(s_rest), G2);
  }
  ChainOut co;
  if (i < g.P) chain_vjp<true>(v, g, i, n != 0, n ? clampw[i] : 0u, G2, WANT_MEANS, co);
  lm_epilogue<WANT_MEANS, true>((v.D + 1) * (v.D + 1), g, co, o, s_rest, s_dot);
}

// The SH-rest group of one view's Krylov space (GSLM_MV_SH_REST_PROJECTED): with one view every
// Gaussian's SH-rest column of J is B_rest(dir) (x) (d rgb), so J^T J + D (D a scalar on the group) maps
// span{B_rest(dir) (x) e_c} into itself, and every CG iterate started from J^T b stays there: 3
// coordinates per Gaussian along the unit direction Bh = B_rest / |B_rest| replace 3(M-1) floats.
//   mode 0 (expand):  out[i, k-1, c] = Bh_k in[i, c]         (k < nc; 0 for inactive coefficients)
//   mode 1 (project): out[i, c] = sum_k Bh_k in[i, k-1, c]
__global__ __launch_bounds__(256) void k_sh_rest_project(ViewK v, GaussK g, int mode, const float* __restrict__ in,
                                                         int64_t in_stride, float* __restrict__ out,
                                                         int64_t out_stride) {
  // the block's [256, M-1, 3] rows go through LDS so the full-layout side is read / written coalesced
  extern __shared__ __attribute__((aligned(16))) float s_rows[];
  const int R = 3 * (g.M - 1);
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
  const int64_t nv = min((int64_t)blockDim.x, g.P - i0);
  const int64_t i = i0 + threadIdx.x;
  if (mode == 1) {  // gather the rows to project
    for (int64_t e = threadIdx.x; e < nv * R; e += blockDim.x) {
      const int64_t ii = e / R, r = e - ii * R;
      s_rows[e] = in[(i0 + ii) * in_stride + r];
    }
    __syncthreads();
  }
  if (i < g.P) {
    const float x = g.means3D[3 * i + 0], y = g.means3D[3 * i + 1], z = g.means3D[3 * i + 2];
    const float dx = x - v.campos[0], dy = y - v.campos[1], dz = z - v.campos[2];
    const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
    float B[16];
    sh_basis(v.D, dx / len, dy / len, dz / len, B);
    const int nc = (v.D + 1) * (v.D + 1);
    const float nb = sh_rest_norm(B, nc);
    const float inv = nb > 0.f ? 1.f / nb : 0.f;
    float* row = s_rows + (int64_t)threadIdx.x * R;
    if (mode == 0) {
      for (int k = 1; k < g.M; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) row[3 * (k - 1) + c] = k < nc ? (B[k] * inv) * in[i * in_stride + c] : 0.f;
    } else {
      float acc[3] = {0.f, 0.f, 0.f};
      for (int k = 1; k < g.M && k < nc; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) acc[c] += (B[k] * inv) * row[3 * (k - 1) + c];
#pragma unroll
      for (int c = 0; c < 3; ++c) out[i * out_stride + c] = acc[c];
    }
  }
  if (mode == 0) {  // scatter the expanded rows
    __syncthreads();
    for (int64_t e = threadIdx.x; e < nv * R; e += blockDim.x) {
      const int64_t ii = e / R, r = e - ii * R;
      out[(i0 + ii) * out_stride + r] = s_rows[e];
    }
  }
}

// ---------------------------------------------------------------- launchers
int launch_sh_rest_project(const ViewK& v, const GaussK& g, int mode, const float* in, int64_t in_stride, float* out,
                           int64_t out_stride, hipStream_t s) {
  if (g.P == 0 || g.M < 2) return GSLM_OK;
  const size_t lds = (size_t)256 * 3 * (g.M - 1) * sizeof(float);
  hipLaunchKernelGGL(k_sh_rest_project, dim3((unsigned)((g.P + 255) / 256)), dim3(256), lds, s, v, g, mode, in,
                     in_stride, out, out_stride);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_preprocess_bwd(const ViewK& v, const GaussK& g, const GeomBufs& gb, const BinBufs& bb,
                          const ScratchBufs& sb, const GradK& out, bool want_means, hipStream_t s) {
  (void)bb;
  if (g.P == 0) return GSLM_OK;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  // the factored SH stage and the block's <dres, sh_k> (256 x SHB_STRIDE floats)
  const size_t sh_lds = (sh_stage_floats<true>(g.M) + (size_t)256 * SHB_STRIDE) * sizeof(float);
  const size_t chunk_lds = (size_t)GATHER_CHUNK * 3 * sizeof(float4);
  // (staging the primal SH rows here as k_preprocess_jvp does measured 221 -> 229 us at 1M: the 48 KB of LDS cost
  // more occupancy than the strided reads; profiles/r04/ab/dropin_staging -- only the 15 dot products with dres
  // are needed, formed from coalesced reads instead)
  const size_t lds = sh_lds > chunk_lds ? sh_lds : chunk_lds;
  if (g.raw)
    hipLaunchKernelGGL(k_preprocess_bwd<true>, dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.contrib, out, want_means ? 1 : 0);
  else
    hipLaunchKernelGGL(k_preprocess_bwd<false>, dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.contrib, out, want_means ? 1 : 0);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_gather_lm(const ViewK& v, const GaussK& g, const GeomBufs& gb, const ScratchBufs& sb, const GradK& y,
                     const GradK& vin, const double* damp7, bool overwrite, bool mask_xyz, double* dot_part,
                     hipStream_t s, bool rest_proj) {
  if (g.P == 0) return GSLM_OK;
  FlatK o;
  const int st = make_flatk(g, y, vin, damp7, overwrite, dot_part, &o, rest_proj);
  if (st) return st;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  const size_t rest_lds = sh_stage_floats<true>(g.M) * sizeof(float);
  const size_t chunk_lds = (size_t)GATHER_CHUNK * (mask_xyz ? 2 : 3) * sizeof(float4);
  const size_t lds = (rest_lds > chunk_lds ? rest_lds : chunk_lds) + 16;
  if (mask_xyz && o.rest_proj)
    hipLaunchKernelGGL((k_gather_lm<false, 2, true>), dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.hscan, sb.contrib, o);
  else if (mask_xyz)
    hipLaunchKernelGGL((k_gather_lm<false, 2, false>), dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.hscan, sb.contrib, o);
  else if (o.rest_proj)
    hipLaunchKernelGGL((k_gather_lm<true, 3, true>), dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.hscan, sb.contrib, o);
  else
    hipLaunchKernelGGL((k_gather_lm<true, 3, false>), dim3(nb), dim3(256), lds, s, v, g, gb.clampw, gb.tiles, gb.goff,
                       sb.hscan, sb.contrib, o);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
