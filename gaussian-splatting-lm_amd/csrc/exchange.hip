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

// COORDS: the SH-rest group in gslm_rest_basis coordinates -- view b's rest gradient B_rest(dir_b) (x) dres_b adds
// R[j][view_base + b] dres_b to coordinate j (j <= view_base + b), accumulated in dsh[1 + j]; nothing else changes.
template <bool COORDS>
__global__ __launch_bounds__(256) void k_gather_screen(ViewsK vs, GaussK g, const float4* __restrict__ screen,
                                                        int64_t sstride, FlatK o, RestK rc) {
  extern __shared__ __attribute__((aligned(16))) float s_rest[];  // [256 * rest width]
  __shared__ double s_dot[4];
  if (cg_stopped(vs.v[0])) return;  // a stopped solve (gslm_matvec_opts.cg_ctl): block-uniform, before any barrier
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
      if constexpr (COORDS) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) acc.dsh[0][ch] += co.dsh[0][ch];
        const int col = rc.view_base + b;
        const float* Rc = rc.R + i * rest_basis_floats(rc.V) + rest_basis_floats(col);
#pragma unroll
        for (int j = 0; j < MAX_REST_VIEWS; ++j)
          if (j <= col) {
            const float r = Rc[j];
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) acc.dsh[1 + j][ch] += r * co.dres[ch];
          }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          acc.dsh[k][0] += co.dsh[k][0];
          acc.dsh[k][1] += co.dsh[k][1];
          acc.dsh[k][2] += co.dsh[k][2];
        }
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
                         hipStream_t s, const RestK& rc) {
  if (g.P == 0) return GSLM_OK;
  FlatK o;
  const int st = make_flatk(g, y, vin, damp7, overwrite, dot_part, &o, false, rc.R ? rc.V : 0);
  if (st) return st;
  if (nviews < 1 || nviews > MAX_SCREEN_VIEWS) {
    set_error("gather_screen: 1..16 views per call");
    return GSLM_ERR_INVALID;
  }
  ViewsK vs;
  for (int b = 0; b < nviews; ++b) vs.v[b] = views[b];
  vs.n = nviews;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  const float4* sc = reinterpret_cast<const float4*>(screen);
  if (o.rest_V) {
    const size_t lds = (size_t)256 * 3 * o.rest_V * sizeof(float) + 16;
    hipLaunchKernelGGL(k_gather_screen<true>, dim3(nb), dim3(256), lds, s, vs, g, sc, sstride, o, rc);
  } else {
    const size_t lds = sh_stage_floats<false>(g.M) * sizeof(float) + 16;
    hipLaunchKernelGGL(k_gather_screen<false>, dim3(nb), dim3(256), lds, s, vs, g, sc, sstride, o, rc);
  }
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

namespace gslm {

// ---------------------------------------------------------------- SH-rest coordinates (gslm_rest_basis)
// The SH-rest basis vector of view v at Gaussian i: B[k], k = 1..nc-1, the fp32 values chain_jvp / chain_vjp use
// (same direction arithmetic as chain_eval).
__device__ __forceinline__ void rest_basis_vec(const ViewK& v, const float* __restrict__ m, int64_t i, float B[16]) {
  const float dx = m[3 * i + 0] - v.campos[0], dy = m[3 * i + 1] - v.campos[1], dz = m[3 * i + 2] - v.campos[2];
  const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
  sh_basis(v.D, dx / len, dy / len, dz / len, B);
}

__device__ __forceinline__ double rest_gram(const float A[16], const float B[16], int nc) {
  double acc = 0.0;
#pragma unroll
  for (int k = 1; k < 16; ++k)
    if (k < nc) acc += (double)A[k] * (double)B[k];
  return acc;
}

// One thread per Gaussian: the Gram matrix G[a][b] = <B_a, B_b> of the V views' SH-rest vectors (double), its
// upper Cholesky factor column by column (G = R^T R, i.e. Gram-Schmidt of B_0, B_1, .. in view order), R packed by
// columns (float).  A view adding less than sqrt(1e-7) = 3.2e-4 of its norm to the earlier ones' span is dropped (row
// zeroed): gslm_rest_coords divides by the float R[b][b], so a kept view's relative R[b][b] bounds how far the float
// rounding of R (6e-8) is amplified -- at most ~2e-4 here (a 1e-6 cut, round 3, allowed ~6%), and a dropped view's
// part outside the span is below 3.2e-4 of its direction.
__global__ __launch_bounds__(256) void k_rest_basis(ViewsK vs, GaussK g, float* __restrict__ R) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P) return;
  const int V = vs.n, nc = (vs.v[0].D + 1) * (vs.v[0].D + 1);
  double Rm[MAX_REST_VIEWS][MAX_REST_VIEWS];
  float* out = R + i * rest_basis_floats(V);
#pragma unroll
  for (int b = 0; b < MAX_REST_VIEWS; ++b) {
    if (b >= V) break;
    float Bb[16], Ba[16];
    rest_basis_vec(vs.v[b], g.means3D, i, Bb);
    double Gc[MAX_REST_VIEWS];
#pragma unroll
    for (int a = 0; a < MAX_REST_VIEWS; ++a)
      if (a < b) {
        rest_basis_vec(vs.v[a], g.means3D, i, Ba);
        Gc[a] = rest_gram(Ba, Bb, nc);
      }
    const double gbb = rest_gram(Bb, Bb, nc);
    double d = gbb;
#pragma unroll
    for (int j = 0; j < MAX_REST_VIEWS; ++j)
      if (j < b) {
        double r = 0.0;
        if (Rm[j][j] != 0.0) {
          r = Gc[j];
#pragma unroll
          for (int q = 0; q < MAX_REST_VIEWS; ++q)
            if (q < j) r -= Rm[q][j] * Rm[q][b];
          r /= Rm[j][j];
        }
        Rm[j][b] = r;
        d -= r * r;
      }
    Rm[b][b] = (gbb > 0.0 && d > 1e-7 * gbb) ? sqrt(d) : 0.0;
#pragma unroll
    for (int j = 0; j < MAX_REST_VIEWS; ++j)
      if (j <= b) out[rest_basis_floats(b) + j] = (float)Rm[j][b];
  }
}

// mode 0 (expand): t = Q c = B_K R_KK^-1 c over the kept views K (back substitution); mode 1 (project):
// c = Q^T t = R_KK^-T B_K^T t (forward substitution).  One thread per Gaussian, double arithmetic.
__global__ __launch_bounds__(256) void k_rest_coords(ViewsK vs, GaussK g, const float* __restrict__ R, int mode,
                                                     const float* __restrict__ in, int64_t in_stride,
                                                     float* __restrict__ out, int64_t out_stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P) return;
  const int V = vs.n, nc = (vs.v[0].D + 1) * (vs.v[0].D + 1), M = g.M;
  const float* Rp = R + i * rest_basis_floats(V);
  auto Rjb = [&](int j, int b) { return (double)Rp[rest_basis_floats(b) + j]; };
  double y[MAX_REST_VIEWS][3];
  float B[16];
  if (mode == 0) {
#pragma unroll
    for (int b = MAX_REST_VIEWS - 1; b >= 0; --b) {
      if (b >= V) continue;
      const double rbb = Rjb(b, b);
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        double acc = in[i * in_stride + 3 * b + ch];
#pragma unroll
        for (int j = 0; j < MAX_REST_VIEWS; ++j)
          if (j > b && j < V) acc -= Rjb(b, j) * y[j][ch];
        y[b][ch] = rbb != 0.0 ? acc / rbb : 0.0;
      }
    }
    double t[15][3];
#pragma unroll
    for (int k = 0; k < 15; ++k) t[k][0] = t[k][1] = t[k][2] = 0.0;
#pragma unroll
    for (int b = 0; b < MAX_REST_VIEWS; ++b) {
      if (b >= V) break;
      rest_basis_vec(vs.v[b], g.means3D, i, B);
#pragma unroll
      for (int k = 1; k < 16; ++k)
        if (k < nc)
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) t[k - 1][ch] += (double)B[k] * y[b][ch];
    }
#pragma unroll
    for (int k = 1; k < 16; ++k)
      if (k < M)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) out[i * out_stride + 3 * (k - 1) + ch] = k < nc ? (float)t[k - 1][ch] : 0.f;
  } else {
#pragma unroll
    for (int b = 0; b < MAX_REST_VIEWS; ++b) {
      if (b >= V) break;
      rest_basis_vec(vs.v[b], g.means3D, i, B);
      const double rbb = Rjb(b, b);
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        double z = 0.0;
#pragma unroll
        for (int k = 1; k < 16; ++k)
          if (k < nc && k < M) z += (double)B[k] * (double)in[i * in_stride + 3 * (k - 1) + ch];
#pragma unroll
        for (int j = 0; j < MAX_REST_VIEWS; ++j)
          if (j < b) z -= Rjb(j, b) * y[j][ch];
        y[b][ch] = rbb != 0.0 ? z / rbb : 0.0;
        out[i * out_stride + 3 * b + ch] = (float)y[b][ch];
      }
    }
  }
}

int launch_rest_basis(const ViewK* views, int nviews, const GaussK& g, float* R, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  ViewsK vs;
  for (int b = 0; b < nviews; ++b) vs.v[b] = views[b];
  vs.n = nviews;
  hipLaunchKernelGGL(k_rest_basis, dim3((unsigned)((g.P + 255) / 256)), dim3(256), 0, s, vs, g, R);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_rest_coords(const ViewK* views, int nviews, const GaussK& g, const float* R, int mode, const float* in,
                       int64_t in_stride, float* out, int64_t out_stride, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  ViewsK vs;
  for (int b = 0; b < nviews; ++b) vs.v[b] = views[b];
  vs.n = nviews;
  hipLaunchKernelGGL(k_rest_coords, dim3((unsigned)((g.P + 255) / 256)), dim3(256), 0, s, vs, g, R, mode, in, in_stride,
                     out, out_stride);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
