// jvp.hip -- forward-mode tangent of the rasterizer and the fused LM normal-equations product.
//
//   k_preprocess_jvp   one thread per visible Gaussian: tangent render record (48 B) from the
//                      input tangents (chain_jvp, exact transpose of chain_vjp).
//   k_render_jvp       per tile, front-to-back over the *primal's* sorted list (no re-sort), the
//                      skip/stop decisions frozen at the primal (bounded by n_contrib):
//                        dC += drgb a T + rgb (da T + a dT),  dT <- dT (1 - a) - T da.
//   k_render_matvec    the fused pair: JVP pass -> u = 2 w (.) J v in registers -> VJP pass ->
//                      one reduced row per (tile, Gaussian); the per-pixel J v never touches HBM.
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

template <bool RAW>
__global__ __launch_bounds__(256) void k_preprocess_jvp(ViewK v, GaussK g, GaussK t, const float* __restrict__ m2t,
                                                         const float4* __restrict__ rec,
                                                         const uint32_t* __restrict__ tiles,
                                                         float4* __restrict__ trec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.P) return;
  if (tiles[i] == 0) return;  // never gathered by the render passes
  float T2[10];
  chain_jvp<RAW>(v, g, t, m2t, i, rec, T2);
  trec[3 * i + 0] = make_float4(T2[0], T2[1], T2[2], T2[3]);
  trec[3 * i + 1] = make_float4(T2[4], T2[5], T2[6], T2[7]);
  trec[3 * i + 2] = make_float4(T2[8], T2[9], 0.f, 0.f);
}

struct JvpPix {
  float T, dT, dC[3], dD;
};

// Front-to-back tangent pass over the tile.  Block-uniform; blockDim = 256.
template <bool WITH_XY, bool WITH_INV>
__device__ __forceinline__ void jvp_tile(JvpPix& o, bool inside, float pxf, float pyf, uint32_t last, uint2 range,
                                         const uint32_t* __restrict__ point_list, const float4* __restrict__ rec,
                                         const float4* __restrict__ trec, float4* s_r0, float4* s_r1, float4* s_r2,
                                         float4* s_t0, float4* s_t1, float4* s_t2) {
  const int tid = threadIdx.x;
  o.T = 1.f;
  o.dT = 0.f;
  o.dC[0] = o.dC[1] = o.dC[2] = 0.f;
  o.dD = 0.f;
  bool done = !inside || last == 0;
  const int n = (int)(range.y - range.x);
  const int rounds = (n + TILE_PIX - 1) / TILE_PIX;
  uint32_t contributor = 0;
  int todo = n;
  for (int r = 0; r < rounds; ++r, todo -= TILE_PIX) {
    const int num_done = __syncthreads_count(done);
    if (num_done == TILE_PIX) break;
    const int k = r * TILE_PIX + tid;
    if (k < n) {
      const uint32_t g = point_list[range.x + k];
      s_r0[tid] = rec[3 * (int64_t)g + 0];
      s_r1[tid] = rec[3 * (int64_t)g + 1];
      s_r2[tid] = rec[3 * (int64_t)g + 2];
      s_t0[tid] = trec[3 * (int64_t)g + 0];
      s_t1[tid] = trec[3 * (int64_t)g + 1];
      s_t2[tid] = trec[3 * (int64_t)g + 2];
    }
    __syncthreads();
    const int cnt = min(TILE_PIX, todo);
    for (int j = 0; !done && j < cnt; ++j) {
      ++contributor;
      const float4 a = s_r0[j];
      const float4 b = s_r1[j];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = -0.5f * (a.z * dx * dx + b.x * dy * dy) - a.w * dx * dy;
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      if (!(power > 0.0f) && alpha >= 1.0f / 255.0f) {
        const float4 c = s_r2[j];
        const float4 t0 = s_t0[j];
        const float4 t1 = s_t1[j];
        float dpower = -0.5f * (t0.z * dx * dx + t1.x * dy * dy) - t0.w * dx * dy;
        if (WITH_XY) {
          const float ddx = t0.x, ddy = t0.y;
          dpower += -(a.z * dx * ddx + b.x * dy * ddy) - a.w * (ddx * dy + dx * ddy);
        }
        const float dalpha = G * (t1.y + b.y * dpower);
        const float w = alpha * o.T;
        const float dw = dalpha * o.T + alpha * o.dT;
        o.dC[0] += t1.z * w + b.z * dw;
        o.dC[1] += t1.w * w + b.w * dw;
        if (WITH_INV) {
          const float4 t2 = s_t2[j];
          o.dC[2] += t2.x * w + c.x * dw;
          o.dD += t2.y * w + c.y * dw;
        } else {
          o.dC[2] += s_t2[j].x * w + c.x * dw;
        }
        o.dT = o.dT * (1.f - alpha) - o.T * dalpha;
        o.T = o.T * (1.f - alpha);
        if (contributor == last) done = true;
      }
    }
  }
}

template <bool WITH_XY>
__global__ __launch_bounds__(256) void k_render_jvp(ViewK v, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ point_list,
                                                     const float4* __restrict__ rec, const float4* __restrict__ trec,
                                                     const uint32_t* __restrict__ n_contrib,
                                                     float* __restrict__ out_color_t, float* __restrict__ out_inv_t) {
  __shared__ float4 s_r0[TILE_PIX], s_r1[TILE_PIX], s_r2[TILE_PIX];
  __shared__ float4 s_t0[TILE_PIX], s_t1[TILE_PIX], s_t2[TILE_PIX];
  const int tile = blockIdx.x;
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  const int px = tile_x * TILE_X + (tid & 15), py = tile_y * TILE_Y + (tid >> 4);
  const bool inside = px < v.W && py < v.H;
  const int64_t pid = (int64_t)py * v.W + px;
  const uint32_t last = inside ? n_contrib[pid] : 0u;
  JvpPix o;
  jvp_tile<WITH_XY, true>(o, inside, (float)px, (float)py, last, ranges[tile], point_list, rec, trec, s_r0, s_r1,
                          s_r2, s_t0, s_t1, s_t2);
  if (inside) {
    const int64_t HW = (int64_t)v.H * v.W;
    out_color_t[pid] = o.dC[0] + o.dT * v.bg[0];
    out_color_t[HW + pid] = o.dC[1] + o.dT * v.bg[1];
    out_color_t[2 * HW + pid] = o.dC[2] + o.dT * v.bg[2];
    if (out_inv_t) out_inv_t[pid] = o.dD;
  }
}

// Fused (J^T W J) v for one view: JVP pass, per-pixel weight, VJP pass.
template <bool WITH_XY>
__global__ __launch_bounds__(256) void k_render_matvec(ViewK v, const uint2* __restrict__ ranges,
                                                        const uint32_t* __restrict__ point_list,
                                                        const float4* __restrict__ rec, const float4* __restrict__ trec,
                                                        const uint2* __restrict__ rect,
                                                        const uint32_t* __restrict__ goff,
                                                        const float* __restrict__ final_T,
                                                        const uint32_t* __restrict__ n_contrib,
                                                        const float* __restrict__ weight, float4* __restrict__ contrib) {
  __shared__ float4 s_r0[TILE_PIX], s_r1[TILE_PIX], s_r2[TILE_PIX];
  __shared__ float4 s_t0[TILE_PIX], s_t1[TILE_PIX], s_t2[TILE_PIX];
  __shared__ float s_acc[vjp_acc_floats<WITH_XY, false>()];
  __shared__ int s_misc[4];
  const int tile = blockIdx.x;
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  const int px = tile_x * TILE_X + (tid & 15), py = tile_y * TILE_Y + (tid >> 4);
  const bool inside = px < v.W && py < v.H;
  const int64_t pid = (int64_t)py * v.W + px;
  const int64_t HW = (int64_t)v.H * v.W;
  const uint2 range = ranges[tile];
  uint32_t last = 0;
  float Tf = 0.f, w0 = 0.f, w1 = 0.f, w2 = 0.f;
  if (inside) {
    last = n_contrib[pid];
    Tf = final_T[pid];
    w0 = weight[pid];
    w1 = weight[HW + pid];
    w2 = weight[2 * HW + pid];
  }
  JvpPix o;
  jvp_tile<WITH_XY, false>(o, inside, (float)px, (float)py, last, range, point_list, rec, trec, s_r0, s_r1, s_r2,
                           s_t0, s_t1, s_t2);
  // u = 2 * w (.) (J v)   -- factor 2: the [r; r] residual aliasing of batch_training_loss.py:17
  const float u0 = 2.f * w0 * (o.dC[0] + o.dT * v.bg[0]);
  const float u1 = 2.f * w1 * (o.dC[1] + o.dT * v.bg[1]);
  const float u2 = 2.f * w2 * (o.dC[2] + o.dT * v.bg[2]);
  VjpPix st;
  vjp_init(st, v, inside, Tf, last, u0, u1, u2, 0.f);
  vjp_tile<WITH_XY, false, WITH_XY ? 3 : 2>(st, inside, (float)px, (float)py, tile_x, tile_y, range, point_list, rec,
                                            rect, goff, s_r0, s_r1, s_r2, s_acc, s_misc, contrib);
}

// ------------------------------------------------------------------ launchers
int launch_tangent_pre(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
                       const ScratchBufs& sb, hipStream_t s) {
  if (g.P == 0) return GSLM_OK;
  const unsigned nb = (unsigned)((g.P + 255) / 256);
  if (g.raw)
    hipLaunchKernelGGL(k_preprocess_jvp<true>, dim3(nb), dim3(256), 0, s, v, g, t, m2t, gb.rec, gb.tiles, sb.trec);
  else
    hipLaunchKernelGGL(k_preprocess_jvp<false>, dim3(nb), dim3(256), 0, s, v, g, t, m2t, gb.rec, gb.tiles, sb.trec);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
               const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb, float* out_color_t, float* out_inv_t,
               hipStream_t s) {
  int st = launch_tangent_pre(v, g, t, m2t, gb, sb, s);
  if (st) return st;
  const int ntiles = v.gx * v.gy;
  const bool xy = t.means3D != nullptr || m2t != nullptr;
  if (xy)
    hipLaunchKernelGGL(k_render_jvp<true>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list, gb.rec,
                       sb.trec, ib.n_contrib, out_color_t, out_inv_t);
  else
    hipLaunchKernelGGL(k_render_jvp<false>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list, gb.rec,
                       sb.trec, ib.n_contrib, out_color_t, out_inv_t);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_matvec_render(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                         const ScratchBufs& sb, const float* weight, bool mask_xyz, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (mask_xyz)
    hipLaunchKernelGGL(k_render_matvec<false>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, sb.trec, gb.rect, gb.goff, ib.final_T, ib.n_contrib, weight, sb.contrib);
  else
    hipLaunchKernelGGL(k_render_matvec<true>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.point_list,
                       gb.rec, sb.trec, gb.rect, gb.goff, ib.final_T, ib.n_contrib, weight, sb.contrib);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
