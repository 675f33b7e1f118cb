// render_fwd.hip -- the rasterizer forward's per-tile blend (upstream renderCUDA semantics, SURVEY App. A
// step 11): one 16x16 tile per 256-thread block, wave w on the tile's 8x8 quadrant w (tile_pixel), each wave
// visiting only the list entries whose alpha region reaches its quadrant (the point list's quadrant masks),
// front to back until T < 1e-4.
//
// Compiled apart from the per-Gaussian kernels with -fno-slp-vectorize (Makefile), like the other tile
// passes: the loop body is scalar f32 math and one branch, the per-lane stop kept as a lane mask (the wave
// leaves when every lane has stopped), no software pipelining of the next records (measured: no gain).
#include "gslm_tile.hpp"

namespace gslm {

// One independent wave per 8x8 quadrant: 64 list positions per round, each lane fetches one, the entries whose
// mask holds the quadrant stage their record in the wave's own LDS slots (lane-indexed), and the wave walks the
// round's hit bits in list order.  No block barrier: a wave leaves as soon as all of its pixels have stopped,
// however far the tile's other quadrants still go (a block-cooperative version with 256-entry LDS batches
// measured 1.5% slower on the full forward).
// MODE (the epilogue): FWD_FULL colour + inverse depth + final_T / n_contrib (gslm_rasterize, the drop-in forward);
// FWD_NO_INV the same without the inverse-depth accumulation (out_invdepth NULL: the LM paths); FWD_LOSS the
// validation loss of the LM line search without any image: per pixel r = m clamp(C + T bg) - gt (gslm_lm_residual's
// arithmetic), sum r^2 in double per tile -> part[tile] (gslm_rasterize_loss).
enum { FWD_FULL = 0, FWD_NO_INV = 1, FWD_LOSS = 2 };

// SLOT (FWD_LOSS only): the line search's union list (gslm_rasterize_loss_slot) -- an entry is visited by its set's
// bits of amask (k_slot_masks: the set's own quadrant mask, 0 outside the set's rect) instead of the point list's.
template <int MODE, bool SLOT = false>
__global__ __launch_bounds__(256) void k_render_fwd_wave(ViewK v, const uint2* __restrict__ ranges,
                                                          const uint32_t* __restrict__ tile_order,
                                                          const uint32_t* __restrict__ point_list,
                                                          const float4* __restrict__ rec, float* __restrict__ out_color,
                                                          float* __restrict__ out_invdepth, float* __restrict__ final_T,
                                                          uint32_t* __restrict__ n_contrib, const float* __restrict__ gt,
                                                          const float* __restrict__ mask, double* __restrict__ part,
                                                          const uint32_t* __restrict__ amask = nullptr, int shift = 0) {
  __shared__ float4 s_rec[4][3 * 64];
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x, q = tid >> 6, lane = tid & 63;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
  const bool inside = px < v.W && py < v.H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);
  const uint32_t* pl = point_list + range.x;
  float4* s = s_rec[q];

  // A stopped lane (or one outside the image) carries T <= 0: minus its transmittance at the stop, which a live lane
  // (T >= 1e-4) never is.  Every visit then runs the same per-lane arithmetic with no boolean lane state across
  // iterations (each one would cost a few scalar mask instructions per visit; with them the loop was bound by its
  // scalar instructions, not VALU): a stopped lane's test_T = T (1 - u) <= 0 stops it again, with weight 0, and
  // -|T| keeps T -- one select with source modifiers, where a separate stop-transmittance register cost two VALU.
  float T = inside ? 1.0f : 0.0f;
  uint32_t last = 0;
  float C0 = 0.f, C1 = 0.f, C2 = 0.f, Dp = 0.f;
  uint64_t live = __builtin_amdgcn_ballot_w64(inside);  // lanes not yet stopped (inside the image), wave-uniform
  for (int base = 0; base < n; base += 64) {
    if (live == 0ull) break;  // every pixel of this quadrant has stopped
    const int k = base + lane;
    bool hit = false;
    if (k < n) {
      const uint32_t e = pl[k];
      if (((SLOT ? amask[range.x + k] >> shift : pl_mask(e)) >> q) & 1u) {
        hit = true;
        const uint32_t g = pl_id(e);
        s[lane] = rec[RECS * (size_t)g + 0];
        s[64 + lane] = rec[RECS * (size_t)g + 1];
        s[128 + lane] = rec[RECS * (size_t)g + 2];
      }
    }
    uint64_t hb = __ballot(hit);
    wave_lds_sync();
    while (hb) {
      const int j = (int)__builtin_ctzll(hb);
      hb = clear_bit(hb, j);
      const float4 a = s[j], b = s[64 + j], cc = s[128 + j];
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(cc.x), "v"(cc.y));
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float alpha = fminf(0.99f, b.y * gexp(power));
      // u: the alpha the reference blends, 0 where it skips the Gaussian (power > 0, alpha < 1/255): T * (1 - 0)
      // and colour * 0 leave T and the sums unchanged bitwise (the sums start at +0, colours and 1/depth are >= 0)
      float u = alpha >= 1.0f / 255.0f ? alpha : 0.0f;
      u = power > 0.0f ? 0.0f : u;
      const float test_T = T * (1.0f - u);
      // a live lane has T >= 1e-4, so with u = 0 it never stops here; a stopped lane (T = 0) re-stops harmlessly
      const bool stop = test_T < 0.0001f;
      const float wt = stop ? 0.0f : u * T;
      // the colour sums decide nothing (the stop and skip tests above are upstream's roundings): one FMA each
      C0 = __builtin_fmaf(b.z, wt, C0);
      C1 = __builtin_fmaf(b.w, wt, C1);
      C2 = __builtin_fmaf(cc.x, wt, C2);
      if (MODE == FWD_FULL) Dp = __builtin_fmaf(cc.y, wt, Dp);
      T = stop ? -fabsf(T) : test_T;
      if (MODE != FWD_LOSS) last = wt > 0.0f ? (uint32_t)(base + j + 1) : last;  // blended: 1-based list position
      // the stop compare's lane mask (no VGPR round trip) leaves `live`; the round ends when no lane is
      live_update(live, hb, __builtin_amdgcn_ballot_w64(stop));
    }
    wave_lds_sync();
  }
  T = T > 0.0f ? T : -T;  // the transmittance the reference keeps: at the stop, else after the last Gaussian
  const int64_t pid = (int64_t)py * v.W + px;
  const int64_t HW = (int64_t)v.H * v.W;
  if constexpr (MODE == FWD_LOSS) {
    __shared__ double s_sum[4];
    double acc = 0.0;
    if (inside) {
      const float m = mask ? mask[pid] : 1.0f;
      const float R[3] = {C0 + T * v.bg[0], C1 + T * v.bg[1], C2 + T * v.bg[2]};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float r = m * clamp01(R[c]) - gt[c * HW + pid];
        acc += (double)r * (double)r;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (lane == 0) s_sum[q] = acc;
    __syncthreads();
    if (tid == 0) part[tile] = ((s_sum[0] + s_sum[1]) + s_sum[2]) + s_sum[3];
  } else if (inside) {
    final_T[pid] = T;
    n_contrib[pid] = last;
    out_color[pid] = C0 + T * v.bg[0];
    out_color[HW + pid] = C1 + T * v.bg[1];
    out_color[2 * HW + pid] = C2 + T * v.bg[2];
    if (MODE == FWD_FULL) out_invdepth[pid] = Dp;
  }
}

// The line search's union list blended for all NS parameter sets in ONE pass (gslm_rasterize_loss_sets): per wave the
// list is walked once -- each round's 64 entries and their mask words loaded once -- and set a's round is
// k_render_fwd_wave<FWD_LOSS, true>'s round for slot a: its hits (bit 4a + q) staged from set a's records, the same
// visit arithmetic on set a's own pixel state, the same per-set stop.  Set a + 1's records are loaded while set a's
// hits are visited, so a round waits on two dependent loads (entries, set 0's records) instead of two per set.
// Every set's visits and their order are the single-set kernel's: the same losses, bitwise.
template <int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NS <= 6 ? 8 : 1))) void k_render_loss_sets(ViewK v, const uint2* __restrict__ ranges,
                                                           const uint32_t* __restrict__ tile_order,
                                                           const uint32_t* __restrict__ point_list,
                                                           const uint32_t* __restrict__ amask, SetRecsK sr,
                                                           const float* __restrict__ gt, const float* __restrict__ mask,
                                                           double* __restrict__ part, int shift) {
  __shared__ float4 s_rec[4][3 * 64];
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x, q = tid >> 6, lane = tid & 63;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
  const bool inside = px < v.W && py < v.H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);
  const uint32_t* pl = point_list + range.x;
  const uint32_t* am = amask + range.x;
  float4* s = s_rec[q];
  float T[NS], C0[NS], C1[NS], C2[NS];  // T: k_render_fwd_wave's stopped-lane encoding (-|T| at the stop)
  uint64_t live[NS];  // per set: lanes not yet stopped
  const uint64_t in0 = __builtin_amdgcn_ballot_w64(inside);
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    T[a] = inside ? 1.0f : 0.0f;
    C0[a] = C1[a] = C2[a] = 0.f;
    live[a] = in0;
  }
  for (int base = 0; base < n; base += 64) {
    bool all = true;
#pragma unroll
    for (int a = 0; a < NS; ++a) all = all && live[a] == 0ull;
    if (all) break;  // every pixel of this quadrant has stopped in every set
    const int k = base + lane;
    uint32_t g = 0u, m = 0u;
    if (k < n) {
      g = pl_id(pl[k]);
      m = am[k] >> shift;  // sets first_set.. of the union binning (gslm_rasterize_loss_sets' first_set)
    }
    // set 0's records of this lane's entry (if it is a hit of a set still blending)
    bool hit = live[0] != 0ull && ((m >> q) & 1u);
    float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra, rc = ra;
    if (hit) {
      const float4* r = sr.rec[0] + RECS * (size_t)g;
      ra = r[0];
      rb = r[1];
      rc = r[2];
    }
#pragma unroll
    for (int a = 0; a < NS; ++a) {
      if (hit) {
        s[lane] = ra;
        s[64 + lane] = rb;
        s[128 + lane] = rc;
      }
      uint64_t hb = __ballot(hit);
      wave_lds_sync();
      if (a + 1 < NS) {  // the next set's records while this set's hits are visited
        hit = live[a + 1] != 0ull && ((m >> (4 * (a + 1) + q)) & 1u);
        if (hit) {
          const float4* r = sr.rec[a + 1] + RECS * (size_t)g;
          ra = r[0];
          rb = r[1];
          rc = r[2];
        }
      }
      float Ta = T[a], c0 = C0[a], c1 = C1[a], c2 = C2[a];
      uint64_t lv = live[a];
      while (hb) {
        const int j = (int)__builtin_ctzll(hb);
        hb = clear_bit(hb, j);
        const float4 x = s[j], y = s[64 + j], z = s[128 + j];
        asm volatile("" : : "v"(y.z), "v"(y.w), "v"(z.x));
        const float dx = x.x - pxf, dy = x.y - pyf;
        const float power = gpower(x.z, x.w, y.x, dx, dy);
        const float alpha = fminf(0.99f, y.y * gexp(power));
        float u = alpha >= 1.0f / 255.0f ? alpha : 0.0f;
        u = power > 0.0f ? 0.0f : u;
        const float test_T = Ta * (1.0f - u);
        const bool stop = test_T < 0.0001f;
        const float wt = stop ? 0.0f : u * Ta;
        c0 = __builtin_fmaf(y.z, wt, c0);  // k_render_fwd_wave's colour FMAs
        c1 = __builtin_fmaf(y.w, wt, c1);
        c2 = __builtin_fmaf(z.x, wt, c2);
        Ta = stop ? -fabsf(Ta) : test_T;
        live_update(lv, hb, __builtin_amdgcn_ballot_w64(stop));
      }
      T[a] = Ta;
      C0[a] = c0;
      C1[a] = c1;
      C2[a] = c2;
      live[a] = lv;
      wave_lds_sync();  // this set's hits read before the next set's are staged
    }
  }
  const int64_t HW = (int64_t)v.H * v.W;
  __shared__ double s_sum[NS][4];
  float gtc[3] = {0.f, 0.f, 0.f};
  float mv = 1.0f;
  if (inside) {
    const int64_t pid = (int64_t)(int)pyf * v.W + (int)pxf;  // from the loop's live pixel centre, not a kept index
    mv = mask ? mask[pid] : 1.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) gtc[c] = gt[c * HW + pid];
  }
#pragma unroll
  for (int a = 0; a < NS; ++a) {
    double acc = 0.0;
    if (inside) {
      const float Tf = T[a] > 0.0f ? T[a] : -T[a];
      const float R[3] = {C0[a] + Tf * v.bg[0], C1[a] + Tf * v.bg[1], C2[a] + Tf * v.bg[2]};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float r = mv * clamp01(R[c]) - gtc[c];
        acc += (double)r * (double)r;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (lane == 0) s_sum[a][q] = acc;
  }
  __syncthreads();
  if (tid < NS) part[(int64_t)tid * (v.gx * v.gy) + tile] = ((s_sum[tid][0] + s_sum[tid][1]) + s_sum[tid][2]) + s_sum[tid][3];
}

// per set a (block a): the sum of its per-tile partials in tile order, times 2, into *loss[a] (k_tile_loss_final);
// nsets (or NULL): the union binning's recorded set count -- slot first_set + a at or past it (masks that were never
// built) gets a NaN loss, as gslm_rasterize_loss_slot gives it
__global__ __launch_bounds__(256) void k_tile_loss_final_sets(const double* __restrict__ part, int np, int accumulate,
                                                               LossPtrsK lp, const uint32_t* __restrict__ nsets,
                                                               int first_set) {
  __shared__ double s[4];
  const int a = blockIdx.x;
  double acc = strided_sum_in_order(part + (int64_t)a * np, np);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double l = 2.0 * (((s[0] + s[1]) + s[2]) + s[3]);
    if (nsets && (uint32_t)(first_set + a) >= *nsets) l = __longlong_as_double(0x7ff8000000000000ll);  // quiet NaN
    double* out = lp.loss[a];
    *out = accumulate ? *out + l : l;
  }
}

int launch_render_loss_sets(const ViewK& v, const SetRecsK& sr, int nsets, const BinBufs& bb, const uint32_t* amask,
                            const float* gt, const float* mask, double* part, const LossPtrsK& lp, int accumulate,
                            hipStream_t s, int first_set, const uint32_t* nsets_dev) {
  const int ntiles = v.gx * v.gy;
  if (ntiles == 0) {
    if (!accumulate)
      for (int a = 0; a < nsets; ++a) GSLM_HIP_CHECK(hipMemsetAsync(lp.loss[a], 0, sizeof(double), s));
    return GSLM_OK;
  }
  const dim3 grid(ntiles), block(TILE_PIX);
  switch (nsets) {
#define GSLM_LOSS_SETS(NS)                                                                                           \
  case NS:                                                                                                           \
    hipLaunchKernelGGL(k_render_loss_sets<NS>, grid, block, 0, s, v, bb.ranges, bb.tile_order, bb.point_list, amask, \
                       sr, gt, mask, part, 4 * first_set);                                                           \
    break;
    GSLM_LOSS_SETS(1) GSLM_LOSS_SETS(2) GSLM_LOSS_SETS(3) GSLM_LOSS_SETS(4)
    GSLM_LOSS_SETS(5) GSLM_LOSS_SETS(6) GSLM_LOSS_SETS(7) GSLM_LOSS_SETS(8)
#undef GSLM_LOSS_SETS
    default:
      set_error("rasterize_loss_sets: 1..8 parameter sets");
      return GSLM_ERR_INVALID;
  }
  hipLaunchKernelGGL(k_tile_loss_final_sets, dim3(nsets), dim3(256), 0, s, (const double*)part, ntiles, accumulate, lp,
                     amask ? nsets_dev : nullptr, first_set);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// sum of the per-tile loss partials in tile order (deterministic), times 2 (the [r; r] aliasing)
// nsets (or NULL): the union binning's recorded set count; slot >= *nsets (masks that were never built) -> NaN loss
__global__ __launch_bounds__(256) void k_tile_loss_final(const double* __restrict__ part, int np, int accumulate,
                                                          double* __restrict__ loss, const uint32_t* __restrict__ nsets,
                                                          int slot) {
  __shared__ double s[4];
  double acc = strided_sum_in_order(part, np);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double l = 2.0 * (((s[0] + s[1]) + s[2]) + s[3]);
    if (nsets && (uint32_t)slot >= *nsets) l = __longlong_as_double(0x7ff8000000000000ll);  // quiet NaN
    *loss = accumulate ? *loss + l : l;
  }
}

int launch_render_fwd(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib, float* out_color,
                      float* out_invdepth, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (ntiles == 0) return GSLM_OK;
  if (out_invdepth)
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_FULL, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, out_color, out_invdepth, ib.final_T, ib.n_contrib, (const float*)nullptr,
                       (const float*)nullptr, (double*)nullptr, (const uint32_t*)nullptr, 0);
  else
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_NO_INV, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, out_color, (float*)nullptr, ib.final_T, ib.n_contrib, (const float*)nullptr,
                       (const float*)nullptr, (double*)nullptr, (const uint32_t*)nullptr, 0);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_render_loss(const ViewK& v, const GeomBufs& gb, const BinBufs& bb, const float* gt, const float* mask,
                       double* part, double* loss, int accumulate, hipStream_t s, const uint32_t* amask, int shift,
                       const uint32_t* nsets) {
  const int ntiles = v.gx * v.gy;
  if (ntiles == 0) {
    if (!accumulate) GSLM_HIP_CHECK(hipMemsetAsync(loss, 0, sizeof(double), s));
    return GSLM_OK;
  }
  if (amask)
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_LOSS, true>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges,
                       bb.tile_order, bb.point_list, gb.rec, (float*)nullptr, (float*)nullptr, (float*)nullptr,
                       (uint32_t*)nullptr, gt, mask, part, amask, shift);
  else
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_LOSS, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges,
                       bb.tile_order, bb.point_list, gb.rec, (float*)nullptr, (float*)nullptr, (float*)nullptr,
                       (uint32_t*)nullptr, gt, mask, part, (const uint32_t*)nullptr, 0);
  hipLaunchKernelGGL(k_tile_loss_final, dim3(1), dim3(256), 0, s, (const double*)part, ntiles, accumulate, loss,
                     amask ? nsets : nullptr, shift / 4);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
