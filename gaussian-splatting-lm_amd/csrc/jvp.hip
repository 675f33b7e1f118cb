// jvp.hip -- tile passes of the forward-mode tangent and of the fused LM normal-equations product
// (the per-Gaussian tangent records come from tangent.hip).
//
//   k_render_jvp       per tile, front-to-back over the *primal's* sorted list (no re-sort), the
//                      skip/stop decisions frozen at the primal (bounded by n_contrib):
//                        dC += drgb a T + rgb (da T + a dT),  dT <- dT (1 - a) - T da.
//   k_render_matvec    the fused pair: JVP pass -> u = 2 w (.) J v in registers -> VJP pass ->
//                      one reduced row per (tile, Gaussian); the per-pixel J v never touches HBM.
//                      With the compact LM records the JVP pass runs one independent wave per quadrant
//                      (jvp_wave_packed, no block barrier; k_render_jv_wave is the J v-only form).
#include "gslm_tile.hpp"
#include "gslm_chain.hpp"

namespace gslm {

constexpr int MATVEC_BATCH = 128;

struct JvpPix {
  float T, dT, dC[3], dD;
};

// Front-to-back tangent pass over the tile, BATCH list entries staged in LDS per round.
// Block-uniform; blockDim = 256.  Wave w visits only the batch elements whose alpha region reaches its
// 8x8 quadrant (publish_quad_masks) and that lie before the last position any of its pixels blends (the
// primal's n_contrib; the same per-wave bound as vjp_tile); a lane blends entry `pos` only while
// pos < its own n_contrib -- the stop decision frozen at the primal, without a per-iteration done flag.
template <bool WITH_XY, bool WITH_INV, int BATCH>
__device__ __forceinline__ void jvp_tile(JvpPix& o, bool inside, float pxf, float pyf, int tile_x, int tile_y,
                                         uint32_t last, uint2 range, const uint32_t* __restrict__ point_list,
                                         const float4* __restrict__ rec, const float4* __restrict__ trec,
                                         float4* s_r0, float4* s_r1, float2* s_r2, float4* s_t0, float4* s_t1,
                                         float2* s_t2, uint64_t* s_bits, int* s_cnt) {
  constexpr bool PACKED = !WITH_XY && !WITH_INV;  // the LM product's records (see the staging below)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  o.T = 1.f;
  o.dT = 0.f;
  o.dC[0] = o.dC[1] = o.dC[2] = 0.f;
  o.dD = 0.f;
  const uint32_t my_last = inside ? last : 0u;
  const int wmax = wave_max_u((int)my_last);
  if (lane == 0) s_cnt[w] = wmax;
  __syncthreads();
  const int wm0 = s_cnt[0], wm1 = s_cnt[1], wm2 = s_cnt[2], wm3 = s_cnt[3];
  const int n_eff = min(max(max(wm0, wm1), max(wm2, wm3)), (int)(range.y - range.x));
  const int rounds = (n_eff + BATCH - 1) / BATCH;
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();  // the previous batch has been consumed
    const int k = r * BATCH + tid;
    uint32_t m = 0u;
    if (tid < BATCH && k < n_eff) {
      const uint32_t e = point_list[range.x + k];
      const int64_t g = pl_id(e);
      // quadrants it can touch, and only the waves that still blend at this list position
      m = pl_mask(e) & ((k < wm0 ? 1u : 0u) | (k < wm1 ? 2u : 0u) | (k < wm2 ? 4u : 0u) | (k < wm3 ? 8u : 0u));
      s_r0[tid] = rec[RECS * g + 0];
      s_r1[tid] = rec[RECS * g + 1];
      const float4 r2 = rec[RECS * g + 2];
      if (PACKED) {
        // the LM rows' compact tangent record (store_trec): [da db dc dop | dr dg db 0].  The product's 9 primal +
        // 7 tangent floats as 4 float4 at one LDS stride: the hit loop reads them with one address register;
        // the tangent conic carries its power factors (-1/2, -1, -1/2)
        const float4 c0 = trec[2 * g + 0], c1 = trec[2 * g + 1];
        s_t0[tid] = make_float4(r2.x, -0.5f * c0.x, -c0.y, -0.5f * c0.z);  // blue, da', db', dc'
        s_t1[tid] = make_float4(c0.w, c1.x, c1.y, c1.z);                    // dopacity, dr, dg, db
      } else {
        const float4 t0 = trec[3 * g + 0], t1 = trec[3 * g + 1], t2 = trec[3 * g + 2];
        s_r2[tid] = make_float2(r2.x, r2.y);
        s_t0[tid] = t0;
        s_t1[tid] = t1;
        s_t2[tid] = make_float2(t2.x, t2.y);
      }
    }
    publish_quad_masks(m, s_bits);
    __syncthreads();
    // this wave's hits in list order (latency is hidden by occupancy -- 8 waves per SIMD -- rather than
    // by register prefetch, which costs issue slots and occupancy)
    HitIter it(s_bits, w);
    if constexpr (PACKED) {
      for (int j = it.next(); j >= 0; j = it.next()) {
        const float4 a = s_r0[j], b = s_r1[j], C = s_t0[j], D = s_t1[j];
        asm volatile("" : : "v"(b.z), "v"(b.w), "v"(C.x), "v"(C.y), "v"(C.z), "v"(C.w), "v"(D.x), "v"(D.y), "v"(D.z),
                     "v"(D.w));
        const uint32_t pos = (uint32_t)(r * BATCH + j);
        const float dx = a.x - pxf, dy = a.y - pyf;
        const float power = gpower(a.z, a.w, b.x, dx, dy);
        const float G = gexp(power);
        const float alpha = fminf(0.99f, b.y * G);
        if (pos < my_last && !(power > 0.0f) && alpha >= 1.0f / 255.0f) {
#pragma clang fp contract(fast)
          const float dpower = fmaf(dx, fmaf(C.y, dx, C.z * dy), C.w * dy * dy);  // 5 VALU, not 6
          const float dalpha = G * (D.x + b.y * dpower);
          const float wt = alpha * o.T;
          const float dw = dalpha * o.T + alpha * o.dT;
          // two FMAs into the accumulator per channel (not mul + fma + add)
          o.dC[0] = fmaf(b.z, dw, fmaf(D.y, wt, o.dC[0]));
          o.dC[1] = fmaf(b.w, dw, fmaf(D.z, wt, o.dC[1]));
          o.dC[2] = fmaf(C.x, dw, fmaf(D.w, wt, o.dC[2]));
          o.dT = o.dT * (1.f - alpha) - o.T * dalpha;
          o.T = o.T * (1.f - alpha);
        }
      }
      continue;
    }
    for (int j = it.next(); j >= 0; j = it.next()) {
      const float4 a = s_r0[j], b = s_r1[j], t0 = s_t0[j], t1 = s_t1[j];
      const float2 cc = s_r2[j], t2 = s_t2[j];
      // all of the entry's primal and tangent record in one LDS round trip (the empty asm pins the
      // loads here; otherwise the tangent half is fetched inside the branch, a second exposed latency)
      asm volatile("" : : "v"(t0.z), "v"(t0.w), "v"(t1.x), "v"(t1.y), "v"(t1.z), "v"(t1.w), "v"(t2.x), "v"(b.z),
                   "v"(b.w), "v"(cc.x));
      const uint32_t pos = (uint32_t)(r * BATCH + j);
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      if (pos < my_last && !(power > 0.0f) && alpha >= 1.0f / 255.0f) {
        // the tangent arithmetic decides nothing (stop is frozen at the primal): FMA-contracted
#pragma clang fp contract(fast)
        float dpower = -0.5f * (t0.z * dx * dx + t1.x * dy * dy) - t0.w * dx * dy;
        if (WITH_XY) {
          const float ddx = t0.x, ddy = t0.y;
          dpower += -(a.z * dx * ddx + b.x * dy * ddy) - a.w * (ddx * dy + dx * ddy);
        }
        const float dalpha = G * (t1.y + b.y * dpower);
        const float wt = alpha * o.T;
        const float dw = dalpha * o.T + alpha * o.dT;
        o.dC[0] += t1.z * wt + b.z * dw;
        o.dC[1] += t1.w * wt + b.w * dw;
        o.dC[2] += t2.x * wt + cc.x * dw;
        if (WITH_INV) o.dD += t2.y * wt + cc.y * dw;
        o.dT = o.dT * (1.f - alpha) - o.T * dalpha;
        o.T = o.T * (1.f - alpha);
      }
    }
  }
}

// Front-to-back tangent pass of ONE wave over its 8x8 quadrant q, independent of the tile's other waves (no
// block barrier): 64 list positions per round, each lane fetches one; the entries whose quadrant mask holds q
// stage the compact LM record in the wave's own LDS slots (lane-indexed), and the wave walks the round's hit
// bits in list order.  Same per-lane arithmetic and decisions as jvp_tile's PACKED branch.
__device__ __forceinline__ void jvp_wave_packed(JvpPix& o, float pxf, float pyf, uint32_t my_last, int wm, int q,
                                                const uint32_t* __restrict__ pl, const float4* __restrict__ rec,
                                                const float4* __restrict__ trec, float4* s) {
  const int lane = threadIdx.x & 63;
  o.T = 1.f;
  o.dT = 0.f;
  o.dC[0] = o.dC[1] = o.dC[2] = 0.f;
  o.dD = 0.f;
  for (int base = 0; base < wm; base += 64) {
    const int k = base + lane;
    bool hit = false;
    if (k < wm) {
      const uint32_t e = pl[k];
      if ((pl_mask(e) >> q) & 1u) {
        hit = true;
        const uint32_t g = pl_id(e);
        const float4 r0 = rec[RECS * (size_t)g + 0], r1 = rec[RECS * (size_t)g + 1], r2 = rec[RECS * (size_t)g + 2];
        const float4 c0 = trec[2 * (size_t)g + 0], c1 = trec[2 * (size_t)g + 1];
        s[lane] = r0;
        s[64 + lane] = r1;
        s[128 + lane] = make_float4(r2.x, -0.5f * c0.x, -c0.y, -0.5f * c0.z);  // blue, da', db', dc'
        s[192 + lane] = make_float4(c0.w, c1.x, c1.y, c1.z);                    // dopacity, dr, dg, db
      }
    }
    uint64_t hb = __ballot(hit);
    // pos = base + j < my_last as j < my_last - base: the lane's bound once per round, the hit's index compared as
    // the SGPR it is (no scalar add per visit)
    const int rel = (int)my_last - base;
    wave_lds_sync();
    while (hb) {
      const int j = (int)__builtin_ctzll(hb);
      hb = clear_bit(hb, j);
      const float4 a = s[j], b = s[64 + j], C = s[128 + j], D = s[192 + j];
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(C.x), "v"(C.y), "v"(C.z), "v"(C.w), "v"(D.x), "v"(D.y), "v"(D.z),
                   "v"(D.w));
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      if (j < rel && !(power > 0.0f) && alpha >= 1.0f / 255.0f) {
#pragma clang fp contract(fast)
        const float dpower = fmaf(dx, fmaf(C.y, dx, C.z * dy), C.w * dy * dy);  // 5 VALU, not 6
        const float dalpha = G * (D.x + b.y * dpower);
        const float wt = alpha * o.T;
        const float dw = dalpha * o.T + alpha * o.dT;
        // two FMAs into the accumulator per channel (not mul + fma + add)
        o.dC[0] = fmaf(b.z, dw, fmaf(D.y, wt, o.dC[0]));
        o.dC[1] = fmaf(b.w, dw, fmaf(D.z, wt, o.dC[1]));
        o.dC[2] = fmaf(C.x, dw, fmaf(D.w, wt, o.dC[2]));
        o.dT = o.dT * (1.f - alpha) - o.T * dalpha;
        o.T = o.T * (1.f - alpha);
      }
    }
    wave_lds_sync();
  }
}

// J v only, compact LM records, one independent wave per quadrant (jvp_wave_packed).
__global__ __launch_bounds__(256) void k_render_jv_wave(ViewK v, const uint2* __restrict__ ranges,
                                                         const uint32_t* __restrict__ tile_order,
                                                         const uint32_t* __restrict__ point_list,
                                                         const float4* __restrict__ rec, const float4* __restrict__ trec,
                                                         const uint32_t* __restrict__ n_contrib,
                                                         float* __restrict__ out_color_t) {
  __shared__ float4 s_rec[4][4 * 64];
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x, q = tid >> 6;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
  const bool inside = px < v.W && py < v.H;
  const int64_t pid = (int64_t)py * v.W + px;
  const uint32_t last = inside ? n_contrib[pid] : 0u;
  const uint2 range = ranges[tile];
  const int wm = __builtin_amdgcn_readfirstlane(min(wave_max_u((int)last), (int)(range.y - range.x)));
  JvpPix o;
  jvp_wave_packed(o, (float)px, (float)py, last, wm, q, point_list + range.x, rec, trec, s_rec[q]);
  if (inside) {
    const int64_t HW = (int64_t)v.H * v.W;
    out_color_t[pid] = o.dC[0] + o.dT * v.bg[0];
    out_color_t[HW + pid] = o.dC[1] + o.dT * v.bg[1];
    out_color_t[2 * HW + pid] = o.dC[2] + o.dT * v.bg[2];
  }
}

template <bool WITH_XY>
__global__ __launch_bounds__(256) void k_render_jvp(ViewK v, const uint2* __restrict__ ranges,
                                                     const uint32_t* __restrict__ tile_order,
                                                     const uint32_t* __restrict__ point_list,
                                                     const float4* __restrict__ rec, const float4* __restrict__ trec,
                                                     const uint32_t* __restrict__ n_contrib,
                                                     float* __restrict__ out_color_t, float* __restrict__ out_inv_t) {
  constexpr int B = TILE_PIX;
  __shared__ float4 s_r0[B], s_r1[B], s_t0[B], s_t1[B];
  __shared__ float2 s_r2[B], s_t2[B];
  __shared__ uint64_t s_bits[16];
  __shared__ int s_cnt[4];
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
  const bool inside = px < v.W && py < v.H;
  const int64_t pid = (int64_t)py * v.W + px;
  const uint32_t last = inside ? n_contrib[pid] : 0u;
  JvpPix o;
  jvp_tile<WITH_XY, true, B>(o, inside, (float)px, (float)py, tile_x, tile_y, last, ranges[tile], point_list, rec,
                                 trec, s_r0, s_r1, s_r2, s_t0, s_t1, s_t2, s_bits, s_cnt);
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
__global__ __launch_bounds__(256, WITH_XY ? 6 : 8) void k_render_matvec(ViewK v, const uint2* __restrict__ ranges,
                                                        const uint32_t* __restrict__ tile_order,
                                                        const uint32_t* __restrict__ point_list,
                                                        const float4* __restrict__ rec, const float4* __restrict__ trec,
                                                        const uint32_t* __restrict__ slots,
                                                        const uint2* __restrict__ rect,
                                                        const uint32_t* __restrict__ goff,
                                                        const float* __restrict__ final_T,
                                                        const uint32_t* __restrict__ n_contrib,
                                                        const float* __restrict__ weight, float4* __restrict__ contrib,
                                                        int write_tail) {
  // 128-entry batches.  The LM instantiation (WITH_XY = false): 20.1 KB of LDS and 47 VGPRs -> 8 blocks per CU, 8
  // waves per SIMD (hipcc -Rpass-analysis=kernel-resource-usage; profiles/r04/resource_usage.txt); the drop-in
  // one (screen-position tangents): 23.8 KB, 64 VGPRs -> 6 blocks per CU
  constexpr int B = MATVEC_BATCH;
  __shared__ uint64_t s_bits[16];
  __shared__ int s_cnt[4];
  // The JVP pass's records and the VJP pass's staged records, per-wave partials (+ its n_eff scratch) are never
  // live together (vjp_tile starts with a block barrier): one LDS region.  Without screen-position tangents
  // the JVP pass runs one independent wave per quadrant (jvp_wave_packed: 4 x 256 float4 of wave-private
  // records); with them the block-cooperative jvp_tile.
  // float4; rounded up to 512 B: vjp_tile's record planes then start on a ds_read2st64 stride (no address add per visit)
  constexpr int kAcc = (vjp_acc_floats<WITH_XY, false, B>() + 3) / 4 + 31 & ~31;
  constexpr int kVjp = kAcc + B + B + B / 2;  // + s_r0, s_r1, s_r2 (vjp_tile: 5 float2 planes)
  constexpr int kJvp = WITH_XY ? 0 : 4 * 256;
  static_assert(!WITH_XY || kAcc >= 2 * B + B / 2, "jvp_tile's tangent records must fit below s_r0");
  __shared__ float4 s_lds[kVjp > kJvp ? kVjp : kJvp];
  float* s_acc = reinterpret_cast<float*>(s_lds);
  int* s_misc = reinterpret_cast<int*>(s_lds);
  float4* s_r0 = s_lds + kAcc;
  float4* s_r1 = s_r0 + B;
  float2* s_r2 = reinterpret_cast<float2*>(s_r1 + B);
  float4* s_t0 = s_lds;  // jvp_tile's tangent records (WITH_XY), below s_r0
  float4* s_t1 = s_t0 + B;
  float2* s_t2 = reinterpret_cast<float2*>(s_t1 + B);
  if (cg_stopped(v)) return;
  const int tile = (int)tile_order[blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = threadIdx.x;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
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
  if constexpr (WITH_XY) {
    jvp_tile<WITH_XY, false, B>(o, inside, (float)px, (float)py, tile_x, tile_y, last, range, point_list, rec, trec,
                                s_r0, s_r1, s_r2, s_t0, s_t1, s_t2, s_bits, s_cnt);
  } else {
    const int q = tid >> 6;
    const int wm = __builtin_amdgcn_readfirstlane(min(wave_max_u(inside ? (int)last : 0), (int)(range.y - range.x)));
    jvp_wave_packed(o, (float)px, (float)py, inside ? last : 0u, wm, q, point_list + range.x, rec, trec,
                    s_lds + 256 * q);
  }
  // u = 2 * w (.) (J v)   -- factor 2: the [r; r] residual aliasing of batch_training_loss.py:17
  const float u0 = 2.f * w0 * (o.dC[0] + o.dT * v.bg[0]);
  const float u1 = 2.f * w1 * (o.dC[1] + o.dT * v.bg[1]);
  const float u2 = 2.f * w2 * (o.dC[2] + o.dT * v.bg[2]);
  VjpPix st;
  vjp_init(st, v, inside, Tf, last, u0, u1, u2, 0.f);
  vjp_tile<WITH_XY, false, WITH_XY ? 3 : 2, B>(st, inside, (float)px, (float)py, tile_x, tile_y, range, point_list, rec,
                                            slots, rect, goff, reinterpret_cast<float2*>(s_r0), s_bits, s_acc, s_misc, contrib,
                                            write_tail != 0);
}

// ------------------------------------------------------------------ launchers
int launch_jvp(const ViewK& v, const GaussK& g, const GaussK& t, const float* m2t, const GeomBufs& gb,
               const BinBufs& bb, const ImgBufs& ib, const ScratchBufs& sb, float* out_color_t, float* out_inv_t,
               hipStream_t s) {
  int st = launch_tangent_pre(v, g, t, m2t, gb, sb, nullptr, s, false);  // the drop-in JVP: 12-float records
  if (st) return st;
  const int ntiles = v.gx * v.gy;
  const bool xy = t.means3D != nullptr || m2t != nullptr;
  if (xy)
    hipLaunchKernelGGL(k_render_jvp<true>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list, gb.rec,
                       sb.trec, ib.n_contrib, out_color_t, out_inv_t);
  else
    hipLaunchKernelGGL(k_render_jvp<false>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list, gb.rec,
                       sb.trec, ib.n_contrib, out_color_t, out_inv_t);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_render_jv(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                     const ScratchBufs& sb, bool mask_xyz, float* jv_out, hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  if (mask_xyz)  // the TANGENT stage of the LM rows wrote compact records
    hipLaunchKernelGGL(k_render_jv_wave, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, sb.trec, ib.n_contrib, jv_out);
  else
    hipLaunchKernelGGL(k_render_jvp<true>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,
                       bb.point_list, gb.rec, sb.trec, ib.n_contrib, jv_out, (float*)nullptr);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

int launch_matvec_render(const ViewK& v, const GaussK& t, const GeomBufs& gb, const BinBufs& bb, const ImgBufs& ib,
                         const ScratchBufs& sb, int64_t N, const float* weight, bool mask_xyz, bool tail_clean,
                         hipStream_t s) {
  const int ntiles = v.gx * v.gy;
  // the LM row map (head entries only; ScratchBufs::hscan): computed by the first product on a geometry
  if (!tail_clean) {
    const int st = launch_lm_rowmap(v, gb, bb, ib, sb, N, s);
    if (st) return st;
  }
  if (mask_xyz)
    hipLaunchKernelGGL(k_render_matvec<false>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list,
                       gb.rec, sb.trec, bb.slots, gb.rect, gb.goff, ib.final_T, ib.n_contrib, weight, sb.contrib,
                       0);  // no tail rows: the row map holds head entries only
  else
    hipLaunchKernelGGL(k_render_matvec<true>, dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order, bb.point_list,
                       gb.rec, sb.trec, bb.slots, gb.rect, gb.goff, ib.final_T, ib.n_contrib, weight, sb.contrib,
                       0);  // no tail rows: the row map holds head entries only
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
