// gslm_tile.hpp -- per-tile back-to-front (VJP) pass shared by the drop-in backward and the fused
// LM matvec kernels.
//
// VJP accumulation strategy (MI355X-specific): instead of upstream's per-pixel global atomicAdd
// (10 atomics per pixel-Gaussian pair), every wave reduces a Gaussian's per-pixel contributions
// with a 6-step DPP reduction, the 4 waves' partials meet in LDS, and each (tile, Gaussian) pair
// writes ONE row with plain stores.  Rows are grouped by Gaussian index (row_slot), so the
// per-Gaussian sum over tiles in the gather kernel reads contiguous memory.  No float atomics
// anywhere: results are bitwise reproducible run to run.
#pragma once
#include "gslm_kernels.hpp"

namespace gslm {

template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, BANK_MASK, true));
}

// Sum over the 64 lanes of a wave; the total lands in lane 63.  Requires all 64 lanes active.
__device__ __forceinline__ float wave_sum_lane63(float x) {
  x += dpp_f<0x111>(x);       // row_shr:1
  x += dpp_f<0x112>(x);       // row_shr:2
  x += dpp_f<0x114>(x);       // row_shr:4
  x += dpp_f<0x118>(x);       // row_shr:8   -> lane 15 of each row holds the row sum
  x += dpp_f<0x142, 0xa>(x);  // row_bcast:15 into rows 1 and 3
  x += dpp_f<0x143, 0xc>(x);  // row_bcast:31 into rows 2 and 3 -> lane 63 holds the total
  return x;
}

// Transposed ("reduce-scatter") sum of 8 values per lane over the 64 lanes of a wave, using the
// gfx950 permlane swaps for the cross-half steps and DPP inside rows.  On return every lane of the
// 8-lane group k (lanes 8k..8k+7) holds sum over the wave of v[k].  18 instructions instead of
// 8 x 6 DPP adds.  Requires all 64 lanes active.
__device__ __forceinline__ float perm32_add(float a, float b, float& hi_part) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  (void)hi_part;
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float perm16_add(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float wave_reduce8_t(const float v[8], int lane) {
  float dummy = 0.f;
  // step 1 (lanes l <-> l+32): lower half keeps values 0..3, upper half values 4..7
  const float w0 = perm32_add(v[0], v[4], dummy), w1 = perm32_add(v[1], v[5], dummy);
  const float w2 = perm32_add(v[2], v[6], dummy), w3 = perm32_add(v[3], v[7], dummy);
  // step 2 (rows r <-> r^1): even rows keep w0, w1; odd rows keep w2, w3
  const float u0 = perm16_add(w0, w2), u1 = perm16_add(w1, w3);
  // step 3 (lanes l <-> l^8 inside a row): bit3 = 0 keeps u0, bit3 = 1 keeps u1
  const bool hi8 = (lane & 8) != 0;
  const float give = hi8 ? u0 : u1;
  float x = hi8 ? u1 : u0;
  x += dpp_f<0x128>(give);  // row_ror:8
  // step 4: sum the 8 lanes of the group
  x += dpp_f<0xB1>(x);      // quad_perm [1,0,3,2]
  x += dpp_f<0x4E>(x);      // quad_perm [2,3,0,1]
  x += dpp_f<0x141>(x);     // row_half_mirror
  return x;                 // value index of this lane: (lane >> 3) & 7
}

// Orders a wave's LDS stores before its later loads of other lanes' slots (a wave's LDS operations complete in
// order; this only stops the compiler from moving them across).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The blend loops' exit test in two scalar ALU instructions (clang's `dmask |= stopped; if (dmask == ~0) break;`
// was 6-8 per visit, the uniform exit lowered through a VCC select; with clear_bit, gslm_kernels.hpp).
// live &= ~stopped, and the round's remaining hits dropped once no lane is live (s_andn2_b64 sets SCC = live != 0):
// the loop's `while (hb)` is then its only exit test
__device__ __forceinline__ void live_update(uint64_t& live, uint64_t& hb, uint64_t stopped) {
  asm("s_andn2_b64 %0, %0, %2\n\ts_cselect_b64 %1, %1, 0" : "+s"(live), "+s"(hb) : "s"(stopped) : "scc");
}

// Block-wide count of `pred` over 256 threads (4 waves) with one barrier; s_cnt = 4 ints of LDS the
// caller owns.  Replaces __syncthreads_count, whose lowering reserves 256 B of LDS per block -- the
// difference between 3 and 4 resident blocks per CU for k_render_matvec.  Safe to call once per
// round as long as another barrier separates consecutive calls (the batch-load barrier does).
__device__ __forceinline__ int block_count(bool pred, int* s_cnt) {
  const uint64_t b = __ballot(pred);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = __popcll(b);
  __syncthreads();
  return (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
}

// Wave-wide max of a non-negative int (all lanes active); every lane gets the result.
__device__ __forceinline__ int wave_max_u(int x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o));
  return x;
}

// Screen-space gradient of one (tile, Gaussian) pair, value index q:
//   0 dL/dx_pix  1 dL/dy_pix  2 dL/dconic.a  3 dL/dconic.b  4 dL/dconic.c  5 dL/dopacity_eff
//   6..8 dL/drgb  9 dL/dinvdepth
// Row formats: ROWF4 = 3 (general): [x y a b | c o r g | b inv 0 0]
//              ROWF4 = 2 (LM, xyz frozen, no depth term): [a b c o | r g b 0]
constexpr int NV = 10;

template <bool WITH_XY, bool WITH_INV>
__host__ __device__ constexpr bool q_used(int q) {
  return (q >= 2 && q <= 8) || (q < 2 && WITH_XY) || (q == 9 && WITH_INV);
}
template <bool WITH_XY, bool WITH_INV>
__host__ __device__ constexpr int n_used() {
  return 7 + (WITH_XY ? 2 : 0) + (WITH_INV ? 1 : 0);
}
template <bool WITH_XY, bool WITH_INV>
__host__ __device__ constexpr int q_slot(int q) {
  int s = 0;
  for (int k = 0; k < q; ++k) s += q_used<WITH_XY, WITH_INV>(k) ? 1 : 0;
  return s;
}

template <int ROWF4>
__device__ __forceinline__ void store_row(float4* __restrict__ rows, uint32_t slot, const float t[NV]) {
  if (ROWF4 == 3) {
    rows[3 * (size_t)slot + 0] = make_float4(t[0], t[1], t[2], t[3]);
    rows[3 * (size_t)slot + 1] = make_float4(t[4], t[5], t[6], t[7]);
    rows[3 * (size_t)slot + 2] = make_float4(t[8], t[9], 0.f, 0.f);
  } else {
    rows[2 * (size_t)slot + 0] = make_float4(t[2], t[3], t[4], t[5]);
    rows[2 * (size_t)slot + 1] = make_float4(t[6], t[7], t[8], 0.f);
  }
}

template <int ROWF4>
__device__ __forceinline__ void load_row(const float4* __restrict__ rows, size_t slot, float t[NV]) {
  if (ROWF4 == 3) {
    const float4 a = rows[3 * slot + 0], b = rows[3 * slot + 1], c = rows[3 * slot + 2];
    t[0] = a.x; t[1] = a.y; t[2] = a.z; t[3] = a.w; t[4] = b.x; t[5] = b.y; t[6] = b.z; t[7] = b.w;
    t[8] = c.x; t[9] = c.y;
  } else {
    const float4 a = rows[2 * slot + 0], b = rows[2 * slot + 1];
    t[0] = 0.f; t[1] = 0.f; t[2] = a.x; t[3] = a.y; t[4] = a.z; t[5] = a.w; t[6] = b.x; t[7] = b.y;
    t[8] = b.z; t[9] = 0.f;
  }
}

struct VjpPix {
  float T;          // running transmittance (starts at final_T)
  float T_final;
  uint32_t last;    // n_contrib (1-based index of the last blended Gaussian)
  float dpix[3];    // dL/dcolor of this pixel
  float dinv;       // dL/dinvdepth of this pixel
  float bg_dot;     // <bg, dL/dpix>
  // Upstream keeps the colour (and inverse depth) accumulated behind the current Gaussian per channel,
  // but only its dot product with dL/dpix enters dL/dalpha; the recurrence is linear, so the dot
  // itself is carried: accd = <acc, dL/dpix> (+ acc_inv dL/dinvdepth).  Upstream folds the previous
  // Gaussian in at the start of the next visit (accum = last_alpha last_colour + (1 - last_alpha) accum);
  // here each visit folds its own Gaussian in at its end -- the same operands and FMA, so the same values,
  // without carrying last_alpha / last_colour across iterations.
  float accd;
  float tb;         // -T_final <bg, dL/dpix>: the background term of dL/dalpha is tb / (1 - alpha)
};

__device__ __forceinline__ void vjp_init(VjpPix& s, const ViewK& v, bool inside, float T_final, uint32_t last,
                                         float d0, float d1, float d2, float dinv) {
  s.T_final = inside ? T_final : 0.f;
  s.T = s.T_final;
  s.last = inside ? last : 0u;
  s.dpix[0] = d0; s.dpix[1] = d1; s.dpix[2] = d2;
  s.dinv = dinv;
  s.bg_dot = (v.bg[0] * d0 + v.bg[1] * d1) + v.bg[2] * d2;
  s.tb = -s.T_final * s.bg_dot;
  s.accd = 0.f;
}

// LDS floats needed by vjp_tile's per-wave partial sums: [wave][value slot][batch element], rows padded
// to BATCH + 1 floats so the 8 lanes storing one element's 8 slots hit 8 different banks.
template <int BATCH>
constexpr int acc_stride() { return BATCH + 1; }
template <bool WITH_XY, bool WITH_INV, int BATCH>
constexpr int vjp_acc_floats() { return 4 * n_used<WITH_XY, WITH_INV>() * acc_stride<BATCH>(); }

// Back-to-front pass over the tile's list (upstream BACKWARD::renderCUDA semantics), writing one
// reduced row per (tile, Gaussian) pair.  Block-uniform control flow; requires blockDim = 256.
// slots != NULL (the LM row map): rows exist for head entries only -- those some wave still blending at their list
// position visits (a non-empty mask below) -- and the others are not written.
// s_rp: the batch's records as five float2 planes of BATCH entries ((x, y), (conic a, b), (conic c, opacity), (r, g),
// (b, 1/depth)): a visit reads entry j of each plane from ONE address (8 j) with plane offsets -- two
// ds_read2st64_b64 and a ds_read_b64, issued together -- where the float4 / float2 arrays needed two addresses of
// different scale and the float2 read waited behind the float4 pair.
template <bool WITH_XY, bool WITH_INV, int ROWF4, int BATCH>
__device__ __forceinline__ void vjp_tile(VjpPix& st, bool inside, float pxf, float pyf, int tile_x, int tile_y,
                                         uint2 range, const uint32_t* __restrict__ point_list,
                                         const float4* __restrict__ rec, const uint32_t* __restrict__ slots,
                                         const uint2* __restrict__ rect, const uint32_t* __restrict__ goff,
                                         float2* s_rp, uint64_t* s_bits, float* s_acc, int* s_misc,
                                         float4* __restrict__ rows, bool write_tail) {
  constexpr int NU = n_used<WITH_XY, WITH_INV>();
  constexpr int ACC_STRIDE = acc_stride<BATCH>();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // Positions >= max over pixels of n_contrib are never blended: their rows are zero.  The leading
  // barrier lets s_misc alias LDS the caller used before this pass (k_render_matvec's JVP buffers).
  __syncthreads();
  const int wmax = wave_max_u((int)st.last);
  if (lane == 0) s_misc[w] = wmax;
  __syncthreads();
  // per-wave bound: wave w's lanes blend nothing at list positions >= wm[w]
  const int wm0 = s_misc[0], wm1 = s_misc[1], wm2 = s_misc[2], wm3 = s_misc[3];
  const int n_eff = max(max(wm0, wm1), max(wm2, wm3));
  if (write_tail) {
    float z[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) z[q] = 0.f;
    for (int64_t k = (int64_t)range.x + n_eff + tid; k < (int64_t)range.y; k += TILE_PIX) {
      uint32_t slot;
      if (slots) {
        slot = slots[k];
      } else {
        const uint32_t g = pl_id(point_list[k]);
        slot = row_slot(goff[g], rect[g], tile_x, tile_y);
      }
      store_row<ROWF4>(rows, slot, z);
    }
  }
  const int rounds = (n_eff + BATCH - 1) / BATCH;
  for (int r = 0; r < rounds; ++r) {
    const int base = n_eff - 1 - r * BATCH;  // list position of batch element 0
    const int cnt = min(BATCH, base + 1);
    __syncthreads();
    uint32_t my_slot = 0;
    uint32_t my_mask = 0u;
    if (tid < cnt) {
      const uint32_t e = point_list[range.x + base - tid];
      const uint32_t g = pl_id(e);
      my_mask = pl_mask(e);
      const float4 r0 = rec[RECS * (int64_t)g + 0], r1 = rec[RECS * (int64_t)g + 1], r2 = rec[RECS * (int64_t)g + 2];
      s_rp[tid] = make_float2(r0.x, r0.y);
      s_rp[BATCH + tid] = make_float2(r0.z, r0.w);
      s_rp[2 * BATCH + tid] = make_float2(r1.x, r1.y);
      s_rp[3 * BATCH + tid] = make_float2(r1.z, r1.w);
      s_rp[4 * BATCH + tid] = make_float2(r2.x, r2.y);
      // and only the waves that still blend at this list position
      const int pos = base - tid;
      my_mask &= (pos < wm0 ? 1u : 0u) | (pos < wm1 ? 2u : 0u) | (pos < wm2 ? 4u : 0u) | (pos < wm3 ? 8u : 0u);
      // the row slot of an entry that gets a row (below): the LM row map, or the drop-in's rectangle slot
      if (my_mask || (!slots && write_tail))
        my_slot = slots ? slots[range.x + base - tid] : row_slot(goff[g], rect[g], tile_x, tile_y);
    }
    // which waves' quadrants this element can touch; wave w visits only its hits, and the combine below
    // takes zero for the others (exactly what a visit with no valid lane would have produced)
    publish_quad_masks(my_mask, s_bits);
    __syncthreads();
    // the batch's hit words in order, each walked by s_ff1 (HitIter's single loop cost ~5 more scalar instructions per
    // visit: the word switch, a sign test of the index and a branch through the iterator's exit)
#pragma unroll 1
    for (int wd = 0; wd < (BATCH + 63) / 64; ++wd) {
    uint64_t hits = wave_bits(s_bits, w, wd);
    while (hits) {
      const int hb = (int)__builtin_ctzll(hits);
      hits = clear_bit(hits, hb);
      const int j = 64 * wd + hb;
      const float2 p0 = s_rp[j], p1 = s_rp[BATCH + j], p2 = s_rp[2 * BATCH + j], p3 = s_rp[3 * BATCH + j];
      const float2 c = s_rp[4 * BATCH + j];
      const float4 a = make_float4(p0.x, p0.y, p1.x, p1.y), b = make_float4(p2.x, p2.y, p3.x, p3.y);
      // the whole record in one LDS round trip at the top of the iteration (the empty asm pins the loads
      // here; otherwise the colour half is fetched after the alpha test, a second exposed LDS latency;
      // prefetching the next hit's record instead measured 9% slower: it costs issue slots, not latency)
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(c.x), "v"(c.y));
      {
        const uint32_t contributor = (uint32_t)(base - j);  // 0-based list position
        const float dx = a.x - pxf, dy = a.y - pyf;
        const float power = gpower(a.z, a.w, b.x, dx, dy);
        const float G = gexp(power);
        const float alpha = fminf(0.99f, b.y * G);
        const bool c_last = contributor < st.last, c_pow = !(power > 0.0f), c_alpha = alpha >= 1.0f / 255.0f;
        const bool valid = c_last && c_pow && c_alpha;  // st.last = 0 outside the image
        // <colour, dL/dpix> for every lane (the colour is already in registers)
        float cd;
        {
#pragma clang fp contract(fast)
          cd = (b.z * st.dpix[0] + b.w * st.dpix[1]) + c.x * st.dpix[2];
          if (WITH_INV) cd += c.y * st.dinv;
        }
        // A visit some lane blends runs the body in every lane, an invalid lane with alpha = G = 0: its row
        // values are 0, T is unchanged (rcp(1) = 1) and its accumulation update adds 0 * (...).  No per-lane
        // branch and no zeroing of the row values per visit.
        // (per-condition ballots fold into their compares' lane masks: no VGPR round trip of `valid`)
        const bool any = (__builtin_amdgcn_ballot_w64(c_last) & __builtin_amdgcn_ballot_w64(c_pow) &
                          __builtin_amdgcn_ballot_w64(c_alpha)) != 0ull;
        float gv[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) gv[q] = 0.f;
        const float a_e = valid ? alpha : 0.f;
        const float G_e = valid ? G : 0.f;
        if (any) {
          // Only the primal tests above (power, alpha) must round exactly as the forward's; the
          // derivative arithmetic below decides nothing and is contracted to FMAs.
#pragma clang fp contract(fast)
          const float inv1ma = rcp_f(1.f - a_e);
          st.T = st.T * inv1ma;
          const float dchannel = a_e * st.T;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch) gv[6 + ch] = dchannel * st.dpix[ch];
          if (WITH_INV) gv[9] = dchannel * st.dinv;
          // dL/dalpha = (<c, u> - acc) T - T_final / (1 - alpha) <bg, u>   (tb = -T_final <bg, u>)
          const float cd_acc = cd - st.accd;
          const float dL_dalpha = cd_acc * st.T + st.tb * inv1ma;
          st.accd = st.accd + a_e * cd_acc;  // this Gaussian joins the accumulation behind the next one
          gv[5] = G_e * dL_dalpha;
          // h = G dL/dG = o gv5 with G = exp(power): dL/dpower = h; the conic rows carry gv5 dx^2, gv5 dx dy,
          // gv5 dy^2 and their factors o (-1/2, -1, -1/2) are applied once per row at the combine (the entry's
          // opacity o is the same at every pixel: one VALU less per visit)
          const float hdx = gv[5] * dx, hdy = gv[5] * dy;
          // the screen-position rows: the conic is the entry's, so dL/dx = -(A sum h dx + B sum h dy) and dL/dy =
          // -(C sum h dy + B sum h dx) are formed from the two sums once per row at the combine (not per lane)
          if (WITH_XY) {
            gv[0] = hdx;
            gv[1] = hdy;
          }
          gv[2] = hdx * dx;
          gv[3] = hdx * dy;
          gv[4] = hdy * dy;
        }
        if constexpr (NU <= 8) {
          // transposed reduction: value slot k ends in lanes 8k..8k+7; lane 8k stores it
          float rr = 0.f;
          if (any) {
            float pv[8];
#pragma unroll
            for (int q = 0; q < NV; ++q)
              if (q_used<WITH_XY, WITH_INV>(q)) pv[q_slot<WITH_XY, WITH_INV>(q)] = gv[q];
            // unused slots (7 with the LM rows) are never stored and never mix into a stored one (slot k + 4 stays in
            // the other half-wave through every step): any register will do -- a dead one (dy), which the permlane swap
            // may overwrite in place; an alias of a live slot cost a copy per visit
#pragma unroll
            for (int k = NU; k < 8; ++k) pv[k] = k == 7 ? dy : pv[k - 4];
            rr = wave_reduce8_t(pv, lane);
          }
          const int k = lane >> 3;
          if ((lane & 7) == 0 && k < NU) s_acc[(w * NU + k) * ACC_STRIDE + j] = rr;
        } else {
          // slots 0..7 by the transposed reduction, the 1-2 extra slots (drop-in: means2D, invdepth)
          // by lane-63 sums
          constexpr int NX = NU - 8;
          float rr = 0.f, ex[NX];
#pragma unroll
          for (int e = 0; e < NX; ++e) ex[e] = 0.f;
          if (any) {
            float pv[8];
#pragma unroll
            for (int q = 0; q < NV; ++q)
              if (q_used<WITH_XY, WITH_INV>(q)) {
                const int sq = q_slot<WITH_XY, WITH_INV>(q);
                if (sq < 8) pv[sq] = gv[q];
                else ex[sq - 8] = gv[q];
              }
            rr = wave_reduce8_t(pv, lane);
#pragma unroll
            for (int e = 0; e < NX; ++e) ex[e] = wave_sum_lane63(ex[e]);
          }
          if ((lane & 7) == 0) s_acc[(w * NU + (lane >> 3)) * ACC_STRIDE + j] = rr;
          if (lane == 63)
#pragma unroll
            for (int e = 0; e < NX; ++e) s_acc[(w * NU + 8 + e) * ACC_STRIDE + j] = ex[e];
        }
      }
    }
    }
    __syncthreads();
    // rows only for the entries some wave visited: the LM rows (slots) exist for head entries only (k_row_flags); the
    // drop-in's rectangle rows of every other entry are the zeros its caller filled the buffer with (write_tail = 0),
    // or were written by the tail loop above (write_tail)
    if (tid < cnt && (my_mask || (!slots && write_tail))) {
      float t[NV];
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        t[q] = 0.f;
        if (q_used<WITH_XY, WITH_INV>(q)) {
          const int sq = q_slot<WITH_XY, WITH_INV>(q);
          // every wave's slot read, the ones it never wrote (no hit) then dropped by a select: plain LDS loads and
          // v_cndmask instead of an exec-mask branch around each load
          const float a0 = s_acc[(0 * NU + sq) * ACC_STRIDE + tid], a1 = s_acc[(1 * NU + sq) * ACC_STRIDE + tid];
          const float a2 = s_acc[(2 * NU + sq) * ACC_STRIDE + tid], a3 = s_acc[(3 * NU + sq) * ACC_STRIDE + tid];
          const float p0 = (my_mask & 1u) ? a0 : 0.f;
          const float p1 = (my_mask & 2u) ? a1 : 0.f;
          const float p2 = (my_mask & 4u) ? a2 : 0.f;
          const float p3 = (my_mask & 8u) ? a3 : 0.f;
          t[q] = ((p0 + p1) + p2) + p3;
        }
      }
      // the conic rows' factors o (-1/2, -1, -1/2) (see the hit loop)
      const float op = s_rp[2 * BATCH + tid].y;
      t[2] *= -0.5f * op;
      t[3] *= -op;
      t[4] *= -0.5f * op;
      if (WITH_XY) {  // o sum gv5 dx, o sum gv5 dy -> dL/d(x, y) with the entry's conic (A, B, C)
#pragma clang fp contract(fast)
        const float cA = s_rp[BATCH + tid].x, cB = s_rp[BATCH + tid].y, cC = s_rp[2 * BATCH + tid].x, sx = op * t[0], sy = op * t[1];
        t[0] = -(cA * sx + cB * sy);
        t[1] = -(cC * sy + cB * sx);
      }
      store_row<ROWF4>(rows, my_slot, t);
    }
  }
}

}  // namespace gslm
