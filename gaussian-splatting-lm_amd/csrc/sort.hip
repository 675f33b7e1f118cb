// sort.hip -- stable LSD radix sort of (u32 key, u32 value) pairs and an exclusive u32 scan.
//
// Replaces cub::DeviceRadixSort::SortPairs / cub::DeviceScan::InclusiveSum of the upstream
// rasterizer_impl (SURVEY §2 kernel table).  Written for wave64: the stable in-block ranking uses
// 8 wave ballots per digit (a "match" of equal digits), per-wave digit counts in LDS and a
// 4-wave prefix, so every block scatters its 4096 keys in input order (stability is what keeps
// depth ties in Gaussian-index order).
//
// Per pass: hist (read keys) -> per-digit scan over blocks -> scatter (read keys+vals, write both).
#include "gslm_internal.hpp"

namespace gslm {

namespace {

// Orders a wave's LDS stores before its later loads of other lanes' slots: a wave's LDS operations complete in
// order, so this costs no instruction; it only stops the compiler from moving them across (as wave_lds_sync in
// gslm_tile.hpp).
__device__ __forceinline__ void wave_order_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// Block-wide inclusive scan for 256 threads.  Returns inclusive value; *total = block sum.
__device__ __forceinline__ uint32_t block_incl_scan256(uint32_t x, uint32_t* s_w, uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t inc = wave_incl_scan(x, lane);
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v = s_w[k];
    if (k < w) off += v;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return inc + off;
}

// The exclusive prefix of the first b of a scan's per-block sums (written raw by the reduce pass), summed by the
// block's threads (b <= SCAN_INLINE_MAX_BLOCKS: L2-resident loads).  In the apply pass this replaces the
// scan-of-block-sums launch between the two passes (a single-block kernel at its ~5 us floor, twice per forward).
// The loads grow as nb^2 / 2 over the grid, so longer scans (the LM row map over N pairs at 5M Gaussians or 4K frames:
// nb ~ 12k-49k) scan the block sums in a launch of their own (k_scan_top, SCANNED = true) and read their prefix.
template <bool SCANNED>
__device__ __forceinline__ uint32_t block_sums_before(const uint32_t* __restrict__ bs, int b, uint32_t* s_w) {
  if (SCANNED) return bs[b];
  const uint32_t acc = strided_sum_in_order(bs, b);  // loads 8 deep
  uint32_t tot;
  block_incl_scan256(acc, s_w, &tot);
  return tot;
}

// One block per sequence of nb block sums (bs + blockIdx.x * nb): in-place exclusive scan, chunks of 8 x 256 loaded
// together (as k_radix_scan).
__global__ __launch_bounds__(256) void k_scan_top(uint32_t* __restrict__ bs, int nb) {
  __shared__ uint32_t s_w[4];
  uint32_t* h = bs + (int64_t)blockIdx.x * nb;
  const int tid = threadIdx.x;
  uint32_t carry = 0;
  for (int base0 = 0; base0 < nb; base0 += 8 * 256) {
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = base0 + k * 256 + tid;
      x[k] = i < nb ? h[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int base = base0 + k * 256;
      if (base >= nb) break;  // block-uniform
      const int i = base + tid;
      uint32_t tot;
      const uint32_t inc = block_incl_scan256(x[k], s_w, &tot);
      if (i < nb) h[i] = carry + inc - x[k];
      carry += tot;
    }
  }
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor(x, o, 64));
  return x;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor(x, o, 64));
  return x;
}

// The depth sort's key range (radix_sort_pairs(..., key_range = true); VERDICT r05 item 2: sort only the bits the
// frame's depths use).  Pass 0 sorts the low byte of key - kmin, which is the raw low byte rotated by kmin's: its
// histogram kernel counts raw digits and records each block's (min, max) over the keys other than 0xFFFFFFFF (the
// Gaussians behind the near plane), and block 0 of its scan reduces those into w: kmin, the sort value t of the
// 0xFFFFFFFF keys (the least value past max - kmin whose low byte is (0xFF - kmin) mod 256, so pass 0's rotation
// holds for them too) and the working pass count (the bytes of t).  Later passes sort the bytes of
// key' = key - kmin (t for 0xFFFFFFFF), monotone in key with the 0xFFFFFFFF keys last: the stable order is the
// 32-bit sort's.  Past the working passes every key' byte is 0 and the pass is the identity: the histogram and scan
// kernels return at once and the scatter copies (same ping-pong parity, the last pass's gather kept).
struct KeyRange {
  uint32_t* w;   // [0] kmin, [1] t, [2] working passes
  uint2* blk;    // [blocks] (min, max) of each pass-0 histogram block's keys other than 0xFFFFFFFF
  int pass;
};
__device__ __forceinline__ uint32_t range_key(uint32_t k, uint32_t kmin, uint32_t t) {
  return k == 0xFFFFFFFFu ? t : k - kmin;
}

// n_dev (or NULL): the key count is min(n, *n_dev), read on the device (a capacity-sized launch whose count the host
// has not read back: gslm_rasterize_dev); blocks past it count nothing
template <int ITEMS, bool RANGE = false>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_hist(const uint32_t* __restrict__ keys, int64_t n,
                                                             int shift, uint32_t dmask, uint32_t* __restrict__ hist,
                                                             int nblocks, const uint32_t* __restrict__ n_dev,
                                                             KeyRange kr = KeyRange{}) {
  __shared__ uint32_t cnt[RADIX];
  __shared__ uint32_t s_mm[2][4];
  const int tid = threadIdx.x;
  uint32_t kmin = 0u, t = 0u;
  if (RANGE && kr.pass > 0) {
    if (kr.pass >= (int)kr.w[2]) return;  // past the span (block-uniform)
    kmin = kr.w[0];
    t = kr.w[1];
  }
  if (n_dev) n = min(n, (int64_t)*n_dev);
  cnt[tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * (SORT_THREADS * ITEMS);
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll 4
  for (int r = 0; r < ITEMS; ++r) {
    const int64_t i = base + r * SORT_THREADS + tid;
    if (i < n) {
      const uint32_t k = keys[i];
      if (RANGE && kr.pass == 0 && k != 0xFFFFFFFFu) {
        lo = min(lo, k);
        hi = max(hi, k);
      }
      const uint32_t kk = (RANGE && kr.pass > 0) ? range_key(k, kmin, t) : k;  // pass 0: the raw digit
      atomicAdd(&cnt[(kk >> shift) & dmask], 1u);
    }
  }
  if (RANGE && kr.pass == 0) {
    lo = wave_min_u32(lo);
    hi = wave_max_u32(hi);
    if ((tid & 63) == 0) {
      s_mm[0][tid >> 6] = lo;
      s_mm[1][tid >> 6] = hi;
    }
  }
  __syncthreads();
  hist[(int64_t)tid * nblocks + blockIdx.x] = cnt[tid];
  if (RANGE && kr.pass == 0 && tid == 0)
    kr.blk[blockIdx.x] = make_uint2(min(min(s_mm[0][0], s_mm[0][1]), min(s_mm[0][2], s_mm[0][3])),
                                    max(max(s_mm[1][0], s_mm[1][1]), max(s_mm[1][2], s_mm[1][3])));
}

// One block per digit: exclusive scan of that digit's per-block counts; digit total -> totals[d].
// RANGE, pass 0: block 0 first reduces the histogram blocks' key ranges into kr.w (KeyRange).
template <bool RANGE = false>
__global__ __launch_bounds__(256) void k_radix_scan(uint32_t* __restrict__ hist, int nblocks,
                                                    uint32_t* __restrict__ totals, KeyRange kr = KeyRange{}) {
  __shared__ uint32_t s_w[4];
  const int d = blockIdx.x, tid = threadIdx.x;
  if (RANGE && kr.pass > 0 && kr.pass >= (int)kr.w[2]) return;
  if (RANGE && kr.pass == 0 && d == 0) {
    __shared__ uint32_t s_mm[2][4];
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    for (int b = tid; b < nblocks; b += 256) {
      const uint2 m = kr.blk[b];
      lo = min(lo, m.x);
      hi = max(hi, m.y);
    }
    lo = wave_min_u32(lo);
    hi = wave_max_u32(hi);
    if ((tid & 63) == 0) {
      s_mm[0][tid >> 6] = lo;
      s_mm[1][tid >> 6] = hi;
    }
    __syncthreads();
    if (tid == 0) {
      lo = min(min(s_mm[0][0], s_mm[0][1]), min(s_mm[0][2], s_mm[0][3]));
      hi = max(max(s_mm[1][0], s_mm[1][1]), max(s_mm[1][2], s_mm[1][3]));
      uint32_t kmin = 0u, t = 0xFFu;  // no key other than 0xFFFFFFFF: one digit value, one pass
      if (lo <= hi) {
        kmin = lo;
        const uint32_t r1 = hi - kmin + 1u;              // past every other key's key'
        const uint32_t lowb = (0xFFu - kmin) & 0xFFu;    // (0xFFFFFFFF - kmin) mod 256
        t = r1 + ((lowb - r1) & 0xFFu);                  // <= 0xFFFFFFFF - kmin: no wrap
      }
      const int bits = 32 - __clz((int)t);
      kr.w[0] = kmin;
      kr.w[1] = t;
      kr.w[2] = (uint32_t)max(1, (bits + 7) / 8);
    }
  }
  uint32_t* h = hist + (int64_t)d * nblocks;
  uint32_t carry = 0;
  // up to 8 chunks of 256 counts loaded together (the tile sort's ~1200 blocks: 5 chunks, one load latency instead of
  // five), then scanned chunk by chunk; each count is read before its own slot is rewritten
  for (int base0 = 0; base0 < nblocks; base0 += 8 * 256) {
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = base0 + k * 256 + tid;
      x[k] = i < nblocks ? h[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int base = base0 + k * 256;
      if (base >= nblocks) break;  // block-uniform
      const int i = base + tid;
      uint32_t tot;
      const uint32_t inc = block_incl_scan256(x[k], s_w, &tot);
      if (i < nblocks) h[i] = carry + inc - x[k];
      carry += tot;
    }
  }
  if (tid == 0) totals[d] = carry;
}

// Scatter of one pass.  Each wave ranks a contiguous quarter of the block's 4096 keys on its own (16 rounds of
// 64 consecutive keys): a digit "match" from nbits wave ballots gives the key's rank among equal digits of the
// round, and a wave-private LDS counter per digit carries the wave's running count across rounds (LDS accesses
// of one wave are ordered, so no barrier inside the loop).  One block-wide prefix then turns the four waves'
// counts into local positions: block order = wave order, round order, lane order = input order (stable).  The
// keys are reordered through LDS into digit runs and each run is written to its global offset by consecutive
// threads (coalesced segments instead of one scattered 4-byte store per key).
// PAY: a second value array moves with the pairs (pin -> pout; the line search's union list carries each entry's
// per-set quadrant masks through the tile sort, gslm_union_binning).
// RANGE: the digits of key' (KeyRange; pass 0 the low byte of key - kmin, i.e. digit run d' holds raw digit
// (d' + kmin) mod 256's counts); past the working passes a plain copy.
template <int ITEMS, bool PAY = false, bool RANGE = false>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout, int64_t n, int shift, int nbits, const uint32_t* __restrict__ hist, int nblocks,
    const uint32_t* __restrict__ totals, const uint32_t* __restrict__ kgather, const uint32_t* __restrict__ n_dev,
    const uint32_t* __restrict__ pin = nullptr, uint32_t* __restrict__ pout = nullptr, KeyRange kr = KeyRange{}) {
  static_assert(SORT_THREADS == 256 && RADIX == 256, "one digit per thread, four waves");
  constexpr int TILE = SORT_THREADS * ITEMS;
  constexpr int WAVE_KEYS = TILE / 4;
  __shared__ uint32_t s_keys[TILE], s_vals[TILE];
  __shared__ uint32_t s_pay[PAY ? TILE : 1];
  __shared__ uint32_t s_wcnt[4][RADIX];  // per-wave running digit count, then the wave's offset in the digit run
  __shared__ uint32_t s_loc[RADIX];      // block-local start of each digit's run
  __shared__ uint32_t s_gbase[RADIX];    // global offset of this block's run of each digit
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (n_dev) n = min(n, (int64_t)*n_dev);  // as k_radix_hist; a block past the count moves nothing (nvalid <= 0)
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const int nvalid = (int)max<int64_t>(-1, min<int64_t>(TILE, n - base));
  const int wbase = w * WAVE_KEYS;
  const uint32_t dmask = (1u << nbits) - 1u;
  uint32_t kmin = 0u, kt = 0u, rot = 0u;
  if (RANGE) {
    kmin = kr.w[0];
    kt = kr.w[1];
    if (kr.pass >= (int)kr.w[2]) {  // past the span: the identity pass (block-uniform)
      for (int e = tid; e < TILE; e += SORT_THREADS) {
        const int64_t i = base + e;
        if (i < n) {
          const uint32_t val = vin ? vin[i] : (uint32_t)i;
          kout[i] = kgather ? kgather[val] : kin[i];
          vout[i] = val;
        }
      }
      return;
    }
    if (kr.pass == 0) rot = kmin & 0xFFu;
  }
  // this pass's digit of a key
  auto digit = [&](uint32_t k) -> uint32_t {
    if (!RANGE) return (k >> shift) & dmask;
    if (kr.pass == 0) return (k - kmin) & dmask;  // == key' & dmask, the 0xFFFFFFFF keys included (t's low byte)
    return (range_key(k, kmin, kt) >> shift) & dmask;
  };

#pragma unroll
  for (int k = 0; k < 4; ++k) s_wcnt[w][lane + 64 * k] = 0u;
  wave_order_lds();  // the zeroes before any lane's first counter read
  // all loads first (16 keys + 16 values per lane in flight), wave w on keys [wbase, wbase + 1024) of the block
  uint32_t key[ITEMS], val[ITEMS], lrank[ITEMS];
  uint32_t pay[PAY ? ITEMS : 1];
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const int64_t i = base + wbase + r * 64 + lane;
    key[r] = i < n ? kin[i] : 0u;
    val[r] = i < n ? (vin ? vin[i] : (uint32_t)i) : 0u;  // vin == NULL: the values are the indices
    if (PAY) pay[r] = i < n ? pin[i] : 0u;
  }
  {
    // global base of each digit's run for this block = exclusive prefix of digit totals + this block's offset
    const uint32_t draw = (tid + rot) & 0xFFu;  // the raw digit whose counts digit run tid holds (rot 0: itself)
    const uint32_t t = totals[draw];
    uint32_t tot;
    const uint32_t inc = block_incl_scan256(t, s_w, &tot);
    s_gbase[tid] = inc - t + hist[(int64_t)draw * nblocks + blockIdx.x];
  }
  // 1. wave-local stable rank of every key among equal digits
  const unsigned long long lt_mask = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    const bool valid = wbase + r * 64 + lane < nvalid;
    const uint32_t d = digit(key[r]);
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (b >= nbits) break;
      const bool bit = (d >> b) & 1u;
      const unsigned long long bb = __ballot(bit);
      m &= bit ? bb : ~bb;
    }
    const uint32_t rank = __popcll(m & lt_mask);
    const uint32_t cnt = s_wcnt[w][d];
    lrank[r] = cnt + rank;
    if (valid && rank == 0) s_wcnt[w][d] = cnt + (uint32_t)__popcll(m);
    wave_order_lds();  // this round's counter updates before the next round's reads by other lanes
  }
  __syncthreads();
  // 2. the four waves' offsets inside each digit's run, and each run's block-local start
  {
    const uint32_t c0 = s_wcnt[0][tid], c1 = s_wcnt[1][tid], c2 = s_wcnt[2][tid], c3 = s_wcnt[3][tid];
    const uint32_t c = c0 + c1 + c2 + c3;
    s_wcnt[0][tid] = 0u;
    s_wcnt[1][tid] = c0;
    s_wcnt[2][tid] = c0 + c1;
    s_wcnt[3][tid] = c0 + c1 + c2;
    uint32_t tot;
    const uint32_t inc = block_incl_scan256(c, s_w, &tot);
    s_loc[tid] = inc - c;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < ITEMS; ++r) {
    if (wbase + r * 64 + lane < nvalid) {
      const uint32_t d = digit(key[r]);
      const uint32_t lp = s_loc[d] + s_wcnt[w][d] + lrank[r];
      s_keys[lp] = key[r];
      s_vals[lp] = val[r];
      if (PAY) s_pay[lp] = pay[r];
    }
  }
  __syncthreads();
  // 3. each run to its global offset, consecutive threads on consecutive elements
  for (int e = tid; e < nvalid; e += SORT_THREADS) {
    const uint32_t k = s_keys[e];
    const uint32_t d = digit(k);
    const uint32_t pos = s_gbase[d] + ((uint32_t)e - s_loc[d]);
    const uint32_t val = s_vals[e];
    // kgather (the last pass of the depth sort): the sorted keys are not needed afterwards, so their slot carries
    // kgather[value] in sorted order instead (the tile counts the depth-order scan reads, gathered once here)
    kout[pos] = kgather ? kgather[val] : k;
    vout[pos] = val;
    if (PAY) pout[pos] = s_pay[e];
  }
}

// ---------------- scan ----------------
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_reduce(const uint32_t* __restrict__ in,
                                                              const uint32_t* __restrict__ idx, int64_t n,
                                                              uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) acc += in[idx ? idx[i] : i];
  }
  uint32_t tot;
  block_incl_scan256(acc, s_w, &tot);
  if (tid == 0) block_sums[blockIdx.x] = tot;
}

// In-place form of k_scan_apply (data = in = out, no index gather): one pointer without __restrict__, so the
// compiler keeps every thread's loads of its elements ahead of its stores to them.
template <bool SCANNED>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_apply_inplace(uint32_t* data, int64_t n,
                                                                     const uint32_t* __restrict__ block_sums,
                                                                     uint32_t* __restrict__ total) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
  const uint32_t before = block_sums_before<SCANNED>(block_sums, blockIdx.x, s_w);
  uint32_t v[SCAN_ITEMS];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    v[k] = i < n ? data[i] : 0u;
    acc += v[k];
  }
  uint32_t tot;
  const uint32_t inc = block_incl_scan256(acc, s_w, &tot);
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *total = before + tot;
  uint32_t run = before + inc - acc;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) data[i] = run;
    run += v[k];
  }
}

template <bool SCANNED>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_apply(const uint32_t* __restrict__ in,
                                                             const uint32_t* __restrict__ idx, int64_t n,
                                                             const uint32_t* __restrict__ block_sums,
                                                             uint32_t* __restrict__ out, uint32_t* __restrict__ total) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
  const uint32_t before = block_sums_before<SCANNED>(block_sums, blockIdx.x, s_w);
  uint32_t v[SCAN_ITEMS];
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    v[k] = i < n ? in[idx ? idx[i] : i] : 0u;
    acc += v[k];
  }
  uint32_t tot;
  const uint32_t inc = block_incl_scan256(acc, s_w, &tot);
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *total = before + tot;
  uint32_t run = before + inc - acc;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
}

// Two exclusive scans of the same counts in one pass: in index order (out_a) and gathered through idx
// (out_b).  block_sums holds 2 nb partials: [0, nb) for a, [nb, 2 nb) for b.
// in_b (or NULL: in gathered through idx) is the second sequence
__global__ __launch_bounds__(SCAN_THREADS) void k_scan2_reduce(const uint32_t* __restrict__ in,
                                                               const uint32_t* __restrict__ idx,
                                                               const uint32_t* __restrict__ in_b, int64_t n,
                                                               uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
  uint32_t acc_a = 0, acc_b = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) {
      acc_a += in[i];
      acc_b += in_b ? in_b[i] : in[idx[i]];
    }
  }
  uint32_t tot_a, tot_b;
  block_incl_scan256(acc_a, s_w, &tot_a);
  block_incl_scan256(acc_b, s_w, &tot_b);
  if (tid == 0) {
    block_sums[blockIdx.x] = tot_a;
    block_sums[gridDim.x + blockIdx.x] = tot_b;
  }
}

template <bool SCANNED>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan2_apply(const uint32_t* __restrict__ in,
                                                              const uint32_t* __restrict__ idx,
                                                              const uint32_t* __restrict__ in_b, int64_t n,
                                                              const uint32_t* __restrict__ block_sums,
                                                              uint32_t* __restrict__ out_a, uint32_t* __restrict__ out_b,
                                                              uint32_t* __restrict__ total_a,
                                                              uint32_t* __restrict__ total_b) {
  __shared__ uint32_t s_w[4];
  const int tid = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
  const uint32_t before_a = block_sums_before<SCANNED>(block_sums, blockIdx.x, s_w);
  const uint32_t before_b = block_sums_before<SCANNED>(block_sums + gridDim.x, blockIdx.x, s_w);
  uint32_t va[SCAN_ITEMS], vb[SCAN_ITEMS];
  uint32_t acc_a = 0, acc_b = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    va[k] = i < n ? in[i] : 0u;
    vb[k] = i < n ? (in_b ? in_b[i] : in[idx[i]]) : 0u;
    acc_a += va[k];
    acc_b += vb[k];
  }
  uint32_t tot_a, tot_b;
  const uint32_t inc_a = block_incl_scan256(acc_a, s_w, &tot_a);
  const uint32_t inc_b = block_incl_scan256(acc_b, s_w, &tot_b);
  if (blockIdx.x == gridDim.x - 1 && tid == 0) {
    *total_a = before_a + tot_a;
    *total_b = before_b + tot_b;
  }
  uint32_t ra = before_a + inc_a - acc_a;
  uint32_t rb = before_b + inc_b - acc_b;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) {
      out_a[i] = ra;
      out_b[i] = rb;
    }
    ra += va[k];
    rb += vb[k];
  }
}

}  // namespace

int exclusive_scan_u32_dual(const uint32_t* in, const uint32_t* idx, uint32_t* out_a, uint32_t* out_b, int64_t n,
                            uint32_t* tmp, uint32_t* total_a, uint32_t* total_b, hipStream_t s, const uint32_t* in_b) {
  if (n <= 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(total_a, 0, 4, s));
    GSLM_HIP_CHECK(hipMemsetAsync(total_b, 0, 4, s));
    return GSLM_OK;
  }
  const int nb = (int)scan_blocks(n);
  hipLaunchKernelGGL(k_scan2_reduce, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, in_b, n, tmp);
  if (nb > SCAN_INLINE_MAX_BLOCKS) {
    hipLaunchKernelGGL(k_scan_top, dim3(2), dim3(256), 0, s, tmp, nb);
    hipLaunchKernelGGL(k_scan2_apply<true>, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, in_b, n, tmp, out_a, out_b,
                       total_a, total_b);
  } else {
    hipLaunchKernelGGL(k_scan2_apply<false>, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, in_b, n, tmp, out_a, out_b,
                       total_a, total_b);
  }
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

// one pass of a key_range sort (KeyRange)
template <int ITEMS>
static void launch_range_pass(const uint32_t* ki, const uint32_t* vin, uint32_t* ko, uint32_t* vo, int64_t n, int shift,
                              int nbits, uint32_t dmask, uint32_t* hist, int nb, uint32_t* totals, const uint32_t* kg,
                              KeyRange kr, hipStream_t s) {
  hipLaunchKernelGGL((k_radix_hist<ITEMS, true>), dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb,
                     (const uint32_t*)nullptr, kr);
  hipLaunchKernelGGL(k_radix_scan<true>, dim3(RADIX), dim3(256), 0, s, hist, nb, totals, kr);
  hipLaunchKernelGGL((k_radix_scatter<ITEMS, false, true>), dim3(nb), dim3(SORT_THREADS), 0, s, ki, vin, ko, vo, n, shift,
                     nbits, hist, nb, totals, kg, (const uint32_t*)nullptr, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                     kr);
}

int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int64_t n, int end_bit,
                     uint32_t* hist, bool* result_in_alt, hipStream_t s, bool iota_values, const uint32_t* last_gather,
                     const uint32_t* n_dev, uint32_t* p0, uint32_t* p1, bool key_range) {
  *result_in_alt = false;
  if (n <= 0) return GSLM_OK;
  const bool pay = p0 != nullptr;
  if (key_range && (pay || n_dev || end_bit != 32)) {
    set_error("radix_sort_pairs: key_range needs 32-bit keys, no payload, a host-known count");
    return GSLM_ERR_INVALID;
  }
  const int nb = (int)sort_blocks(n, pay);
  const bool small = sort_items(n, pay) != SORT_ITEMS;
  uint32_t* totals = hist + (size_t)RADIX * nb;
  KeyRange kr{};
  if (key_range) {
    kr.w = totals + RADIX;
    kr.blk = reinterpret_cast<uint2*>(kr.w + 4);
  }
  uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1, *pi = p0, *po = p1;
  bool first = true;  // iota_values: the first scatter generates value = index instead of reading v0
  bool alt = false;
  // ceil(end_bit / 8) passes with the bits split evenly (13-bit tile ids: 7 + 6, not 8 + 5): fewer, longer
  // digit runs per block in the scatter (coalesced writes) for the same pass count
  const int passes = (end_bit + 7) / 8;
  const int per = (end_bit + passes - 1) / passes;
  for (int shift = 0; shift < end_bit; shift += per) {
    const int nbits = end_bit - shift < per ? end_bit - shift : per;  // digit bits of this pass
    const uint32_t dmask = (1u << nbits) - 1u;
    const uint32_t* vin = (first && iota_values) ? (const uint32_t*)nullptr : vi;
    const uint32_t* kg = (shift + per >= end_bit) ? last_gather : nullptr;  // the last pass
    if (key_range) {
      if (small) launch_range_pass<SORT_ITEMS_SMALL>(ki, vin, ko, vo, n, shift, nbits, dmask, hist, nb, totals, kg, kr, s);
      else launch_range_pass<SORT_ITEMS>(ki, vin, ko, vo, n, shift, nbits, dmask, hist, nb, totals, kg, kr, s);
      ++kr.pass;
    } else if (small) {
      hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS_SMALL>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb,
                         n_dev);
      hipLaunchKernelGGL(k_radix_scan<false>, dim3(RADIX), dim3(256), 0, s, hist, nb, totals, KeyRange{});
      if (pay)
        hipLaunchKernelGGL((k_radix_scatter<SORT_ITEMS_SMALL, true>), dim3(nb), dim3(SORT_THREADS), 0, s, ki, vin, ko, vo,
                           n, shift, nbits, hist, nb, totals, kg, n_dev, (const uint32_t*)pi, po);
      else
        hipLaunchKernelGGL((k_radix_scatter<SORT_ITEMS_SMALL, false>), dim3(nb), dim3(SORT_THREADS), 0, s, ki, vin, ko,
                           vo, n, shift, nbits, hist, nb, totals, kg, n_dev, (const uint32_t*)nullptr, (uint32_t*)nullptr);
    } else {
      hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb, n_dev);
      hipLaunchKernelGGL(k_radix_scan<false>, dim3(RADIX), dim3(256), 0, s, hist, nb, totals, KeyRange{});
      hipLaunchKernelGGL((k_radix_scatter<SORT_ITEMS, false>), dim3(nb), dim3(SORT_THREADS), 0, s, ki, vin, ko, vo, n,
                         shift, nbits, hist, nb, totals, kg, n_dev, (const uint32_t*)nullptr, (uint32_t*)nullptr);
    }
    first = false;
    GSLM_LAUNCH_CHECK();
    std::swap(ki, ko);
    std::swap(vi, vo);
    std::swap(pi, po);
    alt = !alt;
  }
  *result_in_alt = alt;
  return GSLM_OK;
}

int exclusive_scan_u32(const uint32_t* in, const uint32_t* idx, uint32_t* out, int64_t n, uint32_t* tmp,
                       uint32_t* total, hipStream_t s, int64_t inline_max_blocks) {
  if (n <= 0) {
    GSLM_HIP_CHECK(hipMemsetAsync(total, 0, 4, s));
    return GSLM_OK;
  }
  const int nb = (int)scan_blocks(n);
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, n, tmp);
  const bool top = nb > inline_max_blocks;
  if (top) hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, tmp, nb);
  if (out == in && !idx) {  // in place (the LM row map's head-flag scan)
    if (top) hipLaunchKernelGGL(k_scan_apply_inplace<true>, dim3(nb), dim3(SCAN_THREADS), 0, s, out, n, tmp, total);
    else hipLaunchKernelGGL(k_scan_apply_inplace<false>, dim3(nb), dim3(SCAN_THREADS), 0, s, out, n, tmp, total);
  } else {
    if (top) hipLaunchKernelGGL(k_scan_apply<true>, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, n, tmp, out, total);
    else hipLaunchKernelGGL(k_scan_apply<false>, dim3(nb), dim3(SCAN_THREADS), 0, s, in, idx, n, tmp, out, total);
  }
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}

}  // namespace gslm
