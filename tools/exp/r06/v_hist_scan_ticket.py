# variant (round 6, VERDICT r05 item 2's proposal): each radix pass's per-digit scan over blocks folded into its
# histogram kernel -- every block publishes its counts (device-scope release) and takes a ticket; the last 256 blocks to
# arrive wait for the others and scan one digit each (as k_radix_scan's 256 blocks do), so the pass loses its scan
# launch.  Per-pass tickets in 4 extra words of the histogram buffer, zeroed by one memset per sort.  Bounded waits.
s = open("gslm_internal.hpp").read()
a = "  return (size_t)RADIX * (size_t)sort_blocks(n, payload) * 4 + 4 * RADIX;"
assert a in s
s = s.replace(a, "  return (size_t)RADIX * (size_t)sort_blocks(n, payload) * 4 + 4 * RADIX + 16;")
open("gslm_internal.hpp", "w").write(s)

s = open("sort.hip").read()
k = r'''
#ifndef GSLM_TICKET_SPIN_MAX
#define GSLM_TICKET_SPIN_MAX (1 << 22)
#endif
template <int ITEMS>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_hist_scan(const uint32_t* __restrict__ keys, int64_t n,
                                                                  int shift, uint32_t dmask, uint32_t* __restrict__ hist,
                                                                  int nblocks, const uint32_t* __restrict__ n_dev,
                                                                  uint32_t* __restrict__ totals, uint32_t* ctr) {
  __shared__ uint32_t cnt[RADIX];
  __shared__ uint32_t s_w[4];
  __shared__ int s_ticket;
  const int tid = threadIdx.x;
  if (n_dev) n = min(n, (int64_t)*n_dev);
  cnt[tid] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * (SORT_THREADS * ITEMS);
#pragma unroll 4
  for (int r = 0; r < ITEMS; ++r) {
    const int64_t i = base + r * SORT_THREADS + tid;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & dmask], 1u);
  }
  __syncthreads();
  hist[(int64_t)tid * nblocks + blockIdx.x] = cnt[tid];
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    s_ticket = (int)atomicAdd(ctr, 1u);
  }
  __syncthreads();
  const int first = nblocks - RADIX;  // the host launches this form only with nblocks >= RADIX
  if (s_ticket < first) return;
  const int d = s_ticket - first;
  if (tid == 0) {
    for (int it = 0; it < GSLM_TICKET_SPIN_MAX; ++it) {
      if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)nblocks) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __threadfence();
  uint32_t* h = hist + (int64_t)d * nblocks;
  uint32_t carry = 0;
  for (int base0 = 0; base0 < nblocks; base0 += 8 * 256) {
    uint32_t x[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int i = base0 + kk * 256 + tid;
      x[kk] = i < nblocks ? __hip_atomic_load(h + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int bb = base0 + kk * 256;
      if (bb >= nblocks) break;
      const int i = bb + tid;
      uint32_t tot;
      const uint32_t inc = block_incl_scan256(x[kk], s_w, &tot);
      if (i < nblocks) h[i] = carry + inc - x[kk];
      carry += tot;
    }
  }
  if (tid == 0) totals[d] = carry;
}
'''
marker = "// Scatter of one pass."
assert marker in s
s = s.replace(marker, k + "\n" + marker, 1)

a = """  const bool small = sort_items(n, pay) != SORT_ITEMS;
  uint32_t* totals = hist + (size_t)RADIX * nb;"""
assert a in s
s = s.replace(a, """  const bool small = sort_items(n, pay) != SORT_ITEMS;
  uint32_t* totals = hist + (size_t)RADIX * nb;
  uint32_t* tickets = totals + RADIX;  // one per pass
  const bool fused = nb >= RADIX;
  if (fused) GSLM_HIP_CHECK(hipMemsetAsync(tickets, 0, 16, s));
  int pass = 0;""")
a = """      hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS_SMALL>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb,
                         n_dev);
      hipLaunchKernelGGL(k_radix_scan, dim3(RADIX), dim3(256), 0, s, hist, nb, totals);"""
assert a in s
s = s.replace(a, """      if (fused) {
        hipLaunchKernelGGL(k_radix_hist_scan<SORT_ITEMS_SMALL>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask,
                           hist, nb, n_dev, totals, tickets + pass);
      } else {
        hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS_SMALL>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist,
                           nb, n_dev);
        hipLaunchKernelGGL(k_radix_scan, dim3(RADIX), dim3(256), 0, s, hist, nb, totals);
      }""")
a = """      hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb, n_dev);
      hipLaunchKernelGGL(k_radix_scan, dim3(RADIX), dim3(256), 0, s, hist, nb, totals);"""
assert a in s
s = s.replace(a, """      if (fused) {
        hipLaunchKernelGGL(k_radix_hist_scan<SORT_ITEMS>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist,
                           nb, n_dev, totals, tickets + pass);
      } else {
        hipLaunchKernelGGL(k_radix_hist<SORT_ITEMS>, dim3(nb), dim3(SORT_THREADS), 0, s, ki, n, shift, dmask, hist, nb,
                           n_dev);
        hipLaunchKernelGGL(k_radix_scan, dim3(RADIX), dim3(256), 0, s, hist, nb, totals);
      }""")
a = """    first = false;
    GSLM_LAUNCH_CHECK();"""
assert a in s
s = s.replace(a, """    first = false;
    ++pass;
    GSLM_LAUNCH_CHECK();""")
open("sort.hip", "w").write(s)
