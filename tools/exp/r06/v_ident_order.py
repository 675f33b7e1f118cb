# variant: the forward's binning without k_tile_order -- the blend launches tiles in identity order, written by
# k_duplicate's grid-stride range zeroing (one single-block launch less per binning; the LM product's cost order and
# the union binning untouched)
s = open("forward.hip").read()
a = """__device__ __forceinline__ void zero_tile_ranges(uint2* __restrict__ ranges, int ntiles) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x)
    ranges[t] = make_uint2(0u, 0u);
}"""
assert a in s
s = s.replace(a, """__device__ __forceinline__ void zero_tile_ranges(uint2* __restrict__ ranges, int ntiles, uint32_t* order = nullptr) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
    ranges[t] = make_uint2(0u, 0u);
    if (order) order[t] = (uint32_t)t;
  }
}""")
a = """                                                    uint2* __restrict__ zero_ranges, int ntiles) {
  __shared__ QuadCull s_q[256];"""
assert a in s
s = s.replace(a, """                                                    uint2* __restrict__ zero_ranges, int ntiles,
                                                    uint32_t* __restrict__ ident_order) {
  __shared__ QuadCull s_q[256];""")
a = """  zero_tile_ranges(zero_ranges, ntiles);
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * 256, s = s0 + tid;
  const int64_t slast = min(s0 + 255, P - 1);"""
assert a in s, "dup body"
s = s.replace(a, """  zero_tile_ranges(zero_ranges, ntiles, ident_order);
  const int tid = threadIdx.x;
  const int64_t s0 = (int64_t)blockIdx.x * 256, s = s0 + tid;
  const int64_t slast = min(s0 + 255, P - 1);""")
a = """                       gb.offsets, (uint32_t)N, n_dev, gb.rect, gb.rec, bb.keys0, bb.vals0, bb.ranges, ntiles);"""
assert s.count(a) == 1
s = s.replace(a, """                       gb.offsets, (uint32_t)N, n_dev, gb.rect, gb.rec, bb.keys0, bb.vals0, bb.ranges, ntiles,
                       bb.tile_order);""")
a = """  hipLaunchKernelGGL(k_ranges, dim3(nbN), dim3(256), 0, s, N, bb.keys_sorted, bb.ranges, n_dev, n_out);
  GSLM_LAUNCH_CHECK();
  if (int st = launch_tile_order(ntiles, bb.ranges, bb.tile_order, nullptr, s)) return st;
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;"""
assert a in s
s = s.replace(a, """  hipLaunchKernelGGL(k_ranges, dim3(nbN), dim3(256), 0, s, N, bb.keys_sorted, bb.ranges, n_dev, n_out);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;""")
open("forward.hip", "w").write(s)
