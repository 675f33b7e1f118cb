# variant: the forward blend (FWD_FULL / FWD_NO_INV) as one 64-thread block per (tile, quadrant) instead of one
# 256-thread block per tile -- its waves never meet at a barrier, so each retires on its own and the dispatcher can
# refill a single wave slot (the loss mode keeps its block reduction and 256-thread blocks)
s = open("render_fwd.hip").read()
a = """template <int MODE, bool SLOT = false>
__global__ __launch_bounds__(256) void k_render_fwd_wave(ViewK v, const uint2* __restrict__ ranges,"""
assert a in s
s = s.replace(a, """template <int MODE, bool SLOT = false>
__global__ __launch_bounds__(MODE == 2 ? 256 : 64) void k_render_fwd_wave(ViewK v, const uint2* __restrict__ ranges,""")
a = """  __shared__ float4 s_rec[4][3 * 64];
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

  // A stopped lane"""
assert a in s
s = s.replace(a, """  constexpr bool WB = MODE != FWD_LOSS;  // one wave per block
  __shared__ float4 s_rec[WB ? 1 : 4][3 * 64];
  const int tile = (int)tile_order[WB ? (blockIdx.x >> 2) : blockIdx.x];
  const int tile_x = tile % v.gx, tile_y = tile / v.gx;
  const int tid = WB ? (int)(blockIdx.x & 3u) * 64 + (int)threadIdx.x : (int)threadIdx.x, q = tid >> 6, lane = tid & 63;
  int px, py;
  tile_pixel(tile_x, tile_y, tid, px, py);
  const bool inside = px < v.W && py < v.H;
  const float pxf = (float)px, pyf = (float)py;
  const uint2 range = ranges[tile];
  const int n = (int)(range.y - range.x);
  const uint32_t* pl = point_list + range.x;
  float4* s = s_rec[WB ? 0 : q];

  // A stopped lane""")
a = """  if (out_invdepth)
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_FULL, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,"""
assert a in s
s = s.replace(a, """  if (out_invdepth)
    hipLaunchKernelGGL((k_render_fwd_wave<FWD_FULL, false>), dim3(4 * ntiles), dim3(64), 0, s, v, bb.ranges, bb.tile_order,""")
a = """    hipLaunchKernelGGL((k_render_fwd_wave<FWD_NO_INV, false>), dim3(ntiles), dim3(TILE_PIX), 0, s, v, bb.ranges, bb.tile_order,"""
assert a in s
s = s.replace(a, """    hipLaunchKernelGGL((k_render_fwd_wave<FWD_NO_INV, false>), dim3(4 * ntiles), dim3(64), 0, s, v, bb.ranges, bb.tile_order,""")
open("render_fwd.hip", "w").write(s)
