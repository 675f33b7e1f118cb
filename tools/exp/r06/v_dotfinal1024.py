# timing variant (round 6): k_dot_final as one block of 1024 threads (one batch of loads for <= 8192 partials)
# instead of 256 -- a different (still fixed) summation order
s = open("cg.hip").read()
a = """__global__ __launch_bounds__(DOT_THREADS) void k_dot_final(const double* __restrict__ part, int np,
                                                           double* __restrict__ out) {
  __shared__ double s[DOT_THREADS / 64];
  const double acc = strided_sum_in_order(part, np);
  const double t = block_sum_d(acc, s);
  if (threadIdx.x == 0) *out = t;
}"""
assert a in s
s = s.replace(a, """__global__ __launch_bounds__(1024) void k_dot_final(const double* __restrict__ part, int np,
                                                   double* __restrict__ out) {
  __shared__ double s[16];
  double acc = strided_sum_in_order(part, np);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if (lane == 0) s[w] = acc;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += s[k];
    *out = t;
  }
}""")
s = s.replace("hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(DOT_THREADS),", "hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(1024),")
open("cg.hip", "w").write(s)
