// valu_rate.hip -- issue rate of scalar f32 FMAs (v_fma_f32) against packed ones (v_pk_fma_f32) on gfx950, at
// the occupancy of the tile passes (8 waves per SIMD), to price the "two pixels per lane with packed f32 math"
// design for k_render_matvec (round-1 verdict).  Each lane runs CHAINS independent FMA chains of ITERS steps;
// the packed kernel does the same flops as float2 lanes, half the instructions.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate && ./tools/valu_rate  (profiles/r02/valu_rate.json)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef float float2v __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;
constexpr int CHAINS = 8;  // scalar chains per lane (packed: CHAINS / 2 float2 chains)

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
  float x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fmaf(x[c], a, b);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c];
  if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(256) void k_pk_fma(float* out, float a, float b) {
  float2v x[CHAINS / 2];
  const float2v av = {a, a}, bv = {b, b};
#pragma unroll
  for (int c = 0; c < CHAINS / 2; ++c) x[c] = float2v{threadIdx.x * 1e-3f + 2 * c, threadIdx.x * 1e-3f + 2 * c + 1};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS / 2; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHAINS / 2; ++c) s += x[c].x + x[c].y;
  if (s == 1234.5f) out[0] = s;
}

int main() {
  float* out;
  CHECK(hipMalloc(&out, 64));
  const int blocks = 256 * 8 * 4;  // 8 blocks (32 waves, 8 per SIMD) per CU, 4 rounds
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double lanes = (double)blocks * 256;
  struct K { const char* name; void (*f)(float*, float, float); double flops_per_lane; double insts_per_lane; };
  const K ks[] = {
      {"v_fma_f32", k_fma, 2.0 * CHAINS * ITERS, (double)CHAINS * ITERS},
      {"v_pk_fma_f32", k_pk_fma, 2.0 * CHAINS * ITERS, (double)CHAINS / 2 * ITERS},
  };
  std::printf("{");
  for (int r = 0; r < 2; ++r) {
    for (int k = 0; k < 2; ++k) {
      hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (r == 1)
        std::printf("%s\"%s\": {\"ms\": %.4f, \"tflops\": %.2f, \"wave_insts_per_ns\": %.2f}", k ? ", " : "", ks[k].name, ms,
                    lanes * ks[k].flops_per_lane / (ms * 1e9), lanes / 64 * ks[k].insts_per_lane / (ms * 1e6));
    }
  }
  std::printf("}\n");
  CHECK(hipFree(out));
  return 0;
}
