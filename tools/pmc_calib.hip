// pmc_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of
// the tile passes (MI355X_MICROARCH.md: FETCH_SIZE reports half of a wide coalesced streaming read; other
// widths are uncalibrated).  Each kernel moves a known number of bytes through a 1 GiB table (4x the
// Infinity Cache, so the reads reach HBM); run under rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in
// separate passes and divide the reported bytes by the known ones (tools/pmc_calib.sh).
//
//   k_stream16   coalesced 16-B-per-lane read of the whole table             known: table bytes
//   k_stream4    coalesced 4-B-per-lane read of the whole table              known: table bytes
//   k_gather48   per lane one random 48-B record (3 x 16-B loads), as the tile passes stage render records
//   k_gather48a  the same 48 B per lane, each record alone in its own 128-B line (separates the counter's
//                tally of a request from the bytes a 48-B-stride record pulls across line boundaries)
//   k_gather32   per lane one random 32-B record (2 x 16-B loads), the compact LM tangent records
//   k_store16    coalesced 16-B-per-lane store of 512 MiB                      known: bytes written
//   k_store32r   one 32-B row per lane at a random row index, as the LM rows   known: bytes written
//
//   hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib && ./tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void k_stream16(const float4* __restrict__ t, int64_t n4, float* __restrict__ sink) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = t[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) sink[0] = acc;  // keeps the loads
}

__global__ void k_stream4(const float* __restrict__ t, int64_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += t[i];
  if (acc == 1234.5f) sink[0] = acc;
}

__global__ void k_gather48(const float4* __restrict__ t, const uint32_t* __restrict__ idx, int64_t m,
                           float* __restrict__ sink) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t g = idx[i];
  const float4 a = t[3 * (size_t)g], b = t[3 * (size_t)g + 1], c = t[3 * (size_t)g + 2];
  const float s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w;
  if (s == 1234.5f) sink[0] = s;
}

__global__ void k_gather48a(const float4* __restrict__ t, const uint32_t* __restrict__ idx, int64_t m,
                            float* __restrict__ sink) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t g = idx[i];
  const float4 a = t[8 * (size_t)g], b = t[8 * (size_t)g + 1], c = t[8 * (size_t)g + 2];
  const float s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w;
  if (s == 1234.5f) sink[0] = s;
}

__global__ void k_gather32(const float4* __restrict__ t, const uint32_t* __restrict__ idx, int64_t m,
                           float* __restrict__ sink) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t g = idx[i];
  const float4 a = t[2 * (size_t)g], b = t[2 * (size_t)g + 1];
  const float s = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  if (s == 1234.5f) sink[0] = s;
}

__global__ void k_store16(float4* __restrict__ t, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    t[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

__global__ void k_store32r(float4* __restrict__ t, const uint32_t* __restrict__ idx, int64_t m) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t r = idx[i];
  t[2 * (size_t)r] = make_float4((float)i, 1.f, 2.f, 3.f);
  t[2 * (size_t)r + 1] = make_float4(4.f, 5.f, 6.f, 7.f);
}

int main() {
  const size_t table_bytes = (size_t)1 << 30;      // 1 GiB
  const int64_t n4 = (int64_t)(table_bytes / 16);   // float4 elements
  const int64_t m = 8 << 20;                         // gathered records / scattered rows per launch
  float4* table;
  float* sink;
  uint32_t *idx48, *idx48a, *idx32, *idxrow;
  CHECK(hipMalloc(&table, table_bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&idx48, m * 4));
  CHECK(hipMalloc(&idx48a, m * 4));
  CHECK(hipMalloc(&idx32, m * 4));
  CHECK(hipMalloc(&idxrow, m * 4));
  CHECK(hipMemset(table, 0, table_bytes));
  // distinct random records: a random permutation prefix of the table's record slots, so every gathered
  // byte is a different byte (no reuse in any cache)
  const uint32_t n48 = (uint32_t)(table_bytes / 48), n32 = (uint32_t)(table_bytes / 32);
  const uint32_t n128 = (uint32_t)(table_bytes / 128);
  std::vector<uint32_t> h(m);
  auto fill = [&](uint32_t nrec, uint32_t* dst, uint64_t seed) {
    std::vector<uint32_t> perm(nrec);
    for (uint32_t i = 0; i < nrec; ++i) perm[i] = i;
    uint64_t s = seed;
    for (int64_t i = 0; i < m; ++i) {  // partial Fisher-Yates
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      const uint32_t j = (uint32_t)(i + (s >> 33) % (uint64_t)(nrec - i));
      std::swap(perm[i], perm[j]);
      h[i] = perm[i];
    }
    CHECK(hipMemcpy(dst, h.data(), m * 4, hipMemcpyHostToDevice));
  };
  fill(n48, idx48, 1);
  fill(n128, idx48a, 4);
  fill(n32, idx32, 2);
  fill(n32, idxrow, 3);
  const int blocks = 256 * 16, threads = 256;
  const unsigned gb = (unsigned)((m + threads - 1) / threads);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_stream16, dim3(blocks), dim3(threads), 0, 0, table, n4, sink);
    hipLaunchKernelGGL(k_stream4, dim3(blocks), dim3(threads), 0, 0, reinterpret_cast<const float*>(table), 4 * n4,
                       sink);
    hipLaunchKernelGGL(k_gather48, dim3(gb), dim3(threads), 0, 0, table, idx48, m, sink);
    hipLaunchKernelGGL(k_gather48a, dim3(gb), dim3(threads), 0, 0, table, idx48a, m, sink);
    hipLaunchKernelGGL(k_gather32, dim3(gb), dim3(threads), 0, 0, table, idx32, m, sink);
    hipLaunchKernelGGL(k_store16, dim3(blocks), dim3(threads), 0, 0, table, n4 / 2);
    hipLaunchKernelGGL(k_store32r, dim3(gb), dim3(threads), 0, 0, table, idxrow, m);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  std::printf("{\"known_bytes\": {\"k_stream16\": %zu, \"k_stream4\": %zu, \"k_gather48\": %lld, \"k_gather48a\": %lld, \"k_gather32\": %lld, "
              "\"k_store16\": %zu, \"k_store32r\": %lld}}\n",
              table_bytes, table_bytes, (long long)(48 * m), (long long)(48 * m), (long long)(32 * m), table_bytes / 2,
              (long long)(32 * m));
  CHECK(hipFree(table));
  CHECK(hipFree(sink));
  CHECK(hipFree(idx48));
  CHECK(hipFree(idx48a));
  CHECK(hipFree(idx32));
  CHECK(hipFree(idxrow));
  return 0;
}
