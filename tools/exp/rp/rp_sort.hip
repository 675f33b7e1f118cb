// Measurement only (not product code): rocPRIM's device radix sort (onesweep) on the forward's two sort shapes, as
// a yardstick for the in-tree LSD sort (sort.hip).  1M 32-bit depth keys with index values; 4.87M 13-bit tile keys
// with u32 values.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float time_sort(size_t n, int end_bit, unsigned seed, int reps) {
  std::vector<unsigned> hk(n), hv(n);
  std::mt19937 rng(seed);
  for (size_t i = 0; i < n; ++i) {
    hk[i] = end_bit == 32 ? (0x3E000000u + (rng() % 0x05000000u)) : (rng() % 8160u);
    hv[i] = (unsigned)i;
  }
  unsigned *k0, *k1, *v0, *v1;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
  size_t tmp_bytes = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 0, end_bit));
  void* tmp;
  CK(hipMalloc(&tmp, tmp_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 3; ++r) CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, end_bit));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, end_bit));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  // check sortedness
  std::vector<unsigned> ok(n);
  CK(hipMemcpy(ok.data(), k1, n * 4, hipMemcpyDeviceToHost));
  for (size_t i = 1; i < n; ++i) if (ok[i - 1] > ok[i]) { printf("not sorted at %zu\n", i); break; }
  CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(v0)); CK(hipFree(v1)); CK(hipFree(tmp));
  return ms / reps * 1000.f;
}

int main() {
  printf("{\"rocprim_depth_1M_32bit_us\": %.1f, ", time_sort(1000000, 32, 1, 20));
  printf("\"rocprim_tile_4.87M_13bit_us\": %.1f}\n", time_sort(4867236, 13, 2, 20));
  return 0;
}
