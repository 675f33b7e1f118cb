// diag.hip -- device self-tests of the wave-level primitives the tile passes rely on.
#include "gslm_tile.hpp"

namespace gslm {

// in: [64 lanes][8 values] (value-major per lane); out[lane] = primitive result of that lane.
__global__ void k_selftest(int which, const float* __restrict__ in, float* __restrict__ out) {
  const int lane = threadIdx.x;
  if (which == 0) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = in[lane * 8 + k];
    out[lane] = wave_reduce8_t(v, lane);
  } else {
    out[lane] = wave_sum_lane63(in[lane * 8]);
  }
}

}  // namespace gslm

extern "C" int gslm_selftest(int32_t which, const float* in, float* out, void* stream) {
  hipLaunchKernelGGL(gslm::k_selftest, dim3(1), dim3(64), 0, (hipStream_t)stream, which, in, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    gslm::set_error(std::string("selftest launch: ") + hipGetErrorString(e));
    return GSLM_ERR_HIP;
  }
  return GSLM_OK;
}

extern "C" int gslm_selftest_scan(const uint32_t* in, uint32_t* out, int64_t n, int32_t force_top, void* tmp,
                                  size_t tmp_bytes, uint32_t* total, void* stream) {
  if (n < 0 || (n > 0 && (!in || !out || !tmp || !total))) {
    gslm::set_error("selftest_scan: n < 0 or NULL buffer");
    return GSLM_ERR_INVALID;
  }
  if (tmp_bytes < gslm::scan_tmp_bytes(n)) {
    gslm::set_error("selftest_scan: tmp below 8 ceil(n / 2048) + 64 bytes rounded up to 256");
    return GSLM_ERR_CAPACITY;
  }
  return gslm::exclusive_scan_u32(in, nullptr, out, n, static_cast<uint32_t*>(tmp), total, (hipStream_t)stream,
                                  force_top ? 0 : gslm::SCAN_INLINE_MAX_BLOCKS);
}
