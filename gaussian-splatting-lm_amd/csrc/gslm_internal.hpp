// gslm_internal.hpp -- host-side internal interfaces between the .hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>
#include "gslm.h"
#include "gslm_device.hpp"

namespace gslm {

void set_error(const std::string& msg);

#define GSLM_HIP_CHECK(expr)                                                                  \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      ::gslm::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                   \
      return GSLM_ERR_HIP;                                                                    \
    }                                                                                         \
  } while (0)

// Debug mode (gslm_view.debug, the rasterizer settings' `debug`, arguments/__init__.py:70): upstream's CHECK_CUDA
// synchronises after each kernel and throws on an error, so a failing launch is reported where it happened instead of
// as a late status of some later call.  The drop-in entry points open a DebugScope for their stream; inside it every
// GSLM_LAUNCH_CHECK synchronises that stream and names the launch site.
struct DebugSync {
  hipStream_t s = nullptr;
  bool on = false;
};
extern thread_local DebugSync g_debug;
struct DebugScope {
  DebugSync prev;
  DebugScope(bool on, void* stream) : prev(g_debug) {
    if (on) g_debug = DebugSync{(hipStream_t)stream, true};
  }
  ~DebugScope() { g_debug = prev; }
};
int launch_failed(hipError_t e, const char* file, int line);  // sets the error (debug: with the launch site)

#define GSLM_LAUNCH_CHECK()                                                                   \
  do {                                                                                        \
    hipError_t _e = hipGetLastError();                                                        \
    if (_e == hipSuccess && ::gslm::g_debug.on) _e = hipStreamSynchronize(::gslm::g_debug.s);  \
    if (_e != hipSuccess) return ::gslm::launch_failed(_e, __FILE__, __LINE__);               \
  } while (0)

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// ---------------- radix sort (LSD, 8-bit digits, stable) ----------------
constexpr int SORT_THREADS = 256;
constexpr int SORT_ITEMS = 16;                       // items per thread per block (large sorts)
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS; // 4096 keys per block
// Sorts that would launch fewer than SORT_FULL_BLOCKS blocks of SORT_TILE keys (the depth sort of 1M
// Gaussians: 245 blocks, one per CU, one wave per SIMD) use SORT_ITEMS_SMALL items per thread instead, so
// the launch fills the chip's 256 CUs several times over.
#ifndef GSLM_SORT_ITEMS_SMALL
#define GSLM_SORT_ITEMS_SMALL 8
#endif
constexpr int SORT_ITEMS_SMALL = GSLM_SORT_ITEMS_SMALL;
constexpr int64_t SORT_FULL_BLOCKS = 1024;
constexpr int RADIX = 256;

// A sort that moves a payload array with the pairs always takes SORT_ITEMS_SMALL items per thread: at 16 the third
// per-item register array pushes the scatter to 143 VGPRs (two waves per SIMD, 2x the time of the pair scatter).
inline int sort_items(int64_t n, bool payload = false) {
  return !payload && (n + SORT_TILE - 1) / SORT_TILE >= SORT_FULL_BLOCKS ? SORT_ITEMS : SORT_ITEMS_SMALL;
}
inline int64_t sort_blocks(int64_t n, bool payload = false) {
  const int64_t t = (int64_t)SORT_THREADS * sort_items(n, payload);
  return (n + t - 1) / t;
}
// [RADIX][blocks] counts, RADIX digit totals, then the key range of a key_range sort: 4 words and a (min, max) pair
// per block
inline size_t sort_hist_bytes(int64_t n, bool payload = false) {
  const size_t nb = (size_t)sort_blocks(n, payload);
  return (size_t)RADIX * nb * 4 + 4 * RADIX + 16 + 8 * nb;
}

// Sorts (keys, vals) of length n on bits [0, end_bit).  Uses k0/v0 as input and k1/v1 as the
// ping-pong buffers; *result_in_alt tells which pair holds the output.  hist: sort_hist_bytes(n, p0 != NULL).
// last_gather (or NULL): the last pass writes last_gather[value] in place of each sorted key.
// n_dev (or NULL): n is a capacity (grid and hist sized for it) and the kernels sort the first min(n, *n_dev) pairs.
// p0 / p1 (or NULL): a second value array (p0 input, p1 its ping-pong partner) moved with the pairs; the result is
// in p1 exactly when *result_in_alt.
// key_range (the depth sort: end_bit 32, no n_dev / payload): the passes sort key - min over the keys other than
// 0xFFFFFFFF (those sort last, as before), and the passes past the span's bytes run as copies -- the 32-bit sort's
// order bit for bit, in fewer working passes when the keys span fewer than 32 bits (sort.hip KeyRange).
int radix_sort_pairs(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int64_t n, int end_bit,
                     uint32_t* hist, bool* result_in_alt, hipStream_t s, bool iota_values = false,
                     const uint32_t* last_gather = nullptr, const uint32_t* n_dev = nullptr, uint32_t* p0 = nullptr,
                     uint32_t* p1 = nullptr, bool key_range = false);

// ---------------- exclusive scan of uint32 (optionally gathered through idx) ----------------
constexpr int SCAN_THREADS = 256;
#ifndef GSLM_SCAN_ITEMS
#define GSLM_SCAN_ITEMS 8
#endif
constexpr int SCAN_ITEMS = GSLM_SCAN_ITEMS;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;
inline int64_t scan_blocks(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }
// Above this many blocks a scan's apply pass no longer sums its prefix of block sums itself (O(nb^2) loads over the
// grid) but reads it from a scanned copy (k_scan_top, one more launch).  The bench's forward scans (1M Gaussians,
// nb = 489) and its LM row map (4.87M pairs, nb = 2377) keep the two-launch form.
#ifndef GSLM_SCAN_INLINE_MAX_BLOCKS
#define GSLM_SCAN_INLINE_MAX_BLOCKS 4096
#endif
constexpr int64_t SCAN_INLINE_MAX_BLOCKS = GSLM_SCAN_INLINE_MAX_BLOCKS;
inline size_t scan_tmp_bytes(int64_t n) { return align_up((size_t)scan_blocks(n) * 8 + 64); }  // dual scans: 2 nb
// out[i] = sum_{j<i} in[idx ? idx[j] : j];  *total (device) = full sum.
// inline_max_blocks: the largest block count whose apply pass sums its own prefix of block sums (above it, k_scan_top)
int exclusive_scan_u32(const uint32_t* in, const uint32_t* idx, uint32_t* out, int64_t n, uint32_t* tmp,
                       uint32_t* total, hipStream_t s, int64_t inline_max_blocks = SCAN_INLINE_MAX_BLOCKS);
// out_a[i] = sum_{j<i} in[j], out_b[i] = sum_{j<i} b[j] in one pass (tmp: scan_tmp_bytes(n)), b = in_b, or in
// gathered through idx when in_b is NULL.
int exclusive_scan_u32_dual(const uint32_t* in, const uint32_t* idx, uint32_t* out_a, uint32_t* out_b, int64_t n,
                            uint32_t* tmp, uint32_t* total_a, uint32_t* total_b, hipStream_t s,
                            const uint32_t* in_b = nullptr);

}  // namespace gslm
