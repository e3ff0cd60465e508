// Request grouping on the device (the batching layer's locality order, inside the evaluation step).
//
// A throughput batch is evaluated in an order that puts requests with the same (action, resource
// type), the same principal key ancestors and the same hot attribute values side by side, so the
// requests of a wave probe the same scope-index buckets and run the same candidate policies
// (round 1: +30 % on C3, profiles/r01/group_ab). Round 2 sorted the rows on the host at submit
// (~50 ns per request, one thread, outside the timed step).
//
// Here the order is computed on the device in every step from the 32-bit grouping key the encoder
// writes per request (Batch::gkeys: a hash of fields it encodes anyway, on the encoding threads):
// rocPRIM's radix sort (onesweep, stable) orders (key, request) pairs: ord[k] = the request
// evaluated k-th. The first-pass kernels read each request's row through the order (whole 64-byte
// lines at random); results and scan lists stay at each request's own index. (Round 3 copied the
// rows into order first, so that those kernels read them contiguously: the copy cost 0.077 ms per
// 1M and 0.26 GB of traffic, and saved the kernels 0.016 ms: 690 vs 718 M decisions/s on C3,
// gpurun_out/r04gab; CEDARGPU_GROUP_GATHER=1 brings it back.)
// A bucket sort with one atomic per request into 2^20-2^22 counters was 3-5x slower: popular
// principals' identical keys serialize their atomics (0.52-1.34 ms per 1M, profiles/r03/ab6).
// Ordering only within tiles of 4-16k requests (one block-local LDS radix sort per tile, one
// launch: 0.027-0.058 ms) made the scan 0.11 ms slower: equal keys must meet across the whole
// batch (round 5, profiles/r05/ab/r05v). 24 key bits stay best: 16 bits sort in 0.061 ms but the
// scan loses 0.036 ms, 32 bits cost 0.022 ms more sort for a 0.014 ms slower scan (r05w).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>

#include "image.h"

using namespace cgi;

namespace {

// GSEG lanes per request copy its row (uint4 pieces) to its grouped position
constexpr uint32_t GSEG = 8;
__global__ __launch_bounds__(256) void cedar_group_gather(const uint32_t* __restrict__ ord, uint32_t n,
                                                          const uint4* __restrict__ rows, uint32_t row_vec,
                                                          uint4* __restrict__ grows) {
  const uint32_t lane = threadIdx.x & 63, sl = lane % GSEG;
  const uint32_t k = (blockIdx.x * 256 + threadIdx.x) / GSEG;
  if (k >= n) return;
  const uint4* src = rows + (size_t)ord[k] * row_vec;
  uint4* dst = grows + (size_t)k * row_vec;
  for (uint32_t j = sl; j < row_vec; j += GSEG) dst[j] = src[j];
}

// vals[i] = i, four per lane (vals 16-byte aligned; the tail of the last uint4 past n is scratch)
__global__ __launch_bounds__(256) void cedar_group_iota(uint4* __restrict__ vals, uint32_t n, uint32_t* __restrict__ zero,
                                                        uint32_t zero_n) {
  const uint32_t i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i < n) vals[i / 4] = make_uint4(i, i + 1, i + 2, i + 3);
  if (blockIdx.x == 0 && threadIdx.x < zero_n) zero[threadIdx.x] = 0u;
}

}  // namespace

namespace cg {

// rocPRIM's onesweep configuration for (u32 key, u32 request) pairs. Its gfx950 default sorts
// 1024 x 16 = 16384 pairs per block: 64 blocks per 1M requests, a quarter of the CUs, each pass
// latency-bound (~27 us per 8-bit pass, profiles/r04/final2). CEDARGPU_SORT_CFG picks a smaller
// block (A/B): 1 = 256x16, 2 = 512x8, 3 = 256x8, 4 = 512x16, 5 = 256x12, 6 = 512x8 with a
// 512x8 histogram, 7 = 1024x4 with a 512x8 histogram (the default: 256 blocks, group 0.086-0.092
// ms per 1M vs 0.121-0.129 at 0, gpurun_out/r05n, r05o); 0 = rocPRIM's default. (12-bit digits,
// two places for 24 bits: the histogram kernel needs 192 KB of LDS.)
template <unsigned B, unsigned I, unsigned HB = 1024, unsigned HI = 16, unsigned BITS = 8>
using OneSweep = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<HB, HI>, rocprim::kernel_config<B, I>, BITS,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

static int sort_cfg() {
  static const int c = [] {
    const char* e = std::getenv("CEDARGPU_SORT_CFG");
    const int v = e ? std::atoi(e) : 7;
    return v < 0 || v > 7 ? 7 : v;
  }();
  return c;
}

template <class Cfg>
hipError_t sort_with(void* temp, size_t& bytes, uint32_t* keys, uint32_t* keys2, const uint32_t* vals, uint32_t* ord,
                     uint32_t n, uint32_t lo, hipStream_t s) {
  return rocprim::radix_sort_pairs<Cfg>(temp, bytes, keys, keys2, vals, ord, n, lo, 32, s);
}

static hipError_t group_sort(void* temp, size_t& bytes, uint32_t* keys, uint32_t* keys2, const uint32_t* vals, uint32_t* ord,
                             uint32_t n, uint32_t lo, hipStream_t s) {
  switch (sort_cfg()) {
    case 1: return sort_with<OneSweep<256, 16>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 2: return sort_with<OneSweep<512, 8>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 3: return sort_with<OneSweep<256, 8>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 4: return sort_with<OneSweep<512, 16>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 5: return sort_with<OneSweep<256, 12>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 6: return sort_with<OneSweep<512, 8, 512, 8>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    case 7: return sort_with<OneSweep<1024, 4, 512, 8>>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
    default: return sort_with<SortConfig>(temp, bytes, keys, keys2, vals, ord, n, lo, s);
  }
}

// key bits sorted, from the top: CEDARGPU_GROUP_BITS (24 by default: three onesweep passes, the
// (action, resource type) and principal fields; 0.19 vs 0.22 ms per 1M at 32, profiles/r03/ab11)
uint32_t group_bits() {
  static const uint32_t b = [] {
    const char* e = std::getenv("CEDARGPU_GROUP_BITS");
    const int v = e ? std::atoi(e) : 24;
    return (uint32_t)(v < 8 ? 8 : v > 32 ? 32 : v);
  }();
  return b;
}

// CEDARGPU_GROUP_GATHER=1: the rows copied into group order (grows) for the first-pass kernels
bool group_gather() {
  static const bool g = [] { const char* e = std::getenv("CEDARGPU_GROUP_GATHER"); return e && *e == '1'; }();
  return g;
}

// Temporary storage rocPRIM's radix sort needs for n pairs (onesweep at every size: the default
// takes its merge-sort path up to 2^20 pairs, ~0.16 ms per 1M on gfx950, profiles/r03/ab1).
size_t group_temp_bytes(uint32_t n) {
  size_t bytes = 0;
  uint32_t* none = nullptr;
  if (group_sort(nullptr, bytes, none, none, none, none, n, 32 - group_bits(), nullptr) != hipSuccess)
    return 0;
  return bytes;
}

// Enqueues the grouping of n requests on `stream`: ord[k] = the request evaluated k-th, grows its
// row (row_words a multiple of 4). keys2 / vals: n words of scratch each; temp: group_temp_bytes.
int group_enqueue(const uint32_t* keys, const uint32_t* rows, uint32_t n, uint32_t row_words, uint32_t* grows,
                  uint32_t* ord, uint32_t* keys2, uint32_t* vals, void* temp, size_t temp_bytes, void* stream,
                  uint32_t* zero, uint32_t zero_n) {
  hipStream_t s = (hipStream_t)stream;
  if (row_words % 4) return -1;
  // The request indices are written out (one pass over n words) rather than read from a counting
  // iterator: rocPRIM copies a counting iterator and the keys into its buffers (two passes) before
  // an odd number of digit places.
  if (zero_n > 256) return -1;
  hipLaunchKernelGGL(cedar_group_iota, dim3((n + 1023) / 1024), dim3(256), 0, s, reinterpret_cast<uint4*>(vals), n, zero,
                     zero ? zero_n : 0u);
  size_t bytes = temp_bytes;
  if (group_sort(temp, bytes, const_cast<uint32_t*>(keys), keys2, vals, ord, n, 32 - group_bits(), s) != hipSuccess)
    return -1;
  if (!group_gather()) return hipGetLastError() == hipSuccess ? 0 : -1;
  hipLaunchKernelGGL(cedar_group_gather, dim3((n + 256 / GSEG - 1) / (256 / GSEG)), dim3(256), 0, s, ord, n,
                     reinterpret_cast<const uint4*>(rows), row_words / 4, reinterpret_cast<uint4*>(grows));
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cg
