// Request grouping on the device (the batching layer's locality order, inside the evaluation step).
//
// A throughput batch is evaluated in an order that puts requests with the same (action, resource
// type), the same principal key ancestors and the same hot attribute values side by side, so the
// requests of a wave probe the same scope-index buckets and run the same candidate policies
// (round 1: +30 % on C3, profiles/r01/group_ab). Round 2 sorted the rows on the host at submit
// (~50 ns per request, outside the timed step). Here the order is computed on the device as part
// of every step: one kernel hashes each request's row into a 32-bit grouping key, rocPRIM's radix
// sort (stable) orders (key, request) pairs, and the first-pass kernels read requests through the
// resulting order (KArgs::ord). Rows never move and results stay at each request's own index, so
// nothing on the host changes.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "image.h"

using namespace cgi;

namespace {

__device__ __forceinline__ uint32_t gmix(uint32_t h, uint32_t x) {
  h ^= x;
  h *= 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x85EBCA77u;
  return h ^ (h >> 13);
}

// key = 10 bits of (action, resource type) | 14 bits of the principal's type and key ancestors |
// 8 bits of its hot values. Equal fields group; unequal values that share a field only cost locality.
constexpr uint32_t GROUP_ANC = 32;  // key ancestors hashed (the scope-index keys a request probes)

// one request per lane: its row header, its first key ancestors and its hot values
__global__ __launch_bounds__(256) void cedar_group_key(const uint32_t* __restrict__ rows, const uint32_t* __restrict__ heap,
                                                       uint32_t n, uint32_t row_words, uint32_t n_hot,
                                                       uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t* row = rows + (size_t)i * row_words;
  const uint32_t ar = gmix(gmix(0x51ED27Fu, row[RW_A + 1]), row[RW_R]);
  const uint32_t pn = row[RW_PN];
  const uint32_t nk = min((pn >> AN_KEYS_SHIFT) & AN_KEYS, GROUP_ANC);
  const uint32_t* anc = heap + row[RW_BLK] + row[RW_PANC];
  uint32_t g = gmix(0x2545F491u, row[RW_P]);
  for (uint32_t j = 0; j < nk; j++) g = gmix(gmix(g, anc[2 * j]), anc[2 * j + 1]);
  uint32_t hv = 0x6C8E9CF5u;
  for (uint32_t j = 0; j < 2 * n_hot; j++) hv = gmix(hv, row[RW_HDR + j]);
  keys[i] = (ar & 0xFFC00000u) | ((g >> 18) << 8) | (hv >> 24);
  vals[i] = i;
}

}  // namespace

namespace cg {

// Temporary storage rocPRIM's radix sort needs for n pairs.
size_t group_temp_bytes(uint32_t n) {
  size_t bytes = 0;
  uint32_t* none = nullptr;
  if (rocprim::radix_sort_pairs(nullptr, bytes, none, none, none, none, n, 0, 32) != hipSuccess) return 0;
  return bytes;
}

// Enqueues the grouping of n requests on `stream`: ord[k] = the request evaluated k-th.
// keys / keys2 / vals: n words each of scratch; temp: group_temp_bytes(n) bytes.
int group_enqueue(const uint32_t* rows, const uint32_t* heap, uint32_t n, uint32_t row_words, uint32_t n_hot,
                  uint32_t* keys, uint32_t* keys2, uint32_t* vals, uint32_t* ord, void* temp, size_t temp_bytes,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(cedar_group_key, dim3((n + 255) / 256), dim3(256), 0, s, rows, heap, n, row_words, n_hot, keys, vals);
  if (hipGetLastError() != hipSuccess) return -1;
  size_t bytes = temp_bytes;
  if (rocprim::radix_sort_pairs(temp, bytes, keys, keys2, vals, ord, n, 0, 32, s) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cg
