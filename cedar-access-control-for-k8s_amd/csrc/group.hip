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

#include <cstdlib>
#include <string>

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

// key = 10 bits of (action, resource type) | 14 bits of the principal's type and key-ancestor set |
// 8 bits of its hot values. Equal fields group; unequal values that share a field only cost
// locality. The set and value hashes are sums of per-element mixes (order-independent), so the 8
// lanes that read a request's row and ancestor list in coalesced pieces combine them by shuffles.
constexpr uint32_t GROUP_ANC = 32;  // key ancestors hashed (the scope-index keys a request probes)
constexpr uint32_t GSEG = 8;        // lanes per request

__device__ __forceinline__ uint32_t gfin(uint32_t h) {
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  return h;
}

// ANC: hash the principal's key-ancestor set (one dependent load into the request block); else the
// principal's UID stands for it (CEDARGPU_GROUP_KEY=uid, A/B)
template <bool ANC>
__global__ __launch_bounds__(256) void cedar_group_key(const uint32_t* __restrict__ rows, const uint32_t* __restrict__ heap,
                                                       uint32_t n, uint32_t row_words, uint32_t n_hot,
                                                       uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t lane = threadIdx.x & 63, sl = lane % GSEG, sbase = lane - sl;
  const uint32_t i = (blockIdx.x * 256 + threadIdx.x) / GSEG;
  const bool valid = i < n;
  const uint32_t* row = rows + (size_t)(valid ? i : 0u) * row_words;
  const uint32_t h0 = valid ? row[sl] : 0u, h1 = valid ? row[GSEG + sl] : 0u;  // header words 0..15
  auto hdr = [&](uint32_t k) -> uint32_t {
    return (uint32_t)__shfl((int)(k < GSEG ? h0 : h1), (int)(sbase + (k % GSEG)));
  };
  const uint32_t ar = gmix(gmix(0x51ED27Fu, hdr(RW_A + 1)), hdr(RW_R));
  const uint32_t pn = hdr(RW_PN);
  const uint32_t nk = (ANC && valid) ? min((pn >> AN_KEYS_SHIFT) & AN_KEYS, GROUP_ANC) : 0u;
  const uint32_t* anc = heap + hdr(RW_BLK) + hdr(RW_PANC);
  uint32_t g = 0, hv = 0;
  for (uint32_t j = sl; j < nk; j += GSEG) {
    const uint2 u = *reinterpret_cast<const uint2*>(anc + 2 * j);
    g += gmix(gmix(0x2545F491u, u.x), u.y);
  }
  for (uint32_t j = sl; valid && j < 2 * n_hot; j += GSEG) hv += gmix(0x6C8E9CF5u + j, row[RW_HDR + j]);
  for (uint32_t o = GSEG / 2; o; o >>= 1) {
    g += (uint32_t)__shfl_xor((int)g, (int)o);
    hv += (uint32_t)__shfl_xor((int)hv, (int)o);
  }
  g = gfin(g + gmix(0x3C6EF372u, hdr(RW_P)) + (ANC ? 0u : gmix(0x1B873593u, hdr(RW_P + 1))));
  hv = gfin(hv);
  if (valid && sl == 0) {
    keys[i] = (ar & 0xFFC00000u) | ((g >> 18) << 8) | (hv >> 24);
    vals[i] = i;
  }
}

}  // namespace

namespace cg {

// Temporary storage rocPRIM's radix sort needs for n pairs.
// Onesweep at every size: rocPRIM's default takes its merge-sort path up to 2^20 pairs of 32-bit
// keys, ~0.16 ms per 1M on gfx950 (profiles/r03/ab1).
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

size_t group_temp_bytes(uint32_t n) {
  size_t bytes = 0;
  uint32_t* none = nullptr;
  if (rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, none, none, none, none, n, 0, 32) != hipSuccess) return 0;
  return bytes;
}

// Enqueues the grouping of n requests on `stream`: ord[k] = the request evaluated k-th.
// keys / keys2 / vals: n words each of scratch; temp: group_temp_bytes(n) bytes.
int group_enqueue(const uint32_t* rows, const uint32_t* heap, uint32_t n, uint32_t row_words, uint32_t n_hot,
                  uint32_t* keys, uint32_t* keys2, uint32_t* vals, uint32_t* ord, void* temp, size_t temp_bytes,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  static const bool uid = std::getenv("CEDARGPU_GROUP_KEY") && std::string(std::getenv("CEDARGPU_GROUP_KEY")) == "uid";
  if (uid)
    hipLaunchKernelGGL(cedar_group_key<false>, dim3((n + 256 / GSEG - 1) / (256 / GSEG)), dim3(256), 0, s, rows, heap, n,
                       row_words, n_hot, keys, vals);
  else
    hipLaunchKernelGGL(cedar_group_key<true>, dim3((n + 256 / GSEG - 1) / (256 / GSEG)), dim3(256), 0, s, rows, heap, n,
                       row_words, n_hot, keys, vals);
  if (hipGetLastError() != hipSuccess) return -1;
  size_t bytes = temp_bytes;
  if (rocprim::radix_sort_pairs<SortConfig>(temp, bytes, keys, keys2, vals, ord, n, 0, 32, s) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cg
