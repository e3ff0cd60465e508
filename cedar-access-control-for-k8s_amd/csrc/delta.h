// Delta images ("delta images" for policy hot reload). The reference applies every
// CRD informer event to its PolicySet in place (internal/server/store/crd.go:45-118: Add / Remove
// at :62,85,102,114) and the directory store swaps a re-read set on a ticker (directory.go:41-82).
// Here the root compiles the new epoch (incrementally, compiler.cpp LowerState) and ships only the
// bytes that differ from the image every rank already holds: a delta blob of copy / literal
// operations over the new image's bytes. Each rank rebuilds the new blob on its GPU from its device
// copy of the base (dev_blob_patch), checks it against the new blob's checksum, and loads it.
//
// Delta blob (little-endian):
//   u32 magic "CGDL", u32 version, u64 base_len, u64 new_len, u64 new_sum (blob_sum of the new
//   blob), u64 n_ops, u64 lit_len, u64 n_fix, then n_ops (dst, len, src) u64 triples in dst order
//   covering [0, new_len) exactly (src: a base-blob offset, or DL_LIT | an offset into the
//   literals), then n_fix (word index, value) u32 pairs applied after the operations (a copied
//   block that differs in a few words: a scope-index entry whose first-head index moved when a
//   document was added), then lit_len literal bytes.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace cg {

constexpr uint32_t DL_MAGIC = 0x4C444743u;  // "CGDL"
constexpr uint32_t DL_VERSION = 3;
constexpr size_t DL_HEAD = 56;

// 64-bit checksum of a blob: the sum (mod 2^64) over its 8-byte little-endian words (the last one
// zero-padded) of mix(word ^ index * K), plus the length. Order-keyed by the index and
// associative, so up to 16 host threads or a GPU kernel (dev_blob_sum) compute it in any split.
inline uint64_t blob_word_mix(uint64_t w, uint64_t i) {
  uint64_t z = w ^ (i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t blob_sum(const uint8_t* p, size_t n);

// The delta that turns `base` into `next`. Both are image blobs: the diff pairs their regions
// (header, each device section, the host part), so a section that grew or shrank does not shift
// the comparison of the others; within a region, equal runs at the current shift become copies
// and a run of mismatches starts a search (rolling hash over the base region) for the new shift.
// Any two byte strings work (one region each when either is no image blob).
std::vector<uint8_t> image_delta(const uint8_t* base, size_t base_len, const uint8_t* next, size_t next_len);

// A parsed, checked delta: every operation in range, the operations covering the new blob once.
struct DeltaPlan {
  uint64_t base_len = 0, new_len = 0, new_sum = 0, n_ops = 0;
  std::vector<uint64_t> pieces;  // (dst, len, src) triples of at most DL_PIECE bytes (device.h)
  const uint8_t* lit = nullptr;  // into the delta blob
  size_t lit_len = 0;
  const uint32_t* fix = nullptr;  // (word index, value) pairs, into the delta blob (4-byte aligned)
  size_t n_fix = 0;
};
DeltaPlan delta_plan(const uint8_t* delta, size_t len);  // throws CedarError when malformed

// The new blob on the host (base bytes + delta), checked against new_sum.
std::vector<uint8_t> image_patch(const uint8_t* base, size_t base_len, const uint8_t* delta, size_t len);

}  // namespace cg
