// Host engine: compiled image, batch encoder, result renderer, device bridge.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "cedar.h"
#include "image.h"

namespace cg {

// Lists deduplicated while built (parents, groups) scan linearly up to this many entries and hash
// beyond, so a principal in thousands of groups encodes in time linear in its size.
constexpr size_t DEDUP_SCAN = 32;

// huge-page-backed anonymous mappings (encoder.cpp): huge_map returns null on failure (the caller
// falls back to the heap); huge_unmap returns false for a block huge_map did not make
bool hugepages_on();
void* huge_map(size_t bytes);
bool huge_unmap(void* p, size_t bytes);

// Pinned (page-locked, device-mapped) blocks for the host arrays a batch uploads (cedar_eval.hip;
// the host-only build has none): a small batch's heap and rows are encoded straight into memory
// the copy engine reads, so its upload needs no staging copy. pinned_take returns null when pinned
// blocks are off (no device context yet, CEDARGPU_PINNED_ARRAYS=0, or the cap is reached);
// pinned_give returns false for a block it did not hand out; pinned_block tells whether [p, p+n)
// lies in one of its blocks.
void* pinned_take(size_t bytes);
bool pinned_give(void* p, size_t bytes);
bool pinned_block(const void* p, size_t bytes);
void pinned_stats(uint64_t* held_bytes, uint64_t* idle_blocks);
extern std::atomic<uint64_t> g_pinned_kept;  // batches closed in flight that kept their arrays
constexpr size_t PIN_MIN = 64u << 10, PIN_MAX = 16u << 20;  // array sizes that take pinned blocks

// An allocator whose resize() leaves new elements uninitialised: a batch's large arrays are
// written in full right after they grow (Batch::concat), so zero-filling them first would be a
// serial pass over hundreds of MB.

template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U> struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <class U> NoInitAlloc(const NoInitAlloc<U>&) {}
  template <class U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
  // CEDARGPU_HUGEPAGES=1: blocks of >= 2 MiB (a bulk encode's batch parts and the concatenated
  // batch: ~1 GB per 1M SARs) from huge-page-backed mappings, whose first touches fault 2 MiB at a
  // time (A/B: with the kernel's synchronous compaction on advised regions it can lose).
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= huge_min() && huge_on()) {
      if (void* p = huge_map(bytes)) return static_cast<T*>(p);
    }
    return std::allocator<T>::allocate(n);
  }
  void deallocate(T* p, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= huge_min() && huge_on() && huge_unmap(p, bytes)) return;
    std::allocator<T>::deallocate(p, n);
  }
  static constexpr size_t huge_min() { return 2u << 20; }
  static bool huge_on() { return hugepages_on(); }
};
template <class T> using PodVec = std::vector<T, NoInitAlloc<T>>;

// A batch's uploaded arrays: NoInitAlloc, with arrays of PIN_MIN..PIN_MAX bytes in pinned blocks
// when there are any (pinned_take), which the upload copies from without staging.
template <class T>
struct PinAlloc : NoInitAlloc<T> {
  template <class U> struct rebind { using other = PinAlloc<U>; };
  PinAlloc() = default;
  template <class U> PinAlloc(const PinAlloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= PIN_MIN && bytes <= PIN_MAX)
      if (void* p = pinned_take(bytes)) return static_cast<T*>(p);
    return NoInitAlloc<T>::allocate(n);
  }
  void deallocate(T* p, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= PIN_MIN && bytes <= PIN_MAX && pinned_give(p, bytes)) return;
    NoInitAlloc<T>::deallocate(p, n);
  }
};
template <class T> using PinVec = std::vector<T, PinAlloc<T>>;
// n elements appended by one copy (a range insert into these vectors constructs element by
// element through the allocator: ~8 % of a SAR encode)
template <class T, class A>
inline void append_pod(std::vector<T, A>& v, const T* p, size_t n) {
  const size_t o = v.size();
  v.resize(o + n);
  if (n) std::memcpy(v.data() + o, p, n * sizeof(T));
}

struct PolicyMeta {
  std::string id, filename;
  Position pos;
  uint32_t tier = 0;
  bool forbid = false;
};

struct EncCache;  // encode_impl.h

// 64-bit key -> 31-bit value, open addressing at load <= 1/2 (the encoder's per-UID lookups of
// static entities: a std::unordered_map's modulo and node walk were ~10 % of a SAR encode)
struct U64Table {
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;  // value + 1 (0: empty slot)
  size_t n = 0;
  void clear() { keys.clear(); vals.clear(); n = 0; }
  static size_t slot(uint64_t k, size_t mask) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 32) & mask; }
  // (the first value put for a key stays)
  void put(uint64_t k, uint32_t v) {
    if (2 * (n + 1) > keys.size()) {
      std::vector<uint64_t> ok;
      std::vector<uint32_t> ov;
      ok.swap(keys);
      ov.swap(vals);
      keys.assign(std::max<size_t>(16, ok.size() * 2), 0);
      vals.assign(keys.size(), 0);
      n = 0;
      for (size_t i = 0; i < ok.size(); i++)
        if (ov[i]) put(ok[i], ov[i] - 1);
    }
    const size_t mask = keys.size() - 1;
    for (size_t h = slot(k, mask);; h = (h + 1) & mask) {
      if (!vals[h]) { keys[h] = k; vals[h] = v + 1; n++; return; }
      if (keys[h] == k) return;
    }
  }
  int32_t find(uint64_t k) const {
    if (!n) return -1;
    const size_t mask = keys.size() - 1;
    for (size_t h = slot(k, mask);; h = (h + 1) & mask) {
      if (!vals[h]) return -1;
      if (keys[h] == k) return (int32_t)(vals[h] - 1);
    }
  }
};

// Word arrays whose resize() leaves new words unwritten: the builder zeroes or fills a large
// section on several threads (a serial zero fill faults in every page on one thread: ~45 ms of a
// 100k-policy build's 70 MB record stream)
template <class T>
struct RawAlloc : std::allocator<T> {
  RawAlloc() = default;
  template <class U>
  RawAlloc(const RawAlloc<U>&) {}
  template <class U>
  struct rebind { using other = RawAlloc<U>; };
  template <class U>
  void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
using RawWords = std::vector<uint32_t, RawAlloc<uint32_t>>;

// A compiled, immutable policy image (one per policy epoch). Device sections are the vectors
// uploaded verbatim; the rest is host-side metadata for rendering diagnostics. An image read from a
// blob (deserialize) leaves the device-only sections empty (pstream, btab, bfilt, bstream, sctx,
// sbits, svals: dev_len holds their sizes): the host never reads them after the upload.
struct Image {
  uint64_t epoch = 0;
  std::vector<uint32_t> pol, tier_end, code, cpool, gstr_off, hot;  // hot: HOT_WORDS per hot path
  // device policy stream: per policy a record [descriptor (POL_WORDS) | code, padded to 4 words]
  // with PW_CODE relative to the record; records grouped into chunks of <= CHUNK_WORDS words
  // that never cross a tier. chunks: (word offset, words, first policy, end policy) per chunk;
  // tier_cend[t] = end chunk index of tier t.
  RawWords pstream;
  std::vector<uint32_t> chunks, tier_cend;
  std::vector<uint32_t> act;  // action table: (type sid, id sid) pairs of every action entity in scopes
  uint32_t amask_ok = 0;      // 1 when act has <= MAX_ACT entries (PW_AMASK* valid)
  uint32_t n_atomic = 0;      // policies compiled to atoms (statistics)
  uint32_t lane_need = 0;     // most lane-scratch words a bytecode policy uses (image.h LANE_MAX)
  // scope index over atomic policies (image.h "scope index"); indexed = every policy is atomic
  // btab: the scope index's entries, BT_WORDS each (one all-zero entry when it has none). The
  // open-addressed table of btab_slots slots (image.h "scope index") is built on the device from
  // them at load (cedar_btab_build), so blobs and reload broadcasts carry no empty slots.
  RawWords btab, bstream;
  std::vector<uint32_t> bfilt;  // bfilt: key filter, 2 words per block
  // duplicate classes (host side, image.h "duplicate classes"): the members of the class whose
  // representative (lowest member) is policy p are cls_mem[cls_off[p] .. cls_off[p + 1]), ascending;
  // both empty when no two policies share a record. The first pass may report a class by its
  // representative (a reason word with RS_CLASS set), which Batch::reason_ids expands.
  std::vector<uint32_t> cls_off, cls_mem;
  uint32_t btab_slots = 1;
  uint32_t indexed = 0;
  uint32_t combo_mask = 0;  // level-1 key combos in use (bit key_combo(..))
  // entity components of the scope index's level-1 keys, (type sid << 32 | id sid), sorted: the
  // encoder lists a request's ancestors that are among them first (image.h RW_PN)
  std::vector<uint64_t> key_ents;
  // scope bitsets (image.h "scope bitsets"): context table and one row of sbits_words per context
  RawWords sbits;
  std::vector<uint32_t> sctx, svals;  // sbits: (bits, rank) per word; svals: SVAL_WORDS per set bit
  std::vector<uint32_t> sbloom;              // context filter (image.h ctx_bloom_*), 64-bit words
  uint32_t sbits_words = 0;
  uint32_t l2_vmask = 0, l2_lmask = 0;  // hot slots with level-2 value keys / list keys under entity-principal combos
  // index of `uid` in key_ents, KIDX_NONE when it is no key entity
  uint32_t key_index(uint64_t uid) const {
    if (!is_key_ent(uid)) return cgi::KIDX_NONE;
    return (uint32_t)(std::lower_bound(key_ents.begin(), key_ents.end(), uid) - key_ents.begin());
  }
  // static entities (image.h "static entities"): device rows and UID hash; closure rows and
  // direct-parent lists in cpool ([n, (type, id) x n]; ER_ANC / ER_PAD offsets)
  std::vector<uint32_t> srows, shash;
  uint32_t n_static() const { return (uint32_t)srows.size() / cgi::ENT_WORDS; }
  // host lookups, rebuilt by build_lookup
  U64Table sindex;          // UID key -> static row
  U64Table static_targets;  // UIDs some static entity names as a parent (value 0)
  std::vector<uint64_t> key_bloom;  // 1-bit-per-hash prefilter over key_ents
  bool is_static_target(uint64_t uid) const { return static_targets.find(uid) >= 0; }
  int32_t static_row(uint64_t uid) const { return sindex.find(uid); }
  bool is_key_ent(uint64_t uid) const {
    if (key_ents.empty()) return false;
    const uint64_t h = (uid * 0x9E3779B97F4A7C15ull) >> 40;
    if (!((key_bloom[(h >> 6) % key_bloom.size()] >> (h & 63)) & 1)) return false;
    return std::binary_search(key_ents.begin(), key_ents.end(), uid);
  }
  std::vector<uint8_t> gstr_bytes;
  std::vector<PolicyMeta> meta;
  std::vector<std::string> strings;
  std::unordered_map<std::string, uint32_t> sid;
  std::vector<std::string> ext_msgs;
  uint32_t n_tiers() const { return (uint32_t)tier_end.size(); }
  uint32_t n_pol() const { return (uint32_t)meta.size(); }
  uint32_t n_gstr() const { return (uint32_t)strings.size(); }
  uint32_t n_hot() const { return (uint32_t)hot.size() / cgi::HOT_WORDS; }
  // hot slots with set-membership level-2 keys (image.h BT_CKEY): rows then carry n_hot more words
  uint32_t cslot_mask = 0;
  // hot slots with prefix level-2 keys (image.h "prefix level-2 keys") and their prefix lengths,
  // PFX_LENS per hot slot (0 = unused)
  uint32_t pslot_mask = 0;
  std::vector<uint32_t> pfx;
  uint32_t list_mask() const { return cslot_mask | pslot_mask; }
  // hot slots an inline `like` atom reads (image.h AK_LIKEI): rows then carry LIKE_WORDS per slot
  // after the list offsets
  uint32_t lslot_mask = 0;
  uint32_t n_like() const { return (uint32_t)__builtin_popcount(lslot_mask); }
  // hot slots some `like` atom reads (~0: one past slot 31). The device reads a request string's
  // bytes only there when every policy is atomic (bytecode may read any string, ip() / decimal()
  // parse them), so a batch then uploads the bytes of those slots' strings alone (Batch dstr_*)
  uint32_t lread_mask = 0;
  bool dev_all_strings() const { return n_atomic < n_pol() || lread_mask == 0xFFFFFFFFu || n_hot() > 32; }
  // (one list-offset word per slot of list_mask, in slot order: image.h "set-membership keys")
  uint32_t like_off() const { return cgi::RW_HDR + 2 * n_hot() + (uint32_t)__builtin_popcount(list_mask()); }
  uint32_t row_words() const { return (like_off() + cgi::LIKE_WORDS * n_like() + 3) & ~3u; }
  // string -> id over a string_view: open addressing, entries (hash high 32 bits << 32 | id + 1),
  // 0 = empty; size is a power of two. Built by build_lookup once the table is final.
  std::vector<uint64_t> lookup;
  void build_lookup();
  uint64_t cache_id = 0;  // unique per build_lookup (per final image): keys the encoder's caches
  // the encoder's ancestor-record cache (encode_impl.h EncCache), made on first use
  mutable std::shared_ptr<EncCache> enc_cache;
  int32_t find(std::string_view s) const {
    if (lookup.empty()) {
      auto it = sid.find(std::string(s));
      return it == sid.end() ? -1 : (int32_t)it->second;
    }
    const uint64_t h = str_hash(s);
    const uint32_t tag = (uint32_t)(h >> 32);
    const size_t mask = lookup.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const uint64_t v = lookup[i];
      if (!v) return -1;
      if ((uint32_t)(v >> 32) == tag && strings[(uint32_t)v - 1] == s) return (int32_t)((uint32_t)v - 1);
    }
  }
  static uint64_t str_hash(std::string_view s) {  // 8 bytes a step, multiply-xorshift mixing
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (s.size() * 0xC2B2AE3D27D4EB4Full);
    const char* p = s.data();
    size_t n = s.size();
    for (; n >= 8; n -= 8, p += 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      h = (h ^ (w * 0xBF58476D1CE4E5B9ull)) * 0x94D049BB133111EBull;
      h ^= h >> 31;
    }
    if (n) {
      uint64_t w = 0;
      std::memcpy(&w, p, n);
      h = (h ^ (w * 0xBF58476D1CE4E5B9ull)) * 0x94D049BB133111EBull;
      h ^= h >> 31;
    }
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
  }
  std::vector<uint8_t> serialize() const;
  uint8_t* serialize_malloc(size_t* len) const;  // the blob in one malloc'd buffer (cg_free)
  size_t blob_size() const;
  void serialize_into(uint8_t* out) const;  // blob_size() bytes; large sections on several threads
  void write_blob(void* writer) const;
  // device region of the blob this image was read from (image.h DevSection): section offsets and
  // byte sizes, and the region's bounds (blob offsets)
  uint64_t dev_off[cgi::DS_COUNT] = {}, dev_len[cgi::DS_COUNT] = {};
  uint64_t dev_begin = 0, dev_end = 0;
  uint64_t blob_len = 0;  // the blob's size (deserialize)
  static std::shared_ptr<Image> deserialize(const uint8_t* p, size_t n);
};

// One document (a policy file / CRD content / AVP statement) inside a tier.
struct DocSpec {
  std::string filename, text, id_prefix, id_suffix;
  std::string explicit_id;  // when set: the document holds exactly one policy with this ID
  bool zero_position = false;  // policies built from AST (e.g. allow-all-admission) carry Position{}
  // a document that does not parse is left out of the build and reported (the directory / CRD /
  // AVP stores log and skip it: directory.go:69-73, crd.go:51-55,91-95,
  // verified_permissions.go:89-93); else it fails the build (cedar.NewPolicySetFromBytes, memory.go:18)
  bool skip_invalid = false;
};
struct DocError {
  std::string filename, error;
};

// Parsed documents kept across builds (the incremental compiler): a rebuild after a store change
// parses only the documents whose (filename, text) it has not seen; the rest reuse their ASTs.
// Entries a build does not use are dropped after it.
struct ParseCache {
  struct Entry {
    std::string filename, text;
    std::shared_ptr<const std::vector<Policy>> policies;
    uint64_t used = 0;  // generation of the last build that used it
  };
  std::unordered_map<uint64_t, std::vector<Entry>> map;  // by hash of (filename, text)
  uint64_t generation = 0;
  uint64_t hits = 0, misses = 0;  // over the last build
};

// Entity input for the encoder (already decoded from JSON or built by the k8s model).
struct EntityIn {
  std::string type, id;
  HVal attrs;  // Record
  std::vector<std::pair<std::string, std::string>> parents;
};

// Lowered documents kept across builds (the incremental compiler, compiler.cpp): a full build
// records every document's lowered policies against persistent arenas (string table, code,
// constant pool, action table); a later build lowers only the documents it has not seen and
// copies the rest, as long as the image-wide choices it made stay valid (the hot attribute paths,
// the action table within MAX_ACT, the static entities). Otherwise, or once the arenas hold more
// garbage than live words, the build is a full one again.
struct LowerState;
struct LowerDeleter { void operator()(LowerState* s) const; };
std::unique_ptr<LowerState, LowerDeleter> make_lower_state();
struct BuildInfo {
  bool incremental = false;      // the last build copied cached documents' lowered policies
  uint64_t lowered = 0;          // policies it lowered
  uint64_t reused = 0;           // policies it copied from the cache
  const char* why_full = "";     // a full build's reason (first build, hot paths, actions, ...)
};

// Compiles the tiers. With a cache, unseen documents are parsed on worker threads and reused
// next time; without `inc` the image is byte-identical to a build without the cache. `statics`:
// the image's static entities (cg_compiler_set_entities), `statics_gen` their version. With `inc`
// a build after a document change lowers only the changed documents: its image decides every
// request as a fresh build would, but its arenas keep the removed documents' words (not byte-
// identical to a fresh build).
std::shared_ptr<Image> compile_image(const std::vector<std::vector<DocSpec>>& tiers, uint64_t epoch,
                                     ParseCache* cache = nullptr, const std::vector<EntityIn>* statics = nullptr,
                                     std::vector<DocError>* skipped = nullptr, LowerState* inc = nullptr,
                                     uint64_t statics_gen = 0, BuildInfo* info = nullptr);
struct RequestIn {
  std::pair<std::string, std::string> principal, action, resource;
  HVal context;  // Record
};

// One request encoded position-independently, so that any thread can encode it and a batch
// appends it with plain copies: heap references are block-relative, and strings absent from the
// image's table are numbered request-locally (id n_gstr + j names strs[j]; the device adds the
// request's string base, stored at RH_SBASE when the block is appended).
struct EncodedRequest {
  std::vector<uint32_t> blk, row;  // heap block; columnar row (RW_BLK set on append)
  // Ancestor lists ([n, (type, id) x n] + the key-entity indices of a scope-bitset image), kept out
  // of the block: record k starts at anc[anc_at[k]]. The block's ER_ANC words and the row's
  // RW_*ANC words name records (k, and k + 1 with 0 = none) until Batch::append interns each
  // record in the batch heap (one copy per distinct list) and points them at it.
  std::vector<uint32_t> anc, anc_at;
  std::vector<uint64_t> anc_hash;  // per record: its content hash when known (a cached record), else 0
  // grouping key (group.hip): (action, resource type) | principal key ancestors | hot values,
  // hashed fields of the row, most significant first; the device bucket-sorts on its top bits
  uint32_t gkey = 0;
  std::vector<std::string> strs;   // request-local strings (few per request: found by linear scan)
  std::vector<uint8_t> str_dev;    // per string: its bytes are read on the device (Image::lread_mask)
  static constexpr size_t STRS_SCAN = 16;
  std::unordered_multimap<uint64_t, uint32_t> strs_ix;  // str_hash -> index, once strs outgrows STRS_SCAN
  // interning memo over the source bytes' address: a value repeated from the same bytes (a group
  // name as entity id, parent and attribute; a type-name literal) is looked up once
  static constexpr uint32_t MEMO = 32;
  const char* memo_p[MEMO];
  uint32_t memo_len[MEMO], memo_id[MEMO], n_memo = 0;
  void clear() { blk.clear(); row.clear(); anc.clear(); anc_at.clear(); anc_hash.clear(); strs.clear(); str_dev.clear(); strs_ix.clear(); n_memo = 0; }
  // words of record k / the first pair of the list a row word (k + 1) names
  const uint32_t* anc_rec(uint32_t k) const { return anc.data() + anc_at[k]; }
  const uint32_t* anc_pairs(uint32_t row_word) const { return anc_rec(row_word - 1) + 1; }
};
// Encodes (EntityMap, Request) for `img`. Thread-safe: reads the image only.
void encode_request(const Image& img, const std::vector<EntityIn>& ents, const RequestIn& req, EncodedRequest& out);
// The webhook's host steps for one SubjectAccessReview JSON body (GetAuthorizerAttributes,
// Authorize's fast paths, RecordToCedarResource, encode_request) without intermediate trees.
// Returns 1 with `out` encoded, 2 with a fast-path decision in fast/reason, or 0 when the body
// uses something this path does not take (escapes, numbers, duplicate keys, malformed JSON ...):
// the caller then runs the general path, which gives the identical encoding or error.
int encode_sar_direct(const Image& img, const char* json, size_t n, EncodedRequest& out, int& fast, std::string& reason);

// Host side of a device batch: encoded request heap + string table; results after evaluation.
struct Batch {
  std::shared_ptr<const Image> img;
  PinVec<uint32_t> heap, req_base;
  PinVec<uint32_t> rows;  // columnar request rows (image.h RowW), row_words each
  PinVec<uint32_t> gkeys;  // one grouping key per request (EncodedRequest::gkey)
  uint32_t row_words = 0;
  // request-local strings of every request, appended as requests arrive: string j is
  // bstr_bytes[bstr_off[j] .. bstr_off[j + 1]) (bstr_off keeps a trailing end offset)
  PinVec<uint32_t> bstr_off{0};
  PinVec<uint8_t> bstr_bytes;
  uint32_t n_bstr() const { return (uint32_t)bstr_off.size() - 1; }
  // the device's copy of the table when the image reads few strings (Image::dev_all_strings false):
  // the same numbering, and bytes only for the strings a `like` atom reads (the rest empty); the
  // host renders diagnostics from the full table above
  bool dstr = false;
  PinVec<uint32_t> dstr_off{0};
  PinVec<uint8_t> dstr_bytes;
  const PinVec<uint32_t>& dev_str_off() const { return dstr ? dstr_off : bstr_off; }
  const PinVec<uint8_t>& dev_str_bytes() const { return dstr ? dstr_bytes : bstr_bytes; }
  // Interned ancestor lists (EncodedRequest::anc): content hash -> heap offset of the copy that
  // later blocks reference (image.h "ancestor lists"). Requests of one principal share one list,
  // so a batch carries each distinct list once and grouped neighbours read the same lines.
  // (open addressing over one array, so a part's memo is one block, not a node per list: freeing
  // thousands of nodes after every bulk encode left the allocator's bins to sort on the next
  // large allocation, 50-90 us on the serving path)
  PodVec<uint64_t> memo;  // (hash | 1) << 0 in the even word, heap offset in the odd one; 0: empty
  size_t memo_used = 0;
  uint64_t anc_words = 0, anc_shared_words = 0;  // list words appended / list words served by a copy
  uint32_t intern_list(const uint32_t* w, uint32_t n, uint64_t room, uint64_t hash = 0);
  // results
  uint32_t capr = 8, cape = 4;
  // on-device follow-up sizing (device.h FuKind), from the previous batch on the same image:
  // entries wanted per worklist (0: the default) and reasons per FU_BIG entry (0: 256)
  uint32_t fu_want[3] = {0, 0, 0};
  uint32_t fu_capr_hint = 0, fu_capr_gen_hint = 0;  // reasons per FU_BIG / FU_GEN entry (0: default)
  // the batching layer's locality order is computed on the device inside each step (group.hip)
  bool dev_group = false;
  bool prof = false;  // cg_batch_set_profile: device events around the upload, the step and the download
  // first-pass results, read in place from the batch's pinned staging block (device.h DevBatch;
  // valid while the batch lives): res[2i], [2i+1] per request, capr reasons of each effect, cape
  // error records. res is written back by overflow re-runs.
  uint32_t* res = nullptr;
  const uint32_t *reasons_f = nullptr, *reasons_p = nullptr, *errs = nullptr;
  // Results are laid out by position in the device's launch order (device.h DevBatch::res): request
  // i's slot is pos_of[i] for a batch grouped on the device, else i. Everything indexed by slot
  // (res, the lists, bigs, the worklists' and re-runs' ids) uses positions; only the accessors
  // below take request indices.
  const uint32_t* pos_of = nullptr;
  uint32_t slot(uint32_t i) const { return pos_of ? pos_of[i] : i; }
  // per-request overflow re-run results (index -> reasons / errors)
  // Re-run results: request i's reason / error list read in place from the re-run's pinned result
  // block, which the owning cg_batch keeps until it is destroyed (big stays empty until a re-run
  // fills one; ptr null = the first pass's lists).
  // the on-device follow-up worklists (device.h DevBatch::fu_*), read in the pinned block
  struct FollowUp {
    const uint32_t *ids = nullptr, *res = nullptr, *rf = nullptr, *rp = nullptr, *er = nullptr;
    uint32_t cap = 0, capr = 0, cape = 0;
  } fu[3];
  // requests each worklist's gather found (may exceed cap); [FU_KINDS]: requests whose key-entity
  // indices were not the image's (device.h DevBatch::fu_cnt)
  const uint32_t* fu_cnt = nullptr;
  struct BigRef { const uint32_t *r = nullptr, *e = nullptr; uint32_t nr = 0, ne_words = 0; };
  std::vector<BigRef> bigs;      // lists held outside the first pass's slots
  std::vector<uint32_t> big_ix;  // per slot: 1 + its index in bigs, or 0 (empty: none)
  const BigRef* big_of(uint32_t p) const { return (!big_ix.empty() && big_ix[p]) ? &bigs[big_ix[p] - 1] : nullptr; }
  void set_big(uint32_t p, const uint32_t* reasons, uint32_t nr, const uint32_t* errs, uint32_t nerr_words);

  uint32_t n() const { return (uint32_t)req_base.size(); }
  // string `id` as request i sees it
  std::string str(uint32_t i, uint32_t id) const;
  void add(const std::vector<EntityIn>& ents, const RequestIn& req);  // encode_request + append
  void append(EncodedRequest& e);                                     // moves e's strings
  // Appends whole batches encoded on other threads (same image), in order: each part's heap, rows,
  // grouping keys and strings are copied at their offsets and its block-relative words stay valid
  // (request bases, RW_BLK and RH_SBASE are shifted). `threads` copy the parts side by side.
  void concat(std::vector<Batch>& parts, unsigned threads);
  void finalize_strings();
  // (by request index i) decision: 1 allow, 0 deny; the deciding tier; the Go-JSON rendering of
  // the cedar.Diagnostic
  bool decision(uint32_t i) const;
  uint32_t tier(uint32_t i) const;
  void diagnostic_json(uint32_t i, std::string& out, bool reasons_only) const;
  void reason_ids(uint32_t i, std::vector<uint32_t>& out) const;
  void error_recs(uint32_t i, std::vector<uint32_t>& out) const;
  std::string error_message(uint32_t i, const uint32_t* rec) const;
};

// Parses a Cedar-JSON request item {"entities": [...], "request": {...}} into encoder input.
void decode_json_item(const JVal& item, std::vector<EntityIn>& ents, RequestIn& req);
// Parses a Cedar-JSON entity array.
void decode_json_entities(const JVal& arr, std::vector<EntityIn>& ents);

}  // namespace cg
