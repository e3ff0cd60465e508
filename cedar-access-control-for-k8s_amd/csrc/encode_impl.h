// The request encoder's one implementation, shared by the general path (EntityIn / HVal trees
// decoded from Cedar JSON or built by sar.cpp) and the direct SubjectAccessReview path (views
// into the request body), so both produce the same words for the same (EntityMap, Request).
//
// Source interface (Src):
//   uint32_t n_ents();  std::string_view type(i), id(i);
//   uint32_t n_parents(i);  std::pair<sv, sv> parent(i, k);
//   std::pair<sv, sv> principal(), action(), resource();
//   void emit_ctx(out, img, E, w0, w1);  void emit_attrs(i, out, img, E, w0, w1);
//     (emit the context / entity attributes record into `out` exactly as emit_heap_value does)
#pragma once
#include <algorithm>
#include <mutex>
#include <memory>
#include <atomic>
#include <cstdlib>
#include <string_view>
#include <unordered_map>
#include <unordered_set>

#include "engine.h"

namespace cg {

uint32_t request_sid(const Image& img, EncodedRequest& e, std::string_view s);
uint64_t list_hash(const uint32_t* w, uint32_t n);  // an ancestor-list record's content hash (encoder.cpp)

namespace enc {
using namespace cgi;

// memory-form record lookup (the device's rec_get, on the host): the record lives in the emitted
// request block or, for a static entity's attributes, in the image's constant pool
inline bool blk_rec_get(const std::vector<uint32_t>& blk, const std::vector<uint32_t>& cpool, uint32_t rw0, uint32_t n,
                        uint32_t key, uint32_t& w0, uint32_t& w1) {
  const uint32_t off = rw0 & OFF_MASK;
  const std::vector<uint32_t>& m = ((rw0 & X_MASK) >> SPACE_SHIFT) == SP_CPOOL ? cpool : blk;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (m[off + 1 + 3 * mid] < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && m[off + 1 + 3 * lo] == key) {
    w0 = m[off + 2 + 3 * lo];
    w1 = m[off + 3 + 3 * lo];
    return true;
  }
  return false;
}

// element hash (image.h chash_*) of a memory-form value held in the block or the constant pool:
// primitives canonically, records over (key sid, primitive field hash) in key order; anything else
// by its tag (no set-membership key has such an element)
inline uint32_t mem_chash(const std::vector<uint32_t>& blk, const std::vector<uint32_t>& cpool, uint32_t w0, uint32_t w1,
                          bool nested = false) {
  auto mem = [&](uint32_t x) -> const uint32_t* {
    return ((x >> SPACE_SHIFT) == SP_CPOOL ? cpool.data() : blk.data()) + (x & OFF_MASK);
  };
  const uint32_t tag = w0 >> TAG_SHIFT;
  switch (tag) {
    case T_BOOL: case T_STR: return chash_prim(tag, w1, 0);
    case T_LONG: return chash_prim(T_LONG, w1, (int32_t)w1 < 0 ? 0xFFFFFFFFu : 0u);
    case T_LONGREF: { const uint32_t* q = mem(w0 & X_MASK); return chash_prim(T_LONG, q[0], q[1]); }
    case T_ENT: return chash_prim(T_ENT, w0 & X_MASK, w1);
    case T_REC: {
      if (nested) break;
      const uint32_t* q = mem(w0 & X_MASK);
      uint32_t h = chash_mix(CHASH_REC, q[0]);
      for (uint32_t j = 0; j < q[0]; j++) h = chash_mix(chash_mix(h, q[1 + 3 * j]), mem_chash(blk, cpool, q[2 + 3 * j], q[3 + 3 * j], true));
      return h;
    }
    default: break;
  }
  return chash_prim(tag, 0, 0);
}

// [n, (type, id) x n] list at cpool[off] as UID keys
inline void cpool_uids(const Image& img, uint32_t off, std::vector<uint64_t>& out) {
  const uint32_t n = img.cpool[off];
  for (uint32_t k = 0; k < n; k++) out.push_back(((uint64_t)img.cpool[off + 1 + 2 * k] << 32) | img.cpool[off + 2 + 2 * k]);
}

// Orders an ancestor list for the probe kernel (image.h RW_PN): scope-index key entities first,
// each part sorted; returns how many lead.
inline uint32_t order_ancestors(const Image& img, std::vector<uint64_t>& anc) {
  if (!img.indexed) {
    std::sort(anc.begin(), anc.end());
    return 0;
  }
  auto mid = std::partition(anc.begin(), anc.end(), [&](uint64_t u) { return img.is_key_ent(u); });
  std::sort(anc.begin(), mid);
  std::sort(mid, anc.end());
  return (uint32_t)(mid - anc.begin());
}

inline uint32_t mem_tname(uint32_t w0) {
  switch (w0 >> TAG_SHIFT) {
    case T_BOOL: return TN_BOOL;
    case T_LONG: case T_LONGREF: return TN_LONG;
    case T_STR: return TN_STRING;
    case T_ENT: return TN_ENTITY;
    case T_SET: return TN_SET;
    case T_REC: return TN_RECORD;
    case T_DEC: return TN_DECIMAL;
    case T_IP: return TN_IP;
    default: return TN_UNKNOWN;
  }
}

inline uint64_t uid_key(uint32_t t, uint32_t id) { return ((uint64_t)t << 32) | id; }

// UID -> entity-table index: a linear scan for the few entities of a webhook request, a hash
// map beyond that.
struct UidIndex {
  std::vector<uint64_t> keys;
  std::unordered_map<uint64_t, uint32_t> map;
  int32_t find(uint64_t k) const {
    if (map.empty()) {
      for (size_t i = 0; i < keys.size(); i++)
        if (keys[i] == k) return (int32_t)i;
      return -1;
    }
    auto it = map.find(k);
    return it == map.end() ? -1 : (int32_t)it->second;
  }
  void add(uint64_t k) {
    keys.push_back(k);
    if (!map.empty()) map.emplace(k, (uint32_t)keys.size() - 1);
    else if (keys.size() > 32)
      for (size_t i = 0; i < keys.size(); i++) map.emplace(keys[i], (uint32_t)i);
  }
};

// An ancestor-list record (EncodedRequest::anc) of `owner` over the ancestor set `anc` (any order,
// no repeats): [n, (type, id) x n] in order_ancestors order, then on a scope-bitset image the key-
// entity index of the owner and of each leading key ancestor. Returns the key-ancestor count.
inline uint32_t make_record(const Image& img, uint64_t owner, std::vector<uint64_t>& anc, std::vector<uint32_t>& out) {
  const uint32_t keys = order_ancestors(img, anc);
  out.push_back((uint32_t)anc.size());
  for (const uint64_t a : anc) { out.push_back((uint32_t)(a >> 32)); out.push_back((uint32_t)a); }
  if (img.sbits_words) {
    out.push_back(img.key_index(owner));
    for (uint32_t j = 0; j < keys; j++) out.push_back(img.key_index(anc[j]));
  }
  return keys;
}

}  // namespace enc

// Per-image cache of ancestor-list records for the common request shape (a SubjectAccessReview's
// user with its groups, over a static group hierarchy): a table entity without request-given
// parents has its static closure row as ancestry (or none), and an entity whose request-given
// parents have none of their own has the union of its parents' closures. Both are pure functions of
// the image and, for the latter, of (entity, merged parent list), so every encoding thread shares
// one computation of each: static rows are published once (compare-and-swap), the rest live in a
// sharded map under per-shard locks. The image holds the cache (Image::enc_cache).
struct EncCache {
  struct Rec {
    std::vector<uint32_t> words;
    uint32_t keys = 0;
    uint64_t hash = 0;  // list_hash(words): Batch::append interns the record without rehashing it
  };
  std::unique_ptr<std::atomic<const Rec*>[]> srec;  // static row -> record (null: not built yet)
  size_t n_static = 0;
  struct Ent {
    uint64_t uid = 0;
    std::vector<uint64_t> parents;
    Rec rec;
  };
  static constexpr uint32_t SHARDS = 64;
  static constexpr size_t MAX_PER_SHARD = 4096;
  struct alignas(64) Shard {
    std::mutex mu;
    std::unordered_map<uint64_t, Ent> map;  // by hash of (uid, parents)
  } shards[SHARDS];
  explicit EncCache(size_t ns) : srec(new std::atomic<const Rec*>[ns ? ns : 1]), n_static(ns) {
    for (size_t i = 0; i < ns; i++) srec[i].store(nullptr, std::memory_order_relaxed);
  }
  ~EncCache() {
    for (size_t i = 0; i < n_static; i++) delete srec[i].load();
  }
};
// (per thread, the last image's cache without touching the shared_ptr: libstdc++'s atomic
// shared_ptr operations take a mutex from a small address-hashed pool, one and the same for every
// thread encoding against one image, and copying the pointer bounces its reference count between
// the cores; the thread keeps its own reference until it encodes against another image)
inline EncCache& enc_cache(const Image& img) {
  thread_local uint64_t t_id = 0;
  thread_local std::shared_ptr<EncCache> t_keep;
  if (t_keep && img.cache_id && t_id == img.cache_id) return *t_keep;
  std::shared_ptr<EncCache> p = std::atomic_load(&img.enc_cache);
  if (!p) {
    auto n = std::make_shared<EncCache>(img.n_static());
    if (std::atomic_compare_exchange_strong(&img.enc_cache, &p, n)) p = n;  // (else p: the winner's)
  }
  t_keep = p;
  t_id = img.cache_id;
  return *p;
}
namespace enc {
// set on a thread to encode with the general walk only (cg_encode_sar_check compares the two)
inline thread_local bool t_no_closure_cache = false;
inline bool closure_cache_on() {
  static const bool on = !(std::getenv("CEDARGPU_CLOSURE_CACHE") && *std::getenv("CEDARGPU_CLOSURE_CACHE") == '0');
  return on;
}

// The encoder's working lists, kept per thread so that a request costs no allocations once a
// thread has encoded a few (each call clears them; capacities stay).
struct Scratch {
  std::vector<uint32_t> table, n_key, hs;
  UidIndex index;
  std::vector<std::vector<uint64_t>> parents;
  std::unordered_set<uint64_t> seen_p, seen_big;
  std::vector<uint64_t> anc, nodes, cl, sp, extended;
  std::vector<uint32_t> attrs;  // a table entity's attributes emitted for the static comparison
  void reset() {
    table.clear(); n_key.clear(); hs.clear(); attrs.clear();
    index.keys.clear(); index.map.clear();
    for (auto& p : parents) p.clear();
    seen_p.clear(); seen_big.clear();
    anc.clear(); nodes.clear(); cl.clear(); sp.clear(); extended.clear();
  }
};
inline Scratch& scratch() {
  thread_local Scratch s;
  return s;
}

// CEDARGPU_STATIC_ELIDE=0 keeps every request entity in the table (A/B, tests)
inline bool static_elide_on() {
  static const bool on = [] { const char* e = std::getenv("CEDARGPU_STATIC_ELIDE"); return !(e && *e == '0'); }();
  return on;
}

// a request entity's attributes (record w0, w1 emitted into `m`) equal a static entity's (record
// sw0, sw1 in the constant pool) field for field, every field an inline primitive (bool, string,
// small long, entity UID): equal words are then equal values
inline bool static_attrs_equal(const Image& img, uint32_t sw0, uint32_t sw1, const std::vector<uint32_t>& m, uint32_t w0,
                               uint32_t w1) {
  if ((sw0 >> TAG_SHIFT) != T_REC || (w0 >> TAG_SHIFT) != T_REC || sw1 != w1) return false;
  if (((sw0 & X_MASK) >> SPACE_SHIFT) != SP_CPOOL || ((w0 & X_MASK) >> SPACE_SHIFT) != SP_HEAP) return false;
  const uint32_t so = sw0 & OFF_MASK, ro = w0 & OFF_MASK;
  if ((size_t)so + 1 + 3 * (size_t)sw1 > img.cpool.size() || (size_t)ro + 1 + 3 * (size_t)w1 > m.size()) return false;
  for (uint32_t j = 0; j < w1; j++) {
    const uint32_t* a = &img.cpool[so + 1 + 3 * j];
    const uint32_t* b = &m[ro + 1 + 3 * j];
    const uint32_t tag = a[1] >> TAG_SHIFT;
    if (tag != T_BOOL && tag != T_STR && tag != T_LONG && tag != T_ENT) return false;
    if (a[0] != b[0] || a[1] != b[1] || a[2] != b[2]) return false;
  }
  return true;
}

// CEDARGPU_HOST_CTX=0: the scan looks every request's contexts up itself (A/B)
inline bool host_ctx_on() {
  static const bool on = [] { const char* e = std::getenv("CEDARGPU_HOST_CTX"); return !(e && *e == '0'); }();
  return on;
}

// The request's scope contexts (image.h RH_SCTX), looked up in the image's context table exactly as
// cedar_scan_kernel's bitset pass would: per entity-principal combo its level-1 context, one per
// value slot of l2_vmask with the request's value, one per element (or marker) of each list slot
// of l2_lmask. Written only when the scan would take its bitset path with these contexts (the SAR
// shape: at most one action / resource key entity, a principal list, at most CTX_CAP contexts) and
// at most CTXR_SLOTS of them exist; the row's RW_ASELF then carries ASELF_CTXR.
inline void resolve_contexts(const Image& img, EncodedRequest& E) {
  std::vector<uint32_t>& blk = E.blk;
  uint32_t* row = E.row.data();
  for (uint32_t k = 0; k < CTXR_SLOTS; k++) blk[RH_SCTX + k] = CTXR_EMPTY;
  const size_t slots = img.sctx.size() / SCTX_WORDS;
  if (!host_ctx_on() || !img.indexed || !img.sbits_words || slots < 2 || !row[RW_PANC]) return;
  const uint32_t cm = img.combo_mask;
  uint32_t pe = 0, ae = 0, re = 0;  // combos with an entity principal / action / resource component
  for (uint32_t cb = 0; cb < 32; cb++) {
    if ((cb & 3) == KC_ENT) pe |= 1u << cb;
    if (((cb >> 2) & 1) == KC_ENT) ae |= 1u << cb;
    if ((cb >> 3) == KC_ENT) re |= 1u << cb;
  }
  pe &= cm;
  const uint32_t pn = row[RW_PN], an = row[RW_AN], rn = row[RW_RN];
  auto nkeys = [](uint32_t w) { return (w >> 31) + ((w >> AN_KEYS_SHIFT) & AN_KEYS); };
  const uint32_t nP = nkeys(pn), nA = nkeys(an), nR = nkeys(rn);
  if (!pe || !((!(cm & ae) || nA <= 1) && (!(cm & re) || nR <= 1) && nP < 2048)) return;
  // the action / resource component of the keys: the UID when it is a key entity, else its one key
  // ancestor (the first of its list)
  auto key1 = [&](uint32_t n, uint32_t w_n, uint32_t w_anc, uint32_t t, uint32_t i) -> std::pair<uint32_t, uint32_t> {
    if (n != 1) return {KW_ANY, KW_ANY};
    if (row[w_n] & AN_SELF) return {t, i};
    const uint32_t* l = E.anc_pairs(row[w_anc]);
    return {l[0], l[1]};
  };
  const auto ka1 = key1(nA, RW_AN, RW_AANC, row[RW_A], row[RW_A + 1]);
  const auto kr1 = key1(nR, RW_RN, RW_RANC, row[RW_R], row[RW_R + 1]);
  const uint32_t nh = img.n_hot(), vm = img.l2_vmask, lm = img.l2_lmask, hl = img.list_mask();
  // per combo: level 1, the value slots, the list entries (CTX_CAP in all at most)
  struct Key { uint32_t hs, v0, v1; };
  Key keys[CTX_CAP];
  uint32_t per = 1;
  keys[0] = {SCTX_L1, 0u, 0u};
  for (uint32_t m = vm; m; m &= m - 1) {
    const uint32_t h = (uint32_t)__builtin_ctz(m);
    const uint32_t w0 = row[RW_HDR + 2 * h], w1 = row[RW_HDR + 2 * h + 1];
    const bool ok = (w0 >> TAG_SHIFT) != T_NONE;
    if (per < CTX_CAP) keys[per] = {h, ok ? w0 : MISSING_W0, ok ? w1 : 0u};
    per++;
  }
  for (uint32_t m = lm; m && hl; m &= m - 1) {
    const uint32_t h = (uint32_t)__builtin_ctz(m);
    const uint32_t lo = row[RW_HDR + 2 * nh + (uint32_t)__builtin_popcount(hl & ((1u << h) - 1u))];
    const uint32_t hd = blk[lo];
    if (hd & 0x80000000u) {
      if (per < CTX_CAP) keys[per] = {h | BT_CKEY, hd == CL_MISSING ? MISSING_W0 : NOTSET_W0, 0u};
      per++;
    } else {
      for (uint32_t e = 0; e < hd; e++) {
        if (per < CTX_CAP) keys[per] = {h | BT_CKEY, blk[lo + 1 + e], 1u};
        per++;
      }
    }
  }
  if ((uint64_t)__builtin_popcount(pe) * per > CTX_CAP) return;  // the scan enumerates this request's keys
  uint32_t found[CTXR_SLOTS], nf = 0;
  for (uint32_t m = pe; m; m &= m - 1) {
    const uint32_t cb = (uint32_t)__builtin_ctz(m);
    const auto q = ((cb >> 2) & 1) == KC_ENT ? ka1 : std::make_pair(KW_ANY, KW_ANY);
    const uint32_t rkc = cb >> 3;
    const auto r = rkc == KC_ENT ? kr1 : rkc == KC_TYPE ? std::make_pair(row[RW_R], KW_ANY) : std::make_pair(KW_ANY, KW_ANY);
    const uint32_t pre = key_pre(cb, q.first, q.second, r.first, r.second);
    for (uint32_t t = 0; t < per; t++) {
      const Key& k = keys[t];
      const uint32_t w0c = ctx_w0(cb, k.hs);
      for (size_t h = ctx_key(pre, k.hs, k.v0, k.v1) & (slots - 1);; h = (h + 1) & (slots - 1)) {
        const uint32_t* x = &img.sctx[h * SCTX_WORDS];
        if (!x[0]) break;
        if (x[0] == w0c && x[1] == q.first && x[2] == q.second && x[3] == r.first && x[4] == r.second && x[5] == k.v0 &&
            x[6] == k.v1) {
          if (nf == CTXR_SLOTS || x[7] >= (1u << (32 - CTXR_ROW))) return;  // (more than the block holds)
          found[nf++] = cb | (x[7] << CTXR_ROW);
          break;
        }
      }
    }
  }
  for (uint32_t k = 0; k < nf; k++) blk[RH_SCTX + k] = found[k];
  row[RW_ASELF] |= ASELF_CTXR;
}

inline void emit_empty_record(std::vector<uint32_t>& out, uint32_t& w0, uint32_t& w1) {
  const uint32_t off = (uint32_t)out.size();
  out.push_back(0);
  w0 = mk_w0(T_REC, mk_ref(SP_HEAP, off));
  w1 = 0;
}

}  // namespace enc

template <class Src>
void encode_impl(const Image& img, const Src& src, EncodedRequest& E) {
  using namespace enc;
  E.clear();
  auto sid = [&](std::string_view s) { return request_sid(img, E, s); };
  std::vector<uint32_t>& blk = E.blk;
  // entity table (EntityMap semantics: a repeated UID replaces the earlier entity)
  Scratch& S = scratch();
  S.reset();
  std::vector<uint32_t>& table = S.table;  // source entity of each table slot
  UidIndex& index = S.index;
  const uint32_t n_in = src.n_ents();
  for (uint32_t e = 0; e < n_in; e++) {
    const uint32_t t = sid(src.type(e)), id = sid(src.id(e));
    const uint64_t k = uid_key(t, id);
    const int32_t at = index.find(k);
    if (at >= 0) { table[(size_t)at] = e; continue; }
    index.add(k);
    table.push_back(e);
  }
  auto uid_of = [&](const std::pair<std::string_view, std::string_view>& u) {
    const uint32_t t = sid(u.first);
    return std::make_pair(t, sid(u.second));
  };
  // parent adjacency (ids of parents that exist in the map are followed; absent ones are leaves)
  std::vector<std::vector<uint64_t>>& parents = S.parents;
  if (parents.size() < table.size()) parents.resize(table.size());
  std::unordered_set<uint64_t>& seen_p = S.seen_p;  // a parent list past DEDUP_SCAN entries dedups by hashing
  auto add_parent = [&](std::vector<uint64_t>& l, uint64_t key) {
    if (l.size() < DEDUP_SCAN) {
      if (std::find(l.begin(), l.end(), key) == l.end()) l.push_back(key);
      return;
    }
    if (l.size() == DEDUP_SCAN || seen_p.empty()) seen_p = std::unordered_set<uint64_t>(l.begin(), l.end());
    if (seen_p.insert(key).second) l.push_back(key);
  };
  for (uint32_t i = 0; i < table.size(); i++) {
    const uint32_t np = src.n_parents(table[i]);
    seen_p.clear();
    for (uint32_t k = 0; k < np; k++) {
      const auto u = uid_of(src.parent(table[i], k));
      add_parent(parents[i], uid_key(u.first, u.second));
    }
  }
  // Static entities merged into the map (image.h "static entities"). A table entity that is also
  // static gains the static parents. A static entity outside the table keeps its compiled closure
  // row, which is its merged ancestry unless that row names a table entity with parents of its own
  // (the request extends the hierarchy above it): such static entities join the table (rare: the
  // SAR path gives only the principal parents, and no static edge names a principal).
  const bool has_static = img.n_static() != 0;
  constexpr uint32_t FROM_STATIC = 0x80000000u;  // table slot holding static row (slot & ~FROM_STATIC)
  if (has_static) {
    const uint32_t n0 = (uint32_t)table.size();
    std::vector<uint64_t>& extended = S.extended;  // table entities with parents that some static edge names
    for (uint32_t i = 0; i < n0; i++)
      if (!parents[i].empty() && img.is_static_target(index.keys[i])) extended.push_back(index.keys[i]);
    if (!extended.empty()) {
      std::sort(extended.begin(), extended.end());
      std::vector<uint64_t> cl;
      for (uint32_t s = 0; s < img.n_static(); s++) {
        const uint32_t* r = &img.srows[(size_t)s * ENT_WORDS];
        const uint64_t k = uid_key(r[ER_TYPE], r[ER_ID]);
        if (index.find(k) >= 0) continue;
        cl.clear();
        cpool_uids(img, r[ER_ANC] & OFF_MASK, cl);
        bool hit = false;
        for (size_t a = 0; a < cl.size() && !hit; a++) hit = std::binary_search(extended.begin(), extended.end(), cl[a]);
        if (!hit) continue;
        index.add(k);
        table.push_back(FROM_STATIC | s);
        if (parents.size() < table.size()) parents.resize(table.size());  // (a cleared list from the scratch)
      }
    }
    for (uint32_t i = 0; i < table.size(); i++) {
      const int32_t s = (table[i] & FROM_STATIC) ? (int32_t)(table[i] & ~FROM_STATIC) : img.static_row(index.keys[i]);
      if (s < 0) continue;
      std::vector<uint64_t>& sp = S.sp;
      sp.clear();
      cpool_uids(img, img.srows[(size_t)s * ENT_WORDS + ER_PAD], sp);
      seen_p.clear();
      for (const uint64_t p : sp) add_parent(parents[i], p);
    }
  }
  const auto pu = uid_of(src.principal()), au = uid_of(src.action()), ru = uid_of(src.resource());
  // A table entity that merges to exactly its static entity (no parents of its own, attributes equal
  // to the static ones field for field) leaves the table: lookups of its UID then find the static
  // row, whose attributes and closure row are what the merge would give. (The SAR path's group
  // entities, {name} with no parents, over a static group hierarchy: ~140 B per request.) P / A / R
  // stay, and only records of inline primitives are compared.
  if (has_static && static_elide_on()) {
    const uint64_t pk = uid_key(pu.first, pu.second), ak = uid_key(au.first, au.second), rk = uid_key(ru.first, ru.second);
    uint32_t kept = 0;
    bool dropped = false;
    for (uint32_t i = 0; i < (uint32_t)table.size(); i++) {
      const uint64_t k = index.keys[i];
      bool elide = false;
      if (!(table[i] & FROM_STATIC) && k != pk && k != ak && k != rk && src.n_parents(table[i]) == 0) {
        const int32_t s = img.static_row(k);
        if (s >= 0) {
          const uint32_t* sr = &img.srows[(size_t)s * ENT_WORDS];
          S.attrs.clear();
          uint32_t w0, w1;
          src.emit_attrs(table[i], S.attrs, img, E, w0, w1);
          elide = static_attrs_equal(img, sr[ER_ATTR0], sr[ER_ATTR1], S.attrs, w0, w1);
        }
      }
      if (elide) { dropped = true; continue; }
      table[kept] = table[i];
      index.keys[kept] = k;
      std::swap(parents[kept], parents[i]);
      kept++;
    }
    if (dropped) {
      table.resize(kept);
      index.keys.resize(kept);
      index.map.clear();
      if (kept > 32)
        for (uint32_t i = 0; i < kept; i++) index.map.emplace(index.keys[i], i);
    }
  }
  const uint32_t n = (uint32_t)table.size();
  blk.resize(RH_WORDS + (size_t)n * ENT_WORDS, 0);
  for (auto* u : {&pu, &au, &ru})
    if (u->first > X_MASK) throw CedarError("string table overflow");
  blk[RH_NENT] = n;
  // entity index of a UID: the request's table, else the image's static entities (ENT_STATIC)
  auto idx_of = [&](const std::pair<uint32_t, uint32_t>& u) {
    const int32_t i = index.find(uid_key(u.first, u.second));
    if (i >= 0) return (uint32_t)i;
    const int32_t s = has_static ? img.static_row(uid_key(u.first, u.second)) : -1;
    return s < 0 ? NO_ENT : (ENT_STATIC | (uint32_t)s);
  };
  blk[RH_PIDX] = idx_of(pu);
  blk[RH_AIDX] = idx_of(au);
  blk[RH_RIDX] = idx_of(ru);
  {
    uint32_t w0, w1;
    src.emit_ctx(blk, img, E, w0, w1);
    blk[RH_CTX] = w0; blk[RH_CTX + 1] = w1;
  }
  std::vector<uint64_t>& anc = S.anc;
  std::vector<uint64_t>& nodes = S.nodes;
  std::vector<uint64_t>& cl = S.cl;
  std::vector<uint32_t>& n_key = S.n_key;
  n_key.assign(n, 0);
  std::unordered_set<uint64_t>& seen_big = S.seen_big;
  // one ancestor-list record (EncodedRequest::anc): the pairs of `anc` and, on an image with scope
  // bitsets, the key-entity index of its owner and of each of its `keys` leading (key-entity)
  // ancestors (image.h "scope bitsets"); returns the record's index
  std::vector<uint32_t>& al = E.anc;
  auto put_list = [&](uint64_t owner, uint32_t keys) {
    E.anc_at.push_back((uint32_t)al.size());
    al.push_back((uint32_t)anc.size());
    for (const uint64_t a : anc) { al.push_back((uint32_t)(a >> 32)); al.push_back((uint32_t)a); }
    if (img.sbits_words) {
      al.push_back(img.key_index(owner));
      for (uint32_t j = 0; j < keys; j++) al.push_back(img.key_index(anc[j]));
    }
    return (uint32_t)E.anc_at.size() - 1;
  };
  auto put_words = [&](const EncCache::Rec& r) {
    E.anc_hash.resize(E.anc_at.size(), 0);
    E.anc_hash.push_back(r.hash);
    E.anc_at.push_back((uint32_t)al.size());
    al.insert(al.end(), r.words.begin(), r.words.end());
    return (uint32_t)E.anc_at.size() - 1;
  };
  // The closure cache (EncCache) applies when no table entity with request-given parents is the
  // target of a static edge: then no static path leads back into the request's own edges.
  bool shortcut = closure_cache_on() && !t_no_closure_cache;
  for (uint32_t i = 0; i < n && shortcut; i++)
    if (table[i] & FROM_STATIC) shortcut = false;
    else if (has_static && src.n_parents(table[i]) && img.is_static_target(index.keys[i])) shortcut = false;
  EncCache* cc = shortcut ? &enc_cache(img) : nullptr;
  auto req_parents = [&](uint32_t i) { return !(table[i] & FROM_STATIC) && src.n_parents(table[i]) > 0; };
  // the record of table entity i from the cache; false: the general walk below
  auto cached = [&](uint32_t i) -> bool {
    const uint64_t uid = index.keys[i];
    if (!req_parents(i)) {
      const int32_t s = has_static ? img.static_row(uid) : -1;
      if (s < 0) {  // no parents anywhere
        anc.clear();
        n_key[i] = 0;
        blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = put_list(uid, 0);
        return true;
      }
      const EncCache::Rec* r = cc->srec[(size_t)s].load(std::memory_order_acquire);
      if (!r) {
        auto* nr = new EncCache::Rec();
        anc.clear();
        cpool_uids(img, img.srows[(size_t)s * ENT_WORDS + ER_ANC] & OFF_MASK, anc);
        std::sort(anc.begin(), anc.end());
        anc.erase(std::unique(anc.begin(), anc.end()), anc.end());
        nr->keys = make_record(img, uid, anc, nr->words);
        nr->hash = list_hash(nr->words.data(), (uint32_t)nr->words.size());
        const EncCache::Rec* expect = nullptr;
        if (cc->srec[(size_t)s].compare_exchange_strong(expect, nr, std::memory_order_acq_rel)) r = nr;
        else { delete nr; r = expect; }  // another thread published the same record first
      }
      n_key[i] = r->keys;
      blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = put_words(*r);
      return true;
    }
    const std::vector<uint64_t>& ps = parents[i];
    // The record names its owner only as a key entity (make_record: key_index), so an owner that is
    // none caches under its parents alone: users with one group set share a record (and a user's
    // UID string, request-local, never splits the cache).
    const uint64_t cu = img.is_key_ent(uid) ? uid : ~0ull;
    uint64_t h = cu * 0x9E3779B97F4A7C15ull;
    for (const uint64_t p : ps) {
      const int32_t at = index.find(p);
      if (at >= 0 && req_parents((uint32_t)at)) return false;  // a request edge above a request edge
      h = (h ^ p) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    }
    EncCache::Shard& sh = cc->shards[(h >> 58) & (EncCache::SHARDS - 1)];
    {
      std::lock_guard<std::mutex> g(sh.mu);
      auto it = sh.map.find(h);
      if (it != sh.map.end() && it->second.uid == cu && it->second.parents == ps) {
        n_key[i] = it->second.rec.keys;
        blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = put_words(it->second.rec);
        return true;
      }
    }
    anc.clear();
    for (const uint64_t p : ps) {
      anc.push_back(p);
      const int32_t s = has_static ? img.static_row(p) : -1;
      if (s >= 0) cpool_uids(img, img.srows[(size_t)s * ENT_WORDS + ER_ANC] & OFF_MASK, anc);
    }
    std::sort(anc.begin(), anc.end());
    anc.erase(std::unique(anc.begin(), anc.end()), anc.end());
    EncCache::Ent e;
    e.uid = cu;
    e.parents = ps;
    e.rec.keys = make_record(img, uid, anc, e.rec.words);
    e.rec.hash = list_hash(e.rec.words.data(), (uint32_t)e.rec.words.size());
    n_key[i] = e.rec.keys;
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = put_words(e.rec);
    std::lock_guard<std::mutex> g(sh.mu);
    if (sh.map.size() >= EncCache::MAX_PER_SHARD) sh.map.clear();
    sh.map[h] = std::move(e);
    return true;
  };
  for (uint32_t i = 0; i < n; i++) {
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_TYPE] = (uint32_t)(index.keys[i] >> 32);
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ID] = (uint32_t)index.keys[i];
    uint32_t w0, w1;
    if (table[i] & FROM_STATIC) {  // the static entity's attributes (constant-pool record)
      w0 = img.srows[(size_t)(table[i] & ~FROM_STATIC) * ENT_WORDS + ER_ATTR0];
      w1 = img.srows[(size_t)(table[i] & ~FROM_STATIC) * ENT_WORDS + ER_ATTR1];
    } else {
      src.emit_attrs(table[i], blk, img, E, w0, w1);
    }
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ATTR0] = w0;
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ATTR1] = w1;
    if (shortcut && cached(i)) continue;
    // transitive ancestors (through the merged map; cycles tolerated)
    anc.clear();
    seen_big.clear();
    auto seen = [&](uint64_t p) {
      return anc.size() <= 64 ? std::find(anc.begin(), anc.end(), p) != anc.end() : seen_big.count(p) > 0;
    };
    auto add = [&](uint64_t p) {
      anc.push_back(p);
      if (anc.size() == 65) seen_big.insert(anc.begin(), anc.end());  // switch to hashing
      else if (anc.size() > 65) seen_big.insert(p);
    };
    nodes.assign(1, index.keys[i]);  // table entities still to expand
    while (!nodes.empty()) {
      const int32_t at = index.find(nodes.back());
      nodes.pop_back();
      for (const uint64_t p : parents[(uint32_t)at]) {
        if (seen(p)) continue;
        add(p);
        if (index.find(p) >= 0) { nodes.push_back(p); continue; }
        const int32_t s = has_static ? img.static_row(p) : -1;
        if (s < 0) continue;  // in neither map: no parents
        // a static entity outside the table: its compiled closure row
        cl.clear();
        cpool_uids(img, img.srows[(size_t)s * ENT_WORDS + ER_ANC] & OFF_MASK, cl);
        for (const uint64_t q : cl) {
          if (seen(q)) continue;
          add(q);
          if (index.find(q) >= 0) nodes.push_back(q);  // a table entity a static edge names
        }
      }
    }
    n_key[i] = order_ancestors(img, anc);
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = put_list(index.keys[i], n_key[i]);  // a record index until appended
  }
  // ---- columnar row: UIDs, ancestor lists, hot paths resolved as attribute access would ----
  E.row.assign(img.row_words(), 0);
  uint32_t* row = E.row.data();
  row[RW_P] = pu.first; row[RW_P + 1] = pu.second;
  row[RW_A] = au.first; row[RW_A + 1] = au.second;
  row[RW_R] = ru.first; row[RW_R + 1] = ru.second;
  // ancestor lists of P / A / R (a static entity outside the table: its closure row as a record of
  // its own, so the probe kernel reads every list the same way), with the key counts; the row names
  // record k as k + 1 until appended
  auto anc_into = [&](uint32_t idx, const std::pair<uint32_t, uint32_t>& self, uint32_t w_off, uint32_t w_n) {
    uint32_t cnt = 0, keys = 0;
    if (idx != NO_ENT && (idx & ENT_STATIC)) {
      anc.clear();
      cpool_uids(img, img.srows[(size_t)(idx & ~ENT_STATIC) * ENT_WORDS + ER_ANC] & OFF_MASK, anc);
      keys = order_ancestors(img, anc);
      row[w_off] = put_list(uid_key(self.first, self.second), keys) + 1;
      cnt = (uint32_t)anc.size();
    } else if (idx != NO_ENT) {
      const uint32_t rec = blk[RH_WORDS + idx * ENT_WORDS + ER_ANC];
      row[w_off] = rec + 1;
      cnt = E.anc_rec(rec)[0];
      keys = n_key[idx];
    }
    if (cnt > AN_COUNT || keys > AN_KEYS) throw CedarError("entity has too many ancestors for the device row format");
    row[w_n] = cnt | (keys << AN_KEYS_SHIFT) | (img.is_key_ent(uid_key(self.first, self.second)) ? AN_SELF : 0u);
  };
  anc_into(blk[RH_PIDX], pu, RW_PANC, RW_PN);
  anc_into(blk[RH_RIDX], ru, RW_RANC, RW_RN);
  anc_into(blk[RH_AIDX], au, RW_AANC, RW_AN);
  // action masks over the image action table, as the probe kernel tests scopes against them
  row[RW_ASELF] = ASELF_MASK;  // (absent; bit 31, ASELF_CTXR, is resolve_contexts')
  if (img.amask_ok) {
    uint64_t am = 0;
    const uint32_t n_act = (uint32_t)img.act.size() / 2;
    const uint32_t an = row[RW_AN] & AN_COUNT;
    const uint32_t* al_ = an ? E.anc_pairs(row[RW_AANC]) : nullptr;
    for (uint32_t k = 0; k < n_act; k++) {
      const uint32_t qt = img.act[2 * k], qi = img.act[2 * k + 1];
      const bool self = au.first == qt && au.second == qi;
      bool hit = self;
      for (uint32_t j = 0; j < an && !hit; j++) hit = al_[2 * j] == qt && al_[2 * j + 1] == qi;
      if (hit) am |= 1ull << k;
      if (self) row[RW_ASELF] = k;
    }
    row[RW_AM0] = (uint32_t)am;
    row[RW_AM1] = (uint32_t)(am >> 32);
  }
  const uint32_t nh = img.n_hot();
  for (uint32_t h = 0; h < nh; h++) {
    const uint32_t* hp = &img.hot[(size_t)h * HOT_WORDS];
    const uint32_t var = hp[0], depth = hp[1];
    uint32_t w0, w1;
    if (var == 3) { w0 = blk[RH_CTX]; w1 = blk[RH_CTX + 1]; }
    else { const auto& u = var == 0 ? pu : var == 1 ? au : ru; w0 = mk_w0(T_ENT, u.first); w1 = u.second; }
    uint32_t code = E_NONE, aux = 0, k = 0, et = 0, ei = 0;
    bool fin = false;
    for (uint32_t j = 0; j < depth && code == E_NONE; j++) {
      const uint32_t key = hp[2 + j], tag = w0 >> TAG_SHIFT;
      const bool last = j + 1 == depth;
      if (tag == T_ENT) {
        const uint32_t t = w0 & X_MASK, id = w1;
        const uint32_t at = idx_of({t, id});
        if (at == NO_ENT) { code = E_ENTITY_MISSING; et = t; ei = id; fin = last; break; }
        const uint32_t* er = (at & ENT_STATIC) ? &img.srows[(size_t)(at & ~ENT_STATIC) * ENT_WORDS]
                                               : &blk[RH_WORDS + (size_t)at * ENT_WORDS];
        const uint32_t a0 = er[ER_ATTR0], a1 = er[ER_ATTR1];
        if (!blk_rec_get(blk, img.cpool, a0, a1, key, w0, w1)) { code = E_ATTR_ENTITY; k = key; et = t; ei = id; fin = last; }
      } else if (tag == T_REC) {
        if (!blk_rec_get(blk, img.cpool, w0, w1, key, w0, w1)) { code = E_ATTR_RECORD; k = key; fin = last; }
      } else {
        code = E_TYPE;
        aux = TN_ENTITY_OR_RECORD | (mem_tname(w0) << 8);
      }
    }
    if (code == E_NONE) {
      row[RW_HDR + 2 * h] = w0;
      row[RW_HDR + 2 * h + 1] = w1;
      if (h < ASELF_PRES_SLOTS) row[RW_ASELF] |= 1u << (ASELF_PRES_SHIFT + h);  // (image.h "presence masks")
    } else {
      const uint32_t off = (uint32_t)blk.size();
      blk.push_back(code | (aux << 8)); blk.push_back(k); blk.push_back(et); blk.push_back(ei);
      row[RW_HDR + 2 * h] = mk_w0(T_NONE, code | (fin ? HS_FINAL : 0u));
      row[RW_HDR + 2 * h + 1] = off;
    }
  }
  // set-membership keys (image.h BT_CKEY): each such slot's element hashes, after the hot slots;
  // prefix keys (image.h "prefix level-2 keys"): a string's prefix hashes at the slot's lengths
  if (img.list_mask()) {
    std::vector<uint32_t>& hs = S.hs;
    for (uint32_t m = img.list_mask(); m; m &= m - 1) {
      const uint32_t h = (uint32_t)__builtin_ctz(m);
      const uint32_t w0 = row[RW_HDR + 2 * h], w1 = row[RW_HDR + 2 * h + 1], tag = w0 >> TAG_SHIFT;
      hs.clear();
      const bool pfx = (img.pslot_mask >> h) & 1;
      const uint32_t want = pfx ? T_STR : T_SET;
      uint32_t head = tag == T_NONE ? CL_MISSING : tag != want ? CL_NOTSET : 0u;
      if (pfx && tag == T_STR) {
        const std::string_view sv = w1 < img.n_gstr() ? std::string_view(img.strings[w1]) : std::string_view(E.strs[w1 - img.n_gstr()]);
        for (uint32_t j = 0; j < PFX_LENS; j++) {
          const uint32_t len = img.pfx[(size_t)h * PFX_LENS + j];
          if (len && len <= sv.size()) hs.push_back(pfx_hash(reinterpret_cast<const uint8_t*>(sv.data()), len));
        }
        head = (uint32_t)hs.size();
      } else if (!pfx && tag == T_SET) {
        const uint32_t x = w0 & X_MASK;
        const std::vector<uint32_t>& mm = (x >> SPACE_SHIFT) == SP_CPOOL ? img.cpool : blk;
        const uint32_t off = x & OFF_MASK, n = mm[off];
        head = n;
        for (uint32_t k = 0; k < n; k++) hs.push_back(mem_chash(blk, img.cpool, mm[off + 1 + 2 * k], mm[off + 2 + 2 * k]));
      }
      // (the slot's word: its rank among the image's list slots)
      row[RW_HDR + 2 * nh + (uint32_t)__builtin_popcount(img.list_mask() & ((1u << h) - 1u))] = (uint32_t)blk.size();
      blk.push_back(head);
      blk.insert(blk.end(), hs.begin(), hs.end());
    }
  }
  // like words (image.h AK_LIKEI): per like slot the string's length, first and last 8 bytes
  if (img.lslot_mask) {
    uint32_t* lw = row + img.like_off();
    for (uint32_t m = img.lslot_mask; m; m &= m - 1, lw += LIKE_WORDS) {
      const uint32_t h = (uint32_t)__builtin_ctz(m);
      const uint32_t w0 = row[RW_HDR + 2 * h], w1 = row[RW_HDR + 2 * h + 1];
      for (uint32_t j = 0; j < LIKE_WORDS; j++) lw[j] = 0;
      if ((w0 >> TAG_SHIFT) != T_STR) continue;  // (the atom's type check decides first)
      const std::string_view sv = w1 < img.n_gstr() ? std::string_view(img.strings[w1]) : std::string_view(E.strs[w1 - img.n_gstr()]);
      const size_t n = sv.size(), k = std::min<size_t>(n, 8);
      uint64_t pre = 0, suf = 0;
      for (size_t j = 0; j < k; j++) pre |= (uint64_t)(uint8_t)sv[j] << (8 * j);
      for (size_t j = 0; j < k; j++) suf |= (uint64_t)(uint8_t)sv[n - 1 - j] << (8 * (7 - j));
      lw[0] = n > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)n;
      lw[1] = (uint32_t)pre; lw[2] = (uint32_t)(pre >> 32);
      lw[3] = (uint32_t)suf; lw[4] = (uint32_t)(suf >> 32);
    }
  }
  // the request-local strings whose bytes the device reads: the values of the image's like-read
  // slots (Image::lread_mask); none of the others is ever read as bytes there
  if (!img.dev_all_strings() && !E.strs.empty()) {
    E.str_dev.assign(E.strs.size(), 0);
    for (uint32_t m = img.lread_mask; m; m &= m - 1) {
      const uint32_t h = (uint32_t)__builtin_ctz(m);
      if (h >= nh) break;
      const uint32_t w0 = row[RW_HDR + 2 * h], w1 = row[RW_HDR + 2 * h + 1];
      if ((w0 >> TAG_SHIFT) == T_STR && w1 >= img.n_gstr() && w1 - img.n_gstr() < E.strs.size()) E.str_dev[w1 - img.n_gstr()] = 1;
    }
  }
  resolve_contexts(img, E);
  if (blk.size() > OFF_MASK) throw CedarError("request too large for the device heap format");
  // grouping key: 8 bits of (action, resource type) | 16 of the principal's type and key ancestors |
  // 8 of its hot values (group.hip sorts on the top 24). Round-5 A/B of the field order
  // (profiles/r05/ab/r05x): hot values before the principal, 0.52-0.54 ms of scan for 0.45;
  // the principal first, 0.51 ms and a 0.04 ms slower candidate pass.
  {
    auto mix = [](uint32_t h, uint32_t x) {
      h ^= x;
      h *= 0x9E3779B1u;
      h ^= h >> 15;
      h *= 0x85EBCA77u;
      return h ^ (h >> 13);
    };
    const uint32_t ar = mix(mix(0x51ED27Fu, row[RW_A + 1]), row[RW_R]);
    uint32_t g = mix(0x3C6EF372u, row[RW_P]);
    const uint32_t nk = std::min<uint32_t>((row[RW_PN] >> AN_KEYS_SHIFT) & AN_KEYS, 32u);
    const uint32_t* pl = nk ? E.anc_pairs(row[RW_PANC]) : nullptr;
    for (uint32_t j = 0; j < nk; j++) g += mix(mix(0x2545F491u, pl[2 * j]), pl[2 * j + 1]);
    g = mix(g, 0x7FEB352Du);
    uint32_t hv = 0x6C8E9CF5u;
    // (a request-local string, in no image key, mixes as one value: its id is a table position)
    for (uint32_t j = 0; j < nh; j++) {
      const uint32_t w0 = row[RW_HDR + 2 * j], w1 = row[RW_HDR + 2 * j + 1];
      hv = mix(mix(hv, w0), (w0 >> TAG_SHIFT) == T_STR && w1 >= img.n_gstr() ? img.n_gstr() : w1);
    }
    E.gkey = (ar & 0xFF000000u) | ((g >> 16) << 8) | (hv >> 24);
  }
}

}  // namespace cg
