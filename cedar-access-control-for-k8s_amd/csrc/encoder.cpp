// Request encoder: (EntityMap, Request) -> one request block of the device heap.
//
// The reference builds a Go `cedartypes.EntityMap` + `cedar.Request` per webhook call
// (internal/server/authorizer/authorizer.go:89-111, admission/handler.go:82-153) and hands them
// to (*PolicySet).IsAuthorized (store/store.go:31). The encoder lays the same facts out flat:
//   header (P/A/R UIDs, context, entity-table indices of P/A/R) | entity table | data
// Strings are interned against the image's global table first (so policy constants and request
// strings compare by ID), then request-locally, so encoding needs no batch-wide state: any thread
// encodes a request (encode_request) and the batch appends it with copies (Batch::append). Each entity row carries a pointer to its
// transitive ancestor list (the closure of `parents` through the map), so `in` is a linear scan.
#include <sys/mman.h>
#include <algorithm>
#include <atomic>
#include <thread>

#include "encode_impl.h"

namespace cg {
std::atomic<uint64_t> g_pinned_kept{0};
}  // namespace cg

namespace cg {

bool hugepages_on() {
  static const bool on = [] { const char* e = std::getenv("CEDARGPU_HUGEPAGES"); return e && *e == '1'; }();
  return on;
}

// 2 MiB-aligned (the tag huge_unmap checks: the heap never returns such a block), advised huge
void* huge_map(size_t bytes) {
  constexpr size_t H = 2u << 20;
  const size_t len = (bytes + H - 1) & ~(H - 1);
  void* raw = mmap(nullptr, len + H, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (raw == MAP_FAILED) return nullptr;
  const uintptr_t r = (uintptr_t)raw, a = (r + H - 1) & ~(uintptr_t)(H - 1);
  if (a > r) munmap(raw, a - r);
  if (r + len + H > a + len) munmap((void*)(a + len), r + len + H - (a + len));
  (void)madvise((void*)a, len, MADV_HUGEPAGE);
  return (void*)a;
}

bool huge_unmap(void* p, size_t bytes) {
  constexpr size_t H = 2u << 20;
  if (!p || ((uintptr_t)p & (H - 1))) return false;
  munmap(p, (bytes + H - 1) & ~(H - 1));
  return true;
}

using namespace cgi;

void emit_heap_value(const HVal& v, std::vector<uint32_t>& out, const Image& img, EncodedRequest& e, uint32_t& w0,
                     uint32_t& w1);

std::string Batch::str(uint32_t i, uint32_t id) const {
  const uint32_t ng = img->n_gstr();
  if (id < ng) return img->strings[id];
  if (i >= req_base.size()) return std::string();
  const size_t j = (size_t)heap[req_base[i] + RH_SBASE] + (id - ng);
  if (j >= n_bstr()) return std::string();
  return std::string((const char*)bstr_bytes.data() + bstr_off[j], bstr_off[j + 1] - bstr_off[j]);
}

namespace {
// (EntityIn, RequestIn) trees as an encode_impl source
struct HSrc {
  const std::vector<EntityIn>& ents;
  const RequestIn& req;
  using SV = std::pair<std::string_view, std::string_view>;
  uint32_t n_ents() const { return (uint32_t)ents.size(); }
  std::string_view type(uint32_t i) const { return ents[i].type; }
  std::string_view id(uint32_t i) const { return ents[i].id; }
  uint32_t n_parents(uint32_t i) const { return (uint32_t)ents[i].parents.size(); }
  SV parent(uint32_t i, uint32_t k) const { return {ents[i].parents[k].first, ents[i].parents[k].second}; }
  SV principal() const { return {req.principal.first, req.principal.second}; }
  SV action() const { return {req.action.first, req.action.second}; }
  SV resource() const { return {req.resource.first, req.resource.second}; }
  static void emit(const HVal& v, std::vector<uint32_t>& out, const Image& img, EncodedRequest& E, uint32_t& w0,
                   uint32_t& w1) {
    if (v.k != VK::Rec) enc::emit_empty_record(out, w0, w1);  // a non-record is encoded as {}
    else emit_heap_value(v, out, img, E, w0, w1);
  }
  void emit_ctx(std::vector<uint32_t>& out, const Image& img, EncodedRequest& E, uint32_t& w0, uint32_t& w1) const {
    emit(req.context, out, img, E, w0, w1);
  }
  void emit_attrs(uint32_t i, std::vector<uint32_t>& out, const Image& img, EncodedRequest& E, uint32_t& w0,
                  uint32_t& w1) const {
    emit(ents[i].attrs, out, img, E, w0, w1);
  }
};
}  // namespace

void encode_request(const Image& img, const std::vector<EntityIn>& ents, const RequestIn& req, EncodedRequest& E) {
  encode_impl(img, HSrc{ents, req}, E);
}

void Batch::append(EncodedRequest& e) {
  if (!row_words) row_words = img->row_words();
  if (e.row.size() != row_words || e.blk.size() < RH_WORDS) throw CedarError("request encoded for another image");
  if (heap.size() + e.blk.size() + e.anc.size() > 0xFFFFFFFFull) throw CedarError("batch heap exceeds 16 GiB");
  // (the probe kernel addresses a row's words by a 32-bit offset, PCtx::rowo)
  if (rows.size() + row_words > 0xFFFFFFFFull) throw CedarError("batch rows exceed 16 GiB");
  size_t sbytes = 0;
  for (auto& s : e.strs) sbytes += s.size();
  if (n_bstr() + e.strs.size() >= 0xFFFFFFFFull || bstr_bytes.size() + sbytes > 0xFFFFFFFFull)
    throw CedarError("batch string table overflow");
  // ancestor-list records: interned ahead of the block, which points back at them
  const uint32_t n_rec = (uint32_t)e.anc_at.size();
  uint32_t at_small[16];
  std::vector<uint32_t> at_big;
  uint32_t* at = n_rec <= 16 ? at_small : (at_big.resize(n_rec), at_big.data());
  const uint64_t room = (uint64_t)e.anc.size() + 16;  // the block starts at most this far past a new record
  for (uint32_t k = 0; k < n_rec; k++) {
    const uint32_t s = e.anc_at[k], t = k + 1 < n_rec ? e.anc_at[k + 1] : (uint32_t)e.anc.size();
    at[k] = intern_list(e.anc.data() + s, t - s, room, k < e.anc_hash.size() ? e.anc_hash[k] : 0);
  }
  const uint32_t B = (uint32_t)heap.size();
  const uint32_t nent = e.blk[RH_NENT];
  for (uint32_t i = 0; i < nent; i++) {
    uint32_t& w = e.blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC];
    if (w >= n_rec) throw CedarError("request encoded without its ancestor lists");
    w = mk_ref(SP_HEAP, (at[w] - B) & OFF_MASK);
  }
  for (const uint32_t f : {RW_PANC, RW_RANC, RW_AANC}) {
    uint32_t& w = e.row[f];
    if (w > n_rec) throw CedarError("request encoded without its ancestor lists");
    if (w) w = at[w - 1] - B + 1;  // (mod 2^32: negative)
  }
  e.blk[RH_SBASE] = n_bstr();
  e.row[RW_BLK] = B;
  req_base.push_back(B);
  append_pod(heap, e.blk.data(), e.blk.size());
  append_pod(rows, e.row.data(), e.row.size());
  gkeys.push_back(e.gkey);
  for (auto& s : e.strs) {
    append_pod(bstr_bytes, (const uint8_t*)s.data(), s.size());
    bstr_off.push_back((uint32_t)bstr_bytes.size());
  }
  if (!img->dev_all_strings()) {  // the device's table: the same ids, bytes of the read strings only
    dstr = true;
    for (size_t k = 0; k < e.strs.size(); k++) {
      if (k < e.str_dev.size() && e.str_dev[k]) append_pod(dstr_bytes, (const uint8_t*)e.strs[k].data(), e.strs[k].size());
      dstr_off.push_back((uint32_t)dstr_bytes.size());
    }
  }
}

// One ancestor-list record into the heap, or the copy an earlier block appended (equal words,
// close enough that a block starting `room` words past the heap end still reaches it).
uint64_t list_hash(const uint32_t* w, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
  for (uint32_t k = 0; k < n; k++) {
    h = (h ^ w[k]) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
  }
  return h | 1;  // (never 0: 0 means "not computed")
}

uint32_t Batch::intern_list(const uint32_t* w, uint32_t n, uint64_t room, uint64_t hash) {
  const uint64_t h = hash ? hash : list_hash(w, n);
  anc_words += n;
  const uint64_t key = h | 1u;
  if (2 * (memo_used + 1) > memo.size() / 2) {  // (load <= 1/2; pairs of words)
    PodVec<uint64_t> old;
    old.swap(memo);
    memo.assign(std::max<size_t>(512, old.size() * 2), 0);
    const size_t mask = memo.size() / 2 - 1;
    for (size_t j = 0; j < old.size(); j += 2)
      if (old[j]) {
        size_t s = (size_t)(old[j] >> 1) & mask;
        while (memo[2 * s]) s = (s + 1) & mask;
        memo[2 * s] = old[j];
        memo[2 * s + 1] = old[j + 1];
      }
  }
  const size_t mask = memo.size() / 2 - 1;
  size_t s = (size_t)(key >> 1) & mask;
  while (memo[2 * s] && memo[2 * s] != key) s = (s + 1) & mask;
  if (memo[2 * s]) {
    const uint32_t o = (uint32_t)memo[2 * s + 1];
    if (heap.size() + room - o <= ANC_REACH && std::equal(w, w + n, heap.begin() + o)) {
      anc_shared_words += n;
      return o;
    }
  } else {
    memo_used++;
  }
  if (heap.size() + n > 0xFFFFFFFFull) throw CedarError("batch heap exceeds 16 GiB");
  const uint32_t o = (uint32_t)heap.size();
  append_pod(heap, w, n);
  memo[2 * s] = key;
  memo[2 * s + 1] = o;
  return o;
}

void Batch::concat(std::vector<Batch>& parts, unsigned threads) {
  if (!row_words) row_words = img->row_words();
  const size_t np = parts.size();
  std::vector<size_t> ho(np), ro(np), so(np), bo(np), dbo(np);
  size_t H = heap.size(), R = req_base.size(), S = n_bstr(), SB = bstr_bytes.size(), DB = dstr_bytes.size();
  dstr = dstr || !img->dev_all_strings();
  for (size_t k = 0; k < np; k++) {
    const Batch& p = parts[k];
    if (p.n() && p.row_words != row_words) throw CedarError("request encoded for another image");
    if (dstr && p.dstr_off.size() != p.bstr_off.size()) throw CedarError("batch part without its device string table");
    ho[k] = H; ro[k] = R; so[k] = S; bo[k] = SB; dbo[k] = DB;
    H += p.heap.size(); R += p.n(); S += p.n_bstr(); SB += p.bstr_bytes.size(); DB += p.dstr_bytes.size();
    anc_words += p.anc_words;
    anc_shared_words += p.anc_shared_words;
  }
  if (H > 0xFFFFFFFFull) throw CedarError("batch heap exceeds 16 GiB");
  if (R * row_words > 0xFFFFFFFFull) throw CedarError("batch rows exceed 16 GiB");
  if (S >= 0xFFFFFFFFull || SB > 0xFFFFFFFFull || DB > 0xFFFFFFFFull) throw CedarError("batch string table overflow");
  heap.resize(H);
  req_base.resize(R);
  rows.resize(R * row_words);
  gkeys.resize(R);
  bstr_off.resize(S + 1);
  bstr_bytes.resize(SB);
  if (dstr) {
    dstr_off.resize(S + 1);
    dstr_bytes.resize(DB);
  }
  auto copy = [&](size_t k) {
    Batch& p = parts[k];
    const uint32_t hs = (uint32_t)ho[k], ss = (uint32_t)so[k], bs = (uint32_t)bo[k];
    if (!p.heap.empty()) std::memcpy(heap.data() + ho[k], p.heap.data(), p.heap.size() * 4);
    for (uint32_t i = 0; i < p.n(); i++) {
      const uint32_t base = p.req_base[i] + hs;
      req_base[ro[k] + i] = base;
      heap[base + RH_SBASE] += ss;  // request-local strings: the part's numbering, shifted
      uint32_t* row = rows.data() + (ro[k] + i) * row_words;
      std::memcpy(row, p.rows.data() + (size_t)i * row_words, (size_t)row_words * 4);
      row[RW_BLK] += hs;
      gkeys[ro[k] + i] = p.gkeys[i];
    }
    for (uint32_t j = 0; j < p.n_bstr(); j++) bstr_off[ss + 1 + j] = p.bstr_off[1 + j] + bs;
    if (!p.bstr_bytes.empty()) std::memcpy(bstr_bytes.data() + bo[k], p.bstr_bytes.data(), p.bstr_bytes.size());
    if (dstr) {
      const uint32_t ds = (uint32_t)dbo[k];
      for (uint32_t j = 0; j < p.n_bstr(); j++) dstr_off[ss + 1 + j] = p.dstr_off[1 + j] + ds;
      if (!p.dstr_bytes.empty()) std::memcpy(dstr_bytes.data() + dbo[k], p.dstr_bytes.data(), p.dstr_bytes.size());
    }
    p = Batch();  // its memory goes back as soon as it is copied
  };
  threads = std::max(1u, std::min<unsigned>(threads, (unsigned)np));
  if (threads <= 1) {
    for (size_t k = 0; k < np; k++) copy(k);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> ws;
  for (unsigned t = 1; t < threads; t++)
    ws.emplace_back([&] { for (size_t k; (k = next++) < np;) copy(k); });
  for (size_t k; (k = next++) < np;) copy(k);
  for (auto& w : ws) w.join();
}

void Batch::add(const std::vector<EntityIn>& ents, const RequestIn& req) {
  EncodedRequest e;
  encode_request(*img, ents, req, e);
  append(e);
}

// The string table is built as requests are appended; the device reads at least one byte and word.
void Batch::finalize_strings() {
  if (bstr_bytes.empty()) bstr_bytes.push_back(0);
  if (dstr && dstr_bytes.empty()) dstr_bytes.push_back(0);
  if (heap.empty()) heap.push_back(0);
}

static std::pair<std::string, std::string> uid_from_json(const JVal& j) {
  const JVal* u = j.get("__entity");
  const JVal& x = u ? *u : j;
  return {x.str_or("type"), x.str_or("id")};
}

void decode_json_entities(const JVal& es, std::vector<EntityIn>& ents) {
  if (es.t != JVal::Arr) throw CedarError("\"entities\" must be an array");
  for (auto& e : es.arr) {
    EntityIn ei;
    const JVal* uid = e.get("uid");
    if (!uid) throw CedarError("entity without uid");
    auto u = uid_from_json(*uid);
    ei.type = u.first; ei.id = u.second;
    const JVal* at = e.get("attrs");
    if (at) ei.attrs = hval_from_json(*at);
    else ei.attrs.k = VK::Rec;
    if (ei.attrs.k != VK::Rec) throw CedarError("entity attrs must be an object");
    const JVal* ps = e.get("parents");
    if (ps) for (auto& p : ps->arr) ei.parents.push_back(uid_from_json(p));
    ents.push_back(std::move(ei));
  }
}

void decode_json_item(const JVal& item, std::vector<EntityIn>& ents, RequestIn& req) {
  const JVal* es = item.get("entities");
  const JVal* rq = item.get("request");
  if (!rq || rq->t != JVal::Obj) throw CedarError("item needs a \"request\" object");
  ents.clear();
  if (es) decode_json_entities(*es, ents);
  const JVal* p = rq->get("principal");
  const JVal* a = rq->get("action");
  const JVal* r = rq->get("resource");
  if (!p || !a || !r) throw CedarError("request needs principal, action and resource");
  req.principal = uid_from_json(*p);
  req.action = uid_from_json(*a);
  req.resource = uid_from_json(*r);
  const JVal* c = rq->get("context");
  if (c) req.context = hval_from_json(*c);
  else { req.context = HVal(); req.context.k = VK::Rec; }
}

}  // namespace cg
