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
#include <algorithm>
#include <unordered_set>

#include "engine.h"

namespace cg {
using namespace cgi;

void emit_heap_value(const HVal& v, std::vector<uint32_t>& out, const Image& img, EncodedRequest& e, uint32_t& w0,
                     uint32_t& w1);
uint32_t request_sid(const Image& img, EncodedRequest& e, const std::string& s);

const std::string& Batch::str(uint32_t i, uint32_t id) const {
  static const std::string empty;
  const uint32_t ng = img->n_gstr();
  if (id < ng) return img->strings[id];
  if (i >= req_base.size()) return empty;
  const size_t j = (size_t)heap[req_base[i] + RH_SBASE] + (id - ng);
  return j < bstrings.size() ? bstrings[j] : empty;
}

namespace {
// memory-form record lookup inside an emitted request block (the device's rec_get, on the host)
bool blk_rec_get(const std::vector<uint32_t>& blk, uint32_t rw0, uint32_t n, uint32_t key, uint32_t& w0, uint32_t& w1) {
  const uint32_t off = rw0 & OFF_MASK;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blk[off + 1 + 3 * mid] < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && blk[off + 1 + 3 * lo] == key) {
    w0 = blk[off + 2 + 3 * lo];
    w1 = blk[off + 3 + 3 * lo];
    return true;
  }
  return false;
}
uint32_t mem_tname(uint32_t w0) {
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
struct PairHash {
  size_t operator()(const std::pair<uint32_t, uint32_t>& p) const { return ((size_t)p.first << 32) ^ p.second; }
};
}  // namespace

void encode_request(const Image& img, const std::vector<EntityIn>& ents, const RequestIn& req, EncodedRequest& E) {
  E.clear();
  auto sid = [&](const std::string& s) { return request_sid(img, E, s); };
  std::vector<uint32_t>& blk = E.blk;
  // entity table (EntityMap semantics: a repeated UID replaces the earlier entity)
  std::vector<const EntityIn*> table;
  std::unordered_map<std::pair<uint32_t, uint32_t>, uint32_t, PairHash> index;
  std::vector<std::pair<uint32_t, uint32_t>> uids;
  for (auto& e : ents) {
    std::pair<uint32_t, uint32_t> u{sid(e.type), sid(e.id)};
    auto it = index.find(u);
    if (it != index.end()) { table[it->second] = &e; continue; }
    index.emplace(u, (uint32_t)table.size());
    table.push_back(&e);
    uids.push_back(u);
  }
  const uint32_t n = (uint32_t)table.size();
  blk.resize(RH_WORDS + (size_t)n * ENT_WORDS, 0);
  auto uid_of = [&](const std::pair<std::string, std::string>& u) { return std::make_pair(sid(u.first), sid(u.second)); };
  auto pu = uid_of(req.principal), au = uid_of(req.action), ru = uid_of(req.resource);
  for (auto* u : {&pu, &au, &ru}) if (u->first > X_MASK) throw CedarError("string table overflow");
  blk[RH_NENT] = n;
  blk[RH_P] = mk_w0(T_ENT, pu.first); blk[RH_P + 1] = pu.second;
  blk[RH_A] = mk_w0(T_ENT, au.first); blk[RH_A + 1] = au.second;
  blk[RH_R] = mk_w0(T_ENT, ru.first); blk[RH_R + 1] = ru.second;
  auto idx_of = [&](const std::pair<uint32_t, uint32_t>& u) { auto it = index.find(u); return it == index.end() ? NO_ENT : it->second; };
  blk[RH_PIDX] = idx_of(pu);
  blk[RH_AIDX] = idx_of(au);
  blk[RH_RIDX] = idx_of(ru);
  {
    uint32_t w0, w1;
    HVal ctx = req.context;
    if (ctx.k != VK::Rec) { ctx = HVal(); ctx.k = VK::Rec; }
    emit_heap_value(ctx, blk, img, E, w0, w1);
    blk[RH_CTX] = w0; blk[RH_CTX + 1] = w1;
  }
  // parent adjacency (ids of parents that exist in the map are followed; absent ones are leaves)
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> parents(n);
  for (uint32_t i = 0; i < n; i++)
    for (auto& p : table[i]->parents) {
      auto u = uid_of(p);
      if (std::find(parents[i].begin(), parents[i].end(), u) == parents[i].end()) parents[i].push_back(u);
    }
  for (uint32_t i = 0; i < n; i++) {
    uint32_t* row = &blk[RH_WORDS + (size_t)i * ENT_WORDS];
    row[ER_TYPE] = uids[i].first;
    row[ER_ID] = uids[i].second;
    uint32_t w0, w1;
    HVal attrs = table[i]->attrs;
    if (attrs.k != VK::Rec) { attrs = HVal(); attrs.k = VK::Rec; }
    emit_heap_value(attrs, blk, img, E, w0, w1);
    row = &blk[RH_WORDS + (size_t)i * ENT_WORDS];  // blk may have reallocated
    row[ER_ATTR0] = w0; row[ER_ATTR1] = w1;
    // transitive ancestors (BFS through the map; cycles tolerated)
    std::vector<std::pair<uint32_t, uint32_t>> anc;
    std::unordered_set<std::pair<uint32_t, uint32_t>, PairHash> seen;
    std::vector<uint32_t> stack{i};
    while (!stack.empty()) {
      uint32_t cur = stack.back();
      stack.pop_back();
      for (auto& p : parents[cur]) {
        if (!seen.insert(p).second) continue;
        anc.push_back(p);
        auto it = index.find(p);
        if (it != index.end()) stack.push_back(it->second);
      }
    }
    std::sort(anc.begin(), anc.end());
    uint32_t off = (uint32_t)blk.size();
    blk.push_back((uint32_t)anc.size());
    for (auto& a : anc) { blk.push_back(a.first); blk.push_back(a.second); }
    blk[RH_WORDS + (size_t)i * ENT_WORDS + ER_ANC] = mk_ref(SP_HEAP, off);
  }
  // ---- columnar row: UIDs, ancestor lists, hot paths resolved as attribute access would ----
  E.row.assign(img.row_words(), 0);
  std::vector<uint32_t>& rows = E.row;
  const size_t r0 = 0;
  uint32_t* row = rows.data();
  row[RW_P] = pu.first; row[RW_P + 1] = pu.second;
  row[RW_A] = au.first; row[RW_A + 1] = au.second;
  row[RW_R] = ru.first; row[RW_R + 1] = ru.second;
  auto anc_into = [&](uint32_t idx, uint32_t w_off, uint32_t w_n) {
    if (idx == NO_ENT) return;
    const uint32_t ref = blk[RH_WORDS + idx * ENT_WORDS + ER_ANC] & OFF_MASK;
    rows[r0 + w_off] = ref + 1;
    rows[r0 + w_n] = blk[ref];
  };
  anc_into(blk[RH_PIDX], RW_PANC, RW_PN);
  anc_into(blk[RH_RIDX], RW_RANC, RW_RN);
  anc_into(blk[RH_AIDX], RW_AANC, RW_AN);
  const uint32_t nh = img.n_hot();
  for (uint32_t h = 0; h < nh; h++) {
    const uint32_t* hp = &img.hot[(size_t)h * HOT_WORDS];
    const uint32_t var = hp[0], depth = hp[1];
    uint32_t w0, w1;
    if (var == 3) { w0 = blk[RH_CTX]; w1 = blk[RH_CTX + 1]; }
    else { const uint32_t o = var == 0 ? RH_P : var == 1 ? RH_A : RH_R; w0 = blk[o]; w1 = blk[o + 1]; }
    uint32_t code = E_NONE, aux = 0, k = 0, et = 0, ei = 0;
    bool fin = false;
    for (uint32_t j = 0; j < depth && code == E_NONE; j++) {
      const uint32_t key = hp[2 + j], tag = w0 >> TAG_SHIFT;
      const bool last = j + 1 == depth;
      if (tag == T_ENT) {
        const uint32_t t = w0 & X_MASK, id = w1;
        auto it = index.find({t, id});
        if (it == index.end()) { code = E_ENTITY_MISSING; et = t; ei = id; fin = last; break; }
        const uint32_t* er = &blk[RH_WORDS + it->second * ENT_WORDS];
        if (!blk_rec_get(blk, er[ER_ATTR0], er[ER_ATTR1], key, w0, w1)) { code = E_ATTR_ENTITY; k = key; et = t; ei = id; fin = last; }
      } else if (tag == T_REC) {
        if (!blk_rec_get(blk, w0, w1, key, w0, w1)) { code = E_ATTR_RECORD; k = key; fin = last; }
      } else {
        code = E_TYPE;
        aux = TN_ENTITY_OR_RECORD | (mem_tname(w0) << 8);
      }
    }
    if (code == E_NONE) {
      rows[r0 + RW_HDR + 2 * h] = w0;
      rows[r0 + RW_HDR + 2 * h + 1] = w1;
    } else {
      const uint32_t off = (uint32_t)blk.size();
      blk.push_back(code | (aux << 8)); blk.push_back(k); blk.push_back(et); blk.push_back(ei);
      rows[r0 + RW_HDR + 2 * h] = mk_w0(T_NONE, code | (fin ? HS_FINAL : 0u));
      rows[r0 + RW_HDR + 2 * h + 1] = off;
    }
  }
  if (blk.size() > OFF_MASK) throw CedarError("request too large for the device heap format");
}

void Batch::append(EncodedRequest& e) {
  if (!row_words) row_words = img->row_words();
  if (e.row.size() != row_words || e.blk.size() < RH_WORDS) throw CedarError("request encoded for another image");
  if (heap.size() + e.blk.size() > 0xFFFFFFFFull) throw CedarError("batch heap exceeds 16 GiB");
  if (bstrings.size() + e.strs.size() > 0xFFFFFFFFull) throw CedarError("batch string table overflow");
  e.blk[RH_SBASE] = (uint32_t)bstrings.size();
  e.row[RW_BLK] = (uint32_t)heap.size();
  req_base.push_back((uint32_t)heap.size());
  heap.insert(heap.end(), e.blk.begin(), e.blk.end());
  rows.insert(rows.end(), e.row.begin(), e.row.end());
  for (auto& s : e.strs) bstrings.push_back(std::move(s));
}

void Batch::add(const std::vector<EntityIn>& ents, const RequestIn& req) {
  EncodedRequest e;
  encode_request(*img, ents, req, e);
  append(e);
}

void Batch::finalize_strings() {
  bstr_off.clear();
  bstr_bytes.clear();
  for (auto& s : bstrings) {
    bstr_off.push_back((uint32_t)bstr_bytes.size());
    bstr_bytes.insert(bstr_bytes.end(), s.begin(), s.end());
  }
  bstr_off.push_back((uint32_t)bstr_bytes.size());
  if (bstr_bytes.empty()) bstr_bytes.push_back(0);
  if (heap.empty()) heap.push_back(0);
}

static std::pair<std::string, std::string> uid_from_json(const JVal& j) {
  const JVal* u = j.get("__entity");
  const JVal& x = u ? *u : j;
  return {x.str_or("type"), x.str_or("id")};
}

void decode_json_item(const JVal& item, std::vector<EntityIn>& ents, RequestIn& req) {
  const JVal* es = item.get("entities");
  const JVal* rq = item.get("request");
  if (!rq || rq->t != JVal::Obj) throw CedarError("item needs a \"request\" object");
  ents.clear();
  if (es) {
    if (es->t != JVal::Arr) throw CedarError("\"entities\" must be an array");
    for (auto& e : es->arr) {
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
