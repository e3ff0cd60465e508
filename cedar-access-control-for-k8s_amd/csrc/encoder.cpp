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

#include "encode_impl.h"

namespace cg {
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
  if (heap.size() + e.blk.size() > 0xFFFFFFFFull) throw CedarError("batch heap exceeds 16 GiB");
  // (the probe kernel addresses a row's words by a 32-bit offset, PCtx::rowo)
  if (rows.size() + row_words > 0xFFFFFFFFull) throw CedarError("batch rows exceed 16 GiB");
  size_t sbytes = 0;
  for (auto& s : e.strs) sbytes += s.size();
  if (n_bstr() + e.strs.size() >= 0xFFFFFFFFull || bstr_bytes.size() + sbytes > 0xFFFFFFFFull)
    throw CedarError("batch string table overflow");
  e.blk[RH_SBASE] = n_bstr();
  e.row[RW_BLK] = (uint32_t)heap.size();
  req_base.push_back((uint32_t)heap.size());
  heap.insert(heap.end(), e.blk.begin(), e.blk.end());
  rows.insert(rows.end(), e.row.begin(), e.row.end());
  gkeys.push_back(e.gkey);
  for (auto& s : e.strs) {
    bstr_bytes.insert(bstr_bytes.end(), s.begin(), s.end());
    bstr_off.push_back((uint32_t)bstr_bytes.size());
  }
}

void Batch::add(const std::vector<EntityIn>& ents, const RequestIn& req) {
  EncodedRequest e;
  encode_request(*img, ents, req, e);
  append(e);
}

// The string table is built as requests are appended; the device reads at least one byte and word.
void Batch::finalize_strings() {
  if (bstr_bytes.empty()) bstr_bytes.push_back(0);
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
