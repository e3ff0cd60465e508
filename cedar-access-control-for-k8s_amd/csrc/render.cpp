// Result renderer: device result records -> (Decision, cedar.Diagnostic) exactly as the reference
// returns them from TieredPolicyStores.IsAuthorized (internal/server/store/store.go:25-42) and
// serialises them with json.Marshal (authorizer.go:113-124; admission handler.go:64-66).
//
// Diagnostic JSON shape (cedar-go types.Diagnostic, omitempty slices):
//   {"reasons":[{"policy":ID,"position":{"filename":F,"offset":O,"line":L,"column":C}}],
//    "errors":[{"policy":ID,"position":{...},"message":M}]}
// Reasons/errors are listed in policy insertion order (canonical order; cedar-go's own order
// comes from Go map iteration and is not defined).
#include <algorithm>

#include "engine.h"

namespace cg {
using namespace cgi;

bool Batch::decision(uint32_t i) const { return (res[2 * (size_t)slot(i)] & 0xFF) == DEC_ALLOW; }
uint32_t Batch::tier(uint32_t i) const { return (res[2 * (size_t)slot(i)] >> 8) & 0xFF; }

void Batch::reason_ids(uint32_t i, std::vector<uint32_t>& out) const {
  out.clear();
  const uint32_t p = slot(i);
  uint32_t n = res[2 * (size_t)p + 1] & 0xFFFF;
  if (const BigRef* b = big_of(p)) {
    out.assign(b->r, b->r + b->nr);
  } else {
    uint32_t flags = res[2 * (size_t)p] >> 16;
    const uint32_t* src = (flags & RF_FORBID) ? reasons_f : reasons_p;
    for (uint32_t k = 0; k < n && k < capr; k++) out.push_back(src[(size_t)p * capr + k]);
  }
  // duplicate classes reported by their representative: every member, then policy order again
  // (the classes and the single policies are disjoint, so the list stays duplicate-free)
  bool cls = false;
  for (const uint32_t r : out) cls |= (r & RS_CLASS) != 0;
  if (!cls) return;
  const size_t n0 = out.size();
  for (size_t k = 0; k < n0; k++) {
    const uint32_t r = out[k];
    if (!(r & RS_CLASS)) continue;
    const uint32_t p = r & ~RS_CLASS;
    // (a word naming no class representative: an empty member range would be read past its end)
    if (img->cls_off.empty() || p + 1 >= img->cls_off.size() || img->cls_off[p] >= img->cls_off[p + 1] ||
        img->cls_off[p + 1] > img->cls_mem.size())
      throw CedarError("reason names an unknown duplicate class");
    out[k] = img->cls_mem[img->cls_off[p]];
    out.insert(out.end(), img->cls_mem.begin() + img->cls_off[p] + 1, img->cls_mem.begin() + img->cls_off[p + 1]);
  }
  std::sort(out.begin(), out.end());
}

void Batch::set_big(uint32_t p, const uint32_t* reasons, uint32_t nr, const uint32_t* errs, uint32_t nerr_words) {
  if (big_ix.empty()) big_ix.assign(n(), 0u);
  if (big_ix[p]) {
    bigs[big_ix[p] - 1] = BigRef{reasons, errs, nr, nerr_words};
  } else {
    bigs.push_back(BigRef{reasons, errs, nr, nerr_words});
    big_ix[p] = (uint32_t)bigs.size();
  }
}

void Batch::error_recs(uint32_t i, std::vector<uint32_t>& out) const {
  out.clear();
  const uint32_t p = slot(i);
  uint32_t n = res[2 * (size_t)p + 1] >> 16;
  if (const BigRef* b = big_of(p)) {
    out.assign(b->e, b->e + b->ne_words);
    return;
  }
  for (uint32_t k = 0; k < n && k < cape; k++)
    for (uint32_t w = 0; w < ERR_WORDS; w++) out.push_back(errs[((size_t)p * cape + k) * ERR_WORDS + w]);
}

static const char* type_name(uint32_t t) {
  switch (t) {
    case TN_BOOL: return "bool";
    case TN_LONG: return "long";
    case TN_STRING: return "string";
    case TN_ENTITY: return "entity";
    case TN_SET: return "set";
    case TN_RECORD: return "record";
    case TN_DECIMAL: return "decimal";
    case TN_IP: return "IP";
    case TN_ENTITY_OR_RECORD: return "entity or record";
    case TN_SET_OR_ENTITY: return "set or entity";
    default: return "unknown";
  }
}

static void quote(std::string& o, const std::string& s) {
  o += '"';
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  o += '"';
}

std::string Batch::error_message(uint32_t i, const uint32_t* rec) const {
  const PolicyMeta& m = img->meta[rec[0]];
  uint32_t code = rec[1] & 0xFF, aux = rec[1] >> 8;
  std::string body;
  switch (code) {
    case E_TYPE:
      body = std::string("type error: expected ") + type_name(aux & 0xFF) + ", got " + type_name((aux >> 8) & 0xFF);
      break;
    case E_ENTITY_MISSING:
      body = "entity `" + str(i, rec[3]) + "::";
      quote(body, str(i, rec[4]));
      body += "` does not exist";
      break;
    case E_ATTR_ENTITY:
      body = "`" + str(i, rec[3]) + "::";
      quote(body, str(i, rec[4]));
      body += "` does not have the attribute `" + str(i, rec[2]) + "`";
      break;
    case E_ATTR_RECORD: body = "record does not have the attribute `" + str(i, rec[2]) + "`"; break;
    case E_OVERFLOW: body = "integer overflow"; break;
    case E_EXT: body = aux < img->ext_msgs.size() ? img->ext_msgs[aux] : "extension error"; break;
    case E_EXT_ARG: body = std::string(aux ? "decimal" : "ip") + " takes one string argument"; break;
    case E_EXT_PARSE: body = std::string("error parsing ") + (aux ? "decimal" : "ip") + " value: " + str(i, rec[2]); break;
    case E_DEPTH: body = "value nesting exceeds the device evaluator limit"; break;
    case E_LANE: body = "device lane scratch exhausted"; break;
    default: body = "unknown evaluation error"; break;
  }
  return "while evaluating policy `" + m.id + "`: " + body;
}

static void pos_json(std::string& o, const PolicyMeta& m) {
  o += "{\"filename\":";
  go_json_string(o, m.filename);
  o += ",\"offset\":" + std::to_string(m.pos.offset) + ",\"line\":" + std::to_string(m.pos.line) +
       ",\"column\":" + std::to_string(m.pos.column) + "}";
}

void Batch::diagnostic_json(uint32_t i, std::string& out, bool reasons_only) const {
  std::vector<uint32_t> rs, es;
  reason_ids(i, rs);
  error_recs(i, es);
  std::string rj;
  rj += '[';
  for (size_t k = 0; k < rs.size(); k++) {
    const PolicyMeta& m = img->meta[rs[k]];
    if (k) rj += ',';
    rj += "{\"policy\":";
    go_json_string(rj, m.id);
    rj += ",\"position\":";
    pos_json(rj, m);
    rj += '}';
  }
  rj += ']';
  out.clear();
  if (reasons_only) { out = rj; return; }
  out += '{';
  bool any = false;
  if (!rs.empty()) { out += "\"reasons\":"; out += rj; any = true; }
  if (!es.empty()) {
    if (any) out += ',';
    out += "\"errors\":[";
    for (size_t k = 0; k < es.size() / ERR_WORDS; k++) {
      const uint32_t* rec = &es[k * ERR_WORDS];
      const PolicyMeta& m = img->meta[rec[0]];
      if (k) out += ',';
      out += "{\"policy\":";
      go_json_string(out, m.id);
      out += ",\"position\":";
      pos_json(out, m);
      out += ",\"message\":";
      go_json_string(out, error_message(i, rec));
      out += '}';
    }
    out += ']';
  }
  out += '}';
}

}  // namespace cg
