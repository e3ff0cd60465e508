// Host engine: compiled image, batch encoder, result renderer, device bridge.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "cedar.h"
#include "image.h"

namespace cg {

struct PolicyMeta {
  std::string id, filename;
  Position pos;
  uint32_t tier = 0;
  bool forbid = false;
};

// A compiled, immutable policy image (one per policy epoch). Device sections are the vectors
// uploaded verbatim; the rest is host-side metadata for rendering diagnostics.
struct Image {
  uint64_t epoch = 0;
  std::vector<uint32_t> pol, tier_end, code, cpool, gstr_off, hot;  // hot: HOT_WORDS per hot path
  // device policy stream: per policy a record [descriptor (POL_WORDS) | code, padded to 4 words]
  // with PW_CODE relative to the record; records grouped into chunks of <= CHUNK_WORDS words
  // that never cross a tier. chunks: (word offset, words, first policy, end policy) per chunk;
  // tier_cend[t] = end chunk index of tier t.
  std::vector<uint32_t> pstream, chunks, tier_cend;
  std::vector<uint32_t> act;  // action table: (type sid, id sid) pairs of every action entity in scopes
  uint32_t amask_ok = 0;      // 1 when act has <= MAX_ACT entries (PW_AMASK* valid)
  uint32_t n_atomic = 0;      // policies compiled to atoms (statistics)
  // scope index over atomic policies (image.h "scope index"); indexed = every policy is atomic
  std::vector<uint32_t> btab, brefs, bstream;
  uint32_t indexed = 0;
  uint32_t combo_mask = 0;  // level-1 key combos in use (bit key_combo(..))
  std::vector<uint8_t> gstr_bytes;
  std::vector<PolicyMeta> meta;
  std::vector<std::string> strings;
  std::unordered_map<std::string, uint32_t> sid;
  std::vector<std::string> ext_msgs;
  uint32_t n_tiers() const { return (uint32_t)tier_end.size(); }
  uint32_t n_pol() const { return (uint32_t)meta.size(); }
  uint32_t n_gstr() const { return (uint32_t)strings.size(); }
  uint32_t n_hot() const { return (uint32_t)hot.size() / cgi::HOT_WORDS; }
  uint32_t row_words() const { return (cgi::RW_HDR + 2 * n_hot() + 3) & ~3u; }
  int32_t find(const std::string& s) const {
    auto it = sid.find(s);
    return it == sid.end() ? -1 : (int32_t)it->second;
  }
  std::vector<uint8_t> serialize() const;
  static std::shared_ptr<Image> deserialize(const uint8_t* p, size_t n);
};

// One document (a policy file / CRD content / AVP statement) inside a tier.
struct DocSpec {
  std::string filename, text, id_prefix, id_suffix;
  std::string explicit_id;  // when set: the document holds exactly one policy with this ID
  bool zero_position = false;  // policies built from AST (e.g. allow-all-admission) carry Position{}
};

std::shared_ptr<Image> compile_image(const std::vector<std::vector<DocSpec>>& tiers, uint64_t epoch);

// Entity input for the encoder (already decoded from JSON or built by the k8s model).
struct EntityIn {
  std::string type, id;
  HVal attrs;  // Record
  std::vector<std::pair<std::string, std::string>> parents;
};
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
  std::vector<std::string> strs;   // request-local strings
  std::unordered_map<std::string, uint32_t> local;
  void clear() { blk.clear(); row.clear(); strs.clear(); local.clear(); }
};
// Encodes (EntityMap, Request) for `img`. Thread-safe: reads the image only.
void encode_request(const Image& img, const std::vector<EntityIn>& ents, const RequestIn& req, EncodedRequest& out);

// Host side of a device batch: encoded request heap + string table; results after evaluation.
struct Batch {
  std::shared_ptr<const Image> img;
  std::vector<uint32_t> heap, req_base;
  std::vector<uint32_t> rows;  // columnar request rows (image.h RowW), row_words each
  uint32_t row_words = 0;
  std::vector<std::string> bstrings;  // request-local strings of every request, concatenated
  std::vector<uint32_t> bstr_off;
  std::vector<uint8_t> bstr_bytes;
  // results
  uint32_t capr = 8, cape = 4;
  std::vector<uint32_t> res, reasons_f, reasons_p, errs;
  // per-request overflow re-run results (index -> reasons / errors)
  std::unordered_map<uint32_t, std::vector<uint32_t>> big_reasons, big_errs;

  uint32_t n() const { return (uint32_t)req_base.size(); }
  // string `id` as request i sees it
  const std::string& str(uint32_t i, uint32_t id) const;
  void add(const std::vector<EntityIn>& ents, const RequestIn& req);  // encode_request + append
  void append(EncodedRequest& e);                                     // moves e's strings
  void finalize_strings();
  // decision: 1 allow, 0 deny; fills the Go-JSON rendering of the cedar.Diagnostic
  bool decision(uint32_t i) const;
  void diagnostic_json(uint32_t i, std::string& out, bool reasons_only) const;
  void reason_ids(uint32_t i, std::vector<uint32_t>& out) const;
  void error_recs(uint32_t i, std::vector<uint32_t>& out) const;
  std::string error_message(uint32_t i, const uint32_t* rec) const;
};

// Parses a Cedar-JSON request item {"entities": [...], "request": {...}} into encoder input.
void decode_json_item(const JVal& item, std::vector<EntityIn>& ents, RequestIn& req);

}  // namespace cg
