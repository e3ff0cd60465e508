// C-ABI implementation (include/cedargpu.h). No exception crosses this boundary.
#include <algorithm>
#include <array>
#include <chrono>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "admission.h"
#include "capi_internal.h"
#include "delta.h"
#include "encode_impl.h"
#include "sar.h"

namespace {
// CEDARGPU_TRACE_LAT=1: one stderr line per submit / wait with the microseconds of each phase
// (diagnostic only; off by default).
struct LatTrace {
  static bool on() {
    static const bool v = [] { const char* e = std::getenv("CEDARGPU_TRACE_LAT"); return e && *e == '1'; }();
    return v;
  }
  const char* what;
  std::chrono::steady_clock::time_point t;
  std::string line;
  explicit LatTrace(const char* w) : what(w) { if (on()) t = std::chrono::steady_clock::now(); }
  void mark(const char* phase) {
    if (!on()) return;
    auto n = std::chrono::steady_clock::now();
    line += " "; line += phase; line += "=";
    line += std::to_string(std::chrono::duration<double, std::micro>(n - t).count());
    t = n;
  }
  void val(const char* k, double v) {
    if (!on()) return;
    line += " "; line += k; line += "="; line += std::to_string(v);
  }
  ~LatTrace() { if (on() && !line.empty()) std::fprintf(stderr, "LAT %s%s\n", what, line.c_str()); }
};
}  // namespace

using namespace cg;

struct cg_compiler {
  std::vector<std::vector<DocSpec>> tiers;
  std::vector<EntityIn> statics;  // the image's static entities (cg_compiler_set_entities)
  std::vector<DocError> skipped;  // documents the last build left out (CG_DOC_SKIP_INVALID)
  ParseCache cache;  // parsed documents reused across builds
  std::unique_ptr<LowerState, LowerDeleter> lower = make_lower_state();  // lowered documents (incremental builds)
  bool incremental = true;
  uint64_t statics_gen = 0;  // bumped by every cg_compiler_set_entities that changes them
  std::string statics_json;
  BuildInfo last;
  std::string err;
  std::shared_ptr<Image> built;  // cg_compiler_build_sized's image until cg_compiler_write_image
  size_t built_len = 0;
};

namespace {

// Element texts of a top-level JSON array (bracket / string balance only; each element is parsed
// on its own afterwards). False when the text is not an array. One pass: string bodies are skipped
// with memchr (most of a SubjectAccessReview's bytes), everything else through a byte-class table.
bool split_array_serial(const char* p, size_t n, std::vector<std::pair<size_t, size_t>>& out) {
  enum : uint8_t { C_OTHER = 0, C_WS, C_QUOTE, C_OPEN, C_CLOSE, C_COMMA };
  static const auto cls = [] {
    std::array<uint8_t, 256> t{};
    t[' '] = t['\t'] = t['\n'] = t['\r'] = t['\f'] = t['\v'] = C_WS;
    t['"'] = C_QUOTE;
    t['['] = t['{'] = C_OPEN;
    t[']'] = t['}'] = C_CLOSE;
    t[','] = C_COMMA;
    return t;
  }();
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  size_t i = 0;
  while (i < n && cls[u[i]] == C_WS) i++;
  if (i == n || p[i] != '[') return false;
  i++;
  out.reserve(out.size() + n / 256);
  int depth = 0;
  size_t start = std::string::npos;
  while (i < n) {
    switch (cls[u[i]]) {
      case C_WS:
        i++;
        continue;
      case C_QUOTE: {
        if (start == std::string::npos) start = i;
        size_t j = i + 1;
        for (;;) {  // the closing quote: one not preceded by an odd run of backslashes
          const void* q = std::memchr(p + j, '"', n - j);
          if (!q) return false;
          j = (size_t)((const char*)q - p);
          size_t bs = 0;
          while (j - bs > i + 1 && p[j - 1 - bs] == '\\') bs++;
          if (!(bs & 1)) break;
          j++;
        }
        i = j + 1;
        continue;
      }
      case C_OPEN:
        if (start == std::string::npos) start = i;
        depth++;
        break;
      case C_CLOSE:
        if (depth == 0) {  // end of the top-level array
          if (start != std::string::npos) out.emplace_back(start, i - start);
          return true;
        }
        depth--;
        break;
      case C_COMMA:
        if (depth == 0) {
          if (start == std::string::npos) return false;
          out.emplace_back(start, i - start);
          start = std::string::npos;
        }
        break;
      default:
        if (start == std::string::npos) start = i;
        break;
    }
    i++;
  }
  return false;
}

// The same over a large text on several threads. A quote is unescaped when an even run of
// backslashes precedes it, which each thread sees in the bytes themselves, so its region's quote
// parity and its bracket-depth change (for both string states at its start) need no neighbour;
// prefix sums over the regions then give each region's starting state, and a second pass lists the
// elements that start in each region. Falls back to the serial scan on anything unusual.
bool split_array_regions(const char* p, size_t n, std::vector<std::pair<size_t, size_t>>& out, unsigned T);
bool split_array(const char* p, size_t n, std::vector<std::pair<size_t, size_t>>& out) {
  unsigned T = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (const char* e = std::getenv("CEDARGPU_HOST_THREADS")) T = (unsigned)std::max(1, std::atoi(e));
  if (n < (8u << 20) || T < 2) return split_array_serial(p, n, out);
  return split_array_regions(p, n, out, T);
}
bool split_array_regions(const char* p, size_t n, std::vector<std::pair<size_t, size_t>>& out, unsigned T) {
  T = (unsigned)std::max<size_t>(1, std::min<size_t>(T, n / 2 + 1));
  size_t lo = 0;
  while (lo < n && std::isspace((unsigned char)p[lo])) lo++;
  if (lo == n || p[lo] != '[') return false;
  lo++;
  auto unescaped = [&](size_t j) {  // p[j] == '"' and not escaped
    size_t bs = 0;
    while (j - bs > 0 && p[j - 1 - bs] == '\\') bs++;
    return !(bs & 1);
  };
  struct Reg {
    size_t b, e;
    uint64_t quotes = 0;           // unescaped quotes in the region
    int64_t depth[2] = {0, 0};     // depth change starting outside / inside a string
    bool in = false;               // the string state at its start (from the prefix)
    int64_t d0 = 0;                // the depth at its start
    std::vector<std::pair<size_t, size_t>> el;
    size_t open = std::string::npos;  // an element still open at the region's end (its start)
    bool bad = false, done = false;
  };
  std::vector<Reg> rg(T);
  for (unsigned t = 0; t < T; t++) { rg[t].b = lo + (n - lo) * t / T; rg[t].e = lo + (n - lo) * (t + 1) / T; }
  auto par = [&](auto&& fn) {
    std::vector<std::thread> ws;
    for (unsigned t = 1; t < T; t++) ws.emplace_back(fn, t);
    fn(0u);
    for (auto& w : ws) w.join();
  };
  // pass 1, one sweep: the two string states at a region's start stay complementary at every byte
  // (the same quotes toggle both), so a bracket counts towards the state it is outside of
  par([&](unsigned t) {
    Reg& r = rg[t];
    const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
    bool in = false;  // (starting outside)
    int64_t d[2] = {0, 0};
    uint64_t q = 0;
    for (size_t i = r.b; i < r.e; i++) {
      const unsigned char c = u[i];
      if (c == '"') {
        if (unescaped(i)) { in = !in; q++; }
        continue;
      }
      const int delta = (c == '[' || c == '{') ? 1 : (c == ']' || c == '}') ? -1 : 0;
      if (delta) d[in ? 1 : 0] += delta;
    }
    r.depth[0] = d[0];
    r.depth[1] = d[1];
    r.quotes = q;
  });
  bool in = false;
  int64_t d = 0;
  for (auto& r : rg) {
    r.in = in;
    r.d0 = d;
    d += r.depth[in ? 1 : 0];
    if (r.quotes & 1) in = !in;
  }
  // second pass: the separators at the array's own level (depth 0, outside strings): its commas,
  // and its closing bracket (in the first region that reaches it)
  par([&](unsigned t) {
    Reg& r = rg[t];
    bool in2 = r.in;
    int64_t dd = r.d0;
    for (size_t i = r.b; i < r.e; i++) {
      if (in2) {  // to the closing quote, at memchr speed
        const void* qp = std::memchr(p + i, '"', r.e - i);
        if (!qp) break;
        i = (size_t)((const char*)qp - p);
        if (unescaped(i)) in2 = false;
        continue;
      }
      const char c = p[i];
      if (c == '"') { if (unescaped(i)) in2 = true; continue; }
      if (c == '[' || c == '{') { dd++; continue; }
      if (c == ']' || c == '}') {
        if (dd == 0) { r.el.emplace_back(i, 1); r.done = true; return; }  // the array's end
        dd--;
        continue;
      }
      if (c == ',' && dd == 0) r.el.emplace_back(i, 0);
    }
    if (dd < 0) r.bad = true;
  });
  // elements between consecutive separators, as the serial scan cuts them: from the first
  // non-space byte after a separator up to the next separator; an empty one before a comma is an
  // error, an empty one before the closing bracket ends the array
  size_t prev = lo - 1;  // the '['
  bool ended = false;
  for (unsigned t = 0; t < T && !ended; t++) {
    const Reg& r = rg[t];
    if (r.bad) { out.clear(); return split_array_serial(p, n, out); }
    for (const auto& sp : r.el) {
      size_t st = prev + 1;
      while (st < sp.first && std::isspace((unsigned char)p[st])) st++;
      if (st == sp.first) {
        if (!sp.second) return false;  // `[,` or `,,`
      } else {
        out.emplace_back(st, sp.first - st);
      }
      prev = sp.first;
      if (sp.second) { ended = true; break; }
    }
  }
  return ended;
}

// Worker threads for host-side bulk work: at most 16 (a GPU's share of host cores), and one per
// 256 items.
unsigned host_workers(size_t items) {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  if (const char* e = std::getenv("CEDARGPU_HOST_THREADS")) hw = (unsigned)std::max(1, std::atoi(e));
  else hw = std::min(hw, 16u);
  return (unsigned)std::max<size_t>(1, std::min<size_t>(hw, items / 256));
}

template <class F>
void parallel_for(size_t n, F&& f) {
  const unsigned t = host_workers(n);
  if (t <= 1) { for (size_t i = 0; i < n; i++) f(i); return; }
  std::atomic<size_t> next{0};
  std::vector<std::thread> ws;
  for (unsigned k = 0; k < t; k++)
    ws.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(64)) < n;)
        for (size_t j = i; j < std::min(n, i + 64); j++) f(j);
    });
  for (auto& w : ws) w.join();
}

// Request grouping (batching layer). The batch's rows are ordered by (action, resource type),
// then the principal's type and groups, then its hot attribute values, before upload. The four
// requests of a wave then take the same scope-index buckets and candidate policies, so the wave's
// collective loops converge and neighbouring waves share image lines in L2: C3 1M-request
// launches went from 870M to 1.15B decisions/s (profiles/r01/group_ab). Rows and request bases
// move to their new slots and items map to the slots, so every result accessor reads its own
// request. Throughput batches (>= 65,536 requests) only: a radix sort plus the row permutation
// costs ~50 ns of host time per request (~2 ms at 32,768), more than a smaller batch's kernel
// wins back (C4 at 32,768: kernel 1.32 -> 0.81 ms, submit -> results 7.4 -> 8.0 ms).
// CEDARGPU_GROUP=1 / 0 forces it.
// Round 3: the order is computed on the device inside every evaluation step (group.hip: a grouping
// key per request and a rocPRIM radix sort; the kernels read requests in that order), so a batch
// costs no host sort and the timed step includes its ordering. CEDARGPU_GROUP_DEV=0 keeps the host
// sort below (A/B).
void group_requests(cg_batch* b) {
  Batch& h = b->host;
  const uint32_t n = h.n(), rw = h.row_words;
  bool on = n >= 65536u;
  if (const char* e = std::getenv("CEDARGPU_GROUP")) on = *e == '1';
  static const bool dev = !(std::getenv("CEDARGPU_GROUP_DEV") && *std::getenv("CEDARGPU_GROUP_DEV") == '0');
  h.dev_group = false;
  if (!on || n < 2 || n >= (1u << 24) || !rw || h.rows.size() != (size_t)n * rw) return;
  if (dev) { h.dev_group = true; return; }
  auto mix = [](uint64_t k, uint32_t w) {
    k ^= w;
    k *= 0xff51afd7ed558ccdull;
    return k ^ (k >> 29);
  };
  // one 64-bit key per request: 12 bits of (action, resource type) | the principal's type and
  // groups in the bits left over | 8 bits of its hot values | its position in ceil(log2 n) bits
  // (ties keep batch order).
  // Hash fields group equal values; unequal values sharing a field only cost locality.
  // position bits: just enough for n; the groups field takes the rest between the fixed fields
  uint32_t ib = 1;
  while ((1ull << ib) < n) ib++;
  const uint64_t imask = (1ull << ib) - 1, hmask = 0xFFull << ib;
  const uint64_t gmask = ((1ull << 52) - 1) & ~((1ull << (ib + 8)) - 1);
  std::vector<uint64_t> key(n), tmp(n);
  parallel_for(n, [&](size_t i) {
    const uint32_t* row = h.rows.data() + i * rw;
    const uint64_t ar = mix(mix(0x51ED27Fu, row[cgi::RW_A + 1]), row[cgi::RW_R]);
    // groups: the principal's ancestor (type, id) pairs
    uint64_t g = mix(0x9E3779B97F4A7C15ull, row[cgi::RW_P]);
    const size_t anc = (uint32_t)(row[cgi::RW_BLK] + row[cgi::RW_PANC]);  // (signed offset: mod 2^32)
    for (uint32_t j = 0; j < 2 * (row[cgi::RW_PN] & cgi::AN_COUNT) && anc + j < h.heap.size(); j++) g = mix(g, h.heap[anc + j]);
    uint64_t hv = 0x2545F4914F6CDD1Dull;
    for (uint32_t j = cgi::RW_HDR; j < rw; j++) hv = mix(hv, row[j]);
    key[i] = ((ar >> 52) << 52) | (((g >> 40) << (64 - 12 - 24)) & gmask) | (((hv >> 56) << ib) & hmask) | (uint64_t)i;
  });
  // LSD radix sort on the key bits above the position (11-bit digits)
  for (uint32_t sh = ib; sh < 64; sh += 11) {
    std::vector<uint32_t> cnt(2049, 0);
    for (uint32_t i = 0; i < n; i++) cnt[((key[i] >> sh) & 2047u) + 1]++;
    for (uint32_t d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
    for (uint32_t i = 0; i < n; i++) tmp[cnt[(key[i] >> sh) & 2047u]++] = key[i];
    key.swap(tmp);
  }
  PinVec<uint32_t> rows((size_t)n * rw), base(n), gk(h.gkeys.size());
  std::vector<uint32_t> slot(n);
  parallel_for(n, [&](size_t s) {
    const uint32_t o = (uint32_t)(key[s] & imask);
    std::memcpy(rows.data() + s * rw, h.rows.data() + (size_t)o * rw, (size_t)rw * 4);
    base[s] = h.req_base[o];
    slot[o] = (uint32_t)s;
    if (!gk.empty()) gk[s] = h.gkeys[o];
  });
  h.rows.swap(rows);
  h.req_base.swap(base);
  h.gkeys.swap(gk);
  for (auto& it : b->items)
    if (it.dev >= 0) it.dev = (int32_t)slot[(uint32_t)it.dev];
}

// CG_FAULT_BAD_KIDX: every principal's key-entity indices (image.h "scope bitsets") pushed past
// the image's key entities, as a batch encoded for another image would carry them (lists are
// shared between requests: the change is idempotent).
void corrupt_key_indices(Batch& h) {
  if (!h.img->sbits_words) return;
  const uint32_t rw = h.row_words;
  for (uint32_t i = 0; i < h.n(); i++) {
    const uint32_t* row = h.rows.data() + (size_t)i * rw;
    if (!row[cgi::RW_PANC]) continue;
    const uint32_t pn = row[cgi::RW_PN], n = pn & cgi::AN_COUNT, keys = (pn >> cgi::AN_KEYS_SHIFT) & cgi::AN_KEYS;
    uint32_t* kl = h.heap.data() + (uint32_t)(row[cgi::RW_BLK] + row[cgi::RW_PANC]) + 2 * (size_t)n;
    for (uint32_t j = 0; j <= keys; j++)
      if (kl[j] != cgi::KIDX_NONE) kl[j] |= 0x40000000u;
  }
}

// Bulk encoding (cg_batch_add_sar_json / cg_batch_add_admission_json over a JSON array of at least
// 64 KiB). The elements split into contiguous chunks; worker threads take chunks in turn and encode
// each element straight into the chunk's own Batch part (ancestor lists interned per part), and the
// parts are concatenated in order with their offsets shifted, side by side (Batch::concat). No
// per-element buffers and no serial append. All or nothing: the first failing element's error is
// returned and the batch is left as it was.
struct BulkOut {
  bool host = false;  // decided on the host (fast path / skip / review error): no device request
  int fast = -1;
  std::string reason;
};
template <class F>  // f(element k, EncodedRequest& e, BulkOut& o): encodes e, or sets o.host
int bulk_add(cg_batch* b, size_t n, F&& f) {
  LatTrace tr("bulk");
  const unsigned t = host_workers(n);
  // chunks per worker (CEDARGPU_ENCODE_CHUNKS, default 1): each chunk is a batch part whose
  // ancestor lists are interned on their own, so fewer, larger parts share more (1M C3 SARs:
  // 533 B of upload per request at 8 chunks per worker, 517 at 2, 500 at 1, the encode as fast)
  static const size_t cpt = [] { const char* e = std::getenv("CEDARGPU_ENCODE_CHUNKS"); return e ? (size_t)std::max(1, std::atoi(e)) : 1u; }();
  const size_t per = std::max<size_t>(256, (n + cpt * t - 1) / (cpt * t));
  const size_t nc = (n + per - 1) / per;
  struct Chunk {
    Batch part;
    std::vector<int32_t> fast;  // per element: -1 a device request, else its host result
    std::vector<std::pair<uint32_t, std::string>> reasons;  // (element in chunk, reason / error text)
    int rc = CG_OK;
    std::string err;
  };
  std::vector<Chunk> ch(nc);
  for (auto& c : ch) c.part.img = b->host.img;
  std::atomic<size_t> next{0};
  auto work = [&] {
    EncodedRequest e;
    BulkOut o;
    for (size_t c; (c = next++) < nc;) {
      Chunk& C = ch[c];
      const size_t lo = c * per, hi = std::min(n, lo + per);
      C.fast.reserve(hi - lo);
      for (size_t k = lo; k < hi; k++) {
        o.host = false;
        o.fast = -1;
        o.reason.clear();
        try {
          f(k, e, o);
          if (!o.host) C.part.append(e);
        } catch (const CedarError& x) {
          C.rc = CG_E_PARSE; C.err = x.what();
        } catch (const std::bad_alloc&) {
          C.rc = CG_E_ARG; C.err = "out of host memory";
        } catch (const std::exception& x) {
          C.rc = CG_E_ARG; C.err = x.what();
        }
        if (C.rc) break;
        if (o.host && !o.reason.empty()) C.reasons.emplace_back((uint32_t)(k - lo), std::move(o.reason));
        C.fast.push_back(o.host ? o.fast : -1);
      }
    }
  };
  {
    std::vector<std::thread> ws;
    for (unsigned k = 1; k < t; k++) ws.emplace_back(work);
    work();
    for (auto& w : ws) w.join();
  }
  tr.mark("encode");
  for (auto& c : ch)  // chunks are contiguous and stop at their first failure: the first one in order
    if (c.rc) { b->err = c.err; return c.rc; }
  GUARD(b->err, {
    size_t n_items = b->items.size();
    for (auto& c : ch) n_items += c.fast.size();
    b->items.reserve(n_items);
    int32_t dev = (int32_t)b->host.n();
    std::vector<Batch> parts;
    parts.reserve(nc);
    for (auto& c : ch) {
      const uint32_t i0 = (uint32_t)b->items.size();
      for (const int32_t f : c.fast) b->items.push_back(f < 0 ? cg_batch::Item{dev++, -1} : cg_batch::Item{-1, f});
      for (auto& r : c.reasons) b->fast_reason[i0 + r.first] = std::move(r.second);
      parts.push_back(std::move(c.part));
    }
    ch.clear();
    tr.mark("items");
    b->host.concat(parts, t);
    tr.mark("concat");
    return CG_OK;
  })
}

// cg_encode_sar_check: every SAR of the array through the direct path and the general path.
int encode_sar_check(const void* image, size_t len, const char* sars, size_t n, uint32_t* n_items, uint32_t* n_direct,
                     uint32_t* n_mismatch, int64_t* first_mismatch) {
  auto img = Image::deserialize((const uint8_t*)image, len);
  std::vector<std::pair<size_t, size_t>> elems;
  if (!split_array(sars, n, elems)) throw CedarError("expected a JSON array");
  uint32_t nd = 0, nm = 0;
  int64_t first = -1;
  for (size_t k = 0; k < elems.size(); k++) {
    const char* p = sars + elems[k].first;
    const size_t m = elems[k].second;
    EncodedRequest direct;
    int fast_d = -1;
    std::string reason_d;
    const int d = encode_sar_direct(*img, p, m, direct, fast_d, reason_d);
    if (!d) continue;
    nd++;
    JVal v = json_parse(p, m);
    Attributes at = attributes_from_sar(v);
    std::string reason_g;
    const int fast_g = authorize_fast_path(at, reason_g);
    bool same;
    if (fast_g >= 0) {
      same = d == 2 && fast_d == fast_g && reason_d == reason_g;
    } else {
      std::vector<EntityIn> ents;
      RequestIn req;
      record_to_cedar(at, ents, req);
      EncodedRequest general;
      // the general path walks every hierarchy itself, so the direct path's cached ancestor
      // records (encode_impl.h ClosureCache) are checked against the walk word for word
      enc::t_no_closure_cache = true;
      try {
        encode_request(*img, ents, req, general);
      } catch (...) {
        enc::t_no_closure_cache = false;
        throw;
      }
      enc::t_no_closure_cache = false;
      same = d == 1 && direct.blk == general.blk && direct.row == general.row && direct.strs == general.strs &&
             direct.anc == general.anc && direct.anc_at == general.anc_at;
    }
    if (!same) {
      nm++;
      if (first < 0) first = (int64_t)k;
    }
  }
  if (n_items) *n_items = (uint32_t)elems.size();
  if (n_direct) *n_direct = nd;
  if (n_mismatch) *n_mismatch = nm;
  if (first_mismatch) *first_mismatch = first;
  return CG_OK;
}

// {"entities":[...],"request":{...}} (Cedar JSON) of an (EntityMap, Request)
void cedar_item_json(const std::vector<EntityIn>& ents, const RequestIn& req, std::string& s) {
  auto uid = [&s](const std::pair<std::string, std::string>& u) {
    s += "{\"type\":"; go_json_string(s, u.first); s += ",\"id\":"; go_json_string(s, u.second); s += "}";
  };
  s = "{\"entities\":[";
  for (size_t k = 0; k < ents.size(); k++) {
    if (k) s += ',';
    s += "{\"uid\":";
    uid({ents[k].type, ents[k].id});
    s += ",\"attrs\":";
    hval_to_json(ents[k].attrs, s);
    s += ",\"parents\":[";
    for (size_t p = 0; p < ents[k].parents.size(); p++) { if (p) s += ','; uid(ents[k].parents[p]); }
    s += "]}";
  }
  s += "],\"request\":{\"principal\":";
  uid(req.principal);
  s += ",\"action\":";
  uid(req.action);
  s += ",\"resource\":";
  uid(req.resource);
  s += ",\"context\":";
  hval_to_json(req.context, s);
  s += "}}";
}

}  // namespace

extern "C" {

const char* cg_version(void) { return "cedargpu 0.1.0 (gfx950)"; }
void cg_free(void* p) { std::free(p); }

// ---------------------------------------------------------------------------------------------
int cg_compiler_create(cg_compiler** out) {
  if (!out) return CG_E_ARG;
  *out = new (std::nothrow) cg_compiler();
  return *out ? CG_OK : CG_E_ARG;
}
void cg_compiler_destroy(cg_compiler* c) { delete c; }
const char* cg_compiler_last_error(cg_compiler* c) { return c ? c->err.c_str() : "null compiler"; }

int cg_compiler_clear(cg_compiler* c) {
  if (!c) return CG_E_ARG;
  c->tiers.clear();
  return CG_OK;
}

int cg_compiler_cache_stats(cg_compiler* c, uint64_t* hits, uint64_t* misses, uint64_t* entries) {
  if (!c) return CG_E_ARG;
  if (hits) *hits = c->cache.hits;
  if (misses) *misses = c->cache.misses;
  if (entries) {
    uint64_t n = 0;
    for (auto& kv : c->cache.map) n += kv.second.size();
    *entries = n;
  }
  return CG_OK;
}

int cg_compiler_set_incremental(cg_compiler* c, int on) {
  if (!c) return CG_E_ARG;
  c->incremental = on != 0;
  if (!on) c->lower = make_lower_state();  // drop the arenas
  return CG_OK;
}

int cg_compiler_last_build(cg_compiler* c, int* incremental, uint64_t* lowered, uint64_t* reused, const char** why_full) {
  if (!c) return CG_E_ARG;
  if (incremental) *incremental = c->last.incremental ? 1 : 0;
  if (lowered) *lowered = c->last.lowered;
  if (reused) *reused = c->last.reused;
  if (why_full) *why_full = c->last.why_full;
  return CG_OK;
}

int cg_compiler_set_entities(cg_compiler* c, const char* json, size_t len) {
  if (!c || (!json && len)) return CG_E_ARG;
  GUARD(c->err, {
    if (c->statics_json.size() == len && (!len || std::memcmp(c->statics_json.data(), json, len) == 0)) return CG_OK;
    std::vector<EntityIn> ents;
    if (len) decode_json_entities(json_parse(json, len), ents);
    c->statics = std::move(ents);
    c->statics_json.assign(json ? json : "", len);
    c->statics_gen++;
    return CG_OK;
  })
}

int cg_compiler_add_tier(cg_compiler* c) {
  if (!c) return CG_E_ARG;
  c->tiers.emplace_back();
  return CG_OK;
}

int cg_compiler_add_document_ex(cg_compiler* c, const char* filename, const char* text, size_t len, const char* id_prefix,
                                const char* id_suffix, int flags) {
  if (!c || (!text && len) || (flags & ~CG_DOC_SKIP_INVALID)) return CG_E_ARG;
  GUARD(c->err, {
    DocSpec d;
    d.filename = filename ? filename : "";
    d.text.assign(text ? text : "", len);
    d.id_prefix = id_prefix ? id_prefix : "policy";
    d.id_suffix = id_suffix ? id_suffix : "";
    d.skip_invalid = (flags & CG_DOC_SKIP_INVALID) != 0;
    if (c->tiers.empty()) c->tiers.emplace_back();  // parsed by the build (on workers, cached)
    c->tiers.back().push_back(std::move(d));
    return CG_OK;
  })
}

int cg_compiler_add_document(cg_compiler* c, const char* filename, const char* text, size_t len, const char* id_prefix,
                             const char* id_suffix) {
  return cg_compiler_add_document_ex(c, filename, text, len, id_prefix, id_suffix, 0);
}

int cg_compiler_add_policy(cg_compiler* c, const char* policy_id, const char* filename, const char* text, size_t len,
                           int zero_position) {
  if (!c || !policy_id || !*policy_id || (!text && len)) return CG_E_ARG;
  GUARD(c->err, {
    DocSpec d;
    d.filename = filename ? filename : "";
    d.text.assign(text ? text : "", len);
    d.explicit_id = policy_id;
    d.zero_position = zero_position != 0;
    if (c->tiers.empty()) c->tiers.emplace_back();  // the build checks it holds exactly one policy
    c->tiers.back().push_back(std::move(d));
    return CG_OK;
  })
}

int cg_compiler_doc_errors(cg_compiler* c, char* buf, size_t cap, size_t* need) {
  if (!c) return CG_E_ARG;
  std::string s = "[";
  for (size_t k = 0; k < c->skipped.size(); k++) {
    if (k) s += ",";
    s += "{\"filename\":";
    go_json_string(s, c->skipped[k].filename);
    s += ",\"error\":";
    go_json_string(s, c->skipped[k].error);
    s += "}";
  }
  s += "]";
  if (need) *need = s.size() + 1;
  if (!buf || cap < s.size() + 1) return buf ? CG_E_RANGE : CG_OK;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return CG_OK;
}

int cg_compiler_build(cg_compiler* c, uint64_t epoch, uint8_t** image, size_t* len) {
  if (!c || !image || !len) return CG_E_ARG;
  try {
    c->skipped.clear();
    auto img = compile_image(c->tiers, epoch, &c->cache, &c->statics, &c->skipped, c->incremental ? c->lower.get() : nullptr,
                             c->statics_gen, &c->last);
    size_t n = 0;
    uint8_t* p = img->serialize_malloc(&n);
    if (!p) { c->err = "out of host memory"; return CG_E_ARG; }
    *image = p;
    *len = n;
    return CG_OK;
  } catch (const CedarError& e) {
    c->err = e.what();
    std::string m = e.what();
    return (m.find("device") != std::string::npos || m.find("not supported") != std::string::npos) ? CG_E_COMPILE : CG_E_PARSE;
  } catch (const std::exception& e) {
    c->err = e.what();
    return CG_E_ARG;
  }
}

int cg_compiler_build_sized(cg_compiler* c, uint64_t epoch, size_t* len) {
  if (!c || !len) return CG_E_ARG;
  try {
    c->skipped.clear();
    c->built.reset();
    c->built = compile_image(c->tiers, epoch, &c->cache, &c->statics, &c->skipped, c->incremental ? c->lower.get() : nullptr,
                             c->statics_gen, &c->last);
    *len = c->built_len = c->built->blob_size();
    return CG_OK;
  } catch (const CedarError& e) {
    c->err = e.what();
    std::string m = e.what();
    return (m.find("device") != std::string::npos || m.find("not supported") != std::string::npos) ? CG_E_COMPILE : CG_E_PARSE;
  } catch (const std::exception& e) {
    c->err = e.what();
    return CG_E_ARG;
  }
}

int cg_compiler_write_image(cg_compiler* c, void* out, size_t cap) {
  if (!c || !out) return CG_E_ARG;
  if (!c->built) { c->err = "no image built (cg_compiler_build_sized)"; return CG_E_STATE; }
  if (cap < c->built_len) { c->err = "buffer smaller than the image blob"; return CG_E_RANGE; }
  try {
    c->built->serialize_into((uint8_t*)out);
  } catch (const std::exception& e) {
    c->err = e.what();
    return CG_E_ARG;
  }
  c->built.reset();
  return CG_OK;
}

int cg_image_info(const void* image, size_t len, uint32_t* n_policies, uint32_t* n_tiers, uint64_t* epoch) {
  if (!image) return CG_E_ARG;
  try {
    auto img = Image::deserialize((const uint8_t*)image, len);
    if (n_policies) *n_policies = img->n_pol();
    if (n_tiers) *n_tiers = img->n_tiers();
    if (epoch) *epoch = img->epoch;
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_image_stats(const void* image, size_t len, uint32_t* n_atomic, uint32_t* n_hot, uint32_t* n_actions,
                   uint32_t* stream_words) {
  if (!image) return CG_E_ARG;
  try {
    auto img = Image::deserialize((const uint8_t*)image, len);
    if (n_atomic) *n_atomic = img->n_atomic;
    if (n_hot) *n_hot = (uint32_t)img->hot.size() / cgi::HOT_WORDS;
    if (n_actions) *n_actions = (uint32_t)img->act.size() / 2;
    if (stream_words) *stream_words = (uint32_t)(img->dev_len[cgi::DS_PSTREAM] / 4);
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_image_index_stats(const void* image, size_t len, uint32_t* cslot_mask, uint32_t* pslot_mask, uint32_t* combo_mask,
                         uint32_t* entries, uint32_t* contexts, uint32_t* sbits_words) {
  if (!image) return CG_E_ARG;
  try {
    auto img = Image::deserialize((const uint8_t*)image, len);
    if (cslot_mask) *cslot_mask = img->cslot_mask;
    if (pslot_mask) *pslot_mask = img->pslot_mask;
    if (combo_mask) *combo_mask = img->combo_mask;
    if (entries) *entries = (uint32_t)(img->dev_len[cgi::DS_BTAB] / 4 / cgi::BT_WORDS);
    if (contexts) *contexts = img->sbits_words ? (uint32_t)(img->dev_len[cgi::DS_SBITS] / 8 / img->sbits_words) : 0u;
    if (sbits_words) *sbits_words = img->sbits_words;
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

// ---------------------------------------------------------------------------------------------
int cg_image_like_slots(const void* image, size_t len, uint32_t* row_like_mask, uint32_t* like_read_mask) {
  if (!image) return CG_E_ARG;
  try {
    auto img = Image::deserialize((const uint8_t*)image, len);
    if (row_like_mask) *row_like_mask = img->lslot_mask;
    if (like_read_mask) *like_read_mask = img->lread_mask;
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_image_policy_atomic(const void* image, size_t len, uint32_t i, int* atomic) {
  if (!image || !atomic) return CG_E_ARG;
  try {
    auto img = Image::deserialize((const uint8_t*)image, len);
    if (i >= img->n_pol()) return CG_E_RANGE;
    *atomic = (img->pol[(size_t)i * cgi::POL_WORDS + cgi::PW_FLAGS] & cgi::PF_ATOMIC) ? 1 : 0;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
  return CG_OK;
}

int cg_image_indexed(const void* image, size_t len, int* indexed) {
  if (!image || !indexed) return CG_E_ARG;
  try {
    *indexed = Image::deserialize((const uint8_t*)image, len)->indexed ? 1 : 0;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
  return CG_OK;
}

int cg_device_count(int* n) {
  if (!n) return CG_E_ARG;
  return dev_count(n) ? CG_E_DEVICE : CG_OK;
}

int cg_device_synchronize(int device) { return dev_synchronize(device) ? CG_E_DEVICE : CG_OK; }

int cg_ctx_create(int device, cg_ctx** out) {
  if (!out) return CG_E_ARG;
  *out = nullptr;
  int n = 0;
  if (dev_count(&n) || device < 0 || device >= n) return CG_E_DEVICE;
  auto* c = new (std::nothrow) cg_ctx();
  if (!c) return CG_E_ARG;
  c->device = device;
  if (dev_stream_create(device, &c->stream)) { delete c; return CG_E_DEVICE; }
  if (dev_stream_create(device, &c->rstream)) { dev_stream_destroy(c->stream); delete c; return CG_E_DEVICE; }
  if (dev_pool_create(device, &c->pool)) { dev_stream_destroy(c->rstream); dev_stream_destroy(c->stream); delete c; return CG_E_DEVICE; }
  *out = c;
  return CG_OK;
}

void cg_ctx_destroy(cg_ctx* ctx) {
  if (!ctx) return;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->active.reset();
    ctx->images.clear();
  }
  dev_pool_destroy(ctx->pool);
  dev_stream_destroy(ctx->rstream);
  dev_stream_destroy(ctx->stream);
  delete ctx;
}

const char* cg_last_error(cg_ctx* ctx) { return ctx ? ctx->err.c_str() : dev_last_error(); }

int cg_ctx_inject_fault(cg_ctx* ctx, int kind, uint64_t arg) {
  if (!ctx) return CG_E_ARG;
  switch (kind) {
    case CG_FAULT_NONE: ctx->fault_errors = 0; ctx->fault_stall_us = 0; ctx->fault_kidx = 0; return CG_OK;
    case CG_FAULT_DEVICE_ERROR: ctx->fault_errors = arg; return CG_OK;
    case CG_FAULT_STALL: ctx->fault_stall_us = std::min<uint64_t>(arg, 2000000u); return CG_OK;
    case CG_FAULT_BAD_KIDX: ctx->fault_kidx = arg; return CG_OK;
    default: return CG_E_ARG;
  }
}

int cg_pinned_stats(uint64_t* held_bytes, uint64_t* idle_blocks, uint64_t* kept_batches) {
  cg::pinned_stats(held_bytes, idle_blocks);
  if (kept_batches) *kept_batches = cg::g_pinned_kept.load(std::memory_order_relaxed);
  return CG_OK;
}

int cg_image_load(cg_ctx* ctx, const void* image, size_t len, uint64_t epoch) {
  if (!ctx || !image) return CG_E_ARG;
  std::shared_ptr<Image> img;
  try {
    img = Image::deserialize((const uint8_t*)image, len);
  } catch (const std::exception& e) {
    ctx->err = e.what();
    return CG_E_ARG;
  }
  img->epoch = epoch;
  auto li = std::make_shared<LoadedImage>();
  li->host = img;
  if (dev_image_upload(ctx->device, *img, (const uint8_t*)image, &li->dev)) { ctx->err = dev_last_error(); return CG_E_DEVICE; }
  std::lock_guard<std::mutex> g(ctx->mu);
  li->serial = ctx->next_serial++;
  ctx->images[epoch] = li;
  return CG_OK;
}

int cg_image_load_device(cg_ctx* ctx, void* dev_blob, size_t len, uint64_t epoch, const void* host_blob) {
  if (!ctx || !dev_blob) return CG_E_ARG;
  std::vector<uint8_t> copy;
  if (!host_blob) {  // the host side of the image (encoder tables, reasons' metadata) from the device blob
    try {
      copy.resize(len);
    } catch (const std::exception& e) {
      ctx->err = e.what();
      return CG_E_ARG;
    }
    if (dev_to_host(ctx->device, dev_blob, len, copy.data())) { ctx->err = dev_last_error(); return CG_E_DEVICE; }
    host_blob = copy.data();
  }
  std::shared_ptr<Image> img;
  try {
    img = Image::deserialize((const uint8_t*)host_blob, len);
  } catch (const std::exception& e) {
    ctx->err = e.what();
    return CG_E_ARG;
  }
  img->epoch = epoch;
  auto li = std::make_shared<LoadedImage>();
  li->host = img;
  if (dev_image_adopt(ctx->device, *img, dev_blob, &li->dev)) { ctx->err = dev_last_error(); return CG_E_DEVICE; }
  std::lock_guard<std::mutex> g(ctx->mu);
  li->serial = ctx->next_serial++;
  ctx->images[epoch] = li;
  return CG_OK;
}

int cg_image_delta(const void* base, size_t base_len, const void* next, size_t next_len, uint8_t** delta, size_t* delta_len) {
  if (!base || !next || !delta || !delta_len) return CG_E_ARG;
  try {
    std::vector<uint8_t> d = image_delta((const uint8_t*)base, base_len, (const uint8_t*)next, next_len);
    uint8_t* p = (uint8_t*)std::malloc(d.size());
    if (!p) return CG_E_ARG;
    std::memcpy(p, d.data(), d.size());
    *delta = p;
    *delta_len = d.size();
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_image_patch(const void* base, size_t base_len, const void* delta, size_t delta_len, uint8_t** out, size_t* out_len) {
  if (!base || !delta || !out || !out_len) return CG_E_ARG;
  try {
    std::vector<uint8_t> b = image_patch((const uint8_t*)base, base_len, (const uint8_t*)delta, delta_len);
    uint8_t* p = (uint8_t*)std::malloc(std::max<size_t>(b.size(), 1));
    if (!p) return CG_E_ARG;
    if (!b.empty()) std::memcpy(p, b.data(), b.size());
    *out = p;
    *out_len = b.size();
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_delta_info(const void* delta, size_t len, uint64_t* base_len, uint64_t* new_len, uint64_t* ops, uint64_t* literal_bytes) {
  if (!delta) return CG_E_ARG;
  try {
    const DeltaPlan p = delta_plan((const uint8_t*)delta, len);
    if (base_len) *base_len = p.base_len;
    if (new_len) *new_len = p.new_len;
    if (ops) *ops = p.n_ops;
    if (literal_bytes) *literal_bytes = p.lit_len;
    return CG_OK;
  } catch (const std::exception&) {
    return CG_E_ARG;
  }
}

int cg_image_load_delta(cg_ctx* ctx, uint64_t base_epoch, const void* delta, size_t len, uint64_t epoch) {
  if (!ctx || !delta) return CG_E_ARG;
  std::shared_ptr<LoadedImage> base;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    auto it = ctx->images.find(base_epoch);
    if (it == ctx->images.end()) { ctx->err = "no image loaded for the delta's base epoch"; return CG_E_STATE; }
    base = it->second;
  }
  DeltaPlan plan;
  try {
    plan = delta_plan((const uint8_t*)delta, len);
  } catch (const std::exception& e) {
    ctx->err = e.what();
    return CG_E_ARG;
  }
  if (!base->dev.blob_len || plan.base_len != base->dev.blob_len) {
    ctx->err = "delta image is for another base (length)";
    return CG_E_ARG;
  }
  // the new blob, built on the GPU from the base's device blob; the host tables from a copy of it
  void* nb = nullptr;
  if (dev_blob_patch(ctx->device, base->dev, plan.pieces.data(), plan.pieces.size() / 3, plan.lit, plan.lit_len,
                     plan.fix, plan.n_fix, (size_t)plan.new_len, &nb)) {
    ctx->err = dev_last_error();
    return CG_E_DEVICE;
  }
  std::shared_ptr<Image> img;
  try {
    // the new blob's checksum on the device; then the host reads back only what deserialize reads:
    // the header and section table, the sections the host keeps, and the host part (not the policy
    // stream or the scope index: ~70 % of a large image)
    uint64_t sum = 0;
    if (dev_blob_sum(ctx->device, nb, (size_t)plan.new_len, &sum)) throw std::runtime_error(dev_last_error());
    if (sum != plan.new_sum) throw CedarError("delta image does not reproduce the new image (checksum)");
    std::unique_ptr<uint8_t[]> host(new uint8_t[std::max<uint64_t>(plan.new_len, 1)]);
    const size_t n = (size_t)plan.new_len, table = 16 + 16 * ((size_t)cgi::DS_COUNT + 1);
    auto d2h = [&](size_t lo, size_t hi) {
      if (hi > lo && dev_to_host(ctx->device, (const uint8_t*)nb + lo, hi - lo, host.get() + lo)) throw std::runtime_error(dev_last_error());
    };
    if (n < table) throw CedarError("truncated image");
    d2h(0, table);
    uint64_t off[cgi::DS_COUNT + 1];
    for (uint32_t k = 0; k < cgi::DS_COUNT; k++) std::memcpy(&off[k], host.get() + 16 + 16 * k, 8);
    std::memcpy(&off[cgi::DS_COUNT], host.get() + 16 + 16 * cgi::DS_COUNT + 8, 8);  // the device region's end
    bool ok = true;
    for (uint32_t k = 0; k < cgi::DS_COUNT; k++) ok = ok && off[k] <= off[k + 1] && off[k + 1] <= n;
    if (!ok || off[0] < table) throw CedarError("corrupt image (device region)");
    static_assert(cgi::DS_PSTREAM == 0 && cgi::DS_BTAB + 1 == cgi::DS_BFILT && cgi::DS_BFILT + 1 == cgi::DS_BSTREAM, "section order");
    d2h(table, (size_t)off[cgi::DS_PSTREAM]);
    d2h((size_t)off[cgi::DS_PSTREAM + 1], (size_t)off[cgi::DS_BTAB]);
    d2h((size_t)off[cgi::DS_BSTREAM + 1], n);
    img = Image::deserialize(host.get(), n);
  } catch (const std::exception& e) {
    dev_free(ctx->device, nb);
    ctx->err = e.what();
    return CG_E_ARG;
  }
  img->epoch = epoch;
  auto li = std::make_shared<LoadedImage>();
  li->host = img;
  if (dev_image_adopt(ctx->device, *img, nb, &li->dev)) {
    dev_free(ctx->device, nb);
    ctx->err = dev_last_error();
    return CG_E_DEVICE;
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  li->serial = ctx->next_serial++;
  ctx->images[epoch] = li;
  return CG_OK;
}

int cg_image_load_peer(cg_ctx* dst, cg_ctx* src, uint64_t epoch) {
  if (!dst || !src) return CG_E_ARG;
  std::shared_ptr<LoadedImage> from;
  {
    std::lock_guard<std::mutex> g(src->mu);
    auto it = src->images.find(epoch);
    if (it == src->images.end()) { dst->err = "no image loaded for epoch on the source context"; return CG_E_STATE; }
    from = it->second;
  }
  auto li = std::make_shared<LoadedImage>();
  li->host = from->host;  // one host image (encoder tables, metadata) shared by both contexts
  if (dev_image_copy(dst->device, *from->host, from->dev, &li->dev)) { dst->err = dev_last_error(); return CG_E_DEVICE; }
  std::lock_guard<std::mutex> g(dst->mu);
  li->serial = dst->next_serial++;
  dst->images[epoch] = li;
  return CG_OK;
}

int cg_image_activate(cg_ctx* ctx, uint64_t epoch) {
  if (!ctx) return CG_E_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  auto it = ctx->images.find(epoch);
  if (it == ctx->images.end()) { ctx->err = "no image loaded for epoch"; return CG_E_STATE; }
  if (ctx->active != it->second) ctx->activations++;
  ctx->active = it->second;
  return CG_OK;
}

int cg_image_active(cg_ctx* ctx, uint64_t* epoch) {
  if (!ctx || !epoch) return CG_E_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->active) return CG_E_STATE;
  *epoch = ctx->active->host->epoch;
  return CG_OK;
}

int cg_image_unload(cg_ctx* ctx, uint64_t epoch) {
  if (!ctx) return CG_E_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->images.erase(epoch);  // shared_ptr: batches / active keep it alive
  return CG_OK;
}

// ---------------------------------------------------------------------------------------------
int cg_batch_create(cg_ctx* ctx, cg_batch** out) {
  if (!ctx || !out) return CG_E_ARG;
  std::shared_ptr<LoadedImage> img;
  {
    std::lock_guard<std::mutex> g(ctx->mu);
    img = ctx->active;
  }
  if (!img) { ctx->err = "no active image"; return CG_E_STATE; }
  auto* b = new (std::nothrow) cg_batch();
  if (!b) return CG_E_ARG;
  b->ctx = ctx;
  b->img = img;
  b->host.img = img->host;
  *out = b;
  return CG_OK;
}

void cg_batch_destroy(cg_batch* b) { delete b; }

int cg_batch_add_json(cg_batch* b, const char* json, size_t len) {
  if (!b || !json) return CG_E_ARG;
  if (b->submitted) { b->err = "batch already submitted"; return CG_E_STATE; }
  GUARD(b->err, {
    JVal v = json_parse(json, len);
    std::vector<EntityIn> ents;
    RequestIn req;
    auto one = [&](const JVal& item) {
      decode_json_item(item, ents, req);
      b->items.push_back({(int32_t)b->host.n(), -1});
      b->host.add(ents, req);
    };
    if (v.t == JVal::Arr) for (auto& item : v.arr) one(item);
    else one(v);
    return CG_OK;
  })
}

int cg_batch_add_sar_json(cg_batch* b, const char* json, size_t len) {
  if (!b || !json) return CG_E_ARG;
  if (b->submitted) { b->err = "batch already submitted"; return CG_E_STATE; }
  std::vector<std::pair<size_t, size_t>> elems;
  LatTrace tr("split");
  if (len >= 65536 && split_array(json, len, elems)) {
    tr.mark("split");
    // bulk: parse, convert and encode elements on worker threads into per-chunk parts (bulk_add;
    // one worker too: the direct path per element, no JSON tree of the whole array)
    const Image& img = *b->host.img;
    return bulk_add(b, elems.size(), [&](size_t k, EncodedRequest& e, BulkOut& o) {
      const char* p = json + elems[k].first;
      const size_t m = elems[k].second;
      const int d = encode_sar_direct(img, p, m, e, o.fast, o.reason);
      if (d == 2) { o.host = true; return; }
      if (d == 1) return;
      JVal v = json_parse(p, m);
      Attributes a = attributes_from_sar(v);
      o.reason.clear();
      o.fast = authorize_fast_path(a, o.reason);
      if (o.fast >= 0) { o.host = true; return; }
      std::vector<EntityIn> ents;
      RequestIn req;
      record_to_cedar(a, ents, req);
      encode_request(img, ents, req, e);
    });
  }
  GUARD(b->err, {
    JVal v = json_parse(json, len);
    std::vector<EntityIn> ents;
    RequestIn req;
    auto one = [&](const JVal& sar) {
      Attributes a = attributes_from_sar(sar);  // (array of < 65536 bytes, or one worker)
      std::string reason;
      int fast = authorize_fast_path(a, reason);
      if (fast >= 0) {
        b->fast_reason[(uint32_t)b->items.size()] = reason;
        b->items.push_back({-1, fast});
        return;
      }
      record_to_cedar(a, ents, req);
      b->items.push_back({(int32_t)b->host.n(), -1});
      b->host.add(ents, req);
    };
    if (v.t == JVal::Arr) for (auto& s : v.arr) one(s);
    else one(v);
    return CG_OK;
  })
}

int cg_sar_to_cedar_json(const char* sar_json, size_t len, char* out, size_t cap, size_t* need) {
  if (!sar_json) return CG_E_ARG;
  std::string s, err;
  GUARD(err, {
    JVal v = json_parse(sar_json, len);
    Attributes a = attributes_from_sar(v);
    std::string reason;
    int fast = authorize_fast_path(a, reason);
    if (fast >= 0) {
      s = "{\"fast\":" + std::to_string(fast) + ",\"reason\":";
      go_json_string(s, reason);
      s += "}";
    } else {
      std::vector<EntityIn> ents;
      RequestIn req;
      record_to_cedar(a, ents, req);
      cedar_item_json(ents, req, s);
    }
  })
  if (need) *need = s.size() + 1;
  if (!out || cap < s.size() + 1) return CG_E_RANGE;
  std::memcpy(out, s.c_str(), s.size() + 1);
  return CG_OK;
}

int cg_batch_authz(cg_batch* b, uint32_t i, int* decision, char* reason, size_t cap, size_t* need) {
  if (!b || !decision) return CG_E_ARG;
  if (i >= b->items.size()) return CG_E_RANGE;
  std::string r;
  const auto& it = b->items[i];
  if (it.dev < 0) {
    *decision = it.fast;
    r = b->fast_reason[i];
  } else {
    if (!b->done) return CG_E_STATE;
    // authorizer.go:73-84 + diagnosticToReason (authorizer.go:113-124)
    std::vector<uint32_t> rs;
    GUARD_RESULT(b->err, { b->host.reason_ids((uint32_t)it.dev, rs); })
    if (b->host.decision((uint32_t)it.dev)) {
      *decision = AUTHZ_ALLOW;
    } else if (!rs.empty()) {
      *decision = AUTHZ_DENY;
    } else {
      *decision = AUTHZ_NO_OPINION;
    }
    if (*decision != AUTHZ_NO_OPINION && !rs.empty()) {
      GUARD_RESULT(b->err, { b->host.diagnostic_json((uint32_t)it.dev, r, false); })
    }
  }
  if (need) *need = r.size() + 1;
  if (!reason) return CG_OK;
  if (cap < r.size() + 1) return CG_E_RANGE;
  std::memcpy(reason, r.c_str(), r.size() + 1);
  return CG_OK;
}

int cg_encode_sar_check(const void* image, size_t len, const char* sars, size_t n, uint32_t* n_items,
                        uint32_t* n_direct, uint32_t* n_mismatch, int64_t* first_mismatch) {
  if (!image || !sars) return CG_E_ARG;
  std::string err;
  GUARD(err, { return encode_sar_check(image, len, sars, n, n_items, n_direct, n_mismatch, first_mismatch); })
}

int cg_json_split_check(const char* json, size_t n, uint32_t threads, int64_t* n_elems, int* same) {
  if (!json || !n_elems || !same) return CG_E_ARG;
  std::vector<std::pair<size_t, size_t>> a, b;
  const bool ra = split_array_serial(json, n, a);
  bool rb;
  {
    // the parallel split on `threads` regions whatever the size (CEDARGPU_HOST_THREADS and the
    // 8 MiB floor are bypassed for the check)
    rb = split_array_regions(json, n, b, std::max(2u, threads));
  }
  *n_elems = ra ? (int64_t)a.size() : -1;
  *same = (ra == rb) && (!ra || a == b);
  return CG_OK;
}

int cg_encode_items_check(const void* image, size_t len, const char* items, size_t n, uint32_t* n_items,
                          uint32_t* n_mismatch, int64_t* first_mismatch) {
  if (!image || !items) return CG_E_ARG;
  std::string err;
  GUARD(err, {
    auto img = Image::deserialize((const uint8_t*)image, len);
    JVal v = json_parse(items, n);
    if (v.t != JVal::Arr) throw CedarError("expected a JSON array");
    uint32_t nm = 0;
    int64_t first = -1;
    std::vector<EntityIn> ents;
    RequestIn req;
    for (size_t k = 0; k < v.arr.size(); k++) {
      decode_json_item(v.arr[k], ents, req);
      EncodedRequest a;
      EncodedRequest w;
      encode_request(*img, ents, req, a);  // ancestor records from the closure cache where it applies
      enc::t_no_closure_cache = true;
      try {
        encode_request(*img, ents, req, w);  // the general walk
      } catch (...) {
        enc::t_no_closure_cache = false;
        throw;
      }
      enc::t_no_closure_cache = false;
      if (a.blk != w.blk || a.row != w.row || a.anc != w.anc || a.anc_at != w.anc_at || a.strs != w.strs || a.gkey != w.gkey) {
        nm++;
        if (first < 0) first = (int64_t)k;
      }
    }
    if (n_items) *n_items = (uint32_t)v.arr.size();
    if (n_mismatch) *n_mismatch = nm;
    if (first_mismatch) *first_mismatch = first;
    return CG_OK;
  })
}

int cg_batch_add_admission_json(cg_batch* b, const char* json, size_t len) {
  if (!b || !json) return CG_E_ARG;
  if (b->submitted) { b->err = "batch already submitted"; return CG_E_STATE; }
  std::vector<std::pair<size_t, size_t>> elems;
  if (len >= 65536 && split_array(json, len, elems) && host_workers(elems.size()) > 1) {
    // bulk: parse, flatten and encode reviews on worker threads into per-chunk parts (bulk_add)
    const Image& img = *b->host.img;
    return bulk_add(b, elems.size(), [&](size_t k, EncodedRequest& e, BulkOut& o) {
      JVal v = json_parse(json + elems[k].first, elems[k].second);
      const AdmissionRequest a = admission_request_from_json(v);
      std::vector<EntityIn> ents;
      RequestIn req;
      std::string err;
      const int outcome = admission_to_cedar(a, ents, req, err);
      if (outcome != ADM_EVAL) {
        o.host = true;
        o.fast = outcome;
        if (outcome == ADM_ERROR) o.reason = std::move(err);
        return;
      }
      encode_request(img, ents, req, e);
    });
  }
  GUARD(b->err, {
    JVal v = json_parse(json, len);
    std::vector<EntityIn> ents;
    RequestIn req;
    auto one = [&](const JVal& review) {
      const AdmissionRequest a = admission_request_from_json(review);
      std::string err;
      const int o = admission_to_cedar(a, ents, req, err);
      const uint32_t i = (uint32_t)b->items.size();
      if (o == ADM_EVAL) {
        b->items.push_back({(int32_t)b->host.n(), -1});
        b->host.add(ents, req);
      } else {
        b->items.push_back({-1, o});
        if (o == ADM_ERROR) b->fast_reason[i] = err;
      }
    };
    if (v.t == JVal::Arr) for (auto& r : v.arr) one(r);
    else one(v);
    return CG_OK;
  })
}

int cg_batch_admit(cg_batch* b, uint32_t i, int* allowed, int* code, char* msg, size_t cap, size_t* need) {
  if (!b || !allowed) return CG_E_ARG;
  if (i >= b->items.size()) return CG_E_RANGE;
  std::string m;
  int c = 200;
  const auto& it = b->items[i];
  if (it.dev < 0) {
    if (it.fast == ADM_SKIP) {
      *allowed = 1;
    } else {  // admission.Errored(http.StatusInternalServerError, err)
      *allowed = 0;
      c = 500;
      m = b->fast_reason[i];
    }
  } else {
    if (!b->done) return CG_E_STATE;
    const uint32_t d = (uint32_t)it.dev;
    *allowed = b->host.decision(d) ? 1 : 0;
    std::vector<uint32_t> rs;
    GUARD_RESULT(b->err, { b->host.reason_ids(d, rs); })
    if (!*allowed && !rs.empty()) {  // json.Marshal(diagnostics.Reasons) (handler.go:62-66)
      GUARD_RESULT(b->err, { b->host.diagnostic_json(d, m, true); })
    }
  }
  if (code) *code = c;
  if (need) *need = m.size() + 1;
  if (!msg) return CG_OK;
  if (cap < m.size() + 1) return CG_E_RANGE;
  std::memcpy(msg, m.c_str(), m.size() + 1);
  return CG_OK;
}

int cg_admission_to_cedar_json(const char* review_json, size_t len, char* out, size_t cap, size_t* need) {
  if (!review_json) return CG_E_ARG;
  std::string s, err;
  GUARD(err, {
    JVal v = json_parse(review_json, len);
    const AdmissionRequest a = admission_request_from_json(v);
    std::vector<EntityIn> ents;
    RequestIn req;
    std::string e;
    const int o = admission_to_cedar(a, ents, req, e);
    if (o == ADM_SKIP) {
      s = "{\"skip\":true}";
    } else if (o == ADM_ERROR) {
      s = "{\"error\":";
      go_json_string(s, e);
      s += "}";
    } else {
      cedar_item_json(ents, req, s);
    }
  })
  if (need) *need = s.size() + 1;
  if (!out || cap < s.size() + 1) return CG_E_RANGE;
  std::memcpy(out, s.c_str(), s.size() + 1);
  return CG_OK;
}

uint32_t cg_batch_size(cg_batch* b) { return b ? (uint32_t)b->items.size() : 0; }

int cg_batch_submit(cg_batch* b) {
  if (!b) return CG_E_ARG;
  if (b->submitted) { b->err = "batch already submitted"; return CG_E_STATE; }
  LatTrace tr("submit");
  const int64_t p0 = b->host.prof ? dev_now_ns() : 0;
  auto pmark = [&](int k, int64_t& t) {
    if (!b->host.prof) return;
    const int64_t now = dev_now_ns();
    b->prof_ms[k] = (double)(now - t) * 1e-6;
    t = now;
  };
  int64_t pt = p0;
  b->host.finalize_strings();
  tr.mark("finalize");
  pmark(0, pt);
  if (b->host.n() == 0) { b->submitted = b->done = true; return CG_OK; }
  // First-pass reason capacity: up to the probe kernel's 64-hit stage while the two reason arrays
  // stay within 4 MB (small, latency-bound batches then need no re-run for 9..64 reasons); large
  // throughput batches keep 8 per effect.
  // CEDARGPU_FIRST_CAPR pins it (tests drive the 9..64-reason re-run path with small batches).
  const uint32_t n = b->host.n();
  b->host.capr = std::max<uint32_t>(8u, std::min<uint32_t>(64u, (uint32_t)((4u << 20) / (8ull * n))));
  // Sizing from the last batch on this image (CapHint): each follow-up worklist gets the share
  // that batch needed (+1/4 and 64 spare), so images whose requests mostly collect many reasons
  // (C4) finish on the device; FU_BIG's per-entry reason capacity follows the longest list it
  // produced (+1/8, rounded up to 32; 64..256); the first pass holds the longest list it counted
  // (up to 64) while its two reason arrays stay within 32 MB.
  CapHint h;
  {
    std::lock_guard<std::mutex> g(b->ctx->mu);
    h = b->ctx->hint;
  }
  for (uint32_t k = 0; k < FU_KINDS; k++) b->host.fu_want[k] = 0;
  b->host.fu_capr_hint = b->host.fu_capr_gen_hint = 0;
  if (h.serial && h.serial == b->img->serial) {
    for (uint32_t k = 0; k < FU_KINDS; k++)
      if (h.ppm[k]) b->host.fu_want[k] = (uint32_t)std::min<uint64_t>(n, (uint64_t)h.ppm[k] * n / 1000000u * 5 / 4 + 64);
    if (h.big_maxr) b->host.fu_capr_hint = (h.big_maxr + h.big_maxr / 8 + 8 + 31) & ~31u;
    if (h.gen_maxr) b->host.fu_capr_gen_hint = (h.gen_maxr + h.gen_maxr / 8 + 8 + 31) & ~31u;
    // the longest list the last first pass counted (<= 64), as far as the two reason arrays stay
    // within the budget (CEDARGPU_FIRST_BUDGET_MB, default 32)
    static const uint64_t budget = [] { const char* e = std::getenv("CEDARGPU_FIRST_BUDGET_MB"); return (uint64_t)(e ? std::max(1, std::atoi(e)) : 32) << 20; }();
    const uint32_t want_capr = std::min<uint32_t>(64u, (h.first_maxr + 7) & ~7u);
    const uint32_t fit = (uint32_t)std::min<uint64_t>(64u, budget / (8ull * std::max<uint32_t>(1u, n))) & ~7u;
    if (std::min(want_capr, fit) > b->host.capr) b->host.capr = std::min(want_capr, fit);
  }
  // A small batch runs as one launch whose waves hold up to 1,024 hits each (device.h
  // DevBatch::small) and has no on-device follow-up: its reason lists get room for most of those
  // (within 2 MB per batch), so that a many-hit request seldom needs a host re-run.
  // (Within 512 KB of reasons and 64 KB of errors per batch: the D2H copy carries them all; a
  // longer list takes one of the batch's overflow slots, which travel back only when taken.)
  if (b->img->host->indexed && n <= dev_small_n()) {
    b->host.capr = std::max(b->host.capr, std::min<uint32_t>(1024u, std::max<uint32_t>(32u, (uint32_t)((512u << 10) / (4ull * n)))) & ~7u);
    b->host.cape = std::max(b->host.cape, std::min<uint32_t>(32u, std::max<uint32_t>(2u, (uint32_t)((64u << 10) / (24ull * n)))));
  }
  // First-pass error details per request: indexed batches past the one-launch size keep one in their
  // result block (a request with more takes a long-list slot, with up to 8), so the results copy
  // carries 24 instead of 96 bytes of mostly empty error slots per request. CEDARGPU_FIRST_CAPE pins it.
  if (b->img->host->indexed && n > dev_small_n()) b->host.cape = 1;
  if (const char* e = std::getenv("CEDARGPU_FIRST_CAPE")) b->host.cape = (uint32_t)std::max(1, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("CEDARGPU_FIRST_CAPR")) b->host.capr = (uint32_t)std::max(1, std::min(4096, std::atoi(e)));
  GUARD(b->err, { group_requests(b); })
  tr.mark("group");
  pmark(1, pt);
  for (uint64_t f = b->ctx->fault_errors.load(); f;)
    if (b->ctx->fault_errors.compare_exchange_weak(f, f - 1)) {
      b->err = "injected device error (cg_ctx_inject_fault CG_FAULT_DEVICE_ERROR)";
      return CG_E_DEVICE;
    }
  for (uint64_t f = b->ctx->fault_kidx.load(); f;)
    if (b->ctx->fault_kidx.compare_exchange_weak(f, f - 1)) {
      corrupt_key_indices(b->host);
      break;
    }
  if (dev_batch_upload(b->ctx->device, b->host, &b->dev, b->ctx->stream, b->ctx->pool)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  tr.mark("upload");
  pmark(2, pt);
  if (const uint64_t us = b->ctx->fault_stall_us.load())
    if (dev_stall(b->ctx->device, b->ctx->stream, us)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  if (dev_eval(b->img->dev, b->dev, b->ctx->stream)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  tr.mark("launch");
  if (dev_download_async(b->dev, b->ctx->stream)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  tr.mark("d2h_enqueue");
  pmark(3, pt);
  b->submitted = true;
  return CG_OK;
}

int cg_batch_wait(cg_batch* b, int64_t timeout_ns) {
  if (!b) return CG_E_ARG;
  const int64_t t0 = dev_now_ns();
  const int64_t deadline = timeout_ns < 0 ? -1 : t0 + timeout_ns;
  const int rc = cg::batch_wait(b, deadline, deadline);
  if (b->host.prof && rc == CG_OK) b->prof_ms[4] += (double)(dev_now_ns() - t0) * 1e-6;
  return rc;
}

int cg_batch_set_profile(cg_batch* b, int on) {
  if (!b) return CG_E_ARG;
  if (b->submitted) { b->err = "profile must be set before submit"; return CG_E_STATE; }
  b->host.prof = on != 0;
  return CG_OK;
}

int cg_batch_profile(cg_batch* b, double* ms, size_t n) {
  if (!b || !ms) return CG_E_ARG;
  if (!b->host.prof || !b->downloaded) { b->err = "batch not profiled, or not waited"; return CG_E_STATE; }
  float dev[3] = {0.f, 0.f, 0.f};
  if (!dev_batch_profile(b->dev, &dev[0], &dev[1], &dev[2])) { b->err = "no device profile (small batch or stand-in)"; }
  const double v[8] = {b->prof_ms[0], b->prof_ms[1], b->prof_ms[2], b->prof_ms[3], dev[0], dev[1], dev[2], b->prof_ms[4]};
  for (size_t k = 0; k < n && k < 8; k++) ms[k] = v[k];
  return CG_OK;
}

}  // extern "C"

int cg::batch_wait(cg_batch* b, int64_t download_deadline, int64_t deadline) {
  if (!b->submitted) { b->err = "batch not submitted"; return CG_E_STATE; }
  if (b->done) return CG_OK;
  if (b->failed) return b->failed;
  LatTrace tr("wait");
  if (!b->downloaded) {
    if (const int drc = dev_download_finish(b->dev, b->host, download_deadline)) {
      b->err = dev_last_error();
      return drc == DEV_TIMEOUT ? CG_E_TIMEOUT : CG_E_DEVICE;  // a timeout leaves the batch in flight
    }
    b->downloaded = true;
    if (b->host.fu_cnt && b->host.fu_cnt[FU_KINDS]) {
      // the scan found key-entity indices that are not the image's: the batch was encoded for
      // another image (or corrupted), so none of its answers can be trusted; callers fail safe
      b->err = std::to_string(b->host.fu_cnt[FU_KINDS]) +
               " request(s) carry key-entity indices outside the image's: batch not encoded for this image";
      b->failed = CG_E_DEVICE;
      return CG_E_DEVICE;
    }
  }
  tr.mark("sync_copy");
  // Overflowed result lists: re-run just those requests. Capacity overflows of the probe kernel
  // re-run there with the exact capacities; requests it could not decide (RF_GENERAL) and any
  // stream-kernel overflow re-run on the stream kernel, which reports exact counts, so a second
  // pass with those capacities completes it.
  // Requests the on-device follow-up finished (worklists right behind the first pass, same
  // results block): their lists are final, unless the follow-up itself overflowed (those keep the
  // first pass's RF_OVERFLOW and go to the host re-run below). Their counts size the next batch.
  CapHint h;
  h.serial = b->img->serial;
  const uint32_t n = b->host.n();
  for (uint32_t i = 0; i < n; i++) {  // the first pass's exact list lengths (<= 64 hits)
    const uint32_t fl = b->host.res[2 * (size_t)i] >> 16;
    if ((fl & cgi::RF_VALID) && !(fl & (cgi::RF_GENERAL | cgi::RF_BIG)))
      h.first_maxr = std::max(h.first_maxr, b->host.res[2 * (size_t)i + 1] & 0xFFFF);
  }
  tr.mark("maxr");
  if (b->host.fu_cnt) {
    for (uint32_t q = 0; q < FU_KINDS; q++) {
      const auto& fu = b->host.fu[q];
      h.ppm[q] = (uint32_t)std::min<uint64_t>(1000000u, (uint64_t)b->host.fu_cnt[q] * 1000000u / std::max<uint32_t>(1u, n));
      const uint32_t cnt = std::min(b->host.fu_cnt[q], fu.cap);
      for (uint32_t k = 0; k < cnt; k++) {
        const uint32_t i = fu.ids[k] & ~0x80000000u;  // (FU_DONE: an entry the first pass finished)
        if (i >= n) { b->err = "follow-up worklist out of range"; return CG_E_DEVICE; }
        b->routes.push_back((uint64_t)i << 8 | ((fu.ids[k] & 0x80000000u) ? CG_ROUTE_FIRST_SLOT : (CG_ROUTE_FU_BIG << q)));
        const uint32_t fl = fu.res[2 * k] >> 16;
        if (!(fl & cgi::RF_VALID) || (fl & (cgi::RF_GENERAL | cgi::RF_BIG))) continue;
        const uint32_t nr = fu.res[2 * k + 1] & 0xFFFF, ne = fu.res[2 * k + 1] >> 16;
        if (q == FU_BIG) h.big_maxr = std::max(h.big_maxr, nr);  // exact, overflowed or not
        if (q == FU_GEN) h.gen_maxr = std::max(h.gen_maxr, nr);
        if (fl & cgi::RF_OVERFLOW) continue;
        b->host.res[2 * (size_t)i] = fu.res[2 * k];
        b->host.res[2 * (size_t)i + 1] = fu.res[2 * k + 1];
        b->n_fu[q]++;
        GUARD(b->err, {
          b->host.set_big(i, ((fl & cgi::RF_FORBID) ? fu.rf : fu.rp) + (size_t)k * fu.capr, nr,
                          fu.er + (size_t)k * fu.cape * cgi::ERR_WORDS, ne * cgi::ERR_WORDS);
        })
      }
      if (cnt) tr.val(q == FU_BIG ? "nbig" : "nfu", cnt);
    }
  }
  tr.mark("fu");
  {
    std::lock_guard<std::mutex> g(b->ctx->mu);
    // a batch without FU_BIG / FU_GEN entries keeps the image's last known list lengths
    if (!h.big_maxr && b->ctx->hint.serial == h.serial) h.big_maxr = b->ctx->hint.big_maxr;
    if (!h.gen_maxr && b->ctx->hint.serial == h.serial) h.gen_maxr = b->ctx->hint.gen_maxr;
    b->ctx->hint = h;
  }
  tr.mark("fold");
  std::vector<uint32_t> idx_probe, idx_big, idx_gen;
  uint32_t capr_p = 0, cape_p = 0, capr_b = 0, cape_b = 0, capr_g = 0, cape_g = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t fl = b->host.res[2 * (size_t)i] >> 16;
    if (!(fl & cgi::RF_VALID)) { b->err = "request left unevaluated"; return CG_E_DEVICE; }
    if (!(fl & cgi::RF_OVERFLOW)) continue;
    const uint32_t nr = b->host.res[2 * (size_t)i + 1] & 0xFFFF, ne = b->host.res[2 * (size_t)i + 1] >> 16;
    if ((fl & cgi::RF_GENERAL) || !b->img->dev.indexed) {
      idx_gen.push_back(i); capr_g = std::max(capr_g, nr); cape_g = std::max(cape_g, ne);
    } else if (fl & cgi::RF_BIG) {
      idx_big.push_back(i); capr_b = std::max(capr_b, nr); cape_b = std::max(cape_b, ne);
    } else {
      idx_probe.push_back(i); capr_p = std::max(capr_p, nr); cape_p = std::max(cape_p, ne);
    }
  }
  // Folds one re-run's results (subset order, read in place from the job's pinned block) into the
  // batch. Requests a probe re-run cannot decide move on to `next`; those whose lists overflowed
  // again go to `again` with their exact counts.
  auto apply = [&](const std::vector<uint32_t>& idx, uint32_t capr, uint32_t cape, int mode, const SubsetView& v,
                   std::vector<uint32_t>& again, uint32_t& capr2, uint32_t& cape2, std::vector<uint32_t>& next) {
    for (size_t k = 0; k < idx.size(); k++) {
      uint32_t i = idx[k];
      uint32_t fl = v.res[2 * k] >> 16;
      uint32_t nr = v.res[2 * k + 1] & 0xFFFF, ne = v.res[2 * k + 1] >> 16;
      if (mode && (fl & (cgi::RF_GENERAL | cgi::RF_BIG))) { next.push_back(i); continue; }
      if (fl & cgi::RF_OVERFLOW) {
        again.push_back(i);
        capr2 = std::max(capr2, nr);
        cape2 = std::max(cape2, ne);
        continue;
      }
      const uint32_t* src = (fl & cgi::RF_FORBID) ? v.rf : v.rp;
      b->host.res[2 * (size_t)i] = v.res[2 * k];
      b->host.res[2 * (size_t)i + 1] = v.res[2 * k + 1];
      b->host.set_big(i, src + k * capr, nr, v.er + k * cape * cgi::ERR_WORDS, ne * cgi::ERR_WORDS);
    }
  };
  auto clampr = [](uint32_t c, uint32_t lo) { return std::max(std::min(c, 4096u), lo); };
  // a re-run that missed the deadline is still in flight: its blocks stay with the batch, whose
  // destruction drains the stream first; the batch is failed
  auto timed_out = [&](std::initializer_list<DevSubset*> jobs) {
    b->err = "deadline exceeded during a host re-run";
    for (DevSubset* j : jobs)
      if (j->dblk) b->held.push_back(*j);
    b->dev.pending = true;
    b->failed = CG_E_TIMEOUT;
    return CG_E_TIMEOUT;
  };
  // re-runs a subset (mode: 1 probe kernel, 2 its large-stage variant, 0 stream kernel) until its
  // lists fit, one round trip per pass
  auto rerun = [&](std::vector<uint32_t>& idx, uint32_t capr, uint32_t cape, int mode, std::vector<uint32_t>& next) -> int {
    for (int pass = 0; pass < 3 && !idx.empty(); pass++) {
      capr = clampr(capr, 8u);
      cape = clampr(cape, 4u);
      DevSubset job;
      SubsetView v;
      int src = dev_subset_begin(b->img->dev, b->dev, idx.data(), (uint32_t)idx.size(), capr, cape, mode, b->ctx->rstream, &job);
      if (!src) src = dev_subset_end(&job, &v, deadline);
      if (src == DEV_TIMEOUT) return timed_out({&job});
      if (src) {
        b->err = dev_last_error();
        (void)dev_stream_sync(b->ctx->rstream);
        dev_subset_release(&job);
        return CG_E_DEVICE;
      }
      std::vector<uint32_t> again;
      uint32_t capr2 = 0, cape2 = 0;
      try {
        apply(idx, capr, cape, mode, v, again, capr2, cape2, next);
      } catch (const std::exception& ex) {
        b->err = ex.what();
        dev_subset_release(&job);
        return CG_E_RANGE;
      }
      b->held.push_back(job);  // the batch's lists point into its pinned block
      idx.swap(again);
      capr = capr2;
      cape = cape2;
    }
    if (!idx.empty()) { b->err = "result lists exceed the device re-run capacity"; return CG_E_RANGE; }
    return CG_OK;
  };
  b->n_rerun = (uint32_t)(idx_probe.size() + idx_big.size() + idx_gen.size());
  for (const auto* v : {&idx_probe, &idx_big, &idx_gen})
    for (const uint32_t i : *v) b->routes.push_back((uint64_t)i << 8 | CG_ROUTE_RERUN);
  int rc;
  tr.mark("scan");
  // First round: the three subsets are known from the first pass's flags, so their re-runs are
  // enqueued back to back and share one wait. Leftovers (rare: a probe re-run that found it needs
  // the large stage or the stream kernel, or lists that overflowed again) finish sequentially.
  {
    struct Sub { std::vector<uint32_t>* idx; uint32_t capr, cape; int mode; DevSubset job; SubsetView v; };
    Sub subs[3] = {{&idx_probe, clampr(capr_p, 8u), clampr(cape_p, 4u), 1, {}, {}},
                   {&idx_big, clampr(capr_b, 64u), clampr(cape_b, 16u), 2, {}, {}},
                   {&idx_gen, clampr(capr_g, 64u), clampr(cape_g, 16u), 0, {}, {}}};
    int brc = 0;
    for (auto& u : subs)
      if (!brc && !u.idx->empty())
        brc = dev_subset_begin(b->img->dev, b->dev, u.idx->data(), (uint32_t)u.idx->size(), u.capr, u.cape, u.mode, b->ctx->rstream, &u.job);
    for (auto& u : subs)
      if (!brc) brc = dev_subset_end(&u.job, &u.v, deadline);
    if (brc == DEV_TIMEOUT) return timed_out({&subs[0].job, &subs[1].job, &subs[2].job});
    std::vector<uint32_t> again[3], next_big, next_gen;
    uint32_t capr2[3] = {0, 0, 0}, cape2[3] = {0, 0, 0};
    std::vector<uint32_t>* nexts[3] = {&next_big, &next_gen, &next_gen};
    int arc = CG_OK;
    if (brc) {
      b->err = dev_last_error();
      (void)dev_stream_sync(b->ctx->rstream);  // nothing in flight before the blocks go back
      arc = CG_E_DEVICE;
    } else {
      try {
        for (int k = 0; k < 3; k++)
          if (!subs[k].idx->empty())
            apply(*subs[k].idx, subs[k].capr, subs[k].cape, subs[k].mode, subs[k].v, again[k], capr2[k], cape2[k], *nexts[k]);
      } catch (const std::exception& ex) {
        b->err = ex.what();
        arc = CG_E_RANGE;
      }
    }
    for (auto& u : subs) {
      if (arc) dev_subset_release(&u.job);
      else if (u.job.dblk) b->held.push_back(u.job);  // the batch's lists point into its pinned block
    }
    if (arc) return arc;
    tr.mark("rerun_batched");
    if (!again[0].empty() && (rc = rerun(again[0], capr2[0], cape2[0], 1, next_big))) return rc;
    if (!next_big.empty()) {
      // exact counts unknown for these: the large stage reports them, a second pass completes it
      if ((rc = rerun(next_big, 64u, 16u, 2, next_gen))) return rc;
    }
    if (!again[1].empty() && (rc = rerun(again[1], capr2[1], cape2[1], 2, next_gen))) return rc;
    if (!again[2].empty()) {
      std::vector<uint32_t> none;
      if ((rc = rerun(again[2], capr2[2], cape2[2], 0, none))) return rc;
    }
    if (!next_gen.empty()) {
      std::vector<uint32_t> none;
      if ((rc = rerun(next_gen, 64u, 16u, 0, none))) return rc;
    }
  }
  tr.mark("rerun_big_general");
  if (!idx_big.empty()) {
    // their exact list lengths join the image's sizing hint: the worklist the large stage ran on
    // the device may have held only some of this batch's many-hit requests
    uint32_t mx = 0;
    for (const uint32_t i : idx_big) mx = std::max(mx, b->host.res[2 * (size_t)i + 1] & 0xFFFFu);
    std::lock_guard<std::mutex> g(b->ctx->mu);
    if (b->ctx->hint.serial == b->img->serial) b->ctx->hint.big_maxr = std::max(b->ctx->hint.big_maxr, mx);
  }
  b->done = true;
  return CG_OK;
}

extern "C" {

int cg_batch_route(cg_batch* b, uint32_t i, uint32_t* route, uint32_t* reason_words) {
  if (!b || !route) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  if (i >= b->items.size()) return CG_E_RANGE;
  if (b->items[i].dev < 0) return CG_E_STATE;
  const uint32_t p = b->host.slot((uint32_t)b->items[i].dev);
  if (!b->routes_sorted) {  // (position << 8 | bit) records of the fold, sorted once
    std::sort(b->routes.begin(), b->routes.end());
    b->routes_sorted = true;
  }
  uint32_t r = 0;
  for (auto it = std::lower_bound(b->routes.begin(), b->routes.end(), (uint64_t)p << 8);
       it != b->routes.end() && (*it >> 8) == p; ++it)
    r |= (uint32_t)(*it & 0xFF);
  // a duplicate class reported whole (RS_CLASS: its members listed on the host, Batch::reason_ids)
  const uint32_t nr = b->host.res[2 * (size_t)p + 1] & 0xFFFF;
  const Batch::BigRef* big = b->host.big_of(p);
  const uint32_t* src = big ? big->r : (((b->host.res[2 * (size_t)p] >> 16) & cgi::RF_FORBID) ? b->host.reasons_f : b->host.reasons_p) + (size_t)p * b->host.capr;
  const uint32_t cnt = big ? big->nr : std::min(nr, b->host.capr);
  for (uint32_t k = 0; k < cnt; k++)
    if (src[k] & cgi::RS_CLASS) { r |= CG_ROUTE_CLASS; break; }
  *route = r;
  if (reason_words) *reason_words = cnt;
  return CG_OK;
}

int cg_batch_reruns(cg_batch* b, uint32_t* n) {
  if (!b || !n) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  *n = b->n_rerun;
  return CG_OK;
}

int cg_batch_followups(cg_batch* b, uint32_t* counts) {
  if (!b || !counts) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  for (uint32_t k = 0; k < FU_KINDS; k++) counts[k] = b->n_fu[k];
  return CG_OK;
}

int cg_batch_decision(cg_batch* b, uint32_t i, int* allow, uint32_t* tier) {
  if (!b || !allow) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  if (i >= b->items.size()) return CG_E_RANGE;
  if (b->items[i].dev < 0) return CG_E_STATE;
  i = (uint32_t)b->items[i].dev;
  *allow = b->host.decision(i) ? 1 : 0;
  if (tier) *tier = b->host.tier(i);
  return CG_OK;
}

int cg_batch_diagnostic(cg_batch* b, uint32_t i, int reasons_only, char* buf, size_t cap, size_t* need) {
  if (!b) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  if (i >= b->items.size()) return CG_E_RANGE;
  if (b->items[i].dev < 0) return CG_E_STATE;
  i = (uint32_t)b->items[i].dev;
  std::string s;
  GUARD_RESULT(b->err, { b->host.diagnostic_json(i, s, reasons_only != 0); })
  if (need) *need = s.size() + 1;
  if (!buf || cap < s.size() + 1) return CG_E_RANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return CG_OK;
}

int cg_batch_reasons(cg_batch* b, uint32_t i, uint32_t* idx, uint32_t cap, uint32_t* n, uint32_t* n_errors) {
  if (!b || !n) return CG_E_ARG;
  if (!b->done) return CG_E_STATE;
  if (i >= b->items.size()) return CG_E_RANGE;
  if (b->items[i].dev < 0) return CG_E_STATE;
  i = (uint32_t)b->items[i].dev;
  std::vector<uint32_t> rs, es;
  GUARD_RESULT(b->err, {
    b->host.reason_ids(i, rs);
    b->host.error_recs(i, es);
  })
  *n = (uint32_t)rs.size();
  if (n_errors) *n_errors = (uint32_t)(es.size() / cgi::ERR_WORDS);
  if (idx) for (uint32_t k = 0; k < cap && k < rs.size(); k++) idx[k] = rs[k];
  return rs.size() > cap && idx ? CG_E_RANGE : CG_OK;
}

int cg_batch_time(cg_batch* b, uint32_t iters, float* ms_total) {
  if (!b || !ms_total) return CG_E_ARG;
  if (!b->submitted) return CG_E_STATE;
  if (dev_time_eval(b->img->dev, b->dev, iters, b->ctx->stream, ms_total)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  return CG_OK;
}

int cg_batch_time_split(cg_batch* b, uint32_t iters, float* ms_phase, float* ms_total) {
  if (!b || !ms_phase || !ms_total) return CG_E_ARG;
  if (!b->submitted) return CG_E_STATE;
  if (dev_time_split(b->img->dev, b->dev, iters, b->ctx->stream, ms_phase, ms_total)) { b->err = dev_last_error(); return CG_E_DEVICE; }
  return CG_OK;
}

int cg_batch_bytes(cg_batch* b, uint64_t* batch_bytes, uint64_t* image_bytes, uint64_t* heap_bytes) {
  if (!b) return CG_E_ARG;
  if (batch_bytes) *batch_bytes = b->dev.bytes;
  if (image_bytes) *image_bytes = b->img->dev.bytes;
  if (heap_bytes) *heap_bytes = (uint64_t)b->host.heap.size() * 4;
  return CG_OK;
}

int cg_batch_io(cg_batch* b, uint64_t* h2d_bytes, uint64_t* d2h_bytes, uint64_t* list_words, uint64_t* list_words_shared) {
  if (!b) return CG_E_ARG;
  if (h2d_bytes) *h2d_bytes = b->submitted ? b->dev.bytes - b->dev.out_bytes : 0;
  if (d2h_bytes) *d2h_bytes = b->submitted ? b->dev.out_bytes : 0;
  if (list_words) *list_words = b->host.anc_words;
  if (list_words_shared) *list_words_shared = b->host.anc_shared_words;
  return CG_OK;
}

int cg_is_authorized_json(cg_ctx* ctx, const char* item_json, size_t len, int* allow, char* diag, size_t cap, size_t* need) {
  if (!ctx || !item_json || !allow) return CG_E_ARG;
  cg_batch* b = nullptr;
  int rc = cg_batch_create(ctx, &b);
  if (rc) return rc;
  rc = cg_batch_add_json(b, item_json, len);
  if (!rc) rc = cg_batch_submit(b);
  if (!rc) rc = cg_batch_wait(b, -1);
  if (!rc) rc = cg_batch_decision(b, 0, allow, nullptr);
  if (!rc && (diag || need)) rc = cg_batch_diagnostic(b, 0, 0, diag, cap, need);
  if (rc) ctx->err = b->err;
  cg_batch_destroy(b);
  return rc;
}

}  // extern "C"
