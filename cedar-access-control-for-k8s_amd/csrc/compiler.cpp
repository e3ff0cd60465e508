// Policy compiler: Cedar AST -> flat GPU image (see image.h for the layout).
//
// Lowers what cedar-go v1.1.0 evaluates per request inside (*PolicySet).IsAuthorized (reference
// call site internal/server/store/store.go:31) into:
//   * interned string / entity IDs (policy constants get global IDs; request-only strings get
//     batch-local IDs at encode time, so string equality is ID equality),
//   * a fixed 16-word scope descriptor per policy (principal/action/resource ==, in, is, is-in,
//     action in [..]),
//   * register bytecode for when/unless with explicit short-circuit jumps (forward only), so a
//     wave can walk one policy's program with a wave-uniform PC while lanes (requests) diverge
//     through per-lane skip targets,
//   * constant-folded set/record/extension literals in a constant pool,
//   * `like` patterns pre-split into prefix / middle / suffix literals,
//   * up to NHOT hot attribute paths (var.k0.k1.., depth <= MAX_PATH) that the encoder resolves
//     per request on the host into the columnar request row,
//   * when/unless clauses over those paths as a forward-only branch graph of predicate atoms
//     (image.h "atoms"), and a two-level scope/attribute index over all-atomic images.
// Policy IDs follow the reference store conventions: memory `policy<i>` (memory.go:18),
// directory `<file>.policy<i>` (directory.go:76), CRD `<name><i>-<uid>` (crd.go:60),
// AVP `<id>.<i>` (verified_permissions.go:95), static `allow-all-admission` (main.go:112).
#include <algorithm>
#include <array>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <thread>
#include <tuple>

#include "engine.h"

namespace cg {
using namespace cgi;

namespace {

template <class SidFn>
void emit_value_impl(const HVal& v, std::vector<uint32_t>& out, uint32_t space, SidFn& sid, uint32_t& w0, uint32_t& w1) {
  switch (v.k) {
    case VK::Bool: w0 = mk_w0(T_BOOL, 0); w1 = v.b ? 1u : 0u; return;
    case VK::Long:
      if (v.i >= INT32_MIN && v.i <= INT32_MAX) { w0 = mk_w0(T_LONG, 0); w1 = (uint32_t)(int32_t)v.i; return; }
      {
        uint32_t off = (uint32_t)out.size();
        out.push_back((uint32_t)((uint64_t)v.i & 0xFFFFFFFFu));
        out.push_back((uint32_t)((uint64_t)v.i >> 32));
        w0 = mk_w0(T_LONGREF, mk_ref(space, off)); w1 = 0;
      }
      return;
    case VK::Dec: {
      uint32_t off = (uint32_t)out.size();
      out.push_back((uint32_t)((uint64_t)v.i & 0xFFFFFFFFu));
      out.push_back((uint32_t)((uint64_t)v.i >> 32));
      w0 = mk_w0(T_DEC, mk_ref(space, off)); w1 = 0;
      return;
    }
    case VK::Ip: {
      uint32_t off = (uint32_t)out.size();
      out.push_back((uint32_t)v.ip.v6 | ((uint32_t)v.ip.prefix << 8));
      for (int k = 0; k < 4; k++)
        out.push_back(((uint32_t)v.ip.addr[4 * k] << 24) | ((uint32_t)v.ip.addr[4 * k + 1] << 16) |
                      ((uint32_t)v.ip.addr[4 * k + 2] << 8) | (uint32_t)v.ip.addr[4 * k + 3]);
      w0 = mk_w0(T_IP, mk_ref(space, off)); w1 = 0;
      return;
    }
    case VK::Str: w0 = mk_w0(T_STR, 0); w1 = sid(v.s); return;
    case VK::Ent: {
      uint32_t t = sid(v.etype);
      if (t > X_MASK) throw CedarError("too many strings for entity type ids");
      w0 = mk_w0(T_ENT, t); w1 = sid(v.s);
      return;
    }
    case VK::Set: {
      std::vector<uint32_t> ew;
      ew.reserve(v.elems.size() * 2);
      for (auto& e : v.elems) {
        uint32_t a, b;
        emit_value_impl(e, out, space, sid, a, b);
        ew.push_back(a); ew.push_back(b);
      }
      uint32_t off = (uint32_t)out.size();
      out.push_back((uint32_t)v.elems.size());
      out.insert(out.end(), ew.begin(), ew.end());
      w0 = mk_w0(T_SET, mk_ref(space, off)); w1 = (uint32_t)v.elems.size();
      return;
    }
    case VK::Rec: {
      std::vector<std::array<uint32_t, 3>> fw;
      fw.reserve(v.fields.size());
      for (auto& kv : v.fields) {
        uint32_t a, b;
        emit_value_impl(kv.second, out, space, sid, a, b);
        uint32_t k = sid(kv.first);
        bool dup = false;
        for (auto& f : fw) if (f[0] == k) { f[1] = a; f[2] = b; dup = true; }
        if (!dup) fw.push_back({k, a, b});
      }
      std::sort(fw.begin(), fw.end(), [](const std::array<uint32_t, 3>& x, const std::array<uint32_t, 3>& y) { return x[0] < y[0]; });
      uint32_t off = (uint32_t)out.size();
      out.push_back((uint32_t)fw.size());
      for (auto& f : fw) { out.push_back(f[0]); out.push_back(f[1]); out.push_back(f[2]); }
      w0 = mk_w0(T_REC, mk_ref(space, off)); w1 = (uint32_t)fw.size();
      return;
    }
  }
}

struct Compiler {
  Image& I;
  using Path = std::pair<uint32_t, std::vector<uint32_t>>;  // (var, key sids)
  std::map<Path, uint32_t> hot;                             // hot path -> slot
  // per-policy state
  uint32_t code0 = 0;
  uint32_t max_slot = 0;
  uint32_t lane_off = 0;

  explicit Compiler(Image& img) : I(img) {}

  uint32_t intern(const std::string& s) {
    auto it = I.sid.find(s);
    if (it != I.sid.end()) return it->second;
    uint32_t id = (uint32_t)I.strings.size();
    I.strings.push_back(s);
    I.sid.emplace(s, id);
    return id;
  }

  void value_words(const HVal& v, uint32_t& w0, uint32_t& w1) {
    auto sidf = [this](const std::string& s) { return intern(s); };
    emit_value_impl(v, I.cpool, SP_CPOOL, sidf, w0, w1);
  }
  uint32_t const_val(const HVal& v) {
    uint32_t w0, w1;
    value_words(v, w0, w1);
    uint32_t off = (uint32_t)I.cpool.size();
    I.cpool.push_back(w0);
    I.cpool.push_back(w1);
    return off;
  }

  uint32_t emit(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c, uint32_t imm) {
    uint32_t idx = (uint32_t)(I.code.size() - code0) / 2;
    I.code.push_back(mk_ins(op, d, a, b, c));
    I.code.push_back(imm);
    return idx;
  }
  uint32_t here() const { return (uint32_t)(I.code.size() - code0) / 2; }
  void patch(uint32_t idx, uint32_t imm) { I.code[code0 + 2 * idx + 1] = imm; }

  void slot(uint32_t d) {  // slots NSLOT.. spill to lane scratch (image.h MAX_SLOTS)
    if (d >= MAX_SLOTS) throw CedarError("expression nesting beyond the device evaluator's 64 registers is not supported by the device compiler");
    max_slot = std::max(max_slot, d + 1);
  }
  uint32_t lane(uint32_t words) {  // a region of the policy's lane scratch
    const uint32_t off = lane_off;
    lane_off += words;
    if (lane_off > LANE_MAX) throw CedarError("policy needs more lane scratch than the device provides (not supported by the device compiler)");
    return off;
  }

  static int var_index(const std::string& n) {
    if (n == "principal") return 0;
    if (n == "action") return 1;
    if (n == "resource") return 2;
    return 3;
  }

  // Constant folding of literal-only subtrees (sets, records, extension constructors).
  bool fold(const Expr& e, HVal& out) {
    switch (e.k) {
      case EK::Lit: out = e.lit; return true;
      case EK::Set: {
        HVal s; s.k = VK::Set;
        for (auto& k : e.kids) {
          HVal x;
          if (!fold(*k, x)) return false;
          bool dup = false;
          for (auto& y : s.elems) if (hval_eq(x, y)) { dup = true; break; }
          if (!dup) s.elems.push_back(std::move(x));
        }
        out = std::move(s);
        return true;
      }
      case EK::Rec: {
        HVal r; r.k = VK::Rec;
        for (size_t i = 0; i < e.kids.size(); i++) {
          HVal x;
          if (!fold(*e.kids[i], x)) return false;
          r.fields.emplace_back(e.keys[i], std::move(x));
        }
        out = std::move(r);
        return true;
      }
      case EK::Call: {
        if (e.kids.size() != 1) return false;
        HVal a;
        if (!fold(*e.kids[0], a) || a.k != VK::Str) return false;
        HVal r;
        if (e.name == "decimal") { r.k = VK::Dec; if (!parse_decimal(a.s, &r.i)) return false; out = r; return true; }
        if (e.name == "ip") { r.k = VK::Ip; if (!parse_ip(a.s, &r.ip)) return false; out = r; return true; }
        return false;
      }
      default: return false;
    }
  }

  uint32_t ext_msg(const std::string& m) {
    I.ext_msgs.push_back(m);
    return (uint32_t)I.ext_msgs.size() - 1;
  }

  // `like` pattern -> [flags (bit0 star, bits 8.. #middles), prefix, suffix, middles...], each
  // literal as [len, bytes packed 4 per word]. Appended to `dst`; returns its offset there.
  static uint32_t pattern_into(const std::vector<PatPiece>& pat, std::vector<uint32_t>& dst) {
    // collapse into literal runs separated by stars
    std::vector<std::string> lits;
    bool has_star = false;
    lits.push_back("");
    for (auto& p : pat) {
      if (p.star) { has_star = true; lits.push_back(""); }
      else lits.back() += p.lit;
    }
    // lits[0] = prefix, lits.back() = suffix (when has_star), middles between (empty ones dropped)
    uint32_t off = (uint32_t)dst.size();
    auto put_lit = [&dst](const std::string& s) {
      dst.push_back((uint32_t)s.size());
      for (size_t k = 0; k < s.size(); k += 4) {
        uint32_t w = 0;
        for (size_t j = 0; j < 4 && k + j < s.size(); j++) w |= (uint32_t)(uint8_t)s[k + j] << (8 * j);
        dst.push_back(w);
      }
    };
    if (!has_star) {
      dst.push_back(0);  // flags: no star, 0 middles
      put_lit(lits[0]);
      return off;
    }
    std::vector<std::string> mids;
    for (size_t k = 1; k + 1 < lits.size(); k++) if (!lits[k].empty()) mids.push_back(lits[k]);
    dst.push_back(1u | ((uint32_t)mids.size() << 8));
    put_lit(lits[0]);
    put_lit(lits.back());
    for (auto& m : mids) put_lit(m);
    return off;
  }
  uint32_t pattern(const std::vector<PatPiece>& pat) { return pattern_into(pat, I.cpool); }

  void compile(const Expr& e, uint32_t d) {
    slot(d);
    HVal cv;
    if (e.k != EK::Lit && (e.k == EK::Set || e.k == EK::Rec || e.k == EK::Call) && fold(e, cv)) {
      emit(OP_LDC, d, 0, 0, 0, const_val(cv));
      return;
    }
    switch (e.k) {
      case EK::Lit:
        if (e.lit.k == VK::Bool) emit(OP_LDB, d, 0, 0, 0, e.lit.b ? 1 : 0);
        else if (e.lit.k == VK::Str) emit(OP_LDS, d, 0, 0, 0, intern(e.lit.s));
        else emit(OP_LDC, d, 0, 0, 0, const_val(e.lit));
        return;
      case EK::Var: emit(OP_LDV, d, 0, 0, 0, (uint32_t)var_index(e.name)); return;
      case EK::Attr:
      case EK::Has: {
        const Expr& k0 = *e.kids[0];
        int h = hot_of(e);
        if (h >= 0) {
          emit(e.k == EK::Attr ? OP_HOT : OP_HOTHAS, d, 0, 0, (uint32_t)h, 0);
          return;
        }
        compile(k0, d);
        emit(e.k == EK::Attr ? OP_ATTR : OP_HAS, d, d, 0, 0, intern(e.name));
        return;
      }
      case EK::And:
      case EK::Or: {
        compile(*e.kids[0], d);
        uint32_t j = emit(e.k == EK::And ? OP_JF : OP_JT, 0, d, 0, 0, 0);
        compile(*e.kids[1], d);
        emit(OP_CHKB, 0, d, 0, 0, 0);
        patch(j, here());
        return;
      }
      case EK::Not: compile(*e.kids[0], d); emit(OP_NOT, d, d, 0, 0, 0); return;
      case EK::Neg: compile(*e.kids[0], d); emit(OP_NEG, d, d, 0, 0, 0); return;
      case EK::If: {
        compile(*e.kids[0], d);
        uint32_t jelse = emit(OP_JNF, 0, d, 0, 0, 0);
        compile(*e.kids[1], d);
        uint32_t jend = emit(OP_JMP, 0, 0, 0, 0, 0);
        patch(jelse, here());
        compile(*e.kids[2], d);
        patch(jend, here());
        return;
      }
      case EK::Bin: {
        compile(*e.kids[0], d);
        compile(*e.kids[1], d + 1);
        static const uint32_t ops[] = {OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE, OP_ADD, OP_SUB, OP_MUL, OP_IN};
        emit(ops[(int)e.op], d, d, d + 1, 0, 0);
        return;
      }
      case EK::Like: compile(*e.kids[0], d); emit(OP_LIKE, d, d, 0, 0, pattern(e.pat)); return;
      case EK::Is: {
        if (!e.has_in) { compile(*e.kids[0], d); emit(OP_IS, d, d, 0, 0, intern(e.name)); return; }
        compile(*e.kids[0], d + 1);
        slot(d + 2);
        emit(OP_IS, d, d + 1, 0, 0, intern(e.name));
        uint32_t j = emit(OP_JF, 0, d, 0, 0, 0);
        compile(*e.kids[1], d + 2);
        emit(OP_IN, d, d + 1, d + 2, 0, 0);
        patch(j, here());
        return;
      }
      case EK::Call: {
        // constant extension call that failed to fold => runtime error every evaluation
        HVal a;
        if (e.kids.size() == 1 && fold(*e.kids[0], a) && a.k == VK::Str && (e.name == "decimal" || e.name == "ip")) {
          emit(OP_ERR, 0, 0, 0, E_EXT, ext_msg("error parsing " + std::string(e.name == "ip" ? "ip" : "decimal") + " value: " + a.s));
          return;
        }
        if (e.kids.size() != 1 || (e.name != "decimal" && e.name != "ip")) throw CedarError("unknown extension function " + e.name);
        // ip(x) / decimal(x) over a runtime value: parsed on the device into lane scratch
        compile(*e.kids[0], d);
        const bool ip = e.name == "ip";
        emit(OP_CALL, d, d, 0, ip ? CO_PARSE_IP : CO_PARSE_DEC, lane(ip ? 5u : 2u));
        return;
      }
      case EK::Method: {
        const std::string& m = e.name;
        size_t nargs = e.kids.size() - 1;
        compile(*e.kids[0], d);
        if (m == "contains" || m == "containsAll" || m == "containsAny" || m == "lessThan" || m == "lessThanOrEqual" ||
            m == "greaterThan" || m == "greaterThanOrEqual" || m == "isInRange") {
          if (nargs != 1) throw CedarError(m + " takes exactly one argument");
          compile(*e.kids[1], d + 1);
          if (m == "contains") { emit(OP_CONTAINS, d, d, d + 1, 0, 0); return; }
          uint32_t co = m == "containsAll" ? CO_CONTAINS_ALL : m == "containsAny" ? CO_CONTAINS_ANY
                      : m == "lessThan" ? CO_DEC_LT : m == "lessThanOrEqual" ? CO_DEC_LE
                      : m == "greaterThan" ? CO_DEC_GT : m == "greaterThanOrEqual" ? CO_DEC_GE : CO_IP_IN_RANGE;
          emit(OP_CALL, d, d, d + 1, co, 0);
          return;
        }
        if (nargs != 0) throw CedarError(m + " takes no arguments");
        uint32_t co;
        if (m == "isEmpty") co = CO_IS_EMPTY;
        else if (m == "isIpv4") co = CO_IP_V4;
        else if (m == "isIpv6") co = CO_IP_V6;
        else if (m == "isLoopback") co = CO_IP_LOOPBACK;
        else if (m == "isMulticast") co = CO_IP_MULTICAST;
        else throw CedarError("unknown method " + m);
        emit(OP_CALL, d, d, 0, co, 0);
        return;
      }
      case EK::Set: {
        uint32_t n = (uint32_t)e.kids.size();
        if (n >= MAX_LITERAL) throw CedarError("non-constant set literal of 4096 or more elements is not supported by the device compiler");
        const uint32_t off = lane(1 + 4 * n);  // [n, (w0,w1)*n, (lo,hi)*n spare for 64-bit longs]
        emit(OP_SETNEW, d, 0, 0, 0, off | (n << 20));  // lane offset < 2^20, n < 2^12
        for (uint32_t i = 0; i < n; i++) {
          compile(*e.kids[i], d + 1);
          emit(OP_SETPUT, d, d + 1, 0, 0, i);
        }
        return;
      }
      case EK::Rec: {
        uint32_t n = (uint32_t)e.kids.size();
        if (n >= MAX_LITERAL) throw CedarError("non-constant record literal of 4096 or more fields is not supported by the device compiler");
        const uint32_t off = lane(1 + 5 * n);  // [n, (key,w0,w1)*n, (lo,hi)*n spare]
        std::vector<std::pair<uint32_t, uint32_t>> order;  // (key sid, source index)
        for (uint32_t i = 0; i < n; i++) order.emplace_back(intern(e.keys[i]), i);
        std::vector<uint32_t> pos(n);
        auto sorted = order;
        std::sort(sorted.begin(), sorted.end());
        for (uint32_t k = 0; k < n; k++) pos[sorted[k].second] = k;
        emit(OP_RECNEW, d, 0, 0, 0, off | (n << 20));
        for (uint32_t i = 0; i < n; i++) {
          compile(*e.kids[i], d + 1);
          emit(OP_RECPUT, d, d + 1, pos[i] >> 6, pos[i] & 63, order[i].first);  // position c | b << 6
        }
        return;
      }
    }
    throw CedarError("unsupported expression");
  }

  // Path of an attribute-access / has chain rooted at a variable: `resource.metadata.name` and
  // `resource.metadata has name` both have path (resource, [metadata, name]).
  bool path_of(const Expr& e, Path& out) {
    if (e.k != EK::Attr && e.k != EK::Has) return false;
    std::vector<uint32_t> keys{intern(e.name)};
    const Expr* x = e.kids[0].get();
    while (x->k == EK::Attr) {
      keys.push_back(intern(x->name));
      x = x->kids[0].get();
    }
    if (x->k != EK::Var || keys.size() > MAX_PATH) return false;
    std::reverse(keys.begin(), keys.end());
    out = Path((uint32_t)var_index(x->name), std::move(keys));
    return true;
  }
  void count_hot(const Expr& e, std::map<Path, uint32_t>& cnt) {
    Path p;
    if (path_of(e, p)) cnt[p]++;
    for (auto& k : e.kids) count_hot(*k, cnt);
  }

  // ---- atoms ----------------------------------------------------------------------------------
  int hot_of(const Expr& e) {  // e is an Attr/Has chain over a Var
    Path p;
    if (!path_of(e, p)) return -1;
    auto it = hot.find(p);
    return it == hot.end() ? -1 : (int)it->second;
  }
  std::vector<uint32_t> hot_depth;  // slot -> path depth
  static bool is_prim(const HVal& v) { return v.k == VK::Bool || v.k == VK::Long || v.k == VK::Str || v.k == VK::Ent; }
  void reg_form(const HVal& v, uint32_t* w) {
    switch (v.k) {
      case VK::Bool: w[0] = mk_w0(T_BOOL, 0); w[1] = v.b ? 1 : 0; w[2] = 0; break;
      case VK::Long: w[0] = mk_w0(T_LONG, 0); w[1] = (uint32_t)((uint64_t)v.i & 0xFFFFFFFFu); w[2] = (uint32_t)((uint64_t)v.i >> 32); break;
      case VK::Str: w[0] = mk_w0(T_STR, 0); w[1] = intern(v.s); w[2] = 0; break;
      default: w[0] = mk_w0(T_ENT, intern(v.etype)); w[1] = intern(v.s); w[2] = 0; break;
    }
  }
  bool lit_prim(const Expr& e, HVal& v) {
    if (e.k == EK::Lit && is_prim(e.lit)) { v = e.lit; return true; }
    return false;
  }
  // One leaf predicate -> one atom (kind, h, operands) or false. *neg: the atom's truth is the
  // negation of the expression's (`!=`). Data-carrying atoms get w1 relative to adata and
  // *patch set (re-based to the record once the atom count is known).
  bool atom(const Expr& e0, uint32_t* w, bool* neg, bool* patch) {
    const Expr* e = &e0;
    w[0] = w[1] = w[2] = w[3] = 0;
    *neg = false;
    *patch = false;
    auto put = [&](uint32_t kind, uint32_t h) {
      w[0] = kind | (h << 8);
      // set-membership atoms read the slot's element hashes (image.h "set-membership keys")
      if (kind == AK_CONTAINS || kind == AK_RECSET) I.cslot_mask |= 1u << h;
      return true;
    };
    HVal c;
    int h;
    switch (e->k) {
      case EK::Has:
        if ((h = hot_of(*e)) < 0) return false;
        return put(AK_HAS, (uint32_t)h);
      case EK::Attr:
        if ((h = hot_of(*e)) < 0) return false;
        return put(AK_BOOL, (uint32_t)h);
      case EK::Like: {
        if ((h = hot_of(*e->kids[0])) < 0 || e->kids[0]->k != EK::Attr) return false;
        // one star at most and literals within 8 bytes: inline (AK_LIKEI), nothing to read but the
        // value's first and last 8 bytes (CEDARGPU_NO_LIKEI: the record form everywhere, A/B).
        // CEDARGPU_LIKE_WORDS=1 also ships those bytes in the row (6 words per like slot, image.h
        // LIKE_WORDS): neutral on the step in the round-5 A/B, and 48 B more per C3
        // request to upload, so off by default.
        static const bool no_likei = std::getenv("CEDARGPU_NO_LIKEI") != nullptr;
        // (read per atom, not once per process: a test can build images both ways in one process;
        // the device reads staged words only for slots in the image's lslot_mask)
        const char* lw_env = std::getenv("CEDARGPU_LIKE_WORDS");
        const bool like_words = lw_env && *lw_env == '1';
        std::string pre, suf;
        bool star = false, inl = !no_likei;
        for (auto& pc : e->pat) {
          if (pc.star) {
            if (star && !suf.empty()) inl = false;  // a middle literal
            star = true;
          } else {
            (star ? suf : pre) += pc.lit;
          }
        }
        if (inl && pre.size() + suf.size() <= LIKEI_MAX) {
          uint64_t b = 0;
          const std::string lit = pre + suf;
          for (size_t j = 0; j < lit.size(); j++) b |= (uint64_t)(uint8_t)lit[j] << (8 * j);
          w[1] = (uint32_t)b;
          w[2] = (uint32_t)(b >> 32);
          w[3] = (uint32_t)pre.size() | ((uint32_t)suf.size() << 4) | (star ? 1u << 8 : 0u);
          if (like_words) I.lslot_mask |= 1u << h;
          I.lread_mask |= h < 32 ? 1u << h : 0xFFFFFFFFu;
          return put(AK_LIKEI, (uint32_t)h);
        }
        I.lread_mask |= h < 32 ? 1u << h : 0xFFFFFFFFu;
        w[1] = pattern_into(e->pat, adata);
        *patch = true;
        return put(AK_LIKE, (uint32_t)h);
      }
      case EK::Lit:
        if (e->lit.k != VK::Bool) return false;
        *neg = !e->lit.b;
        return put(AK_TRUE, 0);
      case EK::Is:
        if (e->has_in || e->kids[0]->k != EK::Var || e->kids[0]->name == "context") return false;
        w[1] = intern(e->name);
        return put(AK_IS, (uint32_t)var_index(e->kids[0]->name));
      case EK::Method: {
        if (e->name == "contains" && e->kids.size() == 2 && e->kids[1]->k != EK::Rec) {
        const Expr& recv = *e->kids[0];
        const Expr& arg = *e->kids[1];
        HVal s;
        if (recv.k == EK::Set && fold(recv, s)) {
          if (arg.k != EK::Attr || (h = hot_of(arg)) < 0) return false;
          for (auto& x : s.elems) if (!is_prim(x)) return false;
          bool strs = !s.elems.empty() && s.elems.size() <= 3;
          for (auto& x : s.elems) strs = strs && x.k == VK::Str;
          if (strs) {  // 1 to 3 strings: inline (AK_INSTR), repeats fill the unused words
            for (uint32_t j = 0; j < 3; j++) w[1 + j] = intern(s.elems[std::min<size_t>(j, s.elems.size() - 1)].s);
            return put(AK_INSTR, (uint32_t)h);
          }
          uint32_t off = (uint32_t)adata.size();
          for (auto& x : s.elems) { uint32_t r[3]; reg_form(x, r); adata.insert(adata.end(), r, r + 3); }
          w[1] = off;
          w[2] = (uint32_t)s.elems.size();
          *patch = true;
          return put(AK_INSET, (uint32_t)h);
        }
        if (recv.k == EK::Attr && (h = hot_of(recv)) >= 0 && lit_prim(arg, c)) {
          reg_form(c, &w[1]);
          return put(AK_CONTAINS, (uint32_t)h);
        }
        return false;
      }
      if (e->name == "containsAny" || e->name == "contains") {
        // label-selector shape: hot.containsAny([{k: lit|hot|[lit|hot..]}, ..]) / hot.contains({..})
        if (e->kids.size() != 2) return false;
        const Expr& recv = *e->kids[0];
        const Expr& arg = *e->kids[1];
        if (recv.k != EK::Attr || (h = hot_of(recv)) < 0) return false;
        std::vector<const Expr*> tmpls;
        if (e->name == "contains") {
          if (arg.k != EK::Rec) return false;
          tmpls.push_back(&arg);
        } else {
          if (arg.k != EK::Set) return false;
          for (auto& k : arg.kids) {
            if (k->k != EK::Rec) return false;
            tmpls.push_back(k.get());
          }
        }
        std::vector<uint32_t> holes, body;
        std::vector<std::pair<size_t, uint32_t>> setlits;  // (body index of field word a, body offset of list)
        std::vector<uint32_t> lists;
        auto elem = [&](const Expr& x, uint32_t* o) {  // o: kind + 3 operand words
          HVal v;
          int hh;
          if (lit_prim(x, v)) { o[0] = RF_CONST; reg_form(v, o + 1); return true; }
          if (x.k == EK::Attr && (hh = hot_of(x)) >= 0) {
            o[0] = RF_HOLE; o[1] = (uint32_t)hh; o[2] = o[3] = 0;
            holes.push_back((uint32_t)hh);
            return true;
          }
          return false;
        };
        for (const Expr* t : tmpls) {
          const uint32_t n = (uint32_t)t->kids.size();
          std::vector<std::pair<uint32_t, std::array<uint32_t, 5>>> fields;
          for (uint32_t i = 0; i < n; i++) {  // source order: holes are evaluated in this order
            std::array<uint32_t, 5> f{intern(t->keys[i]), 0, 0, 0, 0};
            const Expr& x = *t->kids[i];
            if (x.k == EK::Set) {
              f[1] = RF_SETLIT;
              f[2] = (uint32_t)lists.size();  // patched below
              f[3] = (uint32_t)x.kids.size();
              for (auto& el : x.kids) {
                uint32_t o[4];
                if (!elem(*el, o)) return false;
                lists.insert(lists.end(), o, o + 4);
              }
            } else {
              uint32_t o[4];
              if (!elem(x, o)) return false;
              f[1] = o[0]; f[2] = o[1]; f[3] = o[2]; f[4] = o[3];
            }
            fields.emplace_back(f[0], f);
          }
          std::sort(fields.begin(), fields.end(), [](auto& a, auto& b) { return a.first < b.first; });
          body.push_back(n);
          for (auto& f : fields) {
            if (f.second[1] == RF_SETLIT) setlits.emplace_back(body.size() + 2, f.second[2]);
            body.insert(body.end(), f.second.begin(), f.second.end());
          }
        }
        // data = [holes][templates][element lists]; offsets relative to the data start for now
        const uint32_t off = (uint32_t)adata.size();
        const uint32_t hdr = 1 + (uint32_t)holes.size();
        const uint32_t lists_at = off + hdr + (uint32_t)body.size();
        for (auto& sl : setlits) body[sl.first] = lists_at + sl.second;
        adata.push_back((uint32_t)holes.size());
        adata.insert(adata.end(), holes.begin(), holes.end());
        adata.insert(adata.end(), body.begin(), body.end());
        adata.insert(adata.end(), lists.begin(), lists.end());
        for (auto& sl : setlits) rs_patch.push_back(off + hdr + (uint32_t)sl.first);
        w[1] = off;
        w[2] = (uint32_t)tmpls.size();
        w[3] = e->name == "contains" ? 1u : 0u;
        *patch = true;
        return put(AK_RECSET, (uint32_t)h);
      }
      return false;
      }
      case EK::Bin: {
        const Expr& l = *e->kids[0];
        const Expr& r = *e->kids[1];
        if (e->op == BinOp::Eq || e->op == BinOp::Ne) {
          if (e->op == BinOp::Ne) *neg = true;
          if (l.k == EK::Attr && (h = hot_of(l)) >= 0 && lit_prim(r, c)) { reg_form(c, &w[1]); return put(AK_EQ, (uint32_t)h); }
          if (r.k == EK::Attr && (h = hot_of(r)) >= 0 && lit_prim(l, c)) { reg_form(c, &w[1]); return put(AK_EQ, (uint32_t)h); }
          const Expr* var = l.k == EK::Var ? &l : (r.k == EK::Var ? &r : nullptr);
          const Expr& other = &l == var ? r : l;
          if (var && var->name != "context" && lit_prim(other, c) && c.k == VK::Ent) {
            w[1] = intern(c.etype);
            w[2] = intern(c.s);
            return put(AK_EQV, (uint32_t)var_index(var->name));
          }
          int h2;
          if (l.k == EK::Attr && r.k == EK::Attr && (h = hot_of(l)) >= 0 && (h2 = hot_of(r)) >= 0) {
            w[1] = (uint32_t)h2;
            return put(AK_EQH, (uint32_t)h);
          }
          return false;
        }
        if (e->op == BinOp::In) {
          if (l.k != EK::Var || l.name == "context") return false;
          if (lit_prim(r, c) && c.k == VK::Ent) {
            w[1] = intern(c.etype);
            w[2] = intern(c.s);
            w[3] = uid_bloom_bit(w[1], w[2]);
            return put(AK_IN, (uint32_t)var_index(l.name));
          }
          HVal sv;
          if (r.k == EK::Set && fold(r, sv)) {  // var in [E1, E2, ..]: entity literals only
            for (auto& x : sv.elems) if (x.k != VK::Ent) return false;
            uint32_t off = (uint32_t)adata.size();
            for (auto& x : sv.elems) { adata.push_back(intern(x.etype)); adata.push_back(intern(x.s)); }
            w[1] = off;
            w[2] = (uint32_t)sv.elems.size();
            *patch = true;
            return put(AK_INANY, (uint32_t)var_index(l.name));
          }
          return false;
        }
        if (e->op == BinOp::Lt || e->op == BinOp::Le || e->op == BinOp::Gt || e->op == BinOp::Ge) {
          static const uint32_t code[] = {0, 1, 2, 3};
          static const uint32_t mirror[] = {2, 3, 0, 1};
          uint32_t op = code[(int)e->op - (int)BinOp::Lt];
          if (l.k == EK::Attr && (h = hot_of(l)) >= 0 && lit_prim(r, c) && c.k == VK::Long) {
          } else if (r.k == EK::Attr && (h = hot_of(r)) >= 0 && lit_prim(l, c) && c.k == VK::Long) {
            op = mirror[op];
          } else {
            return false;
          }
          w[1] = op;
          w[2] = (uint32_t)((uint64_t)c.i & 0xFFFFFFFFu);
          w[3] = (uint32_t)((uint64_t)c.i >> 32);
          return put(AK_LCMP, (uint32_t)h);
        }
        return false;
      }
      default: return false;
    }
  }
  // ---- atom graph ------------------------------------------------------------------------------
  // Labels are forward references to atom indices; L_SAT / L_UNSAT are the policy outcomes.
  static constexpr uint32_t L_SAT = 0xFFFFFFFFu, L_UNSAT = 0xFFFFFFFEu;
  struct AtomB {
    uint32_t w[4];
    uint32_t t, f;  // labels
    bool patch;
  };
  std::vector<AtomB> ab;
  std::vector<int64_t> label_at;
  uint32_t new_label() { label_at.push_back(-1); return (uint32_t)label_at.size() - 1; }
  void place(uint32_t l) { label_at[l] = (int64_t)ab.size(); }
  // Lowers boolean expression e so that control reaches T when it is true and F when false.
  bool gen(const Expr& e, uint32_t T, uint32_t F) {
    switch (e.k) {
      case EK::And: {
        uint32_t l = new_label();
        if (!gen(*e.kids[0], l, F)) return false;
        place(l);
        return gen(*e.kids[1], T, F);
      }
      case EK::Or: {
        uint32_t l = new_label();
        if (!gen(*e.kids[0], T, l)) return false;
        place(l);
        return gen(*e.kids[1], T, F);
      }
      case EK::Not: return gen(*e.kids[0], F, T);
      case EK::If: {
        uint32_t lt = new_label(), le = new_label();
        if (!gen(*e.kids[0], lt, le)) return false;
        place(lt);
        if (!gen(*e.kids[1], T, F)) return false;
        place(le);
        return gen(*e.kids[2], T, F);
      }
      case EK::Is:
        if (e.has_in) {
          // `v is T in E`: the type test short-circuits before E is evaluated
          if (e.kids[0]->k != EK::Var || e.kids[0]->name == "context") return false;
          Expr is = e;
          is.has_in = false;
          is.kids.resize(1);
          Expr in;
          in.k = EK::Bin;
          in.op = BinOp::In;
          in.kids = {e.kids[0], e.kids[1]};
          uint32_t l = new_label();
          if (!gen(is, l, F)) return false;
          place(l);
          return gen(in, T, F);
        }
        break;
      default: break;
    }
    AtomB a;
    bool neg;
    if (!atom(e, a.w, &neg, &a.patch)) return false;
    a.t = neg ? F : T;
    a.f = neg ? T : F;
    ab.push_back(a);
    return ab.size() <= MAX_ATOMS;
  }

  // All when/unless clauses as one atom graph, or false (then the policy uses bytecode).
  // Output: atoms, then their data (INSET element triples, LIKE patterns, ...) addressed relative
  // to the policy record start; *n_atom_words = words of atoms proper.
  std::vector<uint32_t> adata;
  std::vector<uint32_t> rs_patch;  // adata words holding adata-relative offsets
  bool atoms(const Policy& p, std::vector<uint32_t>& out, uint32_t* n_atom_words) {
    adata.clear();
    rs_patch.clear();
    ab.clear();
    label_at.clear();
    for (size_t i = 0; i < p.conds.size(); i++) {
      const bool when = p.conds[i].first;
      const uint32_t next = i + 1 < p.conds.size() ? new_label() : L_SAT;
      if (!gen(*p.conds[i].second, when ? next : L_UNSAT, when ? L_UNSAT : next)) return false;
      if (next != L_SAT) place(next);
    }
    auto target = [&](uint32_t l) -> uint32_t {
      if (l == L_SAT) return AT_SAT;
      if (l == L_UNSAT) return AT_UNSAT;
      if (label_at[l] < 0 || label_at[l] >= (int64_t)ab.size()) throw CedarError("internal: dangling atom label");
      return (uint32_t)label_at[l];
    };
    const uint32_t base = POL_WORDS + ATOM_WORDS * (uint32_t)ab.size();
    out.clear();
    for (size_t i = 0; i < ab.size(); i++) {
      AtomB& a = ab[i];
      const uint32_t t = target(a.t), f = target(a.f);
      if ((t < AT_UNSAT && t <= i) || (f < AT_UNSAT && f <= i)) throw CedarError("internal: backward atom edge");
      out.push_back(a.w[0] | (t << 16) | (f << 24));
      out.push_back(a.patch ? a.w[1] + base : a.w[1]);
      out.push_back(a.w[2]);
      out.push_back(a.w[3]);
    }
    *n_atom_words = (uint32_t)out.size();
    for (uint32_t k : rs_patch) adata[k] += base;
    out.insert(out.end(), adata.begin(), adata.end());
    return true;
  }

  // Attribute key of an atomic policy (image.h "scope index", level 2): the first equality atom
  // on the graph's entry spine (each earlier atom cannot raise and has one edge to UNSAT), whose
  // false edge is UNSAT and whose constant has a canonical memory form.
  struct AttrKey {
    bool ok = false, guarded = false;
    bool contains = false;  // a set-membership key (image.h BT_CKEY): v0 = element hash, v1 = 1
    uint32_t plen = 0;      // a prefix key (image.h "prefix level-2 keys"): prefix bytes hashed into v0
    uint32_t h = 0, v0 = 0, v1 = 0;
    // required presence (image.h "presence masks"): single-level hot slots a `has` atom of the
    // entry spine requires, where no atom before it can raise: mpre before the key atom (or on the
    // whole spine of an unkeyed policy), mpost also after it (exact in a bucket of the key's value,
    // where the key atom cannot raise)
    uint32_t mpre = 0, mpost = 0;
    uint32_t filt = 0;  // the equality after the key atom (image.h "equality filters"), 0: none
  };

  // `has` slots the spine requires from atom i on, up to the first atom that can raise; with
  // `filt`, that atom's equality filter when it is `hot(h) == constant` (image.h "equality filters")
  uint32_t spine_has(const std::vector<uint32_t>& at, uint32_t n, uint32_t i, uint32_t* filt = nullptr) const {
    uint32_t m = 0;
    while (i < n) {
      const uint32_t* a = &at[ATOM_WORDS * i];
      const uint32_t kind = a[0] & 0xFF, h = (a[0] >> 8) & 0xFF, t = (a[0] >> 16) & 0xFF, f = a[0] >> 24;
      const bool no_error = kind == AK_IS || kind == AK_IN || kind == AK_INANY || kind == AK_TRUE || kind == AK_EQV ||
                            (kind == AK_HAS && hot_depth[h] == 1);
      if (!no_error) {
        const uint32_t tag = a[1] >> TAG_SHIFT;
        if (filt && kind == AK_EQ && f == AT_UNSAT && t != AT_UNSAT && h < EQF_SLOTS &&
            (tag == T_STR || tag == T_BOOL || tag == T_ENT))
          *filt = EQF_ON | (h << EQF_SLOT_SHIFT) | eqf_hash(a[1], a[2]);
        break;
      }
      if (f == AT_UNSAT && t < AT_UNSAT) {
        if (kind == AK_HAS && h < ASELF_PRES_SLOTS) m |= 1u << h;  // (the row carries slots 0..14)
        i = t;
      } else if (t == AT_UNSAT && f < AT_UNSAT) {
        i = f;
      } else {
        break;
      }
    }
    return m;
  }

  AttrKey attr_key(const std::vector<uint32_t>& at, uint32_t n_atom_words) const {
    AttrKey k;
    const uint32_t n = n_atom_words / ATOM_WORDS;
    std::vector<uint32_t> present;  // single-level hot slots known present on the spine
    uint32_t i = 0;
    k.mpre = k.mpost = spine_has(at, n, 0);
    while (i < n) {
      const uint32_t* a = &at[ATOM_WORDS * i];
      const uint32_t kind = a[0] & 0xFF, h = (a[0] >> 8) & 0xFF, t = (a[0] >> 16) & 0xFF, f = a[0] >> 24;
      if (kind == AK_EQ && f == AT_UNSAT && t != AT_UNSAT) {
        const uint32_t tag = a[1] >> TAG_SHIFT;
        const bool small_long = tag == T_LONG && a[3] == (((int32_t)a[2] < 0) ? 0xFFFFFFFFu : 0u);
        if (tag == T_STR || tag == T_BOOL || tag == T_ENT || small_long) {
          k.ok = true;
          k.h = h;
          k.v0 = tag == T_LONG ? mk_w0(T_LONG, 0) : a[1];
          k.v1 = a[2];
          k.guarded = std::find(present.begin(), present.end(), h) != present.end();
          k.mpost = k.mpre | spine_has(at, n, t, &k.filt);
        }
        return k;
      }
      // hot(h).contains(primitive) / hot(h).contains({k: primitive, ..}) on the spine: a
      // set-membership key (image.h BT_CKEY)
      if ((kind == AK_CONTAINS || (kind == AK_RECSET && a[3] == 1 && a[2] == 1)) && f == AT_UNSAT && t != AT_UNSAT) {
        uint32_t hv = 0;
        bool keyable = false;
        if (kind == AK_CONTAINS) {
          keyable = reg_chash(a[1], a[2], a[3], hv);
        } else {
          const uint32_t* d = &at[a[1] - POL_WORDS];  // [n_holes, holes.., n_keys, (key, kind, a, b, c)..]
          if (d[0] == 0) {
            const uint32_t nk = d[1];
            keyable = true;
            hv = chash_mix(CHASH_REC, nk);
            for (uint32_t j = 0; j < nk && keyable; j++) {
              const uint32_t* fld = &d[2 + RS_FIELD_WORDS * j];
              uint32_t fh = 0;
              keyable = fld[1] == RF_CONST && reg_chash(fld[2], fld[3], fld[4], fh);
              hv = chash_mix(chash_mix(hv, fld[0]), fh);
            }
          }
        }
        if (keyable) {
          k.ok = true;
          k.contains = true;
          k.h = h;
          k.v0 = hv;
          k.v1 = 1;
          k.guarded = std::find(present.begin(), present.end(), h) != present.end();
          k.mpost = k.mpre | spine_has(at, n, t, &k.filt);
        }
        return k;
      }
      // hot(h) like "lit*..." on the spine: a prefix key on the pattern's opening literal (a
      // pattern without a star is its whole literal, which is also a prefix of every match)
      if ((kind == AK_LIKE || kind == AK_LIKEI) && f == AT_UNSAT && t != AT_UNSAT) {
        uint32_t len = 0;
        uint8_t bytes[PFX_MAX];
        if (kind == AK_LIKE) {
          const uint32_t* pw = &at[a[1] - POL_WORDS];  // [flags, prefix len, prefix bytes ...]
          len = std::min(pw[1], PFX_MAX);
          for (uint32_t j = 0; j < len; j++) bytes[j] = (uint8_t)(pw[2 + (j >> 2)] >> (8 * (j & 3)));
        } else {  // inline: the prefix is the first (w3 & 15) bytes of w1, w2
          len = a[3] & 15u;
          for (uint32_t j = 0; j < len; j++) bytes[j] = (uint8_t)(a[1 + (j >> 2)] >> (8 * (j & 3)));
        }
        if (len > 0) {
          k.ok = true;
          k.contains = true;
          k.plen = len;
          k.h = h;
          k.v0 = pfx_hash(bytes, len);
          k.v1 = 1;
          k.guarded = std::find(present.begin(), present.end(), h) != present.end();
          k.mpost = k.mpre | spine_has(at, n, t, &k.filt);
        }
        return k;
      }
      const bool no_error = kind == AK_IS || kind == AK_IN || kind == AK_INANY || kind == AK_TRUE || kind == AK_EQV ||
                            (kind == AK_HAS && hot_depth[h] == 1);
      if (!no_error) return k;
      uint32_t nxt;
      if (f == AT_UNSAT && t < AT_UNSAT) {
        nxt = t;
        if (kind == AK_HAS) present.push_back(h);
      } else if (t == AT_UNSAT && f < AT_UNSAT) {
        nxt = f;
      } else {
        return k;
      }
      i = nxt;
    }
    return k;
  }

  std::map<std::pair<uint32_t, uint32_t>, uint32_t> act_index;  // action entity -> bit
  void collect_actions(const Scope& s) {
    auto add = [this](const std::pair<std::string, std::string>& e) {
      std::pair<uint32_t, uint32_t> k{intern(e.first), intern(e.second)};
      if (!act_index.count(k)) {
        act_index.emplace(k, (uint32_t)act_index.size());
        I.act.push_back(k.first);
        I.act.push_back(k.second);
      }
    };
    if (s.kind == ScopeKind::Eq || s.kind == ScopeKind::In) add(s.ent);
    if (s.kind == ScopeKind::InSet) for (auto& e : s.ents) add(e);
  }
  uint64_t action_mask(const Scope& s) {
    if (s.kind == ScopeKind::Any) return ~0ull;
    uint64_t m = 0;
    auto bit = [&](const std::pair<std::string, std::string>& e) {
      uint32_t b = act_index.at({intern(e.first), intern(e.second)});
      if (b < 64) m |= 1ull << b;
    };
    if (s.kind == ScopeKind::InSet) for (auto& e : s.ents) bit(e);
    else bit(s.ent);
    return m;
  }

  void scope_words(const Scope& s, uint32_t* w_type, uint32_t* w_et, uint32_t* w_ei) {
    if (s.kind == ScopeKind::Is || s.kind == ScopeKind::IsIn) *w_type = intern(s.etype);
    if (s.kind == ScopeKind::Eq || s.kind == ScopeKind::In || s.kind == ScopeKind::IsIn) {
      *w_et = intern(s.ent.first);
      *w_ei = intern(s.ent.second);
    }
  }

  void policy(const Policy& p, uint32_t tier) {
    uint32_t w[POL_WORDS] = {0};
    w[PW_FLAGS] = (p.forbid ? 1u : 0u) | (tier << 8);
    w[PW_KINDS] = (uint32_t)p.principal.kind | ((uint32_t)p.action.kind << 8) | ((uint32_t)p.resource.kind << 16);
    scope_words(p.principal, &w[PW_P_TYPE], &w[PW_P_ET], &w[PW_P_EI]);
    uint32_t dummy = 0;
    scope_words(p.resource, &w[PW_R_TYPE], &w[PW_R_ET], &w[PW_R_EI]);
    if (p.action.kind == ScopeKind::Eq || p.action.kind == ScopeKind::In) {
      scope_words(p.action, &dummy, &w[PW_A_ET], &w[PW_A_EI]);
    } else if (p.action.kind == ScopeKind::InSet) {
      w[PW_A_ET] = (uint32_t)p.action.ents.size();
      std::vector<uint32_t> pairs;
      for (auto& e : p.action.ents) { pairs.push_back(intern(e.first)); pairs.push_back(intern(e.second)); }
      w[PW_A_EI] = (uint32_t)I.cpool.size();
      I.cpool.insert(I.cpool.end(), pairs.begin(), pairs.end());
    } else if (p.action.kind != ScopeKind::Any) {
      throw CedarError("invalid action scope");
    }
    if (p.principal.kind == ScopeKind::Eq || p.principal.kind == ScopeKind::In || p.principal.kind == ScopeKind::IsIn)
      w[PW_FLAGS] |= uid_bloom_bit(w[PW_P_ET], w[PW_P_EI]) << 16;
    if (p.resource.kind == ScopeKind::Eq || p.resource.kind == ScopeKind::In || p.resource.kind == ScopeKind::IsIn)
      w[PW_FLAGS] |= uid_bloom_bit(w[PW_R_ET], w[PW_R_EI]) << 24;
    uint64_t am = I.amask_ok ? action_mask(p.action) : ~0ull;
    w[PW_AMASK0] = (uint32_t)am;
    w[PW_AMASK1] = (uint32_t)(am >> 32);
    code0 = (uint32_t)I.code.size();
    max_slot = 0;
    lane_off = 0;
    std::vector<uint32_t> at;
    uint32_t n_atom_words = 0;
    AttrKey key;
    if (atoms(p, at, &n_atom_words)) {
      w[PW_FLAGS] |= PF_ATOMIC;
      w[PW_SLOTS] = n_atom_words;
      I.code.insert(I.code.end(), at.begin(), at.end());
      I.n_atomic++;
      key = attr_key(at, n_atom_words);
    } else {
      for (auto& c : p.conds) {
        compile(*c.second, 0);
        emit(OP_COND, 0, 0, 0, c.first ? 0u : 1u, 0);
      }
    }
    w[PW_CODE] = code0;
    w[PW_CODE_N] = (uint32_t)I.code.size() - code0;
    if (!(w[PW_FLAGS] & PF_ATOMIC)) {
      w[PW_SLOTS] = max_slot;
      if (max_slot > NSLOT) (void)lane(3 * (max_slot - NSLOT));  // spilled registers: the lane area's end
      I.lane_need = std::max(I.lane_need, lane_off);
    }
    w[PW_LANE] = lane_off;
    I.pol.insert(I.pol.end(), w, w + POL_WORDS);
    akeys.push_back(key);
  }
  std::vector<AttrKey> akeys;  // per policy (global index)

  // Static entities (image.h "static entities"): one row per UID (a repeated UID replaces the
  // earlier entity, as in an EntityMap), attributes as constant-pool records, and per row the
  // transitive ancestors over the static parent edges (the compiled `in`-closure row, sorted)
  // and the direct parents, both as [n, (type, id) x n] lists in the constant pool.
  void statics(const std::vector<EntityIn>& ents) {
    std::unordered_map<uint64_t, uint32_t> row_of;
    std::vector<const EntityIn*> src;
    auto key = [](uint32_t t, uint32_t i) { return ((uint64_t)t << 32) | i; };
    for (const EntityIn& e : ents) {
      const uint64_t k = key(intern(e.type), intern(e.id));
      auto it = row_of.find(k);
      if (it != row_of.end()) { src[it->second] = &e; continue; }
      row_of.emplace(k, (uint32_t)src.size());
      src.push_back(&e);
    }
    const uint32_t n = (uint32_t)src.size();
    if ((uint64_t)n >= ENT_STATIC) throw CedarError("too many static entities");
    std::vector<uint64_t> uid(n);
    std::vector<std::vector<uint64_t>> par(n);
    for (uint32_t r = 0; r < n; r++) {
      uid[r] = key(intern(src[r]->type), intern(src[r]->id));
      for (auto& p : src[r]->parents) {
        const uint64_t k = key(intern(p.first), intern(p.second));
        if (std::find(par[r].begin(), par[r].end(), k) == par[r].end()) par[r].push_back(k);
      }
    }
    auto put_list = [this](const std::vector<uint64_t>& l) {
      const uint32_t off = (uint32_t)I.cpool.size();
      I.cpool.push_back((uint32_t)l.size());
      for (uint64_t x : l) { I.cpool.push_back((uint32_t)(x >> 32)); I.cpool.push_back((uint32_t)x); }
      return off;
    };
    I.srows.assign((size_t)n * ENT_WORDS, 0);
    std::vector<uint64_t> anc, stack;
    std::vector<uint32_t> mark(n, 0xFFFFFFFFu);
    for (uint32_t r = 0; r < n; r++) {
      uint32_t w0 = mk_w0(T_REC, mk_ref(SP_CPOOL, 0)), w1 = 0;
      value_words(src[r]->attrs, w0, w1);
      anc.clear();
      stack.assign(1, uid[r]);
      while (!stack.empty()) {  // closure over the static edges (cycles tolerated: as a walk)
        const uint64_t cur = stack.back();
        stack.pop_back();
        auto it = row_of.find(cur);
        if (it == row_of.end()) continue;
        for (uint64_t p : par[it->second]) {
          auto pr = row_of.find(p);
          if (pr != row_of.end()) {
            if (mark[pr->second] == r) continue;
            mark[pr->second] = r;
          } else if (std::find(anc.begin(), anc.end(), p) != anc.end()) {
            continue;
          }
          anc.push_back(p);
          stack.push_back(p);
        }
      }
      std::sort(anc.begin(), anc.end());
      uint32_t* row = &I.srows[(size_t)r * ENT_WORDS];
      row[ER_TYPE] = (uint32_t)(uid[r] >> 32);
      row[ER_ID] = (uint32_t)uid[r];
      row[ER_ATTR0] = w0;
      row[ER_ATTR1] = w1;
      row[ER_ANC] = mk_ref(SP_CPOOL, put_list(anc));
      row[ER_PAD] = put_list(par[r]);
    }
    uint32_t size = 1;
    while (size < 2 * n + 1) size <<= 1;
    I.shash.assign((size_t)size * SH_WORDS, 0);
    for (uint32_t r = 0; r < n; r++) {
      const uint32_t t = (uint32_t)(uid[r] >> 32), i = (uint32_t)uid[r];
      uint32_t h = uid_hash(t, i) & (size - 1);
      while (I.shash[(size_t)h * SH_WORDS + 2]) h = (h + 1) & (size - 1);
      I.shash[(size_t)h * SH_WORDS] = t;
      I.shash[(size_t)h * SH_WORDS + 1] = i;
      I.shash[(size_t)h * SH_WORDS + 2] = r + 1;
    }
  }
};

}  // namespace

// std::sort of v over up to `threads` threads: sorted pieces, then merged pairwise (each round's
// merges side by side). Same result as one std::sort for a strict total order.
template <class T>
static void parallel_sort(std::vector<T>& v, unsigned threads) {
  const size_t n = v.size();
  unsigned parts = 1;
  while (parts * 2 <= threads && n / (parts * 2) >= (1u << 14)) parts *= 2;
  if (parts == 1) { std::sort(v.begin(), v.end()); return; }
  std::vector<size_t> cut(parts + 1);
  for (unsigned k = 0; k <= parts; k++) cut[k] = n * k / parts;
  {
    std::vector<std::thread> ts;
    for (unsigned k = 1; k < parts; k++) ts.emplace_back([&, k] { std::sort(v.begin() + (long)cut[k], v.begin() + (long)cut[k + 1]); });
    std::sort(v.begin(), v.begin() + (long)cut[1]);
    for (auto& t : ts) t.join();
  }
  std::vector<T> buf(n);
  std::vector<T>* src = &v;
  std::vector<T>* dst = &buf;
  for (unsigned w = 1; w < parts; w *= 2) {
    std::vector<std::thread> ts;
    for (unsigned k = 0; k < parts; k += 2 * w) {
      const size_t a = cut[k], m = cut[std::min(parts, k + w)], e = cut[std::min(parts, k + 2 * w)];
      ts.emplace_back([=] { std::merge(src->begin() + (long)a, src->begin() + (long)m, src->begin() + (long)m, src->begin() + (long)e, dst->begin() + (long)a); });
    }
    for (auto& t : ts) t.join();
    std::swap(src, dst);
  }
  if (src != &v) v.swap(*src);
}

// fn(i) for i in [0, n) on up to 16 threads (chunks of 4,096)
static void parallel_range(size_t n, const std::function<void(size_t)>& fn) {
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t chunk = 4096;
  const unsigned nt = (unsigned)std::min<size_t>(hw, (n + chunk - 1) / chunk);
  if (nt <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t b; (b = next.fetch_add(chunk)) < n;)
      for (size_t i = b; i < std::min(n, b + chunk); i++) fn(i);
  };
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

// fn(k) for each of n coarse tasks on up to 16 threads (one task at a time; fn must not throw)
static void parallel_tasks(size_t n, const std::function<void(size_t)>& fn) {
  const unsigned nt = (unsigned)std::min<size_t>(std::max(1u, std::min(16u, std::thread::hardware_concurrency())), n);
  if (nt <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t k; (k = next.fetch_add(1)) < n;) fn(k);
  };
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

// v = n zero words, zeroed on several threads (1 MB pieces: the pages fault in side by side)
static void zeroed(RawWords& v, size_t n) {
  v.clear();
  v.resize(n);
  const size_t piece = 1u << 18;
  parallel_tasks((n + piece - 1) / piece, [&](size_t k) {
    std::fill(v.begin() + (long)(k * piece), v.begin() + (long)std::min(n, (k + 1) * piece), 0u);
  });
}

// Scope index (image.h "scope index"): file each policy of an all-atomic image under the key set
// with the fewest competing policies (a level-1 scope key, refined by the policy's attribute key
// when it has one), then lay out fixed record heads bucket by bucket and the full records in the
// ext area.
template <class AK>
static void build_scope_index(Image& img, const std::vector<AK>& akeys_in) {
  using L1 = std::array<uint32_t, 7>;                   // (combo, pt, pi, at, ai, rt, ri)
  using L2 = std::pair<L1, std::array<uint32_t, 3>>;    // (+ h, v0, v1)
  const uint32_t n = img.n_pol();
  img.btab.clear(); img.bfilt.clear(); img.bstream.clear();
  img.key_ents.clear();
  img.sctx.assign(2 * SCTX_WORDS, 0); img.sbits.assign(2, 0); img.svals.assign(SVAL_WORDS, 0); img.sbits_words = 0; img.sbloom.assign(2 * ctx_bloom_words(2), 0);
  img.combo_mask = 0;
  img.pslot_mask = 0;
  img.pfx.assign((size_t)img.n_hot() * PFX_LENS, 0);
  // prefix keys (image.h "prefix level-2 keys"): per slot the PFX_LENS most used prefix lengths;
  // a policy whose length is not among them, or whose slot a contains atom reads, stays unkeyed
  std::vector<AK> akeys = akeys_in;
  {
    static const bool off = std::getenv("CEDARGPU_NO_PREFIX_KEYS") != nullptr;  // A/B studies
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> uses;  // (slot, length) -> policies
    for (auto& k : akeys)
      if (k.ok && k.plen) {
        if (off || ((img.cslot_mask >> k.h) & 1)) k.ok = false;
        else uses[{k.h, k.plen}]++;
      }
    for (uint32_t h = 0; h < img.n_hot(); h++) {
      std::vector<std::pair<uint32_t, uint32_t>> ls;  // (-uses, length)
      for (auto it = uses.lower_bound({h, 0}); it != uses.end() && it->first.first == h; ++it)
        ls.emplace_back(0u - it->second, it->first.second);
      std::sort(ls.begin(), ls.end());
      for (size_t j = 0; j < ls.size() && j < PFX_LENS; j++) img.pfx[(size_t)h * PFX_LENS + j] = ls[j].second;
    }
    for (auto& k : akeys)
      if (k.ok && k.plen) {
        const uint32_t* l = &img.pfx[(size_t)k.h * PFX_LENS];
        if (std::find(l, l + PFX_LENS, k.plen) == l + PFX_LENS) k.ok = false;
        else img.pslot_mask |= 1u << k.h;
      }
  }
  img.indexed = (n > 0 && img.n_atomic == n) ? 1u : 0u;
  if (!img.indexed) {
    img.btab.assign(BT_WORDS, 0); img.bfilt.assign(2, 0); img.bstream.assign(HEAD_WORDS, 0);
    img.btab_slots = 2;
    img.sctx.assign(2 * SCTX_WORDS, 0); img.sbits.assign(2, 0); img.svals.assign(SVAL_WORDS, 0); img.sbits_words = 0; img.sbloom.assign(2 * ctx_bloom_words(2), 0);
    return;
  }
  static const bool times = std::getenv("CEDARGPU_COMPILE_TIMES") != nullptr;
  auto t_mark = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!times) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  index %-14s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t_mark).count());
    t_mark = now;
  };
  // stream record offset / length of every policy
  std::vector<uint32_t> rec_off(n), rec_len(n);
  for (size_t ch = 0; ch < img.chunks.size(); ch += 4) {
    uint32_t off = img.chunks[ch];
    for (uint32_t p = img.chunks[ch + 2]; p < img.chunks[ch + 3]; p++) {
      const uint32_t len = (POL_WORDS + img.pstream[off + PW_CODE_N] + 3) & ~3u;
      rec_off[p] = off; rec_len[p] = len;
      off += len;
    }
  }
  // most specific level-1 keys of every policy: its scope's own entity / type / wildcard
  // filings as flat (key, policy) records, sorted: each key's policies stay in policy order, and
  // buckets are laid out in key order
  // duplicate classes: policies whose records agree word for word (the global index aside, an
  // action list by content) decide alike for every request; only the lowest-index member is filed,
  // and its head lists the class (head word PW_CODE_N: bstream offset of [n, member indices...]),
  // so the probe kernel evaluates the class once and records every member
  // (key: the record with PW_CODE and an action list's offset zeroed, then that list's pairs;
  // hashed on worker threads, classes found among equal hashes)
  std::vector<uint32_t> rep(n), mcnt(n, 0), moff(n + 1, 0), mflat(n);
  {
    static const bool off = std::getenv("CEDARGPU_NO_CLASSES") != nullptr;  // A/B studies
    auto inset = [&](uint32_t q) { return ((img.pol[(size_t)q * POL_WORDS + PW_KINDS] >> 8) & 0xFF) == SK_INSET; };
    auto klen = [&](uint32_t q) { return rec_len[q] + (inset(q) ? 2 * img.pol[(size_t)q * POL_WORDS + PW_A_ET] : 0u); };
    auto kword = [&](uint32_t q, uint32_t j) -> uint32_t {
      if (j < rec_len[q]) return (j == PW_CODE || (j == PW_A_EI && inset(q))) ? 0u : img.pstream[rec_off[q] + j];
      return img.cpool[img.pol[(size_t)q * POL_WORDS + PW_A_EI] + (j - rec_len[q])];
    };
    std::vector<std::pair<uint64_t, uint32_t>> hq(n);
    parallel_range(off ? 0 : n, [&](size_t q) {
      uint64_t h = 1469598103934665603ull;
      const uint32_t L = klen((uint32_t)q);
      for (uint32_t j = 0; j < L; j++) h = (h ^ kword((uint32_t)q, j)) * 1099511628211ull;
      hq[q] = {h, (uint32_t)q};
    });
    for (uint32_t q = 0; q < n; q++) rep[q] = q;
    if (!off) {
      parallel_sort(hq, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
      auto same = [&](uint32_t x, uint32_t y) {
        const uint32_t L = klen(x);
        if (klen(y) != L) return false;
        for (uint32_t j = 0; j < L; j++)
          if (kword(x, j) != kword(y, j)) return false;
        return true;
      };
      std::vector<uint32_t> reps;  // distinct keys of one hash run, lowest member first
      for (size_t i = 0; i < n;) {
        size_t j = i;
        while (j < n && hq[j].first == hq[i].first) j++;
        reps.clear();
        for (size_t k = i; k < j; k++) {  // ascending policy index within the run
          const uint32_t q = hq[k].second;
          for (uint32_t r : reps)
            if (same(r, q)) { rep[q] = r; break; }
          if (rep[q] == q) reps.push_back(q);
        }
        i = j;
      }
    }
    for (uint32_t q = 0; q < n; q++) mcnt[rep[q]]++;
    for (uint32_t q = 0; q < n; q++) moff[q + 1] = moff[q] + mcnt[q];
    std::vector<uint32_t> fill(moff.begin(), moff.end() - 1);
    for (uint32_t q = 0; q < n; q++) mflat[fill[rep[q]]++] = q;  // ascending per class
  }
  img.cls_off.clear();
  img.cls_mem.clear();
  if (std::any_of(mcnt.begin(), mcnt.end(), [](uint32_t c) { return c > 1; })) {
    img.cls_off = moff;
    img.cls_mem = mflat;
  }
  mark("classes");
  constexpr uint32_t NO_POLICY = 0xFFFFFFFFu;  // a level-1 entry that only carries level-2 keys
  std::vector<std::pair<L1, uint32_t>> r1;
  std::vector<std::pair<L2, uint32_t>> r2;
  std::vector<uint64_t> kents;  // entity components of the level-1 keys
  // filed in blocks of policies side by side, the blocks' records then concatenated in order
  // (the same records in the same order as one walk)
  struct Filed {
    std::vector<std::pair<L1, uint32_t>> r1;
    std::vector<std::pair<L2, uint32_t>> r2;
    std::vector<uint64_t> kents;
    uint32_t combo_mask = 0, cslot_mask = 0;
    bool too_large = false;
  };
  const uint32_t fblk = 2048;
  std::vector<Filed> filed((n + fblk - 1) / fblk);
  parallel_tasks(filed.size(), [&](size_t b) {
    Filed& F = filed[b];
    auto& r1 = F.r1;
    auto& r2 = F.r2;
    auto& kents = F.kents;
    std::vector<std::pair<uint32_t, uint32_t>> acts;  // a policy's action components
    for (uint32_t p = (uint32_t)b * fblk; p < std::min<uint32_t>(n, (uint32_t)(b + 1) * fblk); p++) {
      if (rep[p] != p) continue;  // filed through its class representative
      const uint32_t* d = &img.pol[(size_t)p * POL_WORDS];
      const uint32_t pk = d[PW_KINDS] & 0xFF, ak = (d[PW_KINDS] >> 8) & 0xFF, rk = (d[PW_KINDS] >> 16) & 0xFF;
      auto comp = [](uint32_t kind, uint32_t ty, uint32_t et, uint32_t ei, uint32_t& kc, uint32_t& t, uint32_t& i) {
        if (kind == SK_EQ || kind == SK_IN || kind == SK_ISIN) { kc = KC_ENT; t = et; i = ei; }
        else if (kind == SK_IS) { kc = KC_TYPE; t = ty; i = KW_ANY; }
        else { kc = KC_WILD; t = KW_ANY; i = KW_ANY; }
      };
      uint32_t pkc, pt, pi, rkc, rt, ri;
      comp(pk, d[PW_P_TYPE], d[PW_P_ET], d[PW_P_EI], pkc, pt, pi);
      comp(rk, d[PW_R_TYPE], d[PW_R_ET], d[PW_R_EI], rkc, rt, ri);
      acts.clear();
      uint32_t akc = KC_ENT;
      if (ak == SK_EQ || ak == SK_IN) acts.emplace_back(d[PW_A_ET], d[PW_A_EI]);
      else if (ak == SK_INSET) {
        for (uint32_t k = 0; k < d[PW_A_ET]; k++) acts.emplace_back(img.cpool[d[PW_A_EI] + 2 * k], img.cpool[d[PW_A_EI] + 2 * k + 1]);
        std::sort(acts.begin(), acts.end());
        acts.erase(std::unique(acts.begin(), acts.end()), acts.end());  // empty: `action in []` never applies
      } else {
        akc = KC_WILD;
        acts.emplace_back(KW_ANY, KW_ANY);
      }
      const uint32_t combo = key_combo(pkc, akc, rkc);
      if (pkc == KC_ENT) kents.push_back(((uint64_t)pt << 32) | pi);
      if (rkc == KC_ENT) kents.push_back(((uint64_t)rt << 32) | ri);
      for (auto& a : acts) {
        if (akc == KC_ENT) kents.push_back(((uint64_t)a.first << 32) | a.second);
        const L1 k{combo, pt, pi, a.first, a.second, rt, ri};
        if ((pt != KW_ANY && pt >= (1u << 28)) || (rt != KW_ANY && rt >= (1u << 28))) { F.too_large = true; return; }
        F.combo_mask |= 1u << combo;
        if (!akeys[p].ok) { r1.emplace_back(k, p); continue; }
        r1.emplace_back(k, NO_POLICY);  // the level-1 entry carries the hmask even without unkeyed policies
        const uint32_t hk = akeys[p].h | (akeys[p].contains ? BT_CKEY : 0u);
        r2.emplace_back(L2(k, {hk, akeys[p].v0, akeys[p].v1}), p);
        if (!akeys[p].guarded) r2.emplace_back(L2(k, {hk, MISSING_W0, 0u}), p);
        if (akeys[p].contains) {
          r2.emplace_back(L2(k, {hk, NOTSET_W0, 0u}), p);  // contains on a non-set (like on a non-string) raises
          if (!akeys[p].plen) F.cslot_mask |= 1u << akeys[p].h;
        }
      }
    }
  });
  {
    size_t n1 = 0, n2 = 0, nk = 0;
    std::vector<std::array<size_t, 3>> at(filed.size());
    for (size_t b = 0; b < filed.size(); b++) {
      const Filed& F = filed[b];
      if (F.too_large) throw CedarError("string table too large for the scope index");
      img.combo_mask |= F.combo_mask;
      img.cslot_mask |= F.cslot_mask;
      at[b] = {n1, n2, nk};
      n1 += F.r1.size(); n2 += F.r2.size(); nk += F.kents.size();
    }
    r1.resize(n1); r2.resize(n2); kents.resize(nk);
    parallel_tasks(filed.size(), [&](size_t b) {
      Filed& F = filed[b];
      std::copy(F.r1.begin(), F.r1.end(), r1.begin() + (long)at[b][0]);
      std::copy(F.r2.begin(), F.r2.end(), r2.begin() + (long)at[b][1]);
      std::copy(F.kents.begin(), F.kents.end(), kents.begin() + (long)at[b][2]);
      F = Filed();
    });
  }
  if (times) std::fprintf(stderr, "  index filings: r1 %zu r2 %zu kents %zu\n", r1.size(), r2.size(), kents.size());
  mark("filings");
  // Records ordered by (level-1 key hash, level-1 key[, level-2 part], policy): equal keys side by
  // side in policy order, and r1 / r2 in the same level-1 order (merged below). The hash decides
  // almost every comparison, so index records sort instead of the wide ones, on three threads.
  auto l1_hash = [](const L1& k) { return key_hash(k[0], k[1], k[2], k[3], k[4], k[5], k[6]); };
  auto l1_less = [&](const L1& a, uint32_t ha, const L1& b, uint32_t hb) { return ha != hb ? ha < hb : a < b; };
  {
    // 64-bit sort keys: r1 (hash, policy), r2 (hash, level-2 hash) then policy; a run of equal
    // hashes over different keys (a collision) is put in key order afterwards
    auto x_hash = [](const std::array<uint32_t, 3>& x) { return key_hash(x[0], x[1], x[2], 0, 0, 0, 0); };
    struct K1 { uint64_t k; uint32_t i; bool operator<(const K1& o) const { return k != o.k ? k < o.k : i < o.i; } };
    struct K2 { uint64_t k; uint32_t p, i; bool operator<(const K2& o) const { return k != o.k ? k < o.k : (p != o.p ? p < o.p : i < o.i); } };
    std::vector<K1> i1(r1.size());
    std::vector<K2> i2(r2.size());
    std::vector<uint32_t> h1s(r1.size()), h2s(r2.size());  // level-1 hash by record
    parallel_range(r1.size(), [&](size_t i) { h1s[i] = l1_hash(r1[i].first); i1[i] = {((uint64_t)h1s[i] << 32) | r1[i].second, (uint32_t)i}; });
    parallel_range(r2.size(), [&](size_t i) {
      h2s[i] = l1_hash(r2[i].first.first);
      i2[i] = {((uint64_t)h2s[i] << 32) | x_hash(r2[i].first.second), r2[i].second, (uint32_t)i};
    });
    mark("sort keys");
    // (the longest of the three, i2, on half the threads)
    const unsigned hw = std::max(2u, std::min(16u, std::thread::hardware_concurrency()));
    std::thread t1([&] { parallel_sort(i1, hw / 4); });
    std::thread t2([&] { parallel_sort(kents, hw / 4); });
    parallel_sort(i2, hw / 2);
    t1.join();
    t2.join();
    mark("sort core");
    // gathered in hash order, then each run of equal hashes checked (in order, cache-friendly)
    std::vector<std::pair<L1, uint32_t>> s1(r1.size());
    std::vector<std::pair<L2, uint32_t>> s2(r2.size());
    std::vector<uint64_t> k2(r2.size());
    parallel_range(r1.size(), [&](size_t i) { s1[i] = r1[i1[i].i]; });
    parallel_range(r2.size(), [&](size_t i) { s2[i] = r2[i2[i].i]; k2[i] = i2[i].k; });
    for (size_t b0 = 0; b0 < s1.size();) {  // collisions of the level-1 hash
      size_t e = b0 + 1;
      bool mixed = false;
      while (e < s1.size() && (i1[e].k >> 32) == (i1[b0].k >> 32)) mixed |= s1[e++].first != s1[b0].first;
      if (mixed) std::stable_sort(s1.begin() + (long)b0, s1.begin() + (long)e);
      b0 = e;
    }
    for (size_t b0 = 0; b0 < s2.size();) {
      size_t e = b0 + 1;
      bool mixed = false;
      while (e < s2.size() && (k2[e] >> 32) == (k2[b0] >> 32)) {
        mixed |= s2[e].first.first != s2[b0].first.first;
        e++;
      }
      for (size_t c = b0; !mixed && c < e;) {  // equal level-1 keys: level-2 hash collisions
        size_t f = c + 1;
        while (f < e && k2[f] == k2[c]) mixed |= s2[f++].first.second != s2[c].first.second;
        c = f;
      }
      if (mixed) std::stable_sort(s2.begin() + (long)b0, s2.begin() + (long)e);
      b0 = e;
    }
    r1.swap(s1);
    r2.swap(s2);
  }
  r2.erase(std::unique(r2.begin(), r2.end()), r2.end());
  mark("sort");
  kents.erase(std::unique(kents.begin(), kents.end()), kents.end());
  img.key_ents = std::move(kents);
  // groups: [begin, end) ranges of one key; level-1 hmask from the level-2 keys under it
  struct G { size_t b, e; uint32_t hmask = 0, cmask = 0; uint32_t bloom[4] = {0, 0, 0, 0}; };
  std::vector<G> g1, g2;
  // group starts flagged side by side, collected in order
  auto group = [&](const auto& r, std::vector<G>& out) {
    const size_t n = r.size();
    std::vector<uint8_t> st(n);
    parallel_range(n, [&](size_t i) { st[i] = i == 0 || !(r[i].first == r[i - 1].first); });
    for (size_t i = 0; i < n; i++)
      if (st[i]) {
        if (!out.empty()) out.back().e = i;
        out.push_back({i, n});
      }
  };
  group(r1, g1);
  group(r2, g2);
  // each level-2 group's level-1 group by binary search over (hash, key) (both lists in that
  // order), its bits OR-ed in atomically: groups side by side, the same masks as in order
  std::vector<uint32_t> h1g(g1.size());
  parallel_range(g1.size(), [&](size_t k) { h1g[k] = l1_hash(r1[g1[k].b].first); });
  parallel_range(g2.size(), [&](size_t a) {
    const L1& key = r2[g2[a].b].first.first;
    const uint32_t hk = l1_hash(key);
    size_t lo = 0, hi = g1.size();
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      if (l1_less(r1[g1[mid].b].first, h1g[mid], key, hk)) lo = mid + 1;
      else hi = mid;
    }
    const size_t k = lo;
    if (k < g1.size() && r1[g1[k].b].first == key) {
      const auto& x = r2[g2[a].b].first.second;
      if (x[0] & BT_CKEY) __atomic_fetch_or(&g1[k].cmask, 1u << (x[0] & ~BT_CKEY), __ATOMIC_RELAXED);
      else __atomic_fetch_or(&g1[k].hmask, 1u << x[0], __ATOMIC_RELAXED);
      const uint32_t bits = l2_bloom_bits(bucket_hash2(key_hash(key[0], key[1], key[2], key[3], key[4], key[5], key[6]), x[0], x[1], x[2]));
      for (uint32_t j = 0; j < 3; j++) {
        const uint32_t bb = (bits >> (7 * j)) & 127u;
        __atomic_fetch_or(&g1[k].bloom[bb >> 5], 1u << (bb & 31), __ATOMIC_RELAXED);
      }
    }
  });
  mark("buckets");
  // scope bitsets (image.h "scope bitsets"): a row per context of the keys whose principal
  // component is an entity, a bit per key entity: level-1 keys that file policies directly, and
  // every level-2 key. The bits' buckets (svals) are known once the heads are laid out, below.
  // Contexts get their rows in first-seen order (level-1 groups, then level-2), walked in key
  // order below. Keys, hashes and key-entity indices are computed side by side; the rows are then
  // assigned in order through one open-addressing table (290k lookups into a std::map were 87 ms
  // of a 100k-policy build).
  using CtxKey = std::array<uint32_t, 8>;
  auto ctx_hash = [](const CtxKey& a) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint32_t w : a) h = (h ^ w) * 0xBF58476D1CE4E5B9ull, h ^= h >> 29;
    return h;
  };
  std::vector<std::pair<CtxKey, uint32_t>> ctx;  // (key, row) in row order
  struct SBit { uint32_t row, kidx, grp; };  // grp: g1 index, or g2 index | SB_L2
  constexpr uint32_t SB_L2 = 0x80000000u;
  std::vector<SBit> sbit;
  {
    auto kidx = [&](uint32_t t, uint32_t i) {
      const uint64_t u = ((uint64_t)t << 32) | i;
      return (uint32_t)(std::lower_bound(img.key_ents.begin(), img.key_ents.end(), u) - img.key_ents.begin());
    };
    img.l2_vmask = img.l2_lmask = 0;
    // candidates: the level-1 groups that file policies directly, then every level-2 group, of
    // entity-principal combos
    struct Cand { CtxKey key; uint64_t h; uint32_t kidx, grp; };
    std::vector<uint32_t> c1;
    for (size_t gi = 0; gi < g1.size(); gi++) {
      const G& g = g1[gi];
      const L1& k = r1[g.b].first;
      if ((k[0] & 3) != KC_ENT) continue;
      img.l2_vmask |= g.hmask;
      img.l2_lmask |= g.cmask;
      bool direct = false;
      for (size_t i = g.b; i < g.e && !direct; i++) direct = r1[i].second != NO_POLICY;
      if (direct) c1.push_back((uint32_t)gi);
    }
    std::vector<uint32_t> c2;
    c2.reserve(g2.size());
    for (size_t gi = 0; gi < g2.size(); gi++)
      if ((r2[g2[gi].b].first.first[0] & 3) == KC_ENT) c2.push_back((uint32_t)gi);
    std::vector<Cand> cand(c1.size() + c2.size());
    parallel_range(cand.size(), [&](size_t c) {
      Cand& o = cand[c];
      if (c < c1.size()) {
        const L1& k = r1[g1[c1[c]].b].first;
        o.key = CtxKey{k[0], k[3], k[4], k[5], k[6], SCTX_L1, 0u, 0u};
        o.kidx = kidx(k[1], k[2]);
        o.grp = c1[c];
      } else {
        const uint32_t gi = c2[c - c1.size()];
        const L1& k = r2[g2[gi].b].first.first;
        const auto& x = r2[g2[gi].b].first.second;
        o.key = CtxKey{k[0], k[3], k[4], k[5], k[6], x[0], x[1], x[2]};
        o.kidx = kidx(k[1], k[2]);
        o.grp = gi | SB_L2;
      }
      o.h = ctx_hash(o.key);
    });
    size_t slots = 16;
    while (slots < 2 * cand.size()) slots <<= 1;
    std::vector<uint32_t> table(slots, 0);  // row + 1
    sbit.reserve(cand.size());
    for (const Cand& o : cand) {
      size_t h = (size_t)o.h & (slots - 1);
      while (table[h] && ctx[table[h] - 1].first != o.key) h = (h + 1) & (slots - 1);
      if (!table[h]) {
        ctx.emplace_back(o.key, (uint32_t)ctx.size());
        table[h] = (uint32_t)ctx.size();
      }
      sbit.push_back({table[h] - 1, o.kidx, o.grp});
    }
  }
  mark("scope ctx");
  // record heads (bucket order) then the ext area (one full record per policy)
  uint32_t n_heads = 0;
  for (auto& x : r1) n_heads += x.second != NO_POLICY;
  n_heads += (uint32_t)r2.size();
  std::vector<uint32_t> ext(n), mlist(n, 0);
  uint64_t ext_end = (uint64_t)n_heads * HEAD_WORDS;
  for (uint32_t p = 0; p < n; p++) { ext[p] = (uint32_t)ext_end; ext_end += rec_len[p]; }
  for (uint32_t p = 0; p < n; p++)
    if (mcnt[p] > 1) { mlist[p] = (uint32_t)ext_end; ext_end += 1 + mcnt[p]; }
  if (ext_end >= (1ull << 32)) throw CedarError("scope index exceeds 16 GiB");
  // (the candidate pass packs a bucket's first head with its key combination: 27 bits, cedar_eval.hip EF_COMBO)
  if (n_heads >= (1u << 27)) throw CedarError("scope index exceeds 2^27 policy heads");
  zeroed(img.bstream, std::max<uint64_t>(ext_end, HEAD_WORDS));
  parallel_range(n, [&](size_t p) {
    std::copy(img.pstream.begin() + rec_off[p], img.pstream.begin() + rec_off[p] + rec_len[p], img.bstream.begin() + ext[p]);
    if (mlist[p]) {
      img.bstream[mlist[p]] = mcnt[p];
      std::copy(mflat.begin() + moff[p], mflat.begin() + moff[p + 1], img.bstream.begin() + mlist[p] + 1);  // ascending
    }
  });
  mark("ext area");
  const size_t n_entries = g1.size() + g2.size();
  // slots: the power of two >= 8x the entries while the table stays within 64 MB, and >= 2x in any
  // case. Linear-probe chains then average ~1.06 slots, so a probe needs no key filter in front
  // of it (C3 DAG: 3.72e8 decisions/s at 2x with the filter, 4.01e8 at 8-32x without it,
  // profiles/r02/ab_slack). CEDARGPU_BTAB_SLACK=k: >= k/4 x (A/B studies).
  static const size_t slack = [] { const char* e = std::getenv("CEDARGPU_BTAB_SLACK"); return e ? (size_t)std::max(4, std::atoi(e)) : 32u; }();
  uint32_t size = 16;
  while (size * 4 < 8 * n_entries) size <<= 1;
  while (size * 4 < slack * n_entries && (size_t)size * 2 * BT_WORDS * 4 <= (64u << 20)) size <<= 1;
  // the entries only: the device inserts them into `size` slots at load (cedar_btab_build)
  img.btab_slots = size;
  size_t blocks = 16;
  while (blocks * 4 < n_entries) blocks <<= 1;  // >= 16 bits per entry
  img.bfilt.assign(2 * blocks, 0);
  auto filt_add = [&](uint32_t hash) {
    const uint64_t need = filt_need(hash);
    const size_t blk = hash & (blocks - 1);
    img.bfilt[2 * blk] |= (uint32_t)need;
    img.bfilt[2 * blk + 1] |= (uint32_t)(need >> 32);
  };
  mark("tables");
  // Each group's heads sit at its first (prefix sums of its records that file a policy), in group
  // order (level-1 groups, then level-2); the groups' heads and bucket entries are then written
  // side by side, the filter after them.
  std::vector<uint32_t> g1_first(g1.size()), g1_cnt(g1.size()), g2_first(g2.size()), g2_cnt(g2.size());
  parallel_range(g1.size(), [&](size_t gi) {
    uint32_t c = 0;
    for (size_t i = g1[gi].b; i < g1[gi].e; i++) c += r1[i].second != NO_POLICY;
    g1_cnt[gi] = c;
  });
  parallel_range(g2.size(), [&](size_t gi) {
    uint32_t c = 0;
    for (size_t i = g2[gi].b; i < g2[gi].e; i++) c += r2[i].second != NO_POLICY;
    g2_cnt[gi] = c;
  });
  {
    uint32_t head = 0;
    for (size_t gi = 0; gi < g1.size(); gi++) { g1_first[gi] = head; head += g1_cnt[gi]; }
    for (size_t gi = 0; gi < g2.size(); gi++) { g2_first[gi] = head; head += g2_cnt[gi]; }
  }
  auto put_heads = [&](auto begin, auto end, uint32_t head) {
    for (auto it = begin; it != end; ++it) {
      const uint32_t p = it->second;
      if (p == NO_POLICY) continue;
      uint32_t* hd = &img.bstream[(size_t)head * HEAD_WORDS];
      const uint32_t* src = &img.pstream[rec_off[p]];
      std::copy(src, src + std::min<uint32_t>(rec_len[p], HEAD_WORDS), hd);
      hd[PW_EXT] = ext[p];
      hd[PW_CODE_N] = mlist[p];  // heads: the duplicate class's member list (0: the policy alone)
      // heads: the class size in PW_SLOTS' upper half (0xFFFF: read it from the list), so a hit
      // needs no load before its members'
      hd[PW_SLOTS] = (hd[PW_SLOTS] & 0xFFFFu) | (std::min<uint32_t>(mcnt[p], 0xFFFFu) << 16);
      head++;
    }
  };
  zeroed(img.btab, n_entries * BT_WORDS);
  std::vector<uint32_t> h2g(g2.size());  // level-2 bucket hashes (the filter's)
  parallel_range(g1.size(), [&](size_t gi) {
    const G& g = g1[gi];
    const L1& k = r1[g.b].first;
    put_heads(r1.begin() + (long)g.b, r1.begin() + (long)g.e, g1_first[gi]);
    const uint32_t e[BT_WORDS] = {BT_USED | (k[0] << 16), k[1], k[2], k[3], k[4], k[5], k[6], g.cmask, 0, g1_first[gi],
                                  g1_cnt[gi], g.hmask, g.bloom[0], g.bloom[1], g.bloom[2], g.bloom[3]};
    std::copy(e, e + BT_WORDS, img.btab.begin() + (long)(gi * BT_WORDS));
  });
  parallel_range(g2.size(), [&](size_t gi) {
    const G& g = g2[gi];
    const L1& k = r2[g.b].first.first;
    const auto& x = r2[g.b].first.second;
    put_heads(r2.begin() + (long)g.b, r2.begin() + (long)g.e, g2_first[gi]);
    h2g[gi] = bucket_hash2(l1_hash(k), x[0], x[1], x[2]);
    const uint32_t e[BT_WORDS] = {BT_USED | (k[0] << 16) | BT_L2 | x[0], k[1], k[2], k[3], k[4], k[5], k[6], x[1], x[2],
                                  g2_first[gi], g2_cnt[gi], 0, 0, 0, 0, 0};
    std::copy(e, e + BT_WORDS, img.btab.begin() + (long)((g1.size() + gi) * BT_WORDS));
  });
  for (uint32_t h : h1g) filt_add(h);
  for (uint32_t h : h2g) filt_add(h);
  if (img.btab.empty()) img.btab.assign(BT_WORDS, 0);  // never empty buffers
  // each bucket's required presence (image.h "presence masks"): the slots every policy filed in it
  // requires, a value key's bucket with the slots its policies' `has` atoms after the key atom name
  std::vector<uint32_t> g1_need(g1.size()), g2_need(g2.size()), g2_filt(g2.size());
  parallel_range(g1.size(), [&](size_t gi) {
    uint32_t m = ~0u;
    for (size_t i = g1[gi].b; i < g1[gi].e; i++)
      if (r1[i].second != NO_POLICY) m &= akeys[r1[i].second].mpre;
    g1_need[gi] = g1_cnt[gi] ? m : 0u;
  });
  parallel_range(g2.size(), [&](size_t gi) {
    const auto& x = r2[g2[gi].b].first.second;
    const bool value = x[1] != MISSING_W0 && x[1] != NOTSET_W0;
    uint32_t m = ~0u, fl = value && g2_cnt[gi] ? akeys[r2[g2[gi].b].second].filt : 0u;
    for (size_t i = g2[gi].b; i < g2[gi].e; i++) {
      m &= value ? akeys[r2[i].second].mpost : akeys[r2[i].second].mpre;
      if (akeys[r2[i].second].filt != fl) fl = 0;  // the filter only when every policy has the same one
    }
    g2_need[gi] = g2_cnt[gi] ? m : 0u;
    g2_filt[gi] = fl;
  });
  mark("heads+slots");
  // the bitset rows as (bits, rank) word pairs, every set bit's bucket at its rank, and the context
  // table (image.h "scope bitsets")
  const uint64_t words = (img.key_ents.size() + 31) / 32;
  // (a listed key carries its bit's rank in 26 bits: cedar_scan_kernel)
  if (!ctx.empty() && words && (uint64_t)ctx.size() * words * 8 <= SBITS_MAX_BYTES && sbit.size() < (1u << 26)) {
    img.sbits_words = (uint32_t)words;
    RawWords bitw;
    zeroed(bitw, (size_t)ctx.size() * words);
    for (auto& b : sbit) bitw[(size_t)b.row * words + (b.kidx >> 5)] |= 1u << (b.kidx & 31);
    zeroed(img.sbits, 2 * bitw.size());
    uint32_t rank = 0;
    for (size_t w = 0; w < bitw.size(); w++) {
      img.sbits[2 * w] = bitw[w];
      img.sbits[2 * w + 1] = rank;
      rank += (uint32_t)__builtin_popcount(bitw[w]);
    }
    img.svals.assign(SVAL_WORDS * (size_t)std::max<uint32_t>(rank, 1u), 0);
    for (auto& b : sbit) {
      const size_t w = (size_t)b.row * words + (b.kidx >> 5);
      const uint32_t r = img.sbits[2 * w + 1] + (uint32_t)__builtin_popcount(bitw[w] & ((1u << (b.kidx & 31)) - 1u));
      const bool l2 = (b.grp & SB_L2) != 0;
      const uint32_t gi = b.grp & ~SB_L2;
      uint32_t* sv = &img.svals[SVAL_WORDS * (size_t)r];
      sv[0] = l2 ? g2_first[gi] : g1_first[gi];
      sv[1] = l2 ? g2_cnt[gi] : g1_cnt[gi];
      sv[2] = l2 ? g2_need[gi] : g1_need[gi];
      sv[3] = l2 ? g2_filt[gi] : 0u;
    }
    uint32_t slots = 2;
    while (slots < 2 * ctx.size()) slots <<= 1;
    img.sctx.assign((size_t)slots * SCTX_WORDS, 0);
    std::vector<std::pair<CtxKey, uint32_t>> ctx_sorted(ctx.begin(), ctx.end());
    std::sort(ctx_sorted.begin(), ctx_sorted.end());
    for (auto& c : ctx_sorted) {
      const auto& x = c.first;
      uint32_t h = ctx_key(key_pre(x[0], x[1], x[2], x[3], x[4]), x[5], x[6], x[7]) & (slots - 1);
      while (img.sctx[(size_t)h * SCTX_WORDS]) h = (h + 1) & (slots - 1);
      uint32_t* e = &img.sctx[(size_t)h * SCTX_WORDS];
      e[0] = ctx_w0(x[0], x[5]);
      e[1] = x[1]; e[2] = x[2]; e[3] = x[3]; e[4] = x[4]; e[5] = x[6]; e[6] = x[7];
      e[7] = c.second;
    }
    // the context filter: every context's key (the kernel's lookup hash)
    const uint32_t bw = ctx_bloom_words(slots);
    img.sbloom.assign(2 * (size_t)bw, 0);
    for (auto& c : ctx) {
      const auto& x = c.first;
      const uint32_t hash = ctx_key(key_pre(x[0], x[1], x[2], x[3], x[4]), x[5], x[6], x[7]);
      const uint32_t w = ctx_bloom_at(hash, bw);
      const uint64_t b = ctx_bloom_bits(hash);
      img.sbloom[2 * (size_t)w] |= (uint32_t)b;
      img.sbloom[2 * (size_t)w + 1] |= (uint32_t)(b >> 32);
    }
  }
  if (times) {
    size_t masked = 0, filtered = 0;
    for (size_t r = 0; r + SVAL_WORDS <= img.svals.size(); r += SVAL_WORDS) {
      masked += img.svals[r + 2] != 0;
      filtered += img.svals[r + 3] != 0;
    }
    std::fprintf(stderr, "  scope bitsets: %zu contexts x %llu words (%zu key entities, %zu set bits, %zu with a presence mask, "
                 "%zu with an equality filter): %.1f MB%s\n",
                 ctx.size(), (unsigned long long)words, img.key_ents.size(), sbit.size(), masked, filtered, ctx.size() * words * 8 / 1e6,
                 img.sbits_words ? "" : " (over the cap: none)");
  }
  mark("bitsets");
}

// Parses every document of the tiers, through the cache when one is given (unseen documents on
// worker threads).
static std::vector<std::shared_ptr<const std::vector<Policy>>> parse_documents(
    const std::vector<std::vector<DocSpec>>& tiers, ParseCache* cache, std::vector<DocError>* skipped) {
  std::vector<const DocSpec*> docs;
  for (auto& t : tiers)
    for (auto& d : t) docs.push_back(&d);
  std::vector<std::shared_ptr<const std::vector<Policy>>> out(docs.size());
  auto key = [](const DocSpec& d) {
    return std::hash<std::string>()(d.filename) * 0x9E3779B97F4A7C15ull ^ std::hash<std::string>()(d.text);
  };
  std::vector<size_t> todo;
  if (cache) {
    cache->generation++;
    cache->hits = cache->misses = 0;
    for (size_t i = 0; i < docs.size(); i++) {
      auto it = cache->map.find(key(*docs[i]));
      if (it != cache->map.end())
        for (auto& e : it->second)
          if (e.filename == docs[i]->filename && e.text == docs[i]->text) {
            out[i] = e.policies;
            e.used = cache->generation;
            break;
          }
      if (out[i]) cache->hits++;
      else { cache->misses++; todo.push_back(i); }
    }
  } else {
    for (size_t i = 0; i < docs.size(); i++) todo.push_back(i);
  }
  // parse the rest; the first syntax error (in document order) is the one reported
  std::vector<std::string> errs(docs.size());
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = (unsigned)std::min<size_t>(hw, todo.size() / 8 + 1);
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t k; (k = next++) < todo.size();) {
      const size_t i = todo[k];
      try {
        out[i] = std::make_shared<const std::vector<Policy>>(parse_policies(docs[i]->text, docs[i]->filename));
      } catch (const CedarError& e) {
        errs[i] = e.what();
      }
    }
  };
  if (nt <= 1) {
    work();
  } else {
    std::vector<std::thread> ws;
    for (unsigned t = 0; t < nt; t++) ws.emplace_back(work);
    for (auto& w : ws) w.join();
  }
  // a document that does not parse fails the build, unless its store skips such documents: then
  // it contributes no policies and is reported (the first error, in document order, either way)
  static const auto empty = std::make_shared<const std::vector<Policy>>();
  for (size_t i = 0; i < docs.size(); i++) {
    if (errs[i].empty()) continue;
    if (!docs[i]->skip_invalid) throw CedarError(errs[i]);
    if (skipped) skipped->push_back({docs[i]->filename, errs[i]});
    out[i] = empty;
  }
  if (cache) {
    for (size_t i : todo)
      if (errs[i].empty()) cache->map[key(*docs[i])].push_back({docs[i]->filename, docs[i]->text, out[i], cache->generation});
    for (auto it = cache->map.begin(); it != cache->map.end();) {  // drop what this build did not use
      auto& v = it->second;
      v.erase(std::remove_if(v.begin(), v.end(), [&](const ParseCache::Entry& e) { return e.used != cache->generation; }), v.end());
      it = v.empty() ? cache->map.erase(it) : std::next(it);
    }
  }
  return out;
}

// Incremental lowering state (engine.h LowerState): the persistent arenas a full build leaves, the
// compiler's image-wide choices over them, and every document's lowered policies (descriptor with
// the tier bits clear, index key, hot-path uses).
struct LowerState {
  Image arena;  // strings, sid, code, cpool, ext_msgs, act, hot, amask_ok
  Compiler C{arena};
  struct Pol {
    std::array<uint32_t, POL_WORDS> w{};
    Compiler::AttrKey key;
    std::vector<std::pair<Compiler::Path, uint32_t>> uses;  // hot-path candidates it reads
  };
  struct Doc {
    std::shared_ptr<const std::vector<Policy>> keep;  // holds the address the map is keyed by
    std::vector<Pol> pols;
    std::map<Compiler::Path, uint32_t> sum;  // uses over all its policies
    size_t words = 0;                        // arena code + cpool words its lowering appended
    uint64_t used = 0;
  };
  std::unordered_map<const void*, Doc> docs;
  std::vector<uint32_t> srows, shash;  // the static entities as the last full build lowered them
  uint64_t statics_gen = 0, gen = 0;
  size_t base_words = 0, full_strings = 0;  // arena words owned by no document; strings then
  bool valid = false;
  void reset() {  // before a full build (gen carries on)
    arena = Image();
    C.hot.clear(); C.hot_depth.clear(); C.act_index.clear(); C.akeys.clear();
    docs.clear(); srows.clear(); shash.clear();
    statics_gen = 0; base_words = full_strings = 0;
    valid = false;
  }
};
void LowerDeleter::operator()(LowerState* s) const { delete s; }
std::unique_ptr<LowerState, LowerDeleter> make_lower_state() { return std::unique_ptr<LowerState, LowerDeleter>(new LowerState()); }

namespace {
// PolicySet.Add semantics: a repeated ID replaces the earlier policy in place. The tiers refer to
// the parsed ASTs (owned by the parse results / the cache); only ID and position are per use.
struct PRef {
  const Policy* p;
  std::string id;
  const std::string* filename;  // empty for zero-position documents
  Position pos;
  uint32_t doc, idx;  // parsed document (tier order) and the policy's index in it
};
const std::string k_empty_name;

// the NHOT most used paths (ties: path order) -> slot
std::map<Compiler::Path, uint32_t> hot_slots(const std::map<Compiler::Path, uint32_t>& cnt) {
  std::vector<std::pair<uint32_t, const Compiler::Path*>> order;
  for (auto& kv : cnt) order.emplace_back(kv.second, &kv.first);
  std::sort(order.begin(), order.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : *a.second < *b.second; });
  std::map<Compiler::Path, uint32_t> out;
  for (size_t k = 0; k < order.size() && k < NHOT; k++) out.emplace(*order[k].second, (uint32_t)k);
  return out;
}
}  // namespace

// The image's policy stream, scope index, static entities and string table from its lowered
// policies (shared by the full and the incremental build).
template <class AK>
static void finish_image(Image& img, const std::vector<AK>& akeys, const std::function<void()>& statics,
                         const std::function<void(const char*)>& mark) {
  // device policy stream + chunk table: the layout (record offsets, chunks) in order, then the
  // records written side by side (padding words stay zero)
  {
    const uint32_t np = img.n_pol();
    std::vector<size_t> at(np);
    size_t size = 0;
    uint32_t p = 0;
    for (uint32_t t = 0; t < img.n_tiers(); t++) {
      uint32_t pend = img.tier_end[t];
      uint32_t c_off = (uint32_t)size, c_p0 = p;
      auto close = [&](uint32_t flag) {
        uint32_t nw = (uint32_t)size - c_off;
        if (p > c_p0) {
          img.chunks.push_back(c_off); img.chunks.push_back(nw | flag);
          img.chunks.push_back(c_p0); img.chunks.push_back(p);
        }
        c_off = (uint32_t)size;
        c_p0 = p;
      };
      for (; p < pend;) {
        uint32_t rec = (POL_WORDS + img.pol[(size_t)p * POL_WORDS + PW_CODE_N] + 3) & ~3u;
        // a record larger than an LDS chunk gets a chunk of its own, read in place (CHUNK_GLOBAL)
        const bool big = rec > CHUNK_WORDS;
        if (big || (uint32_t)size - c_off + rec > CHUNK_WORDS) close(0);
        at[p] = size;
        size += rec;
        p++;
        if (big) close(CHUNK_GLOBAL);
      }
      close(0);
      img.tier_cend.push_back((uint32_t)img.chunks.size() / 4);
    }
    zeroed(img.pstream, std::max<size_t>(size, 4));
    parallel_range(np, [&](size_t q) {
      const uint32_t* d = &img.pol[q * POL_WORDS];
      uint32_t* o = &img.pstream[at[q]];
      std::copy(d, d + POL_WORDS, o);
      o[PW_CODE] = (uint32_t)q;
      std::copy(img.code.begin() + d[PW_CODE], img.code.begin() + d[PW_CODE] + d[PW_CODE_N], o + POL_WORDS);
    });
  }
  mark("stream");
  build_scope_index(img, akeys);
  mark("scope index");
  statics();
  if (img.shash.empty()) img.shash.assign(SH_WORDS, 0);  // never empty buffers
  mark("static entities");
  // global string table
  img.gstr_off.clear();
  img.gstr_bytes.clear();
  for (auto& s : img.strings) {
    img.gstr_off.push_back((uint32_t)img.gstr_bytes.size());
    img.gstr_bytes.insert(img.gstr_bytes.end(), s.begin(), s.end());
  }
  img.gstr_off.push_back((uint32_t)img.gstr_bytes.size());
  if (img.code.empty()) img.code.push_back(0), img.code.push_back(0);  // never empty buffers
  if (img.cpool.empty()) img.cpool.push_back(0);
  if (img.gstr_bytes.empty()) img.gstr_bytes.push_back(0);
  img.build_lookup();
  mark("strings");
}

// The incremental build (engine.h LowerState): null when the cached lowering cannot serve this
// build (`why` says why), which then runs in full.
static std::shared_ptr<Image> compile_incremental(LowerState& S, const std::vector<std::shared_ptr<const std::vector<Policy>>>& docs,
                                                  const std::vector<std::vector<PRef>>& parsed, uint64_t epoch,
                                                  BuildInfo* info, const char** why, const std::function<void(const char*)>& mark) {
  Compiler& C = S.C;
  Image& A = S.arena;
  S.gen++;
  const size_t nd = docs.size();
  std::vector<LowerState::Doc*> dref(nd, nullptr);
  std::vector<uint32_t> fresh;  // documents to lower
  for (size_t d = 0; d < nd; d++) {
    auto it = S.docs.find(docs[d].get());
    if (it != S.docs.end() && it->second.keep == docs[d]) dref[d] = &it->second;
    else fresh.push_back((uint32_t)d);
  }
  // hot-path uses of the new documents (interned into the arena) and the image-wide totals over
  // the policies that stay (a repeated ID drops the earlier policy)
  std::vector<LowerState::Doc> lowered(fresh.size());
  for (size_t f = 0; f < fresh.size(); f++) {
    const auto& ps = *docs[fresh[f]];
    lowered[f].keep = docs[fresh[f]];
    lowered[f].pols.resize(ps.size());
    for (size_t i = 0; i < ps.size(); i++) {
      std::map<Compiler::Path, uint32_t> c;
      for (auto& cond : ps[i].conds) C.count_hot(*cond.second, c);
      for (auto& kv : c) lowered[f].sum[kv.first] += kv.second;
      lowered[f].pols[i].uses.assign(c.begin(), c.end());
    }
  }
  std::vector<uint32_t> fresh_at(nd, 0xFFFFFFFFu);
  for (size_t f = 0; f < fresh.size(); f++) fresh_at[fresh[f]] = (uint32_t)f;
  auto doc_of = [&](uint32_t d) -> LowerState::Doc& { return dref[d] ? *dref[d] : lowered[fresh_at[d]]; };
  std::vector<uint32_t> kept(nd, 0);
  for (auto& tp : parsed)
    for (auto& r : tp) kept[r.doc]++;
  std::map<Compiler::Path, uint32_t> cnt;
  for (size_t d = 0; d < nd; d++) {
    LowerState::Doc& D = doc_of((uint32_t)d);
    for (auto& kv : D.sum) cnt[kv.first] += kv.second;
  }
  for (size_t d = 0; d < nd; d++) {  // a document with replaced policies: take theirs back out
    LowerState::Doc& D = doc_of((uint32_t)d);
    if (kept[d] == D.pols.size()) continue;
    std::vector<char> live(D.pols.size(), 0);
    for (auto& tp : parsed)
      for (auto& r : tp)
        if (r.doc == d) live[r.idx] = 1;
    for (size_t i = 0; i < D.pols.size(); i++)
      if (!live[i])
        for (auto& u : D.pols[i].uses) {
          auto it = cnt.find(u.first);
          if ((it->second -= u.second) == 0) cnt.erase(it);
        }
  }
  // the hot slots stay as they are while the paths a fresh build would make hot are among them
  // (a slot whose path fell out of use only costs the encoder a column)
  for (auto& kv : hot_slots(cnt))
    if (!C.hot.count(kv.first)) { *why = "hot attribute paths changed"; return nullptr; }
  for (uint32_t d : fresh)
    for (auto& p : *docs[d]) C.collect_actions(p.action);
  if (A.amask_ok && A.act.size() / 2 > MAX_ACT) { *why = "action table outgrew the action masks"; return nullptr; }
  mark("incremental check");
  // lower the new documents into the arenas
  uint64_t n_lowered = 0;
  for (size_t f = 0; f < fresh.size(); f++) {
    const auto& ps = *docs[fresh[f]];
    for (size_t i = 0; i < ps.size(); i++) {
      const size_t w0 = A.code.size() + A.cpool.size();
      C.policy(ps[i], 0);
      auto& P = lowered[f].pols[i];
      std::copy(A.pol.end() - POL_WORDS, A.pol.end(), P.w.begin());
      P.key = C.akeys.back();
      A.pol.clear();
      C.akeys.clear();
      lowered[f].words += A.code.size() + A.cpool.size() - w0;
      n_lowered++;
    }
  }
  for (size_t f = 0; f < fresh.size(); f++) {
    const void* k = docs[fresh[f]].get();
    S.docs.erase(k);
    dref[fresh[f]] = &(S.docs[k] = std::move(lowered[f]));
  }
  mark("lower");
  auto img = std::make_shared<Image>();
  img->epoch = epoch;
  img->strings = A.strings;
  img->sid = A.sid;
  img->code = A.code;
  img->cpool = A.cpool;
  img->ext_msgs = A.ext_msgs;
  img->act = A.act;
  img->hot = A.hot;
  img->amask_ok = A.amask_ok;
  // every slot a contains / containsAny atom of the arenas reads (Compiler::atom sets it while
  // lowering; removed documents' slots linger, which only costs their rows a list): the scope index
  // then never files prefix keys on them, as a fresh build would not
  img->cslot_mask = A.cslot_mask;
  img->lslot_mask = A.lslot_mask;  // (the same: removed documents' like slots linger)
  img->lread_mask = A.lread_mask;
  std::vector<Compiler::AttrKey> akeys;
  size_t total = 0;
  for (auto& tp : parsed) total += tp.size();
  // every policy's words, key and metadata at its index, written side by side
  std::vector<std::pair<uint32_t, uint32_t>> at(total);  // (tier, index in tier)
  {
    size_t q = 0;
    for (size_t t = 0; t < parsed.size(); t++) {
      for (size_t i = 0; i < parsed[t].size(); i++) at[q++] = {(uint32_t)t, (uint32_t)i};
      img->tier_end.push_back((uint32_t)q);
    }
  }
  for (auto& tp : parsed)
    for (auto& r : tp) dref[r.doc]->used = S.gen;
  img->pol.resize(total * POL_WORDS);
  img->meta.resize(total);
  akeys.resize(total);
  std::vector<uint8_t> atomic(total);
  parallel_range(total, [&](size_t q) {
    const uint32_t t = at[q].first;
    const PRef& r = parsed[t][at[q].second];
    const LowerState::Pol& P = dref[r.doc]->pols[r.idx];
    std::copy(P.w.begin(), P.w.end(), img->pol.begin() + (long)(q * POL_WORDS));
    img->pol[q * POL_WORDS + PW_FLAGS] |= t << 8;
    atomic[q] = (P.w[PW_FLAGS] & PF_ATOMIC) != 0;
    akeys[q] = P.key;
    PolicyMeta& m = img->meta[q];
    m.id = r.id; m.filename = *r.filename; m.pos = r.pos; m.tier = t;
    m.forbid = r.p->forbid;
  });
  for (size_t q = 0; q < total; q++) {
    if (atomic[q]) img->n_atomic++;
    else img->lane_need = std::max(img->lane_need, img->pol[q * POL_WORDS + PW_LANE]);
  }
  // documents this build did not use leave the cache; their words stay in the arenas as garbage
  size_t live = S.base_words;
  for (auto it = S.docs.begin(); it != S.docs.end();) {
    if (it->second.used != S.gen) it = S.docs.erase(it);
    else { live += it->second.words; ++it; }
  }
  if (A.code.size() + A.cpool.size() > 2 * live + 1024 || A.strings.size() > 2 * S.full_strings + 256)
    S.valid = false;  // the next build compacts (a full one)
  mark("assemble");
  finish_image(*img, akeys, [&] { img->srows = S.srows; img->shash = S.shash; }, mark);
  if (info) {
    info->incremental = true;
    info->lowered = n_lowered;
    info->reused = total - std::min<uint64_t>(total, n_lowered);
  }
  return img;
}

std::shared_ptr<Image> compile_image(const std::vector<std::vector<DocSpec>>& tiers, uint64_t epoch, ParseCache* cache,
                                     const std::vector<EntityIn>* statics, std::vector<DocError>* skipped,
                                     LowerState* inc, uint64_t statics_gen, BuildInfo* info) {
  if (tiers.empty()) throw CedarError("at least one policy tier is required");
  if (tiers.size() > 255) throw CedarError("too many tiers");
  // CEDARGPU_COMPILE_TIMES=1: phase times to stderr (profiling)
  static const bool times = std::getenv("CEDARGPU_COMPILE_TIMES") != nullptr;
  auto t_mark = std::chrono::steady_clock::now();
  std::function<void(const char*)> mark = [&](const char* what) {
    if (!times) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "compile %-18s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t_mark).count());
    t_mark = now;
  };
  if (info) *info = BuildInfo();
  const auto docs = parse_documents(tiers, cache, skipped);
  mark("parse");
  std::vector<std::vector<PRef>> parsed(tiers.size());
  {
    size_t di = 0;
    for (size_t t = 0; t < tiers.size(); t++) {
      size_t n = 0;
      for (size_t k = 0; k < tiers[t].size(); k++) n += docs[di + k]->size();
      for (size_t k = 0; k < tiers[t].size(); k++)
        if (!tiers[t][k].explicit_id.empty() && docs[di + k]->size() != 1)
          throw CedarError("document for policy " + tiers[t][k].explicit_id + " must hold exactly one policy");
      // every ID built side by side; when no two IDs hash alike (so none repeats) the tier is its
      // documents' policies in order, as the replacing walk below would leave it
      {
        std::vector<size_t> start(tiers[t].size() + 1, 0);
        for (size_t k = 0; k < tiers[t].size(); k++) start[k + 1] = start[k] + docs[di + k]->size();
        parsed[t].resize(n);
        std::vector<std::pair<uint64_t, uint32_t>> hs(n);
        parallel_range(n, [&](size_t q) {
          const size_t k = (size_t)(std::upper_bound(start.begin(), start.end(), q) - start.begin()) - 1;
          const DocSpec& doc = tiers[t][k];
          const std::vector<Policy>& ps = *docs[di + k];
          const size_t i = q - start[k];
          PRef& r = parsed[t][q];
          if (doc.explicit_id.empty()) {
            char nb[24];
            const auto tc = std::to_chars(nb, nb + sizeof nb, i);
            r.id.reserve(doc.id_prefix.size() + (size_t)(tc.ptr - nb) + doc.id_suffix.size());
            r.id.append(doc.id_prefix).append(nb, tc.ptr).append(doc.id_suffix);
          } else {
            r.id = doc.explicit_id;
          }
          r.p = &ps[i];
          r.filename = doc.zero_position ? &k_empty_name : &ps[i].filename;
          r.pos = doc.zero_position ? Position{} : ps[i].pos;
          r.doc = (uint32_t)(di + k);
          r.idx = (uint32_t)i;
          hs[q] = {std::hash<std::string_view>()(r.id), (uint32_t)q};
        });
        parallel_sort(hs, std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
        bool dup = false;
        for (size_t j = 1; j < n && !dup; j++) dup = hs[j].first == hs[j - 1].first;
        if (!dup) {
          di += tiers[t].size();
          continue;
        }
        parsed[t].clear();
      }
      parsed[t].reserve(n);
      // (keys view the IDs in parsed[t], which never reallocates: reserved above)
      std::unordered_map<std::string_view, size_t> ids;
      ids.reserve(n);
      for (auto& doc : tiers[t]) {
        const std::vector<Policy>& ps = *docs[di];
        if (!doc.explicit_id.empty() && ps.size() != 1)
          throw CedarError("document for policy " + doc.explicit_id + " must hold exactly one policy");
        for (size_t i = 0; i < ps.size(); i++) {
          std::string id;
          if (doc.explicit_id.empty()) {
            char nb[24];
            const auto tc = std::to_chars(nb, nb + sizeof nb, i);
            id.reserve(doc.id_prefix.size() + (size_t)(tc.ptr - nb) + doc.id_suffix.size());
            id.append(doc.id_prefix).append(nb, tc.ptr).append(doc.id_suffix);
          } else {
            id = doc.explicit_id;
          }
          PRef r{&ps[i], std::move(id), doc.zero_position ? &k_empty_name : &ps[i].filename,
                 doc.zero_position ? Position{} : ps[i].pos, (uint32_t)di, (uint32_t)i};
          auto it = ids.find(r.id);
          if (it != ids.end()) {  // a repeated ID replaces the earlier policy in its place
            const size_t at = it->second;
            ids.erase(it);
            parsed[t][at] = std::move(r);
            ids.emplace(parsed[t][at].id, at);
          } else {
            parsed[t].push_back(std::move(r));
            ids.emplace(parsed[t].back().id, parsed[t].size() - 1);
          }
        }
        di++;
      }
    }
  }
  mark("assemble");
  const char* why_full = "first build";
  if (inc && inc->valid && inc->statics_gen == statics_gen) {
    const char* why = "";
    if (auto img = compile_incremental(*inc, docs, parsed, epoch, info, &why, mark)) return img;
    why_full = why;
  } else if (inc && inc->valid) {
    why_full = "static entities changed";
  } else if (inc && inc->gen) {
    why_full = "compaction";
  }
  if (inc) inc->reset();  // a full build records afresh

  auto img = std::make_shared<Image>();
  img->epoch = epoch;
  Compiler C(*img);
  // hot attribute paths over the whole image: the NHOT most used
  std::map<Compiler::Path, uint32_t> cnt;
  std::vector<std::vector<std::pair<Compiler::Path, uint32_t>>> uses;  // per policy (incremental state)
  if (inc) {
    size_t total = 0;
    for (auto& tp : parsed) total += tp.size();
    uses.reserve(total);
  }
  for (auto& tp : parsed)
    for (auto& r : tp) {
      if (!inc) {
        for (auto& c : r.p->conds) C.count_hot(*c.second, cnt);
        continue;
      }
      std::map<Compiler::Path, uint32_t> c1;
      for (auto& c : r.p->conds) C.count_hot(*c.second, c1);
      for (auto& kv : c1) cnt[kv.first] += kv.second;
      uses.emplace_back(c1.begin(), c1.end());
    }
  C.hot = hot_slots(cnt);
  C.hot_depth.assign(C.hot.size(), 0);
  img->hot.assign(C.hot.size() * HOT_WORDS, 0);
  for (auto& kv : C.hot) {
    const Compiler::Path& path = kv.first;
    C.hot_depth[kv.second] = (uint32_t)path.second.size();
    uint32_t* h = &img->hot[(size_t)kv.second * HOT_WORDS];
    h[0] = path.first;
    h[1] = (uint32_t)path.second.size();
    for (uint32_t j = 0; j < MAX_PATH; j++) h[2 + j] = j < path.second.size() ? path.second[j] : 0u;
  }
  for (auto& tp : parsed)
    for (auto& r : tp) C.collect_actions(r.p->action);
  img->amask_ok = img->act.size() / 2 <= MAX_ACT ? 1u : 0u;
  std::vector<size_t> words;  // per policy: arena words its lowering appended (incremental state)
  for (size_t t = 0; t < parsed.size(); t++) {
    for (auto& r : parsed[t]) {
      const size_t w0 = img->code.size() + img->cpool.size();
      C.policy(*r.p, (uint32_t)t);
      if (inc) words.push_back(img->code.size() + img->cpool.size() - w0);
      PolicyMeta m;
      m.id = std::move(r.id); m.filename = *r.filename; m.pos = r.pos; m.tier = (uint32_t)t;
      m.forbid = r.p->forbid;
      img->meta.push_back(std::move(m));
    }
    img->tier_end.push_back(img->n_pol());
  }
  mark("lower");
  finish_image(*img, C.akeys, [&] { if (statics && !statics->empty()) C.statics(*statics); }, mark);
  if (inc) {  // the arenas (the static entities' lists included) and every document whose policies all stayed
    LowerState& S = *inc;
    Image& A = S.arena;
    A.strings = img->strings; A.sid = img->sid; A.code = img->code; A.cpool = img->cpool;
    A.ext_msgs = img->ext_msgs; A.act = img->act; A.hot = img->hot; A.amask_ok = img->amask_ok;
    A.cslot_mask = img->cslot_mask;
    A.lslot_mask = img->lslot_mask;
    A.lread_mask = img->lread_mask;
    S.C.hot = C.hot; S.C.hot_depth = C.hot_depth; S.C.act_index = C.act_index;
    S.gen++;
    std::vector<uint32_t> kept(docs.size(), 0);
    for (auto& tp : parsed)
      for (auto& r : tp) kept[r.doc]++;
    std::unordered_map<const void*, uint32_t> owner;  // a document parsed once but listed twice: its first listing
    size_t p = 0, owned = 0;
    for (size_t t = 0; t < parsed.size(); t++)
      for (auto& r : parsed[t]) {
        const auto& keep = docs[r.doc];
        if (kept[r.doc] == keep->size() && owner.emplace(keep.get(), r.doc).first->second == r.doc) {
          LowerState::Doc& D = S.docs[keep.get()];
          if (!D.keep) { D.keep = keep; D.pols.resize(keep->size()); D.used = S.gen; }
          LowerState::Pol& P = D.pols[r.idx];
          std::copy(&img->pol[p * POL_WORDS], &img->pol[p * POL_WORDS] + POL_WORDS, P.w.begin());
          P.w[PW_FLAGS] &= ~(0xFFu << 8);  // the tier is the build's
          P.key = C.akeys[p];
          P.uses = std::move(uses[p]);
          for (auto& u : P.uses) D.sum[u.first] += u.second;
          D.words += words[p];
          owned += words[p];
        }
        p++;
      }
    S.srows = img->srows;
    S.shash = img->shash;
    S.statics_gen = statics_gen;
    S.base_words = A.code.size() + A.cpool.size() - owned;
    S.full_strings = A.strings.size();
    S.valid = true;
    mark("record");
  }
  if (info) {
    info->incremental = false;
    info->lowered = img->n_pol();
    info->why_full = why_full;
  }
  return img;
}

// ---------------------------------------------------------------------------------------------
// Serialization: a versioned little-endian blob (what a Go-side compiler would hand to
// cg_image_load): header, the device-region section table, the device region (image.h
// DevSection: raw arrays at 256-byte-aligned offsets), then the host-only part (u32-length-
// prefixed sections).
// ---------------------------------------------------------------------------------------------
namespace {
static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "the blob's word arrays are copied as little-endian memory");
// Two passes over one writer: with no buffer it only counts bytes, then it fills an exact one.
struct W {
  uint8_t* b = nullptr;
  size_t n = 0;
  // (serialize_into: copies of >= 1 MB are collected here and run on several threads afterwards)
  std::vector<std::tuple<uint8_t*, const void*, size_t>>* defer = nullptr;
  void raw(const void* p, size_t k) {
    if (b && k) {
      if (defer && k >= (1u << 20)) defer->emplace_back(b + n, p, k);
      else std::memcpy(b + n, p, k);
    }
    n += k;
  }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void put64(size_t at, uint64_t v) { if (b) std::memcpy(b + at, &v, 8); }
  void vec(const std::vector<uint32_t>& v) { u32((uint32_t)v.size()); raw(v.data(), v.size() * 4); }
  void str(const std::string& s) { u32((uint32_t)s.size()); raw(s.data(), s.size()); }
  void align(size_t a) {
    const size_t m = (n + a - 1) / a * a;
    if (b) std::memset(b + n, 0, m - n);
    n = m;
  }
};
struct R {
  const uint8_t* p; const uint8_t* e;
  void need(size_t n) { if ((size_t)(e - p) < n) throw CedarError("truncated image"); }
  uint32_t u32() { need(4); uint32_t v; std::memcpy(&v, p, 4); p += 4; return v; }
  uint64_t u64() { uint64_t lo = u32(); return lo | ((uint64_t)u32() << 32); }
  std::vector<uint32_t> vec() { uint32_t n = u32(); need((size_t)n * 4); std::vector<uint32_t> v(n); if (n) std::memcpy(v.data(), p, (size_t)n * 4); p += (size_t)n * 4; return v; }
  std::vector<uint8_t> bytes() { uint32_t n = u32(); need(n); std::vector<uint8_t> v(p, p + n); p += n; return v; }
  std::string str() { uint32_t n = u32(); need(n); std::string s((const char*)p, n); p += n; return s; }
};
}  // namespace

void Image::write_blob(void* wp) const {
  W& w = *static_cast<W*>(wp);
  w.u32(IMG_MAGIC); w.u32(IMG_VERSION); w.u64(epoch);
  const size_t table = w.n;
  for (uint32_t k = 0; k < 2 * DS_COUNT + 2; k++) w.u64(0);  // (offset, bytes) per section, begin, end
  auto words = [](const auto& v) { return std::make_pair((const void*)v.data(), v.size() * 4); };
  const std::pair<const void*, size_t> sec[DS_COUNT] = {
      words(pstream), words(tier_cend), words(chunks), words(cpool), words(gstr_off), words(hot), words(act),
      words(btab), words(bfilt), words(bstream), words(srows), words(shash), words(sctx), words(sbits), words(svals),
      words(sbloom), std::make_pair((const void*)gstr_bytes.data(), gstr_bytes.size())};
  w.align(DS_ALIGN);
  const size_t begin = w.n;
  for (uint32_t k = 0; k < DS_COUNT; k++) {
    w.align(DS_ALIGN);
    w.put64(table + 16 * k, w.n);
    w.put64(table + 16 * k + 8, sec[k].second);
    w.raw(sec[k].first, sec[k].second);
  }
  w.raw("\0\0\0\0", 4);  // no section ends the region: a kernel may read one word of an empty one
  w.align(DS_ALIGN);
  w.put64(table + 16 * DS_COUNT, begin);
  w.put64(table + 16 * DS_COUNT + 8, w.n);
  w.vec(pol); w.vec(tier_end); w.vec(code);
  w.u32(amask_ok); w.u32(n_atomic); w.u32(indexed); w.u32(combo_mask); w.u32(lane_need); w.u32(cslot_mask);
  w.u32(pslot_mask); w.u32(lslot_mask); w.u32(lread_mask); w.vec(pfx); w.u32(btab_slots); w.u32(sbits_words); w.u32(l2_vmask); w.u32(l2_lmask);
  w.u32((uint32_t)key_ents.size());
  w.raw(key_ents.data(), key_ents.size() * 8);
  w.u32((uint32_t)strings.size());
  for (auto& s : strings) w.str(s);
  w.u32((uint32_t)meta.size());
  for (auto& m : meta) {
    w.str(m.id); w.str(m.filename);
    w.u64((uint64_t)m.pos.offset); w.u64((uint64_t)m.pos.line); w.u64((uint64_t)m.pos.column);
    w.u32(m.tier); w.u32(m.forbid ? 1 : 0);
  }
  w.u32((uint32_t)ext_msgs.size());
  for (auto& s : ext_msgs) w.str(s);
  w.vec(cls_off); w.vec(cls_mem);
}

std::vector<uint8_t> Image::serialize() const {
  W c;
  write_blob(&c);
  std::vector<uint8_t> out(c.n);
  W w{out.data(), 0};
  write_blob(&w);
  return out;
}

uint8_t* Image::serialize_malloc(size_t* len) const {
  W c;
  write_blob(&c);
  uint8_t* p = (uint8_t*)std::malloc(std::max<size_t>(c.n, 1));
  if (!p) return nullptr;
  W w{p, 0};
  write_blob(&w);
  *len = c.n;
  return p;
}

size_t Image::blob_size() const {
  W c;
  write_blob(&c);
  return c.n;
}

void Image::serialize_into(uint8_t* out) const {
  std::vector<std::tuple<uint8_t*, const void*, size_t>> big;
  W w{out, 0, &big};
  write_blob(&w);
  // the deferred copies in 4 MB pieces over up to 8 threads
  std::vector<std::tuple<uint8_t*, const uint8_t*, size_t>> pieces;
  for (auto& [d, src, k] : big)
    for (size_t o = 0; o < k; o += (4u << 20))
      pieces.emplace_back(d + o, (const uint8_t*)src + o, std::min<size_t>(4u << 20, k - o));
  const unsigned nt = (unsigned)std::min<size_t>(pieces.size(), std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t i; (i = next++) < pieces.size();) std::memcpy(std::get<0>(pieces[i]), std::get<1>(pieces[i]), std::get<2>(pieces[i]));
  };
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

std::shared_ptr<Image> Image::deserialize(const uint8_t* p, size_t n) {
  R r{p, p + n};
  if (r.u32() != IMG_MAGIC) throw CedarError("bad image magic");
  if (r.u32() != IMG_VERSION) throw CedarError("unsupported image version");
  auto img = std::make_shared<Image>();
  img->epoch = r.u64();
  for (uint32_t k = 0; k < DS_COUNT; k++) { img->dev_off[k] = r.u64(); img->dev_len[k] = r.u64(); }
  img->dev_begin = r.u64();
  img->dev_end = r.u64();
  img->blob_len = n;
  if (img->dev_begin % DS_ALIGN || img->dev_end % DS_ALIGN || img->dev_begin > img->dev_end || img->dev_end > n ||
      img->dev_begin < (size_t)(r.p - p))
    throw CedarError("corrupt image (device region)");
  auto sec_words = [&](uint32_t k, std::vector<uint32_t>& v) {
    const uint64_t off = img->dev_off[k], len = img->dev_len[k];
    if (off % DS_ALIGN || off < img->dev_begin || len % 4 || off + len + 4 > img->dev_end) throw CedarError("corrupt image (section)");
    v.resize(len / 4);
    if (len) std::memcpy(v.data(), p + off, len);  // an empty section (no static entities) has no storage
  };
  // The host keeps the sections it reads (encoder tables, string table, static entities, the
  // context table); the device-only ones (policy stream, scope index, bitsets: ~85 % of a large image) are validated
  // in place and only their sizes kept (Image::dev_len), so a load copies them once, to the device
  auto sec_view = [&](uint32_t k) -> std::pair<const uint32_t*, size_t> {
    const uint64_t off = img->dev_off[k], len = img->dev_len[k];
    if (off % DS_ALIGN || off < img->dev_begin || len % 4 || off + len + 4 > img->dev_end) throw CedarError("corrupt image (section)");
    return {reinterpret_cast<const uint32_t*>(p + off), (size_t)(len / 4)};
  };
  for (uint32_t k : {DS_PSTREAM, DS_BTAB, DS_BFILT, DS_BSTREAM, DS_SCTX, DS_SBITS, DS_SVALS, DS_SBLOOM}) (void)sec_view(k);
  sec_words(DS_TIER_CEND, img->tier_cend); sec_words(DS_CHUNKS, img->chunks);
  sec_words(DS_CPOOL, img->cpool); sec_words(DS_GSTR_OFF, img->gstr_off); sec_words(DS_HOT, img->hot);
  sec_words(DS_ACT, img->act); sec_words(DS_SROWS, img->srows); sec_words(DS_SHASH, img->shash);
  sec_words(DS_SCTX, img->sctx);  // (the encoder resolves requests' scope contexts, image.h RH_SCTX)
  {
    const uint64_t off = img->dev_off[DS_GSTR_BYTES], len = img->dev_len[DS_GSTR_BYTES];
    if (off % DS_ALIGN || off < img->dev_begin || off + len + 4 > img->dev_end) throw CedarError("corrupt image (section)");
    img->gstr_bytes.assign(p + off, p + off + len);
  }
  r.p = p + img->dev_end;
  img->pol = r.vec(); img->tier_end = r.vec(); img->code = r.vec();
  img->amask_ok = r.u32(); img->n_atomic = r.u32(); img->indexed = r.u32(); img->combo_mask = r.u32();
  img->lane_need = r.u32();
  img->cslot_mask = r.u32();
  img->pslot_mask = r.u32();
  img->lslot_mask = r.u32();
  img->lread_mask = r.u32();
  if (img->n_hot() < 32 && (img->lslot_mask >> img->n_hot())) throw CedarError("corrupt image (like slots)");
  img->pfx = r.vec();
  img->btab_slots = r.u32();
  img->sbits_words = r.u32();
  img->l2_vmask = r.u32();
  img->l2_lmask = r.u32();
  if (img->pfx.size() != (size_t)img->n_hot() * PFX_LENS && !(img->pfx.empty() && !img->pslot_mask))
    throw CedarError("corrupt image (prefix lengths)");
  {
    // entries < slots: every insertion finds a free slot and every probe chain ends at one
    const size_t bw = sec_view(DS_BTAB).second, nf = sec_view(DS_BFILT).second;
    const size_t ne = bw / BT_WORDS, nb = img->btab_slots;
    if (!ne || bw % BT_WORDS || nb < 2 || (nb & (nb - 1)) || ne >= nb || nf < 2 || (nf & (nf - 1)))
      throw CedarError("corrupt image (scope index)");
  }
  if (img->lane_need > LANE_MAX) throw CedarError("corrupt image (lane scratch)");
  {
    const auto [sctx, sctx_n] = sec_view(DS_SCTX);
    const auto [sbits, sbits_n] = sec_view(DS_SBITS);
    const size_t svals_n = sec_view(DS_SVALS).second;
    const size_t nc = sctx_n / SCTX_WORDS;
    if (!nc || (nc & (nc - 1)) || sctx_n % SCTX_WORDS || sbits_n % 2 ||
        (img->sbits_words && (sbits_n / 2) % img->sbits_words) || svals_n < SVAL_WORDS || svals_n % SVAL_WORDS ||
        sec_view(DS_SBLOOM).second != 2 * (size_t)ctx_bloom_words((uint32_t)nc))
      throw CedarError("corrupt image (scope bitsets)");
    // every context row in range, a free slot that ends every probe chain, and ranks that number
    // every set bit within svals
    size_t used = 0;
    const size_t rows = img->sbits_words ? sbits_n / 2 / img->sbits_words : 0;
    for (size_t k = 0; k < nc; k++) {
      const uint32_t* e = sctx + k * SCTX_WORDS;
      if (!e[0]) continue;
      used++;
      if (!(e[0] & SCTX_USED) || e[7] >= rows) throw CedarError("corrupt image (scope bitsets)");
    }
    if (used >= nc) throw CedarError("corrupt image (scope bitsets)");
    uint32_t rank = 0;
    for (size_t w = 0; w < sbits_n / 2; w++) {
      if (sbits[2 * w + 1] != rank) throw CedarError("corrupt image (scope bitsets)");
      rank += (uint32_t)__builtin_popcount(sbits[2 * w]);
    }
    if ((size_t)rank * SVAL_WORDS > svals_n) throw CedarError("corrupt image (scope bitsets)");
  }
  {
    const size_t ns = img->shash.size() / SH_WORDS;
    if (!ns || (ns & (ns - 1)) || img->srows.size() % ENT_WORDS || ns <= img->n_static()) throw CedarError("corrupt image (static entities)");
  }
  const uint32_t nk = r.u32();
  r.need((size_t)nk * 8);
  img->key_ents.resize(nk);
  r.need(img->key_ents.size() * 8);
  if (!img->key_ents.empty()) std::memcpy(img->key_ents.data(), r.p, img->key_ents.size() * 8);
  r.p += img->key_ents.size() * 8;
  if (img->sbits_words && img->sbits_words != (img->key_ents.size() + 31) / 32) throw CedarError("corrupt image (scope bitsets)");
  // (no `sid` map: a loaded image finds strings through `lookup`, build_lookup below)
  uint32_t ns = r.u32();
  r.need((size_t)ns * 4);
  img->strings.reserve(ns);
  for (uint32_t i = 0; i < ns; i++) img->strings.push_back(r.str());
  uint32_t nm = r.u32();
  r.need((size_t)nm * 40);  // (two length words, three u64, two u32 each at least)
  img->meta.reserve(nm);
  for (uint32_t i = 0; i < nm; i++) {
    PolicyMeta m;
    m.id = r.str(); m.filename = r.str();
    m.pos.offset = (int64_t)r.u64(); m.pos.line = (int64_t)r.u64(); m.pos.column = (int64_t)r.u64();
    m.tier = r.u32(); m.forbid = r.u32() != 0;
    img->meta.push_back(std::move(m));
  }
  uint32_t ne = r.u32();
  for (uint32_t i = 0; i < ne; i++) img->ext_msgs.push_back(r.str());
  if (img->pol.size() != (size_t)img->meta.size() * POL_WORDS) throw CedarError("corrupt image");
  img->cls_off = r.vec(); img->cls_mem = r.vec();
  {  // every policy in at most one class, the offsets ascending
    const size_t np = img->meta.size();
    bool ok = img->cls_off.empty() ? img->cls_mem.empty()
                                   : img->cls_off.size() == np + 1 && img->cls_off[0] == 0 && img->cls_off[np] == img->cls_mem.size() &&
                                         img->cls_mem.size() <= np;
    for (size_t q = 0; ok && q < np && !img->cls_off.empty(); q++) ok = img->cls_off[q] <= img->cls_off[q + 1];
    for (size_t k = 0; ok && k < img->cls_mem.size(); k++) ok = img->cls_mem[k] < np;
    if (!ok) throw CedarError("corrupt image (duplicate classes)");
  }
  img->build_lookup();
  return img;
}

// exported for the encoder
// Request strings: the image's id when the image holds the string, else a request-local id
// (EncodedRequest).
uint32_t request_sid(const Image& img, EncodedRequest& e, std::string_view s) {
  for (uint32_t k = 0; k < e.n_memo; k++)
    if (e.memo_p[k] == s.data() && e.memo_len[k] == s.size()) return e.memo_id[k];
  uint32_t id;
  const int32_t g = img.find(s);
  if (g >= 0) {
    id = (uint32_t)g;
  } else {
    // a few strings: a linear scan; past STRS_SCAN (a user in thousands of groups) a hash index,
    // so the encode stays linear in the request's size
    size_t j = e.strs.size();
    if (e.strs.size() <= EncodedRequest::STRS_SCAN) {
      for (j = 0; j < e.strs.size() && e.strs[j] != s; j++) {}
    } else {
      if (e.strs_ix.empty())
        for (uint32_t k = 0; k < e.strs.size(); k++) e.strs_ix.emplace(Image::str_hash(e.strs[k]), k);
      auto r = e.strs_ix.equal_range(Image::str_hash(s));
      for (auto it = r.first; it != r.second; ++it)
        if (e.strs[it->second] == s) { j = it->second; break; }
    }
    id = img.n_gstr() + (uint32_t)j;
    if (j == e.strs.size()) {
      id = img.n_gstr() + (uint32_t)e.strs.size();
      if (id > X_MASK) throw CedarError("string table overflow");
      e.strs.emplace_back(s);
      if (!e.strs_ix.empty()) e.strs_ix.emplace(Image::str_hash(s), (uint32_t)e.strs.size() - 1);
    }
  }
  if (e.n_memo < EncodedRequest::MEMO) {
    e.memo_p[e.n_memo] = s.data();
    e.memo_len[e.n_memo] = (uint32_t)s.size();
    e.memo_id[e.n_memo++] = id;
  }
  return id;
}

void Image::build_lookup() {
  static std::atomic<uint64_t> next_id{0};
  cache_id = ++next_id;  // the encoder's per-thread closure caches key on it (encode_impl.h)
  size_t cap = 16;
  while (cap < 2 * strings.size() + 16) cap <<= 1;
  lookup.assign(cap, 0);
  for (uint32_t i = 0; i < strings.size(); i++) {
    const uint64_t hv = str_hash(strings[i]);
    size_t h = hv & (cap - 1);
    while (lookup[h]) {
      if (strings[(uint32_t)lookup[h] - 1] == strings[i]) break;  // first id of a repeated string wins, as in `sid`
      h = (h + 1) & (cap - 1);
    }
    if (!lookup[h]) lookup[h] = ((hv >> 32) << 32) | (i + 1);
  }
  sindex.clear();
  static_targets.clear();
  for (uint32_t r = 0; r < n_static(); r++) {
    sindex.put(((uint64_t)srows[(size_t)r * ENT_WORDS + ER_TYPE] << 32) | srows[(size_t)r * ENT_WORDS + ER_ID], r);
    const uint32_t pl = srows[(size_t)r * ENT_WORDS + ER_PAD];  // direct parents [n, pairs]
    for (uint32_t k = 0; k < cpool[pl]; k++) static_targets.put(((uint64_t)cpool[pl + 1 + 2 * k] << 32) | cpool[pl + 2 + 2 * k], 0);
  }
  key_bloom.assign(std::max<size_t>(1, key_ents.size() / 4 + 1), 0);  // ~16 bits per key entity
  for (uint64_t k : key_ents) {
    const uint64_t h = (k * 0x9E3779B97F4A7C15ull) >> 40;
    key_bloom[(h >> 6) % key_bloom.size()] |= 1ull << (h & 63);
  }
}

void emit_heap_value(const HVal& v, std::vector<uint32_t>& out, const Image& img, EncodedRequest& e, uint32_t& w0,
                     uint32_t& w1) {
  auto sidf = [&img, &e](const std::string& s) { return request_sid(img, e, std::string_view(s)); };
  emit_value_impl(v, out, SP_HEAP, sidf, w0, w1);
}

}  // namespace cg
