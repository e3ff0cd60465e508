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
//   * up to NHOT pre-resolved (var, attribute) pairs evaluated once per request.
// Policy IDs follow the reference store conventions: memory `policy<i>` (memory.go:18),
// directory `<file>.policy<i>` (directory.go:76), CRD `<name><i>-<uid>` (crd.go:60),
// AVP `<id>.<i>` (verified_permissions.go:95), static `allow-all-admission` (main.go:112).
#include <algorithm>
#include <array>
#include <cstring>
#include <map>

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
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> hot;  // (var, key sid) -> hot slot
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

  void slot(uint32_t d) {
    if (d >= NSLOT) throw CedarError("expression too deep for the device register file");
    max_slot = std::max(max_slot, d + 1);
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

  uint32_t pattern(const std::vector<PatPiece>& pat) {
    // collapse into literal runs separated by stars
    std::vector<std::string> lits;
    bool has_star = false;
    std::string cur;
    bool lead_star = !pat.empty() && pat[0].star;
    (void)lead_star;
    lits.push_back("");
    for (auto& p : pat) {
      if (p.star) { has_star = true; lits.push_back(""); }
      else lits.back() += p.lit;
    }
    // lits[0] = prefix, lits.back() = suffix (when has_star), middles between (empty ones dropped)
    uint32_t off = (uint32_t)I.cpool.size();
    auto put_lit = [this](const std::string& s) {
      I.cpool.push_back((uint32_t)s.size());
      for (size_t k = 0; k < s.size(); k += 4) {
        uint32_t w = 0;
        for (size_t j = 0; j < 4 && k + j < s.size(); j++) w |= (uint32_t)(uint8_t)s[k + j] << (8 * j);
        I.cpool.push_back(w);
      }
    };
    if (!has_star) {
      I.cpool.push_back(0);  // flags: no star, 0 middles
      put_lit(lits[0]);
      return off;
    }
    std::vector<std::string> mids;
    for (size_t k = 1; k + 1 < lits.size(); k++) if (!lits[k].empty()) mids.push_back(lits[k]);
    I.cpool.push_back(1u | ((uint32_t)mids.size() << 8));
    put_lit(lits[0]);
    put_lit(lits.back());
    for (auto& m : mids) put_lit(m);
    return off;
  }

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
        if (k0.k == EK::Var) {
          auto it = hot.find({(uint32_t)var_index(k0.name), intern(e.name)});
          if (it != hot.end()) {
            emit(e.k == EK::Attr ? OP_HOT : OP_HOTHAS, d, 0, 0, it->second, 0);
            return;
          }
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
        throw CedarError("extension call " + e.name + "() with a non-constant argument is not supported by the device compiler");
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
        if (n >= 64) throw CedarError("non-constant set literal too large for the device");
        uint32_t off = lane_off;
        lane_off += 1 + 4 * n;  // [n, (w0,w1)*n, (lo,hi)*n spare for 64-bit longs]
        if (lane_off > LANE_WORDS) throw CedarError("policy needs more lane scratch than the device provides");
        emit(OP_SETNEW, d, 0, 0, 0, off | (n << 16));
        for (uint32_t i = 0; i < n; i++) {
          compile(*e.kids[i], d + 1);
          emit(OP_SETPUT, d, d + 1, 0, i, 0);
        }
        return;
      }
      case EK::Rec: {
        uint32_t n = (uint32_t)e.kids.size();
        if (n >= 64) throw CedarError("non-constant record literal too large for the device");
        uint32_t off = lane_off;
        lane_off += 1 + 5 * n;  // [n, (key,w0,w1)*n, (lo,hi)*n spare]
        if (lane_off > LANE_WORDS) throw CedarError("policy needs more lane scratch than the device provides");
        std::vector<std::pair<uint32_t, uint32_t>> order;  // (key sid, source index)
        for (uint32_t i = 0; i < n; i++) order.emplace_back(intern(e.keys[i]), i);
        std::vector<uint32_t> pos(n);
        auto sorted = order;
        std::sort(sorted.begin(), sorted.end());
        for (uint32_t k = 0; k < n; k++) pos[sorted[k].second] = k;
        emit(OP_RECNEW, d, 0, 0, 0, off | (n << 16));
        for (uint32_t i = 0; i < n; i++) {
          compile(*e.kids[i], d + 1);
          emit(OP_RECPUT, d, d + 1, 0, pos[i], order[i].first);
        }
        return;
      }
    }
    throw CedarError("unsupported expression");
  }

  void count_hot(const Expr& e, std::map<std::pair<uint32_t, uint32_t>, uint32_t>& cnt) {
    if ((e.k == EK::Attr || e.k == EK::Has) && e.kids[0]->k == EK::Var)
      cnt[{(uint32_t)var_index(e.kids[0]->name), intern(e.name)}]++;
    for (auto& k : e.kids) count_hot(*k, cnt);
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
    code0 = (uint32_t)I.code.size();
    max_slot = 0;
    lane_off = 0;
    for (auto& c : p.conds) {
      compile(*c.second, 0);
      emit(OP_COND, 0, 0, 0, c.first ? 0u : 1u, 0);
    }
    w[PW_CODE] = code0;
    w[PW_CODE_N] = (uint32_t)I.code.size() - code0;
    w[PW_SLOTS] = max_slot;
    w[PW_LANE] = lane_off;
    I.pol.insert(I.pol.end(), w, w + POL_WORDS);
  }
};

}  // namespace

std::shared_ptr<Image> compile_image(const std::vector<std::vector<DocSpec>>& tiers, uint64_t epoch) {
  if (tiers.empty()) throw CedarError("at least one policy tier is required");
  if (tiers.size() > 255) throw CedarError("too many tiers");
  auto img = std::make_shared<Image>();
  img->epoch = epoch;
  Compiler C(*img);
  // parse every tier; PolicySet.Add semantics: a repeated ID replaces the earlier policy in place
  std::vector<std::vector<Policy>> parsed(tiers.size());
  for (size_t t = 0; t < tiers.size(); t++) {
    std::unordered_map<std::string, size_t> ids;
    for (auto& doc : tiers[t]) {
      std::vector<Policy> ps = parse_policies(doc.text, doc.filename);
      if (!doc.explicit_id.empty() && ps.size() != 1)
        throw CedarError("document for policy " + doc.explicit_id + " must hold exactly one policy");
      for (size_t i = 0; i < ps.size(); i++) {
        Policy& p = ps[i];
        p.id = doc.explicit_id.empty() ? doc.id_prefix + std::to_string(i) + doc.id_suffix : doc.explicit_id;
        if (doc.zero_position) { p.pos = Position{}; p.filename = ""; }
        auto it = ids.find(p.id);
        if (it != ids.end()) parsed[t][it->second] = std::move(p);
        else { ids.emplace(p.id, parsed[t].size()); parsed[t].push_back(std::move(p)); }
      }
    }
  }
  // hot attribute selection over the whole image
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> cnt;
  for (auto& tp : parsed)
    for (auto& p : tp)
      for (auto& c : p.conds) C.count_hot(*c.second, cnt);
  std::vector<std::pair<uint32_t, std::pair<uint32_t, uint32_t>>> order;
  for (auto& kv : cnt) order.emplace_back(kv.second, kv.first);
  std::sort(order.begin(), order.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
  for (size_t k = 0; k < order.size() && k < NHOT; k++) {
    C.hot[order[k].second] = (uint32_t)k;
    img->hot.push_back(order[k].second.first);
    img->hot.push_back(order[k].second.second);
  }
  for (size_t t = 0; t < parsed.size(); t++) {
    for (auto& p : parsed[t]) {
      C.policy(p, (uint32_t)t);
      PolicyMeta m;
      m.id = p.id; m.filename = p.filename; m.pos = p.pos; m.tier = (uint32_t)t; m.forbid = p.forbid;
      img->meta.push_back(std::move(m));
    }
    img->tier_end.push_back(img->n_pol());
  }
  // global string table
  img->gstr_off.clear();
  img->gstr_bytes.clear();
  for (auto& s : img->strings) {
    img->gstr_off.push_back((uint32_t)img->gstr_bytes.size());
    img->gstr_bytes.insert(img->gstr_bytes.end(), s.begin(), s.end());
  }
  img->gstr_off.push_back((uint32_t)img->gstr_bytes.size());
  if (img->code.empty()) img->code.push_back(0), img->code.push_back(0);  // never empty buffers
  if (img->cpool.empty()) img->cpool.push_back(0);
  if (img->gstr_bytes.empty()) img->gstr_bytes.push_back(0);
  return img;
}

// ---------------------------------------------------------------------------------------------
// Serialization: a versioned little-endian blob (what a Go-side compiler would hand to
// cg_image_load). Sections are u32-length-prefixed.
// ---------------------------------------------------------------------------------------------
namespace {
struct W {
  std::vector<uint8_t> b;
  void u32(uint32_t v) { for (int k = 0; k < 4; k++) b.push_back((uint8_t)(v >> (8 * k))); }
  void u64(uint64_t v) { u32((uint32_t)v); u32((uint32_t)(v >> 32)); }
  void vec(const std::vector<uint32_t>& v) { u32((uint32_t)v.size()); for (auto x : v) u32(x); }
  void bytes(const std::vector<uint8_t>& v) { u32((uint32_t)v.size()); b.insert(b.end(), v.begin(), v.end()); }
  void str(const std::string& s) { u32((uint32_t)s.size()); b.insert(b.end(), s.begin(), s.end()); }
};
struct R {
  const uint8_t* p; const uint8_t* e;
  void need(size_t n) { if ((size_t)(e - p) < n) throw CedarError("truncated image"); }
  uint32_t u32() { need(4); uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); p += 4; return v; }
  uint64_t u64() { uint64_t lo = u32(); return lo | ((uint64_t)u32() << 32); }
  std::vector<uint32_t> vec() { uint32_t n = u32(); need((size_t)n * 4); std::vector<uint32_t> v(n); for (auto& x : v) x = u32(); return v; }
  std::vector<uint8_t> bytes() { uint32_t n = u32(); need(n); std::vector<uint8_t> v(p, p + n); p += n; return v; }
  std::string str() { uint32_t n = u32(); need(n); std::string s((const char*)p, n); p += n; return s; }
};
}  // namespace

std::vector<uint8_t> Image::serialize() const {
  W w;
  w.u32(IMG_MAGIC); w.u32(IMG_VERSION); w.u64(epoch);
  w.vec(pol); w.vec(tier_end); w.vec(code); w.vec(cpool); w.vec(gstr_off); w.vec(hot); w.bytes(gstr_bytes);
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
  return w.b;
}

std::shared_ptr<Image> Image::deserialize(const uint8_t* p, size_t n) {
  R r{p, p + n};
  if (r.u32() != IMG_MAGIC) throw CedarError("bad image magic");
  if (r.u32() != IMG_VERSION) throw CedarError("unsupported image version");
  auto img = std::make_shared<Image>();
  img->epoch = r.u64();
  img->pol = r.vec(); img->tier_end = r.vec(); img->code = r.vec(); img->cpool = r.vec();
  img->gstr_off = r.vec(); img->hot = r.vec(); img->gstr_bytes = r.bytes();
  uint32_t ns = r.u32();
  for (uint32_t i = 0; i < ns; i++) { img->strings.push_back(r.str()); img->sid.emplace(img->strings.back(), i); }
  uint32_t nm = r.u32();
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
  return img;
}

// exported for the encoder
void emit_heap_value(const HVal& v, std::vector<uint32_t>& out, Batch& b, uint32_t& w0, uint32_t& w1) {
  auto sidf = [&b](const std::string& s) { return b.sid(s); };
  emit_value_impl(v, out, SP_HEAP, sidf, w0, w1);
}

}  // namespace cg
