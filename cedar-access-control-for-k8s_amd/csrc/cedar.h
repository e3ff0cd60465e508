// Host-side Cedar types for the MI355X evaluator: values, AST, parser, JSON.
//
// This is the C++ host half of the drop-in for cedar-go v1.1.0's PolicySet (the reference calls it
// at internal/server/store/store.go:31 and parses with cedar.NewPolicySetFromBytes at
// internal/server/store/memory.go:18 / cedar.NewPolicyListFromBytes at store/directory.go:69).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace cg {

struct CedarError : std::runtime_error {
  explicit CedarError(const std::string& m) : std::runtime_error(m) {}
};

// ---------------------------------------------------------------------------------------------
// Host values (policy constants and request data before device encoding)
// ---------------------------------------------------------------------------------------------
enum class VK : uint8_t { Bool, Long, Str, Ent, Set, Rec, Dec, Ip };

struct IpVal {
  uint8_t v6 = 0;      // 0 = IPv4, 1 = IPv6
  uint8_t prefix = 32; // prefix length
  uint8_t addr[16] = {0};
};

struct HVal;
using HValP = std::shared_ptr<HVal>;

struct HVal {
  VK k = VK::Bool;
  bool b = false;
  int64_t i = 0;           // Long, Decimal (scaled 1e4)
  std::string s;           // Str; Ent id
  std::string etype;       // Ent type
  std::vector<HVal> elems; // Set elements
  std::vector<std::pair<std::string, HVal>> fields; // Record (key order as given)
  IpVal ip;

  static HVal Bool(bool v) { HVal h; h.k = VK::Bool; h.b = v; return h; }
  static HVal Long(int64_t v) { HVal h; h.k = VK::Long; h.i = v; return h; }
  static HVal Str(std::string v) { HVal h; h.k = VK::Str; h.s = std::move(v); return h; }
  static HVal Ent(std::string t, std::string id) { HVal h; h.k = VK::Ent; h.etype = std::move(t); h.s = std::move(id); return h; }
};

bool hval_eq(const HVal& a, const HVal& b);
bool parse_decimal(const std::string& s, int64_t* out);
bool parse_ip(const std::string& s, IpVal* out);

// ---------------------------------------------------------------------------------------------
// AST
// ---------------------------------------------------------------------------------------------
enum class EK : uint8_t {
  Lit, Var, And, Or, Not, Neg, If, Bin, Has, Like, Is, Attr, Call, Method, Set, Rec
};
enum class BinOp : uint8_t { Eq, Ne, Lt, Le, Gt, Ge, Add, Sub, Mul, In };

struct PatPiece { bool star; std::string lit; };

struct Expr;
using ExprP = std::shared_ptr<Expr>;
struct Expr {
  EK k;
  BinOp op = BinOp::Eq;
  HVal lit;                  // Lit
  std::string name;          // Var name / attr key / type / fn / method
  std::vector<ExprP> kids;   // operands / args / elements
  std::vector<std::string> keys; // Rec keys (parallel to kids)
  std::vector<PatPiece> pat; // Like
  bool has_in = false;       // Is ... in
};

enum class ScopeKind : uint8_t { Any = 0, Eq = 1, In = 2, Is = 3, IsIn = 4, InSet = 5 };

struct Scope {
  ScopeKind kind = ScopeKind::Any;
  std::string etype;                                       // Is / IsIn
  std::pair<std::string, std::string> ent;                 // Eq / In / IsIn  (type, id)
  std::vector<std::pair<std::string, std::string>> ents;   // InSet
};

struct Position { int64_t offset = 0, line = 0, column = 0; };

struct Policy {
  bool forbid = false;
  Scope principal, action, resource;
  std::vector<std::pair<bool, ExprP>> conds;  // (is_when, expr)
  std::vector<std::pair<std::string, std::string>> annotations;
  Position pos;
  std::string filename;
  std::string id;
};

// cedar.NewPolicyListFromBytes restatement. Throws CedarError on syntax errors.
std::vector<Policy> parse_policies(const std::string& src, const std::string& filename);

// ---------------------------------------------------------------------------------------------
// Minimal JSON (entities / requests / SAR documents)
// ---------------------------------------------------------------------------------------------
struct JVal;
using JValP = std::shared_ptr<JVal>;
struct JVal {
  enum T : uint8_t { Null, Bool, Int, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const char* key) const {
    for (auto& kv : obj) if (kv.first == key) return &kv.second;
    return nullptr;
  }
  std::string str_or(const char* key, const char* dflt = "") const {
    const JVal* v = get(key);
    return (v && v->t == Str) ? v->s : std::string(dflt);
  }
};
JVal json_parse(const char* p, size_t n);
// Go encoding/json string escaping (HTML-safe: <, >, & and U+2028/9 escaped).
void go_json_string(std::string& out, const std::string& s);

// Cedar JSON value -> HVal (`__entity`, `__extn` escapes; arrays are sets; objects records).
HVal hval_from_json(const JVal& j);
void hval_to_json(const HVal& v, std::string& out);

}  // namespace cg
