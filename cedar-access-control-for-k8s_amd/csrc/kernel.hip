// gfx950 evaluation kernel: tiered Cedar authorization for a batch of requests.
//
// Replaces, per request, the reference's
//   TieredPolicyStores.IsAuthorized (internal/server/store/store.go:25-42)
//     -> cedar-go (*PolicySet).IsAuthorized (call site store.go:31)
// Mapping onto CDNA4:
//   * one lane = one request; a 64-lane wave walks the policy list of each tier in lock step, so
//     every policy descriptor and bytecode word is a wave-uniform scalar load (SMEM, K$-cached),
//     and opcode dispatch is a scalar branch;
//   * the scope test (principal/action/resource) runs first; a `__ballot` skips the whole policy
//     for the wave when no lane's scope matches (the common case at 1k-100k policies);
//   * conditions run as register bytecode; `&&`/`||`/if-then-else diverge per lane through
//     forward skip targets, never through per-lane program counters;
//   * satisfied forbids/permits and errors are appended to per-request result lists; forbid
//     overrides permit; a tier falls through only on (Deny, no reasons, no errors).
// No MFMA: the work is integer compares, hashing-free ID equality and short scans.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "device.h"
#include "engine.h"
#include "image.h"

using namespace cgi;

namespace {

struct RV {
  uint32_t w0, w1, w2;
};

__device__ __forceinline__ uint32_t tag_of(const RV& v) { return v.w0 >> TAG_SHIFT; }

struct KArgs {
  const uint32_t* __restrict__ pol;
  const uint32_t* __restrict__ tier_end;
  const uint32_t* __restrict__ code;
  const uint32_t* __restrict__ cpool;
  const uint32_t* __restrict__ gstr_off;
  const uint8_t* __restrict__ gstr_bytes;
  const uint32_t* __restrict__ hot;
  const uint32_t* __restrict__ heap;
  const uint32_t* __restrict__ req_base;
  const uint32_t* __restrict__ req_idx;
  const uint32_t* __restrict__ bstr_off;
  const uint8_t* __restrict__ bstr_bytes;
  uint32_t* __restrict__ res;
  uint32_t* __restrict__ reasons_f;
  uint32_t* __restrict__ reasons_p;
  uint32_t* __restrict__ errs;
  uint32_t n_pol, n_tiers, n_gstr, n_hot, n_req, capr, cape;
};

// Per-lane evaluation context.
struct Ctx {
  const uint32_t* blk;      // request block
  const uint32_t* cpool;
  uint32_t* lh;             // lane scratch
  const KArgs* a;
  // request header cache
  uint32_t pt, pi, at, ai, rt, ri;
  uint32_t pidx, aidx, ridx;
  uint32_t nent;
};

__device__ __forceinline__ uint32_t rd(const Ctx& c, uint32_t ref, uint32_t i) {
  uint32_t sp = ref >> SPACE_SHIFT, off = (ref & OFF_MASK) + i;
  if (sp == SP_HEAP) return c.blk[off];
  if (sp == SP_CPOOL) return c.cpool[off];
  return c.lh[off];
}

__device__ __forceinline__ RV load_val(const Ctx& c, uint32_t w0, uint32_t w1) {
  uint32_t t = w0 >> TAG_SHIFT;
  if (t == T_LONG) return RV{mk_w0(T_LONG, 0), w1, ((int32_t)w1 < 0) ? 0xFFFFFFFFu : 0u};
  if (t == T_LONGREF) {
    uint32_t ref = w0 & X_MASK;
    return RV{mk_w0(T_LONG, 0), rd(c, ref, 0), rd(c, ref, 1)};
  }
  return RV{w0, w1, 0};
}

__device__ __forceinline__ uint32_t tname(const RV& v) {
  switch (tag_of(v)) {
    case T_BOOL: return TN_BOOL;
    case T_LONG: return TN_LONG;
    case T_STR: return TN_STRING;
    case T_ENT: return TN_ENTITY;
    case T_SET: return TN_SET;
    case T_REC: return TN_RECORD;
    case T_DEC: return TN_DECIMAL;
    case T_IP: return TN_IP;
    default: return TN_UNKNOWN;
  }
}

// ---- deep equality (bounded nesting) -------------------------------------------------------
template <int D>
__device__ bool veq(const Ctx& c, const RV& a, const RV& b, bool& deep);

template <int D>
__device__ __noinline__ bool veq_composite(const Ctx& c, const RV& a, const RV& b, bool& deep) {
  uint32_t t = tag_of(a);
  uint32_t ra = a.w0 & X_MASK, rb = b.w0 & X_MASK;
  if (t == T_DEC) return rd(c, ra, 0) == rd(c, rb, 0) && rd(c, ra, 1) == rd(c, rb, 1);
  if (t == T_IP) {
    for (uint32_t k = 0; k < 5; k++) if (rd(c, ra, k) != rd(c, rb, k)) return false;
    return true;
  }
  if constexpr (D == 0) {
    deep = true;
    return false;
  } else {
    uint32_t na = a.w1, nb = b.w1;
    if (t == T_SET) {
      // set equality = mutual inclusion (lane-built sets may hold duplicates)
      for (uint32_t i = 0; i < na; i++) {
        RV x = load_val(c, rd(c, ra, 1 + 2 * i), rd(c, ra, 2 + 2 * i));
        bool f = false;
        for (uint32_t j = 0; j < nb && !f; j++) f = veq<D - 1>(c, x, load_val(c, rd(c, rb, 1 + 2 * j), rd(c, rb, 2 + 2 * j)), deep);
        if (!f) return false;
      }
      for (uint32_t j = 0; j < nb; j++) {
        RV y = load_val(c, rd(c, rb, 1 + 2 * j), rd(c, rb, 2 + 2 * j));
        bool f = false;
        for (uint32_t i = 0; i < na && !f; i++) f = veq<D - 1>(c, load_val(c, rd(c, ra, 1 + 2 * i), rd(c, ra, 2 + 2 * i)), y, deep);
        if (!f) return false;
      }
      return true;
    }
    // records: unique sorted keys on both sides
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i++) {
      if (rd(c, ra, 1 + 3 * i) != rd(c, rb, 1 + 3 * i)) return false;
      RV x = load_val(c, rd(c, ra, 2 + 3 * i), rd(c, ra, 3 + 3 * i));
      RV y = load_val(c, rd(c, rb, 2 + 3 * i), rd(c, rb, 3 + 3 * i));
      if (!veq<D - 1>(c, x, y, deep)) return false;
    }
    return true;
  }
}

template <int D>
__device__ __forceinline__ bool veq(const Ctx& c, const RV& a, const RV& b, bool& deep) {
  uint32_t ta = tag_of(a), tb = tag_of(b);
  if (ta != tb) return false;
  switch (ta) {
    case T_BOOL:
    case T_STR: return a.w1 == b.w1;
    case T_LONG: return a.w1 == b.w1 && a.w2 == b.w2;
    case T_ENT: return a.w0 == b.w0 && a.w1 == b.w1;
    case T_SET:
    case T_REC:
    case T_DEC:
    case T_IP: return veq_composite<D>(c, a, b, deep);
    default: return false;
  }
}

// ---- records / entities ---------------------------------------------------------------------
__device__ __forceinline__ bool rec_get(const Ctx& c, const RV& rec, uint32_t key, RV& out) {
  uint32_t ref = rec.w0 & X_MASK, n = rec.w1;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (rd(c, ref, 1 + 3 * mid) < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && rd(c, ref, 1 + 3 * lo) == key) {
    out = load_val(c, rd(c, ref, 2 + 3 * lo), rd(c, ref, 3 + 3 * lo));
    return true;
  }
  return false;
}

__device__ __forceinline__ uint32_t find_ent(const Ctx& c, uint32_t et, uint32_t ei) {
  if (et == c.pt && ei == c.pi) return c.pidx;
  if (et == c.rt && ei == c.ri) return c.ridx;
  if (et == c.at && ei == c.ai) return c.aidx;
  for (uint32_t i = 0; i < c.nent; i++) {
    const uint32_t* row = c.blk + RH_WORDS + i * ENT_WORDS;
    if (row[ER_TYPE] == et && row[ER_ID] == ei) return i;
  }
  return NO_ENT;
}

__device__ __forceinline__ bool anc_has(const Ctx& c, uint32_t idx, uint32_t qt, uint32_t qi) {
  if (idx == NO_ENT) return false;
  uint32_t ref = c.blk[RH_WORDS + idx * ENT_WORDS + ER_ANC];
  uint32_t n = rd(c, ref, 0);
  for (uint32_t k = 0; k < n; k++)
    if (rd(c, ref, 1 + 2 * k) == qt && rd(c, ref, 2 + 2 * k) == qi) return true;
  return false;
}

__device__ __forceinline__ bool ent_in(const Ctx& c, uint32_t et, uint32_t ei, uint32_t qt, uint32_t qi) {
  if (et == qt && ei == qi) return true;
  return anc_has(c, find_ent(c, et, ei), qt, qi);
}

// ---- strings / like -------------------------------------------------------------------------
__device__ __forceinline__ void str_span(const Ctx& c, uint32_t sid, const uint8_t*& p, uint32_t& len) {
  const KArgs& a = *c.a;
  if (sid < a.n_gstr) {
    uint32_t o = a.gstr_off[sid];
    len = a.gstr_off[sid + 1] - o;
    p = a.gstr_bytes + o;
  } else {
    uint32_t j = sid - a.n_gstr;
    uint32_t o = a.bstr_off[j];
    len = a.bstr_off[j + 1] - o;
    p = a.bstr_bytes + o;
  }
}

__device__ __forceinline__ uint32_t pat_byte(const uint32_t* w, uint32_t k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }

__device__ bool lit_at(const uint8_t* s, uint32_t pos, const uint32_t* w, uint32_t n) {
  for (uint32_t k = 0; k < n; k++)
    if (s[pos + k] != pat_byte(w, k)) return false;
  return true;
}

__device__ bool like_match(const Ctx& c, uint32_t sid, uint32_t off) {
  const uint8_t* s;
  uint32_t slen;
  str_span(c, sid, s, slen);
  const uint32_t* cp = c.cpool;
  uint32_t flags = cp[off];
  uint32_t q = off + 1;
  uint32_t plen = cp[q];
  const uint32_t* pw = cp + q + 1;
  q += 1 + ((plen + 3) >> 2);
  if (!(flags & 1)) return slen == plen && lit_at(s, 0, pw, plen);
  uint32_t sl = cp[q];
  const uint32_t* sw = cp + q + 1;
  q += 1 + ((sl + 3) >> 2);
  if (slen < plen + sl) return false;
  if (!lit_at(s, 0, pw, plen)) return false;
  if (!lit_at(s, slen - sl, sw, sl)) return false;
  uint32_t pos = plen, end = slen - sl;
  uint32_t nmid = flags >> 8;
  for (uint32_t m = 0; m < nmid; m++) {
    uint32_t ml = cp[q];
    const uint32_t* mw = cp + q + 1;
    q += 1 + ((ml + 3) >> 2);
    bool found = false;
    while (pos + ml <= end) {
      if (lit_at(s, pos, mw, ml)) { found = true; break; }
      pos++;
    }
    if (!found) return false;
    pos += ml;
  }
  return true;
}

// ---- wave helpers ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, o));
  return __builtin_amdgcn_readfirstlane(x);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

struct Err {
  uint32_t code, aux, k, et, ei;
};

__device__ __forceinline__ void type_err(Err& e, uint32_t expected, const RV& got) {
  e.code = E_TYPE;
  e.aux = expected | (tname(got) << 8);
}

// i64 helpers
__device__ __forceinline__ int64_t as_i64(const RV& v) { return (int64_t)(((uint64_t)v.w2 << 32) | v.w1); }
__device__ __forceinline__ RV from_i64(int64_t x) {
  return RV{mk_w0(T_LONG, 0), (uint32_t)((uint64_t)x & 0xFFFFFFFFu), (uint32_t)((uint64_t)x >> 32)};
}
__device__ __forceinline__ RV mk_bool(bool b) { return RV{mk_w0(T_BOOL, 0), b ? 1u : 0u, 0}; }

// ---- the kernel -----------------------------------------------------------------------------
constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void cedar_eval_kernel(KArgs a) {
  const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
  const bool valid = gid < a.n_req;
  const uint32_t r = valid ? (a.req_idx ? a.req_idx[gid] : gid) : 0;

  uint32_t lane_scratch[LANE_WORDS];
  Ctx c;
  c.blk = a.heap + (valid ? a.req_base[r] : 0);
  c.cpool = a.cpool;
  c.lh = lane_scratch;
  c.a = &a;
  if (valid) {
    c.nent = c.blk[RH_NENT];
    c.pt = c.blk[RH_P] & X_MASK; c.pi = c.blk[RH_P + 1];
    c.at = c.blk[RH_A] & X_MASK; c.ai = c.blk[RH_A + 1];
    c.rt = c.blk[RH_R] & X_MASK; c.ri = c.blk[RH_R + 1];
    c.pidx = c.blk[RH_PIDX]; c.aidx = c.blk[RH_AIDX]; c.ridx = c.blk[RH_RIDX];
  } else {
    c.nent = 0; c.pt = c.pi = c.at = c.ai = c.rt = c.ri = 0xFFFFFFFFu;
    c.pidx = c.aidx = c.ridx = NO_ENT;
  }

  // pre-resolve hot (var, attribute) pairs: value + status (0 ok, else the error code ATTR would raise)
  RV hv[NHOT];
  uint32_t hs[NHOT];
  const uint32_t n_hot = a.n_hot;
#pragma unroll
  for (uint32_t h = 0; h < NHOT; h++) {
    hv[h] = RV{0, 0, 0};
    hs[h] = E_ENTITY_MISSING;
    if (h < n_hot && valid) {
      uint32_t var = a.hot[2 * h], key = a.hot[2 * h + 1];
      if (var == 3) {
        RV ctx = RV{c.blk[RH_CTX], c.blk[RH_CTX + 1], 0};
        hs[h] = rec_get(c, ctx, key, hv[h]) ? 0u : (uint32_t)E_ATTR_RECORD;
      } else {
        uint32_t idx = var == 0 ? c.pidx : var == 1 ? c.aidx : c.ridx;
        if (idx == NO_ENT) {
          hs[h] = E_ENTITY_MISSING;
        } else {
          const uint32_t* row = c.blk + RH_WORDS + idx * ENT_WORDS;
          RV attrs = RV{row[ER_ATTR0], row[ER_ATTR1], 0};
          hs[h] = rec_get(c, attrs, key, hv[h]) ? 0u : (uint32_t)E_ATTR_ENTITY;
        }
      }
    }
  }

  uint32_t S0[NSLOT], S1[NSLOT], S2[NSLOT];
#pragma unroll
  for (uint32_t k = 0; k < NSLOT; k++) { S0[k] = 0; S1[k] = 0; S2[k] = 0; }

  bool decided = !valid;
  uint32_t pbeg = 0;
  const uint32_t n_tiers = a.n_tiers;
  for (uint32_t t = 0; t < n_tiers; t++) {
    const uint32_t pend = uni(a.tier_end[t]);
    uint32_t nf = 0, np = 0, ne = 0;
    for (uint32_t p = pbeg; p < pend; p++) {
      if (__ballot(!decided) == 0) break;
      const uint32_t* d = a.pol + (size_t)p * POL_WORDS;
      const uint32_t kinds = uni(d[PW_KINDS]);
      const uint32_t pk = kinds & 0xFF, ak = (kinds >> 8) & 0xFF, rk = (kinds >> 16) & 0xFF;
      bool ok = !decided;
      // principal scope
      if (pk != SK_ANY) {
        const uint32_t ty = uni(d[PW_P_TYPE]), et = uni(d[PW_P_ET]), ei = uni(d[PW_P_EI]);
        if (pk == SK_EQ) ok = ok && c.pt == et && c.pi == ei;
        else if (pk == SK_IS) ok = ok && c.pt == ty;
        else if (pk == SK_IN) ok = ok && ((c.pt == et && c.pi == ei) || anc_has(c, c.pidx, et, ei));
        else ok = ok && c.pt == ty && ((c.pt == et && c.pi == ei) || anc_has(c, c.pidx, et, ei));
      }
      // action scope
      if (ak != SK_ANY) {
        const uint32_t et = uni(d[PW_A_ET]), ei = uni(d[PW_A_EI]);
        if (ak == SK_EQ) ok = ok && c.at == et && c.ai == ei;
        else if (ak == SK_IN) ok = ok && ((c.at == et && c.ai == ei) || anc_has(c, c.aidx, et, ei));
        else {
          bool any = false;
          for (uint32_t k = 0; k < et; k++) {
            const uint32_t qt = uni(a.cpool[ei + 2 * k]), qi = uni(a.cpool[ei + 2 * k + 1]);
            any = any || (c.at == qt && c.ai == qi) || anc_has(c, c.aidx, qt, qi);
          }
          ok = ok && any;
        }
      }
      // resource scope
      if (rk != SK_ANY) {
        const uint32_t ty = uni(d[PW_R_TYPE]), et = uni(d[PW_R_ET]), ei = uni(d[PW_R_EI]);
        if (rk == SK_EQ) ok = ok && c.rt == et && c.ri == ei;
        else if (rk == SK_IS) ok = ok && c.rt == ty;
        else if (rk == SK_IN) ok = ok && ((c.rt == et && c.ri == ei) || anc_has(c, c.ridx, et, ei));
        else ok = ok && c.rt == ty && ((c.rt == et && c.ri == ei) || anc_has(c, c.ridx, et, ei));
      }
      if (__ballot(ok) == 0) continue;

      // ---- condition bytecode ----
      const uint32_t flags = uni(d[PW_FLAGS]);
      const uint32_t* code = a.code + uni(d[PW_CODE]);
      const uint32_t n_ins = uni(d[PW_CODE_N]) >> 1;
      bool run = ok;
      bool err = false;
      uint32_t skip = 0;
      Err e{0, 0, 0, 0, 0};
      for (uint32_t pc = 0; pc < n_ins;) {
        const bool on = run && skip <= pc;
        if (__ballot(on) == 0) {
          const uint32_t nxt = wave_min(run ? skip : 0xFFFFFFFFu);
          if (nxt >= n_ins) break;
          pc = nxt;
          continue;
        }
        const uint32_t w0 = uni(code[2 * pc]);
        const uint32_t imm = uni(code[2 * pc + 1]);
        const uint32_t op = w0 & 0xFF, D = (w0 >> 8) & 63, A = (w0 >> 14) & 63, B = (w0 >> 20) & 63, C = w0 >> 26;
        if (on) {
          RV va = RV{S0[A], S1[A], S2[A]};
          RV vb = RV{S0[B], S1[B], S2[B]};
          RV out = va;
          bool wr = true;
          switch (op) {
            case OP_LDV: {
              uint32_t o = imm == 0 ? RH_P : imm == 1 ? RH_A : imm == 2 ? RH_R : RH_CTX;
              out = RV{c.blk[o], c.blk[o + 1], 0};
              break;
            }
            case OP_LDC: out = load_val(c, c.cpool[imm], c.cpool[imm + 1]); break;
            case OP_LDB: out = mk_bool(imm != 0); break;
            case OP_LDS: out = RV{mk_w0(T_STR, 0), imm, 0}; break;
            case OP_HOT: {
              uint32_t st = hs[C];
              if (st == 0) { out = hv[C]; break; }
              const uint32_t var = uni(a.hot[2 * C]);
              e.code = st;
              e.k = uni(a.hot[2 * C + 1]);
              e.et = var == 0 ? c.pt : var == 1 ? c.at : c.rt;
              e.ei = var == 0 ? c.pi : var == 1 ? c.ai : c.ri;
              err = true;
              wr = false;
              break;
            }
            case OP_HOTHAS: out = mk_bool(hs[C] == 0); break;
            case OP_ATTR:
            case OP_HAS: {
              const uint32_t t = tag_of(va);
              const bool has = op == OP_HAS;
              if (t == T_ENT) {
                uint32_t et = va.w0 & X_MASK, ei = va.w1;
                uint32_t idx = find_ent(c, et, ei);
                if (idx == NO_ENT) {
                  if (has) { out = mk_bool(false); break; }
                  e.code = E_ENTITY_MISSING; e.et = et; e.ei = ei; err = true; wr = false;
                  break;
                }
                const uint32_t* row = c.blk + RH_WORDS + idx * ENT_WORDS;
                RV got;
                bool f = rec_get(c, RV{row[ER_ATTR0], row[ER_ATTR1], 0}, imm, got);
                if (has) { out = mk_bool(f); break; }
                if (!f) { e.code = E_ATTR_ENTITY; e.k = imm; e.et = et; e.ei = ei; err = true; wr = false; break; }
                out = got;
              } else if (t == T_REC) {
                RV got;
                bool f = rec_get(c, va, imm, got);
                if (has) { out = mk_bool(f); break; }
                if (!f) { e.code = E_ATTR_RECORD; e.k = imm; err = true; wr = false; break; }
                out = got;
              } else {
                type_err(e, TN_ENTITY_OR_RECORD, va); err = true; wr = false;
              }
              break;
            }
            case OP_EQ:
            case OP_NE: {
              bool deep = false;
              bool q = veq<VAL_DEPTH>(c, va, vb, deep);
              if (deep) { e.code = E_DEPTH; err = true; wr = false; break; }
              out = mk_bool(op == OP_EQ ? q : !q);
              break;
            }
            case OP_LT: case OP_LE: case OP_GT: case OP_GE:
            case OP_ADD: case OP_SUB: case OP_MUL: {
              if (tag_of(va) != T_LONG) { type_err(e, TN_LONG, va); err = true; wr = false; break; }
              if (tag_of(vb) != T_LONG) { type_err(e, TN_LONG, vb); err = true; wr = false; break; }
              const int64_t x = as_i64(va), y = as_i64(vb);
              int64_t z = 0;
              bool of = false;
              switch (op) {
                case OP_LT: out = mk_bool(x < y); break;
                case OP_LE: out = mk_bool(x <= y); break;
                case OP_GT: out = mk_bool(x > y); break;
                case OP_GE: out = mk_bool(x >= y); break;
                case OP_ADD: of = __builtin_add_overflow(x, y, &z); out = from_i64(z); break;
                case OP_SUB: of = __builtin_sub_overflow(x, y, &z); out = from_i64(z); break;
                default: of = __builtin_mul_overflow(x, y, &z); out = from_i64(z); break;
              }
              if (of) { e.code = E_OVERFLOW; err = true; wr = false; }
              break;
            }
            case OP_NEG: {
              if (tag_of(va) != T_LONG) { type_err(e, TN_LONG, va); err = true; wr = false; break; }
              const int64_t x = as_i64(va);
              if (x == INT64_MIN) { e.code = E_OVERFLOW; err = true; wr = false; break; }
              out = from_i64(-x);
              break;
            }
            case OP_NOT:
              if (tag_of(va) != T_BOOL) { type_err(e, TN_BOOL, va); err = true; wr = false; break; }
              out = mk_bool(va.w1 == 0);
              break;
            case OP_CHKB:
              wr = false;
              if (tag_of(va) != T_BOOL) { type_err(e, TN_BOOL, va); err = true; }
              break;
            case OP_JF:
            case OP_JT:
            case OP_JNF:
              wr = false;
              if (tag_of(va) != T_BOOL) { type_err(e, TN_BOOL, va); err = true; break; }
              if ((op == OP_JT) == (va.w1 != 0)) skip = imm;
              break;
            case OP_JMP: wr = false; skip = imm; break;
            case OP_IN: {
              if (tag_of(va) != T_ENT) { type_err(e, TN_ENTITY, va); err = true; wr = false; break; }
              const uint32_t et = va.w0 & X_MASK, ei = va.w1;
              const uint32_t tb = tag_of(vb);
              if (tb == T_ENT) { out = mk_bool(ent_in(c, et, ei, vb.w0 & X_MASK, vb.w1)); break; }
              if (tb != T_SET) { type_err(e, TN_SET_OR_ENTITY, vb); err = true; wr = false; break; }
              const uint32_t ref = vb.w0 & X_MASK, n = vb.w1;
              bool bad = false;
              for (uint32_t k = 0; k < n && !bad; k++) {
                RV x = load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k));
                if (tag_of(x) != T_ENT) { type_err(e, TN_ENTITY, x); bad = true; }
              }
              if (bad) { err = true; wr = false; break; }
              const uint32_t idx = find_ent(c, et, ei);
              bool any = false;
              for (uint32_t k = 0; k < n && !any; k++) {
                const uint32_t qt = rd(c, ref, 1 + 2 * k) & X_MASK, qi = rd(c, ref, 2 + 2 * k);
                any = (et == qt && ei == qi) || anc_has(c, idx, qt, qi);
              }
              out = mk_bool(any);
              break;
            }
            case OP_IS:
              if (tag_of(va) != T_ENT) { type_err(e, TN_ENTITY, va); err = true; wr = false; break; }
              out = mk_bool((va.w0 & X_MASK) == imm);
              break;
            case OP_LIKE:
              if (tag_of(va) != T_STR) { type_err(e, TN_STRING, va); err = true; wr = false; break; }
              out = mk_bool(like_match(c, va.w1, imm));
              break;
            case OP_CONTAINS: {
              if (tag_of(va) != T_SET) { type_err(e, TN_SET, va); err = true; wr = false; break; }
              const uint32_t ref = va.w0 & X_MASK, n = va.w1;
              bool deep = false, f = false;
              for (uint32_t k = 0; k < n && !f; k++)
                f = veq<VAL_DEPTH>(c, load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k)), vb, deep);
              if (deep) { e.code = E_DEPTH; err = true; wr = false; break; }
              out = mk_bool(f);
              break;
            }
            case OP_CALL: {
              if (C == CO_CONTAINS_ALL || C == CO_CONTAINS_ANY || C == CO_IS_EMPTY) {
                if (tag_of(va) != T_SET) { type_err(e, TN_SET, va); err = true; wr = false; break; }
                if (C == CO_IS_EMPTY) { out = mk_bool(va.w1 == 0); break; }
                if (tag_of(vb) != T_SET) { type_err(e, TN_SET, vb); err = true; wr = false; break; }
                const uint32_t ra = va.w0 & X_MASK, na = va.w1, rb = vb.w0 & X_MASK, nb = vb.w1;
                bool deep = false;
                bool all = true, any = false;
                for (uint32_t j = 0; j < nb; j++) {
                  RV y = load_val(c, rd(c, rb, 1 + 2 * j), rd(c, rb, 2 + 2 * j));
                  bool f = false;
                  for (uint32_t i = 0; i < na && !f; i++)
                    f = veq<VAL_DEPTH>(c, load_val(c, rd(c, ra, 1 + 2 * i), rd(c, ra, 2 + 2 * i)), y, deep);
                  all = all && f;
                  any = any || f;
                  if (C == CO_CONTAINS_ANY ? any : !all) break;
                }
                if (deep) { e.code = E_DEPTH; err = true; wr = false; break; }
                out = mk_bool(C == CO_CONTAINS_ALL ? all : any);
                break;
              }
              if (C >= CO_DEC_LT && C <= CO_DEC_GE) {
                if (tag_of(va) != T_DEC) { type_err(e, TN_DECIMAL, va); err = true; wr = false; break; }
                if (tag_of(vb) != T_DEC) { type_err(e, TN_DECIMAL, vb); err = true; wr = false; break; }
                const uint32_t ra = va.w0 & X_MASK, rb = vb.w0 & X_MASK;
                const int64_t x = (int64_t)(((uint64_t)rd(c, ra, 1) << 32) | rd(c, ra, 0));
                const int64_t y = (int64_t)(((uint64_t)rd(c, rb, 1) << 32) | rd(c, rb, 0));
                out = mk_bool(C == CO_DEC_LT ? x < y : C == CO_DEC_LE ? x <= y : C == CO_DEC_GT ? x > y : x >= y);
                break;
              }
              // IP methods
              if (tag_of(va) != T_IP) { type_err(e, TN_IP, va); err = true; wr = false; break; }
              const uint32_t ra = va.w0 & X_MASK;
              const uint32_t hdr = rd(c, ra, 0);
              const bool v6 = (hdr & 0xFF) != 0;
              const uint32_t a0 = rd(c, ra, 1);
              if (C == CO_IP_V4) { out = mk_bool(!v6); break; }
              if (C == CO_IP_V6) { out = mk_bool(v6); break; }
              if (C == CO_IP_LOOPBACK) {
                if (!v6) { out = mk_bool((a0 >> 24) == 127); break; }
                out = mk_bool(a0 == 0 && rd(c, ra, 2) == 0 && rd(c, ra, 3) == 0 && rd(c, ra, 4) == 1);
                break;
              }
              if (C == CO_IP_MULTICAST) {
                out = mk_bool(v6 ? ((a0 >> 24) == 0xFF) : ((a0 >> 28) == 0xE));
                break;
              }
              // isInRange(b): same family, b.prefix <= a.prefix, and a's network lies inside b's
              if (tag_of(vb) != T_IP) { type_err(e, TN_IP, vb); err = true; wr = false; break; }
              {
                const uint32_t rb = vb.w0 & X_MASK;
                const uint32_t hb = rd(c, rb, 0);
                if ((hb & 0xFF) != (hdr & 0xFF)) { out = mk_bool(false); break; }
                const uint32_t pa = hdr >> 8, pb = hb >> 8;
                if (pb > pa) { out = mk_bool(false); break; }
                const uint32_t words = v6 ? 4u : 1u;
                bool in = true;
                for (uint32_t k = 0; k < words; k++) {
                  const int bits = (int)pb - (int)(32 * k);
                  const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : bits <= 0 ? 0u : (0xFFFFFFFFu << (32 - bits));
                  if ((rd(c, ra, 1 + k) & mask) != (rd(c, rb, 1 + k) & mask)) in = false;
                }
                out = mk_bool(in);
              }
              break;
            }
            case OP_SETNEW:
            case OP_RECNEW: {
              const uint32_t off = imm & 0xFFFF, n = imm >> 16;
              c.lh[off] = n;
              out = RV{mk_w0(op == OP_SETNEW ? T_SET : T_REC, mk_ref(SP_LANE, off)), n, 0};
              break;
            }
            case OP_SETPUT:
            case OP_RECPUT: {
              // store slot A (register form) into the container in slot D at position C
              wr = false;
              const RV cont = RV{S0[D], S1[D], S2[D]};
              const uint32_t base = cont.w0 & OFF_MASK, n = cont.w1;
              const bool isrec = op == OP_RECPUT;
              const uint32_t stride = isrec ? 3u : 2u;
              uint32_t* slotp = c.lh + base + 1 + stride * C;
              if (isrec) *slotp++ = imm;
              if (tag_of(va) == T_LONG) {
                const int64_t x = as_i64(va);
                if (x >= INT32_MIN && x <= INT32_MAX) { slotp[0] = mk_w0(T_LONG, 0); slotp[1] = va.w1; }
                else {
                  const uint32_t sp = base + 1 + stride * n + 2 * C;
                  c.lh[sp] = va.w1; c.lh[sp + 1] = va.w2;
                  slotp[0] = mk_w0(T_LONGREF, mk_ref(SP_LANE, sp)); slotp[1] = 0;
                }
              } else {
                slotp[0] = va.w0; slotp[1] = va.w1;
              }
              break;
            }
            case OP_COND:
              wr = false;
              if (tag_of(va) != T_BOOL) { type_err(e, TN_BOOL, va); err = true; break; }
              if ((C == 0) != (va.w1 != 0)) run = false;  // when-false or unless-true
              break;
            case OP_ERR:
              wr = false;
              e.code = C; e.aux = imm; err = true;
              break;
            default:
              wr = false;
              break;
          }
          if (err) run = false;
          if (wr) { S0[D] = out.w0; S1[D] = out.w1; S2[D] = out.w2; }
        }
        pc++;
      }
      // ---- record outcome ----
      if (ok) {
        if (err) {
          if (ne < a.cape) {
            uint32_t* er = a.errs + ((size_t)gid * a.cape + ne) * ERR_WORDS;
            er[0] = p; er[1] = e.code | (e.aux << 8); er[2] = e.k; er[3] = e.et; er[4] = e.ei; er[5] = 0;
          }
          ne++;
        } else if (run) {
          if (flags & 1) {
            if (nf < a.capr) a.reasons_f[(size_t)gid * a.capr + nf] = p;
            nf++;
          } else {
            if (np < a.capr) a.reasons_p[(size_t)gid * a.capr + np] = p;
            np++;
          }
        }
      }
    }
    if (!decided) {
      if (t + 1 == n_tiers || nf || np || ne) {
        const uint32_t dec = nf ? DEC_DENY : (np ? DEC_ALLOW : DEC_DENY);
        const uint32_t nr = nf ? nf : np;
        uint32_t fl = RF_VALID | (nf ? RF_FORBID : 0u);
        if (nr > a.capr || ne > a.cape) fl |= RF_OVERFLOW;
        a.res[2 * (size_t)gid] = dec | (t << 8) | (fl << 16);
        a.res[2 * (size_t)gid + 1] = min(nr, 0xFFFFu) | (min(ne, 0xFFFFu) << 16);
        decided = true;
      }
    }
    pbeg = pend;
  }
}

thread_local std::string g_err;

int fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return -5;  // CG_E_DEVICE
}

#define HIPCHK(x, what)                        \
  do {                                         \
    hipError_t _e = (x);                       \
    if (_e != hipSuccess) return fail(_e, what); \
  } while (0)

template <class T>
int up(T** dst, const std::vector<T>& src, size_t& bytes, hipStream_t s) {
  size_t n = std::max<size_t>(src.size(), 1) * sizeof(T);
  HIPCHK(hipMalloc((void**)dst, n), "hipMalloc");
  bytes += n;
  if (!src.empty()) HIPCHK(hipMemcpyAsync(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
  return 0;
}

}  // namespace

namespace cg {

const char* dev_last_error() { return g_err.c_str(); }

int dev_count(int* n) {
  HIPCHK(hipGetDeviceCount(n), "hipGetDeviceCount");
  return 0;
}

int dev_select(int device) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  return 0;
}

int dev_synchronize(int device) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  HIPCHK(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return 0;
}

int dev_stream_create(int device, void** stream) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  *stream = (void*)s;
  return 0;
}
void dev_stream_destroy(void* stream) { if (stream) (void)hipStreamDestroy((hipStream_t)stream); }
int dev_stream_sync(void* stream) {
  HIPCHK(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
  return 0;
}

int dev_image_upload(int device, const Image& img, DevImage* out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  DevImage d;
  d.device = device;
  hipStream_t s = nullptr;
  int rc;
  if ((rc = up(&d.pol, img.pol, d.bytes, s))) return rc;
  if ((rc = up(&d.tier_end, img.tier_end, d.bytes, s))) return rc;
  if ((rc = up(&d.code, img.code, d.bytes, s))) return rc;
  if ((rc = up(&d.cpool, img.cpool, d.bytes, s))) return rc;
  if ((rc = up(&d.gstr_off, img.gstr_off, d.bytes, s))) return rc;
  if ((rc = up(&d.hot, img.hot, d.bytes, s))) return rc;
  if ((rc = up(&d.gstr_bytes, img.gstr_bytes, d.bytes, s))) return rc;
  HIPCHK(hipStreamSynchronize(s), "sync image upload");
  d.n_pol = img.n_pol();
  d.n_tiers = img.n_tiers();
  d.n_gstr = img.n_gstr();
  d.n_hot = (uint32_t)img.hot.size() / 2;
  *out = d;
  return 0;
}

void dev_image_free(DevImage* d) {
  if (d->device < 0) return;
  (void)hipSetDevice(d->device);
  for (void* p : {(void*)d->pol, (void*)d->tier_end, (void*)d->code, (void*)d->cpool, (void*)d->gstr_off,
                  (void*)d->hot, (void*)d->gstr_bytes})
    if (p) (void)hipFree(p);
  *d = DevImage();
}

int dev_batch_upload(int device, const Batch& b, DevBatch* out, void* stream) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  DevBatch d;
  d.device = device;
  d.n = b.n();
  d.heap_words = b.heap.size();
  int rc;
  if ((rc = up(&d.heap, b.heap, d.bytes, s))) return rc;
  if ((rc = up(&d.req_base, b.req_base, d.bytes, s))) return rc;
  if ((rc = up(&d.bstr_off, b.bstr_off, d.bytes, s))) return rc;
  if ((rc = up(&d.bstr_bytes, b.bstr_bytes, d.bytes, s))) return rc;
  const size_t n = std::max<uint32_t>(b.n(), 1);
  d.capr = b.capr;
  d.cape = b.cape;
  HIPCHK(hipMalloc((void**)&d.res, n * 2 * 4), "hipMalloc res");
  HIPCHK(hipMalloc((void**)&d.reasons_f, n * d.capr * 4), "hipMalloc reasons");
  HIPCHK(hipMalloc((void**)&d.reasons_p, n * d.capr * 4), "hipMalloc reasons");
  HIPCHK(hipMalloc((void**)&d.errs, n * d.cape * ERR_WORDS * 4), "hipMalloc errs");
  HIPCHK(hipMemsetAsync(d.res, 0, n * 2 * 4, s), "memset res");
  d.bytes += n * (2 + 2 * d.capr + d.cape * ERR_WORDS) * 4;
  *out = d;
  return 0;
}

void dev_batch_free(DevBatch* d) {
  if (d->device < 0) return;
  (void)hipSetDevice(d->device);
  for (void* p : {(void*)d->heap, (void*)d->req_base, (void*)d->req_idx, (void*)d->bstr_off, (void*)d->bstr_bytes,
                  (void*)d->res, (void*)d->reasons_f, (void*)d->reasons_p, (void*)d->errs})
    if (p) (void)hipFree(p);
  *d = DevBatch();
}

static KArgs make_args(const DevImage& img, const DevBatch& b, const uint32_t* req_idx, uint32_t n, uint32_t* res,
                       uint32_t* rf, uint32_t* rp, uint32_t* er, uint32_t capr, uint32_t cape) {
  KArgs k;
  k.pol = img.pol; k.tier_end = img.tier_end; k.code = img.code; k.cpool = img.cpool;
  k.gstr_off = img.gstr_off; k.gstr_bytes = img.gstr_bytes; k.hot = img.hot;
  k.heap = b.heap; k.req_base = b.req_base; k.req_idx = req_idx;
  k.bstr_off = b.bstr_off; k.bstr_bytes = b.bstr_bytes;
  k.res = res; k.reasons_f = rf; k.reasons_p = rp; k.errs = er;
  k.n_pol = img.n_pol; k.n_tiers = img.n_tiers; k.n_gstr = img.n_gstr; k.n_hot = img.n_hot;
  k.n_req = n; k.capr = capr; k.cape = cape;
  return k;
}

int dev_eval(const DevImage& img, DevBatch& b, void* stream) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  if (b.n == 0) return 0;
  if (img.device != b.device) { g_err = "image and batch live on different devices"; return -2; }
  KArgs k = make_args(img, b, nullptr, b.n, b.res, b.reasons_f, b.reasons_p, b.errs, b.capr, b.cape);
  hipLaunchKernelGGL(cedar_eval_kernel, dim3((b.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, (hipStream_t)stream, k);
  HIPCHK(hipGetLastError(), "launch");
  return 0;
}

// Re-evaluates a subset of requests (overflowed result lists) with larger capacities; results are
// compact in subset order and copied to host before returning.
int dev_eval_subset(const DevImage& img, const DevBatch& b, const uint32_t* idx, uint32_t n, uint32_t capr,
                    uint32_t cape, void* stream, std::vector<uint32_t>& res, std::vector<uint32_t>& rf,
                    std::vector<uint32_t>& rp, std::vector<uint32_t>& er) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  for (uint32_t i = 0; i < n; i++) if (idx[i] >= b.n) { g_err = "request index out of range"; return -2; }
  uint32_t *d_idx = nullptr, *d_res = nullptr, *d_rf = nullptr, *d_rp = nullptr, *d_er = nullptr;
  int rc = 0;
  auto cleanup = [&]() { for (void* p : {(void*)d_idx, (void*)d_res, (void*)d_rf, (void*)d_rp, (void*)d_er}) if (p) (void)hipFree(p); };
  do {
    hipError_t e;
    if ((e = hipMalloc((void**)&d_idx, (size_t)n * 4)) != hipSuccess) { rc = fail(e, "hipMalloc"); break; }
    if ((e = hipMalloc((void**)&d_res, (size_t)n * 2 * 4)) != hipSuccess) { rc = fail(e, "hipMalloc"); break; }
    if ((e = hipMalloc((void**)&d_rf, (size_t)n * capr * 4)) != hipSuccess) { rc = fail(e, "hipMalloc"); break; }
    if ((e = hipMalloc((void**)&d_rp, (size_t)n * capr * 4)) != hipSuccess) { rc = fail(e, "hipMalloc"); break; }
    if ((e = hipMalloc((void**)&d_er, (size_t)n * cape * ERR_WORDS * 4)) != hipSuccess) { rc = fail(e, "hipMalloc"); break; }
    if ((e = hipMemcpyAsync(d_idx, idx, (size_t)n * 4, hipMemcpyHostToDevice, s)) != hipSuccess) { rc = fail(e, "H2D"); break; }
    KArgs k = make_args(img, b, d_idx, n, d_res, d_rf, d_rp, d_er, capr, cape);
    hipLaunchKernelGGL(cedar_eval_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, k);
    if ((e = hipGetLastError()) != hipSuccess) { rc = fail(e, "launch"); break; }
    res.resize((size_t)n * 2); rf.resize((size_t)n * capr); rp.resize((size_t)n * capr); er.resize((size_t)n * cape * ERR_WORDS);
    if ((e = hipMemcpyAsync(res.data(), d_res, res.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) { rc = fail(e, "D2H"); break; }
    if ((e = hipMemcpyAsync(rf.data(), d_rf, rf.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) { rc = fail(e, "D2H"); break; }
    if ((e = hipMemcpyAsync(rp.data(), d_rp, rp.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) { rc = fail(e, "D2H"); break; }
    if ((e = hipMemcpyAsync(er.data(), d_er, er.size() * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) { rc = fail(e, "D2H"); break; }
    if ((e = hipStreamSynchronize(s)) != hipSuccess) { rc = fail(e, "sync"); break; }
  } while (0);
  cleanup();
  return rc;
}

int dev_download(const DevBatch& b, Batch& host, void* stream) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  const size_t n = b.n;
  host.capr = b.capr;
  host.cape = b.cape;
  host.res.resize(n * 2);
  host.reasons_f.resize(n * b.capr);
  host.reasons_p.resize(n * b.capr);
  host.errs.resize(n * b.cape * ERR_WORDS);
  if (n) {
    HIPCHK(hipMemcpyAsync(host.res.data(), b.res, n * 2 * 4, hipMemcpyDeviceToHost, s), "D2H res");
    HIPCHK(hipMemcpyAsync(host.reasons_f.data(), b.reasons_f, n * b.capr * 4, hipMemcpyDeviceToHost, s), "D2H");
    HIPCHK(hipMemcpyAsync(host.reasons_p.data(), b.reasons_p, n * b.capr * 4, hipMemcpyDeviceToHost, s), "D2H");
    HIPCHK(hipMemcpyAsync(host.errs.data(), b.errs, n * b.cape * ERR_WORDS * 4, hipMemcpyDeviceToHost, s), "D2H");
  }
  HIPCHK(hipStreamSynchronize(s), "sync download");
  return 0;
}

int dev_time_eval(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_total) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0), "event");
  HIPCHK(hipEventCreate(&e1), "event");
  KArgs k = make_args(img, b, nullptr, b.n, b.res, b.reasons_f, b.reasons_p, b.errs, b.capr, b.cape);
  HIPCHK(hipEventRecord(e0, s), "event record");
  for (uint32_t i = 0; i < iters; i++)
    hipLaunchKernelGGL(cedar_eval_kernel, dim3((b.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, k);
  HIPCHK(hipGetLastError(), "launch");
  HIPCHK(hipEventRecord(e1, s), "event record");
  HIPCHK(hipEventSynchronize(e1), "event sync");
  HIPCHK(hipEventElapsedTime(ms_total, e0, e1), "elapsed");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 0;
}

}  // namespace cg
